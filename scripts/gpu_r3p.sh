#!/bin/bash
# round 3: flash backward without per-element masks on interior subtiles (numerics + times + GPT bench); MIOpen kernel scan
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or dropout" > gpurun_out/r3p_tests.log 2>&1 || { tail -40 gpurun_out/r3p_tests.log; exit 1; }
tail -2 gpurun_out/r3p_tests.log
for shp in gpt2 gpt3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3p_attn_$shp -o run -- python3 scripts/attn_only.py --shape $shp --iters 20 --dropout 0.1 > gpurun_out/r3p_attn_$shp.log 2>&1 || { tail -20 gpurun_out/r3p_attn_$shp.log; exit 1; }
  db=$(find gpurun_out/r3p_attn_$shp -name "*.db" | head -1)
  python3 scripts/prof_summary.py "$db" 20 6 | tee gpurun_out/r3p_attn_${shp}_summary.txt
done
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3p_bench.log 2>&1 || { tail -20 gpurun_out/r3p_bench.log; exit 1; }
tail -1 gpurun_out/r3p_bench.log
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --steps 8 --warmup 3 --out gpurun_out/r3p_mrcnn.jsonl > gpurun_out/r3p_mrcnn1.log 2>&1 || { tail -20 gpurun_out/r3p_mrcnn1.log; exit 1; }
timeout -k 10 300 python -u scripts/miopen_kernel_scan.py > gpurun_out/r3p_scan.txt 2>&1 || { tail -20 gpurun_out/r3p_scan.txt; exit 1; }
head -12 gpurun_out/r3p_scan.txt
grep -v '"scratch": "0"' gpurun_out/r3p_scan.txt | grep '{' | head -30
