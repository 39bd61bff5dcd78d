#!/bin/bash
# round 3: flash backward dropout-mask rewrite -- numerics, per-kernel times (GPT-2 / GPT-3 shapes), GPT bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or dropout or bda" > gpurun_out/r3n_tests.log 2>&1 || { tail -40 gpurun_out/r3n_tests.log; exit 1; }
tail -2 gpurun_out/r3n_tests.log
for shp in gpt2 gpt3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_attn_$shp -o run -- python3 scripts/attn_only.py --shape $shp --iters 20 --dropout 0.1 > gpurun_out/r3n_attn_$shp.log 2>&1 || { tail -20 gpurun_out/r3n_attn_$shp.log; exit 1; }
  db=$(find gpurun_out/r3n_attn_$shp -name "*.db" | head -1)
  python3 scripts/prof_summary.py "$db" 20 8 | tee gpurun_out/r3n_attn_${shp}_summary.txt
done
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3n_bench.log 2>&1 || { tail -20 gpurun_out/r3n_bench.log; exit 1; }
tail -1 gpurun_out/r3n_bench.log
