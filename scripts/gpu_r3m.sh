#!/bin/bash
# round 3: 8-phase 256x256 GEMM numerics + microbench; row top-k; GEMM stamps; Mask R-CNN bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt or gemm_p8" > gpurun_out/r3m_gemm_tests.log 2>&1 || { tail -40 gpurun_out/r3m_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r3m_gemm_tests.log
timeout -k 10 300 python -u scripts/gemm_nt_bench.py > gpurun_out/r3m_gemm.log 2>&1 || { tail -30 gpurun_out/r3m_gemm.log; exit 1; }
grep -v "^check" gpurun_out/r3m_gemm.log | grep -E "==|torch|v1 |v6 |v9 |v10 |v0 |v3 |total"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vision_ops.py tests/test_maskrcnn_gpu.py -m gpu > gpurun_out/r3m_tests.log 2>&1 || { tail -40 gpurun_out/r3m_tests.log; exit 1; }
tail -2 gpurun_out/r3m_tests.log
timeout -k 10 200 python -u scripts/gemm_stamps.py > gpurun_out/r3m_stamps.log 2>&1 || { tail -20 gpurun_out/r3m_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3m_stamps.log
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 --out gpurun_out/r3m_mrcnn.jsonl > gpurun_out/r3m_mrcnn1.log 2>&1 || { tail -20 gpurun_out/r3m_mrcnn1.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 --out gpurun_out/r3m_mrcnn.jsonl > gpurun_out/r3m_mrcnn4.log 2>&1 || { tail -20 gpurun_out/r3m_mrcnn4.log; exit 1; }
cat gpurun_out/r3m_mrcnn.jsonl
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
