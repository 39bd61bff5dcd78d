#!/bin/bash
# round 3: 8-phase 256x256 GEMM numerics + microbench; row top-k; GEMM stamps; Mask R-CNN bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt or gemm_p8" > gpurun_out/r3m_gemm_tests.log 2>&1 || { tail -40 gpurun_out/r3m_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r3m_gemm_tests.log
timeout -k 10 300 python -u scripts/gemm_nt_bench.py > gpurun_out/r3m_gemm.log 2>&1 || { tail -30 gpurun_out/r3m_gemm.log; exit 1; }
grep -v "^check" gpurun_out/r3m_gemm.log | grep -E "==|torch|v1 |v6 |v9 |v0 |v3 |total"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vision_ops.py tests/test_maskrcnn_gpu.py -m gpu > gpurun_out/r3m_tests.log 2>&1 || { tail -40 gpurun_out/r3m_tests.log; exit 1; }
tail -2 gpurun_out/r3m_tests.log
timeout -k 10 200 python -u scripts/gemm_stamps.py > gpurun_out/r3m_stamps.log 2>&1 || { tail -20 gpurun_out/r3m_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3m_stamps.log
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 --out gpurun_out/r3m_mrcnn.jsonl > gpurun_out/r3m_mrcnn1.log 2>&1 || { tail -20 gpurun_out/r3m_mrcnn1.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 --out gpurun_out/r3m_mrcnn.jsonl > gpurun_out/r3m_mrcnn4.log 2>&1 || { tail -20 gpurun_out/r3m_mrcnn4.log; exit 1; }
cat gpurun_out/r3m_mrcnn.jsonl
