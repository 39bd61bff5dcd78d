#!/bin/bash
# round 3: row top-k numerics, GEMM tile anatomy (stamps), Mask R-CNN 1/4 img bench with the new top-k
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vision_ops.py tests/test_maskrcnn_gpu.py -m gpu > gpurun_out/r3l_tests.log 2>&1 || { tail -40 gpurun_out/r3l_tests.log; exit 1; }
tail -2 gpurun_out/r3l_tests.log
timeout -k 10 200 python -u scripts/gemm_stamps.py > gpurun_out/r3l_stamps.log 2>&1 || { tail -20 gpurun_out/r3l_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3l_stamps.log
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 --out gpurun_out/r3l_mrcnn.jsonl > gpurun_out/r3l_mrcnn1.log 2>&1 || { tail -20 gpurun_out/r3l_mrcnn1.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 --out gpurun_out/r3l_mrcnn.jsonl > gpurun_out/r3l_mrcnn4.log 2>&1 || { tail -20 gpurun_out/r3l_mrcnn4.log; exit 1; }
cat gpurun_out/r3l_mrcnn.jsonl
