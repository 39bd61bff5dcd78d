#!/bin/bash
# round 3, session 3: flash bwd QKV-bias partials + colsum/sumsq/CE changes (numerics), graph
# tests, Mask R-CNN graphed-vs-eager drift printouts, GPT-2 bench, GPT-3 6.7B one-GPU bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_graph_gpu.py tests/test_tp_gpu.py > gpurun_out/r3af_tests.log 2>&1 || { tail -40 gpurun_out/r3af_tests.log; exit 1; }
tail -1 gpurun_out/r3af_tests.log
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 30 --warmup 5 > gpurun_out/r3af_bench.log 2>&1 || { tail -20 gpurun_out/r3af_bench.log; exit 1; }
tail -1 gpurun_out/r3af_bench.log
timeout -k 10 900 python -u -m pytest -s -q --timeout 600 --timeout-method thread tests/test_maskrcnn_gpu.py tests/test_maskrcnn_packet_capture_gpu.py -k "graphed or packet" > gpurun_out/r3af_mrcnn_tests.log 2>&1 || { tail -30 gpurun_out/r3af_mrcnn_tests.log; exit 1; }
grep -E "relative|eager vs graph|passed|failed" gpurun_out/r3af_mrcnn_tests.log
timeout -k 10 900 python -u bench.py --model gpt3-6.7b --micro-batch-size 2 --global-batch-size 2 --no-maskrcnn --steps 10 --warmup 3 > gpurun_out/r3af_bench_gpt3.log 2>&1 || { tail -20 gpurun_out/r3af_bench_gpt3.log; exit 1; }
tail -1 gpurun_out/r3af_bench_gpt3.log
