#!/bin/bash
# round 3, session 3: colsum rewrite numerics, GPT-2 bench, and the GPT-3 6.7B one-GPU
# builder bench (whole model on one 288 GB GPU, mbs 2, seq 2048, dropout 0.1/0.1) with the
# single-pass D 128 attention backward
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "colsum or norm or gpt" > gpurun_out/r3ae_tests.log 2>&1 || { tail -30 gpurun_out/r3ae_tests.log; exit 1; }
tail -1 gpurun_out/r3ae_tests.log
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 30 --warmup 5 > gpurun_out/r3ae_bench.log 2>&1 || { tail -20 gpurun_out/r3ae_bench.log; exit 1; }
tail -1 gpurun_out/r3ae_bench.log
timeout -k 10 900 python -u bench.py --model gpt3-6.7b --micro-batch-size 2 --global-batch-size 2 --no-maskrcnn --steps 10 --warmup 3 > gpurun_out/r3ae_bench_gpt3.log 2>&1 || { tail -20 gpurun_out/r3ae_bench_gpt3.log; exit 1; }
tail -1 gpurun_out/r3ae_bench_gpt3.log
timeout -k 10 900 python -u -m pytest -s -q --timeout 600 --timeout-method thread tests/test_maskrcnn_gpu.py tests/test_maskrcnn_packet_capture_gpu.py -k "graphed or packet" > gpurun_out/r3ae_mrcnn_tests.log 2>&1 || { tail -30 gpurun_out/r3ae_mrcnn_tests.log; exit 1; }
grep -E "relative|eager vs graph|passed|failed" gpurun_out/r3ae_mrcnn_tests.log
