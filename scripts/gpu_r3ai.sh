#!/bin/bash
# round 3, session 3: GPT-3 6.7B one-GPU bench with the size rule (hipBLASLt above 2^35
# multiply-adds), GEMM tests, and the GPT-2 bench for the record
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or linear" > gpurun_out/r3ai_tests.log 2>&1 || { tail -30 gpurun_out/r3ai_tests.log; exit 1; }
tail -1 gpurun_out/r3ai_tests.log
timeout -k 10 900 python -u bench.py --model gpt3-6.7b --micro-batch-size 2 --global-batch-size 2 --no-maskrcnn --steps 10 --warmup 3 > gpurun_out/r3ai_bench_gpt3.log 2>&1 || { tail -20 gpurun_out/r3ai_bench_gpt3.log; exit 1; }
tail -1 gpurun_out/r3ai_bench_gpt3.log
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 30 --warmup 5 > gpurun_out/r3ai_bench.log 2>&1 || { tail -20 gpurun_out/r3ai_bench.log; exit 1; }
tail -1 gpurun_out/r3ai_bench.log | cut -c1-200
