#!/bin/bash
# round 3: GPU tests + GPT bench with the fused-epilogue GEMMs (and the hipBLASLt A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r3i_tests.log 2>&1 || { tail -40 gpurun_out/r3i_tests.log; exit 1; }
tail -2 gpurun_out/r3i_tests.log
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3i_bench.log 2>&1 || { tail -20 gpurun_out/r3i_bench.log; exit 1; }
tail -1 gpurun_out/r3i_bench.log
timeout -k 10 300 python -u bench.py --no-fused-linear --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3i_bench_off.log 2>&1 || { tail -20 gpurun_out/r3i_bench_off.log; exit 1; }
tail -1 gpurun_out/r3i_bench_off.log
