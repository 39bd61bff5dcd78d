#!/bin/bash
# round 3, session 4: full GPU test suite and the driver's default bench (GPT-2 + Mask R-CNN
# 1 / 4 img) with every implicit-GEMM convolution path on (final tree).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3aq_tests.log 2>&1 || { tail -30 gpurun_out/r3aq_tests.log; exit 1; }
tail -2 gpurun_out/r3aq_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3aq_bench.log 2>&1 || { tail -20 gpurun_out/r3aq_bench.log; exit 1; }
tail -1 gpurun_out/r3aq_bench.log
