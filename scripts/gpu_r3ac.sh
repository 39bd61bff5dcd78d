#!/bin/bash
# round 3, session 3: full GPU test suite (incl. the Mask R-CNN packet-capture replay vs
# eager test), then the driver's bench (GPT + Mask R-CNN, packet capture now on by default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 600 --timeout-method thread tests > gpurun_out/r3ac_tests.log 2>&1 || { tail -40 gpurun_out/r3ac_tests.log; exit 1; }
tail -2 gpurun_out/r3ac_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3ac_bench.log 2>&1 || { tail -20 gpurun_out/r3ac_bench.log; exit 1; }
tail -1 gpurun_out/r3ac_bench.log
