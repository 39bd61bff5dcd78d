#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt" > gpurun_out/r3h_tests.log 2>&1 || { tail -30 gpurun_out/r3h_tests.log; exit 1; }
tail -1 gpurun_out/r3h_tests.log
timeout -k 10 200 python -u scripts/gemm_stamps.py > gpurun_out/r3h_stamps.log 2>&1 || { tail -20 gpurun_out/r3h_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3h_stamps.log | head -12
timeout -k 10 300 python -u scripts/gemm_nt_bench.py > gpurun_out/r3h_bench.log 2>&1 || { tail -30 gpurun_out/r3h_bench.log; exit 1; }
grep -v "^check" gpurun_out/r3h_bench.log
