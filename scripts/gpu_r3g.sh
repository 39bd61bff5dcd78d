#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/gemm_stamps.py > gpurun_out/r3g_stamps.log 2>&1; rc=$?
cat gpurun_out/r3g_stamps.log | grep -v amdgpu.ids
exit $rc
