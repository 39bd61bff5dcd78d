#!/bin/bash
# round 3: gemm_nt loop v2 (saddr DMA, unrolled ring, BK32 variants): numerics + timing + PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt" > gpurun_out/r3d_tests.log 2>&1 || { tail -30 gpurun_out/r3d_tests.log; exit 1; }
tail -2 gpurun_out/r3d_tests.log
timeout -k 10 300 python -u scripts/gemm_nt_bench.py > gpurun_out/r3d_bench.log 2>&1 || { tail -30 gpurun_out/r3d_bench.log; exit 1; }
grep -v "^check" gpurun_out/r3d_bench.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU"
ROUNDS=1 REPS=2 timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-include-regex "gemm_nt" -d gpurun_out/r3d_pmc1 -o run -- python3 scripts/gemm_nt_bench.py > gpurun_out/r3d_pmc1.log 2>&1 || exit 1
python3 scripts/rocpd_pmc.py gpurun_out/r3d_pmc1/run_results.db > gpurun_out/r3d_pmc.txt 2>&1
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r3d_counters.txt 2>&1 || true
