#!/bin/bash
# round 3: gemm_nt after DMA spreading: numerics, timing, one PMC pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt" > gpurun_out/r3b_tests.log 2>&1 || { tail -30 gpurun_out/r3b_tests.log; exit 1; }
tail -2 gpurun_out/r3b_tests.log
timeout -k 10 300 python -u scripts/gemm_nt_bench.py > gpurun_out/r3b_bench.log 2>&1 || { tail -30 gpurun_out/r3b_bench.log; exit 1; }
grep -v "^check" gpurun_out/r3b_bench.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  ROUNDS=1 REPS=2 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "gemm_nt" -d gpurun_out/r3b_pmc$i -o run -- python3 scripts/gemm_nt_bench.py > gpurun_out/r3b_pmc$i.log 2>&1 || exit 1
done
python3 scripts/rocpd_pmc.py gpurun_out/r3b_pmc1/run_results.db gpurun_out/r3b_pmc2/run_results.db > gpurun_out/r3b_pmc.txt 2>&1 || ls -R gpurun_out/r3b_pmc1 | head
head -120 gpurun_out/r3b_pmc.txt
