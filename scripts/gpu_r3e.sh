#!/bin/bash
# round 3: why does per-CU GEMM efficiency collapse at full occupancy?  (T=1024 -> 64 tiles of
# 256x256 vs T=4096 -> 256 tiles) + clock / L2 / TA counters
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=1024 ROUNDS=5 timeout -k 10 300 python -u scripts/gemm_nt_bench.py > gpurun_out/r3e_bench_t1024.log 2>&1 || { tail -30 gpurun_out/r3e_bench_t1024.log; exit 1; }
grep -v "^check" gpurun_out/r3e_bench_t1024.log | grep -A10 "fc1_fwd"
PA="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_WAVES SQ_BUSY_CYCLES"
PB="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum SQ_INSTS_VMEM SQ_WAIT_INST_ANY"
i=0
for P in "$PA" "$PB"; do
  i=$((i+1))
  ROUNDS=1 REPS=2 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "gemm_nt" -d gpurun_out/r3e_pmc$i -o run -- python3 scripts/gemm_nt_bench.py > gpurun_out/r3e_pmc$i.log 2>&1 || { tail -5 gpurun_out/r3e_pmc$i.log; exit 1; }
done
python3 scripts/rocpd_pmc_grid.py gpurun_out/r3e_pmc1/run_results.db gpurun_out/r3e_pmc2/run_results.db > gpurun_out/r3e_pmc.txt 2>&1
grep -A17 "true, 2, 4, 8, 4, 64, 2, 1, 2>\|true, 2, 4, 4, 2, 64, 4, 1, 0>" gpurun_out/r3e_pmc.txt
