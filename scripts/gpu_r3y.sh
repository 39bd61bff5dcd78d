#!/bin/bash
# round 3, session 3: (1) graph tests + node probe with the driver-getter rewrite;
# (2) D 128 dK/dV 64-rows-per-step variant: bit-identity + time; (3) capture-only HIP API
# census of the Mask R-CNN step with the training conv search (no replay)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "d128 or flash_attention" > gpurun_out/r3y_tests.log 2>&1 || { tail -40 gpurun_out/r3y_tests.log; exit 1; }
tail -2 gpurun_out/r3y_tests.log
for var in 2 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3y_attn_gpt3_v$var -o run -- python3 scripts/attn_only.py --shape gpt3 --iters 20 --dropout 0.1 --k128 $var > gpurun_out/r3y_attn_gpt3_v$var.log 2>&1 || { tail -20 gpurun_out/r3y_attn_gpt3_v$var.log; exit 1; }
  db=$(find gpurun_out/r3y_attn_gpt3_v$var -name "*.db" | head -1)
  python3 scripts/prof_summary.py "$db" 20 3 | tee gpurun_out/r3y_attn_gpt3_v${var}_summary.txt
done
AMD_LOG_LEVEL=3 timeout -k 10 500 python3 scripts/graph_diag.py --mode graph --batch 1 --capture-only --find-db > gpurun_out/r3y_diag.out 2> /tmp/r3y_diag.err
echo "diag rc=$?"
python3 scripts/capture_memcpy_census.py /tmp/r3y_diag.err > gpurun_out/r3y_memcpy_census.txt
tail -60 gpurun_out/r3y_memcpy_census.txt
grep -m5 "hipMemcpyAsync" /tmp/r3y_diag.err | cut -c1-200 || true
