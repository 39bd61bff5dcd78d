#!/bin/bash
# round 3, session 3: D 128 dK/dV ping-pong variant (3) -- bit-identity + rocprof time
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "d128 or flash_attention" > gpurun_out/r3t_tests.log 2>&1 || { tail -40 gpurun_out/r3t_tests.log; exit 1; }
tail -2 gpurun_out/r3t_tests.log
for var in 3 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3t_attn_gpt3_v$var -o run -- python3 scripts/attn_only.py --shape gpt3 --iters 20 --dropout 0.1 --k128 $var > gpurun_out/r3t_attn_gpt3_v$var.log 2>&1 || { tail -20 gpurun_out/r3t_attn_gpt3_v$var.log; exit 1; }
  db=$(find gpurun_out/r3t_attn_gpt3_v$var -name "*.db" | head -1)
  python3 scripts/prof_summary.py "$db" 20 3 | tee gpurun_out/r3t_attn_gpt3_v${var}_summary.txt
done
timeout -k 10 300 python -u scripts/probe_graph_nodes.py --rounds 300 > gpurun_out/r3t_nodes.log 2>&1 || { tail -20 gpurun_out/r3t_nodes.log; exit 1; }
grep nodes gpurun_out/r3t_nodes.log
