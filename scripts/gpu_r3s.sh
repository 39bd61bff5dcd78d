#!/bin/bash
# round 3, session 3: big-kernarg packet-capture probe; D 128 dK/dV variants (single pass,
# + static priority) numerics and rocprof times at GPT-3 shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/probe_graph_bigargs.py --nodes 2000 > gpurun_out/r3s_bigargs.log 2>&1 || { tail -20 gpurun_out/r3s_bigargs.log; exit 1; }
grep bigargs gpurun_out/r3s_bigargs.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "d128 or flash_attention" > gpurun_out/r3s_tests.log 2>&1 || { tail -40 gpurun_out/r3s_tests.log; exit 1; }
tail -2 gpurun_out/r3s_tests.log
for var in 0 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3s_attn_gpt3_v$var -o run -- python3 scripts/attn_only.py --shape gpt3 --iters 20 --dropout 0.1 --k128 $var > gpurun_out/r3s_attn_gpt3_v$var.log 2>&1 || { tail -20 gpurun_out/r3s_attn_gpt3_v$var.log; exit 1; }
  db=$(find gpurun_out/r3s_attn_gpt3_v$var -name "*.db" | head -1)
  python3 scripts/prof_summary.py "$db" 20 3 | tee gpurun_out/r3s_attn_gpt3_v${var}_summary.txt
done
