#!/bin/bash
# round 3, session 3: memset nodes -> fill-kernel nodes under packet capture (probes and
# tests: no kernel indexes memory with data, cannot fault); fused CE numerics; D 128 dK/dV
# exchange buffers A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in plain kern; do
  extra=""; [ $m = kern ] && extra="--memset-kernels"
  timeout -k 10 200 python -u scripts/probe_graph_memsets.py $extra > gpurun_out/r3aa_memsets_$m.log 2>&1 || { tail -20 gpurun_out/r3aa_memsets_$m.log; exit 1; }
  grep memsets gpurun_out/r3aa_memsets_$m.log
  timeout -k 10 200 python -u scripts/probe_graph_nodes.py --rounds 50 $extra > gpurun_out/r3aa_nodes_$m.log 2>&1 || { tail -20 gpurun_out/r3aa_nodes_$m.log; exit 1; }
  grep nodes gpurun_out/r3aa_nodes_$m.log
done
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_graph_gpu.py > gpurun_out/r3aa_test_graph.log 2>&1; tail -8 gpurun_out/r3aa_test_graph.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "d128 or flash_attention or cross_entropy" > gpurun_out/r3aa_tests.log 2>&1 || { tail -40 gpurun_out/r3aa_tests.log; exit 1; }
tail -2 gpurun_out/r3aa_tests.log
for var in 2 0 2 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3aa_attn_gpt3_v$var -o run -- python3 scripts/attn_only.py --shape gpt3 --iters 20 --dropout 0.1 --k128 $var > gpurun_out/r3aa_attn_gpt3_v$var.log 2>&1 || { tail -20 gpurun_out/r3aa_attn_gpt3_v$var.log; exit 1; }
  db=$(find gpurun_out/r3aa_attn_gpt3_v$var -name "*.db" | head -1)
  python3 scripts/prof_summary.py "$db" 20 1 | tee -a gpurun_out/r3aa_attn_gpt3_summary.txt
  rm -rf gpurun_out/r3aa_attn_gpt3_v$var
done
