#!/bin/bash
# round 3, session 3: (1) memset size/alignment probe under packet capture (no data
# indexing: cannot fault); (2) D 128 dK/dV one vs two exchange buffers, same box;
# (3) graph test; (4) memset census of the Mask R-CNN capture window (capture only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/probe_graph_memsets.py > gpurun_out/r3z_memsets.log 2>&1 || { tail -20 gpurun_out/r3z_memsets.log; exit 1; }
grep memsets gpurun_out/r3z_memsets.log
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graph_gpu.py > gpurun_out/r3z_test_graph.log 2>&1 || { tail -30 gpurun_out/r3z_test_graph.log; exit 1; }
tail -2 gpurun_out/r3z_test_graph.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "d128 or flash_attention" > gpurun_out/r3z_tests.log 2>&1 || { tail -40 gpurun_out/r3z_tests.log; exit 1; }
tail -2 gpurun_out/r3z_tests.log
for var in 2 0 2 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3z_attn_gpt3_v$var -o run -- python3 scripts/attn_only.py --shape gpt3 --iters 20 --dropout 0.1 --k128 $var > gpurun_out/r3z_attn_gpt3_v$var.log 2>&1 || { tail -20 gpurun_out/r3z_attn_gpt3_v$var.log; exit 1; }
  db=$(find gpurun_out/r3z_attn_gpt3_v$var -name "*.db" | head -1)
  python3 scripts/prof_summary.py "$db" 20 1 | tee -a gpurun_out/r3z_attn_gpt3_summary.txt
  rm -rf gpurun_out/r3z_attn_gpt3_v$var
done
AMD_LOG_LEVEL=3 timeout -k 10 500 python3 scripts/graph_diag.py --mode graph --batch 1 --capture-only --find-db > gpurun_out/r3z_diag.out 2> /tmp/r3z_diag.err
echo "diag rc=$?"
python3 scripts/capture_memcpy_census.py /tmp/r3z_diag.err > gpurun_out/r3z_memcpy_census.txt
cat gpurun_out/r3z_memcpy_census.txt | head -80
