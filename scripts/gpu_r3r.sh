#!/bin/bash
# round 3, session 3: single-pass 8-wave D 128 dK/dV kernel -- numerics (all attention
# tests + bit-identity against the two-pass kernels) and kernel times at GPT-3 6.7B shapes
# (rocprofv3, single pass vs two passes, dropout 0.1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention or dropout" > gpurun_out/r3r_tests.log 2>&1 || { tail -40 gpurun_out/r3r_tests.log; exit 1; }
tail -2 gpurun_out/r3r_tests.log
for mode in one two; do
  extra=""; [ $mode = two ] && extra="--two-pass"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3r_attn_gpt3_$mode -o run -- python3 scripts/attn_only.py --shape gpt3 --iters 20 --dropout 0.1 $extra > gpurun_out/r3r_attn_gpt3_$mode.log 2>&1 || { tail -20 gpurun_out/r3r_attn_gpt3_$mode.log; exit 1; }
  db=$(find gpurun_out/r3r_attn_gpt3_$mode -name "*.db" | head -1)
  python3 scripts/prof_summary.py "$db" 20 6 | tee gpurun_out/r3r_attn_gpt3_${mode}_summary.txt
done
# graph packet capture: does a non-uniform dispatch (partial last workgroup) survive it?
timeout -k 10 120 python -u scripts/probe_graph_launch.py > gpurun_out/r3r_probe.log 2>&1 || { tail -20 gpurun_out/r3r_probe.log; exit 1; }
grep probe gpurun_out/r3r_probe.log
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --steps 4 --warmup 2 --out gpurun_out/r3r_mrcnn.jsonl > gpurun_out/r3r_mrcnn1.log 2>&1 || { tail -20 gpurun_out/r3r_mrcnn1.log; exit 1; }
timeout -k 10 300 python -u scripts/miopen_kernel_scan.py > gpurun_out/r3r_scan.txt 2>&1 || { tail -20 gpurun_out/r3r_scan.txt; exit 1; }
grep -c '"name"' gpurun_out/r3r_scan.txt || true
grep -i 'transpose\|"uniform_wg": "0"\|"uniform_wg": "false"' gpurun_out/r3r_scan.txt | head -20 || true
