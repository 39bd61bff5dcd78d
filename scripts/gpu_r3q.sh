#!/bin/bash
# round 3, session 3: full GPU tests after the flash diagonal-branch commit, the driver's
# bench, and the graph packet-capture investigation (bounds-checked launch probe; kernel
# trace of the graphed Mask R-CNN replay with packet capture off -> non-uniform MIOpen
# dispatches; MIOpen code-object scan).  No step of this script replays with capture on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
true
true
timeout -k 10 120 python -u scripts/probe_graph_launch.py > gpurun_out/r3q_probe.log 2>&1 || { tail -20 gpurun_out/r3q_probe.log; exit 1; }
cat gpurun_out/r3q_probe.log | grep probe
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3q_mrcnn_trace -o run -- python3 scripts/bench_maskrcnn.py --batch 1 --steps 6 --warmup 2 --out gpurun_out/r3q_mrcnn_trace.jsonl > gpurun_out/r3q_mrcnn_trace.log 2>&1 || { tail -20 gpurun_out/r3q_mrcnn_trace.log; exit 1; }
csv=$(find gpurun_out/r3q_mrcnn_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/nonuniform_dispatches.py "$csv" > gpurun_out/r3q_nonuniform.txt
head -40 gpurun_out/r3q_nonuniform.txt
rm -f "$csv"
timeout -k 10 300 python -u scripts/miopen_kernel_scan.py > gpurun_out/r3q_scan.txt 2>&1 || { tail -20 gpurun_out/r3q_scan.txt; exit 1; }
grep -c '"name"' gpurun_out/r3q_scan.txt || true
timeout -k 10 600 python -u bench.py > gpurun_out/r3q_bench.log 2>&1 || { tail -20 gpurun_out/r3q_bench.log; exit 1; }
tail -1 gpurun_out/r3q_bench.log
