#!/bin/bash
# round 3, session 3: GPT bench (fused single-pass CE), then Mask R-CNN images/s with the
# graph's memset nodes rewritten into fill kernels: packet capture off (baseline) then ON
# (the configuration that faulted before the rewrite: last steps of the script)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graph_gpu.py tests/test_kernels_gpu.py -k "graph or d128 or cross_entropy" > gpurun_out/r3ab_tests.log 2>&1 || { tail -30 gpurun_out/r3ab_tests.log; exit 1; }
tail -1 gpurun_out/r3ab_tests.log
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3ab_bench.log 2>&1 || { tail -20 gpurun_out/r3ab_bench.log; exit 1; }
tail -1 gpurun_out/r3ab_bench.log
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 --out gpurun_out/r3ab_mrcnn.jsonl > gpurun_out/r3ab_mrcnn_b1_pc0.log 2>&1 || { tail -20 gpurun_out/r3ab_mrcnn_b1_pc0.log; exit 1; }
tail -1 gpurun_out/r3ab_mrcnn.jsonl | cut -c1-400
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 --out gpurun_out/r3ab_mrcnn.jsonl > gpurun_out/r3ab_mrcnn_b1_pc1.log 2>&1 || { tail -20 gpurun_out/r3ab_mrcnn_b1_pc1.log; exit 1; }
tail -1 gpurun_out/r3ab_mrcnn.jsonl | cut -c1-400
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 --out gpurun_out/r3ab_mrcnn.jsonl > gpurun_out/r3ab_mrcnn_b4_pc1.log 2>&1 || { tail -20 gpurun_out/r3ab_mrcnn_b4_pc1.log; exit 1; }
tail -1 gpurun_out/r3ab_mrcnn.jsonl | cut -c1-400
