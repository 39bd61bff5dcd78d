#!/bin/bash
# round 3: which MIOpen kernels the graphed Mask R-CNN step uses and what their code objects
# require at dispatch (read-only scan of the user kernel cache after a short run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --steps 12 --warmup 4 --out gpurun_out/r3o_mrcnn.jsonl > gpurun_out/r3o_mrcnn1.log 2>&1 || { tail -20 gpurun_out/r3o_mrcnn1.log; exit 1; }
timeout -k 10 300 python -u scripts/miopen_kernel_scan.py > gpurun_out/r3o_scan.txt 2>&1 || { tail -20 gpurun_out/r3o_scan.txt; exit 1; }
head -5 gpurun_out/r3o_scan.txt
grep -c '"scratch": "0"' gpurun_out/r3o_scan.txt || true
grep -v '"scratch": "0"' gpurun_out/r3o_scan.txt | head -40
