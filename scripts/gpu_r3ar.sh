#!/bin/bash
# round 3, session 4: is bench.py's 4 img/GPU Mask R-CNN phase (40 steps, 10 warm-up) input
# bound?  Same run with 6 (default) and 12 data-loader workers.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 6 12 6 12; do
  timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 --workers $w > gpurun_out/r3ar_w$w.log 2>&1 || { tail -30 gpurun_out/r3ar_w$w.log; exit 1; }
  echo "workers $w: $(grep Throughput gpurun_out/r3ar_w$w.log)"
done
