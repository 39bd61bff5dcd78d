#!/bin/bash
# round 3, session 3: which round-3 change breaks the deferred-optimizer bit-identity test?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in base nobias noce neither; do
  timeout -k 10 300 python -u scripts/bisect_deferred.py $m > gpurun_out/r3ag_$m.log 2>&1
  grep -E "bisect|passed|failed|assert runs" gpurun_out/r3ag_$m.log | head -5
done
