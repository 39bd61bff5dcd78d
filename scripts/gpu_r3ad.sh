#!/bin/bash
# round 3, session 3: sumsq rewrite numerics + GPT bench A/B: default vs --wgrad-stream
# (weight-gradient GEMMs on a concurrent side stream), interleaved on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adamw or norm or cross_entropy" > gpurun_out/r3ad_tests.log 2>&1 || { tail -30 gpurun_out/r3ad_tests.log; exit 1; }
tail -1 gpurun_out/r3ad_tests.log
for v in base ws base ws; do
  extra=""; [ $v = ws ] && extra="--wgrad-stream"
  timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 30 --warmup 5 $extra > gpurun_out/r3ad_bench_$v.log 2>&1 || { tail -20 gpurun_out/r3ad_bench_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r3ad_bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ad_prof -o run -- python3 bench.py --no-maskrcnn --steps 10 --warmup 3 > gpurun_out/r3ad_prof.log 2>&1 || { tail -20 gpurun_out/r3ad_prof.log; exit 1; }
db=$(find gpurun_out/r3ad_prof -name "*.db" | head -1)
python3 scripts/prof_summary.py "$db" 13 45 > gpurun_out/r3ad_gpt_kernel_table.txt
head -30 gpurun_out/r3ad_gpt_kernel_table.txt
rm -rf gpurun_out/r3ad_prof
