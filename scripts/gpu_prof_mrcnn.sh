# Mask R-CNN launch census: rocprofv3 kernel trace of the eager and the graphed step at
# 1 img/GPU; scripts/step_census.py averages the last 10 steps (one-time work excluded)
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
for mode in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p_mr_$mode -o run -- python3 scripts/bench_maskrcnn.py --batch 1 --steps 40 --warmup 5 --graph $mode --out gpurun_out/mr_$mode.jsonl > gpurun_out/p_mr_$mode.log 2>&1 || exit 1
  db=$(find gpurun_out/p_mr_$mode -name "*.db" | head -1)
  python3 scripts/step_census.py "$db" --top 150 > gpurun_out/census_mr_graph$mode.txt || exit 1
  rm -rf gpurun_out/p_mr_$mode
done
