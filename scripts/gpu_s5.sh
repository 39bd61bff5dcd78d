set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vision_ops.py tests/test_maskrcnn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t5.log 2>&1 || exit 1
for b in 1 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p_mr5_$b -o run -- python3 scripts/bench_maskrcnn.py --batch $b --steps 30 --warmup 5 --out gpurun_out/mr5_prof.jsonl > gpurun_out/p_mr5_$b.log 2>&1 || exit 1
  db=$(find gpurun_out/p_mr5_$b -name "*.db" | head -1)
  python3 scripts/step_census.py "$db" --top 200 > gpurun_out/census_mr5_b$b.txt || exit 1
  rm -rf gpurun_out/p_mr5_$b
done
timeout -k 10 450 python bench.py > gpurun_out/bench5.log 2>&1
