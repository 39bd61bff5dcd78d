set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vision_ops.py tests/test_maskrcnn_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t6.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 --out gpurun_out/mr6.jsonl > gpurun_out/mr6_b1.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 --out gpurun_out/mr6.jsonl > gpurun_out/mr6_b4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p_mr6 -o run -- python3 scripts/bench_maskrcnn.py --batch 1 --steps 30 --warmup 5 --out gpurun_out/mr6_prof.jsonl > gpurun_out/p_mr6.log 2>&1 || exit 1
db=$(find gpurun_out/p_mr6 -name "*.db" | head -1)
python3 scripts/step_census.py "$db" --top 250 > gpurun_out/census_mr6_b1.txt
rm -rf gpurun_out/p_mr6
