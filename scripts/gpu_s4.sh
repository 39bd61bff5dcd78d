set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_vision_ops.py tests/test_maskrcnn_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t4.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 --out gpurun_out/mr4.jsonl > gpurun_out/mr4_b1.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 --out gpurun_out/mr4.jsonl > gpurun_out/mr4_b4.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p_mr4 -o run -- python3 scripts/bench_maskrcnn.py --batch 1 --steps 40 --warmup 5 --out gpurun_out/mr4_prof.jsonl > gpurun_out/p_mr4.log 2>&1 || exit 1
db=$(find gpurun_out/p_mr4 -name "*.db" | head -1)
python3 scripts/step_census.py "$db" --top 150 > gpurun_out/census_mr4.txt || exit 1
rm -rf gpurun_out/p_mr4
bash scripts/gpu_prof_gpt.sh
