set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_vision_ops.py -m gpu -x -q --timeout 200 --timeout-method thread -k nms > gpurun_out/t8.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/op_census_maskrcnn.py --batch 1 > gpurun_out/op_census_b1.txt 2> gpurun_out/op_census_b1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p_mr8 -o run -- python3 scripts/bench_maskrcnn.py --batch 1 --steps 30 --warmup 5 --out gpurun_out/mr8_prof.jsonl > gpurun_out/p_mr8.log 2>&1 || exit 1
db=$(find gpurun_out/p_mr8 -name "*.db" | head -1)
python3 scripts/step_census.py "$db" --top 250 > gpurun_out/census_mr8_b1.txt
rm -rf gpurun_out/p_mr8
