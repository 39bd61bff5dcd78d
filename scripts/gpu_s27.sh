# Mask R-CNN 1 img/GPU: bench + graphed-step census after the unsorted post-NMS top-k
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_maskrcnn_gpu.py -x -q --timeout 250 --timeout-method thread -m gpu > gpurun_out/t27.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 > gpurun_out/b27_mr1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/p_mr27 -o run -- python3 scripts/bench_maskrcnn.py --batch 1 --steps 40 --warmup 5 --graph 1 --out gpurun_out/mr27.jsonl > gpurun_out/p_mr27.log 2>&1 || exit 1
db=$(find gpurun_out/p_mr27 -name "*.db" | head -1)
python3 scripts/step_census.py "$db" --top 150 > gpurun_out/census_mr27.txt || exit 1
rm -rf gpurun_out/p_mr27
