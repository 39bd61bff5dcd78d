mkdir -p gpurun_out/c24
timeout -k 10 200 python -u -m pytest tests/test_vision_ops.py tests/test_maskrcnn_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/c24/tests.log 2>&1 || { tail -30 gpurun_out/c24/tests.log; exit 1; }
tail -2 gpurun_out/c24/tests.log
for b in 1 4; do
timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch $b --out gpurun_out/c24/b$b.jsonl > gpurun_out/c24/b$b.log 2>&1 || { tail -5 gpurun_out/c24/b$b.log; exit 1; }
done
cat gpurun_out/c24/*.jsonl; grep -o "per step.*" gpurun_out/c24/b*.log | tail -2
