mkdir -p gpurun_out/c6
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 1 --graph 1 --out gpurun_out/c6/b1_graph_pc.jsonl > gpurun_out/c6/b1_graph_pc.log 2>&1 && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 python -u scripts/bench_maskrcnn.py --batch 4 --graph 1 --out gpurun_out/c6/b4_graph_pc.jsonl > gpurun_out/c6/b4_graph_pc.log 2>&1
echo "rc=$?"
cat gpurun_out/c6/*.jsonl
