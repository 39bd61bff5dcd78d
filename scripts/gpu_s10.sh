set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t10.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_attn10 -o run -- python3 scripts/kbench.py --only attn,attn128 > gpurun_out/kb10.log 2>&1 || exit 1
db=$(find gpurun_out/p_attn10 -name "*.db" | head -1)
python3 scripts/prof_summary.py "$db" 1 30 > gpurun_out/attn10_summary.txt
rm -rf gpurun_out/p_attn10
timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/bench10.log 2>&1
