set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_wgrad" > gpurun_out/t_gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p_attn3 -o run -- python3 scripts/attn_only.py --shape gpt2 --dropout 0.1 > gpurun_out/p_attn3.log 2>&1 || exit 1
db=$(find gpurun_out/p_attn3 -name "*.db" | head -1); python3 scripts/prof_summary.py "$db" 20 12 > gpurun_out/p_attn3_summary.txt
