set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "attention or gpt_layer" > gpurun_out/t2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p2_attn2 -o run -- python3 scripts/attn_only.py --shape gpt2 --dropout 0.1 > gpurun_out/p2_attn2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p2_attn2n -o run -- python3 scripts/attn_only.py --shape gpt2 --dropout 0.0 > gpurun_out/p2_attn2n.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p2_attn3 -o run -- python3 scripts/attn_only.py --shape gpt3 --dropout 0.1 > gpurun_out/p2_attn3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench2.log 2>&1
