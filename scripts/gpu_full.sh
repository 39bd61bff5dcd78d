set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tall.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p2_attn2 -o run -- python3 scripts/attn_only.py --shape gpt2 --dropout 0.1 > gpurun_out/p2_attn2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench2.log 2>&1
