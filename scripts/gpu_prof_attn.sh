set -o pipefail
cd /root/repo && export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p_attn2 -o run -- python3 scripts/attn_only.py --shape gpt2 --dropout 0.1 > gpurun_out/p_attn2.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/p_attn3 -o run -- python3 scripts/attn_only.py --shape gpt3 --dropout 0.1 > gpurun_out/p_attn3.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p_bench -o run -- python3 bench.py --steps 10 --warmup 3 --no-graph > gpurun_out/p_bench.log 2>&1
