set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gpt -o run -- python3 bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/p_gpt.log 2>&1 || exit 1
db=$(ls gpurun_out/p_gpt/*/run_results.db 2>/dev/null | head -1); [ -z "$db" ] && db=$(find gpurun_out/p_gpt -name "*.db" | head -1)
python3 scripts/prof_summary.py "$db" 26 45 > gpurun_out/p_gpt_summary.txt
