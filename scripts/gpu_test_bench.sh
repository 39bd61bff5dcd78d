set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tall.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/bench_gpt.log 2>&1 || exit 1
