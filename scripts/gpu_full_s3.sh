# full GPU test suite + default bench (GPT + Mask R-CNN) + GPT kernel profile
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/full_bench.log 2>&1 || exit 1
bash scripts/gpu_prof_gpt.sh
