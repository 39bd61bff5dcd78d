set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "deferred or layernorm or bda_norm or rmsnorm or norm" > gpurun_out/t17.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/bench17.log 2>&1 || exit 1
bash scripts/gpu_prof_gpt.sh
