set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "norm or deferred or layernorm" > gpurun_out/t19.log 2>&1 || exit 1
timeout -k 10 200 python scripts/ln_ab.py > gpurun_out/ln19.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/bench19.log 2>&1
