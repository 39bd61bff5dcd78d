set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "attn or flash or attention or dropmask" > gpurun_out/t18.log 2>&1 || exit 1
timeout -k 10 200 python scripts/attn_ab.py > gpurun_out/ab18.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/bench18.log 2>&1
