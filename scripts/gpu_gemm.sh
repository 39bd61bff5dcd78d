set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_wgrad" > gpurun_out/t_gemm.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 || exit 1
