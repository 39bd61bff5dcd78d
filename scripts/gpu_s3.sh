set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "layernorm or bda_norm or gelu or colsum or gpt_layer or swiglu" > gpurun_out/t3.log 2>&1 || exit 1
timeout -k 10 200 python scripts/kbench.py --only lnsplit,norm,gelu > gpurun_out/kbench3.log 2>&1 || exit 1
bash scripts/gpu_prof_mrcnn.sh
