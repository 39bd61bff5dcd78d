set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_vision_ops.py -x -q --timeout 200 --timeout-method thread -m gpu -k "gelu or conv_bias_act" > gpurun_out/t26.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/bench26.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 > gpurun_out/b26_mr1.log 2>&1 || exit 1
bash scripts/gpu_prof_gpt.sh
