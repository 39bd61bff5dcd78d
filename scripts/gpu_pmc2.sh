set -o pipefail
cd /root/repo && export TMPDIR=/tmp
SHAPE=gpt2 DROP=0.1 bash scripts/gpu_pmc_attn.sh || exit 1
MXTRAIN_AUX_STREAM=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_noaux.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p3_bench -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/p3_bench.log 2>&1
