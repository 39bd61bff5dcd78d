# batched attention-dropout masks: all on the main stream vs layers 1.. on a side stream
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/b24_a.log 2>&1 || exit 1
MXTRAIN_AUX_STREAM=1 MXTRAIN_SIDE_DMASKS=1 timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/b24_side.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/b24_b.log 2>&1 || exit 1
MXTRAIN_AUX_STREAM=1 MXTRAIN_SIDE_DMASKS=1 timeout -k 10 300 python bench.py --no-maskrcnn > gpurun_out/b24_side2.log 2>&1 || exit 1
