# 1 img/GPU Mask R-CNN: 1x1 convolutions as hipBLASLt GEMMs vs MIOpen (same box)
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
MXTRAIN_CONV1X1_GEMM=1 timeout -k 10 300 python scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 > gpurun_out/b23_gemm1x1.log 2>&1 || exit 1
timeout -k 10 300 python scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 > gpurun_out/b23_miopen.log 2>&1 || exit 1
