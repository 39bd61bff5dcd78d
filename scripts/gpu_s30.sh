# Mask R-CNN 4 img/GPU: conv-epilogue bias index by mask vs modulo (same box, alternating)
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
for m in 1 0 1 0; do
  MXTRAIN_EPI_MASK=$m timeout -k 10 300 python scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 > gpurun_out/b30_$m.log 2>&1 || exit 1
  echo "mask=$m $(grep Throughput gpurun_out/b30_$m.log | tail -1)" >> gpurun_out/b30_summary.txt
done
