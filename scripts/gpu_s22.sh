# MIOpen NORMAL-mode find (every applicable solver benchmarked) for the Mask R-CNN
# training shapes, written to a fresh user db under gpurun_out/, then the 1 img/GPU bench
# with that db.  Progress: the db's size every 30 s.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_normal
mkdir -p $MIOPEN_USER_DB_PATH
( while true; do echo "$(date +%T) $(du -sb $MIOPEN_USER_DB_PATH | cut -f1)" >> gpurun_out/find_progress.txt; sleep 30; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
MIOPEN_FIND_MODE=NORMAL timeout -k 10 480 python scripts/bench_maskrcnn.py --batch 1 --steps 4 --warmup 2 --graph 0 > gpurun_out/find_1img.log 2>&1 || exit 1
MIOPEN_FIND_MODE=NORMAL timeout -k 10 420 python scripts/bench_maskrcnn.py --batch 4 --steps 3 --warmup 2 --graph 0 > gpurun_out/find_4img.log 2>&1 || exit 1
MIOPEN_FIND_MODE=FAST timeout -k 10 240 python scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 > gpurun_out/bench_1img_normaldb.log 2>&1 || exit 1
