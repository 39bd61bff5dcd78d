set -o pipefail
cd /root/repo && export TMPDIR=/tmp
for cfg in 64,64 128,128 64,128 128,64; do
  d=gpurun_out/qbk_${cfg/,/_}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d -o run -- python3 scripts/attn_only.py --shape gpt2 --dropout 0.1 --iters 40 --qbk $cfg > $d.log 2>&1 || exit 1
done
for cfg in 64_64 128_128 64_128 128_64; do echo "== $cfg"; f=$(find gpurun_out/qbk_$cfg -name "*kernel_stats.csv" | head -1); grep flash "$f" | cut -d, -f1-8; done > gpurun_out/qbk_summary.txt
