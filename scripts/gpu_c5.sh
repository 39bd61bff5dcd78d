mkdir -p gpurun_out/c8
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for t in 1 0; do
MXTRAIN_ROIALIGN_TILED=$t timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_t$t -o run -- python -u scripts/bench_maskrcnn.py --batch 4 --graph 0 --steps 20 --warmup 10 --out gpurun_out/c8/b4_t$t.jsonl > gpurun_out/c8/b4_t$t.log 2>&1 || exit 1
db=$(find /tmp/prof_t$t -name "*.db" | head -1)
python3 scripts/rocpd_stats.py "$db" --csv gpurun_out/c8/kstats_t$t.csv --top 50 > gpurun_out/c8/kstats_t$t.txt
done
cat gpurun_out/c8/*.jsonl
