#!/bin/bash
# round 3 (re-entry): state check -- gemm_nt numerics + microbench, GPU tests, GPT bench fused vs hipBLASLt
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/gemm_nt_bench.py > gpurun_out/r3j_gemm.log 2>&1 || { tail -30 gpurun_out/r3j_gemm.log; exit 1; }
grep -v "^check" gpurun_out/r3j_gemm.log | tail -50
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r3j_tests.log 2>&1 || { tail -40 gpurun_out/r3j_tests.log; exit 1; }
tail -2 gpurun_out/r3j_tests.log
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3j_bench.log 2>&1 || { tail -20 gpurun_out/r3j_bench.log; exit 1; }
tail -1 gpurun_out/r3j_bench.log
timeout -k 10 300 python -u bench.py --no-fused-linear --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3j_bench_off.log 2>&1 || { tail -20 gpurun_out/r3j_bench_off.log; exit 1; }
tail -1 gpurun_out/r3j_bench_off.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3j_prof -o run -- python3 bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3j_prof.log 2>&1 || { tail -20 gpurun_out/r3j_prof.log; exit 1; }
db=$(find gpurun_out/r3j_prof -name "*.db" | head -1)
python3 scripts/prof_summary.py "$db" 26 45 > gpurun_out/r3j_prof_summary.txt && head -50 gpurun_out/r3j_prof_summary.txt
