#!/bin/bash
# round 3: new DP Mask R-CNN GPU test first (own time limit), then the full GPU suite,
# GEMM microbench, GPT bench A/B and a kernel-trace profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 330 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_maskrcnn_dp_gpu.py > gpurun_out/r3k_dp.log 2>&1 || { tail -60 gpurun_out/r3k_dp.log; exit 1; }
tail -3 gpurun_out/r3k_dp.log
timeout -k 10 620 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_tp_gpu.py > gpurun_out/r3k_tp.log 2>&1 || { tail -60 gpurun_out/r3k_tp.log; exit 1; }
tail -5 gpurun_out/r3k_tp.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu --deselect tests/test_tp_gpu.py --deselect tests/test_maskrcnn_dp_gpu.py > gpurun_out/r3k_tests.log 2>&1 || { tail -40 gpurun_out/r3k_tests.log; exit 1; }
tail -2 gpurun_out/r3k_tests.log
timeout -k 10 300 python -u scripts/gemm_nt_bench.py > gpurun_out/r3k_gemm.log 2>&1 || { tail -30 gpurun_out/r3k_gemm.log; exit 1; }
grep -v "^check" gpurun_out/r3k_gemm.log | tail -50
timeout -k 10 300 python -u bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3k_bench.log 2>&1 || { tail -20 gpurun_out/r3k_bench.log; exit 1; }
tail -1 gpurun_out/r3k_bench.log
timeout -k 10 300 python -u bench.py --no-fused-linear --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3k_bench_off.log 2>&1 || { tail -20 gpurun_out/r3k_bench_off.log; exit 1; }
tail -1 gpurun_out/r3k_bench_off.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k_prof -o run -- python3 bench.py --no-maskrcnn --steps 20 --warmup 5 > gpurun_out/r3k_prof.log 2>&1 || { tail -20 gpurun_out/r3k_prof.log; exit 1; }
db=$(find gpurun_out/r3k_prof -name "*.db" | head -1)
python3 scripts/prof_summary.py "$db" 26 45 > gpurun_out/r3k_prof_summary.txt && head -50 gpurun_out/r3k_prof_summary.txt
