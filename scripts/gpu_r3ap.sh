#!/bin/bash
# round 3, session 4: implicit-GEMM conv forward -- tests, per-shape A/B (wgrad / dgrad /
# fwd+bias vs MIOpen), Mask R-CNN 1 img/GPU with the forward off (default) and on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_convwg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ap_tests.log 2>&1 || { tail -40 gpurun_out/r3ap_tests.log; exit 1; }
tail -1 gpurun_out/r3ap_tests.log
timeout -k 10 300 python -u scripts/conv_wgrad_bench.py > gpurun_out/r3ap_convwg.txt 2>&1 || { tail -30 gpurun_out/r3ap_convwg.txt; exit 1; }
cat gpurun_out/r3ap_convwg.txt
timeout -k 10 400 python -u scripts/bench_maskrcnn_ab.py FWD=0 -- --batch 1 --steps 40 --warmup 10 > gpurun_out/r3ap_mrcnn1_fwd0.log 2>&1 || { tail -30 gpurun_out/r3ap_mrcnn1_fwd0.log; exit 1; }
tail -2 gpurun_out/r3ap_mrcnn1_fwd0.log
timeout -k 10 400 python -u scripts/bench_maskrcnn_ab.py FWD=1 -- --batch 1 --steps 40 --warmup 10 > gpurun_out/r3ap_mrcnn1_fwd1.log 2>&1 || { tail -30 gpurun_out/r3ap_mrcnn1_fwd1.log; exit 1; }
tail -2 gpurun_out/r3ap_mrcnn1_fwd1.log
timeout -k 10 400 python -u scripts/bench_maskrcnn_ab.py FWD=1 -- --batch 4 --steps 30 --warmup 8 > gpurun_out/r3ap_mrcnn4_fwd1.log 2>&1 || { tail -30 gpurun_out/r3ap_mrcnn4_fwd1.log; exit 1; }
tail -2 gpurun_out/r3ap_mrcnn4_fwd1.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ap_alltests.log 2>&1 || { tail -30 gpurun_out/r3ap_alltests.log; exit 1; }
tail -2 gpurun_out/r3ap_alltests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3ap_bench.log 2>&1 || { tail -20 gpurun_out/r3ap_bench.log; exit 1; }
tail -1 gpurun_out/r3ap_bench.log
