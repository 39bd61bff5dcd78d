#!/bin/bash
# round 3, session 4: conv weight gradient with the implicit-GEMM forward with fused epilogue: tests,
# graphed per-shape A/B vs MIOpen, Mask R-CNN 1 and 4 img/GPU, kernel trace of the step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_convwg_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3ao_tests.log 2>&1 || { tail -40 gpurun_out/r3ao_tests.log; exit 1; }
tail -1 gpurun_out/r3ao_tests.log
timeout -k 10 300 python -u scripts/conv_wgrad_bench.py > gpurun_out/r3ao_convwg.txt 2>&1 || { tail -30 gpurun_out/r3ao_convwg.txt; exit 1; }
cat gpurun_out/r3ao_convwg.txt
timeout -k 10 400 python -u scripts/bench_maskrcnn.py --batch 1 --steps 40 --warmup 10 --out gpurun_out/r3ao_mrcnn1.jsonl > gpurun_out/r3ao_mrcnn1.log 2>&1 || { tail -30 gpurun_out/r3ao_mrcnn1.log; exit 1; }
tail -2 gpurun_out/r3ao_mrcnn1.log
timeout -k 10 400 python -u scripts/bench_maskrcnn.py --batch 4 --steps 30 --warmup 8 --out gpurun_out/r3ao_mrcnn4.jsonl > gpurun_out/r3ao_mrcnn4.log 2>&1 || { tail -30 gpurun_out/r3ao_mrcnn4.log; exit 1; }
tail -2 gpurun_out/r3ao_mrcnn4.log
