#!/bin/bash
# round 3, session 3: GPT-3 6.7B shapes -- hand-written fused-epilogue GEMMs vs hipBLASLt
# (microbench at T = 4096, H = 4096, and the one-GPU bench with --no-fused-linear)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T=4096 H=4096 ROUNDS=5 timeout -k 10 600 python -u scripts/gemm_nt_bench.py > gpurun_out/r3ah_gemm_gpt3.log 2>&1 || { tail -20 gpurun_out/r3ah_gemm_gpt3.log; exit 1; }
grep -v "^check" gpurun_out/r3ah_gemm_gpt3.log
timeout -k 10 900 python -u bench.py --model gpt3-6.7b --micro-batch-size 2 --global-batch-size 2 --no-maskrcnn --no-fused-linear --steps 10 --warmup 3 > gpurun_out/r3ah_bench_gpt3_blaslt.log 2>&1 || { tail -20 gpurun_out/r3ah_bench_gpt3_blaslt.log; exit 1; }
tail -1 gpurun_out/r3ah_bench_gpt3_blaslt.log | cut -c1-300
