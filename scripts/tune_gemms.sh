#!/bin/bash
# Regenerate a TunableOp GEMM solution table on an MI355X (run through gpurun):
#   gpurun -- 'bash scripts/tune_gemms.sh gpt2-345m [extra bench args]'
# writes gpurun_out/tunableop_<model>0.csv; copy it to mxtrain/tuning/tunableop_<model>_gfx950.csv
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
MODEL=${1:-gpt2-345m}; shift
python -m mxtrain.build > gpurun_out/build.log 2>&1 || exit 2
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_${MODEL}.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-200}
export PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=${ROT_MB:-256}
timeout -k 10 ${T_TUNE:-900} python bench.py --model "$MODEL" --steps 5 --warmup 2 --no-graph --tune-gemm "$@" \
  > gpurun_out/tune_${MODEL}.log 2>&1; rc=$?
tail -2 gpurun_out/tune_${MODEL}.log; exit $rc
