#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
python -m mxtrain.build > gpurun_out/build.log 2>&1 || exit 2
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_results.csv
timeout -k 10 500 python scripts/kbench.py --only gemm > gpurun_out/kbench_tuned.log 2>&1; rc=$?
grep -v "^\[" gpurun_out/kbench_tuned.log | tail -20; echo "tune rc=$rc"; [ $rc -le 1 ] || exit $rc
unset PYTORCH_TUNABLEOP_ENABLED PYTORCH_TUNABLEOP_TUNING PYTORCH_TUNABLEOP_VERBOSE
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA -d "$GRAFT_REPO_ROOT/gpurun_out/pmc" -o pmc --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/kbench.py" --only attn,norm,gelu > "$GRAFT_REPO_ROOT/gpurun_out/pmc.log" 2>&1; rc=$?
echo "pmc rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/gpurun_out/pmc.log"
