#!/bin/bash
# One gpurun session: kernel numerics tests, smoke, bench, rocprof summary.
# Each GPU step has its own time limit; after a crash/timeout (exit >= 124 or signal)
# nothing further touches the GPU.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
python -m mxtrain.build > gpurun_out/build.log 2>&1 || { echo "build failed"; cat gpurun_out/build.log; exit 2; }
STEPS="${STEPS:-tests smoke bench}"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 ${T_TESTS:-600} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?
      tail -30 gpurun_out/gpu_tests.log; echo "tests rc=$rc"; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
      tail -5 gpurun_out/smoke.log; echo "smoke rc=$rc"; ok $rc || exit $rc ;;
    bench)
      timeout -k 10 ${T_BENCH:-400} python bench.py --gpus 1 --steps ${BSTEPS:-20} --warmup ${BWARM:-5} ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
      tail -5 gpurun_out/bench.log; echo "bench rc=$rc"; ok $rc || exit $rc ;;
    slice)
      timeout -k 10 ${T_SLICE:-900} python scripts/gpu_slice.py ${SLICE_ARGS:-} > gpurun_out/slice.log 2>&1; rc=$?
      tail -20 gpurun_out/slice.log; echo "slice rc=$rc"; ok $rc || exit $rc ;;
    mrcnn)
      timeout -k 10 ${T_MRCNN:-600} python scripts/bench_maskrcnn.py ${MRCNN_ARGS:-} > gpurun_out/mrcnn.log 2>&1; rc=$?
      tail -12 gpurun_out/mrcnn.log; echo "mrcnn rc=$rc"; ok $rc || exit $rc ;;
    mrprof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 ${T_PROF:-500} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/mrprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/bench_maskrcnn.py" --steps 12 --warmup 6 ${MRCNN_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/mrprof.log" 2>&1; rc=$?
      cd "$GRAFT_REPO_ROOT"; tail -5 gpurun_out/mrprof.log; echo "mrprof rc=$rc"; ok $rc || exit $rc ;;
    kbench)
      timeout -k 10 300 python scripts/kbench.py ${KBENCH_ARGS:-} > gpurun_out/kbench.log 2>&1; rc=$?
      cat gpurun_out/kbench.log | tail -40; echo "kbench rc=$rc"; ok $rc || exit $rc ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 5 --warmup 3 ${PROF_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; rc=$?
      cd "$GRAFT_REPO_ROOT"; tail -5 gpurun_out/prof.log; echo "prof rc=$rc"; ok $rc || exit $rc ;;
  esac
done
echo ALLDONE
