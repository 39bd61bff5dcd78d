#!/bin/bash
# One gpurun session, parameterised (the one wrapper every GPU call goes through):
#   STEPS="tests smoke bench"  (also: slice mrcnn mrprof kbench prof pmc)
#   PYTEST_K (a -k expression, may contain spaces) / PYTEST_ARGS / BENCH_ARGS / MRCNN_ARGS / KBENCH_ARGS / PROF_ARGS / SLICE_ARGS
#   pmc: PMC_CMD (python script + args, run directly after rocprofv3's --), PMC_REGEX
#        (kernel-name filter), one rocprofv3 pass per counter group (SQ <= 8 per pass)
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
      timeout -k 10 ${T_TESTS:-900} python -u -m pytest ${PYTEST_TARGET:-tests} -m gpu ${PYTEST_X--x} -q --timeout ${T_TEST:-300} --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?
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
      # whole-step kernel census of Mask R-CNN (MRCNN_ARGS e.g. "--batch 4"), summarised on the box
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 ${T_PROF:-500} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${PROF_TAG:-mrprof}" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/bench_maskrcnn.py" --steps ${MR_STEPS:-12} --warmup 6 ${MRCNN_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/${PROF_TAG:-mrprof}.log" 2>&1; rc=$?
      cd "$GRAFT_REPO_ROOT"; tail -5 gpurun_out/${PROF_TAG:-mrprof}.log; echo "mrprof rc=$rc"; ok $rc || exit $rc
      python3 scripts/step_census.py $(find gpurun_out/${PROF_TAG:-mrprof} -name "*.db" | head -1) --last $((${MR_STEPS:-12} - 4)) --top 90 ${CENSUS_DETAIL:+--detail "$CENSUS_DETAIL"} > gpurun_out/${PROF_TAG:-mrprof}_census.txt 2>&1
      find gpurun_out/${PROF_TAG:-mrprof} -name "*.db" -delete ;;
    kbench)
      timeout -k 10 300 python scripts/kbench.py ${KBENCH_ARGS:-} > gpurun_out/kbench.log 2>&1; rc=$?
      cat gpurun_out/kbench.log | tail -40; echo "kbench rc=$rc"; ok $rc || exit $rc ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${PROF_TAG:-prof}" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps ${P_STEPS:-10} --warmup 3 --no-maskrcnn ${PROF_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/${PROF_TAG:-prof}.log" 2>&1; rc=$?
      cd "$GRAFT_REPO_ROOT"; tail -5 gpurun_out/${PROF_TAG:-prof}.log; echo "prof rc=$rc"; ok $rc || exit $rc
      python3 scripts/prof_summary.py $(find gpurun_out/${PROF_TAG:-prof} -name "*.db" | head -1) $((${P_STEPS:-10} + 6)) 60 > gpurun_out/${PROF_TAG:-prof}_summary.txt 2>&1
      [ -n "$CENSUS_MARKER" ] && python3 scripts/step_census.py $(find gpurun_out/${PROF_TAG:-prof} -name "*.db" | head -1) --marker "$CENSUS_MARKER" --last $((${P_STEPS:-10} - 2)) --top 60 ${CENSUS_DETAIL:+--detail "$CENSUS_DETAIL"} > gpurun_out/${PROF_TAG:-prof}_census.txt 2>&1
      find gpurun_out/${PROF_TAG:-prof} -name "*.db" -delete ;;
    rprof)
      # kernel census of any python script: RPROF_CMD="script.py args", RPROF_STEPS (divisor), RPROF_TAG
      cd /tmp && export TMPDIR=/tmp && export PYTHONPATH="$GRAFT_REPO_ROOT${PYTHONPATH:+:$PYTHONPATH}"
      timeout -k 10 ${T_PROF:-400} rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${RPROF_TAG:-rprof}" -o run -- python3 $GRAFT_REPO_ROOT/$RPROF_CMD > "$GRAFT_REPO_ROOT/gpurun_out/${RPROF_TAG:-rprof}.log" 2>&1; rc=$?
      cd "$GRAFT_REPO_ROOT"; tail -5 gpurun_out/${RPROF_TAG:-rprof}.log; echo "rprof rc=$rc"; ok $rc || exit $rc
      python3 scripts/prof_summary.py $(find gpurun_out/${RPROF_TAG:-rprof} -name "*.db" | head -1) ${RPROF_STEPS:-10} 60 > gpurun_out/${RPROF_TAG:-rprof}_summary.txt 2>&1
      [ -n "$CENSUS_MARKER" ] && python3 scripts/step_census.py $(find gpurun_out/${RPROF_TAG:-rprof} -name "*.db" | head -1) --marker "$CENSUS_MARKER" --last ${CENSUS_LAST:-10} --top 60 ${CENSUS_DETAIL:+--detail "$CENSUS_DETAIL"} > gpurun_out/${RPROF_TAG:-rprof}_census.txt 2>&1
      find gpurun_out/${RPROF_TAG:-rprof} -name "*.db" -delete ;;
    gemm)
      timeout -k 10 ${T_GEMM:-400} python scripts/gemm_nt_bench.py > gpurun_out/${GEMM_TAG:-gemm}.txt 2>&1; rc=$?
      tail -20 gpurun_out/${GEMM_TAG:-gemm}.txt; echo "gemm rc=$rc"; ok $rc || exit $rc ;;
    cmd)
      # one arbitrary python command: CMD="scripts/x.py args" (output to gpurun_out/$CMD_TAG.txt)
      timeout -k 10 ${T_CMD:-300} python $CMD > gpurun_out/${CMD_TAG:-cmd}.txt 2>&1; rc=$?
      tail -${CMD_TAIL:-20} gpurun_out/${CMD_TAG:-cmd}.txt; echo "cmd rc=$rc"; ok $rc || exit $rc ;;
    cmds)
      # several python commands: CMDS="a.py args|b.py args", outputs gpurun_out/${CMDS_TAG}_<i>.txt
      IFS='|' read -ra _CMDS <<< "$CMDS"; i=0
      for c in "${_CMDS[@]}"; do
        i=$((i+1))
        timeout -k 10 ${T_CMD:-300} python $c > gpurun_out/${CMDS_TAG:-cmds}_$i.txt 2>&1; rc=$?
        tail -${CMD_TAIL:-20} gpurun_out/${CMDS_TAG:-cmds}_$i.txt; echo "cmds[$i] rc=$rc"; ok $rc || exit $rc
      done ;;
    cmd2)
      timeout -k 10 ${T_CMD2:-300} python $CMD2 > gpurun_out/${CMD2_TAG:-cmd2}.txt 2>&1; rc=$?
      tail -${CMD_TAIL:-20} gpurun_out/${CMD2_TAG:-cmd2}.txt; echo "cmd2 rc=$rc"; ok $rc || exit $rc ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp
      G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
      G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM"
      G3="SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE GRBM_COUNT"
      i=0
      for G in "$G1" "$G2" "$G3"; do
        i=$((i+1))
        timeout -s KILL ${T_PMC:-120} rocprofv3 --pmc $G --kernel-include-regex "${PMC_REGEX:-.*}" -d "$GRAFT_REPO_ROOT/gpurun_out/${PMC_TAG:-pmc}$i" -o run -- python3 $GRAFT_REPO_ROOT/$PMC_CMD > "$GRAFT_REPO_ROOT/gpurun_out/${PMC_TAG:-pmc}$i.log" 2>&1; rc=$?
        echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { cd "$GRAFT_REPO_ROOT"; tail -5 gpurun_out/${PMC_TAG:-pmc}$i.log; exit $rc; }
      done
      cd "$GRAFT_REPO_ROOT"
      python3 scripts/rocpd_pmc.py $(find gpurun_out/${PMC_TAG:-pmc}[123] -name "*.db") > gpurun_out/${PMC_TAG:-pmc}_summary.txt 2>&1
      find gpurun_out/${PMC_TAG:-pmc}[123] -name "*.db" -delete ;;
  esac
done
echo ALLDONE
