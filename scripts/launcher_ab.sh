#!/bin/bash
# Same-box A/B of the Ray-Lightning ResNet-50 launcher (BASELINE config 5, hipGraph step) on an
# environment switch: AB_VAR=<NAME> runs alternating arms NAME=1 / NAME=0, ROUNDS rounds
# (default 2), STEPS steps per run (default 40); prints samples/s per run.
#   gpurun -- 'AB_VAR=MXTRAIN_X bash scripts/launcher_ab.sh'
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in 1 0; do
    env "$AB_VAR=$arm" timeout -k 10 200 python mxtrain/workloads/ray/train_resnet50.py --steps-per-epoch ${STEPS:-40} \
      --storage-path /tmp/launcher_ab_$arm$r > gpurun_out/launcher_ab_${arm}_$r.log 2>&1 || exit 1
    echo "$AB_VAR=$arm round $r: $(grep -o '"samples_per_sec": [0-9.]*' gpurun_out/launcher_ab_${arm}_$r.log)"
  done
done
