cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
  for arm in 1 0; do
    MXTRAIN_BN_CASTS=$arm timeout -k 10 200 python mxtrain/workloads/ray/train_resnet50.py --steps-per-epoch 40 --storage-path /tmp/rn_ab_$arm$r > gpurun_out/rn_ab_${arm}_$r.log 2>&1 || exit 1
    echo "arm casts=$arm round $r: $(grep -o '"samples_per_sec": [0-9.]*' gpurun_out/rn_ab_${arm}_$r.log)"
  done
done
