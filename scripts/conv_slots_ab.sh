# A/B of the conv forward / input-gradient LDS ring depth (MXTRAIN_CONV_*_SLOTS) on the
# Mask R-CNN shapes at 4 images (scripts/conv_wgrad_bench.py), one process per setting
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && python -m mxtrain.build > gpurun_out/build.log 2>&1 || exit 2
for ns in 2 3 4 2; do
  echo "== slots $ns" >> gpurun_out/conv_slots_ab.txt
  IMGS=${IMGS:-4} MXTRAIN_CONV_FWD_SLOTS=$ns MXTRAIN_CONV_DGRAD_SLOTS=$ns timeout -k 10 200 python scripts/conv_wgrad_bench.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/conv_slots_ab.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
echo ABDONE
