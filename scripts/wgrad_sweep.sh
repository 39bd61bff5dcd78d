cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && python -m mxtrain.build > gpurun_out/build.log 2>&1 || exit 2
for imgs in 1 4; do for t in 256 512 1024; do for ms in 4 8 16; do
  echo "== IMGS=$imgs TARGET=$t MIN_STEPS=$ms" >> gpurun_out/wgrad_sweep.txt
  IMGS=$imgs WGRAD_ONLY=1 MXTRAIN_WGRAD_TARGET_WGS=$t MXTRAIN_WGRAD_MIN_STEPS=$ms timeout -k 10 120 python scripts/conv_wgrad_bench.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/wgrad_sweep.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done; done; done
echo SWEEPDONE
