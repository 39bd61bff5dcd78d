# Mask R-CNN: (1) capture-only graph diagnostic with HIP API logging (no replay -> no fault
# risk), (2) MIOpen find-db generation + images/s at 1 and 4 img/GPU
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
mkdir -p gpurun_out/miopen_db
AMD_LOG_LEVEL=3 timeout -k 10 300 python3 scripts/graph_diag.py --mode graph --batch 2 --capture-only > gpurun_out/gdiag.out 2> gpurun_out/gdiag.err; echo "diag rc=$?"
awk '/capture-begin/{f=1} f{print} /capture-end/{f=0}' gpurun_out/gdiag.err | grep -v "hipLaunchKernel\|hipExtModuleLaunchKernel\|hipModuleLaunchKernel\|hipGetLastError\|hipGetDevice\b\|hipSetDevice\|hipPeekAtLastError\|hipStreamIsCapturing\|hipGetDeviceProperties\|hipDeviceGetAttribute\|hipStreamGetCaptureInfo\|ShaderName\|KernelName" | cut -c1-220 | head -400 > gpurun_out/gdiag_capture_api.txt
grep -c . gpurun_out/gdiag.err > gpurun_out/gdiag_lines.txt
rm -f gpurun_out/gdiag.err
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db timeout -k 10 400 python3 scripts/bench_maskrcnn.py --batch 4 --steps 40 --warmup 10 --out gpurun_out/mrcnn.jsonl > gpurun_out/mrcnn_b4.log 2>&1 || exit 1
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db timeout -k 10 400 python3 scripts/bench_maskrcnn.py --batch 1 --steps 60 --warmup 15 --out gpurun_out/mrcnn.jsonl > gpurun_out/mrcnn_b1.log 2>&1
