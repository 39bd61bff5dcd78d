"""Probe: do module launches (the path MIOpen's solvers use: hipExtModuleLaunchKernel with
global work sizes, and hipModuleLaunchKernel with grid sizes) replay correctly from a
captured hipGraph on this HIP runtime?

A tiny code object (one kernel that counts its workgroups and stamps its block index)
is loaded through torch's own libamdhip64 with ctypes, launched eagerly and under
torch.cuda.graph capture, and the replay's workgroup count and output are compared with
the eager launch.  Every write is bounds-checked, so a wrong grid cannot fault.

    python scripts/probe_graph_launch.py        (GPU box)
"""
import ctypes
import os
import subprocess
import sys
import tempfile

KERNEL = r"""
#include <hip/hip_runtime.h>
extern "C" __global__ void probe(int* out, int* count, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (threadIdx.x == 0) atomicAdd(count, 1);
  if (i < n) out[i] = blockIdx.x + 1;
}
// one count per launched work-item: a non-uniform dispatch (global size not a multiple of
// the workgroup size, as OpenCL-style MIOpen kernels are launched) launches fewer items
// in its last workgroup; a replay that rounds the grid up counts more
extern "C" __global__ void probe_items(int* out, int* count, int n_alloc) {
  int i = blockIdx.x * 256 + threadIdx.x;
  atomicAdd(count, 1);
  if (i < n_alloc) out[i] = blockIdx.x + 1;
}
// private (scratch) segment: a dynamically indexed local array the compiler cannot keep
// in registers
extern "C" __global__ void probe_scratch(int* out, int* count, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  volatile int tmp[384];
  for (int k = 0; k < 384; ++k) tmp[k] = k * 3 + i;
  int acc = 0;
  for (int k = 0; k < 384; k += 7) acc += tmp[(k * 13 + i) % 384];
  if (threadIdx.x == 0) atomicAdd(count, 1);
  if (i < n) out[i] = acc;
}
"""


def build_hsaco(extra=()) -> str:
    d = tempfile.mkdtemp()
    src, out = os.path.join(d, "probe.hip"), os.path.join(d, "probe.hsaco")
    with open(src, "w") as f:
        f.write(KERNEL)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--genco", "--offload-arch=gfx950", "-O2", *extra, src, "-o", out])
    return out


def main() -> int:
    import torch
    hsaco = build_hsaco()
    hip = None
    for name in ("libamdhip64.so",):
        p = os.path.join(os.path.dirname(torch.__file__), "lib", name)
        hip = ctypes.CDLL(p if os.path.exists(p) else name)
    torch.zeros(1, device="cuda")
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod), hsaco.encode()) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"probe") == 0
    n_blocks, bs = 64, 256
    n = n_blocks * bs
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")

    a_out, a_cnt, a_n = ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cnt.data_ptr()), ctypes.c_int(n)
    args = (ctypes.c_void_p * 3)(ctypes.cast(ctypes.byref(a_out), ctypes.c_void_p),
                                 ctypes.cast(ctypes.byref(a_cnt), ctypes.c_void_p),
                                 ctypes.cast(ctypes.byref(a_n), ctypes.c_void_p))

    def ext(stream):
        r = hip.hipExtModuleLaunchKernel(fn, ctypes.c_uint32(n), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_uint32(bs), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_size_t(0), ctypes.c_void_p(stream), args, None, None, None,
                                         ctypes.c_uint32(0))
        assert r == 0, r

    def mod_launch(stream):
        r = hip.hipModuleLaunchKernel(fn, ctypes.c_uint32(n_blocks), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                      ctypes.c_uint32(bs), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                      ctypes.c_uint32(0), ctypes.c_void_p(stream), args, None)
        assert r == 0, r

    # MIOpen passes its arguments through ``extra`` (HIP_LAUNCH_PARAM_BUFFER_POINTER to a
    # packed host buffer on its stack) instead of kernelParams.  The buffer is rewritten
    # after capture to point at a decoy output: if the graph kept the pointer instead of
    # copying the bytes, the replay writes the decoy (valid memory, so no fault either way).
    decoy = torch.zeros(n, dtype=torch.int32, device="cuda")
    dcnt = torch.zeros(1, dtype=torch.int32, device="cuda")

    class Args(ctypes.Structure):
        _fields_ = [("out", ctypes.c_void_p), ("count", ctypes.c_void_p), ("n", ctypes.c_int), ("pad", ctypes.c_int)]

    buf = Args(out.data_ptr(), cnt.data_ptr(), n, 0)
    size = ctypes.c_size_t(ctypes.sizeof(Args))
    extra = (ctypes.c_void_p * 5)(ctypes.c_void_p(1), ctypes.cast(ctypes.byref(buf), ctypes.c_void_p),
                                  ctypes.c_void_p(2), ctypes.cast(ctypes.byref(size), ctypes.c_void_p),
                                  ctypes.c_void_p(3))

    def ext_extra(stream):
        buf.out, buf.count = out.data_ptr(), cnt.data_ptr()
        r = hip.hipExtModuleLaunchKernel(fn, ctypes.c_uint32(n), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_uint32(bs), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_size_t(0), ctypes.c_void_p(stream), None, extra, None, None,
                                         ctypes.c_uint32(0))
        assert r == 0, r

    def after_capture():
        buf.out, buf.count = decoy.data_ptr(), dcnt.data_ptr()

    fn_items, fn_scr = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipModuleGetFunction(ctypes.byref(fn_items), mod, b"probe_items") == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn_scr), mod, b"probe_scratch") == 0
    n_items = n - 24          # last workgroup partial: 232 of 256 items

    def ext_nonuniform(stream):
        r = hip.hipExtModuleLaunchKernel(fn_items, ctypes.c_uint32(n_items), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_uint32(bs), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_size_t(0), ctypes.c_void_p(stream), args, None, None, None,
                                         ctypes.c_uint32(0))
        if r != 0:
            hip.hipGetLastError()   # clear the error so later calls do not report it
            raise RuntimeError(f"hipExtModuleLaunchKernel rejected the non-uniform launch: error {r}")

    def ext_scratch(stream):
        r = hip.hipExtModuleLaunchKernel(fn_scr, ctypes.c_uint32(n), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_uint32(bs), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_size_t(0), ctypes.c_void_p(stream), args, None, None, None,
                                         ctypes.c_uint32(0))
        assert r == 0, r

    # the same counting kernel from a code object built WITHOUT the uniform-workgroup
    # assumption (OpenCL-style, like MIOpen's runtime-compiled utility kernels): the runtime
    # accepts a non-uniform global size for it, and the hardware runs a partial last group
    mod2, fn_nu = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod2), build_hsaco(("-fno-offload-uniform-block",)).encode()) == 0
    assert hip.hipModuleGetFunction(ctypes.byref(fn_nu), mod2, b"probe_items") == 0

    def ext_nonuniform_ok(stream):
        r = hip.hipExtModuleLaunchKernel(fn_nu, ctypes.c_uint32(n_items), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_uint32(bs), ctypes.c_uint32(1), ctypes.c_uint32(1),
                                         ctypes.c_size_t(0), ctypes.c_void_p(stream), args, None, None, None,
                                         ctypes.c_uint32(0))
        if r != 0:
            hip.hipGetLastError()
            raise RuntimeError(f"hipExtModuleLaunchKernel rejected the non-uniform launch: error {r}")

    ok = True
    for name, launch, want_count in (("hipExtModuleLaunchKernel non-uniform (items)", ext_nonuniform, n_items),
                                     ("hipExtModuleLaunchKernel non-uniform, no-uniform-block code object (items)",
                                      ext_nonuniform_ok, n_items),
                                     ("hipExtModuleLaunchKernel scratch kernel", ext_scratch, n_blocks)):
        out.zero_(); cnt.zero_()
        try:
            launch(torch.cuda.current_stream().cuda_stream)
        except RuntimeError as e:
            print(f"[probe] {name}: {e}", flush=True)
            continue
        torch.cuda.synchronize()
        eager = (int(cnt.item()), out.clone())
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            launch(s.cuda_stream)
        out.zero_(); cnt.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        same = torch.equal(out, eager[1])
        print(f"[probe] {name}: eager count={eager[0]} (expect {want_count}) replay count={int(cnt.item())} "
              f"output_equal={same} packet_capture={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', 'default')}",
              flush=True)
        ok &= eager[0] == want_count and int(cnt.item()) == want_count and same
    for name, launch in (("hipExtModuleLaunchKernel", ext), ("hipModuleLaunchKernel", mod_launch),
                         ("hipExtModuleLaunchKernel+extra", ext_extra)):
        out.zero_(); cnt.zero_()
        launch(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        eager = (int(cnt.item()), out.clone())
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            launch(s.cuda_stream)
            if launch is ext_extra:   # still inside the capture: MIOpen's stack frame is gone by now
                after_capture()
        out.zero_(); cnt.zero_(); decoy.zero_(); dcnt.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        same = torch.equal(out, eager[1])
        print(f"[probe] {name}: eager workgroups={eager[0]} replay workgroups={int(cnt.item())} "
              f"output_equal={same} decoy_workgroups={int(dcnt.item())}", flush=True)
        ok &= eager[0] == n_blocks and int(cnt.item()) == n_blocks and same
    print("[probe] OK" if ok else "[probe] MISMATCH", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
