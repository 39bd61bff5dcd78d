"""Probe: node kinds of a captured Mask R-CNN step besides plain kernels -- do they keep
their semantics under hipGraph packet capture?

  * memset -> kernel: hipMemsetAsync of an accumulator, then a kernel that adds into it
    (MIOpen's weight-gradient solvers zero a workspace that way before accumulating),
    repeated N times in one graph; every round's result is copied out by a third kernel.
  * memcpy -> kernel: hipMemcpyAsync device-to-device, then a kernel that reads the copy.
  * host-to-device memcpy from PAGEABLE host memory (and from pinned memory) captured into
    the graph, the host buffer rewritten after the capture: does the replay copy the bytes
    the buffer held at capture time (a snapshot) or what it holds at replay time?  (A
    library that stages kernel arguments through a host vector that dies after the call
    would replay garbage in the second case.)
  * dynamic LDS: a module kernel launched with sharedMemBytes (extern __shared__), writing
    and reading back its slots at the top of a 48 KiB dynamic segment -- a packet built
    without the dynamic size would drop those LDS writes (no fault, wrong values).

Every kernel indexes only with its own thread ids into buffers sized for them, so a
broken node shows up as a wrong value, never as a fault.

    python scripts/probe_graph_nodes.py [--rounds 300]      (GPU box)
"""
import argparse
import ctypes
import os
import subprocess
import sys
import tempfile

KERNEL = r"""
#include <hip/hip_runtime.h>
extern "C" __global__ void add_one(int* acc, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) acc[i] += 1;
}
extern "C" __global__ void snap(const int* acc, int* out, int n, int round) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[(size_t)round * n + i] = acc[i];
}
extern "C" __global__ void dyn_lds(int* out, int words) {
  extern __shared__ int sm[];
  const int t = threadIdx.x;
  // fill the whole dynamic segment, then read back from its top quarter
  for (int i = t; i < words; i += blockDim.x) sm[i] = i * 3 + blockIdx.x;
  __syncthreads();
  const int j = words - 1 - t;
  out[blockIdx.x * blockDim.x + t] = j >= 0 ? sm[j] : -7;
}
"""


def build_hsaco() -> str:
    d = tempfile.mkdtemp()
    src, out = os.path.join(d, "nodes.hip"), os.path.join(d, "nodes.hsaco")
    with open(src, "w") as f:
        f.write(KERNEL)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--genco", "--offload-arch=gfx950", "-O2", src, "-o", out])
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=300)
    ap.add_argument("--no-h2d", action="store_true", help="leave the host-to-device copies out of the graph")
    ap.add_argument("--memset-kernels", action="store_true",
                    help="replace the captured memset nodes by fill-kernel nodes (mxtrain.runtime.graphfix)")
    a = ap.parse_args()
    import torch
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    torch.zeros(1, device="cuda")
    mod = ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod), build_hsaco().encode()) == 0
    fns = {}
    for name in ("add_one", "snap", "dyn_lds"):
        f = ctypes.c_void_p()
        assert hip.hipModuleGetFunction(ctypes.byref(f), mod, name.encode()) == 0
        fns[name] = f
    keep = []

    def launch(name, grid, block, stream, *vals, shmem=0):
        cargs = list(vals)   # ctypes values; kept alive until the end (graph capture)
        ptrs = (ctypes.c_void_p * len(cargs))(*[ctypes.cast(ctypes.byref(c), ctypes.c_void_p) for c in cargs])
        keep.append((cargs, ptrs))
        r = hip.hipModuleLaunchKernel(fns[name], grid, 1, 1, block, 1, 1, shmem, ctypes.c_void_p(stream), ptrs, None)
        assert r == 0, (name, r)

    R, n = a.rounds, 4096
    acc = torch.zeros(n, dtype=torch.int32, device="cuda")
    src = torch.arange(n, dtype=torch.int32, device="cuda")
    cpy = torch.zeros(n, dtype=torch.int32, device="cuda")
    out_ms = torch.zeros(R * n, dtype=torch.int32, device="cuda")
    out_cp = torch.zeros(R * n, dtype=torch.int32, device="cuda")
    words, blocks, bs = 48 * 1024 // 4, 64, 256
    out_lds = torch.zeros(blocks * bs, dtype=torch.int32, device="cuda")

    h_page = (ctypes.c_int * n)(*range(100, 100 + n))          # pageable host memory
    h_pin_t = torch.arange(200, 200 + n, dtype=torch.int32).pin_memory()
    d_page = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_pin = torch.zeros(n, dtype=torch.int32, device="cuda")

    def h2d(stream):
        assert hip.hipMemcpyAsync(ctypes.c_void_p(d_page.data_ptr()), ctypes.cast(h_page, ctypes.c_void_p),
                                  ctypes.c_size_t(4 * n), 1, ctypes.c_void_p(stream)) == 0
        assert hip.hipMemcpyAsync(ctypes.c_void_p(d_pin.data_ptr()), ctypes.c_void_p(h_pin_t.data_ptr()),
                                  ctypes.c_size_t(4 * n), 1, ctypes.c_void_p(stream)) == 0

    def body(stream):
        if not a.no_h2d:
            h2d(stream)
        for rd in range(R):
            # memset -> accumulate (x2) -> snapshot: expect 2 everywhere
            assert hip.hipMemsetAsync(ctypes.c_void_p(acc.data_ptr()), 0, ctypes.c_size_t(4 * n), ctypes.c_void_p(stream)) == 0
            launch("add_one", n // 256, 256, stream, ctypes.c_void_p(acc.data_ptr()), ctypes.c_int(n))
            launch("add_one", n // 256, 256, stream, ctypes.c_void_p(acc.data_ptr()), ctypes.c_int(n))
            launch("snap", n // 256, 256, stream, ctypes.c_void_p(acc.data_ptr()), ctypes.c_void_p(out_ms.data_ptr()),
                   ctypes.c_int(n), ctypes.c_int(rd))
            # memcpy src -> cpy, snapshot the copy, then clobber the copy
            assert hip.hipMemcpyAsync(ctypes.c_void_p(cpy.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                      ctypes.c_size_t(4 * n), 3, ctypes.c_void_p(stream)) == 0
            launch("snap", n // 256, 256, stream, ctypes.c_void_p(cpy.data_ptr()), ctypes.c_void_p(out_cp.data_ptr()),
                   ctypes.c_int(n), ctypes.c_int(rd))
            assert hip.hipMemsetAsync(ctypes.c_void_p(cpy.data_ptr()), 0, ctypes.c_size_t(4 * n), ctypes.c_void_p(stream)) == 0
        launch("dyn_lds", blocks, bs, stream, ctypes.c_void_p(out_lds.data_ptr()), ctypes.c_int(words), shmem=4 * words)

    cur = torch.cuda.current_stream().cuda_stream
    body(cur)
    torch.cuda.synchronize()
    ref = (out_ms.clone(), out_cp.clone(), out_lds.clone())
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=s):
        body(s.cuda_stream)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from mxtrain.runtime import graphfix
    print(f"[nodes] census {graphfix.census(g)}", flush=True)
    if a.memset_kernels:
        print(f"[nodes] replaced {graphfix.memsets_to_kernels(g)} memset nodes by fill kernels", flush=True)
    g.instantiate()
    for t in (out_ms, out_cp, out_lds, acc, cpy, d_page, d_pin):
        t.fill_(-1)
    for i in range(n):                      # rewrite both host sources after the capture
        h_page[i] = -5
    h_pin_t.fill_(-6)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    pc = os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "default")
    for name, dst, snap_v, live_v in (("H2D pageable", d_page, 100, -5), ("H2D pinned", d_pin, 200, -6)):
        snap = torch.equal(dst.cpu(), torch.arange(snap_v, snap_v + n, dtype=torch.int32))
        live = bool((dst == live_v).all().item())
        print(f"[nodes] {name} source rewritten after capture: replay copied "
              f"{'the capture-time bytes' if snap else 'the replay-time bytes' if live else 'neither (garbage)'} "
              f"packet_capture={pc}", flush=True)
    ok = True
    exp_ms = torch.full_like(out_ms, 2)
    exp_cp = src.repeat(R)
    exp_lds = torch.tensor([(words - 1 - t) * 3 + b for b in range(blocks) for t in range(bs)], dtype=torch.int32,
                           device="cuda")
    for name, got, eager, exp in (("memset->kernel", out_ms, ref[0], exp_ms), ("memcpy->kernel", out_cp, ref[1], exp_cp),
                                  ("dynamic LDS 48 KiB", out_lds, ref[2], exp_lds)):
        e_ok, r_ok = torch.equal(eager, exp), torch.equal(got, exp)
        bad = int((got != exp).sum().item())
        detail = ""
        if bad and got.numel() % n == 0:
            rows = (got != exp).view(-1, n).any(1).nonzero().flatten().tolist()
            vals = [sorted(set(got.view(-1, n)[r].tolist()))[:4] for r in rows[:4]]
            detail = f" rounds {rows[:8]} values {vals}"
        print(f"[nodes] {name}: eager_ok={e_ok} replay_ok={r_ok} (wrong {bad}){detail} packet_capture={pc} "
              f"h2d_nodes={not a.no_h2d} memset_kernels={a.memset_kernels}", flush=True)
        ok &= e_ok and r_ok
    print("[nodes] OK" if ok else "[nodes] MISMATCH", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
