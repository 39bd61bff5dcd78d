"""Probe: do LARGE by-value kernel arguments survive hipGraph packet capture, alone and
across thousands of captured nodes?

The composable-kernel convolutions MIOpen's find-db picks for the Mask R-CNN step
(kernel_grouped_conv_fwd_xdl_cshuffle_v3, kernel_batched_gemm_xdlops_bwd_weight, ...) take
their tensor descriptors by value: kernarg segments of hundreds of bytes to kilobytes, far
larger than the module kernels scripts/probe_graph_launch.py covers.  With packet capture
the runtime copies every node's arguments into a kernarg pool at instantiation; this probe
captures N launches of a kernel whose argument is a KB-sized struct (node index at its
start, payload words up to its very end), replays the graph, and checks every node's row
(payload checksum, last and first word) against the eager launch.  The argument holds no
pointer: rows land in a module global, bounds-checked by the node index, so a truncated
or stale argument shows up as a wrong row, never as a fault.

    python scripts/probe_graph_bigargs.py [--nodes 2000]        (GPU box)
"""
import argparse
import ctypes
import os
import subprocess
import sys
import tempfile

WORDS = {"small": 8, "1k": 248, "2k": 504, "4k": 1016}

KERNEL = r"""
#include <hip/hip_runtime.h>
// no pointer in the argument: the rows land in a module global, so even a garbage
// argument can only write inside it (node index bounds-checked)
#define MAXN 8192
__device__ int g_out[3 * MAXN];
template <int W> struct Big { long long tag; int node; int n_nodes; int v[W]; };
template <int W> __device__ void body(const Big<W>& b) {
  // node's row: [checksum of v, last word, first word]; only the first lane writes
  if (threadIdx.x != 0 || blockIdx.x != 0 || b.node < 0 || b.node >= b.n_nodes || b.n_nodes > MAXN) return;
  int s = 0;
  for (int i = 0; i < W; ++i) s = s * 31 + b.v[i];
  g_out[3 * b.node] = s;
  g_out[3 * b.node + 1] = b.v[W - 1];
  g_out[3 * b.node + 2] = b.v[0];
}
#define K(NAME, W) extern "C" __global__ void NAME(Big<W> b) { body<W>(b); }
K(big_small, 8)
K(big_1k, 248)
K(big_2k, 504)
K(big_4k, 1016)
"""


def build_hsaco() -> str:
    d = tempfile.mkdtemp()
    src, out = os.path.join(d, "bigargs.hip"), os.path.join(d, "bigargs.hsaco")
    with open(src, "w") as f:
        f.write(KERNEL)
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--genco", "--offload-arch=gfx950", "-O2", src, "-o", out])
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=2000)
    a = ap.parse_args()
    import torch
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    torch.zeros(1, device="cuda")
    mod = ctypes.c_void_p()
    assert hip.hipModuleLoad(ctypes.byref(mod), build_hsaco().encode()) == 0
    ok = True
    for tag, W in WORDS.items():
        fn = ctypes.c_void_p()
        assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, f"big_{tag}".encode()) == 0

        class Big(ctypes.Structure):
            _fields_ = [("tag", ctypes.c_longlong), ("node", ctypes.c_int), ("n_nodes", ctypes.c_int),
                        ("v", ctypes.c_int * W)]

        n = min(a.nodes, 8192)
        gptr, gsize = ctypes.c_void_p(), ctypes.c_size_t()
        assert hip.hipModuleGetGlobal(ctypes.byref(gptr), ctypes.byref(gsize), mod, b"g_out") == 0

        def fetch():
            host = torch.zeros(3 * 8192, dtype=torch.int32)
            assert hip.hipMemcpy(ctypes.c_void_p(host.data_ptr()), gptr, gsize, 2) == 0   # D2H
            return host[:3 * n].clone()

        def clear():
            assert hip.hipMemset(gptr, 0, gsize) == 0

        args = []
        for i in range(n):
            b = Big(0x5EED, i, n)
            for j in range(W):
                b.v[j] = (i * 7919 + j * 104729) & 0x7FFFFFFF
            args.append(b)

        def launch(stream, i):
            p = (ctypes.c_void_p * 1)(ctypes.cast(ctypes.byref(args[i]), ctypes.c_void_p))
            r = hip.hipModuleLaunchKernel(fn, 1, 1, 1, 64, 1, 1, 0, ctypes.c_void_p(stream), p, None)
            assert r == 0, r

        clear()
        cur = torch.cuda.current_stream().cuda_stream
        for i in range(n):
            launch(cur, i)
        torch.cuda.synchronize()
        eager = fetch()
        s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for i in range(n):
                launch(s.cuda_stream, i)
        # scribble over the host argument structs: a graph that kept pointers to them
        # instead of copying would now read these values
        for b in args:
            for j in range(W):
                b.v[j] = -1
        torch.cuda.synchronize()
        clear()
        g.replay()
        torch.cuda.synchronize()
        out = fetch()
        bad = (out != eager).view(n, 3).any(1).nonzero().flatten().tolist()
        print(f"[bigargs] {tag} ({ctypes.sizeof(Big)} B kernarg) x {n} nodes: eager==replay "
              f"{not bad} (bad nodes {len(bad)}{', first ' + str(bad[:8]) if bad else ''}) "
              f"packet_capture={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', 'default')}", flush=True)
        ok &= not bad
        del g
    print("[bigargs] OK" if ok else "[bigargs] MISMATCH", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
