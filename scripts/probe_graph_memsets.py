"""Probe: memset nodes of many sizes / alignments inside a graph replayed with the HIP
runtime's packet capture: each round is [D2D copy] -> [memset region to 0] -> [kernel adds
1 to every int of the region] -> [kernel snapshots the region's checksum]; the replay's
checksums must equal the eager ones.  Sizes span 4 B .. 64 MiB, destinations at offsets
0 / 4 / 8 / 2 bytes, byte counts that are not multiples of 4 (the runtime's unaligned
fill path).  No kernel indexes memory with data, so a misordered node cannot fault.

    python scripts/probe_graph_memsets.py        (GPU box)
"""
import ctypes
import os
import sys

SIZES = [4, 12, 100, 1022, 4096, 65536 + 4, 1 << 20, (1 << 22) + 6, 16 << 20, 64 << 20]
OFFSETS = [0, 4, 8, 2]


def main() -> int:
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--memset-kernels", action="store_true",
                    help="replace the captured memset nodes by fill-kernel nodes (mxtrain.runtime.graphfix)")
    a = ap.parse_args()
    import torch
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    dev = "cuda"
    maxb = max(SIZES) + 64
    buf = torch.zeros(maxb // 4 + 16, dtype=torch.int32, device=dev)
    src = torch.arange(4096, dtype=torch.int32, device=dev)
    dst = torch.zeros(4096, dtype=torch.int32, device=dev)
    cases = [(s, o) for s in SIZES for o in OFFSETS]
    sums = torch.zeros(len(cases), dtype=torch.int64, device=dev)
    base = buf.data_ptr()

    def body(stream):
        with torch.cuda.stream(stream):
            for i, (size, off) in enumerate(cases):
                assert hip.hipMemcpyAsync(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                          ctypes.c_size_t(4 * 4096), 3, ctypes.c_void_p(stream.cuda_stream)) == 0
                buf.fill_(7)                                   # a known non-zero background
                assert hip.hipMemsetAsync(ctypes.c_void_p(base + off), 0, ctypes.c_size_t(size),
                                          ctypes.c_void_p(stream.cuda_stream)) == 0
                buf.add_(1)
                sums[i] = buf.to(torch.int64).sum() + dst[5].to(torch.int64)

    s = torch.cuda.Stream()
    body(s)
    torch.cuda.synchronize()
    eager = sums.clone()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g, stream=s):
        body(s)
    if a.memset_kernels:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from mxtrain.runtime import graphfix
        print(f"[memsets] replaced {graphfix.memsets_to_kernels(g)} memset nodes; census {graphfix.census(g)}",
              flush=True)
    g.instantiate()
    bad_total = 0
    for rep in range(3):
        sums.fill_(-1)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        bad = (sums != eager).nonzero().flatten().tolist()
        bad_total += len(bad)
        print(f"[memsets] replay {rep}: {len(cases) - len(bad)}/{len(cases)} cases exact"
              + (f"; wrong (bytes, offset): {[cases[i] for i in bad[:10]]}" if bad else "")
              + f" packet_capture={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE', 'default')}"
              f" memset_kernels={a.memset_kernels}", flush=True)
    print("[memsets] OK" if bad_total == 0 else "[memsets] MISMATCH", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
