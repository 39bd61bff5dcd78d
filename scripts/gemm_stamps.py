#!/usr/bin/env python3
"""Where does a gemm_nt tile spend its time?  Per-tile s_memtime stamps (diagnostic build of
the forward kernel) at tile start / first K-step data landed / main loop end / epilogue end,
for a few shapes; prints start skew, phase medians (cycles) and the in-kernel clock."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import _lib  # noqa: E402


def run(M, N, K, variant, reps=30):
    dev = "cuda"
    a = (torch.randn(M, K, device=dev)).to(torch.bfloat16)
    b = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    bm, bn = {0: (256, 256), 3: (128, 128), 6: (256, 256)}[variant]
    tiles = (M // bm) * (N // bn)
    st = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
    for _ in range(reps):   # back-to-back launches (clock settles under load)
        _lib.call("mx_gemm_nt_stamps", a.data_ptr(), b.data_ptr(), c.data_ptr(), st.data_ptr(), K, K, N, M, N, K,
                  variant, _lib.stream())
    torch.cuda.synchronize()
    s = st.view(tiles, 8).cpu().tolist()
    t0 = min(r[0] for r in s)
    start = [r[0] - t0 for r in s]
    first = [r[2] - r[0] for r in s]
    loop = [r[4] - r[2] for r in s]
    epi = [r[6] - r[4] for r in s]
    total = max(r[6] for r in s) - t0
    rt = max(r[7] for r in s) - min(r[1] for r in s)   # 100 MHz ticks
    clk = [(r[6] - r[0]) / max(r[7] - r[1], 1) * 100 for r in s]
    med = statistics.median
    flop = 2.0 * M * N * K
    print(f"M{M} N{N} K{K} v{variant} tiles={tiles}: kernel {total} cyc = {rt / 100:.1f} us, clock ~{med(clk):.0f} MHz, "
          f"{flop / (rt / 1e8) / 1e15:.3f} PF/s")
    print(f"   start skew med {med(start)} max {max(start)} | first-data med {med(first)} max {max(first)} | "
          f"loop med {med(loop)} min {min(loop)} max {max(loop)} ({med(loop) / (K // (32 if variant == 0 else 64)):.0f}/step) "
          f"| epilogue med {med(epi)} max {max(epi)}", flush=True)


def main():
    for (M, N, K) in [(4096, 4096, 1024), (4096, 1024, 4096), (1024, 4096, 1024), (4096, 4096, 4096)]:
        for v in (6, 0, 3):
            bm, bn = {0: (256, 256), 3: (128, 128), 6: (256, 256)}[v]
            if M % bm == 0 and N % bn == 0:
                run(M, N, K, v)


if __name__ == "__main__":
    main()
