#!/usr/bin/env python3
"""Per-kernel PMC counter means (summed over XCD/SE instances per dispatch, averaged over
dispatches) from rocprofv3 SQLite outputs, plus derived rates when their counters are there:
  MFMA pipe busy %  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
  VALU per MFMA     = SQ_INSTS_VALU / SQ_INSTS_MFMA
  wait share        = SQ_WAIT_ANY / SQ_WAVE_CYCLES
    python scripts/rocpd_pmc.py gpurun_out/pmc_attn1/run_results.db [more.db ...]
    python scripts/rocpd_pmc.py --text profiles/r5_s1/pmc_conv_kernels_4img_final.txt  (re-derive)"""
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


SIMDS, XCDS = 1024, 8   # MI355X: 256 CUs x 4 SIMDs, GRBM_GUI_ACTIVE summed over 8 XCDs


def derived(m):
    """Derived rates from per-dispatch counter means ``m`` (name -> value)."""
    out = []
    busy, gui = m.get("SQ_VALU_MFMA_BUSY_CYCLES"), m.get("GRBM_GUI_ACTIVE")
    if busy is not None and gui:
        out.append(("MFMA pipe busy %", 100.0 * busy / (gui / XCDS * SIMDS)))
    if m.get("SQ_INSTS_MFMA"):
        if m.get("SQ_INSTS_VALU") is not None:
            out.append(("VALU per MFMA", m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"]))
        if m.get("SQ_INSTS_LDS") is not None:
            out.append(("LDS per MFMA", m["SQ_INSTS_LDS"] / m["SQ_INSTS_MFMA"]))
    if m.get("SQ_WAVE_CYCLES") and m.get("SQ_WAIT_ANY") is not None:
        out.append(("wait share %", 100.0 * m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]))
    return out


def from_text(path):
    """{kernel: {counter: mean}} parsed back from this script's own text output."""
    res, cur = {}, None
    for line in open(path):
        if not line.strip():
            continue
        if not line.startswith(" "):
            cur = res.setdefault(line.strip(), {})
        elif cur is not None:
            parts = line.split()
            try:
                cur[parts[0]] = float(parts[1])
            except (IndexError, ValueError):
                pass
    return res


def main():
    if sys.argv[1:2] == ["--text"]:
        rows = []
        for k, m in from_text(sys.argv[2]).items():
            rows.append((k, dict(derived(m))))
        print(f"{'kernel':48s} {'MFMA busy %':>12s} {'VALU/MFMA':>10s} {'LDS/MFMA':>9s} {'wait %':>7s}")
        for k, d in sorted(rows, key=lambda r: -r[1].get("MFMA pipe busy %", 0)):
            print(f"{k[:48]:48s} {d.get('MFMA pipe busy %', float('nan')):12.1f} "
                  f"{d.get('VALU per MFMA', float('nan')):10.2f} {d.get('LDS per MFMA', float('nan')):9.2f} "
                  f"{d.get('wait share %', float('nan')):7.1f}")
        return
    agg = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for db in sys.argv[1:]:
        con = sqlite3.connect(db)
        names = {r[0]: r[1] for r in con.execute("select dispatch_id, name from kernels")}
        for disp, cn, val in con.execute("select dispatch_id, counter_name, counter_value from pmc_events"):
            agg[short(names.get(disp, "?"))][cn][disp] += val
    for k, d in agg.items():
        print(k)
        means = {}
        for cn in sorted(d):
            v = list(d[cn].values())
            means[cn] = sum(v) / len(v)
            print(f"   {cn:32s} {means[cn]:16.0f}  (dispatches={len(v)})")
        for name, val in derived(means):
            print(f"   {'= ' + name:32s} {val:16.2f}")


if __name__ == "__main__":
    main()
