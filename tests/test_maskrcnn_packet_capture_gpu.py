"""The Mask R-CNN whole-step hipGraph in the benchmark configuration (training shapes,
torch benchmark mode + MIOpen find with the in-repo find-db) replayed with the HIP
runtime's graph packet capture ON, against the eager step on the same batches.

Before the graph's memset nodes were rewritten into fill-kernel nodes (csrc/graph.hip),
this configuration took an illegal-address fault after a few replays
(profiles/r3_s4/maskrcnn_packet_capture_on_fault.log); the memset probes behind the fix
are in tests/test_graph_gpu.py.  Both runs are child processes: the packet-capture flag
and MIOpen's find-db are read when the runtime / the MIOpen handle initialise."""
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(mode, steps, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "graph_diag.py"), "--mode", mode,
                        "--batch", "1", "--steps", str(steps), "--find-db"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, (mode, r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    losses = [float(m.group(1)) for m in re.finditer(r"\[diag\] mode=\w+ step=\d+ .*total_loss=([-\d.eE+na]+)", r.stdout)]
    assert len(losses) == steps, r.stdout[-2000:]
    return losses, r.stdout


def test_maskrcnn_graph_replays_under_packet_capture_like_eager():
    steps = 12
    eager, _ = _run("eager", steps, {})
    graph, out = _run("graph", steps, {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "1"})
    m = re.search(r"captures=(\d+) replays=(\d+)", out)
    assert m and int(m.group(1)) == 1 and int(m.group(2)) == steps - 1, out[-1000:]
    assert "'memsets_as_kernels': " in out and "'memsets_as_kernels': 0" not in out, out[-1000:]
    print("eager vs graph (packet capture on) total loss per step:",
          [(round(a, 4), round(b, 4)) for a, b in zip(eager, graph)])
    for s, (a, b) in enumerate(zip(eager, graph)):
        assert b == b and abs(b) < 1e4, (s, b)
        # first steps close; later ones may drift through the discrete proposal / RoI sampling
        tol = 0.05 if s < 2 else 0.08   # (measured: <= 4.2 %, profiles/r3_s4/)
        assert abs(a - b) <= tol * abs(a) + 1e-3, (s, a, b, eager, graph)
