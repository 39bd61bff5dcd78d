"""A/B wrapper: scripts/bench_maskrcnn.py with ops.convwg module switches set first.
usage: bench_maskrcnn_ab.py FWD=1 [DGRAD=0 ...] -- <bench_maskrcnn.py args>"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxtrain.ops import convwg  # noqa: E402

i = sys.argv.index("--")
for kv in sys.argv[1:i]:
    k, v = kv.split("=")
    setattr(convwg, k, type(getattr(convwg, k))(int(v)) if isinstance(getattr(convwg, k), (bool, int)) else v)
    print(f"convwg.{k} = {getattr(convwg, k)}", flush=True)
sys.argv = [os.path.join(os.path.dirname(os.path.abspath(__file__)), "bench_maskrcnn.py")] + sys.argv[i + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
