"""A/B of tests/test_kernels_gpu.py::test_deferred_optimizer_matches_inline with the round-3
fusions switched off one at a time (module switches, no environment variables).
    python scripts/bisect_deferred.py base|nobias|noce|neither"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mode = sys.argv[1]
    import mxtrain.models.gpt as gpt
    import mxtrain.ops.fused as fused
    gpt.FUSED_QKV_BIAS_GRAD = mode not in ("nobias", "neither")
    fused.SINGLE_PASS_CE = mode not in ("noce", "neither")
    rc = pytest.main(["-x", "-q", "-p", "no:cacheprovider", os.path.join(ROOT, "tests", "test_kernels_gpu.py"),
                      "-k", "deferred_optimizer"])
    print(f"[bisect] {mode}: pytest rc={rc}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
