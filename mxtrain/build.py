"""Build the mxtrain native libraries in-tree for gfx950.

* ``mxtrain/lib/libmxkernels.so`` -- every ``csrc/*.hip`` (and ``csrc/comm/*.hip``)
  compiled with ``hipcc --offload-arch=gfx950`` and linked into one shared object with
  a plain C ABI (bound from Python with ctypes, see ``mxtrain/ops/_lib.py``).
* ``mxtrain/lib/libmxruntime.so`` -- host-only C++ runtime pieces (indexed-dataset
  sample-index builder, ...), compiled with g++.

Objects are rebuilt only when their source (or any header) is newer.  Usage::

    python -m mxtrain.build            # build everything
    python -m mxtrain.build --clean
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(ROOT, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("MXTRAIN_ARCH", "gfx950")

KERNEL_LIB = os.path.join(LIBDIR, "libmxkernels.so")
RUNTIME_LIB = os.path.join(LIBDIR, "libmxruntime.so")

HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-mcode-object-version=5",
    "-fvisibility=hidden",
    "-ffp-contract=fast",
    "-Wno-unused-result",
]


def _newer(src_list, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def hip_sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "comm", "*.hip")))


def headers():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def build_kernels(jobs: int = 8, verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = hip_sources()
    hdrs = headers()
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(OBJDIR, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer([s] + hdrs, o):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        cmd = [HIPCC] + HIP_FLAGS + ["-I", CSRC, "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
        return o

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(compile_one, todo))
    if _newer(objs, KERNEL_LIB) or todo:
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", KERNEL_LIB] + objs)
    return KERNEL_LIB


def build_runtime(verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return ""
    os.makedirs(LIBDIR, exist_ok=True)
    if _newer(srcs + headers(), RUNTIME_LIB):
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-pthread",
               "-I", CSRC, "-o", RUNTIME_LIB] + srcs
        if verbose:
            print(" ".join(cmd), flush=True)
        _run(cmd)
    return RUNTIME_LIB


def build_all(jobs: int = 8, verbose: bool = False):
    k = build_kernels(jobs, verbose)
    r = build_runtime(verbose)
    return k, r


def clean():
    if os.path.isdir(LIBDIR):
        shutil.rmtree(LIBDIR)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    if a.clean:
        clean()
    k, r = build_all(a.jobs, a.verbose)
    print(f"built {k}" + (f" and {r}" if r else ""))


if __name__ == "__main__":
    sys.exit(main())
