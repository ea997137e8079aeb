"""Build libdse.so (HIP, gfx950) in-tree with hipcc.

    python -m quantumsimulations_amd.build          # or __graft_entry__.build()

The shared library lands next to this file so it travels with the repo snapshot
to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libdse.so")
SOURCES = ["dse_kernels.hip", "dse_interval.hip", "dse_wht.hip", "dse_small.hip", "dse_dense.hip", "dse_matrix.hip",
           "dse_sytrd.hip", "dse_eig2.hip", "dse_span.hip", "dse_real.hip", "dse_nufft.hip", "dse_runtime.hip",
           "dse_host.cpp"]
HEADERS = ["dse_internal.h", "dse_device.h", "dse_wht.h", "dse_small.h", "dse_dense.h"]
ARCH = os.environ.get("DSE_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: libdse.so needs ROCm's hipcc")


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "dse.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, out: str | None = None) -> str:
    """Compiles libdse.so (or, with ``out``, a variant library of the same ABI at that path).
    Sources compile to objects in parallel (one hipcc per file), then link."""
    target = out or LIB
    if not force and out is None and not needs_build():
        return LIB
    hipcc = _hipcc()
    tmp = target + ".tmp"
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
             "-Wno-unused-function", "-Wno-unused-result", "-I", os.path.join(ROOT, "include")]
    flags += os.environ.get("DSE_EXTRA_FLAGS", "").split()  # e.g. -DDSE_ACC_BLOCK=2 for a variant library
    with tempfile.TemporaryDirectory(prefix="dse_build_") as tdir:
        objs = [os.path.join(tdir, s + ".o") for s in SOURCES]
        cmds = [[hipcc, *flags, "-c", os.path.join(CSRC, s), "-o", o] for s, o in zip(SOURCES, objs)]
        jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
        with ThreadPoolExecutor(jobs) as ex:
            results = list(ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds))
        for c, res in zip(cmds, results):
            if verbose:
                print(" ".join(c), flush=True)
            if res.returncode != 0:
                raise RuntimeError("hipcc failed:\n" + res.stdout + res.stderr)
            if verbose and (res.stdout or res.stderr):
                print(res.stdout + res.stderr)
        link = [hipcc, f"--offload-arch={ARCH}", "-fPIC", "-shared", *objs, "-L", "/opt/rocm/lib",
                "-lrccl", "-lrocsolver", "-lrocblas", "-lrocfft", "-Wl,-rpath,/opt/rocm/lib", "-o", tmp]
        res = subprocess.run(link, capture_output=True, text=True)
        if verbose:
            print(" ".join(link), flush=True)
        if res.returncode != 0:
            raise RuntimeError("hipcc link failed:\n" + res.stdout + res.stderr)
    os.replace(tmp, target)
    return target


if __name__ == "__main__":
    out = None
    if "--out" in sys.argv:
        out = os.path.abspath(sys.argv[sys.argv.index("--out") + 1])
    print(build(force="--force" in sys.argv or out is not None, verbose=True, out=out))
