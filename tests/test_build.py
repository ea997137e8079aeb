"""Build-level checks of the HIP sources (CPU only: hipcc cross-compiles for gfx950)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quantumsimulations_amd", "csrc")


def _hipcc():
    for c in ("/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    pytest.skip("hipcc not available")


def test_interval_kernel_does_not_spill(tmp_path):
    """k_interval holds w_{k-2} and w_k (16 amplitudes each) in registers at 2 waves per SIMD:
    every variant must fit the 256-VGPR budget without scratch spills (a spilling build gave
    run-to-run differences of ~1e-9 on 2-tile problems)."""
    res = subprocess.run(
        [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
         "--cuda-device-only", "-c", os.path.join(CSRC, "dse_interval.hip"), "-o",
         str(tmp_path / "iv.o"), "-Rpass-analysis=kernel-resource-usage"],
        capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-2000:]
    names = re.findall(r"Function Name: (\S+)", res.stderr)
    spills = [int(v) for v in re.findall(r"VGPRs Spill: (\d+)", res.stderr)]
    kernels = [(n, s) for n, s in zip(names, spills) if "k_interval" in n]
    assert len(kernels) == 8, names
    assert all(s == 0 for _, s in kernels), kernels


def test_wht_passes_do_not_spill(tmp_path):
    """The Walsh-Hadamard passes (2 tile sizes x 5 passes x 3 modes) and the table kernels stay
    spill-free."""
    res = subprocess.run(
        [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
         "--cuda-device-only", "-c", os.path.join(CSRC, "dse_wht.hip"), "-o",
         str(tmp_path / "wht.o"), "-Rpass-analysis=kernel-resource-usage"],
        capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-2000:]
    names = re.findall(r"Function Name: (\S+)", res.stderr)
    spills = [int(v) for v in re.findall(r"VGPRs Spill: (\d+)", res.stderr)]
    kernels = [(n, s) for n, s in zip(names, spills) if "k_wht" in n]
    assert len(kernels) == 34, names
    assert all(s == 0 for _, s in kernels), kernels
