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


def _resources(stderr):
    """(function name, VGPR spill count, scratch bytes per lane) per kernel of a
    -Rpass-analysis=kernel-resource-usage compile."""
    rows = {}
    name = None
    for line in stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            rows[name] = [None, None]
        m = re.search(r"VGPRs Spill: (\d+)", line)
        if m and name:
            rows[name][0] = int(m.group(1))
        m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
        if m and name:
            rows[name][1] = int(m.group(1))
    return [(n, sp, sc) for n, (sp, sc) in rows.items()]


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
    kernels = [k for k in _resources(res.stderr) if "k_interval" in k[0]]
    assert len(kernels) == 8, kernels
    assert all(sp == 0 and sc == 0 for _, sp, sc in kernels), kernels


def test_wht_passes_do_not_spill(tmp_path):
    """The Walsh-Hadamard passes (2 tile sizes x 5 passes x 3 modes, FWD / MID / INV also per
    vector of a partitioned register; the half-LDS forms of option wht_half within 128 VGPRs) stay spill-free and keep their tile arrays out of scratch
    (a run-time vector selector once put them there: N = 30 went from 68 to 353 ms per H); the
    one-thread-per-tile table kernels run once per problem and may use scratch."""
    res = subprocess.run(
        [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
         "--cuda-device-only", "-c", os.path.join(CSRC, "dse_wht.hip"), "-o",
         str(tmp_path / "wht.o"), "-Rpass-analysis=kernel-resource-usage"],
        capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-2000:]
    kernels = [k for k in _resources(res.stderr) if "k_wht" in k[0]]
    persistent = [k for k in kernels if "k_wht_mid_p" in k[0]]
    half = [k for k in kernels if "k_wht_h" in k[0]]
    passes = [k for k in kernels if "k_wht_tables" not in k[0] and "k_wht_qtab" not in k[0] and k not in persistent
              and k not in half]
    assert len(passes) == 2 * (3 * 3 + 3 * 3 * 3), [k[0] for k in passes]  # FIRST, FINAL, FINAL_NEXT x mode
    assert len(persistent) == 2 * 3 * 3, [k[0] for k in persistent]  # tile x mode x vectors
    assert len(half) == 3 + 3 * 3 * 3, [k[0] for k in half]  # 13-bit tiles: FIRST x mode, FWD/MID/INV x mode x vectors
    passes += persistent + half
    assert all(sp == 0 for _, sp, _ in kernels), kernels
    assert all(sc == 0 for _, _, sc in passes), passes


def test_span_kernel_does_not_spill(tmp_path):
    """k_span (dse_span.hip) keeps out, w_{k-2} and the pipelined partner rows in registers at two
    waves per SIMD for the 512-thread configurations (2^11 tiles x 4 rows, 2^10 x 2 rows)."""
    res = subprocess.run(
        [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-c",
         os.path.join(CSRC, "dse_span.hip"), "-o", str(tmp_path / "span.o"), "-Rpass-analysis=kernel-resource-usage"],
        capture_output=True, text=True)
    assert res.returncode == 0, res.stderr[-2000:]
    kernels = [k for k in _resources(res.stderr) if "k_span" in k[0]]
    assert len(kernels) >= 4, kernels
    assert all(sp == 0 and sc == 0 for _, sp, sc in kernels), kernels


def test_real_kernel_does_not_spill(tmp_path):
    """k_real (dse_real.hip, option real): the production instantiation k_real<0> holds out and
    w_{k-2} (32 real rows each) in registers at two waves per SIMD without scratch spills (the
    diagnostic ablation instantiations may spill)."""
    res = subprocess.run(
        [_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-c",
         os.path.join(CSRC, "dse_real.hip"), "-o", str(tmp_path / "real.o"), "-Rpass-analysis=kernel-resource-usage"],
        capture_output=True, text=True)
    assert res.returncode == 0, res.stderr[-2000:]
    kernels = [k for k in _resources(res.stderr) if "k_realILi0E" in k[0]]
    assert len(kernels) == 1, _resources(res.stderr)
    assert all(sp == 0 and sc == 0 for _, sp, sc in kernels), kernels


def test_coef_schedule_covers_every_term_once(tmp_path):
    """coef_nterm (dse_internal.h): for every update phase (k_span staggers output j to phase
    j % 3) and series degree d, the terms accumulated at k = 1..d are exactly a_0..a_d, each once,
    and no update reaches further back than w_{k-2}; phase 0 is the k_interval / k_real schedule
    (updates at k = 1, 4, 7, ... and the remainder at k = d)."""
    src = tmp_path / "sched.cpp"
    src.write_text(r'''
#include "dse_internal.h"
#include <cstdio>
int main() {
  for (int ph = 0; ph < 3; ++ph)
    for (int d = 1; d <= 400; ++d) {
      int next = 0;  // first term not yet accumulated
      for (int k = 1; k <= d + 1; ++k) {
        const int n = dse::coef_nterm(k, d, ph);
        if (k > d) { if (n) return 1; continue; }
        if (n > 3 || (k == 1 && n != 2)) return 2;
        if (n == 0) continue;
        if (k - n + 1 != (k == 1 ? 0 : next) && !(k == 1 && next == 0)) return 3;
        next = k + 1;
      }
      if (next != d + 1) return 4;
      if (ph == 0)
        for (int k = 2; k <= d; ++k)
          if ((dse::coef_nterm(k, d, 0) == 3) != ((k - 1) % 3 == 0)) return 5;
    }
  std::puts("ok");
  return 0;
}
''')
    exe = tmp_path / "sched"
    res = subprocess.run([_hipcc(), "-std=c++17", "-I", CSRC, "-I", os.path.join(ROOT, "include"),
                          "-x", "hip", "--offload-arch=gfx950", str(src), "-o", str(exe)],
                         capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-2000:]
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert run.returncode == 0 and run.stdout.strip() == "ok", (run.returncode, run.stdout, run.stderr)
