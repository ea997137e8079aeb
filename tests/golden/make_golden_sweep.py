"""Generate the sweep-level golden fixtures from the reference's own sweep code.

Run ONLY in the build container (reads /root/reference, absent on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_sweep.py

The reference's ``sweep_sea_detuning.py`` is imported by path with the QuTiP stand-in of
``_qutip_standin`` first on sys.path and the reference's own ``dipolar_ensemble_with_rare.py``
registered under its module name (the same route as make_golden.py).  Nothing of the reference
is copied: only the numbers and files its functions produce are stored.

Fixtures written:
  sweep_metrics.json   coarse_grain / iz_slope_from_coarse on the N = 7 traces of traces_n7.npz
                       for several windows and edge cases, contrast_michelson_with_t_gate cases
  sweep_n7/            the data files of one complete reference sweep (n_sea = 6, 3 detunings,
                       t_final 2e-4 s, 60 outputs, coarse_window 5, the sweep's ZVODE tolerances):
                       every .npz and .json of the tree, plus manifest.json listing every file
                       of the tree (PNG / PDF included) relative to the sweep directory
  sweep2d_c4/          BASELINE config 4 in miniature: the reference's sweeps at f1A = 5 and 20 kHz
                       (n_sea = 6, 3 detunings in [0, 3 f1A], 4e-4 s, 80 outputs) and its 2D
                       aggregation over both trees (config4_fixture)
  sweep2d/             synthetic multi-sweep summary.json files (4 f1A values, NaN / missing
                       entries, a sweep without f1A) and expected.json: the reference's
                       aggregate_points, compute_stable_region for several criteria and the
                       files make_plots / make_plots_and_analyze write (2D_sweep_report*.py).
                       Both scripts import tkinter at module level (absent here) for their folder
                       picker only; a bare placeholder module satisfies that import and is never
                       called (the root directory is always passed).
"""
from __future__ import annotations

import importlib.util
import json
import os
import shutil
import sys
import tempfile

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "_qutip_standin"))

import matplotlib  # noqa: E402

matplotlib.use("Agg")


def _load(name, file):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, file))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


_load("dipolar_ensemble_with_rare", "dipolar_ensemble_with_rare.py")
sweep = _load("ref_sweep_sea_detuning", "sweep_sea_detuning.py")

SWEEP_N7 = dict(n_sea=6, sea_detunings_Hz=[0.0, 25000.0, 75000.0], t_final=2e-4, steps=60,
                coarse_window=5)


def _jsonable(d):
    return {k: (None if isinstance(v, float) and not np.isfinite(v) else v) for k, v in d.items()}


def metrics_fixture():
    tr = np.load(os.path.join(HERE, "traces_n7.npz"))
    t = tr["t"]
    cases = []
    for src in ("center_off_ref_Iz_sea", "center_on_ref_Iz_sea", "shell_off_exact_Iz_sea"):
        y = tr[src]
        for w in (-2, 1, 3, 10, 25, 50, 67, 100, 201, 300):
            tc, yc = sweep.coarse_grain(t, y, window=w)
            cases.append({"trace": src, "window": w, "t_coarse": tc.tolist(),
                          "y_coarse": yc.tolist(),
                          "slope": _jsonable(sweep.iz_slope_from_coarse(tc, yc))})
    # degenerate envelopes: constant (R undefined), 4 points, 5 points, linear (zero residual)
    extra = {"constant": (np.linspace(0, 1, 10), np.full(10, 0.25)),
             "four": (np.array([0.0, 1.0, 2.0, 3.0]), np.array([0.1, 0.3, 0.2, 0.5])),
             "five": (np.arange(5.0), np.array([1.0, -2.0, 0.5, 4.0, 3.0])),
             "linear": (np.arange(12.0), 0.5 + 2.0 * np.arange(12.0)),
             "three": (np.arange(3.0), np.array([1.0, 2.0, 4.0]))}
    for name, (tc, yc) in extra.items():
        cases.append({"trace": name, "window": None, "t_coarse": tc.tolist(),
                      "y_coarse": yc.tolist(), "slope": _jsonable(sweep.iz_slope_from_coarse(tc, yc))})
    contrast = []
    for args in ((1e-3, 5e-4, 3.0, 2.0), (1e-3, 5e-4, 0.5, 2.0), (1e-3, 5e-4, 3.0, 0.2),
                 (1e-3, 5e-4, 0.1, 0.2), (-2e-3, 1e-3, -4.0, 5.0), (float("nan"), 1e-3, 2.0, 2.0),
                 (1e-3, 1e-3, float("nan"), 2.0), (0.0, 0.0, 5.0, 5.0), (1e-17, 1e-17, 5.0, 5.0),
                 (3e-4, -3e-4, 1.0, -1.0)):
        c = sweep.contrast_michelson_with_t_gate(*args)
        contrast.append({"args": [None if not np.isfinite(a) else a for a in args],
                         "value": None if not np.isfinite(c) else c})
    with open(os.path.join(HERE, "sweep_metrics.json"), "w") as f:
        json.dump({"coarse_and_slope": cases, "contrast": contrast}, f, indent=1)


def sweep_fixture():
    out = os.path.join(HERE, "sweep_n7")
    shutil.rmtree(out, ignore_errors=True)
    os.makedirs(out)
    with tempfile.TemporaryDirectory() as tmp:
        f_az = 8.1812e7 * 3.0 / (2 * np.pi)
        base = sweep.run_sweep_sea_detuning(
            f_Az=f_az, f1A=50_000, target_sea_detuning=50_000, gamma_sea=8.1812e7,
            gamma_rare=6.976e7, phi_sea=np.pi / 2.0, phi_rare=np.pi / 2.0, out_root=tmp,
            is_spin_three_half=False, solver_atol=1e-10, solver_rtol=1e-9,
            solver_nsteps=10_000_000, solver_max_step=1e-5, **SWEEP_N7)
        files = []
        for root, _, names in os.walk(base):
            for nm in names:
                rel = os.path.relpath(os.path.join(root, nm), base)
                files.append(rel)
                if nm.endswith((".npz", ".json")):
                    dst = os.path.join(out, rel)
                    os.makedirs(os.path.dirname(dst), exist_ok=True)
                    shutil.copyfile(os.path.join(root, nm), dst)
    with open(os.path.join(out, "manifest.json"), "w") as f:
        json.dump({"config": SWEEP_N7, "files": sorted(files)}, f, indent=1)


def _synthetic_summaries(root):
    rng = np.random.default_rng(2024)
    for s_i, f1a in enumerate((5000.0, 20000.0, 35000.0, 50000.0)):
        rows = []
        for d in np.linspace(0.0, 3.0 * f1a, 13):
            x = d / f1a
            row = {"delta_Hz": float(d),
                   "contrast_rare_center": float(-0.6 * np.exp(-(x - 1.2) ** 2) + 0.15 * rng.standard_normal()),
                   "DeltaOmega_over_geff": float((np.sqrt(d * d + f1a * f1a) - np.sqrt(2) * f1a) / 40.0),
                   "I_z_slope_off_center": float(rng.standard_normal() * 1e-3),
                   "I_z_slope_on_center": float(rng.standard_normal() * 1e-3)}
            rows.append(row)
        rows[2]["contrast_rare_center"] = float("nan")
        rows[3]["DeltaOmega_over_geff"] = None
        del rows[4]["I_z_slope_on_center"]
        rows[5]["I_z_slope_off_center"] = float("inf")
        sub = os.path.join(root, f"f1A_{int(f1a)}", f"sea_detuning_sweep_2026010{s_i}_000000")
        os.makedirs(sub)
        with open(os.path.join(sub, "summary.json"), "w") as f:
            json.dump({"global_params": {"f1A_Hz": f1a}, "sweep_results": rows}, f, indent=2)
    os.makedirs(os.path.join(root, "no_f1a"))
    with open(os.path.join(root, "no_f1a", "summary.json"), "w") as f:
        json.dump({"global_params": {}, "sweep_results": [{"delta_Hz": 1.0}]}, f)


def sweep2d_fixture():
    import types
    tk = types.ModuleType("tkinter")
    tk.filedialog = types.ModuleType("tkinter.filedialog")
    sys.modules["tkinter"], sys.modules["tkinter.filedialog"] = tk, tk.filedialog
    rep = _load("ref_2d_sweep_report", "2D_sweep_report.py")
    stab = _load("ref_2d_sweep_report_stable_region", "2D_sweep_report_stable_region.py")
    out = os.path.join(HERE, "sweep2d")
    shutil.rmtree(out, ignore_errors=True)
    root = os.path.join(out, "root")
    _synthetic_summaries(root)
    pts = stab.aggregate_points(root)
    assert json.dumps(pts) == json.dumps(rep.aggregate_points(root))
    x = np.array([p["delta_Hz"] / p["f1A_Hz"] for p in pts])
    c = np.array([p["contrast"] for p in pts])
    regions = []
    for c_min, p_min, dec, neg in ((0.2, 0.8, 3, True), (0.1, 0.5, 2, True), (0.3, 0.9, 1, True),
                                   (0.05, 0.5, 3, False), (0.2, 0.5, 0, True)):
        stats, best = stab.compute_stable_region(x, c, c_min, p_min, dec, require_negative=neg)
        regions.append({"args": [c_min, p_min, dec, neg], "stats": stats, "best": best})
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "a"))
        os.makedirs(os.path.join(tmp, "b"))
        rep.make_plots(root, os.path.join(tmp, "a", "summary.pdf"))
        stab.make_plots_and_analyze(root, os.path.join(tmp, "b", "summary.pdf"), 0.2, 0.8, 3,
                                    os.path.join(tmp, "b", "stable.json"), True)
        with open(os.path.join(tmp, "b", "stable.json")) as f:
            stable_json = json.load(f)
        files_a = sorted(os.listdir(os.path.join(tmp, "a", "graphs")))
        files_b = sorted(os.listdir(os.path.join(tmp, "b", "graphs")))
    with open(os.path.join(out, "expected.json"), "w") as f:
        json.dump({"points": pts, "regions": regions, "stable_json": stable_json,
                   "graphs_make_plots": files_a, "graphs_stable": files_b}, f, indent=1)


CONFIG4 = dict(f1a=(5000.0, 20000.0), n_sea=6, n_det=3, t_final=4e-4, steps=80, coarse_window=5)


def config4_fixture():
    """BASELINE config 4 in miniature: the reference's sweep for two drive strengths (its __main__
    pattern: target = f1A, detunings linspace(0, 3 f1A, n), sweep_sea_detuning.py:1220-1240), then
    its 2D aggregation over both sweep trees (2D_sweep_report.py:288-303,
    2D_sweep_report_stable_region.py:260-364).  Stored: the trees' .npz/.json files under
    sweep2d_c4/root/f1A_<Hz>/sweep/ and expected.json (points, stable-region results)."""
    import types
    tk = types.ModuleType("tkinter")
    tk.filedialog = types.ModuleType("tkinter.filedialog")
    sys.modules["tkinter"], sys.modules["tkinter.filedialog"] = tk, tk.filedialog
    stab = _load("ref_2d_sweep_report_stable_region", "2D_sweep_report_stable_region.py")
    out = os.path.join(HERE, "sweep2d_c4")
    shutil.rmtree(out, ignore_errors=True)
    root = os.path.join(out, "root")
    f_az = 8.1812e7 * 3.0 / (2 * np.pi)
    with tempfile.TemporaryDirectory() as tmp:
        for f1a in CONFIG4["f1a"]:
            base = sweep.run_sweep_sea_detuning(
                f_Az=f_az, f1A=f1a, target_sea_detuning=f1a, gamma_sea=8.1812e7,
                gamma_rare=6.976e7, sea_detunings_Hz=np.linspace(0.0, 3.0 * f1a, CONFIG4["n_det"]),
                n_sea=CONFIG4["n_sea"], t_final=CONFIG4["t_final"], steps=CONFIG4["steps"],
                phi_sea=np.pi / 2.0, phi_rare=np.pi / 2.0, out_root=os.path.join(tmp, "x"),
                is_spin_three_half=False, solver_atol=1e-10, solver_rtol=1e-9,
                solver_nsteps=10_000_000, solver_max_step=1e-5,
                coarse_window=CONFIG4["coarse_window"])
            dst_root = os.path.join(root, f"f1A_{int(f1a)}", "sweep")
            for rt, _, names in os.walk(base):
                for nm in names:
                    if nm.endswith((".npz", ".json")):
                        rel = os.path.relpath(os.path.join(rt, nm), base)
                        dst = os.path.join(dst_root, rel)
                        os.makedirs(os.path.dirname(dst), exist_ok=True)
                        shutil.copyfile(os.path.join(rt, nm), dst)
            shutil.rmtree(os.path.join(tmp, "x"))
    pts = stab.aggregate_points(root)
    x = np.array([p["delta_Hz"] / p["f1A_Hz"] for p in pts])
    c = np.array([p["contrast"] for p in pts])
    regions = []
    for c_min, p_min, dec, neg in ((0.2, 0.8, 3, True), (0.05, 0.5, 1, True), (0.0, 0.5, 2, False)):
        stats, best = stab.compute_stable_region(x, c, c_min, p_min, dec, require_negative=neg)
        regions.append({"args": [c_min, p_min, dec, neg], "stats": stats, "best": best})
    with open(os.path.join(out, "expected.json"), "w") as f:
        json.dump({"config": {**CONFIG4, "f1a": list(CONFIG4["f1a"])}, "points": pts,
                   "regions": regions}, f, indent=1)


if __name__ == "__main__":
    if "--config4" in sys.argv:
        config4_fixture()
    else:
        metrics_fixture()
        sweep_fixture()
        sweep2d_fixture()
        config4_fixture()
    print("ok")
