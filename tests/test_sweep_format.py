"""Sweep outputs: metrics and the on-disk tree against fixtures the
reference's own sweep code produced (tests/golden/make_golden_sweep.py).

CPU tests: the metric functions are bit-identical to the reference's on the same envelopes, and
``run_sweep_sea_detuning`` writes the same tree (file names, npz keys / dtypes / shapes, JSON
records) when fed the reference's traces in place of the GPU evolutions (the evolution step is
replaced by the fixture data; there is no CPU evolution path in the product).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from quantumsimulations_amd import metrics as M
from quantumsimulations_amd import sweep_runner
from quantumsimulations_amd.sweep import VARIANTS, detuning_label

SWEEP_DIR = os.path.join(GOLDEN, "sweep_n7")


def _nan_eq(a, b):
    if a is None:
        return b is None or (isinstance(b, float) and np.isnan(b))
    if isinstance(a, float) and np.isnan(a):
        return isinstance(b, float) and np.isnan(b)
    return a == b


def test_coarse_grain_and_slope_bit_exact(golden):
    fx = golden("sweep_metrics.json")
    tr = golden("traces_n7.npz")
    for case in fx["coarse_and_slope"]:
        if case["window"] is not None:
            tc, yc = M.coarse_grain(tr["t"], tr[case["trace"]], window=case["window"])
            assert tc.tolist() == case["t_coarse"] and yc.tolist() == case["y_coarse"], case["trace"]
        else:
            tc, yc = np.array(case["t_coarse"]), np.array(case["y_coarse"])
        got = M.iz_slope_from_coarse(tc, yc)
        assert list(got) == list(case["slope"])
        for k, v in case["slope"].items():
            assert _nan_eq(v, got[k]), (case["trace"], case["window"], k, v, got[k])


def test_coarse_grain_zero_window_raises():
    with pytest.raises(ZeroDivisionError):
        M.coarse_grain(np.arange(4.0), np.arange(4.0), window=0)


def test_contrast_bit_exact(golden):
    for case in golden("sweep_metrics.json")["contrast"]:
        args = [np.nan if a is None else a for a in case["args"]]
        assert _nan_eq(case["value"], M.contrast_michelson_with_t_gate(*args)), case


def _load_tree(base):
    out = {}
    for root, _, names in os.walk(base):
        for nm in names:
            out[os.path.relpath(os.path.join(root, nm), base)] = os.path.join(root, nm)
    return out


def _reference_traces():
    man = json.load(open(os.path.join(SWEEP_DIR, "manifest.json")))
    traces = []
    for d in man["config"]["sea_detunings_Hz"]:
        for tag in VARIANTS:
            z = np.load(os.path.join(SWEEP_DIR, detuning_label(d), f"time_and_obs_{tag}.npz"))
            traces.append((z["t"], {k: z[k] for k in z.files if k != "t"}))
    return man, traces


def test_point_metrics_match_reference_sweep():
    """metrics.json of every point, recomputed from the reference's own traces: bit-identical."""
    man, traces = _reference_traces()
    gp = json.load(open(os.path.join(SWEEP_DIR, "global_params.json")))
    for i, d in enumerate(man["config"]["sea_detunings_Hz"]):
        per = {tag: (traces[3 * i + j][0], traces[3 * i + j][1]["Iz_sea"])
               for j, tag in enumerate(VARIANTS)}
        ref = json.load(open(os.path.join(SWEEP_DIR, detuning_label(d), "metrics.json")))
        got, _ = M.point_metrics(d, gp["f_Az_Hz"] - d, gp["f1A_Hz"], gp["f1R_Hz"],
                                 gp["rms_b_AR_Hz"], per, gp["coarse_window"])
        assert list(got) == list(ref)
        for k in ref:
            assert _nan_eq(ref[k], got[k]), (d, k, ref[k], got[k])


@pytest.mark.parametrize("report", ["full", "none"])
def test_sweep_tree_matches_reference(tmp_path, monkeypatch, report):
    """The dispatcher's output tree, with the evolutions replaced by the reference's traces."""
    man, traces = _reference_traces()
    cfg = man["config"]
    calls = []

    def fake_evolve(params_list, devices=None, tol=1e-14):
        calls.append(len(params_list))
        assert len(params_list) == len(traces)
        return traces
    monkeypatch.setattr(sweep_runner, "evolve_many", fake_evolve)
    f_az = 8.1812e7 * 3.0 / (2 * np.pi)
    timings = {}
    base = sweep_runner.run_sweep_sea_detuning(
        f_Az=f_az, f1A=50_000, target_sea_detuning=50_000, gamma_sea=8.1812e7, gamma_rare=6.976e7,
        phi_sea=np.pi / 2.0, phi_rare=np.pi / 2.0, out_root=str(tmp_path), solver_atol=1e-10,
        solver_rtol=1e-9, solver_nsteps=10_000_000, solver_max_step=1e-5, report=report,
        timings=timings, verbose=False, **cfg)
    assert calls == [3 * len(cfg["sea_detunings_Hz"])]
    assert os.path.basename(base).startswith("sea_detuning_sweep_")
    assert set(timings) == {"evolve_s", "outputs_s", "report_s"}
    tree = _load_tree(base)
    want = set(man["files"])
    if report == "none":
        want = {f for f in want if not f.endswith((".png", ".pdf"))}
    assert set(tree) == want
    for rel in want:
        if rel.endswith(".json"):
            a = json.load(open(os.path.join(SWEEP_DIR, rel)))
            b = json.load(open(tree[rel]))
            assert json.dumps(a, sort_keys=False) == json.dumps(b, sort_keys=False), rel
        elif rel.endswith(".npz"):
            a, b = np.load(os.path.join(SWEEP_DIR, rel)), np.load(tree[rel])
            assert a.files == b.files, rel
            for k in a.files:
                assert a[k].dtype == b[k].dtype and a[k].shape == b[k].shape, (rel, k)
                np.testing.assert_array_equal(a[k], b[k], err_msg=f"{rel}:{k}")


def test_lpt_assignment_balances():
    costs = [5.0, 4.0, 3.0, 3.0, 2.0, 2.0, 1.0]
    bins = sweep_runner.assign_lpt(costs, 3)
    assert sorted(i for b in bins for i in b) == list(range(len(costs)))
    loads = [sum(costs[i] for i in b) for b in bins]
    assert max(loads) - min(loads) <= 1.0
    assert sweep_runner.assign_lpt([1.0], 4) == [[0], [], [], []]


# ------------------------------------------------------------------------------------------
# headless 2D report against the reference's 2D_sweep_report*.py
# ------------------------------------------------------------------------------------------
def _sweep2d():
    from quantumsimulations_amd import sweep2d
    exp = json.load(open(os.path.join(GOLDEN, "sweep2d", "expected.json")))
    return sweep2d, exp, os.path.join(GOLDEN, "sweep2d", "root")


def test_sweep2d_aggregate_points():
    sweep2d, exp, root = _sweep2d()
    assert json.dumps(sweep2d.aggregate_points(root)) == json.dumps(exp["points"])


def test_sweep2d_stable_region():
    sweep2d, exp, _ = _sweep2d()
    x = np.array([p["delta_Hz"] / p["f1A_Hz"] for p in exp["points"]])
    c = np.array([p["contrast"] for p in exp["points"]])
    for case in exp["regions"]:
        c_min, p_min, dec, neg = case["args"]
        stats, best = sweep2d.compute_stable_region(x, c, c_min, p_min, dec, require_negative=neg)
        assert json.loads(json.dumps(stats)) == case["stats"]
        assert json.loads(json.dumps(best)) == case["best"]
    with pytest.raises(RuntimeError):
        sweep2d.compute_stable_region(np.array([np.nan]), np.array([1.0]), 0.2, 0.8, 3)


def test_sweep2d_cli_outputs(tmp_path):
    sweep2d, exp, root = _sweep2d()
    out_a, out_b = tmp_path / "a", tmp_path / "b"
    assert sweep2d.main([root, "-o", str(out_a / "s.pdf")]) == 0
    assert sorted(os.listdir(out_a / "graphs")) == exp["graphs_make_plots"]
    assert (out_a / "s.pdf").stat().st_size > 0
    assert sweep2d.main([root, "-o", str(out_b / "s.pdf"), "--stable", "--add-stability-page",
                         "--stable-json", str(out_b / "stable.json")]) == 0
    assert sorted(os.listdir(out_b / "graphs")) == exp["graphs_stable"]
    assert json.load(open(out_b / "stable.json")) == exp["stable_json"]
    assert sweep2d.main([str(tmp_path / "missing")]) == 2


# ------------------------------------------------------------------------------------------
# BASELINE config 4 in miniature (tests/golden/sweep2d_c4): the reference's own sweeps at two
# f1A values and its 2D aggregation over them
# ------------------------------------------------------------------------------------------
def test_sweep2d_config4_reference_trees():
    """The headless 2D port reproduces the reference's aggregation of the reference's sweep trees."""
    from quantumsimulations_amd import sweep2d
    exp = json.load(open(os.path.join(GOLDEN, "sweep2d_c4", "expected.json")))
    root = os.path.join(GOLDEN, "sweep2d_c4", "root")
    pts = sweep2d.aggregate_points(root)
    key = lambda p: (p["f1A_Hz"], p["delta_Hz"])  # noqa: E731  (walk order is the filesystem's)
    assert json.dumps(sorted(pts, key=key)) == json.dumps(sorted(exp["points"], key=key))
    x = np.array([p["delta_Hz"] / p["f1A_Hz"] for p in exp["points"]])
    c = np.array([p["contrast"] for p in exp["points"]])
    for case in exp["regions"]:
        c_min, p_min, dec, neg = case["args"]
        stats, best = sweep2d.compute_stable_region(x, c, c_min, p_min, dec, require_negative=neg)
        assert json.loads(json.dumps(stats)) == case["stats"]
        assert json.loads(json.dumps(best)) == case["best"]
