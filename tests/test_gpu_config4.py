"""BASELINE config 4 on the GPU, in miniature: the 2D driver (quantumsimulations_amd.sweep2d_run)
runs one sweep per f1A (5 and 20 kHz; n_sea = 6, 3 detunings in [0, 3 f1A], 4e-4 s, 80 outputs)
through evolve_many, writes every sweep tree from a worker process and aggregates them with the
headless 2D report.  Compared with the reference's own sweeps and 2D aggregation of the same
configuration (tests/golden/sweep2d_c4, make_golden_sweep.py config4_fixture):

* traces: the reference integrates with ZVODE at rtol 1e-9 (~1e-5 from exact here): abs 2e-5;
  against the exact oracle (dense eigh of the reference-built H): 1e-10
* the 2D points: same (f1A, delta) set; coupling metric to 1e-12; contrast and slope difference to
  the accuracy the reference's own trace allows (abs 1e-6 / 2e-6); the stable-region bins exactly
"""
import glob
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import propagate as pg
from oracle import reference_model as rm
from quantumsimulations_amd.sweep import VARIANTS, detuning_label

pytestmark = pytest.mark.gpu
C4 = os.path.join(GOLDEN, "sweep2d_c4")


def test_config4_driver_matches_reference(tmp_path):
    from quantumsimulations_amd import sweep2d
    from quantumsimulations_amd.sweep2d_run import run_2d_sweep
    exp = json.load(open(os.path.join(C4, "expected.json")))
    cfg = exp["config"]
    out = run_2d_sweep(str(tmp_path), cfg["f1a"], n_det=cfg["n_det"], n_sea=cfg["n_sea"],
                       t_final=cfg["t_final"], steps=cfg["steps"], coarse_window=cfg["coarse_window"],
                       devices=[0], report="none", stable=True, verbose=False)
    assert out["evolutions"] == 2 * 3 * cfg["n_det"] and len(out["sweep_dirs"]) == 2
    for f1a, base in zip(cfg["f1a"], out["sweep_dirs"]):
        ref_base = os.path.join(C4, "root", f"f1A_{int(f1a)}", "sweep")
        for d in np.linspace(0.0, 3.0 * f1a, cfg["n_det"]):
            lab = detuning_label(d)
            for tag in VARIANTS:
                ours = np.load(os.path.join(base, lab, f"time_and_obs_{tag}.npz"))
                ref = np.load(os.path.join(ref_base, lab, f"time_and_obs_{tag}.npz"))
                assert ours.files == ref.files
                np.testing.assert_array_equal(ours["t"], ref["t"])
                for k in ref.files[1:]:
                    np.testing.assert_allclose(ours[k], ref[k], rtol=0, atol=2e-5, err_msg=f"{f1a} {lab} {tag} {k}")
                p = json.load(open(os.path.join(base, lab, f"params_{tag}.json")))
                assert p == json.load(open(os.path.join(ref_base, lab, f"params_{tag}.json")))
                H, obs, psi0, _ = rm.build(p)
                ex = pg.eigh_trace(H, psi0, ours["t"], obs)
                for k in ex:
                    assert np.max(np.abs(ex[k] - ours[k])) < 1e-10, (f1a, lab, tag, k)
    # the 2D aggregation over the GPU-produced tree vs the reference's over its own tree
    key = lambda p: (p["f1A_Hz"], p["delta_Hz"])  # noqa: E731
    got = sorted(sweep2d.aggregate_points(str(tmp_path)), key=key)
    ref_pts = sorted(exp["points"], key=key)
    assert [key(p) for p in got] == [key(p) for p in ref_pts]
    for g, r in zip(got, ref_pts):
        assert g["coupling_metric"] == pytest.approx(r["coupling_metric"], rel=1e-12)
        assert g["contrast"] == pytest.approx(r["contrast"], rel=1e-3, abs=1e-6)
        # |slope_on - slope_off| is a difference of two fitted slopes: the reference's ZVODE trace
        # error (~1e-5 here) moves it by a few 1e-7 absolute
        assert g["abs_delta_slope_center"] == pytest.approx(r["abs_delta_slope_center"], rel=1e-3, abs=2e-6)
    stable = json.load(open(os.path.join(str(tmp_path), "stable_region_stats.json")))
    ref_bins = exp["regions"][0]["stats"]
    assert [(b["x"], b["N"]) for b in stable["per_bin"]] == [(b["x"], b["N"]) for b in ref_bins]
    assert glob.glob(os.path.join(str(tmp_path), "graphs", "*.png"))
