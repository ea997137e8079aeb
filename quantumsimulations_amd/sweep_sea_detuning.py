"""Drop-in for the reference's ``sweep_sea_detuning`` module (sweep_sea_detuning.py).

Same public names: ``run_sweep_sea_detuning`` (batched over GPUs, same output tree),
``coarse_grain``, ``iz_slope_from_coarse``, ``contrast_michelson_with_t_gate``,
``SLOPE_T_MIN``, ``detuning_label``, ``f1R_for_resonance``.  Run as a script it performs the
reference's ``__main__`` sweep (:1201-1251: Ga/Al at 3 T, f1A = 50 kHz, 13 detunings in
[0, 150 kHz], n_sea = 6, t_final = 30 s, 20000 outputs); the command-line options override it.
"""
from __future__ import annotations

import argparse

import numpy as np

from .metrics import (SLOPE_T_MIN, coarse_grain, contrast_michelson_with_t_gate,  # noqa: F401
                      iz_slope_from_coarse)
from .sweep import detuning_label, f1R_for_resonance  # noqa: F401
from .sweep_runner import run_sweep_sea_detuning  # noqa: F401


def _safe_normalized_difference(num: float, denom: float) -> float:
    """num / denom, NaN when denom is 0 or NaN (reference sweep_sea_detuning.py:324-335)."""
    if denom == 0.0 or np.isnan(denom):
        return float("nan")
    return num / denom


def main(argv=None) -> str:
    ap = argparse.ArgumentParser(description="Sea-detuning sweep on MI355X GPUs")
    ap.add_argument("--n-sea", type=int, default=6)
    ap.add_argument("--t-final", type=float, default=30.0)
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--n-det", type=int, default=13)
    ap.add_argument("--f1a", type=float, default=50_000.0)
    ap.add_argument("--out-root", default="results/sweep_f1A_3x_target_detune_extra_long")
    ap.add_argument("--devices", default=None, help="comma-separated GPU ids (default: all)")
    ap.add_argument("--report", default="full", choices=("full", "png", "none"))
    ap.add_argument("--coarse-window", type=int, default=100)
    a = ap.parse_args(argv)
    gamma_sea, gamma_rare, b0 = 8.1812e7, 6.976e7, 3.0
    f_az = gamma_sea * b0 / (2 * np.pi)
    target = a.f1a
    devices = None if a.devices is None else [int(x) for x in a.devices.split(",")]
    return run_sweep_sea_detuning(
        f_Az=f_az, f1A=a.f1a, target_sea_detuning=target, gamma_sea=gamma_sea,
        gamma_rare=gamma_rare, sea_detunings_Hz=np.linspace(0.0, 3.0 * target, a.n_det),
        n_sea=a.n_sea, t_final=a.t_final, steps=a.steps, phi_sea=np.pi / 2.0,
        phi_rare=np.pi / 2.0, out_root=a.out_root, is_spin_three_half=False, solver_atol=1e-10,
        solver_rtol=1e-9, solver_nsteps=10_000_000, solver_max_step=1e-5,
        coarse_window=a.coarse_window, devices=devices, report=a.report)


if __name__ == "__main__":
    main()
