"""Sea-detuning sweep points (host side of sweep_sea_detuning.py).

``sweep_point_params`` forms the DipolarRareParams of one (detuning, variant)
exactly as ``run_sweep_sea_detuning`` does (sweep_sea_detuning.py:414-668) with
the Ga/Al constants of its ``__main__`` (:1201-1251).  Variants:
``center_off`` / ``center_on`` (rare at the center, rare drive off / on) and
``shell_off`` (sea-as-center control), :660-668.
"""
from __future__ import annotations

import dataclasses
from typing import List, Sequence

import numpy as np

from .model import DipolarRareParams

GAMMA_SEA = 8.1812e7         # 71Ga, rad s^-1 T^-1 (sweep_sea_detuning.py:1206)
GAMMA_RARE = 6.976e7         # 27Al (:1211)
B0_TESLA = 3.0               # (:1214)
F1A_HZ = 50_000              # (:1220)
PHI = (np.pi / 2.0) * 1.0    # (:1227-1228)
DIPOLAR_SCALE_SI = 1.0e-7 * 1.054571817e-34   # mu0/4pi * hbar (:434-436)
SHELL_SCALE_M = 0.282393e-9  # (:437)
SWEEP_TOL = dict(solver_atol=1e-10, solver_rtol=1e-9, solver_nsteps=10_000_000, solver_max_step=1e-5)
VARIANTS = ("center_off", "center_on", "shell_off")


def f_az_hz(gamma_sea: float = GAMMA_SEA, b0: float = B0_TESLA) -> float:
    return gamma_sea * b0 / (2 * np.pi)


def f1R_for_resonance(f1A_Hz: float, deltaA_Hz: float, deltaR_Hz: float = 0.0) -> float:
    """sqrt(dA^2 + f1A^2) = sqrt(dR^2 + f1R^2) solved for f1R (sweep_sea_detuning.py:1168-1194)."""
    lhs_sq = deltaA_Hz ** 2 + f1A_Hz ** 2
    return (lhs_sq - deltaR_Hz ** 2) ** 0.5


def detuning_label(delta_Hz: float) -> str:
    """Per-detuning directory name, e.g. +1000.0 -> 'delta_p1000.0Hz' (sweep_sea_detuning.py:342-349)."""
    return f"delta_{delta_Hz:+.1f}Hz".replace("+", "p").replace("-", "m")


def sweep_point_params(n_sea: int, delta_Hz: float, variant: str, t_final: float, steps: int,
                       f1A: float = F1A_HZ, target_sea_detuning: float | None = None,
                       gamma_sea: float = GAMMA_SEA, gamma_rare: float = GAMMA_RARE,
                       f_Az: float | None = None, phi_sea: float = PHI, phi_rare: float = PHI,
                       is_spin_three_half: bool = False, solver=SWEEP_TOL) -> DipolarRareParams:
    """DipolarRareParams of one sweep point, as built at sweep_sea_detuning.py:414-668."""
    if target_sea_detuning is None:
        target_sea_detuning = f1A
    if f_Az is None:
        f_Az = f_az_hz(gamma_sea)
    f1R = f1R_for_resonance(f1A, target_sea_detuning, 0.0)
    B0_common = 2 * np.pi * f_Az / gamma_sea
    f_Rz = gamma_rare * B0_common / (2 * np.pi)
    B1_sea = 2 * np.pi * f1A / gamma_sea
    B1_rare = 2 * np.pi * f1R / gamma_rare if gamma_rare != 0.0 else 0.0
    f_rf_sea = f_Az - delta_Hz
    base = DipolarRareParams(
        n_sea=n_sea, gamma_sea=gamma_sea, gamma_rare=gamma_rare,
        B0_sea=B0_common, B0_rare=B0_common, B1_sea=B1_sea, B1_rare=B1_rare,
        omega_rf_sea=2 * np.pi * f_rf_sea, omega_rf_rare=2 * np.pi * f_Rz,
        phi_sea=phi_sea, phi_rare=phi_rare, dipolar_scale=DIPOLAR_SCALE_SI,
        shell_scale=SHELL_SCALE_M, t_final=t_final, steps=steps, drive_sea=True,
        drive_rare=False, init_x_sign=-1, init_rare_level=3,
        is_spin_three_half=is_spin_three_half, is_center_rare=True, **dict(solver or {}))
    if variant == "center_off":
        return dataclasses.replace(base, drive_rare=False, is_center_rare=True)
    if variant == "center_on":
        return dataclasses.replace(base, drive_rare=True, is_center_rare=True)
    if variant == "shell_off":
        return dataclasses.replace(base, drive_rare=False, is_center_rare=False)
    raise ValueError(f"unknown variant {variant!r}")


def sweep_params(n_sea: int, detunings_Hz: Sequence[float], t_final: float, steps: int,
                 **kw) -> List[DipolarRareParams]:
    """All 3 x len(detunings) evolutions of one sweep, detuning-major, variant order of :694-702."""
    return [sweep_point_params(n_sea, float(d), v, t_final, steps, **kw)
            for d in detunings_Hz for v in VARIANTS]
