"""Physical model of the driven heteronuclear dipolar spin ensemble (host side).

This module is the host-side restatement of the parameter/geometry layer of the
reference's ``dipolar_ensemble_with_rare.py``.  It has no QuTiP dependency: it
produces plain floats and numpy arrays that ``problem.py`` reduces to
coefficient tables for the HIP engine.

Floating-point expressions follow the reference's evaluation order so the
derived frequencies, positions and couplings agree bit-for-bit (checked against
the golden fixtures in ``tests/golden``).

Reference map
-------------
* ``DipolarRareParams``               dipolar_ensemble_with_rare.py:307-384
* ``get_derived_frequencies``         dipolar_ensemble_with_rare.py:387-450
* ``_platonic_vertices``              dipolar_ensemble_with_rare.py:107-202
* ``shell_positions_with_rare_center``dipolar_ensemble_with_rare.py:205-251
* ``dipolar_couplings_from_positions``dipolar_ensemble_with_rare.py:255-299
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict

import numpy as np


# ---------------------------------------------------------------------------
# Parameter record (dipolar_ensemble_with_rare.py:307-384).  The field list is
# kept identical (names, order, defaults) because callers serialise it with
# dataclasses.asdict (sweep_sea_detuning.py:683).
# ---------------------------------------------------------------------------

@dataclass
class DipolarRareParams:
    """All knobs of one evolution of n_sea spin-1/2 "sea" nuclei + one rare nucleus.

    Angular frequencies are derived: omega_z = gamma * B0, omega_1 = gamma * B1.
    A species whose drive is off is described in the frame rotating at its own
    Larmor frequency (zero detuning, no Zeeman term).
    """

    n_sea: int = 12

    gamma_sea: float = 1.0
    gamma_rare: float = 1.0

    B0_sea: float = 1.0
    B0_rare: float = 1.0

    B1_sea: float = 0.0
    B1_rare: float = 0.0

    omega_rf_sea: float | None = None
    omega_rf_rare: float | None = None

    phi_sea: float = 0.0
    phi_rare: float = 0.0

    dipolar_scale: float = 2 * np.pi

    shell_scale: float = 0.282393

    t_final: float = 0.02
    steps: int = 2_000

    drive_sea: bool = False
    drive_rare: bool = False

    # Used as the z-basis sign of the sea spins (dipolar_ensemble_with_rare.py:599);
    # the rare spin takes the opposite sign (:602).
    init_x_sign: int = -1
    # Present in the reference record but never read (:375).
    init_rare_level: int = 3

    is_spin_three_half: bool = True
    is_center_rare: bool = True

    solver_atol: float | None = None
    solver_rtol: float | None = None
    solver_nsteps: int | None = None
    solver_max_step: float | None = None


def get_derived_frequencies(params: DipolarRareParams) -> Dict[str, float]:
    """Larmor/Rabi/rf angular frequencies, detunings and their Hz copies.

    Mirrors dipolar_ensemble_with_rare.py:387-450, including the rule that a
    detuning is exactly 0.0 when its drive is off.
    """
    omega_Az = params.gamma_sea * params.B0_sea
    omega_Rz = params.gamma_rare * params.B0_rare
    omega1_sea = params.gamma_sea * params.B1_sea
    omega1_rare = params.gamma_rare * params.B1_rare

    omega_rf_sea = omega_Az if params.omega_rf_sea is None else params.omega_rf_sea
    omega_rf_rare = omega_Rz if params.omega_rf_rare is None else params.omega_rf_rare

    delta_sea = (omega_Az - omega_rf_sea) if params.drive_sea else 0.0
    delta_rare = (omega_Rz - omega_rf_rare) if params.drive_rare else 0.0

    two_pi = 2 * np.pi
    angular = {
        "omega_Az": omega_Az,
        "omega_Rz": omega_Rz,
        "omega1_sea": omega1_sea,
        "omega1_rare": omega1_rare,
        "omega_rf_sea": omega_rf_sea,
        "omega_rf_rare": omega_rf_rare,
        "delta_sea": delta_sea,
        "delta_rare": delta_rare,
    }
    hz_names = {
        "f_Az": "omega_Az",
        "f_Rz": "omega_Rz",
        "f1_sea": "omega1_sea",
        "f1_rare": "omega1_rare",
        "f_rf_sea": "omega_rf_sea",
        "f_rf_rare": "omega_rf_rare",
        "delta_sea_Hz": "delta_sea",
        "delta_rare_Hz": "delta_rare",
    }
    out: Dict[str, float] = dict(angular)
    for hz_key, ang_key in hz_names.items():
        out[hz_key] = angular[ang_key] / two_pi
    return out


# ---------------------------------------------------------------------------
# Geometry (dipolar_ensemble_with_rare.py:107-251)
# ---------------------------------------------------------------------------

def _platonic_vertices(n_sea: int) -> np.ndarray:
    """Unit-sphere vertices of the Platonic solid with n_sea vertices.

    Vertex order matches dipolar_ensemble_with_rare.py:117-194 (the order fixes
    which site is which qubit, so it is part of the contract).
    """
    golden = (1.0 + np.sqrt(5.0)) / 2.0
    inv_golden = 1.0 / golden
    if n_sea == 4:
        verts = [(1, 1, 1), (-1, -1, 1), (-1, 1, -1), (1, -1, -1)]
    elif n_sea == 6:
        verts = []
        for axis in range(3):
            for sgn in (1.0, -1.0):
                v = [0.0, 0.0, 0.0]
                v[axis] = sgn
                verts.append(tuple(v))
    elif n_sea == 8:
        verts = [(sx, sy, sz) for sx in (1.0, -1.0) for sy in (1.0, -1.0) for sz in (1.0, -1.0)]
    elif n_sea == 12:
        # cyclic permutations of (0, +-1, +-golden), grouped as in the reference
        verts = [
            (0.0, 1.0, golden), (0.0, -1.0, golden), (0.0, 1.0, -golden), (0.0, -1.0, -golden),
            (1.0, golden, 0.0), (-1.0, golden, 0.0), (1.0, -golden, 0.0), (-1.0, -golden, 0.0),
            (golden, 0.0, 1.0), (golden, 0.0, -1.0), (-golden, 0.0, 1.0), (-golden, 0.0, -1.0),
        ]
    elif n_sea == 20:
        verts = [(sx, sy, sz) for sx in (-1.0, 1.0) for sy in (-1.0, 1.0) for sz in (-1.0, 1.0)]
        verts += [(0.0, y, z) for y in (-inv_golden, inv_golden) for z in (-golden, golden)]
        verts += [(x, y, 0.0) for x in (-inv_golden, inv_golden) for y in (-golden, golden)]
        verts += [(x, 0.0, z) for x in (-golden, golden) for z in (-inv_golden, inv_golden)]
    else:
        raise ValueError(f"No Platonic solid with {n_sea} vertices.")
    pts = np.array(verts, dtype=float)
    return pts / np.linalg.norm(pts, axis=1, keepdims=True)


def shell_positions_with_rare_center(n_sea: int, radius: float = 0.282393) -> np.ndarray:
    """(n_sea+1, 3) positions: sea sites on a sphere of ``radius``, rare at the origin (last row).

    Platonic solids for n_sea in {4, 6, 8, 12, 20}; otherwise the Fibonacci
    sphere of dipolar_ensemble_with_rare.py:233-247.
    """
    if n_sea < 1:
        raise ValueError("n_sea must be at least 1.")
    try:
        sea = radius * _platonic_vertices(n_sea)
    except ValueError:
        golden = (1.0 + np.sqrt(5.0)) / 2.0
        sea = np.zeros((n_sea, 3), dtype=float)
        for i in range(n_sea):
            y = 1.0 - 2.0 * (i + 0.5) / n_sea
            r_xy = np.sqrt(max(0.0, 1.0 - y * y))
            azim = 2.0 * np.pi * i / golden
            sea[i] = radius * np.array([r_xy * np.cos(azim), y, r_xy * np.sin(azim)], dtype=float)
    return np.vstack([sea, np.zeros((1, 3), dtype=float)])


def dipolar_couplings_from_positions(
    positions: np.ndarray,
    scale: float,
    gamma_sea: float,
    gamma_rare: float,
) -> np.ndarray:
    """Symmetric secular dipolar couplings b_ij = g_i g_j scale (1 - 3 cos^2 th) / r^3.

    The last row of ``positions`` is the rare site (gamma_rare); theta is the
    angle of r_i - r_j to z.  dipolar_ensemble_with_rare.py:255-299.
    """
    pos = np.asarray(positions, dtype=float)
    n = pos.shape[0]
    gam = np.full(n, gamma_sea, dtype=float)
    gam[n - 1] = gamma_rare
    b = np.zeros((n, n), dtype=float)
    for i in range(n):
        for j in range(i + 1, n):
            d = pos[i] - pos[j]
            dist = np.sqrt(d.dot(d))
            if dist == 0:
                raise ValueError("Two sites have identical positions.")
            c = d[2] / dist
            geom = (1.0 - 3.0 * c**2) / (dist**3)
            b[i, j] = b[j, i] = gam[i] * gam[j] * scale * geom
    return b
