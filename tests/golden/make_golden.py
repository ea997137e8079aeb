"""Generate the golden fixtures in tests/golden/ from the reference's own code.

Run ONLY in the build container (it reads /root/reference, which the GPU box
does not have):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

How: QuTiP is not installed (and cannot be installed offline), so the
reference's ``dipolar_ensemble_with_rare.py`` is imported *by path* with
``tests/golden/_qutip_standin`` first on sys.path, a minimal stand-in for the
QuTiP calls it makes (Kronecker products, Qobj arithmetic, eigenstates and an
``sesolve`` restating QuTiP 5's ZVODE-Adams integrator).  Everything physical
-- which terms, their coefficients, the site ordering, the initial state, the
observables, the geometry and the derived frequencies -- therefore comes from
the reference's own functions.  No reference source is copied; only the
numbers it produces are stored here.

Sweep-point parameters are formed with the expressions of
sweep_sea_detuning.py:414-668 and the __main__ constants of :1201-1251.

Fixtures written (all small):
  geometry.npz         positions / couplings for several n_sea
  freqs.json           get_derived_frequencies for sweep points (3 variants x 5 detunings)
  hamiltonian_n7.npz   H (CSR), psi0 index, O @ v for N = 7, 3 variants x 3 detunings
  hpsi_n12.npz         H @ v and <v|O|v> for a seeded random v, N = 12, 3 variants
  traces_n7.npz        N = 7, delta = 50 kHz, t_final 2e-3, 201 points, 3 variants:
                       exact (eigh of the reference H) + simulate_rare (ZVODE at the
                       sweep's tolerances) + tight ZVODE (rtol 1e-13, atol 1e-14)
  traces_n12.npz       N = 12 center_on, same grid: exact + simulate_rare
"""
from __future__ import annotations

import dataclasses
import importlib.util
import json
import os
import sys
import time

import numpy as np
import scipy.linalg as la

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

sys.path.insert(0, os.path.join(HERE, "_qutip_standin"))
import qutip  # noqa: E402  (the stand-in)


def _load_reference():
    spec = importlib.util.spec_from_file_location(
        "ref_dipolar", os.path.join(REF, "dipolar_ensemble_with_rare.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["ref_dipolar"] = mod
    spec.loader.exec_module(mod)
    return mod


ref = _load_reference()

# --- sweep constants (sweep_sea_detuning.py:1201-1251) ---
GAMMA_SEA = 8.1812e7
GAMMA_RARE = 6.976e7
B0 = 3.0
F_AZ = GAMMA_SEA * B0 / (2 * np.pi)
F1A = 50_000
TARGET = F1A
PHI = (np.pi / 2.0) * 1.0
SWEEP_TOL = dict(solver_atol=1e-10, solver_rtol=1e-9, solver_nsteps=10_000_000, solver_max_step=1e-5)


def sweep_params(n_sea, delta_hz, variant, t_final, steps, f1a=F1A, target=TARGET, tol=SWEEP_TOL):
    """sweep_sea_detuning.py:414-668 for one (detuning, variant)."""
    lhs_sq = target ** 2 + f1a ** 2                               # f1R_for_resonance :1168-1194
    f1r = (lhs_sq - 0.0 ** 2) ** 0.5
    b0 = 2 * np.pi * F_AZ / GAMMA_SEA
    f_rz = GAMMA_RARE * b0 / (2 * np.pi)
    b1_sea = 2 * np.pi * f1a / GAMMA_SEA
    b1_rare = 2 * np.pi * f1r / GAMMA_RARE
    f_rf_sea = F_AZ - delta_hz
    base = ref.DipolarRareParams(
        n_sea=n_sea, gamma_sea=GAMMA_SEA, gamma_rare=GAMMA_RARE, B0_sea=b0, B0_rare=b0,
        B1_sea=b1_sea, B1_rare=b1_rare, omega_rf_sea=2 * np.pi * f_rf_sea,
        omega_rf_rare=2 * np.pi * f_rz, phi_sea=PHI, phi_rare=PHI,
        dipolar_scale=1.0e-7 * 1.054571817e-34, shell_scale=0.282393e-9,
        t_final=t_final, steps=steps, drive_sea=True, drive_rare=False, init_x_sign=-1,
        init_rare_level=3, is_spin_three_half=False, is_center_rare=True, **tol)
    if variant == "center_off":
        return dataclasses.replace(base, drive_rare=False, is_center_rare=True)
    if variant == "center_on":
        return dataclasses.replace(base, drive_rare=True, is_center_rare=True)
    if variant == "shell_off":
        return dataclasses.replace(base, drive_rare=False, is_center_rare=False)
    raise ValueError(variant)


VARIANTS = ("center_off", "center_on", "shell_off")
OBS = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R")


def rand_state(dim, seed=1234):
    rng = np.random.default_rng(seed)
    v = rng.standard_normal(dim) + 1j * rng.standard_normal(dim)
    return v / np.linalg.norm(v)


def exact_trace(H, psi0, t, eops):
    w, V = la.eigh(H.full())
    c0 = V.conj().T @ psi0
    st = (V @ (np.exp(-1j * np.outer(w, t)) * c0[:, None])).T
    out = {k: np.real(np.einsum("td,td->t", st.conj(), (eops[k].data @ st.T).T)) for k in OBS}
    out["state_norm"] = np.linalg.norm(st, axis=1)
    return out


def main():
    t_start = time.time()
    # 1. geometry + couplings
    geo = {}
    for n in (1, 2, 3, 4, 5, 6, 7, 8, 11, 12, 13, 20, 29):
        pos = ref.shell_positions_with_rare_center(n, radius=0.282393e-9)
        geo[f"pos_{n}"] = pos
        geo[f"b_center_{n}"] = ref.dipolar_couplings_from_positions(
            pos, 1.0e-7 * 1.054571817e-34, GAMMA_SEA, GAMMA_RARE)
        geo[f"b_shell_{n}"] = ref.dipolar_couplings_from_positions(
            pos, 1.0e-7 * 1.054571817e-34, GAMMA_SEA, GAMMA_SEA)
    np.savez(os.path.join(HERE, "geometry.npz"), **geo)

    # 2. derived frequencies at sweep points
    rows = []
    for v in VARIANTS:
        for d in (0.0, 12500.0, 25000.0, 50000.0, 150000.0):
            p = sweep_params(6, d, v, 2e-3, 201)
            rows.append({"variant": v, "delta_Hz": d, "params": dataclasses.asdict(p),
                         "freqs": ref.get_derived_frequencies(p)})
    with open(os.path.join(HERE, "freqs.json"), "w") as f:
        json.dump(rows, f, indent=1)

    # 3. Hamiltonians at N = 7
    h7 = {}
    for v in VARIANTS:
        for d in (0.0, 25000.0, 150000.0):
            p = sweep_params(6, d, v, 2e-3, 201)
            H, eops = ref.build_hamiltonian_rare(p)
            psi0 = ref.initial_state_rare(p).full().ravel()
            key = f"{v}_{int(d)}"
            m = H.data.tocsr()
            m.sort_indices()
            h7[f"{key}_data"], h7[f"{key}_indices"], h7[f"{key}_indptr"] = m.data, m.indices, m.indptr
            h7[f"{key}_psi0_index"] = int(np.argmax(np.abs(psi0)))
            vec = rand_state(m.shape[0], 7)
            h7[f"{key}_v"] = vec
            for k in OBS:
                h7[f"{key}_O_{k}"] = eops[k].data @ vec
    np.savez(os.path.join(HERE, "hamiltonian_n7.npz"), **h7)

    # 4. H @ v at N = 12
    h12 = {}
    for v in VARIANTS:
        p = sweep_params(11, 50000.0, v, 2e-3, 201)
        H, eops = ref.build_hamiltonian_rare(p)
        vec = rand_state(H.shape[0], 1234)
        h12[f"{v}_v"] = vec
        h12[f"{v}_Hv"] = H.data @ vec
        h12[f"{v}_psi0_index"] = int(np.argmax(np.abs(ref.initial_state_rare(p).full().ravel())))
        for k in OBS:
            h12[f"{v}_expect_{k}"] = np.real(np.vdot(vec, eops[k].data @ vec))
    np.savez(os.path.join(HERE, "hpsi_n12.npz"), **h12)

    # 5. traces at N = 7
    tr7 = {}
    for v in VARIANTS:
        p = sweep_params(6, 50000.0, v, 2e-3, 201)
        H, eops = ref.build_hamiltonian_rare(p)
        psi0 = ref.initial_state_rare(p).full().ravel()
        t, obs_ref = ref.simulate_rare(p)
        tr7[f"{v}_rhs_ref"] = qutip.LAST_SOLVE_INFO["rhs"]
        ex = exact_trace(H, psi0, t, eops)
        ptight = dataclasses.replace(p, solver_atol=1e-14, solver_rtol=1e-13)
        _, obs_tight = ref.simulate_rare(ptight)
        tr7["t"] = t
        for k in OBS + ("state_norm",):
            tr7[f"{v}_exact_{k}"] = ex[k]
            tr7[f"{v}_ref_{k}"] = obs_ref[k]
            tr7[f"{v}_tight_{k}"] = obs_tight[k]
        print(v, "N=7 exact-vs-ref", max(np.max(np.abs(ex[k] - obs_ref[k])) for k in OBS),
              "exact-vs-tight", max(np.max(np.abs(ex[k] - obs_tight[k])) for k in OBS), flush=True)
    np.savez(os.path.join(HERE, "traces_n7.npz"), **tr7)

    # 6. trace at N = 12, center_on
    tr12 = {}
    p = sweep_params(11, 50000.0, "center_on", 2e-3, 201)
    H, eops = ref.build_hamiltonian_rare(p)
    psi0 = ref.initial_state_rare(p).full().ravel()
    ex = exact_trace(H, psi0, np.linspace(0.0, p.t_final, p.steps), eops)
    t, obs_ref = ref.simulate_rare(p)
    tr12["t"] = t
    tr12["rhs_ref"] = qutip.LAST_SOLVE_INFO["rhs"]
    for k in OBS + ("state_norm",):
        tr12[f"exact_{k}"] = ex[k]
        tr12[f"ref_{k}"] = obs_ref[k]
    print("N=12 exact-vs-ref", max(np.max(np.abs(ex[k] - obs_ref[k])) for k in OBS), flush=True)
    np.savez(os.path.join(HERE, "traces_n12.npz"), **tr12)
    print(f"done in {time.time() - t_start:.1f} s")


if __name__ == "__main__":
    main()
