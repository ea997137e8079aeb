"""Kronecker-product restatement of the reference Hamiltonian (TEST INFRASTRUCTURE).

Independent of ``quantumsimulations_amd``: this builds H exactly the way the
reference does -- local 2x2 spin operators embedded with Kronecker products,
site 0 as the most significant factor -- but with scipy.sparse instead of QuTiP.

Reference map (TimHarrelson/QuantumSimulations, dipolar_ensemble_with_rare.py):
    local operators          :15-19
    embed / total over sea   :37-52
    derived frequencies      :387-450
    geometry + couplings     :107-299
    Hamiltonian + observables:453-588
    initial product state    :591-606
"""
from __future__ import annotations

from itertools import combinations
from typing import Dict, List, Tuple

import numpy as np
import scipy.sparse as sp

SX = np.array([[0.0, 1.0], [1.0, 0.0]], dtype=complex)
SY = np.array([[0.0, -1.0j], [1.0j, 0.0]], dtype=complex)
SZ = np.array([[1.0, 0.0], [0.0, -1.0]], dtype=complex)
IX, IY, IZ = 0.5 * SX, 0.5 * SY, 0.5 * SZ          # :16-18
ID2 = np.eye(2, dtype=complex)

OBS_ORDER = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R")


def embed(op: np.ndarray, site: int, n_sites: int) -> sp.csr_matrix:
    """op on ``site`` of an n_sites register; site 0 is the leftmost Kronecker factor (:37-45)."""
    left = sp.identity(2 ** site, dtype=complex, format="csr")
    right = sp.identity(2 ** (n_sites - site - 1), dtype=complex, format="csr")
    return sp.kron(sp.kron(left, sp.csr_matrix(op)), right, format="csr")


def total(op: np.ndarray, sites: List[int], n_sites: int) -> sp.csr_matrix:
    acc = sp.csr_matrix((2 ** n_sites, 2 ** n_sites), dtype=complex)
    for s in sites:
        acc = acc + embed(op, s, n_sites)
    return acc


def derived_frequencies(p: Dict) -> Dict[str, float]:
    """:387-450 (keys restricted to what H needs plus the Hz copies used in fixtures)."""
    wA = p["gamma_sea"] * p["B0_sea"]
    wR = p["gamma_rare"] * p["B0_rare"]
    w1A = p["gamma_sea"] * p["B1_sea"]
    w1R = p["gamma_rare"] * p["B1_rare"]
    rfA = wA if p["omega_rf_sea"] is None else p["omega_rf_sea"]
    rfR = wR if p["omega_rf_rare"] is None else p["omega_rf_rare"]
    dA = wA - rfA if p["drive_sea"] else 0.0
    dR = wR - rfR if p["drive_rare"] else 0.0
    return {"omega_Az": wA, "omega_Rz": wR, "omega1_sea": w1A, "omega1_rare": w1R,
            "omega_rf_sea": rfA, "omega_rf_rare": rfR, "delta_sea": dA, "delta_rare": dR}


def positions(n_sea: int, radius: float) -> np.ndarray:
    """:205-251 with the Platonic vertex tables of :107-202."""
    phi = (1.0 + np.sqrt(5.0)) / 2.0
    ip = 1.0 / phi
    table = {
        4: [[1, 1, 1], [-1, -1, 1], [-1, 1, -1], [1, -1, -1]],
        6: [[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]],
        8: [[1, 1, 1], [1, 1, -1], [1, -1, 1], [1, -1, -1],
            [-1, 1, 1], [-1, 1, -1], [-1, -1, 1], [-1, -1, -1]],
        12: [[0, 1, phi], [0, -1, phi], [0, 1, -phi], [0, -1, -phi],
             [1, phi, 0], [-1, phi, 0], [1, -phi, 0], [-1, -phi, 0],
             [phi, 0, 1], [phi, 0, -1], [-phi, 0, 1], [-phi, 0, -1]],
    }
    if n_sea == 20:
        pts = [[x, y, z] for x in (-1.0, 1.0) for y in (-1.0, 1.0) for z in (-1.0, 1.0)]
        pts += [[0.0, y, z] for y in (-ip, ip) for z in (-phi, phi)]
        pts += [[x, y, 0.0] for x in (-ip, ip) for y in (-phi, phi)]
        pts += [[x, 0.0, z] for x in (-phi, phi) for z in (-ip, ip)]
        table[20] = pts
    if n_sea in table:
        v = np.array(table[n_sea], dtype=float)
        sea = radius * (v / np.linalg.norm(v, axis=1, keepdims=True))
    else:
        sea = np.zeros((n_sea, 3))
        for i in range(n_sea):
            y = 1.0 - 2.0 * (i + 0.5) / n_sea
            rxy = np.sqrt(max(0.0, 1.0 - y * y))
            ang = 2.0 * np.pi * i / phi
            sea[i] = radius * np.array([rxy * np.cos(ang), y, rxy * np.sin(ang)])
    return np.vstack([sea, np.zeros((1, 3))])


def couplings(pos: np.ndarray, scale: float, g_sea: float, g_rare: float) -> np.ndarray:
    """:255-299."""
    n = pos.shape[0]
    b = np.zeros((n, n))
    for i, j in combinations(range(n), 2):
        r = pos[i] - pos[j]
        d = np.linalg.norm(r)
        c = r[2] / d
        gi = g_rare if i == n - 1 else g_sea
        gj = g_rare if j == n - 1 else g_sea
        b[i, j] = b[j, i] = gi * gj * scale * ((1.0 - 3.0 * c ** 2) / d ** 3)
    return b


def build(p: Dict) -> Tuple[sp.csr_matrix, Dict[str, sp.csr_matrix], np.ndarray, Dict]:
    """(H, observables, psi0, aux) for a parameter dict with DipolarRareParams field names.

    Follows :453-606 term by term (including the -1/4 (IxIx - IyIy) pair term
    and the shell-geometry re-labelling n_sea := n_total).
    """
    if p.get("is_spin_three_half", False):
        raise ValueError("spin-3/2 rare spin is not constructible in the reference (dims mismatch)")
    n_sea = p["n_sea"]
    n_tot = n_sea + 1
    rare = n_sea
    center = p["is_center_rare"]
    n_s = n_sea if center else n_tot
    sea = list(range(n_s))
    f = derived_frequencies(p)
    dim = 2 ** n_tot
    H = sp.csr_matrix((dim, dim), dtype=complex)
    if p["drive_sea"] and f["delta_sea"] != 0.0:
        H = H + f["delta_sea"] * total(IZ, sea, n_tot)
    if center and p["drive_rare"] and f["delta_rare"] != 0.0:
        H = H + f["delta_rare"] * embed(IZ, rare, n_tot)
    if p["drive_sea"] and f["omega1_sea"] != 0.0:
        H = H + f["omega1_sea"] * (np.cos(p["phi_sea"]) * total(IX, sea, n_tot)
                                   + np.sin(p["phi_sea"]) * total(IY, sea, n_tot))
    if center and p["drive_rare"] and f["omega1_rare"] != 0.0:
        H = H + f["omega1_rare"] * (np.cos(p["phi_rare"]) * embed(IX, rare, n_tot)
                                    + np.sin(p["phi_rare"]) * embed(IY, rare, n_tot))
    pos = positions(n_sea, p["shell_scale"])
    b = couplings(pos, p["dipolar_scale"], p["gamma_sea"],
                  p["gamma_rare"] if center else p["gamma_sea"])
    for i, j in combinations(range(n_tot), 2):
        if i < n_s and j < n_s:
            zi, zj = embed(IZ, i, n_tot), embed(IZ, j, n_tot)
            xi, xj = embed(IX, i, n_tot), embed(IX, j, n_tot)
            yi, yj = embed(IY, i, n_tot), embed(IY, j, n_tot)
            H = H + b[i, j] * (zi @ zj - 0.25 * (xi @ xj - yi @ yj))
        elif i == rare or j == rare:
            s = i if j == rare else j
            H = H + b[i, j] * (embed(IZ, s, n_tot) @ embed(IZ, rare, n_tot))
    obs = {
        "Ix_sea": total(IX, sea, n_tot), "Iy_sea": total(IY, sea, n_tot),
        "Iz_sea": total(IZ, sea, n_tot), "Iz_R": embed(IZ, rare, n_tot),
        "Ix_R": embed(IX, rare, n_tot), "Iy_R": embed(IY, rare, n_tot),
    }
    sea_idx = 0 if p["init_x_sign"] >= 0 else 1
    rare_idx = 0 if -p["init_x_sign"] >= 0 else 1
    bits = [sea_idx] * n_tot
    if center:
        bits[rare] = rare_idx
    index = 0
    for s in range(n_tot):
        index = (index << 1) | bits[s]
    psi0 = np.zeros(dim, dtype=complex)
    psi0[index] = 1.0
    return H.tocsr(), obs, psi0, {"freqs": f, "positions": pos, "b": b, "psi0_index": index}


def bitwise_apply(tables: Dict[str, np.ndarray], psi: np.ndarray) -> np.ndarray:
    """H psi from engine coefficient tables (numpy, vectorised over the basis).

    ``tables`` holds n, field, zz, pair, flip, shift in register-bit order, with
    the same meaning as ``include/dse.h`` (s_b = 1/2 - bit_b, flip index = output bit).
    Used to check the product's table builder against ``build`` and to check the
    GPU kernels at sizes where a CSR matrix is too large.
    """
    n = int(tables["n"])
    x = np.arange(1 << n, dtype=np.int64)
    bits = [((x >> b) & 1) for b in range(n)]
    s = [0.5 - bt for bt in bits]
    diag = np.full(x.shape, float(tables["shift"]))
    for k in range(n):
        diag += tables["field"][k] * s[k]
    for i in range(n):
        for j in range(i + 1, n):
            if tables["zz"][i, j] != 0.0:
                diag += tables["zz"][i, j] * (s[i] * s[j])
    out = diag * psi
    for k in range(n):
        f = tables["flip"][k]
        if not np.any(f != 0.0):
            continue
        c = np.where(bits[k] == 0, f[0] + 1j * f[1], f[2] + 1j * f[3])
        out = out + c * psi[x ^ (1 << k)]
    for i in range(n):
        for j in range(i + 1, n):
            g = tables["pair"][i, j]
            if g == 0.0:
                continue
            eq = bits[i] == bits[j]
            out = out + np.where(eq, g, 0.0) * psi[x ^ ((1 << i) | (1 << j))]
    return out


def observables_bitwise(psi: np.ndarray, n: int, sea_mask: int, rare_bit: int,
                        rare_z_const: float = 0.0) -> np.ndarray:
    """The six expectations + norm of a register state (un-normalised sums, then / norm^2)."""
    x = np.arange(1 << n, dtype=np.int64)
    p2 = np.abs(psi) ** 2
    norm2 = p2.sum()
    res = np.zeros(7)
    for k in range(n):
        if not (sea_mask >> k) & 1:
            continue
        lo = ((x >> k) & 1) == 0
        ov = np.sum(np.conj(psi[lo]) * psi[x[lo] ^ (1 << k)])
        res[0] += ov.real
        res[1] += ov.imag
        res[2] += np.sum(p2 * (0.5 - ((x >> k) & 1)))
    if rare_bit >= 0:
        k = rare_bit
        lo = ((x >> k) & 1) == 0
        ov = np.sum(np.conj(psi[lo]) * psi[x[lo] ^ (1 << k)])
        res[3] = np.sum(p2 * (0.5 - ((x >> k) & 1)))
        res[4] = ov.real
        res[5] = ov.imag
    else:
        res[3] = rare_z_const * norm2
    res[:6] /= norm2
    res[6] = np.sqrt(norm2)
    return res
