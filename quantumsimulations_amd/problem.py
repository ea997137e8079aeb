"""Reduce a ``DipolarRareParams`` to the coefficient tables the HIP engine consumes.

The reference builds H as a sum of Kronecker-embedded QuTiP operators
(``build_hamiltonian_rare``, dipolar_ensemble_with_rare.py:453-588).  Every
term there is a Pauli-like bit operation on qubits, so the engine only needs,
per register bit b (s_b(x) = 1/2 - bit_b(x), bit value 0 = spin up):

* ``field[b]``       diagonal  D(x) += field[b] * s_b(x)          (detunings, :505-512)
* ``zz[i, j]``       diagonal  D(x) += zz[i, j] * s_i(x) s_j(x)   (secular ZZ, :559-568), i < j
* ``pair[i, j]``     <x ^ e_i ^ e_j| H |x> = pair[i, j] when bit_i(x) == bit_j(x), i < j
                     (the -1/4 (IxIx - IyIy) "double-quantum" term, :559-561: pair = -b/8)
* ``flip[b]``        <x ^ e_b| H |x> = flip[b, 2v] + i flip[b, 2v+1] where v is the bit value
                     of the *output* state (rf drives, :515-530)
* ``shift``          constant energy offset

Qubit -> bit mapping ("order"):

* ``"reference"``: site 0 is the most significant bit (QuTiP ``tensor`` order), so
  state vectors are directly comparable with the reference's ``Qobj.full()``.
* ``"engine"``: bit b = site b, so the rare site (last site) is the top bit and
  lands outside the LDS tile (its only off-diagonal term is its own drive).

When the rare spin sits at the center and is not driven, its bit is conserved
(sea-rare coupling is ZZ only, :562-568); with ``reduce=True`` the register then
holds only the sea spins and the rare spin enters as a static field.  This is
exact and halves the state.
"""
from __future__ import annotations

from dataclasses import dataclass, field as dc_field
from typing import Dict, Tuple

import numpy as np

from .model import (
    DipolarRareParams,
    dipolar_couplings_from_positions,
    get_derived_frequencies,
    shell_positions_with_rare_center,
)

OBS_NAMES: Tuple[str, ...] = ("Ix_sea", "Iy_sea", "Iz_sea", "Iz_R", "Ix_R", "Iy_R", "state_norm")


@dataclass
class Problem:
    n_qubits: int
    field: np.ndarray          # (n,)
    zz: np.ndarray             # (n, n) upper triangle used
    pair: np.ndarray           # (n, n) upper triangle used
    flip: np.ndarray           # (n, 4): re0, im0, re1, im1
    shift: float
    psi0_index: int
    sea_mask: int
    rare_bit: int              # -1 when the rare spin is not in the register
    rare_z_const: float        # <Iz_R> when the rare spin is not in the register
    site_of_bit: np.ndarray    # reference site index of every register bit
    n_sites: int
    reduced: bool
    order: str
    meta: Dict[str, float] = dc_field(default_factory=dict)

    @property
    def dim(self) -> int:
        return 1 << self.n_qubits


def _validate(params: DipolarRareParams) -> None:
    if params.is_spin_three_half:
        # The reference forces the rare local dimension to 2 in the center geometry
        # (dipolar_ensemble_with_rare.py:486) and then multiplies 4x4 rare operators
        # into it; in the shell geometry it embeds 2x2 sea operators on a 4-level site.
        # Both raise a dimension mismatch inside QuTiP.  We raise the same way.
        raise ValueError(
            "is_spin_three_half=True is not constructible in the reference model "
            "(operator dimension mismatch, dipolar_ensemble_with_rare.py:486/499-501)"
        )
    if params.n_sea < 1:
        raise ValueError("n_sea must be at least 1.")


def site_tables(params: DipolarRareParams):
    """Per-site coefficient tables of the full (unreduced) Hamiltonian, site-indexed.

    Returns (field, zz, pair, flip, sea_sites, rare_site, psi0_bits, freqs, b).
    """
    _validate(params)
    n_sea = params.n_sea
    n_sites = n_sea + 1
    rare = n_sea
    center = bool(params.is_center_rare)
    n_s = n_sea if center else n_sites          # :488-489  (shell: every site is "sea")
    sea_sites = list(range(n_s))

    freqs = get_derived_frequencies(params)
    w1_sea, w1_rare = freqs["omega1_sea"], freqs["omega1_rare"]
    d_sea, d_rare = freqs["delta_sea"], freqs["delta_rare"]

    field = np.zeros(n_sites)
    zz = np.zeros((n_sites, n_sites))
    pair = np.zeros((n_sites, n_sites))
    flip = np.zeros((n_sites, 4))

    if params.drive_sea and d_sea != 0.0:                      # :505-508
        for k in sea_sites:
            field[k] += d_sea
    if center and params.drive_rare and d_rare != 0.0:         # :510-512
        field[rare] += d_rare

    def _drive(w1: float, phi: float) -> np.ndarray:
        # w1 (cos(phi) Ix + sin(phi) Iy):  <1|.|0> = w1/2 e^{+i phi},  <0|.|1> = w1/2 e^{-i phi}
        re = w1 * (np.cos(phi) * 0.5)
        im = w1 * (np.sin(phi) * 0.5)
        return np.array([re, -im, re, im])

    if params.drive_sea and w1_sea != 0.0:                     # :515-519
        for k in sea_sites:
            flip[k] = _drive(w1_sea, params.phi_sea)
    if center and params.drive_rare and w1_rare != 0.0:        # :523-528
        flip[rare] = _drive(w1_rare, params.phi_rare)

    positions = shell_positions_with_rare_center(n_sea, radius=params.shell_scale)   # :533-536
    if positions.shape != (n_sites, 3):
        raise RuntimeError("Shell geometry returned unexpected number of sites.")
    b = dipolar_couplings_from_positions(                      # :540-545
        positions, params.dipolar_scale, params.gamma_sea,
        params.gamma_rare if center else params.gamma_sea,
    )
    for i in range(n_sites):                                   # :549-568
        for j in range(i + 1, n_sites):
            if i < n_s and j < n_s:
                zz[i, j] = b[i, j]
                pair[i, j] = b[i, j] * -0.125
            elif i == rare or j == rare:
                zz[i, j] = b[i, j]

    sea_bit = 0 if params.init_x_sign >= 0 else 1              # :599, basis_sea :70-72
    rare_bit_val = 0 if -params.init_x_sign >= 0 else 1        # :602, basis_rare argmax/argmin of Iz
    psi0_bits = [sea_bit] * n_sites
    if center:
        psi0_bits[rare] = rare_bit_val
    return field, zz, pair, flip, sea_sites, rare, psi0_bits, freqs, b


def build_problem(params: DipolarRareParams, order: str = "engine", reduce: bool = True) -> Problem:
    """Coefficient tables of ``params`` in the requested register order (see module doc)."""
    if order not in ("engine", "reference"):
        raise ValueError("order must be 'engine' or 'reference'")
    field_s, zz_s, pair_s, flip_s, sea_sites, rare, psi0_bits, freqs, b = site_tables(params)
    n_sites = params.n_sea + 1
    center = bool(params.is_center_rare)
    rare_flipped = bool(np.any(flip_s[rare] != 0.0))
    reduced = bool(reduce and center and not rare_flipped)

    sites = list(range(params.n_sea)) if reduced else list(range(n_sites))
    n = len(sites)
    if order == "engine":
        bit_of_site = {s: i for i, s in enumerate(sites)}
    else:
        bit_of_site = {s: n - 1 - i for i, s in enumerate(sites)}
    site_of_bit = np.empty(n, dtype=np.int64)
    for s, bt in bit_of_site.items():
        site_of_bit[bt] = s

    field = np.zeros(n)
    zz = np.zeros((n, n))
    pair = np.zeros((n, n))
    flip = np.zeros((n, 4))
    shift = 0.0
    rare_z_const = 0.0
    for s in sites:
        field[bit_of_site[s]] = field_s[s]
        flip[bit_of_site[s]] = flip_s[s]
    if reduced:
        s_r = 0.5 - psi0_bits[rare]
        rare_z_const = s_r
        for s in sites:
            # b_sR s_s s_R with s_R frozen  ->  static field on the sea spin
            a, c = min(s, rare), max(s, rare)
            field[bit_of_site[s]] += zz_s[a, c] * s_r
        shift += field_s[rare] * s_r
    for ia, sa in enumerate(sites):
        for sb in sites[ia + 1:]:
            i, j = bit_of_site[sa], bit_of_site[sb]
            lo, hi = min(i, j), max(i, j)
            zz[lo, hi] = zz_s[sa, sb]
            pair[lo, hi] = pair_s[sa, sb]

    psi0 = 0
    for s in sites:
        psi0 |= psi0_bits[s] << bit_of_site[s]
    sea_mask = 0
    for s in sea_sites:
        if s in bit_of_site:
            sea_mask |= 1 << bit_of_site[s]
    rare_bit = -1 if reduced else bit_of_site[rare]

    meta = {"delta_sea": freqs["delta_sea"], "delta_rare": freqs["delta_rare"],
            "omega1_sea": freqs["omega1_sea"], "omega1_rare": freqs["omega1_rare"]}
    return Problem(n, field, zz, pair, flip, shift, psi0, sea_mask, rare_bit, rare_z_const,
                   site_of_bit, n_sites, reduced, order, meta)


def spectral_bounds(prob: Problem) -> Tuple[float, float]:
    """Rigorous [E_min, E_max] of H by Weyl's inequality over one- and two-qubit pieces.

    One-qubit piece of bit k: field_k Iz + drive -> eigenvalues +-sqrt(field^2/4 + |c|^2).
    Two-qubit piece (i, j): zz s_i s_j + pair flip -> {zz/4 +- |g|} U {-zz/4}.
    Exact for the non-interacting part, which dominates the spectral width.
    (Mirrors dse_spectral_bounds in the C library; used by host-side tests.)
    """
    lo = hi = prob.shift
    n = prob.n_qubits
    for k in range(n):
        c = np.hypot(prob.flip[k, 2], prob.flip[k, 3])
        r = np.sqrt(0.25 * prob.field[k] ** 2 + c * c)
        lo -= r
        hi += r
    for i in range(n):
        for j in range(i + 1, n):
            q, g = 0.25 * prob.zz[i, j], abs(prob.pair[i, j])
            lo += min(q - g, -q)
            hi += max(q + g, -q)
    return lo, hi


def time_grid(params: DipolarRareParams) -> np.ndarray:
    """Output times, dipolar_ensemble_with_rare.py:620-626."""
    if params.steps < 2 or params.t_final <= 0.0:
        raise ValueError("Bad time grid: steps >= 2 and t_final > 0.")
    return np.linspace(0.0, params.t_final, params.steps)
