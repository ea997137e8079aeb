"""The identity the Walsh-Hadamard engine (csrc/dse_wht.hip) is built on, checked on the CPU:

    H = D_Z + W D_X W + V D_Y V^+,   W = H_had^{(x)n} (unnormalised),  V = S^{(x)n} W,
    D_X(z) = 2^-n [sum_b Re c1_b z_b + sum_{i<j} (g_ij / 2) z_i z_j]
    D_Y(z) = 2^-n [sum_b Im c1_b z_b - sum_{i<j} (g_ij / 2) z_i z_j],   z_b = 1 - 2 bit_b,

against the oracle's bitwise H (oracle/reference_model.py bitwise_apply, the include/dse.h term
conventions).  The GPU passes are checked against the same oracle in test_gpu_wht.py.
"""
import numpy as np

from oracle import reference_model as rm


def _fwht(v):
    """Unnormalised Walsh-Hadamard transform over all bits."""
    v = v.copy()
    n = v.size.bit_length() - 1
    for b in range(n):
        v = v.reshape(-1, 2, 1 << b)
        a, c = v[:, 0, :].copy(), v[:, 1, :].copy()
        v[:, 0, :], v[:, 1, :] = a + c, a - c
        v = v.reshape(-1)
    return v


def _tables(n, seed, imag_drive=False):
    rng = np.random.default_rng(seed)
    flip = np.zeros((n, 4))
    for b in range(n):
        c = (rng.standard_normal() * (0.0 if imag_drive else 1.0) + 1j * rng.standard_normal()) * 1e3
        flip[b] = [c.real, c.imag, c.real, -c.imag]   # (re0, im0) = conj(re1, im1): (re1, im1) = c*
    return {"n": n, "field": rng.standard_normal(n) * 500.0,
            "zz": np.triu(rng.standard_normal((n, n)), 1) * 300.0,
            "pair": np.triu(rng.standard_normal((n, n)), 1) * 100.0, "flip": flip, "shift": 17.0}


def _wht_apply(t, psi):
    n = t["n"]
    x = np.arange(1 << n)
    z = [1.0 - 2.0 * ((x >> b) & 1) for b in range(n)]
    pc = np.array([bin(int(i)).count("1") for i in x])
    dx = np.zeros(1 << n)
    dy = np.zeros(1 << n)
    for b in range(n):
        dx += t["flip"][b, 2] * z[b]
        dy += t["flip"][b, 3] * z[b]
        for j in range(b + 1, n):
            dx += 0.5 * t["pair"][b, j] * z[b] * z[j]
            dy -= 0.5 * t["pair"][b, j] * z[b] * z[j]
    sc = 2.0 ** -n
    diag_only = dict(t, flip=np.zeros_like(t["flip"]), pair=np.zeros_like(t["pair"]))
    out = rm.bitwise_apply(diag_only, psi)                         # D_Z psi
    out = out + _fwht(sc * dx * _fwht(psi))                         # W D_X W psi
    u = _fwht((-1j) ** pc * psi)                                    # W S^+ psi
    out = out + (1j) ** pc * _fwht(sc * dy * u)                     # S W D_Y W S^+ psi
    return out


def test_wht_identity_matches_bitwise_h():
    for n, seed, imag in ((1, 1, False), (2, 2, False), (5, 3, False), (7, 4, True), (8, 5, False)):
        t = _tables(n, seed, imag)
        rng = np.random.default_rng(seed)
        psi = rng.standard_normal(1 << n) + 1j * rng.standard_normal(1 << n)
        ref = rm.bitwise_apply(t, psi)
        got = _wht_apply(t, psi)
        assert np.max(np.abs(got - ref)) <= 1e-12 * np.max(np.abs(ref)), (n, seed)
