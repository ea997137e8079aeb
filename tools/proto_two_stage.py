#!/usr/bin/env python3
"""Numpy prototype of the two-stage symmetric eigensolver planned for the dense engine (design
check, not product code): dense -> band b by blocked Householder panels, band -> tridiagonal by
bulge chasing (one reflector of length <= b per task (s, t), each task touching the 3b-wide strip
[s + (t-1) b + 1, s + (t+2) b]), and the orders the GPU kernels must respect:
  * pipelined chase: task (s + 1, t) may run once tasks 0 .. t + 3 of sweep s are done;
  * Q2 Z in blocks G(s0, t) = {H(s, t): s0 <= s < s0 + nb}: s-blocks last to first, t ascending
    within a block, s descending within a group.

    python3 tools/proto_two_stage.py [n] [b] [nb]
"""
import sys

import numpy as np


def house(x):
    """v (v[0] = 1), tau, beta with (I - tau v v^T) x = beta e1 (LAPACK dlarfg)."""
    alpha = x[0]
    xn = np.linalg.norm(x[1:])
    v = np.zeros_like(x)
    v[0] = 1.0
    if xn == 0.0:
        return v, 0.0, alpha
    beta = -np.copysign(np.hypot(alpha, xn), alpha)
    tau = (beta - alpha) / beta
    v[1:] = x[1:] / (alpha - beta)
    return v, tau, beta


def sy2sb(A, b):
    """Dense symmetric -> lower band b; returns the band matrix and the panels (i, V, T)."""
    A = A.copy()
    n = len(A)
    panels = []
    for i in range(0, n - b - 1, b):
        m = n - i - b
        P = A[i + b:, i:i + b].copy()
        k = min(m, b)
        V = np.zeros((m, k))
        tau = np.zeros(k)
        for j in range(k):
            v, t, beta = house(P[j:, j])
            V[j:, j] = v
            tau[j] = t
            P[j:, j:] -= t * np.outer(v, v @ P[j:, j:])
        T = np.zeros((k, k))  # forward, columnwise (dlarft): H = I - V T V^T
        for j in range(k):
            T[:j, j] = -tau[j] * T[:j, :j] @ (V[:, :j].T @ V[:, j])
            T[j, j] = tau[j]
        A[i + b:, i:i + b] = np.triu(P)
        A[i:i + b, i + b:] = A[i + b:, i:i + b].T
        A22 = A[i + b:, i + b:]
        Y = A22 @ V @ T
        W = Y - 0.5 * V @ (T.T @ (V.T @ Y))
        A[i + b:, i + b:] = A22 - V @ W.T - W @ V.T
        panels.append((i, V, T))
    return A, panels


def chase_task(A, s, t, b, local=True):
    """Task (s, t) of the bulge chase on the full symmetric array A (in place). Returns the
    reflector (r0, v, tau) or None past the matrix."""
    n = len(A)
    if t == 0:
        col, r0 = s, s + 1
    else:
        col, r0 = s + (t - 1) * b + 1, s + t * b + 1
    if r0 > n - 1:
        return None
    r1 = min(r0 + b - 1, n - 1)
    x = A[r0:r1 + 1, col].copy()
    v, tau, beta = house(x)
    if local:
        lo, hi = col, min(n - 1, r1 + b)
    else:
        lo, hi = 0, n - 1
    J = slice(r0, r1 + 1)
    K = slice(lo, hi + 1)
    # outside the strip the rows J must be zero (what the GPU kernel will not touch)
    if local:
        outside = np.concatenate([A[J, :lo].ravel(), A[J, hi + 1:].ravel()])
        assert np.max(np.abs(outside), initial=0.0) < 1e-12, ("strip", s, t, np.max(np.abs(outside)))
    H = np.eye(r1 - r0 + 1) - tau * np.outer(v, v)
    A[J, K] = H @ A[J, K]
    A[K, J] = A[K, J] @ H
    return (r0, v, tau)


def tasks_of_sweep(n, s, b):
    t = 0
    while True:
        r0 = s + 1 if t == 0 else s + t * b + 1
        if r0 > n - 1:
            return t
        t += 1


def sb2st(B, b, order="sequential"):
    A = B.copy()
    n = len(A)
    refl = {}
    nt = [tasks_of_sweep(n, s, b) for s in range(n - 1)]
    if order == "sequential":
        seq = [(s, t) for s in range(n - 1) for t in range(nt[s])]
    else:  # the pipelined schedule: every step, each sweep advances by one task when allowed
        done = [0] * (n - 1)
        seq = []
        while any(done[s] < nt[s] for s in range(n - 1)):
            step = []
            for s in range(n - 1):
                t = done[s]
                if t >= nt[s]:
                    continue
                if s > 0 and not (done[s - 1] >= min(nt[s - 1], t + 4)):
                    continue
                step.append((s, t))
            # tasks of one step run concurrently: their strips must not overlap
            strips = []
            for s, t in step:
                lo = s if t == 0 else s + (t - 1) * b + 1
                hi = s + (t + 2) * b
                strips.append((lo, hi))
            strips.sort()
            for (a0, a1), (b0, b1) in zip(strips, strips[1:]):
                assert a1 < b0, ("concurrent strips overlap", strips)
            for s, t in step:
                done[s] += 1
            seq += step
    for s, t in seq:
        r = chase_task(A, s, t, b)
        if r is not None:
            refl[(s, t)] = r
    return A, refl, nt


def apply_q2(Z, refl, nt, b, nb):
    """V = Q2 Z in the blocked order of the GPU kernel."""
    Z = Z.copy()
    n = len(Z)
    ns = n - 1
    for s0 in reversed(range(0, ns, nb)):
        tmax = max(nt[s] for s in range(s0, min(ns, s0 + nb)))
        for t in range(tmax):
            for s in reversed(range(s0, min(ns, s0 + nb))):
                if (s, t) not in refl:
                    continue
                r0, v, tau = refl[(s, t)]
                J = slice(r0, r0 + len(v))
                Z[J, :] -= tau * np.outer(v, v @ Z[J, :])
    return Z


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    rng = np.random.default_rng(1)
    A0 = rng.standard_normal((n, n))
    A0 = A0 + A0.T
    lam0 = np.linalg.eigvalsh(A0)
    B, panels = sy2sb(A0, b)
    band_err = np.max(np.abs(np.tril(B, -b - 1)))
    print("stage 1: outside band", band_err, "eig diff", np.max(np.abs(np.linalg.eigvalsh(B) - lam0)))
    Q1 = np.eye(n)
    for i, V, T in panels:
        H = np.eye(n)
        H[i + b:, i + b:] -= V @ T @ V.T
        Q1 = Q1 @ H
    print("stage 1: Q1^T A Q1 - B", np.max(np.abs(Q1.T @ A0 @ Q1 - B)))
    Tseq, refl, nt = sb2st(B, b, "sequential")
    Tpip, refl_p, _ = sb2st(B, b, "pipelined")
    off = np.max(np.abs(np.tril(Tseq, -2)))
    print("stage 2: below subdiagonal", off, "pipelined == sequential", np.max(np.abs(Tpip - Tseq)))
    d, e = np.diag(Tseq), np.diag(Tseq, -1)
    Tt = np.diag(d) + np.diag(e, -1) + np.diag(e, 1)
    lam, Z = np.linalg.eigh(Tt)
    print("stage 2: eig diff", np.max(np.abs(lam - lam0)))
    Q2Z = apply_q2(Z, refl, nt, b, nb)
    # reference: Q2 as the product of the reflectors in sequential order
    Q2 = np.eye(n)
    for s in range(n - 1):
        for t in range(nt[s]):
            if (s, t) in refl:
                r0, v, tau = refl[(s, t)]
                H = np.eye(n)
                J = slice(r0, r0 + len(v))
                H[J, J] -= tau * np.outer(v, v)
                Q2 = Q2 @ H
    print("Q2 blocked order vs product", np.max(np.abs(Q2Z - Q2 @ Z)))
    V = Q1 @ Q2Z
    print("residual |A V - V L| / |A|", np.max(np.abs(A0 @ V - V * lam)) / np.max(np.abs(A0)),
          "orthogonality", np.max(np.abs(V.T @ V - np.eye(n))))
    print("reflectors", len(refl), "max tasks per sweep", max(nt))


if __name__ == "__main__":
    main()
