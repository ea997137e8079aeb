"""Index-level check of the bulge chase's hand-off protocol (csrc/dse_eig2.hip, k_sb2st_pf), CPU only.

Task (s, t) of sweep s touches three blocks of the band (lower storage): L = A(r0 .. r0+m-1,
col .. col+nL-1), D = A(r0 .. r0+m-1, r0 .. r0+m-1) (i >= j), R = A(r0+m .. r0+m+mr-1, r0 .. r0+m-1),
with col = s, r0 = s + 1 for t = 0 and col = s + (t-1) b + 1, r0 = s + t b + 1 after.  The kernel
lets task (s, t) run once task (s-1, t+1) is done and task (s-1, t+2) has published its beta,
prefetches D and R of task t + 1 during task t, and carries R of task t in registers as the L of
task t + 1.  That is valid when (checked here for every task of a few (n, b)):

* (s, t) and the concurrently running (s-1, t+2) share exactly one entry, E = R_t(b-1, b-1) =
  L_{(s-1, t+2)}(0, 0), the head of the column (s-1, t+2) annihilates (handed over by mailbox);
* no task (s-1, t') with t' >= t + 2 touches D_t or R_t other than E (so the prefetch, issued
  after (s-1, t+1) is done, reads final values);
* no task (s-1, t') with t' >= t + 1 touches the carried L_t, other than (s-1, t+1)'s annihilated
  head (the entry task (s, t-1) took from the mailbox);
* task t's R is task t+1's L (same entries), and R exists exactly when task t + 1 exists.
"""
import pytest


def tasks(n, b, s):
    return 1 + (n - 2 - s) // b


def blocks(n, b, s, t):
    col = s if t == 0 else s + (t - 1) * b + 1
    r0 = s + 1 if t == 0 else s + t * b + 1
    m = min(b, n - r0)
    nl = 1 if t == 0 else b
    mr = max(0, min(b, n - r0 - m))
    L = {(r0 + i, col + j) for i in range(m) for j in range(nl)}
    D = {(r0 + i, r0 + j) for i in range(m) for j in range(m) if i >= j}
    R = {(r0 + m + i, r0 + j) for i in range(mr) for j in range(m)}
    return L, D, R, (r0, col, m, mr)


@pytest.mark.parametrize("n,b", [(40, 4), (67, 4), (100, 8), (131, 8)])
def test_chase_prefetch_and_mailbox_protocol(n, b):
    for s in range(1, n - 1):
        nt, ntp = tasks(n, b, s), tasks(n, b, s - 1)
        for t in range(nt):
            L, D, R, (r0, col, m, mr) = blocks(n, b, s, t)
            mine = L | D | R
            e = (s + (t + 2) * b, s + (t + 1) * b)
            # the concurrently running producer
            if t + 2 < ntp:
                pl, pd, pr, _ = blocks(n, b, s - 1, t + 2)
                shared = mine & (pl | pd | pr)
                assert shared <= {e}, (s, t, sorted(shared))
                assert (e in R) == (mr == b), (s, t)
            # nothing later in sweep s - 1 touches the prefetched D / R but E
            for tp in range(t + 2, ntp):
                ql, qd, qr, _ = blocks(n, b, s - 1, tp)
                assert not ((D | R) - {e}) & (ql | qd | qr), (s, t, tp)
            # the carried L: untouched by (s-1, t') for t' >= t+2; (s-1, t+1) only at its own head
            if t >= 1:
                head = (s + (t + 1) * b, s + t * b)  # R_{t-1}(b-1, b-1), task (s, t-1)'s mailbox entry
                for tp in range(t + 1, ntp):
                    ql, qd, qr, _ = blocks(n, b, s - 1, tp)
                    touched = L & (ql | qd | qr)
                    assert touched <= ({head} if tp == t + 1 else set()), (s, t, tp, sorted(touched))
            # R of task t is L of task t + 1, and exists exactly when task t + 1 does
            if t + 1 < nt:
                nl_, _, _, _ = blocks(n, b, s, t + 1)
                assert R == nl_, (s, t)
            else:
                assert not R, (s, t)


def test_annihilated_head_is_the_consumers_corner():
    # the producer (s-1, t+2)'s L(0, 0) is the consumer (s, t)'s R(b-1, b-1)
    n, b = 100, 8
    for s in range(1, n - 1):
        for t in range(tasks(n, b, s)):
            if t + 2 >= tasks(n, b, s - 1):
                continue
            _, _, _, (r0p, colp, _, _) = blocks(n, b, s - 1, t + 2)
            _, _, _, (r0, col, m, mr) = blocks(n, b, s, t)
            if mr == b:
                assert (r0p, colp) == (r0 + m + b - 1, r0 + b - 1)
