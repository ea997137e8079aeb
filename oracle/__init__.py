"""CPU oracle for the dipolar spin-ensemble evolution path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``quantumsimulations_amd`` imports this
package; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg use it, and only as the checker / the timed CPU baseline.

Contents
--------
* ``reference_model``  independent restatement of the reference's Hamiltonian
  construction (dipolar_ensemble_with_rare.py:15-52, 387-606) as scipy.sparse
  Kronecker products in QuTiP's site order (site 0 = most significant factor).
* ``propagate``        exact propagators (dense ``eigh`` for N <= 12,
  ``expm_multiply`` above) and the QuTiP-5 ``sesolve`` equivalent
  (scipy ZVODE Adams, normalised output) used as the CPU baseline.

Pinning: ``tests/test_oracle_golden.py`` checks this oracle against golden
vectors produced by the reference's own ``dipolar_ensemble_with_rare.py``
(see ``tests/golden/make_golden.py`` for how, and DESIGN.md §Oracle for what is
pinned and what is not).
"""
