"""One register partitioned over GPUs (SURVEY.md §8(e), configs with N >= 28).

The top ``shard_bits`` engine qubits are global: rank r of 2^shard_bits (one process per GPU)
holds the amplitudes whose global bits equal r.  On the Walsh-Hadamard engine (default) every H
application index-swaps the X / Y vectors around its MID pass (local top bits <-> shard bits: an
RCCL all-to-all inside libdse, twice per vector).  On the step kernels (option wht = 0): in
engine order the rare spin is the top qubit, so it is always global; its only off-diagonal term
is its own drive flip (sea-rare coupling is ZZ only, dipolar_ensemble_with_rare.py:562-568), so
the global set {rare, s1, s2} needs partner masks {rare, s1, s2, s1^s2}: at most 4 full-shard
exchanges per term (RCCL send/recv pairs, include/dse.h dse_add_problem_sharded).  Either way
one all-reduce of the observable sums at the end.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_partitioned.py

``simulate_rare_partitioned`` is the collective counterpart of ``simulate_rare``: every rank calls
it with the same parameters and gets the same (t, obs).
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

from .engine import Engine
from .model import DipolarRareParams
from .problem import OBS_NAMES, build_problem, time_grid


def shard_bits_for(world: int) -> int:
    if world not in (2, 4, 8):
        raise ValueError("a partitioned register needs 2, 4 or 8 ranks")
    return world.bit_length() - 1


def join(engine: Engine, rank: int, world: int, dist) -> None:
    """RCCL communicator of the engine: rank 0's unique id broadcast over ``dist``
    (an initialised torch.distributed)."""
    box = [Engine.dist_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    engine.dist_init(rank, world, box[0])


def simulate_rare_partitioned(params: DipolarRareParams, engine: Engine, rank: int, world: int,
                              tol: float = 1e-14) -> Tuple[np.ndarray, Dict[str, np.ndarray], dict]:
    """Evolves one register split over ``world`` ranks (engine already joined); returns the
    time grid, the whole-register observables (identical on every rank) and the call's stats."""
    t = time_grid(params)
    prob = build_problem(params, order="engine", reduce=True)
    engine.clear()
    pid = engine.add_sharded(prob, shard_bits_for(world), rank)
    obs, st = engine.evolve(t, tol=tol)
    return t, {k: obs[pid, j].copy() for j, k in enumerate(OBS_NAMES)}, st
