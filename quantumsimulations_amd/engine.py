"""Python handle on one device's engine context (libdse.so).

``Engine`` owns a ``dse_ctx``: problems (coefficient tables from ``problem.py``)
are added, then evolved together on one MI355X with the exact Chebyshev
propagator.  Errors from the library surface as ``ValueError`` (bad arguments,
as the reference raises for a bad grid, dipolar_ensemble_with_rare.py:620-621)
or ``RuntimeError`` (HIP / allocation / degree-cap failures).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Tuple

import numpy as np

from . import _lib
from .problem import Problem

DEFAULT_TOL = 1e-14


def device_count() -> int:
    return int(_lib.lib().dse_device_count())


def device_memory(device: int) -> Tuple[float, float]:
    """(free, total) bytes of a device's memory (hipMemGetInfo)."""
    out = np.empty(2)
    rc = _lib.lib().dse_device_memory(int(device), _lib.ptr(out))
    if rc != 0:
        raise RuntimeError(f"dse_device_memory({device}) failed ({rc})")
    return float(out[0]), float(out[1])


def problem_bytes(prob: Problem) -> float:
    """Upper estimate of one problem's device footprint in a context: 3 state buffers, one
    intermediate output of a two-output launch, the Walsh-Hadamard engine's 2 extra vectors or the
    2-tile hand-off ring (the larger: 2 vectors), plus tables and coefficients."""
    return 16.0 * (3 + 1 + 2) * (1 << prob.n_qubits) + (4 << 20)


# A libdse evolve runs its persistent interval kernel only when every register that is not on the
# small-register engine fits one or two 2^13-amplitude tiles (dse_runtime.hip, dse_evolve's mode
# choice); one larger register in the call drops all of them to the streaming kernels.
PERSISTENT_MAX_QUBITS = 14


def engine_class(prob: Problem) -> int:
    """0: a register the persistent kernel (or the small-register engine) takes, 1: a larger one."""
    return 0 if prob.n_qubits <= PERSISTENT_MAX_QUBITS else 1


def evolve_groups(grid_keys, probs) -> Dict[Tuple, list]:
    """Indices of problems that share one evolve call: the same time grid and the same engine
    class, so a mixed batch keeps its tile-sized registers on the persistent kernel."""
    groups: Dict[Tuple, list] = {}
    for i, (key, p) in enumerate(zip(grid_keys, probs)):
        groups.setdefault((*key, engine_class(p)), []).append(i)
    return groups


# Device memory a context holds besides its problems: observable partials (up to 256 MiB), the
# intermediate outputs and hand-off slots of the interval kernel beyond the per-problem estimate,
# flags, coefficient arenas.
CONTEXT_BYTES = 512 << 20


def batches_for_memory(probs, device: int, headroom: float = 0.8):
    """Index batches of ``probs`` whose summed footprint fits ``headroom`` of the free memory of
    ``device`` less one context's fixed arenas (at least one problem per batch; a problem too large
    alone still gets its own).  Call it with the context cleared, so its last batch's buffers are
    not counted as used."""
    free, _ = device_memory(device)
    budget = headroom * free - CONTEXT_BYTES
    out, cur, used = [], [], 0.0
    for i, p in enumerate(probs):
        b = problem_bytes(p)
        if cur and used + b > budget:
            out.append(cur)
            cur, used = [], 0.0
        cur.append(i)
        used += b
    if cur:
        out.append(cur)
    return out


class Engine:
    def __init__(self, device: int = 0, tile_bits: int | None = None, time_kernels: bool = True):
        self._L = _lib.lib()
        h = self._L.dse_create(int(device))
        if not h:
            raise RuntimeError("dse_create failed: " + self._L.dse_create_error().decode())
        self._h = C.c_void_p(h)
        self.device = device
        self.problems: list[Problem] = []
        self._dims: list[int] = []       # state size the hooks of each problem id take
        if tile_bits is not None:
            self.set_option("tile_bits", tile_bits)
        self.set_option("time_kernels", 1.0 if time_kernels else 0.0)

    # -- plumbing --
    def _check(self, rc: int) -> int:
        if rc >= 0:
            return rc
        msg = self._L.dse_last_error(self._h).decode()
        if rc == _lib.DSE_ERR_ARG:
            raise ValueError(msg)
        raise RuntimeError(f"libdse error {rc}: {msg}")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.dse_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_option(self, key: str, value: float) -> None:
        self._check(self._L.dse_set_option(self._h, key.encode(), float(value)))

    # -- problems --
    @staticmethod
    def _tables(prob: Problem):
        n = prob.n_qubits
        return (np.ascontiguousarray(prob.field, dtype=np.float64),
                np.ascontiguousarray(prob.zz, dtype=np.float64).reshape(n * n),
                np.ascontiguousarray(prob.pair, dtype=np.float64).reshape(n * n),
                np.ascontiguousarray(prob.flip, dtype=np.float64).reshape(4 * n))

    def add(self, prob: Problem) -> int:
        tabs = self._tables(prob)
        pid = self._check(self._L.dse_add_problem(
            self._h, prob.n_qubits, *[_lib.ptr(a) for a in tabs],
            float(prob.shift), int(prob.psi0_index), int(prob.sea_mask), int(prob.rare_bit),
            float(prob.rare_z_const)))
        self.problems.append(prob)
        self._dims.append(1 << prob.n_qubits)
        return pid

    def add_sharded(self, prob: Problem, shard_bits: int, rank: int = -1) -> int:
        """A register partitioned by its top ``shard_bits`` qubits (include/dse.h): all shards
        on this device (rank -1, returns shard 0's id; its hooks take whole-register states) or
        this process's shard ``rank`` of a register spread over processes (after dist_init)."""
        tabs = self._tables(prob)
        pid = self._check(self._L.dse_add_problem_sharded(
            self._h, prob.n_qubits, *[_lib.ptr(a) for a in tabs],
            float(prob.shift), int(prob.psi0_index), int(prob.sea_mask), int(prob.rare_bit),
            float(prob.rare_z_const), int(shard_bits), int(rank)))
        n_members = 1 if rank >= 0 else (1 << shard_bits)
        for i in range(n_members):
            self.problems.append(prob)
            self._dims.append((1 << prob.n_qubits) if (rank < 0 and i == 0)
                              else int(self._L.dse_problem_dim(self._h, pid + i)))
        return pid

    @staticmethod
    def dist_unique_id() -> bytes:
        buf = C.create_string_buffer(_lib.DSE_DIST_ID_BYTES)
        if _lib.lib().dse_dist_unique_id(buf) != 0:
            raise RuntimeError("dse_dist_unique_id (ncclGetUniqueId) failed")
        return buf.raw

    def dist_init(self, rank: int, world: int, uid: bytes) -> None:
        """Join the RCCL communicator of a register partitioned over ``world`` processes."""
        if len(uid) != _lib.DSE_DIST_ID_BYTES:
            raise ValueError("unique id must have DSE_DIST_ID_BYTES bytes")
        self._check(self._L.dse_dist_init(self._h, int(rank), int(world), uid))

    def dist_init_exchange(self, rank: int, world: int, dist) -> None:
        """Join a partitioned register's ranks over ``dist`` (an initialised torch.distributed,
        e.g. gloo) instead of RCCL: libdse hands every exchange to this host callback
        (include/dse.h dse_dist_init_exchange)."""
        import torch

        def view(addr, nbytes, dtype):
            buf = (C.c_uint8 * nbytes).from_address(addr)
            return torch.from_numpy(np.frombuffer(buf, dtype=dtype))

        def fn(_user, op, send, recv, nbytes, peer):
            try:
                if op == _lib.DSE_XCHG_ALLTOALL:
                    dist.all_to_all_single(view(recv, nbytes * world, np.uint8),
                                           view(send, nbytes * world, np.uint8))
                elif op == _lib.DSE_XCHG_SENDRECV:
                    reqs = [dist.isend(view(send, nbytes, np.uint8), peer),
                            dist.irecv(view(recv, nbytes, np.uint8), peer)]
                    for r in reqs:
                        r.wait()
                elif op == _lib.DSE_XCHG_ALLREDUCE_F64:
                    dist.all_reduce(view(send, nbytes, np.float64))
                else:
                    return 1
                return 0
            except Exception:  # reported to the library as a failed exchange
                return 1

        self._xfn = _lib.EXCHANGE_FN(fn)   # kept alive with the engine
        self._check(self._L.dse_dist_init_exchange(self._h, int(rank), int(world), self._xfn, None))

    def clear(self) -> None:
        self._check(self._L.dse_clear(self._h))
        self.problems = []
        self._dims = []

    # -- hot path --
    def apply_h(self, pid: int, psi: np.ndarray) -> np.ndarray:
        dim = self._dims[pid]
        x = np.ascontiguousarray(psi, dtype=np.complex128)
        if x.shape != (dim,):
            raise ValueError(f"state must have shape ({dim},)")
        out = np.empty_like(x)
        self._check(self._L.dse_apply_h(self._h, pid, _lib.ptr(x), _lib.ptr(out)))
        return out

    def observables(self, pid: int, psi: np.ndarray) -> np.ndarray:
        dim = self._dims[pid]
        x = np.ascontiguousarray(psi, dtype=np.complex128)
        if x.shape != (dim,):
            raise ValueError(f"state must have shape ({dim},)")
        out = np.empty(7)
        self._check(self._L.dse_observables(self._h, pid, _lib.ptr(x), _lib.ptr(out)))
        return out

    def evolve(self, t: np.ndarray, tol: float = DEFAULT_TOL) -> Tuple[np.ndarray, Dict[str, float]]:
        """obs[problem, 7, n_t] for all problems, and the call's counters."""
        tt = np.ascontiguousarray(t, dtype=np.float64)
        out = np.empty((len(self.problems), _lib.DSE_N_OBS, len(tt)))
        st = _lib.DseStats()
        self._check(self._L.dse_evolve(self._h, _lib.ptr(tt), len(tt), float(tol), _lib.ptr(out),
                                       C.byref(st)))
        return out, st.as_dict()

    def state(self, pid: int) -> np.ndarray:
        out = np.empty(self._dims[pid], dtype=np.complex128)
        self._check(self._L.dse_get_state(self._h, pid, _lib.ptr(out)))
        return out

    def energy(self, pid: int) -> Tuple[float, float]:
        """(<psi|H|psi> / <psi|psi>, <psi|psi>) of the final state after evolve, on the device."""
        out = np.empty(2)
        self._check(self._L.dse_energy(self._h, pid, _lib.ptr(out)))
        return float(out[0]), float(out[1])

    def time_step_kernel(self, reps: int = 20) -> Tuple[float, float]:
        ms = C.c_double()
        by = C.c_double()
        self._check(self._L.dse_time_step_kernel(self._h, int(reps), C.byref(ms), C.byref(by)))
        return ms.value, by.value


def spectral_bounds_native(prob: Problem) -> Tuple[float, float]:
    """dse_spectral_bounds (host-only library function)."""
    L = _lib.lib()
    n = prob.n_qubits
    arrs = [np.ascontiguousarray(a, dtype=np.float64).ravel() for a in (prob.field, prob.zz, prob.pair, prob.flip)]
    lo, hi = C.c_double(), C.c_double()
    rc = L.dse_spectral_bounds(n, *[_lib.ptr(a) for a in arrs], float(prob.shift), C.byref(lo), C.byref(hi))
    if rc != 0:
        raise ValueError("dse_spectral_bounds failed")
    return lo.value, hi.value


def bessel_native(z: float, kmax: int, tol: float = 1e-14) -> Tuple[np.ndarray, int]:
    """dse_bessel_j (host-only library function): J_0..J_kmax(z) and the truncation degree."""
    L = _lib.lib()
    out = np.empty(kmax + 1)
    deg = C.c_int()
    rc = L.dse_bessel_j(float(z), int(kmax), _lib.ptr(out), float(tol), C.byref(deg))
    if rc != 0:
        raise ValueError("dse_bessel_j failed")
    return out, deg.value
