"""Batched sea-detuning sweep: the GPU dispatcher behind ``run_sweep_sea_detuning``.

The reference's sweep (sweep_sea_detuning.py:356-1165) loops over detunings and calls
``simulate_rare`` three times per point, serially, writing each point's files as it goes.
Here every (detuning, variant) evolution of the sweep is submitted at once: the evolutions
are spread over the visible GPUs (longest-processing-time first by their Chebyshev work,
||H|| * t_final), each GPU evolves its share concurrently inside one libdse context, and only
then are the per-point outputs produced in detuning order, with the same file tree, names,
keys and JSON records as the reference:

    <out_root>/sea_detuning_sweep_<YYYYmmdd_HHMMSS>/
        geometry_and_couplings.npz  global_params.json  summary.json
        sea_detuning_report.pdf  contrast_rare_center_vs_DeltaOmega_over_geff.png
        delta_p<...>Hz/ time_and_obs_{center_off,center_on,shell_off}.npz
                        params_<tag>.json  freqs_<tag>.json  metrics.json  4 x PNG

(:483-502, :677-685, :791, :814-1049, :1143-1157).  The plots and the PDF are produced on the
host after the GPU work (``report="full"``, the reference's content), only the PNGs
(``report="png"``) or not at all (``report="none"``); their time is reported separately from
the evolution time in ``timings``.

There is no CPU fallback: the evolutions run through libdse or the call raises.
"""
from __future__ import annotations

import datetime as _dt
import json
import os
import threading
import time
from dataclasses import asdict, dataclass, replace
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .metrics import coupling_stats, point_metrics
from .model import (DipolarRareParams, dipolar_couplings_from_positions, get_derived_frequencies,
                    shell_positions_with_rare_center)
from .problem import OBS_NAMES, build_problem, spectral_bounds, time_grid
from .sweep import VARIANTS, detuning_label, f1R_for_resonance

Trace = Tuple[np.ndarray, Dict[str, np.ndarray]]


# ------------------------------------------------------------------------------------------
# multi-GPU evolution of many parameter sets
# ------------------------------------------------------------------------------------------
def _visible_devices() -> List[int]:
    from .engine import device_count
    n = device_count()
    if n <= 0:
        raise RuntimeError("no HIP device visible: the sweep runs on MI355X GPUs only")
    return list(range(n))


def assign_lpt(costs: Sequence[float], n_bins: int) -> List[List[int]]:
    """Longest-processing-time-first assignment of jobs to ``n_bins`` devices."""
    bins: List[List[int]] = [[] for _ in range(n_bins)]
    load = [0.0] * n_bins
    for i in sorted(range(len(costs)), key=lambda k: (-costs[k], k)):
        b = min(range(n_bins), key=lambda k: (load[k], k))
        bins[b].append(i)
        load[b] += costs[i]
    for b in bins:
        b.sort()
    return bins


# One libdse context per (engine class, device), kept across evolve_many calls of this process: a
# driver that evolves sweep after sweep (sweep2d_run: one call per group of f1A sweeps) pays the
# context set-up and the first call's allocations once instead of per call (~0.1-0.2 s each).
# DSE_ENGINE_CACHE=0 opens and closes a context per call, as before.
_ENGINES: Dict[Tuple[type, int], Any] = {}
_ENGINES_LOCK = threading.Lock()
# A cached context is not thread-safe (include/dse.h): whoever uses one holds its lock for the whole
# clear / add / evolve sequence, so duplicate device ids or concurrent evolve_many calls serialise.
_ENGINE_USE: Dict[Tuple[type, int], threading.Lock] = {}


def _use_lock(cls, dev: int) -> threading.Lock:
    with _ENGINES_LOCK:
        return _ENGINE_USE.setdefault((cls, dev), threading.Lock())


def _engine_for(cls, dev: int):
    if os.environ.get("DSE_ENGINE_CACHE", "1") == "0":
        return cls(dev), True
    with _ENGINES_LOCK:
        eng = _ENGINES.get((cls, dev))
        if eng is None:
            eng = _ENGINES[(cls, dev)] = cls(dev)
    return eng, False


def close_engines() -> None:
    """Closes the contexts evolve_many keeps (also at interpreter exit)."""
    with _ENGINES_LOCK:
        for eng in _ENGINES.values():
            close = getattr(eng, "close", None)
            if close is not None:
                close()
        _ENGINES.clear()


import atexit as _atexit  # noqa: E402
_atexit.register(close_engines)


def evolve_many(params_list: Sequence[DipolarRareParams], devices: Optional[Sequence[int]] = None,
                tol: Optional[float] = None) -> List[Trace]:
    """``simulate_rare`` for every parameter set, spread over ``devices`` (one host thread and one
    libdse context per GPU; the ctypes call releases the GIL).  Results in input order.  Each
    device evolves its share in batches that fit its free memory (the reference runs one
    evolution at a time, so a sweep of large registers must not allocate all of them at once).
    ``tol``: Chebyshev truncation, default DSE_TOL as in simulate_rare."""
    from .dipolar_ensemble_with_rare import _tol
    tol = _tol() if tol is None else float(tol)
    grids = [time_grid(p) for p in params_list]
    probs = [build_problem(p, order="engine", reduce=True) for p in params_list]
    devices = list(devices) if devices is not None else _visible_devices()
    costs = []
    for p, pr in zip(params_list, probs):
        lo, hi = spectral_bounds(pr)
        costs.append(0.5 * (hi - lo) * float(p.t_final) + 30.0 * int(p.steps))
    shares = assign_lpt(costs, len(devices))
    results: List[Optional[Trace]] = [None] * len(params_list)
    errors: List[BaseException] = []

    def work(dev: int, idxs: List[int]) -> None:
        from .engine import Engine
        with _use_lock(Engine, dev):
            _work(dev, idxs)

    def _work(dev: int, idxs: List[int]) -> None:
        from .engine import Engine, batches_for_memory, evolve_groups
        eng, own = None, False
        try:
            eng, own = _engine_for(Engine, dev)
            # one evolve per time grid and engine class, within the device's memory
            sub = evolve_groups([(float(params_list[i].t_final), int(params_list[i].steps))
                                 for i in idxs], [probs[i] for i in idxs])
            for local in sub.values():
                group = [idxs[j] for j in local]
                eng.clear()
                for batch in batches_for_memory([probs[i] for i in group], dev):
                    eng.clear()
                    members = [group[b] for b in batch]
                    for i in members:
                        eng.add(probs[i])
                    t = grids[members[0]]
                    obs, _ = eng.evolve(t, tol=tol)
                    for slot, i in enumerate(members):
                        results[i] = (t.copy(), {name: obs[slot, j].copy()
                                                 for j, name in enumerate(OBS_NAMES)})
            eng.clear()
        except BaseException as exc:  # re-raised in the caller's thread
            errors.append(exc)
            if eng is not None and not own:  # a failed context is not reused
                with _ENGINES_LOCK:
                    if _ENGINES.get((Engine, dev)) is eng:
                        del _ENGINES[(Engine, dev)]
                        own = True
        finally:
            if eng is not None and own and hasattr(eng, "close"):
                eng.close()

    threads = [threading.Thread(target=work, args=(d, s)) for d, s in zip(devices, shares) if s]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    if errors:
        raise errors[0]
    return results  # type: ignore[return-value]


# ------------------------------------------------------------------------------------------
# output tree
# ------------------------------------------------------------------------------------------
def _json_dump(path: str, obj: Any) -> None:
    with open(path, "w", encoding="utf-8") as f:
        json.dump(obj, f, indent=2, default=float)


def _sweep_base_params(n_sea, gamma_sea, gamma_rare, B0, B1_sea, B1_rare, omega_rf_sea,
                       omega_rf_rare, phi_sea, phi_rare, dipolar_scale, shell_scale, t_final,
                       steps, is_spin_three_half, solver) -> DipolarRareParams:
    """The per-detuning base record of sweep_sea_detuning.py:631-657."""
    return DipolarRareParams(
        n_sea=n_sea, gamma_sea=gamma_sea, gamma_rare=gamma_rare, B0_sea=B0, B0_rare=B0,
        B1_sea=B1_sea, B1_rare=B1_rare, omega_rf_sea=omega_rf_sea, omega_rf_rare=omega_rf_rare,
        phi_sea=phi_sea, phi_rare=phi_rare, dipolar_scale=dipolar_scale, shell_scale=shell_scale,
        t_final=t_final, steps=steps, drive_sea=True, drive_rare=False, init_x_sign=-1,
        init_rare_level=3, is_spin_three_half=is_spin_three_half, is_center_rare=True, **solver)


def _variant(base: DipolarRareParams, tag: str) -> DipolarRareParams:
    """:660-668"""
    if tag == "center_off":
        return replace(base, drive_rare=False, is_center_rare=True)
    if tag == "center_on":
        return replace(base, drive_rare=True, is_center_rare=True)
    return replace(base, drive_rare=False, is_center_rare=False)


@dataclass
class SweepPlan:
    """Everything of one sweep that precedes its evolutions (sweep_sea_detuning.py:414-610)."""
    base_dir: str
    dets: np.ndarray
    f_Az: float
    f1A: float
    f1R: float
    coarse_window: int
    rms_b_AR: float
    global_params: Dict[str, Any]
    point_params: List[Dict[str, DipolarRareParams]]

    @property
    def flat(self) -> List[DipolarRareParams]:
        """The 3 x n_det evolutions, detuning-major in the reference's variant order (:694-702)."""
        return [pp[tag] for pp in self.point_params for tag in VARIANTS]


def plan_sweep(
    *,
    f_Az: float,
    f1A: float,
    target_sea_detuning: float,
    gamma_sea: float,
    gamma_rare: float,
    sea_detunings_Hz: Sequence[float],
    n_sea: int = 12,
    t_final: float = 3.0e-2,
    steps: int = 2000,
    phi_sea: float = 0.0,
    phi_rare: float = 0.0,
    out_root: str = "results",
    is_spin_three_half: bool = False,
    solver_atol: float | None = None,
    solver_rtol: float | None = None,
    solver_nsteps: int | None = None,
    solver_max_step: float | None = None,
    coarse_window: int = 50,
    verbose: bool = True,
) -> SweepPlan:
    """The sweep directory, its geometry file, global parameters and the parameter records of every
    evolution (:414-668), before any evolution runs."""
    say = print if verbose else (lambda *a, **k: None)
    f1R = f1R_for_resonance(f1A, target_sea_detuning, 0.0)
    dets = np.asarray(sea_detunings_Hz, dtype=float)
    B0 = 2 * np.pi * f_Az / gamma_sea
    f_Rz = gamma_rare * B0 / (2 * np.pi)
    B1_sea = 2 * np.pi * f1A / gamma_sea
    B1_rare = 2 * np.pi * f1R / gamma_rare if gamma_rare != 0.0 else 0.0
    dipolar_scale = 1.0e-7 * 1.054571817e-34       # mu0/4pi * hbar (:434-436)
    shell_scale = 0.282393e-9                      # (:437)

    positions = shell_positions_with_rare_center(n_sea=n_sea, radius=shell_scale)
    b = dipolar_couplings_from_positions(positions=positions, scale=dipolar_scale,
                                         gamma_sea=gamma_sea, gamma_rare=gamma_rare)
    cs = coupling_stats(b, n_sea)
    say("Estimated dipolar couplings from geometry + physical scales:")
    for name, key, rms in (("Sea–rare b_ij (all sea ↔ rare)", "sea_rare_abs_Hz", "sea_rare_rms_Hz"),
                           ("Sea–sea b_ij (all i<j)", "sea_sea_abs_Hz", "sea_sea_rms_Hz")):
        a = cs[key]
        say(f"  {name}, |b| in Hz: avg {a.mean():.2f}  rms {cs[rms]:.2f}  "
            f"min {a.min():.2f}  max {a.max():.2f}")

    base_dir = os.path.join(out_root, "sea_detuning_sweep_"
                            + _dt.datetime.now().strftime("%Y%m%d_%H%M%S"))
    os.makedirs(base_dir, exist_ok=True)
    np.savez(os.path.join(base_dir, "geometry_and_couplings.npz"), positions=positions, b=b,
             sea_indices=np.array(list(range(n_sea)), dtype=int), idx_rare=int(n_sea),
             sea_rare_vals=cs["sea_rare_vals"], sea_sea_vals=cs["sea_sea_vals"])
    solver = dict(solver_atol=solver_atol, solver_rtol=solver_rtol, solver_nsteps=solver_nsteps,
                  solver_max_step=solver_max_step)
    global_params = {
        "f_Az_Hz": float(f_Az), "f_Rz_Hz": float(f_Rz), "f1A_Hz": float(f1A), "f1R_Hz": float(f1R),
        "gamma_sea": float(gamma_sea), "gamma_rare": float(gamma_rare),
        "B0_common_T": float(B0), "B1_sea_T": float(B1_sea), "B1_rare_T": float(B1_rare),
        "dipolar_scale_SI": float(dipolar_scale), "shell_scale_m": float(shell_scale),
        "t_final_s": float(t_final), "steps": int(steps), "n_sea": int(n_sea),
        "phi_sea_rad": float(phi_sea), "phi_rare_rad": float(phi_rare),
        "sea_detunings_Hz": [float(x) for x in dets], "sea_spin_type": "1/2",
        "rare_spin_type": "3/2" if is_spin_three_half else "1/2",
        **solver,
        "target_sea_detuning": target_sea_detuning, "coarse_window": int(coarse_window),
        "avg_b_AR_Hz": float(cs["sea_rare_abs_Hz"].mean()),
        "rms_b_AR_Hz": float(cs["sea_rare_rms_Hz"]),
        "avg_b_AA_Hz": float(cs["sea_sea_abs_Hz"].mean()),
        "rms_b_AA_Hz": float(cs["sea_sea_rms_Hz"]),
    }
    say(f"Sea detuning sweep: {len(dets)} points x 3 variants -> {base_dir}", flush=True)
    point_params: List[Dict[str, DipolarRareParams]] = []
    for delta in dets:
        f_rf_sea = f_Az - delta
        base = _sweep_base_params(n_sea, gamma_sea, gamma_rare, B0, B1_sea, B1_rare,
                                  2 * np.pi * f_rf_sea, 2 * np.pi * f_Rz, phi_sea, phi_rare,
                                  dipolar_scale, shell_scale, t_final, steps, is_spin_three_half,
                                  solver)
        point_params.append({tag: _variant(base, tag) for tag in VARIANTS})
    return SweepPlan(base_dir, dets, float(f_Az), float(f1A), float(f1R), int(coarse_window),
                     float(cs["sea_rare_rms_Hz"]), global_params, point_params)


def writer_count() -> int:
    """Worker processes for sweep trees and figures: this process's CPU share less the one driving
    the GPUs, at most 16 (the GPU box's share; os.cpu_count() there is the whole machine's)."""
    if os.environ.get("DSE_REPORT_WORKERS"):  # explicit count (1: the serial report)
        return max(1, int(os.environ["DSE_REPORT_WORKERS"]))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        n = os.cpu_count() or 2
    return max(1, min(16, n - 1))


def _png_chunk(details, base_dir: Optional[str] = None, rows=None) -> float:
    """Worker task: the PNGs of a chunk of points (and the sweep's contrast plot, once)."""
    from . import report as rep
    t0 = time.perf_counter()
    rep.write_point_pngs(details)
    if base_dir is not None:
        rep.write_contrast_png(base_dir, rows)
    return time.perf_counter() - t0


def write_sweep(plan: SweepPlan, traces: Sequence[Trace], report: str = "full",
                timings: Optional[Dict[str, float]] = None, verbose: bool = True,
                details_out: Optional[list] = None, workers: Optional[int] = None) -> str:
    """Per-point files and metrics in detuning order, the report, global_params.json and
    summary.json (:611-1157) from the evolutions' traces (in ``plan.flat`` order).
    ``details_out``: receives the (det_dir, per, metrics, det) rows a report is drawn from.
    ``workers`` (default writer_count()): with more than one and at least 8 points, the per-point
    PNGs (most of a report's time: ~1.4 s per point at 300 dpi) are drawn by that many spawned
    processes in 4-point chunks while this process writes the PDF pages, whose order is fixed."""
    if report not in ("full", "png", "none"):
        raise ValueError(f"report must be 'full', 'png' or 'none', not {report!r}")
    say = print if verbose else (lambda *a, **k: None)
    t1 = time.perf_counter()
    base_dir = plan.base_dir
    summary: Dict[str, Any] = {"global_params": plan.global_params, "sweep_results": []}
    details = []
    for idx, delta in enumerate(plan.dets):
        det_dir = os.path.join(base_dir, detuning_label(delta))
        os.makedirs(det_dir, exist_ok=True)
        per = {}
        for j, tag in enumerate(VARIANTS):
            t_arr, obs = traces[3 * idx + j]
            p = plan.point_params[idx][tag]
            np.savez(os.path.join(det_dir, f"time_and_obs_{tag}.npz"), t=t_arr, **obs)
            _json_dump(os.path.join(det_dir, f"params_{tag}.json"), asdict(p))
            _json_dump(os.path.join(det_dir, f"freqs_{tag}.json"), get_derived_frequencies(p))
            per[tag] = (t_arr, obs)
        metrics, det = point_metrics(delta, plan.f_Az - delta, plan.f1A, plan.f1R, plan.rms_b_AR,
                                     {k: (v[0], v[1]["Iz_sea"]) for k, v in per.items()},
                                     plan.coarse_window)
        _json_dump(os.path.join(det_dir, "metrics.json"), metrics)
        summary["sweep_results"].append(metrics)
        details.append((det_dir, per, metrics, det))
    t2 = time.perf_counter()
    if details_out is not None:
        details_out.extend(details)

    if report != "none":
        from . import report as rep
        nw = writer_count() if workers is None else int(workers)
        if nw > 1 and len(details) >= 8:
            import multiprocessing as mp
            from concurrent.futures import ProcessPoolExecutor
            chunk = 4
            n_chunks = (len(details) + chunk - 1) // chunk
            with ProcessPoolExecutor(max_workers=min(nw, n_chunks),
                                     mp_context=mp.get_context("spawn")) as pool:
                futs = [pool.submit(_png_chunk, details[i:i + chunk],
                                    base_dir if i == 0 else None,
                                    summary["sweep_results"] if i == 0 else None)
                        for i in range(0, len(details), chunk)]
                if report == "full":
                    rep.write_sweep_report(base_dir, plan.global_params, summary["sweep_results"],
                                           details, pdf=True, pngs=False)
                for f in futs:
                    f.result()
        else:
            rep.write_sweep_report(base_dir, plan.global_params, summary["sweep_results"], details,
                                   pdf=(report == "full"))
    t3 = time.perf_counter()

    _json_dump(os.path.join(base_dir, "global_params.json"), summary["global_params"])
    _json_dump(os.path.join(base_dir, "summary.json"), summary)
    if timings is not None:
        timings.update(outputs_s=t2 - t1, report_s=t3 - t2)
    say(f"Sweep written: {base_dir} (files {t2 - t1:.2f} s, report {t3 - t2:.2f} s)", flush=True)
    return base_dir


def run_sweep_sea_detuning(
    *,
    f_Az: float,
    f1A: float,
    target_sea_detuning: float,
    gamma_sea: float,
    gamma_rare: float,
    sea_detunings_Hz: Sequence[float],
    n_sea: int = 12,
    t_final: float = 3.0e-2,
    steps: int = 2000,
    phi_sea: float = 0.0,
    phi_rare: float = 0.0,
    out_root: str = "results",
    is_spin_three_half: bool = False,
    solver_atol: float | None = None,
    solver_rtol: float | None = None,
    solver_nsteps: int | None = None,
    solver_max_step: float | None = None,
    coarse_window: int = 50,
    devices: Optional[Sequence[int]] = None,
    report: str = "full",
    timings: Optional[Dict[str, float]] = None,
    verbose: bool = True,
) -> str:
    """Same arguments, outputs and return value (the sweep directory) as
    sweep_sea_detuning.py:356-1165, plus ``devices`` (GPU ids, default all visible),
    ``report`` ("full" | "png" | "none") and ``timings`` (filled with evolve_s / outputs_s /
    report_s)."""
    if report not in ("full", "png", "none"):
        raise ValueError(f"report must be 'full', 'png' or 'none', not {report!r}")
    plan = plan_sweep(f_Az=f_Az, f1A=f1A, target_sea_detuning=target_sea_detuning,
                      gamma_sea=gamma_sea, gamma_rare=gamma_rare, sea_detunings_Hz=sea_detunings_Hz,
                      n_sea=n_sea, t_final=t_final, steps=steps, phi_sea=phi_sea, phi_rare=phi_rare,
                      out_root=out_root, is_spin_three_half=is_spin_three_half,
                      solver_atol=solver_atol, solver_rtol=solver_rtol, solver_nsteps=solver_nsteps,
                      solver_max_step=solver_max_step, coarse_window=coarse_window, verbose=verbose)
    t0 = time.perf_counter()
    traces = evolve_many(plan.flat, devices)
    t1 = time.perf_counter()
    if verbose:
        print(f"  evolved {len(plan.flat)} evolutions in {t1 - t0:.2f} s", flush=True)
    base_dir = write_sweep(plan, traces, report=report, timings=timings, verbose=verbose)
    if timings is not None:
        timings["evolve_s"] = t1 - t0
    return base_dir
