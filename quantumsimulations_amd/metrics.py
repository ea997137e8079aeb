"""Per-point sweep metrics (host side), restating sweep_sea_detuning.py:116-335 and :748-790.

These run on the host after the evolutions, on the ``Iz_sea`` traces the engine returns:

* ``coarse_grain``        block means of ``window`` consecutive samples      (:116-141)
* ``iz_slope_from_coarse`` line fit over the central 60 % of the envelope   (:148-268)
* ``contrast_michelson_with_t_gate``  t-gated Michelson contrast of slopes  (:279-317)
* ``point_metrics``       the ``metrics.json`` record of one detuning       (:704-790)

The arithmetic (numpy reductions, ``np.polyfit``) is the same as the reference's so the
numbers are bit-identical on identical traces; tests/test_sweep_format.py checks that against
metrics the reference's own functions produced (tests/golden/sweep_metrics.json).
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

SLOPE_T_MIN: float = 1.0    # sweep_sea_detuning.py:276

_SLOPE_KEYS = ("I_z_slope", "t_start", "t_end", "I_z_start", "I_z_end", "slope", "slope_std",
               "t_value", "R_value", "R2_value")


def coarse_grain(t: np.ndarray, y: np.ndarray, window: int = 25) -> Tuple[np.ndarray, np.ndarray]:
    """Block-average (t, y) over ``window`` samples; the ragged tail is dropped (:116-141).
    ``window`` 0 raises ZeroDivisionError and ``window`` <= 1 returns the input, as there."""
    m = len(t) // window
    if window <= 1 or m <= 0:
        return t, y
    keep = m * window
    return (np.asarray(t)[:keep].reshape(m, window).mean(axis=1),
            np.asarray(y)[:keep].reshape(m, window).mean(axis=1))


def _nan_slope() -> Dict[str, float]:
    return {k: np.nan for k in _SLOPE_KEYS}


def iz_slope_from_coarse(t_coarse: np.ndarray, iz_coarse: np.ndarray) -> Dict[str, float]:
    """Drift of a coarse <Iz_sea> envelope from a least-squares line over its central 60 %.

    Same window, clamping, fit, R and slope t-statistic as sweep_sea_detuning.py:179-268.
    """
    n = t_coarse.size
    if n < 4 or iz_coarse.size < 4:
        return _nan_slope()
    lo = max(0, min(int(0.2 * n), n - 2))
    hi = max(lo + 2, min(int(0.8 * n), n))
    ts, ys = t_coarse[lo:hi], iz_coarse[lo:hi]
    if ts.size < 2:
        return _nan_slope()
    slope, icpt = np.polyfit(ts, ys, 1)
    t0, t1 = float(ts[0]), float(ts[-1])
    y0, y1 = float(icpt + slope * t0), float(icpt + slope * t1)

    dt, dy = ts - np.mean(ts), ys - np.mean(ys)
    sxx, syy = float(np.sum(dt * dt)), float(np.sum(dy * dy))
    if sxx > 0.0 and syy > 0.0:
        r = float(np.dot(dt, dy) / np.sqrt(sxx * syy))
        r2 = float(r * r)
    else:
        r = r2 = np.nan

    slope_std = t_val = np.nan
    if ts.size > 2 and sxx > 0.0:
        res = ys - (icpt + slope * ts)
        var = float(np.sum(res ** 2)) / (ts.size - 2) / sxx
        slope_std = float(np.sqrt(var)) if var > 0.0 else np.nan
        if slope_std > 0.0 and np.isfinite(slope_std):
            t_val = float(slope / slope_std)
    return {"I_z_slope": float(y1 - y0), "t_start": t0, "t_end": t1, "I_z_start": y0,
            "I_z_end": y1, "slope": float(slope), "slope_std": slope_std, "t_value": t_val,
            "R_value": r, "R2_value": r2}


def contrast_michelson_with_t_gate(slope_on: float, slope_off: float, t_on: float, t_off: float,
                                   t_min: float = SLOPE_T_MIN) -> float:
    """(|s_on| - |s_off|) / (|s_on| + |s_off|), a slope with |t| < t_min counting as 0 (:279-317)."""
    if not all(np.isfinite(v) for v in (slope_on, slope_off, t_on, t_off)):
        return float("nan")
    a = 0.0 if abs(t_on) < t_min else slope_on
    b = 0.0 if abs(t_off) < t_min else slope_off
    s = abs(a) + abs(b)
    if not np.isfinite(s) or s <= 1e-16:
        return 0.0
    return (abs(a) - abs(b)) / s


def coupling_stats(b: np.ndarray, n_sea: int) -> Dict[str, object]:
    """Sea-rare and sea-sea coupling values and |b| statistics in Hz (:451-466)."""
    sea_rare = np.array([b[i, n_sea] for i in range(n_sea)], dtype=float)
    sea_sea = np.array([b[i, j] for i in range(n_sea) for j in range(i + 1, n_sea)], dtype=float)
    two_pi = 2 * np.pi
    return {
        "sea_rare_vals": sea_rare,
        "sea_sea_vals": sea_sea,
        "sea_rare_abs_Hz": np.abs(sea_rare) / two_pi,
        "sea_rare_rms_Hz": np.sqrt(np.mean(np.abs(sea_rare) ** 2)) / two_pi,
        "sea_sea_abs_Hz": np.abs(sea_sea) / two_pi,
        "sea_sea_rms_Hz": np.sqrt(np.mean(np.abs(sea_sea) ** 2)) / two_pi,
    }


def point_metrics(delta_Hz: float, f_rf_sea: float, f1A: float, f1R: float,
                  sea_rare_rms_Hz: float, traces: Dict[str, Tuple[np.ndarray, np.ndarray]],
                  coarse_window: int) -> Tuple[Dict[str, float], Dict[str, dict]]:
    """``metrics.json`` of one detuning (:704-790) from the (t, Iz_sea) trace of each variant.

    Returns (metrics, details) where details holds the coarse envelopes and the slope fits the
    report plots draw.
    """
    env, fit = {}, {}
    for tag in ("center_off", "center_on", "shell_off"):
        t, iz = traces[tag]
        env[tag] = coarse_grain(t, iz, window=coarse_window)
        fit[tag] = iz_slope_from_coarse(*env[tag])
    off, on, sea = fit["center_off"], fit["center_on"], fit["shell_off"]
    c_rare = contrast_michelson_with_t_gate(on["I_z_slope"], off["I_z_slope"], on["t_value"],
                                            off["t_value"])
    c_sea = contrast_michelson_with_t_gate(on["I_z_slope"], sea["I_z_slope"], on["t_value"],
                                           sea["t_value"])
    # Delta Omega / |g_eff| with the RMS sea-rare coupling; rare driven on resonance (:748-767)
    om_a = np.sqrt(delta_Hz ** 2 + f1A ** 2)
    om_r = np.sqrt(0.0 ** 2 + f1R ** 2)
    d_om = om_a - om_r
    sin_a = f1A / om_a if om_a != 0.0 else 0.0
    sin_r = f1R / om_r if om_r != 0.0 else 0.0
    g_eff = (sea_rare_rms_Hz / 4.0) * sin_a * sin_r
    ratio = float("nan") if (g_eff == 0.0 or np.isnan(g_eff)) else float(d_om / abs(g_eff))
    metrics = {
        "delta_Hz": float(delta_Hz),
        "f_rf_sea_Hz": float(f_rf_sea),
        "I_z_slope_off_center": float(off["I_z_slope"]),
        "R_off_center": float(off["R_value"]),
        "t_off_center": float(off["t_value"]),
        "I_z_slope_on_center": float(on["I_z_slope"]),
        "R_on_center": float(on["R_value"]),
        "t_on_center": float(on["t_value"]),
        "contrast_rare_center": float(c_rare),
        "I_z_slope_off_sea_center": float(sea["I_z_slope"]),
        "R_off_sea_center": float(sea["R_value"]),
        "t_off_sea_center": float(sea["t_value"]),
        "contrast_sea_center": float(c_sea),
        "DeltaOmega_Hz": float(d_om),
        "g_eff_Hz": float(g_eff),
        "DeltaOmega_over_geff": float(ratio),
    }
    return metrics, {"envelopes": env, "fits": fit}
