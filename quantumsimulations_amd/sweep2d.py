"""Headless 2D sweep report: aggregation over many sweeps.

Restates the analysis of ``2D_sweep_report.py`` (aggregate_points :199-303, make_plots
:306-463) and ``2D_sweep_report_stable_region.py`` (compute_stable_region :251-364,
make_plots_and_analyze :367-548) without their module-level ``tkinter`` import, which keeps
both scripts from even starting on a display-less node: the root directory is a required
argument here instead of a folder-picker dialog.  Outputs are the same files:
``<root>/contrast_vs_coupling_summary.pdf``, ``<root>/graphs/0[1-5]_*.png`` and
``<root>/stable_region_stats.json``.

    python -m quantumsimulations_amd.sweep2d ROOT [--stable] [--c-min 0.2] [--p-min 0.8]
                                                    [--bin-decimals 3] [--add-stability-page]
"""
from __future__ import annotations

import argparse
import json
import math
import os
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np

POINT_ALPHA = 0.85
POINT_SIZE = 24
ZOOM_PERCENTILES = (1.0, 99.0)
F1A_COLOR_VMIN_KHZ = 5.0
F1A_COLOR_VMAX_KHZ = 50.0
F1A_COLORBAR_TICKS_KHZ = np.arange(5.0, 50.0 + 0.001, 5.0)


# ------------------------------------------------------------------------------------------
# aggregation
# ------------------------------------------------------------------------------------------
def find_sweep_summaries(root_dir: str) -> Iterator[str]:
    """Every summary.json below root_dir, in os.walk order (:199-207)."""
    for dirpath, _, filenames in os.walk(root_dir):
        if "summary.json" in filenames:
            yield os.path.join(dirpath, "summary.json")


def _finite_float(v) -> Optional[float]:
    try:
        f = float(v)
    except (TypeError, ValueError):
        return None
    return f


def load_data_from_summary(summary_path: str) -> List[Dict[str, float]]:
    """The usable points of one sweep (:210-285): rows whose coupling metric, contrast, detuning
    and the sweep's f1A are all finite (f1A != 0), with |slope_on - slope_off| when present."""
    with open(summary_path, "r", encoding="utf-8") as f:
        data = json.load(f)
    f1a = data.get("global_params", {}).get("f1A_Hz", None)
    if f1a is None:
        return []
    pts = []
    for row in data.get("sweep_results", []):
        eta = row.get("DeltaOmega_over_geff", float("nan"))
        con = row.get("contrast_rare_center", float("nan"))
        dlt = row.get("delta_Hz", float("nan"))
        s_off, s_on = row.get("I_z_slope_off_center", None), row.get("I_z_slope_on_center", None)
        dslope = float("nan")
        if s_off is not None and s_on is not None:
            a, b = _finite_float(s_off), _finite_float(s_on)
            if a is not None and b is not None and math.isfinite(a) and math.isfinite(b):
                dslope = abs(b - a)
        if eta is None or con is None or dlt is None:
            continue
        vals = [_finite_float(v) for v in (eta, con, dlt, f1a)]
        if any(v is None for v in vals):
            continue
        eta, con, dlt, f1 = vals
        if not all(math.isfinite(v) for v in (eta, con, dlt, f1)) or f1 == 0.0:
            continue
        pts.append({"coupling_metric": eta, "contrast": con, "f1A_Hz": f1, "delta_Hz": dlt,
                    "abs_delta_slope_center": dslope})
    return pts


def aggregate_points(root_dir: str) -> List[Dict[str, float]]:
    """All points of all sweeps below root_dir (:288-303)."""
    out: List[Dict[str, float]] = []
    for path in find_sweep_summaries(root_dir):
        out.extend(load_data_from_summary(path))
    return out


# ------------------------------------------------------------------------------------------
# stable region in x = delta_A / f1A
# ------------------------------------------------------------------------------------------
def _mad(x: np.ndarray) -> float:
    x = np.asarray(x, dtype=float)
    x = x[np.isfinite(x)]
    if x.size == 0:
        return float("nan")
    return float(np.median(np.abs(x - float(np.median(x)))))


def compute_stable_region(detuning_ratio: np.ndarray, contrast: np.ndarray, c_min: float,
                          p_min: float, bin_decimals: int, require_negative: bool = True
                          ) -> Tuple[List[dict], Optional[dict]]:
    """Per-bin pass fraction and the best contiguous run of qualifying bins (:260-364).

    Bins are x rounded to ``bin_decimals``; a point passes when its contrast has the required
    sign and |C| >= c_min; bins with p >= p_min qualify; the best run is the longest, then the
    one with most points, then (require_negative) the most negative median contrast.
    """
    x = np.asarray(detuning_ratio, dtype=float)
    c = np.asarray(contrast, dtype=float)
    keep = np.isfinite(x) & np.isfinite(c)
    x, c = x[keep], c[keep]
    if x.size == 0:
        raise RuntimeError("No finite (x, contrast) points for stable-region analysis.")
    groups: Dict[float, List[float]] = {}
    for xb, cb in zip(np.round(x, decimals=bin_decimals), c):
        groups.setdefault(float(xb), []).append(float(cb))
    centers = np.array(sorted(groups), dtype=float)
    stats = []
    for xc in centers:
        v = np.array(groups[float(xc)], dtype=float)
        ok = ((v < 0.0) if require_negative else (v > 0.0)) & (np.abs(v) >= c_min)
        stats.append({"x": float(xc), "N": int(v.size),
                      "p": float(np.mean(ok)) if v.size else float("nan"),
                      "median_C": float(np.median(v)) if v.size else float("nan"),
                      "mad_C": _mad(v)})
    good = [s["p"] >= p_min for s in stats]
    best = None
    i = 0
    while i < len(good):
        if not good[i]:
            i += 1
            continue
        j = i
        while j < len(good) and good[j]:
            j += 1
        run = stats[i:j]
        vals = np.asarray([cv for s in run for cv in groups[s["x"]]], dtype=float)
        med = float(np.median(vals)) if vals.size else float("nan")
        n_pts = sum(s["N"] for s in run)
        key = (j - i, n_pts, (-med if require_negative and math.isfinite(med) else 0.0))
        if best is None or key > best["key"]:
            best = {"i0": i, "i1": j - 1, "x_lo": float(centers[i]), "x_hi": float(centers[j - 1]),
                    "run_len": int(j - i), "run_N": int(n_pts), "run_median_C": med, "key": key}
        i = j
    return stats, best


# ------------------------------------------------------------------------------------------
# figures (matplotlib Agg)
# ------------------------------------------------------------------------------------------
def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def _zoom(ax, x, y, percentiles=ZOOM_PERCENTILES) -> None:
    x, y = np.asarray(x, dtype=float), np.asarray(y, dtype=float)
    m = np.isfinite(x) & np.isfinite(y)
    if np.count_nonzero(m) < 5:
        return
    xf, yf = x[m], y[m]
    lo, hi = percentiles
    x_lo, x_hi = np.percentile(xf, [lo, hi])
    yz = yf
    if math.isfinite(x_lo) and math.isfinite(x_hi) and x_hi > x_lo:
        ax.set_xlim(x_lo, x_hi)
        inside = (xf >= x_lo) & (xf <= x_hi)
        if np.count_nonzero(inside) >= 5:
            yz = yf[inside]
    y_lo, y_hi = np.percentile(yz, [lo, hi])
    if math.isfinite(y_lo) and math.isfinite(y_hi) and y_hi > y_lo:
        pad = 0.05 * (y_hi - y_lo)
        ax.set_ylim(y_lo - pad, y_hi + pad)


def _scatter(plt, ax, x, y, col, label) -> None:
    from matplotlib.colors import Normalize
    x, y, col = (np.asarray(a, dtype=float) for a in (x, y, col))
    f = np.isfinite(x) & np.isfinite(y)
    x, y, col = x[f], y[f], col[f]
    cf = np.isfinite(col)
    if np.any(cf):
        sc = ax.scatter(x[cf], y[cf], s=POINT_SIZE, c=col[cf], alpha=POINT_ALPHA,
                        norm=Normalize(vmin=F1A_COLOR_VMIN_KHZ, vmax=F1A_COLOR_VMAX_KHZ, clip=True))
        cb = plt.colorbar(sc, ax=ax)
        cb.set_label(label)
        cb.set_ticks(F1A_COLORBAR_TICKS_KHZ)
    if np.any(~cf):
        ax.scatter(x[~cf], y[~cf], s=POINT_SIZE, alpha=POINT_ALPHA, color="0.5",
                   label="color missing")
        ax.legend(loc="best")


def _arrays(points):
    a = {k: np.array([p[k] for p in points], dtype=float)
         for k in ("coupling_metric", "contrast", "f1A_Hz", "delta_Hz", "abs_delta_slope_center")}
    m = (np.isfinite(a["coupling_metric"]) & np.isfinite(a["contrast"]) & np.isfinite(a["f1A_Hz"])
         & np.isfinite(a["delta_Hz"]) & (a["f1A_Hz"] != 0.0))
    return {k: v[m] for k, v in a.items()}


def _write_pages(plt, pdf, graphs_dir, a, x_label_ratio, extra=None) -> List[str]:
    written = []
    ratio = a["delta_Hz"] / a["f1A_Hz"]
    f1k = a["f1A_Hz"] / 1000.0
    eta_label = r"Coupling metric $\eta = \Delta\Omega / |g_{\mathrm{eff}}|$"
    slope_label = r"$| \Delta I^z_{\mathrm{slope,center}} |$"

    def save(fig, name):
        fig.tight_layout()
        pdf.savefig(fig)
        fig.savefig(os.path.join(graphs_dir, name), dpi=300)
        plt.close(fig)
        written.append(name)

    pages = [(a["coupling_metric"], a["contrast"], f1k, eta_label, "Contrast",
              "Contrast vs coupling metric\n(all detuning points across all sweeps)",
              "01_contrast_vs_eta.png", False),
             (ratio, a["contrast"], f1k, x_label_ratio[0], "Contrast", x_label_ratio[1],
              "02_contrast_vs_scaled_detuning.png", False)]
    ms = np.isfinite(a["abs_delta_slope_center"])
    if np.any(ms):
        pages += [(a["coupling_metric"][ms], a["abs_delta_slope_center"][ms], f1k[ms], eta_label,
                   slope_label, "Absolute slope difference vs coupling metric"
                   "\n(all detuning points across all sweeps)",
                   "03_abs_slope_diff_vs_eta_zoom.png", True),
                  (ratio[ms], a["abs_delta_slope_center"][ms], f1k[ms], x_label_ratio[0],
                   slope_label, x_label_ratio[2], "04_abs_slope_diff_vs_scaled_detuning_zoom.png",
                   True)]
    for x, y, c, xl, yl, title, name, zoom in pages:
        fig, ax = plt.subplots(figsize=(8, 5))
        _scatter(plt, ax, x, y, c, r"$f_{1A}$ (kHz)")
        if zoom:
            _zoom(ax, x, y)
        ax.set_xlabel(xl)
        ax.set_ylabel(yl)
        ax.set_title(title)
        ax.grid(True, alpha=0.3)
        save(fig, name)
    if extra is not None:
        save(extra(plt), "05_pass_fraction_vs_scaled_detuning.png")
    return written


def make_plots(root_dir: str, pdf_path: str) -> List[str]:
    """The four pages of 2D_sweep_report.py (:306-463); returns the PNG names written."""
    points = aggregate_points(root_dir)
    if not points:
        raise RuntimeError(f"No valid data points found under {root_dir!r}")
    plt = _plt()
    from matplotlib.backends.backend_pdf import PdfPages
    graphs = os.path.join(os.path.dirname(pdf_path), "graphs")
    os.makedirs(graphs, exist_ok=True)
    labels = (r"Scaled detuning $\delta_A / f_{1A}$",
              r"Contrast vs $\delta_A / f_{1A}$" "\n(all detuning points across all sweeps)",
              r"Absolute slope difference vs $\delta_A / f_{1A}$"
              "\n(all detuning points across all sweeps)")
    with PdfPages(pdf_path) as pdf:
        names = _write_pages(plt, pdf, graphs, _arrays(points), labels)
    print(f"Wrote summary PDF to: {pdf_path}")
    return names


def make_plots_and_analyze(root_dir: str, pdf_path: str, c_min: float, p_min: float,
                           bin_decimals: int, stable_json_path: str,
                           add_stability_page: bool) -> dict:
    """2D_sweep_report_stable_region.py (:367-548): stable-region JSON + pages; returns the JSON."""
    points = aggregate_points(root_dir)
    if not points:
        raise RuntimeError(f"No valid data points found under {root_dir!r}")
    a = _arrays(points)
    stats, best = compute_stable_region(a["delta_Hz"] / a["f1A_Hz"], a["contrast"], c_min, p_min,
                                        bin_decimals, require_negative=True)
    print("\n=== Stable-region analysis in x = delta_A / f1A ===")
    print(f"Criterion: pass = (C < 0) and (|C| >= {c_min:g});  p_min = {p_min:g}")
    print(f"Binning: x rounded to {bin_decimals} decimals\n")
    print("   x        N     p(pass)   median(C)    MAD(C)")
    print("----------------------------------------------------")
    for s in stats:
        print(f"{s['x']:7.3f}  {s['N']:6d}   {s['p']:7.3f}   {s['median_C']:10.4f}  {s['mad_C']:9.4f}")
    if best is None:
        print("\nNo contiguous stable region found for the chosen thresholds.")
    else:
        print("\nBest stable region (largest contiguous run with p>=p_min):")
        print(f"  x in [{best['x_lo']:.3f}, {best['x_hi']:.3f}]")
        print(f"  bins = {best['run_len']}, points = {best['run_N']}, "
              f"median(C) = {best['run_median_C']:.4f}")
    out = {"criteria": {"c_min": float(c_min), "p_min": float(p_min),
                        "bin_decimals": int(bin_decimals), "require_negative": True},
           "per_bin": stats, "best_region": best}
    with open(stable_json_path, "w", encoding="utf-8") as f:
        json.dump(out, f, indent=2)
    print(f"\nWrote: {stable_json_path}")

    plt = _plt()
    from matplotlib.backends.backend_pdf import PdfPages
    graphs = os.path.join(os.path.dirname(pdf_path), "graphs")
    os.makedirs(graphs, exist_ok=True)
    labels = (r"Scaled detuning $x=\delta_A / f_{1A}$",
              r"Contrast vs $x=\delta_A / f_{1A}$" "\n(all detuning points across all sweeps)",
              r"Absolute slope difference vs $x=\delta_A / f_{1A}$"
              "\n(all detuning points across all sweeps)")

    def stability_page(plt_):
        fig, ax = plt_.subplots(figsize=(8, 5))
        ax.plot([s["x"] for s in stats], [s["p"] for s in stats], marker="o")
        ax.axhline(p_min, linestyle="--")
        ax.set_xlabel(r"Scaled detuning $x=\delta_A / f_{1A}$")
        ax.set_ylabel(r"Pass fraction $p(x)$")
        title = f"Stable-region pass fraction (C<0 and |C|>={c_min:g})"
        if best is not None:
            ax.axvspan(best["x_lo"], best["x_hi"], alpha=0.2)
            title += f"\nBest band: [{best['x_lo']:.3f}, {best['x_hi']:.3f}]"
        ax.set_title(title)
        ax.grid(True, alpha=0.3)
        return fig

    with PdfPages(pdf_path) as pdf:
        _write_pages(plt, pdf, graphs, a, labels,
                     extra=stability_page if add_stability_page else None)
    print(f"\nWrote summary PDF to: {pdf_path}")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Headless 2D aggregation of detuning sweeps "
                                 "(contrast vs coupling metric / scaled detuning, stable region)")
    ap.add_argument("root", help="directory holding sea_detuning_sweep_* folders (summary.json)")
    ap.add_argument("-o", "--output", default=None,
                    help="PDF path (default <root>/contrast_vs_coupling_summary.pdf)")
    ap.add_argument("--stable", action="store_true",
                    help="also run the stable-region analysis (2D_sweep_report_stable_region.py)")
    ap.add_argument("--c-min", type=float, default=0.2)
    ap.add_argument("--p-min", type=float, default=0.8)
    ap.add_argument("--bin-decimals", type=int, default=3)
    ap.add_argument("--stable-json", default=None)
    ap.add_argument("--add-stability-page", action="store_true")
    a = ap.parse_args(argv)
    root = os.path.abspath(a.root)
    if not os.path.isdir(root):
        print(f"Root folder does not exist: {root}")
        return 2
    pdf = os.path.abspath(a.output) if a.output else os.path.join(root, "contrast_vs_coupling_summary.pdf")
    os.makedirs(os.path.dirname(pdf), exist_ok=True)
    if a.stable:
        sj = os.path.abspath(a.stable_json) if a.stable_json else os.path.join(root, "stable_region_stats.json")
        os.makedirs(os.path.dirname(sj), exist_ok=True)
        make_plots_and_analyze(root, pdf, a.c_min, a.p_min, a.bin_decimals, sj, a.add_stability_page)
    else:
        make_plots(root, pdf)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
