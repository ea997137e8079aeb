"""Sweep report figures (host, matplotlib Agg): the per-point PNGs and the PDF of
sweep_sea_detuning.py:557-1150, drawn from traces the engine already returned.

Off the GPU path: ``run_sweep_sea_detuning`` calls this after every evolution has finished and
times it separately.  Figure content follows the reference (same file names, titles, labels,
curves, slope segments and metric annotations); styling details are not a parity target.
"""
from __future__ import annotations

import os
from typing import Dict, List

import numpy as np


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def _segment(ax, fit: Dict[str, float], style: str, label: str) -> None:
    if not np.isnan(fit["I_z_slope"]):
        ax.plot([fit["t_start"], fit["t_end"]], [fit["I_z_start"], fit["I_z_end"]], style,
                linewidth=2.0, markersize=6, label=label)


def _slope_note(ax, fit: Dict[str, float], dy: float, sign: float, text: str) -> None:
    if np.isnan(fit["I_z_slope"]) or np.isnan(fit["t_start"]):
        return
    tm = 0.5 * (fit["t_start"] + fit["t_end"])
    ym = 0.5 * (fit["I_z_start"] + fit["I_z_end"]) + sign * 0.03 * dy
    ax.text(tm, ym, text, fontsize=6, ha="center", va="bottom", family="monospace",
            bbox=dict(boxstyle="round", alpha=0.2, linewidth=0))


def _zoom(ax, y: np.ndarray) -> float:
    lo, hi = float(np.min(y)), float(np.max(y))
    if hi > lo:
        pad = 0.05 * (hi - lo)
        ax.set_ylim(lo - pad, hi + pad)
    return max(1e-8, hi - lo)


def _side_text(ax, text: str) -> None:
    ax.text(1.02, 0.98, text, transform=ax.transAxes, va="top", ha="left", fontsize=7,
            family="monospace", bbox=dict(boxstyle="round", alpha=0.08), clip_on=False)


def point_figures(per, metrics, det):
    """The four figures of one detuning (:795-1052), as (file name, figure) pairs."""
    plt = _plt()
    d = metrics["delta_Hz"]
    env, fit = det["envelopes"], det["fits"]
    figs = []

    f, ax = plt.subplots()
    for tag, lab in (("center_off", "rare OFF (center)"), ("center_on", "rare ON (center)")):
        ax.plot(per[tag][0], per[tag][1]["Iz_sea"],
                label=r"$\langle I^z_{\mathrm{sea}}\rangle$, " + lab)
    ax.set_xlabel("Time (s)")
    ax.set_ylabel(r"$\langle I^z_{\mathrm{sea}}\rangle$")
    ax.set_title(f"δ_A = {d:+.1f} Hz (rare at center)")
    ax.legend()
    f.tight_layout()
    figs.append(("Iz_sea_off_on_center.png", f))

    f, ax = plt.subplots()
    f.subplots_adjust(right=0.75)
    ax.plot(*env["center_off"], "o-", markersize=3, label="OFF, rare center (envelope)")
    ax.plot(*env["center_on"], "o--", markersize=3, label="ON, rare center (envelope)")
    _segment(ax, fit["center_off"], "s-", "OFF slope, rare center")
    _segment(ax, fit["center_on"], "s--", "ON slope, rare center")
    ax.set_xlabel("Time (s)")
    ax.set_ylabel(r"$\langle I^z_{\mathrm{sea}}\rangle$")
    ax.set_title(f"δ_A = {d:+.1f} Hz (coarse envelopes, rare at center)")
    dy = _zoom(ax, np.concatenate([env["center_off"][1], env["center_on"][1]]))
    s_off, s_on = metrics["I_z_slope_off_center"], metrics["I_z_slope_on_center"]
    _slope_note(ax, fit["center_off"], dy, -1.0, f"OFF slope = {s_off:+.2e}")
    _slope_note(ax, fit["center_on"], dy, +1.0, f"ON slope = {s_on:+.2e}")
    _side_text(ax, f"I_z_slope_off(center)   = {s_off:+.3e}\n"
                   f"t_off(center)           = {metrics['t_off_center']:+.3f}\n"
                   f"I_z_slope_on(center)    = {s_on:+.3e}\n"
                   f"t_on(center)            = {metrics['t_on_center']:+.3f}\n"
                   f"contrast_rare_center    = {metrics['contrast_rare_center']:+.3e}\n"
                   f"ΔΩ/|g_eff|              = {metrics['DeltaOmega_over_geff']:+.3e}")
    ax.legend(fontsize=7, loc="upper left")
    f.tight_layout()
    figs.append(("Iz_sea_detection_envelopes_center.png", f))

    f, ax = plt.subplots()
    f.subplots_adjust(right=0.75)
    ax.plot(*env["shell_off"], "x-", markersize=3, label="Sea-center control (envelope)")
    _segment(ax, fit["shell_off"], "D-", "Slope, sea-center control")
    ax.set_xlabel("Time (s)")
    ax.set_ylabel(r"$\langle I^z_{\mathrm{sea}}\rangle$")
    ax.set_title(f"δ_A = {d:+.1f} Hz (coarse envelope, sea-center control)")
    dy = _zoom(ax, env["shell_off"][1])
    s_sea = metrics["I_z_slope_off_sea_center"]
    _slope_note(ax, fit["shell_off"], dy, +1.0, f"Slope = {s_sea:+.2e}")
    _side_text(ax, f"I_z_slope_sea-center    = {s_sea:+.3e}\n"
                   f"t_sea-center            = {metrics['t_off_sea_center']:+.3f}\n"
                   f"contrast_sea_center     = {metrics['contrast_sea_center']:+.3e}")
    ax.legend(fontsize=7, loc="upper left")
    f.tight_layout()
    figs.append(("Iz_sea_detection_envelopes_sea_center.png", f))

    f, ax = plt.subplots()
    for tag, lab in (("center_off", "rare OFF (center)"), ("center_on", "rare ON (center)")):
        ax.plot(per[tag][0], per[tag][1]["state_norm"], label=r"$\|\psi(t)\|$, " + lab)
    ax.set_xlabel("Time (s)")
    ax.set_ylabel(r"State norm $\|\psi\|$")
    ax.set_title(f"δ_A = {d:+.1f} Hz (state norm, rare at center)")
    ax.legend()
    f.tight_layout()
    figs.append(("state_norm_off_on_center.png", f))
    return figs


def _global_page(plt, gp):
    f, ax = plt.subplots(figsize=(8.27, 11.69))
    ax.axis("off")
    lines = ["Sea detuning sweep report (Ga sea / Al rare)", "",
             "Global parameters (constant across sweep):",
             f"  f_Az (sea Larmor)     = {gp['f_Az_Hz'] / 1e6:.3f} MHz",
             f"  f_Rz (rare Larmor)    = {gp['f_Rz_Hz'] / 1e6:.3f} MHz",
             f"  f1A (sea Rabi)        = {gp['f1A_Hz'] / 1e3:.3f} kHz",
             f"  f1R (rare Rabi)       = {gp['f1R_Hz'] / 1e3:.3f} kHz",
             f"  Target sea detuning   = {gp['target_sea_detuning'] / 1e3:.3f} kHz",
             f"  gamma_sea             = {gp['gamma_sea']:.3e} rad·s⁻¹·T⁻¹",
             f"  gamma_rare            = {gp['gamma_rare']:.3e} rad·s⁻¹·T⁻¹",
             f"  B0_common             = {gp['B0_common_T']:.3f} T",
             f"  B1_sea                = {gp['B1_sea_T']:.3e} T",
             f"  B1_rare               = {gp['B1_rare_T']:.3e} T",
             f"  dipolar_scale_SI      = {gp['dipolar_scale_SI']:.3e}",
             f"  shell_scale           = {gp['shell_scale_m'] * 1e9:.3f} nm",
             f"  t_final               = {gp['t_final_s']:.3e} s",
             f"  steps                 = {gp['steps']:d}",
             f"  n_sea                 = {gp['n_sea']:d}",
             f"  phi_sea               = {gp['phi_sea_rad']:.3f} rad",
             f"  phi_rare              = {gp['phi_rare_rad']:.3f} rad",
             "  sea_spin_type         = 1/2",
             f"  rare_spin_type        = {gp['rare_spin_type']}", ""]
    for k in ("solver_atol", "solver_rtol", "solver_nsteps", "solver_max_step"):
        lines.append(f"  {k:<22}= {gp[k]}")
    lines += ["", f"  coarse_window         = {gp['coarse_window']}", "",
              "Sea detunings (δ_A = f_Az - f_rf,A) in Hz:"]
    ds = [f"{x:+.1f}" for x in gp["sea_detunings_Hz"]]
    lines += ["  " + ", ".join(ds[i:i + 6]) for i in range(0, len(ds), 6)]
    ax.text(0.02, 0.98, "\n".join(lines), transform=ax.transAxes, va="top", family="monospace")
    return f


def _table_page(plt, rows):
    f, ax = plt.subplots(figsize=(8.27, 11.69))
    ax.axis("off")
    cols = ["δ_A (Hz)", "slope_off(center)", "t_off(center)", "slope_on(center)", "t_on(center)",
            "contrast_rare_center", "slope_sea-center", "t_sea-center", "contrast_sea_center"]
    fmt = [("delta_Hz", "+.1f"), ("I_z_slope_off_center", "+.3e"), ("t_off_center", "+.3f"),
           ("I_z_slope_on_center", "+.3e"), ("t_on_center", "+.3f"),
           ("contrast_rare_center", "+.3e"), ("I_z_slope_off_sea_center", "+.3e"),
           ("t_off_sea_center", "+.3f"), ("contrast_sea_center", "+.3e")]
    cells = [[format(r[k], spec) for k, spec in fmt] for r in rows]
    if cells:
        tab = ax.table(cellText=cells, colLabels=cols, loc="center")
        tab.auto_set_font_size(False)
        tab.set_fontsize(6)
        tab.scale(1.0, 1.3)
    ax.set_title("Contrast metrics from coarse-grained ⟨I^z_sea⟩ slopes", pad=20)
    return f


def _contrast_figure(plt, rows):
    x = np.array([r.get("DeltaOmega_over_geff", np.nan) for r in rows], dtype=float)
    y = np.array([r.get("contrast_rare_center", np.nan) for r in rows], dtype=float)
    keep = ~np.isnan(x) & ~np.isnan(y)
    x, y = x[keep], y[keep]
    if x.size == 0:
        return None
    o = np.argsort(x)
    f, ax = plt.subplots(figsize=(6, 4))
    ax.plot(x[o], y[o], "o-", markersize=4)
    ax.set_xlabel(r"$\Delta\Omega / |g_{\mathrm{eff}}|$")
    ax.set_ylabel(r"$\mathrm{contrast\_rare\_center}$")
    ax.set_title(r"Rare-center contrast vs $\Delta\Omega/|g_{\mathrm{eff}}|$")
    ax.grid(True, alpha=0.3)
    f.tight_layout()
    return f


def write_point_pngs(details, dpi: int = 300) -> int:
    """The per-point PNGs of ``details`` ((det_dir, per, metrics, det) rows of write_sweep) only:
    a unit of work a worker process can take on its own (PNG reports have no page order)."""
    plt = _plt()
    n = 0
    for det_dir, per, metrics, det in details:
        for name, f in point_figures(per, metrics, det):
            f.savefig(os.path.join(det_dir, name), dpi=dpi)
            plt.close(f)
            n += 1
    return n


def write_contrast_png(base_dir: str, rows: List[dict], dpi: int = 300) -> None:
    """The sweep-level contrast plot of a PNG report (as write_sweep_report writes it)."""
    plt = _plt()
    try:
        f = _contrast_figure(plt, rows)
        if f is not None:
            f.savefig(os.path.join(base_dir, "contrast_rare_center_vs_DeltaOmega_over_geff.png"), dpi=dpi)
            plt.close(f)
    except Exception as exc:  # the reference only warns here (:1149-1150)
        print(f"Warning: could not build ΔΩ/|g_eff| contrast plot: {exc}")


def write_sweep_report(base_dir: str, global_params: dict, rows: List[dict], details,
                       pdf: bool = True, dpi: int = 300, pngs: bool = True) -> None:
    """PNGs of every point (+ the contrast plot) and, with ``pdf``, sea_detuning_report.pdf;
    ``pngs=False``: the PDF alone (the PNGs drawn elsewhere, e.g. by worker processes)."""
    plt = _plt()
    from matplotlib.backends.backend_pdf import PdfPages
    pages = PdfPages(os.path.join(base_dir, "sea_detuning_report.pdf")) if pdf else None
    try:
        if pages is not None:
            f = _global_page(plt, global_params)
            pages.savefig(f)
            plt.close(f)
        for det_dir, per, metrics, det in details:
            if not pngs and pages is None:
                break
            for name, f in point_figures(per, metrics, det):
                if pngs:
                    f.savefig(os.path.join(det_dir, name), dpi=dpi)
                if pages is not None:
                    pages.savefig(f)
                plt.close(f)
        if pages is not None:
            f = _table_page(plt, rows)
            pages.savefig(f)
            plt.close(f)
        try:
            f = _contrast_figure(plt, rows)
            if f is not None:
                if pngs:
                    f.savefig(os.path.join(base_dir, "contrast_rare_center_vs_DeltaOmega_over_geff.png"),
                              dpi=dpi)
                if pages is not None:
                    pages.savefig(f)
                plt.close(f)
        except Exception as exc:  # the reference only warns here (:1149-1150)
            print(f"Warning: could not build ΔΩ/|g_eff| contrast plot: {exc}")
    finally:
        if pages is not None:
            pages.close()
