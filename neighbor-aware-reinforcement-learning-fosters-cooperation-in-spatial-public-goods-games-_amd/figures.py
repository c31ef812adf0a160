"""Paper figures from the experiment files this package writes.

Restates the reference's plot consumers -- `src/visualization/plotting.py:1-362`
(`setup_matplotlib_for_publication`, `load_data`, `plot_figure_2/4/6/7/8/9`,
`plot_state_comparison`), `scripts/plot_figures.py:19-126` (which experiment
folder feeds which figure) and `scripts/plot_state_comparison.py:19-80` -- over
the per-experiment `data/experiment_data.h5` files that `SPGG.run` and the
batched sweep (`sweep.py`) write.  Those files are HDF5 (h5py, or the HDF5 C
library through `h5native` when h5py is absent) or, without any HDF5 library, an
.npz archive under the same name with the same datasets (`h5io.py`); `load_data`
reads each, so the figures regenerate from this build's output whichever writer
produced it.

Same function names, arguments, dataset names, axes, limits and file names as
the reference; missing files or datasets print a warning and leave the curve
out, as there.  Host-only (matplotlib), nothing here touches the GPU.

    python -m spgg_amd.figures --data-dir results --output-dir paper_figures --figures all
    python -m spgg_amd.figures --state-comparison --data-dir results --r 4.6
"""
from __future__ import annotations

import argparse
import os
from typing import Dict, Iterable, Optional, Sequence, Tuple

import numpy as np

import matplotlib

if not os.environ.get("DISPLAY"):
    matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

from .h5io import read_dataset  # noqa: E402

DATA_FILE = os.path.join("data", "experiment_data.h5")
FIGURES = ("2", "4", "6", "7", "8", "9")
KAPPAS_FIG2 = (0.0, 0.5, 1.0, 1.5, 2.0)          # plot_figures.py:61-63
R_SNAPSHOT_TIMES = (100, 1000, 10000)             # plotting.py:197


def setup_matplotlib_for_publication(font_size_pt=12):
    """One rcParams style for every figure (plotting.py:11-35)."""
    plt.rcParams.update({
        "font.size": font_size_pt,
        "axes.titlesize": font_size_pt,
        "axes.labelsize": font_size_pt,
        "xtick.labelsize": font_size_pt - 2,
        "ytick.labelsize": font_size_pt - 2,
        "legend.fontsize": font_size_pt - 2,
        "figure.titlesize": font_size_pt + 2,
        "font.family": "serif",
        "font.serif": ["Times New Roman", "DejaVu Serif"],
        "text.usetex": False,
        "figure.dpi": 300,
    })
    print(f"Matplotlib style updated for {font_size_pt}pt font.")


def _read_one(filepath: str, name: str) -> Optional[np.ndarray]:
    # HDF5 (h5py, or the HDF5 C library when h5py is absent) or h5io's .npz sink
    return read_dataset(filepath, name)


def load_data(filepath, dataset_name):
    """One dataset of an experiment file, or None (plotting.py:38-67: a missing
    file or dataset is a printed warning, an unreadable file a printed error)."""
    if not os.path.exists(filepath):
        print(f"Warning: Data file not found at {filepath}")
        return None
    try:
        arr = _read_one(filepath, dataset_name)
    except Exception as e:  # noqa: BLE001 - the reference reports and carries on
        print(f"Error loading {filepath}: {e}")
        return None
    if arr is None:
        print(f"Warning: Dataset '{dataset_name}' not found in {filepath}")
    return arr


# ---------------------------------------------------------------------------
# building blocks: a history per curve on a log-t axis
# ---------------------------------------------------------------------------

def _curves(ax, entries: Iterable[Tuple[str, str, Optional[str]]], dataset: str, **kw) -> int:
    """Plot dataset over t = 1..len for each (label, path, color); returns curves drawn."""
    drawn = 0
    for label, path, color in entries:
        y = load_data(path, dataset)
        if y is None:
            continue
        extra = dict(kw)
        if color is not None:
            extra["color"] = color
        ax.plot(np.arange(1, len(y) + 1), y, label=label, **extra)
        drawn += 1
    return drawn


def _log_t(ax, title=None, ylabel=None, xlabel="$t$", legend=True, grid=None, xlim=None, ylim=None):
    if title is not None:
        ax.set_title(title)
    ax.set_xlabel(xlabel)
    if ylabel is not None:
        ax.set_ylabel(ylabel)
    ax.set_xscale("log")
    if xlim is not None:
        ax.set_xlim(*xlim)
    if ylim is not None:
        ax.set_ylim(*ylim)
    if legend:
        ax.legend()
    ax.grid(True, **(grid or {}))


def _save(fig, output_filename, what, tight=True):
    if tight:
        plt.tight_layout()
    plt.savefig(output_filename, bbox_inches="tight")
    plt.close(fig)
    print(f"{what} saved to {output_filename}")


_GRID_BOTH = dict(which="both", ls="--", alpha=0.6)
_GRID_FINE = dict(which="both", ls="--", linewidth=0.5)
_GRID = dict(ls="--", alpha=0.6)


# ---------------------------------------------------------------------------
# the figures (plotting.py:70-362)
# ---------------------------------------------------------------------------

def plot_figure_2(data_paths, output_filename, total_iterations=1000000):
    """f_c(t) per kappa, M=1 | M=2 panels (plotting.py:70-118).
    data_paths: {kappa: {'M1': path, 'M2': path}}."""
    fig, (ax1, ax2) = plt.subplots(1, 2, figsize=(8, 3.5), sharey=True)
    kappas = sorted(data_paths.keys())
    for ax, key, title, ylabel in ((ax1, "M1", "(a) $M=1$", "$f_c$"), (ax2, "M2", "(b) $M=2$", None)):
        _curves(ax, [(f"$\\kappa={k}$", data_paths[k][key], None) for k in kappas], "coop_rate_history")
        _log_t(ax, title, ylabel, grid=_GRID_BOTH, xlim=(1, total_iterations),
               ylim=(0, 1.05) if key == "M1" else None)
    _save(fig, output_filename, "Figure 2")


def plot_figure_4(data_paths, output_filename):
    """Neighbour-influence contribution (%) per kappa (plotting.py:121-148).
    data_paths: {kappa: path}."""
    fig, ax = plt.subplots(figsize=(5.5, 4))
    _curves(ax, [(f"$\\kappa={k}$", data_paths[k], None) for k in sorted(data_paths)],
            "neighbor_influence_percent")
    _log_t(ax, None, r"NI Contribution (%)", xlabel="$t$ ", grid=_GRID_FINE)
    _save(fig, output_filename, "Figure 4")


_MECHANISM_COLORS = {"Hybrid": "C0", "Sole reputation": "C2", "Sole NI": "C1"}


def plot_figure_6(data_paths, output_filename):
    """f_c(t) of the three mechanisms, M=1 | M=2 (plotting.py:151-188).
    data_paths: {'M1': {label: path}, 'M2': {label: path}}."""
    fig, (ax1, ax2) = plt.subplots(1, 2, figsize=(8, 3.5), sharey=True)
    for ax, key, title, ylabel in ((ax1, "M1", "(a) $M=1$", "$f_c$"), (ax2, "M2", "(b) $M=2$", None)):
        _curves(ax, [(lab, p, _MECHANISM_COLORS[lab]) for lab, p in data_paths[key].items()],
                "coop_rate_history")
        _log_t(ax, title, ylabel, legend=key == "M1", grid=_GRID)
    _save(fig, output_filename, "Figure 6")


def plot_figure_7(data_paths, output_filename):
    """Reputation lattices at t = 100, 1000, 10000, one row per mechanism
    (plotting.py:191-240).  data_paths: {label: path} (3 rows)."""
    fig, axes = plt.subplots(nrows=3, ncols=3, figsize=(7, 7.5),
                             gridspec_kw={"hspace": 0.4, "wspace": 0.1})
    cmap, vmin, vmax = plt.cm.viridis, -10, 10
    im = None
    for i, (label, path) in enumerate(data_paths.items()):
        axes[i, 0].set_ylabel(label, fontsize=plt.rcParams["axes.labelsize"], rotation=90, labelpad=20)
        for j, t in enumerate(R_SNAPSHOT_TIMES):
            ax = axes[i, j]
            snap = load_data(path, f"R_snapshot_{t}")
            if snap is None:
                ax.text(0.5, 0.5, "Data Missing", ha="center", va="center", fontsize=8)
            else:
                im = ax.imshow(snap, cmap=cmap, vmin=vmin, vmax=vmax, interpolation="nearest")
            if i == 0:
                ax.set_title(f"$t={t}$")
            ax.set_xticks([])
            ax.set_yticks([])
    fig.subplots_adjust(right=0.85)
    cax = fig.add_axes([0.88, 0.15, 0.03, 0.7])
    if im is None:  # no snapshot anywhere: a colour bar of the fixed range
        im = plt.cm.ScalarMappable(cmap=cmap, norm=plt.Normalize(vmin=vmin, vmax=vmax))
        im.set_array([])
    fig.colorbar(im, cax=cax).set_label("Reputation Value")
    _save(fig, output_filename, "Figure 7", tight=False)


def plot_figure_8(data_paths, output_filename):
    """f_c(t) per neighbourhood order with NI (kappa=1) | without (plotting.py:243-282).
    data_paths: {'with_ni': {M: path}, 'no_ni': {M: path}}."""
    fig, (ax1, ax2) = plt.subplots(1, 2, figsize=(8, 3.5), sharey=True)
    for ax, key, title, ylabel in ((ax1, "with_ni", r"(a) with NI ($\kappa=1.0$)", "$f_c$"),
                                   (ax2, "no_ni", r"(b) no NI ($\kappa=0$)", None)):
        _curves(ax, [(f"$M={M}$", p, None) for M, p in sorted(data_paths[key].items())],
                "coop_rate_history")
        _log_t(ax, title, ylabel, grid=dict(ls="--", alpha=0.6))
    _save(fig, output_filename, "Figure 8")


def plot_figure_9(data_filepath, output_filename):
    """Share of NI from second-order neighbours (%) (plotting.py:285-310); no file
    is written when the dataset is missing."""
    y = load_data(data_filepath, "best_neighbor_second_order_percent")
    if y is None:
        return
    fig, ax = plt.subplots(figsize=(5.5, 4))
    ax.plot(np.arange(1, len(y) + 1), y)
    _log_t(ax, None, r"NI from 2nd-order neighbors (%)", xlabel="$t$ ", legend=False, grid=_GRID_FINE,
           ylim=(50, 80))
    ax.set_xlim(left=1)
    _save(fig, output_filename, "Figure 9")


def plot_state_comparison(data_paths, output_filename, total_iterations=100001):
    """Reputation vs previous-action state: f_c(t) | strategy switches per
    iteration (plotting.py:313-362).  data_paths: {label: path}."""
    fig, (ax1, ax2) = plt.subplots(1, 2, figsize=(10, 4))
    t_all = np.arange(1, total_iterations + 1)
    for label, path in data_paths.items():
        y = load_data(path, "coop_rate_history")
        if y is not None:  # padded with NaN to the nominal length (absorbed runs stop early)
            padded = np.full(total_iterations, np.nan)
            padded[:len(y)] = y
            ax1.plot(t_all, padded, label=label, lw=1.5)
    _log_t(ax1, "(a) Cooperation Rate", "$f_c$", xlabel="$t$ ", grid=_GRID_BOTH,
           xlim=(1, total_iterations), ylim=(-0.05, 1.05))
    for label, path in data_paths.items():
        cd, dc = load_data(path, "switch_C_to_D"), load_data(path, "switch_D_to_C")
        if cd is not None and dc is not None:
            sw = cd + dc
            ax2.plot(np.arange(1, len(sw) + 1), sw, label=label, lw=1.5)
    _log_t(ax2, "(b) System Stability", "Number of Strategy Switches", xlabel="$t$ ", grid=_GRID_BOTH,
           ylim=(-5, 10005))
    _save(fig, output_filename, "State comparison figure")


# ---------------------------------------------------------------------------
# which experiment feeds which figure (scripts/plot_figures.py, plot_state_comparison.py)
# ---------------------------------------------------------------------------

def experiment_file(base_path, r, kappa, use_second_order, w_p, algorithm="qlearning",
                    alpha=0.8, rep_gain_C=1.0, state_representation="reputation"):
    """Data file of one experiment folder (plot_figures.py:19-22: alpha 0.8, rep_gain_C 1.0)."""
    from .sweep import get_folder_name
    return os.path.join(base_path, get_folder_name(r, kappa, use_second_order, alpha, w_p, rep_gain_C,
                                                   state_representation, algorithm), DATA_FILE)


def figure_inputs(base_path, algorithm="qlearning") -> Dict[str, object]:
    """Inputs of figures 2-9 (plot_figures.py:58-124): r=3.6 kappa grid with w_P=1
    for 2/4; the r=3.0 mechanism set (hybrid kappa=1 w_P=0.95, sole reputation
    kappa=0 w_P=0.95, sole NI kappa=1 w_P=1) for 6-9."""
    f = lambda r, k, m2, wp: experiment_file(base_path, r, k, m2, wp, algorithm)  # noqa: E731
    mech = lambda m2: {"Hybrid": f(3.0, 1.0, m2, 0.95),  # noqa: E731
                       "Sole reputation": f(3.0, 0.0, m2, 0.95),
                       "Sole NI": f(3.0, 1.0, m2, 1.0)}
    return {
        "2": {k: {"M1": f(3.6, k, False, 1.0), "M2": f(3.6, k, True, 1.0)} for k in KAPPAS_FIG2},
        "4": {k: f(3.6, k, False, 1.0) for k in KAPPAS_FIG2},
        "6": {"M1": mech(False), "M2": mech(True)},
        "7": {"Sole reputation": f(3.0, 0.0, False, 0.95), "Sole NI": f(3.0, 1.0, False, 1.0),
              "Hybrid mechanism": f(3.0, 1.0, False, 0.95)},
        "8": {"with_ni": {1: f(3.0, 1.0, False, 0.95), 2: f(3.0, 1.0, True, 0.95)},
              "no_ni": {1: f(3.0, 0.0, False, 0.95), 2: f(3.0, 0.0, True, 0.95)}},
        "9": f(3.0, 1.0, True, 0.95),
    }


_PLOTTERS = {"2": plot_figure_2, "4": plot_figure_4, "6": plot_figure_6, "7": plot_figure_7,
             "8": plot_figure_8, "9": plot_figure_9}


def plot_figures(data_dir=".", output_dir="paper_figures", figures: Sequence[str] = ("all",),
                 algorithm="qlearning", total_iterations=1000000) -> Dict[str, str]:
    """Generate the requested paper figures as PDFs (plot_figures.py:27-126);
    returns {figure: output path}."""
    os.makedirs(output_dir, exist_ok=True)
    wanted = list(FIGURES) if "all" in figures else [f for f in FIGURES if f in figures]
    inputs = figure_inputs(data_dir, algorithm)
    out = {}
    for fig in wanted:
        print(f"\n--- Generating Figure {fig} (algorithm: {algorithm}) ---")
        path = os.path.join(output_dir, f"Figure_{fig}.pdf")
        if fig == "2":
            plot_figure_2(inputs[fig], path, total_iterations=total_iterations)
        else:
            _PLOTTERS[fig](inputs[fig], path)
        out[fig] = path
    print("\nAll plotting tasks are complete.")
    return out


def state_comparison(data_dir=".", output_dir="paper_figures", r=4.6, kappa=0.0, use_second_order=False,
                     alpha=0.8, w_p=1.0, rep_gain_c=1.0, total_iterations=100001) -> str:
    """Reputation- vs action-state runs of one parameter point (plot_state_comparison.py:19-80)."""
    os.makedirs(output_dir, exist_ok=True)
    paths = {
        "State: Reputation": experiment_file(data_dir, r, kappa, use_second_order, w_p, "qlearning",
                                             alpha, rep_gain_c, "reputation"),
        "State: Previous Action": experiment_file(data_dir, r, kappa, use_second_order, w_p, "qlearning",
                                                  alpha, rep_gain_c, "action"),
    }
    print("\n--- Generating State Comparison Figure ---")
    out = os.path.join(output_dir, "State_Comparison.pdf")
    plot_state_comparison(paths, out, total_iterations=total_iterations)
    print("\nState comparison plotting complete.")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description="Generate publication figures")
    ap.add_argument("--data-dir", type=str, default=".", help="Base directory containing experiment results")
    ap.add_argument("--output-dir", type=str, default="paper_figures", help="Output directory for figures")
    ap.add_argument("--figures", type=str, nargs="+", choices=list(FIGURES) + ["all"], default=["all"])
    ap.add_argument("--algorithm", type=str, default="qlearning",
                    choices=["qlearning", "sarsa", "expected_sarsa", "double_qlearning"])
    ap.add_argument("--state-comparison", action="store_true",
                    help="the reputation-vs-action figure (scripts/plot_state_comparison.py) instead")
    ap.add_argument("--r", type=float, default=4.6)
    ap.add_argument("--kappa", type=float, default=0.0)
    ap.add_argument("--use-second-order", action="store_true")
    ap.add_argument("--alpha", type=float, default=0.8)
    ap.add_argument("--w-p", type=float, default=1.0)
    ap.add_argument("--rep-gain-c", type=float, default=1.0)
    args = ap.parse_args(argv)
    setup_matplotlib_for_publication(font_size_pt=12)
    if args.state_comparison:
        state_comparison(args.data_dir, args.output_dir, args.r, args.kappa, args.use_second_order,
                         args.alpha, args.w_p, args.rep_gain_c)
    else:
        plot_figures(args.data_dir, args.output_dir, args.figures, args.algorithm)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
