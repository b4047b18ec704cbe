"""Benchmark plots from ``metrics.csv`` (reference: scripts/plot.py:13-110).

Same five files, titles and axes as the reference (matplotlib Agg, 10x6 in, 150 dpi):
``tokens_per_sec_vs_gpu.png``, ``step_time_vs_gpu.png``, ``vram_vs_seqlen.png`` (only when more
than one sequence length is present), ``scaling_efficiency.png`` (0-110 %, dashed ideal line) and
``gbps_vs_gpu.png``; one line per strategy, labelled in upper case.  A result set that mixes sequence
lengths, tiers or world sizes (e.g. the 1-GPU multi-sequence suite, configs/suite/multiseq_1gpu.txt) gets one
line per strategy AND per value of the columns that vary and are not the plot's x axis (``ZERO3 seq4096``,
``ZERO3 tier B``): the reference's per-strategy lines would join points of different shapes.
"""
import argparse
from pathlib import Path

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import pandas as pd  # noqa: E402

PLOTS = [
    # file, x column, y column, x label, y label, title, sort key
    ("tokens_per_sec_vs_gpu.png", "world_size", "tokens_per_sec", "World Size (GPUs)", "Tokens/sec",
     "Tokens/sec vs GPU Count"),
    ("step_time_vs_gpu.png", "world_size", "mean_step_time_sec", "World Size (GPUs)", "Mean Step Time (sec)",
     "Step Time vs GPU Count"),
    ("vram_vs_seqlen.png", "seq_len", "peak_vram_gb", "Sequence Length", "Peak VRAM (GB)",
     "Peak VRAM vs Sequence Length"),
    ("scaling_efficiency.png", "world_size", "scaling_efficiency_pct", "World Size (GPUs)",
     "Scaling Efficiency (%)", "Scaling Efficiency vs GPU Count"),
    ("gbps_vs_gpu.png", "world_size", "h2d_gbps_per_gpu", "World Size (GPUs)", "H2D GB/s per GPU",
     "Data Transfer Rate vs GPU Count"),
]


def _series(df, xcol):
    """(label, rows) per line: strategy, plus every shape column that varies and is not the x axis."""
    extra = [c for c in ("seq_len", "tier", "world_size") if c != xcol and c in df.columns and df[c].nunique() > 1]
    tag = {"seq_len": "seq{}", "tier": "tier {}", "world_size": "ws{}"}
    out = []
    for key, sub in df.groupby(["strategy"] + extra, sort=False):
        key = key if isinstance(key, tuple) else (key,)
        label = " ".join([str(key[0]).upper()] + [tag[c].format(v) for c, v in zip(extra, key[1:])])
        out.append((label, sub))
    return out


def _one(df, out, fname, xcol, ycol, xlabel, ylabel, title):
    fig, ax = plt.subplots(figsize=(10, 6))
    for label, sub in _series(df, xcol):
        sub = sub.sort_values(xcol)
        ax.plot(sub[xcol], sub[ycol], marker="o", linewidth=2, label=label)
    if ycol == "scaling_efficiency_pct":
        ax.axhline(y=100, color="gray", linestyle="--", alpha=0.5, label="Ideal (100%)")
        ax.set_ylim(0, 110)
    ax.set_xlabel(xlabel, fontsize=12)
    ax.set_ylabel(ylabel, fontsize=12)
    ax.set_title(title, fontsize=14, fontweight="bold")
    ax.legend()
    ax.grid(True, alpha=0.3)
    fig.tight_layout()
    path = out / fname
    fig.savefig(path, dpi=150)
    plt.close(fig)
    print(f"Plot saved: {path}")
    return path


def plot_metrics(csv_path: str, output_dir: str):
    df = pd.read_csv(csv_path)
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    print(f"Loaded {len(df)} records from {csv_path}")
    written = []
    for fname, xcol, ycol, xl, yl, title in PLOTS:
        if fname == "vram_vs_seqlen.png" and df["seq_len"].nunique() <= 1:
            continue
        written.append(_one(df, out, fname, xcol, ycol, xl, yl, title))
    print(f"\nAll plots saved to: {output_dir}")
    return written


def main(argv=None):
    ap = argparse.ArgumentParser(description="Generate benchmark plots")
    ap.add_argument("--results", required=True, help="Path to metrics.csv")
    ap.add_argument("--out", required=True, help="Output directory for plots")
    a = ap.parse_args(argv)
    plot_metrics(a.results, a.out)


if __name__ == "__main__":
    main()
