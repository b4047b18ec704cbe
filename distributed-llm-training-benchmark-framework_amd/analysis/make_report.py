"""``BENCHMARK_REPORT.md`` from ``metrics.csv`` (reference: scripts/make_report.py:11-136).

Section structure and table columns follow the reference report — header (timestamp, platform),
Summary table, per-strategy tables (with H2D GB/s), Key Findings (best throughput, best scaling,
lowest peak VRAM), strategy trade-offs, visualisation links, footer — with the platform line naming
the MI355X node instead of OKE/A10 and trade-off notes describing this framework's engines.  When
``metrics_extended.csv`` sits next to the CSV, a "Corrected scaling" section reports efficiency
against the WS=1 baseline and per-GPU throughput.
"""
import argparse
import os
from datetime import datetime
from pathlib import Path

import pandas as pd

PLATFORM = "AMD Instinct MI355X (gfx950, 288 GB HBM3E per GPU), single node, RCCL over xGMI"

SUMMARY_HDR = ("| Strategy | World Size | Seq Len | Tier | Tokens/sec | Step Time (s) | Peak VRAM (GB) | "
               "Scaling Eff (%) |\n"
               "|----------|-----------|---------|------|------------|---------------|----------------|"
               "------------------|\n")
STRAT_HDR = ("| World Size | Seq Len | Tokens/sec | Step Time (s) | Peak VRAM (GB) | H2D GB/s/GPU | "
             "Scaling Eff (%) |\n"
             "|-----------|---------|------------|---------------|----------------|--------------|"
             "------------------|\n")

TRADEOFFS = {
    "DDP": ["Full bf16 replica per GPU, fp32 master weights + Adam moments for the whole model",
            "Gradients live in one flat bf16 buffer; 64 MiB buckets are all-reduced over RCCL as soon as "
            "their last block finishes backward",
            "Highest per-GPU throughput while the model fits (288 GB HBM3E fits TinyGPT A/B and 7B)",
            "Memory: O(model) per GPU (16 bytes/param of model state)"],
    "FSDP": ["One flat bf16 shard per transformer block (plus a root unit); blocks are all-gathered just in "
             "time with next-block prefetch and released after use (FULL_SHARD)",
             "Gradients are reduce-scattered per block, overlapping the rest of the backward",
             "`auto_wrap_policy: size_based` reproduces the reference's single FlatParameter",
             "Memory: O(model / world_size) + one gathered block"],
    "ZERO2": ["Parameters replicated, gradients reduce-scattered every micro-step into fp32 owner shards",
              "Fused AdamW + global-norm clipping run on the 1/N shard; the bf16 result is all-gathered in place",
              "Optimizer step every grad_accum micro-steps (DeepSpeed semantics, WarmupLR)",
              "Memory: parameters replicated, optimizer state and gradients sharded"],
    "ZERO3": ["Parameters sharded per module and fetched on demand with prefetch; small tensors (LayerNorm, "
              "biases) persist replicated",
              "Gathered parameters stay resident for the step when the model fits stage3_max_live_parameters",
              "Largest models per GPU, extra all-gather traffic per step",
              "Memory: O(model / world_size) + live gathered parameters"],
}


def _row_summary(r):
    return (f"| {str(r['strategy']).upper():8s} | {int(r['world_size']):9d} | {int(r['seq_len']):7d} | "
            f"{str(r['tier']):4s} | {r['tokens_per_sec']:10,.0f} | {r['mean_step_time_sec']:13.4f} | "
            f"{r['peak_vram_gb']:14.2f} | {r['scaling_efficiency_pct']:16.1f} |\n")


def _row_strategy(r):
    return (f"| {int(r['world_size']):9d} | {int(r['seq_len']):7d} | {r['tokens_per_sec']:10,.0f} | "
            f"{r['mean_step_time_sec']:13.4f} | {r['peak_vram_gb']:14.2f} | {r['h2d_gbps_per_gpu']:12.3f} | "
            f"{r['scaling_efficiency_pct']:16.1f} |\n")


def generate_report(csv_path: str, output_dir: str, platform: str = PLATFORM) -> Path:
    df = pd.read_csv(csv_path, dtype={"tier": str})
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    path = out / "BENCHMARK_REPORT.md"
    lines = ["# Distributed Training Benchmark Report\n\n",
             f"**Generated:** {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}\n\n",
             f"**Platform:** {platform}\n\n", "---\n\n", "## Summary\n\n", SUMMARY_HDR]
    lines += [_row_summary(r) for _, r in df.iterrows()]
    lines += ["\n---\n\n", "## Strategy Comparison\n\n"]
    for strategy in df["strategy"].unique():
        sub = df[df["strategy"] == strategy].sort_values(["world_size", "seq_len"])
        lines.append(f"### {str(strategy).upper()}\n\n")
        if sub.empty:
            lines.append("No data available.\n\n")
            continue
        lines.append(STRAT_HDR)
        lines += [_row_strategy(r) for _, r in sub.iterrows()]
        lines.append("\n")
    lines += ["---\n\n", "## Key Findings\n\n"]
    best = df.loc[df["tokens_per_sec"].idxmax()]
    eff = df.loc[df["scaling_efficiency_pct"].idxmax()]
    low = df.loc[df["peak_vram_gb"].idxmin()]
    lines.append(f"- **Best Throughput:** {best['tokens_per_sec']:,.0f} tokens/sec "
                 f"({str(best['strategy']).upper()}, WS={int(best['world_size'])}, SeqLen={int(best['seq_len'])})\n")
    lines.append(f"- **Best Scaling Efficiency:** {eff['scaling_efficiency_pct']:.1f}% "
                 f"({str(eff['strategy']).upper()}, WS={int(eff['world_size'])})\n")
    lines.append(f"- **Lowest Peak VRAM:** {low['peak_vram_gb']:.2f} GB "
                 f"({str(low['strategy']).upper()}, WS={int(low['world_size'])})\n")
    ext_path = Path(os.path.dirname(os.path.abspath(csv_path))) / "metrics_extended.csv"
    if ext_path.exists():
        ext = pd.read_csv(ext_path, dtype={"tier": str})
        lines += ["\n---\n\n", "## Corrected Scaling\n\n",
                  "`Scaling Eff` above uses the reference formula (baseline = smallest world size in the group, "
                  "so a group starting at 2 GPUs reads 50 %). The table below normalises to the WS=1 run "
                  "and to the smallest world size.\n\n",
                  "| Strategy | World Size | Tokens/sec/GPU | Eff vs WS=1 (%) | Eff vs min WS (%) |\n",
                  "|----------|-----------|----------------|-----------------|-------------------|\n"]
        for _, r in ext.iterrows():
            v1 = "" if pd.isna(r["efficiency_vs_ws1_pct"]) else f"{r['efficiency_vs_ws1_pct']:.1f}"
            lines.append(f"| {str(r['strategy']).upper():8s} | {int(r['world_size']):9d} | "
                         f"{r['tokens_per_sec_per_gpu']:14,.0f} | {v1:>15s} | {r['efficiency_vs_min_ws_pct']:17.1f} |\n")
        if "tokens_per_gpu_hour" in ext.columns:
            priced = "tokens_per_sec_per_usd_hr" in ext.columns
            lines += ["\n## Cost View\n\n",
                      "Tokens one GPU processes per hour"
                      + (f", and the reference's tokens/sec per $/hr at ${float(ext['gpu_hour_usd'].iloc[0]):.2f} "
                         "per GPU-hour (tps / (world size x price))" if priced else
                         " (set `--gpu-hour-usd` or `DLTB_GPU_HOUR_USD` for the $ columns)") + ".\n\n",
                      "| Strategy | World Size | Seq Len | Tokens/GPU-hour |" + (" Tokens/sec per $/hr | Tokens/$ |" if priced else "") + "\n",
                      "|----------|-----------|---------|-----------------|" + ("---------------------|----------|" if priced else "") + "\n"]
            for _, r in ext.iterrows():
                row = (f"| {str(r['strategy']).upper():8s} | {int(r['world_size']):9d} | {int(r['seq_len']):7d} | "
                       f"{r['tokens_per_gpu_hour']:15,.0f} |")
                if priced:
                    row += f" {r['tokens_per_sec_per_usd_hr']:19,.0f} | {r['tokens_per_usd']:8,.0f} |"
                lines.append(row + "\n")
    lines += ["\n---\n\n", "## Strategy Trade-offs\n\n"]
    titles = {"DDP": "DDP (Distributed Data Parallel)", "FSDP": "FSDP (Fully Sharded Data Parallel)",
              "ZERO2": "ZeRO-2", "ZERO3": "ZeRO-3"}
    for key, notes in TRADEOFFS.items():
        lines.append(f"### {titles[key]}\n")
        lines += [f"- {n}\n" for n in notes]
        lines.append("\n")
    lines += ["---\n\n", "## Visualizations\n\n",
              "![Tokens per second](plots/tokens_per_sec_vs_gpu.png)\n\n",
              "![Step time](plots/step_time_vs_gpu.png)\n\n",
              "![Scaling efficiency](plots/scaling_efficiency.png)\n\n",
              "![Peak VRAM](plots/vram_vs_seqlen.png)\n\n",
              "![Data transfer rate](plots/gbps_vs_gpu.png)\n\n",
              "---\n\n", "**Generated by:** dltb - MI355X Distributed LLM Training Benchmark\n"]
    path.write_text("".join(lines))
    print(f"Report generated: {path}")
    return path


def main(argv=None):
    ap = argparse.ArgumentParser(description="Generate benchmark report")
    ap.add_argument("--csv", required=True, help="Path to metrics.csv")
    ap.add_argument("--out", required=True, help="Output directory for report")
    ap.add_argument("--platform", default=PLATFORM)
    a = ap.parse_args(argv)
    generate_report(a.csv, a.out, a.platform)


if __name__ == "__main__":
    main()
