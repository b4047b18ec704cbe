"""Aggregate ``result.json`` files into ``metrics.csv`` (reference: scripts/parse_metrics.py:12-87).

Output contract:

* input: every file named exactly ``result.json`` below ``--results-dir`` (the collector layout
  ``<job>_results/result.json``; the harness-side ``result_*.json`` names are NOT matched, as in the
  reference);
* rows sorted by ``[strategy, world_size, seq_len]``; columns = the 13 record keys in record order
  plus ``scaling_efficiency_pct``;
* ``scaling_efficiency_pct`` uses the reference formula per (strategy, seq_len) group with more than
  one row: ``tps / (tps_of_first_row_at_min_ws * ws) * 100`` (single-row groups keep 100.0).  When
  the smallest world size in a group is 2 this reads 50 % for the 2-GPU row — reproduced verbatim
  for CSV compatibility, including the grouping: a result set that mixes tiers at one (strategy,
  seq_len) takes the first row at the smallest world size as the base, as the reference does.

The corrected numbers go to ``metrics_extended.csv``: the reference formula grouped by tier too
(``efficiency_tier_aware_pct``: the reference's long-sequence Tier B rows, run_all_benchmarks.sh:49-51,
are otherwise the 1-GPU base of the Tier A rows -- a 1-GPU Tier A row reads 487 % against the Tier B
row of the same strategy and sequence length), efficiency normalised to the group's WS=1 row (true
weak-scaling efficiency), efficiency normalised to the smallest world size
(``tps / (tps_min * ws / ws_min)``), per-GPU tokens/s, the cost view (tokens per GPU-hour; with a GPU
price -- ``--gpu-hour-usd`` / ``DLTB_GPU_HOUR_USD`` -- the reference's "tokens/sec per $/hr" =
tps / (ws x price), README.md:266-277 of the reference), and the harness' extended sidecar fields when
a ``result.extended.json`` / ``result_*.extended.json`` sits next to the record.
"""
import os
import argparse
import json
from pathlib import Path

import pandas as pd

SUMMARY_COLS = ["strategy", "world_size", "seq_len", "tier", "tokens_per_sec", "mean_step_time_sec",
                "peak_vram_gb", "h2d_gbps_per_gpu", "scaling_efficiency_pct"]


def load_records(results_dir):
    root = Path(results_dir)
    files = sorted(root.rglob("result.json"))
    records, sources = [], []
    for path in files:
        try:
            with open(path) as f:
                records.append(json.load(f))
            sources.append(path)
        except Exception as e:  # noqa: BLE001 - a broken file must not stop the aggregation
            print(f"WARNING: Failed to parse {path}: {e}")
    return records, sources


def reference_efficiency(df: pd.DataFrame, by_tier: bool = False) -> pd.Series:
    """The reference formula (scripts/parse_metrics.py:51-63): groups by (strategy, seq_len); ``by_tier``
    adds the tier to the key (the extended CSV's corrected column)."""
    eff = pd.Series(100.0, index=df.index)
    keys = ["strategy", "seq_len"] + (["tier"] if by_tier and "tier" in df.columns else [])
    for _, grp in df.groupby(keys, sort=False):
        if len(grp) < 2:
            continue
        base = grp[grp["world_size"] == grp["world_size"].min()].iloc[0]["tokens_per_sec"]
        for idx, row in grp.iterrows():
            ideal = base * row["world_size"]
            eff[idx] = (row["tokens_per_sec"] / ideal * 100.0) if ideal > 0 else 0.0
    return eff


def gpu_hour_price(price=None):
    """$ per GPU-hour for the cost view: the argument, else DLTB_GPU_HOUR_USD, else None (no $ column)."""
    if price is None:
        price = os.environ.get("DLTB_GPU_HOUR_USD")
    try:
        price = float(price) if price not in (None, "") else None
    except ValueError:
        price = None
    return price if price and price > 0 else None


def extended_frame(df: pd.DataFrame, sources, gpu_hour_usd=None) -> pd.DataFrame:
    ext = df[["strategy", "world_size", "seq_len", "tier", "tokens_per_sec", "mean_step_time_sec",
              "peak_vram_gb"]].copy()
    ext["tokens_per_sec_per_gpu"] = ext["tokens_per_sec"] / ext["world_size"]
    ext["efficiency_tier_aware_pct"] = reference_efficiency(df, by_tier=True)
    # cost view: tokens one GPU processes per hour; with a price, the reference's tokens/sec per $/hr
    ext["tokens_per_gpu_hour"] = ext["tokens_per_sec_per_gpu"] * 3600.0
    price = gpu_hour_price(gpu_hour_usd)
    if price is not None:
        ext["gpu_hour_usd"] = price
        ext["tokens_per_sec_per_usd_hr"] = ext["tokens_per_sec"] / (ext["world_size"] * price)
        ext["tokens_per_usd"] = ext["tokens_per_gpu_hour"] / price
    ext["efficiency_vs_ws1_pct"] = float("nan")
    ext["efficiency_vs_min_ws_pct"] = float("nan")
    for (_, _, _), grp in ext.groupby(["strategy", "seq_len", "tier"], sort=False):
        ws_min = grp["world_size"].min()
        base_min = grp[grp["world_size"] == ws_min].iloc[0]["tokens_per_sec"]
        one = grp[grp["world_size"] == 1]
        for idx, row in grp.iterrows():
            ext.loc[idx, "efficiency_vs_min_ws_pct"] = row["tokens_per_sec"] / (base_min * row["world_size"] / ws_min) * 100.0
            if len(one):
                ext.loc[idx, "efficiency_vs_ws1_pct"] = row["tokens_per_sec"] / (one.iloc[0]["tokens_per_sec"] * row["world_size"]) * 100.0
    # sidecar fields (harness extended records), matched by directory
    extras = []
    for src in sources:
        cand = list(Path(src).parent.glob("*.extended.json"))
        data = {}
        if cand:
            try:
                with open(cand[0]) as f:
                    e = json.load(f)
                data = {k: e.get(k) for k in ("tflops_per_gpu", "mfu_vs_2.5PF_dense_bf16", "wall_time_timed_sec",
                                               "comm_bytes_per_step_per_gpu", "peak_vram_reserved_gb",
                                               "optimizer_steps", "engine", "accum_semantics")}
            except Exception:
                data = {}
        extras.append(data)
    if any(extras):
        side = pd.DataFrame(extras, index=df.index)
        ext = pd.concat([ext, side], axis=1)
    return ext


def parse_results(results_dir: str, output_dir: str, gpu_hour_usd=None):
    out = Path(output_dir)
    out.mkdir(parents=True, exist_ok=True)
    records, sources = load_records(results_dir)
    if not records:
        print(f"WARNING: No result.json files found in {results_dir}")
        print("Expected files like: bench-master-*_results/result.json")
        return None
    print(f"Found {len(records)} result files")
    df = pd.DataFrame(records)
    order = df.sort_values(by=["strategy", "world_size", "seq_len"]).index
    df = df.loc[order]
    srcs = [sources[i] for i in order]
    df["scaling_efficiency_pct"] = reference_efficiency(df)
    csv = out / "metrics.csv"
    df.to_csv(csv, index=False)
    print(f"\nMetrics saved to: {csv}")
    ext = extended_frame(df, srcs, gpu_hour_usd)
    ext.to_csv(out / "metrics_extended.csv", index=False)
    print("\n=== Summary ===")
    print(df[SUMMARY_COLS].to_string(index=False))
    return df


def main(argv=None):
    ap = argparse.ArgumentParser(description="Parse benchmark results to CSV")
    ap.add_argument("--results-dir", required=True, help="Directory containing result JSON files")
    ap.add_argument("--out", required=True, help="Output directory for metrics.csv")
    ap.add_argument("--gpu-hour-usd", type=float, default=None,
                    help="$ per GPU-hour for the cost columns of metrics_extended.csv (default: $DLTB_GPU_HOUR_USD)")
    a = ap.parse_args(argv)
    parse_results(a.results_dir, a.out, a.gpu_hour_usd)


if __name__ == "__main__":
    main()
