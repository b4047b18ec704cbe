#!/usr/bin/env python3
"""One page for the first multi-GPU run of the suite (scripts/run_all_benchmarks.sh step 4).

    python scripts/first_multigpu_report.py --results results --out results/summary/first_multigpu_report.md

Reads what the suite wrote under ``--results``:

* ``summary/metrics.csv`` + ``metrics_extended.csv`` -- the measured curve: tokens/s, step time and the
  efficiency against the same row at 1 GPU, per strategy and world size;
* the newest shipped emulated-fabric prediction table (``bench.prediction_tables()``) -- per row the predicted
  job tokens/s of the same (strategy label, dtype, N) and the error measured / predicted - 1, so a real
  curve grades the emulator (docs/ARCHITECTURE.md section 6.1);
* ``summary/xgmi_buckets.json`` -- the collective sweep, fitted per world size and collective to
  time = alpha + bytes x ring factor / bus bandwidth (comm/topology.fit_alpha_beta), next to the emulator's
  default model;
* ``summary/transport_ab.jsonl`` -- the flagship under each RCCL transport variant;
* ``summary/rccl_equivalence.json`` -- every engine at N ranks against one rank on the global batch.

Everything missing is reported as missing; the script never fails on absent inputs (a 1-GPU suite run still
gets a page that says no multi-GPU row exists).
"""
import argparse
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# suite row -> (prediction-table strategy label, dtype when the sidecar does not say)
ROW_LABEL = {"ddp": ("ddp", "fp16"), "ddp_bf16": ("ddp", "bf16"), "fsdp": ("fsdp", "fp16"),
             "fsdp_bf16": ("fsdp", "bf16"), "fsdp_root": ("fsdp_root", "fp16"), "zero2": ("zero2", "bf16"),
             "zero3": ("zero3", "bf16"), "ddp_zero1": ("ddp_zero1", "bf16")}


def _sidecar(results, strategy, ws, seq):
    """The harness' extended record of one suite row (dtype, comm bytes ...), or {}."""
    pat = os.path.join(results, f"bench-master-{strategy}-ws{ws}-seq{seq}*_results", "*.extended.json")
    for p in sorted(glob.glob(pat)):
        try:
            return json.load(open(p))
        except (OSError, ValueError):
            pass
    return {}


def _fmt(v, spec=",.0f"):
    return "" if v is None else format(v, spec)


def measured_rows(results):
    import pandas as pd
    csv = os.path.join(results, "summary", "metrics.csv")
    if not os.path.exists(csv):
        return []
    df = pd.read_csv(csv, dtype={"tier": str})
    ext_path = os.path.join(results, "summary", "metrics_extended.csv")
    ext = pd.read_csv(ext_path, dtype={"tier": str}) if os.path.exists(ext_path) else None
    rows = []
    for i, r in df.iterrows():
        e = ext.iloc[i] if ext is not None and len(ext) == len(df) else None
        rows.append({"strategy": r["strategy"], "world_size": int(r["world_size"]), "seq_len": int(r["seq_len"]),
                     "tier": str(r["tier"]), "tokens_per_sec": float(r["tokens_per_sec"]),
                     "step_ms": float(r["mean_step_time_sec"]) * 1e3, "peak_vram_gb": float(r["peak_vram_gb"]),
                     "eff_vs_ws1": (None if e is None or e["efficiency_vs_ws1_pct"] != e["efficiency_vs_ws1_pct"]
                                    else float(e["efficiency_vs_ws1_pct"]))})
    return rows


def with_predictions(rows, results):
    import bench
    for r in rows:
        r["predicted"] = r["error"] = r["table"] = None
        lab = ROW_LABEL.get(r["strategy"])
        if lab is None or r["world_size"] < 2:
            continue
        dtype = _sidecar(results, r["strategy"], r["world_size"], r["seq_len"]).get("dtype") or lab[1]
        if r["tier"] != "A":                 # the shipped predictions are TinyGPT-A runs
            continue
        p = bench.predicted_row(f"{lab[0]}-dp{r['world_size']}", dtype, r["world_size"], r["seq_len"])
        if p and p.get("value"):
            r["predicted"], r["table"] = float(p["value"]), p["table"]
            r["error"] = r["tokens_per_sec"] / r["predicted"] - 1.0
    return rows


def fabric_fits(results):
    from dltb.comm.topology import DEFAULT_ALPHA_US, default_bus_gbps, fit_alpha_beta
    path = os.path.join(results, "summary", "xgmi_buckets.json")
    try:
        prof = json.load(open(path))
    except (OSError, ValueError):
        return None, []
    out = []
    for ws, rws in sorted(prof.get("worlds", {}).items(), key=lambda kv: int(kv[0])):
        for op in ("reduce_scatter", "all_gather", "all_reduce"):
            fit = fit_alpha_beta(rws, op, int(ws))
            out.append({"world": int(ws), "op": op, "alpha_us": fit[0] if fit else None,
                        "bus_GBps": fit[1] if fit else None, "model_alpha_us": DEFAULT_ALPHA_US,
                        "model_bus_GBps": default_bus_gbps(int(ws))})
    return prof.get("backend"), out


def transport(results):
    path = os.path.join(results, "summary", "transport_ab.jsonl")
    if not os.path.exists(path):
        return []
    out = []
    for ln in open(path):
        try:
            d = json.loads(ln)
        except ValueError:
            continue
        out.append({"transport": d.get("transport"), "n_gpus": d.get("n_gpus"), "value": d.get("value"),
                    "ms_per_step": d.get("ms_per_step"), "comm_wait_ms": d.get("comm_wait_ms")})
    return out


def write_report(results, out):
    rows = with_predictions(measured_rows(results), results)
    backend, fits = fabric_fits(results)
    tab = transport(results)
    try:
        eq = json.load(open(os.path.join(results, "summary", "rccl_equivalence.json")))
    except (OSError, ValueError):
        eq = None
    multi = [r for r in rows if r["world_size"] > 1]
    L = ["# First multi-GPU run: measured curve, prediction error, fabric fit\n\n",
         f"Results directory: `{os.path.relpath(results, ROOT) if results.startswith(ROOT) else results}`. "
         f"{len(rows)} suite rows, {len(multi)} of them at more than one GPU.\n\n"]
    L += ["## Measured curve\n\n",
          "| Strategy | GPUs | Seq | Tier | Tokens/s (job) | ms / micro-step | Eff vs 1 GPU (%) | Predicted tokens/s | "
          "Error vs prediction |\n", "|---|---:|---:|---|---:|---:|---:|---:|---:|\n"]
    for r in sorted(rows, key=lambda r: (r["strategy"], r["seq_len"], r["world_size"])):
        err = "" if r["error"] is None else f"{100 * r['error']:+.1f} %"
        L.append(f"| {r['strategy']} | {r['world_size']} | {r['seq_len']} | {r['tier']} | {_fmt(r['tokens_per_sec'])} | "
                 f"{r['step_ms']:.2f} | {_fmt(r['eff_vs_ws1'], '.1f')} | {_fmt(r['predicted'])} | {err} |\n")
    if not multi:
        L.append("\nNo row ran on more than one GPU: the predictions stay ungraded.\n")
    errs = [abs(r["error"]) for r in multi if r["error"] is not None]
    if errs:
        tables = sorted({r["table"] for r in multi if r["table"]})
        L.append(f"\nPrediction error over {len(errs)} rows: mean |error| {100 * sum(errs) / len(errs):.1f} %, "
                 f"max {100 * max(errs):.1f} % (prediction table: {', '.join('`' + t + '`' for t in tables)}).\n")
    L += ["\n## Fabric: alpha-beta fit of the collective sweep\n\n"]
    if fits:
        L += [f"Backend `{backend}`. time = alpha + bytes x ring factor / bus bandwidth, least squares over the swept "
              "sizes (comm/topology.fit_alpha_beta); the emulator's default model alongside.\n\n",
              "| GPUs | Collective | alpha (us) | bus (GB/s) | model alpha (us) | model bus (GB/s) |\n",
              "|---:|---|---:|---:|---:|---:|\n"]
        for f in fits:
            L.append(f"| {f['world']} | {f['op']} | {_fmt(f['alpha_us'], '.1f')} | {_fmt(f['bus_GBps'], '.1f')} | "
                     f"{f['model_alpha_us']:.1f} | {f['model_bus_GBps']:.1f} |\n")
    else:
        L.append("No collective sweep (`summary/xgmi_buckets.json`) in this run.\n")
    L += ["\n## RCCL transport A/B (ZeRO-2 flagship, largest world size)\n\n"]
    if tab:
        base = next((t["value"] for t in tab if t["transport"] == "default"), None)
        L += ["| Variant | GPUs | Tokens/s | ms / micro-step | Exposed comm wait (ms) | vs default |\n",
              "|---|---:|---:|---:|---:|---:|\n"]
        for t in tab:
            rel = "" if not (base and t["value"]) else f"{100 * (t['value'] / base - 1):+.1f} %"
            L.append(f"| {t['transport']} | {t['n_gpus']} | {_fmt(t['value'])} | {_fmt(t['ms_per_step'], '.3f')} | "
                     f"{_fmt(t['comm_wait_ms'], '.3f')} | {rel} |\n")
    else:
        L.append("Not run (needs at least 2 GPUs; TRANSPORT_AB=0 skips it).\n")
    L += ["\n## RCCL equivalence (N ranks against one rank on the global batch)\n\n"]
    if eq:
        L.append(f"Verdict: **{'pass' if eq.get('pass') else 'FAIL'}** on device `{eq.get('device')}`.\n\n")
        for ws, v in sorted(eq.get("world_sizes", {}).items(), key=lambda kv: int(kv[0])):
            L.append(f"* {ws} ranks: {len(v.get('cases', []))} cases, {len(v.get('mismatches', []))} mismatches\n")
    else:
        L.append("Not run in this suite.\n")
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        f.write("".join(L))
    print(f"first multi-GPU report: {out}")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--results", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args(argv)
    write_report(os.path.abspath(a.results), a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
