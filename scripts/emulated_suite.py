#!/usr/bin/env python3
"""Reference-format suite output (result.json per job -> metrics.csv -> plots -> report) from the
PREDICTED emulated-fabric runs of scripts/emulated_scaling.py.

Every N > 1 row is a prediction (one MI355X playing rank 0 of an N-rank job, collectives as
alpha-beta-paced kernels, DLTB_COMM=emulate:N); N = 1 rows are real 1-GPU measurements.  Every
strategy label carries a ``_pred`` suffix (``zero2_pred``) and every result.json a ``prediction``
flag and ``emulated_world``, so metrics.csv, the plots and any aggregator see which rows are
predicted; the report's platform line and a PREDICTED banner say so too, and each job's
result.extended.json keeps the bench record (comm model, exposed comm, per-rank peak HBM).

    python scripts/emulated_suite.py profiles/emulated_scaling_r3.jsonl results/example_output_mi355x_emulated
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PLATFORM = ("PREDICTED: emulated 8x MI355X xGMI fabric on ONE MI355X (DLTB_COMM=emulate:N, alpha-beta "
            "collective model); WS=1 rows measured")


def main():
    src, out = sys.argv[1], sys.argv[2]
    from dltb.results.record import make_record
    os.makedirs(out, exist_ok=True)
    n = 0
    for ln in open(src):
        rec = json.loads(ln)
        label = rec["config"]["parallelism"].rsplit("-dp", 1)[0]
        if label.split("_")[0] in ("ddp", "fsdp") and rec.get("dtype") == "bf16":
            label += "_bf16"                 # BASELINE configs #2 / #3 (the reference runs fp16 there)
        ws = int(rec.get("emulated_world") or rec["n_gpus"])
        seq = int(rec["config"]["seq_len"])
        tier = "M7B" if "Mistral" in rec["config"]["model"] else "A"
        if tier == "M7B":
            label = f"{label}_m7b"
        peak = rec.get("peak_hbm_gb_per_rank", rec.get("peak_hbm_gb", 0.0))
        # every row of a predicted series carries the "_pred" label (its WS=1 row is the measured
        # 1-GPU baseline the series is predicted from, kept in the group so the efficiency columns
        # have their baseline), and result.json says per row whether it is a prediction
        pred = bool(rec.get("prediction"))
        # grad_accum: the CLI value, as the harness writes it (the reference's DDP/FSDP ignore it,
        # the engine's accum is 1 there); bench records without the field come from --grad-accum 4
        accum_cli = int(rec["config"].get("grad_accum_cli", 4))
        r = make_record(f"{label}_pred", ws, 0, seq, tier, rec["steps"], rec["config"]["micro_batch_per_gpu"],
                        accum_cli, rec["ms_per_step"] / 1e3, rec.get("mean_loss", 0.0), peak * 1e9)
        r["prediction"] = pred
        r["emulated_world"] = ws if pred else None
        label = f"{label}_pred"
        job = os.path.join(out, f"bench-master-{label}-ws{ws}-seq{seq}_results")
        os.makedirs(job, exist_ok=True)
        with open(os.path.join(job, "result.json"), "w") as f:
            json.dump(r, f, indent=2)
        with open(os.path.join(job, "result.extended.json"), "w") as f:
            json.dump(rec, f, indent=2)
        n += 1
    summ = os.path.join(out, "summary")
    py = sys.executable
    subprocess.run([py, os.path.join(ROOT, "scripts", "parse_metrics.py"), "--results-dir", out, "--out", summ], check=True)
    subprocess.run([py, os.path.join(ROOT, "scripts", "plot.py"), "--results", os.path.join(summ, "metrics.csv"),
                    "--out", os.path.join(summ, "plots")], check=True)
    subprocess.run([py, os.path.join(ROOT, "scripts", "make_report.py"), "--csv", os.path.join(summ, "metrics.csv"),
                    "--out", summ, "--platform", PLATFORM], check=True)
    rep = os.path.join(summ, "BENCHMARK_REPORT.md")
    with open(rep) as f:
        body = f.read()
    with open(rep, "w") as f:
        f.write("> **PREDICTED RESULTS.** Every multi-GPU row below comes from the emulated fabric on a single "
                "MI355X (`bench.py --emulate N`, docs/ARCHITECTURE.md §6.1), not from N GPUs.\n\n" + body)
    print(f"[emulated_suite] {n} jobs -> {summ}")


if __name__ == "__main__":
    main()
