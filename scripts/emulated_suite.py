#!/usr/bin/env python3
"""Reference-format suite output (result.json per job -> metrics.csv -> plots -> report) from the
PREDICTED emulated-fabric runs of scripts/emulated_scaling.py.

Every N > 1 row is a prediction (one MI355X playing rank 0 of an N-rank job, collectives as
alpha-beta-paced kernels, DLTB_COMM=emulate:N); N = 1 rows are real 1-GPU measurements.  The
report's platform line and a PREDICTED banner say so, and each job's result.extended.json keeps the
bench record (prediction flag, comm model, exposed comm, per-rank peak HBM).

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
        ws = int(rec.get("emulated_world") or rec["n_gpus"])
        seq = int(rec["config"]["seq_len"])
        tier = "M7B" if "Mistral" in rec["config"]["model"] else "A"
        if tier == "M7B":
            label = f"{label}_m7b"
        peak = rec.get("peak_hbm_gb_per_rank", rec.get("peak_hbm_gb", 0.0))
        r = make_record(label, ws, 0, seq, tier, rec["steps"], rec["config"]["micro_batch_per_gpu"],
                        rec["config"]["grad_accum"], rec["ms_per_step"] / 1e3, rec.get("mean_loss", 0.0),
                        peak * 1e9)
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
