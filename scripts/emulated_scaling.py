#!/usr/bin/env python3
"""PREDICTED scaling table from the emulated fabric (DLTB_COMM=emulate:N) on ONE MI355X.

For every strategy this runs the measured 1-GPU bench (real, no collectives) and then
``bench.py --emulate N`` for N in --worlds: one process plays rank 0 of the N-rank job with the
real N-rank layouts, shards, bucket plans and per-rank memory, and every collective is an
alpha-beta-paced kernel on a high-priority side stream (csrc/comm_emu.hip).  The step time it
measures is a PREDICTION of the N-GPU step: overlap, exposed communication and CU/HBM contention
are real, the xGMI fabric is the model of comm/topology.py.  Efficiency columns are predictions
too: per-GPU predicted throughput / measured 1-GPU throughput.

    python scripts/emulated_scaling.py --out profiles/emulated_scaling_r3.txt [--worlds 2 4 8]
                                       [--strategies ddp fsdp fsdp_root zero2 zero3] [--m7b]

Reference rows this must eventually predict: /root/reference/README.md:214-223 (2 / 4 GPUs).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# label -> bench.py flags (the reference's precision per strategy: bench.py --dtype auto)
STRATS = {
    "ddp": ["--strategy", "ddp"],
    "fsdp": ["--strategy", "fsdp"],
    "fsdp_root": ["--strategy", "fsdp", "--fsdp-wrap", "root"],
    "zero2": ["--strategy", "zero2"],
    "zero3": ["--strategy", "zero3"],
    # BASELINE configs #2 / #3 name DDP and FSDP full-shard in bf16
    "ddp_bf16": ["--strategy", "ddp", "--dtype", "bf16"],
    "fsdp_bf16": ["--strategy", "fsdp", "--dtype", "bf16"],
    # FSDP SHARD_GRAD_OP (configs/fsdp/fsdp_config.yaml's alternative, SURVEY §7.4 phase 3): the parameters
    # gathered for the forward stay until the backward, so the backward re-gathers nothing (288 GB holds them)
    "fsdp_sgo": ["--strategy", "fsdp", "--fsdp-sharding", "shard_grad_op"],
    "fsdp_bf16_sgo": ["--strategy", "fsdp", "--dtype", "bf16", "--fsdp-sharding", "shard_grad_op"],
    # DDP + ZeroRedundancyOptimizer: config #2's update with the optimizer state sharded (reduce-scatter +
    # all-gather, the all-reduce's wire bytes) -- the replicated full-model AdamW every micro-step goes
    "ddp_bf16_zero1": ["--strategy", "ddp", "--dtype", "bf16", "--ddp-shard-optimizer"],
}


def run(args, timeout, env_extra=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DLTB_COMM"):
        env.pop(k, None)
    env.update(env_extra or {})
    t0 = time.time()
    try:
        r = subprocess.run(["timeout", "-k", "10", str(timeout), sys.executable, os.path.join(ROOT, "bench.py"), *args],
                           capture_output=True, text=True, env=env)
    except OSError as e:
        return None, str(e)
    recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not recs:
        return None, f"rc={r.returncode} {r.stderr[-800:]}"
    rec = recs[0]
    rec["_wall_s"] = time.time() - t0
    return rec, None


def fmt_row(label, n, rec, base):
    ms = rec["ms_per_step"]
    tps = rec["value"]
    eff = (tps / n) / base["value"] if base else None
    cw = rec.get("comm_wait_ms")
    cm = rec.get("comm_model_ms_per_step")
    host = rec.get("host_over_gpu")
    peak = rec.get("peak_hbm_gb_per_rank", rec.get("peak_hbm_gb"))
    return (f"{label:<10} {n:>2} {'pred' if rec.get('prediction') else 'meas':>4} {ms:9.3f} {tps:12.0f} "
            f"{tps / n:10.0f} {('%6.1f%%' % (100 * eff)) if eff else '     -':>7} "
            f"{('%7.3f' % cw) if cw is not None else '      -':>7} {('%8.3f' % cm) if cm else '       -':>8} "
            f"{peak:8.2f} {('%5.2f' % host) if host else '    -':>5}  {rec['config']['parallelism']}")


HEADER = (f"{'strategy':<10} {'N':>2} {'kind':>4} {'ms/step':>9} {'tok/s(job)':>12} {'tok/s/GPU':>10} "
          f"{'eff':>7} {'cwait':>7} {'comm_mdl':>8} {'peakGB':>8} {'h/g':>5}  parallelism")


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "emulated_scaling.txt"))
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--strategies", nargs="*", default=list(STRATS))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--m7b", action="store_true", help="also Mistral-7B-shape ZeRO-3 at N = 8 (BASELINE config #5)")
    ap.add_argument("--extra", nargs=argparse.REMAINDER, default=[], help="more bench.py flags for every run")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    jsonl = os.path.splitext(a.out)[0] + ".jsonl"
    lines = []
    model = {}

    def emit(s):
        print(s, flush=True)
        lines.append(s)
        with open(a.out, "w") as f:
            f.write("\n".join(lines) + "\n")

    def keep(rec):
        with open(jsonl, "a") as f:
            f.write(json.dumps(rec) + "\n")

    emit("# PREDICTED scaling on the emulated fabric (DLTB_COMM=emulate:N) -- ONE MI355X plays rank 0;")
    emit("# collectives are alpha-beta-paced kernels on a side stream; N>1 rows are predictions, not")
    emit("# measurements of N GPUs. kind=meas rows are real 1-GPU runs. eff = predicted tok/s/GPU / measured 1-GPU.")
    emit("# cwait = exposed collective wait after the last backward kernel (ms/step); comm_mdl = modelled")
    emit("# fabric busy time (ms/step, overlapped or not); h/g = host enqueue / GPU time per step.")
    emit(HEADER)
    common = ["--steps", str(a.steps), "--warmup", str(a.warmup), *a.extra]
    for label in a.strategies:
        flags = STRATS[label]
        base, err = run(flags + common, 300)
        if base is None:
            emit(f"{label:<10}  1 meas FAILED {err}")
            continue
        keep(base)
        emit(fmt_row(label, 1, base, base))
        for n in a.worlds:
            host = ["--host-check"] if n == max(a.worlds) else []
            rec, err = run(flags + common + ["--emulate", str(n)] + host, 300)
            if rec is None:
                emit(f"{label:<10} {n:>2} pred FAILED {err}")
                continue
            keep(rec)
            model = rec.get("comm_model") or model
            emit(fmt_row(label, n, rec, base))
    if a.m7b:
        m7 = ["--strategy", "zero3", "--tier", "M7B", "--seq-len", "4096", "--steps", "6", "--warmup", "6"]
        for cfg in ("zero3.json", "zero3_mi355x_288gb.json"):
            ds = ["--deepspeed-config", os.path.join(ROOT, "configs", "deepspeed", cfg)]
            rec, err = run(m7 + ds + ["--emulate", "8", "--host-check"], 900)
            if rec is None:
                emit(f"M7B-zero3  8 pred FAILED ({cfg}) {err}")
                continue
            keep(rec)
            emit(fmt_row("M7B-z3", 8, rec, None) + f"  [{cfg}] trainable={rec.get('trainable_params')}")
    emit("# comm model: " + json.dumps(model))


if __name__ == "__main__":
    main()
