"""Benchmark result record and export — byte-compatible with the reference
(train_harness.py:399-456).

* the 13-key record in the reference's key order (the CSV columns follow it);
* ``result_{strategy}_ws{ws}_seq{seq}_tier{tier}.json`` written with ``indent=2`` by rank 0;
* the stdout block ``BENCHMARK_RESULT_JSON_START`` / ``..._END`` framed by 80 '=' rules, which the
  collector scrapes into ``<job>_results/result.json``.

Anything new (synchronised wall time, TFLOP/s, MFU, comm bytes, memory breakdown, grad norm ...)
goes into a sidecar ``result_...extended.json`` — never into the record, because pandas turns every
key into a CSV column and would shift ``scaling_efficiency_pct``.
"""
import json
import os
from collections import OrderedDict

RESULT_KEYS = ("strategy", "world_size", "rank", "seq_len", "tier", "steps", "per_device_batch",
               "grad_accum", "tokens_per_sec", "mean_step_time_sec", "mean_loss", "peak_vram_gb",
               "h2d_gbps_per_gpu")
MARK_START = "BENCHMARK_RESULT_JSON_START"
MARK_END = "BENCHMARK_RESULT_JSON_END"
RULE = "=" * 80


def make_record(strategy, world_size, rank, seq_len, tier, steps, per_device_batch, grad_accum,
                mean_step_time_sec, mean_loss, peak_vram_bytes) -> "OrderedDict":
    tokens_per_step = per_device_batch * seq_len * world_size
    tps = tokens_per_step / mean_step_time_sec if mean_step_time_sec > 0 else 0.0
    # reference "H2D" proxy: 4 bytes/token of one rank's micro-batch per step (train_harness.py:412-413)
    h2d = (per_device_batch * seq_len * 4 / mean_step_time_sec) / 1e9 if mean_step_time_sec > 0 else 0.0
    vals = (strategy, world_size, rank, seq_len, tier, steps, per_device_batch, grad_accum, tps,
            mean_step_time_sec, mean_loss, peak_vram_bytes / 1e9, h2d)
    return OrderedDict(zip(RESULT_KEYS, vals))


def result_filename(strategy, world_size, seq_len, tier) -> str:
    return f"result_{strategy}_ws{world_size}_seq{seq_len}_tier{tier}.json"


def write_result(record, results_dir, extended=None) -> str:
    os.makedirs(results_dir, exist_ok=True)
    path = os.path.join(results_dir, result_filename(record["strategy"], record["world_size"],
                                                     record["seq_len"], record["tier"]))
    with open(path, "w") as f:
        json.dump(record, f, indent=2)
    if extended is not None:
        with open(path[:-len(".json")] + ".extended.json", "w") as f:
            json.dump(extended, f, indent=2, default=str)
    return path


def print_result(record):
    print("\n" + RULE)
    print("Benchmark Results:")
    print(f"  Tokens/sec:       {record['tokens_per_sec']:,.0f}")
    print(f"  Mean step time:   {record['mean_step_time_sec']:.4f}s")
    print(f"  Peak VRAM/GPU:    {record['peak_vram_gb']:.2f} GB")
    print(f"  H2D GB/s/GPU:     {record['h2d_gbps_per_gpu']:.3f}")
    print(f"  Mean loss:        {record['mean_loss']:.4f}")
    print(RULE + "\n")


def print_markers(record):
    print("\n" + RULE)
    print(MARK_START)
    print(json.dumps(record, indent=2))
    print(MARK_END)
    print(RULE + "\n", flush=True)


def extract_from_log(text: str):
    """Parse the JSON between the markers of a log (collect_results.sh equivalent)."""
    if MARK_START not in text:
        return None
    body = text.split(MARK_START, 1)[1].split(MARK_END, 1)[0]
    return json.loads(body)
