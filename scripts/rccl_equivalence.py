#!/usr/bin/env python3
"""RCCL correctness check of every engine on a multi-GPU node (the first step of the 8-GPU campaign).

    python scripts/rccl_equivalence.py --ws 2 8 --out results/summary/rccl_equivalence.json

For each world size N: ``scripts/multirank_check.py`` trains every case (DDP bf16 / fp32 all-reduce,
ZeRO-2 per-micro-step and per-window, ZeRO-3 with re-gathers, FSDP per-block and root, Mistral-shape
GQA under ZeRO-3) with N ranks over RCCL -- one rank per GPU, real asynchronous collectives over
xGMI -- and once with one rank on the concatenated batch; the parameter updates must agree within
bf16 tolerance (tests/multirank_util.compare, the bounds tests/test_multirank_gpu.py uses for the
host-staged run).  Writes one JSON verdict per world size and exits non-zero on any mismatch.
(Reference: train_harness.py:210-271 -- at any world size the trained model is the one the global
batch defines.)
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from multirank_util import compare, run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ws", type=int, nargs="+", default=[2, 8])
    ap.add_argument("--out", default=None)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--timeout", type=int, default=900)
    ap.add_argument("--cases", default=None, help="comma-separated multirank_check.py cases (default: all)")
    ap.add_argument("--seq-len", type=int, default=None)
    a = ap.parse_args()
    ref_batch = 1
    for w in a.ws:                      # every world size must divide the global rows
        while ref_batch % w:
            ref_batch += 1
    extra = ("--ref-batch", str(ref_batch))
    if a.cases:
        extra += ("--cases", a.cases)
    if a.seq_len:
        extra += ("--seq-len", str(a.seq_len))
    env = {k: v for k, v in os.environ.items() if k not in ("DLTB_COMM", "DLTB_COMM_LAZY")}
    verdict, ok = {"ref_batch": ref_batch, "device": a.device, "world_sizes": {}}, True
    with tempfile.TemporaryDirectory() as d:
        os.environ.clear()
        os.environ.update(env)
        ws1 = run(os.path.join(d, "ws1.pt"), 1, a.device, extra=extra, timeout=a.timeout)
        for w in a.ws:
            got = run(os.path.join(d, f"ws{w}.pt"), w, a.device, extra=extra, timeout=a.timeout)
            bad = compare(ws1, got, loss_tol=1e-2, upd_tol=0.08, cos_min=0.995, param_tol=0.2)
            verdict["world_sizes"][str(w)] = {"cases": sorted(got), "mismatches": [list(map(str, b)) for b in bad]}
            print(f"[rccl_equivalence] ws={w}: {len(got)} cases, {len(bad)} mismatches", flush=True)
            ok = ok and not bad
    verdict["pass"] = ok
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(verdict, f, indent=1)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
