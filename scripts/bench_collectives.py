#!/usr/bin/env python3
"""RCCL collective sweep over xGMI (the data behind the engines' bucket-size defaults).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \\
        scripts/bench_collectives.py [--min-mb 1] [--max-mb 1024] [--dtype bf16] [--ops all_reduce,...]

For every op and message size (powers of two) it times ``iters`` calls between barriers and
reports algorithm bandwidth (bytes / time) and bus bandwidth (the NCCL-tests convention:
all_reduce x 2(n-1)/n, reduce_scatter / all_gather / all_to_all x (n-1)/n), max over ranks.
Rank 0 prints a table and, with --json, writes the rows.  ``--backend gloo --device cpu`` runs the
same sweep on the CPU (used by the tests).
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist

DT = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}


def bus_factor(op, n):
    return 2.0 * (n - 1) / n if op == "all_reduce" else (n - 1) / n


def run_op(op, buf, out, world):
    if op == "all_reduce":
        dist.all_reduce(buf)
    elif op == "reduce_scatter":
        dist.reduce_scatter_tensor(out, buf)
    elif op == "all_gather":
        dist.all_gather_into_tensor(buf, out)
    elif op == "all_to_all":
        dist.all_to_all_single(out if out.numel() == buf.numel() else buf.clone(), buf)
    else:
        raise ValueError(op)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-mb", type=float, default=1)
    ap.add_argument("--max-mb", type=float, default=1024)
    ap.add_argument("--dtype", default="bf16", choices=list(DT))
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather,all_to_all")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if a.device == "cuda":
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        dist.init_process_group(a.backend, rank=rank, world_size=world, device_id=dev)
        sync = torch.cuda.synchronize
    else:
        dev = torch.device("cpu")
        dist.init_process_group(a.backend, rank=rank, world_size=world)
        sync = (lambda: None)
    dt = DT[a.dtype]
    esz = torch.tensor([], dtype=dt).element_size()
    rows = []
    size = a.min_mb
    while size <= a.max_mb + 1e-9:
        nbytes = int(size * (1 << 20))
        n = max(world, nbytes // esz // world * world)
        buf = torch.ones(n, dtype=dt, device=dev)
        out = torch.empty(n // world, dtype=dt, device=dev)
        for op in a.ops.split(","):
            o = out if op != "all_to_all" else torch.empty_like(buf)
            for _ in range(a.warmup):
                run_op(op, buf, o, world)
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                run_op(op, buf, o, world)
            sync()
            dt_s = (time.perf_counter() - t0) / a.iters
            t = torch.tensor([dt_s], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt_s = float(t.item())
            bytes_ = n * esz
            algbw = bytes_ / dt_s / 1e9
            rows.append({"op": op, "bytes": bytes_, "time_us": dt_s * 1e6, "algbw_GBps": algbw,
                         "busbw_GBps": algbw * bus_factor(op, world), "world": world})
        size *= 2
    if rank == 0:
        print(f"{'op':16s} {'size':>10s} {'time(us)':>10s} {'algbw GB/s':>11s} {'busbw GB/s':>11s}  (world {world})")
        for r in rows:
            print(f"{r['op']:16s} {r['bytes'] / (1 << 20):9.1f}M {r['time_us']:10.1f} {r['algbw_GBps']:11.1f} "
                  f"{r['busbw_GBps']:11.1f}")
        if a.json:
            with open(a.json, "w") as f:
                json.dump(rows, f, indent=1)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
