#!/usr/bin/env python3
"""Flagship benchmark: TinyGPT Tier A training throughput on N MI355X GPUs (one process per GPU).

Metric and config are the ones BASELINE.json names: tokens/sec (+ step time + peak HBM) of TinyGPT
Tier A (236.4M params, d1024 / 16 heads / 16 layers, vocab 32000), seq 2048, per-device batch 1,
grad-accum 4, default strategy ZeRO-2 (the reference's headline: 18,147 tok/s on 4x A10), bf16,
synthetic tokens, random init.  A "step" is one micro-batch, as in the reference
(train_harness.py:351-393); ZeRO-2 runs its optimizer step (fused AdamW + clip + WarmupLR + bf16
all-gather) at every 4th micro-step, and the timed region is aligned to whole accumulation windows
so it contains exactly steps/4 optimizer steps.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strategy zero2|ddp|fsdp|zero3]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

K steps are timed between a barrier + torch.cuda.synchronize() on both sides; the time is the MAX over
ranks; rank 0 prints one JSON line.  ``value`` is the whole-job tokens/s over all N GPUs.
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE_TPS = 18147.0   # best published (ZeRO-2 @ 4x A10), README.md:207,221
BASELINES = {"ddp": {2: 8369.4557, 4: 12220.3415}, "fsdp": {2: 6771.0, 4: 9424.0},
             "zero2": {2: 10999.0, 4: 18147.0}, "zero3": {2: 10560.0, 4: 15977.0}}


def _model_name(tier, c):
    if c.arch == "mistral":
        return (f"Mistral-7B-shape ({c.num_params() / 1e9:.2f}B params, d{c.n_embd}/h{c.n_head}/kv{c.kv_heads}/"
                f"L{c.n_layer}, ffn {c.ffn_dim}, vocab {c.vocab_size})")
    return f"TinyGPT-{tier} ({c.num_params() / 1e6:.1f}M params, d{c.n_embd}/h{c.n_head}/L{c.n_layer}, vocab {c.vocab_size})"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--strategy", default="zero2", choices=["ddp", "fsdp", "zero2", "zero3"])
    ap.add_argument("--tier", default="A")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--per-device-batch", type=int, default=1)
    ap.add_argument("--grad-accum", type=int, default=4)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--accum-semantics", default="reference", choices=["reference", "uniform"])
    ap.add_argument("--grad-reduce", default="auto", choices=["auto", "micro", "window"],
                    help="ZeRO-2 gradient reduce-scatter: every micro-step (DeepSpeed) or once per "
                         "accumulation window; auto = window on N > 1 (xGMI is point-to-point: 1/4 "
                         "of the traffic), no collective at all on N = 1")
    ap.add_argument("--no-align", action="store_true", help="do not align warmup to accumulation windows")
    ap.add_argument("--graphs", default="auto", choices=["auto", "on", "off"],
                    help="replay each micro-step as a captured HIP graph (DLTB_GRAPHS overrides)")
    ap.add_argument("--tunableop", default="auto", choices=["auto", "use", "tune", "off"],
                    help="hipBLASLt GEMM solutions from configs/tunableop (auto = use if present)")
    args = ap.parse_args()

    import dltb
    from dltb.data import SyntheticDataset, make_batcher
    from dltb.harness import _engine_for
    from dltb.models import build_model, get_model_config
    from dltb.ops._ext import ext
    from dltb.parallel import GraphedStep, graphs_enabled
    from dltb.utils.dist import all_reduce_max, barrier, cleanup_distributed, setup_distributed
    from dltb.utils.gemm_tuning import flush_tunableop, setup_tunableop

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    device = setup_distributed(world, rank, local, device_type="cuda")
    ext()   # fail loudly if the HIP extension is missing
    tmode = setup_tunableop(args.tunableop if (args.tunableop != "tune" or rank == 0) else "use")
    torch.manual_seed(42)
    mcfg = get_model_config(args.tier, args.seq_len)
    with torch.device(device):          # random init straight into HBM (7B-class models never touch host RAM)
        model = build_model(mcfg)
    grad_reduce = args.grad_reduce
    if grad_reduce == "auto":
        grad_reduce = "window" if (world > 1 and args.strategy == "zero2") else "micro"
    h = argparse.Namespace(strategy=args.strategy, deepspeed_config=None, fsdp_config=None,
                           grad_accum=args.grad_accum, accum_semantics=args.accum_semantics, dtype="bf16",
                           bucket_mb=args.bucket_mb, seed=42, grad_reduce=grad_reduce)
    engine, ecfg = _engine_for(h, model, device)
    ds = SyntheticDataset(mcfg.vocab_size, args.seq_len, 1000, 42)
    batches = make_batcher("device", ds, args.per_device_batch, world, rank, args.strategy, device)
    engine.train()
    accum = engine.accum
    warm = args.warmup
    if not args.no_align and accum > 1:
        warm = int(math.ceil(warm / accum) * accum)      # timed region starts at a window boundary

    use_graphs = graphs_enabled(args.graphs, device, world)
    runner = GraphedStep(engine) if use_graphs else None

    def one_step():
        b = next(batches)
        if runner is not None:
            return runner(b, b)
        loss = engine(b, b)[1]
        engine.backward(loss)
        engine.step()
        return loss

    torch.cuda.reset_peak_memory_stats(device)
    for _ in range(warm):
        loss = one_step()
    opt0 = engine.opt_steps
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = one_step()
    barrier()
    torch.cuda.synchronize(device)
    elapsed = all_reduce_max(time.perf_counter() - t0, device)
    opt_steps = engine.opt_steps - opt0
    final_loss = float(loss.item())
    peak_gb = torch.cuda.max_memory_allocated(device) / 1e9
    peak_gb = all_reduce_max(peak_gb, device)
    ms = elapsed / args.steps * 1e3
    tokens = args.per_device_batch * args.seq_len * world * args.steps
    value = tokens / elapsed
    if rank == 0:
        flops = mcfg.train_flops_per_token(args.seq_len)
        out = {
            "metric": "tokens_per_sec",
            "value": value,
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": warm,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": value / BASELINE_TPS if (args.tier == "A" and args.seq_len == 2048) else None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": _model_name(args.tier, mcfg),
                       "global_batch": args.per_device_batch * accum * world,
                       "micro_batch_per_gpu": args.per_device_batch,
                       "grad_accum": accum,
                       "seq_len": args.seq_len,
                       "parallelism": f"{args.strategy}-dp{world}",
                       "grad_reduce": grad_reduce if args.strategy == "zero2" else None},
            "strategy": args.strategy,
            "optimizer_steps_timed": opt_steps,
            "peak_hbm_gb": peak_gb,
            "tflops_per_gpu": value / world * flops / 1e12,
            "mfu_dense_bf16": value / world * flops / 2.5e15,
            "final_loss": final_loss,
            "baseline_note": "vs_baseline = value / 18147 tok/s (reference best: ZeRO-2 on 4x A10, BASELINE.md)",
            "same_strategy_published": BASELINES.get(args.strategy),
            "gemm_tuning": tmode,
            "hip_graphs": use_graphs,
        }
        print(json.dumps(out), flush=True)
    flush_tunableop()
    cleanup_distributed()


if __name__ == "__main__":
    main()
