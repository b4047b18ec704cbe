#!/usr/bin/env python3
"""Flagship benchmark: TinyGPT Tier A training throughput on N MI355X GPUs (one process per GPU).

Metric and config are the ones BASELINE.json names: tokens/sec (+ step time + peak HBM) of TinyGPT
Tier A (236.4M params, d1024 / 16 heads / 16 layers, vocab 32000), seq 2048, per-device batch 1,
grad-accum 4, default strategy ZeRO-2 (the reference's headline: 18,147 tok/s on 4x A10), bf16,
synthetic tokens, random init.  A "step" is one micro-batch, as in the reference
(train_harness.py:351-393).  ZeRO-2 is DeepSpeed stage 2 at every world size: the gradients are
reduce-scattered after EVERY micro-step (configs/deepspeed/zero2.json, ``reduce_scatter: true``)
and the optimizer step (fused AdamW + clip + WarmupLR + bf16 all-gather) runs at every 4th
micro-step; ``--grad-reduce window`` (one reduce-scatter per accumulation window) is ZeRO-1
communication and is labelled ``zero1-dpN``.  Any K consecutive micro-steps contain K/4 optimizer
steps, so the timed region needs no alignment: exactly W warm-up steps run, then exactly K are
timed.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--strategy zero2|ddp|fsdp|zero3]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Launch modes (reference: scripts/launch_multi.sh:38-82 starts one pod per rank; here one process
per GPU on one node):
* ``WORLD_SIZE`` set (torchrun / the driver): this process is one rank.
* ``WORLD_SIZE`` unset and ``--gpus N > 1``: this process is only a launcher.  It never touches the
  GPU; it starts ``torch.distributed.run`` with N ranks as a CHILD process (no exec), streams its
  output (rank 0 prints the JSON line) and exits with the child's status, which is non-zero if any
  rank failed.
* ``--device cpu`` runs the same code on gloo / CPU (tests).  ``DLTB_COMM=host`` on a GPU makes
  every rank use gloo with host-staged buffers, so N ranks can share one GPU (tests of the
  multi-rank code paths on a one-GPU box; not a performance mode).

K steps are timed between a barrier + torch.cuda.synchronize() on both sides; the time is the MAX over
ranks; rank 0 prints one JSON line.  ``value`` is the whole-job tokens/s over all N GPUs.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

# multi-process GPU work on this platform needs dmabuf IPC (RCCL's peer buffers): set before any ROCm
# runtime loads in this rank, whether the ranks came from launch() below or from an outside torchrun
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TPS = 18147.0   # best published (ZeRO-2 @ 4x A10), README.md:207,221
BASELINES = {"ddp": {2: 8369.4557, 4: 12220.3415}, "fsdp": {2: 6771.0, 4: 9424.0},
             "zero2": {2: 10999.0, 4: 18147.0}, "zero3": {2: 10560.0, 4: 15977.0}}


def build_parser():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1, help="number of ranks (one per GPU)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--strategy", default="zero2", choices=["ddp", "fsdp", "zero2", "zero3"])
    ap.add_argument("--tier", default="A")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--per-device-batch", type=int, default=1)
    ap.add_argument("--grad-accum", type=int, default=4)
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="gradient bucket cap in MiB (default: comm.topology's measured/modelled choice)")
    ap.add_argument("--accum-semantics", default="reference", choices=["reference", "uniform"])
    ap.add_argument("--grad-reduce", default="micro", choices=["micro", "window"],
                    help="ZeRO-2 gradient reduce-scatter every micro-step (DeepSpeed stage 2, default) or "
                         "once per accumulation window (ZeRO-1 communication, reported as zero1-dpN)")
    ap.add_argument("--dtype", default="auto", choices=["auto", "bf16", "fp16"],
                    help="compute dtype; auto = the reference's precision per strategy (as the harness): bf16 "
                         "for ZeRO-2/3 (zero2.json), fp16 + dynamic loss scaling for DDP/FSDP (autocast)")
    ap.add_argument("--grad-comm-dtype", default="auto", choices=["auto", "compute", "fp32"],
                    help="DDP gradient all-reduce dtype; auto = fp32 for fp16 DDP (the reference's torch DDP "
                         "reduces fp32 grads), else the compute dtype")
    ap.add_argument("--deepspeed-config", default=None,
                    help="DeepSpeed JSON for zero2/zero3 (default configs/deepspeed/<strategy>.json)")
    ap.add_argument("--fsdp-wrap", default="block", choices=["block", "root"],
                    help="FSDP unit layout: per transformer block, or the reference's single root FlatParameter")
    ap.add_argument("--ddp-shard-optimizer", action="store_true",
                    help="ddp: shard the AdamW state over the ranks (torch DDP + ZeroRedundancyOptimizer; reported "
                         "as ddp_zero1): reduce-scatter + all-gather instead of all-reduce, same update")
    ap.add_argument("--fsdp-sharding", default=None, choices=["full_shard", "shard_grad_op"],
                    help="FSDP sharding_strategy (default: configs/fsdp/fsdp_config.yaml's full_shard); "
                         "shard_grad_op keeps the gathered parameters from forward to backward (no re-gather)")
    ap.add_argument("--graphs", default="auto", choices=["auto", "on", "off"],
                    help="replay each micro-step as a captured HIP graph (DLTB_GRAPHS overrides)")
    ap.add_argument("--tunableop", default="auto", choices=["auto", "use", "tune", "off"],
                    help="hipBLASLt GEMM solutions from configs/tunableop (auto = use if present)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = gloo / CPU reference ops (tests of the launcher and the engines)")
    ap.add_argument("--timeout-min", type=int, default=10, help="collective timeout")
    ap.add_argument("--fail-rank", type=int, default=None, help="(tests) this rank raises before timing")
    ap.add_argument("--emulate", type=int, default=0, metavar="N",
                    help="PREDICTION mode: one process on one GPU plays rank 0 of an N-rank job -- real N-rank "
                         "layouts, shards and buckets, every collective an alpha-beta-paced kernel on a "
                         "side stream (DLTB_COMM=emulate:N, comm/collectives.py); value = N x this rank's tok/s")
    ap.add_argument("--no-calibrate", action="store_true",
                    help="skip the in-job collective calibration at world > 1 (bucket size and comm model then "
                         "come from profiles/xgmi_buckets.json or the defaults)")
    ap.add_argument("--host-check", action="store_true",
                    help="after the timed steps: host enqueue time per step while the GPU is held busy "
                         "(is the eager step host-bound?)")
    return ap


def _model_name(tier, c):
    if c.arch == "mistral":
        return (f"Mistral-7B-shape ({c.num_params() / 1e9:.2f}B params, d{c.n_embd}/h{c.n_head}/kv{c.kv_heads}/"
                f"L{c.n_layer}, ffn {c.ffn_dim}, vocab {c.vocab_size})")
    return f"TinyGPT-{tier} ({c.num_params() / 1e6:.1f}M params, d{c.n_embd}/h{c.n_head}/L{c.n_layer}, vocab {c.vocab_size})"


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# shipped emulated-fabric predictions (scripts/emulated_scaling.py): a real N-GPU run reports the prediction
# for its own (strategy label, dtype, N) so the prediction error reads off one JSON line.  Tables are searched
# newest first: by round, then a round's "_final" table before its earlier ones, then the letter suffix.
def prediction_tables():
    import glob
    import re

    def key(path):
        m = re.match(r"emulated_scaling_r(\d+)([a-z]*)(_final)?", os.path.basename(path))
        return (int(m.group(1)), bool(m.group(3)), m.group(2)) if m else (-1, False, "")
    paths = glob.glob(os.path.join(ROOT, "profiles", "emulated_scaling_r*.jsonl"))
    return [os.path.relpath(p, ROOT) for p in sorted(paths, key=key, reverse=True)]


def predicted_row(parallelism: str, dtype: str, world: int, seq_len: int = None, model: str = None):
    """The shipped prediction for this configuration, or None: {ms_per_step, value, table, seq_len, model}.
    ``seq_len`` / ``model`` (the JSON line's config fields), when given, must match the predicted run too."""
    for rel in prediction_tables():
        path = os.path.join(ROOT, rel)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            for line in f:
                try:
                    d = json.loads(line)
                except ValueError:
                    continue
                c = d.get("config", {})
                if (d.get("prediction") and d.get("emulated_world") == world and d.get("dtype") == dtype
                        and c.get("parallelism") == parallelism
                        and (seq_len is None or c.get("seq_len") == seq_len)
                        and (model is None or c.get("model") == model)):
                    return {"ms_per_step": d.get("ms_per_step"), "value": d.get("value"), "table": rel,
                            "seq_len": c.get("seq_len"), "model": c.get("model")}
    return None


def comm_environment():
    """The RCCL build and the communication knobs in effect in this rank (for a real N > 1 run)."""
    import torch
    ver = None
    try:
        v = torch.cuda.nccl.version()
        ver = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 - gloo / CPU runs have no RCCL
        pass
    knobs = {k: v for k, v in sorted(os.environ.items())
             if k.startswith(("NCCL_", "RCCL_", "HSA_", "TORCH_NCCL_", "HIP_", "GPU_MAX_HW_QUEUES"))}
    return {"rccl_version": ver, "hip_version": getattr(torch.version, "hip", None), "knobs": knobs}


def launch(args, argv) -> int:
    """Launcher mode: N ranks under torch.distributed.run as a child process.  Nothing here
    initialises the GPU (no torch import at all), so the parent never holds a device context."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "--max-restarts=0",
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    env["PYTHONUNBUFFERED"] = "1"
    proc = subprocess.run(cmd, env=env, cwd=ROOT)
    return proc.returncode


def resolve_precision(args):
    """--dtype / --grad-comm-dtype auto -> the reference's precision per strategy (harness.py)."""
    if args.dtype == "auto":
        args.dtype = "fp16" if args.strategy in ("ddp", "fsdp") else "bf16"
        if args.strategy in ("zero2", "zero3"):   # the DeepSpeed config's precision (the default one as the harness)
            from dltb.parallel.ds_config import ds_precision
            from dltb.parallel.strategy import default_config_path, load_deepspeed_config
            args.dtype = ds_precision(load_deepspeed_config(args.deepspeed_config or default_config_path(args.strategy)))
    if args.grad_comm_dtype == "auto":
        args.grad_comm_dtype = "fp32" if (args.strategy == "ddp" and args.dtype == "fp16") else "compute"
    return args


def run_rank(args) -> int:
    import torch
    import dltb  # noqa: F401
    from dltb.data import SyntheticDataset, make_batcher
    from dltb.harness import _engine_for
    from dltb.models import build_model, get_model_config
    from dltb.parallel import GraphedStep, graphs_enabled
    from dltb.comm.topology import recommend_bucket_mb
    from dltb.utils.dist import all_reduce_max, barrier, cleanup_distributed, setup_distributed
    from dltb.utils.timers import PhaseTimers
    from dltb.ops import functional as F_

    resolve_precision(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.emulate:
        if world != 1:
            raise SystemExit("--emulate runs in ONE process (it plays rank 0 of the N-rank job)")
        os.environ["DLTB_COMM"] = f"emulate:{args.emulate}"
    device = setup_distributed(world, rank, local, device_type=args.device, timeout_min=args.timeout_min)
    cuda = device.type == "cuda"
    try:
        tmode = "off"
        if cuda:
            from dltb.ops._ext import ext
            from dltb.utils.gemm_tuning import setup_tunableop
            ext()   # fail loudly if the HIP extension is missing
            tmode = setup_tunableop(args.tunableop if (args.tunableop != "tune" or rank == 0) else "use")
        torch.manual_seed(42)
        mcfg = get_model_config(args.tier, args.seq_len)
        with torch.device(device):          # random init straight into HBM
            model = build_model(mcfg)
        eworld = args.emulate or world     # the job's rank count (emulated or real)
        fabric = None
        from dltb.comm.topology import calibrate_fabric, measured_params
        if (world > 1 and not args.no_calibrate and measured_params(world)[2] == "default"
                and (not cuda or os.environ.get("DLTB_COMM", "rccl") != "host")):
            # no measured sweep for this world size (profiles/xgmi_buckets.json): the alpha-beta of
            # THIS job's fabric (RCCL over xGMI on the GPU node) before the buckets are planned;
            # outside the timed region
            fabric = calibrate_fabric(device, sizes_mb=(4, 16, 64) if cuda else (0.25, 1.0))
        bucket_mb = args.bucket_mb if args.bucket_mb is not None else recommend_bucket_mb(eworld)
        h = argparse.Namespace(strategy=args.strategy, deepspeed_config=args.deepspeed_config, fsdp_config=None,
                               grad_accum=args.grad_accum, accum_semantics=args.accum_semantics, dtype=args.dtype,
                               bucket_mb=bucket_mb, seed=42, grad_reduce=args.grad_reduce,
                               grad_comm_dtype=args.grad_comm_dtype,
                               fsdp_wrap=args.fsdp_wrap, fsdp_sharding=args.fsdp_sharding,
                               ddp_shard_optimizer=args.ddp_shard_optimizer)
        engine, ecfg = _engine_for(h, model, device)
        ds = SyntheticDataset(mcfg.vocab_size, args.seq_len, 1000, 42)
        batches = make_batcher("device", ds, args.per_device_batch, eworld, engine.comm.rank, args.strategy, device)
        engine.train()
        accum = engine.accum
        use_graphs = graphs_enabled(args.graphs, device, eworld)
        if use_graphs and args.graphs == "auto" and args.warmup <= accum and os.environ.get("DLTB_GRAPHS") is None:
            # the graphs are captured at the first window start after one eager window (micro-step
            # accum + 1); with a shorter warm-up that capture would land inside the timed steps, so
            # run eagerly instead (measured as fast: 7.34 vs 7.36 ms TinyGPT-A, 32.9 vs 32.7 ms Tier B)
            use_graphs = False
        runner = GraphedStep(engine) if use_graphs else None
        timers = PhaseTimers(device) if runner is None else None   # eager: exposed-comm time from HIP events

        def one_step(timed):
            b = next(batches)
            if runner is not None:
                return runner(b, b)
            if timed and timers is not None:
                engine.timers = timers
                timers.begin_step()
            loss = engine(b, b)[1]
            engine._phase("fwd_end")
            engine.backward(loss)
            engine._phase("bwd_end")
            engine.step()
            if timed and timers is not None:
                timers.end_step()
                engine.timers = None
            return loss

        sync = (lambda: torch.cuda.synchronize(device)) if cuda else (lambda: None)
        if cuda:
            torch.cuda.reset_peak_memory_stats(device)
        for _ in range(args.warmup):
            loss = one_step(False)
        if args.fail_rank is not None and rank == args.fail_rank:
            raise RuntimeError(f"injected failure on rank {rank} (--fail-rank)")
        opt0 = engine.opt_steps
        loss_hist = torch.zeros(max(1, args.steps), dtype=torch.float32, device=device)
        barrier()
        sync()
        engine.comm.reset_stats()
        t0 = time.perf_counter()
        for i in range(args.steps):
            loss = one_step(True)
            loss_hist[i].copy_(loss.detach().reshape(()))   # a copy: graph replays reuse one loss tensor
        barrier()
        sync()
        elapsed = all_reduce_max(time.perf_counter() - t0, device)
        wire_timed = engine.comm.wire_bytes()      # the timed steps' collectives (before finalize)
        opt_steps = engine.opt_steps - opt0
        comm_model_ms = engine.comm.modelled_us() / 1e3 / max(1, args.steps) if args.emulate else None
        host_ms = host_note = None
        if args.host_check and cuda:
            # fewer held steps when the enqueue outruns the hold: a deep model's launches can fill the
            # runtime's launch queue before 6 steps are enqueued (the host then blocks on the queue)
            for k in sorted({min(args.steps, 6), 2, 1}, reverse=True):
                host_ms, host_note = host_enqueue_ms(one_step, k, device,
                                                     step_ms=elapsed / max(1, args.steps) * 1e3)
                if "INVALID" not in host_note:
                    break
        engine.finalize()                    # a deferred update of the last window: outside the timed region
        mean_loss = float(loss_hist[:args.steps].mean().item()) if args.steps else 0.0
        final_loss = float(loss.item())
        peak_gb = torch.cuda.max_memory_allocated(device) / 1e9 if cuda else 0.0
        peak_gb = all_reduce_max(peak_gb, device)
        phases = timers.summary() if timers is not None else None
        comm_wait = all_reduce_max(phases["comm_wait"], device) if phases else 0.0
        graphed = bool(runner is not None and runner.graphs and not runner.disabled)
        wire = wire_timed / args.steps if (args.steps and not graphed) else None
        ms = elapsed / max(1, args.steps) * 1e3
        tokens = args.per_device_batch * args.seq_len * eworld * args.steps
        value = tokens / elapsed if elapsed > 0 else 0.0
        label = args.strategy
        if args.strategy == "zero2" and ecfg.zero_stage == 1:
            label = "zero1"                  # window-reduced: ZeRO-1 communication
        if args.strategy == "ddp" and ecfg.zero_stage == 1:
            label = "ddp_zero1"              # DDP + sharded optimizer state
        if args.strategy == "fsdp" and ecfg.wrap == "root":
            label = "fsdp_root"
        if args.strategy == "fsdp" and not ecfg.reshard_after_forward:
            label += "_sgo"                  # shard_grad_op: no re-gather in backward
        if rank == 0:
            world = eworld if args.emulate else world
            flops = mcfg.train_flops_per_token(args.seq_len)
            same = BASELINES.get(args.strategy) if label == args.strategy else None
            ref_dtype = "fp16" if args.strategy in ("ddp", "fsdp") else "bf16"
            out = {
                "metric": "tokens_per_sec",
                "value": value,
                "unit": "tokens/s",
                "n_gpus": world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": ms,
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": value / BASELINE_TPS if (args.tier == "A" and args.seq_len == 2048) else None,
                "dtype": args.dtype if cuda else "fp32",
                "data": "synthetic tokens (fixed random table, seed 42), random-init weights",
                "config": {"model": _model_name(args.tier, mcfg),
                           "global_batch": args.per_device_batch * accum * world,
                           "micro_batch_per_gpu": args.per_device_batch,
                           "grad_accum": accum,
                           "grad_accum_cli": args.grad_accum,
                           "seq_len": args.seq_len,
                           "parallelism": f"{label}-dp{world}",
                           "grad_reduce": ecfg.extra.get("grad_reduce"),
                           "grad_comm_dtype": getattr(engine, "grad_comm_dtype", args.grad_comm_dtype)
                           if args.strategy == "ddp" else None,
                           "bucket_mb": bucket_mb},
                "strategy": args.strategy,
                "world_size_seen": engine.comm.world,
                "backend": engine.comm.backend,
                "warmup_requested": args.warmup,
                "warmup_used": args.warmup,
                "optimizer_steps_timed": opt_steps,
                "mean_loss": mean_loss,
                "final_loss": final_loss,
                "peak_hbm_gb": peak_gb,
                "trainable_params": mcfg.num_params(),   # every parameter trains (config count: sharded engines free storage)
                "comm_wait_ms": comm_wait if phases else None,
                "phase_ms": phases,
                "wire_bytes_per_step": wire,
                "wire_bytes_per_step_model": engine.comm_bytes_per_step,
                "tflops_per_gpu": value / world * flops / 1e12,
                "mfu_dense_bf16": value / world * flops / 2.5e15,
                "baseline_note": "vs_baseline = value / 18147 tok/s (reference best: ZeRO-2 on 4x A10, BASELINE.md); "
                                 "vs_baseline_per_gpu = (value / n_gpus) / (18147 / 4), the per-GPU ratio",
                "vs_baseline_per_gpu": (value / world) / (BASELINE_TPS / 4) if (args.tier == "A" and args.seq_len == 2048) else None,
                "same_strategy_published": same,
                "same_strategy_precision_matches": (args.dtype == ref_dtype) if same else None,
                "loss_scaler": engine.scaler.stats() if engine.scaler is not None else None,
                "gemm_tuning": tmode,
                "torch_gemm_fallbacks": dict(F_.torch_fallbacks) or None,
                "hip_graphs": graphed,
                "ds_config_keys_ignored": sorted((ecfg.extra.get("ds_keys") or {}).get("ignored", {})),
                "fabric_calibration": ({"fits": fabric["fits"], "rows": fabric["rows"],
                                        "bucket_mb_from": "calibrated" if args.bucket_mb is None else "flag"}
                                       if fabric else None),
            }
            if world > 1 and not args.emulate:
                # a real multi-rank run explains itself: RCCL build and knobs, the in-job fabric fit
                # (fabric_calibration), the measured phase split (phase_ms, eager ranks) and the
                # shipped prediction for exactly this configuration
                pred = predicted_row(f"{label}-dp{world}", out["dtype"], world, out["config"]["seq_len"],
                                     out["config"]["model"])
                out["comm_env"] = comm_environment()
                out["predicted"] = pred
                out["prediction_error"] = ((ms - pred["ms_per_step"]) / pred["ms_per_step"]
                                           if pred and pred.get("ms_per_step") else None)
            if args.emulate:
                out.update({
                    "metric": "tokens_per_sec_predicted",
                    "n_gpus": 1, "emulated_world": eworld, "prediction": True,
                    "prediction_note": (f"ONE MI355X playing rank {engine.comm.rank} of a {eworld}-rank job: real "
                                        f"{eworld}-rank layouts / shards / buckets, collectives replaced by alpha-beta "
                                        "paced kernels on a high-priority side stream (DLTB_COMM=emulate:N); "
                                        "value = N x this rank's tokens/s; NOT a measurement of N GPUs"),
                    "comm_model": {op: {"alpha_us": a, "bus_GBps": b, "source": src}
                                   for op, (a, b, src) in engine.comm.emu_params.items()
                                   if op in ("all_reduce", "reduce_scatter", "all_gather")},
                    "emu_channels": engine.comm.emu_channels,
                    "emu_hbm_passes": engine.comm.emu_pass_of,
                    "emu_host_us_per_call": engine.comm.emu_host_us,
                    # what of the model is measured and what is assumed (no N-GPU RCCL run backs the latter)
                    "emu_assumptions": {
                        "hbm_passes": "ASSUMED: ring-algorithm estimate (reduce-scatter 3, all-gather 2, all-reduce 5 "
                                      "passes over the buffer), not measured on RCCL",
                        "channels": f"ASSUMED: {engine.comm.emu_channels}-workgroup stand-in for RCCL's CU footprint",
                        "host_us": "MEASURED: 1-rank RCCL communicator, async calls with the GPU held busy "
                                   "(profiles/pg_host_cost.json); the sync scalar norm all-reduce has its own 9.7 us row"
                                   if engine.comm.emu_host_us else "none (no host-cost profile)",
                        "alpha_beta": {op: src for op, (a, b, src) in engine.comm.emu_params.items()
                                       if op in ("all_reduce", "reduce_scatter", "all_gather")},
                    },
                    "comm_model_ms_per_step": comm_model_ms,
                    "vs_baseline": None, "vs_baseline_per_gpu": None,
                    "predicted_ms_per_step": ms,
                    "peak_hbm_gb_per_rank": peak_gb,
                })
            if host_ms is not None:
                out["host_enqueue_ms_per_step"] = host_ms
                out["host_over_gpu"] = host_ms / ms if ms else None
                out["host_check_note"] = host_note
            print(json.dumps(out), flush=True)
        if cuda:
            from dltb.utils.gemm_tuning import flush_tunableop
            flush_tunableop()
        return 0
    finally:
        cleanup_distributed()


def host_enqueue_ms(one_step, k, device, step_ms=0.0):
    """Host time to enqueue ``k`` eager micro-steps while the GPU is held busy by one long wait
    kernel in front of them (so no launch waits for the GPU): the host cost per step.  The hold
    lasts at least 3 x the GPU time of the k steps, so the enqueue never outlasts it while the host
    is ahead.  Returns (ms per step, note): the note flags a run whose enqueue still reached the
    hold -- a host sync in the step, or the launch queue full (the runtime blocks the host once its
    hardware queues hold that many packets) -- in which case the ratio is a lower bound of nothing
    and must not be read as host cost."""
    import torch
    from dltb.ops._ext import ext
    hold_us = max(3e5 + 5e4 * k, 3.0 * k * step_ms * 1e3)
    for _ in range(2):      # the first pass grows the allocator's cache: blocks still recorded on a
        torch.cuda.synchronize(device)     # collective stream cannot be reused while the GPU is held
        ext().comm_emu(None, 1, None, None, 1.0, 1, 0, hold_us, 0.0, 1, 0)   # one paced wave: GPU busy
        t0 = time.perf_counter()
        for _ in range(k):
            one_step(False)
        t1 = time.perf_counter()
        torch.cuda.synchronize(device)
    ms = (t1 - t0) / k * 1e3
    note = f"hold {hold_us / 1e3:.0f} ms for {k} steps"
    if ms * k * 1e3 > 0.9 * hold_us:
        note += "; INVALID: the enqueue reached the hold (host sync or launch queue full)"
        print(f"[host-check] enqueue took {ms * k:.1f} ms of a {hold_us / 1e3:.0f} ms hold: a step waits for "
              "the GPU (host sync or full launch queue)", flush=True)
    return ms, note


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = build_parser().parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch(args, argv)
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
