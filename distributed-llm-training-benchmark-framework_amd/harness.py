"""train_harness-compatible benchmark driver for MI355X.

Reference: ``benchmarking/train_harness.py`` (``main`` :465-504, ``train`` :278-458).  Same CLI
flags, same result record / file name / stdout markers, same per-strategy semantics by default,
re-implemented on dltb's fused HIP kernels and native parallelism engines:

    setup_distributed -> seed -> TinyGPT(tier) -> engine (ddp | fsdp | zero2 | zero3)
    -> synthetic data -> STEP LOOP (engine(batch) / engine.backward / engine.step)
    -> metrics (rank 0) -> result_{S}_ws{WS}_seq{T}_tier{X}.json + JSON markers

Differences that make the numbers honest (recorded in the extended sidecar):
* the timed region is bracketed by a barrier and a device synchronisation; mean step time is the
  synchronised wall time of the post-warmup steps divided by their count, max over ranks;
* per-step losses stay on the device and are read once at the end (the reference syncs every step).
Extra flags (all optional): --accum-semantics, --grad-reduce, --dtype, --device, --bucket-mb, --dropout, --seed,
--profile, --debug-collectives, --fail-at-step, --timeout-min, --data-loader, --model-tier.
"""
import argparse
import json
import math
import os
import sys
import time

import torch

from .data import SyntheticDataset, make_batcher
from .models import build_model, get_model_config
from .parallel.checkpoint import export_consolidated, load_checkpoint, save_checkpoint
from .parallel.graphs import GraphedStep, graphs_enabled
from .ops._ext import available as ext_available, so_path
from .ops.functional import torch_fallbacks
from .comm import describe as comm_describe
from .parallel import STRATEGIES, engine_config, make_engine
from .parallel.ds_config import ds_precision
from .parallel.strategy import default_config_path, load_deepspeed_config, load_fsdp_config
from .results import make_record, print_markers, print_result, write_result
from .utils.dist import all_reduce_max, barrier, cleanup_distributed, resolve_ranks, setup_distributed
from .utils.gemm_tuning import flush_tunableop, setup_tunableop
from .utils.platform import MI355X_DENSE_BF16_FLOPS, device_info
from .utils.timers import PhaseTimers

# bf16: the ZeRO configs' precision; fp16: the reference's DDP/FSDP autocast + GradScaler path
DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def build_parser():
    p = argparse.ArgumentParser(description="MI355X Distributed Training Benchmark (dltb)")
    # strategy / distributed (reference flags; rank/world default to the torchrun environment)
    p.add_argument("--strategy", type=str, required=True, choices=list(STRATEGIES))
    p.add_argument("--world-size", type=int, default=None, help="Total number of GPUs (default: $WORLD_SIZE or 1)")
    p.add_argument("--rank", type=int, default=None, help="Global rank (default: $RANK or 0)")
    p.add_argument("--local-rank", type=int, default=None, help="Local rank (default: $LOCAL_RANK or 0)")
    p.add_argument("--master-addr", type=str, default=None)
    p.add_argument("--master-port", type=int, default=None)
    # model & data
    p.add_argument("--tier", type=str, required=True, choices=["A", "B", "default", "M7B", "M7B_narrow", "tiny", "mtiny"])
    p.add_argument("--seq-len", type=int, required=True)
    p.add_argument("--synthetic", action="store_true", help="accepted for compatibility (data is always synthetic)")
    # training
    p.add_argument("--steps", type=int, required=True)
    p.add_argument("--warmup-steps", type=int, default=5)
    p.add_argument("--per-device-batch", type=int, required=True)
    p.add_argument("--grad-accum", type=int, required=True)
    # configs
    p.add_argument("--deepspeed-config", type=str, default=None, help="DeepSpeed JSON (read without DeepSpeed)")
    p.add_argument("--fsdp-config", type=str, default=None, help="FSDP YAML (honoured, unlike the reference)")
    # output
    p.add_argument("--results-dir", type=str, required=True)
    # MI355X extras
    p.add_argument("--accum-semantics", choices=["reference", "uniform"], default="reference")
    p.add_argument("--ddp-shard-optimizer", action="store_true",
                   help="ddp: shard the AdamW state over the ranks (torch DDP + ZeroRedundancyOptimizer): "
                        "reduce-scatter + all-gather instead of all-reduce, same update")
    p.add_argument("--grad-reduce", choices=["micro", "window"], default="micro",
                   help="ZeRO-2 gradient reduce-scatter every micro-step (DeepSpeed) or once per "
                        "accumulation window")
    p.add_argument("--grad-comm-dtype", choices=["auto", "bf16", "fp16", "fp32"], default="auto",
                   help="DDP gradient all-reduce dtype: the compute dtype or fp32; auto = fp32 when DDP "
                        "runs the reference's fp16 path (torch DDP reduces fp32 grads), else the compute dtype")
    p.add_argument("--dtype", choices=["auto"] + list(DTYPES), default="auto",
                   help="compute dtype; auto = the reference's precision per strategy: fp16 + dynamic loss "
                        "scaling for ddp / fsdp (autocast + GradScaler), bf16 for zero2 / zero3 (DS configs)")
    p.add_argument("--device", choices=["cuda", "cpu"], default="cuda" if torch.cuda.is_available() else "cpu")
    p.add_argument("--bucket-mb", type=float, default=None,
                   help="gradient bucket cap (MiB); default: comm.topology.recommend_bucket_mb(world), "
                        "from the measured xGMI sweep (profiles/xgmi_buckets.json) when present")
    p.add_argument("--strategy-label", type=str, default=None,
                   help="name of this run in the result record / file name / CSV (e.g. fsdp_root, "
                        "ddp_uniform); default: --strategy")
    p.add_argument("--dropout", type=float, default=None, help="override the model dropout (reference: 0.1)")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--data-loader", choices=["device", "host"], default="device")
    p.add_argument("--profile", type=str, default=None, help="write a torch.profiler chrome trace to this dir")
    p.add_argument("--profile-steps", type=int, default=3)
    p.add_argument("--phase-timers", action="store_true",
                   help="per-phase times (forward / backward / exposed comm wait / optimizer) from HIP events; "
                        "runs eagerly (a graph replay has no phase boundaries)")
    p.add_argument("--debug-collectives", action="store_true", help="TORCH_DISTRIBUTED_DEBUG=DETAIL")
    p.add_argument("--fail-at-step", type=int, default=None, help="inject a failure (tests the suite runner)")
    p.add_argument("--timeout-min", type=int, default=30, help="collective timeout")
    p.add_argument("--log-every", type=int, default=None,
                   help="log cadence in steps (default: the DeepSpeed config's steps_per_print, else 10)")
    p.add_argument("--no-extended", action="store_true", help="do not write the extended sidecar")
    p.add_argument("--resume", type=str, default=None, help="load a sharded checkpoint dir before training")
    p.add_argument("--save-dir", type=str, default=None, help="write a sharded checkpoint at the end (window boundary)")
    p.add_argument("--export-model", type=str, default=None, help="write the consolidated bf16 model (.safetensors)")
    p.add_argument("--graphs", default="auto", choices=["auto", "on", "off"],
                   help="replay micro-steps as captured HIP graphs (parallel/graphs.py; off with --profile)")
    p.add_argument("--tunableop", default="auto", choices=["auto", "use", "tune", "off"],
                   help="hipBLASLt GEMM solutions (TunableOp results shipped in configs/tunableop)")
    return p


def _engine_for(args, model, device):
    ds = fc = None
    if args.strategy in ("zero2", "zero3"):
        path = args.deepspeed_config or default_config_path(args.strategy)
        ds = load_deepspeed_config(path)
        # train_harness.py:251-262: batch keys are injected at runtime
        for k in ("train_batch_size", "train_micro_batch_size_per_gpu", "gradient_accumulation_steps"):
            ds.pop(k, None)
    if args.strategy == "fsdp":
        path = args.fsdp_config or default_config_path("fsdp")
        if path and os.path.exists(path):
            fc = load_fsdp_config(path)
        if getattr(args, "fsdp_wrap", None) == "root":      # the reference's single root FlatParameter
            fc = dict(fc or {}, auto_wrap_policy="size_based")
        if getattr(args, "fsdp_sharding", None):            # bench.py --fsdp-sharding (FSDP sharding_strategy)
            fc = dict(fc or {}, sharding_strategy=args.fsdp_sharding)
    cfg = engine_config(args.strategy, args.grad_accum, args.accum_semantics, ds, fc,
                        compute_dtype=DTYPES[args.dtype], bucket_mb=args.bucket_mb, seed=args.seed,
                        grad_reduce=getattr(args, "grad_reduce", "micro"))
    cfg.extra["grad_comm_dtype"] = "fp32" if getattr(args, "grad_comm_dtype", None) == "fp32" else "compute"
    if args.strategy == "ddp" and getattr(args, "ddp_shard_optimizer", False):
        cfg.extra["shard_optimizer"] = True       # DDP + ZeroRedundancyOptimizer (parallel/replicated.py)
    return make_engine(model, cfg, device), cfg


def train(args):
    world, rank, local_rank = resolve_ranks(args.world_size, args.rank, args.local_rank)
    args.world_size, args.rank, args.local_rank = world, rank, local_rank
    auto_bucket = args.bucket_mb is None
    label = args.strategy_label or args.strategy
    if not args.strategy_label and args.strategy == "ddp" and getattr(args, "ddp_shard_optimizer", False):
        label = "ddp_zero1"          # DDP + sharded optimizer state: its own row in metrics.csv
    ds_cfg = None
    if args.strategy in ("zero2", "zero3"):
        ds_cfg = load_deepspeed_config(args.deepspeed_config or default_config_path(args.strategy))
    if args.dtype == "auto":
        args.dtype = "fp16" if args.strategy in ("ddp", "fsdp") else ds_precision(ds_cfg)
    if args.log_every is None:               # DeepSpeed's steps_per_print (zero2/3.json: 10)
        args.log_every = int((ds_cfg or {}).get("steps_per_print", 10))
    if (ds_cfg or {}).get("wall_clock_breakdown"):
        args.phase_timers = True             # DeepSpeed's wall-clock breakdown: per-phase HIP-event timers
    if args.grad_comm_dtype == "auto":
        args.grad_comm_dtype = "fp32" if (args.strategy == "ddp" and args.dtype == "fp16") else args.dtype
    if args.grad_comm_dtype not in ("fp32", args.dtype):
        raise ValueError(f"--grad-comm-dtype {args.grad_comm_dtype}: must be fp32 or the compute dtype {args.dtype}")
    device = setup_distributed(world, rank, local_rank, args.master_addr, args.master_port, args.device,
                               args.timeout_min, args.debug_collectives)
    is_main = rank == 0
    fabric = None
    if auto_bucket:
        from .comm.topology import calibrate_fabric, measured_params, recommend_bucket_mb
        if (world > 1 and measured_params(world)[2] == "default"
                and (device.type != "cuda" or os.environ.get("DLTB_COMM", "rccl") != "host")):
            # this job's own collective alpha-beta before the engine plans its buckets (bench.py does the same)
            fabric = calibrate_fabric(device, sizes_mb=(4, 16, 64) if device.type == "cuda" else (0.25, 1.0))
        args.bucket_mb = recommend_bucket_mb(world)
    try:
        if device.type == "cuda" and not ext_available():
            raise RuntimeError("dltb._C is not built: run `python csrc/build.py` (the GPU path has no fallback)")
        gemm_mode = setup_tunableop(args.tunableop if (args.tunableop != "tune" or is_main) else "use") \
            if device.type == "cuda" else "off"
        torch.manual_seed(args.seed)        # identical init on every rank (the reference uses 42+rank + DDP broadcast)
        if is_main:
            print("\n" + "=" * 80)
            print(f"Benchmark Config: {args.strategy.upper()} | Tier {args.tier} | WS={world} | SeqLen={args.seq_len}")
            print("=" * 80 + "\n", flush=True)
        mcfg = get_model_config(args.tier, args.seq_len)
        if args.dropout is not None:
            mcfg.dropout = args.dropout
        with torch.device(device):      # init directly on the GPU (no fp32 host copy of a 7B model)
            model = build_model(mcfg)
        n_params = model.num_params()
        if is_main:
            print(f"Model initialized: {n_params / 1e6:.2f}M parameters", flush=True)
        engine, ecfg = _engine_for(args, model, device)
        if is_main:
            print(f"[Rank {rank}] engine={type(engine).__name__} accum={engine.accum} clip={ecfg.grad_clip} "
                  f"sched={'WarmupLR' if ecfg.scheduler else 'constant'} dtype={engine.compute_dtype}", flush=True)
        ds = SyntheticDataset(mcfg.vocab_size, args.seq_len, size=1000, seed=42)
        if is_main:
            print(f"SyntheticDataset: {len(ds)} samples, seq_len={args.seq_len}", flush=True)
        batches = make_batcher(args.data_loader, ds, args.per_device_batch, world, rank, args.strategy, device)
        if device.type == "cuda":
            torch.cuda.reset_peak_memory_stats(device)
        if is_main:
            print(f"Starting training: {args.steps} steps, warmup={args.warmup_steps}")
            print(f"Per-device batch: {args.per_device_batch}, Grad accum: {args.grad_accum}\n", flush=True)
        if args.resume:
            meta = load_checkpoint(engine, args.resume)
            if is_main:
                print(f"Resumed from {args.resume}: optimizer step {meta['opt_steps']}", flush=True)
        engine.train()
        # (auto: a warm-up no longer than one accumulation window would put the graph capture, at the
        # first window start after an eager window, inside the timed steps -> eager; as fast)
        short_warmup = (args.graphs == "auto" and args.warmup_steps <= engine.accum
                        and os.environ.get("DLTB_GRAPHS") is None)
        runner = GraphedStep(engine) if (graphs_enabled(args.graphs, device, world) and not args.profile
                                         and not args.phase_timers and not short_warmup) else None
        timers = PhaseTimers(device) if args.phase_timers else None
        timed_n = max(0, args.steps - args.warmup_steps)
        # per-step losses are COPIED into a device buffer: a graph replay returns the same static
        # loss tensor for every replay of a window position, so keeping the tensors would alias
        loss_hist = torch.zeros(max(1, timed_n), dtype=torch.float32, device=device)
        n_loss = 0
        step_events = []
        host_times = []
        prof = None
        t_start = None
        t_log = [time.perf_counter(), 0]
        sync = (lambda: torch.cuda.synchronize(device)) if device.type == "cuda" else (lambda: None)
        for step in range(args.steps):
            if step == args.warmup_steps:
                barrier()
                sync()
                engine.comm.reset_stats()     # wire accounting over the timed steps only
                t_start = time.perf_counter()
                if args.profile and is_main:
                    from torch.profiler import ProfilerActivity, profile
                    prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=False)
                    prof.__enter__()
            if args.fail_at_step is not None and step == args.fail_at_step:
                raise RuntimeError(f"injected failure at step {step} (--fail-at-step)")
            batch = next(batches)
            targets = batch          # unshifted targets = inputs (train_harness.py:359)
            ev0 = ev1 = None
            if device.type == "cuda" and step >= args.warmup_steps:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev0.record()
            h0 = time.perf_counter()
            timed_phase = timers is not None and step >= args.warmup_steps
            if timed_phase:
                engine.timers = timers
                timers.begin_step()
            if runner is not None:
                loss = runner(batch, targets)
            else:
                loss = engine(batch, targets)[1]
                if timed_phase:
                    timers.mark("fwd_end")
                engine.backward(loss)
                if timed_phase:
                    timers.mark("bwd_end")
                engine.step()
            if timed_phase:
                timers.end_step()
                engine.timers = None
            h1 = time.perf_counter()
            if ev1 is not None:
                ev1.record()
                step_events.append((ev0, ev1))
            if step >= args.warmup_steps:
                loss_hist[n_loss].copy_(loss.detach().reshape(()))
                n_loss += 1
                host_times.append(h1 - h0)
            if prof is not None and step >= args.warmup_steps + args.profile_steps - 1:
                sync()
                prof.__exit__(None, None, None)
                os.makedirs(args.profile, exist_ok=True)
                prof.export_chrome_trace(os.path.join(args.profile, f"trace_{label}_ws{world}_rank{rank}.json"))
                prof = None
            if is_main and args.log_every and step % args.log_every == 0:
                lv = loss.item()             # synchronises: Time is the mean device-synchronised
                now = time.perf_counter()    # step time since the previous log line
                dt = (now - t_log[0]) / max(1, step - t_log[1]) if step > 0 else h1 - h0
                t_log[:] = [now, step]
                print(f"[Step {step:04d}] Loss: {lv:.4f}, Time: {dt:.4f}s", flush=True)
        barrier()
        sync()
        timed = args.steps - args.warmup_steps
        # the timed region ends here: finalize / checkpoint / export below are not step time
        wall = (time.perf_counter() - t_start) if (t_start is not None and timed > 0) else 0.0
        wall = all_reduce_max(wall, device)
        engine.finalize()            # a deferred optimizer step of the last window (outside the timed region)
        if args.save_dir:
            if engine.micro % engine.accum == 0:
                save_checkpoint(engine, args.save_dir, {"tier": args.tier, "seq_len": args.seq_len})
                if is_main:
                    print(f"Checkpoint written to {args.save_dir}", flush=True)
            elif is_main:
                print("WARNING: --save-dir skipped: the run did not end on an accumulation boundary", flush=True)
        if args.export_model:
            export_consolidated(engine, args.export_model)
        mean_step = wall / timed if timed > 0 else 0.0
        mean_loss = float(loss_hist[:n_loss].mean().item()) if n_loss else 0.0
        peak = torch.cuda.max_memory_allocated(device) if device.type == "cuda" else 0
        record = make_record(label, world, rank, args.seq_len, args.tier, args.steps,
                             args.per_device_batch, args.grad_accum, mean_step, mean_loss, peak)
        ev_times = [a.elapsed_time(b) / 1e3 for a, b in step_events] if step_events else []
        tokens_step = args.per_device_batch * args.seq_len * world
        flops_tok = mcfg.train_flops_per_token(args.seq_len)
        tflops_gpu = (tokens_step / world) * flops_tok / mean_step / 1e12 if mean_step > 0 else 0.0
        extended = {
            "record_file_semantics": "tokens_per_sec = per_device_batch*seq_len*world_size / mean_step_time_sec "
                                     "(reference formula; one micro-batch per step)",
            "timing": "barrier + device sync around the timed region; max over ranks (reference: rank-0 host "
                      "perf_counter without sync)",
            "wall_time_timed_sec": wall, "timed_steps": timed,
            "host_step_time_mean_sec": (sum(host_times) / len(host_times)) if host_times else 0.0,
            "device_step_time_p50_sec": sorted(ev_times)[len(ev_times) // 2] if ev_times else None,
            "device_step_time_max_sec": max(ev_times) if ev_times else None,
            "tflops_per_gpu": tflops_gpu, "mfu_vs_2.5PF_dense_bf16": tflops_gpu * 1e12 / MI355X_DENSE_BF16_FLOPS,
            "train_flops_per_token": flops_tok, "params": n_params, "trainable_params": n_params,
            "model": mcfg.to_dict(), "engine": type(engine).__name__,
            "hip_graphs": bool(runner is not None and runner.graphs and not runner.disabled),
            "engine_config": {k: (str(v) if isinstance(v, torch.dtype) else v) for k, v in vars(ecfg).items()},
            "optimizer_steps": engine.opt_steps, "last_lr": engine.last_lr,
            "grad_norm": float(engine.grad_norm.item()) if engine.grad_norm is not None else None,
            "comm_bytes_per_step_per_gpu": engine.comm_bytes_per_step,
            # measured by the comm layer (host-issued calls; graph replays issue none from Python)
            "comm_wire_bytes_per_step_measured": (engine.comm.wire_bytes() / timed
                                                  if timed > 0 and not (runner is not None and runner.graphs
                                                                        and not runner.disabled) else None),
            "comm_ops_timed": {k: dict(v) for k, v in engine.comm.stats.items()},
            "comm_topology": comm_describe(world) if (is_main and device.type == "cuda") else None,
            "fabric_calibration": fabric,
            "memory": engine.memory_report(),
            "peak_vram_reserved_gb": (torch.cuda.max_memory_reserved(device) / 1e9) if device.type == "cuda" else 0.0,
            "accum_semantics": args.accum_semantics, "grad_reduce": args.grad_reduce, "dtype": args.dtype,
            "grad_comm_dtype": getattr(engine, "grad_comm_dtype", args.grad_comm_dtype), "strategy_engine": args.strategy, "bucket_mb": args.bucket_mb, "data_loader": args.data_loader,
            "kernels": so_path(), "platform": device_info(device), "gemm_tuning": gemm_mode,
            "torch_gemm_fallbacks": dict(torch_fallbacks) or None,
            "phase_times_ms": timers.summary() if timers is not None else None,
            "loss_scaler": engine.scaler.stats() if engine.scaler is not None else None,
            "deepspeed_config_keys": ecfg.extra.get("ds_keys") or None,
            "config_keys_ignored": sorted((ecfg.extra.get("ds_keys") or {}).get("ignored", {})),
        }
        if is_main:
            print_result(record)
            path = write_result(record, args.results_dir, None if args.no_extended else extended)
            print(f"Results saved to: {path}")
            print_markers(record)
        flush_tunableop()
        return record, extended
    finally:
        cleanup_distributed()


def main(argv=None):
    args = build_parser().parse_args(argv)
    if args.strategy in ("zero2", "zero3") and not args.deepspeed_config:
        args.deepspeed_config = default_config_path(args.strategy)
        print(f"[dltb] --deepspeed-config not given; using {args.deepspeed_config}", flush=True)
    train(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
