"""Strategy dispatcher: the MI355X-native replacement of the reference's ``wrap_model``
(train_harness.py:207-275).

``--strategy ddp | fsdp | zero2 | zero3`` selects an engine; the DeepSpeed JSON
(``--deepspeed-config``) and FSDP YAML (``--fsdp-config``) are read by our own schema readers (no
DeepSpeed dependency; the reference never reads its FSDP YAML at all).

Step semantics (``--accum-semantics``):
  reference (default) — what the reference actually runs: DDP/FSDP step the optimizer every
      micro-batch (``--grad-accum`` ignored, no clipping, constant lr 1e-4, wd 0.01,
      train_harness.py:328-382); ZeRO-2/3 accumulate ``grad_accum`` micro-batches, clip the global
      grad norm to 1.0 and use WarmupLR (zero2.json).
  uniform — every strategy gets the ZeRO semantics (accumulation + clipping + schedule).
"""
import json
import os
from typing import Optional

import torch

from .ds_config import apply_deepspeed_config
from .engine import EngineConfig
from .replicated import DDPEngine, Zero2Engine
from .sharded import FSDPEngine, Zero3Engine

STRATEGIES = ("ddp", "fsdp", "zero2", "zero3")
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def default_config_path(strategy: str) -> Optional[str]:
    if strategy in ("zero2", "zero3"):
        return os.path.join(_ROOT, "configs", "deepspeed", f"{strategy}.json")
    if strategy == "fsdp":
        return os.path.join(_ROOT, "configs", "fsdp", "fsdp_config.yaml")
    return None


def load_deepspeed_config(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


def load_fsdp_config(path: str) -> dict:
    import yaml
    with open(path) as f:
        data = yaml.safe_load(f) or {}
    return data.get("fsdp_config", data)


def engine_config(strategy: str, grad_accum: int = 1, semantics: str = "reference",
                  ds_config: Optional[dict] = None, fsdp_config: Optional[dict] = None,
                  compute_dtype=torch.bfloat16, bucket_mb: float = 64.0, seed: int = 42,
                  overrides: Optional[dict] = None, grad_reduce: str = "micro") -> EngineConfig:
    """``grad_reduce`` (ZeRO-2 only): ``micro`` reduce-scatters the gradients after every micro-step
    (DeepSpeed stage 2, configs/deepspeed/zero2.json); ``window`` accumulates them locally over the
    ``grad_accum`` window and reduce-scatters once, during the boundary micro-step's backward
    (ZeRO-1 communication: 1/grad_accum of the xGMI traffic).  Optimizer state stays sharded
    either way, and the engine's flat gradient buffer is full-size in both modes, so HBM is the
    same."""
    if grad_reduce not in ("micro", "window"):
        raise ValueError(f"grad_reduce must be micro or window, not {grad_reduce}")
    if strategy not in STRATEGIES:
        raise ValueError(f"unknown strategy {strategy}")
    cfg = EngineConfig(strategy=strategy, compute_dtype=compute_dtype, bucket_mb=bucket_mb, seed=seed)
    ds = ds_config or {}
    zero_like = strategy in ("zero2", "zero3") or semantics == "uniform"
    if zero_like:
        # defaults = the reference's DeepSpeed configs; the DS JSON (if any) overrides them below
        cfg.lr, cfg.betas, cfg.eps, cfg.weight_decay = 1e-4, (0.9, 0.999), 1e-8, 0.01
        cfg.grad_accum = max(1, int(grad_accum))
        cfg.grad_clip = 1.0 if not ds else 0.0
        cfg.scheduler = None if ds else {"type": "WarmupLR", "params": {
            "warmup_min_lr": 0, "warmup_max_lr": cfg.lr, "warmup_num_steps": 5}}
    else:   # reference DDP / FSDP: AdamW(lr=1e-4, wd=0.01) every micro-step
        cfg.lr, cfg.weight_decay, cfg.grad_accum, cfg.grad_clip, cfg.scheduler = 1e-4, 0.01, 1, 0.0, None
    if strategy == "zero2":
        cfg.zero_stage = 2
    if strategy == "zero3":
        cfg.zero_stage = 3
        cfg.persistence_threshold, cfg.max_live_parameters, cfg.max_reuse_distance = int(1e5), int(1e9), int(1e9)
        cfg.extra["prefetch_elems"] = int(5e8)
    # every DeepSpeed key is honoured, satisfied by construction, or rejected (parallel/ds_config.py)
    cfg.extra["ds_keys"] = apply_deepspeed_config(cfg, ds, strategy, zero_like) if ds else {}
    if strategy == "zero2":
        if grad_reduce == "window":
            cfg.zero_stage = 1
        cfg.extra["grad_reduce"] = "window" if cfg.zero_stage == 1 else "micro"
    if strategy == "zero3":
        cfg.reshard_after_forward = True
        cfg.wrap = "unit"
    if strategy == "fsdp":
        fc = fsdp_config or {}
        ss = str(fc.get("sharding_strategy", "full_shard")).lower()
        cfg.reshard_after_forward = ss != "shard_grad_op"
        if ss == "no_shard":
            cfg.extra["no_shard"] = True
        pol = str(fc.get("auto_wrap_policy", "transformer_block")).lower()
        cfg.wrap = "root" if pol in ("size_based", "root", "none") else "block"
        bp = str(fc.get("backward_prefetch", "backward_pre")).lower()
        cfg.prefetch = 0 if bp in ("none", "false", "no") else 1
        # forward_prefetch (fsdp_config.yaml:9): gather unit i+1 while unit i computes.  False (torch's
        # default, fsdp_reference_root.yaml) issues each unit's all-gather only when it is needed
        cfg.extra["forward_prefetch"] = bool(fc.get("forward_prefetch", True)) and cfg.prefetch > 0
        if fc.get("mixed_precision") is False and fc.get("param_dtype") == "float32":
            cfg.compute_dtype = torch.float32
    if cfg.compute_dtype == torch.float16:
        cfg.extra["loss_scaling"] = True     # GradScaler semantics (train_harness.py:334-335, 371-376)
    cfg.extra["semantics"] = semantics
    for k, v in (overrides or {}).items():
        setattr(cfg, k, v)
    return cfg


def make_engine(model, cfg: EngineConfig, device, group=None):
    """Instantiate the engine for ``cfg.strategy`` (reference ``wrap_model`` equivalent)."""
    s = cfg.strategy
    if s == "ddp" or (s == "fsdp" and cfg.extra.get("no_shard")):
        return DDPEngine(model, cfg, device, group)
    if s == "zero2":
        return Zero2Engine(model, cfg, device, group)
    if s == "fsdp":
        return FSDPEngine(model, cfg, device, group)
    if s == "zero3":
        return Zero3Engine(model, cfg, device, group)
    raise ValueError(s)
