"""Learning-rate schedules.

``WarmupLR`` reproduces DeepSpeed's WarmupLR used by configs/deepspeed/zero{2,3}.json
(``warmup_min_lr 0 -> warmup_max_lr 1e-4 over warmup_num_steps 5``).  DeepSpeed's default
``warmup_type`` is "log": for optimizer step k (0-based) below the warmup length,
``lr = min + (max - min) * log(k + 1) / log(warmup_num_steps)`` (so the very first optimizer step
runs at ``min``), afterwards ``max``.  ``warmup_type: linear`` uses ``k / warmup_num_steps``.
The DDP/FSDP paths of the reference use a constant lr (train_harness.py:329).
"""
import math


class ConstantLR:
    def __init__(self, lr: float):
        self.base = lr

    def __call__(self, k: int) -> float:
        return self.base


class WarmupLR:
    def __init__(self, warmup_min_lr=0.0, warmup_max_lr=1e-4, warmup_num_steps=1000,
                 warmup_type="log"):
        self.min = float(warmup_min_lr)
        self.max = float(warmup_max_lr)
        self.n = max(1, int(warmup_num_steps))
        self.type = warmup_type
        self.inv_log = 1.0 / math.log(self.n) if self.n > 1 else 1.0

    def __call__(self, k: int) -> float:
        if k < self.n:
            if self.type == "log":
                gamma = math.log(k + 1) * self.inv_log if self.n > 1 else 1.0
            else:
                gamma = min(1.0, k / self.n)
            return self.min + (self.max - self.min) * gamma
        return self.max


def build_scheduler(spec, default_lr: float):
    """``spec``: None or a DeepSpeed-style ``{"type": ..., "params": {...}}`` dict."""
    if not spec:
        return ConstantLR(default_lr)
    typ = spec.get("type", "")
    params = dict(spec.get("params", {}))
    if typ == "WarmupLR":
        return WarmupLR(**params)
    raise ValueError(f"unsupported scheduler type {typ!r}")
