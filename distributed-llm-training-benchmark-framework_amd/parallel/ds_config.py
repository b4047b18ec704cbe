"""DeepSpeed-JSON schema reader: every key of a ZeRO config is honoured, satisfied by construction,
or rejected loudly -- nothing is dropped silently.

Reference: ``configs/deepspeed/zero2.json:1-49`` and ``configs/deepspeed/zero3.json:1-51``, read by
``deepspeed.initialize`` at ``benchmarking/train_harness.py:240-271``.  DeepSpeed is not a dependency:
``apply_deepspeed_config`` maps the keys onto the native engines' ``EngineConfig`` and returns a
report, which the harness writes into the result sidecar (``deepspeed_config_keys``) and bench.py
prints in its JSON line:

* ``honoured``        key -> value: the engine does what the key says;
* ``by_construction`` key -> why: the engine's design already gives the key's effect (or its value
                      is the only behaviour offered), so no switch is needed;
* ``ignored``         key -> why: accepted, no effect on the run (documentation / logging keys of
                      DeepSpeed subsystems that do not exist here).

A value the engines cannot honour (CPU / NVMe offload, another optimizer, a bucket cap smaller than
one unit, ...) raises ``ValueError`` naming the key.

Semantics of the size keys (elements, as in DeepSpeed):

* ``reduce_bucket_size`` / ``allgather_bucket_size`` (stage 1/2): upper bounds of one reduce-scatter /
  one parameter all-gather.  The replicated engines reduce and re-gather per gradient bucket, so the
  bucket planner closes a bucket before a unit would push it past ``min(reduce, allgather)``.  Buckets
  are unit-granular (a transformer block is the smallest bucket); a cap below the largest unit is
  rejected.
* ``reduce_bucket_size`` (stage 3): each ZeRO-3 reduce-scatter is one unit's gradient, issued the
  moment that unit's backward completes (per-unit overlap), so the cap is honoured when it is at
  least the largest unit and rejected otherwise.
* ``stage3_prefetch_bucket_size``: an element budget -- the sharded engine gathers the next units
  ahead (forward and backward) while their summed size stays within the budget (at least one).
* ``stage3_max_live_parameters`` / ``stage3_max_reuse_distance``: a unit gathered for the forward is
  kept for its backward instead of being released and re-gathered when the parameters touched
  between its two uses (reuse distance: the later units' forward and backward) stay within
  ``max_reuse_distance`` and the gathered total stays within ``max_live_parameters``; when the whole
  model fits both, every unit stays gathered for the accumulation window.
* ``sub_group_size`` (stage 3): the fused AdamW updates the owner space in launches of at most this
  many elements (DeepSpeed's optimizer sub-groups).
"""
from typing import Optional

_OFFLOAD_OK = (None, "none")
_OPTIMIZERS = ("adamw", "adam")     # DeepSpeed's "Adam" is FusedAdam(adam_w_mode=True): decoupled decay


def _num(v, default=None):
    if v is None or v == "auto":
        return default
    return float(v) if not isinstance(v, bool) else v


class DSReport:
    def __init__(self):
        self.honoured = {}
        self.by_construction = {}
        self.ignored = {}

    def ok(self, key, value):
        self.honoured[key] = value

    def built_in(self, key, why):
        self.by_construction[key] = why

    def skip(self, key, why):
        self.ignored[key] = why

    def as_dict(self):
        return {"honoured": dict(self.honoured), "by_construction": dict(self.by_construction),
                "ignored": dict(self.ignored)}


def _reject(key, value, why):
    raise ValueError(f"DeepSpeed config {key}={value!r}: {why}")


def apply_deepspeed_config(cfg, ds: Optional[dict], strategy: str, zero_like: bool) -> dict:
    """Map the DeepSpeed JSON ``ds`` onto ``cfg`` (an EngineConfig) for ``strategy``.  ``zero_like``:
    the run uses the ZeRO step semantics (optimizer / clipping / scheduler keys apply).  Returns the
    key report (``DSReport.as_dict``)."""
    rep = DSReport()
    ds = dict(ds or {})
    if not ds:
        return rep.as_dict()
    for key in list(ds):
        if key.startswith("_"):                      # _comment and friends
            ds.pop(key)
    # ---- batch keys: injected from the CLI at run time (train_harness.py:251-262)
    for key in ("train_batch_size", "train_micro_batch_size_per_gpu", "gradient_accumulation_steps"):
        if key in ds:
            rep.built_in(key, "set from --per-device-batch / --grad-accum / world size at run time "
                              "(the reference pops and re-injects them, train_harness.py:251-262)")
            ds.pop(key)
    # ---- precision
    bf16 = bool((ds.pop("bf16", None) or {}).get("enabled", False))
    fp16_spec = ds.pop("fp16", None) or {}
    fp16 = bool(fp16_spec.get("enabled", False))
    if bf16 and fp16:
        _reject("bf16.enabled+fp16.enabled", True, "both precisions enabled")
    if bf16:
        rep.ok("bf16.enabled", True)
    if fp16:
        rep.ok("fp16.enabled", True)
        cfg.extra["ds_dtype"] = "fp16"
        for k in ("loss_scale", "initial_scale_power", "loss_scale_window", "hysteresis", "min_loss_scale"):
            if k in fp16_spec:
                rep.skip(f"fp16.{k}", "dynamic loss scaling follows torch GradScaler's schedule "
                                      "(optim/amp.py: 2^16, x0.5 on overflow, x2 after 2000 clean steps)")
    elif bf16:
        cfg.extra["ds_dtype"] = "bf16"
    # ---- optimizer / schedule / clipping (ZeRO step semantics)
    opt = ds.pop("optimizer", None)
    if opt is not None:
        typ = str(opt.get("type", "AdamW"))
        if typ.lower() not in _OPTIMIZERS:
            _reject("optimizer.type", typ, "only AdamW / Adam (fused AdamW, csrc/adamw.hip) is implemented")
        p = dict(opt.get("params", {}))
        if p.get("adam_w_mode", True) is False:
            _reject("optimizer.params.adam_w_mode", False, "L2-coupled Adam is not implemented")
        if p.get("torch_adam"):
            rep.skip("optimizer.params.torch_adam", "the fused HIP AdamW is always used")
        p.pop("adam_w_mode", None), p.pop("torch_adam", None)
        if zero_like:
            cfg.lr = _num(p.pop("lr", None), 1e-4)
            cfg.betas = tuple(p.pop("betas", (0.9, 0.999)))
            cfg.eps = _num(p.pop("eps", None), 1e-8)
            cfg.weight_decay = _num(p.pop("weight_decay", None), 0.01)
            rep.ok("optimizer", {"type": typ, "lr": cfg.lr, "betas": list(cfg.betas), "eps": cfg.eps,
                                 "weight_decay": cfg.weight_decay})
        for k in p:
            _reject(f"optimizer.params.{k}", p[k], "unknown AdamW parameter")
    if "gradient_clipping" in ds:
        v = _num(ds.pop("gradient_clipping"), 0.0)
        if zero_like:
            cfg.grad_clip = v
            rep.ok("gradient_clipping", v)
    sched = ds.pop("scheduler", None)
    if sched is not None:
        if sched.get("type") != "WarmupLR":
            _reject("scheduler.type", sched.get("type"), "only WarmupLR is implemented (optim/sched.py)")
        if zero_like:
            cfg.scheduler = sched
            rep.ok("scheduler", sched)
    # ---- logging / profiling
    if "steps_per_print" in ds:
        v = int(ds.pop("steps_per_print"))
        cfg.extra["steps_per_print"] = v
        rep.ok("steps_per_print", v)                 # the harness's log cadence (unless --log-every)
    if "wall_clock_breakdown" in ds:
        v = bool(ds.pop("wall_clock_breakdown"))
        cfg.extra["wall_clock_breakdown"] = v
        rep.ok("wall_clock_breakdown", v)            # true: per-phase HIP-event timers (--phase-timers)
    fp = ds.pop("flops_profiler", None)
    if fp is not None:
        rep.built_in("flops_profiler", "model FLOPs per token / TFLOP/s per GPU / MFU are always reported "
                                       "(tflops_per_gpu in the sidecar and bench.py's JSON line)")
    # ---- ZeRO
    z = dict(ds.pop("zero_optimization", None) or {})
    if z:
        _apply_zero(cfg, z, strategy, rep)
    for key, val in ds.items():                      # anything else at top level
        rep.skip(key, "not a ZeRO / optimizer / precision key this framework models")
    return rep.as_dict()


def _apply_zero(cfg, z, strategy, rep):
    stage = int(z.pop("stage", 2 if strategy == "zero2" else 3))
    if strategy == "zero2" and stage not in (1, 2):
        _reject("zero_optimization.stage", stage, "--strategy zero2 runs stage 1 or 2")
    if strategy == "zero3" and stage != 3:
        _reject("zero_optimization.stage", stage, "--strategy zero3 runs stage 3")
    rep.ok("zero_optimization.stage", stage)
    for k in ("offload_optimizer", "offload_param"):
        spec = z.pop(k, None)
        dev = (spec or {}).get("device") if isinstance(spec, dict) else spec
        if dev not in _OFFLOAD_OK:
            _reject(f"zero_optimization.{k}.device", dev,
                    "no host / NVMe offload: optimizer state and parameters live in HBM (288 GB per MI355X)")
        if spec is not None:
            rep.ok(f"zero_optimization.{k}.device", "none")
    if "contiguous_gradients" in z:
        z.pop("contiguous_gradients")
        rep.built_in("zero_optimization.contiguous_gradients",
                     "gradients are always written in place into flat, bucket-contiguous buffers (parallel/flat.py)")
    overlap = z.pop("overlap_comm", None)
    if overlap is not None:
        cfg.extra["overlap_comm"] = bool(overlap)
        rep.ok("zero_optimization.overlap_comm", bool(overlap))
    rb = _num(z.pop("reduce_bucket_size", None))
    if rb:
        cfg.extra["reduce_bucket_elems"] = int(rb)
        rep.ok("zero_optimization.reduce_bucket_size", int(rb))
    if strategy == "zero2":
        cfg.zero_stage = stage
        if "reduce_scatter" in z:
            v = bool(z.pop("reduce_scatter"))
            cfg.extra["reduce_scatter"] = v
            rep.ok("zero_optimization.reduce_scatter", v)
        if "allgather_partitions" in z:
            v = bool(z.pop("allgather_partitions"))
            cfg.extra["allgather_partitions"] = v
            rep.ok("zero_optimization.allgather_partitions", v)
        ab = _num(z.pop("allgather_bucket_size", None))
        if ab:
            cfg.extra["allgather_bucket_elems"] = int(ab)
            rep.ok("zero_optimization.allgather_bucket_size", int(ab))
        if "round_robin_gradients" in z:
            z.pop("round_robin_gradients")
            rep.built_in("zero_optimization.round_robin_gradients",
                         "every bucket is split into world-size equal chunks, so each rank's gradient "
                         "partition already takes an equal share of every bucket")
    else:
        cfg.zero_stage = 3
        cfg.persistence_threshold = int(_num(z.pop("stage3_param_persistence_threshold", None), 1e5))
        rep.ok("zero_optimization.stage3_param_persistence_threshold", cfg.persistence_threshold)
        cfg.max_live_parameters = int(_num(z.pop("stage3_max_live_parameters", None), 1e9))
        rep.ok("zero_optimization.stage3_max_live_parameters", cfg.max_live_parameters)
        cfg.max_reuse_distance = int(_num(z.pop("stage3_max_reuse_distance", None), 1e9))
        rep.ok("zero_optimization.stage3_max_reuse_distance", cfg.max_reuse_distance)
        pf = int(_num(z.pop("stage3_prefetch_bucket_size", None), 5e8))
        cfg.prefetch = 1 if pf > 0 else 0
        cfg.extra["prefetch_elems"] = pf
        rep.ok("zero_optimization.stage3_prefetch_bucket_size", pf)
        sg = _num(z.pop("sub_group_size", None))
        if sg:
            cfg.extra["sub_group_elems"] = int(sg)
            rep.ok("zero_optimization.sub_group_size", int(sg))
        if "stage3_gather_16bit_weights_on_model_save" in z:
            v = bool(z.pop("stage3_gather_16bit_weights_on_model_save"))
            rep.built_in("zero_optimization.stage3_gather_16bit_weights_on_model_save",
                         "--export-model always gathers the consolidated 16-bit weights "
                         "(parallel/checkpoint.py); the reference never saves a model")
            cfg.extra["gather_16bit_on_save"] = v
        for k in ("reduce_scatter", "allgather_partitions", "allgather_bucket_size", "round_robin_gradients"):
            if k in z:
                rep.skip(f"zero_optimization.{k}", "a stage 1/2 key; stage 3 reduce-scatters per unit and "
                                                   "gathers per unit")
                z.pop(k)
    for k, v in z.items():
        rep.skip(f"zero_optimization.{k}", "not modelled by the native ZeRO engines")


def check_bucket_caps(cfg, unit_numels, strategy: str):
    """Reject bucket caps the unit-granular engines cannot honour (called by the engines with the
    model's unit sizes, which the config reader does not know)."""
    caps = [("zero_optimization.reduce_bucket_size", cfg.extra.get("reduce_bucket_elems"))]
    if strategy != "zero3":
        caps.append(("zero_optimization.allgather_bucket_size", cfg.extra.get("allgather_bucket_elems")))
    big = max(unit_numels) if unit_numels else 0
    for key, cap in caps:
        if cap and cap < big:
            _reject(key, cap, f"smaller than the largest unit ({big} elements): buckets hold whole units "
                              "(a transformer block, the embedding, the head)")


def ds_precision(ds: Optional[dict]) -> str:
    """Compute dtype a DeepSpeed config asks for: "fp16" when ``fp16.enabled``, else "bf16" (the
    reference's zero2/3.json; fp32 compute is not offered on the GPU path)."""
    return "fp16" if ((ds or {}).get("fp16") or {}).get("enabled") else "bf16"
