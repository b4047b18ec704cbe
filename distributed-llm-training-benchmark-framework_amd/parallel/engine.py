"""Common training-engine machinery shared by the DDP / ZeRO / FSDP engines.

An engine owns the model's parameter storage (flat bf16 buffers), its gradient storage, the fused
optimizer over the rank's fp32 owner space and the collectives.  Its public API mirrors what the
reference harness drives (DeepSpeed's engine interface, train_harness.py:364-368, and the AMP
loop, :370-382):

    loss = engine(batch, targets)[1]       # forward (one micro-batch)
    engine.backward(loss)                  # backward + gradient collectives
    engine.step()                          # optimizer step at accumulation boundaries

Micro-step bookkeeping: ``grad_accum`` micro-steps form one accumulation window; the last one is
the *boundary* where the optimizer runs (with gradient clipping and the LR schedule when
configured).  Gradients are averaged over ranks and micro-steps by folding ``1/(world*accum)``
(and the clipping coefficient) into the optimizer's device-side gradient scale — no extra pass
over the gradients and no host synchronisation.
"""
from dataclasses import dataclass, field
from typing import Optional

import torch

from ..comm import Comm
from ..ops._ext import ext
from ..ops.rng import StepSeed
from ..optim.amp import DynamicLossScaler
from ..optim.sched import build_scheduler
from .runtime import ParamRuntime, Unit


@dataclass
class EngineConfig:
    strategy: str = "ddp"
    lr: float = 1e-4
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.01
    grad_accum: int = 1
    grad_clip: float = 0.0
    scheduler: Optional[dict] = None          # DeepSpeed-style {"type": "WarmupLR", "params": {...}}
    compute_dtype: torch.dtype = torch.bfloat16
    bucket_mb: float = 64.0                   # gradient bucket cap (xGMI-tuned default)
    seed: int = 42
    # sharded engines
    reshard_after_forward: bool = True
    prefetch: int = 1                         # units gathered ahead (forward and backward)
    persistence_threshold: int = 0            # ZeRO-3: params below this numel stay replicated
    max_live_parameters: int = 0              # ZeRO-3: keep gathered params if the model fits
    max_reuse_distance: int = 0
    wrap: str = "block"                       # FSDP: "block" (per transformer block) | "root"
    zero_stage: int = 0
    extra: dict = field(default_factory=dict)


class Engine(ParamRuntime):
    name = "engine"

    def __init__(self, model, cfg: EngineConfig, device, group=None):
        super().__init__()
        self.model = model
        self.cfg = cfg
        self.device = torch.device(device)
        self.group = group
        self.comm = Comm(group)          # every collective of the engine goes through this
        self.world, self.rank = self.comm.world, self.comm.rank
        self.accum = max(1, int(cfg.grad_accum))
        self.compute_dtype = cfg.compute_dtype if self.device.type == "cuda" else torch.float32
        # fp16 compute (the reference's DDP/FSDP autocast): dynamic loss scaling, decided on the device
        self.scaler = DynamicLossScaler(self.device, **cfg.extra.get("loss_scale_args", {})) \
            if cfg.extra.get("loss_scaling") else None
        self.seed = StepSeed(cfg.seed, self.rank, self.device)
        self.sched = build_scheduler(cfg.scheduler, cfg.lr)
        self.micro = 0
        self.opt_steps = 0
        self._is_boundary = self.accum == 1
        self._window_pos = 0
        self._written = {}
        self.last_lr = None
        self.grad_norm = None
        self._norm_sq = torch.zeros(1, device=self.device, dtype=torch.float32)
        self._gscale = torch.ones(1, device=self.device, dtype=torch.float32)
        self._comm_static = 0            # modelled wire bytes per micro-step (set by the engines)
        self._sparse_model = 0.0         # + the token-row exchange (parallel/replicated.py), per micro-step
        self.timers = None               # utils.timers.PhaseTimers while the harness times phases
        self._reported = set()   # id(unit) of the units whose backward reported this micro-step
        self._cache_wt = False   # subclasses: True where parameters stay resident between steps
        self._wt = {}            # (unit index, param index) -> (W view, W^T view of a stacked buffer)
        self._wt_stack = {}      # (param index, shape) -> [units, K, N] buffer of transposes
        self._wt_epoch = -1      # optimizer step the cached transposes belong to
        model.rt = self
        self._setup()

    @property
    def comm_bytes_per_step(self) -> int:
        """Modelled wire bytes one rank sends per micro-step (ring algorithms): the engine's static
        collectives plus, once the batch shape is known, the sparse token-row exchange."""
        return int(self._comm_static + self._sparse_model)

    @comm_bytes_per_step.setter
    def comm_bytes_per_step(self, v):
        self._comm_static = v

    def _model_sparse(self, rows: int, d: int, elem: int, idx_elem: int, every: float):
        """Model of the token-row exchange: two all-gathers (rows x d, rows ids) per exchange,
        ``every`` exchanges per micro-step."""
        frac = (self.world - 1) / self.world
        self._sparse_model = frac * self.world * rows * (d * elem + idx_elem) * every

    def _phase(self, name: str):
        if self.timers is not None:
            self.timers.mark(name)

    # ------------------------------------------------------------------ subclass hooks
    def _setup(self):
        raise NotImplementedError

    def _on_begin_micro(self):
        pass

    def _finish_backward(self):
        pass

    def _optimizer_step(self, lr: float):
        raise NotImplementedError

    # ------------------------------------------------------------------ public API
    def __call__(self, idx, targets=None):
        return None, self.forward(idx, targets)

    def forward(self, idx, targets=None):
        self._begin_micro()
        _, loss = self.model(idx, targets)
        return loss

    def backward(self, loss):
        loss.backward(self.scaler.grad_output if self.scaler is not None else None)
        self._finish_backward()

    def step(self):
        if self._is_boundary:
            lr = self.sched(self.opt_steps)
            self.last_lr = lr
            if self._defer_opt:
                self._pending_lr = lr             # runs at the start of the next micro-step
            else:
                self._optimizer_step(lr)
            self.opt_steps += 1
        self.micro += 1

    # Deferred optimizer step (replicated ZeRO-1/2 at world > 1): the window's clip + AdamW run at
    # the beginning of the NEXT micro-step and the bf16 parameter all-gather is issued per bucket,
    # asynchronously, in forward order -- each unit waits only for its own bucket (``acquire``), so
    # the all-gather hides behind the forward instead of ending the window exposed.  The work per
    # window is unchanged; ``finalize()`` runs a pending update (end of training, checkpoints).
    _defer_opt = False
    _pending_lr = None

    def _run_pending_opt(self):
        if self._pending_lr is not None:
            lr, self._pending_lr = self._pending_lr, None
            self._phase("opt_begin")
            self._deferred_optimizer_step(lr)
            self._phase("opt_end")

    def _deferred_optimizer_step(self, lr: float):
        self._optimizer_step(lr)

    def finalize(self):
        """Apply a pending (deferred) optimizer step and wait for outstanding collectives."""
        self._run_pending_opt()
        self._wait_param_gathers()

    def _wait_param_gathers(self):
        pass

    # ------------------------------------------------------------------ HIP-graph support
    def replay_host_step(self):
        """The host-side effects of one micro-step (what forward/backward/step do besides GPU
        work), for a step whose GPU work is a HIP-graph replay: new dropout seed on the device,
        window position, and the scheduler LR uploaded for the optimizer update this graph runs
        (at the window boundary, or -- deferred -- at the next window's first micro-step)."""
        if self._pending_lr is not None:
            lr, self._pending_lr = self._pending_lr, None
            self.opt.prepare(lr)
        self.seed.next()
        self._window_pos = self.micro % self.accum
        self._is_boundary = self._window_pos == self.accum - 1
        if self._is_boundary:
            lr = self.sched(self.opt_steps)
            self.last_lr = lr
            if self._defer_opt:
                self._pending_lr = lr
            else:
                self.opt.prepare(lr)
            self.opt_steps += 1
        self.micro += 1

    def upload_step_state(self):
        """After a capture (whose host effects already ran): push the current seed / optimizer
        hyper-parameters to the device before the first replay."""
        self.seed.upload()
        if self.opt.step_count > 0:
            self.opt.upload()

    def train(self, mode=True):
        self.model.train(mode)
        return self

    def eval(self):
        return self.train(False)

    def zero_grad(self, set_to_none=True):   # grads are overwritten at window start; kept for API parity
        pass

    @property
    def is_boundary(self):
        return self._is_boundary

    # ------------------------------------------------------------------ cached weight transposes
    def weight_t(self, unit, i, w):
        """Cached W^T for the NT-form data-gradient GEMM (engines whose parameters stay resident
        between optimizer steps: replicated ones, sharded ones at world size 1).  The transposes of
        one parameter kind live in one stacked buffer, one row per unit holding that kind in
        reversed unit order (the order of the parameters in the flat buffers), so after an
        optimizer step all of them are refreshed by ONE batched LDS-tiled transpose launch per kind
        instead of one launch per block."""
        if not self._cache_wt or w.dim() != 2 or not w.is_cuda:
            return None
        if self._wt_epoch != self.opt_steps:
            self._refresh_weight_t()
            self._wt_epoch = self.opt_steps
        key = (unit.index, i)
        hit = self._wt.get(key)
        if hit is not None:
            return hit[1]
        g = (i, tuple(w.shape))
        stack = self._wt_stack.get(g)
        # one row per unit holding a parameter of this kind, in the order of the parameters in the
        # engine's flat buffers (reversed unit order unless the engine says otherwise), so the
        # refresh finds W and W^T equally spaced and batches them
        units = self.model.units()
        order = reversed(units) if getattr(self, "wgrad_rows_reversed", True) else units
        rows = [u.index for u in order if len(u.shapes) > i and u.shapes[i] == g[1]]
        if stack is None:
            stack = torch.empty((len(rows), w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device)
            self._wt_stack[g] = stack
        wt = stack[rows.index(unit.index)]
        ext().transpose_into(w, wt)          # first use: transpose now
        self._wt[key] = (w, wt)
        return wt

    def _refresh_weight_t(self):
        from .wgrad import strided_batch
        groups = {}
        for (uidx, i), (w, wt) in self._wt.items():
            groups.setdefault((i, tuple(w.shape)), []).append((w, wt))
        C = ext()
        for items in groups.values():
            items.sort(key=lambda it: it[1].data_ptr())
            W = strided_batch([it[0] for it in items])
            WT = strided_batch([it[1] for it in items], out=True)
            if W is not None and WT is not None and len(items) > 1:
                C.transpose_batched(items[0][0], items[0][1], len(items), W.stride(0), WT.stride(0))
            else:
                for w, wt in items:
                    C.transpose_into(w, wt)

    # ------------------------------------------------------------------ micro-step bookkeeping
    def _begin_micro(self):
        self._run_pending_opt()
        self.seed.next()
        self._window_pos = self.micro % self.accum
        self._is_boundary = self._window_pos == self.accum - 1
        if self._window_pos == 0:
            self._written.clear()
        self._on_begin_micro()

    def _mark(self, unit: Unit, i: int) -> bool:
        """Returns True when the slot already holds data of this accumulation window."""
        key = (id(unit), i)
        acc = self._written.get(key, False)
        self._written[key] = True
        return acc

    def _zero_unreported(self):
        """Units whose backward did not run this micro-step (parameters the loss does not use: torch
        DDP's ``find_unused_parameters`` case, which the reference turns off, train_harness.py:221):
        every gradient slot of theirs that holds nothing of the current accumulation window is
        zeroed (and marked written), so a stale gradient of an earlier step is never reduced or
        applied.  Returns those units."""
        units = self.model.units()
        if len(self._reported) >= len(units):
            self._reported.clear()
            return []
        out = []
        for u in units:
            if id(u) in self._reported:
                continue
            for i in range(len(u.params)):
                t, acc = self.grad_slot(u, i)
                if not acc:
                    t.zero_()
            out.append(u)
        self._reported.clear()
        return out

    # ------------------------------------------------------------------ helpers
    def _wait_works(self):
        self.comm.wait_all()

    def _sumsq_into(self, t: torch.Tensor, out: torch.Tensor):
        if t.is_cuda:
            ext().sumsq_(t, out)
        else:
            out += t.float().pow(2).sum()

    def _apply_update(self, g, lr: float, extra_scale: float, sharded: bool):
        """Clip coefficient (+ loss-scale unscale / skip decision) and the fused AdamW update of the
        owner gradient ``g``.  With a loss scaler the AdamW hyper-parameters are uploaded first:
        ``amp_step`` overwrites their bias corrections (device step count) and the skip flag."""
        if self.scaler is None:
            self.opt.step(g, lr, self._clip_coef([g], extra_scale, sharded))
        elif g.is_cuda:
            self.opt.prepare(lr)
            self.opt.launch(g, self._clip_coef([g], extra_scale, sharded))
        else:
            gscale = self._clip_coef([g], extra_scale, sharded)
            if not self.scaler.last_skipped:
                self.opt.step(g, lr, gscale)

    def _clip_coef(self, grads, extra_scale: float, sharded: bool):
        """Device gradient scale = extra_scale * min(1, clip / ||extra_scale * g||).  Also records
        the global gradient norm in ``self.grad_norm`` (device tensor).  With a loss scaler the norm
        pass is also the inf check and the scale folds 1/S in (optim/amp.py)."""
        if self.scaler is not None:
            self._norm_sq.zero_()
            for g in grads:
                self._sumsq_into(g, self._norm_sq)
            if sharded and self.world > 1:
                self.comm.all_reduce(self._norm_sq, async_op=False)
            if self.grad_norm is None:
                self.grad_norm = torch.zeros(1, device=self.device)
            self.scaler.step(self._norm_sq, self._gscale, self.grad_norm, self.opt.hp, float(self.cfg.grad_clip),
                             extra_scale, self.opt.betas)
            return self._gscale
        want_norm = self.cfg.grad_clip > 0 or self.cfg.extra.get("track_grad_norm", False)
        if not want_norm:
            self._gscale.fill_(extra_scale)
            return self._gscale
        self._norm_sq.zero_()
        for g in grads:
            self._sumsq_into(g, self._norm_sq)
        if sharded and self.world > 1:
            self.comm.all_reduce(self._norm_sq, async_op=False)
        if self.device.type == "cuda":
            if self.grad_norm is None:
                self.grad_norm = torch.zeros(1, device=self.device)
            ext().clip_coef(self._norm_sq, float(self.cfg.grad_clip), self._gscale, self.grad_norm, extra_scale)
        else:
            nrm = self._norm_sq.sqrt() * extra_scale
            c = torch.clamp(self.cfg.grad_clip / (nrm + 1e-6), max=1.0) if self.cfg.grad_clip > 0 else torch.ones_like(nrm)
            self._gscale.copy_(c * extra_scale)
            self.grad_norm = nrm
        return self._gscale

    # ------------------------------------------------------------------ checkpoint / resume
    def state_dict(self) -> dict:
        self.finalize()
        return self._state_dict()

    def _state_dict(self) -> dict:
        """This rank's resumable state: optimizer partition (fp32 master, exp_avg, exp_avg_sq,
        step), micro/optimizer-step counters and the dropout seed stream.  Only at a window
        boundary (no half-accumulated gradients to carry)."""
        if self.micro % self.accum != 0:
            raise RuntimeError("checkpoint only at a gradient-accumulation boundary")
        return {"format": "dltb-engine-v1", "engine": type(self).__name__, "strategy": self.cfg.strategy,
                "world": self.world, "rank": self.rank, "accum": self.accum, "micro": self.micro,
                "opt_steps": self.opt_steps, "seed_state": str(self.seed.state),
                "optimizer": self.opt.state_dict(),
                "loss_scaler": self.scaler.state_dict() if self.scaler is not None else None}

    def load_state_dict(self, sd: dict):
        if sd.get("format") != "dltb-engine-v1":
            raise ValueError("not a dltb engine checkpoint")
        for k, mine in (("engine", type(self).__name__), ("world", self.world), ("rank", self.rank)):
            if sd[k] != mine:
                raise ValueError(f"checkpoint {k}={sd[k]!r} does not match this run ({mine!r})")
        if sd["optimizer"]["master"].numel() != self.opt.master.numel():
            raise ValueError("checkpoint partition size differs (different model or layout)")
        self._pending_lr = None
        self._wait_param_gathers()
        self.micro, self.opt_steps = int(sd["micro"]), int(sd["opt_steps"])
        self.seed.state = int(sd["seed_state"])
        self.seed.value = self.seed.state
        self.opt.load_state_dict(sd["optimizer"])
        if self.scaler is not None and sd.get("loss_scaler") is not None:
            self.scaler.load_state_dict(sd["loss_scaler"])
        self._after_param_load()

    def _after_param_load(self):
        """Rebuild the compute-dtype parameters from the freshly loaded master partition."""

    # ------------------------------------------------------------------ introspection
    def memory_report(self) -> dict:
        return {}

    def full_state_dict(self) -> dict:
        """Gather a full fp32 state dict (master weights) on every rank."""
        raise NotImplementedError
