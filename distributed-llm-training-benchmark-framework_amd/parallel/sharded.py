"""Sharded-parameter engines: FSDP (full-shard / shard-grad-op) and ZeRO-3.

Reference strategies: torch FSDP at train_harness.py:225-238 (size-based wrap -> one root
FlatParameter of the whole model) and DeepSpeed ZeRO-3 at :240-271 + configs/deepspeed/zero3.json.

MI355X-native design on ``torch.distributed`` (RCCL over xGMI):

* Parameters are grouped into *shard groups*: FSDP ``wrap=block`` -> one group per transformer block
  plus a root group {embedding, final norm / head}; ``wrap=root`` reproduces the reference's single
  FlatParameter; ZeRO-3 -> one group per unit (module-granular fetch).  Each group is one flat bf16
  buffer padded to ``world*128`` elements; a rank keeps only its chunk (its *shard*).
* Forward: ``acquire`` all-gathers a group's shard into a transient full buffer (RCCL
  ``all_gather_into_tensor``), prefetching the next ``prefetch`` groups so the gather of block i+1
  overlaps the compute of block i.  After the group's forward it is released (FULL_SHARD /
  ZeRO-3) or kept (SHARD_GRAD_OP, root group, or ZeRO-3 when the whole model fits under
  ``stage3_max_live_parameters`` / ``stage3_max_reuse_distance`` as in the reference config).
* Backward: released groups are re-gathered (previous groups prefetched); each group's full
  gradient buffer is reduce-scattered into this rank's owner space as soon as the group's backward
  completes, overlapping the rest of the backward.
* ZeRO-3 persistence: parameters smaller than ``stage3_param_persistence_threshold`` (LayerNorm
  weights, biases) stay replicated in one flat buffer that is reduce-scattered/all-gathered like
  ZeRO-2, so they never cost a fetch.
* Optimizer: one fused AdamW launch over the rank's owner space [persistent chunk | group shards];
  the bf16 shard is written in place and becomes the next all-gather's input.
* Precision of the reduction: gradients are reduce-scattered in the compute dtype.  In the fp16
  (reference-precision FSDP) runs that is the loss-scaled fp16 gradient, where the reference's
  torch FSDP (no mixed precision) reduces fp32: a sum over N ranks reaches fp16's range about N
  times sooner, so the dynamic loss scaler may back off more often at 8 ranks than the reference
  would.  Parity unpinned; bench.py and the harness report the scaler's skipped-step count
  (``loss_scaler.optimizer_steps_skipped``) so a run shows whether it happened.  DDP has the fp32
  communication option (``grad_comm_dtype``, replicated.py).
"""
import os

import torch

from ..ops._ext import ext
from ..optim.adamw import FlatAdamW
from .engine import Engine
from .flat import ALIGN, plan_layout
from .wgrad import WgradQueue

_HUGE = 1 << 62


class _Group:
    def __init__(self, gid, units):
        self.gid = gid
        self.units = units
        self.layout = None
        self.total = 0
        self.chunk = 0
        self.owner_start = 0
        self.shard = None            # this rank's bf16 chunk (view of the engine's shard buffer)
        self.full = None             # gathered full buffer (None when released)
        self.work = None             # in-flight all-gather
        self.grad = None             # full gradient buffer of the current backward (= grad_buf, or None)
        self.grad_buf = None         # the group's gradient buffer, allocated once
        self.fwd_left = 0
        self.bwd_left = 0
        self.root = False


class ShardedEngine(Engine):
    name = "sharded"

    def _group_units(self):
        units = self.model.units()
        if self.cfg.wrap == "root":
            return [units]
        if self.cfg.wrap == "unit":
            return [[u] for u in units]
        # "block": transformer blocks own a group each; embedding + head form the root group.  (Splitting the
        # tied head into a group of its own, reduced right after the head's backward, measured no better at
        # emulated N = 2 / 8: the exposed tail is the per-block re-gather + reduce-scatter queue of the
        # backward, not the table: profiles/fsdp_split_root_ab_r6.txt.)
        root = [units[0], units[-1]]
        return [root] + [[u] for u in units[1:-1]]

    def _setup(self):
        cfg, dev, dt = self.cfg, self.device, self.compute_dtype
        thr = int(cfg.persistence_threshold or 0)
        self._persistent = lambda u, i: thr > 0 and u.numels[i] < thr
        groups = [_Group(g, us) for g, us in enumerate(self._group_units())]
        if cfg.wrap == "block" and len(groups) > 1:
            groups[0].root = True
        if len(groups) == 1:
            groups[0].root = True
        self.groups = groups
        self._group_of = {}
        for g in groups:
            for u in g.units:
                self._group_of[id(u)] = g
        # forward order of first use
        order = []
        for u in self.model.units():
            g = self._group_of[id(u)]
            if g not in order:
                order.append(g)
        self._order = order
        self._pos = {g.gid: k for k, g in enumerate(order)}
        # persistent (replicated) parameters: one ZeRO-2 style bucket
        self.p_layout = plan_layout(list(reversed(self.model.units())), self.world, _HUGE, ALIGN, shard=True,
                                    param_filter=lambda u, i: self._persistent(u, i))
        p_total = self.p_layout.total
        p_chunk = self.p_layout.owner_numel
        # sharded groups
        owner = p_chunk
        for g in groups:
            g.layout = plan_layout(g.units, self.world, _HUGE, ALIGN, shard=True,
                                   param_filter=lambda u, i: not self._persistent(u, i))
            g.total = g.layout.total
            g.chunk = g.layout.owner_numel
            g.owner_start = owner
            owner += g.chunk
            g.fwd_left = len(g.units)
            g.bwd_left = len(g.units)
        self.n_owner = owner
        master = torch.zeros(owner, dtype=torch.float32, device=dev)
        self.shard_buf = torch.zeros(owner - p_chunk, dtype=dt, device=dev)
        self.p_flat = torch.zeros(p_total, dtype=dt, device=dev)
        self.p_grad = torch.zeros(p_total, dtype=dt, device=dev)
        # persistent params: full replicated copy + my chunk of master
        if p_total:
            pfull = torch.zeros(p_total, dtype=torch.float32, device=dev)
            for s in self.p_layout.slots.values():
                p = s.unit.params[s.index]
                pfull[s.offset:s.offset + s.numel] = p.detach().reshape(-1).to(dev, torch.float32)
            self.p_flat.copy_(pfull)
            master[:p_chunk] = pfull[self.rank * p_chunk:(self.rank + 1) * p_chunk]
            del pfull
        for g in groups:
            gfull = torch.zeros(g.total, dtype=torch.float32, device=dev)
            for s in g.layout.slots.values():
                p = s.unit.params[s.index]
                gfull[s.offset:s.offset + s.numel] = p.detach().reshape(-1).to(dev, torch.float32)
            mine = gfull[self.rank * g.chunk:(self.rank + 1) * g.chunk]
            master[g.owner_start:g.owner_start + g.chunk] = mine
            g.shard = self.shard_buf[g.owner_start - p_chunk:g.owner_start - p_chunk + g.chunk]
            g.shard.copy_(mine)
            del gfull
        # nn.Parameters no longer own storage: sharded ones become empty, persistent ones views
        empty = torch.empty(0, dtype=dt, device=dev)
        for u in self.model.units():
            for i, p in enumerate(u.params):
                s = self.p_layout.slots.get((id(u), i))
                if s is not None:
                    p.data = self.p_flat[s.offset:s.offset + s.numel].view(s.shape)
                elif (id(u), i) in self._group_of[id(u)].layout.slots:
                    p.data = empty
                p.grad = None
        segs = []
        if p_chunk:
            segs.append((0, p_chunk, self.p_flat[self.rank * p_chunk:(self.rank + 1) * p_chunk]))
        if owner > p_chunk:
            segs.append((p_chunk, owner - p_chunk, self.shard_buf))
        self.opt = FlatAdamW(master, segs, cfg.lr, cfg.betas, cfg.eps, cfg.weight_decay,
                             sub_group=int(cfg.extra.get("sub_group_elems", 0)))
        self.rs_out = torch.zeros(owner, dtype=dt, device=dev)
        self.acc = torch.zeros(owner, dtype=torch.float32, device=dev) if (self.accum > 1 and self.world > 1) else None
        total_sharded = sum(g.total for g in groups)
        self.keep_all = bool(cfg.max_live_parameters) and total_sharded <= cfg.max_live_parameters and \
            total_sharded <= (cfg.max_reuse_distance or _HUGE)
        # ZeRO-3 (parallel/ds_config.py): stage3_prefetch_bucket_size is an element budget of units
        # gathered ahead; without one (FSDP) ``cfg.prefetch`` units are.  A unit gathered for the
        # forward is kept for its backward when the parameters touched in between (the later units'
        # forward and backward) stay within stage3_max_reuse_distance and the gathered total within
        # stage3_max_live_parameters (DeepSpeed's release rule), instead of released and re-gathered
        self._prefetch_elems = int(cfg.extra.get("prefetch_elems", 0)) if cfg.zero_stage == 3 else 0
        tu = getattr(self.model, "tok_slot", (None,))[0]
        self._tied_group = self._group_of.get(id(tu)) if (tu is not None and self.world > 1) else None
        self._reuse_keep = set()
        if cfg.zero_stage == 3 and not self.keep_all and cfg.max_reuse_distance:
            after = 0
            for g in reversed(order):
                if 2 * after <= cfg.max_reuse_distance:
                    self._reuse_keep.add(g.gid)
                after += g.total
        self._overlap = bool(cfg.extra.get("overlap_comm", True))
        # ZeRO-3 / FSDP inside an accumulation window (world > 1): a micro-step that does not end its
        # window leaves its reduce-scatters in flight instead of waiting for them at the end of its
        # backward; the next backward's first gradient write waits for them and folds the chunks into
        # the fp32 accumulator (one launch), a forward later, when they are long done.  The window's
        # last micro-step drains everything before the optimizer (as the replicated engines do).
        # (resident group gradient buffers only, models below 2B parameters: with the transient
        # per-micro-step buffers of a larger model, deferring the drain would keep a full model of
        # bf16 gradients alive through the next forward -- ~14.5 GB per rank at Mistral-7B -- which
        # DeepSpeed / torch FSDP free at the end of the backward)
        self._grad_resident = sum(u.numel for u in self.model.units()) < 2_000_000_000
        self._tail_defer = (self.world > 1 and self.acc is not None and self._overlap and self._grad_resident and
                            bool(cfg.extra.get("defer_tail_reduce", True)))
        self._rs_inflight = []       # reduce-scatter works of the current / deferred micro-step
        self._deferred = False       # a finished micro-step's reduce-scatters are still to be drained
        self._deferred_first = False
        if cfg.zero_stage == 3 and cfg.extra.get("reduce_bucket_elems"):
            from .ds_config import check_bucket_caps
            check_bucket_caps(cfg, [g.total for g in groups] + [p_total], "zero3")   # (+ the persistent block)
        self._p_pending = len([u for u in self.model.units()
                               if any(self._persistent(u, i) for i in range(len(u.params)))])
        self._p_left = self._p_pending
        self._held_grads = []
        # (id(unit), id(gathered buffer)) -> parameter views into that buffer.  Gathered buffers come
        # from a per-size pool and are reused across gathers, so after the first micro-steps every
        # acquire is a dict hit instead of one slice + view per parameter (12 per block: ~0.1 ms of
        # host time per acquire, 36 acquires per FSDP micro-step)
        self._view_cache = {}
        self._gpool = {}             # numel -> free gathered buffers (returned by _release)
        self._pool_on = bool(cfg.extra.get("gather_pool", True))
        self._gviews = {}            # (id(unit), i) -> (gradient slot view, its group or None)
        # resident group gradient buffers at world > 1 for models below 2B parameters (a full model's
        # worth of bf16 gradients per rank: 0.47 GB at TinyGPT-A; Mistral-7B keeps transient ones):
        # self._grad_resident, set above
        self._reduced = set()        # group ids reduce-scattered in this micro-step
        self._p_reduced = False      # the persistent block reduce-scattered in this micro-step
        self._sparse = None          # (token slot, persistent?, gathered rows, gathered ids, works)
        # inside an accumulation window the token rows are carried into the next micro-step's dense
        # head-group gradient instead of exchanged (as the replicated engines do; the window's sum is
        # unchanged); only the window's last micro-step exchanges them
        self._carry_on = (self.world > 1 and self.accum > 1 and
                          bool(cfg.extra.get("carry_token_rows", True)))
        self._carry = None
        # single process: the dW products of all blocks run as strided-batched GEMMs at the end of
        # backward (parallel/wgrad.py).  World > 1 with resident gradient buffers: the groups'
        # buffers are one arena in forward order (equal-size block groups -> equally spaced gradient
        # slots), a completed group waits until ``_group_batch`` groups are complete, and their dW
        # products run as ONE strided-batched GEMM per kind before their reduce-scatters (a 1-block
        # dW product costs 110 us per TinyGPT-A block against 58 for 4 batched,
        # profiles/wgrad_batch_size_r2.txt); otherwise the products are issued immediately
        batch = bool(cfg.extra.get("batch_wgrad", os.environ.get("DLTB_BATCH_WGRAD", "1") == "1"))
        self._group_batch = int(cfg.extra.get("group_wgrad_batch", 4))
        self._arena = None
        if self.world > 1 and self._grad_resident and batch and self._group_batch > 1:
            self._arena = torch.empty(sum(g.total for g in self._order), dtype=dt, device=dev)
            off = 0
            for g in self._order:                      # forward order: block i's slots below block i+1's
                g.grad_buf = self._arena[off:off + g.total]
                g.grad = g.grad_buf
                self._zero_padding(g)
                g.grad = None
                off += g.total
        self.defer_wgrad = batch and (self.world == 1 or self._arena is not None)
        self._wq = WgradQueue()
        # world 1: nothing reads a bias / norm-weight gradient before the end of the backward (the
        # persistent slots are handed over in _finish_backward), so every block's column sums go to one
        # shared reducer flushed there -- one or two colreduce launches instead of one per block, and the
        # QKV-bias partials ride along with the next colpart launch, as in the replicated engines
        from ..ops import functional as F_
        self._red = F_.GradReducer(64, defer_plain=True) if (
            dev.type == "cuda" and self.world == 1 and os.environ.get("DLTB_SHARED_RED", "1") == "1") else None
        self._pend = []              # completed groups whose dW / reduce-scatter wait for a batch
        self.wgrad_rows_reversed = self._blocks_reversed() if self.world == 1 else False
        # world 1: every group's gathered view IS its resident shard, so W^T can be cached per
        # optimizer step like the replicated engines do (NT-form dgrad GEMMs).  Measured
        # (profiles/cache_weight_t_sharded_r2.txt): TinyGPT-A ZeRO-3 (4 micro-steps per refresh)
        # 8.04 -> 7.83 ms; FSDP with the reference's one micro-step per optimizer step 8.80 -> 8.93
        # (the refresh every step costs more than it saves; 8.66 vs 8.68 once the refresh is batched,
        # profiles/cache_weight_t_sharded_r2.txt); Mistral-7B ZeRO-3 neutral (GEMMs
        # -2.4 ms, transposes +1.5 ms per micro-step) for 14.5 GB more HBM.  So: accumulation
        # windows only, and models below 2B parameters.
        nparam = sum(u.numel for u in self.model.units())
        self._cache_wt = (self.world == 1 and self.accum > 1 and nparam < 2_000_000_000
                          and bool(cfg.extra.get("cache_weight_t", True)))
        # world > 1: the gathered W is a transient buffer, so the cache keeps its own transposed copy,
        # made the first time a unit's backward needs it in an accumulation window (the parameters
        # do not change inside a window) and reused by the window's other micro-steps -- one LDS
        # transpose per matrix per window buys the NT-form data-gradient GEMMs.  Same policy as
        # world 1 (windows, models below 2B parameters: the copy is a full model's worth of W^T)
        self._wt_multi = {} if (self.world > 1 and self.accum > 1 and nparam < 2_000_000_000
                                and dev.type == "cuda" and bool(cfg.extra.get("cache_weight_t", True))) else None
        if self.world > 1:
            # modelled wire bytes one rank sends per micro-step (ring algorithms), per group: its
            # all-gathers (once per optimizer step when everything stays gathered; once per
            # micro-step for SHARD_GRAD_OP and the FSDP root group, which stays gathered from its
            # forward through its backward; else forward + backward re-gather) and one reduce-scatter;
            # the persistent (replicated) parameters: a reduce-scatter per micro-step and an
            # all-gather per optimizer step
            e = self.shard_buf.element_size()
            frac = (self.world - 1) / self.world
            per = 0.0
            for g in groups:
                if self.keep_all:
                    ng = 1.0 / self.accum
                elif not cfg.reshard_after_forward or g.root:
                    ng = 1.0
                else:
                    ng = 2.0
                per += frac * g.total * e * (ng + 1.0)
            per += frac * p_total * e * (1.0 + 1.0 / self.accum)
            self.comm_bytes_per_step = int(per)

    def weight_t(self, unit, i, w):
        if self._wt_multi is None:
            return super().weight_t(unit, i, w)
        if w.dim() != 2 or not w.is_cuda:
            return None
        key = (unit.index, i)
        ent = self._wt_multi.get(key)
        if ent is None:
            ent = self._wt_multi[key] = [torch.empty((w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device), -1]
        if ent[1] != self.opt_steps:           # first use in this window: transpose the gathered W
            ext().transpose_into(w, ent[0])
            ent[1] = self.opt_steps
        return ent[0]

    def _slot_key(self, unit, i):
        """(buffer, element offset) of gradient slot ``i`` of ``unit`` at world size 1."""
        s = self.p_layout.slots.get((id(unit), i))
        if s is not None:
            return 0, s.offset                              # persistent parameters: p_grad
        g = self._group_of[id(unit)]
        return 1, g.owner_start + g.layout.slot(unit, i).offset     # owner space (rs_out)

    def _blocks_reversed(self) -> bool:
        """Whether consecutive blocks' matrix gradients sit at decreasing addresses (the order the
        model's layer-strided buffers must follow for batched weight gradients)."""
        blocks = getattr(self.model, "unit_blocks", None) or []
        if len(blocks) < 2:
            return False
        i = next((j for j, shp in enumerate(blocks[0].shapes) if len(shp) == 2), None)
        if i is None:
            return False
        (b0, o0), (b1, o1) = self._slot_key(blocks[0], i), self._slot_key(blocks[1], i)
        return b0 == b1 and o1 < o0

    # ------------------------------------------------------------------ gather / release
    def _launch_gather(self, g):
        if g.full is not None:
            return
        if self.world == 1 or g.total == 0:
            g.full = g.shard
            return
        free = self._gpool.get(g.total)
        # a pooled buffer's previous readers are kernels already enqueued on the compute stream: the
        # all-gather is ordered after them (RCCL / the emulated fabric wait on the issuing stream)
        g.full = free.pop() if free else torch.empty(g.total, dtype=self.shard_buf.dtype, device=self.device)
        g.work = self.comm.all_gather(g.full, g.shard, track=False)

    def _ensure(self, g):
        self._launch_gather(g)
        if g.work is not None:
            g.work.wait()
            g.work = None

    def _release(self, g):
        if self.world == 1 or g.full is None:
            return
        if g.work is not None:
            g.work.wait()
            g.work = None
        if self._pool_on:
            self._gpool.setdefault(g.total, []).append(g.full)   # views into it stay cached
        else:
            for u in g.units:         # (A/B: fresh buffers) cached views would keep the storage alive
                self._view_cache.pop((id(u), id(g.full)), None)
        g.full = None

    def _views(self, unit):
        g = self._group_of[id(unit)]
        key = (id(unit), id(g.full))
        hit = self._view_cache.get(key)
        if hit is not None and hit[0] is g.full:
            return hit[1]
        out = []
        for i in range(len(unit.params)):
            s = self.p_layout.slots.get((id(unit), i))
            if s is not None:
                out.append(self.p_flat[s.offset:s.offset + s.numel].view(s.shape))
            else:
                s = g.layout.slot(unit, i)
                out.append(g.full[s.offset:s.offset + s.numel].view(s.shape))
        self._view_cache[key] = (g.full, out)
        return out

    def _prefetch(self, g, direction):
        k = self._pos[g.gid]
        if self._prefetch_elems > 0:
            budget, kk = self._prefetch_elems, k + direction
            while 0 <= kk < len(self._order):
                nxt = self._order[kk]
                if budget < nxt.total and kk != k + direction:
                    break                            # (the next unit is always prefetched)
                budget -= nxt.total
                self._launch_gather(nxt)
                kk += direction
            return
        for j in range(1, max(0, int(self.cfg.prefetch)) + 1):
            kk = k + direction * j
            if 0 <= kk < len(self._order):
                self._launch_gather(self._order[kk])

    def _live(self) -> int:
        return sum(g.total for g in self.groups if g.full is not None)

    # ------------------------------------------------------------------ runtime interface
    def acquire(self, unit):
        g = self._group_of[id(unit)]
        tg = self._tied_group
        if tg is not None and tg.full is None and tg is not g and self._pos[g.gid] == 0:
            # the tied token table (the head unit's parameter) is read by the embedding, the first
            # forward op: at the first unit's acquire its gather goes out ahead of the embedding's own
            # and of the prefetched blocks, which it would otherwise queue behind on the collective stream
            self._launch_gather(tg)
        self._ensure(g)
        if self.cfg.extra.get("forward_prefetch", True):
            self._prefetch(g, +1)
        return self._views(unit)

    def release_forward(self, unit):
        g = self._group_of[id(unit)]
        g.fwd_left -= 1
        if g.fwd_left == 0:
            g.fwd_left = len(g.units)
            if self.model.training and self.cfg.reshard_after_forward and not g.root and not self.keep_all:
                if not (g.gid in self._reuse_keep and self._live() <= self.cfg.max_live_parameters):
                    self._release(g)

    def acquire_tied(self, unit):
        """Parameters of another unit used by a tied consumer (lm_head = wte): no prefetch, no
        forward-release accounting."""
        self._ensure(self._group_of[id(unit)])
        return self._views(unit)

    def acquire_backward(self, unit):
        g = self._group_of[id(unit)]
        self._ensure(g)
        self._prefetch(g, -1)
        return self._views(unit)

    def grad_slot(self, unit, i):
        if self._deferred:
            self._drain_all()        # the previous micro-step's reduce-scatters read these buffers
        key = (id(unit), i)
        v = self._gviews.get(key)
        if v is not None:
            g = v[1]
            if g is not None and g.grad is None:
                g.grad = g.grad_buf
            return v[0], self._mark(unit, i)
        s = self.p_layout.slots.get(key)
        if s is not None:
            self._gviews[key] = (self.p_grad[s.offset:s.offset + s.numel].view(s.shape), None)
            return self._gviews[key][0], self._mark(unit, i)
        g = self._group_of[id(unit)]
        if not self._grad_resident and self.world > 1:
            # large models: a transient full gradient buffer per group and micro-step
            if g.grad is None:
                g.grad = torch.empty(g.total, dtype=self.shard_buf.dtype, device=self.device)
                self._zero_padding(g)
            s = g.layout.slot(unit, i)
            return g.grad[s.offset:s.offset + s.numel].view(s.shape), self._mark(unit, i)
        if g.grad_buf is None:
            # ONE gradient buffer per group for the whole run (world 1: the group's owner space; world
            # > 1: the full flat buffer its reduce-scatter reads, reused every micro-step once the
            # previous reduce-scatter is waited -- no allocation, no padding fill, cached slot views);
            # its padding is zeroed once (it is reduced and enters the gradient norm; nothing writes it)
            g.grad_buf = self.rs_out[g.owner_start:g.owner_start + g.chunk] if self.world == 1 else \
                torch.empty(g.total, dtype=self.shard_buf.dtype, device=self.device)
            g.grad = g.grad_buf
            self._zero_padding(g)
        if g.grad is None:
            g.grad = g.grad_buf
        s = g.layout.slot(unit, i)
        self._gviews[key] = (g.grad_buf[s.offset:s.offset + s.numel].view(s.shape), g)
        return self._gviews[key][0], self._mark(unit, i)

    def _zero_padding(self, g):
        cur = 0
        for s in sorted(g.layout.slots.values(), key=lambda s: s.offset):
            if s.offset > cur:
                g.grad[cur:s.offset].zero_()
            cur = s.offset + s.numel
        if cur < g.total:
            g.grad[cur:g.total].zero_()

    def wgrad(self, unit, i, dy, x, dw, accumulate):
        if self.defer_wgrad:
            self._wq.add(unit, i, dy, x, dw, accumulate)
        else:
            super().wgrad(unit, i, dy, x, dw, accumulate)

    def grad_reducer(self):
        return self._red

    def grads_ready(self, unit):
        self._reported.add(id(unit))
        if self._carry is not None and self._carry[0][0] is unit:
            from ..ops import functional as F_
            tok, rows, ids = self._carry
            self._carry = None
            F_.embed_bwd(rows, ids, self.grad_slot(*tok)[0], None, False, 0.0, None, 0)
        g = self._group_of[id(unit)]
        if any(self._persistent(unit, i) for i in range(len(unit.params))):
            self._p_left -= 1
            if self._p_left == 0 and self.world > 1:
                self._reduce_persistent()
            # (world 1: the persistent slots are final only after the batched dW flush -- a 2-D
            # parameter below the persistence threshold gets its gradient from the queue -- so
            # they are handed to the owner space in _finish_backward)
        g.bwd_left -= 1
        if g.bwd_left == 0:
            if self._arena is not None and self._wq.has(g.units):
                self._pend.append(g)
                if len(self._pend) >= self._group_batch:
                    self._flush_pending()
            elif self._arena is not None:        # nothing queued (the head, the embedding): reduce now,
                self._flush_pending()            # after the groups completed before it
                self._reduce_group(g)
            else:
                self._reduce_group(g)

    def _flush_pending(self):
        """The queued dW products of the pending groups (one strided-batched GEMM per kind), then
        their reduce-scatters in completion order (the same on every rank)."""
        if not self._pend:
            return
        self._wq.flush([u for g in self._pend for u in g.units])
        pend, self._pend = self._pend, []
        for g in pend:
            self._reduce_group(g)

    def embedding_backward(self, tok, pos, dx, idx, p, seed, site):
        """As the replicated engines (parallel/replicated.py): when the token table's group (or the
        persistent block, for a small table) was already reduce-scattered this micro-step -- ZeRO-3
        reduces the head's group right after the head's backward -- the token rows and ids are
        all-gathered and scatter-added into this rank's owner shard in ``_finish_backward``."""
        unit, i = tok
        persistent = (id(unit), i) in self.p_layout.slots
        done = self._p_reduced if persistent else self._group_of[id(unit)].gid in self._reduced
        if self.world > 1 and not persistent and id(unit) in self._reported \
                and (pos is None or self._group_of[id(pos[0])] is not self._group_of[id(unit)]):
            self._model_sparse(idx.numel(), dx.shape[-1], dx.element_size(), idx.element_size(),
                               1.0 / self.accum if self._carry_on else 1.0)
        if self.world == 1 or not done:
            return super().embedding_backward(tok, pos, dx, idx, p, seed, site)
        from ..ops import functional as F_
        d = dx.shape[-1]
        dx2 = dx.reshape(-1, d)
        rows = F_.dropout(None, dx2, p, seed, site) if p > 0 else dx2.contiguous()
        if pos is not None:
            dwpe, acc_p = self.grad_slot(*pos)
            F_.embed_bwd(dx, idx, None, dwpe, acc_p, p, seed, site)
        if self._carry_on and not self._is_boundary and not persistent:
            self._carry = (tok, rows, idx.reshape(1, -1).clone())
            return
        rows_all = rows.new_empty((self.world * rows.shape[0], d))
        idx_all = idx.new_empty((self.world * idx.shape[0], idx.shape[1]))
        works = [self.comm.all_gather(rows_all, rows, track=False),
                 self.comm.all_gather(idx_all.view(-1), idx.reshape(-1).contiguous(), track=False)]
        self._sparse = (tok, persistent, rows_all, idx_all, works)

    def _apply_sparse(self):
        """Gathered token rows -> a transient dense table -> this rank's chunk of it added into
        its owner gradient (rs_out, before it is folded into the fp32 accumulator)."""
        from ..ops import functional as F_
        (unit, i), persistent, rows_all, idx_all, works = self._sparse
        self._sparse = None
        for w in works:
            w.wait()
        if persistent:
            sl, c0, chunk, base = self.p_layout.slot(unit, i), self.rank * self.p_layout.owner_numel, \
                self.p_layout.owner_numel, 0
        else:
            g = self._group_of[id(unit)]
            sl, c0, chunk, base = g.layout.slot(unit, i), self.rank * g.chunk, g.chunk, g.owner_start
        lo, hi = max(c0, sl.offset), min(c0 + chunk, sl.offset + sl.numel)
        if hi <= lo:
            return
        dense = torch.zeros(sl.shape, dtype=self.rs_out.dtype, device=self.rs_out.device)
        F_.embed_bwd(rows_all, idx_all, dense, None, False, 0.0, None, 0)
        o = base + (lo - c0)
        self.rs_out[o:o + hi - lo] += dense.view(-1)[lo - sl.offset:hi - sl.offset]

    def _reduce_group(self, g):
        if g.grad is None:
            return
        self._reduced.add(g.gid)
        if self.world > 1:
            out = self.rs_out[g.owner_start:g.owner_start + g.chunk]
            if self._tail_defer:
                self._rs_inflight.append(self.comm.reduce_scatter(out, g.grad, track=False))
            else:
                self.comm.reduce_scatter(out, g.grad, async_op=self._overlap)
            self._held_grads.append(g.grad)
        g.grad = None

    def _reduce_persistent(self):
        pc = self.p_layout.owner_numel
        if pc == 0:
            return
        if self.world > 1 and len(self._wq):
            self._wq.flush()          # a 2-D parameter below the persistence threshold is in the queue
        self._p_reduced = True
        if self.world > 1 and self._tail_defer:
            self._rs_inflight.append(self.comm.reduce_scatter(self.rs_out[:pc], self.p_grad, track=False))
        elif self.world > 1:
            self.comm.reduce_scatter(self.rs_out[:pc], self.p_grad, async_op=self._overlap)
        else:
            self.rs_out[:pc].copy_(self.p_grad)

    def release_backward(self, unit):
        g = self._group_of[id(unit)]
        if g.bwd_left == 0:
            g.bwd_left = len(g.units)
            if not self.keep_all:
                self._release(g)

    # ------------------------------------------------------------------ step lifecycle
    def _on_begin_micro(self):
        self._reduced.clear()
        self._p_reduced = False
        if self.world > 1:
            self._written.clear()    # full gradient buffers are reduced every micro-step
        # ws == 1: the group gradient buffers ARE the owner gradients; accumulate in place

    def _finish_backward(self):
        if self._red is not None:
            self._red.flush()
        self._wq.flush()
        self._flush_pending()                     # (their dW products were just issued)
        self._zero_unreported()                   # slots of units that never reported: zero
        # persistent parameters: world 1 hands p_grad to the owner space here; world > 1 reduces it
        # here unless the last unit holding some already did (grads_ready)
        if self.p_layout.owner_numel and (self.world == 1 or self._p_left > 0):
            self._reduce_persistent()
        self._p_left = self._p_pending
        for g in self.groups:                     # groups whose backward did not run fully
            self._reduce_group(g)
            g.bwd_left = len(g.units)
        self._phase("comm_wait_begin")
        self._wait_works()
        if self._tail_defer and not self._is_boundary:
            # left in flight: drained at the next backward's first gradient write (grad_slot)
            self._deferred, self._deferred_first = True, self._window_pos == 0
            self._phase("comm_wait_end")
            return
        self._deferred, self._deferred_first = True, self._window_pos == 0
        self._drain_all()
        self._phase("comm_wait_end")

    def _drain_all(self):
        """Wait for the reduce-scatters of the finished micro-step, add the exchanged token rows,
        and fold the owner chunks into the fp32 accumulator (one launch)."""
        if not self._deferred:
            return
        self._deferred = False
        for w in self._rs_inflight:
            w.wait()
        self._rs_inflight = []
        if self._sparse is not None:
            self._apply_sparse()
        self._held_grads.clear()
        if self.acc is not None:
            first = self._deferred_first
            if self.acc.is_cuda:
                ext().f32_from_bf16_(self.acc, self.rs_out, not first)
            elif first:
                self.acc.copy_(self.rs_out)
            else:
                self.acc += self.rs_out

    def _wait_param_gathers(self):
        self._drain_all()                         # (finalize / checkpoint / graph capture)

    def _optimizer_step(self, lr):
        g = self.acc if self.acc is not None else self.rs_out
        self._apply_update(g, lr, 1.0 / (self.world * self.accum), sharded=True)
        for grp in self.groups:                   # gathered copies are stale now
            self._release(grp)
        pc = self.p_layout.owner_numel
        if pc and self.world > 1:
            mine = self.p_flat[self.rank * pc:(self.rank + 1) * pc]
            self.comm.all_gather(self.p_flat, mine, async_op=False)

    def _after_param_load(self):
        self._wt_epoch = -1                       # cached transposes are stale
        if self._wt_multi:
            for ent in self._wt_multi.values():
                ent[1] = -1
        for grp in self.groups:                   # gathered copies (if any) are stale
            self._release(grp)
        pc = self.p_layout.owner_numel
        if pc and self.world > 1:
            mine = self.p_flat[self.rank * pc:(self.rank + 1) * pc]
            self.comm.all_gather(self.p_flat, mine, async_op=False)

    # ------------------------------------------------------------------ introspection
    def memory_report(self):
        e = self.shard_buf.element_size()
        return {"shard_param_bytes": self.shard_buf.numel() * e, "persistent_param_bytes": self.p_flat.numel() * e,
                "optimizer_bytes": self.opt.state_bytes, "groups": len(self.groups),
                "largest_group_mb": round(max(g.total for g in self.groups) * e / 2**20, 2),
                "keep_all_gathered": self.keep_all,
                # speed-for-HBM buffers beyond DeepSpeed / torch FSDP's footprint (models < 2B params,
                # world > 1): full-size per-group gradient buffers reused every micro-step, and the
                # per-window W^T copies of the NT-form data-gradient GEMMs.  peak_vram_gb includes them.
                "resident_grad_bytes": sum(g.grad_buf.numel() * e for g in self.groups
                                           if g.grad_buf is not None and self.world > 1),
                # transient gradient buffers still referenced after their reduce-scatter was issued
                # (freed when it is waited; with the tail deferral only resident buffers are held)
                "held_grad_bytes": sum(t.numel() * t.element_size() for t in self._held_grads
                                       if not any(t is g.grad_buf for g in self.groups)),
                "weight_t_cache_bytes": sum(t.numel() * t.element_size() for t, _ in (self._wt_multi or {}).values()),
                "gather_pool_bytes": sum(b.numel() * e for bufs in self._gpool.values() for b in bufs)}

    def full_state_dict(self):
        out = {}
        pc = self.p_layout.owner_numel
        if self.p_layout.total:
            pfull = torch.zeros(self.p_layout.total, dtype=torch.float32, device=self.device)
            pfull[self.rank * pc:(self.rank + 1) * pc] = self.opt.master[:pc]
            if self.world > 1:
                self.comm.all_reduce(pfull, async_op=False)
            for s in self.p_layout.slots.values():
                out[s.unit.names[s.index]] = pfull[s.offset:s.offset + s.numel].view(s.shape).clone()
        for g in self.groups:
            gfull = torch.zeros(g.total, dtype=torch.float32, device=self.device)
            gfull[self.rank * g.chunk:(self.rank + 1) * g.chunk] = self.opt.master[g.owner_start:g.owner_start + g.chunk]
            if self.world > 1:
                self.comm.all_reduce(gfull, async_op=False)
            for s in g.layout.slots.values():
                out[s.unit.names[s.index]] = gfull[s.offset:s.offset + s.numel].view(s.shape).clone()
        return out


class FSDPEngine(ShardedEngine):
    name = "fsdp"


class Zero3Engine(ShardedEngine):
    name = "zero3"

    def __init__(self, model, cfg, device, group=None):
        if cfg.wrap == "block":
            cfg.wrap = "unit"
        super().__init__(model, cfg, device, group)
