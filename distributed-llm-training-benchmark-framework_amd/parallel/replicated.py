"""Replicated-parameter engines: DDP and ZeRO-1/2.

Reference strategies (train_harness.py:210-223 torch DDP; :240-271 + configs/deepspeed/zero2.json
DeepSpeed ZeRO-2), re-built on ``torch.distributed`` (RCCL over xGMI on MI355X):

* Parameters: ONE flat bf16 buffer in backward order (head, block L-1 ... block 0, embedding), every
  ``nn.Parameter`` a view into it.  Gradients: a flat bf16 buffer with the same layout, written in
  place by the fused block backward (no autograd hooks, no bucket copies).
* Buckets: consecutive units grouped up to ``bucket_mb`` (xGMI-tuned default 64 MiB); the last two
  units of the backward (block 0 and the embedding) get a bucket each, so the collective that no
  compute can hide is only the embedding's.  When the last unit of a bucket finishes its backward
  the engine launches the bucket's collective immediately (async, on the process group's stream)
  so communication overlaps the remaining backward.
* DDP (``zero_stage=0``): SUM all-reduce per bucket; the 1/world average is folded into the fused
  AdamW's gradient scale.  fp32 master / Adam moments for the whole model on every rank.
* ZeRO-2: reduce-scatter per bucket, every micro-step, into this rank's chunk; chunks accumulate
  in an fp32 owner buffer across the ``grad_accum`` window; at the boundary: global grad-norm
  (one float all-reduce), clipping coefficient on device, fused AdamW on the owner shard writing
  the bf16 chunk in place, then an in-place all-gather per bucket re-replicates the parameters.
* ZeRO-1: like ZeRO-2 but gradients accumulate unsharded and are reduce-scattered at the boundary.
  This is also ZeRO-2 with ``--grad-reduce window`` (reported as ``zero1``; bench.py's default is
  the per-micro-step ZeRO-2 reduction at every world size).  xGMI links are
  point-to-point, so a ring reduce-scatter is per-link bound, and one reduce-scatter per window
  moves 1/grad_accum of the per-micro-step traffic.  The flat gradient buffer is full-size in both
  modes, so HBM use is the same.  Micro-steps without a collective leave every dW product queued
  for one batched flush, as at world size 1.  Precision differs: window mode sums the micro-steps
  in the bf16 flat buffer (the GEMMs accumulate with beta = 1) before one bf16 reduce-scatter,
  while micro mode adds each reduce-scattered chunk into an fp32 owner buffer.
  tests/test_multirank_gpu.py bounds both against the world-1 run of the same global batch.
* DDP ``grad_comm_dtype="fp32"``: each bucket is widened to fp32 right before its all-reduce (the
  reference's torch DDP reduces fp32 gradients), AdamW reads the fp32 sum.
"""
import os

import torch

from ..ops import functional as F_
from ..ops._ext import ext
from ..optim.adamw import FlatAdamW
from .ds_config import check_bucket_caps
from .engine import Engine
from .flat import ALIGN, owner_segments, plan_layout
from .wgrad import WgradQueue


def _dtype_name(dt):
    return {torch.bfloat16: "bf16", torch.float16: "fp16", torch.float32: "fp32"}.get(dt, str(dt))


def grad_comm_dtype(stage: int, world: int, want_f32: bool, dt) -> str:
    """The dtype the replicated engines' gradient collectives carry.  DDP (stage 0) widens each bucket to
    fp32 on request (the reference's torch DDP reduces fp32 gradients); the sharded-optimizer DDP and
    ZeRO-1/2 reduce-scatter the flat compute-dtype buffer, so an fp32 request is overridden there (half the
    wire bytes of the fp32 all-reduce row; fp16 sums stay loss-scaled) and this is what results report."""
    if want_f32 and stage == 0:
        return "fp32"
    return _dtype_name(dt)


class ReplicatedEngine(Engine):
    name = "ddp"
    grad_write_ahead = True      # every gradient slot is a view of the flat buffer from the start

    def _setup(self):
        cfg, model = self.cfg, self.model
        self.stage = int(cfg.zero_stage)
        units = list(reversed(model.units()))
        elem = torch.tensor([], dtype=self.compute_dtype).element_size()
        bucket_elems = int(cfg.bucket_mb * (1 << 20) / elem) if cfg.bucket_mb > 0 else 0
        # DeepSpeed's reduce_bucket_size / allgather_bucket_size (elements): hard upper bounds of one
        # reduce-scatter / one parameter all-gather; both run per bucket here (parallel/ds_config.py)
        caps = [int(c) for c in (cfg.extra.get("reduce_bucket_elems"), cfg.extra.get("allgather_bucket_elems")) if c]
        ds_cap = min(caps) if caps else 0
        if ds_cap:
            check_bucket_caps(cfg, [u.numel for u in units], cfg.strategy)
            bucket_elems = min(bucket_elems, ds_cap) if bucket_elems else ds_cap
        # weight gradients queued and issued as strided-batched GEMMs (parallel/wgrad.py): world 1
        # flushes once per backward, world > 1 per bucket right before its collective
        self.defer_wgrad = bool(cfg.extra.get("batch_wgrad", os.environ.get("DLTB_BATCH_WGRAD", "1") == "1"))
        # World > 1: a bucket's dW products are one batched GEMM per kind, so the bucket's block count
        # is the batch size.  hipBLASLt's batched kernels run 4 or 8 TinyGPT-A blocks at 52-58 us per
        # block but 2-3 blocks at 75-80 and 6 at 68 (profiles/wgrad_batch_size_r2.txt): buckets are
        # rounded up to a multiple of 4 of the model's repeated unit (64 MiB -> 4 blocks, 101 MB).
        # Only the embedding (the unit that finishes last) then keeps a bucket of its own: a solo block 0
        # would be a 1-block batch (110 us) and leave 3 blocks for the group before it.
        mult = int(cfg.extra.get("bucket_unit_multiple", 4))
        solo_tail, solo_head = 2, 0
        if self.world > 1 and self.defer_wgrad and bucket_elems > 0 and mult > 1:
            sizes = sorted(u.numel for u in units)
            grp = mult * sizes[len(sizes) // 2]          # the repeated unit: a transformer block
            bucket_elems = -(-bucket_elems // grp) * grp
            solo_tail = 1
            # the head (the tied 65.5 MB token table at TinyGPT-A) is a bucket of its own: otherwise it
            # shares the first bucket with two blocks and the blocks' dW batches come out 2/4/4/4/2
            # (a 2-block batch costs 75 us per block against 58 for 4, profiles/wgrad_batch_size_r2.txt)
            solo_head = int(cfg.extra.get("solo_head_units", 1))
            if self._ddp_pipe_wanted() or cfg.extra.get("shard_optimizer"):
                # DDP with the optimizer pipelined per bucket: the last bucket's all-reduce is the exposed
                # tail, so blocks 0 and 1 get buckets of their own (1-block dW batches, +~0.1 ms) and the
                # tail shrinks from a 4-block bucket to one block: emulated ddp_bf16 N = 8 10.09 -> 9.97 ms
                # (profiles/emulated_ddp_pipeline_r5.txt).  DDP + sharded optimizer: the last bucket's
                # reduce-scatter is the exposed tail the same way: 9.46 -> 9.36 ms (emulated_ddp_zero1_r5.txt)
                solo_tail = 3
        # the first bucket(s) after the head: twice the size (fewer collectives early in the backward,
        # while compute hides them; the buckets at its end -- the first parameter all-gathers of the
        # next forward -- keep the usual size): emulated ZeRO-2 N = 8 -0.7 %, N = 2 -0.5 %
        # (profiles/emulated_ab_early_bucket_r4.txt).  cfg.extra["early_buckets"] (count; 0 = off).
        # (ZeRO-2 only: DDP and ZeRO-1 wait for every bucket before the optimizer of the same
        # micro-step / window, and there a later first collective only lengthens the exposed tail --
        # DDP fp16 with fp32 all-reduce N = 8 63.6 -> 60.3 %, profiles/emulated_ab_early_bucket_r4.txt)
        early = int(cfg.extra.get("early_buckets", 1)) \
            if (self.world > 1 and bucket_elems > 0 and self.stage == 2) else 0
        shard = self.stage >= 1
        self.layout = L = plan_layout(units, self.world, bucket_elems, ALIGN, shard=shard,
                                      solo_tail=int(cfg.extra.get("solo_tail_units",
                                                                  solo_tail)),
                                      bucket_max=ds_cap, solo_head=solo_head,
                                      early_elems=2 * bucket_elems
                                      if early else 0, early_count=early)
        # DeepSpeed switches (zero2.json; all true there and by default): overlap_comm false waits
        # for every collective where it is issued; reduce_scatter false all-reduces each bucket and
        # keeps this rank's chunk; allgather_partitions false re-replicates the updated parameters
        # by one broadcast per owner chunk instead of an all-gather
        self._overlap = bool(cfg.extra.get("overlap_comm", True))
        self._use_rs = bool(cfg.extra.get("reduce_scatter", True))
        self._use_ag = bool(cfg.extra.get("allgather_partitions", True))
        dev, dt = self.device, self.compute_dtype
        master_full = torch.zeros(L.total, dtype=torch.float32, device=dev)
        for s in L.slots.values():
            p = s.unit.params[s.index]
            master_full[s.offset:s.offset + s.numel] = p.detach().reshape(-1).to(device=dev, dtype=torch.float32)
        self.flat_param = master_full.to(dt)
        self.flat_grad = torch.zeros(L.total, dtype=dt, device=dev)
        # DDP all-reduce dtype.  bf16: the flat gradient buffer itself is reduced.  fp32: what the
        # reference's torch DDP reduces (fp32 grads under fp16 autocast, train_harness.py:217-222):
        # each bucket is widened into an fp32 buffer right before its all-reduce, summed over the
        # ranks in fp32, and AdamW reads the fp32 sum (2x the wire bytes, no bf16 rounding per hop)
        self.comm_f32 = None
        want_f32 = cfg.extra.get("grad_comm_dtype") == "fp32"
        self.grad_comm_dtype = grad_comm_dtype(self.stage, self.world, want_f32, dt)
        if self.grad_comm_dtype == "fp32" and self.world > 1 and dt != torch.float32:
            # (fp16 grads are S-scaled: their fp32 sum cannot overflow)
            self.comm_f32 = torch.zeros(L.total, dtype=torch.float32, device=dev)
        elif want_f32 and self.world > 1 and dt != torch.float32:
            import warnings
            warnings.warn(f"grad_comm_dtype fp32 is not implemented for ZeRO stage {self.stage}: gradients are "
                          f"reduced in {self.grad_comm_dtype}")
        for s in L.slots.values():
            p = s.unit.params[s.index]
            p.data = self.flat_param[s.offset:s.offset + s.numel].view(s.shape)
            p.grad = None
        if shard:
            segs = owner_segments(L, self.rank)
            master = torch.empty(L.owner_numel, dtype=torch.float32, device=dev)
            opt_segs = []
            for ostart, ln, fstart in segs:
                master[ostart:ostart + ln] = master_full[fstart:fstart + ln]
                opt_segs.append((ostart, ln, self.flat_param[fstart:fstart + ln]))
            self.rs_out = torch.zeros(L.owner_numel, dtype=dt, device=dev) if self.world > 1 else None
            # ws == 1: nothing to reduce, gradients accumulate in place in the bf16 flat buffer
            self.acc = torch.zeros(L.owner_numel, dtype=torch.float32, device=dev) \
                if (self.stage == 2 and self.accum > 1 and self.world > 1) else None
        else:
            master = master_full
            opt_segs = [(0, L.total, self.flat_param)]
            self.rs_out = self.acc = None
        # DDP at world > 1 without a loss scaler and without clipping (the reference's DDP in bf16:
        # train_harness.py:210-223 + :328-329 -- AdamW on every micro-step, no clip, no schedule):
        # the optimizer is pipelined under the all-reduce tail.  Each bucket is one AdamW segment;
        # the update waits for its OWN bucket's all-reduce only (a device-side stream wait), so the
        # buckets reduced early in the backward are updated while the last ones are still on the
        # wire and only the last bucket's rows stay exposed behind the comm tail.  (fp16 with dynamic
        # loss scaling needs the global inf check over every bucket first, and clipping the global
        # norm: both keep the whole-model update after the last wait.)
        self._ddp_pipe = self._ddp_pipe_wanted()
        self._ar_works = {}      # bucket -> its all-reduce (untracked) while the pipeline is on
        # (a bucket's update on a side stream right behind its all-reduce, under the rest of the backward,
        # measured slower -- emulated ddp_bf16 N = 8 10.07 -> 10.25 ms, profiles/ddp_early_update_ab_r5.txt --
        # and was removed in round 6)
        if self._ddp_pipe:
            g_full = self.comm_f32 if self.comm_f32 is not None else self.flat_grad
            opt_segs = [(bk.start, bk.end - bk.start, self.flat_param[bk.start:bk.end]) for bk in L.buckets]
            assert sum(x[1] for x in opt_segs) == g_full.numel() == L.total
        del master_full
        self.opt = FlatAdamW(master, opt_segs, cfg.lr, cfg.betas, cfg.eps, cfg.weight_decay)
        self._ag_pending = {}    # bucket -> async all-gather of updated parameters (deferred step)
        self._defer_opt = (self.stage >= 1 and self.world > 1 and self._overlap and
                           bool(cfg.extra.get("defer_opt", os.environ.get("DLTB_DEFER_OPT", "1") == "1")))
        self._cache_wt = True    # cached W^T of every matrix for the NT-form dgrad GEMMs (engine.py)
        self._pending = [len(b.units) for b in L.buckets]
        self._bucket_of = L.unit_bucket
        self._wq = WgradQueue()
        # Window-wide weight gradients: where no collective reads a gradient before the window ends
        # (world 1, or the window-reduced ZeRO-1 / DDP paths), the model keeps every micro-step's
        # dW operands and the window's dW = sum_m dY_m^T X_m runs at its last micro-step as one
        # batched product over accum x 2048 tokens (K = 8192 at TinyGPT-A): the batched GEMMs run at
        # 0.93-1.05 PFLOP/s instead of 0.79-0.93 at K = 2048, and the sum is accumulated in fp32
        # inside the GEMM instead of being rounded to bf16 after every micro-step.
        self._window_wgrad = (self.defer_wgrad and self.accum > 1 and (self.world == 1 or self.stage != 2)
                              and bool(cfg.extra.get("window_wgrad", os.environ.get("DLTB_WINDOW_WGRAD", "1") == "1")))
        # world 1: nothing reads a gradient slot before the backward ends, so the bias / norm-weight
        # column sums of ALL blocks are reduced by one or two colreduce_multi launches at its end
        # instead of one launch per block, and the QKV-bias partials of block i ride along with
        # block i-1's dropout colpart launch instead of a launch of their own
        # (world > 1: the shared reducer is flushed right before each bucket's collective, so one
        # or two colreduce launches serve a 4-block bucket instead of one per block)
        self._red = F_.GradReducer(64, defer_plain=True) if (
            dev.type == "cuda" and (self.world == 1 or os.environ.get("DLTB_SHARED_RED", "1") == "1")) else None
        # buckets are reduced strictly in bucket order (torch DDP's Reducer does the same): every
        # rank must issue its collectives in one sequence, and a unit that does not report on some
        # rank (an unused parameter) would otherwise reorder that rank's sequence
        self._next = 0
        # ZeRO-2 per-micro-step reduce-scatter, world > 1: a micro-step that does not end its window
        # leaves its buckets' reduce-scatters in flight instead of waiting at the end of backward; the
        # next backward waits for bucket b (and folds its chunk into the fp32 accumulator) only when it
        # first writes that bucket's gradient slots, so the tail buckets (block 0, the 70 MB
        # embedding) reduce under the next forward instead of after the backward.  The window's
        # last micro-step drains everything before the optimizer.
        self._tail_defer = (self.stage == 2 and self.world > 1 and self.acc is not None and
                            self._overlap and self._use_rs and bool(cfg.extra.get("defer_tail_reduce", True)))
        self._rs_inflight = {}   # bucket -> (work, first micro-step of its window)
        self._sparse = None      # (token slot, gathered rows, gathered ids, works) of this backward
        # ZeRO-2 per-micro-step reduce-scatter, inside a window: the token rows of micro-step m's
        # embedding backward are not exchanged; they are scatter-added into micro-step m+1's dense
        # token-table gradient (after the head's dW, before its bucket's reduce-scatter).  The
        # window's sum is unchanged (the reduce-scatter is linear); only the window's last micro-step
        # exchanges its rows.  2048 rows scattered locally instead of an all-gather of world x 2048
        # rows + ids and a sort-path scatter every micro-step.
        self._carry_on = (self._tail_defer and
                          bool(cfg.extra.get("carry_token_rows", True)))
        self._carry = None       # (token slot, rows, ids) waiting for the next micro-step's head
        nbytes = L.total * (4 if self.comm_f32 is not None else elem)
        if self.world > 1:
            # modelled wire bytes one rank sends per micro-step (ring algorithms): DDP one all-reduce
            # per optimizer step; ZeRO-2 a reduce-scatter every micro-step; ZeRO-1 one per window;
            # ZeRO-1/2 also one parameter all-gather per window
            frac = (self.world - 1) / self.world
            if self.stage == 0:
                per = 2 * frac * nbytes / self.accum
            else:
                per = frac * nbytes * (1.0 if self.stage == 2 else 1.0 / self.accum) + frac * nbytes / self.accum
            self.comm_bytes_per_step = int(per)

    # ------------------------------------------------------------------ runtime interface
    def acquire(self, unit):
        if self._ag_pending:
            b = self._bucket_of.get(id(unit))
            w = self._ag_pending.pop(b, None)
            if w is not None:
                w.wait()
        return [p.detach() for p in unit.params]

    acquire_backward = acquire

    def acquire_tied(self, unit):
        return self.acquire(unit)

    def grad_slot(self, unit, i):
        if self._rs_inflight:
            b = self._bucket_of.get(id(unit))
            if b in self._rs_inflight:
                self._drain_all()               # the previous micro-step's reduce-scatters read these slots
        s = self.layout.slot(unit, i)
        return self.flat_grad[s.offset:s.offset + s.numel].view(s.shape), self._mark(unit, i)

    def _reduce_now(self) -> bool:
        if self.world == 1:
            return False
        if self.stage == 2:
            return True
        return self._is_boundary

    def wgrad(self, unit, i, dy, x, dw, accumulate):
        if self.defer_wgrad:
            self._wq.add(unit, i, dy, x, dw, accumulate)
        else:
            super().wgrad(unit, i, dy, x, dw, accumulate)

    def wgrad_window(self):
        return (self._window_pos, self.accum) if self._window_wgrad else None

    def grad_reducer(self):
        return self._red

    def grads_ready(self, unit):
        self._reported.add(id(unit))
        if self._carry is not None and self._carry[0][0] is unit:
            self._apply_carry()
        b = self._bucket_of.get(id(unit))
        if b is None:
            return
        self._pending[b] -= 1
        if self._pending[b] == 0 and self._reduce_now():
            while self._next < len(self._pending) and self._pending[self._next] == 0:
                nb = self._next
                self._wq.flush(self.layout.buckets[nb].units)   # this bucket's dW, then its collective
                if self._red is not None:
                    self._red.flush()                           # ... and its column sums
                self._launch(nb)
                self._next += 1
        # (micro-steps without a collective -- inside a ZeRO-1 / window-reduced accumulation
        # window -- leave every dW queued for the single batched flush at the end of the backward)

    def embedding_backward(self, tok, pos, dx, idx, p, seed, site):
        """The tied token table's bucket is reduced right after the head's backward (it sits in the
        first bucket); when that collective already ran this micro-step, the embedding's token rows
        are exchanged instead: this rank's rows after the dropout backward and its token ids are
        all-gathered (world x 2048 x 1024 bf16 = 4 MB per rank at TinyGPT-A, instead of the 65.5 MB
        dense table reduced after the last backward op) and every rank scatter-adds all of them
        into the reduced gradient in ``_finish_backward`` (``_apply_sparse``)."""
        b = self._bucket_of.get(id(tok[0]))
        # the exchange happens only when the token table's unit is not the one running this backward
        # (the tied-in-head table: its unit reported first); an untied table (Mistral) is reduced
        # densely with its own bucket, after this backward
        if self.world > 1 and b is not None and id(tok[0]) in self._reported \
                and (pos is None or self._bucket_of.get(id(pos[0])) != b):
            # structurally exchanged: every micro-step (ZeRO-2), at each window boundary (ZeRO-1, DDP
            # windows, and ZeRO-2 carrying the rows of the window's other micro-steps)
            self._model_sparse(idx.numel(), dx.shape[-1], dx.element_size(), idx.element_size(),
                               1.0 if (self.stage == 2 and not self._carry_on) else 1.0 / self.accum)
        if self.world == 1 or b is None or not (self._reduce_now() and b < self._next):
            return super().embedding_backward(tok, pos, dx, idx, p, seed, site)
        d = dx.shape[-1]
        dx2 = dx.reshape(-1, d)
        rows = F_.dropout(None, dx2, p, seed, site) if p > 0 else dx2.contiguous()
        if pos is not None:
            dwpe, acc_p = self.grad_slot(*pos)
            F_.embed_bwd(dx, idx, None, dwpe, acc_p, p, seed, site)
        if self._carry_on and not self._is_boundary:
            self._carry = (tok, rows, idx.reshape(1, -1).clone())
            return
        rows_all = rows.new_empty((self.world * rows.shape[0], d))
        idx_all = idx.new_empty((self.world * idx.shape[0], idx.shape[1]))
        works = [self.comm.all_gather(rows_all, rows, track=False),
                 self.comm.all_gather(idx_all.view(-1), idx.reshape(-1).contiguous(), track=False)]
        self._sparse = (tok, rows_all, idx_all, works)

    def _apply_carry(self):
        """The previous micro-step's token rows, scatter-added into this micro-step's dense token-table
        gradient (written by the head's dW GEMM, already queued on the stream)."""
        tok, rows, ids = self._carry
        self._carry = None
        s = self.layout.slot(*tok)
        F_.embed_bwd(rows, ids, self.flat_grad[s.offset:s.offset + s.numel].view(s.shape), None, False, 0.0, None, 0)

    def _apply_sparse(self):
        """Scatter-add the gathered token rows into the reduced token-table gradient: DDP into the
        all-reduced buffer (bf16 in place, or through a bf16 scratch into the fp32 one), ZeRO-1/2
        into this rank's owner chunk (the slot's range of the flat gradient is free again once its
        reduce-scatter has read it, and serves as the scratch).  Every rank adds the same rows in
        the same order: the result is identical on all ranks and deterministic."""
        tok, rows_all, idx_all, works = self._sparse
        self._sparse = None
        for w in works:
            w.wait()
        s = self.layout.slot(*tok)
        region = self.flat_grad[s.offset:s.offset + s.numel]
        if self.stage == 0 and self.comm_f32 is None:
            F_.embed_bwd(rows_all, idx_all, region.view(s.shape), None, False, 0.0, None, 0)
            return
        region.zero_()
        F_.embed_bwd(rows_all, idx_all, region.view(s.shape), None, False, 0.0, None, 0)
        if self.stage == 0:
            dst = self.comm_f32[s.offset:s.offset + s.numel]
            if dst.is_cuda:
                ext().f32_from_bf16_(dst, region, True)
            else:
                dst += region.float()
            return
        b = self._bucket_of[id(tok[0])]
        bk = self.layout.buckets[b]
        c0 = bk.start + self.rank * bk.chunk
        lo, hi = max(c0, s.offset), min(c0 + bk.chunk, s.offset + s.numel)
        if hi <= lo:
            return
        src = self.flat_grad[lo:hi]
        o = bk.owner_start + (lo - c0)
        if self._tail_defer:                      # acc already holds this micro-step's chunk
            dst = self.acc[o:o + hi - lo]
            if dst.is_cuda:
                ext().f32_from_bf16_(dst, src, True)
            else:
                dst += src.float()
        else:                                     # rs_out, before it is folded into acc (if any)
            self.rs_out[o:o + hi - lo] += src

    def _launch(self, b):
        if b in self._rs_inflight:
            self._drain_all()         # the previous micro-step's reduce-scatters (this bucket's among them)
        bk = self.layout.buckets[b]
        g = self.flat_grad[bk.start:bk.end]
        sync = not self._overlap
        if self.stage == 0:
            if self.comm_f32 is not None:
                c = self.comm_f32[bk.start:bk.end]
                if c.is_cuda:
                    ext().f32_from_bf16_(c, g, False)
                else:
                    c.copy_(g)
                g = c
            if self._ddp_pipe:       # waited by its own AdamW segment (or the token rows), not wait_all
                self._ar_works[b] = self.comm.all_reduce(g, async_op=True, track=False)
            else:
                self.comm.all_reduce(g, async_op=not sync)
        elif not self._use_rs:
            # reduce_scatter: false -- DeepSpeed all-reduces the bucket and keeps its own partition
            self.comm.all_reduce(g, async_op=False)
            self.rs_out[bk.owner_start:bk.owner_start + bk.chunk].copy_(g[self.rank * bk.chunk:(self.rank + 1) * bk.chunk])
        elif self._tail_defer:
            w = self.comm.reduce_scatter(self.rs_out[bk.owner_start:bk.owner_start + bk.chunk], g, track=False)
            self._rs_inflight[b] = (w, self._window_pos == 0)
        else:
            self.comm.reduce_scatter(self.rs_out[bk.owner_start:bk.owner_start + bk.chunk], g, async_op=not sync)

    def _drain_bucket(self, b):
        """Wait for bucket ``b``'s reduce-scatter and add its chunk into the fp32 accumulator (then
        the token rows exchanged for the tied table, when this is its bucket)."""
        w, first = self._rs_inflight.pop(b)
        w.wait()
        bk = self.layout.buckets[b]
        a = self.acc[bk.owner_start:bk.owner_start + bk.chunk]
        r = self.rs_out[bk.owner_start:bk.owner_start + bk.chunk]
        if a.is_cuda:
            ext().f32_from_bf16_(a, r, not first)
        elif first:
            a.copy_(r)
        else:
            a += r
        if self._sparse is not None and self._bucket_of[id(self._sparse[0][0])] == b:
            self._apply_sparse()

    def _drain_all(self):
        """Wait for every in-flight reduce-scatter and fold the chunks into the fp32 accumulator.  When
        the whole owner space is in flight (the normal case: every bucket of the previous micro-step,
        drained at this backward's first gradient write, a forward later), the fold is ONE launch
        over the owner space instead of one per bucket."""
        if not self._rs_inflight:
            return
        firsts = {f for _, f in self._rs_inflight.values()}
        if len(self._rs_inflight) == len(self.layout.buckets) and len(firsts) == 1:
            for w, _ in self._rs_inflight.values():
                w.wait()
            self._rs_inflight.clear()
            first = firsts.pop()
            if self.acc.is_cuda:
                ext().f32_from_bf16_(self.acc, self.rs_out, not first)
            elif first:
                self.acc.copy_(self.rs_out)
            else:
                self.acc += self.rs_out
            if self._sparse is not None:
                self._apply_sparse()
            return
        for b in sorted(self._rs_inflight):
            self._drain_bucket(b)

    # ------------------------------------------------------------------ step lifecycle
    def _on_begin_micro(self):
        if self.stage == 2 and self.world > 1:
            self._written.clear()         # the full gradient buffer is reduced every micro-step

    def _finish_backward(self):
        if self._red is not None:
            self._red.flush()
        self._wq.flush()                                        # world 1: every block in one batch
        self._zero_unreported()
        if self._reduce_now():
            for b in range(self._next, len(self._pending)):   # buckets holding units that never reported
                self._launch(b)
        self._phase("comm_wait_begin")
        self._wait_works()
        if self._tail_defer and self._is_boundary:
            self._drain_all()                   # the optimizer reads the window's full sum next (one
            #                                     fold launch; the token rows are applied in it)
        # (DDP pipeline at the optimizer boundary: the token rows' all-gathers were issued by the
        # embedding backward, i.e. behind every bucket's all-reduce on the comm stream -- waiting for
        # them here exposed the whole all-reduce tail.  _update applies them right before the tied
        # table's own AdamW segment, which it runs last.)
        pipe_rows = self._ddp_pipe and self._is_boundary
        if self._sparse is not None and not pipe_rows and \
                not (self._tail_defer and not self._is_boundary):
            b = self._bucket_of[id(self._sparse[0][0])]
            if b in self._rs_inflight:
                self._drain_bucket(b)          # the token table's chunk, then its sparse rows
            self._wait_allreduce(b)            # (DDP pipeline: the rows add into the reduced bucket)
            if self._sparse is not None:
                self._apply_sparse()
        # (ZeRO-2 inside a window: the row all-gathers stay in flight with the table's reduce-
        # scatter and are applied when that bucket is drained, under the next forward)
        self._phase("comm_wait_end")
        self._pending = [len(b.units) for b in self.layout.buckets]
        self._next = 0
        if self.stage == 2 and self.acc is not None and not self._tail_defer:
            src = self.rs_out if self.world > 1 else self.flat_grad
            first = self._window_pos == 0
            if self.acc.is_cuda:
                ext().f32_from_bf16_(self.acc, src, not first)
            elif first:
                self.acc.copy_(src)
            else:
                self.acc += src

    def _owner_grad(self):
        if self.stage == 0:
            return self.comm_f32 if self.comm_f32 is not None else self.flat_grad
        if self.acc is not None and self.stage == 2:
            return self.acc
        return self.rs_out if self.world > 1 else self.flat_grad

    def _ddp_pipe_wanted(self):
        cfg = self.cfg
        return (int(cfg.zero_stage) == 0 and self.world > 1 and bool(cfg.extra.get("overlap_comm", True))
                and self.scaler is None and not cfg.grad_clip > 0 and not cfg.extra.get("track_grad_norm", False)
                and bool(cfg.extra.get("ddp_opt_pipeline", True)))

    def _tied_bucket(self):
        tu = getattr(self.model, "tok_slot", (None,))[0]
        return self._bucket_of.get(id(tu)) if tu is not None else None

    def _wait_allreduce(self, b):
        w = self._ar_works.pop(b, None)
        if w is not None:
            w.wait()

    def _update(self, lr):
        if self._ddp_pipe:
            # per bucket, in all-reduce issue order: wait for that bucket's sum, then its AdamW rows;
            # the tied token table's bucket goes last: its gathered token rows (issued after every
            # all-reduce) are scatter-added into it first
            g = self._owner_grad()
            gscale = self._clip_coef([g], 1.0 / (self.world * self.accum), False)   # (no clip: a fill)
            self.opt.prepare(lr)
            order = list(range(len(self.layout.buckets)))
            bt = self._bucket_of[id(self._sparse[0][0])] if self._sparse is not None else None
            if bt is not None:
                order.remove(bt)
                order.append(bt)
            for b in order:
                self._wait_allreduce(b)
                if b == bt:
                    self._apply_sparse()
                self.opt.launch_segment(b, g, gscale)
            return
        self._apply_update(self._owner_grad(), lr, 1.0 / (self.world * self.accum), sharded=self.stage >= 1)

    def _deferred_optimizer_step(self, lr):
        g = self._owner_grad()
        if (self._use_ag and self.scaler is None and g.is_cuda and not self.opt.sub_group
                and bool(self.cfg.extra.get("opt_pipeline", True))):
            # clip coefficient once, then per bucket (gather order): its AdamW rows, then its
            # all-gather -- the all-gather of the tied table's bucket starts after that bucket's
            # update instead of after the whole shard's, and every later one earlier by the rest
            gscale = self._clip_coef([g], 1.0 / (self.world * self.accum), True)
            self.opt.prepare(lr)
            seg = {b: i for i, b in enumerate(i for i, bk in enumerate(self.layout.buckets) if bk.chunk > 0)}
            for b in self._gather_order():
                if b in seg:
                    self.opt.launch_segment(seg[b], g, gscale)
                self._issue_gather(b)
            return
        self._update(lr)
        if not self._use_ag:
            self._regather(async_op=False)
            return
        for b in self._gather_order():
            self._issue_gather(b)

    def _issue_gather(self, b):
        bk = self.layout.buckets[b]
        full = self.flat_param[bk.start:bk.end]
        mine = full[self.rank * bk.chunk:(self.rank + 1) * bk.chunk]
        self._ag_pending[b] = self.comm.all_gather(full, mine, track=False)

    def _gather_order(self):
        """Bucket order of the deferred parameter all-gathers: forward order, except that the bucket of
        the tied token table (the head unit's parameter, which the embedding reads first of all) leads.
        In plain forward order it came last, and the all-gathers run in issue order on one stream, so
        the embedding's forward waited for every bucket's all-gather of the window."""
        order = list(reversed(range(len(self.layout.buckets))))
        tu = getattr(self.model, "tok_slot", (None,))[0]
        bt = self._bucket_of.get(id(tu)) if tu is not None else None
        if bt is not None and bt in order:
            order.remove(bt)
            order.insert(0, bt)
        return order

    def _regather(self, async_op=True):
        """Re-replicate the updated parameter chunks: an all-gather per bucket, or (DeepSpeed's
        ``allgather_partitions: false``) one broadcast per owner chunk."""
        for bk in self.layout.buckets:
            full = self.flat_param[bk.start:bk.end]
            if self._use_ag:
                mine = full[self.rank * bk.chunk:(self.rank + 1) * bk.chunk]
                self.comm.all_gather(full, mine, async_op=async_op)
            else:
                for r in range(self.world):
                    self.comm.broadcast(full[r * bk.chunk:(r + 1) * bk.chunk], src=self.comm.global_rank(r))

    def _wait_param_gathers(self):
        for b in list(self._ar_works):
            self._wait_allreduce(b)
        self._drain_all()
        for w in self._ag_pending.values():
            w.wait()
        self._ag_pending.clear()

    def _optimizer_step(self, lr):
        # (ZeRO-1 reduce-scattered its window-accumulated gradients during the boundary backward)
        self._update(lr)
        if self.stage >= 1 and self.world > 1:
            self._regather()
            self._wait_works()

    def _after_param_load(self):
        self._wt_epoch = -1                  # cached transposes are stale
        if self.stage >= 1 and self.world > 1:   # other ranks' owner parts
            self._regather(async_op=False)

    # ------------------------------------------------------------------ introspection
    def memory_report(self):
        e = self.flat_param.element_size()
        return {"param_bytes": self.flat_param.numel() * e, "grad_bytes": self.flat_grad.numel() * e,
                "optimizer_bytes": self.opt.state_bytes,
                "buckets": len(self.layout.buckets),
                "bucket_mb": [round(b.numel * e / 2**20, 2) for b in self.layout.buckets]}

    def full_state_dict(self):
        self.finalize()
        out = {}
        if self.stage >= 1 and self.world > 1:
            full = torch.zeros(self.layout.total, dtype=torch.float32, device=self.device)
            for ostart, ln, fstart in owner_segments(self.layout, self.rank):
                full[fstart:fstart + ln] = self.opt.master[ostart:ostart + ln]
            self.comm.all_reduce(full, async_op=False)
        elif self.stage >= 1:
            full = torch.zeros(self.layout.total, dtype=torch.float32, device=self.device)
            for ostart, ln, fstart in owner_segments(self.layout, self.rank):
                full[fstart:fstart + ln] = self.opt.master[ostart:ostart + ln]
        else:
            full = self.opt.master
        for s in self.layout.slots.values():
            out[s.unit.names[s.index]] = full[s.offset:s.offset + s.numel].view(s.shape).clone()
        return out


class DDPEngine(ReplicatedEngine):
    """torch DDP semantics (reference ``wrap_model`` ddp).  ``cfg.extra["shard_optimizer"]``
    (``--ddp-shard-optimizer``, torch's DDP + ZeroRedundancyOptimizer) keeps the step's math --
    every rank ends the step with the same full parameters, same per-element AdamW -- but shards the
    optimizer: the gradients are reduce-scattered instead of all-reduced (the same wire bytes), each
    rank updates its 1/N of the master weights and moments, and the updated bf16 parameters are
    all-gathered per bucket under the next forward (the ZeRO-1 path of this engine at grad_accum 1).
    The replicated full-model AdamW of plain DDP (1.2 ms per micro-step at TinyGPT-A, HBM-bound)
    shrinks by N, and optimizer state memory by N."""
    name = "ddp"

    def __init__(self, model, cfg, device, group=None):
        cfg.zero_stage = 1 if cfg.extra.get("shard_optimizer") else 0
        super().__init__(model, cfg, device, group)


class Zero2Engine(ReplicatedEngine):
    name = "zero2"

    def __init__(self, model, cfg, device, group=None):
        if cfg.zero_stage not in (1, 2):
            cfg.zero_stage = 2
        super().__init__(model, cfg, device, group)
