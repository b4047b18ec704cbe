"""Fused AdamW over a flat fp32 owner space.

Replaces ``torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01)``
(train_harness.py:328-329) and DeepSpeed's FusedAdam (``"optimizer": {"type": "AdamW"}`` in
configs/deepspeed/zero{2,3}.json).  The rank's optimizer state — fp32 master weights, exp_avg,
exp_avg_sq — lives in three flat tensors; one HIP launch (csrc/adamw.hip) reads master/m/v/grad
once and writes master/m/v plus the bf16 compute copy of every parameter straight into its
destination (the replicated flat parameter buffer, or this rank's parameter shard).
"""
import math
from typing import List, Sequence, Tuple

import torch

from ..ops import ref
from ..ops._ext import ext


class FlatAdamW:
    def __init__(self, master: torch.Tensor, segments: Sequence[Tuple[int, int, torch.Tensor]],
                 lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, sub_group: int = 0):
        """``segments``: (owner_start, length, dst) with ``dst`` a contiguous 1-D view of length
        ``length`` receiving the compute-dtype copy of ``master[owner_start:owner_start+length]``.
        ``sub_group`` (DeepSpeed ZeRO-3 ``sub_group_size``, elements): update the owner space in
        launches of at most this many elements (0: one launch)."""
        assert master.dtype == torch.float32 and master.dim() == 1
        self.master = master
        self.exp_avg = torch.zeros_like(master)
        self.exp_avg_sq = torch.zeros_like(master)
        self.segments = list(segments)
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.step_count = 0
        self._lr_now = float(lr)
        self._tables = None
        self._seg_blocks = []    # segment -> (first, end) rows of the block tables (contiguous)
        self.sub_group = int(sub_group or 0)
        self._sub_ranges = None  # sub-group -> (first, end) rows of the block tables
        self.hp = None
        # compute-dtype copies written by the kernel: bf16 or fp16 (all segments share one)
        dts = {dst.dtype for _, _, dst in self.segments}
        assert len(dts) <= 1, "AdamW segments must share one compute dtype"
        self.dst_f16 = dts == {torch.float16}
        if master.is_cuda:
            self._build_tables()
            self.hp = torch.zeros(4, dtype=torch.float32, device=master.device)

    def _build_tables(self):
        chunk = ext().adamw_chunk()
        blk_seg: List[int] = []
        blk_start: List[int] = []
        so, sl, sd = [], [], []
        for i, (ostart, length, dst) in enumerate(self.segments):
            assert dst.is_contiguous() and dst.numel() == length
            assert length % 4 == 0 and ostart % 4 == 0 and dst.data_ptr() % 8 == 0, "AdamW segments must be 4-aligned"
            so.append(ostart)
            sl.append(length)
            sd.append(dst.data_ptr())
            first = len(blk_seg)
            for s in range(ostart, ostart + length, chunk):
                blk_seg.append(i)
                blk_start.append(s)
            self._seg_blocks.append((first, len(blk_seg)))
        if self.sub_group > 0:
            per = max(1, self.sub_group // chunk)        # block-table rows per launch
            self._sub_ranges = [(lo, min(lo + per, len(blk_seg))) for lo in range(0, len(blk_seg), per)]
        dev = self.master.device
        self._tables = (torch.tensor(blk_seg, dtype=torch.int32, device=dev),
                        torch.tensor(blk_start, dtype=torch.int64, device=dev),
                        torch.tensor(so, dtype=torch.int64, device=dev),
                        torch.tensor(sl, dtype=torch.int64, device=dev),
                        torch.tensor(sd, dtype=torch.int64, device=dev))

    # ---- step-dependent hyper-parameters live on the device ([lr, lr/bc1, 1/sqrt(bc2)]) so a
    # captured HIP graph of the optimizer step stays valid across replays: ``prepare`` advances
    # the host step counter and uploads the values (skipped while a graph is being captured;
    # the graph runner calls ``upload`` before every replay).
    def prepare(self, lr: float):
        self.step_count += 1
        self._lr_now = float(lr)
        if self.master.is_cuda and not torch.cuda.is_current_stream_capturing():
            self.upload()

    def upload(self):
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        vals = (self._lr_now, self._lr_now / bc1, 1.0 / math.sqrt(bc2), 0.0)
        if self.hp.is_cuda:
            # one fill per value: the scalars travel as kernel arguments.  A copy_ from a (pageable)
            # host tensor would synchronize the stream -- a full pipeline drain at every window
            # boundary of an eager (multi-rank) run
            for i, v in enumerate(vals):
                self.hp[i:i + 1].fill_(v)
        else:
            self.hp.copy_(torch.tensor(vals))

    def launch(self, grad: torch.Tensor, gscale: torch.Tensor = None):
        b1, b2 = self.betas
        if self._sub_ranges is not None and len(self._sub_ranges) > 1:
            for lo, hi in self._sub_ranges:
                self._launch_rows(lo, hi, grad, gscale)
            return
        ext().adamw(self.master, self.exp_avg, self.exp_avg_sq, grad, *self._tables, gscale,
                    self._lr_now, b1, b2, self.eps, self.weight_decay, self.step_count, self.hp, self.dst_f16)

    @property
    def launches_per_step(self) -> int:
        return len(self._sub_ranges) if self._sub_ranges else 1

    def _launch_rows(self, lo, hi, grad, gscale, grid_cap=0):
        b1, b2 = self.betas
        ext().adamw(self.master, self.exp_avg, self.exp_avg_sq, grad, self._tables[0][lo:hi],
                    self._tables[1][lo:hi], *self._tables[2:], gscale,
                    self._lr_now, b1, b2, self.eps, self.weight_decay, self.step_count, self.hp, self.dst_f16,
                    grid_cap)

    def launch_segment(self, i: int, grad: torch.Tensor, gscale: torch.Tensor = None, grid_cap: int = 0):
        """The update of segment ``i`` alone (one launch over a slice of the block tables; the
        blocks of a segment are contiguous rows).  With ``prepare`` called once per step, the
        per-segment launches together are exactly ``launch`` -- the engine uses them to let each
        bucket's forward wait for its own parameters only.  ``grid_cap`` > 0 runs the rows on at most
        that many workgroups (a side-stream update that should leave the CUs to concurrent kernels)."""
        if not self.master.is_cuda:              # CPU reference: the same update on the segment's rows
            b1, b2 = self.betas
            ostart, length, dst = self.segments[i]
            sl = slice(ostart, ostart + length)
            ref.adamw_flat(self.master[sl], self.exp_avg[sl], self.exp_avg_sq[sl], grad[sl], self._lr_now, b1, b2,
                           self.eps, self.weight_decay, self.step_count, gscale)
            dst.copy_(self.master[sl])
            return
        lo, hi = self._seg_blocks[i]
        self._launch_rows(lo, hi, grad, gscale, grid_cap)

    @torch.no_grad()
    def step(self, grad: torch.Tensor, lr: float, gscale: torch.Tensor = None):
        assert grad.numel() == self.master.numel()
        b1, b2 = self.betas
        if self.master.is_cuda:
            self.prepare(lr)
            self.launch(grad, gscale)
            return
        self.step_count += 1
        n = self.master.numel()
        sg = self.sub_group if self.sub_group > 0 else n
        for lo in range(0, n, sg):              # sub-groups: same update, launch by launch
            hi = min(n, lo + sg)
            ref.adamw_flat(self.master[lo:hi], self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi], grad[lo:hi], lr, b1,
                           b2, self.eps, self.weight_decay, self.step_count, gscale)
        for ostart, length, dst in self.segments:
            dst.copy_(self.master[ostart:ostart + length])

    def state_dict(self):
        return {"step": self.step_count, "master": self.master, "exp_avg": self.exp_avg,
                "exp_avg_sq": self.exp_avg_sq, "lr": self.lr, "betas": self.betas, "eps": self.eps,
                "weight_decay": self.weight_decay}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        for ostart, length, dst in self.segments:
            dst.copy_(self.master[ostart:ostart + length])

    @property
    def state_bytes(self) -> int:
        return 3 * self.master.numel() * 4
