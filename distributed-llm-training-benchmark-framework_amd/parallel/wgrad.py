"""Deferred weight gradients, issued as strided-batched GEMMs over consecutive blocks.

A TinyGPT-A layer's dW products (dY^T X over 2048 tokens, 1024-4096 wide) are too small to fill the
256 CUs of an MI355X one at a time: hipBLASLt runs them at 250-610 TFLOP/s.  None of them is on the
critical path of the backward (only the dX chain is), so the engine queues them and issues the
products of several blocks at once.  Because

* the gradient slots of one parameter in consecutive blocks sit at a constant stride in the flat
  gradient buffer (``flat.py`` lays whole blocks out back to back), and
* the model writes the GEMM operands of every block (X: LN outputs, attention output, GELU output;
  dY: the incoming gradients) into layer-strided activation buffers,

a group of blocks is ONE strided-batched hipBLASLt call per parameter kind (``bmm`` / ``baddbmm_``
on ``as_strided`` views, no copies).  Measured on MI355X (scripts/bench_batched_wgrad.py): per
layer qkv 27.0 -> 14.3 us, out-proj 16.4 -> 4.3 us, fc1 30.0 -> 18.4 us, fc2 29.5 -> 18.5 us
(16 blocks batched, accumulate form) -- 0.76 ms of a 9.2 ms micro-step.

Engines flush a group when its gradients are due: at world size 1 once at the end of backward (all
16 blocks in one batch); at world size > 1 per gradient bucket, right before the bucket's RCCL
collective, so communication still overlaps the rest of the backward.  Anything that does not form
an equally-spaced batch (other layouts, CPU copies in other storages) falls back to one GEMM per
block, so correctness never depends on the layout.
"""
from collections import defaultdict
from typing import Dict, List, Optional

import torch

from ..ops import blaslt as _blt
from ..ops import functional as F_


def strided_batch(ts: List[torch.Tensor], out: bool = False) -> Optional[torch.Tensor]:
    """A [n, *shape] view covering the equally spaced same-shape 2-D tensors ``ts`` (in order) of
    one storage, or None.  ``out``: the matrices must not overlap (the view is written)."""
    t0 = ts[0]
    if len(ts) == 1:
        return t0.unsqueeze(0)
    es = t0.element_size()
    step = ts[1].data_ptr() - t0.data_ptr()
    if step <= 0 or step % es:
        return None
    base = t0.untyped_storage().data_ptr()
    for a, b in zip(ts, ts[1:]):
        if (b.data_ptr() - a.data_ptr() != step or b.shape != t0.shape or b.stride() != t0.stride()
                or b.untyped_storage().data_ptr() != base):
            return None
    step //= es
    if out and step < (t0.shape[0] - 1) * t0.stride(0) + (t0.shape[1] - 1) * t0.stride(1) + 1:
        return None
    return t0.as_strided((len(ts),) + tuple(t0.shape), (step,) + tuple(t0.stride()))


class WgradQueue:
    """Queued ``dw (+)= dy^T x`` products keyed by unit; ``flush`` issues them batched."""

    def __init__(self):
        self._items: Dict[int, list] = defaultdict(list)     # id(unit) -> [(i, dy, x, dw, acc)]
        self.batched_calls = 0
        self.single_calls = 0
        self.tn_calls = 0            # batched products that ran on the own token-major kernel (gemm_tn)

    def add(self, unit, i, dy, x, dw, accumulate):
        self._items[id(unit)].append((i, dy, x, dw, bool(accumulate)))

    def has(self, units) -> bool:
        """Whether any of ``units`` has queued products."""
        return any(id(u) in self._items for u in units)

    def pending(self, units) -> list:
        """The queued items of ``units`` (references that keep their operands alive)."""
        return [it for u in units for it in self._items.get(id(u), ())]

    def __len__(self):
        return sum(len(v) for v in self._items.values())

    def flush(self, units=None):
        keys = list(self._items) if units is None else [id(u) for u in units if id(u) in self._items]
        groups = defaultdict(list)                           # (param index, accumulate) -> items
        for k in keys:
            for i, dy, x, dw, acc in self._items.pop(k):
                groups[(i, acc)].append((dy, x, dw))
        for (_, acc), items in groups.items():
            items.sort(key=lambda it: it[2].data_ptr())      # flat-buffer order of the slots
            self._issue(items, acc)

    def _issue(self, items, acc):
        if len(items) > 1:
            DW = strided_batch([it[2] for it in items], out=True)
            DY = strided_batch([it[0] for it in items])
            X = strided_batch([it[1] for it in items])
            if DW is not None and DY is not None and X is not None:
                if X.stride(-2) == 1 and X.stride(-1) != 1:
                    # BLAS TN batched: hipBLASLt's heuristic solution for it faulted the GPU
                    # (profiles/dw_layout_probe_fault_r4.txt); the layer buffers are row-major
                    raise RuntimeError("batched dW with a column-major X operand (BLAS TN) is refused")
                if F_.own_wgrad(DY, X, DW, acc):
                    self.tn_calls += 1
                elif _blt.mm(DY.transpose(1, 2), X, DW, acc):
                    pass
                elif acc:
                    DW.baddbmm_(DY.transpose(1, 2), X)
                else:
                    torch.bmm(DY.transpose(1, 2), X, out=DW)
                self.batched_calls += 1
                return
        for dy, x, dw in items:                              # not equally spaced: one GEMM each
            F_.linear_wgrad(dy, x, dw, None, acc)
            self.single_calls += 1
