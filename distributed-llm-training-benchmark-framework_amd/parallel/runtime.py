"""Parameter runtime interface between the fused model Functions and a parallelism engine.

The models in :mod:`dltb.models` are chains of fused autograd Functions (embedding, one Function
per transformer block, head+loss).  Each Function works on one *unit* of parameters and talks to
the runtime instead of to ``nn.Parameter.grad``:

    forward : params = rt.acquire(unit)            ... compute ...   rt.release_forward(unit)
    backward: params = rt.acquire_backward(unit)   (re-gathers / prefetches under FSDP, ZeRO-3)
              slot, acc = rt.grad_slot(unit, i)    (flat-buffer gradient view + overwrite/accumulate)
              ... GEMMs write dW straight into the slots (rt.wgrad: now, or queued and batched
                  over blocks by engines that defer them) ...
              rt.grads_ready(unit)                 (DDP: bucket all-reduce; ZeRO/FSDP: reduce-scatter)
              rt.release_backward(unit)

This is the MI355X-native replacement for the reference's reliance on autograd hooks inside
torch DDP's C++ Reducer / FSDP / DeepSpeed (train_harness.py:207-275): the engines know exactly
when a unit's gradients are complete, launch their RCCL collective right then on the process
group's stream, and never copy gradients between buffers.
"""
from typing import List, Sequence, Tuple

import torch
import torch.nn as nn


class Unit:
    """An ordered group of parameters gathered / reduced together."""

    def __init__(self, name: str, params: Sequence[Tuple[str, nn.Parameter]], index: int = 0):
        self.name = name
        self.names = [n for n, _ in params]
        self.params = [p for _, p in params]
        self.index = index
        self.shapes = [tuple(p.shape) for p in self.params]
        self.numels = [p.numel() for p in self.params]

    @property
    def numel(self) -> int:
        return sum(self.numels)

    def __repr__(self):
        return f"Unit({self.name}, {len(self.params)} params, {self.numel} elems)"


class ParamRuntime:
    """Interface + the eager default used when no engine is attached (CPU tests, oracles).

    Eager semantics mirror autograd: gradients accumulate into ``param.grad`` (allocated on the first
    write), so a model without an engine behaves like a plain nn.Module under ``loss.backward()``.
    """

    def __init__(self):
        self.seed = None          # dltb.ops.rng.StepSeed
        self.compute_dtype = None

    # forward
    def acquire(self, unit: Unit) -> List[torch.Tensor]:
        return [p.detach() for p in unit.params]

    def release_forward(self, unit: Unit):
        pass

    def acquire_tied(self, unit: Unit) -> List[torch.Tensor]:
        """Parameters of another unit used by a tied consumer (the head reads wte)."""
        return self.acquire(unit)

    def weight_t(self, unit: Unit, i: int, w: torch.Tensor):
        """A contiguous transpose of 2-D parameter ``i`` of ``unit`` (the value ``w`` holds now), or
        None.  Engines whose parameters stay put for a whole accumulation window cache it, so the
        data-gradient GEMM dY W runs in hipBLASLt's fast NT form (dY (W^T)^T) -- 20-30 % faster at
        M = 2048 -- for the price of one transpose per optimizer step."""
        return None

    # backward
    def acquire_backward(self, unit: Unit) -> List[torch.Tensor]:
        return [p.detach() for p in unit.params]

    def grad_slot(self, unit: Unit, i: int) -> Tuple[torch.Tensor, bool]:
        p = unit.params[i]
        if p.grad is None:
            p.grad = torch.empty_like(p)
            return p.grad, False
        return p.grad, True

    # weight gradients (dW (+)= dY^T X of a linear layer)
    # True: a gradient slot of a unit may be written before that unit's own backward runs (the
    # consumer block forms the previous block's fc2 bias gradient, models/tinygpt.py)
    grad_write_ahead = False
    defer_wgrad = False     # True: the engine queues them (parallel/wgrad.py) and issues batches
    # order of the blocks' gradient slots in the engine's flat buffer: True = last block first
    # (backward-ordered replicated layouts); the model's layer-strided buffers follow it
    wgrad_rows_reversed = True

    def wgrad_window(self):
        """(position, accum) when the engine consumes gradients only at the accumulation-window
        boundary and wants the window's weight gradients as ONE product per parameter over all its
        micro-steps' tokens (the model then keeps every micro-step's GEMM operands in its layer
        buffers and hands over full-window views at the last micro-step); None otherwise."""
        return None

    def grad_reducer(self):
        """A column-sum reducer shared by every block's backward (flushed by the engine once per
        backward), or None: each block reduces its own bias / norm-weight sums before it reports
        its gradients (``grads_ready``)."""
        return None

    def wgrad(self, unit: Unit, i: int, dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor,
              accumulate: bool):
        """Write ``dy^T x`` into gradient slot ``dw`` (``accumulate``: add).  The default issues it
        now; engines with ``defer_wgrad`` run it later, batched with the other blocks' products."""
        from ..ops import functional as F_
        F_.linear_wgrad(dy, x, dw, None, accumulate)

    def embedding_backward(self, tok, pos, dx: torch.Tensor, idx: torch.Tensor, p: float, seed, site: int):
        """The token-embedding backward: scatter-add the (dropout-backward'd) rows of ``dx`` into the
        token table's gradient slot ``tok = (unit, i)`` by ``idx``, and their per-position sums
        into the position table's slot ``pos`` (or None).  When the token table is tied to the
        head, its slot already holds the head's dense gradient and the rows are added to it.
        Engines whose collective for ``tok`` already ran this micro-step (the tied table is
        reduced right after the head's backward) override this with a sparse exchange."""
        from ..ops import functional as F_
        dwte, acc = self.grad_slot(*tok)
        if not acc:
            dwte.zero_()
        dwpe, acc_p = self.grad_slot(*pos) if pos is not None else (None, False)
        F_.embed_bwd(dx, idx, dwte, dwpe, acc_p, p, seed, site)

    def grads_ready(self, unit: Unit):
        pass

    def release_backward(self, unit: Unit):
        pass


EAGER = ParamRuntime()
