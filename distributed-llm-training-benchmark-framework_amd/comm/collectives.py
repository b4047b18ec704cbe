"""RCCL-over-xGMI collective layer used by every engine.

The reference issues no collective itself: torch DDP's C++ Reducer, FSDP and DeepSpeed issue them
(train_harness.py:190-204 only initialises and tears down).  Here the
engines own their communication, and this module is the one place that talks to
``torch.distributed``:

* ``Comm`` wraps one process group ("nccl" = RCCL on ROCm, or gloo on the CPU).  Every bulk op takes
  a contiguous slice of a flat bf16/fp32 buffer, so a bucket is one RCCL call with no packing
  kernel.  Ops are asynchronous by default; the returned work is kept in the comm's pending list
  until ``wait_all()`` (``work.wait()`` on a GPU work makes the *compute stream* wait on RCCL's
  stream; the host does not block).
* Wire accounting: each call adds the bytes one rank sends under ring algorithms (all-reduce
  2(n-1)/n of the buffer, reduce-scatter and all-gather (n-1)/n), so ``stats`` reports what the
  step actually moved over xGMI, per op.
* ``world == 1``: every op is a no-op that returns a completed work, so engines need no
  single-process special cases around their collectives.
* Host-staged mode (gloo process group, device tensors; ``DLTB_COMM=host`` in
  ``utils.dist.setup_distributed``): every collective copies its device buffer to host memory,
  runs the gloo op there (bf16 / fp16 / fp32 are all supported) and copies the result back,
  synchronously.  RCCL refuses two ranks on one GPU; this mode lets N ranks share the single
  MI355X of a test box, so every code path that exists only at world > 1 (bf16 flat buckets, the
  per-bucket batched weight gradients, deferred all-gathers waited in ``acquire``, fp32
  accumulation of reduce-scattered chunks, ZeRO-3 transient gather buffers) runs with the real
  HIP kernels.  It is a correctness mode, not a performance mode.
* Lazy mode (``DLTB_COMM_LAZY=1``, tests): an asynchronous collective runs only when its work is
  waited -- it reads its input and writes its output at ``wait()``, the latest moment RCCL could.
  A rank that overwrites a buffer still being reduced, reads a result before waiting for it, or
  never waits at all then computes different numbers, so the world-size equivalence tests catch
  missing or misplaced waits deterministically (the host-staged and CPU gloo paths are otherwise
  synchronous or racy, and only RCCL on several GPUs runs truly asynchronously).
"""
import os
from collections import OrderedDict

import torch
import torch.distributed as dist


class _Done:
    """Completed work (single process, or a synchronous call)."""

    def wait(self):
        return True

    def is_completed(self):
        return True


_DONE = _Done()


class _Lazy:
    """Work whose collective runs at the first ``wait()`` (lazy mode)."""

    def __init__(self, fn):
        self._fn = fn

    def wait(self):
        if self._fn is not None:
            fn, self._fn = self._fn, None
            fn()
        return True

    def is_completed(self):
        return self._fn is None

_REDUCE_OPS = {"sum": "SUM", "max": "MAX", "min": "MIN", "avg": "AVG"}


def ring_factor(op: str, world: int) -> float:
    """Bytes one rank sends per byte of the (full) buffer, ring algorithms."""
    if world <= 1:
        return 0.0
    if op == "all_reduce":
        return 2.0 * (world - 1) / world
    return (world - 1) / world


class Comm:
    def __init__(self, group=None):
        self.group = group
        self.enabled = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.rank = dist.get_rank(group) if self.enabled else 0
        self.backend = dist.get_backend(group) if self.enabled else "none"
        self.staged = self.backend == "gloo"      # device tensors go through host memory
        self.lazy = os.environ.get("DLTB_COMM_LAZY", "0") == "1"
        self._pending = []
        self.stats = OrderedDict()            # op -> {"calls": n, "wire_bytes": b}

    # ------------------------------------------------------------------ accounting
    def _count(self, op: str, t: torch.Tensor):
        s = self.stats.setdefault(op, {"calls": 0, "wire_bytes": 0})
        s["calls"] += 1
        s["wire_bytes"] += int(t.numel() * t.element_size() * ring_factor(op, self.world))

    def wire_bytes(self) -> int:
        return sum(s["wire_bytes"] for s in self.stats.values())

    def reset_stats(self):
        self.stats.clear()

    # ------------------------------------------------------------------ outstanding work
    def _track(self, w, async_op: bool):
        if w is None:
            return _DONE
        if async_op:
            self._pending.append(w)
            return w
        w.wait()
        return _DONE

    def wait_all(self):
        for w in self._pending:
            w.wait()
        self._pending.clear()

    @property
    def pending(self) -> int:
        return len(self._pending)

    # ------------------------------------------------------------------ host staging (gloo)
    def _host(self, t: torch.Tensor) -> torch.Tensor:
        return t.to("cpu") if t.is_cuda else t

    def _back(self, dst: torch.Tensor, h: torch.Tensor):
        if dst.data_ptr() != h.data_ptr() or dst.device != h.device:
            dst.copy_(h)

    # ------------------------------------------------------------------ collectives
    def _lazy(self, fn, async_op: bool, track: bool):
        if not async_op:
            fn()
            return _DONE
        w = _Lazy(fn)
        return self._track(w, True) if track else w

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = True, track: bool = True):
        """In-place all-reduce of a flat buffer slice (DDP bucket, grad-norm scalar)."""
        if self.world == 1:
            return _DONE
        self._count("all_reduce", t)
        if self.lazy:
            return self._lazy(lambda: self._all_reduce(t, op), async_op, track)
        return self._all_reduce(t, op, async_op, track)

    def _all_reduce(self, t, op, async_op=False, track=True):
        if self.staged and t.is_cuda:
            h = self._host(t)
            dist.all_reduce(h, op=getattr(dist.ReduceOp, _REDUCE_OPS[op]), group=self.group)
            self._back(t, h)
            return _DONE
        w = dist.all_reduce(t, op=getattr(dist.ReduceOp, _REDUCE_OPS[op]), group=self.group,
                            async_op=async_op)
        return self._track(w, async_op) if track else (w if async_op else _DONE)

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = True,
                       track: bool = True):
        """SUM-reduce ``inp`` (world x chunk) and keep this rank's chunk in ``out``."""
        if self.world == 1:
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp)
            return _DONE
        assert inp.numel() == out.numel() * self.world, "reduce_scatter: input must be world x output"
        self._count("reduce_scatter", inp)
        if self.lazy:
            return self._lazy(lambda: self._reduce_scatter(out, inp), async_op, track)
        return self._reduce_scatter(out, inp, async_op, track)

    def _reduce_scatter(self, out, inp, async_op=False, track=True):
        if self.staged and (inp.is_cuda or out.is_cuda):
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.reduce_scatter_tensor(h, self._host(inp), group=self.group)
            self._back(out, h)
            return _DONE
        w = dist.reduce_scatter_tensor(out, inp, group=self.group, async_op=async_op)
        return self._track(w, async_op) if track else (w if async_op else _DONE)

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = True,
                   track: bool = True):
        """Gather every rank's ``inp`` chunk into ``out`` (world x chunk); in place when ``inp`` is
        this rank's slice of ``out``."""
        if self.world == 1:
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp)
            return _DONE
        assert out.numel() == inp.numel() * self.world, "all_gather: output must be world x input"
        self._count("all_gather", out)
        if self.lazy:
            return self._lazy(lambda: self._all_gather(out, inp), async_op, track)
        return self._all_gather(out, inp, async_op, track)

    def _all_gather(self, out, inp, async_op=False, track=True):
        if self.staged and (inp.is_cuda or out.is_cuda):
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather_into_tensor(h, self._host(inp), group=self.group)
            self._back(out, h)
            return _DONE
        w = dist.all_gather_into_tensor(out, inp, group=self.group, async_op=async_op)
        return self._track(w, async_op) if track else (w if async_op else _DONE)

    def broadcast(self, t: torch.Tensor, src: int = 0):
        if self.world == 1:
            return
        self._count("broadcast", t)
        if self.staged and t.is_cuda:
            h = self._host(t)
            dist.broadcast(h, src=src, group=self.group)
            self._back(t, h)
            return
        dist.broadcast(t, src=src, group=self.group)

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        if self.world == 1:
            out.copy_(inp)
            return _DONE
        self._count("all_to_all", inp)
        if self.staged and (inp.is_cuda or out.is_cuda):
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(h, self._host(inp), group=self.group)
            self._back(out, h)
            return _DONE
        w = dist.all_to_all_single(out, inp, group=self.group, async_op=async_op)
        return self._track(w, async_op)

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    def max_scalar(self, x: float, device) -> float:
        """Host float max over ranks (timings, peak memory)."""
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if self.staged else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())
