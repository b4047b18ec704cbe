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
* Emulated fabric (``DLTB_COMM=emulate:N``, one process, one GPU): ``world = N`` and ``rank =
  $DLTB_EMU_RANK`` (default 0) with NO process group, so the engines build the real N-rank layouts,
  shards, bucket plans, tail-deferral and per-rank memory footprint.  Each collective runs, on a
  high-priority side stream with RCCL's event semantics (the caller's stream waits only at
  ``wait()``), ONE paced kernel (csrc/comm_emu.hip) that keeps ``$DLTB_EMU_CHANNELS`` (32)
  workgroups resident for the alpha-beta-modelled duration of that collective at N ranks
  (comm/topology.py), reads its buffer through HBM and writes a local stand-in for its result
  (reduce-scatter: N x the own chunk; all-reduce: x N; all-gather into a fresh buffer: the own
  shard replicated; in place: unchanged).  The step time it produces is a PREDICTION of the N-GPU
  step -- overlap, exposed communication and the CU/HBM contention of the collectives are real,
  the fabric itself is the model.  On the CPU only the numerics run (wire-byte accounting tests).
* Lazy mode (``DLTB_COMM_LAZY=1``, tests): an asynchronous collective runs only when its work is
  waited -- it reads its input and writes its output at ``wait()``, the latest moment RCCL could.
  A rank that overwrites a buffer still being reduced, reads a result before waiting for it, or
  never waits at all then computes different numbers, so the world-size equivalence tests catch
  missing or misplaced waits deterministically (the host-staged and CPU gloo paths are otherwise
  synchronous or racy, and only RCCL on several GPUs runs truly asynchronously).
"""
import os
import time
from collections import OrderedDict

import torch
import torch.distributed as dist


class _EmuWork:
    """Emulated collective in flight on the emulation stream (an event the caller's stream waits
    for at ``wait()``, like a ProcessGroupNCCL work)."""

    def __init__(self, ev, keep):
        self._ev = ev
        self._keep = keep            # tensors the side stream still uses

    def wait(self):
        if self._ev is not None:
            torch.cuda.current_stream().wait_event(self._ev)
            self._keep = None
        return True

    def is_completed(self):
        return self._ev is None or self._ev.query()


def emulated_world():
    """N of ``DLTB_COMM=emulate:N`` (0 when not emulating)."""
    mode = os.environ.get("DLTB_COMM", "")
    if not mode.startswith("emulate"):
        return 0
    try:
        n = int(mode.split(":", 1)[1])
    except (IndexError, ValueError):
        raise ValueError(f"DLTB_COMM={mode!r}: expected emulate:N") from None
    if n < 1:
        raise ValueError("DLTB_COMM=emulate:N needs N >= 1")
    return n


class _Done:
    """Completed work (single process, or a synchronous call)."""

    def wait(self):
        return True

    def is_completed(self):
        return True


_DONE = _Done()


class _Lazy:
    """Work whose collective runs at the first ``wait()`` (lazy mode).  Collectives still run in
    the order they were issued, as on RCCL's stream: waiting for one first runs every earlier
    collective of the same comm still queued (ranks may wait in different orders -- a rank whose
    unit did not report drains its buckets elsewhere -- but they issue in the same order)."""

    def __init__(self, fn, queue):
        self._fn = fn
        self._queue = queue
        queue.append(self)

    def _run(self):
        if self._fn is not None:
            fn, self._fn = self._fn, None
            fn()

    def wait(self):
        if self._fn is not None:
            while self._queue:
                w = self._queue.pop(0)
                w._run()
                if w is self:
                    break
        return True

    def is_completed(self):
        return self._fn is None

_REDUCE_OPS = {"sum": "SUM", "max": "MAX", "min": "MIN", "avg": "AVG"}

# emulated fabric: local HBM passes over the full buffer per collective (see Comm.__init__)
EMU_HBM_PASSES = {"reduce_scatter": 3, "all_gather": 2, "all_reduce": 5, "broadcast": 2, "all_to_all": 2}


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
        self.emulate = emulated_world()
        self.enabled = dist.is_available() and dist.is_initialized() and not self.emulate
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.rank = dist.get_rank(group) if self.enabled else 0
        self.backend = dist.get_backend(group) if self.enabled else "none"
        if self.emulate:
            self.world, self.rank, self.backend = self.emulate, int(os.environ.get("DLTB_EMU_RANK", "0")), "emulate"
            if not 0 <= self.rank < self.world:
                raise ValueError(f"DLTB_EMU_RANK={self.rank} outside emulate:{self.world}")
            from .topology import measured_params, pg_host_cost_us
            self.emu_channels = int(os.environ.get("DLTB_EMU_CHANNELS", "32"))
            # local HBM passes over the full buffer per op (ring algorithms, N ranks): reduce-scatter
            # reads its input and writes + re-reads every received chunk (~3), all-gather writes and
            # re-reads the forwarded chunks (~2), all-reduce is both (~5).  DLTB_EMU_HBM_PASSES
            # overrides every op (0: no traffic stream -- the N-rank code path alone)
            env_p = os.environ.get("DLTB_EMU_HBM_PASSES")
            self.emu_pass_of = {op: (int(env_p) if env_p is not None else n) for op, n in EMU_HBM_PASSES.items()}
            self.emu_passes = max(self.emu_pass_of.values())      # (reported; 0 only if all are)
            # host time of the ProcessGroupNCCL call each emulated collective stands in for
            # (profiles/pg_host_cost.json, scripts/probes/pg_host_cost.py); spun on the host before
            # the paced kernel is launched, so an eager emulated step pays what a real one would
            self.emu_host_us = pg_host_cost_us()
            self.emu_null = os.environ.get("DLTB_EMU_NULL", "0") == "1"
            self.emu_params = {}          # op -> (alpha_us, bus_GBps, source)
            for op in ("all_reduce", "reduce_scatter", "all_gather", "broadcast", "all_to_all"):
                a, b, src = measured_params(self.world, "all_reduce" if op == "all_reduce" else "reduce_scatter")
                a = float(os.environ.get("DLTB_EMU_ALPHA_US", a))
                b = float(os.environ.get("DLTB_EMU_BUS_GBPS", b))
                self.emu_params[op] = (a, b, src)
            self._emu_stream = None
        self.staged = self.backend == "gloo"      # device tensors go through host memory
        self.lazy = os.environ.get("DLTB_COMM_LAZY", "0") == "1" and not self.emulate
        self._pending = []
        self._lazy_queue = []                 # lazy mode: issued, not yet run (issue order)
        self.stats = OrderedDict()            # op -> {"calls": n, "wire_bytes": b}

    # ------------------------------------------------------------------ accounting
    def _count(self, op: str, t: torch.Tensor):
        s = self.stats.setdefault(op, {"calls": 0, "wire_bytes": 0})
        s["calls"] += 1
        s["wire_bytes"] += int(t.numel() * t.element_size() * ring_factor(op, self.world))
        if self.emulate:
            a, b = self._emu_time(op, t)
            s["model_us"] = s.get("model_us", 0.0) + a + b

    def modelled_us(self) -> float:
        """Emulated fabric: the summed alpha-beta time of every collective issued since the last
        ``reset_stats`` (what the fabric would be busy for, overlapped or not)."""
        return sum(s.get("model_us", 0.0) for s in self.stats.values())

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

    # ------------------------------------------------------------------ emulated fabric
    def _emu_time(self, op, full):
        """(alpha_us, beta_us) of ``op`` on the full buffer ``full`` at ``self.world`` ranks."""
        a, bus, _ = self.emu_params["all_to_all" if op == "all_to_all" else op]
        nbytes = full.numel() * full.element_size()
        return a, nbytes * ring_factor(op, self.world) / (bus * 1e3)

    def _emu(self, op, full, dst=None, src=None, scale=1.0, replicas=1, rep_stride=0,
             async_op=True, track=True):
        """One emulated collective: numerics stand-in ``dst[r*rep_stride + j] = scale * src[j]``
        plus, on a GPU, the paced kernel on the emulation stream."""
        if not full.is_cuda:
            if src is not None:
                v = src * scale if scale != 1.0 else src
                for r in range(replicas):
                    dst.view(-1)[r * rep_stride:r * rep_stride + src.numel()].copy_(v.view(-1))
            return _DONE
        from ..ops._ext import ext
        if self.emu_null:
            # DLTB_EMU_NULL=1 (timing only): no collective kernel and no numerics stand-in at all --
            # the step time of the N-rank code path alone (the results are NOT the N-rank numerics)
            return _DONE
        if self._emu_stream is None:
            self._emu_stream = torch.cuda.Stream(device=full.device, priority=-1)
            self._emu_handle = self._emu_stream.cuda_stream
        side = self._emu_stream
        side.wait_stream(torch.cuda.current_stream(full.device))   # starts after its producers
        alpha, beta = self._emu_time(op, full)
        host = self.emu_host_us.get(op, 0.0)
        if op == "all_reduce" and not async_op and full.numel() <= 16 and "all_reduce_scalar_sync" in self.emu_host_us:
            host = self.emu_host_us["all_reduce_scalar_sync"]   # the clip norm's own measured (sync, 1 float) cost
        if host > 0:                          # the ProcessGroupNCCL call's host time
            t_end = time.perf_counter() + host * 1e-6
            while time.perf_counter() < t_end:
                pass
        passes = self.emu_pass_of.get(op, 1)
        # (DLTB_EMU_HBM_PASSES=0: no traffic stream, the numerics stand-in only -- isolates the
        # N-rank code path from the collectives' HBM contention)
        ext().comm_emu(full if passes > 0 else None, max(1, passes), dst, src, float(scale),
                       int(replicas), int(rep_stride), float(alpha), float(beta), self.emu_channels,
                       self._emu_handle)
        keep = (full, dst, src)
        for t in keep:
            if t is not None:
                t.record_stream(side)
        ev = torch.cuda.Event()
        ev.record(side)
        w = _EmuWork(ev, keep)
        if not async_op:
            w.wait()
            return _DONE
        return self._track(w, True) if track else w

    def _emu_gather(self, out, inp, async_op, track):
        n = inp.numel()
        off = out.data_ptr() + self.rank * n * out.element_size()
        if inp.data_ptr() == off and inp.dtype == out.dtype:     # in place: the own chunk is already there
            return self._emu("all_gather", out, async_op=async_op, track=track)
        if self.emu_null and out.is_cuda:
            return _DONE
        if out.is_cuda and out.dtype not in (torch.bfloat16, torch.float16, torch.float32):
            # integer payloads (the embedding's token ids): replicate with a torch copy on the
            # emulation stream, the paced kernel models the transfer
            if self._emu_stream is None:
                self._emu_stream = torch.cuda.Stream(device=out.device, priority=-1)
            self._emu_stream.wait_stream(torch.cuda.current_stream(out.device))
            with torch.cuda.stream(self._emu_stream):
                out.view(self.world, n).copy_(inp.reshape(1, n).expand(self.world, n))
            # the caller may free ``inp`` right away: its memory must not be handed to later work
            # on the compute stream before this copy has read it
            inp.record_stream(self._emu_stream)
            return self._emu("all_gather", out, async_op=async_op, track=track)
        return self._emu("all_gather", out, out.view(-1), inp.reshape(-1), 1.0, self.world, n,
                         async_op=async_op, track=track)

    # ------------------------------------------------------------------ collectives
    def _flush_lazy(self):
        while self._lazy_queue:                   # earlier collectives complete first
            self._lazy_queue.pop(0)._run()

    def _lazy(self, fn, async_op: bool, track: bool):
        if not async_op:
            self._flush_lazy()
            fn()
            return _DONE
        w = _Lazy(fn, self._lazy_queue)
        return self._track(w, True) if track else w

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = True, track: bool = True):
        """In-place all-reduce of a flat buffer slice (DDP bucket, grad-norm scalar)."""
        if self.world == 1:
            return _DONE
        self._count("all_reduce", t)
        if self.emulate:
            sc = float(self.world) if op == "sum" else 1.0
            return self._emu("all_reduce", t, t.view(-1), t.view(-1), sc, async_op=async_op, track=track)
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
        if self.emulate:
            n = out.numel()
            mine = inp.reshape(-1)[self.rank * n:(self.rank + 1) * n]
            return self._emu("reduce_scatter", inp, out.view(-1), mine, float(self.world),
                             async_op=async_op, track=track)
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
        if self.emulate:
            return self._emu_gather(out, inp, async_op, track)
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

    def global_rank(self, r: int) -> int:
        """Global rank of group rank ``r`` (``broadcast``'s ``src`` is a global rank)."""
        if self.group is None or not self.enabled:
            return r
        return dist.get_global_rank(self.group, r)

    def broadcast(self, t: torch.Tensor, src: int = 0):
        if self.world == 1:
            return
        self._flush_lazy()
        self._count("broadcast", t)
        if self.emulate:
            self._emu("broadcast", t, async_op=False)
            return
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
        self._flush_lazy()
        self._count("all_to_all", inp)
        if self.emulate:
            return self._emu("all_to_all", inp, out.view(-1), inp.reshape(-1), async_op=async_op)
        if self.staged and (inp.is_cuda or out.is_cuda):
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(h, self._host(inp), group=self.group)
            self._back(out, h)
            return _DONE
        w = dist.all_to_all_single(out, inp, group=self.group, async_op=async_op)
        return self._track(w, async_op)

    def barrier(self):
        if self.world > 1 and not self.emulate:
            self._flush_lazy()
            dist.barrier(group=self.group)

    def max_scalar(self, x: float, device) -> float:
        """Host float max over ranks (timings, peak memory)."""
        if self.world == 1 or self.emulate:
            return x
        self._flush_lazy()
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if self.staged else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())
