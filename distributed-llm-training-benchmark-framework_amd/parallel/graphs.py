"""HIP-graph replay of whole training micro-steps.

A TinyGPT-A micro-step is ~480 kernel launches (GEMMs, the HIP kernels of dltb._C, RCCL calls)
issued from Python autograd Functions; measured on the MI355X, the host needs as long to issue
them as the GPU needs to run them (scripts/host_bound_check.py: enqueue/wall = 0.99), so the
Python side sets the step time.  ``GraphedStep`` captures the GPU work of each position in the
gradient-accumulation window (first micro-step overwrites gradient slots, middle ones
accumulate, the last also runs clipping + fused AdamW + parameter all-gather) into one
``torch.cuda.CUDAGraph`` per position -- HIP graphs on ROCm -- and replays it:

    step k:  engine.replay_host_step()        host bookkeeping + seed / LR uploads (3 tiny ops)
             static_idx.copy_(batch)          the next synthetic batch into the captured input
             graph[k % accum].replay()        ~480 kernels, one launch

Everything inside a captured region reads step-dependent values from device memory: the dropout
seed (``StepSeed.device_tensor``), AdamW's lr / bias corrections (``FlatAdamW.hp``), the clip
coefficient (computed on the device).  Graphs share one memory pool and are replayed in capture
order.  Capture happens at the start of the first window after an eager warm-up window
(hipBLASLt handles, TunableOp lookups, allocator pools and lazily built tables exist by then):
all ``accum`` positions are captured back to back -- a capture runs no GPU work, it only
advances the host bookkeeping -- then the host state is rewound and position 0 is replayed.  A
run therefore replays from its ``accum + 1``-th micro-step on, so a short warm-up (bench.py's
``--warmup 5`` at grad-accum 4) keeps every capture out of the timed region.  The loss returned
by a replay is the graph's static output tensor: callers that keep per-step losses copy it.  Collectives (RCCL
reduce-scatter / all-gather / all-reduce on the process group's stream) are captured with the
rest; ``DLTB_GRAPHS=0`` or ``--graphs off`` restores eager execution.
"""
import os

import torch


def graphs_enabled(flag: str, device, world: int = 1) -> bool:
    """``on`` / ``off``, or ``auto``: on for a single process, off for multi-rank runs.  Captured
    RCCL collectives work on this stack (scripts/rccl_graph_check.py) but a multi-rank capture
    cannot be validated on a one-GPU box, and at 1 GPU replay gains ~1 % (the step is GPU-bound),
    so multi-rank runs stay eager unless asked (``--graphs on`` / ``DLTB_GRAPHS=1``)."""
    if torch.device(device).type != "cuda":
        return False
    env = os.environ.get("DLTB_GRAPHS")
    if env is not None:
        return env == "1"
    if flag == "auto":
        return world == 1
    return flag == "on"


class GraphedStep:
    """``step(idx, targets) -> loss`` for one micro-step; eager until ``capture_after`` micro-steps
    have run (that window warms everything up), then capture-and-replay per window position."""

    def __init__(self, engine, capture_after: int = None):
        self.e = engine
        self.accum = engine.accum
        self.capture_after = self.accum if capture_after is None else capture_after
        self.graphs = {}
        self.pool = None
        self.static_idx = None
        self.static_tgt = None
        self.n = 0
        self.disabled = False
        if getattr(engine, "_tail_defer", False):
            # reduce-scatters left in flight across micro-steps would cross graph boundaries
            engine._drain_all()
            engine._tail_defer = False
        if getattr(engine, "_carry_on", False):
            # token rows carried into the next micro-step would be a tensor of one graph read by the
            # next graph, whose captured allocations may reuse its memory: exchange every micro-step
            engine._carry_on = False

    def _eager(self, idx, tgt):
        loss = self.e(idx, tgt)[1]
        self.e.backward(loss)
        self.e.step()
        return loss

    def __call__(self, idx, tgt):
        e = self.e
        pos = e.micro % self.accum
        self.n += 1
        if self.disabled or self.n <= self.capture_after or (not self.graphs and pos != 0):
            return self._eager(idx, tgt)            # warm-up, then start capturing at a window start
        if not self.graphs and not self._capture_window(idx, tgt):
            return self._eager(idx, tgt)
        g, loss = self.graphs[pos]
        e.replay_host_step()
        self.static_idx.copy_(idx)
        if tgt is not idx:
            self.static_tgt.copy_(tgt)
        g.replay()
        return loss

    def _capture_window(self, idx, tgt) -> bool:
        """Capture one graph per window position (called at a window start).  Returns False (and
        disables graphs for good) when a capture fails; the host state is rewound either way."""
        if self.static_idx is None:
            self.static_idx = idx.clone()
            self.static_tgt = self.static_idx if tgt is idx else tgt.clone()
        torch.cuda.synchronize()
        snap = self._host_state()
        graphs = {}
        try:
            for k in range(self.accum):
                g = torch.cuda.CUDAGraph()
                # thread_local: the process group's watchdog thread may query events meanwhile
                with torch.cuda.graph(g, pool=self.pool, capture_error_mode="thread_local"):
                    loss = self._eager(self.static_idx, self.static_tgt)
                self.pool = g.pool()
                graphs[k] = (g, loss)
        except Exception as exc:  # noqa: BLE001 - fall back to eager execution for good
            self._restore_host_state(snap)
            self.disabled = True
            print(f"[dltb] HIP-graph capture failed ({type(exc).__name__}: {exc}); running eagerly", flush=True)
            torch.cuda.synchronize()
            return False
        self._restore_host_state(snap)       # the captures ran no GPU work: replay from position 0
        if self.e.opt.step_count > 0:
            self.e.opt.upload()
        self.graphs = graphs
        return True

    def _host_state(self):
        e = self.e
        return (e.seed.state, e.seed.value, e.micro, e.opt_steps, e.opt.step_count, dict(e._written),
                e._window_pos, e._is_boundary, e.last_lr, e._pending_lr, e.opt._lr_now)

    def _restore_host_state(self, s):
        e = self.e
        (e.seed.state, e.seed.value, e.micro, e.opt_steps, e.opt.step_count, written,
         e._window_pos, e._is_boundary, e.last_lr, e._pending_lr, e.opt._lr_now) = s
        e._written.clear()
        e._written.update(written)
        if hasattr(e, "_wt_epoch"):
            e._wt_epoch = -1            # transposes "refreshed" inside the failed capture never ran
        e.seed.upload()
