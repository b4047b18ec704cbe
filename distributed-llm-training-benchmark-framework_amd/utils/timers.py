"""Per-phase step timers: forward / backward / exposed collective wait / optimizer.

SURVEY.md §5.1 asks for hipEvent-based per-phase timing (the reference only times whole steps on
the host, train_harness.py:361,384-385).  The harness and the engines drop named *marks* into the
stream as a micro-step runs; the interval from one mark to the next is charged to the phase the
first mark opens:

    step_begin ─forward─▶ [opt_begin ─optimizer─▶ opt_end ─forward─▶] fwd_end ─backward─▶
    [comm_wait_begin ─comm_wait─▶ comm_wait_end ─backward─▶] bwd_end ─optimizer─▶ step_end

(``opt_*`` appear where a deferred ZeRO update runs at the start of the next micro-step; the
``comm_wait`` interval is the time the compute stream waits for the bucket collectives after the
last backward kernel -- the communication the overlap did not hide.)  On a GPU the marks are HIP
events on the current stream, read once at the end (no per-step synchronisation); on the CPU they
are ``time.perf_counter`` stamps.  Whole-step HIP-graph replay has no phase boundaries, so the
harness runs eagerly while the timers are on.
"""
import time
from collections import defaultdict

import torch

_PHASE_OF = {"step_begin": "forward", "opt_begin": "optimizer", "opt_end": "forward",
             "fwd_end": "backward", "comm_wait_begin": "comm_wait", "comm_wait_end": "backward",
             "bwd_end": "optimizer"}
PHASES = ("forward", "backward", "comm_wait", "optimizer")


class PhaseTimers:
    def __init__(self, device):
        self.cuda = torch.device(device).type == "cuda"
        self.steps = []
        self._cur = None

    def begin_step(self):
        self._cur = []
        self.mark("step_begin")

    def mark(self, name: str):
        if self._cur is None:
            return
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._cur.append((name, ev))
        else:
            self._cur.append((name, time.perf_counter()))

    def end_step(self):
        if self._cur is None:
            return
        self.mark("step_end")
        self.steps.append(self._cur)
        self._cur = None

    def summary(self) -> dict:
        """Mean milliseconds per step and phase over the recorded steps."""
        if not self.steps:
            return {}
        if self.cuda:
            torch.cuda.synchronize()
        tot = defaultdict(float)
        for marks in self.steps:
            for (a, ta), (_, tb) in zip(marks, marks[1:]):
                phase = _PHASE_OF.get(a)
                if phase is None:
                    continue
                tot[phase] += ta.elapsed_time(tb) if self.cuda else (tb - ta) * 1e3
        n = len(self.steps)
        return {p: tot[p] / n for p in PHASES}
