"""Side-stream scheduling of parameter-gradient work.

A transformer block's backward is two independent dependency chains:

* the activation-gradient chain (dX GEMMs, norm dx, dropout masks, attention dK/dV) that the next
  block's backward waits for — the critical path;
* the parameter-gradient work (dW GEMMs, bias / gamma / beta column reductions, attention dQ's
  sibling) whose results only land in the flat gradient buffers.

At TinyGPT's per-GPU size (2048 tokens) each of these kernels under-fills the 256 CUs of an
MI355X, so the engine runs the second chain on a side HIP stream concurrently with the first.
``fork`` makes the side stream wait for everything queued on the main stream so far, runs the body
on the side stream and marks the main-stream tensors it reads (``record_stream``) so the caching
allocator cannot recycle them early; ``join`` makes the main stream wait for the side stream (done
before a unit's gradients are handed to the collectives).  On the CPU everything runs inline.
Measured on MI355X (TinyGPT-A, ZeRO-2, 1 GPU): eager, OFF 10.7 ms/step vs ON 18.1 ms/step (the
~10 cross-stream event waits per layer sit on the host's critical path).  Re-measured with the
micro-step replayed as a HIP graph (the waits become graph edges; scripts/ab_bench.sh,
profiles/ab_side_streams_graphs_1gpu.jsonl): OFF 8.97 ms, ``wgrad`` 10.15 ms, ``attn`` 9.44 ms, all kinds 10.32 ms --
two concurrent kernels of this size slow each other down by more than the idle CUs they fill
(hipBLASLt solutions are tuned for a whole chip; dQ beside dK/dV contends for LDS and L2).  The
overlap is therefore OFF by default; ``DLTB_SIDE_STREAM=1|wgrad|attn`` enables it.
"""
import contextlib
import os

import torch

_SIDE = {}


def _side_stream(device):
    idx = torch.device(device).index or 0
    s = _SIDE.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _SIDE[idx] = s
    return s


class GradStreams:
    """``DLTB_SIDE_STREAM``: 0 (off), 1 (every kind), ``wgrad`` (weight-gradient GEMMs only) or
    ``attn`` (attention dQ beside dK/dV only)."""

    def __init__(self, device, enabled=None):
        device = torch.device(device)
        mode = os.environ.get("DLTB_SIDE_STREAM", "0") if enabled is None else ("1" if enabled else "0")
        self.enabled = mode != "0" and device.type == "cuda"
        self.wgrad = mode in ("1", "wgrad")
        self.attn = mode in ("1", "attn")
        if self.enabled:
            self.main = torch.cuda.current_stream(device)
            self.side = _side_stream(device)

    @contextlib.contextmanager
    def fork(self, *tensors):
        if not self.enabled:
            yield
            return
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            yield
        for t in tensors:
            if t is not None:
                t.record_stream(self.side)

    def join(self):
        if self.enabled:
            self.main.wait_stream(self.side)


class _Inline:
    enabled = False
    wgrad = attn = False

    @contextlib.contextmanager
    def fork(self, *tensors):
        yield

    def join(self):
        pass


INLINE = _Inline()
