"""Deferred / batched weight gradients (parallel/wgrad.py) on the CPU.

* ``strided_batch`` recognises equally spaced matrices of one storage (and only those);
* ``WgradQueue.flush`` gives the same dW as one GEMM per block, in overwrite and accumulate mode,
  batched when the slots and operands are layer-strided and one GEMM per item otherwise;
* the engines batch TinyGPT's dW products end to end (every strategy at world size 1).
"""
import pytest
import torch

import dltb  # noqa: F401
from dltb.models import get_model_config
from dltb.models.tinygpt import TinyGPT
from dltb.parallel import engine_config, make_engine
from dltb.parallel.runtime import Unit
from dltb.parallel.wgrad import WgradQueue, strided_batch


def test_strided_batch_detects_equal_spacing():
    flat = torch.arange(10 * 64, dtype=torch.float32)
    ts = [flat[i * 96:i * 96 + 32].view(4, 8) for i in range(5)]       # stride 96 > 32 elements
    b = strided_batch(ts, out=True)
    assert b is not None and b.shape == (5, 4, 8) and b.stride() == (96, 8, 1)
    for i, t in enumerate(ts):
        assert torch.equal(b[i], t)
    assert strided_batch([ts[0], ts[2], ts[3]]) is None                    # not equally spaced
    assert strided_batch([ts[1], ts[0]]) is None                           # descending
    other = torch.zeros(64)[:32].view(4, 8)
    assert strided_batch([ts[0], other]) is None                           # another storage
    over = [flat[i * 16:i * 16 + 32].view(4, 8) for i in range(3)]         # overlapping outputs
    assert strided_batch(over, out=True) is None and strided_batch(over) is not None


@pytest.mark.parametrize("layer_strided", [True, False])
@pytest.mark.parametrize("accumulate", [False, True])
def test_queue_flush_matches_per_block_gemms(layer_strided, accumulate):
    torch.manual_seed(0)
    L, M, N, K, gap = 4, 16, 6, 5, 7
    units = [Unit(f"b{i}", [(f"w{i}", torch.nn.Parameter(torch.zeros(N, K)))], i) for i in range(L)]
    grad = torch.randn(L * (N * K + gap))
    slots = [grad[i * (N * K + gap):i * (N * K + gap) + N * K].view(N, K) for i in range(L)]
    if layer_strided:
        dyb, xb = torch.randn(L, M, N), torch.randn(L, M, K)
        dys, xs = [dyb[i] for i in range(L)], [xb[i] for i in range(L)]
    else:
        dys, xs = [torch.randn(M, N) for _ in range(L)], [torch.randn(M, K) for _ in range(L)]
    expect = [(s.clone() if accumulate else torch.zeros_like(s)) + dy.t() @ x for s, dy, x in zip(slots, dys, xs)]
    q = WgradQueue()
    for u, s, dy, x in zip(reversed(units), reversed(slots), reversed(dys), reversed(xs)):
        q.add(u, 0, dy, x, s, accumulate)                   # queued in backward order
    q.flush(units[:2])                                      # a bucket's worth first
    q.flush()
    assert len(q) == 0
    for s, e in zip(slots, expect):
        assert torch.allclose(s, e, atol=1e-5)
    if layer_strided:
        assert q.batched_calls == 2 and q.single_calls == 0
    else:
        assert q.batched_calls == 0 and q.single_calls == L


@pytest.mark.parametrize("strategy", ["ddp", "zero2", "zero3", "fsdp"])
def test_engines_batch_tinygpt_wgrads(strategy):
    """Batched (default) and per-block weight gradients train identically."""
    out = []
    for batch in (True, False):
        torch.manual_seed(0)
        m = TinyGPT(get_model_config("tiny", 16, dropout=0.0))
        cfg = engine_config(strategy, 2, "uniform")
        cfg.extra["batch_wgrad"] = batch
        e = make_engine(m, cfg, "cpu")
        e.train()
        x = torch.randint(0, 128, (2, 16), generator=torch.Generator().manual_seed(1))
        for _ in range(4):
            loss = e(x, x)[1]
            e.backward(loss)
            e.step()
        assert (e._wq.batched_calls > 0 and e._wq.single_calls == 0) if batch else e._wq.batched_calls == 0
        out.append(e.full_state_dict())
    for n in out[0]:
        assert torch.allclose(out[0][n], out[1][n], atol=2e-5), n     # GEMM summation order only


@pytest.mark.parametrize("strategy,stage", [("zero2", None), ("zero2", 1), ("ddp", None)])
def test_window_wide_wgrad_matches_per_micro(strategy, stage):
    """World 1 (and window-reduced paths): the window's dW as ONE product over all its micro-steps'
    tokens (layer buffers hold accum x tokens rows) trains like per-micro-step products."""
    out = []
    for window in (True, False):
        torch.manual_seed(0)
        m = TinyGPT(get_model_config("tiny", 16, dropout=0.0))
        cfg = engine_config(strategy, 3, "uniform")
        cfg.extra["window_wgrad"] = window
        if stage is not None:
            cfg.zero_stage = stage
        e = make_engine(m, cfg, "cpu")
        assert e._window_wgrad == window
        e.train()
        g = torch.Generator().manual_seed(1)
        for _ in range(6):
            x = torch.randint(0, 128, (2, 16), generator=g)
            loss = e(x, x)[1]
            e.backward(loss)
            e.step()
        rows = m._lbufs.h1.shape[1]
        assert rows == (3 * 2 * 16 if window else 2 * 16)
        out.append(e.full_state_dict())
    for n in out[0]:
        assert torch.allclose(out[0][n], out[1][n], atol=2e-5), n
