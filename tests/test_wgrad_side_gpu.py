"""World-1 batched dW on a side stream (DLTB_WGRAD_SIDE, parallel/replicated.py): the window's
weight gradients of every G finished blocks are issued beside the rest of the backward; the
training curve must match the single end-of-backward batch."""
import pytest
import torch

import dltb  # noqa: F401


def _losses(monkeypatch, side, windows=3):
    from dltb.models import build_model, get_model_config
    from dltb.parallel import engine_config, make_engine
    monkeypatch.delenv("DLTB_COMM", raising=False)
    monkeypatch.setenv("DLTB_WGRAD_SIDE", str(side))
    torch.manual_seed(0)
    cfg = get_model_config("A", 256)
    cfg.n_layer = 6
    dev = torch.device("cuda", 0)
    with torch.device(dev):
        model = build_model(cfg)
    eng = make_engine(model, engine_config("zero2", 4), dev)
    assert eng._side_group == side
    eng.train()
    g = torch.Generator().manual_seed(5)
    out = []
    for _ in range(4 * windows):
        x = torch.randint(0, cfg.vocab_size, (1, 256), generator=g).to(dev)
        loss = eng(x, x)[1]
        eng.backward(loss)
        eng.step()
        out.append(float(loss.item()))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("side", [2, 4])
def test_side_stream_wgrad_matches_single_batch(side, monkeypatch):
    base = _losses(monkeypatch, 0)
    got = _losses(monkeypatch, side)
    assert base[:4] == got[:4]                     # the first window's forwards see the same weights
    for a, b in zip(base, got):
        assert abs(a - b) < 2e-3 * a, (base, got)
