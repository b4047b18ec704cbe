"""Dynamic loss scaling (fp16 path of the reference's DDP/FSDP: train_harness.py:334-335, 371-376)
against torch.amp.GradScaler semantics, and engine-level behaviour on the CPU."""
import math

import pytest
import torch

import dltb
from dltb.models import build_model, get_model_config
from dltb.optim.amp import DynamicLossScaler
from dltb.parallel import engine_config, make_engine


def test_scaler_matches_torch_gradscaler():
    interval = 3
    ref = torch.amp.GradScaler("cpu", init_scale=1024.0, growth_factor=2.0, backoff_factor=0.5,
                               growth_interval=interval)
    p = torch.nn.Parameter(torch.ones(4))
    opt = torch.optim.SGD([p], lr=0.1)
    mine = DynamicLossScaler("cpu", init_scale=1024.0, growth_interval=interval)
    coef, nrm = torch.zeros(1), torch.zeros(1)
    pattern = [False, False, True, False, False, False, False, True, True, False, False, False, False]
    for bad in pattern:
        g = torch.full((4,), 0.5)
        ref.scale(torch.ones(()))              # (GradScaler creates its scale lazily)
        S = ref.get_scale()
        assert mine.scale() == S
        p.grad = g * S
        if bad:
            p.grad[1] = float("inf")
        nsq = torch.tensor([float((p.grad.double() ** 2).sum())])     # before unscale_ rewrites p.grad
        before = p.detach().clone()
        ref.step(opt)
        ref.update()
        ref_skipped = torch.equal(before, p.detach())
        mine.step(nsq, coef, nrm, None, 0.0, 1.0, (0.9, 0.999))
        assert mine.last_skipped == ref_skipped == bad
        if not bad:
            assert math.isclose(float(coef), 1.0 / S) and math.isclose(float(nrm), 1.0, rel_tol=1e-6)
    assert mine.scale() == ref.get_scale()
    st = mine.stats()
    assert st["optimizer_steps_skipped"] == sum(pattern) and st["optimizer_steps_taken"] == len(pattern) - sum(pattern)


def _train(strategy, dtype, steps=6, inject=None):
    torch.manual_seed(0)
    cfg = get_model_config("tiny", 32, dropout=0.0)
    model = build_model(cfg)
    ecfg = engine_config(strategy, 2, "uniform", compute_dtype=dtype)
    eng = make_engine(model, ecfg, "cpu")
    eng.train()
    g = torch.Generator().manual_seed(1)
    losses = []
    for k in range(steps):
        idx = torch.randint(0, cfg.vocab_size, (2, 32), generator=g)
        loss = eng(idx, idx)[1]
        eng.backward(loss)
        if inject is not None and k == inject:
            eng._owner_grad()[7] = float("inf")
        eng.step()
        losses.append(float(loss.detach()))
    return eng, losses


@pytest.mark.parametrize("strategy", ["ddp", "zero2"])
def test_loss_scaling_is_exact_with_power_of_two_scale(strategy):
    e32, l32 = _train(strategy, torch.float32)
    e16, l16 = _train(strategy, torch.float16)           # CPU computes fp32; the scaler still runs
    assert e16.scaler is not None and e32.scaler is None
    assert l16 == l32
    s32, s16 = e32.full_state_dict(), e16.full_state_dict()
    for k in s32:
        assert torch.allclose(s32[k], s16[k], rtol=1e-5, atol=1e-7), k
    assert e16.scaler.stats()["optimizer_steps_taken"] == 3


def test_inf_gradient_skips_the_step_and_backs_off():
    eng, _ = _train("ddp", torch.float16, steps=2)
    before = eng.full_state_dict()
    S = eng.scaler.scale()
    eng2, _ = _train("ddp", torch.float16, steps=2, inject=1)   # inf in the 2nd micro-step's window sum
    st = eng2.scaler.stats()
    assert st["optimizer_steps_skipped"] == 1 and st["optimizer_steps_taken"] == 0
    assert eng2.scaler.scale() == S / 2
    torch.manual_seed(0)
    init = build_model(get_model_config("tiny", 32, dropout=0.0))
    after = eng2.full_state_dict()
    for n, p in init.named_parameters():
        assert torch.equal(after[n], p.detach().float()), n      # skipped: master never moved
    assert eng.scaler.stats()["optimizer_steps_taken"] == 1 and before.keys() == after.keys()
