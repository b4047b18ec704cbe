"""Fused TinyGPT (manual per-block backward, eager runtime, CPU/fp64) vs the stock-module oracle."""
import copy

import pytest
import torch

import dltb
from dltb.models import get_model_config
from dltb.models.oracle import OracleTinyGPT
from dltb.models.tinygpt import TinyGPT
from dltb.ops.rng import StepSeed


def _pair(dropout=0.0, T=16):
    cfg = get_model_config("tiny", T, dropout=dropout)
    torch.manual_seed(0)
    m = TinyGPT(cfg).double()
    o = OracleTinyGPT(cfg).double()
    o.load_state_dict(m.state_dict())
    return cfg, m, o


def test_param_names_and_count_match_reference_layout():
    cfg = get_model_config("A", 2048)
    assert cfg.num_params() == 236_406_784
    cfg, m, o = _pair()
    assert list(m.state_dict().keys()) == list(o.state_dict().keys())
    assert m.num_params() == cfg.num_params()
    assert m.transformer["wte"].weight is m.lm_head.weight


def test_forward_backward_matches_oracle():
    cfg, m, o = _pair()
    m.train(), o.train()
    idx = torch.randint(0, cfg.vocab_size, (3, 16))
    tgt = idx.clone()
    tgt[0, :3] = -1
    _, loss = m(idx, tgt)
    _, lo = o(idx, tgt)
    assert torch.allclose(loss, lo, atol=1e-10), (loss.item(), lo.item())
    loss.backward()
    lo.backward()
    got = dict(m.named_parameters())
    for name, p in o.named_parameters():
        assert got[name].grad is not None, name
        assert torch.allclose(got[name].grad, p.grad, atol=1e-9, rtol=1e-7), name


def test_eval_logits_match_oracle():
    cfg, m, o = _pair()
    m.eval(), o.eval()
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    lg, _ = m(idx)
    lo, _ = o(idx)
    assert torch.allclose(lg, lo, atol=1e-10)
    lg2, loss = m(idx, idx, return_logits=True)
    assert torch.allclose(lg2, lo, atol=1e-10)


def test_dropout_is_deterministic_per_seed_and_changes_loss():
    cfg, m, _ = _pair(dropout=0.1)
    m.train()
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    s = StepSeed(1)
    m.rt.seed = s
    try:
        s.next()
        val = s.value
        l1 = m(idx, idx)[1].item()
        s.value = val
        l2 = m(idx, idx)[1].item()
        s.next()
        l3 = m(idx, idx)[1].item()
        m.eval()
        l0 = m(idx, idx)[1].item()
    finally:
        m.rt.seed = None
    assert l1 == l2
    assert l1 != l3 and l1 != l0


def test_dropout_grads_match_autograd_of_masked_oracle():
    """Backward through all three dropout sites equals finite differences of the fused forward."""
    cfg, m, _ = _pair(dropout=0.2, T=8)
    m.train()
    idx = torch.randint(0, cfg.vocab_size, (1, 8))
    s = StepSeed(5)
    s.next()
    m.rt.seed = s
    try:
        _, loss = m(idx, idx)
        loss.backward()
        p = m.transformer["h"][0].mlp[0].weight
        g = p.grad[3, 5].item()
        eps = 1e-6
        with torch.no_grad():
            p[3, 5] += eps
            lp = m(idx, idx)[1].item()
            p[3, 5] -= 2 * eps
            lm = m(idx, idx)[1].item()
            p[3, 5] += eps
        assert abs((lp - lm) / (2 * eps) - g) < 1e-6
    finally:
        m.rt.seed = None
