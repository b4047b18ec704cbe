"""Fused Mistral-shape decoder (RMSNorm, RoPE, causal GQA attention, SwiGLU, untied head; manual
per-layer backward) vs the stock-module oracle in fp64 on the CPU."""
import pytest
import torch

import dltb
from dltb.models import build_model, get_model_config
from dltb.models.mistral import MistralLM
from dltb.models.oracle import OracleMistral
from dltb.parallel import make_engine, engine_config


def _pair(T=32):
    cfg = get_model_config("mtiny", T)
    torch.manual_seed(0)
    m = MistralLM(cfg).double()
    o = OracleMistral(cfg).double()
    o.load_state_dict(m.state_dict())
    return cfg, m, o


def test_m7b_shape_and_names():
    cfg = get_model_config("M7B", 4096)
    assert cfg.num_params() == 7_241_732_096
    assert (cfg.head_dim, cfg.kv_heads, cfg.ffn_dim) == (128, 8, 14336)
    cfg, m, o = _pair()
    assert isinstance(build_model(cfg), MistralLM)
    assert list(m.state_dict().keys()) == list(o.state_dict().keys())
    assert m.num_params() == cfg.num_params()
    assert m.lm_head.weight is not m.model.embed_tokens.weight
    names = [n for u in m.units() for n in u.names]
    assert names == list(dict(m.named_parameters()).keys())


def test_forward_backward_matches_oracle():
    cfg, m, o = _pair()
    idx = torch.randint(0, cfg.vocab_size, (2, 32))
    tgt = idx.roll(-1, 1)
    tgt[1, -5:] = -1
    _, loss = m(idx, tgt)
    _, lo = o(idx, tgt)
    assert torch.allclose(loss, lo, atol=1e-10), (loss.item(), lo.item())
    loss.backward()
    lo.backward()
    got = dict(m.named_parameters())
    for name, p in o.named_parameters():
        assert got[name].grad is not None, name
        assert torch.allclose(got[name].grad, p.grad, atol=1e-9, rtol=1e-7), name


def test_logits_match_oracle():
    cfg, m, o = _pair(T=16)
    idx = torch.randint(0, cfg.vocab_size, (2, 16))
    lg, _ = m(idx)
    lo, _ = o(idx)
    assert torch.allclose(lg, lo, atol=1e-10)


def _train(strategy, batches, accum):
    cfg = get_model_config("mtiny", 32)
    torch.manual_seed(0)
    m = MistralLM(cfg)
    ecfg = engine_config(strategy, accum, "reference", bucket_mb=0.05)
    ecfg.lr = 1e-3
    eng = make_engine(m, ecfg, "cpu")
    eng.train()
    for b in batches:
        micro = b.shape[0] // accum
        for a in range(accum):
            x = b[a * micro:(a + 1) * micro]
            eng.backward(eng(x, x.roll(-1, 1))[1])
            eng.step()
    return eng.full_state_dict()


def _batches(n=3):
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, 256, (2, 32), generator=g) for _ in range(n)]


def test_ddp_engine_matches_torch_adamw_on_oracle():
    batches = _batches()
    sd = _train("ddp", batches, 1)
    cfg = get_model_config("mtiny", 32)
    torch.manual_seed(0)
    init = MistralLM(cfg).state_dict()
    o = OracleMistral(cfg)
    o.load_state_dict(init)
    opt = torch.optim.AdamW(o.parameters(), lr=1e-3, weight_decay=0.01)
    for b in batches:
        o(b, b.roll(-1, 1))[1].backward()
        opt.step()
        opt.zero_grad()
    for n, p in o.named_parameters():
        # Adam normalises each element's update, so entries whose true gradient is ~0 turn rounding
        # noise into up to +-lr steps; require 99.9 % of entries tight and bound the rest.
        d = (sd[n].float() - p.detach()).abs()
        assert (d > 2e-5).float().mean() < 1e-3 and d.max() < 3e-4, (n, d.max().item())


@pytest.mark.parametrize("strategy", ["zero3", "fsdp"])
def test_sharded_engines_agree_on_mistral(strategy):
    batches = _batches()
    accum = 2 if strategy == "zero3" else 1
    base = _train("zero2" if strategy == "zero3" else "ddp", batches, accum)
    got = _train(strategy, batches, accum)
    for n in base:
        assert torch.allclose(got[n].float(), base[n].float(), atol=1e-6), (strategy, n)
