"""Mistral-shape decoder on the MI355X: HIP path (RMSNorm, RoPE, causal GQA flash attention at
head_dim 128, SwiGLU, xent kernels + hipBLASLt) against the fp32 CPU reference path of the same
fused Functions, and ZeRO-3 / FSDP training steps."""
import copy

import pytest
import torch

import dltb
from dltb.models import build_model, get_model_config
from dltb.parallel import ParamRuntime, engine_config, make_engine

pytestmark = pytest.mark.gpu


def _m7b_slice(T=256, layers=2):
    """Full Mistral-7B width (d4096, 32q/8kv heads x 128, ffn 14336) with fewer layers."""
    c = get_model_config("M7B", T)
    c.n_layer = layers
    return c


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm().clamp(min=1e-12)).item()


@pytest.mark.parametrize("tier", ["mtiny", "M7B"])
def test_mistral_hip_matches_cpu_reference(tier):
    torch.manual_seed(0)
    cfg = get_model_config("mtiny", 256) if tier == "mtiny" else _m7b_slice(256, 1)
    m_cpu = build_model(cfg)
    m_gpu = copy.deepcopy(m_cpu).to("cuda", torch.bfloat16)
    m_cpu.rt, m_gpu.rt = ParamRuntime(), ParamRuntime()
    idx = torch.randint(0, cfg.vocab_size, (2, 256))
    tgt = idx.roll(-1, 1)
    _, l_cpu = m_cpu(idx, tgt)
    _, l_gpu = m_gpu(idx.cuda(), tgt.cuda())
    assert abs(l_cpu.item() - l_gpu.item()) < 1e-2 * abs(l_cpu.item())
    l_cpu.backward()
    l_gpu.backward()
    gp = dict(m_gpu.named_parameters())
    for n, p in m_cpu.named_parameters():
        r = rel(gp[n].grad, p.grad)
        assert r < 6e-2, (n, r)


@pytest.mark.parametrize("strategy", ["zero3", "fsdp", "zero2"])
def test_mistral_engine_steps(strategy):
    torch.manual_seed(0)
    cfg = _m7b_slice(512, 2)
    with torch.device("cuda"):
        model = build_model(cfg)
    eng = make_engine(model, engine_config(strategy, 2, "reference"), "cuda:0")
    eng.train()
    idx = torch.randint(0, cfg.vocab_size, (1, 512), device="cuda")
    losses = []
    for _ in range(6):
        loss = eng(idx, idx.roll(-1, 1))[1]
        eng.backward(loss)
        eng.step()
        losses.append(loss.item())
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0], losses
