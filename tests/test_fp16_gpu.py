"""fp16 compute path (the reference's DDP/FSDP precision: autocast fp16 + GradScaler,
train_harness.py:334-335, 371-376) on the MI355X: every HIP kernel has an fp16 build
(csrc/build.py compiles each kernel file for bf16 and fp16), the engines keep fp32 masters and
scale the loss dynamically on the device (optim/amp.py)."""
import copy
import math

import pytest
import torch

import dltb
from dltb.models import build_model, get_model_config
from dltb.ops import ref
from dltb.ops._ext import ext
from dltb.ops.rng import StepSeed
from dltb.parallel import GraphedStep, ParamRuntime, engine_config, make_engine

from test_kernels_gpu import close, rnd, seed_obj

pytestmark = pytest.mark.gpu
F16 = torch.float16


@pytest.mark.parametrize("B,T,Hq,Hkv,D,causal,p", [(2, 256, 4, 4, 64, False, 0.1), (1, 256, 8, 2, 128, True, 0.0),
                                                   (2, 256, 4, 2, 64, True, 0.1)])
def test_attention_fp16(B, T, Hq, Hkv, D, causal, p):
    C = ext()
    W = (Hq + 2 * Hkv) * D
    qkv = rnd(B * T, W, dtype=F16)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    scale = 1.0 / math.sqrt(D)
    sd = seed_obj(42)
    amask = C.attn_mask(B, T, Hq, p, sd.device_tensor, 11, q) if p else None
    o, lse = C.attn_fwd(q, k, v, amask, B, T, Hq, Hkv, scale, causal, p)
    assert o.dtype == F16
    ro, rlse = ref.attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p, sd, 11)
    close(lse, rlse, 2e-3, 1e-3, "lse")
    close(o, ro, 5e-3, 1e-2, "O")                     # fp16: 3 more mantissa bits than bf16
    do = rnd(B * T, Hq * D, dtype=F16)
    dqkv, rdqkv = torch.empty_like(qkv), torch.empty_like(qkv)
    sl = lambda t: (t[:, :Hq * D], t[:, Hq * D:(Hq + Hkv) * D], t[:, (Hq + Hkv) * D:])
    C.attn_bwd(q, k, v, o, do, lse, amask, *sl(dqkv), B, T, Hq, Hkv, scale, causal, p)
    ref.attn_bwd(q, k, v, o, do, lse, *sl(rdqkv), B, T, Hq, Hkv, scale, causal, p, sd, 11)
    for name, a, b in zip("qkv", sl(dqkv), sl(rdqkv)):
        close(a, b, 2e-2, 2e-2, "d" + name)


def test_mixed_formats_in_one_call_are_rejected():
    C = ext()
    x = rnd(64, 256, dtype=F16)
    with pytest.raises(RuntimeError, match="all be bf16 or all fp16"):
        C.norm_fwd(x, None, torch.ones(256, device="cuda", dtype=torch.bfloat16),
                   torch.zeros(256, device="cuda", dtype=torch.bfloat16), 1e-5, False, 0.0, None, 0)


def test_tinygpt_fp16_hip_matches_cpu_reference():
    """Every kernel of the TinyGPT step in fp16 (embedding, LayerNorm fwd/bwd, attention, GELU,
    dropout, xent, column sums) against the fp32 CPU reference path with identical masks."""
    torch.manual_seed(0)
    cfg = get_model_config("A", 256)
    cfg.n_layer = 2
    m_cpu = build_model(cfg)
    m_gpu = copy.deepcopy(m_cpu).to("cuda", F16)
    m_cpu.rt, m_gpu.rt = ParamRuntime(), ParamRuntime()
    s_cpu, s_gpu = StepSeed(7), StepSeed(7, device="cuda")
    s_cpu.next(), s_gpu.next()
    m_cpu.rt.seed, m_gpu.rt.seed = s_cpu, s_gpu
    m_cpu.train(), m_gpu.train()
    idx = torch.randint(0, cfg.vocab_size, (2, cfg.block_size))
    _, l_cpu = m_cpu(idx, idx)
    _, l_gpu = m_gpu(idx.cuda(), idx.cuda())
    assert abs(l_cpu.item() - l_gpu.item()) < 5e-3 * abs(l_cpu.item())
    l_cpu.backward()
    l_gpu.backward(torch.tensor(1024.0, device="cuda"))     # a loss scale, as the engines seed it
    gp = dict(m_gpu.named_parameters())
    for n, p in m_cpu.named_parameters():
        g = gp[n].grad.float().cpu() / 1024.0
        r = ((g - p.grad).norm() / p.grad.norm().clamp(min=1e-12)).item()
        tol = 0.5 if n.endswith("in_proj_bias") else 3e-2
        assert r < tol, (n, r)


def _train(strategy, dtype, graphed=False, steps=12, semantics="reference"):
    torch.manual_seed(0)
    cfg = get_model_config("A", 256)
    cfg.n_layer = 2
    with torch.device("cuda"):
        model = build_model(cfg)
    eng = make_engine(model, engine_config(strategy, 4, semantics, compute_dtype=dtype), "cuda:0")
    eng.train()
    runner = GraphedStep(eng) if graphed else None
    g = torch.Generator(device="cuda").manual_seed(1)
    idx = torch.randint(0, cfg.vocab_size, (1, 256), device="cuda", generator=g)
    losses = []
    for _ in range(steps):
        if runner is not None:
            loss = runner(idx, idx)
        else:
            loss = eng(idx, idx)[1]
            eng.backward(loss)
            eng.step()
        losses.append(loss.item())
    return eng, losses


@pytest.mark.parametrize("strategy", ["ddp", "fsdp", "zero2", "zero3"])
def test_fp16_training_every_strategy(strategy):
    e16, l16 = _train(strategy, F16)
    e32, lbf = _train(strategy, torch.bfloat16)
    assert e16.flat_param.dtype == F16 if hasattr(e16, "flat_param") else e16.shard_buf.dtype == F16
    st = e16.scaler.stats()
    assert st["optimizer_steps_skipped"] == 0 and st["loss_scale"] == 2.0 ** 16
    assert st["optimizer_steps_taken"] == e16.opt_steps
    assert l16[-1] < l16[0]
    assert all(abs(a - b) < 3e-2 * abs(b) for a, b in zip(l16, lbf)), (l16, lbf)


def test_fp16_graph_replay_matches_eager():
    _, l0 = _train("ddp", F16, graphed=False)
    _, l1 = _train("ddp", F16, graphed=True)
    assert all(abs(a - b) < 1e-3 * abs(a) for a, b in zip(l0, l1)), (l0, l1)


def test_fp16_overflow_skips_on_device_and_backs_off():
    torch.manual_seed(0)
    cfg = get_model_config("A", 256)
    cfg.n_layer = 2
    with torch.device("cuda"):
        model = build_model(cfg)
    eng = make_engine(model, engine_config("ddp", 1, "reference", compute_dtype=F16), "cuda:0")
    eng.train()
    idx = torch.randint(0, cfg.vocab_size, (1, 256), device="cuda")
    master0 = eng.opt.master.clone()
    eng.scaler.state[0] = 2.0 ** 40                 # overflows the fp16 gradients (65504 max)
    loss = eng(idx, idx)[1]
    eng.backward(loss)
    eng.step()
    torch.cuda.synchronize()
    st = eng.scaler.stats()
    assert st["optimizer_steps_skipped"] == 1 and st["optimizer_steps_taken"] == 0
    assert st["loss_scale"] == 2.0 ** 39
    assert torch.equal(eng.opt.master, master0)      # AdamW returned at once: nothing moved
    eng.scaler.state[0] = 2.0 ** 12
    for _ in range(2):
        loss = eng(idx, idx)[1]
        eng.backward(loss)
        eng.step()
    st = eng.scaler.stats()
    assert st["optimizer_steps_taken"] == 2 and not torch.equal(eng.opt.master, master0)
