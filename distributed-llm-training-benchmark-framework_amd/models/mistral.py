"""Mistral-7B-shape decoder (BASELINE.json config #5: ZeRO-3 bf16 on 8x MI355X).

Not part of the reference (it only names a Mistral image, scripts/build.sh:4, and a 7B sizing note,
docs/ARCHITECTURE.md:452-460); built from the same fused per-unit Functions as TinyGPT so every
strategy engine handles it unchanged:

    x = embed_tokens[idx]
    per layer:  h1 = RMSNorm(x); qkv = h1 Wqkv^T (fused q|k|v, GQA: 32 q / 8 kv heads x 128);
                RoPE(q, k) in place; o = causal FlashAttn(qkv); x1 = x + o Wo^T;
                h2 = RMSNorm(x1) (fused with the residual add); gu = h2 Wgu^T (gate|up);
                x2 = x1 + SiLU(gate) * up Wd^T
    logits = RMSNorm(x) lm_head^T (untied), softmax-xent fused

Parameter names follow the common fused-projection layout:
``model.embed_tokens.weight``, ``model.layers.{i}.{input_layernorm,post_attention_layernorm}.weight``,
``model.layers.{i}.self_attn.{qkv_proj,o_proj}.weight``, ``model.layers.{i}.mlp.{gate_up_proj,down_proj}.weight``,
``model.norm.weight``, ``lm_head.weight``.  RMSNorm / RoPE / SwiGLU / causal-GQA attention / xent
run as dltb HIP kernels on the GPU.
"""
import math

import torch
import torch.nn as nn

from ..ops import functional as F_
from ..ops import ref
from ..parallel.runtime import EAGER, Unit
from .config import ModelConfig


class _RMSNorm(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))


class _Attn(nn.Module):
    def __init__(self, d, kvd):
        super().__init__()
        self.qkv_proj = nn.Linear(d, d + 2 * kvd, bias=False)
        self.o_proj = nn.Linear(d, d, bias=False)


class _MLP(nn.Module):
    def __init__(self, d, f):
        super().__init__()
        self.gate_up_proj = nn.Linear(d, 2 * f, bias=False)
        self.down_proj = nn.Linear(f, d, bias=False)


class MistralLayer(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        d = cfg.n_embd
        self.input_layernorm = _RMSNorm(d)
        self.self_attn = _Attn(d, cfg.kv_heads * cfg.head_dim)
        self.post_attention_layernorm = _RMSNorm(d)
        self.mlp = _MLP(d, cfg.ffn_dim)

    def param_list(self):
        return [("input_layernorm.weight", self.input_layernorm.weight),
                ("self_attn.qkv_proj.weight", self.self_attn.qkv_proj.weight),
                ("self_attn.o_proj.weight", self.self_attn.o_proj.weight),
                ("post_attention_layernorm.weight", self.post_attention_layernorm.weight),
                ("mlp.gate_up_proj.weight", self.mlp.gate_up_proj.weight),
                ("mlp.down_proj.weight", self.mlp.down_proj.weight)]


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, idx, model):
        rt, unit = model.rt, model.unit_embed
        (wte,) = rt.acquire(unit)
        x = wte.index_select(0, idx.reshape(-1))
        rt.release_forward(unit)
        ctx.model, ctx.idx = model, idx
        return x

    @staticmethod
    def backward(ctx, dx):
        model = ctx.model
        rt, unit = model.rt, model.unit_embed
        rt.acquire_backward(unit)
        rt.embedding_backward((unit, 0), None, dx.contiguous(), ctx.idx, 0.0, rt.seed, 0)
        rt.grads_ready(unit)
        rt.release_backward(unit)
        return None, None, None


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, i):
        rt, unit = model.rt, model.unit_blocks[i]
        (w_in, wqkv, wo, w_post, wgu, wd) = rt.acquire(unit)
        cfg = model.cfg
        B, T = model._cur_bt
        Hq, Hkv, D = cfg.n_head, cfg.kv_heads, cfg.head_dim
        cos, sin = model.rope(x.device, T)
        _, h1, _, rstd1 = F_.norm_fwd(x, None, w_in, None, cfg.norm_eps, True)
        qkv = F_.linear_fwd(h1, wqkv)
        F_.rope_(qkv, cos, sin, T, Hq + Hkv, D, False)
        qd, kd = Hq * D, Hkv * D
        o, lse, aux = F_.attn_fwd(qkv[:, :qd], qkv[:, qd:qd + kd], qkv[:, qd + kd:], B, T, Hq, Hkv,
                                  1.0 / math.sqrt(D), True, 0.0, rt.seed, 0)
        a = F_.linear_fwd(o, wo)
        x1, h2, _, rstd2 = F_.norm_fwd(x, a, w_post, None, cfg.norm_eps, True)
        gu = F_.linear_fwd(h2, wgu)
        hh = F_.swiglu_fwd(gu)
        m = F_.linear_fwd(hh, wd)
        x2 = F_.dropout(x1, m, 0.0, rt.seed, 0)
        rt.release_forward(unit)
        ctx.model, ctx.i = model, i
        ctx.saved = (x, h1, rstd1, qkv, o, lse, aux, x1, h2, rstd2, gu, hh)
        return x2

    @staticmethod
    def backward(ctx, dx2):
        model, i = ctx.model, ctx.i
        rt, unit = model.rt, model.unit_blocks[i]
        (x, h1, rstd1, qkv, o, lse, aux, x1, h2, rstd2, gu, hh) = ctx.saved
        ctx.saved = None
        (w_in, wqkv, wo, w_post, wgu, wd) = rt.acquire_backward(unit)
        cfg = model.cfg
        B, T = model._cur_bt
        Hq, Hkv, D = cfg.n_head, cfg.kv_heads, cfg.head_dim
        cos, sin = model.rope(dx2.device, T)
        dx2 = dx2.contiguous()
        s = [rt.grad_slot(unit, j) for j in range(6)]
        F_.linear_wgrad(dx2, hh, s[5][0], None, s[5][1])
        dhh = F_.linear_dgrad(dx2, wd, rt.weight_t(unit, 5, wd))
        dgu = F_.swiglu_bwd(dhh, gu)
        F_.linear_wgrad(dgu, h2, s[4][0], None, s[4][1])
        dh2 = F_.linear_dgrad(dgu, wgu, rt.weight_t(unit, 4, wgu))
        shared = rt.grad_reducer()
        red = shared if shared is not None else F_.GradReducer()
        dx1 = F_.norm_bwd(dh2, x1, w_post, None, rstd2, dx2, s[3][0], None, s[3][1], True, red=red)
        F_.linear_wgrad(dx1, o, s[2][0], None, s[2][1])
        do = F_.linear_dgrad(dx1, wo, rt.weight_t(unit, 2, wo))
        qd, kd = Hq * D, Hkv * D
        dqkv = torch.empty_like(qkv)
        F_.attn_bwd(qkv[:, :qd], qkv[:, qd:qd + kd], qkv[:, qd + kd:], o, do, lse, aux,
                    dqkv[:, :qd], dqkv[:, qd:qd + kd], dqkv[:, qd + kd:], B, T, Hq, Hkv,
                    1.0 / math.sqrt(D), True, 0.0, rt.seed, 0)
        F_.rope_(dqkv, cos, sin, T, Hq + Hkv, D, True)      # RoPE is orthogonal: grad = R(-theta) g
        F_.linear_wgrad(dqkv, h1, s[1][0], None, s[1][1])
        dh1 = F_.linear_dgrad(dqkv, wqkv, rt.weight_t(unit, 1, wqkv))
        dx = F_.norm_bwd(dh1, x, w_in, None, rstd1, dx1, s[0][0], None, s[0][1], True, red=red)
        if shared is None:
            red.flush()
        rt.grads_ready(unit)
        rt.release_backward(unit)
        return dx, None, None


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, targets, return_logits):
        rt, unit = model.rt, model.unit_head
        w_norm, w_head = rt.acquire(unit)
        _, h, _, rstd = F_.norm_fwd(x, None, w_norm, None, model.cfg.norm_eps, True)
        logits = F_.linear_fwd(h, w_head)
        if targets is None:
            rt.release_forward(unit)
            ctx.mark_non_differentiable(logits)
            ctx.no_loss = True
            return logits, logits.new_zeros(())
        kept = logits.clone() if return_logits else None
        tg = targets.reshape(-1)
        loss_rows = F_.xent_fwd_bwd_(logits, tg, -1)
        lc = F_.xent_mean(loss_rows, tg, -1)          # (mean, count) on the device
        loss, count = lc[0], lc[1:2]
        rt.release_forward(unit)
        ctx.model, ctx.no_loss = model, False
        ctx.saved = (x, h, rstd, logits, count)
        out_logits = kept if kept is not None else logits.new_empty(0)
        ctx.mark_non_differentiable(out_logits)
        return out_logits, loss

    @staticmethod
    def backward(ctx, dlogits_unused, dloss):
        if ctx.no_loss:
            return None, None, None, None
        model = ctx.model
        rt, unit = model.rt, model.unit_head
        (x, h, rstd, dl, count) = ctx.saved
        ctx.saved = None
        w_norm, w_head = rt.acquire_backward(unit)
        dwh, acc_h = rt.grad_slot(unit, 1)
        hs, g = F_.scale_by(h, dloss, count)                      # g = dloss / count (device)
        F_.linear_wgrad(dl, hs, dwh, None, acc_h)
        dh = F_.head_dgrad(dl, w_head, rt.weight_t(unit, 1, w_head), g)
        gw, acc = rt.grad_slot(unit, 0)
        dx = F_.norm_bwd(dh, x, w_norm, None, rstd, None, gw, None, acc, True)
        rt.grads_ready(unit)
        rt.release_backward(unit)
        return dx, None, None, None


class MistralLM(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        assert cfg.n_embd % cfg.n_head == 0 and cfg.n_head % cfg.kv_heads == 0
        self.cfg = cfg
        self.model = nn.Module()
        self.model.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.n_embd)
        self.model.layers = nn.ModuleList([MistralLayer(cfg) for _ in range(cfg.n_layer)])
        self.model.norm = _RMSNorm(cfg.n_embd)
        self.lm_head = nn.Linear(cfg.n_embd, cfg.vocab_size, bias=False)
        for mod in self.modules():
            if isinstance(mod, (nn.Linear, nn.Embedding)):
                nn.init.normal_(mod.weight, mean=0.0, std=0.02)
        self.rt = EAGER
        self.drop_p = 0.0
        self._rope = {}
        self.unit_embed = Unit("embed", [("model.embed_tokens.weight", self.model.embed_tokens.weight)], 0)
        self.unit_blocks = [Unit(f"layers.{i}", [(f"model.layers.{i}.{n}", p) for n, p in layer.param_list()], i + 1)
                            for i, layer in enumerate(self.model.layers)]
        self.unit_head = Unit("head", [("model.norm.weight", self.model.norm.weight),
                                       ("lm_head.weight", self.lm_head.weight)], len(self.unit_blocks) + 1)

    def units(self):
        return [self.unit_embed] + self.unit_blocks + [self.unit_head]

    def rope(self, device, T):
        key = (str(device), T)
        if key not in self._rope:
            self._rope[key] = ref.rope_tables(T, self.cfg.head_dim, self.cfg.rope_theta, device)
        return self._rope[key]

    def num_params(self):
        return sum(p.numel() for p in self.parameters())

    def forward(self, idx, targets=None, return_logits=False):
        B, T = idx.shape
        assert T <= self.cfg.block_size
        self._cur_bt = (B, T)
        anchor = torch.empty((), requires_grad=True)
        x = _EmbedFn.apply(anchor, idx, self)
        for i in range(len(self.unit_blocks)):
            x = _LayerFn.apply(x, self, i)
        logits, loss = _HeadFn.apply(x, self, targets, return_logits)
        if targets is None:
            return logits.view(B, T, -1), None
        return (logits.view(B, T, -1) if return_logits else None), loss
