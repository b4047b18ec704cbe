"""Plain-torch oracles of the model families (autograd through stock nn modules).

``OracleTinyGPT`` follows the reference architecture of ``train_harness.py:36-131`` op for op —
``nn.MultiheadAttention`` with no mask, pre-LN residual blocks, exact GELU, tied head — so the
fused TinyGPT can be checked against it parameter-for-parameter (same state-dict names).  It is
used only by tests and for parity checks; it is not a training path.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .config import ModelConfig


class _OracleBlock(nn.Module):
    def __init__(self, d, h, p):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d)
        self.attn = nn.MultiheadAttention(d, h, dropout=p, batch_first=True)
        self.ln_2 = nn.LayerNorm(d)
        self.mlp = nn.Sequential(nn.Linear(d, 4 * d), nn.GELU(), nn.Linear(4 * d, d), nn.Dropout(p))

    def forward(self, x):
        a = self.ln_1(x)
        y, _ = self.attn(a, a, a, need_weights=False)
        x = x + y
        return x + self.mlp(self.ln_2(x))


class OracleTinyGPT(nn.Module):
    def __init__(self, cfg: ModelConfig):
        super().__init__()
        d = cfg.n_embd
        self.transformer = nn.ModuleDict({
            "wte": nn.Embedding(cfg.vocab_size, d),
            "wpe": nn.Embedding(cfg.block_size, d),
            "drop": nn.Dropout(cfg.dropout),
            "h": nn.ModuleList([_OracleBlock(d, cfg.n_head, cfg.dropout) for _ in range(cfg.n_layer)]),
            "ln_f": nn.LayerNorm(d),
        })
        self.lm_head = nn.Linear(d, cfg.vocab_size, bias=False)
        self.transformer["wte"].weight = self.lm_head.weight

    def forward(self, idx, targets=None):
        T = idx.shape[1]
        pos = torch.arange(T, device=idx.device)[None]
        x = self.transformer["drop"](self.transformer["wte"](idx) + self.transformer["wpe"](pos))
        for blk in self.transformer["h"]:
            x = blk(x)
        logits = self.lm_head(self.transformer["ln_f"](x))
        loss = None
        if targets is not None:
            loss = F.cross_entropy(logits.view(-1, logits.size(-1)), targets.view(-1), ignore_index=-1)
        return logits, loss


class _RMSNorm(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.eps = eps

    def forward(self, x):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + self.eps) * self.weight


def _rope(x, cos, sin):
    half = x.shape[-1] // 2
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], -1)


class OracleMistral(nn.Module):
    """Stock-op Mistral-shape decoder with the same parameter names as dltb.models.mistral."""

    def __init__(self, cfg: ModelConfig):
        super().__init__()
        self.cfg = cfg
        d, hd = cfg.n_embd, cfg.head_dim
        kvd = cfg.kv_heads * hd
        self.model = nn.Module()
        self.model.embed_tokens = nn.Embedding(cfg.vocab_size, d)
        self.model.layers = nn.ModuleList()
        for _ in range(cfg.n_layer):
            layer = nn.Module()
            layer.input_layernorm = _RMSNorm(d, cfg.norm_eps)
            layer.self_attn = nn.Module()
            layer.self_attn.qkv_proj = nn.Linear(d, d + 2 * kvd, bias=False)
            layer.self_attn.o_proj = nn.Linear(d, d, bias=False)
            layer.post_attention_layernorm = _RMSNorm(d, cfg.norm_eps)
            layer.mlp = nn.Module()
            layer.mlp.gate_up_proj = nn.Linear(d, 2 * cfg.ffn_dim, bias=False)
            layer.mlp.down_proj = nn.Linear(cfg.ffn_dim, d, bias=False)
            self.model.layers.append(layer)
        self.model.norm = _RMSNorm(d, cfg.norm_eps)
        self.lm_head = nn.Linear(d, cfg.vocab_size, bias=False)

    def forward(self, idx, targets=None):
        cfg = self.cfg
        B, T = idx.shape
        H, Hkv, hd = cfg.n_head, cfg.kv_heads, cfg.head_dim
        inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, hd // 2, dtype=torch.float64) * 2.0 / hd))
        ang = torch.arange(T, dtype=torch.float64)[:, None] * inv[None]
        cos = ang.cos().float().to(idx.device)[None, None]
        sin = ang.sin().float().to(idx.device)[None, None]
        x = self.model.embed_tokens(idx)
        for layer in self.model.layers:
            h = layer.input_layernorm(x)
            qkv = layer.self_attn.qkv_proj(h)
            q = qkv[..., :H * hd].view(B, T, H, hd).transpose(1, 2)
            k = qkv[..., H * hd:(H + Hkv) * hd].view(B, T, Hkv, hd).transpose(1, 2)
            v = qkv[..., (H + Hkv) * hd:].view(B, T, Hkv, hd).transpose(1, 2)
            q, k = _rope(q, cos, sin), _rope(k, cos, sin)
            k = k.repeat_interleave(H // Hkv, 1)
            v = v.repeat_interleave(H // Hkv, 1)
            o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
            x = x + layer.self_attn.o_proj(o.transpose(1, 2).reshape(B, T, H * hd))
            gu = layer.mlp.gate_up_proj(layer.post_attention_layernorm(x))
            g, u = gu.chunk(2, -1)
            x = x + layer.mlp.down_proj(F.silu(g) * u)
        logits = self.lm_head(self.model.norm(x))
        loss = None
        if targets is not None:
            loss = F.cross_entropy(logits.view(-1, logits.size(-1)), targets.view(-1), ignore_index=-1)
        return logits, loss
