"""Pure-torch reference implementations of every dltb kernel.

They reproduce the HIP kernels' semantics — same dropout masks (counter hash of
:mod:`dltb.ops.rng`), same rounding points (the residual stream ``s`` is rounded to the storage
dtype before normalisation, softmax-xent writes unscaled dlogits, ...) — computed in fp32.  They
are the CPU execution path of the model (unit tests, gloo multi-process tests) and the oracle the
GPU kernel tests compare against.
"""
import math

import torch
import torch.nn.functional as F

from .rng import attn_keep_mask, keep_mask, keep_mask_2d, site_seed


def _f(t):
    """fp32 compute copy (fp64 inputs stay fp64 for precision tests)."""
    return t if t.dtype == torch.float64 else t.float()


def _seed(seed, site):
    return site_seed(int(seed.value), site)


def _drop(x32, p, seed, site, row_offset=0):
    if p <= 0.0:
        return x32
    s = _seed(seed, site)
    n_cols = x32.shape[-1]
    keep = keep_mask_2d(s, x32.numel() // n_cols, n_cols, p, device=x32.device,
                        row_offset=row_offset).view(x32.shape)
    return torch.where(keep, x32 * (1.0 / (1.0 - p)), torch.zeros((), device=x32.device))


# ------------------------------------------------------------------------------ norms
def norm_fwd(x, r, w, b, eps, rms, p, seed, site):
    dt = x.dtype
    x32 = _f(x)
    s = None
    if r is not None:
        s = (x32 + _drop(_f(r), p, seed, site)).to(dt)
        x32 = _f(s)
    if rms:
        var = x32.pow(2).mean(-1, keepdim=True)
        rstd = torch.rsqrt(var + eps)
        y = x32 * rstd * _f(w)
        mean = None
    else:
        mean = x32.mean(-1, keepdim=True)
        var = (x32 - mean).pow(2).mean(-1, keepdim=True)
        rstd = torch.rsqrt(var + eps)
        y = (x32 - mean) * rstd * _f(w) + _f(b)
        mean = mean.reshape(-1)
    return s, y.to(dt), mean, rstd.reshape(-1)


def _write_slot(slot, val, accumulate):
    if slot is None:
        return
    v = val.reshape(slot.shape).float()
    if accumulate:
        v = v + _f(slot)
    slot.copy_(v)


def norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms):
    d = dy.shape[-1]
    dy32 = _f(dy).reshape(-1, d)
    x32 = _f(s).reshape(-1, d)
    rstd = rstd.reshape(-1, 1)
    mu = 0.0 if rms else mean.reshape(-1, 1)
    xh = (x32 - mu) * rstd
    g = dy32 * _f(w)
    s2 = (g * xh).mean(-1, keepdim=True)
    if rms:
        dx = rstd * (g - xh * s2)
    else:
        s1 = g.mean(-1, keepdim=True)
        dx = rstd * (g - s1 - xh * s2)
    if dres is not None:
        dx = dx + _f(dres).reshape(-1, d)
    _write_slot(gw, (dy32 * xh).sum(0), accumulate)
    if not rms:
        _write_slot(gb, dy32.sum(0), accumulate)
    return dx.to(dy.dtype).view_as(dy)


# ------------------------------------------------------------------------------ elementwise
def gelu_fwd(f):
    return F.gelu(_f(f)).to(f.dtype)


def gelu_bwd(dg, f, db, accumulate):
    x = _f(f)
    cdf = 0.5 * (1.0 + torch.erf(x * (1.0 / math.sqrt(2.0))))
    pdf = torch.exp(-0.5 * x * x) / math.sqrt(2.0 * math.pi)
    df = (_f(dg) * (cdf + x * pdf)).to(dg.dtype)
    if db is not None:
        _write_slot(db, _f(df).reshape(-1, df.shape[-1]).sum(0), accumulate)
    return df


def colsum_into(src, out, accumulate):
    _write_slot(out, _f(src).reshape(-1, src.shape[-1]).sum(0), accumulate)


def dropout(x, r, p, seed, site):
    out = _drop(_f(r), p, seed, site)
    if x is not None:
        out = out + _f(x)
    return out.to(r.dtype)


def swiglu_fwd(gu):
    F2 = gu.shape[-1] // 2
    g, u = _f(gu)[..., :F2], _f(gu)[..., F2:]
    return (F.silu(g) * u).to(gu.dtype)


def swiglu_bwd(dh, gu):
    F2 = gu.shape[-1] // 2
    g, u = _f(gu)[..., :F2], _f(gu)[..., F2:]
    s = torch.sigmoid(g)
    d = _f(dh)
    dg = d * u * s * (1 + g * (1 - s))
    du = d * g * s
    return torch.cat([dg, du], -1).to(gu.dtype)


def rope_tables(T, D, theta, device=None):
    half = D // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2.0 / D))
    ang = torch.arange(T, dtype=torch.float64)[:, None] * inv[None, :]
    return ang.cos().float().to(device), ang.sin().float().to(device)


def rope_(qkv2d, cos, sin, T, heads, D, inverse=False):
    N = qkv2d.shape[0]
    half = D // 2
    x = _f(qkv2d[:, :heads * D]).view(N // T, T, heads, D)
    x1, x2 = x[..., :half], x[..., half:]
    c = cos[:T].view(1, T, 1, half)
    s = sin[:T].view(1, T, 1, half)
    if inverse:
        s = -s
    o1 = x1 * c - x2 * s
    o2 = x2 * c + x1 * s
    qkv2d[:, :heads * D] = torch.cat([o1, o2], -1).reshape(N, heads * D).to(qkv2d.dtype)


# ------------------------------------------------------------------------------ embedding
def embed_fwd(idx, wte, wpe, p, seed, site):
    B, T = idx.shape
    x = _f(wte)[idx] + _f(wpe)[:T][None]
    return _drop(x.reshape(B * T, -1), p, seed, site).reshape(B, T, -1).to(wte.dtype)


def embed_bwd(dx, idx, dwte, dwpe, accumulate_wpe, p, seed, site):
    B, T = idx.shape
    d = dx.shape[-1]
    g = _drop(_f(dx).reshape(B * T, d), p, seed, site)
    if dwpe is not None:
        full = torch.zeros(dwpe.shape, dtype=torch.float32, device=dx.device)
        full[:T] = g.view(B, T, d).sum(0)
        _write_slot(dwpe, full, accumulate_wpe)
    if dwte is not None:
        acc = _f(dwte)
        acc.index_add_(0, idx.reshape(-1), g)
        dwte.copy_(acc)


# ------------------------------------------------------------------------------ xent
def xent_fwd_bwd_(logits, targets, ignore_index):
    """Returns per-row loss; overwrites logits with unscaled (softmax - onehot)."""
    z = _f(logits)
    valid = targets != ignore_index
    lse = torch.logsumexp(z, -1)
    t = targets.clamp(min=0)
    tl = z.gather(-1, t[:, None])[:, 0]
    loss = torch.where(valid, lse - tl, torch.zeros_like(lse))
    pr = torch.softmax(z, -1)
    pr.scatter_add_(-1, t[:, None], -torch.ones_like(tl)[:, None])
    pr = torch.where(valid[:, None], pr, torch.zeros_like(pr))
    logits.copy_(pr.to(logits.dtype))
    return loss


# ------------------------------------------------------------------------------ attention
def _attn_probs(q, k, B, T, Hq, Hkv, D, scale, causal):
    qh = _f(q).reshape(B, T, Hq, D).transpose(1, 2)              # [B,Hq,T,D]
    kh = _f(k).reshape(B, T, Hkv, D).transpose(1, 2)
    if Hq != Hkv:
        kh = kh.repeat_interleave(Hq // Hkv, dim=1)
    s = torch.matmul(qh, kh.transpose(-1, -2)) * scale
    if causal:
        m = torch.ones(T, T, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(m, float("-inf"))
    return s


def _attn_keep(B, Hq, T, p, seed, site, device):
    if p <= 0.0:
        return None
    s = _seed(seed, site)
    rows = torch.arange(B * Hq * T, dtype=torch.int64, device=device)[:, None]
    cols = torch.arange(T, dtype=torch.int64, device=device)[None, :]
    return attn_keep_mask(s, rows, cols, p).view(B, Hq, T, T)


def attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p, seed, site):
    D = q.shape[1] // Hq
    s = _attn_probs(q, k, B, T, Hq, Hkv, D, scale, causal)
    lse = torch.logsumexp(s, -1)                                      # [B,Hq,T]
    pr = torch.exp(s - lse[..., None])
    keep = _attn_keep(B, Hq, T, p, seed, site, q.device)
    if keep is not None:
        pr = torch.where(keep, pr / (1.0 - p), torch.zeros((), device=q.device))
    vh = _f(v).reshape(B, T, Hkv, D).transpose(1, 2)
    if Hq != Hkv:
        vh = vh.repeat_interleave(Hq // Hkv, dim=1)
    o = torch.matmul(pr, vh).transpose(1, 2).reshape(B * T, Hq * D)
    return o.to(q.dtype), _f(lse).contiguous()


def attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, T, Hq, Hkv, scale, causal, p, seed, site):
    D = q.shape[1] // Hq
    G = Hq // Hkv
    s = _attn_probs(q, k, B, T, Hq, Hkv, D, scale, causal)
    pr = torch.exp(s - lse.view(B, Hq, T)[..., None])
    keep = _attn_keep(B, Hq, T, p, seed, site, q.device)
    z = torch.ones_like(pr) if keep is None else _f(keep) / (1.0 - p)
    qh = _f(q).reshape(B, T, Hq, D).transpose(1, 2)
    kh = _f(k).reshape(B, T, Hkv, D).transpose(1, 2).repeat_interleave(G, dim=1)
    vh = _f(v).reshape(B, T, Hkv, D).transpose(1, 2).repeat_interleave(G, dim=1)
    doh = _f(do).reshape(B, T, Hq, D).transpose(1, 2)
    oh = _f(o).reshape(B, T, Hq, D).transpose(1, 2)
    delta = (doh * oh).sum(-1, keepdim=True)
    pd = pr * z
    dvh = torch.matmul(pd.transpose(-1, -2), doh)                     # [B,Hq,T,D]
    dp = torch.matmul(doh, vh.transpose(-1, -2))
    ds = pr * (dp * z - delta)
    dqh = torch.matmul(ds, kh) * scale
    dkh = torch.matmul(ds.transpose(-1, -2), qh) * scale
    if G > 1:
        dkh = dkh.view(B, Hkv, G, T, D).sum(2)
        dvh = dvh.view(B, Hkv, G, T, D).sum(2)
    dq.copy_(dqh.transpose(1, 2).reshape(B * T, Hq * D).to(dq.dtype))
    dk.copy_(dkh.transpose(1, 2).reshape(B * T, Hkv * D).to(dk.dtype))
    dv.copy_(dvh.transpose(1, 2).reshape(B * T, Hkv * D).to(dv.dtype))


# ------------------------------------------------------------------------------ optimizer
def adamw_flat(master, exp_avg, exp_avg_sq, grad, lr, beta1, beta2, eps, wd, step, gscale=None):
    g = _f(grad)
    if gscale is not None:
        g = g * _f(gscale)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    master.mul_(1.0 - lr * wd)
    exp_avg.lerp_(g, 1.0 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    master.addcdiv_(exp_avg, denom, value=-(lr / bc1))
