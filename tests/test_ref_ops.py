"""CPU checks of the torch reference ops (the oracle of the GPU kernel tests and the CPU execution
path): manual backward formulas vs autograd, forward vs torch built-ins, RNG properties."""
import math

import pytest
import torch
import torch.nn.functional as F

import dltb
from dltb.ops import ref, rng
from dltb.ops.rng import StepSeed

torch.manual_seed(0)


def seed(v=7):
    s = StepSeed(v)
    s.next()
    return s


def test_rng_properties():
    s = rng.site_seed(12345, 3)
    keep = rng.keep_mask_2d(s, 512, 1024, 0.1)
    frac = keep.float().mean().item()
    assert abs(frac - (1 - 6554 / 65536)) < 0.003
    # different sites / rows decorrelated
    k2 = rng.keep_mask_2d(rng.site_seed(12345, 4), 512, 1024, 0.1)
    agree = (keep == k2).float().mean().item()
    assert abs(agree - (0.9 * 0.9 + 0.1 * 0.1)) < 0.01
    # row offset consistency
    sub = rng.keep_mask_2d(s, 10, 1024, 0.1, row_offset=100)
    assert torch.equal(sub, keep[100:110])


@pytest.mark.parametrize("site", [5, 6])
def test_attention_mask_hash_statistics(site):
    """attn_keep_mask (one multiply-xorshift round on two independently mixed keys, csrc/common.h
    rng_attn_pair): keep rate, neighbour correlations, byte uniformity, and the rectangle statistic that
    a plain XOR of row and column keys fails (k(r,c) k(r,c') k(r',c) k(r',c') centred: ~0.05 for XOR)."""
    s = rng.site_seed(2024, site)
    R, C = 1024, 2048
    rows = torch.arange(R, dtype=torch.int64)[:, None]
    cols = torch.arange(C, dtype=torch.int64)[None, :]
    keep = rng.attn_keep_mask(s, rows, cols, 0.1).double()
    assert abs(keep.mean().item() - (1 - 6554 / 65536)) < 0.003
    k = keep - keep.mean()
    var = k.var()
    assert abs(((k[:, :-1] * k[:, 1:]).mean() / var).item()) < 0.01          # column pair halves, neighbours
    assert abs(((k[:-1] * k[1:]).mean() / var).item()) < 0.01                  # neighbouring rows
    g = torch.Generator().manual_seed(site)
    ra, rb = torch.randint(0, R, (200000,), generator=g), torch.randint(0, R, (200000,), generator=g)
    ca, cb = torch.randint(0, C, (200000,), generator=g), torch.randint(0, C, (200000,), generator=g)
    rect = ((k[ra, ca] * k[ra, cb] * k[rb, ca] * k[rb, cb]).mean() / var ** 2).item()
    assert abs(rect) < 0.015, rect
    # the raw 16-bit values behind the decisions: uniform top bytes (chi-square, 255 dof)
    rk = rng._fmix32((rng._mul32(rows, rng.C_ROW) + ((s >> 32) & rng.MASK32)) & rng.MASK32)
    ck = rng._fmix32((rng._mul32(cols >> 1, rng.C_COL) + (s & rng.MASK32)) & rng.MASK32)
    h = rng._mul32(rk ^ ck, 0x85EBCA6B)
    h = h ^ (h >> 16)
    r16 = torch.where((cols & 1) == 1, h >> 16, h & 0xFFFF)
    hist = torch.bincount((r16 >> 8).flatten(), minlength=256).double()
    e = R * C / 256
    chi2 = (((hist - e) ** 2) / e).sum().item()
    assert chi2 < 255 + 6 * math.sqrt(2 * 255), chi2
    assert torch.equal(r16 >= 6554, keep.bool())


def test_mul32_matches_uint32():
    a = torch.tensor([0, 1, 0xFFFFFFFF, 0x12345678, 0xDEADBEEF], dtype=torch.int64)
    for c in (rng.C_ROW, rng.C_COL, 0x85EBCA6B):
        got = rng._mul32(a, c).tolist()
        want = [(int(x) * c) & 0xFFFFFFFF for x in a.tolist()]
        assert got == want


@pytest.mark.parametrize("rms", [False, True])
def test_norm_ref_vs_autograd(rms):
    N, d = 37, 64
    x = torch.randn(N, d, dtype=torch.float64)
    r = torch.randn(N, d, dtype=torch.float64)
    w = torch.randn(d, dtype=torch.float64)
    b = torch.randn(d, dtype=torch.float64)
    sd = seed()
    s, y, mean, rstd = ref.norm_fwd(x, r, w, b, 1e-5, rms, 0.0, sd, 0)
    xs = (x + r).requires_grad_()
    wt, bt = w.clone().requires_grad_(), b.clone().requires_grad_()
    if rms:
        yt = xs * torch.rsqrt(xs.pow(2).mean(-1, keepdim=True) + 1e-5) * wt
    else:
        yt = F.layer_norm(xs, (d,), wt, bt, 1e-5)
    assert torch.allclose(y.double(), yt, atol=1e-6)
    dy = torch.randn(N, d, dtype=torch.float64)
    yt.backward(dy)
    gw = torch.zeros(d, dtype=torch.float64)
    gb = torch.zeros(d, dtype=torch.float64)
    dres = torch.randn(N, d, dtype=torch.float64)
    dx = ref.norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, False, rms)
    assert torch.allclose(dx, xs.grad + dres, atol=1e-6)
    assert torch.allclose(gw, wt.grad, atol=1e-6)
    if not rms:
        assert torch.allclose(gb, bt.grad, atol=1e-6)


@pytest.mark.parametrize("causal,Hq,Hkv", [(False, 4, 4), (True, 4, 2)])
def test_attention_ref_vs_sdpa_and_autograd(causal, Hq, Hkv):
    B, T, D = 2, 16, 8
    q = torch.randn(B * T, Hq * D, dtype=torch.float64)
    k = torch.randn(B * T, Hkv * D, dtype=torch.float64)
    v = torch.randn(B * T, Hkv * D, dtype=torch.float64)
    sc = 1 / math.sqrt(D)
    o, lse = ref.attn_fwd(q, k, v, B, T, Hq, Hkv, sc, causal, 0.0, None, 0)
    qh = q.view(B, T, Hq, D).transpose(1, 2).requires_grad_()
    kh = k.view(B, T, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1).detach().requires_grad_()
    vh = v.view(B, T, Hkv, D).transpose(1, 2).repeat_interleave(Hq // Hkv, 1).detach().requires_grad_()
    ot = F.scaled_dot_product_attention(qh, kh, vh, is_causal=causal)
    assert torch.allclose(o.double(), ot.transpose(1, 2).reshape(B * T, Hq * D), atol=1e-6)
    do = torch.randn(B * T, Hq * D, dtype=torch.float64)
    ot.transpose(1, 2).reshape(B * T, Hq * D).backward(do)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    ref.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, T, Hq, Hkv, sc, causal, 0.0, None, 0)
    G = Hq // Hkv
    assert torch.allclose(dq, qh.grad.transpose(1, 2).reshape(B * T, Hq * D), atol=1e-6)
    dk_want = kh.grad.view(B, Hkv, G, T, D).sum(2).transpose(1, 2).reshape(B * T, Hkv * D)
    dv_want = vh.grad.view(B, Hkv, G, T, D).sum(2).transpose(1, 2).reshape(B * T, Hkv * D)
    assert torch.allclose(dk, dk_want, atol=1e-6)
    assert torch.allclose(dv, dv_want, atol=1e-6)


def test_attention_dropout_ref_vs_autograd():
    """attn_bwd with dropout against autograd through an explicit masked softmax."""
    B, T, H, D, p = 1, 16, 2, 8, 0.25
    q = torch.randn(B * T, H * D, dtype=torch.float64)
    k = torch.randn(B * T, H * D, dtype=torch.float64)
    v = torch.randn(B * T, H * D, dtype=torch.float64)
    sd = seed(3)
    o, lse = ref.attn_fwd(q, k, v, B, T, H, H, 0.3, False, p, sd, 5)
    keep = ref._attn_keep(B, H, T, p, sd, 5, "cpu")
    qt, kt, vt = (t.clone().requires_grad_() for t in (q, k, v))
    s = torch.matmul(qt.view(B, T, H, D).transpose(1, 2), kt.view(B, T, H, D).transpose(1, 2).transpose(-1, -2)) * 0.3
    pr = torch.softmax(s, -1) * keep / (1 - p)
    ot = torch.matmul(pr, vt.view(B, T, H, D).transpose(1, 2)).transpose(1, 2).reshape(B * T, H * D)
    assert torch.allclose(o.double(), ot, atol=1e-8)
    do = torch.randn_like(o)
    ot.backward(do)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    ref.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, T, H, H, 0.3, False, p, sd, 5)
    assert torch.allclose(dq, qt.grad, atol=1e-6)  # lse is stored in fp32
    assert torch.allclose(dk, kt.grad, atol=1e-6)
    assert torch.allclose(dv, vt.grad, atol=1e-6)


def test_xent_ref():
    z = torch.randn(10, 50, dtype=torch.float64)
    t = torch.randint(0, 50, (10,))
    t[3] = -1
    zt = z.clone().requires_grad_()
    want = F.cross_entropy(zt, t, ignore_index=-1, reduction="sum")
    want.backward()
    zz = z.clone()
    loss = ref.xent_fwd_bwd_(zz, t, -1)
    assert torch.allclose(loss.sum(), want)
    assert torch.allclose(zz, zt.grad)


def test_gelu_swiglu_rope_refs():
    f = torch.randn(20, 16, dtype=torch.float64, requires_grad=True)
    F.gelu(f).backward(torch.ones_like(f))
    db = torch.zeros(16, dtype=torch.float64)
    df = ref.gelu_bwd(torch.ones_like(f), f.detach(), db, False)
    assert torch.allclose(df, f.grad)
    assert torch.allclose(db, f.grad.sum(0))
    gu = torch.randn(5, 32, dtype=torch.float64, requires_grad=True)
    h = F.silu(gu[:, :16]) * gu[:, 16:]
    dh = torch.randn(5, 16, dtype=torch.float64)
    h.backward(dh)
    assert torch.allclose(ref.swiglu_bwd(dh, gu.detach()), gu.grad)
    T, D = 8, 16
    cos, sin = ref.rope_tables(T, D, 10000.0)
    x = torch.randn(2 * T, 3 * D)
    y = x.clone()
    ref.rope_(y, cos, sin, T, 2, D)
    assert torch.allclose(y[:, 2 * D:], x[:, 2 * D:])      # v untouched
    ref.rope_(y, cos, sin, T, 2, D, inverse=True)
    assert torch.allclose(y, x, atol=1e-5)


def test_adamw_ref_matches_torch():
    p0 = torch.randn(1000)
    master, m, v = p0.clone(), torch.zeros(1000), torch.zeros(1000)
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([tp], lr=1e-3, weight_decay=0.01)
    for step in range(1, 4):
        g = torch.randn(1000)
        tp.grad = g.clone()
        opt.step()
        ref.adamw_flat(master, m, v, g, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)
    assert torch.allclose(master, tp.detach(), atol=1e-7)
