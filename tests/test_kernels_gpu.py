"""Numerics of every gfx950 HIP kernel against a plain-torch fp32 reference of the same op.

The references live in dltb.ops.ref and share the dropout counter hash with the kernels, so
dropout masks must match exactly (any mask mismatch shows up as O(1) errors).
"""
import math

import pytest
import torch

import dltb
from dltb.ops import ref
from dltb.ops._ext import ext
from dltb.ops.rng import StepSeed

pytestmark = pytest.mark.gpu
DEV = "cuda"


def close(a, b, atol, rtol, what=""):
    a = a.float()
    b = b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).float().mean().item()
    assert bad == 0.0, f"{what}: {bad*100:.3f}% elements out of tolerance, max err {err.max().item():.4g}"


def rnd(*shape, scale=1.0, dtype=torch.bfloat16):
    return (torch.randn(*shape, device=DEV) * scale).to(dtype)


@pytest.fixture(scope="module", autouse=True)
def _ext_loaded():
    C = ext()
    assert C.arch() == "gfx950"
    torch.manual_seed(0)


def seed_obj(v=1234):
    s = StepSeed(v, 0, device=DEV)
    s.next()
    return s


# ------------------------------------------------------------------------------ norms
@pytest.mark.parametrize("d", [64, 768, 1024, 2048, 4096])
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("res_p", [None, 0.0, 0.1])
def test_norm_fwd_bwd(d, rms, res_p):
    N = 300
    x, w, b = rnd(N, d), rnd(d, scale=0.5) + 1, rnd(d, scale=0.1)
    r = rnd(N, d) if res_p is not None else None
    p = res_p or 0.0
    sd = seed_obj()
    C = ext()
    s, y, mean, rstd = C.norm_fwd(x, r, w, None if rms else b, 1e-5, rms, p, sd.device_tensor, 3)
    rs, ry, rmean, rrstd = ref.norm_fwd(x, r, w, None if rms else b, 1e-5, rms, p, sd, 3)
    if r is not None:
        close(s, rs, 1e-2, 1e-2, "s")
    close(y, ry, 2e-2, 2e-2, "y")
    close(rstd, rrstd, 1e-4, 1e-3, "rstd")
    # backward
    dy = rnd(N, d)
    dres = rnd(N, d) if r is not None else None
    sin = s if r is not None else x
    gw = torch.zeros(d, device=DEV, dtype=torch.bfloat16)
    gb = torch.zeros(d, device=DEV, dtype=torch.bfloat16)
    rgw, rgb = gw.clone(), gb.clone()
    dx = C.norm_bwd(dy, sin, w, None if rms else mean, rstd, dres, gw, None if rms else gb, False, rms)
    rdx = ref.norm_bwd(dy, sin, w, rmean, rrstd, dres, rgw, rgb, False, rms)
    close(dx, rdx, 3e-2, 3e-2, "dx")
    close(gw, rgw, 0.15, 2e-2, "dgamma")
    if not rms:
        close(gb, rgb, 0.15, 2e-2, "dbeta")
    # accumulate mode adds onto the slot
    gw2 = gw.clone()
    C.norm_bwd(dy, sin, w, None if rms else mean, rstd, dres, gw2, None if rms else gb.clone(), True, rms)
    close(gw2, 2 * gw.float(), 0.3, 3e-2, "dgamma accumulate")


# ------------------------------------------------------------------------------ elementwise
def test_gelu_and_bias_grad():
    N, k = 512, 4096
    f = rnd(N, k)
    C = ext()
    close(C.gelu_fwd(f), ref.gelu_fwd(f), 1e-2, 1e-2, "gelu")
    f_odd = rnd(7, 24)                           # 21 chunks of 8: the two-chunk pass's tail
    close(C.gelu_fwd(f_odd), ref.gelu_fwd(f_odd), 1e-2, 1e-2, "gelu odd")
    dg = rnd(N, k)
    db = torch.zeros(k, device=DEV, dtype=torch.bfloat16)
    rdb = db.clone()
    df = C.gelu_bwd(dg, f, db, False)
    rdf = ref.gelu_bwd(dg, f, rdb, False)
    close(df, rdf, 1e-2, 2e-2, "dgelu")
    close(db, rdb, 0.2, 2e-2, "gelu bias grad")


def test_colsum_and_dropout():
    C = ext()
    src = rnd(1000, 3072)
    out = rnd(3072)
    expect = out.float() + src.float().sum(0)
    C.colsum_into(src, out, True)
    close(out, expect, 0.3, 2e-2, "colsum accumulate")
    sd = seed_obj(99)
    x, r = rnd(257, 1024), rnd(257, 1024)
    y = C.dropout(x, r, 0.1, sd.device_tensor, 7)
    ry = ref.dropout(x, r, 0.1, sd, 7)
    close(y, ry, 1e-2, 1e-2, "dropout_add")
    kept = (C.dropout(None, torch.ones_like(r), 0.1, sd.device_tensor, 7).float() > 0).float().mean().item()
    assert abs(kept - 0.9) < 0.01


@pytest.mark.parametrize("N", [2048, 300])
def test_batched_column_reductions(N):
    """colpart (PLAIN / GELU / DROP / LN / RMS segments, 3 per launch) + colreduce_multi vs torch."""
    from dltb.ops.functional import GradReducer, _DROP, _GELU, _LN, _PLAIN, _RMS
    C = ext()
    d, k3 = 1024, 3072
    dy, s_, dq, f = rnd(N, d), rnd(N, d), rnd(N, k3), rnd(N, k3)
    dg = rnd(N, k3)
    mean = torch.randn(N, device=DEV)
    rstd = torch.rand(N, device=DEV) + 0.5
    sd = seed_obj(77)
    df, dm = torch.empty_like(dg), torch.empty_like(dy)
    parts_a = C.colpart([_LN, _PLAIN, _GELU], [dy, dq, dg], [s_, None, f], [None, None, df],
                        [mean, None, None], [rstd, None, None], 0.0, None, [0, 0, 0])
    parts_b = C.colpart([_RMS, _DROP], [dy, dy], [s_, None], [None, dm], [None, None], [rstd, None], 0.1,
                        sd.device_tensor, [0, 5])
    outs = [torch.zeros(n, device=DEV, dtype=torch.bfloat16) for n in (d, d, k3, k3, d, d)]
    outs[1].fill_(1.0)                                       # accumulate into a non-zero slot
    red = GradReducer()
    red.add(parts_a[0][0], outs[0], False)
    red.add(parts_a[0][1], outs[1], True)
    red.add(parts_a[1][0], outs[2], False)
    red.add(parts_a[2][0], outs[3], False)
    red.add(parts_b[0][0], outs[4], False)
    red.add(parts_b[1][0], outs[5], False)
    red.flush()
    x32 = s_.float()
    xh = (x32 - mean[:, None]) * rstd[:, None]
    close(outs[0], (dy.float() * xh).sum(0), 0.5, 2e-2, "LN dgamma")
    close(outs[1], dy.float().sum(0) + 1.0, 0.5, 2e-2, "LN dbeta (accumulate)")
    close(outs[2], dq.float().sum(0), 0.5, 2e-2, "plain colsum")
    rdf = ref.gelu_bwd(dg, f, None, False)
    close(df, rdf, 2e-2, 2e-2, "gelu df")
    close(outs[3], df.float().sum(0), 0.5, 2e-2, "gelu bias")
    close(outs[4], (dy.float() * x32 * rstd[:, None]).sum(0), 0.5, 2e-2, "RMS dgamma")
    rdm = ref.dropout(None, dy, 0.1, sd, 5)
    assert torch.equal(dm, rdm), "dropout mask / scale"
    close(outs[5], dm.float().sum(0), 0.5, 2e-2, "dropout bias")


@pytest.mark.parametrize("N,d", [(2048, 1024), (300, 768), (4096, 2048), (64, 64)])
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("bias_src", [None, "dx", "ext"])
def test_norm_bwd_fused(N, d, rms, bias_src):
    """One-launch norm backward (dx + gamma / beta partials + column partials of dx) through
    functional.norm_bwd vs an fp32 torch reference; the dqkv-style external bias source too."""
    from dltb.ops import functional as F_
    C = ext()
    assert C.norm_bwd_fused_supported(d)
    dy, s_, dres = rnd(N, d), rnd(N, d), rnd(N, d)
    w = rnd(d, scale=0.5) + 1
    mean = None if rms else torch.randn(N, device=DEV) * 0.1
    rstd = torch.rand(N, device=DEV) + 0.5
    gw = torch.zeros(d, device=DEV, dtype=torch.bfloat16)
    gb = None if rms else torch.full((d,), 1.0, device=DEV, dtype=torch.bfloat16)
    ext_src = rnd(N, 3 * d) if bias_src == "ext" else None
    bslot = torch.zeros(3 * d if bias_src == "ext" else d, device=DEV, dtype=torch.bfloat16)
    bias = None if bias_src is None else (("dx" if bias_src == "dx" else ext_src), bslot, False)
    red = F_.GradReducer()
    dx = F_.norm_bwd(dy, s_, w, mean, rstd, dres, gw, gb, gb is not None, rms, red=red, bias=bias)
    red.flush()
    x32 = s_.float()
    xh = (x32 - (0.0 if rms else mean[:, None])) * rstd[:, None]
    g = dy.float() * w.float()
    s1 = 0.0 if rms else g.mean(-1, keepdim=True)
    s2 = (g * xh).mean(-1, keepdim=True)
    rdx = rstd[:, None] * (g - s1 - xh * s2) + dres.float()
    close(dx, rdx, 3e-2, 3e-2, "dx")
    close(gw, (dy.float() * xh).sum(0), 0.5, 2e-2, "dgamma")
    if not rms:
        close(gb, dy.float().sum(0) + 1.0, 0.5, 2e-2, "dbeta (accumulate)")
    if bias_src == "dx":
        close(bslot, dx.float().sum(0), 0.5, 2e-2, "dx column sum")
    elif bias_src == "ext":
        close(bslot, ext_src.float().sum(0), 0.5, 2e-2, "external column sum")


@pytest.mark.parametrize("N,d", [(2048, 1024), (300, 768)])
@pytest.mark.parametrize("p", [0.1, 0.0])
def test_norm_bwd_fused_dropout(N, d, p):
    """LayerNorm backward that also forms the previous layer's Dropout backward dm of its dx (and
    dm's column sum): dm bitwise the standalone dropout kernel's, dx as without it."""
    from dltb.ops import functional as F_
    dy, s_, dres = rnd(N, d), rnd(N, d), rnd(N, d)
    w = rnd(d, scale=0.5) + 1
    mean = torch.randn(N, device=DEV) * 0.1
    rstd = torch.rand(N, device=DEV) + 0.5
    sd = seed_obj(9)
    outs = [torch.zeros(d, device=DEV, dtype=torch.bfloat16) for _ in range(3)]
    red = F_.GradReducer()
    dx, dm = F_.norm_bwd(dy, s_, w, mean, rstd, dres, outs[0], outs[1], False, False, red=red,
                         drop=(p, sd, 7, None, outs[2], False))
    red.flush()
    ref_outs = [torch.zeros(d, device=DEV, dtype=torch.bfloat16) for _ in range(2)]
    red2 = F_.GradReducer()
    dx2 = F_.norm_bwd(dy, s_, w, mean, rstd, dres, ref_outs[0], ref_outs[1], False, False, red=red2)
    red2.flush()
    assert torch.equal(dx, dx2), "dx"
    assert torch.equal(outs[0], ref_outs[0]) and torch.equal(outs[1], ref_outs[1]), "dgamma / dbeta"
    rdm = ref.dropout(None, dx, p, sd, 7) if p > 0 else dx
    assert torch.equal(dm, rdm), "dropout backward"
    close(outs[2], dm.float().sum(0), 0.5, 2e-2, "dm column sum")


@pytest.mark.parametrize("R,C", [(1024, 3072), (4096, 1024), (100, 36)])
def test_transpose_into(R, C):
    C_ = ext()
    src = rnd(R, C)
    dst = torch.empty(C, R, device=DEV, dtype=torch.bfloat16)
    C_.transpose_into(src, dst)
    assert torch.equal(dst, src.t())


def test_sumsq_is_deterministic():
    C_ = ext()
    x = rnd(3_000_000)
    outs = []
    for _ in range(3):
        o = torch.zeros(1, device=DEV)
        C_.sumsq_(x, o)
        outs.append(o.item())
    assert outs[0] == outs[1] == outs[2]
    assert abs(outs[0] - x.float().pow(2).sum().item()) < 1e-3 * outs[0]


@pytest.mark.parametrize("tn", [False, True])
@pytest.mark.parametrize("M,N,K,cfg,splits", [(256, 384, 512, 0, 1), (512, 256, 1024, 0, 4),
                                               (512, 256, 256, 1, 1), (256, 512, 192, 2, 2),
                                               (256, 192, 512, 3, 1), (192, 256, 320, 4, 2),
                                               (192, 320, 256, 5, 1)])
@pytest.mark.parametrize("pf,gm,stages", [(0, 1, 0), (3, 2, 0), (0, 1, 2)])
def test_gemm(tn, M, N, K, cfg, splits, pf, gm, stages):
    """dltb GEMM (NT: a[M,K] b[N,K]; TN: a[K,M] b[K,N]) vs fp32 torch, incl. bias / accumulate /
    split-K, row-strided operand views and the double-buffered (two workgroups / CU) variant."""
    C_ = ext()
    if not C_.gemm_supported(M, N, K, tn, cfg):
        pytest.skip("tile config not offered for this layout")
    if tn:
        a_full, b_full = rnd(K, M + 64), rnd(K, N)
        a, b = a_full[:, 64:], b_full                 # strided view of a wider buffer
        ref32 = a.float().t() @ b.float()
    else:
        a_full, b_full = rnd(M, K + 64), rnd(N, K)
        a, b = a_full[:, :K], b_full
        ref32 = a.float() @ b.float().t()
    bias = rnd(N)
    out = C_.gemm(a, b, None, bias, tn, False, splits, cfg, pf, gm, stages=stages)
    close(out, ref32 + bias.float(), 0.1, 2e-2, "gemm + bias")
    prev = rnd(M, N)
    acc = prev.clone()
    C_.gemm(a, b, acc, None, tn, True, splits, cfg, pf, gm, stages=stages)
    close(acc, ref32 + prev.float(), 0.1, 2e-2, "gemm accumulate")


def test_swiglu_rope():
    C = ext()
    gu = rnd(256, 2 * 512)
    close(C.swiglu_fwd(gu), ref.swiglu_fwd(gu), 1e-2, 2e-2, "swiglu")
    dh = rnd(256, 512)
    close(C.swiglu_bwd(dh, gu), ref.swiglu_bwd(dh, gu), 1e-2, 3e-2, "swiglu bwd")
    T, Hq, Hkv, D = 128, 4, 2, 128
    qkv = rnd(2 * T, (Hq + 2 * Hkv) * D)
    cos, sin = ref.rope_tables(T, D, 10000.0, DEV)
    a, b = qkv.clone(), qkv.clone()
    C.rope_(a, cos, sin, T, Hq + Hkv, D, False)
    ref.rope_(b, cos, sin, T, Hq + Hkv, D, False)
    close(a, b, 1e-2, 1e-2, "rope")
    C.rope_(a, cos, sin, T, Hq + Hkv, D, True)
    close(a, qkv, 3e-2, 3e-2, "rope inverse")


def test_embedding():
    C = ext()
    V, d, B, T = 1000, 256, 2, 128
    wte, wpe = rnd(V, d), rnd(T, d)
    idx = torch.randint(0, 50, (B, T), device=DEV)   # many repeated ids
    sd = seed_obj(5)
    x = C.embed_fwd(idx, wte, wpe, 0.1, sd.device_tensor, 0)
    close(x, ref.embed_fwd(idx, wte, wpe, 0.1, sd, 0), 1e-2, 1e-2, "embed fwd")
    dx = rnd(B, T, d)
    dwte, dwpe = rnd(V, d), torch.zeros(T, d, device=DEV, dtype=torch.bfloat16)
    rdwte, rdwpe = dwte.clone(), dwpe.clone()
    C.embed_bwd(dx, idx, dwte, dwpe, False, 0.1, sd.device_tensor, 0)
    ref.embed_bwd(dx, idx, rdwte, rdwpe, False, 0.1, sd, 0)
    close(dwpe, rdwpe, 2e-2, 2e-2, "dwpe")
    close(dwte, rdwte, 5e-2, 2e-2, "dwte")


def test_xent():
    C = ext()
    N, V = 300, 32000
    logits = rnd(N, V, scale=2.0)
    tgt = torch.randint(0, V, (N,), device=DEV)
    tgt[::7] = -1
    a, b = logits.clone(), logits.clone()
    la = C.xent_fwd_bwd_(a, tgt, -1)
    lb = ref.xent_fwd_bwd_(b, tgt, -1)
    close(la, lb, 1e-3, 1e-3, "xent loss")
    close(a, b, 1e-4, 2e-2, "dlogits")
    # against torch's own cross entropy
    valid = tgt != -1
    want = torch.nn.functional.cross_entropy(logits.float(), tgt, ignore_index=-1)
    got = la.sum() / valid.sum()
    assert abs(got.item() - want.item()) < 1e-3
    # device-side mean (one launch) and the head-gradient scale helpers
    lc = C.xent_mean(la, tgt, -1)
    assert abs(lc[0].item() - want.item()) < 1e-3 and lc[1].item() == valid.sum().item()
    h = rnd(64, 256)
    dloss = torch.tensor(3.0, device=DEV)
    g = torch.empty(1, device=DEV)
    hs = C.scale_by(h, dloss, lc[1:2], g)
    assert abs(g.item() - 3.0 / valid.sum().item()) < 1e-6
    close(hs, (h.float() * g.item()), 1e-3, 1e-2, "scale_by")


def test_embedding_sort_free_matches_sorted():
    """The scan (no sort) token-gradient path equals a float64 scatter-add, ids with many repeats
    and ignored (-1) positions; deterministic across calls."""
    C = ext()
    V, d, B, T = 500, 192, 2, 256
    idx = torch.randint(0, 20, (B, T), device=DEV)
    idx[0, ::9] = -1
    dx = rnd(B, T, d)
    outs = []
    for _ in range(2):
        dwte = torch.zeros(V, d, device=DEV, dtype=torch.bfloat16)
        C.embed_bwd(dx, idx, dwte, None, False, 0.0, None, 0)
        outs.append(dwte)
    assert torch.equal(outs[0], outs[1])
    want = torch.zeros(V, d, dtype=torch.float64, device=DEV)
    flat = idx.reshape(-1)
    keep = flat >= 0
    want.index_add_(0, flat[keep], dx.reshape(-1, d)[keep].double())
    close(outs[0], want, 2e-2, 2e-2, "dwte scan")


def test_gemm_device_alpha():
    C = ext()
    M, N, K = 256, 256, 2048
    a, b = rnd(M, K), rnd(N, K)
    al = torch.tensor([0.37], device=DEV)
    ref32 = (a.float() @ b.float().t()) * 0.37
    for sp in (1, 4):
        out = C.gemm(a, b, None, None, False, False, sp, 2 if sp == 4 else 0, 0, 1, al)
        close(out, ref32, 0.05, 2e-2, f"gemm alpha splits={sp}")


# ------------------------------------------------------------------------------ attention
ATTN_CASES = [
    # B, T, Hq, Hkv, D, causal, p
    (2, 256, 4, 4, 64, False, 0.0),
    (2, 256, 4, 4, 64, False, 0.1),
    (1, 512, 2, 2, 64, True, 0.0),
    (1, 256, 8, 2, 128, True, 0.0),
    (1, 256, 4, 4, 128, False, 0.1),
    # causal GQA: the dK/dV pass splits each KV group's query heads over workgroups (fp32 partials)
    (1, 512, 8, 2, 128, True, 0.1),
    (2, 256, 4, 2, 64, True, 0.1),
    # non-causal D = 64 (the pipelined dK/dV kernel): one query tile pair per split, and GQA (jobs over heads)
    (1, 128, 2, 2, 64, False, 0.1),
    (1, 512, 8, 2, 64, False, 0.1),
]


@pytest.mark.parametrize("B,T,Hq,Hkv,D,causal,p", ATTN_CASES)
def test_attention(B, T, Hq, Hkv, D, causal, p):
    C = ext()
    W = (Hq + 2 * Hkv) * D
    qkv = rnd(B * T, W)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    scale = 1.0 / math.sqrt(D)
    sd = seed_obj(42)
    amask = C.attn_mask(B, T, Hq, p, sd.device_tensor, 11, q) if p else None
    o, lse = C.attn_fwd(q, k, v, amask, B, T, Hq, Hkv, scale, causal, p)
    ro, rlse = ref.attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p, sd, 11)
    # the kernels form the scores from Q * scale * log2(e) rounded to bf16 once per element (the
    # softmax scale folded into the operand): |score error| <= ~2^-9 |score|, the rounding the
    # reference's own bf16 bmm applies to every score (torch MHA under autocast).  A causal row with
    # one visible key has lse = that score, so the absolute lse tolerance is a few 2^-9 |score|.
    close(lse, rlse, 8e-3, 1e-3, "lse")
    close(o, ro, 2e-2, 3e-2, "O")
    do = rnd(B * T, Hq * D)
    dqkv = torch.empty_like(qkv)
    rdqkv = torch.empty_like(qkv)
    sl = lambda t: (t[:, :Hq * D], t[:, Hq * D:(Hq + Hkv) * D], t[:, (Hq + Hkv) * D:])
    C.attn_bwd(q, k, v, o, do, lse, amask if p else None, *sl(dqkv), B, T, Hq, Hkv, scale, causal, p)
    ref.attn_bwd(q, k, v, o, do, lse, *sl(rdqkv), B, T, Hq, Hkv, scale, causal, p, sd, 11)
    for name, a, b in zip("qkv", sl(dqkv), sl(rdqkv)):
        close(a, b, 5e-2, 5e-2, "d" + name)
    # the model's path: the dQ pass computes delta = rowsum(dO * O) itself (no delta kernel)
    from dltb.ops import functional as F_
    fdqkv = torch.empty_like(qkv)
    F_.attn_bwd(q, k, v, o, do, lse, amask, *sl(fdqkv), B, T, Hq, Hkv, scale, causal, p, sd, 11)
    for name, a, b in zip("qkv", sl(fdqkv), sl(rdqkv)):
        close(a, b, 5e-2, 5e-2, "fused-delta d" + name)


@pytest.mark.parametrize("B,T,Hq,Hkv,D,causal,p", [
    (1, 2048, 16, 16, 64, False, 0.1),     # TinyGPT-A bench shape (non-causal, dropout 0.1)
    (1, 4096, 32, 8, 128, True, 0.0),      # Mistral-7B shape: causal GQA 32/8, D=128, gsplit dK/dV
    (1, 1024, 4, 4, 64, True, 0.1),        # causal D=64 from T=1024: the dQ pass at 3 key splits
])
def test_attention_full_shape_fwd_bwd(B, T, Hq, Hkv, D, causal, p):
    """The shapes the benchmarks run, forward AND backward, against the fp32 reference."""
    test_attention(B, T, Hq, Hkv, D, causal, p)


def test_attention_tinygpt_shape():
    """Tier-A shape: T=2048, 16 heads, D=64, non-causal, dropout 0.1 (fwd only vs fp32)."""
    C = ext()
    B, T, H, D = 1, 2048, 16, 64
    qkv = rnd(B * T, 3 * H * D)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
    sd = seed_obj(3)
    amask = C.attn_mask(B, T, H, 0.1, sd.device_tensor, 1, q)
    o, lse = C.attn_fwd(q, k, v, amask, B, T, H, H, 0.125, False, 0.1)
    ro, rlse = ref.attn_fwd(q, k, v, B, T, H, H, 0.125, False, 0.1, sd, 1)
    close(o, ro, 2e-2, 3e-2, "O tier A")


# ------------------------------------------------------------------------------ optimizer
def _adam_tables(n, dst, chunk):
    nb = (n + chunk - 1) // chunk
    blk_seg = torch.zeros(nb, dtype=torch.int32, device=DEV)
    blk_start = torch.arange(nb, dtype=torch.int64, device=DEV) * chunk
    so = torch.zeros(1, dtype=torch.int64, device=DEV)
    sl = torch.tensor([n], dtype=torch.int64, device=DEV)
    sdst = torch.tensor([dst.data_ptr()], dtype=torch.int64, device=DEV)
    return blk_seg, blk_start, so, sl, sdst


@pytest.mark.parametrize("gdtype", [torch.float32, torch.bfloat16])
def test_adamw_matches_torch(gdtype):
    C = ext()
    n = 100_000
    p0 = torch.randn(n, device=DEV)
    master, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    out_bf16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    tp = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([tp], lr=1e-3, weight_decay=0.01)
    tabs = _adam_tables(n, out_bf16, C.adamw_chunk())
    for step in range(1, 4):
        g = torch.randn(n, device=DEV).to(gdtype)
        tp.grad = g.float()
        opt.step()
        C.adamw(master, m, v, g, *tabs, None, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, None)
    close(master, tp.detach(), 1e-6, 1e-5, "adamw master")
    close(out_bf16, tp.detach().to(torch.bfloat16), 1e-2, 1e-2, "adamw bf16 copy")


def test_adamw_mixed_alignment_segments():
    """FlatAdamW over two segments, the second neither 8-element aligned in the owner space nor 16-byte
    aligned at its destination: its blocks take the 8-byte path, the first segment's the 16-byte path;
    both match torch.optim.AdamW."""
    from dltb.optim.adamw import FlatAdamW
    n, cut = 100_000, 50_004
    p0 = torch.randn(n, device=DEV)
    out_bf16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    opt = FlatAdamW(p0.clone(), [(0, cut, out_bf16[:cut]), (cut, n - cut, out_bf16[cut:])], lr=1e-3)
    tp = torch.nn.Parameter(p0.clone())
    ref = torch.optim.AdamW([tp], lr=1e-3, weight_decay=0.01)
    for _ in range(3):
        g = torch.randn(n, device=DEV).to(torch.bfloat16)
        tp.grad = g.float()
        ref.step()
        opt.step(g, 1e-3)
    close(opt.master, tp.detach(), 1e-6, 1e-5, "adamw master (two segments)")
    close(out_bf16, tp.detach().to(torch.bfloat16), 1e-2, 1e-2, "adamw bf16 copy (two segments)")


def test_adamw_grid_cap_bitwise():
    """A capped grid (launch_segment(grid_cap=...): an update trickled beside other kernels) walks the block table
    block-strided: bitwise the one-block-per-row launch."""
    C = ext()
    n = 300_000
    p0 = torch.randn(n, device=DEV)
    outs = []
    for cap in (0, 7):
        master, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
        out_bf16 = torch.empty(n, device=DEV, dtype=torch.bfloat16)
        tabs = _adam_tables(n, out_bf16, C.adamw_chunk())
        assert tabs[0].numel() > 7
        for step in range(1, 3):
            g = torch.randn(n, device=DEV, generator=torch.Generator(DEV).manual_seed(step)).to(torch.bfloat16)
            C.adamw(master, m, v, g, *tabs, None, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, None, False, cap)
        outs.append((master, m, v, out_bf16))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_sumsq_clip():
    C = ext()
    x = torch.randn(1 << 20, device=DEV)
    acc = torch.zeros(1, device=DEV)
    C.sumsq_(x, acc)
    C.sumsq_(x.to(torch.bfloat16), acc)
    want = 2 * (x.double() ** 2).sum().item()
    assert abs(acc.item() - want) / want < 1e-3
    coef = torch.zeros(1, device=DEV)
    nrm = torch.zeros(1, device=DEV)
    C.clip_coef(acc, 1.0, coef, nrm, 1.0)
    assert abs(nrm.item() - math.sqrt(want)) / math.sqrt(want) < 1e-3
    assert abs(coef.item() - 1.0 / (math.sqrt(want) + 1e-6)) < 1e-6


def test_transpose_batched():
    """nb equally spaced matrices of a flat buffer transposed into a stacked buffer in one launch."""
    C = ext()
    R, Cc, nb, gap = 1024, 3072, 5, 4096
    flat = rnd(nb * (R * Cc + gap))
    src = [flat[i * (R * Cc + gap):i * (R * Cc + gap) + R * Cc].view(R, Cc) for i in range(nb)]
    dst = torch.empty(nb, Cc, R, device=DEV, dtype=torch.bfloat16)
    C.transpose_batched(src[0], dst[0], nb, R * Cc + gap, Cc * R)
    for i in range(nb):
        assert torch.equal(dst[i], src[i].t()), i


@pytest.mark.parametrize("with_res", [False, True])
def test_norm_fwd_mask_fused_matches_separate(with_res):
    """norm_fwd_mask (one launch: LN rows + attention-dropout mask blocks) is bitwise the separate
    norm_fwd and attn_mask launches."""
    C = ext()
    B, T, H, d = 1, 512, 8, 1024
    x, w, b = rnd(B * T, d), rnd(d, scale=0.1) + 1, rnd(d, scale=0.1)
    r = rnd(B * T, d) if with_res else None
    sd = seed_obj(77)
    p = 0.1 if with_res else 0.0
    s0, y0, m0, rs0 = C.norm_fwd(x, r, w, b, 1e-5, False, p, sd.device_tensor if p else None, 4, None)
    mk0 = C.attn_mask(B, T, H, 0.1, sd.device_tensor, 9, x)
    s1, y1, m1, rs1, mk1 = C.norm_fwd_mask(x, r, w, b, 1e-5, False, p, sd.device_tensor, 4, None, B, T, H, 0.1, 9)
    assert torch.equal(y0, y1) and torch.equal(m0, m1) and torch.equal(rs0, rs1)
    if with_res:
        assert torch.equal(s0, s1)
    assert torch.equal(mk0, mk1)


def test_attn_mask_words_match_reference():
    """The packed attention-dropout words are bit-exact with ops/rng.py attn_keep_mask: word
    (bh, t, h, q) bit mask_bit(n, i) <-> key 64t + 32n + (i&3) + 8(i>>2) + 4h (csrc/attn_mask.h)."""
    from dltb.ops import rng
    C = ext()
    B, T, H, p, site = 2, 256, 3, 0.1, 13
    sd = seed_obj(2024)
    q = rnd(B * T, H * 64)
    words = C.attn_mask(B, T, H, p, sd.device_tensor, site, q).view(B * H, T // 64, 2, T)
    u = words.to(torch.int64) & 0xFFFFFFFF
    bit = torch.arange(32, device=DEV)
    j = torch.where(bit < 16, 15 - bit, 31 - bit)                 # pair index of each bit
    i = 2 * (j & 7) + (bit >= 16).to(torch.int64)
    n = j >> 3
    got = torch.empty(B * H, T, T, dtype=torch.bool, device=DEV)
    for t in range(T // 64):
        for h in range(2):
            keys = 64 * t + 32 * n + (i & 3) + 8 * (i >> 2) + 4 * h          # [32]
            bits = ((u[:, t, h, :, None] >> bit) & 1).bool()                 # [BH, T(q), 32]
            got[:, :, keys] = bits
    s = rng.site_seed(int(sd.value), site)
    rows = torch.arange(B * H * T, dtype=torch.int64, device=DEV)[:, None]
    cols = torch.arange(T, dtype=torch.int64, device=DEV)[None, :]
    want = rng.attn_keep_mask(s, rows, cols, p).view(B * H, T, T)
    assert torch.equal(got, want)

