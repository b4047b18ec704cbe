"""Device dispatch of the dltb ops: GPU tensors run the gfx950 HIP kernels of ``dltb._C``
(raising if the extension is missing), CPU tensors run the torch references of :mod:`.ref`.

GEMMs run on hipBLASLt: the problems of the shipped tuning table through the extension API with
their tuned (solution, split-K, wgm) triple (:mod:`.blaslt`), everything else as plain ``torch``
matmuls (TunableOp); gradient-producing GEMMs write straight into the engine's flat gradient slots
(``out=`` / ``addmm_``) so no gradient is ever copied.
"""
import torch

from . import blaslt as _blt
from . import ref
from ._ext import ext


def _gpu(t):
    return t.is_cuda


def _sd(seed):
    return None if seed is None else seed.device_tensor


# ------------------------------------------------------------------------------ norms
def _into(out, t):
    """CPU path of an op with a caller-provided output: copy the reference result into it."""
    if out is None:
        return t
    out.copy_(t)
    return out


def norm_fwd(x, r, w, b, eps, rms, p=0.0, seed=None, site=0, y_out=None):
    """Returns (s, y, mean, rstd); s = x + dropout(r) when r is given (else None).  ``y_out``: write
    y into this (layer-strided activation buffer) view."""
    if _gpu(x):
        s, y, mean, rstd = ext().norm_fwd(x, r, w, b, eps, rms, p, _sd(seed) if p > 0 else None, site, y_out)
        return (s if r is not None else None), y, (None if rms else mean), rstd
    s, y, mean, rstd = ref.norm_fwd(x, r, w, b, eps, rms, p, seed, site)
    return s, _into(y_out, y), mean, rstd


def norm_fwd_mask(x, r, w, b, eps, rms, p, seed, site, y_out, B, T, Hq, p_attn, attn_site, mask_out=None,
                  part=None):
    """norm_fwd plus the attention-dropout mask of (B, T, Hq) at ``attn_site``, on the GPU in one
    launch (csrc/norm.hip norm_fwd_mask_kernel).  Returns (s, y, mean, rstd, mask); mask is None on
    the CPU or without attention dropout.  ``part`` = 0 / 1: only the first / second half of the
    mask's tile groups, written into ``mask_out`` (or a new mask for part 0) -- a mask generated
    by two launches, each beside a latency-bound row norm."""
    if _gpu(x) and p_attn > 0:
        g0, g1 = 0, -1
        if part is not None:
            half = (B * Hq * (T // 64) * 2) // 2
            g0, g1 = (0, half) if part == 0 else (half, -1)
        s_, y, mean, rstd, mask = ext().norm_fwd_mask(x, r, w, b, eps, rms, p, seed.device_tensor, site, y_out,
                                                      B, T, Hq, p_attn, attn_site, mask_out, g0, g1)
        return (s_ if r is not None else None), y, (None if rms else mean), rstd, mask
    s_, y, mean, rstd = norm_fwd(x, r, w, b, eps, rms, p, seed, site, y_out)
    return s_, y, mean, rstd, (attn_mask(B, T, Hq, p_attn, seed, attn_site, x) if part is None else None)


# colpart segment kinds (csrc/colreduce.hip)
_PLAIN, _GELU, _DROP, _LN, _RMS = 0, 1, 2, 3, 4

class GradReducer:
    """Batches the column reductions of one backward unit: producer kernels write fp32 column
    partials (``colpart``) and register them here; :meth:`flush` sums every set into its bf16
    gradient slot with ONE ``colreduce_multi`` launch (instead of one reduce launch per bias /
    norm weight).  On the CPU the ops reduce immediately and this is a no-op."""

    MAX = 64                     # csrc/launchers.h DLTB_COLRED_MAX

    def __init__(self, max_sets: int = 12, defer_plain: bool = False):
        self.max_sets = min(int(max_sets), self.MAX)
        self.parts, self.outs, self.acc = [], [], []
        # plain column sums whose partials may ride along with the NEXT colpart launch (the
        # engine's shared reducer: the QKV bias sum of block i joins block i-1's dropout colpart)
        self.defer_plain = bool(defer_plain)
        self.pending = []

    def take_pending(self, n: int):
        out, self.pending = self.pending[:n], self.pending[n:]
        return out

    def add(self, part2d, out, accumulate):
        if out is None:
            return
        if len(self.parts) == self.max_sets:
            self.flush()
        self.parts.append(part2d)
        self.outs.append(out)
        self.acc.append(bool(accumulate))

    def flush(self):
        while self.pending:
            extra = self.take_pending(3)
            parts = ext().colpart([_PLAIN] * len(extra), [e[0] for e in extra], [None] * len(extra),
                                  [None] * len(extra), [None] * len(extra), [None] * len(extra), 0.0, None,
                                  [0] * len(extra))
            for (src, out, acc), pt in zip(extra, parts):
                self.add(pt[0], out, acc)
        if self.parts:
            ext().colreduce_multi(self.parts, self.outs, self.acc)
            self.parts, self.outs, self.acc = [], [], []


def norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms, red=None, bias=None,
             dx_out=None, drop=None):
    """dx, and dgamma/dbeta written into their gradient slots.

    With a :class:`GradReducer` the dgamma/dbeta partials (and, with ``bias=(src, slot, acc)``, the
    column sum of ``src`` -- ``src="dx"`` meaning this call's output) come from ONE colpart launch
    and are reduced at ``red.flush()``.

    ``drop=(p, seed, site, dm_out, db, db_acc)``: also return dm = Dropout_backward(dx) of dropout
    site ``site`` with its column sum into ``db`` -- ``(dx, dm)`` -- fused into the same kernel on
    the GPU (the previous block's MLP dropout and fc2 bias gradient)."""
    if drop is not None:
        dp, dseed, dsite, dm_out, db, db_acc = drop
        if red is not None and _gpu(dy) and ext().norm_bwd_fused_supported(dy.shape[-1]):
            C = ext()
            dm = torch.empty_like(s) if dm_out is None else dm_out
            dx, part = C.norm_bwd_fused(dy, s, w, mean, rstd, dres, rms, False, dx_out, dm, dp,
                                        _sd(dseed) if dp > 0 else None, dsite)
            red.add(part[0], gw, accumulate)
            if not rms:
                red.add(part[1], gb, accumulate)
            red.add(part[-1], db, db_acc)
            if bias is not None and bias[1] is not None:
                assert not isinstance(bias[0], str), "drop and a dx bias sum are exclusive"
                if red.defer_plain:
                    red.pending.append((bias[0], bias[1], bias[2]))
                else:
                    parts = C.colpart([_PLAIN], [bias[0]], [None], [None], [None], [None], 0.0, None, [0])
                    red.add(parts[0][0], bias[1], bias[2])
            return dx, dm
        dx = norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms, red, bias, dx_out)
        red_local = red if red is not None else GradReducer()
        dm = dropout_bwd_bias(dx, dp, dseed, dsite, db, db_acc, red_local, out=dm_out)
        if red is None:
            red_local.flush()
        return dx, dm
    if red is not None:
        if _gpu(dy) and ext().norm_bwd_fused_supported(dy.shape[-1]):
            # one kernel: dx + gamma / beta partials (+ the column partials of dx itself)
            C = ext()
            has_bias = bias is not None and bias[1] is not None
            dx_sum = has_bias and isinstance(bias[0], str)
            dx, part = C.norm_bwd_fused(dy, s, w, mean, rstd, dres, rms, dx_sum, dx_out)
            red.add(part[0], gw, accumulate)
            if not rms:
                red.add(part[1], gb, accumulate)
            if dx_sum:
                red.add(part[-1], bias[1], bias[2])
            elif has_bias and red.defer_plain:
                red.pending.append((bias[0], bias[1], bias[2]))
            elif has_bias:
                parts = C.colpart([_PLAIN], [bias[0]], [None], [None], [None], [None], 0.0, None, [0])
                red.add(parts[0][0], bias[1], bias[2])
            return dx
        if _gpu(dy):
            C = ext()
            dx = _into(dx_out, C.norm_bwd_dx(dy, s, w, mean, rstd, dres, rms))
            kinds, a, b, mn, rs = [_RMS if rms else _LN], [dy], [s], [mean], [rstd]
            if bias is not None and bias[1] is not None:
                src = dx if isinstance(bias[0], str) else bias[0]
                kinds.append(_PLAIN), a.append(src), b.append(None), mn.append(None), rs.append(None)
            parts = C.colpart(kinds, a, b, [None] * len(kinds), mn, rs, 0.0, None, [0] * len(kinds))
            red.add(parts[0][0], gw, accumulate)
            if not rms:
                red.add(parts[0][1], gb, accumulate)
            if len(parts) > 1:
                red.add(parts[1][0], bias[1], bias[2])
            return dx
        dx = _into(dx_out, ref.norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms))
        if bias is not None and bias[1] is not None:
            ref.colsum_into(dx if isinstance(bias[0], str) else bias[0], bias[1], bias[2])
        return dx
    if _gpu(dy):
        return ext().norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms)
    return ref.norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms)


# ------------------------------------------------------------------------------ elementwise
def gelu_fwd(f, out=None):
    return ext().gelu_fwd(f, out) if _gpu(f) else _into(out, ref.gelu_fwd(f))


def gelu_fwd_grad(f, out=None, gp_out=None):
    """(g, gp) = (GELU(f), GELU'(f)) in one pass (GPU): the forward of the dGELU-epilogue path."""
    return tuple(ext().gelu_fwd_grad(f, out, gp_out))


# dGELU in the fc2 data gradient's epilogue: own-GEMM table rows with bias = 2 (``gemm_rs_aux``)
_DGELU = 2


_GELU_OUT = 3              # own-GEMM table rows with bias = 3: bias + GELU-output epilogue (fc1 forward)


def _nt_operands_ok(*ts):
    """Row-major 2-D bf16 operands with 16-byte aligned base and row stride (the own GEMM's 16-byte loads)."""
    return all(t.dim() == 2 and t.dtype == torch.bfloat16 and t.stride(1) == 1 and t.stride(0) % 8 == 0
               and t.data_ptr() % 16 == 0 for t in ts)


def linear_fwd_gelu(x2d, w, b, g_out=None):
    """(f, GELU(f)) = (x W^T + b, its GELU) from ONE own-GEMM launch (the epilogue writes both; GELU of
    the rounded f, bitwise gelu_fwd's), when the own-GEMM table has a bias = 3 row for the shape whose tile
    config supports the GELU-output epilogue; else None (the caller runs GEMM + gelu_fwd)."""
    global own_gemm_calls
    if not (x2d.is_cuda and b is not None and _nt_operands_ok(x2d, w)):
        return None
    M, K = x2d.shape
    N = w.shape[0]
    hit = rs_table().get((M, N, K, _GELU_OUT))
    if hit is None or not (b.dtype == torch.bfloat16 and b.is_contiguous() and b.data_ptr() % 8 == 0
                           and ext().gemm_rs_gelu_supported(M, N, K, hit[0])):
        return None
    f = torch.empty(M, N, dtype=x2d.dtype, device=x2d.device)
    g = g_out if g_out is not None else torch.empty_like(f)
    if g.stride(0) != f.stride(0) or g.stride(1) != 1 or g.data_ptr() % 16:
        return None
    own_gemm_calls += 1
    ext().gemm_rs(x2d, w, f, b, False, hit[0], hit[1], gelu_out=g)
    return f, g


def dgelu_fused(M, N, K, dtype=torch.bfloat16):
    """True when the fc2 data gradient (M tokens, N = the MLP width, K = the model width) runs with the dGELU
    epilogue: the forward then keeps GELU'(f) instead of f (models/tinygpt.py).  Requires a bf16 step (the
    GELU'-writing forward kernel is bf16-only) and a table row whose tile config supports the aux epilogue;
    the backward still falls back (:func:`dgelu_backward`) when the engine has no cached W^T."""
    hit = rs_table().get((M, N, K, _DGELU))
    return hit is not None and dtype == torch.bfloat16 and ext().gemm_rs_aux_supported(M, N, K, hit[0])


def linear_dgrad_dgelu(dy2d, wt, gp, db, accumulate, red, out=None):
    """df = (dY W) * GELU'(f) with the fc1 bias gradient's column partials, one own-GEMM launch
    (C = dY (W^T)^T; the epilogue multiplies by gp = GELU'(f) from the forward, rounds once and sums the rounded
    columns per 128-row tile; the partials are reduced at ``red.flush()``).  None when the table has no row or
    an operand's layout does not fit the kernel (the caller then takes :func:`dgelu_backward`'s fallback)."""
    global own_gemm_calls
    if wt is None or red is None:
        return None
    M, K = dy2d.shape
    N = wt.shape[0]
    hit = rs_table().get((M, N, K, _DGELU))
    if hit is None or not _nt_operands_ok(dy2d, wt, gp) or not ext().gemm_rs_aux_supported(M, N, K, hit[0]):
        return None
    if out is not None and not (_nt_operands_ok(out) and out.stride(0) == gp.stride(0)):
        return None
    own_gemm_calls += 1
    df, part = ext().gemm_rs_aux(dy2d, wt, out, gp, hit[0], hit[1])
    red.add(part, db, accumulate)
    return df


def dgelu_backward(dm, w2, w2t, gp, db, accumulate, red, out=None):
    """df = (dm W2) * GELU'(f) when the forward saved gp = GELU'(f): the fused own-GEMM epilogue, or -- when
    that cannot run (no cached W^T on this engine, an operand layout the kernel refuses) -- the plain data
    gradient, the product with gp in fp32 rounded once, and the fc1 bias column sum of the rounded df."""
    df = linear_dgrad_dgelu(dm, w2t, gp, db, accumulate, red, out=out)
    if df is not None:
        return df
    dg = linear_dgrad(dm, w2, w2t)
    res = (dg.float() * gp.float()).to(dg.dtype)
    df = _into(out, res)
    if red is not None and df.is_cuda:
        parts = ext().colpart([_PLAIN], [df], [None], [None], [None], [None], 0.0, None, [0])
        red.add(parts[0][0], db, accumulate)
    else:
        colsum_into(df, db, accumulate)
    return df


def gelu_bwd(dg, f, db, accumulate, red=None, out=None):
    """df = dg * gelu'(f); the fc1 bias gradient colsum(df) is fused (reduced at red.flush())."""
    if _gpu(dg):
        if red is None:
            return _into(out, ext().gelu_bwd(dg, f, db, accumulate))
        df = torch.empty_like(dg) if out is None else out
        extra = _take_row_matched(red, dg, 2)        # deferred plain sums ride along (same row count)
        n = len(extra)
        parts = ext().colpart([_GELU] + [_PLAIN] * n, [dg] + [e[0] for e in extra], [f] + [None] * n,
                              [df] + [None] * n, [None] * (n + 1), [None] * (n + 1), 0.0, None, [0] * (n + 1))
        red.add(parts[0][0], db, accumulate)
        for (src, o, acc), pt in zip(extra, parts[1:]):
            red.add(pt[0], o, acc)
        return df
    return _into(out, ref.gelu_bwd(dg, f, db, accumulate))


def _take_row_matched(red, t, limit):
    """Up to ``limit`` of the reducer's deferred plain column sums whose source has ``t``'s row count
    (colpart segments must share it); they are removed from ``red.pending``."""
    rows, keep, extra = t.numel() // t.shape[-1], [], []
    for e in red.pending:
        (extra if len(extra) < limit and e[0].numel() // e[0].shape[-1] == rows else keep).append(e)
    red.pending = keep
    return extra


def dropout_bwd_bias(g, p, seed, site, db, accumulate, red, out=None):
    """dm = dropout_mask(g) / (1-p) (the Dropout backward) with colsum(dm) -> db fused."""
    if _gpu(g):
        dm = torch.empty_like(g) if out is None else out
        extra = _take_row_matched(red, g, 2)
        n = len(extra)
        parts = ext().colpart([_DROP] + [_PLAIN] * n, [g] + [e[0] for e in extra], [None] * (n + 1),
                              [dm] + [None] * n, [None] * (n + 1), [None] * (n + 1), p,
                              _sd(seed) if p > 0 else None, [site] + [0] * n)
        red.add(parts[0][0], db, accumulate)
        for (src, o, acc), pt in zip(extra, parts[1:]):
            red.add(pt[0], o, acc)
        return dm
    dm = _into(out, ref.dropout(None, g, p, seed, site))
    if db is not None:
        ref.colsum_into(dm, db, accumulate)
    return dm


def colsum_into(src, out, accumulate):
    if out is None:
        return
    if _gpu(src):
        ext().colsum_into(src, out, accumulate)
    else:
        ref.colsum_into(src, out, accumulate)


def dropout(x, r, p, seed, site):
    """x + dropout(r) (x may be None -> dropout(r) alone, also used as the mask-replay backward)."""
    if _gpu(r):
        return ext().dropout(x, r, p, _sd(seed) if p > 0 else None, site)
    return ref.dropout(x, r, p, seed, site)


def swiglu_fwd(gu):
    return ext().swiglu_fwd(gu) if _gpu(gu) else ref.swiglu_fwd(gu)


def swiglu_bwd(dh, gu):
    return ext().swiglu_bwd(dh, gu) if _gpu(dh) else ref.swiglu_bwd(dh, gu)


def rope_(qkv2d, cos, sin, T, heads, D, inverse=False):
    if _gpu(qkv2d):
        ext().rope_(qkv2d, cos, sin, T, heads, D, inverse)
    else:
        ref.rope_(qkv2d, cos, sin, T, heads, D, inverse)


# ------------------------------------------------------------------------------ embedding / loss
def embed_fwd(idx, wte, wpe, p, seed, site):
    if _gpu(wte):
        return ext().embed_fwd(idx, wte, wpe, p, _sd(seed) if p > 0 else None, site)
    return ref.embed_fwd(idx, wte, wpe, p, seed, site)


def embed_bwd(dx, idx, dwte, dwpe, accumulate_wpe, p, seed, site):
    if _gpu(dx):
        ext().embed_bwd(dx, idx, dwte, dwpe, accumulate_wpe, p, _sd(seed) if p > 0 else None, site)
    else:
        ref.embed_bwd(dx, idx, dwte, dwpe, accumulate_wpe, p, seed, site)


def xent_fwd_bwd_(logits2d, targets1d, ignore_index=-1):
    if _gpu(logits2d):
        return ext().xent_fwd_bwd_(logits2d, targets1d, ignore_index)
    return ref.xent_fwd_bwd_(logits2d, targets1d, ignore_index)


def xent_mean(loss_rows, targets1d, ignore_index=-1):
    """f32[2] = (mean loss over non-ignored rows, max(count, 1)), computed on the device (one
    launch on MI355X instead of compare / sum / clamp / cast / div)."""
    if _gpu(loss_rows):
        return ext().xent_mean(loss_rows, targets1d, ignore_index)
    count = (targets1d != ignore_index).sum().clamp(min=1).to(torch.float32)
    return torch.stack([loss_rows.sum() / count, count])


def scale_by(x, num, den=None):
    """(x * num/den, g = num/den as f32[1]) with the scale kept on the device (no host sync)."""
    num = num.to(torch.float32).reshape(-1)
    if _gpu(x):
        g = torch.empty(1, device=x.device, dtype=torch.float32)
        return ext().scale_by(x.contiguous(), num, den, g), g
    g = num[:1] / den.reshape(-1)[:1] if den is not None else num[:1].clone()
    return (x * g).to(x.dtype), g


def head_dgrad(dl, w, wt, g):
    """dX = g * dL W for an LM head with weight W [V, d].  K = V is long and the output (tokens x d)
    small.  With a cached W^T both operands are K-contiguous: a tuned hipBLASLt split-K solution
    when the table has the problem (TinyGPT-A: 116 us vs 149 us for the own kernel + reduce,
    profiles/head_dgrad_blaslt_r2.txt), then g applied by one small scale kernel; otherwise the
    own split-K MFMA GEMM with g as a device alpha in its split-K reduction."""
    if _gpu(dl) and wt is not None and dl.stride(1) == 1 and dl.dtype == torch.bfloat16:
        M, K = dl.shape
        N = wt.shape[0]
        if _blt.active():
            dh = torch.empty(M, N, dtype=dl.dtype, device=dl.device)
            if _blt.mm(dl, wt.t(), dh, False):
                return ext().scale_by(dh, g, None, None)
        C = ext()
        if C.gemm_supported(M, N, K, False, 2):
            return C.gemm(dl, wt, None, None, False, False, 4, 2, 0, 1, g)
    if _gpu(dl):
        _note_torch_fallback("head_dgrad", dl.shape, w.shape)
    return (torch.mm(dl, w) * g).to(dl.dtype)


torch_fallbacks = {}        # op -> calls that ran a torch GEMM on the GPU (reported by bench.py / the harness)


def _note_torch_fallback(op, *shapes):
    """A GPU product that neither hipBLASLt's table nor an own kernel took: counted, and warned about once per op."""
    n = torch_fallbacks.get(op, 0)
    torch_fallbacks[op] = n + 1
    if n == 0:
        import warnings
        warnings.warn(f"dltb: {op} {shapes} runs as a plain torch GEMM on the GPU (no tuned or own kernel)")


# ------------------------------------------------------------------------------ attention
def attn_mask(B, T, Hq, p, seed, site, like):
    """Packed dropout keep-bits for attention (GPU only).  Returns None on the CPU or without
    dropout."""
    if p <= 0 or not like.is_cuda:
        return None
    return ext().attn_mask(B, T, Hq, p, seed.device_tensor, site, like)


def attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p, seed, site, mask=None, o_out=None):
    """Returns (o, lse, aux); ``aux`` (the packed dropout mask on the GPU) goes back into attn_bwd."""
    if _gpu(q):
        if p > 0 and mask is None:
            mask = ext().attn_mask(B, T, Hq, p, seed.device_tensor, site, q)
        o, lse = ext().attn_fwd(q, k, v, mask if p > 0 else None, B, T, Hq, Hkv, scale, causal, p, o_out)
        return o, lse, (mask if p > 0 else None)
    o, lse = ref.attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p, seed, site)
    return _into(o_out, o), lse, None


def attn_bwd(q, k, v, o, do, lse, aux, dq, dk, dv, B, T, Hq, Hkv, scale, causal, p, seed, site):
    """dQ (query-major kernel, which also forms delta = rowsum(dO * O) for its rows), then dK/dV
    (key-major kernel, reading that delta)."""
    if _gpu(q):
        C = ext()
        m = aux if p > 0 else None
        delta = torch.empty_like(lse)
        C.attn_bwd_part(1, q, k, v, do, lse, delta, m, dq, None, B, T, Hq, Hkv, scale, causal, p, o)
        C.attn_bwd_part(0, q, k, v, do, lse, delta, m, dk, dv, B, T, Hq, Hkv, scale, causal, p)
    else:
        ref.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, T, Hq, Hkv, scale, causal, p, seed, site)


# ------------------------------------------------------------------------------ linear
# Own MFMA GEMM (csrc/gemm_rs.hip, register-staged, software-pipelined) for the per-layer NT products
# C[M, N] = A[M, K] B[N, K]^T (+ bias) where it beats the tuned hipBLASLt solution: the shapes, tile
# configs and tile walks come from configs/gemm_rs/gemm_rs_gfx950.csv (written by
# scripts/tune_gemm_rs.py from same-process A/B timings); DLTB_OWN_GEMM=0 turns the dispatch off.
import csv as _csv
import os as _os

_RS_FILE = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))),
                         "configs", "gemm_rs", "gemm_rs_gfx950.csv")
_rs_table = None
own_gemm_calls = 0          # products issued through gemm_rs (tests check that the path ran)


def rs_table():
    """(M, N, K, has_bias) -> (cfg, gm) of the shipped own-GEMM table ({} when off or absent)."""
    global _rs_table
    if _rs_table is None:
        _rs_table = {}
        path = _os.environ.get("DLTB_OWN_GEMM_TABLE", _RS_FILE)
        if path != _RS_FILE and path != "none":
            from .blaslt import resolve_config_path
            path = resolve_config_path(path, "DLTB_OWN_GEMM_TABLE")
        if _os.environ.get("DLTB_OWN_GEMM", "1") == "1" and _os.path.exists(path):
            with open(path) as f:
                for r in _csv.DictReader(ln for ln in f if not ln.startswith("#")):
                    _rs_table[(int(r["m"]), int(r["n"]), int(r["k"]), int(r["bias"]))] = (int(r["cfg"]), int(r["gm"]))
    return _rs_table


def _own_nt(a, b_nk, bias=None):
    """a [M, K] @ b_nk[N, K]^T (+ bias) through gemm_rs when the table holds the shape, else None."""
    global own_gemm_calls
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b_nk.dtype == torch.bfloat16 and a.dim() == 2
            and a.stride(1) == 1 and b_nk.stride(1) == 1 and a.stride(0) % 8 == 0 and b_nk.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b_nk.data_ptr() % 16 == 0):      # 16-byte operand loads
        return None
    if bias is not None and not (bias.dtype == torch.bfloat16 and bias.is_contiguous()
                                 and bias.data_ptr() % 8 == 0):               # 8-byte bias loads
        return None
    M, K = a.shape
    N = b_nk.shape[0]
    hit = rs_table().get((M, N, K, int(bias is not None)))
    if hit is None:
        return None
    own_gemm_calls += 1
    return ext().gemm_rs(a, b_nk, None, bias, False, hit[0], hit[1])


def _tuned(a, b, bias=None):
    """a @ b (+ bias) through the tuned hipBLASLt table, or None when the problem is not in it."""
    if not (_blt.active() and a.is_cuda):
        return None
    y = a.new_empty(a.shape[0], b.shape[1])
    return y if _blt.mm(a, b, y, False, bias) else None


def linear_fwd(x2d, w, b=None):
    y = _own_nt(x2d, w, b)
    if y is not None:
        return y
    y = _tuned(x2d, w.t(), b)
    if y is not None:
        return y
    if b is None:
        return torch.mm(x2d, w.t())
    return torch.addmm(b, x2d, w.t())


def linear_dgrad(dy2d, w, wt=None):
    """dX = dY W; with a cached contiguous W^T the product runs as dY (W^T)^T (hipBLASLt NT form)."""
    if wt is not None:
        y = _own_nt(dy2d, wt)            # dY (W^T)^T: the cached W^T is the NT operand
        if y is not None:
            return y
    rhs = wt.t() if wt is not None else w
    y = _tuned(dy2d, rhs)
    return y if y is not None else torch.mm(dy2d, rhs)


# hipBLASLt runs a product fastest with both operands K-contiguous (1.48-1.52 PFLOP/s on
# Mistral-7B's [4096 x 4096-28672] shapes); a weight gradient dY^T X has neither (dY^T is an
# M-contiguous view, X N-contiguous: 1.03-1.04 PFLOP/s), and one K-contiguous side already gives
# 1.22-1.28 (profiles/gemm_layouts_r2.txt).  So for a large product the SMALLER operand is
# transposed into a K-contiguous copy first (an LDS-tiled transpose, ~2 x bytes / 3.5 TB/s) when
# the expected 15 % of the GEMM time pays for it 1.5 times over: the FFN weight gradients of
# Mistral-7B qualify, TinyGPT-A's (K = tokens >> dims, batched over blocks) do not.
_WGRAD_GEMM_FLOPS = 1.1e15
_WGRAD_GAIN = 0.15
_TRANSPOSE_BPS = 3.5e12


def wgrad_operands(dy2d, x2d):
    """(a, b) with dW = a @ b: (dy^T, x), or with the smaller one replaced by a K-contiguous copy."""
    a, b = dy2d.t(), x2d
    if not (dy2d.is_cuda and dy2d.dim() == 2 and dy2d.dtype in (torch.bfloat16, torch.float16)):
        return a, b
    K, M = dy2d.shape
    N = x2d.shape[1]
    gemm_s = 2.0 * M * N * K / _WGRAD_GEMM_FLOPS
    small = dy2d if dy2d.numel() <= x2d.numel() else x2d
    cost_s = 2.0 * small.numel() * small.element_size() / _TRANSPOSE_BPS + 5e-6
    if _WGRAD_GAIN * gemm_s <= 1.5 * cost_s or not small.is_contiguous() or K % 4 or small.shape[1] % 4:
        return a, b
    t = torch.empty(small.shape[1], small.shape[0], dtype=small.dtype, device=small.device)
    ext().transpose_into(small, t)
    return (t, b) if small is dy2d else (a, t.t())


# Own weight-gradient GEMM (csrc/gemm_tn.hip): dW = dY^T X with both operands token-major as the model stores
# them -- the layout hipBLASLt runs 25-45 % below its K-contiguous rate.  DLTB_OWN_WGRAD=0: hipBLASLt.
_OWN_WGRAD = _os.environ.get("DLTB_OWN_WGRAD", "1") == "1"


def own_wgrad(dy, x, dw, accumulate):
    """dw (+)= dy^T x for batched [b, T, *] views on gemm_tn when the shapes and layouts fit; else False."""
    if not (_OWN_WGRAD and dy.is_cuda and dy.dtype == x.dtype == dw.dtype and dy.dtype == torch.bfloat16
            and dy.dim() == x.dim() == dw.dim() and dy.dim() in (2, 3)):
        return False
    if any(t.stride(-1) != 1 or t.stride(-2) % 8 or t.data_ptr() % 16 or (t.dim() == 3 and t.stride(0) % 8)
           for t in (dy, x, dw)):
        return False
    K, M = dy.shape[-2], dy.shape[-1]
    N = x.shape[-1]
    if not ext().gemm_tn_supported(M, N, K):
        return False
    # Batched products only, from one 256 x 256 tile per CU up.  Below one tile per CU (the few-block dW batches
    # of a gradient bucket at world > 1) hipBLASLt's smaller tiles / split-K fill the chip; single products
    # (the tied head's wgrad, Mistral-7B's per-layer dW) run on cold operands where hipBLASLt measured faster in
    # the step: head 115 vs 121-138 us, M7B 200 vs 229 ms per window (profiles/gemm_tn_r6.txt)
    if dy.dim() != 3 or dy.shape[0] < 2 or (M // 256) * (N // 256) * dy.shape[0] < _cu_count(dy.device):
        return False
    ext().gemm_tn(dy, x, dw, bool(accumulate))
    return True


_CUS = {}


def _cu_count(dev):
    if dev not in _CUS:
        _CUS[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
    return _CUS[dev]


def linear_wgrad(dy2d, x2d, dw, db, accumulate):
    """dW (+)= dy^T x written straight into the gradient slot; db (+)= colsum(dy)."""
    if dw is not None and own_wgrad(dy2d, x2d, dw, accumulate):
        if db is not None:
            colsum_into(dy2d, db, accumulate)
        return
    if dw is not None:
        a, b = wgrad_operands(dy2d, x2d)
        if not _blt.mm(a, b, dw, accumulate):
            if accumulate:
                dw.addmm_(a, b)
            else:
                torch.mm(a, b, out=dw)
    if db is not None:
        colsum_into(dy2d, db, accumulate)
