"""Device dispatch of the dltb ops: GPU tensors run the gfx950 HIP kernels of ``dltb._C``
(raising if the extension is missing), CPU tensors run the torch references of :mod:`.ref`.

GEMMs are plain ``torch`` matmuls (hipBLASLt on ROCm); gradient-producing GEMMs write straight
into the engine's flat gradient slots (``out=`` / ``addmm_``) so no gradient is ever copied.
"""
import torch

from . import ref
from ._ext import ext


def _gpu(t):
    return t.is_cuda


def _sd(seed):
    return None if seed is None else seed.device_tensor


# ------------------------------------------------------------------------------ norms
def norm_fwd(x, r, w, b, eps, rms, p=0.0, seed=None, site=0):
    """Returns (s, y, mean, rstd); s = x + dropout(r) when r is given (else None)."""
    if _gpu(x):
        s, y, mean, rstd = ext().norm_fwd(x, r, w, b, eps, rms, p, _sd(seed) if p > 0 else None, site)
        return (s if r is not None else None), y, (None if rms else mean), rstd
    return ref.norm_fwd(x, r, w, b, eps, rms, p, seed, site)


def norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms):
    if _gpu(dy):
        return ext().norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms)
    return ref.norm_bwd(dy, s, w, mean, rstd, dres, gw, gb, accumulate, rms)


# ------------------------------------------------------------------------------ elementwise
def gelu_fwd(f):
    return ext().gelu_fwd(f) if _gpu(f) else ref.gelu_fwd(f)


def gelu_bwd(dg, f, db, accumulate):
    return ext().gelu_bwd(dg, f, db, accumulate) if _gpu(dg) else ref.gelu_bwd(dg, f, db, accumulate)


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


# ------------------------------------------------------------------------------ attention
def attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p, seed, site):
    if _gpu(q):
        o, lse = ext().attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p,
                                _sd(seed) if p > 0 else None, site)
        return o, lse
    return ref.attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p, seed, site)


def attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, T, Hq, Hkv, scale, causal, p, seed, site):
    if _gpu(q):
        ext().attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, T, Hq, Hkv, scale, causal, p,
                       _sd(seed) if p > 0 else None, site)
    else:
        ref.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, B, T, Hq, Hkv, scale, causal, p, seed, site)


# ------------------------------------------------------------------------------ linear
def linear_fwd(x2d, w, b=None):
    if b is None:
        return torch.mm(x2d, w.t())
    return torch.addmm(b, x2d, w.t())


def linear_wgrad(dy2d, x2d, dw, db, accumulate):
    """dW (+)= dy^T x written straight into the gradient slot; db (+)= colsum(dy)."""
    if dw is not None:
        if accumulate:
            dw.addmm_(dy2d.t(), x2d)
        else:
            torch.mm(dy2d.t(), x2d, out=dw)
    if db is not None:
        colsum_into(dy2d, db, accumulate)
