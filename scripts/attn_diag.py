#!/usr/bin/env python3
"""Attention numerics diagnostic: one test case, this build's fwd/bwd outputs and the fp32
reference, saved for offline comparison (DLTB_EXT_PATH selects the build).

    python scripts/attn_diag.py OUT.pt [B T Hq Hkv D causal p]
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops._ext import ext  # noqa: E402
from dltb.ops import ref  # noqa: E402
from dltb.ops.rng import StepSeed  # noqa: E402


def main():
    out = sys.argv[1]
    a = [int(x) for x in sys.argv[2:7]] if len(sys.argv) > 2 else [2, 256, 4, 4, 64]
    causal = bool(int(sys.argv[7])) if len(sys.argv) > 7 else False
    p = float(sys.argv[8]) if len(sys.argv) > 8 else 0.1
    B, T, Hq, Hkv, D = a
    C = ext()
    torch.manual_seed(0)
    W = (Hq + 2 * Hkv) * D
    qkv = torch.randn(B * T, W, device="cuda").to(torch.bfloat16)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    scale = 1.0 / math.sqrt(D)
    sd = StepSeed(42, 0, device="cuda")
    sd.next()
    amask = C.attn_mask(B, T, Hq, p, sd.device_tensor, 11, q) if p else None
    o, lse = C.attn_fwd(q, k, v, amask, B, T, Hq, Hkv, scale, causal, p)
    ro, rlse = ref.attn_fwd(q, k, v, B, T, Hq, Hkv, scale, causal, p, sd, 11)
    do = torch.randn(B * T, Hq * D, device="cuda").to(torch.bfloat16)
    dqkv = torch.empty_like(qkv)
    rdqkv = torch.empty_like(qkv)
    sl = lambda t: (t[:, :Hq * D], t[:, Hq * D:(Hq + Hkv) * D], t[:, (Hq + Hkv) * D:])  # noqa: E731
    C.attn_bwd(q, k, v, o, do, lse, amask, *sl(dqkv), B, T, Hq, Hkv, scale, causal, p)
    ref.attn_bwd(q, k, v, o, do, lse, *sl(rdqkv), B, T, Hq, Hkv, scale, causal, p, sd, 11)
    torch.cuda.synchronize()
    res = dict(qkv=qkv.cpu(), do=do.cpu(), o=o.cpu(), lse=lse.cpu(), ro=ro.cpu(), rlse=rlse.cpu(),
               dqkv=dqkv.cpu(), rdqkv=rdqkv.cpu(), mask=amask.cpu() if amask is not None else None)
    torch.save(res, out)
    for name, x, y in [("o", o, ro), ("lse", lse, rlse)] + [("d" + n, x, y) for n, x, y in zip("qkv", sl(dqkv), sl(rdqkv))]:
        e = (x.float() - y.float()).abs()
        print(f"{name}: max err {e.max().item():.4g} mean err {e.mean().item():.4g} |ref| mean {y.float().abs().mean().item():.4g}")


if __name__ == "__main__":
    main()
