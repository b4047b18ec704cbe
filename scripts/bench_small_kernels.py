#!/usr/bin/env python3
"""Per-call GPU time of the small (memory-bound) kernels of a TinyGPT-A block at M = 2048 tokens:
norms, GELU, dropout, column-partial reductions, batched reduce, transpose (HIP-graph timed)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops._ext import ext  # noqa: E402
from dltb.ops.functional import _DROP, _GELU, _LN, _PLAIN  # noqa: E402


def t_us(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    C = ext()
    M, d, f = 2048, 1024, 4096
    bf = dict(device="cuda", dtype=torch.bfloat16)
    x, r, dy = torch.randn(M, d, **bf), torch.randn(M, d, **bf), torch.randn(M, d, **bf)
    w, b = torch.ones(d, **bf), torch.zeros(d, **bf)
    ff, dg = torch.randn(M, f, **bf), torch.randn(M, f, **bf)
    dq = torch.randn(M, 3 * d, **bf)
    seed = torch.tensor([7], device="cuda", dtype=torch.int64)
    s_, y, mean, rstd = C.norm_fwd(x, r, w, b, 1e-5, False, 0.0, None, 0)
    df, dm = torch.empty_like(dg), torch.empty_like(dy)
    out = torch.empty(f, **bf)
    half = (1 * 16 * (M // 64) * 2) // 2
    mask = C.norm_fwd_mask(x, r, w, b, 1e-5, False, 0.1, seed, 2, None, 1, M, 16, 0.1, 5, None, 0, half)[4]
    parts = C.colpart([_LN, _PLAIN], [dy, dq], [x, None], [None, None], [mean, None], [rstd, None], 0.0, None, [0, 0])
    rows = [
        ("norm_fwd (LN)", lambda: C.norm_fwd(x, None, w, b, 1e-5, False, 0.0, None, 0), 8),
        ("norm_fwd (LN + residual)", lambda: C.norm_fwd(x, r, w, b, 1e-5, False, 0.0, None, 0), 16),
        ("norm_fwd_mask (LN+res, half mask)", lambda: C.norm_fwd_mask(x, r, w, b, 1e-5, False, 0.1, seed, 2, None, 1, M, 16,
                                                                    0.1, 5, mask, 0, half), 20),
        ("norm_fwd_mask (LN+res, other half)", lambda: C.norm_fwd_mask(x, r, w, b, 1e-5, False, 0.0, seed, 0, None, 1, M, 16,
                                                                     0.1, 5, mask, half, -1), 20),
        ("norm_bwd_dx (+dres)", lambda: C.norm_bwd_dx(dy, x, w, mean, rstd, r, False), 16),
        ("norm_bwd_fused (+dres, dx sum)", lambda: C.norm_bwd_fused(dy, x, w, mean, rstd, r, False, True, None, None,
                                                                    0.0, None, 0), 16),
        ("norm_bwd_fused (+dres, drop)", lambda: C.norm_bwd_fused(dy, x, w, mean, rstd, r, False, False, None, dm, 0.1,
                                                                  seed, 4), 20),
        ("gelu_fwd", lambda: C.gelu_fwd(ff), 32),
        ("dropout add", lambda: C.dropout(x, r, 0.1, seed, 3), 12),
        ("colpart DROP", lambda: C.colpart([_DROP], [dy], [None], [dm], [None], [None], 0.1, seed, [3]), 8),
        ("colpart GELU", lambda: C.colpart([_GELU], [dg], [ff], [df], [None], [None], 0.0, None, [0]), 48),
        ("colpart LN + PLAIN(dx)", lambda: C.colpart([_LN, _PLAIN], [dy, x], [x, None], [None, None], [mean, None], [rstd, None], 0.0, None, [0, 0]), 12),
        ("colpart LN + PLAIN(dqkv)", lambda: C.colpart([_LN, _PLAIN], [dy, dq], [x, None], [None, None], [mean, None], [rstd, None], 0.0, None, [0, 0]), 20),
        ("colreduce_multi x8", lambda: C.colreduce_multi([parts[0][0], parts[0][1], parts[1][0]] * 2 + [parts[0][0]] * 2,
                                                          [w, b, torch.empty(3 * d, **bf)] * 2 + [w, b], [False] * 8), 4),
        ("transpose 3072x1024", lambda: C.transpose_into(dq.view(3 * d, d) if False else torch.empty(3 * d, d, **bf), torch.empty(d, 3 * d, **bf)), 12),
    ]
    print(f"{'kernel':28s} {'us':>8s} {'MB':>6s} {'GB/s':>8s}")
    for name, fn, mb in rows:
        us = t_us(fn)
        print(f"{name:28s} {us:8.2f} {mb:6d} {mb * 1e6 / 1.048576 / us / 1e3 * 1.048576:8.0f}")


if __name__ == "__main__":
    main()
