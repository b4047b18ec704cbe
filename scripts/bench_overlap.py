#!/usr/bin/env python3
"""Can independent work hide under the VALU-bound attention / dropout-mask kernels?

TinyGPT-A shapes (B1 T2048 H16 D64, dropout 0.1).  Attention and the dropout-mask generator are
VALU / LDS bound; the weight-gradient GEMMs are MFMA bound.  This times, on one MI355X,
each alone and then concurrently (the second on a side HIP stream):

  A  attention backward (dQ + dK/dV)          B  one block's 4 dW GEMMs (qkv, out, fc1, fc2)
  C  attention forward                         D  the dropout-mask kernel of the next layer
  E  fc1 + fc2 forward GEMMs

and prints alone-sum vs concurrent wall time per pair (interleaved rounds, median).

    python scripts/bench_overlap.py [--iters 30] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops._ext import ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    C = ext()
    dev, bf = "cuda", torch.bfloat16
    B, T, H, D, d, F = 1, 2048, 16, 64, 1024, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    rn = lambda *s: torch.randn(*s, device=dev, dtype=bf, generator=g)  # noqa: E731
    qkv = rn(T, 3 * d)
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    do = rn(T, d)
    seed = torch.tensor([1234], device=dev, dtype=torch.int64)
    mask = C.attn_mask(B, T, H, 0.1, seed, 1, q)
    o, lse = C.attn_fwd(q, k, v, mask, B, T, H, H, 0.125, False, 0.1)
    delta = torch.empty_like(lse)
    dq = torch.empty_like(q)
    dkv = torch.empty(T, 2 * d, device=dev, dtype=bf)
    h1, x_o, h2, gl = rn(T, d), rn(T, d), rn(T, d), rn(T, F)
    dqkv, dx1, df, dm = rn(T, 3 * d), rn(T, d), rn(T, F), rn(T, d)
    w_in, w_o, w1, w2 = rn(3 * d, d), rn(d, d), rn(F, d), rn(d, F)
    dw = [torch.empty_like(w) for w in (w_in, w_o, w1, w2)]

    def attn_bwd():
        C.attn_bwd_part(1, q, k, v, do, lse, delta, mask, dq, None, B, T, H, H, 0.125, False, 0.1, o)
        C.attn_bwd_part(0, q, k, v, do, lse, delta, mask, dkv[:, :d], dkv[:, d:], B, T, H, H, 0.125, False, 0.1)

    def dw_gemms():
        torch.mm(dqkv.t(), h1, out=dw[0])
        torch.mm(dx1.t(), x_o, out=dw[1])
        torch.mm(df.t(), h2, out=dw[2])
        torch.mm(dm.t(), gl, out=dw[3])

    def attn_fwd():
        C.attn_fwd(q, k, v, mask, B, T, H, H, 0.125, False, 0.1)

    def mask_gen():
        C.attn_mask(B, T, H, 0.1, seed, 3, q)

    def mlp_fwd():
        f = torch.mm(h2, w1.t())
        torch.mm(gl, w2.t())
        return f

    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def timed(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters * 1e3

    def pair(f1, f2):
        def run():
            side.wait_stream(main_s)
            f1()
            with torch.cuda.stream(side):
                f2()
            main_s.wait_stream(side)
        return run

    cases = {"A attn_bwd": attn_bwd, "B dW x4": dw_gemms, "C attn_fwd": attn_fwd, "D mask": mask_gen,
             "E mlp fwd": mlp_fwd, "A||B": pair(attn_bwd, dw_gemms), "C||B": pair(attn_fwd, dw_gemms),
             "E||D": pair(mlp_fwd, mask_gen), "C||D": pair(attn_fwd, mask_gen)}
    for fn in cases.values():
        fn()
    torch.cuda.synchronize()
    res = {name: [] for name in cases}
    for _ in range(a.rounds):
        for name, fn in cases.items():
            res[name].append(timed(fn))
    med = {name: statistics.median(v) for name, v in res.items()}
    for name, v in med.items():
        print(f"{name:12s} {v:8.1f} us")
    for p, (x, y) in {"A||B": ("A attn_bwd", "B dW x4"), "C||B": ("C attn_fwd", "B dW x4"),
                      "E||D": ("E mlp fwd", "D mask"), "C||D": ("C attn_fwd", "D mask")}.items():
        print(f"{p:6s} alone-sum {med[x] + med[y]:8.1f} us  concurrent {med[p]:8.1f} us  "
              f"saved {med[x] + med[y] - med[p]:7.1f} us")


if __name__ == "__main__":
    main()
