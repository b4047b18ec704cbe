#!/usr/bin/env python3
"""Attention kernel microbenchmark (forward, dK/dV, dQ, dropout-mask) on the two model shapes.

    python scripts/bench_attn.py [--iters 50]

Prints one line per kernel: time per call and TFLOP/s (causal FLOPs counted over the visible
half).  Shapes: TinyGPT-A (B1 T2048 H16 D64, dropout 0.1, non-causal) and Mistral-7B
(B1 T4096 Hq32 Hkv8 D128, causal).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops._ext import ext  # noqa: E402

SHAPES = {"tinygpt_a": dict(B=1, T=2048, Hq=16, Hkv=16, D=64, causal=False, p=0.1),
          "tinygpt_a_p0": dict(B=1, T=2048, Hq=16, Hkv=16, D=64, causal=False, p=0.0),
          "m7b": dict(B=1, T=4096, Hq=32, Hkv=8, D=128, causal=True, p=0.0),
          # three TinyGPT-A micro-batches: 768 query blocks, so several workgroups share a CU
          "tinygpt_a_b3": dict(B=3, T=2048, Hq=16, Hkv=16, D=64, causal=False, p=0.1),
          # causal D = 64 (mtiny-like): the shapes the causal split caps of csrc/attention.hip act on
          "causal_d64": dict(B=1, T=2048, Hq=16, Hkv=16, D=64, causal=True, p=0.0),
          "causal_d64_short": dict(B=4, T=512, Hq=8, Hkv=8, D=64, causal=True, p=0.0)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def run(name, B, T, Hq, Hkv, D, causal, p, iters):
    C = ext()
    g = torch.Generator(device="cuda").manual_seed(0)
    dev = "cuda"
    qkv = torch.randn(B * T, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16, generator=g)
    q, k, v = qkv[:, :Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    do = torch.randn(B * T, Hq * D, device=dev, dtype=torch.bfloat16, generator=g)
    seed = torch.tensor([1234], device=dev, dtype=torch.int64)
    scale = D ** -0.5
    mask = C.attn_mask(B, T, Hq, p, seed, 1, q) if p > 0 else None
    o, lse = C.attn_fwd(q, k, v, mask, B, T, Hq, Hkv, scale, causal, p)
    delta = C.attn_bwd_delta(o, do, B, T, Hq)
    dq = torch.empty_like(q)
    dkv = torch.empty(B * T, 2 * Hkv * D, device=dev, dtype=torch.bfloat16)
    dk, dv = dkv[:, :Hkv * D], dkv[:, Hkv * D:]
    frac = 0.5 if causal else 1.0
    f_fwd = 4.0 * B * Hq * T * T * D * frac
    res = {}
    res["fwd"] = (timeit(lambda: C.attn_fwd(q, k, v, mask, B, T, Hq, Hkv, scale, causal, p), iters), f_fwd)
    res["dkdv"] = (timeit(lambda: C.attn_bwd_part(0, q, k, v, do, lse, delta, mask, dk, dv, B, T, Hq, Hkv, scale,
                                                  causal, p), iters), f_fwd * 2.0)   # S, dP, dV, dK
    res["dq"] = (timeit(lambda: C.attn_bwd_part(1, q, k, v, do, lse, delta, mask, dq, None, B, T, Hq, Hkv, scale,
                                                causal, p), iters), f_fwd * 1.5)     # S, dP, dQ
    res["delta"] = (timeit(lambda: C.attn_bwd_delta(o, do, B, T, Hq), iters), 0.0)
    if p > 0:
        res["mask"] = (timeit(lambda: C.attn_mask(B, T, Hq, p, seed, 1, q), iters), 0.0)
    tot = 0.0
    for kname, (us, fl) in res.items():
        tot += us
        tf = fl / us / 1e6 if fl else 0.0
        print(f"{name:10s} {kname:6s} {us:9.1f} us  {tf:7.1f} TFLOP/s")
    print(f"{name:10s} total  {tot:9.1f} us per layer (fwd + bwd)")
    return {k: v[0] for k, v in res.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="tinygpt_a,m7b")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = {n: run(n, iters=a.iters, **SHAPES[n]) for n in a.shapes.split(",")}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
