#!/usr/bin/env python3
"""Would dQ and dK/dV gain from running concurrently?  (TinyGPT-A shape, dropout 0.1)

Each pass alone fills one 8-wave workgroup per CU (2 waves / SIMD) and spends ~45 % of its wave
cycles waiting (profiles/attention_pmc_tinygpt_a.txt); together they would hold 4 waves / SIMD.
Times (median of rounds, microseconds per layer):
  serial   dQ (delta fused) -> dK/dV                       (what the model runs)
  split    delta kernel -> dQ -> dK/dV                     (same work, delta separate)
  concur   delta kernel -> [dQ || dK/dV] on two streams
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops._ext import ext  # noqa: E402


def main():
    C = ext()
    dev, bf = "cuda", torch.bfloat16
    B, T, H, D = 1, 2048, 16, 64
    d = H * D
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(T, 3 * d, device=dev, dtype=bf, generator=g)
    q, k, v = qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:]
    do = torch.randn(T, d, device=dev, dtype=bf, generator=g)
    seed = torch.tensor([1234], device=dev, dtype=torch.int64)
    mask = C.attn_mask(B, T, H, 0.1, seed, 1, q)
    o, lse = C.attn_fwd(q, k, v, mask, B, T, H, H, 0.125, False, 0.1)
    delta = torch.empty_like(lse)
    dq = torch.empty_like(q)
    dkv = torch.empty(T, 2 * d, device=dev, dtype=bf)
    side = torch.cuda.Stream()
    main_s = torch.cuda.current_stream()

    def serial():
        C.attn_bwd_part(1, q, k, v, do, lse, delta, mask, dq, None, B, T, H, H, 0.125, False, 0.1, o)
        C.attn_bwd_part(0, q, k, v, do, lse, delta, mask, dkv[:, :d], dkv[:, d:], B, T, H, H, 0.125, False, 0.1)

    def split():
        dl = C.attn_bwd_delta(o, do, B, T, H)
        C.attn_bwd_part(1, q, k, v, do, lse, dl, mask, dq, None, B, T, H, H, 0.125, False, 0.1)
        C.attn_bwd_part(0, q, k, v, do, lse, dl, mask, dkv[:, :d], dkv[:, d:], B, T, H, H, 0.125, False, 0.1)

    def concur():
        dl = C.attn_bwd_delta(o, do, B, T, H)
        side.wait_stream(main_s)
        with torch.cuda.stream(side):
            C.attn_bwd_part(1, q, k, v, do, lse, dl, mask, dq, None, B, T, H, H, 0.125, False, 0.1)
        C.attn_bwd_part(0, q, k, v, do, lse, dl, mask, dkv[:, :d], dkv[:, d:], B, T, H, H, 0.125, False, 0.1)
        main_s.wait_stream(side)

    def timed(fn, iters=30):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters * 1e3

    cases = {"serial": serial, "split": split, "concur": concur}
    for fn in cases.values():
        fn()
    torch.cuda.synchronize()
    res = {n: [] for n in cases}
    for _ in range(7):
        for n, fn in cases.items():
            res[n].append(timed(fn))
    for n, v in res.items():
        print(f"{n:7s} {statistics.median(v):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
