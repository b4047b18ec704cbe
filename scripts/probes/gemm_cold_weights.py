#!/usr/bin/env python3
"""Does a cold weight operand explain the in-step vs microbench gap of the K-long GEMMs?

    python scripts/probes/gemm_cold_weights.py [--copies 48]

TinyGPT-A per-layer products through hipBLASLt (the step's own path, ops/blaslt.py), timed in one HIP
graph of 48 calls: 'warm' re-uses one weight (L2 / MALL resident after the first call, as in
scripts/bench_gemm_nt.py), 'coldW' cycles through --copies weight buffers (> 256 MB of MALL, so each
call reads its weight from HBM, as a layer does inside a step), 'coldAW' cycles the activation too.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops import blaslt  # noqa: E402


def timed(fn, iters):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(i)
    ts = []
    for _ in range(5):
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(ts)[2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--copies", type=int, default=48)
    ap.add_argument("--iters", type=int, default=48)
    a = ap.parse_args()
    blaslt.load()
    M, d, f = 2048, 1024, 4096
    prods = [("qkv.fwd", 3 * d, d, True), ("out.fwd", d, d, True), ("fc1.fwd", f, d, True), ("fc2.fwd", d, f, True),
             ("fc2.dgrad", f, d, False), ("fc1.dgrad", d, f, False), ("out.dgrad", d, d, False),
             ("qkv.dgrad", d, 3 * d, False)]
    for name, N, K, has_bias in prods:
        xs = [torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for _ in range(a.copies)]
        ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05 for _ in range(a.copies)]
        bias = torch.randn(N, device="cuda", dtype=torch.bfloat16) if has_bias else None
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

        def run(x, w):
            wt = w.t()
            if not blaslt.mm(x, wt, y, False, bias):
                torch.mm(x, wt, out=y) if bias is None else torch.addmm(bias, x, wt, out=y)
        c = a.copies
        warm = timed(lambda i: run(xs[0], ws[0]), a.iters)
        cold_w = timed(lambda i: run(xs[0], ws[i % c]), a.iters)
        cold_aw = timed(lambda i: run(xs[i % c], ws[i % c]), a.iters)
        print(f"{name:10s} N{N:5d} K{K:5d}  warm {warm:6.1f} us  coldW {cold_w:6.1f} us (+{cold_w - warm:4.1f})  "
              f"coldAW {cold_aw:6.1f} us (+{cold_aw - warm:4.1f})  W {N * K * 2 / 2**20:4.0f} MiB", flush=True)
        del xs, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
