#!/usr/bin/env python3
"""hipBLASLt GEMM microbenchmark on the exact GEMMs of one TinyGPT / Mistral training step.

    python scripts/bench_gemm.py [--model A|M7B] [--iters 30]

Each linear layer contributes forward (x W^T), dgrad (dY W) and wgrad (dY^T x) products in the
layouts the fused Functions issue them.  Prints time, TFLOP/s and the share of the step's GEMM time.
"""
import argparse
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401


def shapes(model):
    if model == "A":
        M, d, f, V, L = 2048, 1024, 4096, 32000, 16
        lin = [("qkv", 3 * d, d), ("out", d, d), ("fc1", f, d), ("fc2", d, f)]
        return M, [(n, N, K, L) for n, N, K in lin] + [("lm_head", V, d, 1)]
    M, d, f, V, L, kvd = 4096, 4096, 14336, 32000, 32, 1024
    lin = [("qkv", d + 2 * kvd, d), ("o", d, d), ("gate_up", 2 * f, d), ("down", d, f)]
    return M, [(n, N, K, L) for n, N, K in lin] + [("lm_head", V, d, 1)]


def timeit(fn, iters):
    """GPU time per call: ``iters`` calls captured in one HIP graph (no host launch gaps)."""
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="A")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--layouts", action="store_true", help="also time the NT-form alternatives")
    ap.add_argument("--best", action="store_true", help="with --dltb: print only the fastest dltb config per product")
    ap.add_argument("--probe", action="store_true", help="single-workgroup K sweep of each dltb tile config")
    ap.add_argument("--dltb", action="store_true", help="also time the dltb MFMA GEMM (tile configs x split-K)")
    a = ap.parse_args()
    if a.probe:
        return probe(a.iters)
    M, lst = shapes(a.model)
    dt = torch.bfloat16
    rows, total = [], 0.0
    for name, N, K, reps in lst:
        x = torch.randn(M, K, device="cuda", dtype=dt)
        w = torch.randn(N, K, device="cuda", dtype=dt)
        dy = torch.randn(M, N, device="cuda", dtype=dt)
        y = torch.empty(M, N, device="cuda", dtype=dt)
        dx = torch.empty(M, K, device="cuda", dtype=dt)
        dw = torch.empty(N, K, device="cuda", dtype=dt)
        fl = 2.0 * M * N * K
        wT = w.t().contiguous()          # [K, N]
        dyT, xT = dy.t().contiguous(), x.t().contiguous()
        kinds = [("fwd", lambda: torch.mm(x, w.t(), out=y)),
                 ("dgrad", lambda: torch.mm(dy, w, out=dx)),
                 ("wgrad", lambda: torch.mm(dy.t(), x, out=dw))]
        if a.dltb:
            from dltb.ops._ext import ext
            C = ext()
            splits = (1, 2, 4, 8) if max(N, K, M) >= 8192 else (1, 2, 4)
            for cfg, sp, gm, stg in itertools.product(range(6), splits, (1, 4), (0, 2)):
                if gm > 1 and sp > 1:
                    continue
                pf = 0
                tag = f"c{cfg}s{sp}g{gm}n{stg}"
                kw = dict(splits=sp, cfg=cfg, pf=pf, gm=gm, stages=stg)
                if C.gemm_supported(M, N, K, False, cfg):
                    kinds.append((f"fwd[{tag}]", lambda kw=kw: C.gemm(x, w, y, None, False, False, **kw)))
                if C.gemm_supported(M, K, N, False, cfg):
                    kinds.append((f"dgT[{tag}]", lambda kw=kw: C.gemm(dy, wT, dx, None, False, False, **kw)))
                if C.gemm_supported(N, K, M, True, cfg):
                    kinds.append((f"wg[{tag}]", lambda kw=kw: C.gemm(dy, x, dw, None, True, False, **kw)))
        if a.layouts:
            kinds += [("dgradT", lambda: torch.mm(dy, wT.t(), out=dx)),     # W^T cached: NT form
                      ("wgradT", lambda: torch.mm(dyT, xT.t(), out=dw))]    # activations transposed
        for kind, fn in kinds:
            us = timeit(fn, a.iters)
            if kind in ("fwd", "dgrad", "wgrad"):
                total += us * reps
            rows.append((name, kind, M, N, K, reps, us, fl / us / 1e6))
    if a.best:
        best = {}
        for r in rows:
            key = (r[0], r[1][:3] if "[" in r[1] else r[1])
            if "[" in r[1] and (key not in best or r[6] < best[key][6]):
                best[key] = r
        rows = [r for r in rows if "[" not in r[1]] + list(best.values())
    for name, kind, m, n, k, reps, us, tf in rows:
        print(f"{name:8s} {kind:6s} M{m:6d} N{n:6d} K{k:6d} x{reps:3d} {us:8.1f} us {tf:7.1f} TF/s "
              f"{100 * us * reps / total:5.1f}%")
    print(f"total GEMM time per step (1 micro-batch): {total / 1e3:.3f} ms")


def probe(iters):
    """One workgroup (M = BM, N = BN) over growing K: per-64-deep-k-step cycles of the pipeline."""
    from dltb.ops._ext import ext
    C = ext()
    tiles = [(128, 128), (256, 128), (128, 256), (128, 64), (64, 128), (64, 64)]
    for cfg, (bm, bn) in enumerate(tiles):
        for tn in (False, True):
            if not C.gemm_supported(bm, bn, 1024, tn, cfg):
                continue
            out = []
            for K in (1024, 4096, 16384):
                a = torch.randn((K, bm) if tn else (bm, K), device="cuda", dtype=torch.bfloat16)
                b = torch.randn((K, bn) if tn else (bn, K), device="cuda", dtype=torch.bfloat16)
                c = torch.empty(bm, bn, device="cuda", dtype=torch.bfloat16)
                us = timeit(lambda: C.gemm(a, b, c, None, tn, False, 1, cfg), iters)
                out.append((K, us))
            (k0, t0), (k1, t1) = out[1], out[2]
            per = (t1 - t0) / ((k1 - k0) / 64) * 2.4e3      # cycles per k-step at 2.4 GHz
            mf = (bm // 2 // 32) * (bn // 2 // 32) * 4 * 32  # MFMA cycles per k-step per wave
            print(f"cfg{cfg} {bm}x{bn} {'TN' if tn else 'NT'}: " + "  ".join(f"K{k}={t:.1f}us" for k, t in out)
                  + f"  -> {per:.0f} cyc/k-step (MFMA-bound {mf})")


if __name__ == "__main__":
    main()
