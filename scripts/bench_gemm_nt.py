#!/usr/bin/env python3
"""The own NT GEMM (csrc/gemm_nt.hip) against hipBLASLt on the per-layer products of a step.

    python scripts/bench_gemm_nt.py [--model A|M7B] [--iters 50] [--sweep] [--split]

Every product is C[M, N] = A[M, K] B[N, K]^T (+ bias): the forward x W^T and the data gradient
dY (W^T)^T against the engine's cached W^T.  Prints hipBLASLt (the tuned table entry when the
problem has one, else torch / TunableOp), the own kernel at its default pick and, with --sweep,
every (tile config, group) point; each with its max error against an fp32 torch product.
Timing: ``iters`` calls captured in one HIP graph; A/B alternate in rounds inside one process.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops import blaslt  # noqa: E402
from dltb.ops._ext import ext  # noqa: E402

CFGS = {0: "128x64k64", 1: "128x128k64", 2: "128x192k32", 3: "128x256k32", 4: "256x128k32", 5: "64x128k64",
        6: "128x64r4", 7: "128x128s2", 8: "128x64s2", 9: "256x128s2", 10: "128x128s2fix"}
SPLIT = (7, 8, 9)   # split-K configs: fp32 planes [2, M, N], summed by the consumer
FIXUP = (10,)       # split-K with the pair fixup: bf16 output


def products(model):
    if model == "A":
        M, d, f = 2048, 1024, 4096
        return M, [("qkv.fwd", 3 * d, d, True), ("out.fwd", d, d, True), ("fc1.fwd", f, d, True),
                   ("fc2.fwd", d, f, True), ("fc2.dgrad", f, d, False), ("fc1.dgrad", d, f, False),
                   ("out.dgrad", d, d, False), ("qkv.dgrad", d, 3 * d, False)]
    M, d, f, kv = 4096, 4096, 14336, 1024
    return M, [("qkv.fwd", d + 2 * kv, d, False), ("o.fwd", d, d, False), ("gateup.fwd", 2 * f, d, False),
               ("down.fwd", d, f, False), ("down.dgrad", f, d, False), ("gateup.dgrad", d, 2 * f, False),
               ("o.dgrad", d, d, False), ("qkv.dgrad", d, d + 2 * kv, False)]


def graph_time(fns, iters, rounds=5):
    """Per-call GPU time of each fn (median over rounds, the fns interleaved in every round)."""
    graphs = []
    for fn in fns:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        graphs.append(g)
    times = [[] for _ in fns]
    for _ in range(rounds):
        for i, g in enumerate(graphs):
            g.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            times[i].append(s.elapsed_time(e) / iters * 1e3)
    return [sorted(t)[len(t) // 2] for t in times]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="A")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--split", action="store_true", help="also time the split-K configs (fp32 planes)")
    ap.add_argument("--fixup", action="store_true", help="also time the split-K pair-fixup config (bf16 out)")
    a = ap.parse_args()
    C = ext()
    blaslt.load()
    M, prods = products(a.model)
    tot_ref = tot_own = 0.0
    torch.manual_seed(0)
    for name, N, K, has_bias in prods:
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
        bias = torch.randn(N, device="cuda", dtype=torch.bfloat16) if has_bias else None
        ref = x.float() @ w.float().t() + (bias.float() if has_bias else 0)
        y_ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y_own = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        wt = w.t()

        def lib():
            if not blaslt.mm(x, wt, y_ref, False, bias):
                if bias is None:
                    torch.mm(x, wt, out=y_ref)
                else:
                    torch.addmm(bias, x, wt, out=y_ref)
        variants = [("own", -1, 4)]
        if a.sweep:
            variants += [(f"c{c}g{gm}", c, gm) for c in CFGS for gm in (1, 4)
                         if C.gemm_nt_supported(M, N, K, c)]
        if a.split:
            variants += [(f"c{c}g{gm}", c, gm) for c in SPLIT for gm in (1, 4) if C.gemm_nt_supported(M, N, K, c)]
        if a.fixup:
            variants += [(f"c{c}g{gm}", c, gm) for c in FIXUP for gm in (1, 4) if C.gemm_nt_supported(M, N, K, c)]
        planes = torch.empty(2, M, N, device="cuda", dtype=torch.float32)
        ws = torch.empty(M * N, device="cuda", dtype=torch.float32)
        sync = torch.zeros(max(C.gemm_nt_fixup_ints(10, M, N), 1), device="cuda", dtype=torch.int32)

        def own(c, gm):
            if c in FIXUP:
                return C.gemm_nt(x, w, y_own, bias, False, c, gm, ws, sync)
            return C.gemm_nt(x, w, planes if c in SPLIT else y_own, bias, False, c, gm)
        fns = [lib] + [(lambda c=c, gm=gm: own(c, gm)) for _, c, gm in variants]
        ts = graph_time(fns, a.iters)
        lib()
        err_ref = (y_ref.float() - ref).abs().max().item()
        fl = 2.0 * M * N * K
        print(f"{name:11s} M{M} N{N:6d} K{K:6d}  hipBLASLt {ts[0]:7.1f} us {fl / ts[0] / 1e6:6.0f} TF/s "
              f"(err {err_ref:.3g})", flush=True)
        for (tag, c, gm), t in zip(variants, ts[1:]):
            out = own(c, gm)
            torch.cuda.synchronize()
            err = ((out.sum(0) if c in SPLIT else out.float()) - ref).abs().max().item()
            pick = CFGS.get(c, "pick")
            print(f"    {tag:6s} {pick:11s} {t:7.1f} us {fl / t / 1e6:6.0f} TF/s  x{ts[0] / t:4.2f}  err {err:.3g}"
                  + ("  MISMATCH" if err > 2 * err_ref + 0.05 else ""), flush=True)
        tot_ref += ts[0]
        tot_own += ts[1]
    print(f"sum over products: hipBLASLt {tot_ref:.1f} us, own {tot_own:.1f} us")


if __name__ == "__main__":
    main()
