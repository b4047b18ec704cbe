#!/usr/bin/env python3
"""The register-staged NT GEMM (csrc/gemm_rs.hip) against hipBLASLt on the per-layer products of a step.

    python scripts/bench_gemm_rs.py [--model A|M7B] [--iters 50] [--cfgs 0,1,2] [--gm 1,4] [--cold]

Every product is C[M, N] = A[M, K] B[N, K]^T (+ bias): the forward x W^T and the data gradient
dY (W^T)^T against the engine's cached W^T.  For each product prints hipBLASLt (the tuned table
entry when the problem has one, else torch) and every gemm_rs config that fits, with its max error
against an fp32 torch product.  Operands are uniform random (clocks depend on the data).
Timing: ``iters`` calls captured in one HIP graph, A/B interleaved in rounds inside one process;
``--cold`` writes a 512 MB buffer between calls (each call then starts with its operands outside
the L2s, as inside a training step).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops import blaslt  # noqa: E402
from dltb.ops._ext import ext  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_bench_util import graph_time, products  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="A")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cfgs", default="")
    ap.add_argument("--gm", default="4")
    ap.add_argument("--cold", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    C = ext()
    blaslt.load()
    M, prods = products(a.model)
    cfgs = [int(c) for c in a.cfgs.split(",") if c != ""] or list(range(15))
    gms = [int(g) for g in a.gm.split(",")]
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda") if a.cold else None
    tot_ref, tot_best = 0.0, 0.0
    torch.manual_seed(0)
    for name, N, K, has_bias in prods:
        if a.only and name not in a.only.split(","):
            continue
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda", dtype=torch.bfloat16) if has_bias else None
        ref = x.float() @ w.float().t() + (bias.float() if has_bias else 0)
        y_ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y_own = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        wt = w.t()

        def cold():
            if flush is not None:
                flush.fill_(1)

        def lib():
            cold()
            if not blaslt.mm(x, wt, y_ref, False, bias):
                if bias is None:
                    torch.mm(x, wt, out=y_ref)
                else:
                    torch.addmm(bias, x, wt, out=y_ref)

        variants = [(c, gm) for c in cfgs for gm in gms if C.gemm_rs_supported(M, N, K, c)]

        def own(c, gm):
            cold()
            return C.gemm_rs(x, w, y_own, bias, False, c, gm)
        fns = [lib] + [(lambda c=c, gm=gm: own(c, gm)) for c, gm in variants]
        if flush is not None:
            fns.append(cold)
        ts = graph_time(fns, a.iters)
        t_flush = ts[-1] if flush is not None else 0.0
        ts = [t - t_flush for t in ts[:len(fns) - (1 if flush is not None else 0)]]
        lib()
        err_ref = (y_ref.float() - ref).abs().max().item()
        fl = 2.0 * M * N * K
        print(f"{name:11s} M{M} N{N:6d} K{K:6d}  hipBLASLt {ts[0]:7.1f} us {fl / ts[0] / 1e6:6.0f} TF/s "
              f"(err {err_ref:.3g})", flush=True)
        best = ts[0]
        for (c, gm), t in zip(variants, ts[1:]):
            out = own(c, gm)
            torch.cuda.synchronize()
            err = (out.float() - ref).abs().max().item()
            print(f"    rs c{c:<2d} g{gm}  {t:7.1f} us {fl / t / 1e6:6.0f} TF/s  x{ts[0] / t:4.2f}  err {err:.3g}"
                  + ("  MISMATCH" if err > 2 * err_ref + 0.05 else ""), flush=True)
            best = min(best, t)
        tot_ref += ts[0]
        tot_best += best
    print(f"sum over products: hipBLASLt {tot_ref:.1f} us, best-of {tot_best:.1f} us")


if __name__ == "__main__":
    main()
