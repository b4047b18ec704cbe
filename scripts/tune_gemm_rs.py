#!/usr/bin/env python3
"""Pick, per per-layer product of a model, the own MFMA GEMM config (csrc/gemm_rs.hip) that beats the tuned
hipBLASLt solution, and write the own-GEMM table that ops/functional.py dispatches from.

    python scripts/tune_gemm_rs.py [--model A|M7B] [--cfgs 0,9,...] [--min-gain 0.03]
                                   [--out configs/gemm_rs/gemm_rs_gfx950.csv]

Per product (forward x W^T with the bias the model uses, data gradient dY (W^T)^T without): hipBLASLt (the
shipped tuned entry) and every gemm_rs config x tile walk that fits, timed in rounds inside one process
(HIP graphs of ``--iters`` calls, interleaved, median), each checked against an fp32 torch product.  A
config enters the table only when it is correct and faster than hipBLASLt by more than ``--min-gain``.
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

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="A")
    ap.add_argument("--cfgs", default="0,4,5,9,10,11,12,13,14")
    ap.add_argument("--gm", default="1,4")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--min-gain", type=float, default=0.03)
    ap.add_argument("--out", default=os.path.join(ROOT, "configs", "gemm_rs", "gemm_rs_gfx950.csv"))
    a = ap.parse_args()
    C = ext()
    blaslt.load()
    M, prods = products(a.model)
    cfgs = [int(c) for c in a.cfgs.split(",")]
    gms = [int(g) for g in a.gm.split(",")]
    rows = []
    torch.manual_seed(0)
    for name, N, K, has_bias in prods:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
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
        variants = [(c, g) for c in cfgs for g in gms if C.gemm_rs_supported(M, N, K, c)]
        fns = [lib] + [(lambda c=c, g=g: C.gemm_rs(x, w, y_own, bias, False, c, g)) for c, g in variants]
        ts = graph_time(fns, a.iters)
        lib()
        tol = 2 * (y_ref.float() - ref).abs().max().item() + 0.05
        best = None
        for (c, g), t in zip(variants, ts[1:]):
            out = C.gemm_rs(x, w, y_own, bias, False, c, g)
            torch.cuda.synchronize()
            ok = (out.float() - ref).abs().max().item() <= tol
            print(f"{name:10s} M{M} N{N} K{K}  cfg {c:2d} gm {g}: {t:6.1f} us (hipBLASLt {ts[0]:6.1f}){'' if ok else '  WRONG'}",
                  flush=True)
            if ok and (best is None or t < best[2]):
                best = (c, g, t)
        if best is not None and best[2] < ts[0] * (1 - a.min_gain):
            rows.append((M, N, K, int(has_bias), best[0], best[1], best[2], ts[0], name))
            print(f"  -> {name}: cfg {best[0]} gm {best[1]} {best[2]:.1f} us vs hipBLASLt {ts[0]:.1f} us", flush=True)
        else:
            print(f"  -> {name}: hipBLASLt stays ({ts[0]:.1f} us)", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    keep = {}
    if os.path.exists(a.out):                 # other models' rows survive
        with open(a.out) as f:
            for ln in f:
                if ln.startswith(("#", "m,")) or not ln.strip():
                    continue
                v = ln.strip().split(",")
                keep[tuple(int(x) for x in v[:4])] = ln.strip()
    for r in rows:
        keep[r[:4]] = ",".join(str(x) if not isinstance(x, float) else f"{x:.2f}" for x in r)
    with open(a.out, "w") as f:
        f.write("# own MFMA GEMM (csrc/gemm_rs.hip) per product: written by scripts/tune_gemm_rs.py\n")
        f.write("m,n,k,bias,cfg,gm,us,blaslt_us,product\n")
        for k in sorted(keep):
            f.write(keep[k] + "\n")
    print(f"wrote {len(keep)} rows to {a.out}")


if __name__ == "__main__":
    main()
