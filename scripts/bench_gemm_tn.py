#!/usr/bin/env python3
"""The own weight-gradient GEMM (csrc/gemm_tn.hip) against hipBLASLt on the dW products of a training step.

    python scripts/bench_gemm_tn.py [--iters 10] [--only dw.fc1,head.wgrad]

Problems (TinyGPT-A, ZeRO-2 at world 1, grad-accum 4): the window-wide batched dW of each parameter kind over
the 16 blocks (K = 4 x 2048 tokens; operands are views of layer-strided activation buffers, outputs views of
the flat gradient buffer at the block stride, as parallel/wgrad.py issues them) and the tied head's weight
gradient (V = 32000 x d = 1024 over 2048 tokens); plus two Mistral-7B-shape products.  hipBLASLt runs the
shipped tuned solution through the extension API when the problem is in configs/blaslt (what the step runs),
else torch (TunableOp).  Timing: graph replay, interleaved rounds in one process; uniform random operands.
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
from gemm_bench_util import graph_time  # noqa: E402

BLOCK = 12596224            # TinyGPT-A parameters per block (the flat gradient buffer's block stride)


def problems():
    d, f, T = 1024, 4096, 8192
    # name, batch, M (out), N (in), K (tokens), operand row strides, gradient slot stride
    return [("dw.qkv", 16, 3 * d, d, T), ("dw.out", 16, d, d, T), ("dw.fc1", 16, f, d, T), ("dw.fc2", 16, d, f, T),
            ("head.wgrad", 1, 32000, d, 2048), ("m7b.down", 1, 4096, 14336, 4096), ("m7b.gateup", 1, 28672, 4096, 4096)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    C = ext()
    blaslt.load()
    torch.manual_seed(0)
    tot = [0.0, 0.0]
    for name, B, M, N, K in problems():
        if a.only and name not in a.only.split(","):
            continue
        if B > 1:
            dy = ((torch.rand(B, K, M, device="cuda") * 2 - 1)).to(torch.bfloat16)
            x = ((torch.rand(B, K, N, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
            flat = torch.zeros(B * BLOCK, device="cuda", dtype=torch.bfloat16)
            dw_ref = flat.as_strided((B, M, N), (BLOCK, N, 1))
            flat2 = torch.zeros_like(flat)
            dw_own = flat2.as_strided((B, M, N), (BLOCK, N, 1))
        else:
            dy = ((torch.rand(K, M, device="cuda") * 2 - 1)).to(torch.bfloat16)
            x = ((torch.rand(K, N, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
            dw_ref = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            dw_own = torch.empty_like(dw_ref)

        def lib():
            at = dy.transpose(-1, -2)
            if not blaslt.mm(at, x, dw_ref, False):
                if B > 1:
                    torch.bmm(at, x, out=dw_ref)
                else:
                    torch.mm(at, x, out=dw_ref)

        def own():
            C.gemm_tn(dy, x, dw_own, False)
        t_lib, t_own = graph_time([lib, own], a.iters)
        lib()
        own()
        torch.cuda.synchronize()
        ref = (dy.float().transpose(-1, -2) @ x.float())
        e_lib = (dw_ref.float() - ref).abs().max().item()
        e_own = (dw_own.float() - ref).abs().max().item()
        fl = 2.0 * B * M * N * K
        print(f"{name:11s} b{B:2d} M{M:6d} N{N:6d} K{K:6d}  hipBLASLt {t_lib:8.1f} us {fl / t_lib / 1e6:6.0f} TF/s "
              f"(err {e_lib:.3g})   own {t_own:8.1f} us {fl / t_own / 1e6:6.0f} TF/s (err {e_own:.3g})  "
              f"x{t_lib / t_own:4.2f}" + ("  MISMATCH" if e_own > 2 * e_lib + 0.05 else ""),
              flush=True)
        if name.startswith("dw."):
            tot[0] += t_lib
            tot[1] += t_own
        del dy, x
    if tot[0]:
        print(f"window dW sum: hipBLASLt {tot[0]:.1f} us, own {tot[1]:.1f} us  x{tot[0] / tot[1]:.2f}")


if __name__ == "__main__":
    main()
