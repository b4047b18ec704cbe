#!/usr/bin/env python3
"""Weight-gradient GEMMs of L layers as ONE strided-batched hipBLASLt call vs L single calls.

A TinyGPT-A layer's dW products (dY^T X over 2048 tokens) are too small to fill 256 CUs one at a
time.  The gradient slots of the same parameter in consecutive blocks sit at a constant stride in
the flat gradient buffer, so the products of a bucket's blocks can run as one batched GEMM.  This
measures what that buys per shape (overwrite and accumulate forms).

    python scripts/bench_batched_wgrad.py [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from scripts.bench_gemm import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    M = 2048
    dt = torch.bfloat16
    shapes = [("qkv", 3072, 1024), ("out", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096)]
    block_stride = 12_596_224 + 1024            # elements per block in the flat buffer (padded)
    for name, N, K in shapes:
        for L in (3, 16):
            dy = torch.randn(L, M, N, device="cuda", dtype=dt)
            x = torch.randn(L, M, K, device="cuda", dtype=dt)
            flat = torch.zeros(L * block_stride, device="cuda", dtype=dt)
            dw = torch.as_strided(flat, (L, N, K), (block_stride, K, 1))
            single = lambda: [torch.mm(dy[i].t(), x[i], out=dw[i]) for i in range(L)]
            single_acc = lambda: [dw[i].addmm_(dy[i].t(), x[i]) for i in range(L)]
            batched = lambda: torch.bmm(dy.transpose(1, 2), x, out=dw)
            batched_acc = lambda: dw.baddbmm_(dy.transpose(1, 2), x)
            fl = 2.0 * M * N * K * L
            for tag, fn in (("single", single), ("single+acc", single_acc), ("bmm", batched),
                            ("bmm+acc", batched_acc)):
                us = timeit(fn, a.iters)
                print(f"{name:4s} L={L:2d} {tag:11s} {us:8.1f} us  {us / L:6.1f} us/layer  {fl / us / 1e6:7.1f} TF/s",
                      flush=True)
            ref = torch.bmm(dy.transpose(1, 2).float(), x.float())
            batched()
            err = (dw.float() - ref).abs().max().item() / ref.abs().max().item()
            print(f"     bmm rel err {err:.2e}")


if __name__ == "__main__":
    main()
