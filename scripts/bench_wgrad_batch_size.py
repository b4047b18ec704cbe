#!/usr/bin/env python3
"""Per-layer cost of the batched weight-gradient GEMMs vs the number of layers per batch.

At world size > 1 the replicated engines flush the dW products per gradient bucket (right before the
bucket's reduce-scatter), so the batch size is the number of blocks in a bucket: 64 MB buckets hold
~2.5 TinyGPT-A blocks (25 MB of bf16 gradients each).  Times dW = dY^T X (K = 2048 tokens, accumulate
form) for the four matrix kinds of a block, for L blocks per strided-batched call.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.utils.gemm_tuning import setup_tunableop  # noqa: E402


def tm(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    setup_tunableop("use")
    bf, T = torch.bfloat16, 2048
    kinds = {"qkv": (3072, 1024), "out": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096)}
    for L in (1, 2, 3, 4, 6, 8, 16):
        tot = 0.0
        for o, i in kinds.values():
            dy = torch.randn(L, T, o, device="cuda", dtype=bf)
            x = torch.randn(L, T, i, device="cuda", dtype=bf)
            dw = torch.randn(L, o, i, device="cuda", dtype=bf)
            tot += tm(lambda: dw.baddbmm_(dy.transpose(1, 2), x))
        print(f"L={L:2d} blocks per batch: {tot / L:7.1f} us per block (4 dW products)", flush=True)


if __name__ == "__main__":
    main()
