#!/usr/bin/env python3
"""Host cost per GEMM call of the paths a linear layer can take (enqueue only, GPU kept busy):
tuned table entry, heuristic fallback with repeated / fresh operand pointers, torch.mm.

    python scripts/bench_blaslt_host.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops import blaslt  # noqa: E402
from dltb.ops._ext import ext  # noqa: E402


def host_us(fn, n=400):
    torch.cuda.synchronize()
    torch.cuda._sleep(int(5e8))                       # GPU busy: only the enqueue is timed
    t = time.perf_counter()
    for i in range(n):
        fn(i)
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return dt / n * 1e6


def main():
    blaslt.load()
    C = ext()
    dev = "cuda"
    for dt in (torch.bfloat16, torch.float16):
        a = torch.randn(2048, 1024, device=dev, dtype=dt)
        w = torch.randn(4096, 1024, device=dev, dtype=dt)
        out = torch.empty(2048, 4096, device=dev, dtype=dt)
        pool_a = [a.clone() for _ in range(8)]
        pool_o = [out.clone() for _ in range(8)]
        same = host_us(lambda i: C.blaslt_mm(a, w.t(), out, False, None))
        fresh = host_us(lambda i: C.blaslt_mm(pool_a[i % 8], w.t(), pool_o[(i // 8) % 8], False, None))
        tm = host_us(lambda i: torch.mm(a, w.t(), out=out))
        print(f"{dt}: blaslt_mm same pointers {same:.1f} us/call, rotating 64 pointer sets {fresh:.1f} us/call, "
              f"torch.mm {tm:.1f} us/call", flush=True)


if __name__ == "__main__":
    main()
