#!/usr/bin/env python3
"""Run one GEMM shape repeatedly (dltb tile configs and hipBLASLt) for rocprofv3 --pmc runs.

    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --stats -d OUT -- python3 scripts/gemm_pmc_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops._ext import ext  # noqa: E402


def main():
    M, N, K = (int(v) for v in os.environ.get("SHAPE", "2048,1024,1024").split(","))
    cfgs = [int(c) for c in os.environ.get("CFGS", "0,3,5").split(",")]
    C = ext()
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(10):
        torch.mm(x, w.t(), out=y)
    for cfg in cfgs:
        for _ in range(10):
            C.gemm(x, w, y, None, False, False, 1, cfg)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
