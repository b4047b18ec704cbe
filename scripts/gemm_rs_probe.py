#!/usr/bin/env python3
"""One GEMM shape, repeatedly, through hipBLASLt and gemm_rs configs (rocprofv3 --pmc runs).

    SHAPE=2048,1024,4096 CFGS=1,2 rocprofv3 --pmc ... -- python3 scripts/gemm_rs_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops import blaslt  # noqa: E402
from dltb.ops._ext import ext  # noqa: E402


def main():
    M, N, K = (int(v) for v in os.environ.get("SHAPE", "2048,1024,4096").split(","))
    cfgs = [int(c) for c in os.environ.get("CFGS", "1").split(",")]
    C = ext()
    blaslt.load()
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(10):
        if not blaslt.mm(x, w.t(), y, False):
            torch.mm(x, w.t(), out=y)
    for cfg in cfgs:
        for _ in range(10):
            C.gemm_rs(x, w, y, None, False, cfg, 4)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
