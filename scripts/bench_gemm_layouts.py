#!/usr/bin/env python3
"""Best hipBLASLt time for one product in each operand layout (solution sweep per layout).

C[M, N] = A[M, K] B[K, N] (row-major torch terms), A and B each either stored with K contiguous
or as a transposed view; e.g. a weight gradient dW = dY^T X has A = dY^T (a view of dY[K, M]) and
B = X[K, N].  Prints the fastest solution per layout (GPU time, 5 calls averaged).

    python scripts/bench_gemm_layouts.py M N K [M N K ...]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops import blaslt  # noqa: E402
from dltb.ops._ext import ext  # noqa: E402


def main():
    dims = [int(x) for x in sys.argv[1:]] or [14336, 4096, 4096]
    C = ext()
    for M, N, K in zip(dims[0::3], dims[1::3], dims[2::3]):
        fl = 2.0 * M * N * K
        for a_kc in (True, False):
            for b_kc in (True, False):
                A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) if a_kc else \
                    torch.randn(K, M, device="cuda", dtype=torch.bfloat16).t()
                B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16).t() if b_kc else \
                    torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
                out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                key = blaslt.problem(A, B, out, False)
                _, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, beta1, _ = key
                res = C.blaslt_sweep(B, A, out, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, False, None,
                                     5, [0], [0], 0)
                us = res[0][3]
                print(f"M{M} N{N} K{K}  A {'K-contig' if a_kc else 'M-contig'}  B {'K-contig' if b_kc else 'N-contig'}"
                      f"  best {us:8.1f} us  {fl / us / 1e6:7.1f} TF/s  ({len(res)} solutions)", flush=True)
                del A, B, out


if __name__ == "__main__":
    main()
