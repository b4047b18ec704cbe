#!/usr/bin/env python3
"""Split-K x tile search for small-output / long-K products (hipBLASLt extension API).

A [2048 x 1024] output with K = 4096 (TinyGPT-A's fc2 forward and fc1 dgrad) is 256 tiles of
128 x 64: one per CU, each streaming 1.5 MB of operands through L2 at ~43 FLOP/B -- L2-bandwidth
bound.  Larger tiles raise the intensity but leave CUs idle unless K is split; the default sweep
(scripts/tune_blaslt.py) only applies split-K to the solutions that are fastest WITHOUT it, which
are exactly the small-tile ones.  This sweeps every solution under every split-K.

    python scripts/bench_gemm_splitk.py M N K [M N K ...]     (row-major C[M,N] = A[M,K] B[K,N],
                                                                both operands K-contiguous)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops import blaslt  # noqa: E402
from dltb.ops._ext import ext  # noqa: E402


def main():
    dims = [int(x) for x in sys.argv[1:]] or [2048, 1024, 4096]
    C = ext()
    for M, N, K in zip(dims[0::3], dims[1::3], dims[2::3]):
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16).t()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        key = blaslt.problem(A, B, out, False)
        _, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, beta1, _ = key
        res = C.blaslt_sweep(B, A, out, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, False, None,
                             10, [0, 2, 3, 4, 6, 8, 12, 16], [0], 0)
        base = min(r[3] for r in res if r[1] == 0)
        print(f"M{M} N{N} K{K}: best without split-K {base:.1f} us", flush=True)
        for algo, sk, wg, us, name in res[:8]:
            mt = name[name.find("_MT") + 1:].split("_")[0] if "_MT" in name else "?"
            print(f"   {us:7.1f} us  {2.0 * M * N * K / us / 1e6:7.1f} TF/s  algo {algo} splitK {sk} {mt}", flush=True)


if __name__ == "__main__":
    main()
