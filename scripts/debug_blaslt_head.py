#!/usr/bin/env python3
"""Why does the tied head's data-gradient row (algo 618612, split-K 6) fall back under some tables?
Runs the head dgrad product through ops/blaslt.mm with the table given as argv[1], optionally
after a fc2.dgrad-shaped product (argv[2] == 'warm'), and prints mm's result and the raw run code."""
import sys

import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import dltb  # noqa: F401
from dltb.ops import blaslt
from dltb.ops._ext import ext

dev = torch.device("cuda", 0)
n = blaslt.load(sys.argv[1], verbose=True)
C = ext()
if len(sys.argv) > 2 and sys.argv[2] == "warm":
    a = torch.randn(2048, 1024, device=dev, dtype=torch.bfloat16)
    w = torch.randn(4096, 1024, device=dev, dtype=torch.bfloat16)
    c = torch.empty(2048, 4096, device=dev, dtype=torch.bfloat16)
    print("fc2.dgrad-shaped mm:", blaslt.mm(a, w.t(), c, False))
dl = torch.randn(2048, 32000, device=dev, dtype=torch.bfloat16)
wt = torch.randn(1024, 32000, device=dev, dtype=torch.bfloat16)
dh = torch.empty(2048, 1024, device=dev, dtype=torch.bfloat16)
key = blaslt.problem(dl, wt.t(), dh, False, None)
print("head key:", key, "in table:", key in blaslt._table, blaslt._table.get(key))
print("head mm:", blaslt.mm(dl, wt.t(), dh, False))
if key in blaslt._table:
    algo, sk, wg = blaslt._table[key]
    _, opA, opB, m, n_, k, batch, lda, ldb, ldc, sa, sb, sc, beta1, _ = key
    for s in (sk, 0, 2, 4, 8):
        try:
            C.blaslt_run(wt.t(), dl, dh, opA, opB, m, n_, k, batch, lda, ldb, ldc, sa, sb, sc, bool(beta1), None,
                         algo, s, wg)
            print(f"  run algo {algo} splitk {s}: ok")
        except Exception as e:  # noqa: BLE001
            print(f"  run algo {algo} splitk {s}: {e}")
print("name 618612:", C.blaslt_name(618612))
torch.cuda.synchronize()
