#!/usr/bin/env python3
"""Locate wrong output tiles of gemm_rs: per config and shape, the (m-tile, n-tile) blocks whose max error
exceeds the tolerance, over repeated launches (debug aid for the register-staged GEMM)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops._ext import ext  # noqa: E402

TILE = {0: (128, 64), 1: (128, 256), 2: (128, 192), 3: (128, 128), 4: (128, 64), 5: (128, 64), 6: (128, 256),
        7: (128, 192), 8: (128, 64), 9: (128, 64), 10: (128, 64), 11: (128, 64), 12: (128, 64), 13: (128, 64),
        14: (128, 64)}
C = ext()
REPS = int(os.environ.get("REPS", "10"))
torch.manual_seed(0)
for (M, N, K) in [(2048, 3072, 1024), (4096, 1024, 1024), (2048, 1024, 4096), (2048, 4096, 1024)]:
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    for c in [int(v) for v in os.environ.get("CFGS", ",".join(str(c) for c in TILE)).split(",")]:
        if not C.gemm_rs_supported(M, N, K, c):
            continue
        bm, bn = TILE[c]
        bad = set()
        nbad_runs = 0
        for rep in range(REPS):
            y = C.gemm_rs(x, w, None, None, False, c, 1)
            torch.cuda.synchronize()
            e = (y.float() - ref).abs().reshape(M // bm, bm, N // bn, bn).amax(dim=(1, 3))
            b = (e > 0.05).nonzero().tolist()
            nbad_runs += bool(b)
            bad |= {tuple(t) for t in b}
        tiles = (M // bm) * (N // bn)
        ex = sorted(bad)[:12]
        print(f"M{M} N{N} K{K} c{c} tiles {tiles}: bad runs {nbad_runs}/{REPS}, bad tiles {len(bad)} e.g. {ex}", flush=True)
        if bad:
            # which rows / cols inside a bad tile
            y = C.gemm_rs(x, w, None, None, False, c, 1)
            torch.cuda.synchronize()
            mb, nb = sorted(bad)[0]
            d = (y.float() - ref)[mb * bm:(mb + 1) * bm, nb * bn:(nb + 1) * bn].abs() > 0.05
            rows = d.any(1).nonzero().flatten().tolist()
            cols = d.any(0).nonzero().flatten().tolist()
            print(f"   tile {mb},{nb}: bad rows {rows[:40]} ({len(rows)}), bad cols {cols[:40]} ({len(cols)})", flush=True)
