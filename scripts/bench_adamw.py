#!/usr/bin/env python3
"""Fused AdamW launch time at TinyGPT-A size (236.4M fp32 master / moments, bf16 gradient and parameter copy).

    python scripts/bench_adamw.py [--n 236406784] [--iters 20]

Bytes moved per element: read master, m, v (12) + bf16 grad (2), write master, m, v (12) + bf16 param (2)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.optim.adamw import FlatAdamW  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=236406784)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
n = a.n
master = torch.randn(n, device="cuda")
dst = torch.empty(n, device="cuda", dtype=torch.bfloat16)
opt = FlatAdamW(master, [(0, n, dst)], lr=1e-4)
g = torch.randn(n, device="cuda").to(torch.bfloat16)
gs = torch.ones(1, device="cuda")
for _ in range(3):
    opt.step(g, 1e-4, gs)
torch.cuda.synchronize()
ts = []
for _ in range(a.iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    opt.prepare(1e-4)
    s.record()
    opt.launch(g, gs)
    e.record()
    torch.cuda.synchronize()
    ts.append(s.elapsed_time(e) * 1e3)
ts.sort()
med = ts[len(ts) // 2]
print(f"adamw n={n}: median {med:.1f} us, min {ts[0]:.1f} us, "
      f"{28 * n / med / 1e6:.2f} TB/s (28 B/elem)", flush=True)
