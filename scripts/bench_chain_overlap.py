#!/usr/bin/env python3
"""Two independent micro-step chains on two streams: one block's forward (micro-step k+1) beside one block's
backward (micro-step k), TinyGPT-A shapes, HIP-graph timed.  Prints alone / serial / concurrent."""
import os, sys, statistics
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import dltb  # noqa
from dltb.ops import functional as F_
from dltb.ops._ext import ext

C = ext()
dev, bf = "cuda", torch.bfloat16
B, T, H, d, Fd = 1, 2048, 16, 1024, 4096
g = torch.Generator(device=dev).manual_seed(0)
rn = lambda *s: (torch.randn(*s, device=dev, dtype=bf, generator=g) * 0.05)
w_in, b_in, w_o, b_o = rn(3 * d, d), rn(3 * d), rn(d, d), rn(d)
w1, b1, w2, b2 = rn(Fd, d), rn(Fd), rn(d, Fd), rn(d)
wt_in, wt_o, wt1, wt2 = (w.t().contiguous() for w in (w_in, w_o, w1, w2))
seed = torch.tensor([1234], device=dev, dtype=torch.int64)
# forward inputs (micro-step k+1) and backward inputs (micro-step k), separate tensors
h1f, h2f = rn(T, d), rn(T, d)
qkv_b = rn(T, 3 * d); do_b = rn(T, d); dm_b = rn(T, d); df_b = rn(T, Fd); dx1_b = rn(T, d); dqkv_b = rn(T, 3 * d)
mask_b = C.attn_mask(B, T, H, 0.1, seed, 1, qkv_b)
o_b, lse_b = C.attn_fwd(qkv_b[:, :d], qkv_b[:, d:2*d], qkv_b[:, 2*d:], mask_b, B, T, H, H, 0.125, False, 0.1)
delta_b = torch.empty_like(lse_b)
dq_b = torch.empty(T, d, device=dev, dtype=bf); dkv_b = torch.empty(T, 2 * d, device=dev, dtype=bf)

def fwd_chain():
    qkv = F_.linear_fwd(h1f, w_in, b_in)
    mask = C.attn_mask(B, T, H, 0.1, seed, 2, qkv)
    o, lse = C.attn_fwd(qkv[:, :d], qkv[:, d:2*d], qkv[:, 2*d:], mask, B, T, H, H, 0.125, False, 0.1)
    a = F_.linear_fwd(o, w_o, b_o)
    f = F_.linear_fwd(h2f, w1, b1)
    gg = C.gelu_fwd(f)
    m = F_.linear_fwd(gg, w2, b2)
    return a, m

def bwd_chain():
    dg = F_.linear_dgrad(dm_b, w2, wt2)
    dh2 = F_.linear_dgrad(df_b, w1, wt1)
    do = F_.linear_dgrad(dx1_b, w_o, wt_o)
    C.attn_bwd_part(1, qkv_b[:, :d], qkv_b[:, d:2*d], qkv_b[:, 2*d:], do_b, lse_b, delta_b, mask_b, dq_b, None, B, T, H, H, 0.125, False, 0.1, o_b)
    C.attn_bwd_part(0, qkv_b[:, :d], qkv_b[:, d:2*d], qkv_b[:, 2*d:], do_b, lse_b, delta_b, mask_b, dkv_b[:, :d], dkv_b[:, d:], B, T, H, H, 0.125, False, 0.1)
    dh1 = F_.linear_dgrad(dqkv_b, w_in, wt_in)
    return dg, dh2, do, dh1

side = torch.cuda.Stream()
def both():
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        fwd_chain()
    bwd_chain()
    cur.wait_stream(side)

def serial():
    fwd_chain(); bwd_chain()

def graph_time(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps): fn()
    gr.replay(); torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(); gr.replay(); e.record(); torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / reps * 1e3)
    return statistics.median(ts)

res = {}
for r in range(2):
    for name, fn in (("fwd", fwd_chain), ("bwd", bwd_chain), ("serial", serial), ("concurrent", both)):
        res.setdefault(name, []).append(graph_time(fn))
for k, v in res.items():
    print(f"{k:12s} {min(v):8.1f} us  ({', '.join('%.1f' % x for x in v)})")
print(f"concurrent / serial = {min(res['concurrent']) / min(res['serial']):.3f}")
