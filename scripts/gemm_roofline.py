#!/usr/bin/env python3
"""Per-product roofline of the TinyGPT-A step's GEMMs from rocprofv3 kernel traces (VERDICT r4 next #1a).

    python scripts/gemm_roofline.py --off <trace.csv> [--on <trace.csv>] [--all <trace.csv>] > profiles/gemm_roofline_r5.txt

Each trace is scripts/rocprof.sh's run_kernel_trace.csv of bench.py (ZeRO-2, seq 2048).  The steady window is the
last 4 micro-steps (xent launches).  Per-layer products are labelled by their neighbours in the launch sequence:
  forward  qkv = GEMM before attn_fwd, out = GEMM after attn_fwd, fc1 = GEMM before gelu_fwd, fc2 = GEMM after it;
  backward fc2.dgrad = first GEMM of a block's backward (after a colpart), fc1.dgrad = GEMM after the GELU colpart,
           out.dgrad = GEMM after the LN2 norm_bwd_fused, qkv.dgrad = GEMM after attn_bwd_dkdv.
Bounds: MFMA = 2MNK / 2.5 PFLOP/s (dense bf16); stream = (BM + BN) K 2 bytes per CU over a 256-tile grid
(BM = 128, BN = M N / 256 / 128) at 123 GB/s per CU (the register-load rate of profiles/l2_stream_probe_r4.txt).
"""
import argparse
import csv
import re
import statistics

PRODUCTS = {   # name: (M, N, K)
    "qkv.fwd": (2048, 3072, 1024), "out.fwd": (2048, 1024, 1024), "fc1.fwd": (2048, 4096, 1024),
    "fc2.fwd": (2048, 1024, 4096), "fc2.dgrad": (2048, 4096, 1024), "fc1.dgrad": (2048, 1024, 4096),
    "out.dgrad": (2048, 1024, 1024), "qkv.dgrad": (2048, 1024, 3072),
}


def is_gemm(n):
    return "Cijk" in n or "gemm_r" in n


def load(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0) for r in rows]
    x = [i for i, (n, _) in enumerate(seq) if "xent_kernel" in n]
    a, b = x[-5], x[-1]                   # last 4 micro-steps: forward of step k ... forward of step k + 4
    return seq[a - 200 if a >= 200 else 0:b], seq, (x[-5], x[-1])


def label(seq):
    """(product, us, kernel) for every per-layer GEMM in seq."""
    out = []
    for i, (n, t) in enumerate(seq):
        if not is_gemm(n):
            continue
        prev = seq[i - 1][0] if i else ""
        nxt = seq[i + 1][0] if i + 1 < len(seq) else ""
        lab = None
        if "attn_fwd" in nxt:
            lab = "qkv.fwd"
        elif "attn_fwd" in prev:
            lab = "out.fwd"
        elif "gelu_fwd" in nxt:
            lab = "fc1.fwd"
        elif "gelu_fwd" in prev:
            lab = "fc2.fwd"
        elif "attn_bwd_dkdv" in prev:
            lab = "qkv.dgrad"
        elif "norm_bwd_fused" in prev and "attn_bwd_dq" in nxt:
            lab = "out.dgrad"
        elif "colpart" in prev and "norm_bwd_fused" in nxt:
            lab = "fc1.dgrad"
        elif "colpart" in prev and "colpart" in nxt:
            lab = "fc2.dgrad"
        if lab:
            out.append((lab, t, n))
    return out


def per_product(path):
    seq, full, (a, b) = load(path)
    # the steady window: GEMMs between the 5th-last and the last xent launch
    win = full[a - 1:b]
    # forward GEMMs of the window's first micro-step precede xent index a: include the full micro-steps
    lab = label(full[max(0, a - 120):b])
    d = {}
    for p, t, n in lab:
        d.setdefault(p, []).append((t, n))
    return {p: (statistics.median(t for t, _ in v), v[0][1]) for p, v in d.items()}


def short(n):
    if "Cijk" in n:
        m = re.search(r"MT(\d+x\d+x\d+)", n)
        return "hipBLASLt MT" + (m.group(1) if m else "?")
    return n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--off", required=True)
    ap.add_argument("--on", default=None)
    ap.add_argument("--all", default=None)
    a = ap.parse_args()
    arms = [("hipBLASLt", per_product(a.off))]
    if a.on:
        arms.append(("shipped", per_product(a.on)))
    if a.all:
        arms.append(("all-own", per_product(a.all)))
    print(f"{'product':10s} {'M x N x K':>18s} {'GFLOP':>6s} {'B/CU MB':>7s} {'mfma us':>7s} {'strm us':>7s}  "
          + "  ".join(f"{n + ' in-step us':>20s} {'x bound':>7s}" for n, _ in arms))
    tot = {n: 0.0 for n, _ in arms}
    tb = 0.0
    for p, (M, N, K) in PRODUCTS.items():
        fl = 2.0 * M * N * K
        bn = M * N // 256 // 128
        bytes_cu = (128 + bn) * K * 2
        mf = fl / 2.5e15 * 1e6
        st = bytes_cu / 123e9 * 1e6
        bound = max(mf, st)
        tb += bound
        cols = []
        for n, d in arms:
            t = d.get(p, (float("nan"), ""))[0]
            tot[n] += t
            cols.append(f"{t:20.1f} {t / bound:7.2f}")
        print(f"{p:10s} {f'{M}x{N}x{K}':>18s} {fl / 1e9:6.1f} {bytes_cu / 1e6:7.2f} {mf:7.1f} {st:7.1f}  " + "  ".join(cols))
    print(f"{'per layer':10s} {'':>18s} {'':>6s} {'':>7s} {'':>7s} {tb:7.1f}  "
          + "  ".join(f"{tot[n]:20.1f} {tot[n] / tb:7.2f}" for n, _ in arms))
    # head and window-wide weight gradients (hipBLASLt in every arm): MFMA bound only (thousands of tiles)
    _, full, (xa, xb) = load(a.off)
    win = full[xa - 120:xb]
    head = []
    for i, (n, t) in enumerate(win):
        if not is_gemm(n):
            continue
        nxt = win[i + 1][0] if i + 1 < len(win) else ""
        prev2 = " ".join(w[0] for w in win[max(0, i - 3):i])
        if "xent_kernel" in nxt:
            head.append(("head.fwd (logits)", t))
        elif "transpose_kernel" in prev2 or "PostGSU" in n:
            head.append(("head.dgrad + wgrad (+ GSU reduce)", t))
    hd = {}
    for k, t in head:
        hd.setdefault(k, []).append(t)
    print()
    fl_head = 2.0 * 2048 * 32000 * 1024
    for k, v in hd.items():
        per = sum(v) / 4                   # the window holds 4 micro-steps
        nprod = 1 if "fwd" in k else 2
        mf = nprod * fl_head / 2.5e15 * 1e6
        print(f"{k:36s} {nprod * fl_head / 1e9:7.1f} GFLOP  mfma {mf:6.1f} us  in-step {per:7.1f} us per micro-step  x{per / mf:4.2f}")
    dw = [t for n, t in full[xa:xb] if "Cijk_Ailk_Bjlk" in n]
    fl_dw = 2.0 * 8192 * (1024 * 3072 + 1024 * 1024 + 1024 * 4096 + 4096 * 1024) * 16
    if dw:
        mf = fl_dw / 2.5e15 * 1e6
        print(f"{'batched dW (4 kinds x 16 blocks, K 8192)':36s} {fl_dw / 1e9:7.1f} GFLOP  mfma {mf:6.1f} us  in-step "
              f"{sum(dw):7.1f} us per window ({len(dw)} launches)  x{sum(dw) / mf:4.2f}")
    print()
    for n, d in arms:
        print(f"[{n}] kernels: " + "; ".join(f"{p} {short(d[p][1])}" for p in PRODUCTS if p in d))


if __name__ == "__main__":
    main()
