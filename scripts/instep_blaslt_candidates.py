#!/usr/bin/env python3
"""Candidate hipBLASLt solutions for an IN-STEP A/B of chosen per-layer products.

The shipped table (configs/blaslt/blaslt_gfx950.csv, scripts/tune_blaslt.py) keeps each problem's
fastest solution timed isolated and warm (graph-replayed back to back).  In the step the operands
arrive cold from the previous kernel and the neighbours differ, so the isolated winner need not be
the in-step winner (the own GEMM's in-step / isolated gap: profiles/gemm_rs_instep_ab_r5.txt).
This script records the model's problems, sweeps the chosen ones (``--products``), and writes one
table per candidate -- the shipped table with that product's row replaced by the k-th fastest
solution of a different macro tile -- under ``--out-dir`` for bench.py A/Bs
(``DLTB_BLASLT_FILE=<table> python bench.py``).

    python scripts/instep_blaslt_candidates.py --products fc1.fwd,fc2.dgrad,qkv.fwd --top 3
"""
import argparse
import csv
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tune_blaslt import record_problems  # noqa: E402
from dltb.ops import blaslt  # noqa: E402
from dltb.ops._ext import ext  # noqa: E402

# TinyGPT-A per-layer products in the table's key form (opA, opB, m, n, k, bias): hipBLASLt is
# column-major, so a row-major [M, K] x [N, K]^T product is (opA = 1, opB = 0, m = N, n = M)
PRODUCTS = {
    "qkv.fwd": (1, 0, 3072, 2048, 1024, 1),
    "fc1.fwd": (1, 0, 4096, 2048, 1024, 1),
    "fc2.dgrad": (1, 0, 4096, 2048, 1024, 0),
    # the N = 1024 products (own gemm_rsf cfg 34 in the shipped step): a candidate table for these
    # comes with an own-GEMM table lacking the product (<name>_<i>.own.csv, DLTB_OWN_GEMM_TABLE)
    "out.fwd": (1, 0, 1024, 2048, 1024, 1),
    "fc2.fwd": (1, 0, 1024, 2048, 4096, 1),
    "out.dgrad": (1, 0, 1024, 2048, 1024, 0),
    "fc1.dgrad": (1, 0, 1024, 2048, 4096, 0),
    "qkv.dgrad": (1, 0, 1024, 2048, 3072, 0),
    # the tied head: logits, data gradient (K = vocab, split-K), weight gradient
    "head.fwd": (1, 0, 32000, 2048, 1024, 0),
    "head.dgrad": (1, 0, 1024, 2048, 32000, 0),
    "head.wgrad": (1, 1, 1024, 32000, 2048, 0),
}
OWN_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "gemm_rs",
                         "gemm_rs_gfx950.csv")


def macro_tile(name):
    m = re.search(r"MT(\d+x\d+x\d+)", name)
    return m.group(1) if m else name


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--products", default="fc1.fwd,fc2.dgrad,qkv.fwd")
    ap.add_argument("--top", type=int, default=3)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--splitk", default="0", help="split-K factors swept (comma list)")
    ap.add_argument("--table", default=blaslt.DEFAULT_FILE)
    ap.add_argument("--out-dir", default="gpurun_out/blaslt_ab")
    args = ap.parse_args()
    rargs = argparse.Namespace(tier="A", seq_len=2048, strategy="zero2", dtype="bf16", grad_accum=4, emulate=0)
    os.environ["DLTB_OWN_GEMM"] = "0"       # every product through hipBLASLt while recording
    probs, keep = record_problems(rargs)
    with open(OWN_TABLE) as f:
        own_rows = [ln for ln in f if not ln.startswith("#")]
    with open(args.table) as f:
        rows = list(csv.DictReader(f))
    os.makedirs(args.out_dir, exist_ok=True)
    C = ext()
    for prod in args.products.split(","):
        want = PRODUCTS[prod]
        hits = [(k, v) for k, v in probs.items() if k[0] == "bf16" and k[6] == 1 and
                (k[1], k[2], k[3], k[4], k[5], int(bool(k[14]))) == want]
        assert len(hits) == 1, (prod, [h[0] for h in hits])
        key, (a, b, c, acc, bias) = hits[0]
        _, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, beta1, _ = key
        res = C.blaslt_sweep(b, a, c, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, bool(beta1), bias,
                             args.iters, [int(x) for x in args.splitk.split(",")], [0, 1, 2, 4, 8, 16], 24)
        kstr = [str(x) for x in key]
        ship = [r for r in rows if [r[f] for f in blaslt.FIELDS[:15]] == kstr]
        assert len(ship) <= 1, prod
        # the own kernel's row for this product (row-major M = hipBLASLt n, N = hipBLASLt m)
        own_key = f"{n},{m},{k},{int(bool(key[14]))},"
        own_hit = [ln for ln in own_rows if ln.startswith(own_key)]
        seen = {macro_tile(ship[0]["solution"])} if ship and not own_hit else set()
        if ship:
            print(f"[{prod}] table {ship[0]['solution'][:70]} algo {ship[0]['algo']} wgm {ship[0]['wgm']} "
                  f"{ship[0]['us']} us" + ("  (own kernel in the step)" if own_hit else ""), flush=True)
        n_out = 0
        for algo, sk, wg, us, name in res:
            mt = macro_tile(name)
            if mt in seen:
                continue
            seen.add(mt)
            n_out += 1
            alt = [dict(r) for r in rows]
            new = dict(zip(blaslt.FIELDS[:15], kstr))
            new.update(algo=algo, splitk=sk, wgm=wg, us=f"{us:.2f}", torch_us="", solution=name)
            alt = [r for r in alt if [r[f] for f in blaslt.FIELDS[:15]] != kstr] + [new]
            if own_hit:
                with open(os.path.join(args.out_dir, f"{prod}_{n_out}.own.csv"), "w") as f:
                    f.writelines(ln for ln in own_rows if ln not in own_hit)
            path = os.path.join(args.out_dir, f"{prod}_{n_out}.csv")
            with open(path, "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=blaslt.FIELDS)
                w.writeheader()
                for r in alt:
                    w.writerow({kk: r[kk] for kk in blaslt.FIELDS})
            print(f"[{prod}] cand {n_out}: MT{mt} algo {algo} wgm {wg} isolated {us:.2f} us -> {path}", flush=True)
            if n_out >= args.top:
                break
    del keep


if __name__ == "__main__":
    main()
