#!/usr/bin/env python3
"""Tune the model's hipBLASLt GEMMs: solution x split-K x workgroup mapping (ops/blaslt.py).

Runs one eager accumulation window of the model with GEMM recording on (every problem the linear
layers and the batched weight-gradient flushes issue, with exact strides and accumulate flags),
then per problem:

  * times torch's own call for it (TunableOp's shipped pick, the path used without this table);
  * times every hipBLASLt solution, then the fastest ``--refine`` under every (split-K, wgm) pair
    (``dltb._C.blaslt_sweep``, csrc/blaslt.cpp);
  * keeps the winner if it beats torch by more than ``--min-gain``.

and merges the winners into the table (default configs/blaslt/blaslt_gfx950.csv).

    python scripts/tune_blaslt.py --tier A --seq-len 2048 --strategy zero2 [--dtype bf16] [--emulate N]

``--emulate N`` records the problems of rank 0 of an N-rank job (DLTB_COMM=emulate:N): the
per-bucket / per-unit weight gradients and the other shapes that only exist at world size > 1.
"""
import argparse
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.ops import blaslt  # noqa: E402
from dltb.ops._ext import ext  # noqa: E402


def torch_call(a, b, c, acc, bias):
    if a.dim() == 3:
        return (lambda: c.baddbmm_(a, b)) if acc else (lambda: torch.bmm(a, b, out=c))
    if bias is not None:
        return lambda: torch.addmm(bias, a, b, out=c)
    return (lambda: c.addmm_(a, b)) if acc else (lambda: torch.mm(a, b, out=c))


def time_fn(fn, iters):
    """GPU microseconds per call: ``iters`` calls captured in one HIP graph and replayed, so the
    host cost of issuing them (which dominates torch's TunableOp path) is not in the number."""
    for _ in range(3):
        fn()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def host_us(fn, n=200):
    """Host microseconds to issue one call (enqueue only)."""
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return dt / n * 1e6


def record_problems(args):
    from dltb.comm.topology import recommend_bucket_mb
    from dltb.data import SyntheticDataset, make_batcher
    from dltb.harness import _engine_for
    from dltb.models import build_model, get_model_config
    from dltb.utils.dist import setup_distributed
    device = setup_distributed(1, 0, 0, device_type="cuda" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(0)
    mcfg = get_model_config(args.tier, args.seq_len)
    with torch.device(device):
        model = build_model(mcfg)
    h = argparse.Namespace(strategy=args.strategy, deepspeed_config=None, fsdp_config=None, grad_accum=args.grad_accum,
                           accum_semantics="reference", dtype=args.dtype,
                           bucket_mb=recommend_bucket_mb(max(1, args.emulate)), seed=42,
                           grad_reduce="micro", grad_comm_dtype="compute", fsdp_wrap="block")
    engine, _ = _engine_for(h, model, device)
    ds = SyntheticDataset(mcfg.vocab_size, args.seq_len, 64, 0)
    batches = make_batcher("device", ds, 1, 1, 0, args.strategy, device)
    engine.train()
    blaslt.start_recording()
    for _ in range(engine.accum + 1):     # + 1: a window boundary, then a first micro-step again
        b = next(batches)
        loss = engine(b, b)[1]
        engine.backward(loss)
        engine.step()
    engine.finalize()
    torch.cuda.synchronize()
    return blaslt.stop_recording(), (model, engine)


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--tier", default="A")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--strategy", default="zero2")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--grad-accum", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--refine", type=int, default=12)
    ap.add_argument("--splitk", default="0,2,3,4,6,8")
    ap.add_argument("--wgm", default="0,1,2,4,8,16")
    ap.add_argument("--min-gain", type=float, default=-0.02,
                    help="keep an entry unless it is slower than torch's GPU time by more than this fraction "
                         "(entries at parity still pay: a few us of host time per call instead of ~25)")
    ap.add_argument("--out", default=blaslt.DEFAULT_FILE)
    ap.add_argument("--limit", type=int, default=0, help="tune at most this many problems (0 = all)")
    ap.add_argument("--emulate", type=int, default=0, help="record the problems of an N-rank job's rank 0")
    ap.add_argument("--only-new", action="store_true", help="skip problems the table already holds")
    args = ap.parse_args()
    if args.emulate:
        os.environ["DLTB_COMM"] = f"emulate:{args.emulate}"
    from dltb.utils.gemm_tuning import setup_tunableop
    os.environ["DLTB_BLASLT_FILE"] = "none"          # record / compare against the torch path only
    print(f"[tune_blaslt] TunableOp: {setup_tunableop('use')}", flush=True)
    probs, keep = record_problems(args)
    print(f"[tune_blaslt] {len(probs)} distinct GEMM problems recorded", flush=True)
    sks = [int(x) for x in args.splitk.split(",")]
    wgs = [int(x) for x in args.wgm.split(",")]
    rows = {}
    if os.path.exists(args.out):
        with open(args.out) as f:
            for r in csv.DictReader(f):
                rows[tuple(r[k] for k in blaslt.FIELDS[:15])] = r
    items = list(probs.items())
    if args.only_new:
        items = [(k, v) for k, v in items if tuple(str(x) for x in k) not in rows]
        print(f"[tune_blaslt] {len(items)} of them not in {args.out} yet", flush=True)
    if args.limit:
        items = items[:args.limit]
    C = ext()
    tot_t = tot_b = 0.0
    for key, (a, b, c, acc, bias) in items:
        t0 = time.time()
        tu = time_fn(torch_call(a, b, c, acc, bias), args.iters)
        _, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, beta1, _ = key
        res = C.blaslt_sweep(b, a, c, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, bool(beta1), bias,
                             args.iters, sks, wgs, args.refine)
        if not res:
            print(f"  {key}: no supported solution", flush=True)
            continue
        algo, sk, wg, us, name = res[0]
        # confirm through the run path (cached Gemm object, as the model calls it)
        ent = (algo, sk, wg)
        ub = time_fn(lambda: blaslt.run(key, a, b, c, ent, bias), args.iters)
        C.blaslt_table_set([[1 if key[0] == "fp16" else 0, *key[1:], *ent]])
        h_t = host_us(torch_call(a, b, c, acc, bias))
        h_b = host_us(lambda: C.blaslt_mm(a, b, c, bool(acc), bias))
        C.blaslt_table_set([])
        gain = 1.0 - ub / tu
        tot_t += tu
        tot_b += min(ub, tu)
        keep_it = gain > args.min_gain
        print(f"  {'KEEP' if keep_it else 'skip'} {key[:14]} bias={key[14]} torch {tu:7.1f} us  tuned {ub:7.1f} us "
              f"(sweep {us:.1f}; algo {algo} splitK {sk} wgm {wg})  gain {gain * 100:5.1f}%  "
              f"host/call torch {h_t:.1f} us, tuned {h_b:.1f} us  [{time.time() - t0:.0f}s]", flush=True)
        if keep_it:
            r = dict(zip(blaslt.FIELDS[:15], [str(x) for x in key]))
            r.update(algo=algo, splitk=sk, wgm=wg, us=f"{ub:.2f}", torch_us=f"{tu:.2f}", solution=name)
            rows[tuple(r[k] for k in blaslt.FIELDS[:15])] = r
    print(f"[tune_blaslt] per-window sum over distinct problems: torch {tot_t:.1f} us -> {tot_b:.1f} us", flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=blaslt.FIELDS)
        w.writeheader()
        for r in rows.values():
            w.writerow({k: r[k] for k in blaslt.FIELDS})
    print(f"[tune_blaslt] wrote {len(rows)} entries to {args.out}", flush=True)
    del keep


if __name__ == "__main__":
    main()
