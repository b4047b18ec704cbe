#!/usr/bin/env python3
"""World-size equivalence check of every engine on real HIP kernels.

    # 2 ranks sharing one GPU (gloo, host-staged buffers) vs. 1 rank with the concatenated batch
    DLTB_COMM=host python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29531 scripts/multirank_check.py --out ws2.pt
    python scripts/multirank_check.py --out ws1.pt

For every case (DDP bf16 / fp32 all-reduce, ZeRO-2 per-micro-step and per-window reduce-scatter,
ZeRO-3 with release + re-gather, FSDP per-block and the reference's root FlatParameter, and a
Mistral-shape GQA model under ZeRO-3) the same model (same init) trains ``windows`` accumulation
windows of ``accum`` micro-steps.  Rank r of N reads row r of each micro-step's [N_ref, T] token
table; the world-1 run reads all rows as one batch, so the averaged gradients are mathematically
identical.  Dropout is off in the equivalence cases (dropout masks are per-rank streams, so a
world-1 run cannot draw the same masks); the ``dropout`` case turns it on with every rank reading
the SAME rows, which pins that ranks draw distinct masks (their losses differ), that a fixed seed
is deterministic (tests/ re-run it) and that the loss stays within dropout noise of world 1.
``zero3_m7b`` is the Mistral-7B layer at full width (d4096, GQA 32/8, SwiGLU 14336; 2 layers,
vocab 8192) under ZeRO-3 -- BASELINE config #5's shapes through every sharded code path.  AdamW runs with eps = 1 and
no weight decay, which makes an update ~ lr * gradient (not the sign of it), so comparing the
parameter *updates* of two runs compares their reduced gradients.  Rank 0 writes
{case: {"init", "final", "losses"}} (fp32, CPU) to ``--out``; tests/test_multirank_gpu.py compares
the two files.  Reference semantics being checked: train_harness.py:210-271 (DDP / FSDP /
DeepSpeed ZeRO-2/3 wrap) -- at any world size the trained model must be the one the global batch
defines.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CASES = {
    "ddp": dict(strategy="ddp"),
    "ddp_fp32comm": dict(strategy="ddp", grad_comm_dtype="fp32"),
    "zero2": dict(strategy="zero2"),
    "zero2_window": dict(strategy="zero2", grad_reduce="window"),
    "zero3": dict(strategy="zero3"),
    "fsdp": dict(strategy="fsdp"),
    "fsdp_root": dict(strategy="fsdp", wrap="root"),
    "zero3_mistral": dict(strategy="zero3", tier="mtiny", persist=1024),
}
EXTRA_CASES = {
    "zero3_m7b": dict(strategy="zero3", tier="m7b_2l", persist=100_000),
    "dropout": dict(strategy="zero2", dropout=0.1, same_rows=True),
    # DeepSpeed switches (parallel/ds_config.py): overlap_comm / reduce_scatter / allgather_partitions
    # false -> synchronous collectives, all-reduce + own chunk, per-owner broadcasts
    "zero2_ds_switches": dict(strategy="zero2", extra={"overlap_comm": False, "reduce_scatter": False,
                                                       "allgather_partitions": False}),
    # ZeRO-3 with an element prefetch budget (several units ahead), the reuse-distance keep of the
    # last units (not all: reuse distance below the model size) and AdamW sub-groups
    "zero3_ds_budgets": dict(strategy="zero3", extra={"prefetch_elems": 1_700_000, "sub_group_elems": 300_000},
                             over={"max_live_parameters": 10**9, "max_reuse_distance": 2_200_000}),
    # 12 blocks: the replicated engines' bucket plan head | 8 blocks (the early bucket) | 4 blocks | embedding,
    # with the tied table's all-gather first and the per-bucket AdamW + all-gather pipeline
    "zero2_deep": dict(strategy="zero2", layers=12),
}


def model_config(tier, seq_len, dropout=0.0):
    from dltb.models import get_model_config
    if tier == "mtiny":
        return get_model_config("mtiny", seq_len)
    if tier == "m7b_2l":                                 # Mistral-7B width, 2 layers, small vocab
        c = get_model_config("M7B", seq_len)
        c.n_layer, c.vocab_size = 2, 8192
        return c
    c = get_model_config("A", seq_len, dropout=dropout)  # TinyGPT, narrowed: d256 / 4 heads of 64
    c.n_embd, c.n_head, c.n_layer, c.vocab_size = 256, 4, 2, 4096
    return c


def run_case(name, spec, world, rank, device, a):
    from dltb.models import build_model
    from dltb.parallel import engine_config, make_engine
    torch.manual_seed(0)
    mcfg = model_config(spec.get("tier", "A"), a.seq_len, spec.get("dropout", 0.0))
    if "layers" in spec:
        mcfg.n_layer = int(spec["layers"])
    with torch.device(device):
        model = build_model(mcfg)
    init = {n: p.detach().float().cpu().clone() for n, p in model.named_parameters()}
    fc = None
    if spec["strategy"] == "fsdp":
        fc = {"auto_wrap_policy": "size_based" if spec.get("wrap") == "root" else "transformer_block"}
    over = {"lr": a.lr, "eps": 1.0, "weight_decay": 0.0, "scheduler": None}
    if spec["strategy"] == "zero3":
        over["max_live_parameters"] = 0          # release after use: exercise every re-gather
        if "persist" in spec:
            over["persistence_threshold"] = spec["persist"]
    over.update(spec.get("over", {}))
    cfg = engine_config(spec["strategy"], a.accum, "uniform", None, fc, bucket_mb=a.bucket_mb,
                        overrides=over, grad_reduce=spec.get("grad_reduce", "micro"))
    cfg.extra["grad_comm_dtype"] = spec.get("grad_comm_dtype", "compute")
    cfg.extra.update(spec.get("extra", {}))
    eng = make_engine(model, cfg, device)
    eng.train()
    g = torch.Generator().manual_seed(123)
    steps = a.windows * a.accum
    table = torch.randint(0, mcfg.vocab_size, (steps, a.ref_batch, a.seq_len), generator=g)
    per = a.ref_batch // world
    same = spec.get("same_rows", False)
    losses, rank_losses = [], []
    for k in range(steps):
        # same_rows: every rank (and every row of the world-1 batch) reads row 0 of the micro-step
        b = (table[k, :1].expand(per, -1).contiguous() if same else table[k, rank * per:(rank + 1) * per]).to(device)
        loss = eng(b, b)[1]
        eng.backward(loss)
        eng.step()
        lv = torch.zeros(world, dtype=torch.float64)
        lv[rank] = float(loss.item())
        if world > 1:
            dist.all_reduce(lv)
        rank_losses.append(lv.tolist())
        losses.append(float(lv.sum()) / world)
    eng.finalize()
    sd = eng.full_state_dict()
    final = {n: t.detach().float().cpu() for n, t in sd.items()}
    del eng, model
    torch.cuda.empty_cache() if device.type == "cuda" else None
    return {"init": init, "final": final, "losses": losses, "rank_losses": rank_losses}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--seq-len", type=int, default=256)
    ap.add_argument("--ref-batch", type=int, default=2, help="global rows per micro-step")
    ap.add_argument("--accum", type=int, default=2)
    ap.add_argument("--windows", type=int, default=3)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--bucket-mb", type=float, default=1.0, help="small buckets: several per model")
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    from dltb.utils.dist import cleanup_distributed, setup_distributed
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert a.ref_batch % world == 0
    device = setup_distributed(world, rank, local, device_type=a.device, timeout_min=5)
    out = {}
    try:
        for name in a.cases.split(","):
            out[name] = run_case(name, {**CASES, **EXTRA_CASES}[name], world, rank, device, a)
            if rank == 0:
                print(f"[multirank_check] ws={world} {name}: losses {['%.4f' % v for v in out[name]['losses']]}",
                      flush=True)
        if rank == 0:
            torch.save(out, a.out)
    finally:
        cleanup_distributed()


if __name__ == "__main__":
    main()
