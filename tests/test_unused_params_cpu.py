"""Units whose backward does not run in a micro-step (parameters the loss does not use).

The reference's torch DDP runs with ``find_unused_parameters=False`` (train_harness.py:217-222) and
never meets this case; DeepSpeed and FSDP tolerate it.  Here a unit that does not report in a
micro-step must contribute a ZERO gradient: its slots must not carry a stale gradient of an earlier
step, a bucket holding only such units is still reduced (every rank must join the collective), and
a ZeRO-2 reduce-scatter left in flight by the previous micro-step must be folded into the fp32
accumulator before the bucket is reduced again.  The toy model below decides per row which units
take part, so a unit is skipped on one rank (replicated engines only), on every rank, or in whole
windows; world 2 (lazy
collectives, the strictest wait discipline) must reproduce the single-process run, and the
single-process run must match plain autograd + torch.optim.AdamW.
"""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

import dltb  # noqa: F401
from dltb.parallel import engine_config, make_engine
from dltb.parallel.runtime import EAGER, Unit

V, T, K = 64, 6, 3
STEPS = 4


class _Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, model, idx):
        rt = model.rt
        B = idx.shape[0]
        loss = torch.zeros((), dtype=torch.float32)
        for k, u in enumerate(model.units()):
            w, b = rt.acquire(u)
            act = model.active(idx, k)
            if act.any():
                rows = idx[act]
                loss = loss + ((w[rows].float() + b.float()) @ model.c[k]).sum() / B
            rt.release_forward(u)
        ctx.model, ctx.idx = model, idx
        return loss

    @staticmethod
    def backward(ctx, dloss):
        model, idx = ctx.model, ctx.idx
        rt = model.rt
        B = idx.shape[0]
        for k in reversed(range(K)):
            act = model.active(idx, k)
            if not act.any():
                continue                              # this unit does not report this micro-step
            u = model.units()[k]
            rt.acquire_backward(u)
            rows = idx[act]
            gw = torch.zeros(V, 4)
            gw.index_add_(0, rows.reshape(-1), model.c[k].expand(rows.numel(), 4) * (dloss / B))
            gb = model.c[k] * (rows.numel() * dloss / B)
            for i, g in enumerate((gw, gb)):
                slot, acc = rt.grad_slot(u, i)
                if acc:
                    slot += g.to(slot.dtype)
                else:
                    slot.copy_(g)
            rt.grads_ready(u)
            rt.release_backward(u)
        return None, None, None


class Toy(nn.Module):
    """K units of (W [V, 4], b [4]); row r uses unit k unless bit k of its first token is set."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.w = nn.ParameterList([nn.Parameter(torch.randn(V, 4, generator=g) * 0.1) for _ in range(K)])
        self.b = nn.ParameterList([nn.Parameter(torch.randn(4, generator=g) * 0.1) for _ in range(K)])
        self.c = [torch.tensor([1.0, -0.5, 0.25, 2.0]) * (k + 1) for k in range(K)]
        self._units = [Unit(f"u{k}", [(f"w.{k}", self.w[k]), (f"b.{k}", self.b[k])], k) for k in range(K)]
        self.rt = EAGER

    def units(self):
        return self._units

    @staticmethod
    def active(idx, k):
        return (idx[:, 0] >> k) & 1 == 0

    def forward(self, idx, targets=None):
        return None, _Fn.apply(torch.empty((), requires_grad=True), self, idx)


def _batches(global_batch, accum, same_on_ranks):
    """First tokens cycle through every skip pattern (including "every unit skipped").
    ``same_on_ranks``: at world 2 both ranks skip the same units in every micro-step (rank r's
    micro-step a is row r * accum + a).  The sharded engines need that: a unit's backward
    re-gathers its shard, and a collective only some ranks enter cannot complete (torch FSDP
    has the same requirement)."""
    g = torch.Generator().manual_seed(7)
    out = []
    n = 0
    for s in range(STEPS):
        b = torch.randint(0, V, (global_batch, T), generator=g)
        for r in range(global_batch):
            b[r, 0] = ((s * accum + r % accum) * 3) % 8 if same_on_ranks else (n * 3) % 8
            n += 1
        out.append(b)
    return out


def _cfg(strategy, accum, semantics="reference", stage=None):
    ds = None
    if strategy in ("zero2", "zero3"):
        ds = {"gradient_clipping": 1.0,
              "optimizer": {"type": "AdamW", "params": {"lr": 1e-2, "weight_decay": 0.01}},
              "zero_optimization": {"stage": 2 if strategy == "zero2" else 3, "reduce_bucket_size": 5e8,
                                    "stage3_param_persistence_threshold": 100,
                                    "stage3_max_live_parameters": 0, "stage3_max_reuse_distance": 1e9}}
    c = engine_config(strategy, accum, semantics, ds, None, bucket_mb=0.0005)
    c.lr = 1e-2
    c.extra["bucket_unit_multiple"] = 1        # one unit per bucket: a bucket can be wholly unreported
    if stage is not None:
        c.zero_stage = stage
    return c


def _train(strategy, accum, rank, world, semantics="reference", stage=None):
    model = Toy()
    eng = make_engine(model, _cfg(strategy, accum, semantics, stage), "cpu")
    eng.train()
    for b in _batches(2 * accum, accum, strategy in ("zero3", "fsdp")):   # same global batch at world 1, 2
        per = b.shape[0] // world
        mb = b[rank * per:(rank + 1) * per]
        micro = mb.shape[0] // accum
        for a in range(accum):
            x = mb[a * micro:(a + 1) * micro]
            loss = eng(x, x)[1]
            eng.backward(loss)
            eng.step()
    return eng.full_state_dict()


CASES = [("ddp", 1, "reference", None), ("ddp", 2, "uniform", None), ("zero2", 2, "reference", None),
         ("zero2", 2, "reference", 1), ("zero3", 2, "reference", None), ("fsdp", 1, "reference", None)]


def test_single_process_matches_autograd():
    """DDP at world 1 == autograd + torch.optim.AdamW: a unit skipped in a step gets a zero
    gradient (AdamW still decays it and moves it by its moments), not the last step's gradient."""
    sd = _train("ddp", 1, 0, 1)
    ref = Toy()
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.01)
    for b in _batches(2, 1, False):
        loss = torch.zeros(())
        for k in range(K):
            act = Toy.active(b, k)
            if act.any():
                loss = loss + ((ref.w[k][b[act]] + ref.b[k]) @ ref.c[k]).sum() / b.shape[0]
        for p in ref.parameters():
            p.grad = torch.zeros_like(p)
        loss.backward()
        opt.step()
    for k in range(K):
        assert torch.allclose(sd[f"w.{k}"], ref.w[k].detach(), atol=1e-6), k
        assert torch.allclose(sd[f"b.{k}"], ref.b[k].detach(), atol=1e-6), k


def _worker(rank, world, port, case, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("DLTB_COMM_LAZY", "1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        strategy, accum, sem, stage = case
        sd = _train(strategy, accum, rank, world, sem, stage)
        if rank == 0:
            torch.save(sd, out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-acc{c[1]}-{c[2]}-s{c[3]}")
def test_world2_lazy_with_unreported_units(case):
    from tests.test_parallel_cpu import _free_port
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sd.pt")
        mp.spawn(_worker, args=(2, _free_port(), case, out), nprocs=2, join=True)
        got = torch.load(out, weights_only=True)
    strategy, accum, sem, stage = case
    ref = _train(strategy, accum, 0, 1, sem, stage)
    for n in ref:
        assert torch.allclose(got[n], ref[n], atol=2e-5), (case, n, (got[n] - ref[n]).abs().max())
