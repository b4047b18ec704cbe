"""Engine correctness on CPU (gloo "fake cluster").

* single process: every engine == stock torch training (oracle model + torch.optim.AdamW) under
  the reference semantics;
* world_size 2: every strategy (DDP, FSDP block/root wrap, ZeRO-2, ZeRO-3) reproduces the
  single-process run on the concatenated global batch, with gradient accumulation for ZeRO.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dltb
from dltb.models import get_model_config
from dltb.models.oracle import OracleTinyGPT
from dltb.models.tinygpt import TinyGPT
from dltb.parallel import engine_config, make_engine

T = 16
STEPS = 4


def _close(a, b, name, atol):
    """The key part of in_proj_bias has an exactly-zero true gradient (softmax is invariant to a
    per-row constant); Adam turns its rounding noise into +-lr steps, so it is not compared."""
    if name.endswith("attn.in_proj_bias"):
        d = a.numel() // 3
        a = torch.cat([a[:d], a[2 * d:]])
        b = torch.cat([b[:d], b[2 * d:]])
    return torch.allclose(a, b, atol=atol)


def _model():
    torch.manual_seed(0)
    return TinyGPT(get_model_config("tiny", T, dropout=0.0))


def _batches(n_steps, global_batch):
    g = torch.Generator().manual_seed(123)
    return [torch.randint(0, 128, (global_batch, T), generator=g) for _ in range(n_steps)]


def _cfg(strategy, accum, semantics="reference", **kw):
    ds = None
    if strategy in ("zero2", "zero3"):
        ds = {"gradient_clipping": 1.0, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3, "weight_decay": 0.01}},
              "scheduler": {"type": "WarmupLR", "params": {"warmup_min_lr": 0, "warmup_max_lr": 1e-3, "warmup_num_steps": 3}},
              "zero_optimization": {"stage": 2 if strategy == "zero2" else 3, "reduce_bucket_size": 5e8,
                                    "stage3_param_persistence_threshold": 300,
                                    "stage3_max_live_parameters": kw.pop("max_live", 1e9),
                                    "stage3_max_reuse_distance": 1e9}}
    fc = kw.pop("fsdp", None)
    shard_opt = kw.pop("shard_optimizer", False)
    c = engine_config(strategy, accum, semantics, ds, fc, bucket_mb=kw.pop("bucket_mb", 0.01))
    if shard_opt:
        c.extra["shard_optimizer"] = True
    c.lr = 1e-3 if strategy in ("ddp", "fsdp") and semantics == "reference" else c.lr
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def _train(strategy, batches, rank, world, accum, **kw):
    model = _model()
    eng = make_engine(model, _cfg(strategy, accum, **kw), "cpu")
    eng.train()
    for b in batches:
        per = b.shape[0] // world
        mb = b[rank * per:(rank + 1) * per]
        micro = mb.shape[0] // accum
        for a in range(accum):
            x = mb[a * micro:(a + 1) * micro]
            loss = eng(x, x)[1]
            eng.backward(loss)
            eng.step()
    return eng.full_state_dict()


def test_single_process_ddp_matches_torch_adamw():
    batches = _batches(STEPS, 2)
    sd = _train("ddp", batches, 0, 1, 1)
    torch.manual_seed(0)
    ref_model = _model()
    oracle = OracleTinyGPT(ref_model.cfg)
    oracle.load_state_dict(ref_model.state_dict())
    opt = torch.optim.AdamW(oracle.parameters(), lr=1e-3, weight_decay=0.01)
    for b in batches:
        _, loss = oracle(b, b)
        loss.backward()
        opt.step()
        opt.zero_grad()
    for n, p in oracle.named_parameters():
        assert _close(sd[n], p.detach(), n, 2e-5), n


@pytest.mark.parametrize("strategy,kw", [
    ("ddp", {}), ("zero2", {}), ("zero3", {}), ("zero3", {"max_live": 0}), ("fsdp", {}),
    ("fsdp", {"fsdp": {"auto_wrap_policy": "size_based"}}),
    ("fsdp", {"fsdp": {"sharding_strategy": "shard_grad_op"}}),
])
def test_single_process_engines_agree(strategy, kw):
    """Every engine at world_size 1 trains identically to DDP under the same semantics."""
    batches = _batches(STEPS, 2)
    accum = 2 if strategy.startswith("zero") else 1
    base = _train("ddp" if not strategy.startswith("zero") else "zero2", batches, 0, 1, accum)
    got = _train(strategy, batches, 0, 1, accum, **dict(kw))
    for n in base:
        assert _close(got[n], base[n], n, 1e-6), (strategy, n)


# ---------------------------------------------------------------- multi-process (gloo)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, strategy, accum, kw, out_path, global_batch=4):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        sd = _train(strategy, _batches(STEPS, global_batch), rank, world, accum, **kw)
        if rank == 0:
            torch.save(sd, out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("strategy,accum,kw", [
    ("ddp", 1, {}),
    ("ddp", 1, {"shard_optimizer": True}),  # DDP + ZeroRedundancyOptimizer: same training, sharded state
    ("ddp", 2, {"semantics": "uniform"}),
    ("zero2", 2, {}),
    ("zero2", 2, {"zero_stage": 1}),       # --grad-reduce window: one reduce-scatter per window
    ("zero3", 2, {}),
    ("zero3", 1, {"max_live": 0}),
    ("fsdp", 1, {}),
    ("fsdp", 1, {"fsdp": {"auto_wrap_policy": "size_based"}}),
])
def test_world2_matches_single_process(strategy, accum, kw):
    world = 2
    sem = kw.pop("semantics", "reference")
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sd.pt")
        mp.spawn(_worker, args=(world, _free_port(), strategy, accum, dict(kw, semantics=sem) if sem != "reference" else kw, out),
                 nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    # single process on the concatenated batch: same global batch per micro-step
    ref = _train(strategy, _batches(STEPS, 4), 0, 1, accum, **(dict(kw, semantics=sem) if sem != "reference" else kw))
    for n in ref:
        assert _close(got[n], ref[n], n, 2e-5), (strategy, n, (got[n] - ref[n]).abs().max())


@pytest.mark.parametrize("strategy,accum,kw", [("zero2", 2, {}), ("zero2", 2, {"zero_stage": 1}),
                                               ("zero3", 2, {}), ("ddp", 1, {}), ("ddp", 1, {"shard_optimizer": True}),
                                               ("fsdp", 1, {})])
def test_world4_matches_single_process(strategy, accum, kw):
    """Four ranks (uneven bucket chunks, padding on every rank, prefetch across 4 shards) reproduce
    the single-process run on the same global batch -- the rank layout of the 4-GPU baseline."""
    world, gb = 4, 8
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sd.pt")
        mp.spawn(_worker, args=(world, _free_port(), strategy, accum, dict(kw), out, gb), nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    ref = _train(strategy, _batches(STEPS, gb), 0, 1, accum, **dict(kw))
    for n in ref:
        assert _close(got[n], ref[n], n, 2e-5), (strategy, n, (got[n] - ref[n]).abs().max())


def _worker_defer(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        res = {}
        for defer in ("1", "0"):
            os.environ["DLTB_DEFER_OPT"] = defer
            res[defer] = _train("zero2", _batches(STEPS, 4), rank, world, 2)
        if rank == 0:
            torch.save(res, out_path)
    finally:
        dist.destroy_process_group()


def test_world2_deferred_optimizer_step_is_exact():
    """ZeRO-2 at world 2 runs the window's AdamW + parameter all-gather at the start of the next
    micro-step (overlapping the forward); the trained weights must be bitwise identical."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sd.pt")
        mp.spawn(_worker_defer, args=(2, _free_port(), out), nprocs=2, join=True)
        res = torch.load(out, weights_only=True)
    for n in res["1"]:
        assert torch.equal(res["1"][n], res["0"][n]), n


def test_zero3_288gb_config_keeps_gathered_params():
    """configs/deepspeed/zero3_mi355x_288gb.json: a Mistral-7B-sized model fits under
    stage3_max_live_parameters, so the ZeRO-3 engine keeps gathered parameters resident
    (keep_all); the reference's zero3.json (1e9) does not for that size."""
    import json
    import os
    from dltb.parallel.strategy import load_deepspeed_config
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    big = load_deepspeed_config(os.path.join(root, "configs", "deepspeed", "zero3_mi355x_288gb.json"))
    ref = load_deepspeed_config(os.path.join(root, "configs", "deepspeed", "zero3.json"))
    m7b = 7_241_732_096
    for cfg, keep in ((big, True), (ref, False)):
        z = cfg["zero_optimization"]
        assert (m7b <= z["stage3_max_live_parameters"] and m7b <= z["stage3_max_reuse_distance"]) == keep
    assert {k: v for k, v in big.items() if k != "_comment" and k != "zero_optimization"} == \
        {k: v for k, v in ref.items() if k != "_comment" and k != "zero_optimization"}
    torch.manual_seed(0)
    m = TinyGPT(get_model_config("tiny", 16, dropout=0.0))
    e = make_engine(m, engine_config("zero3", 2, "reference", ds_config=big), "cpu")
    assert e.keep_all
    json.dumps(big)


def _worker_lazy(rank, *args):
    os.environ["DLTB_COMM_LAZY"] = "1"        # every async collective runs at its wait()
    _worker(rank, *args)


@pytest.mark.parametrize("strategy,accum,kw", [
    ("ddp", 1, {}),
    ("ddp", 1, {"shard_optimizer": True}),  # DDP + ZeroRedundancyOptimizer: same training, sharded state
    ("ddp", 2, {"semantics": "uniform"}),
    ("zero2", 2, {}),
    ("zero2", 2, {"zero_stage": 1}),
    ("zero3", 2, {}),
    ("zero3", 1, {"max_live": 0}),
    ("fsdp", 1, {}),
    ("fsdp", 2, {"semantics": "uniform"}),
])
def test_world2_lazy_collectives_match_single_process(strategy, accum, kw):
    """Wait discipline: with DLTB_COMM_LAZY=1 a collective reads its input and writes its output
    only when its work is waited (the latest point RCCL could), so a buffer reused before the
    collective finished, a result read before its wait, or a work never waited changes the trained
    weights.  Deferred reduce-scatters across micro-steps, deferred parameter all-gathers waited in
    ``acquire`` and ZeRO-3 / FSDP prefetches must all still reproduce the single-process run."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "sd.pt")
        mp.spawn(_worker_lazy, args=(world, _free_port(), strategy, accum, dict(kw), out), nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    ref = _train(strategy, _batches(STEPS, 4), 0, 1, accum, **dict(kw))
    for n in ref:
        assert _close(got[n], ref[n], n, 2e-5), (strategy, n, (got[n] - ref[n]).abs().max())



def test_reported_grad_comm_dtype_is_the_one_reduced():
    """the sharded-optimizer DDP (stage 1) reduce-scatters the compute-dtype buffer; an fp32 request
    is overridden and the engine reports the dtype its collectives actually carry (bench.py / harness read it)."""
    from dltb.parallel.replicated import grad_comm_dtype
    assert grad_comm_dtype(0, 8, True, torch.float16) == "fp32"       # ddp fp16: fp32 all-reduce
    assert grad_comm_dtype(0, 8, False, torch.bfloat16) == "bf16"
    assert grad_comm_dtype(1, 8, True, torch.float16) == "fp16"       # ddp_zero1: not widened
    assert grad_comm_dtype(1, 8, True, torch.bfloat16) == "bf16"
    assert grad_comm_dtype(2, 8, True, torch.bfloat16) == "bf16"
    eng = make_engine(_model(), _cfg("ddp", 1), "cpu")
    assert eng.grad_comm_dtype == "fp32"                               # CPU engines compute in fp32
