"""Emulated-fabric comm mode (DLTB_COMM=emulate:N) on the CPU.

One process plays rank r of an N-rank job: the engines build their real N-rank layouts and every
collective runs a local stand-in (on a GPU also a paced kernel on a side stream, tests/
test_emulate_gpu.py).  Checked here:

* the stand-in numerics of every collective (identical-ranks semantics);
* for EVERY engine and layout (DDP, ZeRO-1/2, ZeRO-3 with and without keep-all, FSDP block / root /
  SHARD_GRAD_OP), the wire bytes the engine actually issues per micro-step equal its modelled
  ``comm_bytes_per_step`` -- the figure bench.py reports next to the measured one;
* the per-rank footprint: sharded state is 1/N of the world-1 state;
* ``bench.py --emulate N`` prints one prediction record.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

import dltb  # noqa: F401
from dltb.comm import Comm
from dltb.models import build_model, get_model_config
from dltb.models.tinygpt import TinyGPT
from dltb.parallel import engine_config, make_engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def emulate4(monkeypatch):
    monkeypatch.setenv("DLTB_COMM", "emulate:4")
    monkeypatch.setenv("DLTB_EMU_RANK", "1")
    yield 4


def test_collective_stand_ins(emulate4):
    c = Comm()
    assert (c.world, c.rank, c.backend) == (4, 1, "emulate")
    inp = torch.arange(16.)
    out = torch.zeros(4)
    c.reduce_scatter(out, inp)
    assert torch.equal(out, 4 * inp[4:8])                       # N x the own chunk
    full = torch.zeros(16)
    c.all_gather(full, torch.ones(4))                           # fresh buffer: the shard replicated
    assert torch.equal(full, torch.ones(16))
    buf = torch.arange(16.)
    c.all_gather(buf, buf[4:8])                                 # in place: unchanged
    assert torch.equal(buf, torch.arange(16.))
    t = torch.ones(3)
    c.all_reduce(t)
    assert torch.equal(t, torch.full((3,), 4.))
    c.all_reduce(t, op="max")
    assert torch.equal(t, torch.full((3,), 4.))
    assert c.stats["reduce_scatter"]["wire_bytes"] == int(16 * 4 * 3 / 4)
    assert c.modelled_us() > 3 * 25.0                            # alpha per call + bytes / bus


def _cfg(strategy, accum, **kw):
    ds = None
    if strategy in ("zero2", "zero3"):
        ds = {"gradient_clipping": 1.0, "optimizer": {"type": "AdamW", "params": {"lr": 1e-3}},
              "zero_optimization": {"stage": 2 if strategy == "zero2" else 3, "reduce_bucket_size": 5e8,
                                    "stage3_param_persistence_threshold": 300,
                                    "stage3_max_live_parameters": kw.pop("max_live", 1e9),
                                    "stage3_max_reuse_distance": 1e9}}
    shard_opt = kw.pop("shard_optimizer", False)
    c = engine_config(strategy, accum, kw.pop("semantics", "reference"), ds, kw.pop("fsdp", None),
                      bucket_mb=0.01, grad_reduce=kw.pop("grad_reduce", "micro"))
    if shard_opt:
        c.extra["shard_optimizer"] = True
    for k, v in kw.items():
        setattr(c, k, v)
    return c


CASES = [
    ("ddp", 1, {}), ("ddp", 1, {"shard_optimizer": True}), ("ddp", 2, {"semantics": "uniform"}), ("zero2", 4, {}), ("zero2", 4, {"grad_reduce": "window"}),
    ("zero3", 4, {}), ("zero3", 4, {"max_live": 0}), ("fsdp", 1, {}),
    ("fsdp", 1, {"fsdp": {"auto_wrap_policy": "size_based"}}),
    ("fsdp", 1, {"fsdp": {"sharding_strategy": "shard_grad_op"}}),
    ("fsdp", 2, {"semantics": "uniform"}),
    # Mistral shape: untied token table, reduced densely with the embedding's own bucket / group
    ("ddp", 1, {"tier": "mtiny"}), ("zero2", 4, {"tier": "mtiny"}), ("zero3", 4, {"tier": "mtiny"}),
]


@pytest.mark.parametrize("strategy,accum,kw", CASES, ids=[f"{c[0]}-{i}" for i, c in enumerate(CASES)])
def test_wire_bytes_equal_model(emulate4, strategy, accum, kw):
    torch.manual_seed(0)
    kw = dict(kw)
    mcfg = get_model_config(kw.pop("tier", "tiny"), 16)
    mcfg.dropout = 0.0
    model = build_model(mcfg)
    eng = make_engine(model, _cfg(strategy, accum, **kw), "cpu")
    eng.train()
    assert eng.world == 4
    g = torch.Generator().manual_seed(1)

    def window():
        for _ in range(accum):
            x = torch.randint(0, min(128, mcfg.vocab_size), (1, 16), generator=g)
            loss = eng(x, x)[1]
            eng.backward(loss)
            eng.step()

    window()
    eng.finalize()               # a deferred update of window 1 must not land in the count
    eng.comm.reset_stats()
    window()
    window()
    eng.finalize()
    per = eng.comm.wire_bytes() / (2 * accum)
    model_b = eng.comm_bytes_per_step
    assert model_b > 0
    # the one-float grad-norm all-reduce (6 bytes per window at N = 4) is not modelled
    assert abs(per - model_b) <= 8, (strategy, kw, per, model_b, dict(eng.comm.stats))


def test_sharded_footprint_is_one_nth(emulate4, monkeypatch):
    torch.manual_seed(0)
    m4 = TinyGPT(get_model_config("tiny", 16, dropout=0.0))
    e4 = make_engine(m4, _cfg("zero3", 2, max_live=0), "cpu")
    monkeypatch.setenv("DLTB_COMM", "rccl")
    torch.manual_seed(0)
    m1 = TinyGPT(get_model_config("tiny", 16, dropout=0.0))
    e1 = make_engine(m1, _cfg("zero3", 2, max_live=0), "cpu")
    assert e1.world == 1 and e4.world == 4
    r1, r4 = e1.memory_report(), e4.memory_report()
    assert r4["shard_param_bytes"] * 4 >= r1["shard_param_bytes"] >= (r4["shard_param_bytes"] - 4 * 128 * 4 * 32) * 4
    assert e4.opt.master.numel() * 4 < e1.opt.master.numel() * 1.2


def test_bench_emulate_prediction_record():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DLTB_COMM"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--tier", "tiny",
                        "--seq-len", "32", "--steps", "8", "--warmup", "4", "--emulate", "8"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(rec) == 1
    rec = rec[0]
    assert rec["prediction"] is True and rec["emulated_world"] == 8 and rec["n_gpus"] == 1
    assert rec["metric"] == "tokens_per_sec_predicted" and rec["vs_baseline"] is None
    assert rec["config"]["parallelism"] == "zero2-dp8" and rec["world_size_seen"] == 8
    assert rec["comm_model_ms_per_step"] > 0
    assert abs(rec["wire_bytes_per_step"] - rec["wire_bytes_per_step_model"]) <= 8


def test_world_n_wgrad_batches(monkeypatch):
    """World > 1 keeps the weight gradients batched: ZeRO-2 plans the head as a bucket of its own and
    the blocks in whole groups of 4 (one 4-block batched dW per kind and bucket, not 2/4/4/4/2), and
    the sharded engines batch the dW of 4 completed block groups from their gradient arena."""
    monkeypatch.setenv("DLTB_COMM", "emulate:8")
    torch.manual_seed(0)
    mcfg = get_model_config("A", 64)
    mcfg.n_layer, mcfg.n_embd, mcfg.n_head, mcfg.vocab_size, mcfg.dropout = 8, 128, 2, 512, 0.0
    model = build_model(mcfg)
    blk = model.unit_blocks[0].numel
    cfg = engine_config("zero2", 4, "reference", None, bucket_mb=4 * blk * 4 / 2**20 * 0.6)
    eng = make_engine(model, cfg, "cpu")
    names = [[u.name for u in b.units] for b in eng.layout.buckets]
    assert names[0] == ["head"] and names[-1] == ["embed"], names
    assert all(len(n) == 4 for n in names[1:-1]), names
    # 16 blocks: the first bucket after the head takes 8 (fewer collectives early in the backward), the
    # last ones keep 4 (the next forward's first parameter all-gathers)
    mcfg16 = get_model_config("A", 64)
    mcfg16.n_layer, mcfg16.n_embd, mcfg16.n_head, mcfg16.vocab_size, mcfg16.dropout = 16, 128, 2, 512, 0.0
    eng16 = make_engine(build_model(mcfg16), engine_config("zero2", 4, "reference", None,
                                                           bucket_mb=4 * blk * 4 / 2**20 * 0.6), "cpu")
    assert [len(b.units) for b in eng16.layout.buckets] == [1, 8, 4, 4, 1]
    for strategy in ("zero3", "fsdp"):
        torch.manual_seed(0)
        model = build_model(mcfg)
        c = engine_config(strategy, 4, "uniform", None, bucket_mb=1.0)
        c.persistence_threshold = 100             # (ZeRO-3: keep the small blocks' matrices sharded)
        eng = make_engine(model, c, "cpu")
        assert eng.defer_wgrad and eng._arena is not None
        eng.train()
        x = torch.randint(0, 512, (1, 64))
        loss = eng(x, x)[1]
        eng.backward(loss)
        eng.step()
        assert eng._wq.batched_calls == 2 * 4 and eng._wq.single_calls == 0, (strategy, eng._wq.batched_calls,
                                                                              eng._wq.single_calls)
