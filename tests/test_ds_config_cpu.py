"""Every DeepSpeed ZeRO key is honoured, satisfied by construction, or rejected (parallel/ds_config.py).

Reference configs: configs/deepspeed/zero2.json:1-49 and zero3.json:1-51 of the reference, read by
deepspeed.initialize at benchmarking/train_harness.py:240-271.  Each size / switch key's effect is
pinned on the engines: bucket caps on the planned layout, the ZeRO-3 prefetch budget on the gathers
in flight, the reuse-distance keep on the units left gathered after the forward, sub_group_size on
the AdamW launch split, and the three stage-2 switches by a gloo world-2 == world-1 run.
"""
import copy
import json
import os

import pytest
import torch

import dltb  # noqa: F401
from dltb.models.tinygpt import TinyGPT
from dltb.models import get_model_config
from dltb.optim.adamw import FlatAdamW
from dltb.parallel import engine_config, make_engine
from dltb.parallel.ds_config import apply_deepspeed_config, ds_precision
from dltb.parallel.strategy import default_config_path, load_deepspeed_config

from multirank_util import compare, run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ds(strategy):
    return load_deepspeed_config(default_config_path(strategy))


@pytest.mark.parametrize("strategy", ["zero2", "zero3"])
def test_reference_configs_fully_classified(strategy):
    """The shipped configs (same keys / values as the reference's): nothing ignored, and every
    key lands in exactly one class."""
    ds = _ds(strategy)
    cfg = engine_config(strategy, 4, "reference", ds)
    rep = cfg.extra["ds_keys"]
    assert rep["ignored"] == {}, rep["ignored"]
    keys = set(rep["honoured"]) | set(rep["by_construction"])
    z = {f"zero_optimization.{k}" for k in ds["zero_optimization"] if not k.startswith("offload")}
    z |= {f"zero_optimization.{k}.device" for k in ds["zero_optimization"] if k.startswith("offload")}
    top = {"optimizer", "scheduler", "gradient_clipping", "steps_per_print", "wall_clock_breakdown",
           "flops_profiler", "bf16.enabled"}
    assert z | top <= keys, (z | top) - keys
    assert cfg.grad_clip == 1.0 and cfg.lr == 1e-4 and cfg.scheduler["type"] == "WarmupLR"
    if strategy == "zero3":
        assert cfg.extra["prefetch_elems"] == int(5e8) and cfg.extra["sub_group_elems"] == int(1e9)
        assert cfg.persistence_threshold == int(1e5)
    else:
        assert cfg.extra["allgather_bucket_elems"] == int(5e8) and cfg.extra["reduce_scatter"] is True


def test_unknown_keys_are_listed_not_dropped():
    ds = _ds("zero2")
    ds["zero_optimization"]["ignore_unused_parameters"] = True
    ds["amp"] = {"enabled": False}
    rep = engine_config("zero2", 4, "reference", ds).extra["ds_keys"]
    assert "zero_optimization.ignore_unused_parameters" in rep["ignored"] and "amp" in rep["ignored"]


@pytest.mark.parametrize("mutate, key", [
    (lambda d: d["zero_optimization"].update(offload_optimizer={"device": "cpu"}), "offload_optimizer"),
    (lambda d: d["zero_optimization"].update(offload_param={"device": "nvme"}), "offload_param"),
    (lambda d: d["optimizer"].update(type="SGD"), "optimizer.type"),
    (lambda d: d["optimizer"]["params"].update(adam_w_mode=False), "adam_w_mode"),
    (lambda d: d["scheduler"].update(type="OneCycle"), "scheduler.type"),
    (lambda d: d.update(fp16={"enabled": True}), "both precisions"),
    (lambda d: d["zero_optimization"].update(stage=3), "zero_optimization.stage"),
])
def test_unsupported_values_rejected_loudly(mutate, key):
    ds = copy.deepcopy(_ds("zero2"))
    mutate(ds)
    with pytest.raises(ValueError, match=key):
        engine_config("zero2", 4, "reference", ds)


def test_fp16_config_selects_fp16():
    ds = _ds("zero2")
    del ds["bf16"]
    ds["fp16"] = {"enabled": True, "loss_scale": 0}
    assert ds_precision(ds) == "fp16" and ds_precision(_ds("zero2")) == "bf16"
    rep = engine_config("zero2", 4, "reference", ds).extra["ds_keys"]
    assert rep["honoured"]["fp16.enabled"] is True and "fp16.loss_scale" in rep["ignored"]


def _tiny(layers=4):
    c = get_model_config("A", 64, dropout=0.0)
    c.n_embd, c.n_head, c.n_layer, c.vocab_size = 64, 2, layers, 256
    torch.manual_seed(0)
    return TinyGPT(c)


@pytest.mark.parametrize("which", ["reduce_bucket_size", "allgather_bucket_size"])
def test_zero2_bucket_caps_are_upper_bounds(monkeypatch, which):
    """Both stage-2 size keys bound every bucket (unit granularity), below the --bucket-mb threshold."""
    monkeypatch.setenv("DLTB_COMM", "emulate:2")
    model = _tiny(6)
    block = model.unit_blocks[0].numel
    ds = _ds("zero2")
    ds["zero_optimization"][which] = int(2.5 * block)
    cfg = engine_config("zero2", 4, "reference", ds, bucket_mb=1000.0)
    eng = make_engine(model, cfg, "cpu")
    sizes = [b.numel for b in eng.layout.buckets]
    pad = 2 * 128
    assert max(sizes) <= 2.5 * block + pad, sizes
    assert sum(1 for s in sizes if s > 1.5 * block) >= 2        # two blocks per bucket, not one


def test_bucket_cap_below_one_unit_rejected(monkeypatch):
    monkeypatch.setenv("DLTB_COMM", "emulate:2")
    model = _tiny()
    ds = _ds("zero2")
    ds["zero_optimization"]["allgather_bucket_size"] = model.unit_blocks[0].numel // 2
    with pytest.raises(ValueError, match="allgather_bucket_size"):
        make_engine(model, engine_config("zero2", 4, "reference", ds), "cpu")
    ds = _ds("zero3")
    ds["zero_optimization"].update(reduce_bucket_size=model.unit_blocks[0].numel // 2,
                                   stage3_param_persistence_threshold=100)
    with pytest.raises(ValueError, match="reduce_bucket_size"):
        make_engine(_tiny(), engine_config("zero3", 4, "reference", ds), "cpu")


def _zero3(monkeypatch, **z):
    monkeypatch.setenv("DLTB_COMM", "emulate:2")
    model = _tiny(6)
    ds = _ds("zero3")
    ds["zero_optimization"].update(stage3_param_persistence_threshold=100, **z)
    eng = make_engine(model, engine_config("zero3", 4, "reference", ds), "cpu")
    return model, eng


def test_zero3_prefetch_budget_in_elements(monkeypatch):
    """stage3_prefetch_bucket_size: units gathered ahead while their summed size fits the budget."""
    model, _ = _zero3(monkeypatch)
    block = None
    for budget, ahead in ((1, 1), (2.5, 2), (4.2, 4)):
        model, eng = _zero3(monkeypatch, stage3_max_live_parameters=0,
                            stage3_prefetch_bucket_size=int(budget * model.unit_blocks[0].numel))
        block = model.unit_blocks[0]
        eng.acquire(block)                  # block 0: gathers itself + what the budget allows ahead
        gathered = [g for g in eng._order if g.full is not None]
        k = eng._pos[eng._group_of[id(block)].gid]
        assert [eng._pos[g.gid] for g in gathered] == list(range(k, k + 1 + ahead)), (budget, ahead)


def test_zero3_reuse_distance_keeps_last_units(monkeypatch):
    """max_reuse_distance below the model: the units whose backward follows within the distance stay
    gathered after the forward; the others are released (and re-gathered in backward)."""
    model = _tiny(6)
    blk, head = model.unit_blocks[0].numel, model.unit_head.numel
    # head (distance 0) and the last block (2 x head) kept, block 4 (2 x (head + block)) released
    _, eng = _zero3(monkeypatch, stage3_max_reuse_distance=int(2 * head + blk),
                    stage3_max_live_parameters=int(1e9))
    assert not eng.keep_all
    kept = {g.gid for g in eng.groups if g.gid in eng._reuse_keep}
    assert eng._group_of[id(eng.model.unit_head)].gid in kept
    assert eng._group_of[id(eng.model.unit_blocks[-1])].gid in kept
    assert eng._group_of[id(eng.model.unit_blocks[-2])].gid not in kept
    idx = torch.randint(0, 256, (1, 64))
    eng.train()
    loss = eng(idx, idx)[1]                 # forward done: which units are still gathered?
    live = {g.gid for g in eng.groups if g.full is not None}
    assert eng._group_of[id(eng.model.unit_blocks[-1])].gid in live
    assert eng._group_of[id(eng.model.unit_blocks[0])].gid not in live
    eng.backward(loss)
    eng.step()


def test_sub_group_size_same_update():
    """sub_group_size: the owner space updated in pieces gives the identical update."""
    torch.manual_seed(1)
    n = 4096
    master = torch.randn(n)
    g = torch.randn(n)
    outs = []
    for sg in (0, 1000):
        m = master.clone()
        dst = torch.empty(n)
        opt = FlatAdamW(m, [(0, n, dst)], 1e-2, sub_group=sg)
        for _ in range(3):
            opt.step(g, 1e-2)
        outs.append((m, opt.exp_avg.clone(), opt.exp_avg_sq.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_harness_sidecar_lists_keys(tmp_path):
    """The harness writes the key report into the extended sidecar (config_keys_ignored too)."""
    from dltb.harness import main
    cfg = _ds("zero2")
    cfg["some_unknown_key"] = 1
    p = tmp_path / "z2.json"
    p.write_text(json.dumps(cfg))
    os.environ.pop("WORLD_SIZE", None)
    main(["--strategy", "zero2", "--tier", "tiny", "--seq-len", "32", "--steps", "3", "--warmup-steps", "1",
          "--per-device-batch", "1", "--grad-accum", "2", "--deepspeed-config", str(p), "--results-dir",
          str(tmp_path / "res"), "--device", "cpu"])
    ext = [f for f in os.listdir(tmp_path / "res") if f.endswith(".extended.json")]
    side = json.loads((tmp_path / "res" / ext[0]).read_text())
    assert side["config_keys_ignored"] == ["some_unknown_key"]
    assert "zero_optimization.overlap_comm" in side["deepspeed_config_keys"]["honoured"]


def test_ds_switches_world2_equals_world1(tmp_path):
    """overlap_comm / reduce_scatter / allgather_partitions false, and the ZeRO-3 budgets (prefetch
    elements, reuse-distance keep, AdamW sub-groups): gloo world 2 trains the world-1 model."""
    ex = ("--cases", "zero2_ds_switches,zero3_ds_budgets")
    ws1 = run(tmp_path / "ws1.pt", 1, "cpu", extra=ex)
    ws2 = run(tmp_path / "ws2.pt", 2, "cpu", extra=ex)
    bad = compare(ws1, ws2, loss_tol=1e-4, upd_tol=1e-3, cos_min=0.99999, param_tol=1e-3)
    assert not bad, bad
