"""Sharded checkpoint / resume: train -> save -> continue equals fresh -> load -> continue,
single process and 2 ranks (gloo), for replicated (DDP / ZeRO-2) and sharded (ZeRO-3 / FSDP)
engines; consolidated safetensors export carries the reference parameter names."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dltb
from dltb.models import build_model, get_model_config
from dltb.parallel import engine_config, export_consolidated, load_checkpoint, make_engine, save_checkpoint

T = 16


def _engine(strategy, accum):
    torch.manual_seed(0)
    cfg = get_model_config("tiny", T, dropout=0.1)
    model = build_model(cfg)
    c = engine_config(strategy, accum, "reference", bucket_mb=0.01)
    return make_engine(model, c, "cpu")


def _batches(n, rank, world):
    g = torch.Generator().manual_seed(5)
    out = [torch.randint(0, 128, (2 * world, T), generator=g) for _ in range(n)]
    return [b[2 * rank:2 * rank + 2] for b in out]


def _train(eng, batches):
    eng.train()
    for b in batches:
        micro = b.shape[0] // eng.accum
        for a in range(eng.accum):
            x = b[a * micro:(a + 1) * micro]
            eng.backward(eng(x, x)[1])
            eng.step()


def _roundtrip(strategy, accum, rank, world, d):
    batches = _batches(4, rank, world)
    e1 = _engine(strategy, accum)
    _train(e1, batches[:2])
    save_checkpoint(e1, d)
    _train(e1, batches[2:])
    want = e1.full_state_dict()
    e2 = _engine(strategy, accum)
    meta = load_checkpoint(e2, d)
    assert meta["opt_steps"] == e2.opt_steps
    _train(e2, batches[2:])
    got = e2.full_state_dict()
    return want, got


@pytest.mark.parametrize("strategy,accum", [("ddp", 1), ("zero2", 2), ("zero3", 2), ("fsdp", 1)])
def test_resume_single_process(strategy, accum, tmp_path):
    want, got = _roundtrip(strategy, accum, 0, 1, str(tmp_path / "ck"))
    for k in want:
        assert torch.equal(want[k], got[k]), k


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, strategy, accum, d, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        want, got = _roundtrip(strategy, accum, rank, world, d)
        ok = all(torch.equal(want[k], got[k]) for k in want)
        torch.save({"ok": ok}, os.path.join(out, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("strategy,accum", [("zero2", 2), ("zero3", 2)])
def test_resume_world2(strategy, accum):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), strategy, accum, os.path.join(d, "ck"), d), nprocs=2, join=True)
        for r in range(2):
            assert torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)["ok"], r
        assert sorted(f for f in os.listdir(os.path.join(d, "ck"))) == ["meta.json", "rank00000.pt", "rank00001.pt"]


def test_export_and_guards(tmp_path):
    e = _engine("zero2", 2)
    _train(e, _batches(1, 0, 1))
    path = export_consolidated(e, str(tmp_path / "model.safetensors"), torch.float32)
    from safetensors.torch import load_file
    sd = load_file(path)
    assert "transformer.h.0.attn.in_proj_weight" in sd and "lm_head.weight" in sd
    full = e.full_state_dict()
    assert torch.equal(sd["transformer.h.1.mlp.0.weight"], full["transformer.h.1.mlp.0.weight"])
    e.backward(e(_batches(1, 0, 1)[0][:1], _batches(1, 0, 1)[0][:1])[1])
    e.step()
    with pytest.raises(RuntimeError):          # mid-window
        save_checkpoint(e, str(tmp_path / "bad"))
    e2 = _engine("zero3", 2)
    save_checkpoint(_engine("zero2", 2), str(tmp_path / "z2"))
    with pytest.raises(ValueError):
        load_checkpoint(e2, str(tmp_path / "z2"))


def test_harness_save_resume_export(tmp_path):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    base = [sys.executable, os.path.join(root, "benchmarking", "train_harness.py"), "--strategy", "zero2",
            "--tier", "tiny", "--seq-len", "32", "--steps", "4", "--warmup-steps", "1", "--per-device-batch", "1",
            "--grad-accum", "2", "--device", "cpu", "--log-every", "0", "--results-dir", str(tmp_path / "res")]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(base + ["--save-dir", str(tmp_path / "ck"), "--export-model", str(tmp_path / "m.safetensors")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert (tmp_path / "ck" / "rank00000.pt").exists() and (tmp_path / "m.safetensors").exists()
    r = subprocess.run(base + ["--resume", str(tmp_path / "ck")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Resumed from" in r.stdout and "optimizer step 2" in r.stdout
