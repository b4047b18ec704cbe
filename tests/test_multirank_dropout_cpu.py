"""Dropout at world size 2 (gloo / CPU; tests/test_multirank_gpu.py runs the same on the GPU).

The reference seeds every rank the same way and draws dropout from the per-device global CUDA
generator (train_harness.py:283-284), so ranks see different masks; here every rank has its own
counter-hash stream ``StepSeed(seed, rank)`` (ops/rng.py).  With every rank reading the SAME rows:
* the ranks' losses differ at every micro-step (distinct masks -- a regression to one shared
  stream would make them equal and still train);
* a re-run with the same seed is bitwise identical (deterministic streams);
* the mean loss stays within dropout noise of the world-1 run on the same rows.
"""
import pytest
import torch

from multirank_util import run

ARGS = ("--cases", "dropout", "--seq-len", "64")


def test_world2_dropout_streams(tmp_path):
    ws1 = run(tmp_path / "ws1.pt", 1, "cpu", extra=ARGS)["dropout"]
    a = run(tmp_path / "a.pt", 2, "cpu", extra=ARGS)["dropout"]
    b = run(tmp_path / "b.pt", 2, "cpu", extra=ARGS)["dropout"]
    for r0, r1 in a["rank_losses"]:
        assert r0 != r1, "ranks drew the same dropout masks"
    assert a["rank_losses"] == b["rank_losses"]
    for n in a["final"]:
        assert torch.equal(a["final"][n], b["final"][n]), n
    for l1, l2 in zip(ws1["losses"], a["losses"]):
        assert abs(l1 - l2) < 0.02 * abs(l1), (l1, l2)
