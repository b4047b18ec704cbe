"""Every remaining hot-path switch, each supported combination once (round-2 toggle pruning left
five; the side-stream, mask-stream, overlapped-optimizer, standalone-dropout and fused
dropout-backward paths were measured neutral or slower and deleted):

* DLTB_GRAPHS (``--graphs``)      x  DLTB_BATCH_WGRAD (``batch_wgrad``)   x  replicated / sharded
* DLTB_WINDOW_WGRAD (``window_wgrad``, window-wide dW at world 1)  x  DLTB_GRAPHS, replicated
* DLTB_DEFER_OPT                  -- world > 1 only: tests/test_multirank_gpu.py runs ZeRO-1/2 both ways
* DLTB_DKDV_GSPLIT                -- causal GQA dK/dV head split, forced off vs auto, below
* DLTB_COMM_HIGH_PRIORITY         -- an RCCL stream priority (no effect on results; needs >1 GPU)
(The split-K fp32-plane GEMM path, the attention ping-pong forward and the side-stream dW / early DDP update
were measured slower and deleted in round 6; the toggle table is docs/ARCHITECTURE.md "Runtime switches".)
"""
import os
import subprocess
import sys

import pytest
import torch

from test_graphs_gpu import _run

pytestmark = pytest.mark.gpu
_BASE = {}


def _close(l0, s0, l1, s1):
    assert all(abs(a - b) < 2e-3 * abs(a) for a, b in zip(l0, l1)), (l0, l1)
    for k in s0:
        assert torch.allclose(s0[k], s1[k], rtol=2e-2, atol=2e-4), k


@pytest.mark.parametrize("strategy", ["zero2", "zero3"])
@pytest.mark.parametrize("graphed", [False, True])
@pytest.mark.parametrize("batch_wgrad", [True, False])
def test_toggle_matrix(strategy, graphed, batch_wgrad):
    if strategy not in _BASE:
        _BASE[strategy] = _run(strategy, False, windows=2, extra={"batch_wgrad": True})
    l1, s1 = _run(strategy, graphed, windows=2, extra={"batch_wgrad": batch_wgrad})
    l0, s0 = _BASE[strategy]
    _close(l0, s0, l1, s1)


@pytest.mark.parametrize("graphed", [False, True])
def test_window_wgrad_off_matches(graphed):
    if "zero2" not in _BASE:
        _BASE["zero2"] = _run("zero2", False, windows=2, extra={"batch_wgrad": True})
    l1, s1 = _run("zero2", graphed, windows=2, extra={"batch_wgrad": True, "window_wgrad": False})
    l0, s0 = _BASE["zero2"]
    _close(l0, s0, l1, s1)


_GSPLIT_SNIPPET = r"""
import torch, dltb
from dltb.models import build_model, get_model_config
from dltb.parallel import engine_config, make_engine
torch.manual_seed(0)
cfg = get_model_config("mtiny", 512)
with torch.device("cuda"):
    m = build_model(cfg)
eng = make_engine(m, engine_config("zero3", 1, "reference"), "cuda:0")
idx = torch.randint(0, cfg.vocab_size, (1, 512), device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
out = []
for _ in range(3):
    loss = eng(idx, idx)[1]; eng.backward(loss); eng.step(); out.append(loss.item())
print("LOSSES", *out)
"""


def test_dkdv_gsplit_forced_off_matches_auto():
    res = {}
    for v in ("1", "0"):                                 # 1 = no head split, 0 = auto (splits G = 2)
        env = dict(os.environ, DLTB_DKDV_GSPLIT=v)
        r = subprocess.run([sys.executable, "-c", _GSPLIT_SNIPPET], capture_output=True, text=True,
                           env=env, timeout=300, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr[-3000:]
        res[v] = [float(x) for x in r.stdout.split("LOSSES", 1)[1].split()]
    assert all(abs(a - b) < 1e-3 * abs(a) for a, b in zip(res["1"], res["0"])), res
