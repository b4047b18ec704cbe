"""RCCL on the real device: the process group exactly as ``utils.dist.setup_distributed`` builds it
for multi-rank runs (backend "nccl" = RCCL, ``device_id`` eager init, high-priority internal
stream, explicit timeout, warm-up all-reduce), then every collective form the engines issue through
``comm.collectives.Comm`` -- async bf16 / fp32 reduce-scatter into a chunk, in-place all-gather of a
rank's slice, bucket all-reduce, the float64 MAX used for timings -- waited the way the engines wait
(``work.wait()`` orders the compute stream behind RCCL's).  A one-GPU box only allows a one-rank
communicator (RCCL refuses two ranks on one device), so the ring moves no bytes; what this pins is
that the RCCL library, our init options and the tensor/dtype/stream contract work on MI355X.  The
multi-rank engine logic itself runs on the GPU in test_multirank_gpu.py (host-staged gloo)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import os, sys
sys.path.insert(0, sys.argv[1])
import torch, torch.distributed as dist
import dltb  # noqa: F401
from dltb.utils.dist import setup_distributed, cleanup_distributed, all_reduce_max, barrier
from dltb.comm.collectives import Comm
dev = setup_distributed(1, 0, 0, device_type="cuda", timeout_min=2, force_pg=True)
assert dist.is_initialized() and dist.get_backend() == "nccl", dist.get_backend()
comm = Comm()
assert comm.backend == "nccl" and comm.world == 1 and not comm.staged
for dt in (torch.bfloat16, torch.float32):
    x = torch.arange(1 << 20, device=dev, dtype=torch.float32).remainder_(251).to(dt)
    out = torch.empty_like(x)
    w = dist.reduce_scatter_tensor(out, x, async_op=True)
    w.wait()
    assert torch.equal(out, x), dt
    flat = torch.zeros(1 << 20, device=dev, dtype=dt)
    w = dist.all_gather_into_tensor(flat, x, async_op=True)      # rank 0's slice = the whole buffer
    w.wait()
    assert torch.equal(flat, x), dt
    b = x.clone()
    w = dist.all_reduce(b, async_op=True)
    w.wait()
    assert torch.equal(b, x), dt
    y = (b.float() * 2).to(dt)                                   # compute stream after the wait
    assert torch.equal(y, (x.float() * 2).to(dt))
assert all_reduce_max(3.5, dev) == 3.5
t = torch.tensor([2.5], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
assert float(t.item()) == 2.5
barrier()
torch.cuda.synchronize(dev)
cleanup_distributed()
print("rccl ok", torch.cuda.get_device_name(dev))
"""


@pytest.mark.gpu
def test_rccl_process_group_one_rank():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29731", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "rccl ok" in r.stdout
