#!/usr/bin/env python3
"""Host cost of one ProcessGroupNCCL (RCCL) call, per collective form the engines issue.

VERDICT r3 Next #3a: the emulated fabric (DLTB_COMM=emulate:N) launches one paced kernel per
collective -- a few microseconds of host time -- while a real ``dist.reduce_scatter_tensor(...,
async_op=True)`` goes through ProcessGroupNCCL: work object, event record on the compute stream,
stream wait on RCCL's stream, the RCCL enqueue, caching-allocator stream bookkeeping.  That host time
is what an eager N-rank step pays per collective (about 20 per ZeRO-3 micro-step, 55 per FSDP-block
micro-step), so the emulator has to add it.

Measured here on the real RCCL library with a ONE-rank communicator (a one-GPU box cannot hold two
RCCL ranks; the host-side path is the same code up to RCCL's ring, which a 1-rank communicator
short-circuits on the device, not on the host): each form ``--calls`` times back to back while the
GPU is held busy by one long kernel (so no call waits for the device), host time per call, plus
``work.wait()`` (the engines wait every work once).  Written as JSON to ``--out``, which
comm/collectives.py reads as the per-op host cost of emulated collectives
(``profiles/pg_host_cost.json``).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pg_host_cost.json"))
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import dltb  # noqa: F401
    from dltb.ops._ext import ext
    from dltb.utils.dist import cleanup_distributed, setup_distributed
    dev = setup_distributed(1, 0, 0, device_type="cuda", timeout_min=2, force_pg=True)
    n = 25 << 20                                       # a 50 MB bf16 bucket
    x = torch.randn(n, device=dev).to(torch.bfloat16)
    out = torch.empty_like(x)
    f32 = torch.zeros(1, device=dev)
    forms = {
        "reduce_scatter": lambda: dist.reduce_scatter_tensor(out, x, async_op=True),
        "all_gather": lambda: dist.all_gather_into_tensor(out, x, async_op=True),
        "all_reduce": lambda: dist.all_reduce(x, async_op=True),
        "all_reduce_scalar_sync": lambda: dist.all_reduce(f32, async_op=False),
    }
    res = {}
    for name, fn in forms.items():
        for _ in range(5):
            w = fn()
            if w is not None:
                w.wait()
        torch.cuda.synchronize()
        ext().comm_emu(None, 1, None, None, 1.0, 1, 0, 2e5, 0.0, 1, 0)    # hold the GPU 200 ms
        works = []
        t0 = time.perf_counter()
        for _ in range(a.calls):
            works.append(fn())
        t1 = time.perf_counter()
        for w in works:
            if w is not None:
                w.wait()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        res[name] = {"issue_us": (t1 - t0) / a.calls * 1e6, "wait_us": (t2 - t1) / a.calls * 1e6}
        print(f"[pg-host] {name:24s} issue {res[name]['issue_us']:7.1f} us   wait {res[name]['wait_us']:6.1f} us",
              flush=True)
    rec = {"what": "host time per ProcessGroupNCCL call, 1-rank RCCL communicator, GPU held busy",
           "torch": torch.__version__, "calls": a.calls, "per_op_us": {
               k: round(v["issue_us"] + v["wait_us"], 2) for k, v in res.items()}, "detail": res}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec["per_op_us"]), flush=True)
    cleanup_distributed()


if __name__ == "__main__":
    main()
