#!/usr/bin/env python3
"""Is the training step host (launch) bound?  Times K steps twice: the host enqueue time (no sync
inside the loop) and the wall time to drain the GPU.  enqueue ~= wall means the CPU side (Python +
HIP launches) sets the pace, not the kernels.

    python scripts/host_bound_check.py [--tier A] [--strategy zero2] [--steps 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.data import SyntheticDataset, make_batcher  # noqa: E402
from dltb.harness import _engine_for  # noqa: E402
from dltb.models import build_model, get_model_config  # noqa: E402
from dltb.utils.gemm_tuning import setup_tunableop  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tier", default="A")
    ap.add_argument("--strategy", default="zero2")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    setup_tunableop("auto")
    torch.manual_seed(42)
    cfg = get_model_config(a.tier, a.seq_len)
    with torch.device(dev):
        model = build_model(cfg)
    h = argparse.Namespace(strategy=a.strategy, deepspeed_config=None, fsdp_config=None, grad_accum=4,
                           accum_semantics="reference", dtype="bf16", bucket_mb=64.0, seed=42)
    eng, _ = _engine_for(h, model, dev)
    batches = make_batcher("device", SyntheticDataset(cfg.vocab_size, a.seq_len, 1000, 42), 1, 1, 0, a.strategy, dev)
    eng.train()

    def step():
        b = next(batches)
        loss = eng(b, b)[1]
        eng.backward(loss)
        eng.step()

    for _ in range(8):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    enq, wall = (t1 - t0) / a.steps * 1e3, (t2 - t0) / a.steps * 1e3
    print(f"host enqueue {enq:.3f} ms/step   wall {wall:.3f} ms/step   ratio {enq / wall:.2f}")


if __name__ == "__main__":
    main()
