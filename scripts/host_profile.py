#!/usr/bin/env python3
"""Host-side (Python) cost of an eager TinyGPT-A micro-step: cProfile over K eager steps after
warm-up, top functions by own time.  Eager execution is what multi-rank runs use, so every
microsecond of Python per step that exceeds the GPU time is lost wall time.

    python scripts/host_profile.py [--steps 20] [--strategy zero2] [--top 40]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
from dltb.models import build_model, get_model_config  # noqa: E402
from dltb.parallel import engine_config, make_engine  # noqa: E402
from dltb.utils.gemm_tuning import setup_tunableop  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--strategy", default="zero2")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    setup_tunableop("auto")
    torch.manual_seed(0)
    cfg = get_model_config("A", 2048)
    with torch.device("cuda"):
        model = build_model(cfg)
    eng = make_engine(model, engine_config(a.strategy, 4, "reference"), "cuda:0")
    eng.train()
    idx = torch.randint(0, cfg.vocab_size, (1, 2048), device="cuda")

    def step():
        loss = eng(idx, idx)[1]
        eng.backward(loss)
        eng.step()

    for _ in range(8):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    host = (time.perf_counter() - t0) / a.steps
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    print(f"host enqueue {host * 1e3:.3f} ms/step, wall {wall * 1e3:.3f} ms/step")
    # the pure host cost: enqueue 2 steps behind a long GPU sleep, so the queue never makes the
    # host wait (with a shallow backlog "enqueue" above is bounded by the GPU itself)
    for _ in range(3):
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2.4e8))          # ~100 ms of GPU cycles ahead of the steps
        t0 = time.perf_counter()
        for _ in range(2):
            step()
        h2 = (time.perf_counter() - t0) / 2
        torch.cuda.synchronize()
        print(f"host-only cost (GPU busy ahead): {h2 * 1e3:.3f} ms/step")
    # the backward Functions run on autograd's device thread, which cProfile does not see: run the
    # profiled steps with autograd on the calling thread
    torch.autograd.set_multithreading_enabled(False)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    torch.autograd.set_multithreading_enabled(True)
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
