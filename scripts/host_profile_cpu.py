#!/usr/bin/env python3
"""Host-side (Python) cost of the engines' N-rank code paths, measured on the CPU.

    python scripts/host_profile_cpu.py [--strategy fsdp] [--emulate 8] [--steps 16] [--top 25]

A 16-layer TinyGPT of width 64 (the unit / bucket / group structure of Tier A, negligible CPU
arithmetic) runs under ``DLTB_COMM=emulate:N`` on the CPU, so every per-unit engine action of
an N-rank job (gathers, releases, reduce-scatters, bucket bookkeeping, weight-gradient queueing)
executes with the real layouts while the ops themselves cost almost nothing.  cProfile over K
micro-steps then ranks the engine / model / comm functions by own time: the part of an eager
multi-rank step's host time that is framework Python rather than kernel launches.
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--strategy", default="fsdp")
    ap.add_argument("--emulate", type=int, default=8)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    if a.emulate > 1:
        os.environ["DLTB_COMM"] = f"emulate:{a.emulate}"
    import torch
    import dltb  # noqa: F401
    from dltb.models import build_model
    from dltb.models.config import ModelConfig
    from dltb.parallel import engine_config, make_engine

    torch.manual_seed(0)
    cfg = ModelConfig(vocab_size=128, n_embd=64, n_head=4, n_layer=16, block_size=64, dropout=0.1, tier="tiny16")
    model = build_model(cfg)
    ecfg = engine_config(a.strategy, 4, "reference")
    ecfg.compute_dtype = torch.float32
    eng = make_engine(model, ecfg, "cpu")
    eng.train()
    idx = torch.randint(0, cfg.vocab_size, (1, 64))

    def step():
        loss = eng(idx, idx)[1]
        eng.backward(loss)
        eng.step()

    for _ in range(8):
        step()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    per = (time.perf_counter() - t0) / a.steps
    print(f"{a.strategy} emulate:{a.emulate}: {per * 1e3:.3f} ms per micro-step on the CPU (width 64: mostly Python)")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s).sort_stats("tottime")
    st.print_stats("dltb|distributed-llm|parallel|comm|models|ops", a.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
