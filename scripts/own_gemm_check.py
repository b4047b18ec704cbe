#!/usr/bin/env python3
"""Does the own-GEMM table path run in a real step, and does it change the numbers?

    DLTB_OWN_GEMM_TABLE=<csv> python scripts/own_gemm_check.py

Two-block TinyGPT-A at seq 2048 (the bench's per-layer shapes), one forward + backward through the ZeRO-2
engine with the table on, then again with it off (same weights, same tokens): prints the number of products
issued through gemm_rs and the loss difference (the kernels' own numerics: tests/test_gemm_rs_gpu.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import dltb  # noqa: E402,F401
import dltb.ops.functional as F  # noqa: E402
from dltb.models import build_model, get_model_config  # noqa: E402
from dltb.parallel import engine_config, make_engine  # noqa: E402

torch.manual_seed(0)
cfg = get_model_config("A", 2048)
cfg.n_layer = 2
model = build_model(cfg)
eng = make_engine(model, engine_config("zero2", 1, "reference"), "cuda:0")
idx = torch.randint(0, cfg.vocab_size, (1, 2048), device="cuda:0")
tgt = torch.randint(0, cfg.vocab_size, (1, 2048), device="cuda:0")
out = {}
for mode in ("on", "off"):
    F._rs_table = None if mode == "on" else {}
    c0 = F.own_gemm_calls
    loss = eng(idx, tgt)[1]
    eng.backward(loss)
    torch.cuda.synchronize()
    out[mode] = (float(loss.item()), F.own_gemm_calls - c0)
(l1, n1), (l0, n0) = out["on"], out["off"]
print(f"own-GEMM products issued: on {n1}, off {n0}; loss on {l1:.6f} off {l0:.6f} diff {abs(l1 - l0):.2e}")
