#!/usr/bin/env bash
# Offline self-check (replaces the reference's docker --network none verifier, which masked every
# error with `|| true`): imports, extension build, TinyGPT tiers instantiate with the expected
# parameter counts, synthetic data shape, configs present.  Fails loudly on the first problem.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT"
python3 - <<'PY'
import json, os
import torch, yaml, pandas, matplotlib, numpy  # noqa: F401
import dltb
from dltb.models import get_model_config, build_model
from dltb.data import SyntheticDataset
from dltb.ops._ext import available
assert get_model_config("A", 2048).num_params() == 236_406_784
assert get_model_config("B", 2048).num_params() == 1_681_199_104
m = build_model(get_model_config("tiny", 64))
ds = SyntheticDataset(32000, 2048, 8, 42)
assert tuple(ds.data.shape) == (8, 2048)
for p in ("configs/deepspeed/zero2.json", "configs/deepspeed/zero3.json", "configs/fsdp/fsdp_config.yaml"):
    assert os.path.exists(p), p
json.load(open("configs/deepspeed/zero2.json")); yaml.safe_load(open("configs/fsdp/fsdp_config.yaml"))
print("imports / models / data / configs: PASSED; HIP extension:", "built" if available() else "NOT BUILT")
PY
