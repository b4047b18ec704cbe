#!/usr/bin/env python3
"""Entry point with the reference's path and CLI (benchmarking/train_harness.py).

    python benchmarking/train_harness.py --strategy zero2 --world-size 1 --rank 0 --tier A \
        --seq-len 2048 --steps 100 --per-device-batch 1 --grad-accum 4 --results-dir results
    torchrun --standalone --nproc-per-node 8 benchmarking/train_harness.py --strategy ddp ...

All logic lives in dltb.harness (MI355X-native engines and HIP kernels).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dltb.harness import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
