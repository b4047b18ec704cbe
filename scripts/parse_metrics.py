#!/usr/bin/env python3
"""CLI wrapper with the reference's path (scripts/parse_metrics.py); implementation: dltb.analysis.parse_metrics."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dltb.analysis.parse_metrics import main  # noqa: E402

if __name__ == "__main__":
    main()
