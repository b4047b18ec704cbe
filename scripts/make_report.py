#!/usr/bin/env python3
"""CLI wrapper with the reference's path (scripts/make_report.py); implementation: dltb.analysis.make_report."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dltb.analysis.make_report import main  # noqa: E402

if __name__ == "__main__":
    main()
