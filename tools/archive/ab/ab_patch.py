#!/usr/bin/env python3
"""A/B a code path in-process: run bench.py with a Python statement applied first.

    python scripts/ab/ab_patch.py "<statement>" [bench.py flags...]

e.g. ``"import dltb.ops.functional as F; F._WGRAD_GAIN = 0.0"``.  Alternate this with an empty
statement ("pass") in one gpurun call to compare two variants on the same box without a toggle in
the framework itself.
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
stmt = sys.argv[1]
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
exec(stmt)  # noqa: S102 -- a developer's own A/B statement
runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
