#!/usr/bin/env bash
# Analysis-only dependencies (parse_metrics / plot / make_report) for a workstation without the image.
set -euo pipefail
python3 -m pip install --user pandas matplotlib numpy pyyaml
