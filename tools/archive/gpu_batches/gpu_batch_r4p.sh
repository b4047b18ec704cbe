#!/bin/bash
# Round 4 batch P: phase breakdown of the predicted N = 8 ZeRO-2 step on the final round-4 tree.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
STRAT=zero2 N=8 bash scripts/emu_phases.sh
