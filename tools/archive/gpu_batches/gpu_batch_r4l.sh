#!/bin/bash
# Round 4 batch L: where the predicted N = 2 ZeRO-2 micro-step goes (one xGMI link between the two GPUs).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
STRAT=zero2 N=2 bash scripts/emu_phases.sh
