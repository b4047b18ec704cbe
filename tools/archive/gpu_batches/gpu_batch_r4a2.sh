#!/usr/bin/env bash
# Round-4 GPU batch A2: emulated phases incl. the null-collective row, and the kernel-level profile of the
# sharded engines' N-rank code path (ZeRO-3, FSDP).
set -o pipefail
cd "$(dirname "$0")/.."
for S in zero2 zero3 fsdp; do echo "== $S"; STRAT=$S N=8 bash scripts/emu_phases.sh || exit 1; done
for S in zero3 fsdp; do
  STRAT=$S bash scripts/emu_profile.sh > gpurun_out/emu_profile_$S.txt 2>&1 || exit 1
  mkdir -p gpurun_out/emuprof_$S && cp gpurun_out/prof_w1_eager/summary_steady.txt gpurun_out/emuprof_$S/w1.txt \
    && cp gpurun_out/prof_e8_fast/summary_steady.txt gpurun_out/emuprof_$S/e8.txt
done
