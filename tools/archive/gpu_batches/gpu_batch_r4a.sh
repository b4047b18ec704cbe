#!/usr/bin/env bash
# Round-4 GPU batch A: graph-branch probe, ProcessGroupNCCL
# host cost, L2 occupancy probe, emulated phases of the N-rank ZeRO-2 path.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python scripts/probes/graph_branch_probe.py > gpurun_out/graph_branch.txt 2>&1 || exit 1
tail -4 gpurun_out/graph_branch.txt
timeout -k 10 120 python scripts/probes/pg_host_cost.py > gpurun_out/pg_host.txt 2>&1 || exit 1
tail -5 gpurun_out/pg_host.txt
timeout -k 10 120 ./scripts/probes/l2_stream_probe > gpurun_out/l2_probe.txt 2>&1 || exit 1
tail -8 gpurun_out/l2_probe.txt
for S in zero2 zero3 fsdp ddp; do echo "== $S"; STRAT=$S N=8 bash scripts/emu_phases.sh || exit 1; done
