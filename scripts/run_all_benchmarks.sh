#!/usr/bin/env bash
# Full benchmark suite on one 8x MI355X node: every strategy at 1/2/4/8 GPUs (reference:
# scripts/run_all_benchmarks.sh ran {ddp,fsdp,zero2,zero3} x WS{2,4} as K8s jobs).
#  0. RCCL correctness (real GPUs, >= 2 visible): scripts/rccl_equivalence.py trains every engine
#     at the largest and smallest multi-GPU world sizes of WS_LIST over RCCL and against one rank on
#     the concatenated batch -> summary/rccl_equivalence.json (RCCL_CHECK=0 skips it).
#  1. xGMI collective sweep (scripts/bench_collectives.py) at every multi-GPU world size ->
#     summary/xgmi_buckets.json (and profiles/xgmi_buckets.json on real GPUs), which
#     comm/topology.py reads to size the gradient buckets of every following run.
#  1b. RCCL transport A/B on the flagship at the largest world size (NCCL_MIN_NCHANNELS 16 / 32, stream
#      priority) -> summary/transport_ab.jsonl (TRANSPORT_AB=0 skips it).
#  2. Each config: launch (torchrun) -> collect -> failure bookkeeping.  Rows (STRATS):
#       ddp fsdp zero2 zero3      the reference's four strategies, reference semantics and precision
#                                 (DDP / FSDP: fp16 + dynamic loss scaling, DDP fp32 all-reduce;
#                                 ZeRO: bf16 as the DS configs)
#       ddp_bf16 fsdp_bf16        DDP / FSDP in bf16 (bf16 gradient communication)
#       fsdp_root                 FSDP with the reference's effective layout: ONE root FlatParameter
#                                 (configs/fsdp/fsdp_reference_root.yaml)
#       ddp_uniform fsdp_uniform  DDP / FSDP with ZeRO semantics (grad-accum 4, clip 1.0, WarmupLR)
#       zero1                     ZeRO-2 engine with one reduce-scatter per window (opt-in row)
#  2b. BASELINE config #5: Mistral-7B-shape ZeRO-3 (tier M7B, seq 4096) with the reference's
#      zero3.json and with configs/deepspeed/zero3_mi355x_288gb.json (gathered parameters stay
#      resident in 288 GB), rows zero3_m7b / zero3_m7b_288gb at M7B_WS (default "1 8");
#      trainable_params and per-rank peak HBM land in each row's .extended.json sidecar.
#      M7B=0 skips it; M7B_TIER / M7B_SEQ / M7B_STEPS override (the CPU rehearsal uses mtiny).
#  3. parse -> plot -> report.
#  4. summary/first_multigpu_report.md (scripts/first_multigpu_report.py).
# Like the reference it always exits 0; failed configs are listed in results/summary/failures.json.
#
#   ./scripts/run_all_benchmarks.sh [results-dir]
#   env: STEPS, SEQ, SEQ_LIST (several sequence lengths: the vram_vs_seqlen plot), TIER, WS_LIST, STRATS,
#        BENCHMARKS / BENCHMARKS_FILE (explicit "STRATEGY WS SEQ TIER STEPS" rows instead of the
#        STRATS x SEQ_LIST x WS_LIST product, e.g. configs/suite/multiseq_1gpu.txt), TIMEOUT,
#        HARNESS_EXTRA (extra harness flags),
#        M7B, M7B_WS, M7B_TIER, M7B_SEQ, M7B_STEPS (step 2b),
#        FORCE_NPROC (process slots when no GPU is visible, e.g. the gloo/CPU rehearsal),
#        COLLECTIVES=0 (skip step 1), COLL_MAX_MB (largest swept message, default 512)
set -uo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
RESULTS="${1:-$ROOT/results}"
STEPS="${STEPS:-100}"; SEQ="${SEQ:-2048}"; TIER="${TIER:-A}"; TIMEOUT="${TIMEOUT:-900}"
STRATS="${STRATS-ddp fsdp zero2 zero3 fsdp_root ddp_bf16 fsdp_bf16 ddp_uniform fsdp_uniform}"
NGPU="${FORCE_NPROC:-$(python3 -c "import torch; print(torch.cuda.device_count())" 2>/dev/null || echo 0)}"
read -r -a HX <<< "${HARNESS_EXTRA:-}"
WS_LIST="${WS_LIST:-1 2 4 8}"
mkdir -p "$RESULTS/raw" "$RESULTS/summary"
FAILED=(); DONE=0
export HSA_ENABLE_IPC_MODE_LEGACY="${HSA_ENABLE_IPC_MODE_LEGACY:-0}"
echo "=================================================================="
echo "  MI355X Distributed Training Benchmark Suite ($NGPU GPUs visible)"
echo "=================================================================="

# ---- 0. RCCL correctness: every engine at N ranks == 1 rank on the concatenated batch
#      (FORCE_NPROC rehearsal: gloo on the CPU, two cases at a short sequence)
if [[ "${RCCL_CHECK:-1}" != "0" && "$NGPU" -ge 2 ]]; then
  RWS=(); for ws in $WS_LIST; do [[ "$ws" -ge 2 && "$ws" -le "$NGPU" ]] && RWS+=("$ws"); done
  if [[ ${#RWS[@]} -gt 0 ]]; then
    CHK=("${RWS[0]}"); [[ ${#RWS[@]} -gt 1 ]] && CHK+=("${RWS[-1]}")
    RX=(); [[ -n "${FORCE_NPROC:-}" ]] && RX=(--device cpu --cases ddp,zero2 --seq-len 64)
    echo "---- RCCL equivalence ws=${CHK[*]}"
    timeout -k 30 "$((3 * TIMEOUT))" python3 "$ROOT/scripts/rccl_equivalence.py" --ws "${CHK[@]}" \
      ${RX[@]+"${RX[@]}"} --out "$RESULTS/summary/rccl_equivalence.json" > "$RESULTS/rccl_equivalence.log" 2>&1 \
      || { FAILED+=("rccl-equivalence"); echo "     FAILED (see $RESULTS/rccl_equivalence.log)"; }
  fi
fi

# ---- 1. collective sweep -> bucket sizing profile
PROFILE="$RESULTS/summary/xgmi_buckets.json"
if [[ "${COLLECTIVES:-1}" != "0" ]]; then
  if [[ -n "${FORCE_NPROC:-}" ]]; then CARGS=(--backend gloo --device cpu --max-mb "${COLL_MAX_MB:-4}" --iters 3 --warmup 1)
  else CARGS=(--max-mb "${COLL_MAX_MB:-512}"); fi
  for ws in $WS_LIST; do
    [[ "$ws" -lt 2 || "$ws" -gt "$NGPU" ]] && continue
    echo "---- collectives ws=$ws"
    timeout -k 30 "$TIMEOUT" python -m torch.distributed.run --nnodes 1 --nproc-per-node "$ws" --max-restarts 0 \
      --master-addr 127.0.0.1 --master-port "$((29500 + RANDOM % 1000))" "$ROOT/scripts/bench_collectives.py" \
      --ops reduce_scatter,all_gather,all_reduce "${CARGS[@]}" --json "$RESULTS/summary/collectives_ws$ws.json" \
      > "$RESULTS/collectives_ws$ws.log" 2>&1 || { FAILED+=("collectives-ws$ws"); echo "     FAILED"; }
  done
  python3 - "$PROFILE" "$RESULTS/summary" "${FORCE_NPROC:-}" "$ROOT/profiles/xgmi_buckets.json" <<'PY'
import glob, json, os, re, shutil, sys
out, d, forced, repo_copy = sys.argv[1:5]
worlds = {}
for p in sorted(glob.glob(os.path.join(d, "collectives_ws*.json"))):
    worlds[re.search(r"ws(\d+)", p).group(1)] = json.load(open(p))
if worlds:
    json.dump({"source": "scripts/bench_collectives.py via run_all_benchmarks.sh",
               "backend": "gloo-cpu" if forced else "rccl", "worlds": worlds}, open(out, "w"), indent=1)
    if not forced:                      # real GPUs: this node's measurement becomes the default
        shutil.copyfile(out, repo_copy)
PY
  [[ -f "$PROFILE" ]] && export DLTB_XGMI_PROFILE="$PROFILE"
fi

# ---- 1b. RCCL transport knobs on the flagship (ZeRO-2, bench.py) at the largest multi-GPU world size:
#      default, NCCL_MIN_NCHANNELS=16 / 32, the RCCL stream at normal priority -> summary/transport_ab.jsonl
#      (one bench.py JSON line per variant, with a "transport" field; TRANSPORT_AB=0 skips it)
if [[ "${TRANSPORT_AB:-1}" != "0" ]]; then
  TWS=0; for ws in $WS_LIST; do [[ "$ws" -ge 2 && "$ws" -le "$NGPU" && "$ws" -gt "$TWS" ]] && TWS=$ws; done
  if [[ "$TWS" -ge 2 ]]; then
    if [[ -n "${FORCE_NPROC:-}" ]]; then BX=(--device cpu --tier "$TIER" --seq-len "$SEQ" --steps 6 --warmup 5)
    else BX=(--steps "${TRANSPORT_STEPS:-20}" --warmup 5); fi
    : > "$RESULTS/summary/transport_ab.jsonl"
    for knob in default NCCL_MIN_NCHANNELS=16 NCCL_MIN_NCHANNELS=32 DLTB_COMM_HIGH_PRIORITY=0; do
      echo "---- transport ws=$TWS $knob"
      KV=(); [[ "$knob" != default ]] && KV=("$knob")
      tlog="$RESULTS/transport_${knob//=/_}.log"
      if timeout -k 30 "$TIMEOUT" env ${KV[@]+"${KV[@]}"} python3 "$ROOT/bench.py" --gpus "$TWS" --strategy zero2 \
           "${BX[@]}" > "$tlog" 2>&1; then
        python3 - "$tlog" "$knob" "$RESULTS/summary/transport_ab.jsonl" <<'PY' || FAILED+=("transport-$knob")
import json, sys
log, knob, out = sys.argv[1:4]
rec = [json.loads(l) for l in open(log) if l.startswith("{")][-1]
rec["transport"] = knob
open(out, "a").write(json.dumps(rec) + "\n")
PY
      else
        FAILED+=("transport-$knob"); echo "     FAILED (see $tlog)"
      fi
    done
  fi
fi

# ---- 2. benchmark matrix
variant() {   # row name -> "engine strategy|extra harness flags"
  case "$1" in
    ddp|fsdp|zero2|zero3) echo "$1|" ;;
    fsdp_root) echo "fsdp|--fsdp-config $ROOT/configs/fsdp/fsdp_reference_root.yaml --strategy-label fsdp_root" ;;
    ddp_uniform|fsdp_uniform) echo "${1%_uniform}|--accum-semantics uniform --strategy-label $1" ;;
    ddp_bf16|fsdp_bf16) echo "${1%_bf16}|--dtype bf16 --strategy-label $1" ;;
    zero1) echo "zero2|--grad-reduce window --strategy-label zero1" ;;
    *) echo "" ;;
  esac
}
# rows "STRATEGY WS SEQ TIER STEPS" (the reference's BENCHMARKS matrix, run_all_benchmarks.sh:32-52): from
# BENCHMARKS_FILE / BENCHMARKS (one row per line, '#' comments) when given, else STRATS x SEQ_LIST x WS_LIST
ROWS=()
if [[ -n "${BENCHMARKS_FILE:-}" ]]; then BENCHMARKS="$(cat "$BENCHMARKS_FILE")"; fi
if [[ -n "${BENCHMARKS:-}" ]]; then
  while IFS= read -r line; do
    line="${line%%#*}"; read -r -a f <<< "$line"
    [[ ${#f[@]} -eq 0 ]] && continue
    [[ ${#f[@]} -ne 5 ]] && { echo "bad matrix row: $line"; FAILED+=("matrix-row"); continue; }
    ROWS+=("${f[*]}")
  done <<< "$BENCHMARKS"
else
  for s in $STRATS; do for seq in ${SEQ_LIST:-$SEQ}; do for ws in $WS_LIST; do
    ROWS+=("$s $ws $seq $TIER $STEPS")
  done; done; done
fi
for row in "${ROWS[@]}"; do
  read -r s ws seq tier steps <<< "$row"
  spec="$(variant "$s")"
  if [[ -z "$spec" ]]; then echo "unknown row $s"; FAILED+=("$s"); continue; fi
  eng="${spec%%|*}"; read -r -a VX <<< "${spec#*|}"
  if [[ "$ws" -gt "$NGPU" ]]; then echo "skip $s ws=$ws (only $NGPU GPUs)"; continue; fi
  job="bench-master-${s}-ws${ws}-seq${seq}"
  [[ "$tier" != "$TIER" ]] && job="${job}-tier${tier}"
  echo "---- $job"
  if timeout -k 30 "$TIMEOUT" "$ROOT/scripts/launch_local.sh" --strategy "$eng" --world-size "$ws" --seq-len "$seq" \
       --tier "$tier" --steps "$steps" --per-device-batch 1 --grad-accum 4 --results-dir "$RESULTS/raw" \
       -- "${VX[@]}" "${HX[@]}" > "$RESULTS/$job.log" 2>&1 \
     && "$ROOT/scripts/collect_results.sh" "$RESULTS/$job.log" "$RESULTS" "$job" "$RESULTS/raw"; then
    DONE=$((DONE + 1)); echo "     ok"
  else
    FAILED+=("$job"); echo "     FAILED (see $RESULTS/$job.log)"; tail -20 "$RESULTS/$job.log" || true
  fi
done
# ---- 2b. BASELINE config #5: Mistral-7B-shape ZeRO-3 at 1 and 8 GPUs
if [[ "${M7B:-1}" != "0" ]]; then
  M7B_TIER="${M7B_TIER:-M7B}"; M7B_SEQ="${M7B_SEQ:-4096}"; M7B_STEPS="${M7B_STEPS:-20}"
  for row in zero3_m7b zero3_m7b_288gb; do
    cfg="$ROOT/configs/deepspeed/zero3.json"
    [[ "$row" == zero3_m7b_288gb ]] && cfg="$ROOT/configs/deepspeed/zero3_mi355x_288gb.json"
    for ws in ${M7B_WS:-1 8}; do
      if [[ "$ws" -gt "$NGPU" ]]; then echo "skip $row ws=$ws (only $NGPU GPUs)"; continue; fi
      job="bench-master-${row}-ws${ws}-seq${M7B_SEQ}"
      echo "---- $job"
      if timeout -k 30 "$((2 * TIMEOUT))" "$ROOT/scripts/launch_local.sh" --strategy zero3 --world-size "$ws" \
           --seq-len "$M7B_SEQ" --tier "$M7B_TIER" --steps "$M7B_STEPS" --per-device-batch 1 --grad-accum 4 \
           --results-dir "$RESULTS/raw" -- --deepspeed-config "$cfg" --strategy-label "$row" "${HX[@]}" \
           > "$RESULTS/$job.log" 2>&1 \
         && "$ROOT/scripts/collect_results.sh" "$RESULTS/$job.log" "$RESULTS" "$job" "$RESULTS/raw"; then
        DONE=$((DONE + 1)); echo "     ok"
      else
        FAILED+=("$job"); echo "     FAILED (see $RESULTS/$job.log)"; tail -20 "$RESULTS/$job.log" || true
      fi
    done
  done
fi
python3 - "$RESULTS/summary/failures.json" "${FAILED[@]}" <<'PY'
import json, sys
json.dump({"failed": sys.argv[2:]}, open(sys.argv[1], "w"), indent=2)
PY
python3 "$ROOT/scripts/parse_metrics.py" --results-dir "$RESULTS" --out "$RESULTS/summary" \
  && python3 "$ROOT/scripts/plot.py" --results "$RESULTS/summary/metrics.csv" --out "$RESULTS/summary/plots" \
  && python3 "$ROOT/scripts/make_report.py" --csv "$RESULTS/summary/metrics.csv" --out "$RESULTS/summary"
# ---- 4. the multi-GPU summary: measured curve, error of the shipped emulated-fabric prediction per row, the
#      fitted alpha-beta per world size and collective, the transport A/B, the RCCL equivalence verdict
python3 "$ROOT/scripts/first_multigpu_report.py" --results "$RESULTS" \
  --out "$RESULTS/summary/first_multigpu_report.md" || echo "first_multigpu_report failed"
echo "completed: $DONE, failed: ${#FAILED[@]}"
exit 0
