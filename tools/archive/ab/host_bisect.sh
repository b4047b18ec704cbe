cd /root/repo 2>/dev/null || true
run() { local name=$1; shift; timeout -k 10 200 python bench.py --steps 12 --warmup 8 --host-check "$@" > gpurun_out/bisect_$name.log 2>&1 || { echo "$name FAILED"; tail -3 gpurun_out/bisect_$name.log; return 0; }
  tail -n 1 gpurun_out/bisect_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', 'gpu', round(d['ms_per_step'],2), 'host', round(d['host_enqueue_ms_per_step'],2), d.get('host_check_note'))"; }
run narrow_z3_w1 --strategy zero3 --tier M7B_narrow --seq-len 4096
run narrow_z3_e8_s2k --strategy zero3 --tier M7B_narrow --seq-len 2048 --emulate 8
run narrow_z2_e8 --strategy zero2 --tier M7B_narrow --seq-len 4096 --emulate 8
run mtiny_z3_e8 --strategy zero3 --tier mtiny --seq-len 4096 --emulate 8
run a_z3_e8 --strategy zero3 --tier A --seq-len 2048 --emulate 8
