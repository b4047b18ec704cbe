"""Per-phase timers (utils/timers.py, harness ``--phase-timers``) on the CPU.

* the interval bookkeeping charges each span to the phase its opening mark names;
* the harness reports forward / backward / comm_wait / optimizer times in the extended record, at
  world size 1 (in process) and 2 (torchrun + gloo, where the ZeRO-2 reduce-scatter wait appears).
"""
import glob
import json
import os
import socket
import subprocess
import sys
import time

import pytest

import dltb  # noqa: F401
from dltb.harness import main as harness_main
from dltb.utils.timers import PHASES, PhaseTimers

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_marks_are_charged_to_phases():
    t = PhaseTimers("cpu")
    t.mark("fwd_end")                       # outside a step: ignored
    for _ in range(2):
        t.begin_step()
        time.sleep(0.002)
        t.mark("opt_begin")
        time.sleep(0.004)
        t.mark("opt_end")
        time.sleep(0.002)
        t.mark("fwd_end")
        time.sleep(0.003)
        t.mark("comm_wait_begin")
        time.sleep(0.002)
        t.mark("comm_wait_end")
        t.mark("bwd_end")
        t.end_step()
    s = t.summary()
    assert set(s) == set(PHASES)
    assert s["optimizer"] >= 3.5 and s["forward"] >= 3.5 and s["backward"] >= 2.5 and s["comm_wait"] >= 1.5
    assert s["optimizer"] < 40 and s["forward"] < 40


def _extended(results_dir):
    paths = glob.glob(os.path.join(str(results_dir), "**", "*.extended.json"), recursive=True)
    assert paths, os.listdir(results_dir)
    return json.load(open(paths[0]))


def _args(strategy, out):
    return ["--strategy", strategy, "--tier", "tiny", "--seq-len", "32", "--steps", "6", "--warmup-steps", "2",
            "--per-device-batch", "1", "--grad-accum", "2", "--results-dir", str(out), "--device", "cpu",
            "--log-every", "0", "--phase-timers", "--accum-semantics", "uniform"]


def test_harness_phase_times_world1(tmp_path):
    assert harness_main(_args("zero2", tmp_path)) == 0
    ph = _extended(tmp_path)["phase_times_ms"]
    assert set(ph) == set(PHASES)
    assert ph["forward"] > 0 and ph["backward"] > 0 and ph["optimizer"] > 0


@pytest.mark.parametrize("strategy", ["zero2", "zero3"])
def test_harness_phase_times_world2(tmp_path, strategy):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--max-restarts=0",
           "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "dltb.harness", *_args(strategy, tmp_path)]
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    ph = _extended(tmp_path)["phase_times_ms"]
    assert ph["forward"] > 0 and ph["backward"] > 0 and ph["comm_wait"] >= 0
