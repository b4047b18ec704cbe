"""bench.py launcher contract on CPU / gloo (the GPU path runs the same code with RCCL).

* ``python bench.py --gpus 2`` without a torchrun environment starts the ranks itself as a child
  ``torch.distributed.run`` (reference: scripts/launch_multi.sh:38-82 starts one pod per rank),
  and exactly one JSON line comes back with n_gpus == world_size_seen == 2.
* A failing rank makes the launcher exit non-zero.
* Exactly ``--warmup`` untimed steps and ``--steps`` timed steps: the record says so.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--tier", "tiny",
        "--seq-len", "64", "--steps", "8", "--warmup", "5"]


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_bench_self_launch_two_ranks():
    r = subprocess.run(BASE + ["--gpus", "2"], capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = _json_lines(r.stdout)
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == rec["world_size_seen"] == 2
    assert rec["backend"] == "gloo"
    assert rec["steps"] == 8 and rec["warmup"] == 5 == rec["warmup_used"] == rec["warmup_requested"]
    assert rec["config"]["parallelism"] == "zero2-dp2" and rec["config"]["grad_reduce"] == "micro"
    assert rec["optimizer_steps_timed"] == 2          # any 8 consecutive micro-steps hold 2 boundaries
    # ZeRO-2: a reduce-scatter every micro-step + the window's all-gather, measured == modelled
    assert rec["wire_bytes_per_step"] > 0
    assert abs(rec["wire_bytes_per_step"] - rec["wire_bytes_per_step_model"]) / rec["wire_bytes_per_step_model"] < 0.01
    assert rec["comm_wait_ms"] is not None and rec["mean_loss"] > 0
    # the job calibrated its own collectives before planning buckets (gloo here, RCCL on GPUs)
    cal = rec["fabric_calibration"]
    assert {r["op"] for r in cal["rows"]} == {"reduce_scatter", "all_reduce", "all_gather"}
    assert all(r["time_us"] > 0 and r["bytes"] > 0 for r in cal["rows"])
    assert cal["bucket_mb_from"] == "calibrated" and rec["config"]["bucket_mb"] >= 1
    # a real N > 1 line explains itself (VERDICT r4 Next #6): per-op alpha-beta fits of this job's
    # fabric, the communication environment, the measured phase split and the shipped prediction
    assert set(cal["fits"]) == {"reduce_scatter", "all_reduce", "all_gather"}
    assert all(f["alpha_us"] >= 0 and f["bus_GBps"] > 0 for f in cal["fits"].values())
    env = rec["comm_env"]
    assert set(env) == {"rccl_version", "hip_version", "knobs"} and isinstance(env["knobs"], dict)
    assert "HSA_ENABLE_IPC_MODE_LEGACY" in env["knobs"]
    assert set(rec["phase_ms"]) >= {"forward", "backward", "comm_wait", "optimizer"}
    assert "predicted" in rec and "prediction_error" in rec   # None here: no fp32 / tiny row is shipped


def test_bench_window_is_labelled_zero1():
    r = subprocess.run(BASE + ["--gpus", "2", "--grad-reduce", "window", "--steps", "4", "--warmup", "1"],
                       capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["config"]["parallelism"] == "zero1-dp2"
    assert rec["same_strategy_published"] is None


def test_bench_failing_rank_fails_the_launch():
    r = subprocess.run(BASE + ["--gpus", "2", "--fail-rank", "1"], capture_output=True, text=True,
                       env=_env(), timeout=600)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)


def test_bench_single_process_cpu():
    r = subprocess.run(BASE + ["--gpus", "1", "--strategy", "ddp"], capture_output=True, text=True,
                       env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["n_gpus"] == rec["world_size_seen"] == 1 and rec["wire_bytes_per_step"] == 0


def test_bench_prediction_lookup():
    """The shipped emulated-fabric table row for a configuration (what a real N-GPU line is compared to)."""
    sys.path.insert(0, ROOT)
    import bench
    row = bench.predicted_row("zero2-dp8", "bf16", 8)
    assert row is not None and row["ms_per_step"] > 0 and row["table"].startswith("profiles/emulated_scaling")
    assert bench.predicted_row("zero2-dp8", "fp32", 8) is None


def test_own_gemm_table_parsing(tmp_path, monkeypatch):
    """ops/functional.py reads the own-GEMM table (comments skipped) and DLTB_OWN_GEMM=0 turns it off."""
    import dltb.ops.functional as F
    t = tmp_path / "t.csv"
    t.write_text("# note\nm,n,k,bias,cfg,gm\n2048,1024,1024,1,34,1\n2048,1024,4096,0,34,4\n")
    monkeypatch.setenv("DLTB_OWN_GEMM_TABLE", str(t))
    F._rs_table = None
    assert F.rs_table() == {(2048, 1024, 1024, 1): (34, 1), (2048, 1024, 4096, 0): (34, 4)}
    monkeypatch.setenv("DLTB_OWN_GEMM", "0")
    F._rs_table = None
    assert F.rs_table() == {}
    monkeypatch.delenv("DLTB_OWN_GEMM")
    monkeypatch.delenv("DLTB_OWN_GEMM_TABLE")
    F._rs_table = None
    shipped = F.rs_table()
    assert shipped and all(0 <= v[0] <= 14 for v in shipped.values())   # production configs (15+: ablations)
    F._rs_table = None


def test_table_paths_resolve_from_any_cwd(tmp_path, monkeypatch):
    """A relative DLTB_BLASLT_FILE / DLTB_OWN_GEMM_TABLE resolves against the repository root when the
    working directory does not hold it (rocprofv3 runs bench.py from /tmp); a missing table is an error,
    not a silent run without it."""
    import pytest
    from dltb.ops.blaslt import _ROOT, resolve_config_path
    monkeypatch.chdir(tmp_path)
    rel = os.path.join("configs", "blaslt", "blaslt_gfx950.csv")
    assert resolve_config_path(rel, "t") == os.path.join(_ROOT, rel)
    assert resolve_config_path("none", "t") == "none"
    with pytest.raises(FileNotFoundError):
        resolve_config_path("configs/blaslt/no_such_table.csv", "t")
    with pytest.raises(FileNotFoundError):
        resolve_config_path(str(tmp_path / "missing.csv"), "t")


def test_prediction_lookup_reads_the_newest_table():
    """every shipped (parallelism, dtype, N) row resolves from the NEWEST prediction table, so
    the first real multi-GPU run compares against the current prediction, not an older round's."""
    sys.path.insert(0, ROOT)
    import bench
    tables = bench.prediction_tables()
    assert tables, "no shipped prediction table"
    newest = tables[0]
    rows = [json.loads(ln) for ln in open(os.path.join(ROOT, newest)) if ln.strip()]
    rows = [r for r in rows if r.get("prediction")]
    assert rows
    key = lambda r: (r["config"]["parallelism"], r["dtype"], r["emulated_world"], r["config"]["seq_len"],
                     r["config"]["model"])
    counts = {}
    for r in rows:
        counts[key(r)] = counts.get(key(r), 0) + 1
    for r in rows:
        got = bench.predicted_row(*key(r))
        assert got is not None and got["table"] == newest, (r["config"]["parallelism"], got)
        if counts[key(r)] == 1:        # (the M7B rows differ only in their DeepSpeed config file)
            assert got["ms_per_step"] == r["ms_per_step"]
    # a round's "_final" table sorts before the same round's earlier one
    names = [os.path.basename(t) for t in tables]
    for i, n in enumerate(names):
        if n.endswith("_final.jsonl"):
            base = n.replace("_final", "")
            assert base not in names[:i], (base, n)


def test_first_multigpu_report_grades_the_prediction(tmp_path):
    """scripts/first_multigpu_report.py: a Tier A multi-GPU row is compared with the newest shipped prediction of
    the same (strategy, dtype, N, seq); rows of other shapes are not graded."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    sys.path.insert(0, ROOT)
    import bench
    import first_multigpu_report as fmr
    pred = bench.predicted_row("zero2-dp8", "bf16", 8, 2048)
    assert pred is not None and pred["seq_len"] == 2048
    assert bench.predicted_row("zero2-dp8", "bf16", 8, 64) is None
    summ = tmp_path / "summary"
    summ.mkdir()
    hdr = ("strategy,world_size,rank,seq_len,tier,steps,per_device_batch,grad_accum,tokens_per_sec,"
           "mean_step_time_sec,mean_loss,peak_vram_gb,h2d_gbps_per_gpu,scaling_efficiency_pct\n")
    meas = pred["value"] * 0.9
    (summ / "metrics.csv").write_text(hdr + "zero2,1,0,2048,A,100,1,4,280000,0.0073,5.0,9.5,1e-3,100.0\n"
                                      f"zero2,8,0,2048,A,100,1,4,{meas},0.0080,5.0,3.9,1e-3,80.0\n"
                                      "zero2,2,0,64,tiny,100,1,4,5000,0.02,5.0,0.1,1e-3,50.0\n")
    out = fmr.write_report(str(tmp_path), str(summ / "first_multigpu_report.md"))
    rep = open(out).read()
    assert "-10.0 %" in rep and "| zero2 | 2 | 64 | tiny |" in rep
    assert "Prediction error over 1 rows" in rep
