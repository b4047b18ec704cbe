"""End-to-end suite rehearsal on CPU/gloo (BASELINE.json config #1): torchrun launcher -> harness ->
collector -> parse_metrics -> plot -> make_report, including the failure path."""
import json
import os
import subprocess

import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _suite(tmp_path, extra, strats="ddp zero2", m7b="0", **more):
    more.setdefault("TRANSPORT_AB", "0")       # the full sequence runs in test_suite_ddp_zero2_world_1_and_2
    more.setdefault("RCCL_CHECK", "0")
    env = dict(os.environ, STEPS="6", SEQ="64", TIER="tiny", WS_LIST="1 2", STRATS=strats, FORCE_NPROC="2",
               HARNESS_EXTRA=f"--device cpu --warmup-steps 2 --log-every 0 {extra}", TIMEOUT="300",
               OMP_NUM_THREADS="1", M7B=m7b, M7B_TIER="mtiny", M7B_SEQ="64", M7B_STEPS="6", M7B_WS="1 2", **more)
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "run_all_benchmarks.sh"), str(tmp_path)],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return r


def test_suite_ddp_zero2_world_1_and_2(tmp_path):
    """The whole first-multi-GPU sequence, rehearsed on gloo: equivalence check, collective
    sweep, transport A/B on the flagship, the strategy matrix, CSV / plots / report, the multi-GPU summary page."""
    _suite(tmp_path, "", TRANSPORT_AB="1", RCCL_CHECK="1")
    eq = json.load(open(tmp_path / "summary" / "rccl_equivalence.json"))
    assert eq["pass"] and eq["device"] == "cpu" and set(eq["world_sizes"]) == {"2"}
    tab = [json.loads(ln) for ln in open(tmp_path / "summary" / "transport_ab.jsonl")]
    assert [t["transport"] for t in tab] == ["default", "NCCL_MIN_NCHANNELS=16", "NCCL_MIN_NCHANNELS=32",
                                             "DLTB_COMM_HIGH_PRIORITY=0"]
    assert all(t["n_gpus"] == 2 and t["value"] > 0 for t in tab)
    rep = (tmp_path / "summary" / "first_multigpu_report.md").read_text()
    for sec in ("## Measured curve", "## Fabric: alpha-beta fit", "## RCCL transport A/B", "## RCCL equivalence"):
        assert sec in rep, sec
    assert "| zero2 | 2 |" in rep and "reduce_scatter" in rep and "Verdict: **pass**" in rep
    df = pd.read_csv(tmp_path / "summary" / "metrics.csv")
    assert sorted(zip(df.strategy, df.world_size)) == [("ddp", 1), ("ddp", 2), ("zero2", 1), ("zero2", 2)]
    assert (df.loc[df.world_size == 1, "scaling_efficiency_pct"] == 100.0).all()
    assert (tmp_path / "summary" / "BENCHMARK_REPORT.md").exists()
    assert (tmp_path / "summary" / "plots" / "tokens_per_sec_vs_gpu.png").exists()
    assert json.load(open(tmp_path / "summary" / "failures.json")) == {"failed": []}
    ext = pd.read_csv(tmp_path / "summary" / "metrics_extended.csv")
    assert "efficiency_vs_ws1_pct" in ext.columns and ext["efficiency_vs_ws1_pct"].notna().all()
    assert (tmp_path / "bench-master-ddp-ws2-seq64_results" / "result.extended.json").exists()


def test_suite_records_failures_and_still_exits_zero(tmp_path):
    _suite(tmp_path, "--fail-at-step 3", strats="ddp")
    failed = json.load(open(tmp_path / "summary" / "failures.json"))["failed"]
    assert failed == ["bench-master-ddp-ws1-seq64", "bench-master-ddp-ws2-seq64"]


def test_suite_variant_rows_and_measured_bucket_profile(tmp_path, monkeypatch):
    """fsdp_root (the reference's single root FlatParameter) and ddp_uniform rows land in the CSV
    under their own names; the collective sweep writes the bucket profile that sizes the runs."""
    _suite(tmp_path, "", strats="fsdp_root ddp_uniform")
    df = pd.read_csv(tmp_path / "summary" / "metrics.csv")
    assert sorted(zip(df.strategy, df.world_size)) == [("ddp_uniform", 1), ("ddp_uniform", 2),
                                                       ("fsdp_root", 1), ("fsdp_root", 2)]
    prof = json.load(open(tmp_path / "summary" / "xgmi_buckets.json"))
    assert prof["backend"] == "gloo-cpu" and set(prof["worlds"]) == {"2"}
    ops = {r["op"] for r in prof["worlds"]["2"]}
    assert {"reduce_scatter", "all_gather", "all_reduce"} <= ops
    from dltb.comm.topology import measured_params, recommend_bucket_mb
    monkeypatch.setenv("DLTB_XGMI_PROFILE", str(tmp_path / "summary" / "xgmi_buckets.json"))
    assert measured_params(2)[2] == "measured"
    ext = json.load(open(tmp_path / "bench-master-fsdp_root-ws2-seq64_results" / "result.extended.json"))
    assert ext["bucket_mb"] == recommend_bucket_mb(2)
    assert ext["engine_config"]["wrap"] == "root" and ext["strategy_engine"] == "fsdp"
    ext = json.load(open(tmp_path / "bench-master-ddp_uniform-ws2-seq64_results" / "result.extended.json"))
    assert ext["engine_config"]["grad_accum"] == 4 and ext["accum_semantics"] == "uniform"


def test_suite_m7b_rows(tmp_path):
    """Step 2b (BASELINE config #5): the Mistral-shape ZeRO-3 rows with the reference's zero3.json
    and the 288 GB config, rehearsed at the mtiny shape; trainable params + per-rank peak in the
    sidecar."""
    _suite(tmp_path, "", strats="", m7b="1")
    df = pd.read_csv(tmp_path / "summary" / "metrics.csv")
    assert sorted(zip(df.strategy, df.world_size)) == [("zero3_m7b", 1), ("zero3_m7b", 2),
                                                       ("zero3_m7b_288gb", 1), ("zero3_m7b_288gb", 2)]
    assert json.load(open(tmp_path / "summary" / "failures.json")) == {"failed": []}
    ext = json.load(open(tmp_path / "bench-master-zero3_m7b_288gb-ws2-seq64_results" / "result.extended.json"))
    assert ext["trainable_params"] > 0 and ext["peak_vram_reserved_gb"] is not None


def test_suite_multi_seq_matrix(tmp_path):
    """Per-row matrix ("STRATEGY WS SEQ TIER STEPS", the reference's BENCHMARKS format) with several sequence
    lengths and a row of another tier: every row lands in the CSV with its seq_len, and plot.py draws the
    conditional vram_vs_seqlen.png next to the other four plots (reference plot.py:56-71)."""
    rows = "zero2 1 32 tiny 6\nzero2 1 64 tiny 6\nddp 1 32 tiny 6\nddp 1 64 tiny 6\n# comment\nzero3 1 64 mtiny 6\n"
    _suite(tmp_path, "", BENCHMARKS=rows)
    df = pd.read_csv(tmp_path / "summary" / "metrics.csv")
    assert sorted(zip(df.strategy, df.seq_len)) == [("ddp", 32), ("ddp", 64), ("zero2", 32), ("zero2", 64),
                                                    ("zero3", 64)]
    assert json.load(open(tmp_path / "summary" / "failures.json")) == {"failed": []}
    plots = {p.name for p in (tmp_path / "summary" / "plots").iterdir()}
    assert plots == {"tokens_per_sec_vs_gpu.png", "step_time_vs_gpu.png", "vram_vs_seqlen.png",
                     "scaling_efficiency.png", "gbps_vs_gpu.png"}
    assert (tmp_path / "bench-master-zero3-ws1-seq64-tiermtiny_results" / "result.json").exists()


def test_shipped_multiseq_matrix_parses():
    rows = [ln.split("#")[0].split() for ln in open(os.path.join(ROOT, "configs", "suite", "multiseq_1gpu.txt"))]
    rows = [r for r in rows if r]
    assert all(len(r) == 5 for r in rows)
    assert {int(r[2]) for r in rows} == {2048, 4096, 8192}
    assert ["fsdp", "1", "4096", "B", "100"] in rows and ["zero3", "1", "8192", "B", "100"] in rows
