"""Golden tests of the analysis pipeline against the reference's published table
(README.md:214-223, results/example_output/README.md:7-22,87-90), SURVEY.md §4 item 4."""
import json
import os

import pandas as pd
import pytest

import dltb
from dltb.analysis import generate_report, parse_results, plot_metrics
from dltb.results import RESULT_KEYS, extract_from_log, make_record, print_markers

# strategy, ws, tokens/s, step s, peak GB, mean loss, h2d  (DDP rows at full precision from the example
# output, the others as rounded in the README table)
PUBLISHED = [
    ("ddp", 2, 8369.455699192402, 0.4893986117156026, 13.96808448, 6.133937082792583, 1.6738911398384803e-05),
    ("ddp", 4, 12220.341463838564, 0.6703577002525746, 13.96808448, 5.424101734161377, 1.2220341463838563e-05),
    ("fsdp", 2, 6771.0, 0.605, 12.54, 6.1, 1.35e-05),
    ("fsdp", 4, 9424.0, 0.869, 11.84, 5.4, 0.94e-05),
    ("zero2", 2, 10999.0, 0.372, 11.30, 6.1, 2.20e-05),
    ("zero2", 4, 18147.0, 0.451, 10.47, 5.4, 1.81e-05),
    ("zero3", 2, 10560.0, 0.388, 10.62, 6.1, 2.11e-05),
    ("zero3", 4, 15977.0, 0.513, 9.67, 5.4, 1.60e-05),
]
# README rounding: 36.5 / 34.8 / 41.2 / 37.8 (the DDP value is the example output's full precision)
EXPECTED_EFF = {("ddp", 2): 50.0, ("ddp", 4): 36.50279630794195, ("fsdp", 4): 9424 / (6771 * 4) * 100,
                ("zero2", 4): 18147 / (10999 * 4) * 100, ("zero3", 4): 15977 / (10560 * 4) * 100}
CSV_HEADER = ("strategy,world_size,rank,seq_len,tier,steps,per_device_batch,grad_accum,tokens_per_sec,"
              "mean_step_time_sec,mean_loss,peak_vram_gb,h2d_gbps_per_gpu,scaling_efficiency_pct")


def _write_published(root):
    for s, ws, tps, st, vram, loss, h2d in PUBLISHED:
        rec = dict(zip(RESULT_KEYS, (s, ws, 0, 2048, "A", 100, 1, 4, tps, st, loss, vram, h2d)))
        d = root / f"bench-master-{s}-ws{ws}-seq2048_results"
        d.mkdir(parents=True)
        (d / "result.json").write_text(json.dumps(rec, indent=2))
    # decoys the reference glob must ignore
    (root / "result_ddp_ws2_seq2048_tierA.json").write_text("{}")


def test_parse_metrics_reproduces_published_csv(tmp_path):
    _write_published(tmp_path / "results")
    df = parse_results(str(tmp_path / "results"), str(tmp_path / "summary"))
    text = (tmp_path / "summary" / "metrics.csv").read_text().splitlines()
    assert text[0] == CSV_HEADER
    assert len(text) == 9
    assert list(df["strategy"]) == ["ddp", "ddp", "fsdp", "fsdp", "zero2", "zero2", "zero3", "zero3"]
    for (s, ws), want in EXPECTED_EFF.items():
        got = df[(df.strategy == s) & (df.world_size == ws)]["scaling_efficiency_pct"].iloc[0]
        assert got == pytest.approx(want, rel=1e-12), (s, ws)
    # the example output's second CSV line, byte for byte
    assert text[2] == ("ddp,4,0,2048,A,100,1,4,12220.341463838564,0.6703577002525746,5.424101734161377,"
                       "13.96808448,1.2220341463838563e-05,36.50279630794195")
    ext = pd.read_csv(tmp_path / "summary" / "metrics_extended.csv")
    z2 = ext[(ext.strategy == "zero2") & (ext.world_size == 4)].iloc[0]
    assert z2["efficiency_vs_min_ws_pct"] == pytest.approx(18147 / (10999 * 2) * 100)
    assert pd.isna(z2["efficiency_vs_ws1_pct"])   # no WS=1 row was published


def test_single_row_group_keeps_100(tmp_path):
    root = tmp_path / "r" / "x_results"
    root.mkdir(parents=True)
    rec = dict(zip(RESULT_KEYS, ("ddp", 1, 0, 2048, "A", 10, 1, 4, 1000.0, 2.0, 5.0, 1.0, 1e-5)))
    (root / "result.json").write_text(json.dumps(rec))
    df = parse_results(str(tmp_path / "r"), str(tmp_path / "s"))
    assert df["scaling_efficiency_pct"].iloc[0] == 100.0


def test_plots_and_report(tmp_path):
    _write_published(tmp_path / "results")
    parse_results(str(tmp_path / "results"), str(tmp_path / "summary"))
    csv = tmp_path / "summary" / "metrics.csv"
    files = plot_metrics(str(csv), str(tmp_path / "summary" / "plots"))
    names = sorted(os.path.basename(f) for f in files)
    assert names == ["gbps_vs_gpu.png", "scaling_efficiency.png", "step_time_vs_gpu.png", "tokens_per_sec_vs_gpu.png"]
    rep = generate_report(str(csv), str(tmp_path / "summary")).read_text()
    for section in ("## Summary", "## Strategy Comparison", "### ZERO2", "## Key Findings", "## Corrected Scaling",
                    "## Strategy Trade-offs", "## Visualizations"):
        assert section in rep
    assert "- **Best Throughput:** 18,147 tokens/sec (ZERO2, WS=4, SeqLen=2048)" in rep
    assert "- **Best Scaling Efficiency:** 50.0% (DDP, WS=2)" in rep
    assert "- **Lowest Peak VRAM:** 9.67 GB (ZERO3, WS=4)" in rep
    assert "|      DDP |         4 |    2048 | A    |     12,220 |        0.6704 |          13.97 |             36.5 |" \
        .replace("|      DDP |", "| DDP      |") in rep


def test_record_markers_roundtrip(capsys):
    rec = make_record("zero2", 4, 0, 2048, "A", 100, 1, 4, 0.451, 5.4, 10.47e9)
    assert list(rec.keys()) == list(RESULT_KEYS)
    assert rec["tokens_per_sec"] == pytest.approx(1 * 2048 * 4 / 0.451)
    assert rec["h2d_gbps_per_gpu"] == pytest.approx(2048 * 4 / 0.451 / 1e9)
    print_markers(rec)
    out = capsys.readouterr().out
    assert ("=" * 80) in out
    assert extract_from_log(out) == dict(rec)


def test_emulated_suite_labels_predictions(tmp_path):
    """scripts/emulated_suite.py: every predicted series is labelled ``<strategy>_pred`` in
    result.json and metrics.csv, each row says whether it is a prediction, grad_accum is the CLI
    value (4, as the harness writes it) even where the engine's accumulation is 1, and the bf16
    DDP row gets its own series (BASELINE config #2)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    recs = []
    for strat, dtype, ws, ms in (("ddp", "fp16", 1, 8.0), ("ddp", "fp16", 8, 10.0), ("ddp", "bf16", 1, 7.5),
                                 ("ddp", "bf16", 8, 9.0), ("zero2", "bf16", 1, 7.0), ("zero2", "bf16", 8, 8.5)):
        rec = {"metric": "tokens_per_sec", "n_gpus": 1 if ws > 1 else ws, "steps": 20, "ms_per_step": ms,
               "value": 2048 * ws / ms * 1e3, "dtype": dtype, "mean_loss": 10.0, "peak_hbm_gb": 5.0,
               "config": {"model": "TinyGPT-A", "seq_len": 2048, "micro_batch_per_gpu": 1,
                          "grad_accum": 1 if strat == "ddp" else 4, "parallelism": f"{strat}-dp{ws}"}}
        if ws > 1:
            rec.update(prediction=True, emulated_world=ws, peak_hbm_gb_per_rank=4.0)
        recs.append(rec)
    src = tmp_path / "pred.jsonl"
    src.write_text("\n".join(json.dumps(r) for r in recs) + "\n")
    out = tmp_path / "emu"
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "emulated_suite.py"), str(src), str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    df = pd.read_csv(out / "summary" / "metrics.csv")
    assert set(df["strategy"]) == {"ddp_pred", "ddp_bf16_pred", "zero2_pred"}
    assert list(df["prediction"]) == [ws > 1 for ws in df["world_size"]]
    assert (df["grad_accum"] == 4).all()
    z8 = df[(df.strategy == "zero2_pred") & (df.world_size == 8)].iloc[0]
    assert abs(z8["scaling_efficiency_pct"] - 100 * 7.0 / 8.5) < 0.01       # vs its measured WS=1 row
    res = json.loads((out / "bench-master-zero2_pred-ws8-seq2048_results" / "result.json").read_text())
    assert res["prediction"] is True and res["emulated_world"] == 8


def test_cost_view_matches_reference_tokens_per_dollar(tmp_path):
    """The reference's cost table (README.md:266-277): tokens/sec per $/hr = tps / (GPUs x $/GPU-hr), ZeRO-2 on
    4 x A10 at $1.50 = 3,025.  metrics.csv keeps its 13 + 1 columns; the cost view lives in metrics_extended.csv
    and the report."""
    _write_published(tmp_path / "results")
    parse_results(str(tmp_path / "results"), str(tmp_path / "summary"), gpu_hour_usd=1.5)
    assert (tmp_path / "summary" / "metrics.csv").read_text().splitlines()[0] == CSV_HEADER
    ext = pd.read_csv(tmp_path / "summary" / "metrics_extended.csv")
    z2 = ext[(ext.strategy == "zero2") & (ext.world_size == 4)].iloc[0]
    assert z2["tokens_per_sec_per_usd_hr"] == pytest.approx(18147 / (4 * 1.5))      # 3,024.5 -> "3,025"
    assert z2["tokens_per_gpu_hour"] == pytest.approx(18147 / 4 * 3600)
    assert z2["tokens_per_usd"] == pytest.approx(18147 / 4 * 3600 / 1.5)
    rep = generate_report(str(tmp_path / "summary" / "metrics.csv"), str(tmp_path / "summary")).read_text()
    assert "## Cost View" in rep and "3,02" in rep


def test_mixed_tiers_keep_reference_grouping(tmp_path):
    """metrics.csv groups by (strategy, seq_len) exactly as the reference does, even across tiers;
    the tier-aware efficiency is a metrics_extended.csv column."""
    rows = [("zero2", 1, "A", 280000.0), ("zero2", 2, "A", 500000.0), ("zero2", 1, "B", 60000.0)]
    for s, ws, tier, tps in rows:
        d = tmp_path / "r" / f"{s}-{ws}-{tier}_results"
        d.mkdir(parents=True)
        rec = dict(zip(RESULT_KEYS, (s, ws, 0, 2048, tier, 10, 1, 4, tps, 1.0, 5.0, 1.0, 1e-5)))
        (d / "result.json").write_text(json.dumps(rec))
    df = parse_results(str(tmp_path / "r"), str(tmp_path / "s"))
    # reference: base = the first row at the smallest world size of the (strategy, seq_len) group
    base = df[df.world_size == 1].iloc[0]["tokens_per_sec"]
    a2 = df[(df.world_size == 2)].iloc[0]
    assert a2["scaling_efficiency_pct"] == pytest.approx(500000.0 / (base * 2) * 100)
    ext = pd.read_csv(tmp_path / "s" / "metrics_extended.csv", dtype={"tier": str})
    e2 = ext[(ext.world_size == 2)].iloc[0]
    assert e2["efficiency_tier_aware_pct"] == pytest.approx(500000.0 / (280000.0 * 2) * 100)
