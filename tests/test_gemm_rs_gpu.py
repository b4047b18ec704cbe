"""Own MFMA GEMM (csrc/gemm_rs.hip) against an fp32 torch product: every row of the shipped own-GEMM
table (the configs the training step runs), bias / accumulate epilogues, grids with more tiles than CUs
(co-resident workgroups: the case that exposed the LDS race fixed by rs_barrier), and the model path
(ops/functional.py dispatch) actually issuing them."""
import csv
import os

import pytest
import torch

import dltb  # noqa: F401
import dltb.ops.functional as F
from dltb.ops._ext import ext

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "configs", "gemm_rs", "gemm_rs_gfx950.csv")


def _rows():
    with open(TABLE) as f:
        return [{k: int(v) for k, v in r.items()} for r in csv.DictReader(ln for ln in f if not ln.startswith("#"))]


def _check(M, N, K, cfg, gm, bias, accumulate=False):
    torch.manual_seed(M + N + K + cfg)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    bb = torch.randn(N, device="cuda", dtype=torch.bfloat16) if bias else None
    c0 = torch.randn(M, N, device="cuda", dtype=torch.bfloat16) if accumulate else None
    ref = a.float() @ b.float().t()
    if bias:
        ref += bb.float()
    if accumulate:
        ref += c0.float()
    out = c0.clone() if accumulate else None
    y = ext().gemm_rs(a, b, out, bb, accumulate, cfg, gm)
    torch.cuda.synchronize()
    err = (y.float() - ref).abs().max().item()
    # bf16 output: half an ulp of the largest magnitude, plus fp32 accumulation-order noise
    tol = ref.abs().max().item() * 2 ** -8 + 1e-2
    assert err <= tol, f"M{M} N{N} K{K} cfg {cfg} gm {gm}: max err {err:.4g} > {tol:.4g}"


@pytest.mark.parametrize("row", _rows(), ids=lambda r: f"{r['m']}x{r['n']}x{r['k']}b{r['bias']}c{r['cfg']}")
def test_shipped_table_rows(row):
    assert ext().gemm_rs_supported(row["m"], row["n"], row["k"], row["cfg"])
    _check(row["m"], row["n"], row["k"], row["cfg"], row["gm"], bool(row["bias"]))


# cfg -> (N of the test product): 1 / 6 are 128 x 256 tiles, 2 / 7 128 x 192, 3 128 x 128, the rest 128 x 64
_N = {1: 4096, 6: 4096, 2: 3072, 7: 3072, 3: 2048}
# the K-split configs (two wave groups on one tile, alternate k-steps; csrc/gemm_rs.hip KG = 2)
_KSPLIT = [9, 10, 11, 12, 13, 14]


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 7, 8] + _KSPLIT)
def test_fenced_kernels_epilogues(cfg):
    M, N, K = 2048, _N.get(cfg, 1024), 1024
    _check(M, N, K, cfg, 4, bias=True)
    _check(M, N, K, cfg, 1, bias=False, accumulate=True)


@pytest.mark.parametrize("cfg", _KSPLIT)
@pytest.mark.parametrize("K", [512, 3072, 4096])
def test_ksplit_depths(cfg, K):
    """Both k-groups' partial tiles are summed: every K the groups split evenly, incl. the per-group minimum."""
    if not ext().gemm_rs_supported(2048, 1024, K, cfg):
        pytest.skip(f"K {K} not a multiple of cfg {cfg}'s k-steps per group round")
    _check(2048, 1024, K, cfg, 4, bias=True)


def test_ablation_configs_refused():
    """Timing-only ablation configs compute wrong products by construction: refused unless DLTB_GEMM_ABLATION=1."""
    if os.environ.get("DLTB_GEMM_ABLATION") == "1":
        pytest.skip("ablations enabled in this process")
    for cfg in range(15, 25):
        assert not ext().gemm_rs_supported(2048, 1024, 1024, cfg)


@pytest.mark.parametrize("cfg", [0, 4, 9, 11])
def test_coresident_workgroups(cfg):
    # 4096 x 2048 with 128 x 64 tiles = 1024 workgroups (4 per CU over time, 2 resident at once)
    for _ in range(3):
        _check(4096, 2048, 1024, cfg, 4, bias=True)


def test_model_step_issues_own_gemm():
    from dltb.models import build_model, get_model_config
    from dltb.parallel import engine_config, make_engine
    F._rs_table = None
    if not F.rs_table():
        pytest.skip("own-GEMM table off (DLTB_OWN_GEMM=0) or absent")
    torch.manual_seed(0)
    cfg = get_model_config("A", 2048)
    cfg.n_layer = 1
    eng = make_engine(build_model(cfg), engine_config("zero2", 1, "reference"), "cuda:0")
    idx = torch.randint(0, cfg.vocab_size, (1, 2048), device="cuda:0")
    c0 = F.own_gemm_calls
    loss = eng(idx, idx)[1]
    eng.backward(loss)
    torch.cuda.synchronize()
    assert F.own_gemm_calls - c0 == len(_rows()), "every shipped product should run on the own kernel"
    assert 5.0 < float(loss.item()) < 15.0


@pytest.mark.parametrize("cfg", [0, 1, 6, 9])
def test_gelu_out_epilogue(cfg):
    """gemm_rs(..., gelu_out=g): f = a b^T + bias (fp32 reference) and g = GELU(f) of the ROUNDED f, bitwise
    what the separate gelu_fwd kernel writes -- the fc1 forward with its activation fused (table bias = 3)."""
    C = ext()
    M, N, K = 2048, _N.get(cfg, 1024), 1024
    assert C.gemm_rs_gelu_supported(M, N, K, cfg)      # fp32-image epilogue kernels (gemm_rsf)
    torch.manual_seed(cfg)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    bias = (torch.randn(N, device="cuda") * 0.1).to(torch.bfloat16)
    g = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    f = C.gemm_rs(a, b, None, bias, False, cfg, 4, gelu_out=g)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + bias.float()
    tol = ref.abs().max().item() * 2 ** -7 + 1e-2
    assert (f.float() - ref).abs().max().item() <= tol
    assert torch.equal(g, C.gelu_fwd(f, None))
    ref_g = torch.nn.functional.gelu(f.float())
    assert (g.float() - ref_g).abs().max().item() <= 2e-2 * ref_g.abs().max().item() + 1e-2


@pytest.mark.parametrize("cfg", [6, 9])
def test_dgelu_epilogue(cfg):
    """gemm_rs_aux: out = (a b^T) * aux rounded once, part = per-128-row column sums of the rounded out --
    the fc2 data gradient with the GELU backward and the fc1 bias partials fused (aux = GELU'(f))."""
    C = ext()
    M, N, K = 2048, _N.get(cfg, 1024), 1024
    assert C.gemm_rs_aux_supported(M, N, K, cfg)
    assert not C.gemm_rs_aux_supported(2048, 4096, 1024, 1)   # 4 waves: 32 aux chunks per thread, not prefetched
    torch.manual_seed(cfg)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    f = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    g, gp = C.gelu_fwd_grad(f)
    x = f.float()
    ref_g = torch.nn.functional.gelu(x)
    cdf = 0.5 * (1 + torch.erf(x / 2 ** 0.5))
    ref_gp = cdf + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    assert (g.float() - ref_g).abs().max().item() <= 2e-2 * ref_g.abs().max().item()
    assert (gp.float() - ref_gp).abs().max().item() <= 1e-2
    out, part = C.gemm_rs_aux(a, b, None, gp, cfg, 4)
    torch.cuda.synchronize()
    ref = (a.float() @ b.float().t()) * gp.float()
    tol = ref.abs().max().item() * 2 ** -7 + 1e-2
    assert (out.float() - ref).abs().max().item() <= tol
    assert part.shape == (M // 128, N)
    # the partials sum the ROUNDED outputs, per 128-row tile
    ref_part = out.float().view(M // 128, 128, N).sum(1)
    assert torch.allclose(part, ref_part, rtol=1e-4, atol=1e-3)


def _one_layer_grads(monkeypatch, table):
    from dltb.models import build_model, get_model_config
    from dltb.parallel import engine_config, make_engine
    if table is None:
        monkeypatch.delenv("DLTB_OWN_GEMM_TABLE", raising=False)
    else:
        monkeypatch.setenv("DLTB_OWN_GEMM_TABLE", os.path.join(ROOT, "configs", "gemm_rs", table))
    F._rs_table = None
    try:
        torch.manual_seed(0)
        cfg = get_model_config("A", 2048)
        cfg.n_layer = 1
        model = build_model(cfg)
        eng = make_engine(model, engine_config("zero2", 1, "reference"), "cuda:0")
        idx = torch.randint(0, cfg.vocab_size, (1, 2048), generator=torch.Generator().manual_seed(1)).cuda()
        c0 = F.own_gemm_calls
        loss = eng(idx, idx)[1]
        eng.backward(loss)
        torch.cuda.synchronize()
        return float(loss.item()), eng.flat_grad.float().clone(), F.own_gemm_calls - c0
    finally:
        F._rs_table = None


@pytest.mark.parametrize("table", ["ab_gelu6.csv", "ab_gelu1.csv", "ab_dgelu6.csv"])
def test_model_fused_gelu_tables_track_shipped(table, monkeypatch):
    """The model with a fused-GELU table row (forward GELU output, or the backward dGELU epilogue) trains like
    the shipped table: same loss to bf16 noise, gradients within bf16 rounding of the changed products."""
    l0, g0, n0 = _one_layer_grads(monkeypatch, None)
    l1, g1, n1 = _one_layer_grads(monkeypatch, table)
    assert n1 == n0 + 1, (n0, n1)                      # the fused product ran on the own kernel
    assert abs(l1 - l0) < 2e-3 * abs(l0), (l0, l1)
    rel = (g1 - g0).norm().item() / g0.norm().item()
    assert rel < 2e-2, rel
