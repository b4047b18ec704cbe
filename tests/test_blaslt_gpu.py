"""hipBLASLt extension-API GEMMs (csrc/blaslt.cpp, ops/blaslt.py) against fp32 torch products.

Every layout the model issues (forward with bias epilogue, dgrad through W and through cached W^T,
weight gradients overwrite / accumulate, layer-strided batched weight gradients) runs through
``blaslt_run`` with several split-K / workgroup-mapping settings, eagerly and under HIP-graph
capture, and must match ``a.float() @ b.float()`` within bf16 rounding."""
import pytest
import torch

import dltb  # noqa: F401
from dltb.ops import blaslt
from dltb.ops._ext import ext
from dltb.parallel.wgrad import strided_batch

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*s, dtype=BF):
    return (torch.randn(*s, device="cuda") * 0.5).to(dtype)


def best_algo(key, a, b, c, bias=None, splitks=(0,), wgms=(0,)):
    _, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, beta1, _ = key
    res = ext().blaslt_sweep(b, a, c, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, bool(beta1), bias,
                             2, list(splitks), list(wgms), 2)
    assert res, "no hipBLASLt solution for " + str(key)
    return res


def check(got, want, what):
    err = (got.float() - want).abs().max().item()
    tol = 2e-2 * want.abs().max().item() + 1e-2
    assert err <= tol, f"{what}: max err {err} > {tol}"


CASES = ["fwd_bias", "dgrad", "dgrad_wt", "wgrad", "wgrad_acc"]


def operands(case, T=512, din=256, dout=384):
    x, w, dy, bias = rnd(T, din), rnd(dout, din), rnd(T, dout), rnd(dout)
    if case == "fwd_bias":
        return x, w.t(), torch.empty(T, dout, device="cuda", dtype=BF), False, bias
    if case == "dgrad":
        return dy, w, torch.empty(T, din, device="cuda", dtype=BF), False, None
    if case == "dgrad_wt":
        return dy, w.t().contiguous().t(), torch.empty(T, din, device="cuda", dtype=BF), False, None
    return dy.t(), x, rnd(dout, din), case == "wgrad_acc", None


@pytest.mark.parametrize("case", CASES)
def test_blaslt_layouts(case):
    a, b, c, acc, bias = operands(case)
    key = blaslt.problem(a, b, c, acc, bias)
    assert key is not None
    c0 = c.float().clone()
    want = a.float() @ b.float() + (c0 if acc else 0) + (bias.float() if bias is not None else 0)
    res = best_algo(key, a, b, c, bias, splitks=(0, 2, 4), wgms=(0, 4))
    tried = 0
    for algo, sk, wg, _, _ in res[:6]:
        c.copy_(c0.to(BF))
        blaslt.run(key, a, b, c, (algo, sk, wg), bias)
        torch.cuda.synchronize()
        check(c, want, f"{case} algo {algo} splitK {sk} wgm {wg}")
        tried += 1
    assert tried >= 1


@pytest.mark.parametrize("acc", [False, True])
def test_blaslt_batched_strided(acc):
    L, T, din, dout, pad = 4, 512, 256, 384, 128
    dys = rnd(L, T, dout + pad)
    xs = rnd(L, T, din)
    stride = dout * din + 256
    flat = rnd(L * stride)
    DY = strided_batch([dys[i, :, :dout] for i in range(L)])
    X = strided_batch([xs[i] for i in range(L)])
    DW = strided_batch([flat[i * stride:i * stride + dout * din].view(dout, din) for i in range(L)], out=True)
    a = DY.transpose(1, 2)
    key = blaslt.problem(a, X, DW, acc)
    assert key is not None and key[6] == L
    before = flat.clone()
    want = torch.bmm(a.float(), X.float()) + (DW.float() if acc else 0)
    res = best_algo(key, a, X, DW, splitks=(0, 2), wgms=(0, 8))
    flat.copy_(before)
    algo, sk, wg = res[0][:3]
    blaslt.run(key, a, X, DW, (algo, sk, wg))
    torch.cuda.synchronize()
    check(DW, want, "batched")
    # the gaps between the strided matrices are untouched
    for i in range(L):
        lo, hi = i * stride + dout * din, (i + 1) * stride
        assert torch.equal(flat[lo:hi], before[lo:hi])


def test_blaslt_graph_capture_and_table_dispatch(tmp_path):
    """A tuned entry written as a table row dispatches through mm() (functional.linear_fwd), and the
    call replays correctly from a captured HIP graph with a fresh output buffer."""
    from dltb.ops import functional as F_
    x, wt, _, _, bias = operands("fwd_bias")
    w = wt.t()
    y0 = torch.empty(x.shape[0], w.shape[0], device="cuda", dtype=BF)
    key = blaslt.problem(x, w.t(), y0, False, bias)
    algo, sk, wg, us, name = best_algo(key, x, w.t(), y0, bias, splitks=(0, 2), wgms=(0, 4))[0]
    path = tmp_path / "t.csv"
    row = dict(zip(blaslt.FIELDS[:15], key))
    row.update(algo=algo, splitk=sk, wgm=wg, us=us, torch_us=us, solution=name)
    with open(path, "w") as f:
        f.write(",".join(blaslt.FIELDS) + "\n" + ",".join(str(row[k]) for k in blaslt.FIELDS) + "\n")
    try:
        assert blaslt.load(str(path)) == 1
        want = x.float() @ w.float().t() + bias.float()
        check(F_.linear_fwd(x, w, bias), want, "dispatch eager")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            F_.linear_fwd(x, w, bias)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = F_.linear_fwd(x, w, bias)
        x.copy_(rnd(*x.shape))
        g.replay()
        torch.cuda.synchronize()
        check(y, x.float() @ w.float().t() + bias.float(), "graph replay")
    finally:
        blaslt.load()                     # back to the shipped table


@pytest.mark.parametrize("which", ["x_small", "dy_small"])
def test_wgrad_transposed_operand(which):
    """Large weight gradients run with the smaller operand transposed K-contiguous
    (functional.wgrad_operands); the product equals dy^T x, overwrite and accumulate."""
    from dltb.ops import functional as F_
    T = 4096
    out_f, in_f = (14336, 4096) if which == "x_small" else (4096, 14336)
    dy, x = rnd(T, out_f), rnd(T, in_f)
    a, b = F_.wgrad_operands(dy, x)
    if which == "x_small":
        assert a.stride() == dy.t().stride() and b.stride(0) == 1          # x^T copy, viewed back
    else:
        assert a.is_contiguous() and b.data_ptr() == x.data_ptr()          # dy^T copy
    want = dy.float().t() @ x.float()
    dw = torch.empty(out_f, in_f, device="cuda", dtype=BF)
    F_.linear_wgrad(dy, x, dw, None, False)
    check(dw, want, "overwrite")
    F_.linear_wgrad(dy, x, dw, None, True)
    check(dw, 2 * want, "accumulate")
    small = F_.wgrad_operands(rnd(2048, 1024), rnd(2048, 1024))             # small product: untouched
    assert small[1].stride(1) == 1 and not small[0].is_contiguous()


def test_head_dgrad_table_path():
    """TinyGPT-A's tied-head dgrad (2048 x 32000 x 1024, K = vocab) dispatches to the shipped table's
    split-K hipBLASLt entry with the device-scalar g applied afterwards, and matches g * dL W."""
    from dltb.ops import functional as F_
    blaslt.load()
    dl, wte = rnd(2048, 32000), rnd(32000, 1024)
    wt = wte.t().contiguous()
    g = torch.tensor([0.37], device="cuda")
    dh0 = torch.empty(2048, 1024, device="cuda", dtype=BF)
    assert blaslt.problem(dl, wt.t(), dh0, False) is not None
    got = F_.head_dgrad(dl, wte, wt, g)
    want = (dl.float() @ wte.float()) * 0.37
    check(got, want, "head dgrad (table)")
    blaslt.disable()
    try:
        check(F_.head_dgrad(dl, wte, wt, g), want, "head dgrad (own split-K kernel)")
    finally:
        blaslt.load()
