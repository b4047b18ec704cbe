"""The column-major problem keys of ops/blaslt.py describe the torch products they stand for.

The GPU runs these keys through hipBLASLt (tests/test_blaslt_gpu.py); here a NumPy column-major
GEMM reads the raw storages exactly as the key says (op, leading dimension, batch stride) and must
reproduce ``a @ b`` for every operand layout the model and the weight-gradient queue produce.
"""
import numpy as np
import pytest
import torch

import dltb  # noqa: F401
from dltb.ops import blaslt
from dltb.parallel.wgrad import strided_batch


def colmajor(store, off, rows, cols, ld):
    return np.array([[store[off + j * ld + i] for j in range(cols)] for i in range(rows)])


def blas_ref(key, a, b, c, bias=None):
    """D = op(A) op(B) (+ C) (+ bias) from raw storages; BLAS A = torch b, BLAS B = torch a."""
    _, opA, opB, m, n, k, batch, lda, ldb, ldc, sa, sb, sc, beta1, has_bias = key
    SA = b.untyped_storage()
    A_st = torch.tensor([], dtype=b.dtype).set_(b.untyped_storage()).float().numpy()
    B_st = torch.tensor([], dtype=a.dtype).set_(a.untyped_storage()).float().numpy()
    C_st = torch.tensor([], dtype=c.dtype).set_(c.untyped_storage()).float().numpy()
    del SA
    out = []
    for q in range(batch):
        Am = colmajor(A_st, b.storage_offset() + q * sa, k if opA else m, m if opA else k, lda)
        Bm = colmajor(B_st, a.storage_offset() + q * sb, n if opB else k, k if opB else n, ldb)
        D = (Am.T if opA else Am) @ (Bm.T if opB else Bm)
        if beta1:
            D = D + colmajor(C_st, c.storage_offset() + q * sc, m, n, ldc)
        if has_bias:
            D = D + bias.float().numpy()[:, None]
        out.append(D.T)                              # column-major m x n == row-major n x m = torch C
    return np.stack(out) if c.dim() == 3 else out[0]


def _expect(a, b, c, acc, bias=None):
    want = (a.float() @ b.float())
    if acc:
        want = want + c.float()
    if bias is not None:
        want = want + bias.float()
    return want.numpy()


@pytest.mark.parametrize("case", ["fwd", "fwd_bias", "dgrad", "dgrad_wt", "wgrad", "wgrad_acc"])
def test_key_matches_product(case):
    g = torch.Generator().manual_seed(0)
    T, din, dout = 12, 8, 6
    r = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16)  # noqa: E731
    x, w, dy, bias = r(T, din), r(dout, din), r(T, dout), r(dout)
    acc = case == "wgrad_acc"
    if case.startswith("fwd"):
        a, b = x, w.t()
        bias = bias if case == "fwd_bias" else None
        c = torch.zeros(T, dout, dtype=torch.bfloat16)
    elif case == "dgrad":
        a, b, bias = dy, w, None
        c = torch.zeros(T, din, dtype=torch.bfloat16)
    elif case == "dgrad_wt":
        a, b, bias = dy, w.t().contiguous().t(), None
        c = torch.zeros(T, din, dtype=torch.bfloat16)
    else:
        a, b, bias = dy.t(), x, None
        c = r(dout, din)
    key = blaslt.problem(a, b, c, acc, bias)
    assert key is not None
    got = blas_ref(key, a, b, c, bias)
    np.testing.assert_allclose(got, _expect(a, b, c, acc, bias), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("acc", [False, True])
def test_batched_strided_views(acc):
    """The weight-gradient queue's layer-strided views (wgrad.py) map to batched keys."""
    g = torch.Generator().manual_seed(1)
    L, T, din, dout, pad = 3, 10, 8, 6, 4
    dys = torch.randn(L, T, dout + pad, generator=g).to(torch.bfloat16)      # strided activation buffers
    xs = torch.randn(L, T, din, generator=g).to(torch.bfloat16)
    flat = torch.randn(L * (dout * din + 16), generator=g).to(torch.bfloat16)
    dw = [flat[i * (dout * din + 16):i * (dout * din + 16) + dout * din].view(dout, din) for i in range(L)]
    DY = strided_batch([dys[i, :, :dout] for i in range(L)])
    X = strided_batch([xs[i] for i in range(L)])
    DW = strided_batch(dw, out=True)
    key = blaslt.problem(DY.transpose(1, 2), X, DW, acc)
    assert key is not None and key[6] == L
    got = blas_ref(key, DY.transpose(1, 2), X, DW)
    want = np.stack([_expect(DY[i].t(), X[i], DW[i], acc) for i in range(L)])
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-4)


def test_unexpressible_layouts_fall_back():
    a = torch.randn(4, 6, dtype=torch.bfloat16)[:, ::2]          # no unit inner stride
    b = torch.randn(3, 5, dtype=torch.bfloat16)
    c = torch.empty(4, 5, dtype=torch.bfloat16)
    assert blaslt.problem(a, b, c, False) is None
    assert blaslt.problem(torch.randn(4, 3), torch.randn(3, 5), torch.empty(4, 5), False) is None   # fp32
    # no table on the CPU: mm never launches, the caller keeps its torch path
    assert blaslt.mm(torch.randn(4, 3, dtype=torch.bfloat16), b, c) is False


def test_cpp_key_matches_python():
    """dltb._C.blaslt_key (the C++ lookup key of blaslt_mm) equals ops/blaslt.py's problem()."""
    from dltb.ops._ext import ext
    g = torch.Generator().manual_seed(2)
    r = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16)  # noqa: E731
    x, w, dy, bias = r(12, 8), r(6, 8), r(12, 6), r(6)
    L = 3
    dys, xs = r(L, 12, 10), r(L, 12, 8)
    DY = strided_batch([dys[i, :, :6] for i in range(L)])
    X = strided_batch([xs[i] for i in range(L)])
    DW = torch.empty(L, 6, 8, dtype=torch.bfloat16)
    cases = [(x, w.t(), torch.empty(12, 6, dtype=torch.bfloat16), False, bias),
             (dy, w, torch.empty(12, 8, dtype=torch.bfloat16), False, None),
             (dy.t(), x, r(6, 8), True, None),
             (DY.transpose(1, 2), X, DW, True, None),
             (x[:, ::2], r(4, 5), torch.empty(12, 5, dtype=torch.bfloat16), False, None)]
    for a, b, c, acc, bs in cases:
        py = blaslt.problem(a, b, c, acc, bs)
        cc = ext().blaslt_key(a, b, c, acc, bs)
        if py is None:
            assert cc is None
        else:
            assert cc == [1 if py[0] == "fp16" else 0, *py[1:]]


def test_batched_wgrad_is_never_tn():
    """The model's batched weight gradients (layer-strided row-major buffers) are BLAS "NT"
    (opA N, opB T); the batched "TN" form -- whose hipBLASLt heuristic solution faulted the GPU in
    profiles/dw_layout_probe_fault_r4.txt -- is refused by the weight-gradient queue, and its key is
    the one csrc/bindings.cpp refuses (batch > 1, opA T, opB N)."""
    from dltb.parallel.wgrad import WgradQueue
    L, N, dout, din = 4, 64, 48, 32
    dy = torch.randn(L, N, dout).to(torch.bfloat16)          # layer buffers: [L, tokens, width]
    x = torch.randn(L, N, din).to(torch.bfloat16)
    dw = torch.zeros(L, dout, din, dtype=torch.bfloat16)
    key = blaslt.problem(dy.transpose(1, 2), x, dw, False)
    assert key is not None and (key[1], key[2], key[6]) == (0, 1, L)
    # the probe's faulting form: X seen transposed from a K-contiguous [L, din, N] buffer
    xt = x.transpose(1, 2).contiguous()
    bad = blaslt.problem(dy.transpose(1, 2).contiguous(), xt.transpose(1, 2), dw, False)
    assert bad is not None and (bad[1], bad[2], bad[6]) == (1, 0, L)
    q = WgradQueue()

    class U:
        pass
    units = [U() for _ in range(L)]
    for i, u in enumerate(units):
        q.add(u, 0, dy[i], xt[i].t(), dw[i], False)
    with pytest.raises(RuntimeError, match="TN"):
        q.flush()
