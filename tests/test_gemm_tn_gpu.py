"""Weight-gradient GEMM (csrc/gemm_tn.hip): out[b] (+)= a[b]^T b[b] with both operands token-major, against an
fp32 torch product -- 2-D, batched over strided views shaped like the engine's layer buffers and flat gradient
slots (batch stride != rows x row stride), accumulate, and the dispatch that routes the model's batched dW
through it (parallel/wgrad.py)."""
import pytest
import torch

import dltb  # noqa: F401
from dltb.ops._ext import ext

pytestmark = pytest.mark.gpu


def _rand(*shape, scale=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * scale).to(torch.bfloat16)


def _check(out, ref, what):
    err = (out.float() - ref).abs().max().item()
    tol = ref.abs().max().item() * 2 ** -7 + 1e-2
    assert err <= tol, f"{what}: max err {err:.4g} > {tol:.4g}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (1024, 512, 2048), (512, 1024, 640), (3072, 1024, 1024),
                                   (512, 256, 192), (768, 512, 4096)])
def test_gemm_tn_2d(M, N, K):
    torch.manual_seed(M + N + K)
    a, b = _rand(K, M), _rand(K, N, scale=0.05)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ext().gemm_tn(a, b, out, False)
    torch.cuda.synchronize()
    _check(out, a.float().t() @ b.float(), f"gemm_tn {M}x{N}x{K}")


def test_gemm_tn_asymmetric_layout():
    """Exact integer data, asymmetric operands: a transposed / swapped epilogue cannot pass."""
    K, M, N = 128, 256, 512
    a = (torch.arange(K * M, device="cuda") % 7 - 3).reshape(K, M).to(torch.bfloat16)
    b = (torch.arange(K * N, device="cuda") % 5 - 2).reshape(K, N).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ext().gemm_tn(a, b, out, False)
    torch.cuda.synchronize()
    ref = a.float().t() @ b.float()
    assert torch.equal(out.float(), ref)


@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_tn_batched_strided(accumulate):
    # layer buffers [L, T, k] (batch stride T * k) and gradient slots at a block stride larger than M * N
    torch.manual_seed(1 + accumulate)
    L, T, M, N, slot = 4, 1024, 512, 768, 512 * 768 + 4096
    dy, x = _rand(L, T, M), _rand(L, T, N, scale=0.05)
    flat = torch.randn(L * slot, device="cuda").to(torch.bfloat16)
    gaps0 = flat.view(L, slot)[:, M * N:].clone()
    dw = flat.as_strided((L, M, N), (slot, N, 1))
    before = dw.float().clone()
    ext().gemm_tn(dy, x, dw, accumulate)
    torch.cuda.synchronize()
    ref = torch.bmm(dy.float().transpose(1, 2), x.float()) + (before if accumulate else 0)
    _check(dw, ref, f"batched accumulate={accumulate}")
    assert torch.equal(flat.view(L, slot)[:, M * N:], gaps0)      # nothing written between the slots


def test_gemm_tn_refuses_unsupported():
    a, b = _rand(128, 200), _rand(128, 256)
    out = torch.empty(200, 256, device="cuda", dtype=torch.bfloat16)
    assert not ext().gemm_tn_supported(200, 256, 128)
    assert not ext().gemm_tn_supported(256, 256, 64) and not ext().gemm_tn_supported(256, 256, 160)
    with pytest.raises(RuntimeError):
        ext().gemm_tn(a, b, out, False)


@pytest.mark.parametrize("L,T,M,N,own", [(4, 256, 1024, 4096, True),    # 4 x 4 x 16 = 256 tiles: gemm_tn
                                          (3, 512, 256, 512, False)])     # 6 tiles: hipBLASLt fills the chip
def test_wgrad_queue_uses_gemm_tn(L, T, M, N, own):
    """The engine's batched dW (parallel/wgrad.py) runs on gemm_tn from one 256 x 256 tile per CU up (below that
    on hipBLASLt) and matches per-block torch products either way."""
    from dltb.parallel.wgrad import WgradQueue

    class U:
        pass
    torch.manual_seed(3)
    dy, x = _rand(L, T, M), _rand(L, T, N, scale=0.05)
    flat = torch.zeros(L * M * N + 64, device="cuda", dtype=torch.bfloat16)
    q = WgradQueue()
    units = [U() for _ in range(L)]
    for i, u in enumerate(units):
        q.add(u, 0, dy[i], x[i], flat[i * M * N:(i + 1) * M * N].view(M, N), False)
    q.flush()
    torch.cuda.synchronize()
    assert q.batched_calls == 1 and q.tn_calls == (1 if own else 0)
    for i in range(L):
        _check(flat[i * M * N:(i + 1) * M * N].view(M, N), dy[i].float().t() @ x[i].float(), f"block {i}")
