"""World 2 (gloo) == world 1 on the concatenated batch, every engine, fp32 CPU reference ops.

The GPU twin (tests/test_multirank_gpu.py) runs the same script with bf16 HIP kernels and two
ranks sharing one MI355X through host-staged gloo collectives."""
from multirank_util import compare, run


def test_world2_equals_world1_cpu(tmp_path):
    ws1 = run(tmp_path / "ws1.pt", 1, "cpu")
    ws2 = run(tmp_path / "ws2.pt", 2, "cpu")
    assert set(ws1) == set(ws2)
    bad = compare(ws1, ws2, loss_tol=1e-4, upd_tol=1e-3, cos_min=0.99999, param_tol=1e-3)
    assert not bad, bad
