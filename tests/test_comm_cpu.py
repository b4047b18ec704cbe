"""Comm layer (dltb/comm): collectives over gloo at world size 2, wire accounting, the single-process
no-op path, and the xGMI topology / bucket-size model."""
import os
import socket
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import dltb  # noqa: F401
from dltb.comm import Comm, collective_time_us, parse_topology, recommend_bucket_mb, ring_factor


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = Comm()
        assert (c.world, c.rank) == (world, rank)
        n = 8
        # all-reduce of a slice of a flat buffer, asynchronous, then wait_all
        flat = torch.arange(3 * n, dtype=torch.float32) + 100 * rank
        c.all_reduce(flat[n:2 * n])
        assert c.pending == 1
        c.wait_all()
        ar = flat[n:2 * n].clone()
        # reduce-scatter into this rank's chunk
        inp = torch.arange(world * n, dtype=torch.float32) * (rank + 1)
        out = torch.empty(n)
        c.reduce_scatter(out, inp, async_op=False)
        # in-place all-gather (this rank's slice of the output is the input)
        full = torch.zeros(world * n)
        full[rank * n:(rank + 1) * n] = rank + 1
        w = c.all_gather(full, full[rank * n:(rank + 1) * n], track=False)
        w.wait()
        assert c.pending == 0
        mx = c.max_scalar(float(rank), torch.device("cpu"))
        torch.save({"ar": ar, "rs": out, "ag": full, "max": mx, "stats": dict(c.stats),
                    "wire": c.wire_bytes()}, f"{out_path}.{rank}")
    finally:
        dist.destroy_process_group()


def test_comm_world2():
    world, n = 2, 8
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r")
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    base = torch.arange(n, 2 * n, dtype=torch.float32)
    for r in range(world):
        x = res[r]
        assert torch.equal(x["ar"], 2 * base + 100)                      # (b) + (b + 100)
        full_sum = torch.arange(world * n, dtype=torch.float32) * 3      # ranks scale by 1 and 2
        assert torch.equal(x["rs"], full_sum[r * n:(r + 1) * n])
        assert torch.equal(x["ag"], torch.tensor([1.0] * n + [2.0] * n))
        assert x["max"] == 1.0
        st = x["stats"]
        assert st["all_reduce"]["calls"] == 1 and st["reduce_scatter"]["calls"] == 1
        assert st["all_reduce"]["wire_bytes"] == int(n * 4 * ring_factor("all_reduce", 2))
        assert st["reduce_scatter"]["wire_bytes"] == int(world * n * 4 * 0.5)
        assert st["all_gather"]["wire_bytes"] == int(world * n * 4 * 0.5)
        assert x["wire"] == sum(v["wire_bytes"] for v in st.values())


def test_comm_single_process_is_noop():
    c = Comm()
    t = torch.ones(4)
    assert c.all_reduce(t).wait() and torch.equal(t, torch.ones(4))
    out = torch.empty(4)
    c.reduce_scatter(out, torch.full((4,), 3.0))
    assert torch.equal(out, torch.full((4,), 3.0))
    full = torch.zeros(4)
    c.all_gather(full, full)          # in place: nothing to move
    assert c.pending == 0 and c.wire_bytes() == 0


def test_topology_model():
    assert ring_factor("all_reduce", 8) == 2 * 7 / 8 and ring_factor("all_gather", 1) == 0.0
    # the recommended bucket is the smallest power of two whose fixed cost is <= 20 % of its transfer
    alpha = collective_time_us("reduce_scatter", 0, 8)
    for w in (2, 4, 8):
        mb = recommend_bucket_mb(w)
        xfer = collective_time_us("reduce_scatter", int(mb * (1 << 20)), w) - alpha
        half = collective_time_us("reduce_scatter", int(mb * (1 << 19)), w) - alpha
        assert alpha <= 0.2 * xfer and alpha > 0.2 * half
    assert collective_time_us("all_reduce", 1 << 30, 1) == 0.0
    txt = """============================ ROCm System Management Interface ============================
================================ Link Type between two GPUs ================================
       GPU0         GPU1         GPU2
GPU0   0            XGMI         XGMI
GPU1   XGMI         0            XGMI
GPU2   XGMI         XGMI         0
"""
    links = parse_topology(txt)
    assert links[(0, 1)] == "XGMI" and (0, 0) not in links and len(links) == 6


def test_alpha_beta_fit_and_measured_bucket(tmp_path, monkeypatch):
    import json
    from dltb.comm.collectives import ring_factor
    from dltb.comm.topology import fit_alpha_beta, measured_params, recommend_bucket_mb
    alpha, bus, world = 40.0, 250.0, 8
    rows = [{"op": "reduce_scatter", "bytes": b, "time_us": alpha + b * ring_factor("reduce_scatter", world) / (bus * 1e3)}
            for b in (1 << 20, 4 << 20, 16 << 20, 64 << 20)]
    a, g = fit_alpha_beta(rows, "reduce_scatter", world)
    assert abs(a - alpha) < 1e-6 and abs(g - bus) < 1e-6
    p = tmp_path / "prof.json"
    p.write_text(json.dumps({"worlds": {"8": rows}}))
    monkeypatch.setenv("DLTB_XGMI_PROFILE", str(p))
    assert measured_params(8)[2] == "measured" and measured_params(4)[2] == "default"
    # alpha 40 us at 250 GB/s: need 40/0.2 us * 250 GB/s / (7/8) = 57 MB -> 64 MiB
    assert recommend_bucket_mb(8) == 64.0
    monkeypatch.setenv("DLTB_XGMI_PROFILE", str(tmp_path / "missing.json"))
    assert measured_params(8)[2] == "default"
    # noisy timings that fall with size: the largest message as pure bandwidth, alpha 1 us
    noisy = [{"op": "all_gather", "bytes": 4 << 20, "time_us": 300.0}, {"op": "all_gather", "bytes": 16 << 20, "time_us": 200.0}]
    a, g = fit_alpha_beta(noisy, "all_gather", world)
    assert a == 1.0 and abs(g - ring_factor("all_gather", world) * (16 << 20) / 200.0 / 1e3) < 1e-9


def _calib_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dltb.comm import topology as tp
        res = tp.calibrate_fabric(torch.device("cpu"), sizes_mb=(0.25, 1.0), iters=2)
        if rank == 0:
            torch.save({"rows": res["rows"], "fits": res["fits"],
                        "src": tp.measured_params(world)[2],
                        "bucket": tp.recommend_bucket_mb(world)}, out_path)
    finally:
        dist.destroy_process_group()


def test_calibrate_fabric_world2(monkeypatch):
    """In-job calibration on the job's own process group: one row per (op, size), every time
    positive (the max over ranks), and a physical fit -- when it exists -- becomes the process's
    'calibrated' alpha-beta, ahead of a suite profile."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "calib.pt")
        mp.spawn(_calib_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        r = torch.load(out, weights_only=True)
    assert len(r["rows"]) == 6 and {x["op"] for x in r["rows"]} == {"reduce_scatter", "all_reduce", "all_gather"}
    assert all(x["time_us"] > 0 and x["bytes"] > 0 for x in r["rows"])
    if "reduce_scatter" in r["fits"]:
        assert r["src"] == "calibrated" and r["fits"]["reduce_scatter"]["bus_GBps"] > 0
    assert r["bucket"] >= 1


def test_calibrated_params_take_precedence(tmp_path, monkeypatch):
    import json
    from dltb.comm import topology as tp
    p = tmp_path / "prof.json"
    p.write_text(json.dumps({"worlds": {"8": [{"op": "reduce_scatter", "bytes": b, "time_us": 40 + b / 2.5e5}
                                               for b in (1 << 20, 16 << 20)]}}))
    monkeypatch.setenv("DLTB_XGMI_PROFILE", str(p))
    assert tp.measured_params(8)[2] == "measured"
    monkeypatch.setitem(tp._CALIBRATED, (8, "reduce_scatter"), (12.0, 400.0))
    assert tp.measured_params(8) == (12.0, 400.0, "calibrated")
    # 12 us at 400 GB/s: need 12/0.2 us * 400 GB/s / (7/8) = 27 MB -> 32 MiB
    assert tp.recommend_bucket_mb(8) == 32.0
    # an inflated in-job intercept (500 us: would need 171 MB) stays at the validated 4-block bucket size
    monkeypatch.setitem(tp._CALIBRATED, (8, "reduce_scatter"), (500.0, 300.0))
    assert tp.recommend_bucket_mb(8) == tp.BUCKET_MB_MAX == 64.0
