"""xGMI topology and the alpha-beta cost model behind the engines' bucket sizes.

An 8 x MI355X node is fully connected point to point: every GPU has 7 xGMI links of about
153 GB/s each, one to every peer (no switch).  A ring collective therefore runs over ONE link per
hop, so a rank's ring bandwidth is bounded by a single link, while RCCL's multi-ring / direct
algorithms spread one collective over several links.  The model below uses the bus bandwidth
measured by ``scripts/bench_collectives.py`` where available and otherwise a conservative
per-rank figure.

``recommend_bucket_mb`` picks the smallest bucket whose fixed per-call latency (alpha) stays below
a target fraction of its transfer time, so overlap with backward starts early without paying many
launch latencies.  The reference's DDP uses 25 MiB buckets (NVSwitch/PCIe tuned) and DeepSpeed a
single 5e8-element bucket.
"""
import json
import os
import re
import shutil
import subprocess

XGMI_LINKS_PER_GPU = 7
XGMI_LINK_GBPS = 153.0          # per direction, per link
DEFAULT_BUS_GBPS = 300.0        # conservative RCCL bus bandwidth per rank at 8 GPUs (large messages)
DEFAULT_ALPHA_US = 25.0         # fixed cost of one RCCL collective (launch + sync), 8 ranks
LINK_EFFICIENCY = 0.7           # share of a link's rate a ring step sustains (assumed until measured)


def default_bus_gbps(world: int) -> float:
    """Default bus bandwidth at ``world`` ranks of one node: a rank reaches its peers over its
    ``world - 1`` point-to-point links only, so small jobs cannot use the whole 7-link fabric (two GPUs
    share ONE link); capped at the conservative 8-GPU figure."""
    if world <= 1:
        return DEFAULT_BUS_GBPS
    return min(DEFAULT_BUS_GBPS, LINK_EFFICIENCY * XGMI_LINK_GBPS * min(world - 1, XGMI_LINKS_PER_GPU))


def collective_time_us(op: str, nbytes: int, world: int, bus_gbps: float = None,
                       alpha_us: float = DEFAULT_ALPHA_US) -> float:
    """alpha-beta estimate of one collective on ``nbytes`` (full buffer) at ``world`` ranks
    (default bus bandwidth: ``default_bus_gbps(world)``)."""
    from .collectives import ring_factor
    if world <= 1:
        return 0.0
    if bus_gbps is None:
        bus_gbps = default_bus_gbps(world)
    return alpha_us + nbytes * ring_factor(op, world) / (bus_gbps * 1e3)


_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_PROFILE = os.path.join(_ROOT, "profiles", "xgmi_buckets.json")


def load_profile(path: str = None):
    """The measured collective sweep written by scripts/run_all_benchmarks.sh (scripts/
    bench_collectives.py at each world size): {"worlds": {"8": [row, ...]}} with rows
    {"op", "bytes", "time_us", ...}.  ``$DLTB_XGMI_PROFILE`` overrides the default
    ``profiles/xgmi_buckets.json``; None when absent or unreadable."""
    path = path or os.environ.get("DLTB_XGMI_PROFILE") or DEFAULT_PROFILE
    try:
        with open(path) as f:
            data = json.load(f)
        return data if isinstance(data.get("worlds"), dict) else None
    except (OSError, ValueError, AttributeError):
        return None


def fit_alpha_beta(rows, op: str, world: int):
    """Least-squares fit time_us = alpha + bytes * ring_factor / (bus_GBps * 1e3) over the measured
    sizes of ``op``; returns (alpha_us, bus_GBps) or None (fewer than 2 sizes).  A fit with a non-positive
    slope (noisy timings) falls back to the largest size as pure bandwidth."""
    from .collectives import ring_factor
    pts = [(float(r["bytes"]), float(r["time_us"])) for r in rows if r.get("op") == op]
    if len(pts) < 2:
        return None
    n = len(pts)
    mx = sum(x for x, _ in pts) / n
    my = sum(y for _, y in pts) / n
    sxx = sum((x - mx) ** 2 for x, _ in pts)
    if sxx <= 0:
        return None
    slope = sum((x - mx) * (y - my) for x, y in pts) / sxx        # us per byte
    alpha = my - slope * mx
    f = ring_factor(op, world)
    if f <= 0:
        return None
    if slope <= 0:
        # timings that fall with size (noise: a loaded host, a gloo run beside other jobs): no line
        # fits, so take the largest message as pure bandwidth -- a conservative bus rate, alpha 1 us
        xb, yb = max(pts)
        if yb <= 0:
            return None
        slope, alpha = yb / xb, 1.0
    return max(alpha, 1.0), f / (slope * 1e3)


# (world, op) -> (alpha_us, bus_GBps): fitted by calibrate_fabric() in THIS job, on its own ranks
_CALIBRATED = {}


def measured_params(world: int, op: str = "reduce_scatter", path: str = None):
    """(alpha_us, bus_GBps, source) for ``world`` ranks: this job's own calibration
    (:func:`calibrate_fabric`, source "calibrated"), else the fit of the suite's measured sweep when
    the profile holds this world size ("measured"), else the conservative defaults ("default")."""
    cal = _CALIBRATED.get((world, op))
    if cal is not None:
        return cal[0], cal[1], "calibrated"
    prof = load_profile(path)
    rows = (prof or {}).get("worlds", {}).get(str(world)) if prof else None
    fit = fit_alpha_beta(rows, op, world) if rows else None
    if fit is not None:
        return fit[0], fit[1], "measured"
    return DEFAULT_ALPHA_US, default_bus_gbps(world), "default"


def calibrate_fabric(device, sizes_mb=(4, 16, 64), iters: int = 5, dtype=None, group=None,
                     ops=("reduce_scatter", "all_reduce", "all_gather")) -> dict:
    """Time this job's own collectives before the engine builds its buckets: each op at each size,
    ``iters`` calls between a barrier + device sync (the MAX over ranks), then the alpha-beta fit of
    :func:`fit_alpha_beta` per op.  The fits replace the defaults / suite profile for this process
    (``measured_params`` source "calibrated"), so ``recommend_bucket_mb`` and the comm model use the
    fabric the job actually runs on -- the 8 x MI355X xGMI mesh at the driver's scaling runs, where
    no profile from a multi-GPU box exists yet.  Collective calls only (no process-group setup);
    ~0.1-0.3 s at 8 ranks.  Returns {"world", "rows": [...], "fits": {op: {"alpha_us", "bus_GBps"}}}
    (rows in the profile format of scripts/bench_collectives.py)."""
    import time
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    cuda = device.type == "cuda"
    dtype = dtype or (torch.bfloat16 if cuda else torch.float32)
    esz = torch.empty((), dtype=dtype).element_size()
    sync = (lambda: torch.cuda.synchronize(device)) if cuda else (lambda: None)
    rows = []
    for op in ops:
        for mb in sizes_mb:
            n = max(world, (int(mb * (1 << 20)) // esz) // world * world)
            full = torch.ones(n, dtype=dtype, device=device)
            part = torch.ones(n // world, dtype=dtype, device=device)
            if op == "reduce_scatter":
                call = lambda: dist.reduce_scatter_tensor(part, full, group=group)        # noqa: E731
            elif op == "all_gather":
                call = lambda: dist.all_gather_into_tensor(full, part, group=group)        # noqa: E731
            else:
                call = lambda: dist.all_reduce(full, group=group)                          # noqa: E731
            for _ in range(2):
                call()
            sync()
            dist.barrier(group=group)
            t0 = time.perf_counter()
            for _ in range(iters):
                call()
            sync()
            dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                              device=device if dist.get_backend(group) == "nccl" else "cpu")
            dist.all_reduce(dt, op=dist.ReduceOp.MAX, group=group)
            rows.append({"op": op, "bytes": n * esz, "time_us": float(dt.item()) / iters * 1e6,
                         "dtype": str(dtype).replace("torch.", "")})
            del full, part
    fits = {}
    for op in ops:
        fit = fit_alpha_beta(rows, op, world)
        if fit is not None:
            fits[op] = {"alpha_us": fit[0], "bus_GBps": fit[1]}
            _CALIBRATED[(world, op)] = fit
    return {"world": world, "rows": rows, "fits": fits}


DEFAULT_PG_HOST_US = {"reduce_scatter": 20.0, "all_gather": 20.0, "all_reduce": 20.0, "broadcast": 20.0,
                      "all_to_all": 20.0}
PG_HOST_PROFILE = os.path.join(_ROOT, "profiles", "pg_host_cost.json")


def pg_host_cost_us(path: str = None) -> dict:
    """Host microseconds of one ProcessGroupNCCL call per op (issue + wait), measured by
    scripts/probes/pg_host_cost.py on the real RCCL library (``profiles/pg_host_cost.json``);
    ``$DLTB_EMU_HOST_US`` overrides every op (0 disables), else DEFAULT_PG_HOST_US."""
    env = os.environ.get("DLTB_EMU_HOST_US")
    if env is not None:
        return {op: float(env) for op in DEFAULT_PG_HOST_US}
    out = dict(DEFAULT_PG_HOST_US)
    try:
        with open(path or os.environ.get("DLTB_PG_HOST_PROFILE") or PG_HOST_PROFILE) as f:
            per = json.load(f)["per_op_us"]
        for op in out:
            if op in per:
                out[op] = float(per[op])
        out["broadcast"] = out["all_gather"]
        out["all_to_all"] = out["all_gather"]
    except (OSError, ValueError, KeyError, TypeError):
        pass
    return out


def recommend_bucket_mb(world: int, overhead: float = 0.2, bus_gbps: float = None,
                        alpha_us: float = None, op: str = "reduce_scatter") -> float:
    """Smallest power-of-two MiB bucket with alpha <= overhead x transfer time, alpha and bus
    bandwidth from the measured sweep (``load_profile``) when it covers ``world``."""
    from .collectives import ring_factor
    if world <= 1:
        return 64.0
    if bus_gbps is None or alpha_us is None:
        a, b, _ = measured_params(world, op)
        alpha_us = a if alpha_us is None else alpha_us
        bus_gbps = b if bus_gbps is None else bus_gbps
    f = ring_factor(op, world)
    need = alpha_us / overhead * bus_gbps * 1e3 / f       # bytes
    mb = 1.0
    while mb * (1 << 20) < need and mb < BUCKET_MB_MAX:
        mb *= 2
    return min(mb, BUCKET_MB_MAX)


# Upper bound of the recommendation.  The replicated engines round a bucket up to whole groups of 4
# transformer blocks (the batched-dW size, parallel/replicated.py), so every value up to one such
# group (101 MB at TinyGPT-A) gives the same 4-block buckets that the emulated predictions were
# measured with, while a larger one doubles the group and halves the number of collectives that can
# overlap the backward.  An in-job 3-point fit (calibrate_fabric) with an inflated intercept -- a
# first-call or protocol-switch cost at the 4 MiB point -- must not push a job there.
BUCKET_MB_MAX = 64.0


def parse_topology(text: str):
    """Link-type matrix from ``rocm-smi --showtopotype`` output: {(i, j): 'XGMI' | 'PCIE' | ...}."""
    links = {}
    rows = [ln for ln in text.splitlines() if re.match(r"^\s*GPU\d+\s+(?!GPU)\S", ln)]
    for ln in rows:
        parts = ln.split()
        i = int(parts[0][3:])
        for j, tok in enumerate(parts[1:]):
            if tok in ("0", "-"):
                continue
            links[(i, j)] = tok.upper()
    return links


def query_topology():
    """Returns the link matrix of the visible GPUs, or None without rocm-smi."""
    exe = shutil.which("rocm-smi")
    if not exe:
        return None
    try:
        out = subprocess.run([exe, "--showtopotype"], capture_output=True, text=True, timeout=30,
                             env=dict(os.environ)).stdout
    except (OSError, subprocess.SubprocessError):
        return None
    return parse_topology(out) or None


def describe(world: int) -> dict:
    """Summary used in result sidecars and docs."""
    topo = query_topology()
    xgmi = sum(1 for v in (topo or {}).values() if v == "XGMI")
    alpha, bus, src = measured_params(world)
    return {"world": world, "xgmi_pairs": xgmi if topo else None,
            "links_per_gpu": XGMI_LINKS_PER_GPU, "link_GBps": XGMI_LINK_GBPS,
            "alpha_us": alpha, "bus_GBps": bus, "alpha_beta_source": src,
            "recommended_bucket_mb": recommend_bucket_mb(world)}
