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
import os
import re
import shutil
import subprocess

XGMI_LINKS_PER_GPU = 7
XGMI_LINK_GBPS = 153.0          # per direction, per link
DEFAULT_BUS_GBPS = 300.0        # conservative RCCL bus bandwidth per rank at 8 GPUs (large messages)
DEFAULT_ALPHA_US = 25.0         # fixed cost of one RCCL collective (launch + sync), 8 ranks


def collective_time_us(op: str, nbytes: int, world: int, bus_gbps: float = DEFAULT_BUS_GBPS,
                       alpha_us: float = DEFAULT_ALPHA_US) -> float:
    """alpha-beta estimate of one collective on ``nbytes`` (full buffer) at ``world`` ranks."""
    from .collectives import ring_factor
    if world <= 1:
        return 0.0
    return alpha_us + nbytes * ring_factor(op, world) / (bus_gbps * 1e3)


def recommend_bucket_mb(world: int, overhead: float = 0.2, bus_gbps: float = DEFAULT_BUS_GBPS,
                        alpha_us: float = DEFAULT_ALPHA_US, op: str = "reduce_scatter") -> float:
    """Smallest power-of-two MiB bucket with alpha <= overhead x transfer time."""
    from .collectives import ring_factor
    if world <= 1:
        return 64.0
    f = ring_factor(op, world)
    need = alpha_us / overhead * bus_gbps * 1e3 / f       # bytes
    mb = 1.0
    while mb * (1 << 20) < need and mb < 1024:
        mb *= 2
    return mb


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
    return {"world": world, "xgmi_pairs": xgmi if topo else None,
            "links_per_gpu": XGMI_LINKS_PER_GPU, "link_GBps": XGMI_LINK_GBPS,
            "recommended_bucket_mb": recommend_bucket_mb(world)}
