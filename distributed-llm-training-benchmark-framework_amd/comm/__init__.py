"""Communication layer: RCCL (torch.distributed "nccl" on ROCm) over xGMI, or gloo on the CPU."""
from .collectives import Comm, ring_factor
from .topology import collective_time_us, describe, parse_topology, recommend_bucket_mb

__all__ = ["Comm", "ring_factor", "collective_time_us", "describe", "parse_topology", "recommend_bucket_mb"]
