"""Process-group setup / teardown (reference: setup_distributed / cleanup_distributed,
train_harness.py:186-204).

Rank / world / local rank come from the torchrun environment (RANK, WORLD_SIZE, LOCAL_RANK,
MASTER_ADDR, MASTER_PORT) and may be overridden by the reference's explicit CLI flags.  On MI355X
the backend is "nccl", which on ROCm *is* RCCL (collectives over xGMI); on CPU it is gloo.  Unlike
the reference, an explicit collective timeout is always passed and the
single-process case still works for every strategy (the reference's FSDP crashes at WS=1).
"""
import datetime
import os

import torch
import torch.distributed as dist


def env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def resolve_ranks(world_size=None, rank=None, local_rank=None):
    world = world_size if world_size is not None else env_int("WORLD_SIZE", 1)
    r = rank if rank is not None else env_int("RANK", 0)
    lr = local_rank if local_rank is not None else env_int("LOCAL_RANK", 0)
    if os.environ.get("WORLD_SIZE") and world_size is not None and int(os.environ["WORLD_SIZE"]) != world_size:
        raise ValueError(f"--world-size {world_size} disagrees with WORLD_SIZE={os.environ['WORLD_SIZE']}")
    return world, r, lr


def setup_distributed(world_size, rank, local_rank, master_addr=None, master_port=None,
                      device_type="cuda", timeout_min=30, debug_collectives=False, force_pg=False):
    """Initialise the process group when world_size > 1 (or ``force_pg``: a one-rank group, which
    runs the RCCL init options and collectives on a one-GPU box); returns this rank's torch.device."""
    host_comm = device_type == "cuda" and os.environ.get("DLTB_COMM", "rccl") == "host"
    if device_type == "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("no GPU visible (use --device cpu for the gloo/CPU path)")
        if host_comm:     # ranks may outnumber the GPUs: they share them round-robin
            local_rank = local_rank % torch.cuda.device_count()
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    if (world_size > 1 or force_pg) and not dist.is_initialized():
        if debug_collectives:
            os.environ["TORCH_DISTRIBUTED_DEBUG"] = "DETAIL"
        if master_addr:
            os.environ.setdefault("MASTER_ADDR", master_addr)
        if master_port:
            os.environ.setdefault("MASTER_PORT", str(master_port))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        # DLTB_COMM=host: gloo with host-staged device buffers (comm/collectives.py), so several
        # ranks can share one GPU (tests of the world > 1 paths on a one-GPU box)
        backend = "nccl" if (device_type == "cuda" and not host_comm) else "gloo"
        kw = dict(backend=backend, init_method="env://", world_size=world_size, rank=rank,
                  timeout=datetime.timedelta(minutes=timeout_min))
        if backend == "nccl":
            kw["device_id"] = device
            if os.environ.get("DLTB_COMM_HIGH_PRIORITY", "1") == "1":
                # RCCL's internal stream at high priority: when bucket collectives and backward
                # kernels are both queued, the dispatcher places the collective's workgroups first,
                # so the reduce-scatter / all-gather progresses under the compute instead of behind it
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                kw["pg_options"] = opts
        dist.init_process_group(**kw)
        if backend == "nccl":          # warm the communicator up outside the timed region
            t = torch.ones(1, device=device)
            dist.all_reduce(t)
            torch.cuda.synchronize(device)
        print(f"[Rank {rank}/{world_size}] Distributed initialized ({backend})", flush=True)
    elif world_size == 1:
        print("Single-GPU mode (no distributed)" if device_type == "cuda" else "Single-process CPU mode",
              flush=True)
    return device


def cleanup_distributed():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def barrier():
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def all_reduce_max(x: float, device) -> float:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        host = dist.get_backend() == "gloo"
        t = torch.tensor([x], dtype=torch.float64, device="cpu" if host else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return x
