#!/usr/bin/env python3
"""Can RCCL collectives be captured in a HIP graph on this stack?  Runs with torchrun (any world
size, 1 included): captures async all_reduce / reduce_scatter_tensor / all_gather_into_tensor +
wait on the current stream, replays twice and checks the results.  Prints one JSON line per rank."""
import json
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    n = 1 << 20
    x = torch.full((n,), float(rank + 1), device=dev, dtype=torch.bfloat16)
    y = torch.empty(n * world, device=dev, dtype=torch.bfloat16)
    rs = torch.empty(n // world, device=dev, dtype=torch.bfloat16)
    big = torch.zeros(n * world, device=dev, dtype=torch.bfloat16)
    # warm-up (communicator init) outside capture
    dist.all_reduce(x.clone())
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    ok, err = True, ""
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            a = x * 2
            w1 = dist.all_reduce(a, async_op=True)
            w1.wait()
            big.copy_(a.repeat(world))
            w2 = dist.reduce_scatter_tensor(rs, big[: n], async_op=True)
            w2.wait()
            w3 = dist.all_gather_into_tensor(y, a, async_op=True)
            w3.wait()
        for _ in range(2):
            g.replay()
        torch.cuda.synchronize()
        tot = sum(2 * (r + 1) for r in range(world))
        ok = bool((a == tot).all()) and bool((y == tot).all()) and bool((rs == tot * world).all())
    except Exception as e:  # noqa: BLE001
        ok, err = False, repr(e)[:300]
    print(json.dumps({"rank": rank, "world": world, "graph_capture_ok": ok, "error": err}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
