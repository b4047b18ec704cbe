"""Shared helpers of the GEMM microbenchmarks: the per-layer products of a model and a graph-replay timer."""
import torch


def products(model):
    if model == "A":
        M, d, f = 2048, 1024, 4096
        return M, [("qkv.fwd", 3 * d, d, True), ("out.fwd", d, d, True), ("fc1.fwd", f, d, True),
                   ("fc2.fwd", d, f, True), ("fc2.dgrad", f, d, False), ("fc1.dgrad", d, f, False),
                   ("out.dgrad", d, d, False), ("qkv.dgrad", d, 3 * d, False)]
    M, d, f, kv = 4096, 4096, 14336, 1024
    return M, [("qkv.fwd", d + 2 * kv, d, False), ("o.fwd", d, d, False), ("gateup.fwd", 2 * f, d, False),
               ("down.fwd", d, f, False), ("down.dgrad", f, d, False), ("gateup.dgrad", d, 2 * f, False),
               ("o.dgrad", d, d, False), ("qkv.dgrad", d, d + 2 * kv, False)]


def graph_time(fns, iters, rounds=5):
    """Per-call GPU time of each fn (median over rounds, the fns interleaved in every round)."""
    graphs = []
    for fn in fns:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        graphs.append(g)
    times = [[] for _ in fns]
    for _ in range(rounds):
        for i, g in enumerate(graphs):
            g.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            times[i].append(s.elapsed_time(e) / iters * 1e3)
    return [sorted(t)[len(t) // 2] for t in times]
