"""``parallel.rccl.FedAvgAllReduce`` (the bench's N-GPU aggregation, bench.py fl_round) rehearsed over gloo with
world_size 2 on the CPU: sample-weighted mean of the flat model across ranks (fl_server.py:92-105 semantics with the
north-star weighting), every bucket handed to ``on_bucket`` exactly once and the buckets tiling the flat buffer, and
the unweighted (reference) mean."""
import multiprocessing as mp
import os
import socket

import numpy as np


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, n, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from crack_detection_federatedlearning_grpc_amd.parallel.rccl import FedAvgAllReduce
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        flat = torch.randn(n, generator=g)
        own = flat.clone()
        agg = FedAvgAllReduce(flat, world=world, bucket_mb=0.01)       # small buckets: several of them
        seen = []
        ev = agg.average_async(float(10 * (rank + 1)), on_bucket=lambda sl: seen.append((sl.start, sl.stop)))
        weighted = flat.clone()
        flat.copy_(own)
        agg.average(0.0, weighted=False)
        q.put((rank, own.numpy(), weighted.numpy(), flat.numpy(), sorted(seen), len(ev)))
    finally:
        dist.destroy_process_group()


def test_fedavg_allreduce_weighted_and_uniform_gloo_world2():
    world, n = 2, 10_000
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    own = [r[1] for r in res]
    w = np.array([10.0, 20.0]) / 30.0
    want_w = w[0] * own[0] + w[1] * own[1]
    want_u = (own[0] + own[1]) / 2
    for _, _, weighted, uniform, seen, n_events in res:
        np.testing.assert_allclose(weighted, want_w, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(uniform, want_u, rtol=1e-5, atol=1e-6)
        assert n_events == 0                                  # CPU / gloo: synchronous, no HIP events
        assert len(seen) > 1 and seen[0][0] == 0 and seen[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(seen, seen[1:]))   # buckets tile the flat buffer
