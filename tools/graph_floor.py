"""Per-kernel floor inside a replayed hipGraph on this device: N tiny launches (1-element add, and a 1-block
1024-thread kernel of the engine's bn_finalize shape) captured in one graph; wall time per launch."""
import json
import time

import torch


def per_launch(fn, n=200, reps=20):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (reps * n) * 1e6


x = torch.zeros(1, device="cuda")
big = torch.zeros(1 << 20, device="cuda")
print(json.dumps({"tiny_add_us": round(per_launch(lambda: x.add_(1.0)), 2),
                  "add_4MB_us": round(per_launch(lambda: big.add_(1.0)), 2)}))
