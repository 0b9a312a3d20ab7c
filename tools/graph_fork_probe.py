"""Cost of a fork / join inside a captured hipGraph (a second stream branch) on this ROCm build.

Captures (a) a chain of N small elementwise kernels on one stream and (b) the same chain with K kernels moved onto
a side stream (forked after kernel F, joined back after kernel F + J), and times graph replays of each.

    python tools/graph_fork_probe.py [N] [K]
"""
import sys
import time

import torch


def run(n=60, k=8, reps=200, side_prio=0):
    dev = torch.device("cuda")
    x = torch.randn(1 << 20, device=dev)
    ys = [torch.empty_like(x) for _ in range(n)]
    zs = [torch.empty_like(x) for _ in range(k)]
    side = torch.cuda.Stream(device=dev, priority=side_prio)

    def chain(fork: bool):
        cur = torch.cuda.current_stream()
        prev = x
        for i in range(n):
            if fork and i == n // 2:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    a = prev
                    for j in range(k):
                        torch.mul(a, 1.0001, out=zs[j])
                        a = zs[j]
            torch.add(prev, 1.0, out=ys[i])
            prev = ys[i]
            if fork and i == n // 2 + k:
                cur.wait_stream(side)
        return prev

    out = {}
    for fork in (False, True):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            chain(fork)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            chain(fork)
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        out["fork" if fork else "linear"] = (time.perf_counter() - t0) / reps * 1e6
    return out


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    for prio in (0, -1):
        r = run(n, k, side_prio=prio)
        print(f"N={n} kernels, K={k} on the side stream (priority {prio}): linear {r['linear']:.1f} us / replay, "
              f"fork-join {r['fork']:.1f} us / replay", flush=True)
