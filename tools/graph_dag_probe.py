"""Can two independent kernels of ONE captured stream run concurrently? During stream capture the next node's
dependency set is rewritten (hipStreamUpdateCaptureDependencies) so kernel B depends on A's predecessors instead of
on A, and the kernel after them on both: a DAG branch without a second stream (tools/graph_fork_probe.py: a stream
fork / join in a replayed graph costs ~75 us). Times replays of a linear chain vs the same chain with sibling pairs,
and a pair of long-running kernels (sleep) linear vs siblings to see whether siblings overlap at all.

    python tools/graph_dag_probe.py
"""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipStreamGetCaptureInfo_v2.restype = ctypes.c_int
hip.hipStreamUpdateCaptureDependencies.restype = ctypes.c_int


def deps(stream):
    status = ctypes.c_int(0)
    cid = ctypes.c_ulonglong(0)
    graph = ctypes.c_void_p()
    dptr = ctypes.POINTER(ctypes.c_void_p)()
    n = ctypes.c_size_t(0)
    rc = hip.hipStreamGetCaptureInfo_v2(ctypes.c_void_p(stream), ctypes.byref(status), ctypes.byref(cid),
                                        ctypes.byref(graph), ctypes.byref(dptr), ctypes.byref(n))
    assert rc == 0, rc
    return [dptr[i] for i in range(n.value)]


def set_deps(stream, nodes, add=False):
    arr = (ctypes.c_void_p * max(1, len(nodes)))(*nodes)
    rc = hip.hipStreamUpdateCaptureDependencies(ctypes.c_void_p(stream), arr, ctypes.c_size_t(len(nodes)),
                                                 ctypes.c_uint(0 if add else 1))
    assert rc == 0, rc


def build(kind, n=60, pairs=10, sleep_cycles=0):
    dev = torch.device("cuda")
    x = torch.randn(1 << 20, device=dev)
    ys = [torch.empty_like(x) for _ in range(2 * n)]
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device=dev)

    def body(capture):
        st = torch.cuda.current_stream().cuda_stream
        prev = x
        i = 0
        k = 0
        while i < n:
            if kind == "dag" and k < pairs and capture and i % (n // pairs) == 0:
                d0 = deps(st)
                if sleep_cycles:
                    torch.cuda._sleep(sleep_cycles)
                else:
                    torch.add(prev, 1.0, out=ys[i])
                a = deps(st)
                set_deps(st, d0)
                if sleep_cycles:
                    torch.cuda._sleep(sleep_cycles)
                else:
                    torch.mul(prev, 2.0, out=ys[n + i])
                set_deps(st, a, add=True)
                prev = ys[i]
                k += 1
                i += 1
                continue
            if kind in ("linear", "dag") and k < pairs and i % (n // pairs) == 0:
                if sleep_cycles:
                    torch.cuda._sleep(sleep_cycles)
                    torch.cuda._sleep(sleep_cycles)
                else:
                    torch.add(prev, 1.0, out=ys[i])
                    torch.mul(prev, 2.0, out=ys[n + i])
                prev = ys[i]
                k += 1
                i += 1
                continue
            torch.add(prev, 1.0, out=ys[i])
            prev = ys[i]
            i += 1

    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body(False)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        body(True)
    return g


def timeit(g, reps=100):
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


if __name__ == "__main__":
    for sl in (0, 200_000):
        lin = timeit(build("linear", sleep_cycles=sl))
        dag = timeit(build("dag", sleep_cycles=sl))
        print(f"sleep {sl}: 60-kernel chain with 10 pairs: linear {lin:.1f} us, siblings {dag:.1f} us per replay",
              flush=True)
