"""One-node rank launcher: ``python bench.py --gpus N`` without torchrun.

The headline metric is defined at 8 clients (BASELINE.json), and the reference has no launcher at all - its clients
were started by hand (`/root/reference/fl_client.py:178-188`). ``spawn_local_ranks`` starts N fresh child processes
of the same script, one per GPU, each with the torch.distributed environment (``RANK``, ``LOCAL_RANK``,
``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``, ``MASTER_ADDR`` = 127.0.0.1, a free ``MASTER_PORT``) set before it starts, so no
child inherits any GPU state from the parent (the parent makes no GPU call and never execs). Rank 0's stdout is
relayed to the parent's stdout line by line (the bench's JSON result), every other rank's stdout goes to stderr, and
stderr is inherited. The parent exits non-zero if any child fails or the whole run exceeds ``timeout``; the first
failure terminates the other ranks' process groups (each child is started in its own session, so exactly the
processes this launcher started are signalled).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional, Sequence


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket() as so:
        so.bind((host, 0))
        return int(so.getsockname()[1])


def _relay(stream, out, prefix: str) -> None:
    for line in iter(stream.readline, ""):
        out.write(line if not prefix else prefix + line)
        out.flush()
    stream.close()


def spawn_local_ranks(script: str, argv: Sequence[str], nproc: int, *, timeout: Optional[float] = None,
                      env: Optional[dict] = None, master_port: Optional[int] = None,
                      poll_s: float = 0.2) -> int:
    """Run ``python script *argv`` as ``nproc`` ranks of one node; returns 0 iff every rank exited 0."""
    if nproc < 1:
        raise ValueError(f"nproc must be >= 1, got {nproc}")
    base = dict(os.environ if env is None else env)
    # dmabuf IPC only on this host driver: HSA reads this at its initialisation, so every rank gets it from the start
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    port = master_port or free_port()
    procs: List[subprocess.Popen] = []
    relays: List[threading.Thread] = []
    for r in range(nproc):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PYTHONUNBUFFERED="1")
        p = subprocess.Popen([sys.executable, script, *argv], env=e, stdout=subprocess.PIPE, text=True,
                             start_new_session=True)
        procs.append(p)
        t = threading.Thread(target=_relay, args=(p.stdout, sys.stdout if r == 0 else sys.stderr,
                                                   "" if r == 0 else f"[rank {r}] "), daemon=True)
        t.start()
        relays.append(t)
    t0 = time.monotonic()
    rc = 0
    failed = None
    completed = False                       # every rank exited 0: nothing to stop
    prev_term = None

    def _on_term(signum, _frame):           # a SIGTERM to the launcher stops the ranks through the finally below
        raise SystemExit(128 + signum)
    if threading.current_thread() is threading.main_thread():
        prev_term = signal.signal(signal.SIGTERM, _on_term)
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                failed = bad[0]
                rc = 1
                break
            if all(c == 0 for c in codes):
                completed = True
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                failed = (-1, "timeout")
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        if prev_term is not None:
            signal.signal(signal.SIGTERM, prev_term)
        if not completed:
            # a failed rank, the timeout, Ctrl-C or a SIGTERM / any exception in the loop above: the children run in
            # their own sessions (no terminal signal reaches them), so stop every live rank's process group here
            for p in procs:
                if p.poll() is None:
                    try:
                        os.killpg(p.pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
            deadline = time.monotonic() + 10.0
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, deadline - time.monotonic()))
                except subprocess.TimeoutExpired:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except ProcessLookupError:
                        pass
                    p.wait()
        for t in relays:
            t.join(timeout=5.0)
    if failed is not None:
        who = "the run timed out" if failed[0] < 0 else f"rank {failed[0]} exited with {failed[1]}"
        print(f"[spawn] {who}; stopped the other ranks", file=sys.stderr, flush=True)
    return rc
