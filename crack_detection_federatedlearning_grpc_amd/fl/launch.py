"""One-node FL launcher: the gRPC server + one client process per GPU.

    python -m crack_detection_federatedlearning_grpc_amd.fl.launch --num-clients 8 --preset gpu8-256

Replaces the reference's manual procedure (start ``fl_server.py``, then start N ``fl_client.py`` by hand on the
same host, all on one GPU - SURVEY §4). Each client process gets ``LOCAL_RANK`` = its GPU, registers over gRPC,
and - with ``--data-plane rccl`` - joins the RCCL communicator whose rendezvous the server hands out in the READY
reply; the FedAvg of every round is then a weighted all-reduce over xGMI. ``--device cpu`` runs the same topology
with gloo (CPU plumbing).
"""
from __future__ import annotations

import os
import subprocess
import sys
import time
from typing import List, Optional

from .. import config as _config

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    cfg = _config.parse(argv)
    n = cfg.num_clients or 1
    cfg.num_clients = n
    if cfg.data_plane == "rccl":
        from ..parallel.rccl import rccl_placement_error
        err = rccl_placement_error(n, cfg.device, cfg.dist_backend)
        if err:
            print(f"[launch] refused: {err}", file=sys.stderr, flush=True)
            return 2
    from .server import FLServer
    srv = FLServer(cfg)
    port = srv.start()
    print(f"[launch] server on :{port}, starting {n} client process(es) (data plane {cfg.data_plane})", flush=True)
    # the client processes share GPU memory over RCCL: the host driver only supports dmabuf IPC, and HSA reads
    # this at its initialisation, so each child gets it in its environment from the start (fl_client.py also
    # sets it before its first GPU call); plus the RCCL channel cap (parallel/rccl.py rccl_env)
    if cfg.data_plane == "rccl":
        from ..parallel.rccl import rccl_env
        env = rccl_env(os.environ, cfg.rccl_max_channels)
    else:
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    procs = []
    for r in range(n):
        e = dict(env, LOCAL_RANK=str(r), FL_PORT=str(port))
        extra = ["--port", str(port), "--host", "127.0.0.1"]
        if cfg.client_weight_file and n > 1:     # one trainer->driver hand-off file per client process
            root, ext = os.path.splitext(cfg.client_weight_file)
            extra += ["--client-weight-file", f"{root}.rank{r}{ext}"]
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "fl_client.py"), *argv, *extra], env=e))
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            time.sleep(0.5)
        rc = max(p.returncode or 0 for p in procs)
        srv.done.wait(5.0)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        srv.stop(0.5)
    hist = srv.state.history
    if hist:
        print(f"[launch] {len(hist)} round(s); last round wall-clock "
              f"{hist[-1].t_end - hist[-1].t_start:.2f}s; clients {hist[-1].clients}")
    return rc


if __name__ == "__main__":
    sys.exit(main())
