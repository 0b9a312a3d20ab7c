"""FL server entry point - drop-in for the reference's ``python fl_server.py`` (/root/reference/fl_server.py).

Defaults equal the reference literals (port 8889, 10 worker threads, 5 rounds, 10 s registration window, 5 s READY
stall); every literal is a flag / FL_* env var (crack_detection_federatedlearning_grpc_amd/config.py), e.g.
``python fl_server.py --preset cpu-plumbing`` or ``--num-clients 8 --data-plane rccl``.

Module-level names mirror the reference's functions (fl_server.py:23-226) over one locked server object.
"""
from __future__ import annotations

import sys
from typing import List, Optional

import numpy as np

from crack_detection_federatedlearning_grpc_amd import config as _config
from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer
from crack_detection_federatedlearning_grpc_amd.parallel.fedavg import fedavg_lists

SERVER: Optional[FLServer] = None
MAX_NUM_ROUND = 5


class TransportService(FLServer):
    """fl_server.py:209-212 - the servicer; ``transport`` dispatches every verb."""


def send_parameter() -> bytes:
    """fl_server.py:23-24 (the reference pickle a reference client unpickles)."""
    return SERVER.send_parameter(("pickle", "fp32"))


def ready_client(name, config):
    """fl_server.py:45-81 (returns the reply config as plain values)."""
    cr = config["current_round"].scint32 if hasattr(config["current_round"], "scint32") else int(config["current_round"])
    return SERVER.state.ready(name, cr)


def manage_rounds(nclient, current_round, buffer_chunk, n_samples: float = 1.0) -> str:
    """fl_server.py:107-135: returns RESP_ACY / RESP_ARY / FIN (never None)."""
    flat = SERVER.table.from_list(buffer_chunk) if buffer_chunk is not None else None
    return SERVER.state.submit(nclient, current_round, flat, n_samples)[0]


def version_check(Mversion, Cround):
    """fl_server.py:138-149."""
    return SERVER.state.version(Mversion, Cround)


def updateWeight(lists, weights=()):
    """fl_server.py:92-105 as a pure function over a list of client weight lists."""
    return fedavg_lists(lists, weights)


def serve(cfg=None) -> FLServer:
    """fl_server.py:214-226: build the global model, start gRPC, block until FIN (or Ctrl-C)."""
    global SERVER
    cfg = cfg or _config.FLConfig()
    evaluator = None
    try:
        import model_evaluate
        evaluator = model_evaluate.server_evaluator(cfg)
    except Exception as e:  # evaluation is optional (reference: commented out, fl_server.py:65)
        print(f"[fl_server] server-side evaluation disabled: {e}")
    SERVER = FLServer(cfg, evaluator=evaluator)
    port = SERVER.start()
    print(f"[fl_server] listening on {cfg.bind}:{port} ({cfg.max_rounds} rounds, window {cfg.register_window_s}s, "
          f"data plane {cfg.data_plane}, replies in each client's advertised codec, pickle by default)")
    SERVER.serve_forever(exit_on_fin=True)
    return SERVER


def main(argv: Optional[List[str]] = None) -> int:
    cfg = _config.parse(argv)
    serve(cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
