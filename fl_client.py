"""FL client entry point - drop-in for the reference's ``python fl_client.py`` (/root/reference/fl_client.py).

Connects to ``localhost:8889`` by default, registers with a random ``client<N>`` name, and runs the
READY -> PARAM -> TRAINING -> train -> TRAIN_DONE loop until FIN. Local training runs on the MI355X engine when a
GPU is visible (one process per GPU; ``--device cuda``), else on the fp32 CPU reference.
The request builders below keep the reference's names and message shapes (fl_client.py:14-74).
"""
from __future__ import annotations

import os
import random
import sys
from typing import List, Optional

# multi-rank GPU work (RCCL, CUDA-tensor sharing between processes): the host driver only supports dmabuf IPC, so
# the legacy IPC mode must be off - HSA reads this once, at its initialisation, so it is set before this process
# makes any GPU call (with legacy IPC RCCL fails with "hipIpcGetMemHandle: invalid argument")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

from crack_detection_federatedlearning_grpc_amd import config as _config
from crack_detection_federatedlearning_grpc_amd.fl import codec
from crack_detection_federatedlearning_grpc_amd.fl import proto as P
from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
from crack_detection_federatedlearning_grpc_amd.fl.rpc import TransportServiceStub, channel_options

client_name = ""


def request_parameter():
    """fl_client.py:14-17."""
    yield P.transportRequest(update_req=P.UpdateReq(type="P"))


def request_ready():
    """fl_client.py:20-29."""
    global client_name
    client_name = f"client{random.randint(1, 100000)}"
    yield P.transportRequest(ready_req=P.ReadyReq(type="R", cname=client_name, state=P.ON,
                                                  config={"current_round": P.Scalar(scint32=0)}))


def get_file_chunks(filename, chunk_mb: int = 100):
    """fl_client.py:35-43."""
    with open(filename, "rb") as f:
        while True:
            piece = f.read(chunk_mb * 1024 * 1024)
            if not piece:
                return
            yield P.transportRequest(update_req=P.UpdateReq(type="L", buffer_chunk=piece, title=filename,
                                                            file_len=len(piece)))


def send_logs(stub, in_file_name):
    """fl_client.py:46-50."""
    for lr in stub.transport(get_file_chunks(in_file_name)):
        print(f"Finish deliver file: {lr.update_rep.title}, type: {lr.update_rep.type}")


def request_training(nclient):
    """fl_client.py:55-58."""
    yield P.transportRequest(update_req=P.UpdateReq(type="T", cname=nclient, state=P.TRAINING))


def request_traindone(nclient, cr, bc, n_samples: int = 0, codec_name: str = "pickle"):
    """fl_client.py:61-65 (``bc`` = list of weight arrays; pickled like the reference by default)."""
    yield P.transportRequest(update_req=P.UpdateReq(type="D", buffer_chunk=codec.encode(bc, codec_name),
                                                    state=P.TRAIN_DONE, cname=nclient, current_round=cr,
                                                    file_len=n_samples))


def request_model_version(mv, cr):
    """fl_client.py:68-74."""
    yield P.transportRequest(version_req=P.VersionReq(type="P", config={"model_version": P.Scalar(scint32=mv),
                                                                        "current_round": P.Scalar(scint32=cr)}))


def make_client(cfg, name: Optional[str] = None, rank: int = 0) -> FLClient:
    from crack_detection_federatedlearning_grpc_amd.train.factory import make_trainer
    name = name or f"client{random.randint(1, 100000)}"
    agg_factory = None
    if cfg.data_plane == "rccl":
        from crack_detection_federatedlearning_grpc_amd.parallel.rccl import RcclAggregator
        agg_factory = lambda info: RcclAggregator.from_ready_info(info, cfg)  # noqa: E731
    return FLClient(cfg, lambda: make_trainer(cfg, name, rank), name=name, aggregator_factory=agg_factory)


def send_message(stub=None, cfg=None):
    """fl_client.py:77-175 - the whole client loop."""
    cfg = cfg or _config.FLConfig()
    return make_client(cfg).run()


def run(cfg=None):
    """fl_client.py:178-183."""
    cfg = cfg or _config.FLConfig()
    rank = int(os.environ.get("LOCAL_RANK", "0"))
    if cfg.data_plane == "rccl":
        # one GPU per RCCL client: refused here, before any GPU call, instead of rank % device_count putting two
        # ranks on one card (RCCL would fail only at the first collective, after a round of training)
        from crack_detection_federatedlearning_grpc_amd.parallel.rccl import rccl_placement_error
        err = rccl_placement_error(0, cfg.device, cfg.dist_backend, rank=rank)
        if err:
            raise SystemExit(f"fl_client: {err}")
    if cfg.device in ("cuda", "auto"):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.set_device(rank % torch.cuda.device_count())
        except Exception:
            pass
    return make_client(cfg, rank=rank).run()


def main(argv: Optional[List[str]] = None) -> int:
    cfg = _config.parse(argv)
    state = run(cfg)
    return 0 if state == "FIN" else 1


if __name__ == "__main__":
    sys.exit(main())
