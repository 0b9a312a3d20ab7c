"""Single configuration object for server, client, trainer and bench.

The reference has no config system: every knob is a literal. Each literal becomes a field here,
with the reference value as the default, settable from the CLI (``--flag``) and the environment (``FL_FLAG``).

Reference literal sites (all in /root/reference):
  port 8889 ............ fl_server.py:218, fl_client.py:181
  worker threads 10 .... fl_server.py:216
  512 MiB recv limit ... fl_server.py:215, fl_client.py:179
  MAX_NUM_ROUND 5 ...... fl_server.py:18
  10 s window .......... fl_server.py:42       5 s READY stall ... fl_server.py:56
  20 s poll ............ fl_client.py:141      model_version 1 ... fl_server.py:17
  epochs 10 ............ client_fit_model.py:166   batch 16 ...... client_fit_model.py:56
  img 128x128 .......... client_fit_model.py:55,94 val split 6213 ... client_fit_model.py:76
  seed 1337 ............ client_fit_model.py:77-78 Adam/BCE/acc .. client_fit_model.py:157
  log chunk 100 MiB .... fl_client.py:36
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


@dataclass
class FLConfig:
    # --- transport / control plane -------------------------------------------------------------
    host: str = "localhost"              # client target host (fl_client.py:181)
    bind: str = "[::]"                   # server bind address (fl_server.py:218)
    port: int = 8889
    server_threads: int = 10
    max_message_mb: int = 512            # applied to BOTH send and receive (reference typo'd send, §A10)
    rpc_timeout_s: float = 600.0         # per-RPC deadline (reference: none, §A9)
    rpc_retries: int = 3

    # --- round state machine -------------------------------------------------------------------
    max_rounds: int = 5
    register_window_s: float = 10.0
    ready_stall_s: float = 5.0           # reference sleeps 5 s per READY; kept for compat, presets set 0
    num_clients: int = 0                 # >0: close registration as soon as this many registered
    poll_period_s: float = 20.0          # client VERSION poll period (upper bound; server long-polls)
    long_poll_s: float = 20.0            # server holds a VERSION request this long waiting for a new version
    initial_model_version: int = 1
    round_deadline_s: float = 0.0        # 0 = wait forever (reference); >0 = drop stragglers at deadline
    quorum: float = 1.0                  # fraction of registered clients needed at the deadline
    model_type: str = "unet"             # advertised in READY reply; client ignores it (as reference)
    aggregation: str = "weighted"        # weighted (n_k) | uniform (reference mean)
    data_plane: str = "grpc"             # grpc | rccl
    rccl_timeout_s: float = 300.0        # collective timeout; on expiry / peer loss the client aborts the
                                         # communicator and falls back to the gRPC data plane
    dist_backend: str = "nccl"           # rccl data plane backend: nccl (= RCCL over xGMI) | gloo (CPU clients, or
                                         # a rehearsal of N clients sharing one GPU, which RCCL refuses)
    rccl_max_channels: int = -1          # RCCL channel cap (= workgroups an all-reduce occupies): -1 = env
                                         # CFL_RCCL_MAX_CHANNELS or 16 (parallel/rccl.py), 0 = RCCL's own choice
    dist_addr: str = "127.0.0.1"         # rendezvous address the server hands the clients in its READY reply (the
                                         # rank-0 client's TCPStore host; 127.0.0.1 = every client on this node)
    async_upload: bool = True           # rccl data plane: after a successful collective the client starts the next
                                         # round at once and reports TRAIN_DONE (rank 0: + the average) from a
                                         # background thread; its reply is checked before the next report
    codec: str = "flat"                  # client upload / advertised reply format: flat (safe) | pickle (reference
                                         # wire format). The server answers each client in the format it
                                         # advertised, pickle for a reference client that advertises none
    wire_dtype: str = "fp32"             # fp32 | bf16 for the flat codec

    # --- local training ------------------------------------------------------------------------
    epochs: int = 10
    steps_per_epoch: int = 0             # 0 = len(train)//batch (reference Sequence.__len__)
    batch_size: int = 16                 # 0 = planned: largest batch that fits hbm_fraction of HBM (models/memplan.py)
    hbm_fraction: float = 0.85           # HBM share the batch planner may fill (engine + resident dataset shard)
    img_size: int = 128
    val_samples: int = 6213              # reference: FIRST 6213 are train (client_fit_model.py:79)
    shuffle_seed: int = 1337
    lr: float = 1e-3
    beta1: float = 0.9
    beta2: float = 0.999
    adam_eps: float = 1e-7
    bn_momentum: float = 0.99
    bn_eps: float = 1e-3
    loss: str = "bce"                    # bce (reference) | bce_dice
    validate: bool = True
    predict_round: int = 5               # client_fit_model.py:235 (cr == 5)
    device: str = "auto"                 # auto | cpu | cuda
    dtype: str = "bf16"                  # activation dtype on the GPU path (fp32 master weights)
    conv_dtype: str = "bf16"             # bf16 | fp8: decoder 3x3 convs (ConvT fwd + dgrad) on the block-scaled fp8
                                         # MFMA (csrc/kernels/fp8.hip; BASELINE config 5)
    use_graph: bool = True               # capture the train step in a hipGraph
    deterministic: bool = False          # int64 fixed-point cross-block reductions: bitwise-reproducible local
                                         # training (models/engine.py; ~1.4-2.7 % slower, profiles/README.md)

    # --- data ------------------------------------------------------------------------------------
    data: str = "synthetic"              # synthetic | folder
    train_image_dir: str = ""
    train_mask_dir: str = ""
    predict_dir: str = ""
    synthetic_samples: int = 8000        # synthetic dataset size (train+val) per client
    data_seed: int = 0

    # --- persistence / observability -------------------------------------------------------------
    work_dir: str = "."
    client_weight_file: str = "./saved_weight/weights.pickle"
    final_weight_file: str = ""          # where a client writes the model it holds at FIN (rccl data plane: the
                                         # final global average; "" = not written)
    server_weight_file: str = "./server_weights/weights.pickle"
    log_dir: str = "send_logs/logs"
    metrics_file: str = ""               # JSONL metrics sink ("" = stdout only)
    tensorboard: bool = False            # Keras-style tfevents per round under log_dir (client_fit_model.py:153-154)
    histogram_freq: int = 1              # weight histograms every N epochs (the reference's histogram_freq=1)
    upload_logs: bool = False
    log_chunk_mb: int = 100
    snapshot_dir: str = ""               # server per-round snapshot (.h5 + state json) for --resume
    resume: bool = False
    seed: int = 0

    # --- fault injection (tests) ---------------------------------------------------------------
    fault_drop_round: int = 0            # client exits (crash) when this round starts
    fault_delay_s: float = 0.0           # client sleeps before TRAIN_DONE
    fault_corrupt: bool = False          # client sends a corrupted payload

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


PRESETS: Dict[str, Dict[str, Any]] = {
    # BASELINE.json config 1: 2-client FedAvg over gRPC on CPU, tiny U-Net 64x64, synthetic masks.
    "cpu-plumbing": dict(device="cpu", img_size=64, batch_size=4, epochs=1, steps_per_epoch=2,
                         synthetic_samples=48, val_samples=32, register_window_s=3.0, ready_stall_s=0.0,
                         num_clients=2, poll_period_s=0.5, long_poll_s=2.0, dtype="fp32", use_graph=False),
    # config 2: single-client U-Net 256x256 bf16 local fit on one MI355X.
    "gpu1-256": dict(device="cuda", img_size=256, batch_size=16, ready_stall_s=0.0, num_clients=1,
                     register_window_s=1.0, poll_period_s=0.5, long_poll_s=20.0),
    # config 3: 8 clients, RCCL weighted all-reduce.
    "gpu8-256": dict(device="cuda", img_size=256, batch_size=16, ready_stall_s=0.0, num_clients=8,
                     register_window_s=30.0, data_plane="rccl", poll_period_s=0.5, long_poll_s=20.0),
    # config 4: 512x512 large batch, activation memory sized for 288 GB HBM.
    "gpu8-512": dict(device="cuda", img_size=512, batch_size=0, ready_stall_s=0.0, num_clients=8,
                     register_window_s=30.0, data_plane="rccl", poll_period_s=0.5),
    # config 5: config 4 with the block-scaled fp8 ConvT path (+ the asynchronous RCCL aggregation of every rccl run)
    "gpu8-512-fp8": dict(device="cuda", img_size=512, batch_size=0, ready_stall_s=0.0, num_clients=8,
                         register_window_s=30.0, data_plane="rccl", poll_period_s=0.5, conv_dtype="fp8"),
}


def _coerce(v: str, typ: Any) -> Any:
    if typ is bool or typ == "bool":
        return str(v).lower() in ("1", "true", "yes", "on")
    if typ is int or typ == "int":
        return int(v)
    if typ is float or typ == "float":
        return float(v)
    return v


def add_arguments(p: argparse.ArgumentParser) -> None:
    p.add_argument("--preset", default=os.environ.get("FL_PRESET", ""), choices=[""] + sorted(PRESETS))
    for f in dataclasses.fields(FLConfig):
        flag = "--" + f.name.replace("_", "-")
        if f.type in ("bool", bool):
            p.add_argument(flag, dest=f.name, default=None, type=lambda s: _coerce(s, bool), nargs="?", const=True)
        else:
            typ = {"int": int, "float": float, "str": str}.get(f.type if isinstance(f.type, str) else "", None)
            p.add_argument(flag, dest=f.name, default=None, type=typ or str)


def from_args(ns: Optional[argparse.Namespace] = None, **overrides: Any) -> FLConfig:
    """defaults < preset < FL_* environment < CLI flags < explicit overrides."""
    cfg = FLConfig()
    preset = getattr(ns, "preset", "") if ns is not None else overrides.pop("preset", "")
    preset = preset or os.environ.get("FL_PRESET", "")
    if preset:
        for k, v in PRESETS[preset].items():
            setattr(cfg, k, v)
    for f in dataclasses.fields(FLConfig):
        env = os.environ.get("FL_" + f.name.upper())
        if env is not None:
            setattr(cfg, f.name, _coerce(env, f.type))
        if ns is not None and getattr(ns, f.name, None) is not None:
            setattr(cfg, f.name, getattr(ns, f.name))
    for k, v in overrides.items():
        if not hasattr(cfg, k):
            raise KeyError(f"unknown config key {k}")
        setattr(cfg, k, v)
    return cfg


def parse(argv: Optional[List[str]] = None, **overrides: Any) -> FLConfig:
    p = argparse.ArgumentParser()
    add_arguments(p)
    ns = p.parse_args(argv)
    return from_args(ns, **overrides)
