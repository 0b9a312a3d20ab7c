"""FL server: gRPC servicer over the locked ``RoundState``.

Reference: fl_server.py. Same single bidi-stream RPC and verbs (dispatcher fl_server.py:152-207):
  ready_req.type  'R'          -> registration (SW/CTW)                              :154-157
  update_req.type 'P'          -> global parameters                                  :158-161
  update_req.type 'T'          -> training ack (used here as a heartbeat)            :162-169
  update_req.type 'L'          -> log-file chunk upload (appends; reference truncates, §A7)   :170-175
  update_req.type 'D'          -> TRAIN_DONE + weights -> RESP_ACY / RESP_ARY(+params) / FIN  :176-196
  version_req.type 'P'         -> WAIT / NOT_WAIT(+params) / FIN                     :197-207
Extra READY reply keys (ignored by reference clients): ``rank``, ``world_size``, ``dist_addr``, ``dist_port``,
``data_plane`` - the server doubles as the RCCL rendezvous for on-node GPU clients.
``UpdateReq.file_len`` on a 'D' request carries the client's sample count n_k for weighted FedAvg, and
``UpdateReq.title`` = "rccl" says the client's local model already holds the round's average (the RCCL data plane
reduced it on the GPUs): its RESP_ARY / NOT_WAIT replies then carry no parameters (8.2 MB per client per round the
client would discard).

Reply codec per client (drop-in compatibility): a reference client ``pickle.loads`` whatever arrives in
``buffer_chunk`` (client_fit_model.py:51,231) and never says what it can read, so parameters go out as the
reference pickle unless the client advertised the flat codec - a ``codec`` (+ ``wire_dtype``) key in its READY
config, or in the VERSION config / a ``cname`` on the PARAM request that identifies a client that did. A client
whose TRAIN_DONE payload was a pickle is answered in pickle from then on.
"""
from __future__ import annotations

import json
import os
import threading
import time
from concurrent import futures
from typing import Callable, Dict, Optional

import grpc
import numpy as np

from ..config import FLConfig
from ..models.spec import ParamTable
from . import codec
from . import proto as P
from .rpc import TransportServiceServicer, add_TransportServiceServicer_to_server, channel_options
from .state import CTW, FIN, NOT_WAIT, RESP_ACY, RESP_ARY, SW, WAIT, RoundRecord, RoundState


class LatestWorker:
    """One worker thread that runs the NEWEST submitted job: a job submitted while another waits replaces it (a
    round's snapshot / evaluation supersedes the previous round's if that one has not started yet), so slow disk
    or a slow evaluator never queues one 8 MB model copy per round. ``flush`` waits until the worker is idle;
    ``close(cancel)`` drops (or, cancel=False, runs) the pending job and joins the thread."""

    def __init__(self, name: str):
        self._cv = threading.Condition()
        self._job: Optional[Callable[[], None]] = None
        self._busy = False
        self._closed = False
        self._t = threading.Thread(target=self._loop, name=name, daemon=True)
        self._t.start()

    def submit(self, job: Callable[[], None]) -> None:
        with self._cv:
            if self._closed:
                raise RuntimeError("worker closed")
            self._job = job
            self._cv.notify_all()

    def _loop(self) -> None:
        while True:
            with self._cv:
                while self._job is None and not self._closed:
                    self._cv.wait()
                if self._job is None:
                    return
                job, self._job, self._busy = self._job, None, True
            try:
                job()
            except Exception as e:  # a failed write / evaluation must not kill the worker
                print(f"[fl_server] background job failed: {e!r}")
            finally:
                with self._cv:
                    self._busy = False
                    self._cv.notify_all()

    def flush(self, timeout: Optional[float] = None) -> bool:
        end = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while self._job is not None or self._busy:
                rem = None if end is None else end - time.monotonic()
                if rem is not None and rem <= 0:
                    return False
                self._cv.wait(rem)
            return True

    def close(self, cancel: bool = False) -> None:
        with self._cv:
            if cancel:
                self._job = None
            self._closed = True
            self._cv.notify_all()
        self._t.join()


def _scalar(v) -> "P.Scalar":
    if isinstance(v, bool):
        return P.Scalar(scint32=int(v))
    if isinstance(v, int):
        return P.Scalar(scint32=v)
    if isinstance(v, float):
        return P.Scalar(scfloat=v)
    return P.Scalar(scstring=str(v))


def _cfg(d: Dict[str, object]):
    return {k: _scalar(v) for k, v in d.items()}


class FLServer(TransportServiceServicer):
    def __init__(self, cfg: FLConfig, global_flat: Optional[np.ndarray] = None, table: Optional[ParamTable] = None,
                 evaluator: Optional[Callable[[np.ndarray], Dict[str, float]]] = None):
        self.cfg = cfg
        self.table = table or ParamTable()
        start_round, version, snap = 0, cfg.initial_model_version, None
        if global_flat is None:
            global_flat = self.table.init_flat(cfg.seed)
        if cfg.resume and cfg.snapshot_dir:
            snap = load_snapshot(cfg.snapshot_dir, self.table)
            finished = False
            if snap is not None:
                global_flat, start_round, version, finished = snap
                print(f"[fl_server] resumed from snapshot: round {start_round}, version {version}"
                      + (" (run already finished: every client gets FIN)" if finished else ""))
        self.evaluator = evaluator
        self.state = RoundState(global_flat, max_rounds=cfg.max_rounds, register_window_s=cfg.register_window_s,
                                num_clients=cfg.num_clients, initial_version=version,
                                weighted=(cfg.aggregation == "weighted"), round_deadline_s=cfg.round_deadline_s,
                                quorum=cfg.quorum, start_round=start_round, on_aggregate=self._on_aggregate)
        if cfg.resume and cfg.snapshot_dir and snap is not None and finished and start_round > cfg.max_rounds:
            self.state.finished = True       # a completed run stays completed (a larger max_rounds extends it)
        self._blob_lock = threading.Lock()
        self._blob_cache: Dict[tuple, bytes] = {}
        self._codec: Dict[str, tuple] = {}          # client name -> (codec, wire_dtype) it can decode
        self._rccl_round: Dict[str, int] = {}       # client -> round whose average it holds already (RCCL plane)
        self._persist: Optional[LatestWorker] = None       # weight file + snapshot writes (off the lock)
        self._eval_worker: Optional[LatestWorker] = None   # server-side evaluation of the newest global
        self.server: Optional[grpc.Server] = None
        self.port: Optional[int] = None
        self.dist_port = 0
        self.done = threading.Event()
        self.log_root = os.path.abspath(os.path.join(cfg.work_dir, "."))

    # -- parameters --------------------------------------------------------------------------------
    def send_parameter(self, fmt: tuple = ("pickle", "fp32")) -> bytes:
        """fl_server.py:23-24 (``eval_model.get_weights(made_model)``) - here the current global average, encoded
        in the format the requesting client reads (``fmt`` = (codec, wire_dtype); reference pickle by default)."""
        with self.state.cv:
            v, flat = self.state.model_version, self.state.global_flat
        key = (v,) + tuple(fmt)
        with self._blob_lock:
            blob = self._blob_cache.get(key)
            if blob is None:
                blob = codec.encode(self.table.to_list(flat), fmt[0], wire_dtype=fmt[1])
                self._blob_cache = {k: b for k, b in self._blob_cache.items() if k[0] == v}
                self._blob_cache[key] = blob
            return blob

    @staticmethod
    def _advertised(config) -> Optional[tuple]:
        if "codec" not in config or config["codec"].scstring not in ("flat", "pickle"):
            return None
        dt = config["wire_dtype"].scstring if "wire_dtype" in config else "fp32"
        return config["codec"].scstring, dt if dt in ("fp32", "bf16") else "fp32"

    def client_format(self, name: str = "", config=None) -> tuple:
        """The reply codec of a request: advertised in this request's config, else what the named client
        advertised at READY / last uploaded, else the reference pickle."""
        adv = self._advertised(config) if config is not None else None
        if adv is not None:
            return adv
        return self._codec.get(name, ("pickle", "fp32"))

    def global_weights(self):
        with self.state.cv:
            return self.table.to_list(self.state.global_flat)

    def _on_aggregate(self, st: RoundState, rec: RoundRecord) -> None:
        dt = rec.t_end - rec.t_start
        print(f"[fl_server] round {rec.round} aggregated over {len(rec.clients)} client(s) "
              f"(n={[int(n) for n in rec.n_samples]}) in {dt:.2f}s -> version {st.model_version}"
              + (" (FIN)" if st.finished else ""))
        # This hook runs under the RoundState lock: the file writes (8.2 MB pickle, .h5 snapshot) and the evaluation
        # go to worker threads with a copy of the new global, so READY / VERSION long-polls / heartbeats - and the
        # wake-up of the clients waiting for this round - never wait for the disk or the evaluator.
        flat = st.global_flat.copy()
        if self.cfg.server_weight_file or self.cfg.snapshot_dir:
            if self._persist is None:
                self._persist = LatestWorker("fl-persist")
            args = (flat, st.current_round, st.model_version, st.finished)     # bound now, under the lock
            self._persist.submit(lambda: self._write_round(*args))
        if self.evaluator is not None:   # fl_server.py:27-37 (dead code in the reference)
            if self._eval_worker is None:
                self._eval_worker = LatestWorker("fl-eval")
            self._eval_worker.submit(lambda r=rec.round: self._evaluate(r, flat))
        if st.finished:
            self.done.set()

    def _write_round(self, flat: np.ndarray, current_round: int, version: int, finished: bool) -> None:
        """The reference's ./server_weights/weights.pickle (fl_server.py:104-105) + the resume snapshot. Runs on
        the persistence worker; only the newest pending round is written (each file is overwritten per round)."""
        if self.cfg.server_weight_file:
            codec.save_weight_file(os.path.join(self.cfg.work_dir, self.cfg.server_weight_file)
                                   if not os.path.isabs(self.cfg.server_weight_file) else self.cfg.server_weight_file,
                                   self.table.to_list(flat))
        if self.cfg.snapshot_dir:
            save_snapshot(self.cfg.snapshot_dir, self.table, flat, current_round, version, finished)

    def flush_persistence(self, timeout: Optional[float] = None) -> bool:
        """Wait until the latest round's weight file / snapshot is on disk."""
        return self._persist.flush(timeout) if self._persist is not None else True

    def _evaluate(self, rnd: int, flat: np.ndarray) -> None:
        try:
            res = self.evaluator(flat)
            print(f"[fl_server] round {rnd} Evaluate Loss : {res.get('loss')} "
                  f"Evaluate Accuracy : {res.get('accuracy')}")
        except Exception as e:
            print(f"[fl_server] evaluation of round {rnd} failed: {e!r}")

    def _params_for(self, name: str, new_round: int, fmt: tuple) -> bytes:
        """The new global for a client, or nothing for an RCCL client that holds it already (it reported the
        round just aggregated with title "rccl")."""
        if self._rccl_round.get(name) == new_round - 1:
            return b""
        return self.send_parameter(fmt)

    # -- RPC ---------------------------------------------------------------------------------------
    def transport(self, request_iterator, context):
        opened = set()
        for req in request_iterator:
            if req.ready_req.type == "R":
                yield self._ready(req.ready_req)
            elif req.update_req.type == "P":
                fmt = self.client_format(req.update_req.cname)
                yield P.transportResponse(update_rep=P.UpdateRep(type="P", buffer_chunk=self.send_parameter(fmt),
                                                                title="parameters"))
            elif req.update_req.type == "T":
                self.state.heartbeat(req.update_req.cname)
                yield P.transportResponse(update_rep=P.UpdateRep(type="T"))
            elif req.update_req.type == "L":
                self._save_chunk(req.update_req.title, req.update_req.buffer_chunk, opened)
                yield P.transportResponse(update_rep=P.UpdateRep(type="L", title=req.update_req.title))
            elif req.update_req.type == "D":
                yield self._train_done(req.update_req, context)
            elif req.version_req.type == "P":
                yield self._version(req.version_req)
            else:
                yield P.transportResponse()

    def _ready(self, r):
        client_round = r.config["current_round"].scint32 if "current_round" in r.config else 0
        if self.cfg.ready_stall_s > 0:
            time.sleep(self.cfg.ready_stall_s)      # fl_server.py:56 (kept for compat; presets set 0)
        conf = self.state.ready(r.cname, client_round)
        if conf["state"] == SW:
            self._codec[r.cname] = self._advertised(r.config) or ("pickle", "fp32")
            print(f"### Check Train Round ### {r.cname} registered as rank {conf['rank']}")
            conf["model_type"] = self.cfg.model_type
            conf["data_plane"] = self.cfg.data_plane
            if self.cfg.data_plane == "rccl":
                conf["world_size"] = self.state.wait_window_closed(timeout=self.cfg.register_window_s + 5)
                conf["dist_port"] = self.dist_port
                conf["dist_addr"] = self.cfg.dist_addr
        return P.transportResponse(ready_rep=P.ReadyRep(config=_cfg(conf)))

    def _train_done(self, u, context):
        print(f"### Start rounds management ### {u.cname} round {u.current_round}")
        flat = None
        n = float(u.file_len)
        if u.buffer_chunk:
            try:
                arrays, hdr = codec.decode(u.buffer_chunk)
                if u.buffer_chunk[:4] != codec.MAGIC:      # a pickle sender reads pickle replies
                    self._codec[u.cname] = ("pickle", "fp32")
                flat = self.table.from_list(arrays)
                n = float(hdr.get("n_samples") or n or 0.0)   # 0: not reported (reference client)
            except Exception as e:
                print(f"[fl_server] rejected payload from {u.cname}: {e}")
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"bad weight payload: {e}")
        if u.title == "rccl":
            self._rccl_round[u.cname] = u.current_round
        else:
            self._rccl_round.pop(u.cname, None)
        try:
            state, conf = self.state.submit(u.cname, u.current_round, flat, max(n, 0.0))
        except ValueError as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        conf = dict(conf, state=state)
        print(f"### Current state: {state} ###")
        chunk = self._params_for(u.cname, conf["current_round"], self.client_format(u.cname)) \
            if state == RESP_ARY else b""
        return P.transportResponse(update_rep=P.UpdateRep(type="D", buffer_chunk=chunk, config=_cfg(conf)))

    def _version(self, v):
        mv = v.config["model_version"].scint32 if "model_version" in v.config else 0
        cr = v.config["current_round"].scint32 if "current_round" in v.config else 0
        wait = v.config["wait_s"].scfloat if "wait_s" in v.config else 0.0
        state, conf = self.state.version(mv, cr, min(wait, self.cfg.long_poll_s))
        if state == NOT_WAIT:
            name = v.config["cname"].scstring if "cname" in v.config else ""
            chunk = self._params_for(name, conf["current_round"], self.client_format(name, v.config))
            return P.transportResponse(version_rep=P.VersionRep(state=P.NOT_WAIT, buffer_chunk=chunk,
                                                                config=_cfg(conf)))
        if state == FIN:
            return P.transportResponse(version_rep=P.VersionRep(state=P.FIN, config=_cfg(conf)))
        return P.transportResponse(version_rep=P.VersionRep(state=P.WAIT, config=_cfg(conf)))

    def _save_chunk(self, title: str, chunk: bytes, opened: set) -> None:
        """fl_server.py:84-89, with append for multi-chunk files (§A7) and no path escape."""
        rel = title[11:] if title.startswith("./send_logs") else title.lstrip("./")
        dest = os.path.abspath(os.path.join(self.log_root, rel.lstrip("/")))
        if not dest.startswith(self.log_root + os.sep):
            raise ValueError(f"log path escapes the server directory: {title}")
        os.makedirs(os.path.dirname(dest), exist_ok=True)
        with open(dest, "ab" if dest in opened else "wb") as f:
            f.write(chunk)
        opened.add(dest)

    # -- lifecycle -----------------------------------------------------------------------------------
    def start(self, port: Optional[int] = None) -> int:
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=self.cfg.server_threads),
                                  options=channel_options(self.cfg.max_message_mb))
        add_TransportServiceServicer_to_server(self, self.server)
        if self.cfg.data_plane == "rccl" and not self.dist_port:
            self.dist_port = _free_port()     # RCCL rendezvous handed to clients in the READY reply
        port = self.cfg.port if port is None else port
        self.port = self.server.add_insecure_port(f"{self.cfg.bind}:{port}")
        self.server.start()
        return self.port

    def stop(self, grace: float = 0.5) -> None:
        self.state.stop()
        if self.server is not None:
            self.server.stop(grace)
        if self._persist is not None:          # the last round's files are written before stop returns
            self._persist.close(cancel=False)
            self._persist = None
        if self._eval_worker is not None:      # a pending (not yet started) evaluation is dropped
            self._eval_worker.close(cancel=True)
            self._eval_worker = None

    def serve_forever(self, exit_on_fin: bool = True) -> None:
        try:
            while True:
                if exit_on_fin and self.done.wait(1.0):
                    time.sleep(2.0)   # let the last clients collect FIN
                    break
                if not exit_on_fin:
                    time.sleep(3600)
        except KeyboardInterrupt:
            pass
        finally:
            self.stop(0)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# -- snapshot / resume ---------------------------------------------------------------------------------
def save_snapshot(d: str, table: ParamTable, flat: np.ndarray, current_round: int, version: int,
                  finished: bool) -> None:
    from ..ckpt.h5 import save_weights_h5
    os.makedirs(d, exist_ok=True)
    h5 = os.path.join(d, "global.h5")
    save_weights_h5(h5 + ".tmp", table, flat)
    os.replace(h5 + ".tmp", h5)
    st = {"current_round": current_round, "model_version": version, "finished": finished, "time": time.time()}
    with open(os.path.join(d, "state.json.tmp"), "w") as f:
        json.dump(st, f)
    os.replace(os.path.join(d, "state.json.tmp"), os.path.join(d, "state.json"))


def load_snapshot(d: str, table: ParamTable):
    from ..ckpt.h5 import load_weights_h5
    sp = os.path.join(d, "state.json")
    if not os.path.exists(sp):
        return None
    with open(sp) as f:
        st = json.load(f)
    flat = load_weights_h5(os.path.join(d, "global.h5"), table)
    return flat, int(st["current_round"]), int(st["model_version"]), bool(st.get("finished", False))
