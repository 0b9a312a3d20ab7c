"""FL client driver loop.

Reference: fl_client.py:77-175 (``send_message``). Same verb sequence - READY -> PARAM -> TRAINING -> train ->
loop { TRAIN_DONE -> RESP_ACY: poll VERSION until NOT_WAIT | RESP_ARY: TRAINING + train | FIN: exit } - with:
* FIN handled while polling (the reference polls forever);
* server-side long-poll (``wait_s`` in the VERSION config) instead of blind 20 s sleeps;
* RPC deadlines + retry with backoff (reference has none, §5.3);
* optional RCCL data plane: the weighted all-reduce runs between the clients on their GPUs
  (``parallel/rccl.py``); gRPC carries control only and rank 0 uploads the averaged model for the server's copy.
  If a collective fails (a peer died, or ``rccl_timeout_s`` expired) every survivor aborts the communicator and
  sends its local weights over gRPC instead; the server's round deadline + quorum then averages the survivors
  (SURVEY §5.3).
"""
from __future__ import annotations

import json
import os
import random
import sys
import threading
import time
from typing import Callable, Dict, List, Optional, Protocol

import grpc
import numpy as np

from ..config import FLConfig
from . import codec
from . import proto as P
from ..utils.trace import phase as trace_phase
from .rpc import TransportServiceStub, channel_options


class LocalTrainer(Protocol):
    n_samples: int

    def set_weights(self, arrays: List[np.ndarray]) -> None: ...

    def get_weights(self) -> List[np.ndarray]: ...

    def train_round(self, current_round: int) -> Dict[str, float]: ...


def _one(msg):
    yield msg


class FLClient:
    def __init__(self, cfg: FLConfig, trainer_factory: Callable[[], LocalTrainer], name: Optional[str] = None,
                 target: Optional[str] = None, aggregator_factory: Optional[Callable[[Dict], object]] = None):
        self.cfg = cfg
        self.trainer_factory = trainer_factory
        self.name = name or f"client{random.randint(1, 100000)}"     # fl_client.py:26
        self.target = target or f"{cfg.host}:{cfg.port}"
        self.aggregator_factory = aggregator_factory
        self.aggregator = None
        self.trainer: Optional[LocalTrainer] = None
        self.history: List[Dict] = []
        self.phases: List[Dict] = []
        self.info: Dict[str, object] = {}
        self.final_state = ""
        self.fallbacks = 0                      # RCCL -> gRPC data-plane fallbacks (peer loss)
        self._pending = None                    # (thread, result box) of an async round report

    # -- transport helpers ---------------------------------------------------------------------------
    def _call(self, stub, req) -> "P.transportResponse":
        delay = 0.5
        for attempt in range(self.cfg.rpc_retries + 1):
            try:
                last = None
                for rep in stub.transport(_one(req), timeout=self.cfg.rpc_timeout_s):
                    last = rep
                return last
            except grpc.RpcError as e:
                code = e.code() if hasattr(e, "code") else None
                if code not in (grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED) or \
                        attempt == self.cfg.rpc_retries:
                    raise
                time.sleep(delay)
                delay = min(delay * 2, 10.0)

    def _codec_cfg(self) -> Dict[str, "P.Scalar"]:
        """The reply format this client decodes, advertised to the server (a reference client sends none and
        gets pickles)."""
        return {"codec": P.Scalar(scstring=self.cfg.codec), "wire_dtype": P.Scalar(scstring=self.cfg.wire_dtype)}

    def _ready(self, stub):
        req = P.transportRequest(ready_req=P.ReadyReq(type="R", cname=self.name, state=P.ON,
                                                     config={"current_round": P.Scalar(scint32=0),
                                                             **self._codec_cfg()}))
        return self._call(stub, req).ready_rep.config

    def _params(self, stub) -> bytes:
        return self._call(stub, P.transportRequest(update_req=P.UpdateReq(type="P", cname=self.name))
                          ).update_rep.buffer_chunk

    def _log_phase(self, phase: Dict) -> None:
        """Per-round phase wall-clock (aggregate = RCCL all-reduce in rccl mode, upload = TRAIN_DONE RPC incl. the
        server-side FedAvg when this client closes the round, wait = VERSION long-poll until the new global)."""
        rec = dict(phase, client=self.name, kind="phases")
        self.phases.append(rec)
        if self.cfg.metrics_file:
            os.makedirs(os.path.dirname(os.path.abspath(self.cfg.metrics_file)), exist_ok=True)
            with open(self.cfg.metrics_file, "a") as f:
                f.write(json.dumps(rec) + "\n")

    def _training(self, stub) -> None:
        self._call(stub, P.transportRequest(update_req=P.UpdateReq(type="T", cname=self.name, state=P.TRAINING)))

    def _train_done(self, stub, cr: int, payload: bytes, n: int, plane: str = ""):
        """``plane`` = "rccl" (in ``title``): this client's local model already IS the round's average (the
        collective succeeded), so the server sends it no parameters back (a reference client sends no title)."""
        req = P.transportRequest(update_req=P.UpdateReq(type="D", buffer_chunk=payload, state=P.TRAIN_DONE,
                                                        cname=self.name, current_round=cr, file_len=int(n),
                                                        title=plane))
        return self._call(stub, req).update_rep

    def _version(self, stub, mv: int, cr: int, wait_s: float):
        req = P.transportRequest(version_req=P.VersionReq(type="P", config={
            "model_version": P.Scalar(scint32=mv), "current_round": P.Scalar(scint32=cr),
            "wait_s": P.Scalar(scfloat=float(wait_s)), "cname": P.Scalar(scstring=self.name),
            **self._codec_cfg()}))
        return self._call(stub, req).version_rep

    def send_logs(self, stub, root: Optional[str] = None) -> int:
        """fl_client.py:34-50 (call site commented out in the reference, :110-118)."""
        root = root or self.cfg.log_dir
        sent = 0
        chunk = self.cfg.log_chunk_mb * 1024 * 1024
        for dirpath, _, files in os.walk(root):
            for fn in sorted(files):
                full = os.path.join(dirpath, fn)
                title = "./send_logs/" + os.path.relpath(full, os.path.dirname(root.rstrip("/")) or ".")

                def gen():
                    with open(full, "rb") as f:
                        while True:
                            piece = f.read(chunk)
                            if not piece:
                                return
                            yield P.transportRequest(update_req=P.UpdateReq(type="L", buffer_chunk=piece,
                                                                            title=title, file_len=len(piece)))
                for _ in stub.transport(gen(), timeout=self.cfg.rpc_timeout_s):
                    pass
                sent += 1
        return sent

    # -- local work ------------------------------------------------------------------------------------
    def _train(self, cr: int) -> None:
        if self.cfg.fault_drop_round and cr >= self.cfg.fault_drop_round:
            if self._pending is not None:      # the previous round's report went out (async upload) first
                self._pending[0].join()
            print(f"[{self.name}] fault injection: dropping out at round {cr}")
            raise SystemExit(3)
        t0 = time.perf_counter()
        m = self.trainer.train_round(cr)
        m = dict(m, round=cr, client=self.name, train_s=time.perf_counter() - t0)
        self.history.append(m)
        if self.cfg.client_weight_file:   # trainer -> driver hand-off file (client_fit_model.py:238-240)
            codec.save_weight_file(self.cfg.client_weight_file, self.trainer.get_weights())

    def _fallback(self, e: BaseException) -> None:
        print(f"[{self.name}] RCCL aggregation failed ({type(e).__name__}: {e}); aborting the "
              f"communicator, falling back to the gRPC data plane")
        if self.aggregator is not None:
            self.aggregator.abort()
        self.aggregator = None
        self.fallbacks += 1

    def _payload(self, async_ok: bool = False) -> tuple:
        """(weights to upload or None, data plane, pending device FedAvg or None). RCCL mode: the weighted
        all-reduce is issued here (in place on the GPU, or over host arrays). With ``async_ok`` and a device
        buffer the collective is NOT waited for: the ``PendingFedAvg`` goes to the round report, which learns the
        verdict from its watchdog, while this thread starts the next round. Otherwise the verdict is awaited here:
        rank 0 alone uploads the average for the server's copy (host copy of the average kept by the side stream),
        the other ranks send nothing; a failed collective leaves the local model unchanged (rolled back) and the
        client continues on the gRPC plane."""
        n = getattr(self.trainer, "n_samples", 0)
        arrays = None
        plane = ""
        pending = None
        if self.aggregator is not None:
            try:
                adev = getattr(self.trainer, "fedavg_device_async", None)
                pending = adev(self.aggregator, n) if adev is not None else None
                if pending is not None:
                    if async_ok:
                        return None, "rccl", pending
                    self.trainer.settle_fedavg(pending)          # waits for the watchdog's verdict
                    if self.aggregator.rank == 0:
                        arrays = self.trainer.table.to_list(pending.host_average())
                else:
                    dev = getattr(self.trainer, "fedavg_device", None)
                    if dev is not None and dev(self.aggregator, n):
                        pass                                     # averaged in place (no host staging)
                    else:
                        arrays = self.aggregator.average(self.trainer.get_weights(), n)   # host-array trainers
                        self.trainer.set_weights(arrays)         # local model <- global average
            except Exception as e:                               # peer lost / collective timed out
                self._fallback(e)
                arrays = None
                pending = None
            else:
                plane = "rccl"
                if self.aggregator.rank != 0:
                    return None, plane, pending                  # rank 0 alone uploads the server's copy
        if arrays is None:
            arrays = self.trainer.get_weights()
        return arrays, plane, pending

    def _encode(self, arrays) -> bytes:
        if arrays is None:
            return b""
        if self.cfg.fault_corrupt:
            return b"\x80corrupt" + os.urandom(64)
        return codec.encode(arrays, self.cfg.codec, n_samples=getattr(self.trainer, "n_samples", 0),
                            wire_dtype=self.cfg.wire_dtype)

    def _report(self, stub, cr: int, mv: int, arrays, plane: str) -> Dict:
        """TRAIN_DONE of round ``cr`` and, on RESP_ACY, the VERSION long-poll until the server has aggregated the
        round (NOT_WAIT) or finished (FIN): the reference's verb sequence (fl_client.py:121-166). Returns the
        outcome and its phase timings; no local training happens here."""
        t1 = time.perf_counter()
        payload = self._encode(arrays)
        with trace_phase("fl/upload"):
            rep = self._train_done(stub, cr, payload, getattr(self.trainer, "n_samples", 0), plane)
        t2 = time.perf_counter()
        st = rep.config["state"].scstring
        print(f"### Received from state {st} ###")
        out = {"state": st, "cr": cr, "mv": mv, "blob": b"",
               "phase": {"round": cr, "upload_s": t2 - t1, "wait_s": 0.0, "payload_bytes": len(payload),
                         "data_plane": plane or "grpc",
                         "rank": self.aggregator.rank if self.aggregator is not None else -1}}
        if st == "RESP_ACY":
            while True:
                vr = self._version(stub, mv, cr, self.cfg.long_poll_s)
                if vr.state in (P.NOT_WAIT, P.FIN):
                    out["phase"]["wait_s"] = time.perf_counter() - t2
                    out["state"] = "NOT_WAIT" if vr.state == P.NOT_WAIT else "FIN"
                    out["cr"] = vr.config["current_round"].scint32
                    out["mv"] = vr.config["model_version"].scint32
                    out["blob"] = vr.buffer_chunk
                    out["phase"]["reply_bytes"] = len(vr.buffer_chunk)
                    return out
                time.sleep(min(self.cfg.poll_period_s, 1.0) if self.cfg.long_poll_s > 0
                           else self.cfg.poll_period_s)
        if st in ("RESP_ARY", "FIN"):
            out["cr"] = rep.config["current_round"].scint32
            out["mv"] = rep.config["model_version"].scint32
            out["blob"] = rep.buffer_chunk
            if st == "RESP_ARY":
                out["phase"]["reply_bytes"] = len(rep.buffer_chunk)
        return out

    def _apply(self, blob: bytes) -> None:
        if self.aggregator is not None or not blob:
            return                      # RCCL mode: local weights already hold the all-reduced average
        self.trainer.set_weights(codec.decode(blob)[0])

    def _discard_round(self, box: Dict, res: Dict, fell_back: bool) -> None:
        """Undo the round trained while an asynchronous report was pending (its start was not the run's global
        model): drop its history entry and reset the local model to the global one - the server's reply when it
        carries parameters (always after a gRPC fallback), else the average this client's collective produced."""
        pend = box["pending"]
        if self.history:
            self.history.pop()
        if res.get("blob") and (fell_back or self.aggregator is None):
            self.trainer.set_weights(codec.decode(res["blob"])[0])
        elif pend is None:
            self.trainer.set_weights(box["avg"])            # host path: the average taken after the collective
        elif fell_back:
            self.trainer.restore_flat(pend.host_backup())
        else:
            self.trainer.restore_flat(pend.avg)
        if self.cfg.client_weight_file:
            codec.save_weight_file(self.cfg.client_weight_file, self.trainer.get_weights())

    # -- main loop ------------------------------------------------------------------------------------------
    def run(self) -> str:
        with grpc.insecure_channel(self.target, options=channel_options(self.cfg.max_message_mb)) as ch:
            stub = TransportServiceStub(ch)
            print(f"### Ready Client ### {self.name}")
            conf = self._ready(stub)
            if conf["state"].scstring != "SW":
                print(f"[{self.name}] registration closed ({conf['state'].scstring}); exiting")
                self.final_state = conf["state"].scstring
                return self.final_state
            cr = conf["current_round"].scint32
            mtr = conf["max_train_round"].scint32
            mv = conf["model_version"].scint32
            self.info = {k: (v.scstring or v.scint32 or v.scfloat) for k, v in conf.items()}
            if "world_size" in conf and self.aggregator_factory is not None:
                self.aggregator = self.aggregator_factory(self.info)
            print("### Request Global Model Parameter ###")
            self.trainer = self.trainer_factory()
            self.trainer.set_weights(codec.decode(self._params(stub))[0])
            self._training(stub)
            self._train(cr)
            while cr <= mtr:
                join_s = 0.0
                if self._pending is not None:     # the previous round's collective verdict + TRAIN_DONE / VERSION
                    tj = time.perf_counter()
                    th, box = self._pending
                    th.join()
                    self._pending = None
                    join_s = time.perf_counter() - tj
                    if "error" in box:
                        raise box["error"]
                    res, pend = box["res"], box["pending"]
                    fell_back = box.get("fallback", False)
                    self._log_phase(dict(res["phase"], aggregate_s=box["aggregate_s"], join_wait_s=join_s,
                                         exposed_s=box["aggregate_s"] + join_s, async_upload=True,
                                         **(pend.stats() if pend is not None else {})))
                    if pend is not None and pend.engine is not None:
                        pend.engine.stall_log = None
                    if fell_back:                 # the collective failed: this client continues on gRPC
                        self._fallback(pend.error)
                    if res["state"] == "FIN":     # the server finished the run (e.g. fewer rounds than advertised)
                        # the round trained meanwhile is not part of the run: the client ends at the run's global
                        # model (the server's reply after a fallback, else the average this round all-reduced)
                        self._discard_round(box, res, fell_back)
                        cr, mv = res["cr"], res["mv"]
                        self.final_state = "FIN"
                        break
                    if res["state"] not in ("NOT_WAIT", "RESP_ARY"):
                        print(f"[{self.name}] unexpected state {res['state']!r}; exiting")
                        self.final_state = res["state"]
                        break
                    if fell_back or (res["cr"], res["mv"]) != (cr, mv):
                        # the round just trained started from a failed average or a round the server did not
                        # advance to: drop it and train the server's round from the server's model
                        print(f"[{self.name}] server round {res['cr']} / version {res['mv']} (trained {cr} / {mv}"
                              f"{' from a failed collective' if fell_back else ''}); re-training from the global")
                        self._discard_round(box, res, fell_back)
                        cr, mv = res["cr"], res["mv"]
                        self._train(cr)
                        continue
                print(f"### Deliver model state: TRAIN DONE to server ### round {cr}")
                if self.cfg.fault_delay_s:
                    time.sleep(self.cfg.fault_delay_s)
                t0 = time.perf_counter()
                async_ok = self.cfg.async_upload and cr < mtr
                with trace_phase("fl/aggregate"):
                    arrays, plane, pend = self._payload(async_ok)   # RCCL mode: the all-reduce is issued here
                agg_s = time.perf_counter() - t0
                if plane == "rccl" and async_ok:
                    # device path: the collective runs on the GPU's side stream; the round's report (rank 0: upload
                    # of the average) waits for its verdict in a background thread while this thread starts the
                    # next round (whose first step waits per bucket on the device), off the server's aggregation
                    # path. Host-array path: the collective is done; only the report goes to the thread.
                    box: Dict = {"aggregate_s": agg_s, "pending": pend,
                                 "avg": None if pend is not None else self.trainer.get_weights()}
                    rank0 = self.aggregator.rank == 0

                    def report(cr=cr, mv=mv, pend=pend, box=box, rank0=rank0, arrays=arrays):
                        try:
                            if pend is None:
                                arr, pl = arrays, "rccl"
                            elif pend.wait(rollback=False):
                                arr, pl = (self.trainer.table.to_list(pend.host_average()) if rank0 else None), "rccl"
                            else:          # collective lost: report the local model over gRPC
                                print(f"[{self.name}] round {cr} collective failed ({pend.error}); reporting the "
                                      f"local model over gRPC")
                                arr, pl = self.trainer.table.to_list(pend.host_backup()), ""
                                box["fallback"] = True
                            box["res"] = self._report(stub, cr, mv, arr, pl)
                            self._training(stub)
                        except BaseException as e:   # re-raised by the main thread at the join
                            box["error"] = e
                    th = threading.Thread(target=report, name=f"{self.name}-report", daemon=True)
                    th.start()
                    self._pending = (th, box)
                    cr, mv = cr + 1, mv + 1              # what the server's aggregation of round cr yields
                    self._train(cr)
                    continue
                res = self._report(stub, cr, mv, arrays, plane)
                phase = dict(res["phase"], aggregate_s=agg_s, **(pend.stats() if pend is not None else {}))
                if pend is not None and pend.engine is not None:
                    pend.engine.stall_log = None
                st = res["state"]
                self._log_phase(phase)
                if st in ("NOT_WAIT", "RESP_ARY"):
                    if st == "RESP_ARY":
                        self._training(stub)
                    cr, mv = res["cr"], res["mv"]
                    self._apply(res["blob"])
                    if st == "NOT_WAIT":
                        self._training(stub)
                    self._train(cr)
                elif st == "FIN":
                    cr, mv = res["cr"], res["mv"]
                    self.final_state = "FIN"
                    break
                else:
                    print(f"[{self.name}] unexpected state {st!r}; exiting")
                    self.final_state = st
                    break
            if self.cfg.final_weight_file:
                codec.save_weight_file(self.cfg.final_weight_file, self.trainer.get_weights())
            if self.cfg.upload_logs:
                self.send_logs(stub)
            print("all training finish")
            if self.aggregator is not None:
                self.aggregator.close()
            return self.final_state or "FIN"
