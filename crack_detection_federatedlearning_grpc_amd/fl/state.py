"""Locked FL round state machine.

Reference: module globals mutated by 10 gRPC worker threads without a lock (fl_server.py:14-20, 45-81, 107-149;
SURVEY §5.2 / §A8). Here all state lives in one ``RoundState`` guarded by a ``threading.Condition``:

* registration (``ready``)      fl_server.py:45-81   SW / CTW replies, 10 s window from the first READY
* round accounting (``submit``) fl_server.py:107-135 RESP_ACY / RESP_ARY / FIN; aggregation runs EXACTLY once per
  round (fixes the double-aggregate race) over a fresh per-round buffer (fixes §A1); a stale-round submit gets a
  real reply (fixes §A2)
* version check (``version``)   fl_server.py:138-149 WAIT / NOT_WAIT / FIN, plus an optional server-side long-poll
  so a waiting client is released as soon as the round completes instead of on a 20 s sleep boundary
* liveness: optional per-round deadline with a quorum fraction - survivors are re-weighted (§5.3, fixes §A9).
  Clients dropped at a deadline leave the LIVE set, so later rounds close as soon as every live client reported
  (a dead client is not waited for again, and the quorum is a fraction of the live clients); a dropped client
  that speaks again (READY, TRAINING or TRAIN_DONE) rejoins it
"""
from __future__ import annotations

import math
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from ..parallel.fedavg import fedavg_flat

SW, CTW = "SW", "CTW"
RESP_ACY, RESP_ARY, FIN = "RESP_ACY", "RESP_ARY", "FIN"
WAIT, NOT_WAIT = "WAIT", "NOT_WAIT"


@dataclass
class RoundRecord:
    round: int
    clients: List[str]
    n_samples: List[float]
    t_start: float
    t_end: float
    dropped: List[str] = field(default_factory=list)


class RoundState:
    def __init__(self, global_flat: np.ndarray, *, max_rounds: int = 5, register_window_s: float = 10.0,
                 num_clients: int = 0, initial_version: int = 1, weighted: bool = True,
                 round_deadline_s: float = 0.0, quorum: float = 1.0, start_round: int = 0,
                 on_aggregate: Optional[Callable[["RoundState", RoundRecord], None]] = None,
                 clock: Callable[[], float] = time.monotonic):
        self.cv = threading.Condition()
        self.global_flat = np.asarray(global_flat, np.float32).copy()
        self.max_rounds = max_rounds
        self.window_s = register_window_s
        self.num_clients = num_clients
        self.model_version = initial_version
        self.current_round = start_round          # ALL_CURRENT_ROUND (fl_server.py:16)
        self.weighted = weighted
        self.deadline_s = round_deadline_s
        self.quorum = quorum
        self.on_aggregate = on_aggregate
        self.clock = clock
        self.registered: List[str] = []
        self.live: set = set()                    # registered clients not dropped at a deadline
        self.window_started: Optional[float] = None
        self.window_closed = False
        self.updates: Dict[str, Tuple[np.ndarray, float]] = {}
        self.round_started: Optional[float] = None
        self.finished = False
        self.history: List[RoundRecord] = []
        self.heartbeats: Dict[str, float] = {}
        self._timer: Optional[threading.Thread] = None
        self._stop = threading.Event()

    # -- registration -----------------------------------------------------------------------------
    def _window_open_locked(self) -> bool:
        if self.window_closed:
            return False
        if self.window_started is not None and self.clock() - self.window_started >= self.window_s:
            self._close_window_locked()
            return False
        return True

    def _close_window_locked(self) -> None:
        if not self.window_closed:
            self.window_closed = True
            self.round_started = self.clock()
            self.cv.notify_all()

    def ready(self, name: str, client_round: int) -> Dict[str, object]:
        with self.cv:
            if self.finished:                      # e.g. resumed from the snapshot of a finished run
                return dict(self._cfg_locked(), state=FIN)
            if self.window_started is None:
                self.window_started = self.clock()
                self._start_monitor()
            if not self._window_open_locked() and name not in self.registered:
                return {"state": CTW}
            if name not in self.registered:
                self.registered.append(name)
            self._touch_locked(name)
            if self.num_clients and len(self.registered) >= self.num_clients:
                self._close_window_locked()
            if self.current_round == 0 and client_round == 0:
                self.current_round = 1             # fl_server.py:67
            return {"state": SW, "model_version": self.model_version, "current_round": self.current_round,
                    "max_train_round": self.max_rounds, "rank": self.registered.index(name)}

    def wait_window_closed(self, timeout: Optional[float] = None) -> int:
        """Block until registration closes; returns the world size (used by the RCCL data plane)."""
        end = None if timeout is None else self.clock() + timeout
        with self.cv:
            while self._window_open_locked():
                rem = None if end is None else end - self.clock()
                if rem is not None and rem <= 0:
                    break
                self.cv.wait(timeout=min(0.05, rem) if rem is not None else 0.05)
            return len(self.registered)

    def _touch_locked(self, name: str) -> None:
        self.heartbeats[name] = self.clock()
        if name in self.registered and name not in self.live:
            if self.history:
                print(f"[fl_server] {name} is back; expected again from round {self.current_round}")
            self.live.add(name)

    def heartbeat(self, name: str) -> None:
        with self.cv:
            self._touch_locked(name)

    # -- round accounting ---------------------------------------------------------------------------
    def _expected_locked(self) -> int:
        return len(self.live)

    def submit(self, name: str, client_round: int, flat: Optional[np.ndarray], n_samples: float
               ) -> Tuple[str, Dict[str, object]]:
        with self.cv:
            if self.finished:
                return FIN, self._cfg_locked()
            if name not in self.registered:
                return CTW, self._cfg_locked()
            self._touch_locked(name)
            if client_round != self.current_round:
                return RESP_ACY, self._cfg_locked()   # stale: client polls VERSION and picks up new params
            if flat is not None:
                if flat.shape != self.global_flat.shape or not np.all(np.isfinite(flat)):
                    raise ValueError(f"rejected update from {name}: bad shape or non-finite values")
            self.updates[name] = (flat, float(n_samples))
            # aggregation waits for the window to close so a fast early client cannot close a round alone
            if self.window_closed and len(self.updates) >= self._expected_locked():
                return self._aggregate_locked([])
            return RESP_ACY, self._cfg_locked()

    def _aggregate_locked(self, dropped: List[str]) -> Tuple[str, Dict[str, object]]:
        ups = [(f, n) for f, n in self.updates.values() if f is not None]
        if ups:
            # a reference client reports no sample count (n = 0): that round is the reference's plain mean
            self.global_flat = fedavg_flat(ups, self.weighted and all(n > 0 for _, n in ups))
        rec = RoundRecord(self.current_round, list(self.updates), [n for _, n in self.updates.values()],
                          self.round_started or self.clock(), self.clock(), dropped)
        self.live.difference_update(dropped)
        self.history.append(rec)
        self.updates = {}
        done = self.current_round >= self.max_rounds
        self.current_round += 1
        self.model_version += 1
        self.round_started = self.clock()
        if done:
            self.finished = True
        self.cv.notify_all()
        if self.on_aggregate is not None:
            try:
                self.on_aggregate(self, rec)
            except Exception as e:  # snapshot failures must not wedge the round
                print(f"[fl_server] on_aggregate hook failed: {e!r}")
        return (FIN if done else RESP_ARY), self._cfg_locked()

    def _cfg_locked(self) -> Dict[str, object]:
        return {"model_version": self.model_version, "current_round": self.current_round}

    # -- version check / long-poll --------------------------------------------------------------------
    def version(self, client_version: int, client_round: int, wait_s: float = 0.0) -> Tuple[str, Dict[str, object]]:
        end = self.clock() + max(wait_s, 0.0)
        with self.cv:
            while self.model_version == client_version and not self.finished:
                rem = end - self.clock()
                if rem <= 0:
                    break
                self.cv.wait(timeout=min(rem, 0.5))
            if self.model_version == client_version and not self.finished:
                return WAIT, {}
            if self.finished and (client_round >= self.max_rounds or self.current_round > self.max_rounds):
                return FIN, self._cfg_locked()
            return NOT_WAIT, self._cfg_locked()

    # -- deadline monitor -------------------------------------------------------------------------------
    def _start_monitor(self) -> None:
        if self._timer is not None:
            return
        self._timer = threading.Thread(target=self._monitor, name="fl-round-monitor", daemon=True)
        self._timer.start()

    def _monitor(self) -> None:
        while not self._stop.is_set():
            with self.cv:
                if self.finished:
                    return
                if not self.window_closed:
                    self._window_open_locked()
                elif self.updates and len(self.updates) >= self._expected_locked():
                    self._aggregate_locked([])   # window closed after every registered client had reported
                elif self.deadline_s > 0 and self.round_started is not None and \
                        self.clock() - self.round_started >= self.deadline_s and self.updates:
                    need = max(1, math.ceil(self.quorum * len(self.live)))
                    if len(self.updates) >= need:
                        dropped = [c for c in self.live if c not in self.updates]
                        print(f"[fl_server] round {self.current_round} deadline: aggregating "
                              f"{len(self.updates)}/{len(self.live)} live clients, dropped {dropped}")
                        self._aggregate_locked(dropped)
            self._stop.wait(0.05)

    def stop(self) -> None:
        self._stop.set()
        with self.cv:
            self.cv.notify_all()
