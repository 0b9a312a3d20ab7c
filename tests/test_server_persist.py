"""Server persistence runs off the RoundState lock (fl/server.py LatestWorker): a slow disk must not stall the
round's RPCs. Reference: fl_server.py:104-105 writes the pickle inside the aggregation path."""
import threading
import time

import numpy as np

from crack_detection_federatedlearning_grpc_amd.config import FLConfig
from crack_detection_federatedlearning_grpc_amd.fl import server as server_mod
from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer, LatestWorker
from crack_detection_federatedlearning_grpc_amd.fl.state import NOT_WAIT, RESP_ARY


def test_slow_writer_does_not_block_version_long_poll(tmp_path, table, monkeypatch):
    writes = []

    def slow_save(path, arrays):
        time.sleep(2.0)
        writes.append((path, len(arrays)))

    monkeypatch.setattr(server_mod.codec, "save_weight_file", slow_save)
    cfg = FLConfig(register_window_s=5.0, ready_stall_s=0.0, num_clients=2, max_rounds=3, work_dir=str(tmp_path),
                   server_weight_file=str(tmp_path / "w.pickle"), client_weight_file="")
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    st = srv.state
    assert st.ready("a", 0)["state"] == "SW" and st.ready("b", 0)["state"] == "SW"
    mv, cr = st.model_version, st.current_round
    got = {}

    def poll():
        got["res"] = st.version(mv, cr, wait_s=10.0)
        got["t"] = time.monotonic()

    th = threading.Thread(target=poll)
    th.start()
    time.sleep(0.1)
    flat = np.ones(table.total, np.float32)
    st.submit("a", cr, flat, 1.0)
    t0 = time.monotonic()
    state, _ = st.submit("b", cr, flat, 1.0)          # closes the round: aggregation + on_aggregate hook
    t_submit = time.monotonic() - t0
    th.join(5.0)
    assert state == RESP_ARY
    assert t_submit < 0.5, t_submit                    # the hook only queued the write
    assert got["res"][0] == NOT_WAIT and got["t"] - t0 < 0.5
    # a READY / heartbeat during the write is not blocked either
    t1 = time.monotonic()
    st.heartbeat("a")
    assert time.monotonic() - t1 < 0.5
    assert writes == []                                # still writing
    srv.stop()                                         # stop() waits for the last round's files
    assert len(writes) == 1 and writes[0][1] == len(table.entries)


def test_latest_worker_coalesces_pending_jobs():
    ran = []
    gate = threading.Event()
    w = LatestWorker("t")
    w.submit(lambda: (gate.wait(5.0), ran.append(1)))
    time.sleep(0.05)                                   # job 1 running, blocked on the gate
    w.submit(lambda: ran.append(2))
    w.submit(lambda: ran.append(3))                    # replaces job 2 (never started)
    gate.set()
    assert w.flush(5.0)
    assert ran == [1, 3]
    w.submit(lambda: ran.append(4))
    w.close(cancel=False)                              # a pending job still runs on a non-cancelling close
    assert ran == [1, 3, 4]
    w2 = LatestWorker("t2")
    gate2 = threading.Event()
    w2.submit(lambda: gate2.wait(5.0))
    time.sleep(0.05)
    w2.submit(lambda: ran.append(5))
    closer = threading.Thread(target=w2.close, args=(True,))   # drops the pending job at once, then joins
    closer.start()
    time.sleep(0.05)
    gate2.set()
    closer.join(5.0)
    assert 5 not in ran
