"""Failure handling, concurrency and observability of the FL control plane."""
import dataclasses
import json
import os
import threading
import time

import grpc
import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from crack_detection_federatedlearning_grpc_amd.config import FLConfig
from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer
from crack_detection_federatedlearning_grpc_amd.fl.state import (FIN, NOT_WAIT, RESP_ACY, RESP_ARY, SW, WAIT,
                                                                 RoundState)

from fakes import FakeTrainer


def _cfg(tmp_path, **kw):
    base = dict(register_window_s=2.0, ready_stall_s=0.0, num_clients=2, poll_period_s=0.05, long_poll_s=1.0,
                max_rounds=2, client_weight_file="", server_weight_file=str(tmp_path / "server_weights/w.pickle"),
                work_dir=str(tmp_path), rpc_timeout_s=30.0)
    base.update(kw)
    return FLConfig(**base)


def test_corrupt_payload_rejected_and_survivor_finishes(tmp_path, table):
    cfg = _cfg(tmp_path, round_deadline_s=1.0, quorum=0.5)
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    bad_cfg = dataclasses.replace(cfg, fault_corrupt=True)
    res = {}
    good = FLClient(cfg, lambda: FakeTrainer(table, 1.0), name="good", target=f"127.0.0.1:{port}")
    bad = FLClient(bad_cfg, lambda: FakeTrainer(table, 5.0), name="bad", target=f"127.0.0.1:{port}")

    def run_bad():
        try:
            res["bad"] = bad.run()
        except grpc.RpcError as e:
            res["bad"] = e.code()
    ts = [threading.Thread(target=lambda: res.__setitem__("good", good.run())), threading.Thread(target=run_bad)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    srv.stop()
    assert res["good"] == "FIN"
    assert res["bad"] == grpc.StatusCode.INVALID_ARGUMENT
    # the corrupt client's update never entered the average: the global is the survivor's alone
    e = table.entries[0]
    assert np.allclose(srv.state.global_flat[e.offset:e.offset + e.size], 1.0 * cfg.max_rounds)
    assert srv.state.history[0].dropped == ["bad"]


def test_log_upload_multichunk_is_appended(tmp_path, table):
    logs = tmp_path / "client" / "logs" / "run1"
    logs.mkdir(parents=True)
    blob = os.urandom(int(2.5 * 2**20))
    (logs / "events.out").write_bytes(blob)
    (logs / "small.txt").write_bytes(b"hello")
    server_dir = tmp_path / "server"
    server_dir.mkdir()
    cfg = _cfg(tmp_path, num_clients=1, max_rounds=1, upload_logs=True, log_dir=str(tmp_path / "client" / "logs"),
               log_chunk_mb=1, work_dir=str(server_dir))
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    c = FLClient(cfg, lambda: FakeTrainer(table), name="c", target=f"127.0.0.1:{port}")
    assert c.run() == "FIN"
    srv.stop()
    got = list(server_dir.rglob("events.out"))
    assert len(got) == 1 and got[0].read_bytes() == blob           # 3 chunks, appended (reference kept the last)
    assert [p.read_bytes() for p in server_dir.rglob("small.txt")] == [b"hello"]


def test_phase_timings_logged(tmp_path, table):
    cfg = _cfg(tmp_path, metrics_file=str(tmp_path / "m.jsonl"))
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    cs = [FLClient(cfg, lambda: FakeTrainer(table), name=f"c{i}", target=f"127.0.0.1:{port}") for i in range(2)]
    ts = [threading.Thread(target=c.run) for c in cs]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    srv.stop()
    for c in cs:
        assert [p["round"] for p in c.phases] == [1, 2]
        assert all(p["upload_s"] >= 0 and p["wait_s"] >= 0 and p["payload_bytes"] > 0 for p in c.phases)
    recs = [json.loads(x) for x in open(tmp_path / "m.jsonl")]
    assert sum(r.get("kind") == "phases" for r in recs) == 4


def test_stale_round_submit_and_fin_while_polling(table):
    """Appendix A2 (stale submit returned None) and A3 (FIN while polling was never handled)."""
    st_ = RoundState(np.zeros(table.total, np.float32), max_rounds=1, register_window_s=0.2, num_clients=2)
    assert st_.ready("a", 0)["state"] == SW and st_.ready("b", 0)["state"] == SW
    flat = np.ones(table.total, np.float32)
    assert st_.submit("a", 7, flat, 1.0)[0] == RESP_ACY                  # stale round: a real reply, not None
    assert st_.submit("a", 1, flat, 1.0)[0] == RESP_ACY
    out = {}
    t = threading.Thread(target=lambda: out.__setitem__("v", st_.version(1, 1, wait_s=5.0)))
    t.start()
    time.sleep(0.1)
    assert st_.submit("b", 1, flat, 1.0)[0] == FIN                       # last round closes -> FIN
    t.join(5)
    assert out["v"][0] == FIN                                            # the long-poller is released with FIN
    assert st_.version(1, 1)[0] == FIN
    st_.stop()


def test_version_long_poll_wakes_on_new_global(table):
    st_ = RoundState(np.zeros(table.total, np.float32), max_rounds=3, register_window_s=0.2, num_clients=2)
    st_.ready("a", 0)
    st_.ready("b", 0)
    assert st_.version(1, 1, wait_s=0.0)[0] == WAIT
    out = {}
    t0 = time.monotonic()
    t = threading.Thread(target=lambda: out.__setitem__("v", (st_.version(1, 1, wait_s=10.0), time.monotonic())))
    t.start()
    time.sleep(0.2)
    st_.submit("a", 1, np.ones(table.total, np.float32), 1.0)
    assert st_.submit("b", 1, np.ones(table.total, np.float32), 1.0)[0] == RESP_ARY
    t.join(5)
    (state, conf), t_ret = out["v"]
    assert state == NOT_WAIT and conf["current_round"] == 2 and t_ret - t0 < 3.0
    st_.stop()


@settings(max_examples=12, deadline=None)
@given(n_clients=st.integers(2, 6), rounds=st.integers(1, 3), seed=st.integers(0, 1000))
def test_concurrent_submits_aggregate_exactly_once_per_round(n_clients, rounds, seed):
    """Many threads racing TRAIN_DONE: every round is aggregated exactly once with every client's update
    (the reference could double-aggregate or lose counts, Appendix A8)."""
    total = 64
    st_ = RoundState(np.zeros(total, np.float32), max_rounds=rounds, register_window_s=5.0, num_clients=n_clients)
    names = [f"c{i}" for i in range(n_clients)]
    for n in names:
        assert st_.ready(n, 0)["state"] == SW
    rng = np.random.default_rng(seed)
    barrier = threading.Barrier(n_clients)
    errors = []

    def client(i):
        try:
            for r in range(1, rounds + 1):
                barrier.wait(timeout=10)
                time.sleep(float(rng.random()) * 1e-3)
                state, conf = st_.submit(names[i], r, np.full(total, float(i + r), np.float32), 1.0 + i)
                if state == RESP_ACY:                          # wait for the round to close
                    while st_.version(r, r, wait_s=2.0)[0] == WAIT:
                        pass
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    ts = [threading.Thread(target=client, args=(i,)) for i in range(n_clients)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(30)
    st_.stop()
    assert not errors
    assert [h.round for h in st_.history] == list(range(1, rounds + 1))
    assert all(sorted(h.clients) == sorted(names) for h in st_.history)
    w = np.array([1.0 + i for i in range(n_clients)])
    expect = float((w * (np.arange(n_clients) + rounds)).sum() / w.sum())
    assert np.allclose(st_.global_flat, expect)
    assert st_.finished
