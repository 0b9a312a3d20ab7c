"""In-process gRPC server on an ephemeral port + K client threads."""
import threading

import numpy as np
import pytest

from crack_detection_federatedlearning_grpc_amd.config import FLConfig
from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer

from fakes import FakeTrainer


def _cfg(tmp_path, **kw):
    base = dict(register_window_s=2.0, ready_stall_s=0.0, num_clients=2, poll_period_s=0.05, long_poll_s=1.0,
                max_rounds=3, client_weight_file="", server_weight_file=str(tmp_path / "server_weights/w.pickle"),
                work_dir=str(tmp_path), rpc_timeout_s=30.0)
    base.update(kw)
    return FLConfig(**base)


def _run(cfg, deltas, ns, table, names=None):
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    trainers, clients, results = [], [], {}
    for i, (d, n) in enumerate(zip(deltas, ns)):
        tr = FakeTrainer(table, d, n)
        trainers.append(tr)
        c = FLClient(cfg, (lambda tr=tr: tr), name=(names[i] if names else f"c{i}"), target=f"127.0.0.1:{port}")
        clients.append(c)
    ths = [threading.Thread(target=lambda c=c: results.__setitem__(c.name, c.run())) for c in clients]
    for t in ths:
        t.start()
    for t in ths:
        t.join(60)
    srv.stop()
    return srv, trainers, results


@pytest.mark.parametrize("codec", ["flat", "pickle"])
def test_two_clients_fedavg_to_fin(tmp_path, table, codec):
    cfg = _cfg(tmp_path, codec=codec)
    srv, trainers, results = _run(cfg, [1.0, 3.0], [10, 10], table)
    assert results == {"c0": "FIN", "c1": "FIN"}
    # every round: each client adds its delta to the broadcast global; equal n -> plain mean
    # round r global = r * mean(delta) = 2r
    w = srv.state.global_flat
    e = table.entries[0]
    assert np.allclose(w[e.offset:e.offset + e.size], 2.0 * cfg.max_rounds)
    assert [r.round for r in srv.state.history] == [1, 2, 3]
    assert trainers[0].rounds == [1, 2, 3] and trainers[1].rounds == [1, 2, 3]
    assert (tmp_path / "server_weights/w.pickle").exists()


def test_weighted_fedavg(tmp_path, table):
    cfg = _cfg(tmp_path, max_rounds=1)
    srv, _, results = _run(cfg, [1.0, 4.0], [30, 10], table)
    assert set(results.values()) == {"FIN"}
    e = table.entries[0]
    assert np.allclose(srv.state.global_flat[e.offset], (1.0 * 30 + 4.0 * 10) / 40)


def test_late_client_rejected(tmp_path, table):
    cfg = _cfg(tmp_path, num_clients=1, max_rounds=1)
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    c0 = FLClient(cfg, lambda: FakeTrainer(table), name="a", target=f"127.0.0.1:{port}")
    assert c0.run() == "FIN"
    c1 = FLClient(cfg, lambda: FakeTrainer(table), name="b", target=f"127.0.0.1:{port}")
    assert c1.run() in ("CTW", "FIN")
    srv.stop()


def test_straggler_dropped_at_deadline(tmp_path, table):
    # client c1 crashes at round 2; the deadline + quorum lets the survivor finish
    cfg = _cfg(tmp_path, round_deadline_s=1.5, quorum=0.5, max_rounds=3)
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    import dataclasses
    bad = dataclasses.replace(cfg, fault_drop_round=2)
    res = {}
    c0 = FLClient(cfg, lambda: FakeTrainer(table, 1.0), name="good", target=f"127.0.0.1:{port}")
    c1 = FLClient(bad, lambda: FakeTrainer(table, 1.0), name="bad", target=f"127.0.0.1:{port}")

    def run_bad():
        try:
            res["bad"] = c1.run()
        except SystemExit:
            res["bad"] = "crashed"
    ts = [threading.Thread(target=lambda: res.__setitem__("good", c0.run())), threading.Thread(target=run_bad)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    srv.stop()
    assert res == {"good": "FIN", "bad": "crashed"}
    assert any(r.dropped == ["bad"] for r in srv.state.history)
