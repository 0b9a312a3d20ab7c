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


def test_dropped_client_not_waited_for_again(table):
    """A client dropped at a deadline leaves the live set: later rounds close as soon as the live clients report
    (no second deadline wait), the quorum is a fraction of the live clients, and the client rejoins when it
    speaks again."""
    from crack_detection_federatedlearning_grpc_amd.fl.state import RESP_ACY, RESP_ARY, RoundState
    st_ = RoundState(np.zeros(table.total, np.float32), max_rounds=5, register_window_s=0.2, num_clients=3,
                     round_deadline_s=0.5, quorum=0.5)
    for n in "abc":
        st_.ready(n, 0)
    one = np.ones(table.total, np.float32)
    for n in "ab":
        assert st_.submit(n, 1, one, 1.0)[0] == RESP_ACY
    assert st_.submit("c", 1, one, 1.0)[0] == RESP_ARY                # round 1: everyone
    assert st_.submit("a", 2, one, 1.0)[0] == RESP_ACY
    assert st_.submit("b", 2, one, 1.0)[0] == RESP_ACY                # c is silent: deadline drops it
    import time
    t0 = time.monotonic()
    while st_.current_round == 2 and time.monotonic() - t0 < 5:
        time.sleep(0.02)
    assert st_.history[1].dropped == ["c"] and st_.live == {"a", "b"}
    assert st_.submit("a", 3, one, 1.0)[0] == RESP_ACY
    t1 = time.monotonic()
    assert st_.submit("b", 3, one, 1.0)[0] == RESP_ARY                # closes at once: c is not expected
    assert time.monotonic() - t1 < 0.2 and st_.history[2].dropped == []
    assert st_.submit("c", 2, one, 1.0)[0] == RESP_ACY                # c speaks again (stale round) -> live
    assert st_.live == {"a", "b", "c"}
    for n in "ab":
        assert st_.submit(n, 4, one, 1.0)[0] == RESP_ACY              # round 4 waits for c again
    assert st_.submit("c", 4, one, 1.0)[0] == RESP_ARY
    assert sorted(st_.history[3].clients) == ["a", "b", "c"]
    st_.stop()


def test_reference_pickle_client_against_default_server(tmp_path, table):
    """Drop-in wire compatibility: the reference client's exact verb sequence (fl_client.py:77-175) - READY
    without a codec key, PARAM without a name, raw ``pickle.dumps(list[np.ndarray])`` uploads - against the
    DEFAULT server config gets pickles it can ``pickle.loads`` (client_fit_model.py:51,231) on every reply path
    (PARAM, RESP_ARY, NOT_WAIT), while a flat-advertising client on the same server gets flat payloads."""
    import pickle
    import grpc
    from crack_detection_federatedlearning_grpc_amd.fl import codec
    from crack_detection_federatedlearning_grpc_amd.fl import proto as P
    from crack_detection_federatedlearning_grpc_amd.fl.rpc import TransportServiceStub, channel_options
    cfg = _cfg(tmp_path, max_rounds=2)                                   # default codec config
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    got = {}

    def one(stub, req):
        return list(stub.transport(iter([req]), timeout=30))[-1]

    def reference_client():
        with grpc.insecure_channel(f"127.0.0.1:{port}", options=channel_options(512)) as ch:
            stub = TransportServiceStub(ch)
            rep = one(stub, P.transportRequest(ready_req=P.ReadyReq(
                type="R", cname="client42", state=P.ON, config={"current_round": P.Scalar(scint32=0)})))
            conf = rep.ready_rep.config
            cr, mv = conf["current_round"].scint32, conf["model_version"].scint32
            params = pickle.loads(one(stub, P.transportRequest(update_req=P.UpdateReq(type="P"))
                                      ).update_rep.buffer_chunk)              # fl_client.py:98-103
            got["p"] = params
            one(stub, P.transportRequest(update_req=P.UpdateReq(type="T", cname="client42", state=P.TRAINING)))
            while True:
                w = [a + 1.0 for a in params]
                rep = one(stub, P.transportRequest(update_req=P.UpdateReq(
                    type="D", buffer_chunk=pickle.dumps(w), state=P.TRAIN_DONE, cname="client42",
                    current_round=cr))).update_rep
                st = rep.config["state"].scstring
                if st == "FIN":
                    return
                if st == "RESP_ARY":
                    params = pickle.loads(rep.buffer_chunk)
                    got.setdefault("ary", []).append(params)
                    cr, mv = rep.config["current_round"].scint32, rep.config["model_version"].scint32
                    continue
                assert st == "RESP_ACY"
                while True:                                                  # fl_client.py:136-155
                    vr = one(stub, P.transportRequest(version_req=P.VersionReq(type="P", config={
                        "model_version": P.Scalar(scint32=mv), "current_round": P.Scalar(scint32=cr)}))
                             ).version_rep
                    if vr.state == P.NOT_WAIT:
                        params = pickle.loads(vr.buffer_chunk)
                        got.setdefault("nw", []).append(params)
                        cr, mv = vr.config["current_round"].scint32, vr.config["model_version"].scint32
                        break
                    if vr.state == P.FIN:
                        return
                    time.sleep(0.05)

    import time
    flat_trainer = FakeTrainer(table, 3.0)
    ours = FLClient(dataclasses_replace(cfg, codec="flat"), lambda: flat_trainer, name="ours",
                    target=f"127.0.0.1:{port}")
    blobs = []
    orig = ours._params
    ours._params = lambda stub: blobs.append(orig(stub)) or blobs[-1]
    res = {}
    ts = [threading.Thread(target=reference_client), threading.Thread(target=lambda: res.__setitem__("o", ours.run()))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    srv.stop()
    assert res["o"] == "FIN"
    assert len(got["p"]) == len(table.entries) and all(isinstance(a, np.ndarray) for a in got["p"])
    assert len(got.get("ary", [])) + len(got.get("nw", [])) == 1             # round-2 params reached it as pickle
    r2 = (got.get("ary") or got.get("nw"))[0]
    e = table.entries[0]
    assert np.allclose(r2[0], 0.5 * (1.0 + 3.0)) and r2[0].shape == tuple(e.shape)
    assert blobs and blobs[0][:4] == codec.MAGIC                             # the flat client got flat


def dataclasses_replace(cfg, **kw):
    import dataclasses
    return dataclasses.replace(cfg, **kw)
