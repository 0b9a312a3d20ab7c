"""RCCL data plane of the FL client, rehearsed over gloo with world_size 2 (separate processes, CPU)."""
import multiprocessing as mp
import os
import threading

import numpy as np
import pytest


def _client_proc(port, name, delta, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from crack_detection_federatedlearning_grpc_amd.config import FLConfig
    from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    from crack_detection_federatedlearning_grpc_amd.parallel.rccl import RcclAggregator
    from fakes import FakeTrainer
    cfg = FLConfig(device="cpu", data_plane="rccl", num_clients=2, register_window_s=20, ready_stall_s=0,
                   poll_period_s=0.05, long_poll_s=1.0, max_rounds=2, client_weight_file="", rpc_timeout_s=60)
    table = ParamTable()
    tr = FakeTrainer(table, delta, n_samples=10 if delta < 2 else 30)
    c = FLClient(cfg, lambda: tr, name=name, target=f"127.0.0.1:{port}",
                 aggregator_factory=lambda info: RcclAggregator.from_ready_info(info, cfg))
    st = c.run()
    e = table.entries[0]
    q.put((name, st, float(tr.flat[e.offset])))


def test_rccl_mode_two_processes(tmp_path):
    from crack_detection_federatedlearning_grpc_amd.config import FLConfig
    from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    table = ParamTable()
    cfg = FLConfig(device="cpu", data_plane="rccl", num_clients=2, register_window_s=20, ready_stall_s=0,
                   max_rounds=2, work_dir=str(tmp_path), server_weight_file="", long_poll_s=1.0)
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_client_proc, args=(port, f"c{i}", d, q)) for i, d in enumerate([1.0, 5.0])]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(30)
    srv.stop()
    # weighted: round1 avg = (1*10 + 5*30)/40 = 4 ; round2: each adds its delta to 4 -> (5*10 + 9*30)/40 = 8
    vals = {n: v for n, _, v in res}
    assert all(st == "FIN" for _, st, _ in res)
    assert np.isclose(vals["c0"], 8.0) and np.isclose(vals["c1"], 8.0)
    e = table.entries[0]
    assert np.isclose(srv.state.global_flat[e.offset], 8.0)     # rank 0 uploaded the all-reduced model


def _client_proc_faulty(port, name, delta, drop_round, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from crack_detection_federatedlearning_grpc_amd.config import FLConfig
    from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    from crack_detection_federatedlearning_grpc_amd.parallel.rccl import RcclAggregator
    from fakes import FakeTrainer
    cfg = FLConfig(device="cpu", data_plane="rccl", num_clients=3, register_window_s=20, ready_stall_s=0,
                   poll_period_s=0.05, long_poll_s=1.0, max_rounds=3, client_weight_file="", rpc_timeout_s=60,
                   rccl_timeout_s=15.0, fault_drop_round=drop_round)
    table = ParamTable()
    tr = FakeTrainer(table, delta, n_samples=10)
    c = FLClient(cfg, lambda: tr, name=name, target=f"127.0.0.1:{port}",
                 aggregator_factory=lambda info: RcclAggregator.from_ready_info(info, cfg))
    st = c.run()
    q.put((name, st, c.fallbacks))


def test_rccl_peer_loss_falls_back_to_grpc(tmp_path):
    """a client dies after round 1; the survivors' round-2 collective fails, they abort the
    communicator and send their local weights over gRPC; the round deadline + quorum averages the survivors."""
    from crack_detection_federatedlearning_grpc_amd.config import FLConfig
    from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    table = ParamTable()
    cfg = FLConfig(device="cpu", data_plane="rccl", num_clients=3, register_window_s=20, ready_stall_s=0,
                   max_rounds=3, work_dir=str(tmp_path), server_weight_file="", long_poll_s=1.0,
                   round_deadline_s=3.0, quorum=0.6)
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    spec = [("c0", 1.0, 0), ("c1", 2.0, 0), ("c2", 4.0, 2)]
    ps = [ctx.Process(target=_client_proc_faulty, args=(port, n, d, r, q)) for n, d, r in spec]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in ps:
        p.join(30)
    srv.stop()
    assert sorted(n for n, _, _ in res) == ["c0", "c1"]
    assert all(st == "FIN" and fb == 1 for _, st, fb in res), res
    # round 1 over RCCL: (1+2+4)/3; round 2 over gRPC (survivors): mean of +1 / +2; round 3 likewise
    r1 = 7.0 / 3.0
    r2 = r1 + 1.5
    r3 = r2 + 1.5
    e = table.entries[0]
    assert np.isclose(srv.state.global_flat[e.offset], r3, atol=1e-5)
    # c2 left the live set at the round-2 deadline: round 3 closes without waiting for it again
    assert [h.dropped for h in srv.state.history] == [[], ["c2"], []]


def _client_proc_flat(port, name, delta, n, fail_bucket, metrics, q):
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from crack_detection_federatedlearning_grpc_amd.config import FLConfig
    from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    from crack_detection_federatedlearning_grpc_amd.parallel.rccl import RcclAggregator
    from fakes import FakeFlatTrainer
    cfg = FLConfig(device="cpu", data_plane="rccl", dist_backend="gloo", num_clients=2, register_window_s=20,
                   ready_stall_s=0, poll_period_s=0.05, long_poll_s=1.0, max_rounds=2, client_weight_file="",
                   rpc_timeout_s=60, rccl_timeout_s=20.0, metrics_file=metrics)
    table = ParamTable()
    tr = FakeFlatTrainer(table, delta, n_samples=n, fail_bucket=fail_bucket)
    c = FLClient(cfg, lambda: tr, name=name, target=f"127.0.0.1:{port}",
                 aggregator_factory=lambda info: RcclAggregator.from_ready_info(info, cfg))
    st = c.run()
    e = table.entries[0]
    q.put((name, st, float(tr.flat[e.offset]), c.fallbacks, [float(u[e.offset]) for u in tr.uploads]))


def _run_flat_pair(tmp_path, fail_bucket):
    import json
    from crack_detection_federatedlearning_grpc_amd.config import FLConfig
    from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    table = ParamTable()
    cfg = FLConfig(device="cpu", data_plane="rccl", num_clients=2, register_window_s=20, ready_stall_s=0,
                   max_rounds=2, work_dir=str(tmp_path), server_weight_file="", long_poll_s=1.0)
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_client_proc_flat,
                      args=(port, f"c{i}", d, n, fail_bucket, str(tmp_path / f"c{i}.jsonl"), q))
          for i, (d, n) in enumerate([(1.0, 10), (5.0, 30)])]
    for p in ps:
        p.start()
    res = {r[0]: r[1:] for r in (q.get(timeout=120) for _ in ps)}
    for p in ps:
        p.join(30)
    srv.stop()
    phases = {i: [json.loads(x) for x in open(tmp_path / f"c{i}.jsonl") if '"phases"' in x] for i in range(2)}
    return table, srv, res, phases


def test_rccl_device_path_sends_no_parameters(tmp_path):
    """The in-place (device-buffer) RCCL path end to end over gloo: the weighted average lands in every client's
    buffer, rank 0 alone uploads it, rank 1's payload is empty, and the server's RESP_ARY / NOT_WAIT replies carry
    no parameters to clients that hold the average already."""
    table, srv, res, phases = _run_flat_pair(tmp_path, fail_bucket=-1)
    assert all(r[0] == "FIN" and r[2] == 0 for r in res.values()), res
    assert np.isclose(res["c0"][1], 8.0) and np.isclose(res["c1"][1], 8.0)       # (see the two-process test)
    assert np.isclose(srv.state.global_flat[table.entries[0].offset], 8.0)
    assert all(p["data_plane"] == "rccl" for ph in phases.values() for p in ph)
    # ranks follow registration order, not the client names: look the ranks up in the phase records
    by_rank = {ph[0]["rank"]: ph for ph in phases.values()}
    assert sorted(by_rank) == [0, 1] and all(len({p["rank"] for p in ph}) == 1 for ph in phases.values())
    assert [p["payload_bytes"] for p in by_rank[1]] == [0, 0]                      # rank 1 uploads nothing
    assert all(p["payload_bytes"] > 0 for p in by_rank[0])
    # round 1's reply (RESP_ARY or NOT_WAIT) carried no parameters to either client
    assert all(p.get("reply_bytes", 0) == 0 for ph in phases.values() for p in ph), phases
    # async report (cfg.async_upload): round 1 was reported from a background thread while round 2 trained (its
    # phase record carries the exposed part: the collective + the join), the last round synchronously (FIN)
    for ph in phases.values():
        assert [p["round"] for p in ph] == [1, 2]
        assert [p.get("async_upload", False) for p in ph] == [True, False], ph
        assert ph[0]["exposed_s"] >= ph[0]["aggregate_s"] and ph[0]["join_wait_s"] >= 0.0


def test_rccl_failure_mid_bucket_uploads_local_model(tmp_path):
    """A collective lost after some buckets were scaled / reduced: the aggregator aborts the communicator and
    restores the local model, so the gRPC fallback uploads exactly the locally trained weights (not a mix of
    pre-scaled and reduced buckets) and the round is averaged over gRPC."""
    table, srv, res, phases = _run_flat_pair(tmp_path, fail_bucket=2)
    assert all(r[0] == "FIN" and r[2] == 1 for r in res.values()), res
    # each client's uploads: round 1 = its local model (delta), round 2 = 4 + delta (the gRPC average + delta)
    assert res["c0"][3] == [1.0, 5.0] and res["c1"][3] == [5.0, 9.0], res
    assert np.isclose(srv.state.global_flat[table.entries[0].offset], 8.0)
    assert all(p["data_plane"] == "grpc" for ph in phases.values() for p in ph)
    assert all(p["payload_bytes"] > 0 for ph in phases.values() for p in ph)


def _client_proc_fin(port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from crack_detection_federatedlearning_grpc_amd.config import FLConfig
    from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    from crack_detection_federatedlearning_grpc_amd.parallel.rccl import RcclAggregator
    from fakes import FakeTrainer
    cfg = FLConfig(device="cpu", data_plane="rccl", num_clients=1, register_window_s=20, ready_stall_s=0,
                   poll_period_s=0.05, long_poll_s=1.0, max_rounds=3, client_weight_file="", rpc_timeout_s=60)
    table = ParamTable()
    tr = FakeTrainer(table, 1.0, n_samples=10, sleep_s=1.5)
    c = FLClient(cfg, lambda: tr, name="c0", target=f"127.0.0.1:{port}",
                 aggregator_factory=lambda info: RcclAggregator.from_ready_info(info, cfg))
    st = c.run()
    e = table.entries[0]
    q.put((st, float(tr.flat[e.offset]), [h["round"] for h in c.history], list(tr.rounds)))


def test_async_report_fin_restores_the_round_average(tmp_path):
    """Advisor r4: with the asynchronous round report the client trains round r+1 before it learns the server's
    answer to round r. When that answer is FIN (here: the server ends the run after round 1 although it advertised
    3 rounds), the extra round is dropped from the history and the client ends at round 1's global model."""
    from crack_detection_federatedlearning_grpc_amd.config import FLConfig
    from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer
    from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable
    table = ParamTable()
    cfg = FLConfig(device="cpu", data_plane="rccl", num_clients=1, register_window_s=20, ready_stall_s=0,
                   max_rounds=3, work_dir=str(tmp_path), server_weight_file="", long_poll_s=1.0)
    srv = FLServer(cfg, global_flat=np.zeros(table.total, np.float32), table=table)
    port = srv.start(0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_client_proc_fin, args=(port, q))
    p.start()
    try:
        assert srv.state.wait_window_closed(60) == 1
        srv.state.max_rounds = 1                  # the run ends at round 1 (after the READY advertised 3)
        st, final, hist, trained = q.get(timeout=120)
    finally:
        p.join(30)
        srv.stop()
    assert st == "FIN"
    assert trained == [1, 2]                      # round 2 trained while round 1's report was pending ...
    assert hist == [1]                            # ... and was dropped
    assert np.isclose(final, 1.0)                 # the client ends at round 1's average (1 rank: its model)
    assert np.isclose(srv.state.global_flat[table.entries[0].offset], 1.0)
