"""BASELINE config 1: 2-client FedAvg over gRPC on CPU, tiny U-Net 64x64, synthetic masks, to FIN."""
import threading

import numpy as np

from crack_detection_federatedlearning_grpc_amd import config
from crack_detection_federatedlearning_grpc_amd.fl.client import FLClient
from crack_detection_federatedlearning_grpc_amd.fl.server import FLServer
from crack_detection_federatedlearning_grpc_amd.train.factory import make_trainer


def test_two_cpu_clients_real_training(tmp_path, table):
    cfg = config.from_args(None, preset="cpu-plumbing", max_rounds=2, work_dir=str(tmp_path),
                           client_weight_file=str(tmp_path / "saved_weight/weights.pickle"),
                           server_weight_file=str(tmp_path / "server_weights/weights.pickle"),
                           snapshot_dir=str(tmp_path / "snap"), predict_round=2)
    srv = FLServer(cfg, table=table)
    port = srv.start(0)
    res = {}
    clients = [FLClient(cfg, (lambda r=r: make_trainer(cfg, f"c{r}", r, table, "cpu")), name=f"c{r}",
                        target=f"127.0.0.1:{port}") for r in range(2)]
    ts = [threading.Thread(target=lambda c=c: res.__setitem__(c.name, c.run())) for c in clients]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    srv.stop()
    assert res == {"c0": "FIN", "c1": "FIN"}
    assert len(srv.state.history) == 2
    # the server's global equals the mean of the two clients' final local weights (equal n_k)
    w0 = table.from_list(clients[0].trainer.get_weights())
    w1 = table.from_list(clients[1].trainer.get_weights())
    assert np.allclose(srv.state.global_flat, 0.5 * (w0 + w1), atol=1e-6)
    assert all(np.isfinite(h["loss"]) for c in clients for h in c.history)
    assert "predict" in clients[0].history[-1]
    assert (tmp_path / "snap" / "global.h5").exists() and (tmp_path / "saved_weight/weights.pickle").exists()
    # resume: a new server picks up round/version from the snapshot
    cfg2 = config.from_args(None, preset="cpu-plumbing", snapshot_dir=str(tmp_path / "snap"), resume=True,
                            work_dir=str(tmp_path))
    srv2 = FLServer(cfg2, table=table)
    assert srv2.state.current_round == 3 and np.allclose(srv2.state.global_flat, srv.state.global_flat)
    # resuming the snapshot of a FINISHED run under the same max_rounds: READY / VERSION answer FIN, no extra round
    cfg3 = config.from_args(None, preset="cpu-plumbing", snapshot_dir=str(tmp_path / "snap"), resume=True,
                            work_dir=str(tmp_path), max_rounds=2)
    srv3 = FLServer(cfg3, table=table)
    assert srv3.state.finished
    assert srv3.state.ready("late", 0)["state"] == "FIN"
    assert srv3.state.version(srv3.state.model_version, 3)[0] == "FIN"
    assert not srv2.state.finished            # max_rounds 5 > 2 finished rounds: the run continues
