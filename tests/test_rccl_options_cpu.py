"""RCCL group plumbing on the CPU (verdict r5 item 3): the options the FedAvg process group is built with (high-priority
collective stream, channel cap), the rank environment the launchers hand their children, and the refusal of more
RCCL clients than visible GPUs in ``fl/launch.py`` and ``fl_client.py`` (``bench.py`` already refused)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from crack_detection_federatedlearning_grpc_amd.parallel import rccl  # noqa: E402


def test_channel_cap_resolution(monkeypatch):
    monkeypatch.delenv("CFL_RCCL_MAX_CHANNELS", raising=False)
    assert rccl.rccl_channel_cap() == rccl.RCCL_MAX_CHANNELS_DEFAULT == 16
    assert rccl.rccl_channel_cap(-1) == 16                  # config default: env / built-in
    monkeypatch.setenv("CFL_RCCL_MAX_CHANNELS", "8")
    assert rccl.rccl_channel_cap() == 8 and rccl.rccl_channel_cap(-1) == 8
    assert rccl.rccl_channel_cap(24) == 24                  # explicit config wins
    assert rccl.rccl_channel_cap(0) == 0                    # 0 = RCCL's own choice


def test_pg_options_high_priority_stream_and_max_ctas(monkeypatch):
    monkeypatch.delenv("CFL_RCCL_MAX_CHANNELS", raising=False)
    o = rccl.rccl_pg_options()
    assert o.is_high_priority_stream is True and o.config.max_ctas == 16
    o0 = rccl.rccl_pg_options(0)
    assert o0.is_high_priority_stream is True and o0.config.max_ctas < 0     # unset: RCCL default


def test_rank_env_plumbing(monkeypatch):
    monkeypatch.delenv("CFL_RCCL_MAX_CHANNELS", raising=False)
    e = rccl.rccl_env({"PATH": "/bin"})
    assert e["NCCL_MAX_NCHANNELS"] == "16" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin"
    assert rccl.rccl_env({"NCCL_MAX_NCHANNELS": "4"})["NCCL_MAX_NCHANNELS"] == "4"   # the user's choice stays
    assert "NCCL_MAX_NCHANNELS" not in rccl.rccl_env({}, cap=0)
    assert rccl.rccl_env({}, cap=12)["NCCL_MAX_NCHANNELS"] == "12"


def test_placement_refuses_more_rccl_clients_than_gpus(monkeypatch):
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    assert rccl.rccl_placement_error(1, "cuda", "nccl") is None
    err = rccl.rccl_placement_error(2, "auto", "nccl")
    assert err and "2 RCCL clients need 2 visible GPUs" in err and "found 1" in err
    assert rccl.rccl_placement_error(2, "auto", "gloo") is None           # gloo rehearsal may share a card
    assert rccl.rccl_placement_error(2, "cpu", "nccl") is None            # CPU clients run gloo anyway
    assert rccl.rccl_placement_error(0, "cuda", "nccl", rank=0) is None
    assert "rank 1 needs 2" in rccl.rccl_placement_error(0, "cuda", "nccl", rank=1)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert rccl.rccl_placement_error(2, "auto", "nccl") is None           # CPU host: the clients fall back
    assert rccl.rccl_placement_error(2, "cuda", "nccl")                   # asked for GPUs, none there


def test_launch_refuses_before_starting_anything(monkeypatch, capsys):
    from crack_detection_federatedlearning_grpc_amd.fl import launch
    from crack_detection_federatedlearning_grpc_amd.fl import server
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)

    def no_server(*a, **k):
        raise AssertionError("the server must not start")
    monkeypatch.setattr(server, "FLServer", no_server)
    rc = launch.main(["--data-plane", "rccl", "--num-clients", "2", "--device", "cuda", "--port", "0"])
    assert rc == 2 and "refused" in capsys.readouterr().err


def test_fl_client_refuses_a_rank_without_its_own_gpu(monkeypatch):
    import fl_client
    from crack_detection_federatedlearning_grpc_amd import config as C
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    monkeypatch.setenv("LOCAL_RANK", "1")
    cfg = C.FLConfig(data_plane="rccl", device="cuda")
    with pytest.raises(SystemExit, match="rank 1 needs 2 visible GPUs"):
        fl_client.run(cfg)


def test_server_hands_out_the_configured_rendezvous_address():
    from crack_detection_federatedlearning_grpc_amd import config as C
    assert C.FLConfig().dist_addr == "127.0.0.1"
    assert C.from_args(None, dist_addr="10.0.0.5").dist_addr == "10.0.0.5"
