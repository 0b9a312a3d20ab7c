"""HBM batch planner (models/memplan.py): pure shape arithmetic, CPU only. The GPU side (planned bytes vs the
engine's measured allocation) is tests/test_gpu_kernels.py::test_memplan_matches_engine_allocation."""
import pytest

from crack_detection_federatedlearning_grpc_amd.config import PRESETS, from_args
from crack_detection_federatedlearning_grpc_amd.models import memplan as M


def test_activation_bytes_linear_in_batch():
    for S in (64, 256, 512):
        one = M.activation_bytes(1, S)
        assert M.activation_bytes(7, S) == 7 * one
        # 4x the pixels -> 4x the bytes
    assert M.activation_bytes(1, 512) == 4 * M.activation_bytes(1, 256)


def test_bf16_activation_budget_256():
    # 30 bf16 activation/gradient planes per image at 256^2 -> ~50 MiB per image (engine.py layout)
    mib = M.activation_bytes(1, 256) / 2**20
    assert 40 < mib < 60, mib


@pytest.mark.parametrize("S", [256, 512])
def test_plan_respects_hbm_and_index_limits(S):
    p = M.plan_batch(S, 288 * 10**9, 0.85, samples=8000)
    assert p.batch % 8 == 0 and p.batch > 16
    assert p.total_bytes <= p.budget_bytes
    assert M.largest_tensor_elems(p.batch, S) <= M.MAX_ELEMS
    assert p.limit in ("hbm", "index", "max_batch")


def test_512_plan_is_hbm_bound_on_mi355x():
    """With 64-bit element offsets the 512^2 plan on a 288 GB MI355X is bounded by HBM (batch ~1000), not by the
    kernels' index width (the old 2^30-element bound stopped at batch 256 / 58 GB)."""
    p = M.plan_batch(512, 288 * 10**9, 0.85, samples=8000)
    assert p.limit == "hbm" and p.batch >= 512, p.as_dict()
    assert M.largest_tensor_elems(p.batch, 512) > 2**30               # past the old bound
    assert M.largest_tensor_elems(p.batch, 512) <= M.MAX_ELEMS


def test_plan_hbm_bound_when_small():
    # a 16 GiB device is HBM-bound at 512^2
    p = M.plan_batch(512, 16 * 2**30, 0.9, samples=1000)
    assert p.limit == "hbm"
    assert p.total_bytes <= p.budget_bytes
    assert M.engine_bytes(p.batch + 8, 512) + p.dataset_bytes > p.budget_bytes


def test_plan_rejects_impossible():
    with pytest.raises(ValueError):
        M.plan_batch(512, 2**28, 0.9)


def test_preset_512_uses_planner():
    assert PRESETS["gpu8-512"]["batch_size"] == 0
    cfg = from_args(preset="gpu8-512")
    from crack_detection_federatedlearning_grpc_amd.train.factory import planned_batch
    b = planned_batch(cfg, "cpu")
    assert b >= 64 and M.largest_tensor_elems(b, 512) <= M.MAX_ELEMS


def test_deterministic_flag_parses(monkeypatch):
    """--deterministic / FL_DETERMINISTIC select the engine's deterministic reduction mode for the FL product path
    (models/engine.py HipBackend passes it to UNetEngine)."""
    from crack_detection_federatedlearning_grpc_amd.config import parse
    assert parse([]).deterministic is False
    assert parse(["--deterministic"]).deterministic is True
    monkeypatch.setenv("FL_DETERMINISTIC", "1")
    assert parse([]).deterministic is True
