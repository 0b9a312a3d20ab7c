import os
import pickle

import numpy as np
import pytest

from crack_detection_federatedlearning_grpc_amd.fl import codec
from crack_detection_federatedlearning_grpc_amd.fl import proto as P
from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable, forward_flops_per_image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_param_table_matches_keras(table):
    # 112 arrays, 82 trainable, 2,058,145 params, 3,776 non-trainable
    assert len(table) == 112
    assert sum(e.trainable for e in table.entries) == 82
    assert table.num_params == 2058145
    assert table.num_params - table.num_trainable == 3776
    names = [e.keras_name for e in table.entries]
    assert names[:6] == ["conv2d/kernel:0", "conv2d/bias:0", "batch_normalization/gamma:0",
                         "batch_normalization/beta:0", "batch_normalization/moving_mean:0",
                         "batch_normalization/moving_variance:0"]
    assert table.entry("conv2d_transpose_2", "kernel").shape == (3, 3, 128, 256)   # (kh,kw,out,in)
    assert table.entry("separable_conv2d", "depthwise_kernel").shape == (3, 3, 32, 1)
    assert names[-2:] == ["conv2d_8/kernel:0", "conv2d_8/bias:0"]


def test_flops():
    assert abs(forward_flops_per_image(128) / 1e9 - 1.25) < 0.01
    assert abs(forward_flops_per_image(256) / 1e9 - 5.0) < 0.01


def test_flat_list_roundtrip(table):
    f = table.init_flat(3)
    assert np.array_equal(table.from_list(table.to_list(f)), f)
    with pytest.raises(ValueError):
        table.from_list(table.to_list(f)[:-1])


def test_proto_roundtrip_and_schema():
    r = P.transportRequest(update_req=P.UpdateReq(type="D", buffer_chunk=b"xyz", cname="c", state=P.TRAIN_DONE,
                                                  current_round=3, file_len=17))
    r2 = P.transportRequest.FromString(r.SerializeToString())
    assert r2.update_req.current_round == 3 and r2.update_req.state == P.State.TRAIN_DONE
    rep = P.ReadyRep(config={"state": P.Scalar(scstring="SW"), "current_round": P.Scalar(scint32=1)})
    assert P.ReadyRep.FromString(rep.SerializeToString()).config["state"].scstring == "SW"
    assert P.VersionRep(state="FIN").state == P.FIN   # fl_server.py:145/204 passes the string "FIN"
    with open(os.path.join(ROOT, "proto", "transport.proto")) as f:
        assert f.read() == P.to_proto_text()


def test_compat_modules_import():
    import transport_pb2
    import transport_pb2_grpc
    assert transport_pb2.State.WAIT == P.WAIT
    assert hasattr(transport_pb2_grpc, "TransportServiceStub")


@pytest.mark.parametrize("dt", ["fp32", "bf16"])
def test_flat_codec(table, dt):
    arrs = table.to_list(table.init_flat(1))
    blob = codec.encode(arrs, "flat", n_samples=123, wire_dtype=dt)
    out, hdr = codec.decode(blob)
    assert hdr["n_samples"] == 123
    tol = 0 if dt == "fp32" else 1e-2
    for a, b in zip(arrs, out):
        assert a.shape == b.shape
        assert np.allclose(a, b, atol=tol, rtol=tol)
    if dt == "bf16":
        assert len(blob) < 0.6 * len(codec.encode(arrs, "flat"))


def test_pickle_codec_is_reference_format(table):
    arrs = table.to_list(table.init_flat(1))
    blob = codec.encode(arrs, "pickle")
    ref = pickle.loads(blob)    # what the reference does (fl_server.py:179)
    assert len(ref) == 112 and all(np.array_equal(a, b) for a, b in zip(ref, arrs))
    out, _ = codec.decode(blob)
    assert all(np.array_equal(a, b) for a, b in zip(out, arrs))


def test_pickle_codec_refuses_code():
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))
    with pytest.raises(pickle.UnpicklingError):
        codec.decode(pickle.dumps([Evil()]))


def test_bf16_rounding():
    x = np.array([1.0, 1.00390625, 1.01171875, -2.5, np.inf, np.nan], np.float32)
    y = codec.bf16_bits_to_f32(codec.f32_to_bf16_bits(x))
    assert y[0] == 1.0 and y[1] == 1.0 and y[2] == 1.015625 and y[3] == -2.5 and np.isinf(y[4]) and np.isnan(y[5])
