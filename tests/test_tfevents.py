"""TensorBoard event files (native TFRecord framing + descriptor-built Event protos) and the local-fit hook."""
import glob
import os

import numpy as np

from crack_detection_federatedlearning_grpc_amd import config
from crack_detection_federatedlearning_grpc_amd._native_loader import native
from crack_detection_federatedlearning_grpc_amd.train.factory import make_trainer
from crack_detection_federatedlearning_grpc_amd.utils.tfevents import EventWriter, histogram, read_events


def test_crc32c_and_framing():
    t = native().tfrecord
    assert t.crc32c(b"123456789") == 0xE3069283            # CRC-32C check value
    recs = [b"", b"a", os.urandom(1000)]
    assert t.unframe(b"".join(t.frame(r) for r in recs)) == recs
    bad = bytearray(t.frame(b"payload"))
    bad[14] ^= 1
    try:
        t.unframe(bytes(bad))
        raise AssertionError("corruption not detected")
    except RuntimeError:
        pass


def test_event_writer_roundtrip(tmp_path):
    w = EventWriter(str(tmp_path))
    w.add_scalar("epoch_loss", 0.25, 3)
    x = np.random.default_rng(0).standard_normal(1000)
    w.add_histogram("conv2d/kernel_0", x, 3)
    w.close()
    evs = read_events(w.path)
    assert evs[0].file_version == "brain.Event:2"
    assert evs[1].step == 3 and evs[1].summary.value[0].tag == "epoch_loss"
    assert abs(evs[1].summary.value[0].simple_value - 0.25) < 1e-7
    h = evs[2].summary.value[0].histo
    assert h.num == 1000 and abs(h.sum - x.sum()) < 1e-6 and sum(h.bucket) == 1000
    assert list(h.bucket_limit) == sorted(h.bucket_limit)
    assert histogram(np.array([])).num == 0


def test_local_fit_writes_keras_style_logs(tmp_path):
    cfg = config.from_args(None, preset="cpu-plumbing", epochs=2, tensorboard=True, log_dir=str(tmp_path / "logs"))
    fit = make_trainer(cfg, "c", 0, device="cpu")
    fit.train_round(1)
    runs = glob.glob(str(tmp_path / "logs" / "*-1"))
    assert len(runs) == 1
    tr = read_events(glob.glob(os.path.join(runs[0], "train", "events.out.tfevents.*"))[0])
    va = read_events(glob.glob(os.path.join(runs[0], "validation", "events.out.tfevents.*"))[0])
    tags = {v.tag for e in tr[1:] for v in e.summary.value}
    assert {"epoch_loss", "epoch_accuracy", "conv2d/kernel_0"} <= tags
    assert sum(1 for e in va[1:] for v in e.summary.value if v.tag == "epoch_loss") == 2
