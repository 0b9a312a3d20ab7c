"""TensorBoard event files without TensorFlow (the reference's ``TensorBoard(log_dir, histogram_freq=1)`` callback,
/root/reference/client_fit_model.py:153-154,166; SURVEY §2.2 "TensorBoard summary writer").

The ``tensorflow.Event`` / ``Summary`` / ``HistogramProto`` messages are declared from descriptors (same field
numbers as TensorFlow's ``event.proto`` / ``summary.proto``, so TensorBoard reads the files) and framed as
TFRecords by the native module (masked CRC32C, ``csrc/native/tfrecord.cpp``).

Layout written by :class:`KerasTensorBoard` per FL round, as Keras does: ``<log_dir>/<YYYYmmdd-HHMMSS>-<round>/train``
and ``.../validation`` with per-epoch scalars ``epoch_loss`` / ``epoch_accuracy`` and, every ``histogram_freq``
epochs, one histogram per weight array (``<layer>/<weight>_0``).
"""
from __future__ import annotations

import os
import socket
import time
from typing import Dict, Iterable, List, Optional

import numpy as np
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from .._native_loader import native

_F = descriptor_pb2.FieldDescriptorProto


def _build():
    fd = descriptor_pb2.FileDescriptorProto(name="cfl_tb_event.proto", package="tensorflow", syntax="proto3")
    h = fd.message_type.add(name="HistogramProto")
    for i, n in enumerate(["min", "max", "num", "sum", "sum_squares"], 1):
        h.field.add(name=n, number=i, label=_F.LABEL_OPTIONAL, type=_F.TYPE_DOUBLE)
    for i, n in ((6, "bucket_limit"), (7, "bucket")):
        f = h.field.add(name=n, number=i, label=_F.LABEL_REPEATED, type=_F.TYPE_DOUBLE)
        f.options.packed = True
    s = fd.message_type.add(name="Summary")
    v = s.nested_type.add(name="Value")
    v.field.add(name="tag", number=1, label=_F.LABEL_OPTIONAL, type=_F.TYPE_STRING)
    v.field.add(name="simple_value", number=2, label=_F.LABEL_OPTIONAL, type=_F.TYPE_FLOAT, oneof_index=0)
    v.field.add(name="histo", number=5, label=_F.LABEL_OPTIONAL, type=_F.TYPE_MESSAGE,
                type_name=".tensorflow.HistogramProto", oneof_index=0)
    v.oneof_decl.add(name="value")
    s.field.add(name="value", number=1, label=_F.LABEL_REPEATED, type=_F.TYPE_MESSAGE,
                type_name=".tensorflow.Summary.Value")
    e = fd.message_type.add(name="Event")
    e.field.add(name="wall_time", number=1, label=_F.LABEL_OPTIONAL, type=_F.TYPE_DOUBLE)
    e.field.add(name="step", number=2, label=_F.LABEL_OPTIONAL, type=_F.TYPE_INT64)
    e.field.add(name="file_version", number=3, label=_F.LABEL_OPTIONAL, type=_F.TYPE_STRING, oneof_index=0)
    e.field.add(name="summary", number=5, label=_F.LABEL_OPTIONAL, type=_F.TYPE_MESSAGE,
                type_name=".tensorflow.Summary", oneof_index=0)
    e.oneof_decl.add(name="what")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"tensorflow.{n}"))  # noqa: E731
    return get("Event"), get("Summary"), get("HistogramProto")


Event, Summary, HistogramProto = _build()


def _default_buckets() -> np.ndarray:
    """TensorFlow's default histogram bucket limits (histogram.cc: +-1e-12 * 1.1^k up to 1e20, plus +-DBL_MAX)."""
    pos, v = [], 1e-12
    while v < 1e20:
        pos.append(v)
        v *= 1.1
    return np.array([-1.7976931348623157e308] + [-x for x in reversed(pos)] + [0.0] + pos + [1.7976931348623157e308])


_BUCKETS = _default_buckets()


def histogram(values: np.ndarray) -> "HistogramProto":
    x = np.asarray(values, np.float64).ravel()
    h = HistogramProto()
    if x.size == 0:
        return h
    h.min, h.max, h.num = float(x.min()), float(x.max()), float(x.size)
    h.sum, h.sum_squares = float(x.sum()), float((x * x).sum())
    # bucket i counts values in (limit[i-1], limit[i]]; keep the non-empty buckets (TF drops empty runs too)
    idx = np.searchsorted(_BUCKETS, x, side="left")
    counts = np.bincount(idx, minlength=len(_BUCKETS))
    nz = np.nonzero(counts)[0]
    h.bucket_limit.extend(_BUCKETS[nz].tolist())
    h.bucket.extend(counts[nz].astype(np.float64).tolist())
    return h


class EventWriter:
    """One ``events.out.tfevents.<time>.<host>`` file; records are appended and flushed per event."""

    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}")
        self._f = open(self.path, "ab")
        self._write(Event(wall_time=time.time(), step=0, file_version="brain.Event:2"))

    def _write(self, ev) -> None:
        self._f.write(native().tfrecord.frame(ev.SerializeToString()))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        s = Summary()
        s.value.add(tag=tag, simple_value=float(value))
        self._write(Event(wall_time=time.time(), step=int(step), summary=s))

    def add_histogram(self, tag: str, values: np.ndarray, step: int) -> None:
        s = Summary()
        s.value.add(tag=tag, histo=histogram(values))
        self._write(Event(wall_time=time.time(), step=int(step), summary=s))

    def close(self) -> None:
        self._f.close()


def read_events(path: str) -> List["Event"]:
    with open(path, "rb") as f:
        recs = native().tfrecord.unframe(f.read())
    out = []
    for r in recs:
        e = Event()
        e.ParseFromString(r)
        out.append(e)
    return out


class KerasTensorBoard:
    """Per-round Keras-style TensorBoard logs for the local fit (train/ + validation/ writers)."""

    def __init__(self, log_dir: str, current_round: int, histogram_freq: int = 1):
        self.dir = os.path.join(log_dir, time.strftime("%Y%m%d-%H%M%S") + f"-{current_round}")
        self.train = EventWriter(os.path.join(self.dir, "train"))
        self.val = EventWriter(os.path.join(self.dir, "validation"))
        self.histogram_freq = histogram_freq

    def on_epoch_end(self, epoch: int, logs: Dict[str, float], weights: Optional[Iterable] = None) -> None:
        for k in ("loss", "accuracy"):
            if k in logs:
                self.train.add_scalar(f"epoch_{k}", logs[k], epoch)
            if f"val_{k}" in logs:
                self.val.add_scalar(f"epoch_{k}", logs[f"val_{k}"], epoch)
        if weights is not None and self.histogram_freq and epoch % self.histogram_freq == 0:
            for name, arr in weights:
                self.train.add_histogram(name.replace(":0", "_0"), arr, epoch)

    def close(self) -> None:
        self.train.close()
        self.val.close()
