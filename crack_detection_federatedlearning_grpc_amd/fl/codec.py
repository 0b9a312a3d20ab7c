"""Weight payload codecs for the gRPC data plane.

Reference wire format: ``pickle.dumps(list[np.ndarray])`` in ``buffer_chunk`` (fl_client.py:63, fl_server.py:179,
client_fit_model.py:51,231) - 8,236,708 B per 112-array fp32 payload - and ``pickle.loads`` of network bytes.

Two codecs here:
* ``flat`` (default): ``b"CFLW"`` magic, u32 header length, JSON header (dtype, shapes, n_samples, meta), then the
  arrays back to back as little-endian fp32 or bf16 - no code execution on decode, 2x smaller in bf16.
* ``pickle`` (compat): produces exactly what the reference sends; decoding goes through a RESTRICTED unpickler that
  only admits NumPy array reconstruction, so a malicious peer cannot execute code (the reference unpickles
  arbitrary network bytes: fl_server.py:179, client_fit_model.py:51).
``decode`` auto-detects the format.
"""
from __future__ import annotations

import io
import json
import pickle
import struct
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

MAGIC = b"CFLW"


def f32_to_bf16_bits(a: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16 bit pattern (uint16); NaN stays NaN."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = 0x7FC0
    return r


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def encode_flat(arrays: Sequence[np.ndarray], n_samples: int = 0, dtype: str = "fp32",
                meta: Optional[Dict[str, Any]] = None) -> bytes:
    shapes = [list(np.shape(a)) for a in arrays]
    hdr = json.dumps({"v": 1, "dtype": dtype, "shapes": shapes, "n_samples": int(n_samples),
                      "meta": meta or {}}).encode()
    flat = np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in arrays]) if arrays else \
        np.zeros(0, np.float32)
    body = f32_to_bf16_bits(flat).tobytes() if dtype == "bf16" else flat.astype("<f4").tobytes()
    return MAGIC + struct.pack("<I", len(hdr)) + hdr + body


def decode_flat(buf: bytes) -> Tuple[List[np.ndarray], Dict[str, Any]]:
    if buf[:4] != MAGIC:
        raise ValueError("not a flat weight payload")
    (hl,) = struct.unpack("<I", buf[4:8])
    hdr = json.loads(buf[8:8 + hl].decode())
    body = memoryview(buf)[8 + hl:]
    sizes = [int(np.prod(s)) if s else 1 for s in hdr["shapes"]]
    total = sum(sizes)
    if hdr["dtype"] == "bf16":
        if len(body) != 2 * total:
            raise ValueError("truncated bf16 payload")
        flat = bf16_bits_to_f32(np.frombuffer(body, dtype="<u2"))
    elif hdr["dtype"] == "fp32":
        if len(body) != 4 * total:
            raise ValueError("truncated fp32 payload")
        flat = np.frombuffer(body, dtype="<f4").astype(np.float32)
    else:
        raise ValueError(f"unknown dtype {hdr['dtype']}")
    out, off = [], 0
    for s, n in zip(hdr["shapes"], sizes):
        out.append(flat[off:off + n].reshape(s).copy())
        off += n
    return out, hdr


_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("_codecs", "encode"),
    ("numpy.core.numeric", "_frombuffer"), ("numpy._core.numeric", "_frombuffer"),
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module: str, name: str):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to unpickle {module}.{name}")


def encode_pickle(arrays: Sequence[np.ndarray]) -> bytes:
    return pickle.dumps([np.asarray(a, np.float32) for a in arrays])


def decode_pickle(buf: bytes) -> List[np.ndarray]:
    obj = _SafeUnpickler(io.BytesIO(buf)).load()
    if not isinstance(obj, (list, tuple)) or not all(isinstance(a, np.ndarray) for a in obj):
        raise ValueError("pickle payload is not a list of ndarrays")
    return [np.asarray(a) for a in obj]


def encode(arrays: Sequence[np.ndarray], codec: str = "flat", n_samples: int = 0, wire_dtype: str = "fp32") -> bytes:
    if codec == "pickle":
        return encode_pickle(arrays)
    return encode_flat(arrays, n_samples=n_samples, dtype=wire_dtype)


def decode(buf: bytes) -> Tuple[List[np.ndarray], Dict[str, Any]]:
    if not buf:
        raise ValueError("empty weight payload")
    if buf[:4] == MAGIC:
        return decode_flat(buf)
    return decode_pickle(buf), {"n_samples": 0, "dtype": "fp32"}


def load_weight_file(path: str) -> List[np.ndarray]:
    with open(path, "rb") as f:
        return decode(f.read())[0]


def save_weight_file(path: str, arrays: Sequence[np.ndarray]) -> None:
    """Write the reference's ``weights.pickle`` hand-off file (client_fit_model.py:238-240), creating the dir."""
    import os
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)   # reference never creates it
    import threading
    tmp = f"{path}.{os.getpid()}.{threading.get_ident()}.tmp"   # unique per writer (processes and threads)
    with open(tmp, "wb") as f:
        f.write(encode_pickle(arrays))
    os.replace(tmp, path)
