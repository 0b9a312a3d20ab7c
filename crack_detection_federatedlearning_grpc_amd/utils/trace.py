"""Phase markers for rocprofv3 (roctx ranges) and host wall-clock phase timers.

The reference has no tracing beyond the Keras TensorBoard callback. Here every FL phase - local
training epochs, validation, FedAvg aggregation, upload, wait - can be bracketed by a roctx range, so a
``rocprofv3 --marker-trace --kernel-trace`` timeline groups the kernels by phase. Ranges are emitted only when
``CFL_ROCTX=1`` (the roctx library is dlopen-ed from ROCm; without it, or on CPU hosts, markers are no-ops), and
``PhaseTimer`` keeps per-phase host wall-clock totals either way. With ranges on, a phase also synchronises the
GPU when it ends, so the asynchronously replayed hipGraphs of a phase land inside its range (profiling mode: the
cross-phase overlap is given up for an exact attribution).

    with phase("train/epoch"):
        ...
"""
from __future__ import annotations

import ctypes
import os
import time
from contextlib import contextmanager
from typing import Dict, Iterator, Optional

_lib: Optional[ctypes.CDLL] = None
_tried = False


def _roctx() -> Optional[ctypes.CDLL]:
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if os.environ.get("CFL_ROCTX", "0") != "1":
        return None
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so"):
        try:
            lib = ctypes.CDLL(os.path.join(rocm, "lib", name))
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            break
        except (OSError, AttributeError):
            continue
    return _lib


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextmanager
def phase(name: str, timer: Optional["PhaseTimer"] = None) -> Iterator[None]:
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if lib is not None:
            _sync()
        if timer is not None:
            timer.add(name, time.perf_counter() - t0)
        if lib is not None:
            lib.roctxRangePop()


def _sync() -> None:
    import sys
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        torch.cuda.synchronize()


class PhaseTimer:
    """Accumulated host wall-clock seconds per phase name."""

    def __init__(self) -> None:
        self.totals: Dict[str, float] = {}
        self.counts: Dict[str, int] = {}

    def add(self, name: str, seconds: float) -> None:
        self.totals[name] = self.totals.get(name, 0.0) + seconds
        self.counts[name] = self.counts.get(name, 0) + 1

    def as_dict(self) -> Dict[str, float]:
        return {k: round(v, 6) for k, v in self.totals.items()}
