"""Loaders for the two in-tree native modules.

``native()``  -> host C++ module (built on demand with g++; needed by CPU tests too).
``hip()``     -> HIP kernel module ``_C``; on a machine with a GPU a missing/broken module is a hard error (no silent
                 eager fallback), on a CPU-only machine callers get a clear RuntimeError.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_native = None
_hip = None


def native():
    global _native
    if _native is None:
        with _lock:
            if _native is None:
                from . import _build
                if not _build.is_current(_build.native_path(), _build.native_key()):
                    _build.build_native(verbose=False)      # missing or stale (stamp != source hash)
                _native = importlib.import_module(__package__ + "._native")
    return _native


def hip():
    global _hip
    if _hip is None:
        with _lock:
            if _hip is None:
                from . import _build
                if not _build.is_current(_build.hip_path(), _build.hip_key()):
                    # missing, or built from other sources than these (its stamp != the source hash): never
                    # import a stale kernel module silently
                    state = "stale" if os.path.exists(_build.hip_path()) else "not built"
                    if os.environ.get("CFL_NO_JIT_BUILD"):
                        raise RuntimeError(f"HIP extension _C is {state} (run __graft_entry__.build())")
                    print(f"[native] HIP extension _C is {state}; rebuilding", flush=True)
                    _build.build_hip(verbose=True)
                import torch  # noqa: F401  (libtorch must be loaded before _C)
                _hip = importlib.import_module(__package__ + "._C")
                # launch-shape knobs for A/B runs: CFL_TUNE="9=1,3=256" (launch.h TuneKey = value)
                for kv in filter(None, os.environ.get("CFL_TUNE", "").split(",")):
                    k, v = kv.split("=")
                    _hip.set_tune(int(k), int(v))
    return _hip
