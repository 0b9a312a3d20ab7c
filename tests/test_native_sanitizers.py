"""The C++ runtime (HDF5, contours, resize) is clean under AddressSanitizer + UBSan (host code only)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_native_runtime_under_asan_ubsan(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sanitize_native.py"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:] + r.stderr[-3000:])
    assert "sanitized native selftest ok" in r.stdout
