"""Static checks on the gfx950 code objects (CPU-only: hipcc cross-compiles): no kernel spills to scratch memory.

A private array written under a branch, or indexed at run time, is placed in scratch (per-lane memory behind the
vector cache) instead of registers - a silent 2-5x slowdown for the memory-bound kernels. The compiler's
resource remarks report it as ``ScratchSize``.
"""
import glob
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _remarks(src, tmp):
    out = os.path.join(tmp, os.path.basename(src) + ".o")
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", f"-I{ROOT}/csrc",
                        f"-I{ROOT}/csrc/kernels", "-c", src, "-o", out, "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    kernels, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = t.split(":", 1)[1].strip()
            kernels[cur] = {}
        elif cur and ":" in t:
            k, v = t.split(":", 1)
            kernels[cur][k.strip()] = v.strip()
    return kernels


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_no_kernel_uses_scratch(tmp_path):
    srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        results = list(ex.map(lambda s: _remarks(s, str(tmp_path)), srcs))
    bad = []
    n = 0
    for src, ks in zip(srcs, results):
        for name, info in ks.items():
            n += 1
            if int(info.get("ScratchSize [bytes/lane]", "0")) != 0:
                bad.append((os.path.basename(src), name, info.get("ScratchSize [bytes/lane]")))
    assert n > 20
    assert not bad, f"kernels using scratch: {bad}"
