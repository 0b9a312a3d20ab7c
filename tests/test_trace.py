"""utils/trace.py: roctx phase ranges (CFL_ROCTX=1) and host phase timers."""
import subprocess
import sys
import time

from crack_detection_federatedlearning_grpc_amd.utils.trace import PhaseTimer, phase


def test_phase_timer_accumulates():
    t = PhaseTimer()
    for _ in range(3):
        with phase("a", t):
            time.sleep(0.01)
    with phase("b", t):
        pass
    assert t.counts == {"a": 3, "b": 1}
    assert 0.03 <= t.totals["a"] < 1.0 and t.totals["b"] < 0.1


def test_roctx_ranges_load_and_nest():
    code = ("import os; os.environ['CFL_ROCTX']='1'\n"
            "from crack_detection_federatedlearning_grpc_amd.utils import trace\n"
            "with trace.phase('outer'):\n"
            "    with trace.phase('inner'):\n"
            "        trace.mark('m')\n"
            "print('lib' if trace._roctx() is not None else 'nolib')\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() in ("lib", "nolib")
