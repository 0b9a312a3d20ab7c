"""fl.launch on CPU: server + 2 client processes, RCCL data plane rehearsed over gloo, real (tiny) U-Net training."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launch_two_cpu_clients_rccl_gloo(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "crack_detection_federatedlearning_grpc_amd.fl.launch", "--preset", "cpu-plumbing",
           "--data-plane", "rccl", "--max-rounds", "2", "--port", "0", "--work-dir", str(tmp_path),
           "--client-weight-file", str(tmp_path / "w.pickle"), "--server-weight-file", str(tmp_path / "s.pickle"),
           "--register-window-s", "60", "--validate", "0"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "2 round(s)" in r.stdout
    assert (tmp_path / "s.pickle").exists()
