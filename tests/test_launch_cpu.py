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


def test_bench_refuses_world_size_mismatch():
    """bench.py --gpus N must run as N torch.distributed ranks; a mismatch fails loudly (no silent 1-rank number)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"], cwd=root,
                       env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stdout
