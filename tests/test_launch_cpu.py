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


def _bench(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK"), timeout=300):
    env = dict(os.environ)
    for k in drop:
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)


def test_bench_refuses_world_size_mismatch():
    """Under a launcher (WORLD_SIZE set) --gpus N must equal the world size (no silent 1-rank number)."""
    p = _bench(["--gpus", "2", "--steps", "1"], env_extra={"WORLD_SIZE": "1"})
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stdout + p.stderr


def test_bench_self_launch_refuses_more_rccl_ranks_than_gpus():
    """--gpus N without a launcher: with RCCL, N > visible GPUs is refused before any rank starts (no GPU here)."""
    p = _bench(["--gpus", "2", "--steps", "1"])
    assert p.returncode != 0 and "visible GPUs" in p.stdout + p.stderr, p.stdout + p.stderr


def test_bench_self_launch_propagates_rank_failure():
    """--gpus 2 --dist-backend gloo spawns two ranks; here they fail (no GPU): the parent exits non-zero, says which."""
    p = _bench(["--gpus", "2", "--steps", "1", "--dist-backend", "gloo", "--spawn-timeout", "240"])
    assert p.returncode != 0
    assert "[spawn] rank" in p.stderr, p.stderr[-3000:]
    assert '"metric"' not in p.stdout


_CHILD = r"""
import json, os, sys, time
r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
assert int(os.environ["MASTER_PORT"]) > 0 and os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
mode = sys.argv[1]
if mode == "ok":
    print(json.dumps({"rank": r, "world": w, "port": os.environ["MASTER_PORT"]}) if r == 0 else f"noise {r}",
          flush=True)
elif mode == "fail":
    if r == 1:
        sys.exit(3)
    time.sleep(600)
else:
    if os.environ.get("CHILD_PID_DIR"):
        open(os.path.join(os.environ["CHILD_PID_DIR"], f"rank{r}.pid"), "w").write(str(os.getpid()))
    time.sleep(600)
"""


def test_spawn_local_ranks_env_relay_failure_and_timeout(tmp_path, capfd):
    import time
    sys.path.insert(0, ROOT)
    from crack_detection_federatedlearning_grpc_amd.parallel.spawn import spawn_local_ranks
    script = tmp_path / "child.py"
    script.write_text(_CHILD)
    assert spawn_local_ranks(str(script), ["ok"], 3, timeout=120) == 0
    out, err = capfd.readouterr()
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert len(lines) == 1 and '"world": 3' in lines[0]          # only rank 0's stdout on stdout
    assert "[rank 1] noise 1" in err and "[rank 2] noise 2" in err
    t0 = time.monotonic()
    assert spawn_local_ranks(str(script), ["fail"], 2, timeout=120) != 0   # rank 1 fails -> rank 0 stopped
    assert time.monotonic() - t0 < 60
    assert "rank 1 exited with 3" in capfd.readouterr().err
    t0 = time.monotonic()
    assert spawn_local_ranks(str(script), ["hang"], 2, timeout=3) == 124
    assert time.monotonic() - t0 < 30
    assert "timed out" in capfd.readouterr().err


def test_spawn_stops_ranks_when_the_launcher_is_terminated(tmp_path):
    """The ranks run in their own sessions (no terminal signal reaches them): a SIGTERM to the launcher must still
    stop every rank it started (advisor r5: only a failed rank / the timeout used to)."""
    import signal
    import time
    script = tmp_path / "child.py"
    script.write_text(_CHILD)
    launcher = (f"import sys; sys.path.insert(0, {ROOT!r}); "
                f"from crack_detection_federatedlearning_grpc_amd.parallel.spawn import spawn_local_ranks; "
                f"sys.exit(spawn_local_ranks({str(script)!r}, ['hang'], 2))")
    p = subprocess.Popen([sys.executable, "-c", launcher], env=dict(os.environ, CHILD_PID_DIR=str(tmp_path)))
    pids = []
    t0 = time.monotonic()
    while len(pids) < 2 and time.monotonic() - t0 < 60:
        time.sleep(0.1)
        pids = [int(f.read_text()) for f in tmp_path.glob("rank*.pid") if f.read_text()]
    assert len(pids) == 2, "ranks did not start"
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) != 0
    for pid in pids:
        t0 = time.monotonic()
        while True:
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            assert time.monotonic() - t0 < 15, f"rank pid {pid} survived the launcher"
            time.sleep(0.1)
