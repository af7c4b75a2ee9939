"""bench.py contract rehearsed on the CPU: 2 ranks over gloo through
torch.distributed.run (127.0.0.1 rendezvous), one JSON line from rank 0 with
the fields the driver reads; the overlapped and synchronous MIX both run."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("mode", ["overlap", "sync"])
def test_bench_two_ranks_cpu(mode):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--device", "cpu", "--requests", "8",
           "--per-request", "16", "--hash-bits", "12", "--latency-iters", "5", "--mix-mode", mode,
           "--batches-per-step", "2", "--dist-engines", "none"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 2 * 2 * 8 * 16 and mode in out["config"]["mix"]
    assert out["config"]["world_size_observed"] == 2
    assert out["timed_samples_per_rank"] == 2 * 2 * 8 * 16
    assert 0.0 < out["update_fraction"] <= 1.0


def test_bench_spawns_ranks_without_torchrun():
    """--gpus N without WORLD_SIZE: bench.py launches the N ranks itself"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "1", "--device", "cpu", "--requests", "4", "--per-request", "8",
           "--hash-bits", "10", "--latency-iters", "2", "--batches-per-step", "1", "--dist-engines", "none"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == 2 and out["config"]["world_size_observed"] == 2
