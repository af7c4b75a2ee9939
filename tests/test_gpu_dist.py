"""The multi-rank GPU training path (bench.py: GPU request scan, overlapped
MIX with the reference's back-to-back trigger) with two ranks sharing one
GPU over gloo - a functional rehearsal of what the driver runs over RCCL on
an 8-GPU node."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_one_gpu_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "2", "--dist-backend", "gloo",
           "--requests", "64", "--per-request", "32", "--hash-bits", "16", "--latency-iters", "5",
           "--batches-per-step", "3",
           # the distributed engine records at a rehearsal size (the BASELINE-scale
           # fills are the driver's 8-GPU run; tests/test_eight_ranks.py covers them on CPU)
           "--dist-engines", "arow", "--dist-train-seconds", "1", "--dist-engine-rows", "2000"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 2 * 3 * 64 * 32
    assert out["config"]["world_size_observed"] == 2 and out["update_fraction"] > 0
    assert "MIXes in the timed steps" in out["config"]["mix"]
    assert out["heldout_accuracy"] > 0.9
