"""The host worker pool (gome_amd/csrc/host_pool.h) under stress: 300k small jobs back to back, every
task run exactly once, no hang (tools/pool_stress.cpp; its watchdog exits 3 with the pool's state).
The consumer's decode, queue-order passes and render all run on this pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_pool_runs_every_task_once(tmp_path):
    exe = tmp_path / "pool_stress"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", os.path.join(ROOT, "tools", "pool_stress.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, (r.returncode, r.stdout, r.stderr)
