"""Build recipe: libgome.so (HIP for gfx950 + host C++) and the oracle checker.

Everything is built in-tree so the shared objects travel to the GPU box with the
repository snapshot (they are git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gome_amd")
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libgome.so")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "build", "liboracle.so")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ARCH = os.environ.get("GOME_OFFLOAD_ARCH", "gfx950")

SOURCES = [os.path.join(CSRC, "engine.hip"), os.path.join(CSRC, "host.cpp"), os.path.join(CSRC, "loadgen.cpp")]
HEADERS = (sorted(glob.glob(os.path.join(CSRC, "*.h"))) + sorted(glob.glob(os.path.join(CSRC, "*.inc"))) +
           sorted(glob.glob(os.path.join(ROOT, "include", "gome", "*.h"))) + [os.path.abspath(__file__)])


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))
    return r


# SimplifyCFG's common-instruction sinking merges stores to different fields of the hot
# kernel's per-level structs into one store through a phi of pointers, which keeps the
# struct in scratch memory (a memory round trip on the per-order path).  Disable it.
DEVICE_FLAGS = ["-mllvm", "-sink-common-insts=false"]


def build_engine(force: bool = False, extra: list[str] | None = None) -> str:
    if force or _stale(LIB, SOURCES + HEADERS):
        tmp = LIB + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-result", *DEVICE_FLAGS, "-I", os.path.join(ROOT, "include"),
               *SOURCES, "-o", tmp] + (extra or [])
        _run(cmd)
        os.replace(tmp, LIB)
    return LIB


def build_stamps() -> str:
    """Diagnostic build with in-kernel s_memtime phase stamps (never used by the product)."""
    out = os.path.join(PKG, "libgome_stamps.so")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DGOME_STAMPS", *DEVICE_FLAGS,
           "-I", os.path.join(ROOT, "include"), *SOURCES, "-o", out]
    _run(cmd)
    return out


def build_oracle(force: bool = False) -> str:
    src = os.path.join(ORACLE_DIR, "gome_oracle.c")
    deps = [src, os.path.join(ROOT, "include", "gome", "gome_abi.h")]
    if force or _stale(ORACLE_LIB, deps):
        os.makedirs(os.path.dirname(ORACLE_LIB), exist_ok=True)
        tmp = ORACLE_LIB + ".tmp"
        _run(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-Wall", src, "-o", tmp])
        os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


def build_all(force: bool = False) -> None:
    build_engine(force)
    build_oracle(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print(LIB)
    print(ORACLE_LIB)
