"""Build recipe: libgome.so (HIP for gfx950 + host C++) and the oracle checker.

Everything is built in-tree so the shared objects travel to the GPU box with the
repository snapshot (they are git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import glob
import hashlib
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

SOURCES = [os.path.join(CSRC, "engine.hip"), os.path.join(CSRC, "host.cpp"), os.path.join(CSRC, "consume.cpp"),
           os.path.join(CSRC, "loadgen.cpp")]
HEADERS = (sorted(glob.glob(os.path.join(CSRC, "*.h"))) + sorted(glob.glob(os.path.join(CSRC, "*.inc"))) +
           sorted(glob.glob(os.path.join(ROOT, "include", "gome", "*.h"))) + [os.path.abspath(__file__)])


def _digest(deps: list[str], cmd: list[str]) -> str:
    """sha256 over the build command and every source's path and content (not mtimes: the
    snapshot that travels to the GPU box does not keep them in order).  Paths inside the tree are
    hashed relative to it, so a checkout elsewhere (the GPU box's snapshot) is not stale."""
    rel = [os.path.relpath(c, ROOT) if os.path.isabs(c) and c.startswith(ROOT + os.sep) else c for c in cmd]
    h = hashlib.sha256("\0".join(rel).encode())
    for d in sorted(deps):
        h.update(os.path.relpath(d, ROOT).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale(out: str, deps: list[str], cmd: list[str]) -> tuple[bool, str]:
    """(needs a build, digest): the output is current iff its sidecar <out>.sha256 names the
    digest of these sources built by this command."""
    dig = _digest(deps, cmd)
    try:
        with open(out + ".sha256") as f:
            cur = f.read().strip() == dig
    except OSError:
        cur = False
    return (not cur or not os.path.exists(out)), dig


def _stamp(out: str, dig: str) -> None:
    with open(out + ".sha256", "w") as f:
        f.write(dig + "\n")


BUILT: list[str] = []  # what the last build_* calls compiled (build() reports it)


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
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-result", *DEVICE_FLAGS, "-I", os.path.join(ROOT, "include"),
           *SOURCES, "-o", tmp] + (extra or [])
    stale, dig = _stale(LIB, SOURCES + HEADERS, cmd)
    if force or stale:
        _run(cmd)
        os.replace(tmp, LIB)
        _stamp(LIB, dig)
        BUILT.append(LIB)
    return LIB


def build_stamps() -> str:
    """Diagnostic build with in-kernel s_memtime phase stamps (never used by the product)."""
    out = os.path.join(PKG, "libgome_stamps.so")
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-DGOME_STAMPS", *DEVICE_FLAGS,
           "-I", os.path.join(ROOT, "include"), *SOURCES, "-o", out]
    _run(cmd)
    return out


def build_host_sanitized(force: bool = False) -> str:
    """Test-only: the host layer (host.cpp, consume.cpp, loadgen.cpp: JSON decode, interning,
    pre-pool markers, MatchResult render, load generator; no device code) built by g++ with
    AddressSanitizer + UndefinedBehaviorSanitizer into libgome_host_asan.so, never loaded by the
    product.  tests/test_host_sanitizers.py loads it (GOME_LIB, the sanitizer runtimes preloaded)
    under the decoder and consumer tests."""
    out = os.path.join(PKG, "libgome_host_asan.so")
    tmp = out + ".tmp"
    srcs = [s for s in SOURCES if not s.endswith(".hip")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fPIC", "-shared", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-Wall", "-Wno-unused-result",
           "-I", os.path.join(ROOT, "include"), *srcs, "-o", tmp]
    stale, dig = _stale(out, srcs + HEADERS, cmd)
    if force or stale:
        _run(cmd)
        os.replace(tmp, out)
        _stamp(out, dig)
        BUILT.append(out)
    return out


def build_oracle(force: bool = False) -> str:
    src = os.path.join(ORACLE_DIR, "gome_oracle.c")
    deps = [src, os.path.join(ROOT, "include", "gome", "gome_abi.h")]
    tmp = ORACLE_LIB + ".tmp"
    cmd = ["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-Wall", src, "-o", tmp]
    stale, dig = _stale(ORACLE_LIB, deps, cmd)
    if force or stale:
        os.makedirs(os.path.dirname(ORACLE_LIB), exist_ok=True)
        _run(cmd)
        os.replace(tmp, ORACLE_LIB)
        _stamp(ORACLE_LIB, dig)
        BUILT.append(ORACLE_LIB)
    return ORACLE_LIB


def build_all(force: bool = False) -> list[str]:
    """Build what is stale; returns the outputs compiled by this call (empty: all current)."""
    n = len(BUILT)
    build_engine(force)
    build_oracle(force)
    return BUILT[n:]


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print(LIB)
    print(ORACLE_LIB)
