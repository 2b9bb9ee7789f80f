"""The native host layer under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 "race
detection / sanitizers": ASan / UBSan on the C++ CPU code).

consume.cpp parses untrusted AMQP bodies (UTF-8, escapes, nesting to depth 10000) and host.cpp
renders MatchResult JSON; both run on the consumer's host thread pool.  gome_amd/build.py builds
them (no device code) with -fsanitize=address,undefined into libgome_host_asan.so, and the decoder
and consumer tests run against it in a child process (GOME_LIB, the sanitizer runtimes preloaded
into the interpreter): the edge-case and mutated corpora, the Hypothesis damage corpus (truncated
UTF-8, deep nesting, long escapes, duplicate keys), the pre-pool markers and the multi-threaded
renderer.  A sanitizer report aborts the child (abort_on_error, halt_on_error)."""
import os
import subprocess
import sys

import pytest

from gome_amd import build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_host_layer_under_asan_and_ubsan():
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if not asan or not ubsan:
        pytest.skip("gcc's sanitizer runtimes are not installed")
    lib = build.build_host_sanitized()
    env = dict(os.environ, LD_PRELOAD=f"{asan} {ubsan}", GOME_LIB=lib,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:strict_string_checks=1:detect_stack_use_after_return=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("GOME_TEST_POISON", None)
    probe = subprocess.run([sys.executable, "-c", "import gome_amd.abi as a; l = a.load_library(); "
                            "assert not hasattr(l, 'gome_create'); print(l._name)"],
                           env=env, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert probe.returncode == 0 and probe.stdout.strip() == lib, probe.stdout + probe.stderr
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        "tests/test_decode_native.py", "tests/test_consumer.py"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=1500)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-6000:]
    assert r.returncode == 0, out[-6000:]
    assert " passed" in out
