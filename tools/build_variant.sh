#!/bin/bash
# Variant builds of libgome.so for A/B runs in one GPU call (bench.py / tests pick one with
# GOME_LIB=<path>).  usage: bash tools/build_variant.sh <name> <hipcc -D flags...>
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
python3 - "$NAME" "$@" <<'PY'
import sys
from gome_amd import build
name, flags = sys.argv[1], sys.argv[2:]
out = build.LIB.replace("libgome.so", f"libgome_{name}.so")
cmd = [build.HIPCC, f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
       "-Wno-unused-result", *build.DEVICE_FLAGS, "-I", build.os.path.join(build.ROOT, "include"), *build.SOURCES,
       "-o", out, *flags]
build._run(cmd)
print(out)
PY
