#!/bin/bash
# GPU check used during development: parity tests, then a short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
TAG=${1:-chk}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 2; }
tail -1 gpurun_out/${TAG}_bench.log
