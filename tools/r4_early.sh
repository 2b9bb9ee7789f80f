#!/bin/bash
# Early-plan check: its GPU tests, then an A/B with and without it (and the cold books' stream).
set -o pipefail
O=gpurun_out/${1:-r4x}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_early.py tests/test_gpu_device_async.py -x -v --timeout 400 \
  --timeout-method thread > $O/tests.txt 2>&1 || { tail -60 $O/tests.txt; exit 2; }
tail -3 $O/tests.txt
E2E=0 bash tools/r4_abenv.sh ${1:-r4x} "${2:-config3}" 10 "on:GOME_X=0" "off:GOME_EARLY=0" "coldx:GOME_COLD_EARLY=1"
