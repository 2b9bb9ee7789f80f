#!/bin/bash
# Host-path tests, then the e2e leg with the device-written event copy-out (depth 2 / 3).
set -o pipefail
O=gpurun_out/${1:-r4o}
mkdir -p $O
timeout -k 10 900 python -u -m pytest $(grep -ln "submit_async" tests/test_gpu*.py tests/test_consumer.py) -x -q --timeout 400 \
  --timeout-method thread -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 2; }
tail -2 $O/tests.txt
VARIANTS="d2:2: d3:3: d2k:2:GOME_OUT_KERNEL=1" bash tools/r4_e2e2.sh ${1:-r4o} "config2 config3"
