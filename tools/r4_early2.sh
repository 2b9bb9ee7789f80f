#!/bin/bash
# Early plans on the host path: the early tests, then e2e A/B (blit-kernel copies too).
set -o pipefail
O=gpurun_out/${1:-r4x4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_early.py -x -v --timeout 400 --timeout-method thread > $O/tests.txt 2>&1 \
  || { tail -60 $O/tests.txt; exit 2; }
tail -3 $O/tests.txt
VARIANTS="d2:2: d2off:2:GOME_EARLY=0 d3sb:3:GOME_D2H_STREAM=1,HSA_ENABLE_SDMA=0" bash tools/r4_e2e2.sh ${1:-r4x4} "config3 config2"
