#!/bin/bash
# Copy timeline of the e2e leg (config 2, three host batches in flight, events D2H on their own stream).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r4ct}
mkdir -p $O
GOME_D2H_STREAM=1 timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -T --output-format csv -d $O/trace -o run \
  -- python3 bench.py --workload config2 --steps 2 --warmup 1 --e2e-steps 6 --e2e-depth 3 --no-cpu-baseline \
  --consumer-msgs 0 --no-phase-pass > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
ls $O/trace
