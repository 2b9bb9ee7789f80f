#!/bin/bash
# Kernel trace of the sustained config-5 run: the last batches' timelines (what grows with depth).
set -o pipefail
O=gpurun_out/${1:-r4c5t}
export TMPDIR=/tmp
mkdir -p $O
timeout -k 10 900 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/trace -o run \
  -- python3 bench.py --workload config5 --steps ${2:-200} --warmup 3 --pool-levels 335544320 --no-cpu-baseline \
  --no-phase-pass --e2e-steps 0 --consumer-msgs 0 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
f=$(find $O/trace -name "run_kernel_trace.csv" | head -1)
python3 tools/timeline.py $f 2 > $O/timeline_last.txt
python3 tools/timeline.py $f 190 > $O/timeline_early.txt
head -3 $O/timeline_last.txt; head -3 $O/timeline_early.txt
