#!/bin/bash
# Kernel trace (+ stats) of a short bench run of one workload.  usage: tools/trace_workload.sh tag workload
set -o pipefail
cd $GRAFT_REPO_ROOT; out=$GRAFT_REPO_ROOT/gpurun_out/$1; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $2 --steps 3 --warmup 1 --e2e-steps 0 --no-cpu-baseline > $out/bench_trace.log 2>&1 || exit 1
echo "trace $2 done"
