#!/bin/bash
# Kernel + memory-copy trace of the pipelined e2e path of one workload.
# usage: tools/prof_e2e.sh <tag> [workload]
out=gpurun_out/$1; w=${2:-config3}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o e2e --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --steps 3 --warmup 2 --e2e-steps 6 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/prof_bench.json 2> $GRAFT_REPO_ROOT/$out/prof.err
