#!/bin/bash
# Kernel + memory-copy + HIP API trace of the default-length bench (e2e stalls).
# usage: tools/prof_e2e_api.sh <tag> [workload]
out=gpurun_out/$1; w=${2:-config3}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $GRAFT_REPO_ROOT/$out/prof -o e2e --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/$out/prof_bench.json 2> $GRAFT_REPO_ROOT/$out/prof.err
