#!/bin/bash
# Profile recipe (runs on the GPU box): kernel trace + stats, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (they do not fit one pass on gfx950).
# usage: bash profiles/run_rocprof.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run \
  -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/fetch -o run \
  -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1 || exit 2
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/write -o run \
  -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1 || exit 3
echo done
