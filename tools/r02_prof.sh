#!/bin/bash
# Round-2 evidence of the final tree on one MI355X, per workload (configs 3, 4, 5): a kernel
# trace + stats of a short bench run, then FETCH_SIZE and WRITE_SIZE passes (separate runs) of
# the roofline kernel; then a kernel + memory-copy trace of the pipelined e2e leg (config 3).
# usage: bash tools/r02_prof.sh <tag>; summarise with python tools/summarize_r02i.py <tag>
set -o pipefail
tag=${1:-r02i}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for w in config3 config4 config5; do
  mkdir -p $out/$w
  B="$GRAFT_REPO_ROOT/bench.py --workload $w --steps 5 --warmup 2 --e2e-steps 0 --no-cpu-baseline"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$w/trace -o run --output-format csv -- python3 $B \
    > $out/$w/trace_bench.json 2> $out/$w/trace.err || { echo "ktrace $w failed"; exit 1; }
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $pmc --kernel-include-regex "k_flow_plan_head" -d $out/$w/$pmc -o pmc \
      --output-format csv -- python3 $B > $out/$w/$pmc.json 2> $out/$w/$pmc.err || { echo "pmc $w $pmc failed"; exit 1; }
  done
  echo "$w done"
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/e2e -o e2e --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --e2e-steps 6 --no-cpu-baseline \
  > $out/e2e_bench.json 2> $out/e2e.err || { echo "e2e trace failed"; exit 1; }
echo "e2e done"
