#!/bin/bash
# Round-2 evidence set on one MI355X: default bench line (config 3), kernel trace + stats of a
# short config-3 run, FETCH_SIZE / WRITE_SIZE passes (k_flow_plan_head, k_match), PMC SQ pass.
set -o pipefail
tag=${1:-r02f}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag; mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; exit 1; }
echo "bench done"
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --e2e-steps 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 $B > $out/trace_bench.json 2> $out/trace.err || { echo "ktrace failed"; exit 1; }
echo "ktrace done"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "k_match$|k_match\(|k_flow_plan_head" -d $out/p$i -o pmc --output-format csv -- python3 $B > $out/p$i.json 2> $out/p$i.err || { echo "pmc $i failed"; exit 1; }
  echo "pmc $i done"
done
