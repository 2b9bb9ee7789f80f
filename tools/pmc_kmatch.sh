#!/bin/bash
# PMC passes (one per run) on the cold kernel k_match and the hottest book's plan, config-3 bench.
# usage: tools/pmc_kmatch.sh <tag> [workload]
out=$GRAFT_REPO_ROOT/gpurun_out/$1; w=${2:-config3}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --workload $w --steps 2 --warmup 1 --e2e-steps 0 --no-cpu-baseline"
i=0
for pmc in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-include-regex "k_match$|k_match\(|k_flow_plan_head" -d $out/p$i -o pmc --output-format csv -- python3 $B > $out/p$i.json 2> $out/p$i.err || exit $?
  echo "pass $i done"
done
