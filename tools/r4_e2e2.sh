#!/bin/bash
# e2e A/B: host batches in flight (2 / 3) x events D2H on the copy stream / a stream of its own.
set -o pipefail
O=gpurun_out/${1:-r4e3}
mkdir -p $O
Q="--no-cpu-baseline --no-phase-pass --consumer-msgs 0 --steps 4 --warmup 3 --e2e-steps 10"
for w in ${2:-config2 config3}; do
  for rep in 1 2; do
    for v in ${VARIANTS:-"d2:2:" "d3:3:" "d2s:2:GOME_D2H_STREAM=1" "d3s:3:GOME_D2H_STREAM=1"}; do
      n=${v%%:*}; r=${v#*:}; dep=${r%%:*}; e=${r#*:}; e=${e//,/ }
      env $e timeout -k 10 300 python -u bench.py --workload $w $Q --e2e-depth $dep > $O/${w}_${n}_$rep.json 2> $O/${w}_${n}_$rep.err || { tail -20 $O/${w}_${n}_$rep.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['e2e']; print(sys.argv[1], round(e['value']/1e6,1), e['ms_per_step'], e['p50_batch_ms'], e['host_ms_per_step'])" $O/${w}_${n}_$rep.json
    done
  done
done
