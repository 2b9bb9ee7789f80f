#!/bin/bash
# e2e A/B: events D2H on the copy stream (default) vs a stream of its own, with 4 / 8 HW queues.
set -o pipefail
O=gpurun_out/${1:-r4e}
mkdir -p $O
Q="--no-cpu-baseline --no-phase-pass --consumer-msgs 0 --steps 8 --warmup 3 --e2e-steps 8"
for w in config2 config3; do
  for v in "base:" "d2h:GOME_D2H_STREAM=1" "d2h_q8:GOME_D2H_STREAM=1 GPU_MAX_HW_QUEUES=8"; do
    n=${v%%:*}; e=${v#*:}
    env $e timeout -k 10 300 python -u bench.py --workload $w $Q > $O/${w}_$n.json 2> $O/${w}_$n.err || { tail -20 $O/${w}_$n.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['e2e']; print(sys.argv[1], round(d['value']/1e6,1), d['ms_per_step'], 'e2e', round(e['value']/1e6,1), e['ms_per_step'], e['pcie_bound_ms'], e['pcie_peak'])" $O/${w}_$n.json
  done
done
