#!/bin/bash
# Config-3 batch sweep (critical-path fraction per batch size), then quick lines of configs 2/4/5.
set -o pipefail
O=gpurun_out/${1:-r4s}
mkdir -p $O
Q="--no-cpu-baseline --consumer-msgs 0 --e2e-steps 0 --no-phase-pass"
for B in 1048576 2097152 4194304; do
  timeout -k 10 400 python3 -u bench.py --batch $B --steps 12 $Q > $O/sweep_$B.jsonl 2> $O/sweep_$B.log || { tail -20 $O/sweep_$B.log; exit 3; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d['critical_path'], d['early_plans'], d['early_miss'])" $O/sweep_$B.jsonl $B
done
for W in ${2:-config2 config4 config5}; do
  timeout -k 10 400 python3 -u bench.py --workload $W $Q > $O/${W}.jsonl 2> $O/${W}.log || { tail -20 $O/${W}.log; exit 4; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d['early_plans'], d['early_miss'])" $O/${W}.jsonl $W
done
