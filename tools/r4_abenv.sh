#!/bin/bash
# A/B of environment variants (alternating, one box).  usage: r4_abenv.sh OUT "workloads" STEPS "name:ENV=V ..." ...
set -o pipefail
O=gpurun_out/${1:-r4abe}; W=${2:-"config3"}; S=${3:-10}; shift 3
mkdir -p $O
Q="--no-cpu-baseline --no-phase-pass --consumer-msgs 0 --warmup 3 --pool-levels 335544320"
for w in $W; do
  for rep in 1 2; do
    for v in "$@"; do
      n=${v%%:*}; e=${v#*:}
      env $e timeout -k 10 600 python -u bench.py --workload $w $Q --steps $S --e2e-steps ${E2E:-0} --step-log $O/${w}_${n}_$rep.steps.jsonl > $O/${w}_${n}_$rep.json 2> $O/${w}_${n}_$rep.err || { tail -20 $O/${w}_${n}_$rep.err; exit 1; }
      python3 - $O/${w}_${n}_$rep.json $O/${w}_${n}_$rep.steps.jsonl <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
L = [json.loads(l) for l in open(sys.argv[2])]
e = d.get("e2e") or {}
print(sys.argv[1], round(d["value"] / 1e6, 2), d["ms_per_step"], "hot", d["hot_book"]["ns_per_order"],
      "last tot", round(L[-1]["ms_total"], 2), "cold", round(L[-1]["ms_cold"], 2),
      "e2e", round(e.get("value", 0) / 1e6, 2), e.get("ms_per_step"))
PY
    done
  done
done
