#!/bin/bash
# Sustained config 5: 200 timed steps on the default pools, step log with the
# chunk footprint (gome_stats.chunk_bytes) and the cold kernel's time per step.
set -o pipefail
O=gpurun_out/${1:-r4c5}
mkdir -p $O
timeout -k 10 1000 python -u bench.py --workload config5 --steps ${2:-200} --warmup 3 --pool-levels 335544320 --no-cpu-baseline --no-phase-pass \
  --e2e-steps 0 --consumer-msgs 0 --step-log $O/config5_steps.jsonl > $O/config5_long.json 2> $O/config5_long.err \
  || { tail -20 $O/config5_long.err; exit 1; }
python - $O <<'PY'
import json, sys
O = sys.argv[1]
L = [json.loads(l) for l in open(O + "/config5_steps.jsonl")]
for i in (0, 9, 59, 99, 149, len(L) - 1):
    if i < len(L):
        s = L[i]
        print(i, "resting", s["n_resting"], "levels", s["n_levels"], "B/rest", round(s["chunk_bytes"] / s["n_resting"], 1),
              "plan", round(s["ms_flow_plan"], 2), "cold", round(s["ms_cold"], 2), "total", round(s["ms_total"], 2))
d = json.loads(open(O + "/config5_long.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"])
PY
