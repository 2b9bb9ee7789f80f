#!/bin/bash
# Cold-kernel variants on the sustained config 5 (steps) and on configs 3 / 2.
set -o pipefail
O=gpurun_out/${1:-r4cold}; S=${2:-120}; shift 2
mkdir -p $O
for v in base "$@"; do
  e=""; [ "$v" != base ] && e="GOME_LIB=gome_amd/libgome_$v.so"
  env $e timeout -k 10 600 python -u bench.py --workload config5 --steps $S --warmup 3 --pool-levels 335544320 \
    --no-cpu-baseline --no-phase-pass --e2e-steps 0 --consumer-msgs 0 --step-log $O/c5_$v.steps.jsonl > $O/c5_$v.json 2> $O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 1; }
  python3 - $O/c5_$v.steps.jsonl $O/c5_$v.json <<'PY'
import json, sys
L = [json.loads(l) for l in open(sys.argv[1])]
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
f = lambda s: f"tot {s['ms_total']:.1f} cold {s['ms_cold']:.1f} plan {s['ms_flow_plan']:.1f}"
print(sys.argv[2], "value", round(d["value"] / 1e6, 2), "first", f(L[0]), "last", f(L[-1]))
PY
  for w in config3 config2; do
    env $e timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-phase-pass \
      --e2e-steps 0 --consumer-msgs 0 > $O/${w}_$v.json 2> $O/${w}_$v.err || { tail -5 $O/${w}_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d['kernel_ms'].get('k_match'))" $O/${w}_$v.json
  done
done
