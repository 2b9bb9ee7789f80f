#!/bin/bash
# Round-4 bench pass: A/B lines of a chunk-size variant, the quirk-injection stream, config 5's
# chunk footprint.  Usage: tools/r4_bench.sh OUTDIR [variant ...]
set -o pipefail
O=gpurun_out/${1:-r4b}
shift
mkdir -p $O
Q="--no-cpu-baseline --no-phase-pass --e2e-steps 0 --consumer-msgs 0"
run() {  # name, env, args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python - "$O/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
hb = d.get("hot_book", {}); cp = d.get("critical_path", {})
print(sys.argv[1], d["config"]["name"], round(d["value"] / 1e6, 2), "M/s", d["ms_per_step"], "ms",
      "hot", hb.get("ns_per_order"), hb.get("path"), "frac", cp.get("frac"))
PY
}
for v in "" "$@"; do
  e=""; t=base
  if [ -n "$v" ]; then e="GOME_LIB=gome_amd/libgome_$v.so"; t=$v; fi
  run c3_$t "$e" --workload config3 --steps 10 --warmup 3 $Q
  run c5_$t "$e" --workload config5 --steps 10 --warmup 3 $Q --step-log $O/c5_$t.steps.jsonl
done
run c3_heal "" --workload config3 --steps 10 --warmup 3 --inject-quirks heal $Q --step-log $O/c3_heal.steps.jsonl
run c3_stuck "" --workload config3 --steps 4 --warmup 3 --inject-quirks stuck $Q
