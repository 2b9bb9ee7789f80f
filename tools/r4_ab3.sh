#!/bin/bash
# three alternating reps of config 5c: base vs ls0
set -o pipefail
O=gpurun_out/r4ls3; mkdir -p $O
Q="--no-cpu-baseline --no-phase-pass --e2e-steps 0 --consumer-msgs 0 --steps 10 --warmup 3"
for rep in 1 2 3; do
  for v in base ls0; do
    e=""; [ "$v" != base ] && e="GOME_LIB=gome_amd/libgome_$v.so"
    env $e timeout -k 10 300 python -u bench.py --workload config5c $Q > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -20 $O/${v}_$rep.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d['hot_book']['ns_per_order'], d['critical_path']['frac'])" $O/${v}_$rep.json
  done
done
