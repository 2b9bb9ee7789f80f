#!/bin/bash
# A/B of library variants on several workloads (alternating, one box).  usage: r4_ab.sh OUT "wl..." variant...
set -o pipefail
O=gpurun_out/${1:-r4ab}; W=${2:-"config2 config4 config5c"}; shift 2
mkdir -p $O
Q="--no-cpu-baseline --no-phase-pass --e2e-steps 0 --consumer-msgs 0 --steps 10 --warmup 3"
for w in $W; do
  for rep in 1 2; do
    for v in base "$@"; do
      e=""; [ "$v" != base ] && e="GOME_LIB=gome_amd/libgome_$v.so"
      env $e timeout -k 10 300 python -u bench.py --workload $w $Q --step-log $O/${w}_${v}_$rep.steps.jsonl > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=[json.loads(l) for l in open(sys.argv[2])][-1]; print(sys.argv[1], round(d['value']/1e6,2), d['ms_per_step'], d['hot_book']['ns_per_order'], 'B/rest', round(s['chunk_bytes']/max(1,s['n_resting']),1))" $O/${w}_${v}_$rep.json $O/${w}_${v}_$rep.steps.jsonl
    done
  done
done
