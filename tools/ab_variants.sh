#!/bin/bash
# A/B of variant builds (tools/build_variant.py) on one workload, alternating:
#   bash tools/ab_variants.sh TAG WORKLOAD variant1 variant2 ...   (variant "base" = libgome.so)
set -o pipefail
TAG=$1; W=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in "$@"; do
  L=gome_amd/libgome.so; [ "${v%%_*}" != base ] && L=gome_amd/libgome_${v%%_*}.so
  GOME_LIB=$L timeout -k 10 300 python3 -u bench.py --workload $W --no-cpu-baseline --e2e-steps 0 --consumer-msgs 0 > $OUT/$v.jsonl 2> $OUT/$v.log || exit 3
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d['critical_path']['frac'] if d.get('critical_path') else None, d['hot_book']['ns_per_order'])" $OUT/$v.jsonl $v
done
