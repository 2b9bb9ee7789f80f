#!/bin/bash
# A/B of variant builds on the host path (e2e leg) of one workload:
#   bash tools/ab_e2e.sh TAG WORKLOAD variant1 variant2 ...   (variant "base" = libgome.so)
set -o pipefail
TAG=$1; W=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in "$@"; do
  L=gome_amd/libgome.so; [ "${v%%_*}" != base ] && L=gome_amd/libgome_${v%%_*}.so
  GOME_LIB=$L timeout -k 10 300 python3 -u bench.py --workload $W --steps 10 --warmup 4 --no-cpu-baseline --consumer-msgs 0 > $OUT/$v.jsonl 2> $OUT/$v.log || exit 3
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); e=d['e2e']; print(sys.argv[2], round(d['value']/1e6,2), round(e['value']/1e6,2), e['steady_ms_per_step'], e['collect_gaps_ms'])" $OUT/$v.jsonl $v
done
