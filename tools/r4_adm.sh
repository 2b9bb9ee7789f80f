#!/bin/bash
# Admission ahead (k_adm_verify): its tests and the early / pipelined suites, then A/B of the
# dominated non-early workloads (configs 4 and 5c) and config 3, alternating on / off.
set -o pipefail
O=gpurun_out/${1:-r4adm}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_adm_ahead.py tests/test_gpu_early.py -x -v --timeout 400 --timeout-method thread > $O/tests.txt 2>&1 \
  || { tail -60 $O/tests.txt; exit 2; }
tail -3 $O/tests.txt
Q="--no-cpu-baseline --consumer-msgs 0 --e2e-steps 0 --no-phase-pass --steps 12"
for W in ${2:-config4 config5c config3}; do
  for R in 1 2; do
    for A in 1 0; do
      GOME_ADM_AHEAD=$A timeout -k 10 400 python3 -u bench.py --workload $W $Q > $O/${W}_$A$R.jsonl 2> $O/${W}_$A$R.log || { tail -20 $O/${W}_$A$R.log; exit 4; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], d.get('critical_path',{}).get('frac'), d['adm_ahead'], d['adm_redo'], d['early_plans'])" $O/${W}_$A$R.jsonl "$W ahead=$A"
    done
  done
done
