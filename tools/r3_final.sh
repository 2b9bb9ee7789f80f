#!/bin/bash
# Round-3 final measurements (GPU box).  usage: bash tools/r3_final.sh <tag> [parts...]
#   suite: the GPU test suite;  benches: bench lines (e2e + CPU baseline) for configs 3, 2, 4, 5, 5c;
#   prof3 / prof2: rocprofv3 trace + FETCH / WRITE passes (profiles/run_rocprof.sh) + summary
set -o pipefail
TAG=${1:-r03f}; shift
PARTS=${@:-suite benches}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for P in $PARTS; do
  case $P in
  suite)
    timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
      > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 2; }
    tail -3 $OUT/gpu_tests.txt ;;
  benches)
    for W in config3 config2 config4 config5 config5c; do
      timeout -k 10 400 python3 -u bench.py --workload $W > $OUT/${W}_bench.jsonl 2> $OUT/${W}_bench.log \
        || { tail -20 $OUT/${W}_bench.log; exit 3; }
      python3 -c "import json; d=json.loads(open('$OUT/${W}_bench.jsonl').readlines()[-1]); print('$W', d['value'], d['ms_per_step'], d['e2e']['value'], d['hot_book']['ns_per_order'], d['roofline']['kernel'][:40], d['roofline']['frac'])"
    done ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 8; }
    tail -1 $OUT/smoke.txt ;;
  prof3)
    bash profiles/run_rocprof.sh ${TAG}_config3 --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 || exit 4
    python3 profiles/summarize.py ${TAG}_config3 gpurun_out/prof_${TAG}_config3 || exit 5 ;;
  prof2)
    bash profiles/run_rocprof.sh ${TAG}_config2 --workload config2 --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 0 || exit 6
    python3 profiles/summarize.py ${TAG}_config2 gpurun_out/prof_${TAG}_config2 || exit 7 ;;
  esac
done
echo done
