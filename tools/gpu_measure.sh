#!/bin/bash
# Measurements on the GPU box.  usage: bash tools/gpu_measure.sh <tag> [parts...]
#   suite: the GPU test suite;  smoke;  benches: bench lines (e2e, consumer leg, CPU baseline) of
#   configs 3, 2, 4, 5, 5c;  heal / quirks / pg: the quirk-injection line(s) and the RCCL world-1 line;
#   tests=<files, comma-separated>: a subset of the GPU suite (e.g. tests=tests/test_a_layouts_gpu.py);
#   q4: the config-3 bench line in a process whose HIP runtime has 4 hardware queues;
#   prof3 / prof2: rocprofv3 trace + FETCH / WRITE passes (profiles/run_rocprof.sh) + summary
set -o pipefail
TAG=${1:-r04f}; shift
PARTS=${@:-suite benches}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
summ() {
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); e=d.get('e2e') or {}; c=d.get('consumer') or {}; print(sys.argv[2], round(d['value']/1e6,2), d['ms_per_step'], 'e2e', round(e.get('value',0)/1e6,2), 'hot', d['hot_book']['ns_per_order'], d['roofline']['kernel'][:30], d['roofline']['frac'], 'p99dev', d.get('p99_device_batch_ms'), 'consumer', c.get('messages_per_s'))" $1 $2
}
for P in $PARTS; do
  case $P in
  suite)
    timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
      > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 2; }
    tail -3 $OUT/gpu_tests.txt ;;
  tests=*)
    T=${P#tests=}
    timeout -k 10 900 python -u -m pytest ${T//,/ } -m gpu -v --timeout 600 --timeout-method thread \
      > $OUT/gpu_subset.txt 2>&1 || { tail -60 $OUT/gpu_subset.txt; exit 2; }
    tail -8 $OUT/gpu_subset.txt ;;
  q4)
    GOME_HW_QUEUES=4 timeout -k 10 400 python3 -u bench.py --workload config3 --no-cpu-baseline --consumer-msgs 0 \
      > $OUT/config3_q4_bench.jsonl 2> $OUT/config3_q4_bench.log || { tail -20 $OUT/config3_q4_bench.log; exit 9; }
    summ $OUT/config3_q4_bench.jsonl q4 ;;
  pcie)
    timeout -k 10 120 ./tools/pcie_duplex 256 > $OUT/pcie_duplex.json 2>&1 || { cat $OUT/pcie_duplex.json; exit 10; }
    cat $OUT/pcie_duplex.json ;;
  rcclab)
    # the RCCL layout: CU-masked plan stream (plan_cus default) vs every CU shared, alternating, and
    # the plain N=1 line (no process group) beside them
    Q="--steps 10 --warmup 4 --no-cpu-baseline --consumer-msgs 0 --e2e-steps 0 --no-phase-pass"
    for R in 1 2; do
      for V in 0 -1; do
        timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
          --master-port $((29540 + R)) bench.py --gpus 1 --force-pg --backend nccl --plan-cus $V $Q \
          > $OUT/rccl_pc${V}_$R.jsonl 2> $OUT/rccl_pc${V}_$R.log || { tail -20 $OUT/rccl_pc${V}_$R.log; exit 11; }
        summ $OUT/rccl_pc${V}_$R.jsonl rccl_pc$V
      done
      timeout -k 10 300 python3 -u bench.py $Q > $OUT/plain_$R.jsonl 2> $OUT/plain_$R.log || { tail -20 $OUT/plain_$R.log; exit 12; }
      summ $OUT/plain_$R.jsonl plain
    done ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 8; }
    tail -1 $OUT/smoke.txt ;;
  bench3|bench2|bench4|bench5|bench5c|benches)
    WS="config${P#bench}"; [ $P = benches ] && WS="config3 config2 config4 config5 config5c"
    for W in $WS; do
      timeout -k 10 500 python3 -u bench.py --workload $W > $OUT/${W}_bench.jsonl 2> $OUT/${W}_bench.log \
        || { tail -20 $OUT/${W}_bench.log; exit 3; }
      summ $OUT/${W}_bench.jsonl $W
    done ;;
  heal)
    timeout -k 10 400 python3 -u bench.py --workload config3 --inject-quirks heal --no-cpu-baseline --consumer-msgs 0 \
      --step-log $OUT/config3_heal_steps.jsonl > $OUT/config3_heal_bench.jsonl 2> $OUT/config3_heal_bench.log || { tail -20 $OUT/config3_heal_bench.log; exit 4; }
    summ $OUT/config3_heal_bench.jsonl heal ;;
  quirks)
    # quirk injection into the first timed batch (bench.py --inject-quirks): Q2 + Q6 at the bottom /
    # top of the bid book, Q2 alone, Q6 alone
    for M in stuck q2stuck zero zeroheal heal; do
      timeout -k 10 400 python3 -u bench.py --workload config3 --inject-quirks $M --no-cpu-baseline --consumer-msgs 0 \
        > $OUT/config3_${M}_bench.jsonl 2> $OUT/config3_${M}_bench.log || { tail -20 $OUT/config3_${M}_bench.log; exit 4; }
      summ $OUT/config3_${M}_bench.jsonl $M
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); print(json.dumps(d.get('quirk_batch')))" $OUT/config3_${M}_bench.jsonl
    done ;;
  e2e2|e2e3)
    # the host path of config 2 / 3 (records from page-locked host memory, events back) at host depths 2 and 3
    W=config${P#e2e}
    for DP in 2 3; do
      timeout -k 10 300 python3 -u bench.py --workload $W --steps 10 --warmup 4 --no-cpu-baseline --consumer-msgs 0 --e2e-depth $DP \
        > $OUT/${W}_e2e$DP.jsonl 2> $OUT/${W}_e2e$DP.log || { tail -20 $OUT/${W}_e2e$DP.log; exit 13; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); e=d['e2e']; print(sys.argv[2], d['ms_per_step'], e['steady_ms_per_step'], e['pcie_bound_ms'], e['host_ms_per_step'], e.get('device_ms_per_batch_median'), e['pcie_peak'])" $OUT/${W}_e2e$DP.jsonl depth$DP
    done ;;
  pg)
    timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29533 bench.py --gpus 1 --force-pg --backend nccl --no-cpu-baseline --consumer-msgs 0 \
      > $OUT/config3_rccl_bench.jsonl 2> $OUT/config3_rccl_bench.log || { tail -20 $OUT/config3_rccl_bench.log; exit 5; }
    summ $OUT/config3_rccl_bench.jsonl rccl ;;
  prof3)
    bash profiles/run_rocprof.sh ${TAG}_config3 --steps 6 --warmup 3 --no-cpu-baseline --e2e-steps 0 --consumer-msgs 0 --no-phase-pass || exit 6
    python3 profiles/summarize.py ${TAG}_config3 gpurun_out/prof_${TAG}_config3 || exit 7 ;;
  prof4|prof5|prof5c)
    W=config${P#prof}
    bash profiles/run_rocprof.sh ${TAG}_$W --workload $W --steps 6 --warmup 4 --no-cpu-baseline --e2e-steps 0 --consumer-msgs 0 --no-phase-pass || exit 6
    python3 profiles/summarize.py ${TAG}_$W gpurun_out/prof_${TAG}_$W || exit 7 ;;
  prof2)
    bash profiles/run_rocprof.sh ${TAG}_config2 --workload config2 --steps 6 --warmup 4 --no-cpu-baseline --e2e-steps 0 --consumer-msgs 0 --no-phase-pass || exit 6
    python3 profiles/summarize.py ${TAG}_config2 gpurun_out/prof_${TAG}_config2 || exit 7 ;;
  esac
done
echo done
