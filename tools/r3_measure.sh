#!/bin/bash
# Round-3 measurements on the GPU box.  usage: bash tools/r3_measure.sh <tag> [parts...]
#   sweep: config-3 batch-size sweep (2^20, 2^21, 2^22)
#   c2:    config-2 kernel trace (rocprofv3 --kernel-trace --stats)
#   c3t:   config-3 kernel trace at 2^20 and 2^22
#   c5:    config-5 60 timed steps with the per-step log (pools sized for the run)
#   c2grid: config-2 bench lines with GOME_TAIL_GRID = 1024 / 4096 (the tail's per-touch kernels)
#   c3:    config-3 default bench line
#   c5t:   config-5 60 steps under rocprofv3 --kernel-trace (what grows as the books deepen)
#   ab:    config-2 / config-3 bench lines of each gome_amd/libgome_*.so variant beside libgome.so
set -o pipefail
TAG=${1:-r3m}; shift
PARTS=${@:-sweep c2 c3t c5}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for P in $PARTS; do
  case $P in
  sweep)
    for B in 1048576 2097152 4194304; do
      timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --batch $B --no-cpu-baseline \
        > $OUT/c3_b$B.jsonl 2> $OUT/c3_b$B.log || exit 1
      tail -1 $OUT/c3_b$B.jsonl | cut -c100-260
    done ;;
  c2)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/c2trace -o run \
      -- python3 bench.py --workload config2 --steps 5 --warmup 2 --e2e-steps 0 --no-cpu-baseline > $OUT/c2_trace.log 2>&1 || exit 3 ;;
  c3t)
    for B in 1048576 4194304; do
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/c3trace_$B -o run \
        -- python3 bench.py --steps 5 --warmup 2 --batch $B --e2e-steps 0 --no-cpu-baseline > $OUT/c3_trace_$B.log 2>&1 || exit 4
    done ;;
  c5)
    timeout -k 10 500 python3 -u bench.py --workload config5 --steps 60 --warmup 2 --e2e-steps 4 --no-cpu-baseline \
      --pool-nodes 80000000 --pool-levels 160000000 --step-log $OUT/c5_steps.jsonl > $OUT/c5.jsonl 2> $OUT/c5.log || exit 2
    tail -1 $OUT/c5.jsonl | cut -c100-260 ;;
  c2grid)
    for G in 1024 4096; do
      GOME_TAIL_GRID=$G timeout -k 10 300 python3 -u bench.py --workload config2 --steps 10 --warmup 3 --e2e-steps 0 \
        --no-cpu-baseline > $OUT/c2_g$G.jsonl 2> $OUT/c2_g$G.log || exit 5
      tail -1 $OUT/c2_g$G.jsonl | cut -c100-300
    done ;;
  c5t)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/c5trace -o run \
      -- python3 bench.py --workload config5 --steps 60 --warmup 2 --e2e-steps 0 --no-cpu-baseline \
      --pool-nodes 80000000 --pool-levels 160000000 --step-log $OUT/c5t_steps.jsonl > $OUT/c5_trace.log 2>&1 || exit 7 ;;
  ab)  # A/B of the variant builds in gome_amd/libgome_*.so against libgome.so, alternating
    for R in 1 2; do
      for V in "" $(cd gome_amd && ls libgome_*.so 2>/dev/null); do
        N=${V:-libgome.so}
        for W in config2 config3; do
          GOME_LIB=${V:+$PWD/gome_amd/$V} timeout -k 10 300 python3 -u bench.py --workload $W --steps 10 --warmup 3 \
            --e2e-steps 0 --no-cpu-baseline > $OUT/ab_${W}_${N%.so}_$R.jsonl 2> $OUT/ab_${W}_${N%.so}_$R.log || exit 8
          echo "$W $N $R $(tail -1 $OUT/ab_${W}_${N%.so}_$R.jsonl | cut -c1-200)"
        done
      done
    done ;;
  abdeep)  # the same for the deep workloads
    for R in 1 2; do
      for V in "" $(cd gome_amd && ls libgome_*.so 2>/dev/null); do
        N=${V:-libgome.so}
        for W in config5 config5c; do
          GOME_LIB=${V:+$PWD/gome_amd/$V} timeout -k 10 300 python3 -u bench.py --workload $W --steps 8 --warmup 2 \
            --e2e-steps 0 --no-cpu-baseline > $OUT/ab_${W}_${N%.so}_$R.jsonl 2> $OUT/ab_${W}_${N%.so}_$R.log || exit 10
          echo "$W $N $R $(tail -1 $OUT/ab_${W}_${N%.so}_$R.jsonl | grep -o '"ms_per_step": [0-9.]*'; tail -1 $OUT/ab_${W}_${N%.so}_$R.jsonl | grep -o '"ns_per_order": [0-9.]*')"
        done
      done
    done ;;
  c5e2e)  # config 5 with a longer pipelined end-to-end leg (pools sized for 40 + 16 steps)
    timeout -k 10 500 python3 -u bench.py --workload config5 --steps 40 --warmup 2 --e2e-steps 16 --no-cpu-baseline \
      --pool-nodes 80000000 --pool-levels 160000000 > $OUT/c5e2e.jsonl 2> $OUT/c5e2e.log || exit 9
    tail -1 $OUT/c5e2e.jsonl | cut -c100-260 ;;
  c3)
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3.jsonl 2> $OUT/c3.log || exit 6
    tail -1 $OUT/c3.jsonl | cut -c100-300 ;;
  esac
done
echo done
