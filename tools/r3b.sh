#!/bin/bash
# Round-3 session-2 GPU check: new tests first, then the whole GPU suite, then bench lines and a
# config-2 trace.  usage: bash tools/r3b.sh <tag> [parts...]  (parts: new suite c2 c3 c4 c5 c5c c2t)
set -o pipefail
TAG=${1:-r3b}; shift
PARTS=${@:-new suite c2 c3}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
for P in $PARTS; do
  case $P in
  new)
    timeout -k 10 400 python -u -m pytest tests/test_gpu_chains.py -x -v --timeout 300 --timeout-method thread \
      > $OUT/new.log 2>&1 || { tail -40 $OUT/new.log; exit 1; }
    tail -3 $OUT/new.log ;;
  suite)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > $OUT/suite.log 2>&1 || { tail -40 $OUT/suite.log; exit 2; }
    tail -3 $OUT/suite.log ;;
  c2|c3|c4|c5|c5c)
    W=config${P#c}
    timeout -k 10 300 python3 -u bench.py --workload $W --steps 10 --warmup 5 --e2e-steps 0 --no-cpu-baseline \
      > $OUT/$P.jsonl 2> $OUT/$P.log || { tail -20 $OUT/$P.log; exit 3; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/$P.jsonl').readlines()[-1]); print('$P', d['value'], d['ms_per_step'], d['hot_book'], d['kernel_ms'])" ;;
  c2t)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/c2trace -o run \
      -- python3 bench.py --workload config2 --steps 5 --warmup 5 --e2e-steps 0 --no-cpu-baseline > $OUT/c2_trace.log 2>&1 || exit 4 ;;
  c2ts)  # config-2 trace with the tail's events after its writes (solo kernel times)
    GOME_TAIL_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/c2strace -o run \
      -- python3 bench.py --workload config2 --steps 5 --warmup 5 --e2e-steps 0 --no-cpu-baseline --no-phase-pass > $OUT/c2s_trace.log 2>&1 || exit 4 ;;
  pipe)  # synchronous vs pipelined steps (bench.py --sync), configs from ABW, alternating
    for R in 1 2; do
      for M in sync pipe; do
        for W in ${ABW:-config2 config3}; do
          F=""; [ $M = sync ] && F="--sync"
          timeout -k 10 300 python3 -u bench.py --workload $W --steps 10 --warmup 5 --e2e-steps 0 --no-cpu-baseline \
            --no-phase-pass $F > $OUT/${M}_${W}_$R.jsonl 2> $OUT/${M}_${W}_$R.log || { tail -20 $OUT/${M}_${W}_$R.log; exit 12; }
          python3 -c "import json; d=json.loads(open('$OUT/${M}_${W}_$R.jsonl').readlines()[-1]); print('$M $W $R', d['value'], d['ms_per_step'], d['p50_batch_ms'])"
        done
      done
    done ;;
  sweep)  # config 3 batch sweep: value vs the critical-path bound (bench.py critical_path)
    for B in 1048576 2097152 4194304; do
      timeout -k 10 300 python3 -u bench.py --workload config3 --batch $B --steps 10 --warmup 4 --e2e-steps 0 \
        --no-cpu-baseline > $OUT/sweep_$B.jsonl 2> $OUT/sweep_$B.log || { tail -20 $OUT/sweep_$B.log; exit 13; }
      python3 -c "import json; d=json.loads(open('$OUT/sweep_$B.jsonl').readlines()[-1]); print('$B', d['value'], d['ms_per_step'], d['critical_path'])"
    done ;;
  c3t)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/c3trace -o run \
      -- python3 bench.py --workload config3 --steps 5 --warmup 5 --e2e-steps 0 --no-cpu-baseline > $OUT/c3_trace.log 2>&1 || exit 5 ;;
  ubd)  # deep plan ns/record on a one-symbol 4-dp book: VGPR plan vs the LDS plan variant
    for V in "" libgome_ldsdeep.so; do
      GOME_LIB=${V:+$PWD/gome_amd/$V} timeout -k 10 200 python3 -u tools/ubench_deep.py > $OUT/ubd_${V:-main}.log 2>&1 || { tail -20 $OUT/ubd_${V:-main}.log; exit 6; }
      echo "${V:-libgome.so}: $(cat $OUT/ubd_${V:-main}.log | tr '\n' ' ')"
    done ;;
  c5ab)  # config 5 / 5c bench lines, VGPR plan vs the LDS plan variant
    for V in "" libgome_ldsdeep.so; do
      for W in config5 config5c; do
        GOME_LIB=${V:+$PWD/gome_amd/$V} timeout -k 10 300 python3 -u bench.py --workload $W --steps 8 --warmup 3 \
          --e2e-steps 0 --no-cpu-baseline > $OUT/ab_${W}_${V:-main}.jsonl 2> $OUT/ab_${W}_${V:-main}.log || { tail -20 $OUT/ab_${W}_${V:-main}.log; exit 7; }
        python3 -c "import json; d=json.loads(open('$OUT/ab_${W}_${V:-main}.jsonl').readlines()[-1]); print('$W ${V:-main}', d['value'], d['ms_per_step'], d['hot_book'])"
      done
    done ;;
  abv)  # bench lines of each variant build gome_amd/libgome_*.so beside libgome.so (configs from ABW)
    for V in "" $(cd gome_amd && ls libgome_*.so 2>/dev/null); do
      for W in ${ABW:-config2 config3}; do
        GOME_LIB=${V:+$PWD/gome_amd/$V} timeout -k 10 300 python3 -u bench.py --workload $W --steps 8 --warmup 5 \
          --e2e-steps 0 --no-cpu-baseline > $OUT/abv_${W}_${V:-main}.jsonl 2> $OUT/abv_${W}_${V:-main}.log || { tail -20 $OUT/abv_${W}_${V:-main}.log; exit 8; }
        python3 -c "import json; d=json.loads(open('$OUT/abv_${W}_${V:-main}.jsonl').readlines()[-1]); print('$W ${V:-main}', d['value'], d['ms_per_step'], d['hot_book']['ns_per_order'], d['kernel_ms'])"
      done
    done ;;
  split)  # GOME_TAIL_SPLIT A/B on configs 2 and 3, alternating
    for R in 1 2; do
      for SP in 1 0; do
        for W in config2 config3; do
          GOME_TAIL_SPLIT=$SP timeout -k 10 300 python3 -u bench.py --workload $W --steps 8 --warmup 5 --e2e-steps 0 \
            --no-cpu-baseline > $OUT/sp${SP}_${W}_$R.jsonl 2> $OUT/sp${SP}_${W}_$R.log || { tail -20 $OUT/sp${SP}_${W}_$R.log; exit 9; }
          python3 -c "import json; d=json.loads(open('$OUT/sp${SP}_${W}_$R.jsonl').readlines()[-1]); print('split $SP $W $R', d['value'], d['ms_per_step'])"
        done
      done
    done ;;
  envab)  # A/B of an engine env knob: ENVAB="NAME" values 1 / 0, configs from ABW, alternating
    for R in 1 2; do
      for SP in 1 0; do
        for W in ${ABW:-config2 config3}; do
          env $ENVAB=$SP timeout -k 10 300 python3 -u bench.py --workload $W --steps 8 --warmup 5 --e2e-steps 0 \
            --no-cpu-baseline > $OUT/ab${SP}_${W}_$R.jsonl 2> $OUT/ab${SP}_${W}_$R.log || { tail -20 $OUT/ab${SP}_${W}_$R.log; exit 10; }
          python3 -c "import json; d=json.loads(open('$OUT/ab${SP}_${W}_$R.jsonl').readlines()[-1]); print('$ENVAB=$SP $W $R', d['value'], d['ms_per_step'], d['hot_book']['ns_per_order'])"
        done
      done
    done ;;
  pmc)  # FETCH_SIZE / WRITE_SIZE (KiB) and SQ occupancy counters per kernel, one pass each (workload PW)
    W=${PW:-config2}
    i=0
    for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
      i=$((i+1))
      timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --workload $W \
        --steps 3 --warmup 2 --e2e-steps 0 --no-cpu-baseline > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 11; }
    done
    python3 tools/pmc_kernels.py $OUT/pmc1/run_counter_collection.csv $OUT/pmc2/run_counter_collection.csv > $OUT/pmc_bytes.txt
    python3 tools/pmc_kernels.py $OUT/pmc3/run_counter_collection.csv > $OUT/pmc_sq.txt
    head -20 $OUT/pmc_bytes.txt ;;
  esac
done
echo done
