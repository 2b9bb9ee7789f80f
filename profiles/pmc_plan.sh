#!/bin/bash
# SQ counters of the flow plan kernel (one rocprofv3 --pmc pass per counter group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_INSTS_WAVE32"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -T --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || echo "pass $i failed" >> $OUT/status.txt
done
echo done >> $OUT/status.txt
