#!/bin/bash
# SQ counters of the plan loop on the crafted single-book workloads of tools/plan_paths.py
# (diagnostic build libgome_stamps.so); one rocprofv3 --pmc pass per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_paths}
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_IFETCH SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/plan_paths.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed" >> $OUT/status.txt; exit 1; }
done
echo done >> $OUT/status.txt
