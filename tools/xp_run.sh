#!/bin/bash
# Variant comparison: bench lines per (library, workload).  usage: tools/xp_run.sh tag "lib1 lib2" "w1 w2"
set -o pipefail
cd $GRAFT_REPO_ROOT; out=gpurun_out/$1; mkdir -p $out
for L in $2; do
  for w in $3; do
    GOME_LIB=gome_amd/$L timeout -k 10 300 python -u bench.py --workload $w --steps 6 --warmup 2 --e2e-steps 0 --no-cpu-baseline > $out/b_${L}_$w.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$out/b_${L}_$w.json'));print('$L $w', d['value'],d['kernel_ms'],d['hot_book']['ns_per_order'])"
  done
done
