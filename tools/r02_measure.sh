#!/bin/bash
# Round-2 measurement set: bench lines (config 3 / 4 / 5), the kernel-trace stats of the config-3
# line, PMC passes of the cold kernel and the hottest book's plan.  Stops at the first failure.
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02m}; mkdir -p $out
cd $GRAFT_REPO_ROOT
for w in config3 config4 config5; do
  timeout -k 10 400 python -u bench.py --workload $w > $out/bench_$w.json 2> $out/bench_$w.err || { echo "bench $w failed"; exit 1; }
  echo "bench $w done"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/ktrace -o k3 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --e2e-steps 0 --no-cpu-baseline > $out/ktrace_bench.json 2> $out/ktrace.err || { echo "ktrace failed"; exit 1; }
echo "ktrace done"
bash $GRAFT_REPO_ROOT/tools/pmc_kmatch.sh ${1:-r02m}/pmc config3 || exit 1
echo "pmc done"
