#!/bin/bash
# One GPU session: parity tests, then bench lines.  Stops at the first fault / timeout.
# usage: tools/gpu_run.sh <tag> [pytest -k expr] [bench workloads...]
tag=$1; kexpr=${2:-}; shift 2 || true
out=gpurun_out/$tag; mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ "$kexpr" != "none" ]; then
  if [ -n "$kexpr" ]; then K=(-k "$kexpr"); else K=(); fi
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $out/tests.log 2>&1
  rc=$?; tail -5 $out/tests.log; ok $rc || { echo "tests rc=$rc: stopping"; exit $rc; }
fi
for w in "$@"; do
  IFS=: read name steps <<< "$w"
  timeout -k 10 600 python -u bench.py --workload $name --steps ${steps:-10} --warmup 3 > $out/bench_$name.json 2> $out/bench_$name.err
  rc=$?; echo "bench $name rc=$rc"; tail -c 3000 $out/bench_$name.json; [ $rc -eq 0 ] || { tail -20 $out/bench_$name.err; exit $rc; }
done
