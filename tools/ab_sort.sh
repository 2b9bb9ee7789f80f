#!/bin/bash
# A/B of the radix sort: the in-tree sort vs rocPRIM's (variant build libgome_rp.so), config 3.
set -o pipefail
out=gpurun_out/q12; mkdir -p $out
GOME_LIB=gome_amd/libgome_rp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_v4.py tests/test_gpu_parity.py -x -q \
  --timeout 300 --timeout-method thread -k "config3 or config5 or zipf or quirk" > $out/t.log 2>&1 || { tail -20 $out/t.log; exit 1; }
tail -2 $out/t.log
for lib in rp base; do
  if [ $lib = rp ]; then L=gome_amd/libgome_rp.so; else L=gome_amd/libgome.so; fi
  GOME_LIB=$L timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --e2e-steps 0 > $out/$lib.json 2> $out/$lib.err || exit 2
  tail -1 $out/$lib.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['ms_per_step'], d['device_ms_per_batch'], d['kernel_ms'])"
done
