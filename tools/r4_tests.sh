#!/bin/bash
# Round-4 GPU test pass: new tests, the full GPU suite, and the parity subset on a chunk-size variant.
set -o pipefail
O=gpurun_out/${1:-r4t}
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 500 $T -v tests/test_gpu_requal.py tests/test_dup_oid.py tests/test_gpu_r4.py > $O/new.log 2>&1 || { tail -40 $O/new.log; exit 1; }
tail -3 $O/new.log
timeout -k 10 700 $T -m gpu tests > $O/gpu.log 2>&1 || { tail -40 $O/gpu.log; exit 1; }
tail -3 $O/gpu.log
if [ -n "$2" ]; then
  GOME_LIB=gome_amd/libgome_$2.so timeout -k 10 600 $T tests/test_gpu_parity.py tests/test_gpu_flow_cancel.py \
    tests/test_gpu_flow_deep.py tests/test_gpu_requal.py "tests/test_gpu_v4.py::test_bench_config3_exact_4mi_batches" \
    "tests/test_gpu_r3.py::test_bench_config5_exact_4mi_batches" > $O/variant_$2.log 2>&1 || { tail -40 $O/variant_$2.log; exit 1; }
  tail -3 $O/variant_$2.log
fi
