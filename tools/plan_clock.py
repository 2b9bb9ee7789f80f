"""Plan-loop clock check (diagnostic build, libgome_stamps.so built beforehand with
`python -c 'from gome_amd.build import build_stamps; build_stamps()'`): runs the bench
workload (config 3, one GPU) for a few batches and prints, per head book of the last batch,
the plan loop's shader cycles, wall time (s_memrealtime, 100 MHz), the clock they imply and
cycles per order."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

torch.zeros(1, device="cuda")  # the HIP runtime is initialised by torch first, as in bench.py
from gome_amd import abi  # noqa: E402

lib = abi.load_library(os.path.join(ROOT, "gome_amd", os.environ.get("GOME_STAMPS_LIB", "libgome_stamps.so")))
lib.gome_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
import bench  # noqa: E402

gen, share, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
n = 1 << 22
eng = abi.Engine(max_symbols=100000, max_batch=n, max_nodes=max(1 << 20, int(3 * n * 0.3)),
                 max_levels=max(1 << 22, 256 * 100000))
for i in range(3):
    b = torch.from_numpy(gen(n).view(np.uint8)).cuda()
    eng.submit_device(b.data_ptr(), n, seq_base=i * n)
    torch.cuda.synchronize()
NST = 256 * 16
out = (C.c_ulonglong * (NST + 32))()
assert lib.gome_debug_stamps(out, NST + 32) == 0
for h in range(8):
    cyc, rt, no, nt = out[NST + 4 * h: NST + 4 * h + 4]
    if no == 0:
        continue
    print(f"head book {h}: orders {no} touches {nt} cycles {cyc} wall {rt / 1e5:.3f} ms "
          f"clock {cyc / (rt * 10) :.3f} GHz  cycles/order {cyc / no:.1f}  ns/order {rt * 10 / no:.1f}")
