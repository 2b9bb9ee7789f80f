"""Per-path plan-loop costs (diagnostic build libgome_stamps.so, see tools/plan_clock.py):
crafted single-book batches that exercise one outcome of the plan loop each, timed by the
loop's own s_memtime / s_memrealtime stamps.  Prints cycles per order per workload."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

torch.zeros(1, device="cuda")
from gome_amd import abi  # noqa: E402
from gome_amd import workload as wl  # noqa: E402

lib = abi.load_library(os.path.join(ROOT, "gome_amd", os.environ.get("GOME_STAMPS_LIB", "libgome_stamps.so")))
lib.gome_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
NST = 256 * 16
N = 200000
rng = np.random.default_rng(5)


def batch(prices, vols, sides, oid0):
    n = len(prices)
    r = np.zeros(n, wl.ORDER_DTYPE)
    r["price_fx"] = np.asarray(prices, np.int64) * (wl.FX // 100)
    r["volume_fx"] = np.asarray(vols, np.int64) * (wl.FX // 100)
    r["side"] = sides
    r["action"] = wl.ADD
    r["uuid_id"] = 2
    r["oid_id"] = np.arange(oid0, oid0 + n, dtype=np.uint32)
    return r


def run(name, seed_rec, rec):
    eng = abi.Engine(max_symbols=4, max_batch=N + 16, max_nodes=1 << 22, max_levels=1 << 12)
    eng.submit(seed_rec, 0)
    eng.submit(rec, 1000)
    torch.cuda.synchronize()
    out = (C.c_ulonglong * (NST + 32))()
    assert lib.gome_debug_stamps(out, NST + 32) == 0
    cyc, rt, no, nt = out[NST:NST + 4]
    st = eng.stats()
    print(f"{name:34s} orders {no:7d} touches/order {nt / max(no, 1):.2f} cycles/order {cyc / max(no, 1):6.1f} "
          f"clock {cyc / max(rt * 10, 1):.2f} GHz flow_books {st['n_flow_books']}")
    eng.close()


half = rng.integers(0, 2, N).astype(np.uint8)
seed = batch([40] * 200 + [60] * 200, [100] * 400, np.array([0] * 200 + [1] * 200, np.uint8), 1)
# deep rests only: BUY below 40, SALE above 60
p = np.where(half == 0, rng.integers(1, 40, N), rng.integers(61, 101, N))
run("deep rests (random side)", seed, batch(p, rng.integers(1, 101, N), half, 10000))
p = np.where(half == 0, 30, 70)
run("deep rests, one level per side", seed, batch(p, rng.integers(1, 101, N), half, 10000))
# partial fills only: tops with huge depth, small takers crossing the top
seed2 = batch([40] * 200 + [60] * 200, [100000] * 400, np.array([0] * 200 + [1] * 200, np.uint8), 1)
p = np.where(half == 0, 60, 40)
run("partial fills at the top", seed2, batch(p, np.ones(N, np.int64), half, 10000))
# at-top rests
p = np.where(half == 0, 40, 60)
run("rests at the top", seed, batch(p, rng.integers(1, 101, N), half, 10000))
# BUY only deep rests (no side alternation)
p = rng.integers(1, 40, N)
run("deep rests, BUY only", seed, batch(p, rng.integers(1, 101, N), np.zeros(N, np.uint8), 10000))
# doorder distribution on one book
k = np.rint(rng.random(N) * 100).astype(np.int64)
k[k == 0] = 10
v = np.rint(rng.random(N) * 100).astype(np.int64)
v[v == 0] = 100
run("doorder distribution", seed, batch(k, v, half, 10000))
