"""Plan-loop cost per record kind on the flow path (ms_flow_plan of a one-symbol batch):
ADD-only (W32 plan), ADD-only with one no-op DEL (W32C plan), half no-op DELs, half real DELs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gome_amd import workload as wl  # noqa: E402
from gome_amd.abi import Engine  # noqa: E402

N = 1 << 18


def adds(rng, n, oid0):
    r = np.zeros(n, wl.ORDER_DTYPE)
    r["price_fx"] = wl.doorder_prices(rng, n)
    r["volume_fx"] = wl.doorder_volumes(rng, n)
    r["side"] = rng.integers(0, 2, n)
    r["action"] = wl.ADD
    r["uuid_id"] = 2
    r["oid_id"] = np.arange(oid0, oid0 + n)
    return r


def run(tag, mk):
    eng = Engine(max_symbols=1, max_batch=N, max_nodes=1 << 22, max_levels=1 << 20)
    rng = np.random.default_rng(5)
    t = []
    for i in range(6):
        b = mk(rng, i)
        eng.submit(b)
        eng.drain()
        st = eng.stats()
        if i >= 2:
            t.append(st["ms_flow_plan"] * 1e6 / len(b))
    fb = eng.debug_flow_books(1)
    print(f"{tag:34s} ns/record {np.mean(t):7.1f}  kind {int(fb['kind'][0])} decline {int(fb['decline'][0])} "
          f"flow_cancels {st['n_flow_cancels']}")


def add_only(rng, i):
    return adds(rng, N, 1 + i * N)


def one_noop(rng, i):
    b = adds(rng, N, 1 + i * N)
    b[N // 2]["action"] = wl.DEL
    b[N // 2]["oid_id"] = 4_000_000_000
    return b


def half_noop(rng, i):
    b = adds(rng, N, 1 + i * N)
    d = rng.random(N) < 0.5
    b["action"][d] = wl.DEL
    b["oid_id"][d] = 4_000_000_000 - np.arange(int(d.sum()))
    return b


def half_real(rng, i):
    b = adds(rng, N, 1 + i * N)
    # each DEL re-sends an earlier ADD of the batch (uniformly), as the config-4 generator does
    idx = np.arange(N)
    d = rng.random(N) < 0.5
    d[:64] = False
    for j in np.nonzero(d)[0]:
        k = int(rng.integers(0, j))
        while d[k]:
            k = int(rng.integers(0, j))
        b[j] = b[k]
        b[j]["action"] = wl.DEL
    return b


_ns = {}


def native(rng, i):
    if "s" not in _ns:
        _ns["s"] = wl.NativeStream(1, None, seed=3, price_decimals=2, del_frac=0.5, aggressive_frac=0.1)
    return _ns["s"].batch(N)


def _sweeps(rng, i):
    b = adds(rng, N, 1 + i * N)
    ag = rng.random(N) < 0.1
    b["price_fx"][ag] = np.where(b["side"][ag] == 0, wl.FX, wl.FX // 100)
    b["volume_fx"][ag] = rng.integers(1, 17, int(ag.sum())) * 10 * wl.FX
    return b


def recent_dels(aggr):
    """50% DELs, each of a uniformly chosen ADD among the last 256 untargeted ones (windows stay
    short); `aggr` of the ADDs sweep (BUY @ 1.00 / SALE @ 0.01, 10..160 units)."""
    def mk(rng, i):
        b = adds(rng, N, 1 + i * N)
        ag = rng.random(N) < aggr
        b["price_fx"][ag] = np.where(b["side"][ag] == 0, wl.FX, wl.FX // 100)
        b["volume_fx"][ag] = rng.integers(1, 17, int(ag.sum())) * 10 * wl.FX
        d = rng.random(N) < 0.5
        pool = []
        for j in range(N):
            if d[j] and pool:
                k = pool.pop(int(rng.integers(len(pool))))
                b[j] = b[k]
                b[j]["action"] = wl.DEL
            else:
                d[j] = False
                pool.append(j)
                if len(pool) > 256:
                    pool.pop(0)
        return b
    return mk


run("ADD only (W32)", add_only)
run("ADD + one no-op DEL (W32C)", one_noop)
run("50% no-op DELs (W32C)", half_noop)
run("50% DELs of recent ADDs (W32C)", recent_dels(0.0))
run("50% DELs of recent ADDs, 10% sweeps", recent_dels(0.1))
run("ADD only, 10% sweeps (W32)", lambda rng, i: recent_dels(0.1)(rng, i)[:0] if False else _sweeps(rng, i))
