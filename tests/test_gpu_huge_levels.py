"""The hottest book's huge levels (round 6): a level of FC_HUGE (16384) touches or more in a book with
DELs is rebuilt by chunks over many blocks (match_flow_deep.h, k_fcb_*: per-chunk sums, their
prefixes per level, the writes per chunk, then the old FIFO per level) instead of one block walking
it 4096 touches at a time.  Every event, level and FIFO against the C oracle, over two batches (the
second one's DELs reach makers of the first: old targets), for a lane book (2-dp prices, up to 126
levels) and a deep book (4-dp), and at bench size on config 5c's stream; each asserts the chunked
pass took the levels (gome_debug_peek 6: the pass's control blocks)."""
import numpy as np
import pytest

import bench
from gome_amd import workload as wl
from gome_amd.abi import Engine
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books

pytestmark = pytest.mark.gpu

FCB_CTL_BYTES = 22552  # sizeof(FcbCtl): the deep book's control block follows the lane book's


def _huge_taken(eng, deep):
    ctl = np.frombuffer(eng.debug_peek(6, deep * FCB_CTL_BYTES, 16), np.uint32)
    return int(ctl[0]), int(ctl[1])  # (levels taken, chunks)


@pytest.mark.parametrize("decimals,deep", [(2, 0), (4, 1)])
def test_huge_levels_of_one_book(decimals, deep):
    n = 300000
    rec = wl.cancel_mix(2 * n, 1, seed=7 + decimals, price_decimals=decimals)
    eng = Engine(max_symbols=1, max_batch=n, max_nodes=1 << 21, max_levels=1 << 21)
    orc = Oracle(1)
    for k in range(2):
        b = rec[k * n:(k + 1) * n].copy()
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"{decimals}dp batch {k}")
        lv, ch = _huge_taken(eng, deep)
        assert lv >= 1 and ch >= 2 * lv, (lv, ch)
        st = eng.stats()
        assert st["n_flow_cancels"] > 10000, st["n_flow_cancels"]
    _cmp_books(eng, orc, [0], f"{decimals}dp")
    assert eng.stats()["n_resting"] == orc.resting()


def test_huge_levels_config5c_bench_stream():
    """bench.py --workload config5c's stream (1M Zipf symbols, 4-dp prices, 50% DEL, 10% aggressive),
    two 4 Mi-order batches: the hottest (deep) book's 1.00 / 0.01 levels take the chunked pass."""
    n = 1 << 22
    gen, _, _ = bench.make_stream("config5c", 0, 1, 42)
    eng = Engine(max_symbols=1000000, max_batch=n, max_nodes=1 << 25, max_levels=1 << 27)  # (bench.py's sizing)
    orc = Oracle(1000000)
    for i in range(2):
        b = gen(n).copy()
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"config5c batch {i}")
        lv, _ = _huge_taken(eng, 1)
        assert lv >= 1, lv
    z = wl.ZipfSymbols(1000000, 1.0)
    syms = [int(z.rank_to_id[r]) for r in range(8)]
    _cmp_books(eng, orc, syms, "config5c")
    assert eng.stats()["n_resting"] == orc.resting()
