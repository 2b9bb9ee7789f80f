"""Deep head books on the flow path (match_flow_deep.h): more price levels than the lane plans
hold, depths in LDS (gen_plan_asm.py W32D), the two-pass level sort and per-level
reconstruction.  Every case is bit-exact against the C oracle (events, levels, FIFOs, resting
count) and, where stated, identical to the legacy FIFO kernel."""
import numpy as np
import pytest

from gome_amd import workload as wl
from gome_amd.abi import GOME_FLAG_LEGACY_HOT, Engine
from oracle.pyoracle import Oracle

pytestmark = pytest.mark.gpu

DEEP = 3  # FlowHdr::ok of a deep book (debug_flow_books "kind")


def _engine(ns, mb, flags=0):
    return Engine(max_symbols=ns, max_batch=mb, max_nodes=1 << 21, max_levels=1 << 22, flags=flags)


def _cmp(got, exp, tag):
    assert len(got) == len(exp), f"{tag}: {len(got)} events vs oracle {len(exp)}"
    if len(got) and not np.array_equal(got, exp):
        bad = np.nonzero(got != exp)[0][0]
        raise AssertionError(f"{tag}: first mismatch at event {bad}:\n gpu={got[bad]}\n orc={exp[bad]}")


def _state_eq(eng, orc, syms):
    for s in syms:
        lv_g, lv_o = eng.levels(s), orc.levels(s)
        assert np.array_equal(lv_g, lv_o), f"levels of symbol {s}"
        for p in lv_o["price_fx"]:
            assert np.array_equal(eng.fifo(s, int(p)), orc.fifo(s, int(p))), f"fifo {s}@{p}"
    assert eng.stats()["n_resting"] == orc.resting()


def _run(batches, ns, syms=None, mb=None):
    eng = _engine(ns, mb or max(len(b) for b in batches))
    orc = Oracle(ns)
    deep = 0
    for i, b in enumerate(batches):
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"batch {i}")
        deep += int((eng.debug_flow_books()["kind"] == DEEP).sum())
    _state_eq(eng, orc, range(ns) if syms is None else syms)
    return eng, orc, deep


def test_deep_books_4dp_grid():
    """Config 5's price grid: the head books reach thousands of levels."""
    st = wl.Stream(64, seed=5, price_decimals=4)
    eng, orc, deep = _run([st.batch(100000) for _ in range(4)], 64)
    assert deep >= 4 * 6
    assert max(len(orc.levels(s)) for s in range(64)) > 1000


def test_deep_single_book_with_sweeps():
    """One deep book, 10% aggressive takers sweeping many thin levels (promotions by LDS
    scans in both directions), FIFOs at every level."""
    rng = np.random.default_rng(3)
    n = 60000
    batches = []
    oid = 1
    for _ in range(4):
        r = np.zeros(n, wl.ORDER_DTYPE)
        r["side"] = rng.integers(0, 2, n)
        r["price_fx"] = wl.doorder_prices(rng, n, 4)
        r["volume_fx"] = wl.doorder_volumes(rng, n)
        ag = rng.random(n) < 0.1
        r["price_fx"][ag] = np.where(r["side"][ag] == 0, wl.FX, wl.FX // 10000)
        r["volume_fx"][ag] = rng.integers(1, 40, int(ag.sum())) * wl.FX
        r["action"] = wl.ADD
        r["uuid_id"] = 2
        r["oid_id"] = np.arange(oid, oid + n)
        oid += n
        batches.append(r)
    eng, orc, deep = _run(batches, 1)
    assert deep == 4


def test_deep_equals_legacy():
    st = wl.Stream(4, seed=21, price_decimals=4)
    batches = [st.batch(40000) for _ in range(3)]
    a = _engine(4, 40000)
    b = _engine(4, 40000, GOME_FLAG_LEGACY_HOT)
    for bt in batches:
        a.submit(bt)
        b.submit(bt)
        _cmp(a.drain(), b.drain(), "deep vs legacy")
        assert int((a.debug_flow_books()["kind"] == DEEP).sum()) == 4
    for s in range(4):
        assert np.array_equal(a.levels(s), b.levels(s))
        for p in b.levels(s)["price_fx"]:
            assert np.array_equal(a.fifo(s, int(p)), b.fifo(s, int(p)))


@pytest.mark.parametrize("extra", [0, 1])
def test_deep_level_cap(extra):
    """DEEP_CAP - 2 = 16382 distinct prices run on the deep plan; one more declines (legacy)."""
    n = 16382 + extra
    r = np.zeros(n + 2000, wl.ORDER_DTYPE)
    r["price_fx"][:n] = (np.arange(n) + 1) * 1000
    r["side"][:n] = 0
    r["price_fx"][n:] = np.random.default_rng(1).integers(1, n, 2000) * 1000   # sells crossing
    r["side"][n:] = 1
    r["volume_fx"] = 10**6
    r["action"] = wl.ADD
    r["uuid_id"] = 1
    r["oid_id"] = np.arange(1, len(r) + 1)
    eng, orc, deep = _run([r], 1)
    assert deep == (1 if extra == 0 else 0)


def test_deep_shallow_handoff_and_noops():
    """A book deep in one batch and shallow in the next (and back); dropped duplicate ADDs and
    ignored actions inside deep segments."""
    rng = np.random.default_rng(8)
    eng = _engine(2, 30000)
    orc = Oracle(2)
    oid = 1
    kinds = []
    for dec in (4, 2, 4, 2):
        n = 20000
        r = np.zeros(n, wl.ORDER_DTYPE)
        r["symbol_id"] = rng.integers(0, 2, n)
        r["side"] = rng.integers(0, 2, n)
        r["price_fx"] = wl.doorder_prices(rng, n, dec)
        r["volume_fx"] = wl.doorder_volumes(rng, n)
        r["action"] = wl.ADD
        r["uuid_id"] = 4
        r["oid_id"] = np.arange(oid, oid + n)
        oid += n
        dup = r[rng.choice(n, 200, replace=False)].copy()
        ign = r[rng.choice(n, 100, replace=False)].copy()
        ign["action"] = 9
        mix = np.concatenate([r, dup, ign])
        mix = mix[rng.permutation(len(mix))]
        eng.submit(mix)
        _cmp(eng.drain(), orc.submit(mix), f"decimals {dec}")
        kinds.append(sorted(eng.debug_flow_books()["kind"].tolist()))
    _state_eq(eng, orc, range(2))
    assert kinds[0] == [DEEP, DEEP]


def test_deep_tail_books():
    """Config 5's shape at small scale: beyond the 8 head books, mid-size books with more levels
    than lanes take deep slots on the tail's stream (up to DEEP_SLOTS - FL_HEAD per batch)."""
    st = wl.Stream(400, zipf_s=1.0, seed=13, price_decimals=4)
    batches = [st.batch(200000) for _ in range(4)]
    eng, orc, deep = _run(batches, 400, syms=list(range(0, 400, 9)))
    assert deep > 4 * 20
