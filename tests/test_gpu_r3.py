"""HIP engine (MI355X) — round-3 boundary coverage: deferred failures of in-flight batches, the
load-into-a-fresh-engine rule after refused submits, drain collecting in-flight batches."""
import numpy as np
import pytest

from gome_amd import workload as wl
from gome_amd.abi import GOME_E_CAPACITY, GOME_E_INVAL, GOME_OK, Engine, GomeError
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books

pytestmark = pytest.mark.gpu


def _host(eng, b):
    buf = eng.host_buffer(len(b))
    buf[:] = b
    return buf


def test_rejected_async_batch_is_deferred_not_blamed_on_the_next_call():
    """an in-flight batch rejected with E_INVAL (unknown flag bits) that a synchronous
    submit collects does not fail that submit; the submit runs, and gome_take_deferred reports
    the rejected batch once."""
    st = wl.Stream(8, seed=2)
    eng = Engine(max_symbols=8, max_batch=4096)
    orc = Oracle(8)
    good, bad, nxt = st.batch(3000), st.batch(100), st.batch(3000)
    bad[5]["flags"] = 8
    eng.submit_async(_host(eng, good))
    bufb = _host(eng, bad)
    eng.submit_async(bufb)
    eng.submit(nxt)  # collects both: the first's events queue, the second was rejected
    _cmp(eng.drain(), np.concatenate([orc.submit(good), orc.submit(nxt)]), "good + next")
    s, msg = eng.take_deferred()
    assert s == GOME_E_INVAL and "seq_base" in msg
    assert eng.take_deferred() == (GOME_OK, "")
    _cmp_books(eng, orc, range(8), "after deferred")


def test_drain_collects_inflight_batches():
    st = wl.Stream(8, seed=3)
    eng = Engine(max_symbols=8, max_batch=4096)
    orc = Oracle(8)
    b1, b2 = st.batch(2000), st.batch(2000)
    eng.submit_async(_host(eng, b1))
    eng.submit_async(_host(eng, b2))
    _cmp(eng.drain(), np.concatenate([orc.submit(b1), orc.submit(b2)]), "drain after async")
    assert eng.inflight() == 0


def test_load_books_after_refused_submits():
    """refused submits (empty, too large, over capacity) do not count as use: a fresh
    engine still accepts gome_load_books afterwards."""
    eng = Engine(max_symbols=4, max_batch=1024, max_nodes=64, max_levels=1 << 12)
    eng.submit(np.zeros(0, wl.ORDER_DTYPE))
    with pytest.raises(GomeError):
        eng.submit(np.zeros(2048, wl.ORDER_DTYPE))  # > max_batch
    big = wl.Stream(4, seed=1).batch(1000)
    with pytest.raises(GomeError) as ei:
        eng.submit(big)  # headroom: 1000 ADDs > max_nodes
    assert ei.value.status == GOME_E_CAPACITY
    lv = np.zeros(1, wl.LEVEL_DTYPE)
    lv[0] = (50 * 10**6, 3 * 10**6, 1, 1, 0, 0)
    nd = np.zeros(1, wl.NODE_DTYPE)
    nd[0]["volume_fx"], nd[0]["oid_id"], nd[0]["uuid_id"], nd[0]["side"] = 3 * 10**6, 9, 1, 0
    eng.load_books([(2, lv, nd)])
    assert eng.stats()["n_resting"] == 1
    assert np.array_equal(eng.levels(2), lv)


def test_bench_config5_exact_4mi_batches():
    """bench.py --workload config5 exactly (make_stream("config5", 0, 1, 42): 1M Zipf symbols,
    4-dp price grid), three 4 Mi-order batches as the bench runs them:
    every event vs the C oracle, levels and FIFOs of the 8 head books and 100 random books.  At
    4 Mi the tail's deep books (candidates beyond the head, ~2k of them) take the deep plan."""
    import bench
    n = 1 << 22
    gen, _, _ = bench.make_stream("config5", 0, 1, 42)
    eng = Engine(max_symbols=1_000_000, max_batch=n, max_nodes=3 * n + (1 << 20), max_levels=(128 << 20) + 2 * n)
    orc = Oracle(1_000_000)
    deep_tail = 0
    for i in range(3):
        b = gen(n).copy()
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"config5 batch {i}")
        fl = eng.debug_flow_books()
        deep_tail += int(((fl["deep"] != 0) & (np.arange(len(fl)) >= 8)).sum())
        assert eng.stats()["n_flow_books"] > 1000
    assert deep_tail > 1000
    g = wl.NativeStream(1_000_000, 1.0, seed=42, price_decimals=4)
    syms = [int(g.zipf.rank_to_id[r]) for r in range(8)]
    syms += np.random.default_rng(3).choice(1_000_000, 100, replace=False).tolist()
    _cmp_books(eng, orc, syms, "config5")
    assert max(len(orc.levels(s)) for s in syms[:8]) > 2000
    assert eng.stats()["n_resting"] == orc.resting()


@pytest.mark.gpu
def test_bench_config5c_exact():
    """bench.py --workload config5c exactly (config 5's 4-dp grid with config 4's 50% DELs and
    10% aggressive ADDs), three 4 Mi-order batches as the bench runs them: the
    hot books' segments hold ~10k distinct prices and DELs, so they take the deep plan with DELs
    (W32DC, FlowHdr::dc); every event and the books' levels and FIFOs against the C oracle."""
    import bench
    n = 1 << 22
    gen, _, _ = bench.make_stream("config5c", 0, 1, 42)
    eng = Engine(max_symbols=1_000_000, max_batch=n, max_nodes=3 * n + (1 << 20), max_levels=(64 << 20) + 2 * n)
    orc = Oracle(1_000_000)
    for i in range(3):
        b = gen(n).copy()
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"config5c batch {i}")
        st = eng.stats()
        assert st["n_del"] > n // 4 and st["n_flow_cancels"] > n // 20
        fl = eng.debug_flow_books()
        assert (fl["kind"][:8] == 3).all() and (fl["decline"] == 0).all()  # the head: deep books with DELs
    g = wl.NativeStream(1_000_000, 1.0, seed=42, price_decimals=4)
    syms = [int(g.zipf.rank_to_id[r]) for r in range(8)]
    syms += np.random.default_rng(5).choice(1_000_000, 100, replace=False).tolist()
    _cmp_books(eng, orc, syms, "config5c")
    assert eng.stats()["n_resting"] == orc.resting()
