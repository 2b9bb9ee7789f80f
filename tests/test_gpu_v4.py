"""HIP engine (MI355X) — round-2 coverage: parity at the exact bench configurations, the ABI v4
boundary (sequence numbers, record flags, Transaction codes, the pipelined host path, device
events never dropped), cancel-index rebuilds, level-block reuse, and the multi-GPU sharding
with real engine handles.  Every comparison is bit-exact against the C oracle
(oracle/gome_oracle.c) or the literal transliteration (oracle/literal.py)."""
import numpy as np
import pytest

import bench
from gome_amd import workload as wl
from gome_amd.abi import (Engine, GomeError, GOME_FLAG_NO_HEADROOM, GOME_E_INVAL, GOME_E_NOTFOUND, GOME_E_STATE,
                          GOME_ORD_ADM_HOST, GOME_ORD_ADMITTED)
from oracle.pyoracle import Oracle

pytestmark = pytest.mark.gpu


def _cmp(got, exp, tag=""):
    assert len(got) == len(exp), f"{tag}: {len(got)} events vs oracle {len(exp)}"
    if len(got) and not np.array_equal(got, exp):
        bad = np.nonzero(got != exp)[0][0]
        raise AssertionError(f"{tag}: first mismatch at event {bad}:\n gpu={got[bad]}\n orc={exp[bad]}")


def _cmp_books(eng, orc, syms, tag=""):
    for s in syms:
        s = int(s)
        lv_g, lv_o = eng.levels(s), orc.levels(s)
        assert np.array_equal(lv_g, lv_o), f"{tag}: levels of symbol {s}"
        for p in lv_o["price_fx"]:
            assert np.array_equal(eng.fifo(s, int(p)), orc.fifo(s, int(p))), f"{tag}: fifo {s}@{p}"


def _hot_and_random(zipf, n_symbols, k_hot=8, k_rand=100, seed=0):
    hot = [int(zipf.rank_to_id[r]) for r in range(k_hot)]
    rnd = np.random.default_rng(seed).choice(n_symbols, k_rand, replace=False).tolist()
    return hot + [int(x) for x in rnd]


# ---- parity at the bench's own configurations --------------------------------------------
def test_bench_config3_exact_4mi_batches():
    """bench.py's default workload exactly: shard_stream(100000, 1.0, 0, 1, 42), three
    consecutive 4 Mi-order batches, every event vs the oracle; levels and FIFOs of the 8 head
    books and 100 random books.  (Flow-path capacities at full scale: MAX_FLOW candidates,
    FL_HEAD, the touch-log bound, ord8 padding, event-arena regrowth.)"""
    n = 1 << 22
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
    eng = Engine(max_symbols=100000, max_batch=n, max_nodes=int(3 * n * 0.3) + n + (1 << 20),
                 max_levels=1 << 23)
    orc = Oracle(100000)
    for i in range(3):
        b = gen(n)
        eng.submit(b, seq_base=0)
        _cmp(eng.drain(), orc.submit(b), f"config3 batch {i}")
        st = eng.stats()
        assert st["n_flow_books"] > 1000 and st["max_segment"] > 300000
    _cmp_books(eng, orc, _hot_and_random(wl.ZipfSymbols(100000, 1.0), 100000), "config3")
    assert eng.stats()["n_resting"] == orc.resting()


def test_bench_config2_full_batches():
    """bench.py --workload config2 exactly (1k symbols, uniform, 4 Mi-order batches): ~1000 flow
    books of ~4k orders each, nearly all in the tail (per-book claims, per-wave book lookups,
    block-tile arena claims), two batches vs the oracle, levels and FIFOs of 108 books."""
    n = 1 << 22
    gen, _, _ = bench.make_stream("config2", 0, 1, 42)
    eng = Engine(max_symbols=1000, max_batch=n, max_nodes=3 * n, max_levels=1 << 23)
    orc = Oracle(1000)
    for i in range(2):
        b = gen(n).copy()
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"config2 batch {i}")
        st = eng.stats()
        assert st["n_flow_books"] >= 990
    syms = list(range(8)) + np.random.default_rng(1).choice(1000, 100, replace=False).tolist()
    _cmp_books(eng, orc, [int(s) for s in syms], "config2")
    assert eng.stats()["n_resting"] == orc.resting()


def test_bench_config4_native_stream():
    """bench.py --workload config4 exactly (make_stream("config4", 0, 1, 42): 100k Zipf symbols,
    50% DEL, 10% aggressive), two 4 Mi-order batches: every event vs the oracle, the hottest
    book's cancels on the flow path (the Q plan), levels and FIFOs of the 8 head books and 100
    random books."""
    n = 1 << 22
    gen, _, _ = bench.make_stream("config4", 0, 1, 42)
    eng = Engine(max_symbols=100000, max_batch=n, max_nodes=1 << 23, max_levels=1 << 23)
    orc = Oracle(100000)
    for i in range(2):
        b = gen(n).copy()
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"config4 batch {i}")
        st = eng.stats()
        assert st["n_cancels"] > 500000 and st["n_flow_cancels"] > 100000
    g = wl.NativeStream(100000, 1.0, seed=42)
    _cmp_books(eng, orc, _hot_and_random(g.zipf, 100000), "config4")
    assert eng.stats()["n_resting"] == orc.resting()


def test_bench_config5_one_million_symbols():
    """Config 5 at its real symbol count: max_symbols = 2^20 (a 2-pass radix sort of 10-bit
    digits), 4-dp prices (the hottest books reach thousands of levels), 1 Mi batches."""
    n = 1 << 20
    g = wl.NativeStream(1_000_000, 1.0, seed=42, price_decimals=4)
    eng = Engine(max_symbols=1 << 20, max_batch=n, max_nodes=1 << 22, max_levels=1 << 26)
    orc = Oracle(1 << 20)
    for i in range(3):
        b = g.batch(n).copy()
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"config5 batch {i}")
    syms = _hot_and_random(g.zipf, 1_000_000)
    _cmp_books(eng, orc, syms, "config5")
    assert max(len(orc.levels(s)) for s in syms[:8]) > 2000


# ---- ABI v4 ----------------------------------------------------------------------------------
def test_seq_base_in_events():
    st = wl.Stream(20, seed=3)
    b = st.batch(20000)
    eng = Engine(max_symbols=20, max_batch=20000)
    orc = Oracle(20)
    base = (7 << 32) + 123
    eng.submit(b, seq_base=base)
    got = eng.drain()
    exp = orc.submit(b)
    # taker_seq = the low 32 bits of seq_base + batch index (the caller holds seq_base)
    want = (exp["taker_seq"].astype(np.uint64) + np.uint64(base)) & np.uint64(0xFFFFFFFF)
    assert np.array_equal(got["taker_seq"].astype(np.uint64), want)
    got["taker_seq"] = exp["taker_seq"]
    _cmp(got, exp, "seq_base")


def test_device_events_never_dropped():
    """a device submit's undrained events survive a following host submit."""
    torch = pytest.importorskip("torch")
    st = wl.Stream(50, seed=8)
    b1, b2 = st.batch(30000), st.batch(30000)
    eng = Engine(max_symbols=50, max_batch=30000)
    orc = Oracle(50)
    t = torch.from_numpy(b1.view(np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    eng.submit_device(t.data_ptr(), len(b1))
    e1 = orc.submit(b1)
    assert eng.device_events()[1] == len(e1)
    eng.submit(b2)  # before draining the device batch
    e2 = orc.submit(b2)
    _cmp(eng.drain(), np.concatenate([e1, e2]), "device then host")
    # released device events are not moved to the host queue
    b3, b4 = st.batch(1000), st.batch(1000)
    t3 = torch.from_numpy(b3.view(np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    eng.submit_device(t3.data_ptr(), len(b3))
    orc.submit(b3)
    eng.release_device_events()
    eng.submit(b4)
    _cmp(eng.drain(), orc.submit(b4), "after release")


def test_pipelined_async_equals_oracle():
    """gome_submit_batch_async / gome_collect with GOME_MAX_INFLIGHT (3) batches in flight == the oracle."""
    st = wl.NativeStream(300, 1.0, seed=5, del_frac=0.3, aggressive_frac=0.05)
    batches = [st.batch(40000).copy() for _ in range(6)]
    eng = Engine(max_symbols=300, max_batch=40000)
    orc = Oracle(300)
    with pytest.raises(GomeError) as ei:
        eng.collect()
    assert ei.value.status == GOME_E_NOTFOUND
    bufs = [eng.host_buffer(len(b)) for b in batches]
    for buf, b in zip(bufs, batches):
        buf[:] = b
    exp = [orc.submit(b) for b in batches]
    for k in range(3):
        eng.submit_async(bufs[k])
    assert eng.inflight() == 3
    with pytest.raises(GomeError) as ei:
        eng.submit_async(bufs[3])
    assert ei.value.status == GOME_E_STATE
    for k in range(len(batches)):
        ev, stt = eng.collect()
        _cmp(ev, exp[k], f"async batch {k}")
        assert stt["n_orders"] == len(batches[k])
        if k + 3 < len(batches):
            eng.submit_async(bufs[k + 3])
    assert eng.inflight() == 0
    # a synchronous call after async ones collects them into the drain queue first
    b = st.batch(1000).copy()
    buf = eng.host_buffer(len(b))
    buf[:] = b
    eng.submit_async(buf)
    b2 = st.batch(1000).copy()
    eng.submit(b2)
    _cmp(eng.drain(), np.concatenate([orc.submit(b), orc.submit(b2)]), "async then sync")


def test_unknown_record_flags_rejected():
    st = wl.Stream(4, seed=1)
    eng = Engine(max_symbols=4, max_batch=1024)
    orc = Oracle(4)
    good = st.batch(500)
    eng.submit(good)
    _cmp(eng.drain(), orc.submit(good))
    bad = st.batch(100)
    bad[7]["flags"] = 4
    with pytest.raises(GomeError) as ei:
        eng.submit(bad)
    assert ei.value.status == GOME_E_INVAL
    nxt = st.batch(500)
    eng.submit(nxt)
    _cmp(eng.drain(), orc.submit(nxt), "after rejected batch")


def test_host_resolved_admission_flags():
    """GOME_ORD_ADM_HOST: the consumer's pre-pool markers decide (gome_amd/consumer.PrePool).
    A host-rejected ADD is dropped like a missing marker (engine.go:58-60); a host-admitted
    duplicate key in the same batch is admitted (the batch rule would drop it)."""
    st = wl.Stream(2, seed=4)
    b = st.batch(2000)
    eng = Engine(max_symbols=2, max_batch=4096)
    orc = Oracle(2)
    rej = b.copy()
    rej["flags"] = GOME_ORD_ADM_HOST
    rej["flags"][::2] |= GOME_ORD_ADMITTED
    eng.submit(rej)
    ref = b.copy()
    ref["action"][1::2] = 7  # rejected ADDs change nothing (consumed, ignored)
    exp = orc.submit(ref)
    _cmp(eng.drain(), exp, "host admission")
    assert eng.stats()["n_dropped"] == len(b) // 2
    # duplicate key, host-admitted twice in one batch: the second names a node that the first
    # already made (S:node:<oid>): the duplicate-oid rule drops it (gome_abi.h, Q7)
    d = np.zeros(2, wl.ORDER_DTYPE)
    d[:] = (10**6, 10**6, 0, 999999, 5, 0, 1, GOME_ORD_ADM_HOST | GOME_ORD_ADMITTED)
    d[1]["price_fx"] = 2 * 10**6 // 4  # another (non-crossing) price
    eng.submit(d)
    eng.drain()
    st = eng.stats()
    assert st["n_dropped"] == 1 and st["n_dup_oid"] == 1 and st["n_rests"] == 1
    assert eng.dup_records().tolist() == [1]


def test_q8_transaction_codes_on_gpu_vs_literal():
    from oracle.literal import run_batches
    from tests.helpers import Interner, render_events, requests_to_records
    rng = np.random.default_rng(21)
    req = lambda a, oid, tx, p, v: (a, dict(uuid="u1", oid=str(oid), symbol="s", transaction=tx,
                                            price=p, volume=v))
    txs = [0, 1, 257, -3, 2**31 - 1, 1, 0]
    batches, oid = [], 1
    for _ in range(4):
        b = []
        for _ in range(60):
            b.append(req(1, oid, int(rng.choice(txs)), float(rng.choice([0.3, 0.4, 0.5, 0.6])),
                         float(rng.choice([0.1, 0.5, 1.0]))))
            oid += 1
        batches.append(b)
    _, lit = run_batches(batches)
    names = Interner()
    names.id("sym", "s")
    eng = Engine(max_symbols=1, max_batch=64)
    got = []
    for b in batches:
        rec = requests_to_records(b, names)
        eng.submit(rec)
        got += render_events(eng.drain(), rec, names)
    assert got == lit


# ---- cancel index and level pool hygiene ------------------------------------------------
def test_index_rebuild_soak():
    """erases leave tombstones; a small index is rebuilt from the live nodes before it
    fills, cancels of filled / unknown oids stay exact, and every probe terminates."""
    g = wl.NativeStream(64, 1.0, seed=9, del_frac=0.5, aggressive_frac=0.1)
    eng = Engine(max_symbols=64, max_batch=20000, max_nodes=4096, flags=GOME_FLAG_NO_HEADROOM)
    orc = Oracle(64)
    for i in range(40):
        b = g.batch(20000).copy()
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"soak batch {i}")
    st = eng.stats()
    assert st["n_index_rebuilds"] > 0
    _cmp_books(eng, orc, range(64), "soak")


def _buys(sym0, nsym, nprice, oid0, pbase=1):
    rows = []
    oid = oid0
    for s in range(sym0, sym0 + nsym):
        for k in range(nprice):
            rows.append((int((pbase + k) * 10**5), 10**6, s, oid, 1, 0, 1, 0))
            oid += 1
    return np.array(rows, dtype=wl.ORDER_DTYPE), oid


def test_level_blocks_reused():
    """A book that outgrows its level block releases it; blocks of that class are handed to
    other books in later batches instead of carving new ones.  Cold books of
    up to 128 levels grow in LDS and take one block of the final size at write-back; larger
    ones grow block by block in HBM."""
    eng = Engine(max_symbols=256, max_batch=30000, max_levels=1 << 17)
    orc = Oracle(256)
    b1, oid = _buys(0, 100, 40, 1)                  # 100 books of 40 levels: one 64-block each
    eng.submit(b1)
    _cmp(eng.drain(), orc.submit(b1))
    used1 = eng.stats()["lvl_used"]
    assert used1 == 100 * 64
    b2, oid = _buys(0, 100, 60, oid, pbase=41)      # they grow to 100 levels: 128-blocks, the
    eng.submit(b2)                                  # 64-blocks released
    _cmp(eng.drain(), orc.submit(b2))
    used2 = eng.stats()["lvl_used"]
    assert used2 == used1 + 100 * 128
    b3, oid = _buys(100, 100, 40, oid)              # 100 new books of 40 levels: the released
    eng.submit(b3)                                  # 64-blocks
    _cmp(eng.drain(), orc.submit(b3))
    assert eng.stats()["lvl_used"] == used2
    b4, oid = _buys(0, 20, 100, oid, pbase=101)     # 200 levels: beyond the LDS copy, the HBM
    eng.submit(b4)                                  # path (spill to 256-blocks)
    _cmp(eng.drain(), orc.submit(b4))
    assert eng.stats()["lvl_used"] == used2 + 20 * 256
    _cmp_books(eng, orc, list(range(0, 200, 7)) + [0, 19], "levels")


# ---- multi-GPU sharding with real engines ----------------------------------
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_engines_equal_single_engine(world):
    """N engine handles on device 0, one per shard (Zipf rank % N): per-shard events mapped
    back to the global batch index and merged on (seq, fill_idx) == the single engine."""
    n_sym, n = 2000, 1 << 18
    g = wl.Stream(n_sym, zipf_s=1.0, seed=17)
    z = g.zipf
    one = Engine(max_symbols=n_sym, max_batch=n)
    shards = [Engine(max_symbols=n_sym, max_batch=n) for _ in range(world)]
    for bi in range(3):
        b = g.batch(n)
        one.submit(b)
        exp = one.drain()
        ranks = z.id_to_rank[b["symbol_id"]]
        parts = []
        for r in range(world):
            idx = np.nonzero(ranks % world == r)[0]
            shards[r].submit(b[idx])
            ev = shards[r].drain().copy()
            ev["taker_seq"] = idx[ev["taker_seq"]]
            parts.append(ev)
        u = np.concatenate(parts)
        u = u[np.lexsort((u["fill_idx"], u["taker_seq"]))]
        assert u.tobytes() == exp.tobytes(), f"batch {bi}"
    assert sum(s.stats()["n_resting"] for s in shards) == one.stats()["n_resting"]


# ---- transactional capacity errors ------------------------------------------------------
def test_capacity_rejected_before_applying():
    """a batch whose ADDs could push the resting makers past max_nodes is
    rejected with E_CAPACITY before anything is applied: the book is unchanged and the handle
    stays usable (cancels free room, then the same batch is accepted)."""
    from gome_amd.abi import GOME_E_CAPACITY

    def bids(oid0, n):  # BUYs that never cross (no asks): every one rests
        r = np.zeros(n, wl.ORDER_DTYPE)
        r["price_fx"] = (10 + np.arange(n) % 50) * 10**6
        r["volume_fx"] = 10**6
        r["symbol_id"] = np.arange(n) % 4
        r["oid_id"] = np.arange(oid0, oid0 + n)
        r["uuid_id"] = 3
        r["side"] = 0
        r["action"] = wl.ADD
        return r

    eng = Engine(max_symbols=4, max_batch=2000, max_nodes=3000, max_levels=1 << 16)
    orc = Oracle(4)
    for b in (bids(1, 1000), bids(1001, 1000)):
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b))
    assert eng.stats()["n_resting"] == 2000
    b3 = bids(2001, 1500)
    with pytest.raises(GomeError) as ei:
        eng.submit(b3)
    assert ei.value.status == GOME_E_CAPACITY
    assert eng.stats()["n_resting"] == 2000
    _cmp_books(eng, orc, range(4), "after the rejected batch")
    d = bids(1, 800)
    d["action"] = wl.DEL
    eng.submit(d)
    _cmp(eng.drain(), orc.submit(d))
    eng.submit(b3)
    _cmp(eng.drain(), orc.submit(b3))
    assert eng.stats()["n_resting"] == 2700
    _cmp_books(eng, orc, range(4), "after the accepted batch")


# ---- admission (Q4) under heavy key reuse -------------------------------------------------
def _run_admission(batches, n_symbols, syms):
    eng = Engine(max_symbols=n_symbols, max_batch=max(len(b) for b in batches), max_nodes=1 << 20,
                 max_levels=1 << 20)
    orc = Oracle(n_symbols)
    for i, b in enumerate(batches):
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"batch {i}")
    _cmp_books(eng, orc, syms)
    assert eng.stats()["n_resting"] == orc.resting()
    return eng


def test_admission_keys_repeated_within_batches():
    """Every (symbol, uuid, oid) key repeats tens of times inside its batch among ADDs and DELs:
    only an ADD ahead of every other record of its key is admitted (engine.go:58-62,90).  An oid
    names one key (its symbol and uuid) and never recurs in a later batch, so no oid is admitted
    twice (Q7 stays outside the domain, tests/helpers.py:random_batches).  The hot books stay on
    the flow path with most of their ADDs dropped."""
    rec = wl.cancel_mix(160000, 40, seed=19, zipf_s=1.0)
    rng = np.random.default_rng(19)
    batches = wl.split_batches(rec, 40000)
    for k, b in enumerate(batches):
        oid = 1 + k * 200000 + b["symbol_id"].astype(np.int64) * 5000 + rng.integers(0, 250, len(b))
        b["oid_id"] = oid.astype(b["oid_id"].dtype)
        b["uuid_id"] = (1 + oid % 2).astype(b["uuid_id"].dtype)
    eng = _run_admission(batches, 40, range(40))
    assert eng.stats()["n_flow_books"] > 0
