"""HIP engine (MI355X) — quirk books back on the flow path.

A wrong-side cancel (Q2) or a zero-volume maker (Q6) puts a book in a state the aggregate plans
cannot express (BOOK_QUIRK), so the legacy kernel (~23x slower) applies it.  The reference's state
heals (nodepool.go:76-83, engine.go:145-175); k_requalify (match_requal.h) clears the flag once it
has.  On bench.py's config-3 stream, the hottest book gets both quirks injected in batch 1
(workload.inject_quirks, through the engine's own snapshot of the book), and every batch is
compared event for event with the C oracle; the books' levels and FIFOs at the end too."""
import numpy as np
import pytest

import bench
from gome_amd import workload as wl
from gome_amd.abi import Engine
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books, _hot_and_random

pytestmark = pytest.mark.gpu

N = 1 << 20


def _run(mode, batches=5):
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
    z = wl.ZipfSymbols(100000, 1.0)
    hot = int(z.rank_to_id[0])
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=batches * N, max_levels=1 << 22)
    orc = Oracle(100000)
    kinds, req = [], []
    for i in range(batches):
        b = gen(N).copy()
        if i == 1:
            info = wl.inject_quirks(b, hot, eng.levels(hot), lambda p: eng.fifo(hot, p), mode)
            assert info["q2_cancels"] >= 1
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"{mode} batch {i}")
        st = eng.stats()
        fl = eng.debug_flow_books()
        assert int(fl["symbol_id"][0]) == hot
        kinds.append(int(fl["kind"][0]))
        req.append((st["n_quirk_checked"], st["n_requalified"]))
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=50), mode)
    assert eng.stats()["n_resting"] == orc.resting()
    return kinds, req


def test_quirks_heal_and_the_hottest_book_returns_to_the_flow_path():
    kinds, req = _run("heal")
    assert kinds[0] != 0 and kinds[1] == 0, kinds        # flow, then legacy for the injected batch
    healed = [i for i, (c, r) in enumerate(req) if r]
    assert healed and healed[0] <= 2, req                 # healed within two batches
    assert all(k != 0 for k in kinds[healed[0] + 1:]), (kinds, req)


def test_quirk_that_does_not_heal_stays_on_legacy_and_exact():
    kinds, req = _run("stuck", batches=4)
    assert kinds[0] != 0 and all(k == 0 for k in kinds[1:]), kinds
    assert all(r == 0 for _, r in req) and all(c >= 1 for c, _ in req[1:]), req


# ---- stale members on the flow path (Q2 alone) -----------------------------
def test_stale_member_stays_on_the_flow_path():
    """Wrong-side cancels of every maker of the lowest bid (never reached again): batch 1 applies
    them on the legacy kernel (a book with DELs of the wrong side), the level stays in S:BUY with no
    FIFO, k_requalify accepts the stale member, and from batch 2 on the hottest book is planned on
    the flow path with it (n_flow_stale), exact throughout."""
    kinds, req = _run("q2stuck", batches=5)
    assert kinds[0] != 0 and kinds[1] == 0, kinds
    assert all(k != 0 for k in kinds[2:]), (kinds, req)
    assert req[1][1] >= 1, req  # (requalified after batch 1 with the stale level)


def _hand_over(rank, seed, batches=5):
    """Batch 1: wrong-side cancels of every maker of symbol `rank`'s lowest bid (its first records:
    a stale member from then on); batch 2: planned with it; batch 3: the book's first record is a
    SALE at the stale price with a volume above the whole bid side, so it sweeps every real bid and
    rests there: the price is then in both side sets in the reference, where a later SALE taker
    would meet that SALE maker.  k_flow_stale_check hands the book to the legacy kernel after its
    plan; every batch's events and the books at the end are the oracle's."""
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, seed)
    z = wl.ZipfSymbols(100000, 1.0)
    sym = int(z.rank_to_id[rank])
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=(batches + 1) * N, max_levels=1 << 22)
    orc = Oracle(100000)
    stale_p, bails, stales = None, [], []
    for i in range(batches):
        b = gen(N).copy()
        if i == 1:
            stale_p = wl.inject_quirks(b, sym, eng.levels(sym), lambda p: eng.fifo(sym, p), "q2stuck")["q2_price"]
        if i == 3:
            r = np.nonzero(b["symbol_id"] == sym)[0][0]
            b["price_fx"][r], b["side"][r], b["action"][r], b["volume_fx"][r] = stale_p, 1, wl.ADD, 10 ** 14
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"hand-over rank {rank} batch {i}")
        st = eng.stats()
        bails.append(int(st["n_flow_bail"]))
        stales.append(int(st["n_flow_stale"]))
    _cmp_books(eng, orc, [sym] + _hot_and_random(z, 100000, k_rand=30), f"hand-over rank {rank}")
    assert eng.stats()["n_resting"] == orc.resting()
    return stales, bails


def test_order_resting_opposite_a_stale_price_hands_the_book_to_legacy():
    stales, bails = _hand_over(0, 42)
    assert stales[2] >= 1 and stales[3] >= 1 and bails[2] == 0 and bails[3] >= 1, (stales, bails)


def test_near_book_hand_over():
    """The same for the second-hottest book (the near books' reconstruction on the hot stream)."""
    stales, bails = _hand_over(1, 43)
    assert stales[3] >= 1 and bails[3] >= 1, (stales, bails)


# ---- zero-volume ADDs (Q6) on the flow path -----------------------------------------------------
def _zero_run(seed, edit, batches=4):
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, seed)
    z = wl.ZipfSymbols(100000, 1.0)
    hot = int(z.rank_to_id[0])
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=(batches + 1) * N, max_levels=1 << 22)
    orc = Oracle(100000)
    out = []
    for i in range(batches):
        b = gen(N).copy()
        if i == 2:
            edit(b, hot, eng)
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"zero batch {i}")
        st = eng.stats()
        fl = eng.debug_flow_books()
        out.append((int(fl["kind"][0]), int(st["n_flow_zero"]), int(st["n_flow_bail"])))
    _cmp_books(eng, orc, [hot] + _hot_and_random(z, 100000, k_rand=30), "zero")
    assert eng.stats()["n_resting"] == orc.resting()
    return out


def test_zero_volume_takers_stay_on_the_flow_path():
    """Zero-volume ADDs that cross (BUY at 1.00, SALE at 0.01, "Volume": 0 or null in the JSON):
    each takes 0 at the best opposite level, one 0-fill with the maker unchanged (engine.go:176-194),
    on the flow path (the plan's CONS touch of 0): the hottest book stays kind != 0, exact."""
    def edit(b, hot, eng):
        rows = np.nonzero((b["symbol_id"] == hot) & (b["action"] == wl.ADD))[0]
        rows = rows[(np.array([0.0001, 0.01, 0.3, 0.6, 0.95]) * len(rows)).astype(int)]
        for k, r in enumerate(rows):
            sale = k % 2 == 1
            b["volume_fx"][r], b["side"][r] = 0, 1 if sale else 0
            b["price_fx"][r] = 10 ** 6 if sale else 10 ** 8
    out = _zero_run(44, edit)
    assert out[2][0] != 0 and out[2][1] >= 1 and out[2][2] == 0, out
    assert all(k != 0 for k, _, _ in out), out


def test_zero_volume_maker_hands_the_book_to_legacy():
    """A zero-volume ADD that rests (a zero-volume maker, which the reconstruction does not model):
    k_flow_zero_check hands the book to the legacy kernel after its plan, exact; the maker's book is
    a quirk book afterwards (BOOK_QUIRK) until it heals."""
    def edit(b, hot, eng):
        lv = eng.levels(hot)
        bids = np.sort(lv[(lv["in_buy"] != 0) & (lv["n_nodes"] > 0)], order="price_fx")
        r = np.nonzero((b["symbol_id"] == hot) & (b["action"] == wl.ADD))[0][100]
        b["volume_fx"][r], b["side"][r], b["price_fx"][r] = 0, 0, bids["price_fx"][0]
    out = _zero_run(45, edit)
    assert out[2][1] >= 1 and out[2][2] >= 1 and out[2][0] == 0, out
