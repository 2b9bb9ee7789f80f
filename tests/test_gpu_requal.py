"""HIP engine (MI355X) — quirk books back on the flow path.

A wrong-side cancel (Q2) or a zero-volume maker (Q6) puts a book in a state the aggregate plans
cannot express (BOOK_QUIRK), so the legacy kernel (~23x slower) applies it.  The reference's state
heals (nodepool.go:76-83, engine.go:145-175); k_requalify (match_requal.h) clears the flag once it
has.  On bench.py's config-3 stream, the hottest book gets both quirks injected in batch 1
(workload.inject_quirks, through the engine's own snapshot of the book), and every batch is
compared event for event with the C oracle; the books' levels and FIFOs at the end too."""
import struct

import numpy as np
import pytest

import bench
from gome_amd import workload as wl
from gome_amd.abi import Engine
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books, _hot_and_random

pytestmark = pytest.mark.gpu

N = 1 << 20
HAZ_OFF = 144  # FlowHdr::haz (match_flow.h static_assert); HZ_* bits
HZ_STALE = 64


def _run(mode, batches=5):
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
    z = wl.ZipfSymbols(100000, 1.0)
    hot = int(z.rank_to_id[0])
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=batches * N, max_levels=1 << 22)
    orc = Oracle(100000)
    kinds, req, wrong, bails, hazs = [], [], [], [], []
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
        wrong.append(int(st["n_flow_wrong"]))
        bails.append(int(st["n_flow_bail"]))
        hazs.append(struct.unpack("<I", eng.debug_peek(0, HAZ_OFF, 4))[0])  # (FlowHdr::haz of the hottest book)
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=50), mode)
    assert eng.stats()["n_resting"] == orc.resting()
    _run.bails, _run.hazs = bails, hazs
    return kinds, req, wrong


def test_quirks_heal_and_the_hottest_book_returns_to_the_flow_path():
    """The quirks at the best bids, where the stream soon trades.  The zero-volume maker behind the
    second-best bid is popped by a SALE that sweeps that level and goes on (the level-end
    continuation, round 6).  What hands the injected batch to the legacy kernel is the stale bid
    alone (FlowHdr::haz == HZ_STALE): a SALE rests at the stale price (in S:BUY, no FIFO), and a later
    SALE taker reaches that price through S:BUY and fills against the resting SALE -- a same-side
    fill the reference really publishes (the oracle's batch 1: one fill whose maker and taker are
    both SALEs), which no aggregate plan can express.  The batches after it are on the flow path
    again, exact throughout."""
    kinds, req, wrong = _run("heal")
    assert kinds[0] != 0 and wrong[1] >= 1, (kinds, wrong)
    assert kinds[1] == 0 and _run.hazs[1] == HZ_STALE, (kinds, [hex(h) for h in _run.hazs])
    assert all(k != 0 for k in kinds[2:]) and sum(_run.bails) == 1, (kinds, _run.bails)


def test_quirks_that_do_not_heal_stay_on_the_flow_path():
    """The same quirks at the bottom of the bid book, which the stream never reaches again: batch 1
    applies them on the legacy kernel; the stale member (Q2) and the zero-volume maker (Q6, marked
    L_ZERO / BOOK_ZERO by k_requalify) then ride along on the flow path (round 5; in round 4 the book
    stayed on the ~23x slower legacy kernel for good), exact throughout; the injected batch itself runs
    on the flow cancel path (its wrong-side cancels, FlowHdr::nwrong, and the zero-volume ADD resting
    behind a level's makers)."""
    kinds, req, wrong = _run("stuck", batches=5)
    assert all(k != 0 for k in kinds), (kinds, req)   # the injected batch too (round 5)
    assert wrong[1] >= 1, wrong


# ---- stale members on the flow path (Q2 alone) -----------------------------
def _move_away(b, sym, p, after=-1):
    """Records of `sym` at price p (the rows after `after`) move one tick up, so nothing rests or
    trades there: the stale member stays stale."""
    rows = np.nonzero(b["symbol_id"] == sym)[0]
    rows = rows[(rows > after) & (b["price_fx"][rows] == p)]
    b["price_fx"][rows] = p + 10 ** 6


def _stale_inject(b, sym, eng):
    """Wrong-side cancels of every maker of `sym`'s lowest bid (its first records), the rest of the
    symbol's records at that price moved away: a stale member of S:BUY from this batch on."""
    info = wl.inject_quirks(b, sym, eng.levels(sym), lambda p: eng.fifo(sym, p), "q2stuck")
    assert info["q2_cancels"] >= 1
    _move_away(b, sym, info["q2_price"], after=max(info["records"]))
    return info["q2_price"]


def _stale_run(rank, seed, hazard, batches=5, edit1=None):
    """Batch 1: a stale member made (on the legacy kernel: a book with wrong-side DELs); then the
    book on the flow path with it; with `hazard`, batch 2's first record of the book is a SALE at
    the stale price with a volume above the whole bid side, so it sweeps every real bid and rests
    there (the price in both side sets in the reference, where a later SALE taker would meet that
    SALE maker): k_flow_stale_check hands the book to the legacy kernel after its plan.  Every
    batch's events and the books at the end are the oracle's."""
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, seed)
    z = wl.ZipfSymbols(100000, 1.0)
    sym = int(z.rank_to_id[rank])
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=(batches + 1) * N, max_levels=1 << 22)
    orc = Oracle(100000)
    p, out = None, []
    for i in range(batches):
        b = gen(N).copy()
        if i == 1:
            p = _stale_inject(b, sym, eng)
            if edit1 is not None:
                edit1(b, sym, p)
        elif i >= 2:
            _move_away(b, sym, p)
            if hazard and i == 2:
                r = np.nonzero(b["symbol_id"] == sym)[0][0]
                b["price_fx"][r], b["side"][r], b["action"][r], b["volume_fx"][r] = p, 1, wl.ADD, 10 ** 14
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"stale rank {rank} batch {i}")
        st = eng.stats()
        fl = eng.debug_flow_books()
        kind = int(fl["kind"][list(fl["symbol_id"]).index(sym)]) if sym in list(fl["symbol_id"]) else -1
        out.append((kind, int(st["n_flow_stale"]), int(st["n_flow_bail"]), int(st["n_flow_wrong"])))
    _cmp_books(eng, orc, [sym] + _hot_and_random(z, 100000, k_rand=30), f"stale rank {rank}")
    assert eng.stats()["n_resting"] == orc.resting()
    lv = orc.levels(sym)
    return out, lv[lv["price_fx"] == p]


def test_stale_member_stays_on_the_flow_path():
    """The hottest book with a stale member of S:BUY (no FIFO, depth 0) is planned on the flow path
    from the batch after the one that made it (k_requalify accepts it, n_flow_stale), exact, and the
    stale member is still there at the end (levels compared with the oracle's)."""
    out, lv = _stale_run(0, 42, hazard=False)
    assert out[1][0] != 0 and out[1][3] >= 1 and out[1][2] == 0, out  # (the wrong-side cancels: flow)
    assert all(k != 0 and s >= 1 and x == 0 for k, s, x, _ in out[2:]), out
    assert len(lv) == 1 and lv["in_buy"][0] == 1 and lv["n_nodes"][0] == 0, lv


def test_order_resting_opposite_a_stale_price_hands_the_book_to_legacy():
    out, _ = _stale_run(0, 42, hazard=True)
    assert out[2][1] >= 1 and out[2][2] >= 1 and out[2][0] == 0, out


def test_near_book_hand_over():
    """The same for the second-hottest book (the near books' reconstruction on the hot stream)."""
    out, _ = _stale_run(1, 43, hazard=True)
    assert out[2][1] >= 1 and out[2][2] >= 1, out


def test_wrong_side_cancels_then_a_rest_across_in_the_same_batch_hand_over():
    """The wrong-side cancels empty the lowest bid (a stale member of S:BUY from then on) and, later
    in the same batch, a SALE sweeps every bid and rests at that price: k_fc_stale_level finds the
    REST on the other side of the stale price and the book goes to the legacy kernel, exact."""
    def edit1(b, sym, p):
        r = np.nonzero(b["symbol_id"] == sym)[0][5000]
        b["price_fx"][r], b["side"][r], b["action"][r], b["volume_fx"][r] = p, 1, wl.ADD, 10 ** 14
    out, _ = _stale_run(0, 42, hazard=False, edit1=edit1)
    assert out[1][0] == 0 and out[1][2] >= 1 and out[1][3] >= 1, out


def test_wrong_side_cancel_of_a_new_maker():
    """A BUY rests at a price of its own between two bids and a DEL with the SALE side cancels it a
    few records later (the cancel path's new-maker target): the level stays a stale member of
    S:BUY; at a second such price a later BUY rests again, which heals it.  On the flow path
    (n_flow_wrong), exact, the levels compared with the oracle's."""
    def edit1(b, sym, p):
        rows = np.nonzero((b["symbol_id"] == sym) & (b["action"] == wl.ADD))[0]
        for k, (a, heal) in enumerate(((2000, False), (3000, True))):
            pn = p + 10 ** 6 * (k + 2) + 1
            ra, rd, rh = rows[a], rows[a + 5], rows[a + 10]
            b["price_fx"][ra], b["side"][ra], b["volume_fx"][ra] = pn, 0, 10 ** 8
            b["action"][rd], b["flags"][rd], b["price_fx"][rd], b["side"][rd] = wl.DEL, 0, pn, 1
            b["oid_id"][rd], b["uuid_id"][rd], b["volume_fx"][rd] = b["oid_id"][ra], b["uuid_id"][ra], 10 ** 8
            if heal:
                b["price_fx"][rh], b["side"][rh], b["volume_fx"][rh] = pn, 0, 10 ** 8
    out, _ = _stale_run(0, 42, hazard=False, edit1=edit1)
    assert all(k != 0 and x == 0 for k, _, x, _ in out), out
    assert out[1][3] >= 1, out


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


def _hot_rows(b, hot):
    return np.nonzero((b["symbol_id"] == hot) & (b["action"] == wl.ADD))[0]


def test_zero_volume_maker_no_order_reaches_stays_on_the_flow_path():
    """A zero-volume ADD resting at the lowest bid (behind its makers, depth > 0): an ordinary FIFO
    append on the flow path; no order reaches it later, so the book stays on the flow path with the
    zero-volume maker in its FIFO (BOOK_ZERO), exact."""
    def edit(b, hot, eng):
        lv = eng.levels(hot)
        bids = np.sort(lv[(lv["in_buy"] != 0) & (lv["n_nodes"] > 0)], order="price_fx")
        r = _hot_rows(b, hot)[100]
        b["volume_fx"][r], b["side"][r], b["price_fx"][r] = 0, 0, bids["price_fx"][0]
    out = _zero_run(45, edit, batches=5)
    assert all(k != 0 for k, _, _ in out) and all(x == 0 for _, _, x in out), out
    assert all(z >= 1 for _, z, _ in out[2:]), out


def test_zero_volume_maker_popped_by_a_passing_taker_stays_on_the_flow_path():
    """A zero-volume BUY behind the best bid's makers, a BUY of 1.00 behind it, then a SALE at the best
    bid for the level's depth + 0.50: the SALE fills every old maker, pops the zero-volume one with a
    0-fill (MatchOrder's diff > 0 branch, engine.go:145-161) and takes half of the new BUY, leaving the
    level's depth > 0.  The reconstruction pops it (fl_first_back, the intervals), so the book stays
    on the flow path with no hand-over, exact."""
    def edit(b, hot, eng):
        lv = eng.levels(hot)
        bids = np.sort(lv[(lv["in_buy"] != 0) & (lv["n_nodes"] > 0)], order="price_fx")
        best = bids[-1]
        rows = _hot_rows(b, hot)[:3]
        b["volume_fx"][rows[0]], b["side"][rows[0]], b["price_fx"][rows[0]] = 0, 0, best["price_fx"]
        b["volume_fx"][rows[1]], b["side"][rows[1]], b["price_fx"][rows[1]] = 10 ** 8, 0, best["price_fx"]
        b["volume_fx"][rows[2]], b["side"][rows[2]] = int(best["depth_fx"]) + 5 * 10 ** 7, 1
        b["price_fx"][rows[2]] = best["price_fx"]
    out = _zero_run(48, edit)
    assert out[2][0] != 0 and out[2][1] >= 1 and out[2][2] == 0, out


def test_zero_volume_maker_at_a_new_price_hands_the_book_to_legacy():
    """A zero-volume BUY below every level: the reference makes it a side-set member of depth 0
    (SetPoolDepth), which the plans would not visit: k_flow_zero_check hands the book to the legacy
    kernel after its plan, exact."""
    def edit(b, hot, eng):
        r = _hot_rows(b, hot)[100]
        b["volume_fx"][r], b["side"][r], b["price_fx"][r] = 0, 0, 1
    out = _zero_run(46, edit)
    assert out[2][0] == 0 and out[2][1] >= 1 and out[2][2] >= 1, out


def test_zero_volume_maker_at_the_end_of_a_swept_level_stays_on_the_flow_path():
    """A zero-volume BUY at the best bid (the last maker of its FIFO) followed by a SALE sweeping
    every bid: the SALE takes the level's whole depth with volume to spare, so MatchOrder's diff > 0
    branch goes on and pops the zero-volume maker at the level's end with a 0-fill before Match moves
    to the next bid (engine.go:145-161, 129-131).  The level-end continuation (round 6, fl_cont: the
    taker's next touch is its own) pops it in the reconstruction too; until round 6 this handed the
    book to the legacy kernel.  Exact, the book on the flow path, no hand-over."""
    def edit(b, hot, eng):
        lv = eng.levels(hot)
        bids = np.sort(lv[(lv["in_buy"] != 0) & (lv["n_nodes"] > 0)], order="price_fx")
        rows = _hot_rows(b, hot)
        b["volume_fx"][rows[0]], b["side"][rows[0]], b["price_fx"][rows[0]] = 0, 0, bids["price_fx"][-1]
        b["volume_fx"][rows[1]], b["side"][rows[1]], b["price_fx"][rows[1]] = 10 ** 14, 1, 10 ** 6
    out = _zero_run(47, edit)
    assert out[2][0] != 0 and out[2][1] >= 1 and out[2][2] == 0, out
    assert all(k != 0 for k, _, _ in out), out


def _del_of(b, row, eng, hot, price, k=0):
    """Record `row` becomes a DEL of the k-th maker of the hot book's FIFO at `price` (delorder.go)."""
    m = eng.fifo(hot, int(price))[k]
    b["action"][row], b["flags"][row] = wl.DEL, 0
    b["oid_id"][row], b["uuid_id"][row], b["side"][row] = m["oid_id"], m["uuid_id"], m["side"]
    b["price_fx"][row], b["volume_fx"][row] = price, m["volume_fx"]


def test_zero_volume_maker_popped_in_a_batch_with_dels_stays_on_the_flow_path():
    """Round 6: the passing-taker case of the test above in a batch with DELs --
    one of a maker at the lowest bid, one of the best bid's first maker, ahead of the zero-volume maker
    (a cancel that moves it in consumption space) -- so the book takes the cancel path, whose
    reconstruction now pops the zero-volume maker with a 0-fill (fc_fills, the gathers): exact, the
    book on the flow path (kind != 0), no hand-over."""
    def edit(b, hot, eng):
        lv = eng.levels(hot)
        bids = np.sort(lv[(lv["in_buy"] != 0) & (lv["n_nodes"] > 1)], order="price_fx")
        best = bids[-1]
        f = eng.fifo(hot, int(best["price_fx"]))
        rows = _hot_rows(b, hot)[:5]
        _del_of(b, rows[0], eng, hot, bids[0]["price_fx"])
        _del_of(b, rows[1], eng, hot, best["price_fx"])            # (ahead of the zero-volume maker)
        b["volume_fx"][rows[2]], b["side"][rows[2]], b["price_fx"][rows[2]] = 0, 0, best["price_fx"]
        b["volume_fx"][rows[3]], b["side"][rows[3]], b["price_fx"][rows[3]] = 10 ** 8, 0, best["price_fx"]
        left = int(best["depth_fx"]) - int(f[0]["volume_fx"])
        b["volume_fx"][rows[4]], b["side"][rows[4]] = left + 5 * 10 ** 7, 1
        b["price_fx"][rows[4]] = best["price_fx"]
    out = _zero_run(49, edit)
    assert out[2][0] != 0 and out[2][1] >= 1 and out[2][2] == 0, out
    assert all(k != 0 for k, _, _ in out), out


def test_zero_volume_maker_left_at_an_emptied_level_with_dels_hands_over():
    """The hazard the cancel path keeps: a SALE that takes exactly the best bid's depth (every maker
    ahead of the zero-volume one) in a batch with DELs empties the level with the zero-volume maker
    still in its FIFO (the reference leaves it in a FIFO whose level left its set): k_flow_zero_check
    hands the book to the legacy kernel after its plan, exact."""
    def edit(b, hot, eng):
        lv = eng.levels(hot)
        bids = np.sort(lv[(lv["in_buy"] != 0) & (lv["n_nodes"] > 0)], order="price_fx")
        best = bids[-1]
        rows = _hot_rows(b, hot)[:3]
        _del_of(b, rows[0], eng, hot, bids[0]["price_fx"])
        b["volume_fx"][rows[1]], b["side"][rows[1]], b["price_fx"][rows[1]] = 0, 0, best["price_fx"]
        b["volume_fx"][rows[2]], b["side"][rows[2]] = int(best["depth_fx"]), 1
        b["price_fx"][rows[2]] = best["price_fx"]
    out = _zero_run(50, edit)
    assert out[2][0] == 0 and out[2][2] >= 1, out


def test_zero_volume_maker_at_the_end_of_a_swept_level_with_dels_stays_on_the_flow_path():
    """The level-end continuation on the cancel path: the batch of the test above holds a DEL (a
    maker of the lowest bid), a zero-volume BUY rests behind the best bid's makers, and a SALE at the
    best bid for the level's depth + 1.00 takes every maker, pops the zero-volume one at the level's
    end (fc_touch / fc_fills with the consume going on, the gathers' FlowLvl::zcont) and rests its
    remainder there: exact, the book on the flow path, no hand-over."""
    def edit(b, hot, eng):
        lv = eng.levels(hot)
        bids = np.sort(lv[(lv["in_buy"] != 0) & (lv["n_nodes"] > 0)], order="price_fx")
        best = bids[-1]
        rows = _hot_rows(b, hot)[:3]
        _del_of(b, rows[0], eng, hot, bids[0]["price_fx"])
        b["volume_fx"][rows[1]], b["side"][rows[1]], b["price_fx"][rows[1]] = 0, 0, best["price_fx"]
        b["volume_fx"][rows[2]], b["side"][rows[2]] = int(best["depth_fx"]) + 10 ** 8, 1
        b["price_fx"][rows[2]] = best["price_fx"]
    out = _zero_run(51, edit)
    assert out[2][0] != 0 and out[2][1] >= 1 and out[2][2] == 0, out
    assert all(k != 0 for k, _, _ in out), out


def test_zero_volume_takers_in_a_batch_with_dels_stay_on_the_flow_path():
    """Zero-volume takers on the cancel path (round 6): the batch of the zero-taker test above plus a
    DEL (a maker of the lowest bid), so the book takes the cancel plan.  Each taker's CONS of 0 fills
    the head of the best opposite level's FIFO at its time (fc_head_at: the first maker then live,
    a maker cancelled later included) with one 0-fill; exact, the book on the flow path."""
    def edit(b, hot, eng):
        lv = eng.levels(hot)
        bids = np.sort(lv[(lv["in_buy"] != 0) & (lv["n_nodes"] > 0)], order="price_fx")
        rows = _hot_rows(b, hot)
        _del_of(b, rows[0], eng, hot, bids[0]["price_fx"])
        picks = rows[(np.array([0.0002, 0.01, 0.3, 0.6, 0.95]) * len(rows)).astype(int)]
        for k, r in enumerate(picks):
            sale = k % 2 == 1
            b["volume_fx"][r], b["side"][r] = 0, 1 if sale else 0
            b["price_fx"][r] = 10 ** 6 if sale else 10 ** 8
    out = _zero_run(52, edit)
    assert out[2][0] != 0 and out[2][1] >= 1 and out[2][2] == 0, out
    assert all(k != 0 for k, _, _ in out), out
