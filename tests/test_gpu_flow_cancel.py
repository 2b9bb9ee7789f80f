"""Cancels on the flow path (match_flow_cancel.h): hot books whose segment holds DELs, planned by
the W32C aggregate plan (per-side depths only: a DEL removes clamp(depth - Q, 0, v) with Q from
the cancel prep, gen_plan_asm.py) and reconstructed in consumption space.  Every case is
bit-exact against the C oracle (events, levels, FIFOs, resting count) and, where stated,
identical to the legacy FIFO kernel.

The formula itself is checked on the CPU by tools/flow_cancel_model.py (plan_book_q); these are
the device tests proper."""
import numpy as np
import pytest

from gome_amd import workload as wl
from gome_amd.abi import Engine
from oracle.pyoracle import Oracle

pytestmark = pytest.mark.gpu

ADD, DEL = wl.ADD, wl.DEL


def _engine(ns, mb, flags=0):
    return Engine(max_symbols=ns, max_batch=mb, max_nodes=1 << 20, max_levels=1 << 20, flags=flags)


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


ROUTES: list = []   # (batch, debug_flow_books) of the last _run, for assertion messages


def _routes_msg():
    from collections import Counter
    c = Counter()
    for _, fbk in ROUTES:
        for x in fbk:
            c[(int(x["kind"]), int(x["decline"]), int(x["w32"]))] += 1
    bad = [x for _, fbk in ROUTES for x in fbk if x["decline"]]
    worst = [(int(x["wsum"]), int(x["window"]), int(x["orders"]), int(x["levels"])) for x in bad[:6]]
    return "routing (kind, decline bits, w32): " + repr(dict(c)) + "; declined (window sum, window, orders, levels): " + repr(worst)


def _run(batches, ns, check_every=True):
    eng = _engine(ns, max(len(b) for b in batches))
    orc = Oracle(ns)
    fc = fb = 0
    ROUTES.clear()
    for i, b in enumerate(batches):
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"batch {i}")
        st = eng.stats()
        fc += st["n_flow_cancels"]
        fb += st["n_flow_books"]
        ROUTES.append((i, eng.debug_flow_books()))
        if check_every:
            _state_eq(eng, orc, range(ns))
    _state_eq(eng, orc, range(ns))
    return eng, orc, fc, fb


class _Fuzz:
    """Small books with few levels, so FIFOs are consumed, cancelled and refilled within and
    across batches.  DELs re-send earlier ADDs (any batch), some before their ADD, some with
    the wrong price (Q3), a few twice; takers sweep several levels."""

    def __init__(self, seed, ns=2, nprice=6, vmax=9, p_del=0.35, p_aggr=0.08, p_q3=0.03,
                 p_early=0.02, p_dup=0.0, p_q2=0.0):
        self.rng = np.random.default_rng(seed)
        self.ns, self.nprice, self.vmax = ns, nprice, vmax
        self.p_del, self.p_aggr, self.p_q3, self.p_early, self.p_dup, self.p_q2 = \
            p_del, p_aggr, p_q3, p_early, p_dup, p_q2
        self.adds: list[tuple] = []   # (price, vol, sym, oid, uuid, side) of every ADD sent
        self.untargeted: list[int] = []
        self.oid = 1

    def _add(self, out, i):
        rng = self.rng
        sym = int(rng.integers(self.ns))
        side = int(rng.integers(2))
        if rng.random() < self.p_aggr:
            price = 50 + self.nprice if side == 0 else 50 - self.nprice  # sweeps the other side
            vol = int(rng.integers(10, 40))
        else:
            price = 50 + (int(rng.integers(1, self.nprice + 1)) if side == 1 else -int(rng.integers(0, self.nprice)))
            vol = int(rng.integers(1, self.vmax + 1))
        t = (price * 10**6, vol * 10**6, sym, self.oid, 7, side)
        self.oid += 1
        self.adds.append(t)
        self.untargeted.append(len(self.adds) - 1)
        out[i] = (*t, ADD, 0)

    def batch(self, n):
        rng = self.rng
        out = np.zeros(n, wl.ORDER_DTYPE)
        i = 0
        while i < n:
            u = rng.random()
            if u < self.p_del and self.untargeted:
                j = int(rng.integers(len(self.untargeted)))
                k = self.untargeted[j]
                if rng.random() >= self.p_dup:
                    self.untargeted[j] = self.untargeted[-1]
                    self.untargeted.pop()
                p, v, s, o, uu, sd = self.adds[k]
                if rng.random() < self.p_q3:
                    p += 10**6
                if rng.random() < self.p_q2:
                    sd = 1 - sd
                out[i] = (p, v, s, o, uu, sd, DEL, 0)
                i += 1
            elif u < self.p_del + self.p_early and i + 1 < n:
                # a DEL that overtakes its ADD: finds nothing (engine.go:96-98), the ADD rests
                self._add(out, i + 1)
                out[i] = out[i + 1]
                out[i]["action"] = DEL
                i += 2
            else:
                self._add(out, i)
                i += 1
        return out


@pytest.mark.parametrize("seed", range(6))
def test_flow_cancel_fuzz_small_books(seed):
    fz = _Fuzz(100 + seed, ns=2, p_dup=0.04 * (seed % 2))
    batches = [fz.batch(int(n)) for n in np.random.default_rng(seed).integers(300, 3000, 8)]
    eng, orc, fc, fb = _run(batches, 2)
    assert fc > 100, "cancels did not take the flow path; " + _routes_msg()


@pytest.mark.parametrize("seed", range(3))
def test_flow_cancel_fuzz_tail_books(seed):
    """40 symbols: 8 head books (tile-parallel prep) and 32 tail books (one prep block per
    book)."""
    fz = _Fuzz(200 + seed, ns=40, nprice=5)
    batches = [fz.batch(20000) for _ in range(4)]
    eng, orc, fc, fb = _run(batches, 40, check_every=False)
    assert fc > 1000 and fb >= 4 * 30, _routes_msg()


def test_flow_cancel_quirks_decline_exactly():
    """Repeated DELs (the first that can find the maker applies, later ones find nothing) and
    Q2 wrong-side DELs (such books go back to the legacy kernel): exact either way."""
    fz = _Fuzz(7, ns=6, p_dup=0.02, p_q2=0.01)
    batches = [fz.batch(6000) for _ in range(5)]
    _run(batches, 6)


def test_flow_cancel_config4_mix_vs_legacy():
    """The config-4 mix through the flow path and through the legacy FIFO kernel."""
    from gome_amd.abi import GOME_FLAG_LEGACY_HOT
    rec = wl.cancel_mix(120000, 20, seed=4, zipf_s=1.0)
    a = _engine(20, 40000)
    b = _engine(20, 40000, GOME_FLAG_LEGACY_HOT)
    fc = 0
    for bt in wl.split_batches(rec, 40000):
        a.submit(bt)
        b.submit(bt)
        _cmp(a.drain(), b.drain(), "flow vs legacy")
        fc += a.stats()["n_flow_cancels"]
        assert b.stats()["n_flow_books"] == 0
    assert fc > 10000
    for s in range(20):
        assert np.array_equal(a.levels(s), b.levels(s))
        for p in b.levels(s)["price_fx"]:
            assert np.array_equal(a.fifo(s, int(p)), b.fifo(s, int(p)))


def _recs(rows):
    r = np.zeros(len(rows), wl.ORDER_DTYPE)
    for i, x in enumerate(rows):
        r[i] = x
    return r


def test_flow_cancel_long_windows():
    """300 makers at one level, each cancelled later in the batch in arrival order: windows of
    up to 299 targets (the prep's C loop over them), takers in between."""
    rows, oid = [], 1
    for k in range(300):
        rows.append((51 * 10**6, (1 + k % 7) * 10**6, 0, oid, 3, 1, ADD, 0))
        oid += 1
    pad = [(50 * 10**6, 10**6, 0, 10000 + k, 3, 0, ADD, 0) for k in range(40)]   # bids below
    dels, t = [], 0
    for k in range(300):
        dels.append((51 * 10**6, (1 + k % 7) * 10**6, 0, k + 1, 3, 1, DEL, 0))
        if k % 37 == 5:
            dels.append((51 * 10**6, 3 * 10**6, 0, 20000 + t, 3, 0, ADD, 0))   # a taker
            t += 1
    _, _, fc, fb = _run([_recs(rows + pad + dels)], 1)
    assert fc > 250 and fb == 1


def test_flow_cancel_empties_levels_then_sweeps():
    """Cancels empty the best level (the plan's cached top moves on) and a level behind it
    (it leaves the side set); a taker then sweeps through what is left.  Old makers from the
    previous batch are cancelled at every FIFO position, partly consumed ones included."""
    rows, oid = [], 1
    for p in (51, 52, 53, 54):
        for k in range(6):
            rows.append((p * 10**6, (2 + k) * 10**6, 0, oid, 4, 1, ADD, 0))
            oid += 1
    rows += [(40 * 10**6, 10**6, 0, 900 + k, 4, 0, ADD, 0) for k in range(130)]
    b1 = _recs(rows)
    # batch 2: partial consumption of 51, cancels of 51's makers (head partly consumed, middle,
    # tail), all of 53's makers, then a sweep to 54
    b2 = [(51 * 10**6, 3 * 10**6, 0, 5000, 4, 0, ADD, 0)]            # consumes 3 of maker 1 (2+1)
    b2 += [(51 * 10**6, 0, 0, o, 4, 1, DEL, 0) for o in (2, 1, 6)]
    b2 += [(53 * 10**6, 0, 0, o, 4, 1, DEL, 0) for o in range(13, 19)]
    b2 += [(54 * 10**6, 60 * 10**6, 0, 5001, 4, 0, ADD, 0)]           # sweep 51 .. 54
    b2 += [(54 * 10**6, 0, 0, o, 4, 1, DEL, 0) for o in (19, 24)]
    b2 += [(40 * 10**6, 10**6, 0, 6000 + k, 4, 0, ADD, 0) for k in range(130)]
    _, _, fc, fb = _run([b1, _recs(b2)], 1)
    assert fc > 0 and fb == 2


def test_flow_cancel_new_makers_same_batch():
    """DELs of makers that rested earlier in the same batch: untouched, partly consumed, fully
    consumed (no-op), an ADD that never rested (no-op), and a DEL of a cancelled order."""
    P = 10**6
    b = [(60 * P, 5 * P, 0, 1, 2, 1, ADD, 0),        # maker 1
         (60 * P, 4 * P, 0, 2, 2, 1, ADD, 0),        # maker 2
         (60 * P, 3 * P, 0, 3, 2, 1, ADD, 0),        # maker 3
         (60 * P, 7 * P, 0, 10, 2, 0, ADD, 0),       # taker: 5 from 1, 2 from 2
         (60 * P, 0, 0, 2, 2, 1, DEL, 0),            # partly consumed: cancels 2
         (60 * P, 0, 0, 1, 2, 1, DEL, 0),            # fully consumed: no-op
         (60 * P, 2 * P, 0, 11, 2, 0, ADD, 0),       # taker: 2 from 3
         (60 * P, 0, 0, 10, 2, 0, DEL, 0),           # the first taker never rested: no-op
         (60 * P, 0, 0, 3, 2, 1, DEL, 0),            # cancels 1 of 3
         (60 * P, 0, 0, 3, 2, 1, DEL, 0)]            # again: finds nothing
    b += [(30 * P, P, 0, 100 + k, 2, 0, ADD, 0) for k in range(130)]
    c = b[:-131] + b[-130:]                          # without the repeated DEL
    for rows in (c, b):
        _, _, fc, fb = _run([_recs(rows)], 1)
        assert fc == 2 and fb == 1


def test_flow_cancel_generation_wrap():
    """2100 small batches: the (symbol, oid) table's generation tag wraps (cleared every 2048
    batches) without stale entries."""
    fz = _Fuzz(31, ns=1, nprice=3)
    eng = _engine(1, 256)
    orc = Oracle(1)
    for i in range(2100):
        b = fz.batch(160)
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"batch {i}")
    _state_eq(eng, orc, [0])


def test_flow_cancel_long_windows_two_levels():
    """Two levels of 4200 targets each, cancelled in arrival order (DEL windows of up to 4199
    targets, ~15M window entries for the prep's C loops): the book stays on the flow path (no
    FC_BAD_RING decline) and is exact."""
    P = 10**6
    rows, oid = [], 1
    for p in (61, 62):
        for k in range(4200):
            rows.append((p * P, (1 + k % 5) * P, 0, oid, 3, 1, ADD, 0))
            oid += 1
    rows += [(40 * P, P, 0, 90000 + k, 3, 0, ADD, 0) for k in range(200)]   # bids below
    # every maker is a target (a ring counts targets): the first DEL of each level has a
    # window of 4199 targets (C_k = 8192); a taker between them
    rows += [(61 * P, 0, 0, o, 3, 1, DEL, 0) for o in range(1, 2001)]
    rows.append((61 * P, 7 * P, 0, 99000, 3, 0, ADD, 0))
    rows += [(62 * P, 0, 0, o, 3, 1, DEL, 0) for o in range(4201, 8401, 2)]
    rows += [(61 * P, 0, 0, o, 3, 1, DEL, 0) for o in range(2001, 4201)]
    rows.append((62 * P, 9000 * P, 0, 99001, 3, 0, ADD, 0))                 # sweeps both levels
    _, _, fc, fb = _run([_recs(rows)], 1)
    fbk = ROUTES[-1][1]
    assert int(fbk["decline"][0]) == 0 and int(fbk["window"][0]) > 4000, _routes_msg()
    assert fb == 1 and fc > 2000


@pytest.mark.parametrize("seed", range(4))
def test_flow_cancel_fuzz_wide_books(seed):
    """Wider books (up to 80 levels), heavier sweeps and more cancels: DEL targets deep in the
    FIFO, at the cached top, partly consumed heads, old makers several batches old, and levels
    that change side between a maker's rest and its cancel (the Q plan's dead-target case)."""
    fz = _Fuzz(300 + seed, ns=3, nprice=40, vmax=30, p_del=0.45, p_aggr=0.15, p_q3=0.02, p_early=0.02)
    batches = [fz.batch(int(n)) for n in np.random.default_rng(50 + seed).integers(4000, 16000, 6)]
    eng, orc, fc, fb = _run(batches, 3)
    assert fc > 3000, "cancels did not take the flow path; " + _routes_msg()


def test_flow_cancel_fuzz_many_tail_books():
    """200 symbols of a few hundred orders each per batch (all tail books, one prep block per
    book), 10-level books with sweeps and cancels."""
    fz = _Fuzz(400, ns=200, nprice=10, vmax=12, p_del=0.4, p_aggr=0.1)
    batches = [fz.batch(60000) for _ in range(3)]
    eng, orc, fc, fb = _run(batches, 200, check_every=False)
    assert fc > 10000 and fb >= 3 * 150, _routes_msg()
