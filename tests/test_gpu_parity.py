"""HIP engine parity (MI355X): events bit-exact vs the C oracle, MatchResult JSON
byte-exact vs the literal transliteration, book state equal, on every config shape.
All calls go through the C-ABI (libgome.so); there is no CPU fallback."""
import numpy as np
import pytest

from gome_amd import workload as wl
from gome_amd.abi import Engine, GomeError, GOME_E_INVAL
from oracle.literal import run_batches
from oracle.pyoracle import Oracle
from tests.helpers import (Interner, engine_state_to_levels, literal_state_to_levels,
                           random_batches, render_events, requests_to_records)

pytestmark = pytest.mark.gpu


def _engine(max_symbols, max_batch, max_nodes=1 << 20, max_levels=1 << 20):
    return Engine(max_symbols=max_symbols, max_batch=max_batch, max_nodes=max_nodes,
                  max_levels=max_levels)


def _cmp_events(got: np.ndarray, exp: np.ndarray, tag=""):
    assert len(got) == len(exp), f"{tag}: {len(got)} events vs oracle {len(exp)}"
    if len(got) and not np.array_equal(got, exp):
        bad = np.nonzero(got != exp)[0][0]
        raise AssertionError(f"{tag}: first mismatch at event {bad}:\n gpu={got[bad]}\n orc={exp[bad]}")


def _run_pair(batches, max_symbols, sample_syms=(), **kw):
    eng = _engine(max_symbols, max(len(b) for b in batches), **kw)
    orc = Oracle(max_symbols)
    for i, b in enumerate(batches):
        eng.submit(b)
        got = eng.drain()
        exp = orc.submit(b)
        _cmp_events(got, exp, f"batch {i}")
    for s in sample_syms:
        lv_g, lv_o = eng.levels(s), orc.levels(s)
        assert np.array_equal(lv_g, lv_o), f"levels of symbol {s}"
        for p in lv_o["price_fx"]:
            assert np.array_equal(eng.fifo(s, int(p)), orc.fifo(s, int(p))), f"fifo {s}@{p}"
    st = eng.stats()
    assert st["n_resting"] == orc.resting()
    return eng, orc


@pytest.mark.parametrize("seed", range(12))
def test_quirk_streams_vs_literal(seed):
    """Randomized Appendix-A quirk streams: rendered JSON == literal transliteration."""
    symbols = ("eth2usdt", "btc2usdt", "ltc2usdt")
    rng = np.random.default_rng(7000 + seed)
    batches = random_batches(rng, n_batches=5, batch=80, symbols=symbols,
                             del_frac=0.1 + 0.15 * (seed % 4))
    leng, lit = run_batches(batches)
    names = Interner()
    for s in symbols:
        names.id("sym", s)
    eng = _engine(len(symbols), 256)
    got = []
    for b in batches:
        rec = requests_to_records(b, names)
        eng.submit(rec)
        got += render_events(eng.drain(), rec, names)
    assert got == lit
    for s in symbols:
        assert engine_state_to_levels(eng, names.id("sym", s), names) == \
            literal_state_to_levels(leng.book_state(s))


def test_config1_single_symbol():
    st = wl.Stream(1, seed=42)
    batches = [st.batch(20000) for _ in range(5)]
    _run_pair(batches, 1, sample_syms=[0])


def test_config2_uniform_1k():
    st = wl.Stream(1000, seed=42)
    batches = [st.batch(200000) for _ in range(3)]
    _run_pair(batches, 1000, sample_syms=[0, 1, 500, 999])


def test_config3_zipf_100k():
    st = wl.Stream(100000, zipf_s=1.0, seed=42)
    z = st.zipf
    batches = [st.batch(1 << 19) for _ in range(3)]
    hot = [int(z.rank_to_id[r]) for r in (0, 1, 2, 50, 5000)]
    _run_pair(batches, 100000, sample_syms=hot, max_nodes=1 << 21, max_levels=1 << 23)


def test_config4_cancel_mix():
    rec = wl.cancel_mix(300000, 200, seed=42)
    _run_pair(wl.split_batches(rec, 50000), 200, sample_syms=[0, 7, 199])


def test_config4_cancel_mix_zipf_hot():
    rec = wl.cancel_mix(200000, 1000, seed=3, zipf_s=1.0)
    _run_pair(wl.split_batches(rec, 65536), 1000, sample_syms=list(range(0, 1000, 97)))


def test_config5_deep_books():
    """4-dp price grid -> up to 10k levels per book (level arrays far beyond 64 lanes)."""
    st = wl.Stream(64, seed=5, price_decimals=4)
    batches = [st.batch(100000) for _ in range(3)]
    eng, orc = _run_pair(batches, 64, sample_syms=[0, 13, 63])
    assert max(len(orc.levels(s)) for s in range(64)) > 1000


def test_tiny_batches_and_many_batches():
    rng = np.random.default_rng(11)
    batches = random_batches(rng, n_batches=40, batch=7, symbols=("a", "b"), del_frac=0.35)
    names = Interner()
    recs = [requests_to_records(b, names) for b in batches]
    _run_pair(recs, 2, sample_syms=[0, 1])


def test_invalid_batch_rejected_without_state_change():
    st = wl.Stream(4, seed=1)
    good = st.batch(1000)
    eng = _engine(4, 2048)
    orc = Oracle(4)
    eng.submit(good)
    _cmp_events(eng.drain(), orc.submit(good))
    bad = st.batch(10)
    bad[3]["symbol_id"] = 99  # out of range
    with pytest.raises(GomeError) as ei:
        eng.submit(bad)
    assert ei.value.status == GOME_E_INVAL
    bad2 = st.batch(10)
    bad2[0]["volume_fx"] = -5
    with pytest.raises(GomeError):
        eng.submit(bad2)
    nxt = st.batch(1000)
    eng.submit(nxt)
    _cmp_events(eng.drain(), orc.submit(nxt))
    for s in range(4):
        assert np.array_equal(eng.levels(s), orc.levels(s))


def test_empty_batch():
    eng = _engine(2, 16)
    eng.submit(np.zeros(0, wl.ORDER_DTYPE))
    assert len(eng.drain()) == 0


def test_device_submit_and_events():
    """gome_submit_batch_device: records already resident in HBM; events stay on device."""
    torch = pytest.importorskip("torch")
    st = wl.Stream(100, seed=9)
    b = st.batch(50000)
    eng = _engine(100, 65536)
    orc = Oracle(100)
    t = torch.from_numpy(b.view(np.uint8).copy()).cuda()
    torch.cuda.synchronize()
    eng.submit_device(t.data_ptr(), len(b))
    ptr, n = eng.device_events()
    exp = orc.submit(b)
    assert ptr and n == len(exp)
    _cmp_events(eng.drain(), exp)


# ---- hot books (segments >= 2048 orders take the LDS-resident k_match_hot path) -------
def test_hot_book_quirks_vs_literal():
    """One symbol, 2500-order batches (hot path) with every Appendix-A quirk."""
    rng = np.random.default_rng(4242)
    batches = random_batches(rng, n_batches=3, batch=2500, symbols=("eth2usdt",), del_frac=0.3)
    leng, lit = run_batches(batches)
    names = Interner()
    names.id("sym", "eth2usdt")
    eng = _engine(1, 8192)
    got = []
    for b in batches:
        rec = requests_to_records(b, names)
        eng.submit(rec)
        assert eng.stats()["n_hot"] == 1
        got += render_events(eng.drain(), rec, names)
    assert got == lit
    assert engine_state_to_levels(eng, 0, names) == literal_state_to_levels(leng.book_state("eth2usdt"))


def test_hot_books_cancel_heavy():
    """Config-4 mix on 4 symbols: every book is hot, half the stream cancels."""
    rec = wl.cancel_mix(200000, 4, seed=17)
    eng, orc = _run_pair(wl.split_batches(rec, 40000), 4, sample_syms=[0, 1, 2, 3])
    assert eng.stats()["n_hot"] == 4


def test_hot_and_cold_mixed_zipf_cancels():
    rec = wl.cancel_mix(400000, 500, seed=23, zipf_s=1.2)
    eng, orc = _run_pair(wl.split_batches(rec, 100000), 500, sample_syms=list(range(0, 500, 37)))
    assert eng.stats()["n_hot"] >= 1


def test_hot_book_spills_to_hbm():
    """4-dp prices on 2 symbols: a hot book outgrows the LDS level array mid-segment
    (spill to the HBM path), later batches start on the HBM path."""
    st = wl.Stream(2, seed=31, price_decimals=4)
    batches = [st.batch(24000) for _ in range(3)]
    eng, orc = _run_pair(batches, 2, sample_syms=[0, 1])
    assert len(orc.levels(0)) > 1024


def test_hot_book_long_fifo_chunk_chains():
    """Few price points, many resting orders per level: FIFOs span many chunks and the
    head advances across chunk boundaries (cached head reloads, NextNode lookahead)."""
    rng = np.random.default_rng(5)
    n = 60000
    rec = np.zeros(n, wl.ORDER_DTYPE)
    rec["symbol_id"] = 0
    rec["side"] = rng.integers(0, 2, n)
    rec["price_fx"] = np.where(rec["side"] == 0, 49, 51) * 10**6
    big = rng.random(n) < 0.05  # occasional aggressive orders sweeping several levels
    rec["price_fx"][big & (rec["side"] == 0)] = 60 * 10**6
    rec["price_fx"][big & (rec["side"] == 1)] = 40 * 10**6
    rec["volume_fx"] = rng.integers(1, 20, n) * 10**6
    rec["volume_fx"][big] = rng.integers(50, 400, big.sum()) * 10**6
    rec["action"] = 1
    rec["uuid_id"] = 2
    rec["oid_id"] = np.arange(1, n + 1)
    _run_pair(wl.split_batches(rec, 20000), 1, sample_syms=[0])


# ---- golden fixtures (generated by the literal transliteration) --------------------------
from tests.helpers import golden_names, load_golden, replay_fixture  # noqa: E402


class _EngineBackend:
    def __init__(self, ns, mb):
        self.e = _engine(ns, max(mb, 16))

    def submit(self, rec):
        self.e.submit(rec)
        return self.e.drain()

    def levels(self, s):
        return self.e.levels(s)

    def fifo(self, s, p):
        return self.e.fifo(s, p)


_GOLDEN = [fx for n in golden_names() for fx in load_golden(n)]


@pytest.mark.parametrize("fx", _GOLDEN, ids=[fx["name"] for fx in _GOLDEN])
def test_engine_reproduces_golden(fx):
    out, state = replay_fixture(fx, _EngineBackend)
    assert out == fx["results"]
    assert state == fx["state"]


# ---- flow path (match_flow.h): hot ADD-only books via the serial aggregate plan ----------
def _engine_flags(max_symbols, max_batch, flags, max_nodes=1 << 20, max_levels=1 << 20):
    return Engine(max_symbols=max_symbols, max_batch=max_batch, max_nodes=max_nodes,
                  max_levels=max_levels, flags=flags)


def test_flow_path_taken_and_exact_single_symbol():
    st = wl.Stream(1, seed=77)
    batches = [st.batch(30000) for _ in range(4)]
    eng, orc = _run_pair(batches, 1, sample_syms=[0])
    s = eng.stats()
    assert s["n_flow_books"] == 1 and s["n_flow_orders"] == 30000
    assert s["n_flow_touches"] >= 30000


def test_flow_zipf_hot_books_with_fifo_state():
    st = wl.Stream(2000, zipf_s=1.1, seed=8)
    z = st.zipf
    batches = [st.batch(1 << 18) for _ in range(3)]
    hot = [int(z.rank_to_id[r]) for r in (0, 1, 2, 3, 10, 40, 300)]
    eng, orc = _run_pair(batches, 2000, sample_syms=hot)
    assert eng.stats()["n_flow_books"] >= 4


def test_flow_equals_legacy_hot_kernel():
    """The same stream through the flow path and the legacy FIFO kernel: identical events
    and identical book state (FIFOs included)."""
    from gome_amd.abi import GOME_FLAG_LEGACY_HOT
    st = wl.Stream(3, seed=19)
    batches = [st.batch(12000) for _ in range(4)]
    a = _engine_flags(3, 12000, 0)
    b = _engine_flags(3, 12000, GOME_FLAG_LEGACY_HOT)
    for bt in batches:
        a.submit(bt)
        b.submit(bt)
        _cmp_events(a.drain(), b.drain(), "flow vs legacy")
        assert a.stats()["n_flow_books"] == 3 and b.stats()["n_flow_books"] == 0
    for s in range(3):
        assert np.array_equal(a.levels(s), b.levels(s))
        for p in b.levels(s)["price_fx"]:
            assert np.array_equal(a.fifo(s, int(p)), b.fifo(s, int(p)))


def test_flow_then_cancels_then_flow():
    """Book state handed between batches: ADD-only batches, a cancel-heavy batch (cancels of
    makers at every FIFO position, on the flow path's cancel plan), then ADD-only again."""
    rng = np.random.default_rng(99)
    st = wl.Stream(2, seed=99)
    adds1 = [st.batch(8000) for _ in range(2)]
    eng = _engine(2, 16000)
    orc = Oracle(2)
    for b in adds1:
        eng.submit(b)
        _cmp_events(eng.drain(), orc.submit(b), "adds1")
        assert eng.stats()["n_flow_books"] == 2
    # cancel half of the resting book (correct sides/prices), plus new adds
    resting = []
    for s in range(2):
        for lv in orc.levels(s):
            for nd in orc.fifo(s, int(lv["price_fx"])):
                resting.append((s, int(lv["price_fx"]), int(nd["oid_id"]), int(nd["uuid_id"]), int(nd["side"])))
    rng.shuffle(resting)
    dels = np.zeros(len(resting) // 2, wl.ORDER_DTYPE)
    for i, (s, p, o, u, sd) in enumerate(resting[: len(dels)]):
        dels[i] = (p, 10**6, s, o, u, sd, 2, 0)
    mix = np.concatenate([dels, st.batch(4000)])
    eng.submit(mix)
    _cmp_events(eng.drain(), orc.submit(mix), "cancel batch")
    assert eng.stats()["n_flow_books"] == 2 and eng.stats()["n_flow_cancels"] > 1000
    for b in [st.batch(8000) for _ in range(2)]:
        eng.submit(b)
        _cmp_events(eng.drain(), orc.submit(b), "adds2")
        assert eng.stats()["n_flow_books"] == 2
    for s in range(2):
        assert np.array_equal(eng.levels(s), orc.levels(s))
        for p in orc.levels(s)["price_fx"]:
            assert np.array_equal(eng.fifo(s, int(p)), orc.fifo(s, int(p)))


def test_flow_declines_quirky_book():
    """A quirk state that never heals keeps the book on the legacy kernel (the aggregate plan
    cannot express it): a wrong-side cancel (Q2) of the lowest level's first maker, plus a
    zero-volume BUY (Q6) resting on a new level below every price the stream uses (never reached
    again).  A Q2 alone that leaves the level with makers is no quirk at all: the book is back
    on the flow path after the batch (match_requal.h)."""
    st = wl.Stream(1, seed=5)
    eng = _engine(1, 8192)
    orc = Oracle(1)
    b = st.batch(4000)
    eng.submit(b)
    _cmp_events(eng.drain(), orc.submit(b))
    lv = orc.levels(0)[0]
    nd = orc.fifo(0, int(lv["price_fx"]))[0]
    q2 = np.zeros(2, wl.ORDER_DTYPE)
    q2[0] = (int(lv["price_fx"]), 10**6, 0, int(nd["oid_id"]), int(nd["uuid_id"]), 1 - int(nd["side"]), 2, 0)
    q2[1] = (10**5, 0, 0, 4_000_000_000, 1, 0, 1, 0)  # zero-volume BUY at 0.001
    eng.submit(q2)
    _cmp_events(eng.drain(), orc.submit(q2))
    for _ in range(2):
        b = st.batch(4000)
        eng.submit(b)
        _cmp_events(eng.drain(), orc.submit(b))
        assert eng.stats()["n_flow_books"] == 0 and eng.stats()["n_quirk_checked"] == 1
        assert eng.stats()["n_requalified"] == 0
    assert np.array_equal(eng.levels(0), orc.levels(0))


def test_flow_sweeps_and_long_chains_vs_legacy_counts():
    """Aggressive sweeps over few levels with deep FIFOs (many chunks consumed per batch)."""
    rng = np.random.default_rng(12)
    n = 90000
    rec = np.zeros(n, wl.ORDER_DTYPE)
    rec["symbol_id"] = 0
    rec["side"] = rng.integers(0, 2, n)
    base = np.where(rec["side"] == 0, rng.integers(40, 50, n), rng.integers(51, 61, n))
    big = rng.random(n) < 0.08
    base[big & (rec["side"] == 0)] = 70
    base[big & (rec["side"] == 1)] = 30
    rec["price_fx"] = base * 10**6
    rec["volume_fx"] = rng.integers(1, 30, n) * 10**6
    rec["volume_fx"][big] = rng.integers(100, 3000, big.sum()) * 10**6
    rec["action"] = 1
    rec["uuid_id"] = 3
    rec["oid_id"] = np.arange(1, n + 1)
    eng, orc = _run_pair(wl.split_batches(rec, 30000), 1, sample_syms=[0])
    assert eng.stats()["n_flow_books"] == 1


def test_flow_dropped_and_ignored_records():
    """Q4 duplicate ADD keys (later ones dropped) and unknown actions inside an ADD-only hot
    book: they reach the plan as no-op records; events, state and n_flow_books as expected."""
    rng = np.random.default_rng(2024)
    st = wl.Stream(2, seed=2024)
    eng = _engine(2, 20000)
    orc = Oracle(2)
    for _ in range(3):
        b = st.batch(12000)
        dup = rng.choice(len(b), 300, replace=False)
        extra = b[dup].copy()                       # same (S, uuid, oid): admission drops them
        extra["volume_fx"] = 10**6
        ign = b[rng.choice(len(b), 200, replace=False)].copy()
        ign["action"] = 7                           # consumed and ignored (engine.go:46-54)
        mix = np.concatenate([b, extra, ign])
        mix = mix[rng.permutation(len(mix))]
        eng.submit(mix)
        _cmp_events(eng.drain(), orc.submit(mix), "dropped/ignored")
        s = eng.stats()
        assert s["n_flow_books"] == 2 and s["n_dropped"] > 0
    for s_ in range(2):
        assert np.array_equal(eng.levels(s_), orc.levels(s_))
        for p in orc.levels(s_)["price_fx"]:
            assert np.array_equal(eng.fifo(s_, int(p)), orc.fifo(s_, int(p)))


@pytest.mark.parametrize("vmax", [2**20, 2**45])
def test_flow_plan_widths(vmax):
    """Volumes with gcd 1: small ones take the 32-bit plan, volumes up to 2^45 (sum/gcd beyond
    2^32) the 64-bit plan.  Both exact against the oracle, FIFOs included."""
    rng = np.random.default_rng(vmax % 1000003)
    n = 24000
    rec = np.zeros(n, wl.ORDER_DTYPE)
    rec["symbol_id"] = rng.integers(0, 2, n)
    rec["side"] = rng.integers(0, 2, n)
    rec["price_fx"] = rng.integers(1, 90, n) * 10**6
    rec["volume_fx"] = rng.integers(1, vmax, n)
    rec["action"] = 1
    rec["uuid_id"] = 5
    rec["oid_id"] = np.arange(1, n + 1)
    eng, orc = _run_pair(wl.split_batches(rec, 8000), 2, sample_syms=[0, 1])
    assert eng.stats()["n_flow_books"] == 2


# ---- plan-loop edge cases (gen_plan_asm.py): half-group padding, staging flushes inside
#      sweeps, sentinel tops, the level cap, and both plan widths on each

def _book(prices, vols, sides, sym=0, oid0=1, uuid=9):
    n = len(prices)
    r = np.zeros(n, wl.ORDER_DTYPE)
    r["symbol_id"] = sym
    r["price_fx"] = np.asarray(prices, np.int64) * 10**6
    r["volume_fx"] = np.asarray(vols, np.int64)
    r["side"] = sides
    r["action"] = 1
    r["uuid_id"] = uuid
    r["oid_id"] = np.arange(oid0, oid0 + n)
    return r


@pytest.mark.gpu
def test_flow_half_group_padding_residues():
    """Books of 128..135 orders (every residue mod the 8-record half-group) and a few odd sizes,
    one batch each on the same book: exact events, levels and FIFOs after every batch."""
    rng = np.random.default_rng(31)
    batches, oid = [], 1
    for n in list(range(128, 136)) + [999, 1001, 2047]:
        b = _book(rng.integers(30, 71, n), rng.integers(1, 40, n) * 10**6, rng.integers(0, 2, n), oid0=oid)
        oid += n
        batches.append(b)
    eng, orc = _engine(1, 4096), Oracle(1)
    for i, b in enumerate(batches):
        eng.submit(b)
        _cmp_events(eng.drain(), orc.submit(b), f"batch {i} ({len(b)} orders)")
        assert eng.stats()["n_flow_books"] == 1, f"batch {i} not on the flow path"
        assert np.array_equal(eng.levels(0), orc.levels(0)), f"levels after batch {i}"


@pytest.mark.gpu
@pytest.mark.parametrize("unit", [10**6, (1 << 34) + 1])
def test_flow_staging_stress_sweeps(unit):
    """Rounds of 8 small makers on consecutive levels followed by one taker that empties them
    (exact fill or a partial at the last level): 8 level-emptying touches inside one order,
    rounds of 9 orders straddling the 8-record half-groups, so the touch staging is flushed
    inside sweeps.  unit 1e6 runs the 32-bit plan, (2^34 + 1) the 64-bit one."""
    rng = np.random.default_rng(77 if unit == 10**6 else 78)
    prices, vols, sides = [], [], []
    for r in range(2400):
        sell = r % 2 == 0                      # makers' side alternates per round
        lv = np.arange(51, 59) if sell else np.arange(49, 41, -1)
        v = rng.integers(1, 4, 8)
        prices += list(lv)
        vols += list(v)
        sides += [1 if sell else 0] * 8
        prices.append(58 if sell else 42)
        vols.append(int(v.sum()) - int(rng.integers(0, 2)))
        sides.append(0 if sell else 1)
    rec = _book(prices, np.asarray(vols, np.int64) * unit, np.asarray(sides, np.uint8))
    eng, orc = _run_pair(wl.split_batches(rec, 7200), 1, sample_syms=[0])
    s = eng.stats()
    assert s["n_flow_books"] == 1 and s["n_flow_touches"] > 1.7 * s["n_flow_orders"]


@pytest.mark.gpu
def test_flow_one_sided_books_and_sentinel_tops():
    """Symbol 0 sees only BUYs, symbol 1 only SELLs (the opposite top stays at its sentinel
    level); then a batch sweeps each side empty and rests behind the sentinels."""
    rng = np.random.default_rng(5)
    n = 3000
    b0 = _book(rng.integers(10, 60, n), rng.integers(1, 9, n) * 10**6, np.zeros(n, np.uint8), sym=0, oid0=1)
    b1 = _book(rng.integers(40, 90, n), rng.integers(1, 9, n) * 10**6, np.ones(n, np.uint8), sym=1, oid0=1)
    first = np.concatenate([b0, b1])
    tot0, tot1 = int(b0["volume_fx"].sum()), int(b1["volume_fx"].sum())
    # 200 SELLs at the lowest price take every bid of symbol 0, then rest; mirrored for 1
    s0 = _book([1] * 200, [tot0 // 100] * 200, np.ones(200, np.uint8), sym=0, oid0=10**6)
    s1 = _book([99] * 200, [tot1 // 100] * 200, np.zeros(200, np.uint8), sym=1, oid0=10**6)
    second = np.concatenate([s0, s1])
    eng, orc = _run_pair([first, second, first.copy()], 2, sample_syms=[0, 1])
    assert eng.stats()["n_flow_books"] == 2


@pytest.mark.gpu
def test_flow_one_order_sweeps_every_level():
    """100 ask levels, then one BUY that takes all of them (one order logs more touches than the
    staging holds) and rests the remainder; mirrored on the bid side in the next batch."""
    rng = np.random.default_rng(9)
    k = np.repeat(np.arange(2, 102), 3)
    asks = _book(k, rng.integers(1, 5, len(k)) * 10**6, np.ones(len(k), np.uint8), oid0=1)
    big = _book([105], [int(asks["volume_fx"].sum()) + 7 * 10**6], [0], oid0=9000)
    filler = _book(rng.integers(110, 121, 150), [10**6] * 150, np.ones(150, np.uint8), oid0=10000)
    b1 = np.concatenate([asks, big, filler])
    bids = _book(k, rng.integers(1, 5, len(k)) * 10**6, np.zeros(len(k), np.uint8), oid0=20000)
    big2 = _book([1], [int(bids["volume_fx"].sum()) + 7 * 10**6 + 10**8], [1], oid0=30000)
    b2 = np.concatenate([bids, big2, _book([50] * 150, [10**6] * 150, np.zeros(150, np.uint8), oid0=40000)])
    eng, orc = _engine(1, 1024), Oracle(1)
    for i, b in enumerate((b1, b2)):
        eng.submit(b)
        _cmp_events(eng.drain(), orc.submit(b), f"batch {i}")
        st = eng.stats()
        assert st["n_flow_books"] == 1 and st["max_segment"] == len(b)
        assert np.array_equal(eng.levels(0), orc.levels(0))
        for p in orc.levels(0)["price_fx"]:
            assert np.array_equal(eng.fifo(0, int(p)), orc.fifo(0, int(p)))


@pytest.mark.gpu
@pytest.mark.parametrize("nlev", [126, 127])
def test_flow_level_cap(nlev):
    """A batch whose book reaches exactly 126 distinct prices runs on the lane plan; 127 takes
    the deep plan (match_flow_deep.h).  Both exact."""
    rng = np.random.default_rng(nlev)
    n = 4000
    prices = np.concatenate([np.arange(1, nlev + 1), rng.integers(1, nlev + 1, n - nlev)])
    rec = _book(prices, rng.integers(1, 20, n) * 10**6, rng.integers(0, 2, n))
    eng, orc = _run_pair([rec], 1, sample_syms=[0])
    assert eng.stats()["n_flow_books"] == 1
    assert int(eng.debug_flow_books()["kind"][0]) == (1 if nlev == 126 else 3)
