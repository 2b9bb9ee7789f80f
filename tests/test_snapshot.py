"""Checkpoint / resume in the reference's Redis key schema (gome_amd/snapshot.py, SURVEY §5 and
§8f rank 2).  The checker is the literal transliteration (oracle/literal.py), whose FakeRedis
holds exactly the keys the reference would hold after the same request stream."""
import numpy as np
import pytest

from gome_amd import snapshot
from gome_amd.abi import Engine, GomeError, render_link_node
from oracle.literal import NewOrderNode, run_batches
from tests.helpers import Interner, random_batches, render_events, requests_to_records

SYMBOLS = ("eth2usdt", "btc2usdt", "ltc2usdt")


def test_link_node_json_matches_literal():
    """Resting node JSON (SetLinkNode) byte-identical to the literal's encoding/json."""
    rng = np.random.default_rng(3)
    for i in range(300):
        S = str(rng.choice(SYMBOLS))
        req = dict(uuid=f"u{int(rng.integers(9))}", oid=f"o{i}", symbol=S,
                   transaction=int(rng.choice([0, 1, 1, 3])), price=float(rng.choice([0.1, 0.25, 0.5, 1.0, 37.5])),
                   volume=float(rng.choice([0.01, 0.5, 3.0, 1234.5])))
        n = NewOrderNode(req, 8)
        n.Action = 1
        prev = f"o{i - 1}" if rng.random() < 0.6 else None
        nxt = f"o{i + 1}" if rng.random() < 0.6 else None
        n.IsFirst, n.IsLast = prev is None, nxt is None
        n.PrevNode = f"{S}:node:{prev}" if prev else ""
        n.NextNode = f"{S}:node:{nxt}" if nxt else ""
        got = render_link_node(S, int(n.Price), n.Transaction, int(n.Volume), req["uuid"], req["oid"], prev, nxt)
        assert got == n.to_json()


def _literal_keys(lit, symbols):
    """The literal FakeRedis restricted to the book keys of the symbols (zero depth fields
    dropped: see gome_amd/snapshot.py)."""
    h, z = {}, {}
    for key, fields in lit.cache.h.items():
        S = key.split(":")[0]
        if S not in symbols or key.endswith(":comparison"):
            continue
        if key.endswith(":depth"):
            fields = {f: v for f, v in fields.items() if float(v) != 0.0}
            if not fields:
                continue
        h[key] = dict(fields)
    for key, members in lit.cache.z.items():
        if key.split(":")[0] in symbols and members:
            z[key] = dict(members)
    return {"hash": h, "zset": z}


def _run(seed, quirks):
    rng = np.random.default_rng(seed)
    batches = random_batches(rng, n_batches=4, batch=120, symbols=SYMBOLS, del_frac=0.25, quirks=quirks)
    lit, lit_events = run_batches(batches)
    names = Interner()
    for s in SYMBOLS:
        names.id("sym", s)
    eng = Engine(max_symbols=len(SYMBOLS), max_batch=512, max_nodes=1 << 16, max_levels=1 << 14)
    for b in batches:
        eng.submit(requests_to_records(b, names))
        eng.drain()
    return rng, lit, eng, names


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_snapshot_equals_literal_redis(seed):
    """After the same quirk-laden stream, the engine's snapshot equals the reference's Redis
    book keys: both side ZSETs, the depth HASH, every FIFO link HASH with its node JSON."""
    _, lit, eng, names = _run(500 + seed, quirks=True)
    snap = snapshot.redis_snapshot(eng, [names.id("sym", s) for s in SYMBOLS], names)
    exp = _literal_keys(lit, SYMBOLS)
    assert snap["zset"] == exp["zset"]
    assert set(snap["hash"]) == set(exp["hash"])
    for key in exp["hash"]:
        assert snap["hash"][key] == exp["hash"][key], key
    assert snapshot.to_resp(snap).count(b"HSET") == sum(len(v) for v in snap["hash"].values())


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_resume_from_snapshot_continues_identically(seed):
    """Snapshot -> fresh engine (replayed rests, no fill) -> the same snapshot, and the next
    batch gives the reference's MatchResults on both the original and the resumed engine."""
    rng, lit, eng, names = _run(700 + seed, quirks=False)
    sids = [names.id("sym", s) for s in SYMBOLS]
    snap = snapshot.redis_snapshot(eng, sids, names)
    # replayed in chunks of 16 records (FIFO order kept across them)
    eng2 = Engine(max_symbols=len(SYMBOLS), max_batch=4096, max_nodes=1 << 16, max_levels=1 << 14)
    assert snapshot.restore(eng2, snap, names, chunk=16) > 16
    assert snapshot.redis_snapshot(eng2, sids, names) == snap
    nxt = random_batches(rng, n_batches=1, batch=150, symbols=SYMBOLS, del_frac=0.25, quirks=False,
                         oid_base=10**6)
    rec = requests_to_records(nxt[0], names)
    eng.submit(rec)
    a = render_events(eng.drain(), rec, names)
    eng2.submit(rec)
    b = render_events(eng2.drain(), rec, names)
    assert a == b and len(a) > 0


@pytest.mark.gpu
def test_restore_refuses_quirk_books():
    """A wrong-side cancel (Q2, engine.go:87-116) ZREMs the request's side, so the BUY set keeps
    a member with no FIFO and depth 0: the snapshot still equals the reference's Redis, but a
    replay cannot rebuild it, and restore refuses instead of resuming a different book."""
    names = Interner()
    names.id("sym", "eth2usdt")
    add = dict(uuid="u1", oid="o1", symbol="eth2usdt", transaction=0, price=0.5, volume=1.0)
    add2 = dict(uuid="u1", oid="o2", symbol="eth2usdt", transaction=1, price=0.7, volume=2.0)
    dele = dict(add, transaction=1)                 # cancel on the wrong side
    batches = [[(1, add), (1, add2)], [(2, dele)]]
    lit, _ = run_batches(batches)
    eng = Engine(max_symbols=1, max_batch=16, max_nodes=1 << 10, max_levels=1 << 10)
    for b in batches:
        eng.submit(requests_to_records(b, names))
        eng.drain()
    snap = snapshot.redis_snapshot(eng, [0], names)
    assert snap == _literal_keys(lit, ("eth2usdt",))
    assert "50000000" in snap["zset"]["eth2usdt:BUY"]
    with pytest.raises(GomeError):
        snapshot.restore_records(snap, names)


def test_restore_refuses_crossed_book_before_submitting():
    """A snapshot whose best bid >= best ask would fill on replay: refused while validating,
    before any record reaches an engine."""
    names = Interner()
    names.id("sym", "s")
    names.id("uuid", "u")
    node = lambda oid, tx, p, v, prev, nxt: render_link_node("s", p, tx, v, "u", oid, prev, nxt)
    snap = {"hash": {"s:depth": {"s:depth:60000000": "100000000", "s:depth:50000000": "100000000"},
                     "s:link:60000000": {"f": "s:node:a", "l": "s:node:a",
                                         "s:node:a": node("a", 0, 60000000, 100000000, None, None)},
                     "s:link:50000000": {"f": "s:node:b", "l": "s:node:b",
                                         "s:node:b": node("b", 1, 50000000, 100000000, None, None)}},
            "zset": {"s:BUY": {"60000000": 6e7}, "s:SALE": {"50000000": 5e7}}}
    with pytest.raises(GomeError, match="crossed"):
        snapshot.restore_records(snap, names)
    snap["zset"] = {"s:BUY": {"50000000": 5e7}, "s:SALE": {"60000000": 6e7}}
    snap["hash"]["s:link:60000000"]["s:node:a"] = node("a", 1, 60000000, 100000000, None, None)
    snap["hash"]["s:link:50000000"]["s:node:b"] = node("b", 0, 50000000, 100000000, None, None)
    rec = snapshot.restore_records(snap, names)
    assert len(rec) == 2


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_load_quirk_snapshot_continues_identically(seed):
    """Quirk-laden books (Q2 leftovers, zero-volume makers, unusual Transactions) loaded straight
    into a fresh engine (gome_load_books): the same snapshot, and the same MatchResults and
    snapshot as the engine they came from after two more quirk-laden batches."""
    rng, lit, eng, names = _run(900 + seed, quirks=True)
    sids = [names.id("sym", s) for s in SYMBOLS]
    snap = snapshot.redis_snapshot(eng, sids, names)
    eng2 = Engine(max_symbols=len(SYMBOLS), max_batch=512, max_nodes=1 << 16, max_levels=1 << 14)
    assert snapshot.load(eng2, snap, names) == eng.stats()["n_resting"]
    assert snapshot.redis_snapshot(eng2, sids, names) == snap
    assert eng2.stats()["n_resting"] == eng.stats()["n_resting"]
    for k in range(2):
        nxt = random_batches(rng, n_batches=1, batch=150, symbols=SYMBOLS, del_frac=0.25, quirks=True,
                             oid_base=10**6 * (k + 1))
        rec = requests_to_records(nxt[0], names)
        eng.submit(rec)
        a = render_events(eng.drain(), rec, names)
        eng2.submit(rec)
        b = render_events(eng2.drain(), rec, names)
        assert a == b, f"batch {k}"
    assert snapshot.redis_snapshot(eng2, sids, names) == snapshot.redis_snapshot(eng, sids, names)


@pytest.mark.gpu
def test_load_restores_the_q2_book_replay_refuses():
    """The Q2 book restore() refuses (a BUY member without FIFO, depth 0) loads exactly, and a
    later SALE at that price sees the stale member as the reference does."""
    names = Interner()
    names.id("sym", "eth2usdt")
    add = dict(uuid="u1", oid="o1", symbol="eth2usdt", transaction=0, price=0.5, volume=1.0)
    add2 = dict(uuid="u1", oid="o2", symbol="eth2usdt", transaction=1, price=0.7, volume=2.0)
    dele = dict(add, transaction=1)
    sale = dict(uuid="u2", oid="o3", symbol="eth2usdt", transaction=1, price=0.5, volume=0.5)
    batches = [[(1, add), (1, add2)], [(2, dele)]]
    lit, _ = run_batches(batches + [[(1, sale)]])
    eng = Engine(max_symbols=1, max_batch=16, max_nodes=1 << 10, max_levels=1 << 10)
    for b in batches:
        eng.submit(requests_to_records(b, names))
        eng.drain()
    snap = snapshot.redis_snapshot(eng, [0], names)
    eng2 = Engine(max_symbols=1, max_batch=16, max_nodes=1 << 10, max_levels=1 << 10)
    snapshot.load(eng2, snap, names)
    assert snapshot.redis_snapshot(eng2, [0], names) == snap
    rec = requests_to_records([(1, sale)], names)
    eng.submit(rec)
    eng2.submit(rec)
    assert render_events(eng2.drain(), rec, names) == render_events(eng.drain(), rec, names)
    assert snapshot.redis_snapshot(eng2, [0], names) == _literal_keys(lit, ("eth2usdt",))


class _Ids:
    """Names for numeric workload ids (the snapshot renders every id as its decimal text)."""

    def name(self, kind, i):
        return f"{kind}{i}"

    def id(self, kind, s):
        return int(s[len(kind):])


@pytest.mark.gpu
def test_load_flow_books_continues_identically():
    """Clean books deep enough for the flow path (Zipf over 40 symbols, 20k-order batches with
    cancels): loaded into a fresh engine they take the flow path on the next batch and give the
    same events and books as the original engine."""
    from gome_amd import workload as wl
    g = wl.NativeStream(40, 1.0, seed=11, del_frac=0.3, aggressive_frac=0.05)
    mk = lambda: Engine(max_symbols=40, max_batch=20000, max_nodes=1 << 20, max_levels=1 << 16)
    eng = mk()
    for _ in range(2):
        eng.submit(g.batch(20000).copy())
        eng.drain()
    ids = _Ids()
    snap = snapshot.redis_snapshot(eng, range(40), ids)
    eng2 = mk()
    snapshot.load(eng2, snap, ids)
    assert snapshot.redis_snapshot(eng2, range(40), ids) == snap
    b = g.batch(20000).copy()
    eng.submit(b)
    e1 = eng.drain()
    eng2.submit(b)
    e2 = eng2.drain()
    assert eng2.stats()["n_flow_books"] > 0
    assert np.array_equal(e1, e2)
    for s in range(40):
        assert np.array_equal(eng.levels(s), eng2.levels(s))


def test_load_images_keep_quirk_states():
    """book_images (CPU): a member without a FIFO and a depth without nodes are kept as levels."""
    names = Interner()
    names.id("sym", "s")
    snap = {"hash": {"s:depth": {"s:depth:70000000": "200000000"}},
            "zset": {"s:BUY": {"50000000": 5e7}}}
    (sid, lv, nd), = snapshot.book_images(snap, names)
    assert sid == 0 and len(nd) == 0
    assert [(int(x["price_fx"]), int(x["depth_fx"]), int(x["in_buy"]), int(x["in_sale"])) for x in lv] == \
        [(50000000, 0, 1, 0), (70000000, 200000000, 0, 0)]


@pytest.mark.gpu
def test_load_books_rejects_bad_images():
    """gome_load_books checks its image: a used engine (E_STATE), a repeated symbol, prices
    out of order and node counts that do not add up (E_INVAL); nothing is loaded then."""
    from gome_amd.workload import LEVEL_DTYPE, NODE_DTYPE
    lv = np.zeros(2, LEVEL_DTYPE)
    lv[0] = (10, 5, 1, 1, 0, 0)
    lv[1] = (20, 7, 1, 0, 1, 0)
    nd = np.zeros(2, NODE_DTYPE)
    nd[0]["volume_fx"], nd[0]["oid_id"], nd[0]["side"] = 5, 1, 0
    nd[1]["volume_fx"], nd[1]["oid_id"], nd[1]["side"] = 7, 2, 1
    mk = lambda: Engine(max_symbols=4, max_batch=16, max_nodes=1 << 10, max_levels=1 << 10)
    with pytest.raises(GomeError):
        mk().load_books([(0, lv, nd), (0, lv, nd)])          # repeated symbol
    with pytest.raises(GomeError):
        mk().load_books([(0, lv[::-1].copy(), nd)])          # prices not ascending
    with pytest.raises(GomeError):
        mk().load_books([(0, lv, nd[:1].copy())])            # node counts do not add up
    e = mk()
    e.load_books([(1, lv, nd)])
    assert e.stats()["n_resting"] == 2 and len(e.levels(1)) == 2
    with pytest.raises(GomeError):
        e.load_books([(2, lv, nd)])                          # not a fresh engine any more
    used = mk()  # (an empty or refused submit does not count as use: tests/test_gpu_r3.py)
    one = np.zeros(1, __import__("gome_amd.workload", fromlist=["ORDER_DTYPE"]).ORDER_DTYPE)
    one[0] = (10, 5, 3, 9, 1, 0, 1, 0)
    used.submit(one)
    with pytest.raises(GomeError):
        used.load_books([(1, lv, nd)])
