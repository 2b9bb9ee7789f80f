"""Duplicate oids — the boundary rule of include/gome/gome_abi.h.

The reference names a resting node S:node:<oid> without its uuid (ordernode.go:110-112,
nodelink.go:119-122) and assumes oids unique per symbol (README.md:27); a second live node of the
same name corrupts its FIFO.  Rule: an admitted ADD whose (symbol, oid) names a live node when the
ADD is applied is not applied, counted (gome_stats.n_dup_oid) and listed (gome_dup_records).  It
depends on the queue order only, not on where batches start and end.  The literal
transliteration applies it in a wrapper around its faithful consumer loop, before DoOrder
(oracle/literal.py GomeLiteral.consume_boundary), the C oracle in oracle_submit; in the engine the
admission kernels mark the ADDs whose key rests at batch start or repeats in the batch, their books
go to the serial kernels, and those probe the cancel index as each marked ADD is applied."""
import numpy as np
import pytest

from gome_amd import workload as wl
from oracle.literal import run_batches
from oracle.pyoracle import Oracle
from tests.helpers import Interner, render_events, requests_to_records

ADD, DEL = 1, 2


def _req(a, oid, uuid="u1", sym="s", tx=0, p=0.5, v=1.0):
    return (a, dict(uuid=uuid, oid=str(oid), symbol=sym, transaction=tx, price=p, volume=v))


# Each case: batches of requests; expected batch indices rejected per batch.
KATS = {
    # same batch, same (S, oid), another uuid: the second ADD is rejected (it would name the same node)
    "same_batch_other_uuid": ([[_req(ADD, 7, "u1"), _req(ADD, 7, "u2", p=0.6)]], [[1]]),
    # same key twice: Q4 drops the second (no marker left), not the duplicate rule
    "same_key_is_q4": ([[_req(ADD, 7, "u1"), _req(ADD, 7, "u1")]], [[]]),
    # resting from an earlier batch, re-added under another uuid: rejected
    "resting_at_batch_start": ([[_req(ADD, 7, "u1")], [_req(ADD, 7, "u2", p=0.4)]], [[], [0]]),
    # filled in an earlier batch, then reused: an ordinary ADD
    "reuse_after_fill": ([[_req(ADD, 7, "u1", tx=1, p=0.5)], [_req(ADD, 8, "u9", p=0.5)],
                          [_req(ADD, 7, "u2", p=0.3)]], [[], [], []]),
    # cancelled in an earlier batch, then reused
    "reuse_after_cancel": ([[_req(ADD, 7, "u1")], [_req(DEL, 7, "u1")], [_req(ADD, 7, "u2")]], [[], [], []]),
    # filled within the batch, then reused in the same batch: an ordinary ADD (the node is gone)
    "filled_then_reused_same_batch": ([[_req(ADD, 7, "u1", tx=1, p=0.5), _req(ADD, 8, "u9", p=0.5),
                                        _req(ADD, 7, "u2", p=0.3)]], [[]]),
    # partly filled within the batch (still live), then reused: rejected
    "partly_filled_then_reused_same_batch": ([[_req(ADD, 7, "u1", tx=1, p=0.5, v=2.0), _req(ADD, 8, "u9", p=0.5),
                                               _req(ADD, 7, "u2", p=0.3)]], [[2]]),
    # rested in the batch, re-added, then filled and re-added again: rejected, then applied
    "rejected_then_applied_same_batch": ([[_req(ADD, 7, "u1", tx=1, p=0.5), _req(ADD, 7, "u2", p=0.2),
                                           _req(ADD, 8, "u9", p=0.5), _req(ADD, 7, "u3", p=0.3)]], [[1]]),
    # an ADD that admission drops (its DEL came first) does not count as carrying the oid
    "dropped_add_does_not_count": ([[_req(DEL, 7, "u1"), _req(ADD, 7, "u1"), _req(ADD, 7, "u2")]], [[]]),
    # resting at batch start, cancelled earlier in the batch: the re-ADD is an ordinary ADD
    "resting_cancelled_then_readded": ([[_req(ADD, 7, "u1")], [_req(DEL, 7, "u1"), _req(ADD, 7, "u2")]],
                                       [[], []]),
    # resting at batch start, its cancel has the wrong price (Q3: no-op): the re-ADD is rejected
    "resting_wrong_price_cancel_then_readded": ([[_req(ADD, 7, "u1")], [_req(DEL, 7, "u1", p=0.6),
                                                                       _req(ADD, 7, "u2")]], [[], [1]]),
    # another symbol's oid 7 is a different node
    "other_symbol": ([[_req(ADD, 7, "u1", sym="a"), _req(ADD, 7, "u1", sym="b")]], [[]]),
}


def _literal(batches):
    from oracle.literal import GomeLiteral
    eng = GomeLiteral()
    out, dups = [], []
    for b in batches:
        for a, r in b:
            (eng.grpc_do_order if a == ADD else eng.grpc_delete_order)(r)
        eng.consume_boundary()
        out += eng.take_results()
        dups.append(list(eng.dups))
    return out, dups


def _oracle(batches):
    names = Interner()
    for s in sorted({r["symbol"] for b in batches for _, r in b}):
        names.id("sym", s)
    orc = Oracle(len(names.rev["sym"]))
    out, dups = [], []
    for b in batches:
        rec = requests_to_records(b, names)
        out += render_events(orc.submit(rec), rec, names)
        dups.append(orc.dup_records().tolist())
        assert orc.stats()["n_dup_oid"] == len(dups[-1])
    return out, dups


@pytest.mark.parametrize("case", sorted(KATS))
def test_dup_oid_kat_literal_vs_oracle(case):
    batches, want = KATS[case]
    lit, lit_dups = _literal(batches)
    orc, orc_dups = _oracle(batches)
    assert lit == orc
    assert lit_dups == orc_dups == want


def _divergent_stream(n=160000, n_symbols=40, batch=40000, seed=19):
    """The stream on which round 2's engine diverged from the oracle: the
    cancel mix with per-batch oids 1 + k*1000 + U[0,1000) and uuids U{1,2}, so one oid is
    admitted under both uuids in one symbol many times per batch."""
    rec = wl.cancel_mix(n, n_symbols, seed=seed, zipf_s=1.0)
    rng = np.random.default_rng(seed)
    batches = wl.split_batches(rec, batch)
    for k, b in enumerate(batches):
        b["oid_id"] = (1 + k * 1000 + rng.integers(0, 1000, len(b))).astype(b["oid_id"].dtype)
        b["uuid_id"] = rng.integers(1, 3, len(b)).astype(b["uuid_id"].dtype)
    return batches


def _records_to_requests(b):
    out = []
    for r in b:
        out.append((int(r["action"]), dict(uuid="u%d" % r["uuid_id"], oid=str(int(r["oid_id"])),
                                           symbol="s%d" % r["symbol_id"], transaction=int(r["side"]),
                                           price=int(r["price_fx"]) / 1e8, volume=int(r["volume_fx"]) / 1e8)))
    return out


def _host_admitted(b):
    """Admission resolved per record by the host (GOME_ORD_ADM_HOST): every ADD keeps its marker,
    so no verdict depends on the batch (the Q4 batch model would)."""
    b = b.copy()
    b["flags"] = np.where(b["action"] == ADD, 3, 1).astype(b["flags"].dtype)
    return b


def test_dup_rule_does_not_depend_on_batching():
    """the same message stream cut into batches of 4000, 997 and 1 publishes the same
    MatchResults and rejects the same records (C oracle; the literal agrees in the test below)."""
    whole = np.concatenate(_divergent_stream(n=8000, n_symbols=6, batch=4000, seed=29))
    whole["oid_id"] = (1 + np.random.default_rng(1).integers(0, 200, len(whole))).astype(whole["oid_id"].dtype)
    whole = _host_admitted(whole)
    runs = []
    for bs in (4000, 997, 1):
        orc = Oracle(6)
        ev, dups = [], []
        for k in range(0, len(whole), bs):
            e = orc.submit(whole[k:k + bs])
            e["taker_seq"] += k
            ev.append(e)
            dups += [k + int(i) for i in orc.dup_records()]
        runs.append((np.concatenate(ev), dups))
    assert len(runs[0][1]) > 300
    for ev, dups in runs[1:]:
        assert np.array_equal(ev, runs[0][0]) and dups == runs[0][1]


def test_divergent_stream_literal_vs_oracle_small():
    """A 12k-record cut of the divergent stream (3 batches of 4000, oids colliding in every batch
    and, with a narrower oid window, across batches): the literal transliteration (rule in its
    consumer) and the C oracle publish the same MatchResults and reject the same records."""
    batches = _divergent_stream(n=12000, n_symbols=8, batch=4000, seed=23)
    for k, b in enumerate(batches):  # oids 1..300 in every batch: reuse across batches too
        b["oid_id"] = (1 + np.random.default_rng(k).integers(0, 300, len(b))).astype(b["oid_id"].dtype)
    reqs = [_records_to_requests(b) for b in batches]
    lit, lit_dups = _literal(reqs)
    orc, orc_dups = _oracle(reqs)
    assert sum(len(d) for d in orc_dups) > 500
    assert lit_dups == orc_dups
    assert lit == orc


@pytest.mark.gpu
@pytest.mark.parametrize("legacy", [False, True])
def test_divergent_stream_gpu_vs_oracle(legacy):
    """The exact round-2 divergent stream on the GPU, every event and the rejected indices vs the
    C oracle: flow + cold books (default) and every hot book on the legacy kernel."""
    from gome_amd.abi import GOME_FLAG_LEGACY_HOT, Engine
    from tests.test_gpu_v4 import _cmp, _cmp_books
    batches = _divergent_stream()
    eng = Engine(max_symbols=40, max_batch=40000, max_nodes=1 << 20, max_levels=1 << 20,
                 flags=GOME_FLAG_LEGACY_HOT if legacy else 0)
    orc = Oracle(40)
    total = prev_dropped = 0
    for i, b in enumerate(batches):
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"batch {i}")
        d = orc.dup_records()
        assert np.array_equal(eng.dup_records(), d), f"batch {i}: rejected records"
        assert eng.stats()["n_dup_oid"] == len(d)
        dropped = orc.stats()["n_dropped"]  # (the oracle's counters are cumulative)
        assert eng.stats()["n_dropped"] == dropped - prev_dropped
        prev_dropped = dropped
        total += len(d)
    assert total > 1000  # (queue-order rule: a key whose first node was consumed is applied)
    _cmp_books(eng, orc, range(40), "divergent stream")
    assert eng.stats()["n_resting"] == orc.resting()
    # (every book of this stream holds duplicate-oid candidates in every batch: the serial
    # kernels apply them all; tests below cover the flow routing)


def _assign_books(b):
    """Book 0 hot (flow), book 1 ~100 orders (cold), books 2 / 3 quirky with ~5000 / ~500 orders
    (declined: the legacy kernel / the cold kernel)."""
    i = np.arange(len(b))
    b["symbol_id"] = np.select([i % 400 == 0, i % 8 == 1, i % 80 == 3], [1, 2, 3], 0)
    return b


@pytest.mark.gpu
def test_resting_oid_readded_on_flow_cold_and_legacy_books():
    """Oids resting at batch start re-added under another uuid, in a hot book, a cold book and two
    quirky books (legacy and cold kernels), mixed with fresh ADDs: the serial kernels reject each
    one whose node is still live when it is applied, exactly as the oracle does."""
    from gome_amd.abi import Engine
    from tests.test_gpu_v4 import _cmp, _cmp_books
    rng = np.random.default_rng(5)
    g = wl.Stream(4, seed=11)
    eng = Engine(max_symbols=4, max_batch=60000, max_nodes=1 << 20, max_levels=1 << 16)
    orc = Oracle(4)
    first = _assign_books(g.batch(40000))
    q2 = np.zeros(4, wl.ORDER_DTYPE)  # a wrong-side cancel (Q2) marks books 2 and 3 quirky
    q2[:] = (50 * 10**6, 10**6, 2, 10**9, 1, 0, wl.ADD, 0)
    q2[1]["action"], q2[1]["side"] = wl.DEL, 1
    q2[2:] = q2[:2]
    q2["symbol_id"][2:] = 3
    first = np.concatenate([first, q2])
    eng.submit(first)
    _cmp(eng.drain(), orc.submit(first), "first")
    rest = [(s, int(x["oid_id"])) for s in range(4) for p in orc.levels(s)["price_fx"]
            for x in orc.fifo(s, int(p))]
    assert len({s for s, _ in rest}) == 4
    nxt = _assign_books(g.batch(40000))
    pick = rng.choice(len(nxt), 3000, replace=False)
    for j, k in zip(pick, rng.choice(len(rest), 3000)):
        s, o = rest[k]
        nxt[j]["symbol_id"], nxt[j]["oid_id"], nxt[j]["uuid_id"] = s, o, 77 + (j % 3)
    for i in range(3):
        eng.submit(nxt)
        _cmp(eng.drain(), orc.submit(nxt), f"re-added {i}")
        assert np.array_equal(eng.dup_records(), orc.dup_records()), f"batch {i}"
        if i == 0:
            assert len(orc.dup_records()) > 1000
        fl = eng.debug_flow_books()
        if i == 0:  # every book holds re-added oids: the serial kernels decide them
            assert (fl["kind"] == 0).all(), fl
        else:  # fresh oids only: the hot book is back on the flow path
            assert (fl["kind"] > 0).any(), fl
        nxt = _assign_books(g.batch(40000))
    _cmp_books(eng, orc, range(4), "re-added oids")
