"""Batching consumer + pre-pool markers + matchOrder sink (gome_amd/consumer.py) against the
literal transliteration of the reference's gRPC handlers, queue and consumer
(oracle/literal.py: grpc_do_order / grpc_delete_order / consume, rabbitmq.go:116-125,
main.go:39-64, nodepool.go:14-28).

The schedule interleaves gRPC calls and consumption arbitrarily (not batch-aligned): duplicate
ADDs whose markers are re-set while the first is still queued, DELs that overtake their ADD,
cancels of consumed orders.  The consumer drains exactly the messages the reference consumes
at each point, so the published MatchResult bytes must be identical.  The CPU variant runs the
consumer in front of the C oracle (test infrastructure standing in for the engine; it honours
the same GOME_ORD_ADM_HOST flags); the GPU variant in front of libgome."""
import numpy as np
import pytest

from gome_amd.consumer import BatchingConsumer, Ingress, MatchSink, Names, PrePool
from oracle.literal import GomeLiteral
from oracle.pyoracle import Oracle


class _OracleEngine:
    def __init__(self, n_sym, max_batch):
        self.o, self.max_batch, self._ev = Oracle(n_sym), max_batch, None
        self.max_symbols = n_sym

    def submit(self, rec, seq_base=0):
        ev = self.o.submit(rec)
        sq = ev["taker_seq"].astype(np.uint64) + np.uint64(seq_base)
        ev["taker_seq"] = (sq & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        self._ev = ev

    def drain(self):
        ev, self._ev = self._ev, None
        return ev

    def stats(self):
        return self.o.stats()


def _schedule(seed, n_ops=900, symbols=("eth2usdt", "btc2usdt", "a<b&c")):
    """Random interleaving of gRPC calls ("add"/"del", req) and consumption ("take", k)."""
    rng = np.random.default_rng(seed)
    ops, live, oid = [], [], 1
    prices = [0.1, 0.25, 0.3, 0.5, 0.55, 0.7, 1.0]
    vols = [0.01, 0.1, 0.5, 1.0, 2.5]
    sent = taken = 0          # messages enqueued / consumed so far
    last_add_msg = -1         # queue position of the newest ADD
    for _ in range(n_ops):
        u = rng.random()
        if u < 0.12:
            k = int(rng.integers(1, 40))
            ops.append(("take", k))
            taken = min(sent, taken + k)
        elif u < 0.35 and live:
            r = dict(live[int(rng.integers(len(live)))])
            if rng.random() < 0.05:
                r["price"] = float(rng.choice(prices))  # Q3 wrong price
            ops.append(("del", r))
            sent += 1
        else:
            if live and last_add_msg >= taken and rng.random() < 0.06:
                # duplicate ADD while the first is still queued: its marker is set again, the
                # first consumption clears it, the duplicate is dropped (Q4; a duplicate of a
                # consumed ADD would be a duplicate live oid, Q7, outside the domain)
                ops.append(("add", dict(live[-1])))
                sent += 1
                continue
            r = dict(uuid="u" + str(int(rng.integers(3))), oid=str(oid), symbol=str(rng.choice(symbols)),
                     transaction=int(rng.choice([0, 1, 1, 0, 257])), price=float(rng.choice(prices)),
                     volume=float(rng.choice(vols)))
            oid += 1
            if rng.random() < 0.04:
                ops.append(("del", dict(r)))  # the DEL overtakes its ADD
                sent += 1
            ops.append(("add", r))
            last_add_msg = sent
            sent += 1
            live.append(r)
    ops.append(("take", 10**9))
    return ops


def _run(ops, engine, lit_json: bool):
    lit = GomeLiteral()
    pre, sink, names = PrePool(), MatchSink(), Names()
    q: list = []
    ing = Ingress(q, pre)
    cons = BatchingConsumer(engine, pre, sink, names, max_batch=engine.max_batch)
    lit_out = []
    for op, arg in ops:
        if op == "add":
            lit.grpc_do_order(arg)
            if lit_json:  # the reference's own message bytes, marker set as main.go:44-45
                pre.set(arg["symbol"], arg["uuid"], arg["oid"])
                q.append(lit.do_order_q[-1])
            else:
                ing.do_order(arg)
        elif op == "del":
            lit.grpc_delete_order(arg)
            q.append(lit.do_order_q[-1]) if lit_json else ing.delete_order(arg)
        else:
            # the reference consumes one message at a time (and so does the literal here); the
            # consumer drains batches of up to max_batch: the published bytes must not differ
            k = min(arg, len(lit.do_order_q))
            for _ in range(k):
                head, lit.do_order_q = lit.do_order_q[:1], lit.do_order_q[1:]
                saved, lit.do_order_q = lit.do_order_q, head
                lit.consume_boundary()
                lit.do_order_q = saved
                lit_out += lit.take_results()
            while k:
                m = min(k, cons.max_batch)
                cons.process(q[:m])
                del q[:m]
                k -= m
    return lit_out, sink.q, cons


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("lit_json", [True, False])
def test_consumer_matches_literal_cpu(seed, lit_json):
    lit_out, got, cons = _run(_schedule(100 + seed), _OracleEngine(3, 64), lit_json)
    assert len(lit_out) > 100
    assert got == lit_out
    assert cons.rejected == 0


def test_consumer_ignores_bad_json_and_rejects_q5():
    lit_out, got, cons = _run([("take", 1)], _OracleEngine(1, 8), True)
    pre, sink = PrePool(), MatchSink()
    cons = BatchingConsumer(_OracleEngine(1, 8), pre, sink, max_batch=8)
    ing = Ingress([], pre)
    msgs = ["{not json", '{"Action":1,"Symbol":"s","Uuid":"u","Oid":"1","Transaction":0,'
                         '"Price":50000000.5,"Volume":100000000}']
    cons.process(msgs)
    assert cons.consumed == 2 and cons.rejected == 1 and sink.q == []
    # Ingress scaling is exact (NewOrderNode via the decimal path)
    ing.do_order(dict(uuid="u", oid="2", symbol="s", transaction=0, price=0.29, volume=1.0))
    assert '"Price":29000000.0' in ing.q[-1]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(3))
def test_consumer_matches_literal_gpu(seed):
    from gome_amd.abi import Engine
    lit_out, got, cons = _run(_schedule(200 + seed, n_ops=1500), Engine(max_symbols=3, max_batch=128), True)
    assert len(lit_out) > 100
    assert got == lit_out


# ---- Go json.Unmarshal at the boundary ----------------------
def _msg(action=1, sym="s", uuid="u", oid="1", tx=0, price="50000000", vol="100000000", extra=""):
    # (Accuracy is the server's constant in every message the gRPC side writes, ordernode.go:56-58;
    # the renderer echoes the engine's accuracy, so the messages carry it)
    return ('{"Action":%s,"Uuid":"%s","Oid":"%s","Symbol":"%s","Transaction":%s,"Price":%s,"Volume":%s,'
            '"Accuracy":8%s}' % (action, uuid, oid, sym, tx, price, vol, extra))


# messages that decode partially under Go's encoding/json: the mistyped field stays zero and the
# message is still dispatched (rabbitmq.go:118-124)
ODD_MESSAGES = [
    _msg(oid="1", price='"abc"'),                      # Price string -> 0: an ADD at price 0
    _msg(oid="2", price="null"),                       # null -> no effect -> 0
    _msg(oid="3", tx='"x"', price="60000000"),         # Transaction string -> 0 (BUY)
    _msg(oid="4", action="300"),                       # int8 overflow -> Action 0: ignored
    _msg(oid="5", action="1.0"),                       # not an integer literal -> Action 0
    _msg(oid="6", tx="1", price="40000000", vol="1e400"),  # float overflow -> Volume 0 (Q6)
    _msg(oid="7", tx="1", price="40000000", vol="30000000", extra=',"price":45000000'),  # later key wins
    '{"action":1,"uuid":"u","oid":"8","symbol":"s","transaction":1,"price":45000000,"volume":5000000,"accuracy":8}',
    _msg(oid="9", tx="4294967297"),                    # int32 overflow -> 0 (BUY)
    _msg(oid="10", price="true"),                      # bool into float -> 0
    '[1,2,3]', 'null', '{"Action":1', '{"Action":NaN}',  # non-object / syntax errors: zero node
    _msg(oid="11", sym='a\\ud800b', tx="1", price="50000000"),  # lone surrogate -> U+FFFD
    _msg(oid="12", price="5e7", vol="1E8"),            # exponent floats are fine for float64
    _msg(oid="13", vol="-100000000").encode(),         # raw bytes; a negative Volume: rejected
    _msg(oid="14", sym="b\xe2\x82z", tx="1", price="50000000").encode("latin-1"),  # invalid UTF-8:
    _msg(oid="15", sym="b\xed\xa0\x80\xffz", price="50000000").encode("latin-1"),  # U+FFFD per byte
]


def _odd_schedule():
    ops = []
    for m in ODD_MESSAGES:
        ops.append(("raw", m))
    ops.append(("take", 10**9))
    # then ordinary traffic crossing what rested
    for k in range(20):
        ops.append(("add", dict(uuid="v", oid=str(100 + k), symbol="s", transaction=k % 2,
                                price=0.4 + 0.05 * (k % 4), volume=0.5)))
    ops.append(("take", 10**9))
    return ops


def _run_raw(ops, engine):
    """Like _run, but "raw" ops put a message body on the queue as the reference's gRPC side
    would have (its admission marker set for the (Symbol, Uuid, Oid) Go decodes from it)."""
    from oracle.literal import go_unmarshal_order_node
    lit = GomeLiteral()
    pre, sink, names = PrePool(), MatchSink(), Names()
    q: list = []
    cons = BatchingConsumer(engine, pre, sink, names, max_batch=engine.max_batch)
    lit_out = []
    for op, arg in ops:
        if op == "raw":
            nd = go_unmarshal_order_node(arg)
            nd.SetOrderHashKey()
            nd.SetNodeName()
            nd.SetDepthHashKey()
            nd.SetNodeLink()
            nd.SetListZsetKey()
            pre.set(nd.Symbol, nd.Uuid, nd.Oid)
            q.append(arg)
            if nd.Volume < 0:  # outside the exact domain: the consumer rejects it (not compared)
                continue
            lit.SetPrePool(nd)
            lit.do_order_q.append(nd.to_json())  # the literal consumes Go's view of the message
        elif op == "add":
            lit.grpc_do_order(arg)
            pre.set(arg["symbol"], arg["uuid"], arg["oid"])
            q.append(lit.do_order_q[-1])
        else:
            k = min(arg, len(q))
            head, lit.do_order_q = lit.do_order_q[:k], lit.do_order_q[k:]
            saved, lit.do_order_q = lit.do_order_q, head
            lit.consume_boundary()
            lit.do_order_q = saved
            lit_out += lit.take_results()
            while k:
                m = min(k, cons.max_batch)
                cons.process(q[:m])
                del q[:m]
                k -= m
    return lit_out, sink.q, cons


def test_decode_like_go_unmarshal():
    from gome_amd.consumer import decode_order_node
    from oracle.literal import go_unmarshal_order_node
    for m in ODD_MESSAGES:
        a = decode_order_node(m)
        b = go_unmarshal_order_node(m)
        assert a == {k: getattr(b, k) for k in a}, m
    d = decode_order_node(ODD_MESSAGES[0])
    assert d["Action"] == 1 and d["Price"] == 0.0 and d["Volume"] == 1e8
    assert decode_order_node(ODD_MESSAGES[3])["Action"] == 0
    assert decode_order_node(ODD_MESSAGES[6])["Price"] == 45000000.0
    assert decode_order_node(ODD_MESSAGES[7])["Oid"] == "8"
    assert decode_order_node(ODD_MESSAGES[-5])["Symbol"] == "a\ufffdb"
    assert decode_order_node(ODD_MESSAGES[-2])["Symbol"] == "b\ufffd\ufffdz"
    assert decode_order_node(ODD_MESSAGES[-1])["Symbol"] == "b\ufffd\ufffd\ufffd\ufffdz"


def test_consumer_odd_messages_match_literal_cpu():
    lit_out, got, cons = _run_raw(_odd_schedule(), _OracleEngine(4, 64))
    assert len(lit_out) > 5
    assert got == lit_out
    assert cons.consumed == len(ODD_MESSAGES) + 20 and cons.rejected == 1  # (the negative Volume)


def test_consumer_rejects_symbols_beyond_max_symbols_and_negative_volumes():
    """a message the engine would refuse the whole batch for (a Symbol beyond its
    max_symbols, a negative Volume) is rejected on its own; the rest of the batch is applied."""
    pre, sink = PrePool(), MatchSink()
    cons = BatchingConsumer(_OracleEngine(2, 16), pre, sink, max_batch=16)
    msgs = []
    for k, (sym, tx, vol) in enumerate([("a", 0, "100000000"), ("b", 1, "100000000"), ("c", 0, "100000000"),
                                        ("a", 1, "-5"), ("c", 1, "100000000"), ("b", 0, "100000000")]):
        pre.set(sym, "u", str(k))
        msgs.append(_msg(sym=sym, oid=str(k), tx=tx, vol=vol))
    cons.process(msgs)
    assert cons.consumed == 6 and cons.rejected == 3 and len(pre) == 0
    assert len(sink.q) == 1 and '"Oid":"5"' in sink.q[0] and '"Oid":"1"' in sink.q[0]  # b's BUY fills b's SALE


class _RefusingEngine(_OracleEngine):
    """Refuses the first `k` submits as the engine's pool-headroom check does (E_CAPACITY before
    anything is applied)."""

    def __init__(self, n_sym, max_batch, k):
        super().__init__(n_sym, max_batch)
        self.k = k

    def submit(self, rec, seq_base=0):
        from gome_amd.abi import GOME_E_CAPACITY, GomeError
        if self.k:
            self.k -= 1
            raise GomeError(GOME_E_CAPACITY, "batch rejected before it was applied")
        super().submit(rec, seq_base)


def test_consumer_batch_refused_then_resubmitted_cpu():
    """a batch the engine refuses leaves the pre-pool markers untouched, so processing
    the same messages again admits exactly as the first attempt would have."""
    from gome_amd.abi import GomeError
    ops = _schedule(321, n_ops=300)
    lit_out, want, _ = _run(ops, _OracleEngine(3, 64), True)
    lit = GomeLiteral()
    pre, sink, names = PrePool(), MatchSink(), Names()
    cons = BatchingConsumer(_RefusingEngine(3, 64, 0), pre, sink, names, max_batch=64)
    q: list = []
    refused = 0
    for op, arg in ops:
        if op == "add":
            lit.grpc_do_order(arg)
            pre.set(arg["symbol"], arg["uuid"], arg["oid"])
            q.append(lit.do_order_q.pop())
        elif op == "del":
            lit.grpc_delete_order(arg)
            q.append(lit.do_order_q.pop())
        else:
            k = min(arg, len(q))
            while k:
                m = min(k, 64)
                cons.eng.k = 1  # every batch is refused once
                n_pre = len(pre)
                with pytest.raises(GomeError):
                    cons.process(q[:m])
                assert len(pre) == n_pre  # no marker consumed
                refused += 1
                cons.process(q[:m])
                del q[:m]
                k -= m
    assert refused > 5
    assert sink.q == want == lit_out


def test_render_events_long_ids():
    """ids longer than any fixed staging buffer render (no 'unknown id' error); a
    short buffer returns -(bytes needed)."""
    import ctypes as C
    from gome_amd.abi import load_library
    from gome_amd.workload import EVENT_DTYPE, ORDER_DTYPE
    lib = load_library()
    lib.gome_render_events.restype = C.c_int64
    long_oid = "o" * 40000
    rec = np.zeros(1, ORDER_DTYPE)
    rec[0] = (5 * 10**7, 10**8, 0, 0, 0, 0, 1, 0)
    ev = np.zeros(1, EVENT_DTYPE)
    ev[0]["kind"], ev[0]["price_fx"], ev[0]["maker_volume_fx"] = 2, 5 * 10**7, 10**8
    ev[0]["maker_is_last"] = 1
    tab = lambda *s: (C.c_char_p * len(s))(*[x.encode() for x in s])
    sym, uu, oo = tab("s"), tab("u"), tab(long_oid)
    args = lambda buf, cap: (ev.ctypes.data, 1, rec.ctypes.data, 1, 0, 8, C.cast(sym, C.c_void_p), 1,
                             C.cast(uu, C.c_void_p), 1, C.cast(oo, C.c_void_p), 1, None, buf, cap)
    need = lib.gome_render_events(*args(None, 0))
    assert need < 0 and -need > 2 * 40000
    buf = C.create_string_buffer(-need)
    n = lib.gome_render_events(*args(buf, -need))
    assert n == -need
    line = buf.raw[:n].decode()
    assert line.endswith("}\n") and line.count(long_oid) == 6  # Oid, NodeName and OrderHashField, twice


@pytest.mark.gpu
def test_consumer_odd_messages_match_literal_gpu():
    from gome_amd.abi import Engine
    lit_out, got, cons = _run_raw(_odd_schedule(), Engine(max_symbols=4, max_batch=64))
    assert len(lit_out) > 5 and got == lit_out


@pytest.mark.gpu
def test_consumer_capacity_refusal_then_bigger_engine_gpu():
    """A real E_CAPACITY refusal (pool headroom, nothing applied): the markers survive, and the
    same messages processed by an engine with larger pools publish what the literal publishes."""
    from gome_amd.abi import GOME_E_CAPACITY, Engine, GomeError
    ops = [op for op in _schedule(77, n_ops=400) if op[0] != "take"] + [("take", 10**9)]
    lit_out, want, _ = _run(ops, _OracleEngine(3, 512), True)
    lit = GomeLiteral()
    pre, sink = PrePool(), MatchSink()
    q = []
    for op, arg in ops[:-1]:
        (lit.grpc_do_order if op == "add" else lit.grpc_delete_order)(arg)
        if op == "add":
            pre.set(arg["symbol"], arg["uuid"], arg["oid"])
        q.append(lit.do_order_q.pop())
    small = Engine(max_symbols=3, max_batch=512, max_nodes=16, max_levels=1 << 12)
    cons = BatchingConsumer(small, pre, sink, max_batch=512)
    n_pre = len(pre)
    with pytest.raises(GomeError) as ei:
        cons.process(q)
    assert ei.value.status == GOME_E_CAPACITY and len(pre) == n_pre and sink.q == []
    cons.eng = Engine(max_symbols=3, max_batch=512)
    cons.process(q)
    assert sink.q == want == lit_out


# ---- multi-GPU routing (gome_amd/router.py) ------------------------------------
@pytest.mark.parametrize("world", [2, 4])
def test_consumer_through_router_matches_literal_cpu(world):
    """The consumer in front of N handles (symbols owned by load rank mod N; with 3 symbols and
    N = 4 one handle never gets a record): the merged publish stream is byte-identical."""
    from gome_amd.router import Router, owner_table
    r = Router([_OracleEngine(3, 64) for _ in range(world)], owner_table(3, world, np.array([0, 1, 2])))
    lit_out, got, cons = _run(_schedule(400 + world), r, True)
    assert len(lit_out) > 100 and got == lit_out
    r.close()


def test_router_hash_owner_for_unknown_symbols():
    from gome_amd.router import owner_table
    own = owner_table(1000, 4, np.array([5, -1, 7]))
    assert own[0] == 1 and own[2] == 3
    assert set(own[3:].tolist()) == {0, 1, 2, 3}
    assert np.array_equal(own, owner_table(1000, 4, np.array([5, -1, 7])))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_consumer_through_router_matches_literal_gpu(world):
    from gome_amd.abi import Engine
    from gome_amd.router import Router, owner_table
    r = Router([Engine(max_symbols=3, max_batch=128) for _ in range(world)],
               owner_table(3, world, np.array([0, 1, 2])))
    lit_out, got, cons = _run(_schedule(500 + world, n_ops=1500), r, True)
    assert len(lit_out) > 100 and got == lit_out
    r.close()


def _stream_ops(seed, n=6000):
    """A queue of doOrder messages with every marker set before consumption (no interleaving)."""
    ops = [op for op in _schedule(seed, n_ops=n) if op[0] != "take"]
    return ops + [("take", 10**9)]


@pytest.mark.gpu
@pytest.mark.parametrize("packed", [False, True])
def test_consumer_pipelined_stream_matches_literal_gpu(packed):
    """process_stream (two batches in flight, records straight into page-locked buffers, MatchResults
    rendered as each batch is collected) publishes exactly the literal reference's bytes, from a
    list of bodies or from one packed delivery buffer (PackedQueue)."""
    from gome_amd.abi import Engine
    from gome_amd.consumer import PackedQueue
    lit_out, _, _ = _run(_stream_ops(300), _OracleEngine(3, 64), True)
    lit = GomeLiteral()
    pre, sink, names = PrePool(), MatchSink(), Names()
    q = []
    for op, arg in _stream_ops(300)[:-1]:
        if op == "add":
            lit.grpc_do_order(arg)
            pre.set(arg["symbol"], arg["uuid"], arg["oid"])
        else:
            lit.grpc_delete_order(arg)
        q.append(lit.do_order_q[-1])
    cons = BatchingConsumer(Engine(max_symbols=3, max_batch=256), pre, sink, names, max_batch=256)
    batches = PackedQueue(q).batches(256) if packed else (q[k:k + 256] for k in range(0, len(q), 256))
    n = cons.process_stream(batches)
    assert n == len(lit_out) and sink.q == lit_out
    assert cons.consumed == len(q) and len(pre) == 0


def test_render_beside_interning_reads_stable_tables():
    """process_stream renders batch k on a helper thread while this thread interns batch k + 1's
    names; an intern that outgrows an id table moves it (round 6: the r06i GPU run segfaulted in
    the render).  gome_render_events_names reads the tables under the names' lock, so renders beside
    300k interns (every table move included) all give the same bytes."""
    import ctypes as C
    import threading
    from gome_amd.abi import load_library
    from gome_amd.workload import EVENT_DTYPE, ORDER_DTYPE
    lib = load_library()
    names = Names()
    for kind, s in (("sym", "s"), ("uuid", "u"), ("oid", "o")):
        assert names.id(kind, s) == 0
    rec = np.zeros(1, ORDER_DTYPE)
    rec[0] = (5 * 10**7, 10**8, 0, 0, 0, 0, 1, 0)
    ev = np.zeros(64, EVENT_DTYPE)
    ev["kind"], ev["price_fx"], ev["maker_volume_fx"], ev["maker_is_last"] = 2, 5 * 10**7, 10**8, 1
    ev["fill_idx"] = np.arange(64)

    def render():
        buf = C.create_string_buffer(1 << 20)
        n = lib.gome_render_events_names(ev.ctypes.data, len(ev), rec.ctypes.data, 1, 0, 8, names.h, 2, buf, 1 << 20)
        assert n > 0
        return buf.raw[:n]

    want = render()
    got, stop = [], threading.Event()

    def loop():
        while not stop.is_set():
            got.append(render())

    t = threading.Thread(target=loop)
    t.start()
    try:
        for i in range(1, 300000):
            names.id("oid", f"o{i}")
    finally:
        stop.set()
        t.join()
    assert len(got) > 10 and all(g == want for g in got)
