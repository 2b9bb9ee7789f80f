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

    def submit(self, rec, seq_base=0):
        ev = self.o.submit(rec)
        sq = ev["taker_seq"].astype(np.uint64) + np.uint64(seq_base)
        ev["taker_seq"] = (sq & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        ev["seq_hi"] = (sq >> np.uint64(32)).astype(np.uint32)
        self._ev = ev

    def drain(self):
        ev, self._ev = self._ev, None
        return ev


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
            k = min(arg, len(lit.do_order_q))
            head, lit.do_order_q = lit.do_order_q[:k], lit.do_order_q[k:]
            saved, lit.do_order_q = lit.do_order_q, head
            lit.consume()
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
