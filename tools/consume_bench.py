"""The consumer's native record building alone (gome_consume_order_nodes through
BatchingConsumer.records), on the host CPU, no GPU: 2^17 OrderNode JSON messages of config 3's
stream in batches of 2^15, threads 1 and 8, with the call's own split (decode / prepare / queue
order) and how many batches took the parallel queue-order path.
  python tools/consume_bench.py [threads ...]"""
import sys, time; sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import numpy as np, bench
from gome_amd import workload as wl
from gome_amd.consumer import BatchingConsumer, MatchSink, Names, PrePool, _order_node_json, PackedQueue
gen, _, _ = bench.make_stream("config3", 0, 1, 49)
n = 1 << 17
rec = gen(n).copy()
msgs = [_order_node_json(dict(symbol="s%d" % r["symbol_id"], uuid=str(int(r["uuid_id"])), oid=str(int(r["oid_id"])),
        transaction=int(r["side"])), int(r["action"]), float(r["price_fx"]), float(r["volume_fx"]), 8).encode() for r in rec]
for th in [int(x) for x in (sys.argv[1:] or [1, 8])]:
    pre, names = PrePool(), Names()
    for r in rec:
        if r["action"] == wl.ADD: pre.set("s%d" % r["symbol_id"], str(int(r["uuid_id"])), str(int(r["oid_id"])))
    cons = BatchingConsumer(type("E", (), {"max_batch": 1 << 16, "max_symbols": 100000})(), pre, MatchSink(), names, threads=th)
    q = PackedQueue(msgs)
    t = time.perf_counter()
    for b in q.batches(1 << 15):
        cons.records(b); pre.commit()
    w = time.perf_counter() - t
    print(th, round(w * 1e3, 1), "ms", {k: round(v * 1e3, 1) for k, v in cons.phase_s.items() if k.startswith("native")}, "parallel", cons.parallel_batches)
