"""Where the consumer leg's submit time goes, per batch (GPU): bench.consumer_leg's stream through
BatchingConsumer.process_stream with each gome_submit_batch_async timed on its own (wall and the
calling thread's CPU time), twice on the same engine (cold, then warm), at depth 2 and 1.
  python tools/consumer_submit_probe.py [workload ...]"""
import sys, time; sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench
from gome_amd import abi
from gome_amd import workload as wl
from gome_amd.consumer import BatchingConsumer, MatchSink, Names, PrePool, PackedQueue, _order_node_json

orig = abi.Engine.submit_async
log = []


def timed(self, *a, **k):
    t, c = time.perf_counter(), time.thread_time()
    r = orig(self, *a, **k)
    log.append((round((time.perf_counter() - t) * 1e3, 2), round((time.thread_time() - c) * 1e3, 2)))
    return r


abi.Engine.submit_async = timed
for w in sys.argv[1:] or ["config2", "config3"]:
    n_sym, n, B = bench.WORKLOADS[w]["symbols"], 1 << 17, 1 << 15
    gen, _, _ = bench.make_stream(w, 0, 1, 7)
    rec = gen(2 * n).copy()
    msgs = [_order_node_json(dict(symbol="s%d" % r["symbol_id"], uuid=str(int(r["uuid_id"])), oid=str(int(r["oid_id"])),
                                  transaction=int(r["side"])), int(r["action"]), float(r["price_fx"]),
                             float(r["volume_fx"]), 8).encode() for r in rec]
    for depth in (2, 1):
        pre, names = PrePool(), Names()
        for r in rec:
            if r["action"] == wl.ADD:
                pre.set("s%d" % r["symbol_id"], str(int(r["uuid_id"])), str(int(r["oid_id"])))
        eng = abi.Engine(max_symbols=n_sym, max_batch=B, max_nodes=4 * n + (1 << 20), max_levels=(1 << 22) + 4 * n)
        cons = BatchingConsumer(eng, pre, MatchSink(), names, max_batch=B, threads=8)
        for half in range(2):
            log.clear()
            for k in cons.phase_s:
                cons.phase_s[k] = 0.0
            q = PackedQueue(msgs[half * n:(half + 1) * n])
            t = time.perf_counter()
            cons.process_stream(q.batches(B), depth=depth)
            wall = time.perf_counter() - t
            print(w, "depth", depth, "cold" if half == 0 else "warm", round(n / wall), "msg/s",
                  {k: round(v * 1e3, 1) for k, v in cons.phase_s.items()}, "submits (wall, cpu) ms:", log, flush=True)
        eng.close()
