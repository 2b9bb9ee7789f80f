"""Batching consumer, gRPC-ingress admission markers and the matchOrder sink — the host side of
the drop-in (SURVEY.md §8 rows a4, a7, a15, f1 minus Go, f3).

The reference runs one consumer goroutine that takes one `doOrder` message at a time
(gomengine/engine/rabbitmq.go:116-125: json.Unmarshal into an OrderNode, then DoOrder) and
publishes every MatchResult to `matchOrder` (engine.go:109-113,154-194), which a sink process
decodes and logs (rabbitmq.go:132-177).  Admission uses the pre-pool marker S:comparison: the
gRPC DoOrder handler sets it before enqueueing (main.go:39-52, nodepool.go:14-16); the consumer
tests and clears it for an ADD (engine.go:58-62) and clears it for a DEL (engine.go:90).

Here:
  * PrePool       the S:comparison markers, shared by the ingress and the consumer (thread-safe);
  * Ingress       the gRPC Order service counterpart (main.go:39-64): NewOrderNode scaling
                  (gome_fixed_from_double, exact decimal), marker, OrderNode JSON to the queue;
  * BatchingConsumer  drains up to `max_batch` messages or `max_wait_us` after the first one,
                  decodes the OrderNode JSON, converts the already-scaled Price / Volume with
                  gome_fixed_from_scaled (no second scaling), interns Symbol / Uuid / Oid and
                  Transaction codes, resolves admission against PrePool at drain time in queue
                  order (exactly when the reference would consume each message) and hands the
                  verdicts to the engine (GOME_ORD_ADM_HOST), submits the batch, and publishes
                  the rendered MatchResults (gome_render_events, byte-identical Go
                  encoding/json) to the sink in publish order;
  * MatchSink     the matchOrder queue plus ConsumeMatchOrder's decode-and-log.

A message whose JSON does not decode is consumed and ignored (the reference decodes into a
zero OrderNode, whose Action 0 DoOrder ignores).  A message whose Price / Volume is not an
exact scaled integer below 2^53 (quirk Q5) is outside the parity domain: it is counted in
`rejected` and not submitted.
"""
from __future__ import annotations

import ctypes as C
import json
import queue as _queue
import threading
import time

import numpy as np

from .abi import (GOME_ORD_ADM_HOST, GOME_ORD_ADMITTED, GomeError, fixed_from_double,
                  fixed_from_scaled, load_library)
from .workload import ADD, DEL, ORDER_DTYPE


class Names:
    """Host interning: symbol / uuid / oid strings <-> u32 ids, Transaction int32 <-> code."""

    def __init__(self):
        self.fwd = {"sym": {}, "uuid": {}, "oid": {}}
        self.rev = {"sym": [], "uuid": [], "oid": []}
        self._c = {k: [] for k in self.rev}  # bytes kept alive for the C string tables
        self._tab = {k: None for k in self.rev}
        self.tx_fwd = {0: 0, 1: 1}
        self.tx_rev = [0, 1]
        self._txa = None

    def id(self, kind: str, s: str) -> int:
        d = self.fwd[kind]
        i = d.get(s)
        if i is None:
            i = d[s] = len(self.rev[kind])
            self.rev[kind].append(s)
            self._c[kind].append(s.encode())
            self._tab[kind] = None
        return i

    def name(self, kind: str, i: int) -> str:
        return self.rev[kind][i]

    def tx_code(self, raw: int) -> int:
        raw = int(raw)
        c = self.tx_fwd.get(raw)
        if c is None:
            if len(self.tx_rev) == 256:
                raise GomeError(1, "more than 254 distinct Transaction values outside {0, 1}")
            c = self.tx_fwd[raw] = len(self.tx_rev)
            self.tx_rev.append(raw)
            self._txa = None
        return c

    def tx_raw(self, code: int) -> int:
        return self.tx_rev[code] if code < len(self.tx_rev) else code

    def table(self, kind: str):
        t = self._tab[kind]
        if t is None:
            t = self._tab[kind] = (C.c_char_p * max(1, len(self._c[kind])))(*self._c[kind])
        return t

    def tx_array(self) -> np.ndarray:
        if self._txa is None:
            a = np.arange(256, dtype=np.int32)
            a[:len(self.tx_rev)] = self.tx_rev
            self._txa = a
        return self._txa


class PrePool:
    """S:comparison (nodepool.go:14-28): markers keyed (symbol, uuid, oid)."""

    def __init__(self):
        self._s: set = set()
        self._lock = threading.Lock()

    def set(self, symbol: str, uuid: str, oid: str):  # SetPrePool (main.go:44-45)
        with self._lock:
            self._s.add((symbol, uuid, oid))

    def consume_add(self, symbol: str, uuid: str, oid: str) -> bool:
        """ExistsPrePool + DeletePrePool at consume time (engine.go:58-62)."""
        with self._lock:
            k = (symbol, uuid, oid)
            if k in self._s:
                self._s.discard(k)
                return True
            return False

    def consume_del(self, symbol: str, uuid: str, oid: str):  # DeletePrePool (engine.go:90)
        with self._lock:
            self._s.discard((symbol, uuid, oid))

    def __len__(self):
        return len(self._s)


def _order_node_json(req: dict, action: int, price: float, volume: float, accuracy: int) -> str:
    """OrderNode (ordernode.go:9-36) as the doOrder message; key fields as NewOrderNode sets them
    (ordernode.go:89-117).  The consumer only needs the decoded values."""
    S, sale = req["symbol"], int(req["transaction"]) == 1
    P = str(int(price))
    node = {"Action": action, "Uuid": req["uuid"], "Oid": req["oid"], "Symbol": S,
            "Transaction": int(req["transaction"]), "Price": price, "Volume": volume,
            "Accuracy": accuracy, "NodeName": f"{S}:node:{req['oid']}", "IsFirst": False,
            "IsLast": False, "PrevNode": "", "NextNode": "", "NodeLink": f"{S}:link:{P}",
            "OrderHashKey": f"{S}:comparison", "OrderHashField": f"{S}:{req['uuid']}:{req['oid']}",
            "OrderListZsetKey": f"{S}:{'SALE' if sale else 'BUY'}",
            "OrderListZsetRKey": f"{S}:{'BUY' if sale else 'SALE'}",
            "OrderDepthHashKey": f"{S}:depth", "OrderDepthHashField": f"{S}:depth:{P}"}
    return json.dumps(node, separators=(",", ":"))


class Ingress:
    """gRPC `Order` service counterpart (api/order.proto:26-29, main.go:39-64): replies before
    matching; DoOrder sets the marker then enqueues, DeleteOrder only enqueues."""

    def __init__(self, out_queue, prepool: PrePool, accuracy: int = 8):
        self.q, self.pre, self.acc = out_queue, prepool, accuracy

    def _put(self, msg: str):
        (self.q.put if hasattr(self.q, "put") else self.q.append)(msg)

    def do_order(self, req: dict) -> dict:
        p = float(fixed_from_double(req["price"], self.acc))  # NewOrderNode (ordernode.go:76-87)
        v = float(fixed_from_double(req["volume"], self.acc))
        self.pre.set(req["symbol"], req["uuid"], req["oid"])
        self._put(_order_node_json(req, ADD, p, v, self.acc))
        return {"code": 0, "message": "下单执行成功"}

    def delete_order(self, req: dict) -> dict:
        p = float(fixed_from_double(req["price"], self.acc))
        v = float(fixed_from_double(req["volume"], self.acc))
        self._put(_order_node_json(req, DEL, p, v, self.acc))
        return {"code": 0, "message": "删除执行开始成功"}


class MatchSink:
    """The matchOrder queue and its consumer (rabbitmq.go:132-177: decode and log)."""

    def __init__(self, log=None):
        self.q: list[str] = []
        self.log = log
        self.lock = threading.Lock()

    def publish_many(self, lines):
        with self.lock:
            self.q.extend(lines)

    def consume(self) -> list[dict]:
        with self.lock:
            out, self.q = self.q, []
        res = [json.loads(x) for x in out]
        if self.log:
            for r in res:
                self.log(f"撮合结果------：{r}")
        return res


class BatchingConsumer:
    """Replaces ConsumeNewOrder (rabbitmq.go:86-130) in front of one engine handle."""

    def __init__(self, engine, prepool: PrePool, sink: MatchSink, names: Names | None = None,
                 max_batch: int | None = None, max_wait_us: int = 200, accuracy: int = 8):
        self.eng, self.pre, self.sink = engine, prepool, sink
        self.names = names or Names()
        self.max_batch = int(max_batch or engine.max_batch)
        self.max_wait = max_wait_us * 1e-6
        self.acc = accuracy
        self.lib = load_library()
        self.lib.gome_render_events.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_uint64,
                                                C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                                C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t]
        self.lib.gome_render_events.restype = C.c_int64
        self.seq = 0
        self.consumed = self.rejected = self.batches = 0
        self._buf = C.create_string_buffer(1 << 20)

    # ---- draining ------------------------------------------------------------------
    def drain(self, q, block_s: float = 0.0) -> list:
        """Up to max_batch messages: the first waits up to block_s, the rest until max_wait_us
        after the first (a list-like queue is drained without waiting)."""
        if isinstance(q, list):
            msgs, q[:] = q[:self.max_batch], q[self.max_batch:]
            return msgs
        try:
            msgs = [q.get(timeout=block_s) if block_s else q.get_nowait()]
        except _queue.Empty:
            return []
        deadline = time.perf_counter() + self.max_wait
        while len(msgs) < self.max_batch:
            try:
                msgs.append(q.get_nowait())
            except _queue.Empty:
                if time.perf_counter() >= deadline:
                    break
                time.sleep(0)
        return msgs

    # ---- one batch -------------------------------------------------------------------
    def records(self, msgs) -> np.ndarray:
        """Decode, convert and admit (in queue order) -> gome_order records."""
        N = self.names
        rec = np.zeros(len(msgs), ORDER_DTYPE)
        keep = np.ones(len(msgs), bool)
        for i, body in enumerate(msgs):
            try:
                o = json.loads(body)
                act = int(o.get("Action", 0))
                sym, uuid, oid = str(o.get("Symbol", "")), str(o.get("Uuid", "")), str(o.get("Oid", ""))
                tx = int(o.get("Transaction", 0))
                price, vol = o.get("Price", 0.0), o.get("Volume", 0.0)
            except (ValueError, TypeError, AttributeError):
                rec[i]["action"] = 0  # zero OrderNode: DoOrder ignores it
                continue
            if act in (ADD, DEL):
                try:
                    p, v = fixed_from_scaled(price), fixed_from_scaled(vol)
                except GomeError:
                    keep[i] = False  # Q5: outside the exact domain
                    self.rejected += 1
                    if act == ADD:
                        self.pre.consume_add(sym, uuid, oid)
                    else:
                        self.pre.consume_del(sym, uuid, oid)
                    continue
            else:
                p = v = 0
            r = rec[i]
            r["price_fx"], r["volume_fx"] = p, v
            r["symbol_id"], r["uuid_id"], r["oid_id"] = N.id("sym", sym), N.id("uuid", uuid), N.id("oid", oid)
            r["side"] = N.tx_code(tx)
            r["action"] = act & 0xFF if 0 <= act < 256 else 0
            if act == ADD:
                ok = self.pre.consume_add(sym, uuid, oid)
                r["flags"] = GOME_ORD_ADM_HOST | (GOME_ORD_ADMITTED if ok else 0)
            elif act == DEL:
                self.pre.consume_del(sym, uuid, oid)
                r["flags"] = GOME_ORD_ADM_HOST
        return rec[keep]

    def render(self, ev: np.ndarray, rec: np.ndarray, seq_base: int) -> list[str]:
        N = self.names
        while True:
            k = self.lib.gome_render_events(
                ev.ctypes.data, len(ev), rec.ctypes.data, len(rec), seq_base, self.acc,
                C.cast(N.table("sym"), C.c_void_p), len(N.rev["sym"]),
                C.cast(N.table("uuid"), C.c_void_p), len(N.rev["uuid"]),
                C.cast(N.table("oid"), C.c_void_p), len(N.rev["oid"]),
                N.tx_array().ctypes.data, self._buf, len(self._buf))
            if k >= 0:
                break
            if k == -(1 << 63):
                raise GomeError(1, "event references an unknown id")
            self._buf = C.create_string_buffer(int(-k) + (1 << 20))
        return self._buf.raw[:k].decode().split("\n")[:-1]

    def process(self, msgs) -> int:
        """Apply one drained batch; returns the MatchResults published."""
        self.consumed += len(msgs)
        rec = self.records(msgs)
        if len(rec) == 0:
            return 0
        if len(rec) > self.eng.max_batch:
            raise GomeError(1, "batch larger than the engine's max_batch")
        base = self.seq
        self.eng.submit(rec, seq_base=base)
        self.seq += len(rec)
        ev = self.eng.drain()
        lines = self.render(ev, rec, base)
        self.sink.publish_many(lines)
        self.batches += 1
        return len(lines)

    def poll(self, q, block_s: float = 0.0) -> int:
        msgs = self.drain(q, block_s)
        return self.process(msgs) if msgs else 0

    def run(self, q, stop: threading.Event, block_s: float = 0.05):
        """The consumer loop (one thread per engine handle, as the reference has one goroutine)."""
        while not stop.is_set():
            self.poll(q, block_s)
