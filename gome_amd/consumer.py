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

Decoding follows Go's json.Unmarshal into an OrderNode (rabbitmq.go:118-124 prints the error
and still calls DoOrder): a syntax error decodes nothing (a zero OrderNode, whose Action 0
DoOrder ignores); otherwise each field whose JSON value fits its Go type is set and any other
field (wrong type, overflow, null) stays zero, so `"Price":"abc"` is an order at price 0.
`process()` never raises on message content.  A message outside the parity domain is counted
in `rejected` and not submitted: a Price / Volume that is not an exact scaled integer below
2^53 (quirk Q5), a negative Volume, a Symbol beyond the engine's max_symbols distinct symbols,
or a 255th distinct Transaction value outside {0, 1} (the engine carries Transaction as a
one-byte code, gome_abi.h).  Raw bytes decode as Go does: invalid UTF-8 becomes U+FFFD, one
per byte.  The engine applies the duplicate-oid rule (Q7,
gome_abi.h) to the admitted ADDs; `dups` counts them.

Admission markers are resolved against a staged view of the pre-pool and the consumption is
committed only once the engine accepted the batch: a batch the engine refuses (for example
GOME_E_CAPACITY before anything is applied) can be resubmitted with the same verdicts.
"""
from __future__ import annotations

import ctypes as C
import json
import queue as _queue
import threading
import time

import numpy as np

from .abi import GomeError, fixed_from_double, load_library
from .workload import ADD, DEL, ORDER_DTYPE


_KIND = {"sym": 0, "uuid": 1, "oid": 2}  # GOME_NAME_SYMBOL / _UUID / _OID (gome_host.h)


def _b(s) -> bytes:
    return s if isinstance(s, (bytes, bytearray)) else str(s).encode("utf-8", "surrogatepass")


class Names:
    """Host interning (gome_names, gome_host.h): symbol / uuid / oid strings <-> u32 ids,
    Transaction int32 <-> one-byte code."""

    def __init__(self):
        self.lib = load_library()
        self.h = self.lib.gome_names_create()
        if not self.h:
            raise MemoryError("gome_names_create")

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.gome_names_destroy(self.h)
            self.h = None

    def id(self, kind: str, s: str) -> int:
        b = _b(s)
        i = self.lib.gome_names_intern(self.h, _KIND[kind], b, len(b))
        if i < 0:
            raise GomeError(1, "gome_names_intern failed")
        return i

    def find(self, kind: str, s: str) -> int:
        b = _b(s)
        return self.lib.gome_names_find(self.h, _KIND[kind], b, len(b))

    def name(self, kind: str, i: int) -> str:
        n = C.c_size_t()
        p = self.lib.gome_names_get(self.h, _KIND[kind], int(i), C.byref(n))
        if not p:
            raise IndexError(f"{kind} id {i}")
        return C.string_at(p, n.value).decode("utf-8", "surrogatepass")

    def count(self, kind: str) -> int:
        return self.lib.gome_names_count(self.h, _KIND[kind])

    def tx_code(self, raw: int) -> int:
        c = self.lib.gome_names_tx_code(self.h, int(raw))
        if c < 0:
            raise GomeError(1, "more than 254 distinct Transaction values outside {0, 1}")
        return c

    def tx_raw(self, code: int) -> int:
        return int(self.tx_array()[code])

    def table(self, kind: str):
        """The NUL-terminated strings by id (gome_render_events' tables; valid until the next id)."""
        return C.c_void_p(self.lib.gome_names_table(self.h, _KIND[kind]))

    def tx_array(self) -> np.ndarray:
        """The raw Transaction of every code (a view of the native table)."""
        return np.ctypeslib.as_array(self.lib.gome_names_tx_table(self.h), shape=(256,))


class PrePool:
    """S:comparison (nodepool.go:14-28): markers keyed (symbol, uuid, oid) (gome_prepool,
    gome_host.h; markers may be set from any thread).  The consumer consumes them staged
    (gome_consume_order_nodes) and commits once the engine took the batch."""

    def __init__(self):
        self.lib = load_library()
        self.h = self.lib.gome_prepool_create()
        if not self.h:
            raise MemoryError("gome_prepool_create")

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.gome_prepool_destroy(self.h)
            self.h = None

    @staticmethod
    def _key(symbol, uuid, oid):
        a, b, c = _b(symbol), _b(uuid), _b(oid)
        return a, len(a), b, len(b), c, len(c)

    def set(self, symbol: str, uuid: str, oid: str):  # SetPrePool (main.go:44-45)
        self.lib.gome_prepool_set(self.h, *self._key(symbol, uuid, oid))

    def consume_add(self, symbol: str, uuid: str, oid: str) -> bool:
        """ExistsPrePool + DeletePrePool at consume time (engine.go:58-62)."""
        return self.lib.gome_prepool_take(self.h, *self._key(symbol, uuid, oid)) != 0

    def consume_del(self, symbol: str, uuid: str, oid: str):  # DeletePrePool (engine.go:90)
        self.lib.gome_prepool_take(self.h, *self._key(symbol, uuid, oid))

    def commit(self):
        """Remove the markers the last consumed batch took (the engine accepted it)."""
        self.lib.gome_prepool_commit(self.h)

    def abort(self):
        """Forget the last consumed batch's provisional consumption (the engine refused it)."""
        self.lib.gome_prepool_abort(self.h)

    def __len__(self):
        return self.lib.gome_prepool_size(self.h)


# ---- Go encoding/json Unmarshal of the consumed OrderNode (ordernode.go:9-36) -----------------
# Native (gome_decode_order_nodes / gome_consume_order_nodes, gome_host.h): only the fields the
# engine reads; the key fields (OrderHashKey, NodeName, ...) are the ones NewOrderNode derives
# from them at gRPC time (ordernode.go:89-117).
class _Decoded(C.Structure):
    _fields_ = [("price", C.c_double), ("volume", C.c_double), ("transaction", C.c_int32), ("action", C.c_int8),
                ("is_object", C.c_uint8), ("pad", C.c_uint16), ("sym_off", C.c_uint32), ("sym_len", C.c_uint32),
                ("uuid_off", C.c_uint32), ("uuid_len", C.c_uint32), ("oid_off", C.c_uint32), ("oid_len", C.c_uint32)]


class ConsumeStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("messages", "records", "rejected", "ignored", "not_objects", "admitted",
                                          "ns_decode", "ns_prepare", "ns_queue", "queue_parallel")]


def pack_messages(msgs):
    """(one buffer, offsets[n + 1]) of the message bodies (bytes as they are; str as UTF-8)."""
    bodies = [m if isinstance(m, bytes) else _b(m) for m in msgs]
    off = np.zeros(len(bodies) + 1, np.uint64)
    if bodies:
        np.cumsum(np.fromiter(map(len, bodies), np.uint64, len(bodies)), out=off[1:])
    return b"".join(bodies), off


class PackedQueue:
    """doOrder deliveries as one buffer of bodies plus offsets (how an AMQP client reads them off its
    socket): batches are (buf, offsets[k:k + m + 1]) views, no per-message objects and no copy."""

    def __init__(self, msgs):
        self.buf, self.off = pack_messages(msgs)

    def __len__(self):
        return len(self.off) - 1

    def batches(self, m: int):
        for k in range(0, len(self), m):
            yield self.buf, self.off[k:min(k + m, len(self)) + 1]


def decode_order_nodes(msgs, threads: int = 0) -> list[dict]:
    """json.Unmarshal of each body into an OrderNode, the fields the engine reads: {"Action",
    "Uuid", "Oid", "Symbol", "Transaction", "Price", "Volume"} (gome_decode_order_nodes).  Keys
    match exactly or case-insensitively (Go's foldName); later duplicates win; an int field takes
    only an integer literal within its width (Action int8, Transaction int32), a float field any
    finite number, a string field only a string; anything else (and null) leaves the zero value; a
    syntax error or a non-object decodes nothing."""
    lib = load_library()
    buf, off = pack_messages(msgs)
    n = len(off) - 1
    out = (_Decoded * max(n, 1))()
    cap = 3 * len(buf) + 1
    sb = C.create_string_buffer(cap)
    used = lib.gome_decode_order_nodes(buf, off.ctypes.data, n, threads, out, sb, cap)
    if used < 0:
        raise GomeError(1, "gome_decode_order_nodes failed")
    raw = sb.raw
    res = []
    for k in range(n):
        d = out[k]
        st = lambda o, ln: raw[o:o + ln].decode("utf-8", "surrogatepass")  # noqa: E731
        res.append({"Action": d.action, "Uuid": st(d.uuid_off, d.uuid_len), "Oid": st(d.oid_off, d.oid_len),
                    "Symbol": st(d.sym_off, d.sym_len), "Transaction": d.transaction, "Price": d.price,
                    "Volume": d.volume})
    return res


def decode_order_node(body) -> dict:
    return decode_order_nodes([body])[0]


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
    """The matchOrder queue and its consumer (rabbitmq.go:132-177: decode and log).  Rendered batches
    arrive as blocks of newline-terminated MatchResult lines (one message each) and stay bytes until
    something reads them (`q`, consume): splitting each batch into Python strings on the consumer's
    thread cost more than the native render itself."""

    def __init__(self, log=None):
        self._q: list[str] = []
        self._blocks: list[bytes] = []
        self.published = 0  # messages published
        self.log = log
        self.lock = threading.Lock()

    def publish_many(self, lines):
        with self.lock:
            self._flush()
            self._q.extend(lines)
            self.published += len(lines)

    def publish_block(self, block, n: int):
        """n newline-terminated lines, in publish order (bytes or a buffer the sink now owns)."""
        with self.lock:
            self._blocks.append(block)
            self.published += n

    def _flush(self):
        for b in self._blocks:
            self._q.extend(bytes(b).decode().split("\n")[:-1])
        self._blocks.clear()

    @property
    def q(self) -> list[str]:
        """The queued MatchResult lines (str), oldest first."""
        with self.lock:
            self._flush()
            return self._q

    @q.setter
    def q(self, v):
        with self.lock:
            self._blocks.clear()
            self._q = list(v)

    def consume(self) -> list[dict]:
        with self.lock:
            self._flush()
            out, self._q = self._q, []
        res = [json.loads(x) for x in out]
        if self.log:
            for r in res:
                self.log(f"撮合结果------：{r}")
        return res


class BatchingConsumer:
    """Replaces ConsumeNewOrder (rabbitmq.go:86-130) in front of one engine handle.  The per-message
    work is native (gome_consume_order_nodes: Go-Unmarshal decode on `threads` threads, conversion,
    interning, admission in queue order; gome_render_events_mt: the MatchResult lines)."""

    def __init__(self, engine, prepool: PrePool, sink: MatchSink, names: Names | None = None,
                 max_batch: int | None = None, max_wait_us: int = 200, accuracy: int = 8, threads: int = 8,
                 render_threads: int | None = None):
        self.eng, self.pre, self.sink = engine, prepool, sink
        self.names = names or Names()
        self.max_batch = int(max_batch or engine.max_batch)
        self.max_wait = max_wait_us * 1e-6
        self.acc = accuracy
        self.threads = threads
        # (the render's pool: as many threads as the decode's by default -- half measured slower on
        # the GPU box, the render then outlasting the next batch's decode, gpurun_out/r06v)
        self.render_threads = render_threads or threads
        self.lib = load_library()
        self.max_symbols = getattr(engine, "max_symbols", None)
        self.seq = 0
        self.consumed = self.rejected = self.batches = self.dups = 0
        # process_stream's host time per phase (s): decode + admission, submit, collect (waits for
        # the device), render
        self.phase_s = {"records": 0.0, "submit": 0.0, "collect": 0.0, "render": 0.0,
                        "native_decode": 0.0, "native_prepare": 0.0, "native_queue": 0.0}
        self.parallel_batches = 0  # (batches whose queue-order work ran shard by shard)
        # the parallel queue-order path's steps (s, summed over batches; gome_consume_last_steps)
        self.queue_steps_s = [0.0] * 10

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
    def records(self, msgs, out: np.ndarray | None = None) -> np.ndarray:
        """Decode, convert and admit (in queue order) -> gome_order records.  The pre-pool markers
        are consumed staged (process() commits them once the engine took the batch).  A message
        outside the engine's domain is counted in `rejected` and not submitted; an Action other
        than ADD / DEL (a syntax error included) is a zero record, as DoOrder ignores it.
        msgs: the message bodies, or one packed delivery buffer (buf, offsets[n + 1]) (PackedQueue);
        out: where the records go (e.g. a page-locked buffer of the engine's, >= n records)."""
        self.pre.abort()  # (a batch refused earlier left nothing behind)
        buf, off = msgs if isinstance(msgs, tuple) else pack_messages(msgs)
        n = len(off) - 1
        rec = np.zeros(n, ORDER_DTYPE) if out is None else out
        got, st = C.c_size_t(), ConsumeStats()
        s = self.lib.gome_consume_order_nodes(self.names.h, self.pre.h, buf, off.ctypes.data, n,
                                              int(self.max_symbols or 0), self.threads, rec.ctypes.data, None,
                                              C.byref(got), C.byref(st))
        if s != 0:
            raise GomeError(s, "gome_consume_order_nodes failed")
        self.rejected += st.rejected
        for k in ("decode", "prepare", "queue"):  # (the native call's own split, seconds)
            self.phase_s["native_" + k] += getattr(st, "ns_" + k) * 1e-9
        self.parallel_batches += int(st.queue_parallel)
        steps = (C.c_uint64 * len(self.queue_steps_s))()
        self.lib.gome_consume_last_steps(self.names.h, steps, len(steps))
        for i, v in enumerate(steps):
            self.queue_steps_s[i] += v * 1e-9
        return rec[:got.value]

    def render_block(self, ev: np.ndarray, rec: np.ndarray, seq_base: int):
        """The batch's MatchResult lines (newline-terminated), rendered straight into a buffer of
        their own that the caller keeps (a memoryview; no copy of the block afterwards)."""
        cap = 1400 * len(ev) + (1 << 16)
        while True:
            out = np.empty(cap, np.uint8)
            # (the name tables are read under the names' lock: process_stream renders on a helper
            # thread while this thread interns the next batch's names, which may move a table)
            k = self.lib.gome_render_events_names(
                ev.ctypes.data, len(ev), rec.ctypes.data, len(rec), seq_base, self.acc, self.names.h,
                self.render_threads, out.ctypes.data, cap)
            if k >= 0:
                return memoryview(out)[:k]
            if k == -(1 << 63):
                raise GomeError(1, "event references an unknown id")
            cap = int(-k) + (1 << 16)

    def render(self, ev: np.ndarray, rec: np.ndarray, seq_base: int) -> list[str]:
        return bytes(self.render_block(ev, rec, seq_base)).decode().split("\n")[:-1]

    def process(self, msgs) -> int:
        """Apply one drained batch; returns the MatchResults published.  Raises only when the
        engine refuses the batch (GomeError, e.g. E_CAPACITY before anything was applied); the
        pre-pool is then untouched and the same messages can be processed again."""
        rec = self.records(msgs)
        if len(rec) > self.eng.max_batch:
            self.pre.abort()
            raise GomeError(1, "batch larger than the engine's max_batch")
        base = self.seq
        if len(rec):
            try:
                self.eng.submit(rec, seq_base=base)
            except BaseException:
                self.pre.abort()
                raise
        self.pre.commit()  # the engine took the batch: its markers are consumed
        self.consumed += len(msgs)
        if len(rec) == 0:
            return 0
        self.seq += len(rec)
        self.dups += int(self.eng.stats()["n_dup_oid"])
        ev = self.eng.drain()
        self.sink.publish_block(self.render_block(ev, rec, base), len(ev))  # (one line per event)
        self.batches += 1
        return len(ev)

    def process_stream(self, batches, depth: int = 2) -> int:
        """Apply drained batches in order with up to `depth` of them in flight on the engine
        (gome_submit_batch_async / gome_collect): batch k+1's decode, admission and H2D run while
        the device applies batch k, and batch k's MatchResults are rendered (on the renderer's own
        worker pool, by a helper thread) while batch k+2 is decoded.  Publishes exactly what
        process() would, batch after batch (the markers of a batch are committed when the engine
        took it, as there).  Renders queue on one helper thread (in batch order: the sink's order),
        at most two behind the collects.  The engine handle is only ever called from this thread.  Engines
        without the async calls (test doubles) take process() per batch."""
        if not hasattr(self.eng, "submit_async"):
            return sum(self.process(b) for b in batches)
        from collections import deque
        from concurrent.futures import ThreadPoolExecutor
        depth = max(1, min(depth, 3))
        RENDERS = 2  # renders queued on the helper at most (their events are copies, their records in the ring)
        # records stay valid until their batch is rendered: depth in flight, RENDERS queued or
        # rendering, one new
        ring = [self.eng.host_buffer(self.max_batch) for _ in range(depth + RENDERS + 1)]
        flight = deque()  # (records, seq base)
        pending = deque()  # the helper's renders, oldest first
        ph = self.phase_s
        clk = time.perf_counter
        total, slot = 0, 0

        def render(ev, rec, base):  # (helper thread, one batch after another: the sink's order)
            t0 = clk()
            self.sink.publish_block(self.render_block(ev, rec, base), len(ev))
            ph["render"] += clk() - t0

        def finish(ex):
            rec, base = flight.popleft()
            while len(pending) >= RENDERS:  # (a ring slot must not be reused under a render)
                pending.popleft().result()
            t0 = clk()
            # (a copy of the events, ~48 B each: the engine's buffer is the next collect's, and the
            # render need not finish before it)
            ev, st = self.eng.collect(copy=True)
            ph["collect"] += clk() - t0
            self.dups += int(st["n_dup_oid"])
            if len(ev):
                self.batches += 1
                pending.append(ex.submit(render, ev, rec, base))
            return len(ev)

        with ThreadPoolExecutor(max_workers=1) as ex:
            try:
                for msgs in batches:
                    n = (len(msgs[1]) - 1) if isinstance(msgs, tuple) else len(msgs)
                    if n > self.max_batch:
                        raise GomeError(1, "batch larger than the engine's max_batch")
                    t0 = clk()
                    rec = self.records(msgs, out=ring[slot][:n])
                    t1 = clk()
                    slot = (slot + 1) % len(ring)
                    base = self.seq
                    if len(rec):
                        try:
                            self.eng.submit_async(rec, seq_base=base)
                        except BaseException:
                            self.pre.abort()
                            raise
                    self.pre.commit()
                    ph["records"] += t1 - t0
                    ph["submit"] += clk() - t1
                    self.consumed += n
                    if len(rec):
                        self.seq += len(rec)
                        flight.append((rec, base))
                    while len(flight) >= depth:
                        total += finish(ex)
                while flight:
                    total += finish(ex)
            finally:
                while pending:
                    pending.popleft().result()
        return total

    def poll(self, q, block_s: float = 0.0) -> int:
        msgs = self.drain(q, block_s)
        return self.process(msgs) if msgs else 0

    def run(self, q, stop: threading.Event, block_s: float = 0.05):
        """The consumer loop (one thread per engine handle, as the reference has one goroutine)."""
        while not stop.is_set():
            self.poll(q, block_s)
