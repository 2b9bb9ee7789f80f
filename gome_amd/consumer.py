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

import codecs
import ctypes as C
import json
import math
import queue as _queue
import re
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

    def stage(self) -> "StagedMarkers":
        return StagedMarkers(self)

    def commit(self, consumed: set):
        """Remove the markers a staged batch consumed (after the engine accepted the batch)."""
        with self._lock:
            self._s -= consumed

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


class StagedMarkers:
    """One batch's admission verdicts against the pre-pool, in queue order, without consuming
    anything yet: an ADD is admitted iff its marker exists and no earlier record of the batch
    consumed it (ExistsPrePool + DeletePrePool, engine.go:58-62,90)."""

    def __init__(self, pool: PrePool):
        self.pool, self.consumed = pool, set()

    def consume_add(self, symbol: str, uuid: str, oid: str) -> bool:
        k = (symbol, uuid, oid)
        if k in self.consumed:
            return False
        with self.pool._lock:
            ok = k in self.pool._s
        if ok:
            self.consumed.add(k)
        return ok

    def consume_del(self, symbol: str, uuid: str, oid: str):
        with self.pool._lock:
            if (symbol, uuid, oid) in self.pool._s:
                self.consumed.add((symbol, uuid, oid))

    def commit(self):
        self.pool.commit(self.consumed)
        self.consumed = set()


# ---- Go encoding/json Unmarshal of the consumed OrderNode (ordernode.go:9-36) -----------------
# Only the fields the engine reads; the key fields (OrderHashKey, NodeName, ...) are the ones
# NewOrderNode derives from them at gRPC time (ordernode.go:89-117).
_GO_FIELDS = {"action": ("Action", "i", 8), "uuid": ("Uuid", "s", 0), "oid": ("Oid", "s", 0),
              "symbol": ("Symbol", "s", 0), "transaction": ("Transaction", "i", 32),
              "price": ("Price", "f", 0), "volume": ("Volume", "f", 0)}


_LONE_SURROGATE = re.compile("[\ud800-\udfff]")


class _Lit(str):
    """Literal text of a JSON number (Go converts numbers from the literal)."""


class _Pairs(list):
    """A JSON object's (key, value) pairs in document order."""


def _reject_constant(tok):
    raise ValueError(tok)  # NaN / Infinity are not JSON to Go


def _go_bytes_to_str(body) -> str:
    """Go's encoding/json replaces every byte of invalid UTF-8 with U+FFFD, one per byte
    (utf8.DecodeRune returns (RuneError, 1)); Python's 'replace' would merge a truncated sequence."""
    return body.decode("utf-8", errors="gome_go_bytes")


def _go_replace(exc):
    return "\ufffd", exc.start + 1


codecs.register_error("gome_go_bytes", _go_replace)


def decode_order_node(body) -> dict:
    """The OrderNode fields json.Unmarshal leaves: {"Action", "Uuid", "Oid", "Symbol",
    "Transaction", "Price", "Volume"}.  Never raises.  Keys match exactly or case-insensitively
    (Go's field matching); later duplicates win; an int field takes only an integer literal
    within its width (Action int8, Transaction int32), a float field any finite number, a
    string field only a string; anything else (and null) leaves the zero value."""
    out = {"Action": 0, "Uuid": "", "Oid": "", "Symbol": "", "Transaction": 0, "Price": 0.0, "Volume": 0.0}
    if isinstance(body, (bytes, bytearray, memoryview)):
        body = _go_bytes_to_str(bytes(body))
    try:
        doc = json.loads(body, parse_int=_Lit, parse_float=_Lit, parse_constant=_reject_constant,
                         object_pairs_hook=_Pairs)
    except (ValueError, TypeError, RecursionError):
        return out  # syntax error: Unmarshal decodes nothing
    if not isinstance(doc, _Pairs):
        return out
    for key, val in doc:
        f = _GO_FIELDS.get(key.casefold())  # (Unicode folding, as Go's EqualFold: 'ſ' ~ 's')
        if f is None or val is None:
            continue
        name, kind, bits = f
        if kind == "s":
            if isinstance(val, str) and not isinstance(val, _Lit):
                out[name] = _LONE_SURROGATE.sub("\ufffd", val)  # Go decodes a lone \\uD8xx as U+FFFD
        elif isinstance(val, _Lit):
            if kind == "f":
                x = float(val)
                if not math.isinf(x):  # ParseFloat out of range: UnmarshalTypeError, skipped
                    out[name] = x
            else:
                try:
                    x = int(val, 10)  # ParseInt: no fraction, no exponent
                except ValueError:
                    continue
                if -(1 << (bits - 1)) <= x < (1 << (bits - 1)):
                    out[name] = x
    return out


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
        self.max_symbols = getattr(engine, "max_symbols", None)
        self.seq = 0
        self.consumed = self.rejected = self.batches = self.dups = 0
        self._staged = None
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
        """Decode, convert and admit (in queue order) -> gome_order records.  The admission
        verdicts come from a staged view of the pre-pool (committed by process() once the
        engine took the batch)."""
        N = self.names
        pre = self._staged = self.pre.stage()
        rec = np.zeros(len(msgs), ORDER_DTYPE)
        keep = np.ones(len(msgs), bool)
        for i, body in enumerate(msgs):
            o = decode_order_node(body)
            act, sym, uuid, oid = o["Action"], o["Symbol"], o["Uuid"], o["Oid"]
            if act not in (ADD, DEL):
                continue  # DoOrder ignores any other Action (engine.go:46-54): a zero record
            try:
                p, v = fixed_from_scaled(o["Price"]), fixed_from_scaled(o["Volume"])
                if v < 0:  # (the engine's record domain: volume >= 0, gome_abi.h)
                    raise GomeError(1, "negative Volume")
                if self.max_symbols is not None and N.fwd["sym"].get(sym, len(N.rev["sym"])) >= self.max_symbols:
                    raise GomeError(1, "more distinct Symbols than the engine's max_symbols")
                code = N.tx_code(o["Transaction"])
            except GomeError:
                # outside the parity domain (Q5, a negative Volume), or beyond the engine's symbol
                # range or Transaction code space: not submitted, so it cannot refuse the batch
                keep[i] = False
                self.rejected += 1
                if act == ADD:
                    pre.consume_add(sym, uuid, oid)
                else:
                    pre.consume_del(sym, uuid, oid)
                continue
            r = rec[i]
            r["price_fx"], r["volume_fx"] = p, v
            r["symbol_id"], r["uuid_id"], r["oid_id"] = N.id("sym", sym), N.id("uuid", uuid), N.id("oid", oid)
            r["side"] = code
            r["action"] = act
            if act == ADD:
                ok = pre.consume_add(sym, uuid, oid)
                r["flags"] = GOME_ORD_ADM_HOST | (GOME_ORD_ADMITTED if ok else 0)
            else:
                pre.consume_del(sym, uuid, oid)
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
        """Apply one drained batch; returns the MatchResults published.  Raises only when the
        engine refuses the batch (GomeError, e.g. E_CAPACITY before anything was applied); the
        pre-pool is then untouched and the same messages can be processed again."""
        rec = self.records(msgs)
        if len(rec) > self.eng.max_batch:
            raise GomeError(1, "batch larger than the engine's max_batch")
        base = self.seq
        if len(rec):
            self.eng.submit(rec, seq_base=base)
        self._staged.commit()  # the engine took the batch: its markers are consumed
        self.consumed += len(msgs)
        if len(rec) == 0:
            return 0
        self.seq += len(rec)
        self.dups += int(self.eng.stats()["n_dup_oid"])
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
