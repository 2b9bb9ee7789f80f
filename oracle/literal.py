"""Literal oracle: line-faithful Python transliteration of gome's matching engine.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (gome_amd/, include/) imports,
links or executes this file; only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may use oracle/.

PARITY UNPINNED: the reference (Go) ships no tests, golden vectors or fixtures
 and no Go toolchain exists in this image, so this file
cannot be checked against the reference's own outputs.  It is a restatement
that executes the same Redis command sequence the Go code issues, on an
in-memory fake of the Redis data types, so that reference quirks (shared
price-keyed FIFO, stale side membership, zero-volume fills, admission marker
races) fall out of the transliteration rather than being re-derived.

Reference files (paths relative to /root/reference):
  gomengine/engine/engine.go    DoOrder/SetOrder/DeleteOrder/Match/MatchOrder
  gomengine/engine/nodepool.go  Pool (admission marker, depth, side sets)
  gomengine/engine/nodelink.go  NodeLink (per-price doubly-linked FIFO)
  gomengine/engine/ordernode.go OrderNode + fixed-point conversion + key names
  gomengine/engine/rabbitmq.go  ConsumeNewOrder loop (serial, one message at a time)
  gomengine/main.go             gRPC DoOrder/DeleteOrder (marker set before enqueue)

Third-party behaviour restated here (not vendored in the reference; go.mod):
  github.com/shopspring/decimal v1.2.0  NewFromFloat (shortest round-trip decimal),
                                        Mul (exact), Float64 (nearest float64),
                                        String (plain positional, trailing zeros trimmed)
  github.com/go-redis/redis/v8 v8.0.0-beta.8  float64 args -> strconv 'f', -1
  Redis server HINCRBYFLOAT                   long double add, "%.17Lf" trimmed
  Go encoding/json                             struct field order, shortest floats,
                                               'e' form outside [1e-6, 1e21), HTML escaping;
                                               Unmarshal: syntax error -> nothing decoded,
                                               mistyped / overflowing / null field -> left
                                               zero, keys matched case-insensitively
"""
from __future__ import annotations

import json
import math
import re
from decimal import Decimal, getcontext
from fractions import Fraction

getcontext().prec = 80

ADD = 1  # engine.go:14-18
DEL = 2
BUY = 0  # api/order.proto:4-7
SALE = 1


# ---------------------------------------------------------------- formatting
def _shortest_decimal(f: float) -> Decimal:
    """Shortest round-trip decimal of a float64 (Python repr == Go 'g' -1 digits)."""
    return Decimal(repr(float(f)))


def go_fmt_f(f: float) -> str:
    """strconv.FormatFloat(f, 'f', -1, 64) (go-redis arg formatting)."""
    if f == 0:
        return "-0" if math.copysign(1.0, f) < 0 else "0"
    s = format(_shortest_decimal(f), "f")
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    return s


def decimal_string(f: float) -> str:
    """shopspring decimal.NewFromFloat(f).String() (ordernode.go:106,115)."""
    if f == 0:
        return "0"
    return go_fmt_f(f)


def go_json_float(f: float) -> str:
    """encoding/json float64 encoder: 'f' -1, or 'e' -1 outside [1e-6, 1e21)."""
    if math.isinf(f) or math.isnan(f):
        raise ValueError("json: unsupported value")
    a = abs(f)
    if a != 0 and (a < 1e-6 or a >= 1e21):
        d = _shortest_decimal(f)
        sign, digits, exp = d.as_tuple()
        ds = "".join(map(str, digits)).rstrip("0") or "0"
        e10 = exp + len(digits) - 1
        mant = ds[0] + ("." + ds[1:] if len(ds) > 1 else "")
        es = "%+03d" % e10  # Go: at least two exponent digits
        if es[1] == "0" and len(es) == 3 and es[0] == "-":
            es = "-" + es[2]  # encoding/json cleans e-09 -> e-9
        return ("-" if sign else "") + mant + "e" + es
    return go_fmt_f(f)


def go_json_string(s: str) -> str:
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        elif o < 0x20:
            out.append({"\n": "\\n", "\r": "\\r", "\t": "\\t"}.get(ch, "\\u%04x" % o))
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


# ---------------------------------------------------------------- OrderNode
NODE_FIELDS = (
    # (name, kind) in struct declaration order, ordernode.go:9-36
    ("Action", "int"), ("Uuid", "str"), ("Oid", "str"), ("Symbol", "str"),
    ("Transaction", "int"), ("Price", "float"), ("Volume", "float"),
    ("Accuracy", "int"), ("NodeName", "str"), ("IsFirst", "bool"),
    ("IsLast", "bool"), ("PrevNode", "str"), ("NextNode", "str"),
    ("NodeLink", "str"), ("OrderHashKey", "str"), ("OrderHashField", "str"),
    ("OrderListZsetKey", "str"), ("OrderListZsetRKey", "str"),
    ("OrderDepthHashKey", "str"), ("OrderDepthHashField", "str"),
)
_ZERO = {"int": 0, "str": "", "float": 0.0, "bool": False}
_INT_BITS = {"Action": 8, "Transaction": 32, "Accuracy": 64}  # int8 / int32 / int (ordernode.go:10-16)


class _Num(str):
    """A JSON number's literal text (Go decodes numbers from the literal)."""


class _Obj(list):
    """A JSON object as its (key, value) pairs in order."""


def _no_constant(name):
    raise ValueError(f"invalid character in JSON: {name}")  # Go has no NaN / Infinity literals


def _go_field_value(kind: str, name: str, v):
    """encoding/json's literalStore for one struct field (go1.x decode.go): returns the value, or
    None when Go leaves the field unchanged (null, or an UnmarshalTypeError it records and skips)."""
    if v is None:
        return None  # null into a non-pointer field has no effect
    if kind == "str":  # (a lone surrogate escape decodes to U+FFFD)
        return re.sub("[\ud800-\udfff]", "\ufffd", v) if isinstance(v, str) and not isinstance(v, _Num) else None
    if kind == "bool":
        return v if isinstance(v, bool) else None
    if not isinstance(v, _Num):
        return None
    if kind == "float":
        f = float(v)  # strconv.ParseFloat(s, 64): out of range -> ErrRange -> skipped
        return None if math.isinf(f) else f
    # kind == "int": strconv.ParseInt(s, 10, 64) (no fraction or exponent), then OverflowInt
    try:
        n = int(v, 10)
    except ValueError:
        return None
    b = _INT_BITS[name]
    return n if -(1 << (b - 1)) <= n < (1 << (b - 1)) else None


def _go_coerce_utf8(b: bytes) -> str:
    """Go's unquoteBytes coercion (encoding/json decode.go): each byte that does not start a valid
    UTF-8 encoding (utf8.DecodeRune -> (RuneError, 1): bad lead, truncated, overlong, surrogate or
    beyond U+10FFFF) becomes U+FFFD and decoding resumes at the next byte."""
    out, i, n = [], 0, len(b)
    while i < n:
        c = b[i]
        if c < 0x80:
            out.append(chr(c))
            i += 1
            continue
        size, lo, hi = (2, 0x80, 0x7FF) if 0xC2 <= c <= 0xDF else (3, 0x800, 0xFFFF) if 0xE0 <= c <= 0xEF else \
            (4, 0x10000, 0x10FFFF) if 0xF0 <= c <= 0xF4 else (0, 0, 0)
        cp = None
        if size and i + size <= n and all(0x80 <= x <= 0xBF for x in b[i + 1:i + size]):
            v = c & (0x7F >> size)
            for x in b[i + 1:i + size]:
                v = (v << 6) | (x & 0x3F)
            if lo <= v <= hi and not 0xD800 <= v <= 0xDFFF:
                cp = v
        if cp is None:
            out.append("\ufffd")
            i += 1
        else:
            out.append(chr(cp))
            i += size
    return "".join(out)


def go_fold_name(key: str) -> str:
    """encoding/json's case-insensitive key match (Go 1.21 fold.go foldName: ASCII letters to upper
    case, any other rune to the smallest rune of its unicode.SimpleFold orbit; earlier Go:
    bytes.EqualFold, the same orbits).  The field names are ASCII, and the only non-ASCII runes
    whose orbit holds an ASCII letter are U+017F (long s ~ S) and U+212A (Kelvin sign ~ K); every
    other non-ASCII rune is left as it is here, which keeps it from matching any field, as in Go.
    (Python's str.casefold is not this: it maps U+FB01 'fi' to "fi" and U+00DF to "ss".)"""
    return "".join("S" if c == "\u017f" else "K" if c == "\u212a" else c.upper() if "a" <= c <= "z" else c
                   for c in key)


def go_unmarshal_order_node(body) -> "OrderNode":
    """json.Unmarshal(body, &OrderNode{}) as rabbitmq.go:118-121 runs it (the error is printed
    and DoOrder still runs): a syntax error decodes nothing (zero node, Action 0, ignored by
    DoOrder); otherwise every field whose JSON value fits its Go type is set, keys matched
    exactly or case-insensitively, later duplicates winning; a field of the wrong type, an
    overflowing number or a null stays zero."""
    node = OrderNode()
    if isinstance(body, (bytes, bytearray)):
        body = _go_coerce_utf8(bytes(body))
    try:
        d = json.loads(body, parse_int=_Num, parse_float=_Num, parse_constant=_no_constant,
                       object_pairs_hook=_Obj)
    except (ValueError, TypeError):
        return node
    if not isinstance(d, _Obj):
        return node  # null: no effect; any other top-level type: UnmarshalTypeError
    exact = {n: (n, k) for n, k in NODE_FIELDS}
    folded = {go_fold_name(n): (n, k) for n, k in NODE_FIELDS}
    for key, v in d:
        f = exact.get(key) or folded.get(go_fold_name(key))
        if f is None:
            continue
        x = _go_field_value(f[1], f[0], v)
        if x is not None:
            setattr(node, f[0], x)
    return node


class OrderNode:
    __slots__ = tuple(n for n, _ in NODE_FIELDS)

    def __init__(self, **kw):
        for n, k in NODE_FIELDS:
            setattr(self, n, kw.get(n, _ZERO[k]))

    def copy(self) -> "OrderNode":
        return OrderNode(**{n: getattr(self, n) for n, _ in NODE_FIELDS})

    # ordernode.go key builders -------------------------------------------
    def SetOrderHashKey(self):  # ordernode.go:89-92
        self.OrderHashKey = self.Symbol + ":comparison"
        self.OrderHashField = self.Symbol + ":" + self.Uuid + ":" + self.Oid

    def SetListZsetKey(self):  # ordernode.go:94-102 (SALE iff Transaction == 1)
        if SALE == self.Transaction:
            self.OrderListZsetKey = self.Symbol + ":SALE"
            self.OrderListZsetRKey = self.Symbol + ":BUY"
        else:
            self.OrderListZsetKey = self.Symbol + ":BUY"
            self.OrderListZsetRKey = self.Symbol + ":SALE"

    def SetDepthHashKey(self):  # ordernode.go:104-108
        self.OrderDepthHashKey = self.Symbol + ":depth"
        self.OrderDepthHashField = self.Symbol + ":depth:" + decimal_string(self.Price)

    def SetNodeName(self):  # ordernode.go:110-112
        self.NodeName = self.Symbol + ":node:" + self.Oid

    def SetNodeLink(self):  # ordernode.go:114-117
        self.NodeLink = self.Symbol + ":link:" + decimal_string(self.Price)

    # encoding/json ---------------------------------------------------------
    def to_json(self) -> str:
        parts = []
        for n, k in NODE_FIELDS:
            v = getattr(self, n)
            if k == "str":
                s = go_json_string(v)
            elif k == "float":
                s = go_json_float(v)
            elif k == "bool":
                s = "true" if v else "false"
            else:
                s = str(int(v))
            parts.append('"%s":%s' % (n, s))
        return "{" + ",".join(parts) + "}"

    @staticmethod
    def from_json(s: str) -> "OrderNode":
        d = json.loads(s)
        node = OrderNode()
        for n, k in NODE_FIELDS:
            if n in d:
                v = d[n]
                setattr(node, n, float(v) if k == "float" else v)
        return node


def scale(x: float, accuracy: int) -> float:
    """SetVolume/SetPrice, ordernode.go:76-87:
    decimal.NewFromFloat(x).Mul(decimal.NewFromFloat(math.Pow10(acc))).Float64()"""
    d = _shortest_decimal(x) * _shortest_decimal(math.pow(10, accuracy))
    return float(d)  # Decimal -> float is correctly rounded (== big.Rat.Float64)


def NewOrderNode(req: dict, accuracy: int = 8) -> OrderNode:
    """ordernode.go:38-54.  req = OrderRequest{uuid, oid, symbol, transaction, price, volume}."""
    node = OrderNode()
    node.Accuracy = accuracy
    node.Uuid = req["uuid"]
    node.Oid = req["oid"]
    node.Symbol = req["symbol"]
    node.Transaction = int(req["transaction"])
    node.Volume = scale(req["volume"], accuracy)
    node.Price = scale(req["price"], accuracy)
    node.SetOrderHashKey()
    node.SetListZsetKey()
    node.SetDepthHashKey()
    node.SetNodeName()
    node.SetNodeLink()
    return node


# ---------------------------------------------------------------- fake Redis
class FakeRedis:
    """In-memory HASH + ZSET with the Redis semantics the engine relies on."""

    def __init__(self):
        self.h: dict[str, dict[str, str]] = {}
        self.z: dict[str, dict[str, float]] = {}
        self.calls = 0

    # HASH
    def hset(self, key, field, value):
        self.calls += 1
        self.h.setdefault(key, {})[field] = value

    def hget(self, key, field) -> str:  # .Val() is "" on redis.Nil
        self.calls += 1
        return self.h.get(key, {}).get(field, "")

    def hexists(self, key, field) -> bool:
        self.calls += 1
        return field in self.h.get(key, {})

    def hdel(self, key, field):
        self.calls += 1
        d = self.h.get(key)
        if d is not None and field in d:
            del d[field]
            if not d:
                del self.h[key]

    def hincrbyfloat(self, key, field, incr: float):
        """Redis: long double add; stored with "%.17Lf" and trailing zeros trimmed.
        Exact (integer) on the parity domain; Fraction keeps it exact beyond."""
        self.calls += 1
        cur = self.h.get(key, {}).get(field)
        base = Fraction(Decimal(cur)) if cur else Fraction(0)
        val = base + Fraction(Decimal(go_fmt_f(incr)))
        s = format(Decimal(val.numerator) / Decimal(val.denominator), ".17f")
        s = s.rstrip("0").rstrip(".") if "." in s else s
        if s in ("-0", ""):
            s = "0"
        self.h.setdefault(key, {})[field] = s

    # ZSET (member strings; score parsed from the formatted float)
    def zadd(self, key, score: float, member: float):
        self.calls += 1
        self.z.setdefault(key, {})[go_fmt_f(member)] = float(go_fmt_f(score))

    def zrem(self, key, member: float):
        self.calls += 1
        d = self.z.get(key)
        m = go_fmt_f(member)
        if d is not None and m in d:
            del d[m]
            if not d:
                del self.z[key]

    @staticmethod
    def _bound(s: str) -> float:
        if s == "-inf":
            return -math.inf
        if s == "+inf":
            return math.inf
        return float(s)

    def zrangebyscore(self, key, lo: str, hi: str):
        self.calls += 1
        a, b = self._bound(lo), self._bound(hi)
        items = [(sc, m) for m, sc in self.z.get(key, {}).items() if a <= sc <= b]
        items.sort()
        return [m for _, m in items]

    def zrevrangebyscore(self, key, lo: str, hi: str):
        self.calls += 1
        a, b = self._bound(lo), self._bound(hi)
        items = [(sc, m) for m, sc in self.z.get(key, {}).items() if a <= sc <= b]
        items.sort(reverse=True)
        return [m for _, m in items]


# ---------------------------------------------------------------- engine
class GomeLiteral:
    """engine package globals (engine.go:20-22) + the two queues."""

    def __init__(self, accuracy: int = 8):
        self.accuracy = accuracy
        self.cache = FakeRedis()
        self.do_order_q: list[str] = []  # queue "doOrder"
        self.match_q: list[str] = []  # queue "matchOrder"

    # ---- nodepool.go ------------------------------------------------------
    def SetPrePool(self, n):  # :14-16
        self.cache.hset(n.OrderHashKey, n.OrderHashField, "1")

    def ExistsPrePool(self, n):  # :18-22
        return self.cache.hexists(n.OrderHashKey, n.OrderHashField)

    def DeletePrePool(self, n):  # :24-28
        if self.ExistsPrePool(n):
            self.cache.hdel(n.OrderHashKey, n.OrderHashField)

    def SetDepthLink(self, n):  # :31-46
        link = NodeLink(self, n, None)
        first = link.GetFirstNode()
        if first.Oid == "":
            link.InitOrderLink()
            return True
        last = link.GetLast()
        if last.Oid == "":
            raise RuntimeError("expects last node is not empty.")
        link.SetLast()
        return True

    def SetPoolDepthVolume(self, n):  # :61-63
        self.cache.hincrbyfloat(n.OrderDepthHashKey, n.OrderDepthHashField, n.Volume)

    def DeletePoolDepthVolume(self, n):  # :66-68
        self.cache.hincrbyfloat(n.OrderDepthHashKey, n.OrderDepthHashField, n.Volume * -1)

    def SetPoolDepth(self, n):  # :71-73
        self.cache.zadd(n.OrderListZsetKey, n.Price, n.Price)

    def DeletePoolDepth(self, n):  # :76-83
        s = self.cache.hget(n.OrderDepthHashKey, n.OrderDepthHashField)
        try:
            volume = float(s)
        except ValueError:  # strconv.ParseFloat error -> 0
            volume = 0.0
        if volume <= 0:
            self.cache.zrem(n.OrderListZsetKey, n.Price)

    def GetReverseDepth(self, n):  # :86-115
        depths = []
        price = go_fmt_f(n.Price)
        if SALE == n.Transaction:
            prices = self.cache.zrevrangebyscore(n.OrderListZsetRKey, price, "+inf")
        else:
            prices = self.cache.zrangebyscore(n.OrderListZsetRKey, "-inf", price)
        for v in prices:
            vol = self.cache.hget(n.OrderDepthHashKey, n.OrderDepthHashKey + ":" + v)
            depths.append([v, vol])
        return depths

    # ---- engine.go --------------------------------------------------------
    def PublishNewOrder(self, n):  # :35-44
        self.do_order_q.append(n.to_json())

    def publish_match(self, node, match_node, match_volume):
        self.match_q.append(
            '{"Node":%s,"MatchNode":%s,"MatchVolume":%s}'
            % (node.to_json(), match_node.to_json(), go_json_float(match_volume)))

    def DoOrder(self, node):  # :46-54
        if node.Action == ADD:
            self.SetOrder(node)
        elif node.Action == DEL:
            self.DeleteOrder(node)
        return True

    def SetOrder(self, node):  # :56-85
        if not self.ExistsPrePool(node):
            return False
        self.DeletePrePool(node)
        depths = self.GetReverseDepth(node)
        if len(depths) > 0:
            node2 = self.Match(node, depths)  # same pointer as node (:70 shadows)
            if node2.Volume <= 0:
                return True
        self.SetPoolDepth(node)
        self.SetPoolDepthVolume(node)
        self.SetDepthLink(node)
        return True

    def DeleteOrder(self, node):  # :87-116
        self.DeletePrePool(node)
        link = NodeLink(self, node, node)
        nodelink = link.GetLinkNode(node.NodeName)
        if nodelink.Oid == "":
            return False
        node.Volume = nodelink.Volume  # pool.Node aliases &node (:89,:100)
        self.DeletePoolDepthVolume(node)
        self.DeletePoolDepth(node)
        link.DeleteLinkNode(nodelink)
        self.publish_match(node, node, 0.0)
        return True

    def Match(self, node, depths):  # :118-136
        for v in depths:
            price = float(v[0])
            nodelink = node.copy()
            nodelink.Price = price
            nodelink.SetDepthHashKey()
            nodelink.SetNodeLink()
            link = NodeLink(self, nodelink, nodelink)
            node = self.MatchOrder(node, link)
            if node.Volume <= 0:
                break
        return node

    def MatchOrder(self, node, link):  # :138-198 (recursion -> loop on diff > 0)
        while True:
            matchNode = link.GetFirstNode()
            if matchNode.Oid == "":
                return node
            diff = node.Volume - matchNode.Volume
            if diff > 0:
                matchVolume = matchNode.Volume
                node.Volume = node.Volume - matchVolume
                link.DeleteLinkNode(matchNode)
                self.DeletePoolMatchOrder(matchNode)
                self.publish_match(node, matchNode, matchVolume)
                continue  # MatchOrder(node, link) at :161
            elif diff == 0:
                matchVolume = matchNode.Volume
                node.Volume = node.Volume - matchVolume
                link.DeleteLinkNode(matchNode)
                self.DeletePoolMatchOrder(matchNode)
                self.publish_match(node, matchNode, matchVolume)
            else:
                matchVolume = node.Volume
                matchNode.Volume = matchNode.Volume - matchVolume
                link.SetLinkNode(matchNode, matchNode.NodeName)
                updateNode = matchNode.copy()
                updateNode.Volume = matchVolume
                self.DeletePoolMatchOrder(updateNode)
                node.Volume = 0.0
                self.publish_match(node, matchNode, matchVolume)
            return node

    def DeletePoolMatchOrder(self, n):  # :200-206
        self.DeletePoolDepthVolume(n)
        self.DeletePoolDepth(n)

    # ---- gRPC ingress (main.go) and consumer (rabbitmq.go) ------------------
    def grpc_do_order(self, req: dict):  # main.go:39-52
        n = NewOrderNode(req, self.accuracy)
        n.Action = ADD
        self.SetPrePool(n)
        self.PublishNewOrder(n)

    def grpc_delete_order(self, req: dict):  # main.go:54-64
        n = NewOrderNode(req, self.accuracy)
        n.Action = DEL
        self.PublishNewOrder(n)

    def consume(self):  # rabbitmq.go:116-125, one message at a time
        """The reference's consumer loop, faithfully: every queued message is decoded and
        handed to DoOrder (rabbitmq.go:118-124).  A second ADD of a live (Symbol, Oid) corrupts
        the FIFO here exactly as in the reference (Q7); see consume_boundary."""
        q, self.do_order_q = self.do_order_q, []
        for body in q:
            self.DoOrder(go_unmarshal_order_node(body))

    def consume_boundary(self):
        """The same loop behind the drop-in boundary's duplicate-oid rule (gome_abi.h; SURVEY
        Appendix A Q7): an ADD that holds its admission marker but whose (Symbol, Oid) names a
        live node when it is consumed (an S:node:<oid> field of one of the symbol's S:link:<p>
        hashes, nodelink.go:119-122) is consumed (marker cleared, engine.go:62) and not applied.
        The rule depends on the queue order only, not on how the queue is cut into batches.
        `self.dups` = the positions (in this call's messages) of such ADDs."""
        q, self.do_order_q = self.do_order_q, []
        self.dups = []
        for i, body in enumerate(q):
            node = go_unmarshal_order_node(body)
            if node.Action == ADD and self.ExistsPrePool(node) and self.oid_live(node.Symbol, node.Oid):
                self.DeletePrePool(node)
                self.dups.append(i)
                continue
            self.DoOrder(node)

    def oid_live(self, symbol: str, oid: str) -> bool:
        """Does one of the symbol's FIFOs (S:link:<p>) hold the node S:node:<oid>?  The symbol's
        link hashes are listed once per change of the hash keys (a new or deleted price level), not
        per call (the scan of every key per admitted ADD made this quadratic)."""
        pre, field = symbol + ":link:", symbol + ":node:" + oid
        cache = self.__dict__.setdefault("_link_keys", {})
        n = len(self.cache.h)
        got = cache.get(symbol)
        if got is None or got[0] != n:
            got = cache[symbol] = (n, [key for key in self.cache.h if key.startswith(pre)])
        h = self.cache.h
        return any(field in h.get(key, ()) for key in got[1])

    def resting_oids(self) -> set:
        """(Symbol, Oid) of every node resting in a FIFO (an S:node:<oid> field of S:link:<p>)."""
        out = set()
        for key, hv in self.cache.h.items():
            if ":link:" not in key:
                continue
            for f, v in hv.items():
                if f not in ("f", "l"):
                    nd = OrderNode.from_json(v)
                    out.add((nd.Symbol, nd.Oid))
        return out

    def take_results(self) -> list[str]:
        out, self.match_q = self.match_q, []
        return out

    # ---- state dump for parity ---------------------------------------------
    def book_state(self, symbol: str) -> dict:
        """Redis-schema view of one book: side sets, depth fields, FIFOs in link order."""
        buy = sorted(float(m) for m in self.cache.z.get(symbol + ":BUY", {}))
        sale = sorted(float(m) for m in self.cache.z.get(symbol + ":SALE", {}))
        depth = {}
        for f, v in self.cache.h.get(symbol + ":depth", {}).items():
            depth[float(f[len(symbol + ":depth:"):])] = float(v)
        fifos = {}
        pre = symbol + ":link:"
        for key, hv in self.cache.h.items():
            if not key.startswith(pre) or "f" not in hv:
                continue
            out = []
            name = hv["f"]
            while name:
                nd = OrderNode.from_json(hv[name])
                out.append((nd.Oid, nd.Uuid, nd.Transaction, nd.Volume))
                name = nd.NextNode
            fifos[float(key[len(pre):])] = out
        return {"BUY": buy, "SALE": sale, "depth": depth, "fifo": fifos}


class NodeLink:
    """nodelink.go:7-166 — FIFO stored as HASH S:link:<price> {f, l, S:node:<oid> -> JSON}."""

    def __init__(self, eng: GomeLiteral, node, current):
        self.e = eng
        self.Node = node
        self.Current = current

    def InitOrderLink(self):  # :12-19
        self.Node.IsFirst = True
        self.Node.IsLast = True
        self.SetFristPointer(self.Node.NodeName)
        self.SetLastPointer(self.Node.NodeName)
        self.SetLinkNode(self.Node, self.Node.NodeName)

    def GetLinkNode(self, nodeName):  # :21-32 (sets Current)
        v = self.e.cache.hget(self.Node.NodeLink, nodeName)
        if v == "":
            return OrderNode()
        node = OrderNode.from_json(v)
        self.Current = node
        return node

    def SetFristPointer(self, nodename):  # :34-36
        self.e.cache.hset(self.Node.NodeLink, "f", nodename)

    def GetFirstNode(self):  # :38-51
        v = self.e.cache.hget(self.Node.NodeLink, "f")
        if v == "":
            return OrderNode()
        node = self.GetLinkNode(v)
        if node.Uuid != "":
            return node
        self.Current = node
        return node

    def SetLast(self):  # :53-64
        self.GetLast()
        self.Current.IsLast = False
        self.Current.NextNode = self.Node.NodeName
        self.SetLinkNode(self.Current, self.Current.NodeName)
        self.Node.PrevNode = self.Current.NodeName
        self.SetLastPointer(self.Node.NodeName)
        self.Node.IsLast = True
        self.SetLinkNode(self.Node, self.Node.NodeName)

    def SetLastPointer(self, nodename):  # :66-68
        self.e.cache.hset(self.Node.NodeLink, "l", nodename)

    def GetLast(self):  # :70-83
        v = self.e.cache.hget(self.Node.NodeLink, "l")
        if v == "":
            return OrderNode()
        node = self.GetLinkNode(v)
        if node.Uuid == "":
            return node
        self.Current = node
        return node

    def GetCurrent(self):  # :85-87
        return self.Current

    def GetPrev(self):  # :89-102
        current = self.GetCurrent()
        if current.PrevNode == "":
            return OrderNode()
        node = self.GetLinkNode(current.PrevNode)
        if node.Oid == "":
            return OrderNode()
        return node

    def GetNext(self):  # :104-117
        current = self.GetCurrent()
        if current.NextNode == "":
            return OrderNode()
        node = self.GetLinkNode(current.NextNode)
        if node.Oid == "":
            return OrderNode()
        return node

    def SetLinkNode(self, node, nodeName):  # :119-122
        self.e.cache.hset(self.Node.NodeLink, nodeName, node.to_json())

    def DeleteLinkNode(self, node):  # :124-166
        c = self.e.cache
        if node.IsFirst and node.IsLast:
            c.hdel(node.NodeLink, "f")
            c.hdel(node.NodeLink, "l")
            c.hdel(node.NodeLink, node.NodeName)
        elif node.IsFirst and not node.IsLast:
            nxt = self.GetNext()
            if nxt.Oid == "":
                raise RuntimeError("expects next node is not empty.")
            c.hdel(node.NodeLink, node.NodeName)
            nxt.IsFirst = True
            nxt.PrevNode = ""
            self.SetFristPointer(nxt.NodeName)
            self.SetLinkNode(nxt, nxt.NodeName)
        elif not node.IsFirst and node.IsLast:
            prev = self.GetPrev()
            if prev.Oid == "":
                raise RuntimeError("expects prev node is not empty.")
            c.hdel(node.NodeLink, node.NodeName)
            prev.IsLast = True
            prev.NextNode = ""
            self.SetLastPointer(prev.NodeName)
            self.SetLinkNode(prev, prev.NodeName)
        else:
            prev = self.GetPrev()
            current = self.GetNext()
            nxt = self.GetNext()
            if prev.Oid == "" and nxt.Oid == "":
                raise RuntimeError("expects relation node is not empty.")
            c.hdel(current.NodeLink, current.NodeName)
            prev.NextNode = nxt.NodeName
            nxt.PrevNode = prev.NodeName
            self.SetLinkNode(prev, prev.NodeName)
            self.SetLinkNode(nxt, nxt.NodeName)


def run_batches(requests_batches, accuracy: int = 8):
    """Deterministic ingress/consume interleave: every gRPC
    call of batch k happens after batch k-1 is consumed and before batch k is.
    requests_batches: iterable of lists of (action, req-dict).  Returns (engine, results)."""
    eng = GomeLiteral(accuracy)
    results = []
    for batch in requests_batches:
        for action, req in batch:
            if action == ADD:
                eng.grpc_do_order(req)
            elif action == DEL:
                eng.grpc_delete_order(req)
            else:  # a message with any other Action is consumed and ignored (engine.go:46-54)
                n = NewOrderNode(req, accuracy)
                n.Action = action
                eng.PublishNewOrder(n)
        eng.consume_boundary()
        results.extend(eng.take_results())
    return eng, results
