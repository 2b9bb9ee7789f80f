"""Checkpoint / resume in the reference's Redis key schema (SURVEY.md §5 "Checkpoint /
resume", §8f rank 2: "Redis demoted to snapshot/cache").

The reference keeps every book in Redis (nodepool.go:14-115, nodelink.go:12-166,
ordernode.go:89-117); a restart simply continues from Redis.  Here the book lives in HBM,
so a checkpoint is that state rendered in the same key schema, per symbol S:

  ZSET S:BUY / S:SALE      member = price (strconv 'f' -1), score = price    (SetPoolDepth, :71-73)
  HASH S:depth             S:depth:<price> -> depth (HINCRBYFLOAT text)    (:61-68)
  HASH S:link:<price>      f / l -> first / last node name; S:node:<oid> -> the node's JSON
                           (InitOrderLink / SetLast / DeleteLinkNode / SetLinkNode)

Prices and volumes are the reference's scaled float64 values (accuracy 8), integers on the
parity domain, so every number renders as its integer text.  One deliberate difference:
the reference never deletes a depth field, so prices whose depth went back to 0 keep a
"0" field; the engine does not remember them and the snapshot omits zero fields.  The
reference treats a missing field exactly like "0" (HINCRBYFLOAT starts from 0; the
ParseFloat error of an empty HGET gives 0 in DeletePoolDepth, nodepool.go:76-83).

Resume, two ways:
  * `load` writes the books straight into the pools of a fresh engine (gome_load_books): every
    state the reference's Redis can hold, quirk states included (a side-set member without a
    FIFO after a wrong-side cancel, Q2; a depth that differs from the FIFO's sum; a zero-volume
    maker, Q6), comes back exactly;
  * `restore` replays the snapshot into any engine: every resting node becomes an ADD of its
    remaining volume, in FIFO order per level.  A snapshot of an uncrossed book produces no
    fill, so the engine rebuilds the same levels, FIFOs and cancel index.  Books in a quirk
    state cannot be rebuilt this way and are refused.

`names` maps interned ids to the reference's strings: any object with
name(kind, id) -> str and id(kind, str) -> int, kinds "sym", "uuid", "oid" (the host owns
the interning, as the Go consumer would), and optionally tx_raw(code) -> int /
tx_code(raw) -> int for Transaction values outside {0, 1} (gome_abi.h transaction codes;
identity when absent).
"""
from __future__ import annotations

import json
from decimal import Decimal

import numpy as np

from .abi import GOME_E_INVAL, GomeError, render_link_node
from .workload import ADD, LEVEL_DTYPE, NODE_DTYPE, ORDER_DTYPE

GOME_SALE = 1


def _tx_raw(names, code: int) -> int:
    f = getattr(names, "tx_raw", None)
    return f(code) if f else code


def _tx_code(names, raw: int) -> int:
    f = getattr(names, "tx_code", None)
    return f(raw) if f else raw


def redis_snapshot(eng, symbol_ids, names, accuracy: int = 8) -> dict:
    """{"hash": {key: {field: value}}, "zset": {key: {member: score}}} for the symbols."""
    hashes: dict[str, dict[str, str]] = {}
    zsets: dict[str, dict[str, float]] = {}
    for sid in symbol_ids:
        S = names.name("sym", int(sid))
        for lv in eng.levels(int(sid)):
            p = int(lv["price_fx"])
            P = str(p)
            if lv["in_buy"]:
                zsets.setdefault(f"{S}:BUY", {})[P] = float(p)
            if lv["in_sale"]:
                zsets.setdefault(f"{S}:SALE", {})[P] = float(p)
            d = int(lv["depth_fx"])
            if d != 0:
                hashes.setdefault(f"{S}:depth", {})[f"{S}:depth:{P}"] = str(d)
            nodes = eng.fifo(int(sid), p)
            if len(nodes) == 0:
                continue
            oids = [names.name("oid", int(nd["oid_id"])) for nd in nodes]
            link = {"f": f"{S}:node:{oids[0]}", "l": f"{S}:node:{oids[-1]}"}
            for k, nd in enumerate(nodes):
                link[f"{S}:node:{oids[k]}"] = render_link_node(
                    S, p, _tx_raw(names, int(nd["side"])), int(nd["volume_fx"]), names.name("uuid", int(nd["uuid_id"])),
                    oids[k], oids[k - 1] if k else None, oids[k + 1] if k + 1 < len(nodes) else None,
                    accuracy)
            hashes[f"{S}:link:{P}"] = link
    return {"hash": hashes, "zset": zsets}


def _resp(*args: str) -> bytes:
    out = [f"*{len(args)}\r\n".encode()]
    for a in args:
        b = a.encode()
        out.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"".join(out)


def to_resp(snap: dict) -> bytes:
    """The snapshot as a Redis protocol stream (HSET / ZADD), e.g. for `redis-cli --pipe`."""
    out = []
    for key, fields in snap["hash"].items():
        for f, v in fields.items():
            out.append(_resp("HSET", key, f, v))
    for key, members in snap["zset"].items():
        for m, sc in members.items():
            out.append(_resp("ZADD", key, repr(sc) if sc != int(sc) else str(int(sc)), m))
    return b"".join(out)


def restore_records(snap: dict, names) -> np.ndarray:
    """The ADD records that rebuild the snapshot's books (FIFO order per level)."""
    recs = []
    depth = {k: v for k, v in snap["hash"].items() if k.endswith(":depth")}
    for key, link in snap["hash"].items():
        if ":link:" not in key:
            continue
        S, _, P = key.partition(":link:")
        sid, p = names.id("sym", S), int(P)
        name, total = link.get("f"), 0
        seen = 0
        while name:
            nd = json.loads(link[name])
            vol = int(nd["Volume"])
            recs.append((p, vol, sid, names.id("oid", nd["Oid"]), names.id("uuid", nd["Uuid"]),
                         int(nd["Transaction"])))
            total += vol
            seen += 1
            name = nd["NextNode"]
        if seen != len(link) - 2:
            raise GomeError(GOME_E_INVAL, f"{key}: FIFO chain does not cover the level")
        d = int(depth.get(f"{S}:depth", {}).get(f"{S}:depth:{P}", "0"))
        if d != total:
            raise GomeError(GOME_E_INVAL, f"{key}: depth {d} != FIFO total {total} (quirk state)")
    # side sets: a level is in exactly the set of its nodes' side (Transaction 1 = SALE,
    # anything else BUY, ordernode.go:94-102); a member without nodes (a Q2 leftover) or a
    # level in the wrong / both sets cannot come back from a replay
    sides: dict[tuple[str, str], set] = {}
    for (p, v, sid, oid, uuid, side) in recs:
        sides.setdefault((names.name("sym", sid), str(p)), set()).add("SALE" if side == GOME_SALE else "BUY")
    members = {(key.rpartition(":")[0], m, key.rpartition(":")[2])
               for key, ms in snap["zset"].items() for m in ms}
    for (S, P, sd) in members:
        if sides.get((S, P)) != {sd}:
            raise GomeError(GOME_E_INVAL, f"{S}:{sd} member {P} is not a FIFO of that side (quirk state)")
    for (S, P), sd in sides.items():
        if len(sd) != 1 or (S, P, next(iter(sd))) not in members:
            raise GomeError(GOME_E_INVAL, f"{S}:link:{P} is not in its side set (quirk state)")
    # a crossed book (best bid >= best ask) would fill on replay: refuse it before anything
    # reaches the engine
    best: dict[str, list] = {}
    for (S, P, sd) in members:
        b = best.setdefault(S, [None, None])
        p = int(P)
        if sd == "BUY":
            b[0] = p if b[0] is None else max(b[0], p)
        else:
            b[1] = p if b[1] is None else min(b[1], p)
    for S, (bid, ask) in best.items():
        if bid is not None and ask is not None and bid >= ask:
            raise GomeError(GOME_E_INVAL, f"{S}: snapshot book is crossed (bid {bid} >= ask {ask})")
    out = np.zeros(len(recs), ORDER_DTYPE)
    for i, (p, v, sid, oid, uuid, side) in enumerate(recs):
        out[i]["price_fx"] = p
        out[i]["volume_fx"] = v
        out[i]["symbol_id"] = sid
        out[i]["oid_id"] = oid
        out[i]["uuid_id"] = uuid
        out[i]["side"] = _tx_code(names, side)
        out[i]["action"] = ADD
    return out


def restore(eng, snap: dict, names, seq_base: int = 0, chunk: int | None = None) -> int:
    """Rebuild the snapshot's books in an engine (resume), in submits of at most the engine's
    max_batch (or `chunk`) records.  Returns the orders replayed."""
    rec = restore_records(snap, names)  # (validated, crossed books refused: nothing applied yet)
    step = max(1, min(int(getattr(eng, "max_batch", len(rec) or 1)), chunk or (1 << 62)))
    for i in range(0, len(rec), step):  # FIFO order is kept across chunks
        eng.submit(rec[i:i + step], seq_base + i)
        ev = eng.drain()
        if len(ev):
            raise GomeError(GOME_E_INVAL, f"snapshot book is crossed: {len(ev)} fills on replay")
    return len(rec)


def _fifo(key: str, link: dict) -> list:
    """The node JSON objects of one S:link:<price> HASH in FIFO order (f, then NextNode)."""
    out, name = [], link.get("f")
    while name:
        if name not in link or len(out) > len(link):
            raise GomeError(GOME_E_INVAL, f"{key}: broken FIFO chain at {name}")
        nd = json.loads(link[name])
        out.append(nd)
        name = nd["NextNode"]
    if len(out) != len(link) - 2:
        raise GomeError(GOME_E_INVAL, f"{key}: FIFO chain does not cover the level")
    return out


def book_images(snap: dict, names) -> list:
    """The snapshot as gome_load_books images: [(symbol_id, levels, nodes)], one per symbol,
    levels ascending by price.  A level is every price in S:BUY / S:SALE, with a nonzero
    S:depth field or with an S:link HASH; nothing is checked for consistency (quirk states load
    as they are)."""
    per: dict[str, dict[int, list]] = {}

    def lvl(S: str, p: int) -> list:
        return per.setdefault(S, {}).setdefault(p, [0, 0, 0, []])

    for key, members in snap["zset"].items():
        S, _, sd = key.rpartition(":")
        for m in members:
            lvl(S, int(m))[0 if sd == "BUY" else 1] = 1
    for key, fields in snap["hash"].items():
        if key.endswith(":depth"):
            S = key[:-len(":depth")]
            for f, v in fields.items():
                d = int(Decimal(v))
                if d:
                    lvl(S, int(f.rpartition(":")[2]))[2] = d
        elif ":link:" in key:
            S, _, P = key.partition(":link:")
            lvl(S, int(P))[3] = _fifo(key, fields)
    books = []
    for S, lvls in per.items():
        prices = sorted(lvls)
        lv = np.zeros(len(prices), LEVEL_DTYPE)
        nodes = []
        for i, p in enumerate(prices):
            b, a, d, fifo = lvls[p]
            lv[i] = (p, d, len(fifo), b, a, 0)
            for nd in fifo:
                nodes.append((int(nd["Volume"]), names.id("oid", nd["Oid"]), names.id("uuid", nd["Uuid"]),
                              _tx_code(names, int(nd["Transaction"]))))
        na = np.zeros(len(nodes), NODE_DTYPE)
        for i, (v, o, u, t) in enumerate(nodes):
            na[i]["volume_fx"], na[i]["oid_id"], na[i]["uuid_id"], na[i]["side"] = v, o, u, t
        books.append((names.id("sym", S), lv, na))
    return books


def load(eng, snap: dict, names) -> int:
    """Resume: the snapshot's books straight into a fresh engine (gome_load_books), quirk states
    included.  Returns the resting nodes loaded."""
    books = book_images(snap, names)
    eng.load_books(books)
    return sum(len(b[2]) for b in books)
