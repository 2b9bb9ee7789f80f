"""Seeded synthetic order streams for BASELINE.json configs 1-5.

The reference's only load generators are gomengine/doorder.go (1,999 random limit
orders) and gomengine/delorder.go (one cancel).  Their distribution is reproduced
here, not their time-seeded stream (doorder.go:34-35 seeds from the clock):

  side   ~ U{0,1}                                       doorder.go:37
  price  = round2(U[0,1)), 0 -> 0.10                     doorder.go:38-41, :63-67
  volume = round2(U[0,1)), 0 -> 1.00                     doorder.go:43-47

In fixed point at accuracy 8 that is price_fx in {1e6 .. 1e8} step 1e6 and
volume_fx in {1e6 .. 1e8} step 1e6.  Records use the gome_order layout of
include/gome/gome_abi.h (32 bytes).
"""
from __future__ import annotations

import numpy as np

ORDER_DTYPE = np.dtype([
    ("price_fx", "<i8"), ("volume_fx", "<i8"), ("symbol_id", "<u4"), ("oid_id", "<u4"),
    ("uuid_id", "<u4"), ("side", "u1"), ("action", "u1"), ("flags", "<u2"),
])
assert ORDER_DTYPE.itemsize == 32

EVENT_DTYPE = np.dtype([
    ("price_fx", "<i8"), ("match_volume_fx", "<i8"), ("maker_volume_fx", "<i8"),
    ("taker_seq", "<u4"), ("fill_idx", "<u4"), ("maker_oid_id", "<u4"), ("maker_uuid_id", "<u4"),
    ("maker_next_oid_id", "<u4"), ("kind", "u1"), ("maker_side", "u1"),
    ("maker_is_last", "u1"), ("pad0", "u1"),
])
assert EVENT_DTYPE.itemsize == 48


def taker_remaining(ev: np.ndarray, records: np.ndarray, seq_base: int = 0) -> np.ndarray:
    """Node.Volume of each event (gome_abi.h): for a FILL the taker's volume minus its fills so far
    (a taker's events are consecutive in publish order), for a CANCEL the stored remaining volume."""
    idx = ((ev["taker_seq"].astype(np.int64) - seq_base) & 0xFFFFFFFF).astype(np.int64)
    fill = ev["kind"] == 1
    q = np.where(fill, ev["match_volume_fx"], 0)
    start = np.ones(len(ev), bool)
    start[1:] = idx[1:] != idx[:-1]
    grp = np.cumsum(start) - 1
    cs = np.cumsum(q)
    base = np.concatenate([[0], cs])[np.nonzero(start)[0]][grp]  # fills before the taker's first event
    rem = records["volume_fx"][idx] - (cs - base)
    return np.where(fill, rem, ev["maker_volume_fx"])

LEVEL_DTYPE = np.dtype([("price_fx", "<i8"), ("depth_fx", "<i8"), ("n_nodes", "<u4"),
                        ("in_buy", "u1"), ("in_sale", "u1"), ("pad", "<u2")])
NODE_DTYPE = np.dtype([("volume_fx", "<i8"), ("oid_id", "<u4"), ("uuid_id", "<u4"),
                       ("side", "u1"), ("pad", "u1", (7,))])

FX = 10 ** 8  # accuracy 8 (config.yaml.example:24)
ADD, DEL = 1, 2


def doorder_prices(rng: np.random.Generator, n: int, decimals: int = 2) -> np.ndarray:
    """round(U[0,1), decimals) with 0 -> 0.10, in fixed point (doorder.go:38-41)."""
    q = 10 ** decimals
    k = np.rint(rng.random(n) * q).astype(np.int64)
    k[k == 0] = q // 10
    return k * (FX // q)


def doorder_volumes(rng: np.random.Generator, n: int) -> np.ndarray:
    """round2(U[0,1)) with 0 -> 1.00, in fixed point (doorder.go:43-47)."""
    k = np.rint(rng.random(n) * 100).astype(np.int64)
    k[k == 0] = 100
    return k * (FX // 100)


class ZipfSymbols:
    """Symbol ranks ~ Zipf(s) over n symbols, mapped to ids by a fixed permutation."""

    def __init__(self, n_symbols: int, s: float = 1.0, seed: int = 7):
        w = 1.0 / np.arange(1, n_symbols + 1, dtype=np.float64) ** s
        self.cdf = np.cumsum(w / w.sum())
        self.cdf[-1] = 1.0
        self.rank_to_id = np.random.default_rng(seed).permutation(n_symbols).astype(np.uint32)
        self.id_to_rank = np.empty(n_symbols, np.uint32)
        self.id_to_rank[self.rank_to_id] = np.arange(n_symbols, dtype=np.uint32)
        self.n = n_symbols

    def share_of_top(self) -> float:
        return float(self.cdf[0])

    def sample_ranks(self, rng, n):
        return np.searchsorted(self.cdf, rng.random(n), side="right").astype(np.uint32)


class Stream:
    """Deterministic ADD-only doorder-distribution stream over many symbols.

    cfg 1: n_symbols=1 (uuid 2, fresh oids) ; cfg 2: uniform over 1k symbols ;
    cfg 3: Zipf(s) over 100k symbols ; cfg 5: price_decimals=4 over 1M symbols.
    `owner=(rank, world)` keeps only symbols whose Zipf rank % world == rank
    (round-robin over descending expected load).
    """

    def __init__(self, n_symbols: int, zipf_s: float | None = None, seed: int = 42,
                 price_decimals: int = 2, owner: tuple[int, int] | None = None):
        self.rng = np.random.default_rng(seed)
        self.n_symbols = n_symbols
        self.zipf = ZipfSymbols(n_symbols, zipf_s) if zipf_s else None
        self.price_decimals = price_decimals
        self.owner = owner
        self.next_oid = 1

    def _symbols(self, n):
        if self.zipf is None:
            ranks = self.rng.integers(0, self.n_symbols, n, dtype=np.uint32)
            ids = ranks
        else:
            ranks = self.zipf.sample_ranks(self.rng, n)
            ids = self.zipf.rank_to_id[ranks]
        return ids, ranks

    def batch(self, n: int) -> np.ndarray:
        """Next n records of the global stream (before ownership filtering)."""
        rec = np.zeros(n, ORDER_DTYPE)
        ids, ranks = self._symbols(n)
        rec["symbol_id"] = ids
        rec["price_fx"] = doorder_prices(self.rng, n, self.price_decimals)
        rec["volume_fx"] = doorder_volumes(self.rng, n)
        rec["side"] = self.rng.integers(0, 2, n, dtype=np.uint8)
        rec["action"] = ADD
        rec["uuid_id"] = 2
        rec["oid_id"] = np.arange(self.next_oid, self.next_oid + n, dtype=np.uint64).astype(np.uint32)
        self.next_oid += n
        if self.owner is not None:
            r, w = self.owner
            rec = rec[(ranks % w) == r]
        return rec


def cancel_mix(n: int, n_symbols: int, seed: int = 42, del_frac: float = 0.5,
               aggressive_frac: float = 0.10, zipf_s: float | None = None,
               price_decimals: int = 2) -> np.ndarray:
    """Config 4: cancel-heavy mix (sequential generator; use for <= a few M records).

    Each DEL targets a uniformly chosen previously-ADDed, not-yet-cancelled order
    with its original symbol/side/price/uuid (a filled target is a no-op, as in the
    reference, engine.go:96-98).  10% of ADDs are aggressive: BUY @ 1.00 or
    SALE @ 0.01 with volume k * 10.00, k ~ U{1..16} (sweeps several levels).
    """
    rng = np.random.default_rng(seed)
    rec = np.zeros(n, ORDER_DTYPE)
    if zipf_s:
        z = ZipfSymbols(n_symbols, zipf_s)
        syms = z.rank_to_id[z.sample_ranks(rng, n)]
    else:
        syms = rng.integers(0, n_symbols, n, dtype=np.uint32)
    prices = doorder_prices(rng, n, price_decimals)
    vols = doorder_volumes(rng, n)
    sides = rng.integers(0, 2, n, dtype=np.uint8)
    is_del = rng.random(n) < del_frac
    aggr = rng.random(n) < aggressive_frac
    ks = rng.integers(1, 17, n)
    pick = rng.random(n)
    live: list[int] = []  # indices of ADDs not yet targeted
    oid = 1
    for i in range(n):
        if is_del[i] and live:
            j = int(pick[i] * len(live))
            t = live[j]
            live[j] = live[-1]
            live.pop()
            rec[i] = rec[t]
            rec[i]["action"] = DEL
            continue
        rec[i]["action"] = ADD
        rec[i]["symbol_id"] = syms[i]
        rec[i]["side"] = sides[i]
        rec[i]["uuid_id"] = 2
        rec[i]["oid_id"] = oid
        oid += 1
        if aggr[i]:
            rec[i]["price_fx"] = FX if sides[i] == 0 else FX // 100
            rec[i]["volume_fx"] = int(ks[i]) * 10 * FX
        else:
            rec[i]["price_fx"] = prices[i]
            rec[i]["volume_fx"] = vols[i]
        live.append(i)
    return rec


def split_batches(rec: np.ndarray, batch: int):
    return [rec[i:i + batch] for i in range(0, len(rec), batch)]


class NativeStream:
    """The native load generator (include/gome/gome_loadgen.h, libgome.so host code): the same
    distributions as Stream / cancel_mix at bench scale (config 4's cancel mix in C++: each DEL
    re-sends a uniformly chosen earlier ADD no DEL targeted yet).  Symbol ids follow
    ZipfSymbols(n_symbols, s).rank_to_id (uniform symbols: identity)."""

    def __init__(self, n_symbols: int, zipf_s: float | None = None, seed: int = 42,
                 price_decimals: int = 2, del_frac: float = 0.0, aggressive_frac: float = 0.0,
                 rank: int = 0, world: int = 1, uuid: int = 2, first_oid: int = 1):
        import ctypes as C
        from .abi import GomeError, load_library
        self._C = C
        self.lib = load_library()
        self.zipf = ZipfSymbols(n_symbols, zipf_s) if zipf_s else None
        self._perm = (self.zipf.rank_to_id if self.zipf is not None
                      else np.arange(n_symbols, dtype=np.uint32)).astype(np.uint32)

        class Cfg(C.Structure):
            _fields_ = [("n_symbols", C.c_uint32), ("price_decimals", C.c_uint32), ("zipf_s", C.c_double),
                        ("del_frac", C.c_double), ("aggressive_frac", C.c_double), ("seed", C.c_uint64),
                        ("first_oid", C.c_uint64), ("rank_to_id", C.c_void_p), ("rank", C.c_uint32),
                        ("world", C.c_uint32), ("uuid", C.c_uint32), ("accuracy", C.c_uint32)]
        cfg = Cfg(n_symbols, price_decimals, float(zipf_s or 0.0), del_frac, aggressive_frac, seed,
                  first_oid, self._perm.ctypes.data, rank, world, uuid, 8)
        h = C.c_void_p()
        st = self.lib.gome_gen_create(C.byref(cfg), C.byref(h))
        if st != 0:
            raise GomeError(st, "gome_gen_create")
        self.h = h
        own, top = C.c_double(), C.c_double()
        self.lib.gome_gen_shares(h, C.byref(own), C.byref(top))
        self.owned_share, self.top_share = own.value, top.value

    def batch(self, n: int, out: np.ndarray | None = None) -> np.ndarray:
        rec = out if out is not None else np.zeros(n, ORDER_DTYPE)
        assert rec.dtype == ORDER_DTYPE and len(rec) >= n
        st = self.lib.gome_gen_batch(self.h, rec.ctypes.data, n)
        if st != 0:
            raise RuntimeError(f"gome_gen_batch: {st}")
        return rec[:n]

    def close(self):
        if getattr(self, "h", None):
            self.lib.gome_gen_destroy(self.h)
            self.h = None

    __del__ = close


def inject_quirks(rec: np.ndarray, sym: int, levels: np.ndarray, fifo, mode: str = "heal") -> dict:
    """Rewrite the first records of symbol `sym` in `rec` (in place) into the two legal inputs
    that put a book in a quirk state:
      * Q2: wrong-side cancels (`transaction` flipped, price and oid right) of every maker of one
        bid level, which empty its FIFO while DeletePoolDepth ZREMs the *ask* set
        (engine.go:87-116, nodepool.go:76-83): the level stays in S:BUY with no FIFO;
      * Q6: a zero-volume BUY ADD ("Volume": null decodes to 0) at another bid level, which rests
        as a zero-volume maker behind that level's FIFO (engine.go:69-82).
    mode "heal": the Q2 level is the best bid and the Q6 level the second best, where the stream
    soon rests and consumes again (the reference's state heals); mode "stuck": the Q2 level is
    the lowest bid, which the stream never reaches again (the quirk stays).  Modes "q2heal" /
    "q2stuck": the same wrong-side cancels without the zero-volume ADD.  `levels` / `fifo`
    are the book's state before `rec` (gome_snapshot_levels / gome_snapshot_fifo, or the
    oracle's).  Mode "zero": zero-volume ADDs only (Q6, "Volume": 0 or null): six takers that cross
    (BUYs at 1.00, SALEs at 0.01: one 0-fill each at the best opposite level, engine.go:176-194),
    spread over the batch, and one BUY resting behind the lowest bid's makers; "zeroheal": the same
    with the resting one behind the best bid's makers, where the stream's SALEs soon reach it and pop
    it with a 0-fill (engine.go:145-161); "zerodel": that zero-volume maker alone, in a batch with a
    DEL (of the lowest bid's first maker), so the book takes the cancel path.  Returns what was
    injected."""
    bids = levels[(levels["in_buy"] != 0) & (levels["in_sale"] == 0) & (levels["n_nodes"] > 0)]
    if len(bids) < 3:
        raise ValueError("book has fewer than three bid levels")
    bids = np.sort(bids, order="price_fx")
    if mode == "zerodel":
        pos = np.nonzero((rec["symbol_id"] == sym) & (rec["action"] == ADD))[0]
        m = fifo(int(bids[0]["price_fx"]))[0]  # a DEL of the lowest bid's first maker: the cancel path
        d = rec[pos[0]]
        d["action"], d["flags"], d["oid_id"], d["uuid_id"] = DEL, 0, m["oid_id"], m["uuid_id"]
        d["side"], d["price_fx"], d["volume_fx"] = m["side"], bids[0]["price_fx"], m["volume_fx"]
        z = pos[1]  # (right after the DEL: the book is still the snapshot's, so it rests behind the best bid)
        zb = bids[-1]
        rec["volume_fx"][z], rec["side"][z], rec["price_fx"][z] = 0, 0, zb["price_fx"]
        return {"q2_price": None, "q2_cancels": 0, "q6_price": int(zb["price_fx"]),
                "q6_oid": int(rec["oid_id"][z]), "dels": 1, "records": [int(pos[0]), int(z)]}
    if mode in ("zero", "zeroheal"):
        pos = np.nonzero((rec["symbol_id"] == sym) & (rec["action"] == ADD))[0]
        picks = pos[(np.array([0.001, 0.1, 0.3, 0.5, 0.7, 0.9, 0.95]) * len(pos)).astype(int)]
        for k, i in enumerate(picks[:6]):
            sale = k % 2 == 1
            rec["volume_fx"][i], rec["side"][i] = 0, 1 if sale else 0
            rec["price_fx"][i] = FX // 100 if sale else FX
        z = picks[6]
        zb = bids[-1] if mode == "zeroheal" else bids[0]
        rec["volume_fx"][z], rec["side"][z], rec["price_fx"][z] = 0, 0, zb["price_fx"]
        return {"q2_price": None, "q2_cancels": 0, "q6_price": int(zb["price_fx"]),
                "q6_oid": int(rec["oid_id"][z]), "records": [int(i) for i in picks]}
    heal = mode in ("heal", "q2heal")
    q2 = bids[-1] if heal else bids[0]
    q6 = bids[-2] if heal else bids[1]
    makers = fifo(int(q2["price_fx"]))
    pos = np.nonzero((rec["symbol_id"] == sym) & (rec["action"] == ADD))[0]
    if len(pos) < len(makers) + 1:
        raise ValueError("too few records of the symbol to rewrite")
    for i, m in zip(pos, makers):  # the wrong-side cancels
        r = rec[i]
        r["price_fx"], r["volume_fx"] = q2["price_fx"], m["volume_fx"]
        r["oid_id"], r["uuid_id"] = m["oid_id"], m["uuid_id"]
        r["side"] = 0 if m["side"] == 1 else 1
        r["action"], r["flags"] = DEL, 0
    if mode.startswith("q2"):
        return {"q2_price": int(q2["price_fx"]), "q2_cancels": len(makers), "q6_price": None,
                "q6_oid": None, "records": [int(i) for i in pos[:len(makers)]]}
    z = rec[pos[len(makers)]]  # the zero-volume ADD keeps the record's own (fresh) oid
    z["price_fx"], z["volume_fx"], z["side"] = q6["price_fx"], 0, 0
    return {"q2_price": int(q2["price_fx"]), "q2_cancels": len(makers), "q6_price": int(q6["price_fx"]),
            "q6_oid": int(z["oid_id"]), "records": [int(i) for i in pos[:len(makers) + 1]]}
