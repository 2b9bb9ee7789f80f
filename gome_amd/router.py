"""Symbol-sharded routing over N engine handles: the host side of multi-GPU.

The reference has one consumer goroutine applying every message in queue order
(gomengine/engine/rabbitmq.go:116-125).  Books never interact (every key is per symbol,
ordernode.go:89-116), so the books can live on N GPUs: each symbol has one owner handle, a
drained batch is split into N sub-batches in queue order (each keeps its records' relative
order), the handles apply them side by side (one host thread per handle; the ctypes calls release
the GIL), and the N event streams are merged back into the reference's single publish order,
sorted by (sequence number, fill_idx) (engine.go:109-113,154-194).

owner(symbol) = load rank mod N, the round-robin over descending expected load (Zipf rank) that
bench.py's shards use; a symbol without a known load rank goes to hash(symbol_id) mod N.

`Router` has the engine interface BatchingConsumer drives (submit / drain / stats / max_batch /
dup_records), so the consumer runs unchanged in front of N GPUs.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .workload import EVENT_DTYPE, ORDER_DTYPE

_SUM_KEYS = ("n_orders", "n_add", "n_del", "n_dropped", "n_fills", "n_cancels", "n_rests", "n_events",
             "n_resting", "n_levels", "n_segments", "n_hot", "n_hot_orders", "n_hot_fills", "n_hot_rests",
             "n_hot_cancels", "n_flow_books", "n_flow_orders", "n_flow_touches", "n_flow_head_orders",
             "n_flow_head_touches", "n_flow_cancels", "n_dup_oid", "n_flow_tail_fills", "n_index_rebuilds", "idx_tombstones",
             "lvl_used", "n_quirk_checked", "n_requalified")
_TOTAL_KEYS = ("n_resting", "n_levels", "n_index_rebuilds", "idx_tombstones", "lvl_used")
_MAX_KEYS = ("max_segment", "ms_total", "ms_match", "ms_hot", "ms_flow_plan", "ms_cold")


def _mix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x45D9F3B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return x


def owner_table(max_symbols: int, world: int, load_rank: np.ndarray | None = None) -> np.ndarray:
    """owner[symbol_id] for every id: load_rank[id] % world where the load rank is known (>= 0),
    else a hash of the id."""
    ids = np.arange(max_symbols, dtype=np.uint32)
    own = (_mix32(ids) % np.uint64(world)).astype(np.int32)
    if load_rank is not None:
        lr = np.asarray(load_rank, dtype=np.int64)
        k = min(len(lr), max_symbols)
        known = lr[:k] >= 0
        own[:k][known] = (lr[:k][known] % world).astype(np.int32)
    return own


class Router:
    """N engine handles (one per GPU), each owning the symbols owner[] maps to it."""

    def __init__(self, engines, owner: np.ndarray):
        self.engines = list(engines)
        self.world = len(self.engines)
        self.owner = np.asarray(owner, dtype=np.int32)
        assert self.owner.min(initial=0) >= 0 and self.owner.max(initial=0) < self.world
        self.max_batch = min(int(e.max_batch) for e in self.engines)
        # (symbol ids the owner table and every handle accept)
        self.max_symbols = min([len(self.owner)] + [int(getattr(e, "max_symbols", len(self.owner))) for e in self.engines])
        self._pool = ThreadPoolExecutor(max_workers=self.world) if self.world > 1 else None
        self._ev = np.zeros(0, EVENT_DTYPE)
        self._stats: list[dict] = [{} for _ in self.engines]
        self._dups = np.zeros(0, np.uint32)
        self.part_sizes = [0] * self.world

    def close(self):
        if self._pool is not None:
            self._pool.shutdown()
            self._pool = None

    def split(self, rec: np.ndarray) -> list[np.ndarray]:
        """Batch indices owned by each handle, ascending (queue order within each part)."""
        own = self.owner[rec["symbol_id"]]
        return [np.nonzero(own == r)[0] for r in range(self.world)]

    def submit(self, rec: np.ndarray, seq_base: int = 0):
        """Apply one batch: each handle gets its symbols' records in queue order; the events are
        merged into the global publish order (drain())."""
        rec = np.ascontiguousarray(rec, dtype=ORDER_DTYPE)
        parts = self.split(rec)
        self.part_sizes = [len(p) for p in parts]

        def run(r):
            idx = parts[r]
            if len(idx) == 0:
                return np.zeros(0, EVENT_DTYPE), None, np.zeros(0, np.uint32)
            e = self.engines[r]
            e.submit(rec[idx], seq_base=0)
            ev = e.drain()
            ev = ev.copy()
            ev["taker_seq"] = idx[ev["taker_seq"]]  # local -> batch index (seq_base added below)
            dups = idx[e.dup_records()] if hasattr(e, "dup_records") else np.zeros(0, np.int64)
            return ev, e.stats(), dups

        res = list(self._pool.map(run, range(self.world))) if self._pool else [run(0)]
        ev = np.concatenate([x[0] for x in res]) if res else np.zeros(0, EVENT_DTYPE)
        # publish order: (sequence number, fill_idx); each part is already in that order, and a
        # taker's fills all come from its owner, so a stable sort on the sequence number merges
        ev = ev[np.argsort(ev["taker_seq"], kind="stable")]
        sq = ev["taker_seq"].astype(np.uint64) + np.uint64(seq_base)
        ev["taker_seq"] = (sq & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        self._ev = ev
        # a handle with no records this batch: zero per-batch counters, its running totals kept
        self._stats = [x[1] if x[1] is not None else
                       {k: v for k, v in self._stats[r].items() if k in _TOTAL_KEYS} for r, x in enumerate(res)]
        self._dups = np.sort(np.concatenate([x[2] for x in res]).astype(np.uint32))

    def drain(self) -> np.ndarray:
        ev, self._ev = self._ev, np.zeros(0, EVENT_DTYPE)
        return ev

    def dup_records(self) -> np.ndarray:
        return self._dups

    def stats(self) -> dict:
        """The handles' counters of the last batch combined: work summed, times and the hottest
        segment maxed (the handles run side by side)."""
        out = {}
        for k in _SUM_KEYS:
            out[k] = sum(int(s.get(k, 0)) for s in self._stats)
        for k in _MAX_KEYS:
            out[k] = max((s.get(k, 0) for s in self._stats), default=0)
        return out

    def top_of_book(self, symbols) -> np.ndarray:
        """Top-of-book digests of the given symbols, each from its owner handle."""
        from .abi import TOB_DTYPE
        symbols = np.asarray(symbols, dtype=np.uint32)
        out = np.zeros(len(symbols), TOB_DTYPE)
        own = self.owner[symbols]
        for r in range(self.world):
            k = np.nonzero(own == r)[0]
            if len(k):
                out[k] = self.engines[r].top_of_book(symbols[k])
        return out
