"""Publisher summary feed: the per-GPU trade / depth summary that
every rank contributes once per batch (RCCL all_gather over xGMI in bench.py) and the rank-0
consumer that stands in for the reference's matchOrder sink (ConsumeMatchOrder,
gomengine/engine/rabbitmq.go:132-177, which decodes and logs each result; "your code......",
:169).  Instead of one AMQP message per fill, the sink receives one fixed 80-word record per
GPU per batch, checks that the ranks agree on the step, accumulates node-wide totals and keeps
each rank's latest depth digests.

Layout (int64 words):
  [0, len(SUMMARY_FIELDS))      counters, SUMMARY_FIELDS in order
  [DIGEST_BASE, +8 * 7)         top-of-book digests of the rank's DIGEST_N hottest symbols
                                (gome_top_of_book: symbol, best bid price / depth / FIFO length,
                                best ask price / depth / FIFO length; symbol -1 = unused slot),
                                the depth view GetReverseDepth reads (nodepool.go:86-115)
"""
from __future__ import annotations

import json

import numpy as np

SUMMARY_WORDS = 80
SUMMARY_FIELDS = ["n_orders", "n_add", "n_del", "n_dropped", "n_fills", "n_cancels", "n_rests",
                  "n_events", "n_resting", "n_levels", "max_segment", "n_segments", "n_flow_books",
                  "n_flow_orders", "n_hot", "device_us", "rank", "step", "n_dup_oid"]
_IDX = {f: i for i, f in enumerate(SUMMARY_FIELDS)}
DIGEST_BASE, DIGEST_N = 8 + 2 * 8, 8
DIGEST_FIELDS = ["symbol_id", "bid_price_fx", "bid_depth_fx", "bid_nodes", "ask_price_fx", "ask_depth_fx",
                 "ask_nodes"]
DIGEST_W = len(DIGEST_FIELDS)
assert len(SUMMARY_FIELDS) <= DIGEST_BASE and DIGEST_BASE + DIGEST_N * DIGEST_W <= SUMMARY_WORDS


def pack_summary(st: dict, rank: int, step: int, out=None, digests=None):
    """One rank's summary words from its gome_stats dict and (optional) top-of-book digests
    (a gome_top_of_book array, at most DIGEST_N).  out: a torch / numpy int64 vector."""
    vals = np.zeros(SUMMARY_WORDS, np.int64)
    for i, f in enumerate(SUMMARY_FIELDS):
        vals[i] = int(st.get(f, 0))
    vals[_IDX["device_us"]] = int(round(float(st.get("ms_total", 0.0)) * 1000))
    vals[_IDX["rank"]] = rank
    vals[_IDX["step"]] = step
    dg = vals[DIGEST_BASE:DIGEST_BASE + DIGEST_N * DIGEST_W].reshape(DIGEST_N, DIGEST_W)
    dg[:, 0] = -1
    if digests is not None:
        for k, d in enumerate(digests[:DIGEST_N]):
            dg[k] = [int(d[f]) for f in DIGEST_FIELDS]
    if out is None:
        return vals
    if hasattr(out, "copy_"):
        import torch
        out.copy_(torch.from_numpy(vals))
    else:
        out[:] = vals
    return out


def digests_from_levels(levels) -> dict:
    """The digest a book's level snapshot (gome_snapshot_levels, ascending price) implies."""
    d = {"bid_price_fx": 0, "bid_depth_fx": 0, "bid_nodes": 0, "ask_price_fx": 0, "ask_depth_fx": 0, "ask_nodes": 0}
    bids = levels[levels["in_buy"] != 0]
    asks = levels[levels["in_sale"] != 0]
    if len(bids):
        b = bids[-1]
        d.update(bid_price_fx=int(b["price_fx"]), bid_depth_fx=int(b["depth_fx"]), bid_nodes=int(b["n_nodes"]))
    if len(asks):
        a = asks[0]
        d.update(ask_price_fx=int(a["price_fx"]), ask_depth_fx=int(a["depth_fx"]), ask_nodes=int(a["n_nodes"]))
    return d


class SummaryPublisher:
    """Rank-0 consumer of the gathered [world x SUMMARY_WORDS] summaries."""

    def __init__(self, world: int):
        self.world = world
        self.steps = 0
        self.totals = {f: 0 for f in SUMMARY_FIELDS if f not in ("rank", "step", "n_resting", "n_levels")}
        self.resting = [0] * world
        self.max_device_us = 0
        self.digests: list[list[dict]] = [[] for _ in range(world)]
        self.digests_checked = 0
        self.errors: list[str] = []

    def consume(self, gathered) -> dict:
        g = np.asarray(gathered.cpu() if hasattr(gathered, "cpu") else gathered, dtype=np.int64)
        g = g.reshape(self.world, SUMMARY_WORDS)
        steps = set(int(x) for x in g[:, _IDX["step"]])
        if len(steps) != 1:
            self.errors.append(f"ranks disagree on the step: {sorted(steps)}")
        for r in range(self.world):
            if int(g[r, _IDX["rank"]]) != r:
                self.errors.append(f"row {r} carries rank {int(g[r, _IDX['rank']])}")
            self.resting[r] = int(g[r, _IDX["n_resting"]])
            dg = g[r, DIGEST_BASE:DIGEST_BASE + DIGEST_N * DIGEST_W].reshape(DIGEST_N, DIGEST_W)
            self.digests[r] = [dict(zip(DIGEST_FIELDS, (int(x) for x in row))) for row in dg if row[0] >= 0]
        for f in self.totals:
            if f == "max_segment":
                self.totals[f] = max(self.totals[f], int(g[:, _IDX[f]].max()))
            else:
                self.totals[f] += int(g[:, _IDX[f]].sum())
        self.max_device_us = max(self.max_device_us, int(g[:, _IDX["device_us"]].max()))
        self.steps += 1
        return {"step": next(iter(steps)), "orders": int(g[:, _IDX["n_orders"]].sum()),
                "fills": int(g[:, _IDX["n_fills"]].sum()), "events": int(g[:, _IDX["n_events"]].sum())}

    def check(self, orders: int, fills: int, events: int) -> bool:
        """The ranks' summaries add up to the job's totals (computed independently)."""
        ok = (self.totals["n_orders"] == orders and self.totals["n_fills"] == fills
              and self.totals["n_events"] == events and not self.errors)
        if not ok and not self.errors:
            self.errors.append(f"totals {self.totals['n_orders']}/{self.totals['n_fills']}/"
                               f"{self.totals['n_events']} != job {orders}/{fills}/{events}")
        return ok

    def check_digests(self, levels_of) -> bool:
        """Every rank's latest digests against the book snapshots: levels_of(rank, symbol_id) ->
        that rank's gome_snapshot_levels array."""
        ok = True
        for r in range(self.world):
            for d in self.digests[r]:
                want = digests_from_levels(levels_of(r, d["symbol_id"]))
                got = {k: d[k] for k in want}
                if got != want:
                    ok = False
                    self.errors.append(f"rank {r} symbol {d['symbol_id']}: digest {got} != snapshot {want}")
                self.digests_checked += 1
        return ok

    def summary(self) -> dict:
        return {"steps": self.steps, "orders": self.totals["n_orders"], "fills": self.totals["n_fills"],
                "cancels": self.totals["n_cancels"], "events": self.totals["n_events"],
                "dup_oid": self.totals["n_dup_oid"], "resting_per_rank": self.resting,
                "max_device_ms": self.max_device_us / 1000.0,
                "top_of_book": {r: self.digests[r][:2] for r in range(self.world)},
                "digests_checked": self.digests_checked, "errors": self.errors}

    def line(self) -> str:
        return json.dumps(self.summary())
