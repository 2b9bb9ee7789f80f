"""Publisher summary feed: the per-GPU trade / depth summary that
every rank contributes once per batch (RCCL all_gather over xGMI in bench.py) and the rank-0
consumer that stands in for the reference's matchOrder sink (ConsumeMatchOrder,
gomengine/engine/rabbitmq.go:132-177, which decodes and logs each result; "your code......",
:169).  Instead of one AMQP message per fill, the sink receives one fixed 32-word record per
GPU per batch, checks that the ranks agree on the step and accumulates node-wide totals.

Layout (int64 words): SUMMARY_FIELDS in order, the rest zero.
"""
from __future__ import annotations

import json

import numpy as np

SUMMARY_WORDS = 32
SUMMARY_FIELDS = ["n_orders", "n_add", "n_del", "n_dropped", "n_fills", "n_cancels", "n_rests",
                  "n_events", "n_resting", "n_levels", "max_segment", "n_segments", "n_flow_books",
                  "n_flow_orders", "n_hot", "device_us", "rank", "step"]
_IDX = {f: i for i, f in enumerate(SUMMARY_FIELDS)}
assert len(SUMMARY_FIELDS) <= SUMMARY_WORDS


def pack_summary(st: dict, rank: int, step: int, out=None):
    """One rank's summary words from its gome_stats dict (out: a torch / numpy int64 vector)."""
    vals = [int(st.get(f, 0)) for f in SUMMARY_FIELDS]
    vals[_IDX["device_us"]] = int(round(float(st.get("ms_total", 0.0)) * 1000))
    vals[_IDX["rank"]] = rank
    vals[_IDX["step"]] = step
    if out is None:
        out = np.zeros(SUMMARY_WORDS, np.int64)
    out.zero_() if hasattr(out, "zero_") else out.fill(0)
    for i, v in enumerate(vals):
        out[i] = v
    return out


class SummaryPublisher:
    """Rank-0 consumer of the gathered [world x 32] summaries."""

    def __init__(self, world: int):
        self.world = world
        self.steps = 0
        self.totals = {f: 0 for f in SUMMARY_FIELDS if f not in ("rank", "step", "n_resting", "n_levels")}
        self.resting = [0] * world
        self.max_device_us = 0
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

    def summary(self) -> dict:
        return {"steps": self.steps, "orders": self.totals["n_orders"], "fills": self.totals["n_fills"],
                "cancels": self.totals["n_cancels"], "events": self.totals["n_events"],
                "resting_per_rank": self.resting, "max_device_ms": self.max_device_us / 1000.0,
                "errors": self.errors}

    def line(self) -> str:
        return json.dumps(self.summary())
