"""How much of the hottest book's serial plan a look-ahead classify pass could decide without the book
state (VERDICT r5 next #4a).  Replays config 3's hottest book on an aggregate book
(price -> depth per side) and counts, per batch, the orders a state-free bound proves non-crossing:
a BUY below min(best ask at batch start, every earlier SALE price of the batch) cannot cross (a SALE
rests at or above its price), and the mirror for SALEs.  Also counts crossing orders, level fills, emptied levels and rests per order.
  python tools/classify_bound.py"""
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import numpy as np, bench  # noqa: E402
from sortedcontainers import SortedDict
from gome_amd import workload as wl
gen, _, _ = bench.make_stream("config3", 0, 1, 42)
z = wl.ZipfSymbols(100000, 1.0); hot = int(z.rank_to_id[0])
bids, asks = SortedDict(), SortedDict()   # price -> depth
def run(rec, stats):
    p = rec["price_fx"]; v = rec["volume_fx"]; s = rec["side"]
    # static bounds for the batch: best ask >= min(initial best ask, min SALE price before t)
    ba0 = asks.peekitem(0)[0] if asks else 1 << 62
    bb0 = bids.peekitem(-1)[0] if bids else -1
    smin = np.minimum.accumulate(np.where(s == 1, p, 1 << 62)); smin = np.concatenate([[1 << 62], smin[:-1]])
    bmax = np.maximum.accumulate(np.where(s == 0, p, -1)); bmax = np.concatenate([[-1], bmax[:-1]])
    sure = np.where(s == 0, p < np.minimum(ba0, smin), p > np.maximum(bb0, bmax))
    cross = 0; empt = 0; rests = 0; ocross = 0
    for i in range(len(p)):
        pi, vi = int(p[i]), int(v[i])
        if s[i] == 0:
            while vi > 0 and asks and asks.peekitem(0)[0] <= pi:
                a, d = asks.peekitem(0); t = min(d, vi); vi -= t
                if t == d: del asks[a]; empt += 1
                else: asks[a] = d - t
                cross += 1
            ocross += int(vi < int(v[i]))
            if vi > 0: bids[pi] = bids.get(pi, 0) + vi; rests += 1
        else:
            while vi > 0 and bids and bids.peekitem(-1)[0] >= pi:
                b, d = bids.peekitem(-1); t = min(d, vi); vi -= t
                if t == d: del bids[b]; empt += 1
                else: bids[b] = d - t
                cross += 1
            ocross += int(vi < int(v[i]))
            if vi > 0: asks[pi] = asks.get(pi, 0) + vi; rests += 1
    stats.append((len(p), int(sure.sum()), cross, empt, rests, ocross))
st = []
for k in range(6):
    b = gen(1 << 22)
    r = b[(b["symbol_id"] == hot) & (b["action"] == wl.ADD)]
    run(r, st)
    o, sure, cr, em, rs, oc = st[-1]
    print(f"batch {k}: orders {o}, provably non-crossing {sure} ({sure / o:.5f}), crossing orders {oc / o:.3f}, "
          f"level fills {cr / o:.3f} / order, emptied levels {em / o:.3f} / order, rests {rs / o:.3f} / order; "
          f"levels {len(bids)} bid / {len(asks)} ask")
