"""Design check (CPU, not product) of the flow plan with cancels.

Per book, the serial plan keeps per price level k: depth_k (live volume) and R_k (volume that
ever arrived, in arrival coordinates from the old FIFO head).  A targeted maker m (one some DEL
of the batch re-sends) occupies [E_m, E_m + v_m) in arrival coordinates.  At DEL_m:

    r_m = clamp(E_m + v_m - G_k + Xb_m, 0, v_m),   G_k = R_k - depth_k (removed volume)
    Xb_m = sum of v_j over targeted makers j behind m at level k whose DEL came before

Makers behind m live at DEL_m's time are untouched, so their cancels removed v_j exactly;
when m is gone the clamp gives 0.  Xb_m is a window of the level's ring of targeted makers
(ranks rank_m+1 .. rank_m+n_b), ring capacity C_k = max(n_b) + 1 (rounded to a power of 2).
This model replays a book's segment that way and compares every cancel's remaining volume,
every level's final depth and side set with the C oracle.
"""
import sys
from collections import defaultdict

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from gome_amd import workload as wl  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402


def plan_book(old_fifo, seg):
    """old_fifo: {price: [(oid, side, rem), ...]} live resting makers in FIFO order.
    seg: records of one book (one batch, consume order).  Returns (cancel r per DEL index,
    final depth per price, final side per price, max ring sum)."""
    # ---- prep: resolve DEL targets (new: earlier ADD of the segment; old: a live old node)
    old_of = {}
    for p, fifo in old_fifo.items():
        for pos, (oid, side, rem) in enumerate(fifo):
            old_of[oid] = (p, pos, side, rem)
    add_at = {}
    tgt = {}   # del index -> ("new", add index) | ("old", oid)
    for i, r in enumerate(seg):
        oid = int(r["oid_id"])
        if r["action"] == 1:
            add_at[oid] = i
        elif r["action"] == 2:
            if oid in add_at and int(seg[add_at[oid]]["price_fx"]) == int(r["price_fx"]):
                tgt[i] = ("new", add_at[oid])
            elif oid in old_of and old_of[oid][0] == int(r["price_fx"]):
                tgt[i] = ("old", oid)
    # ranks per level: old targets in FIFO order, then new targets in ADD order
    lvl_t = defaultdict(list)   # price -> [(key, target id)]
    for d, (kind, x) in tgt.items():
        if kind == "old":
            p, pos, _, _ = old_of[x]
            lvl_t[p].append(((0, pos), ("old", x)))
        else:
            lvl_t[int(seg[x]["price_fx"])].append(((1, x), ("new", x)))
    rank = {}
    cold = defaultdict(int)
    for p, lst in lvl_t.items():
        lst.sort()
        for k, (_, t) in enumerate(lst):
            rank[t] = (p, k)
        cold[p] = sum(1 for key, _ in lst if key[0] == 0)
    # windows: n_b(DEL d) = #targets at the level arrived before d with rank > rank_m
    arrivals = defaultdict(list)  # price -> sorted add indices of new targets
    for t, (p, k) in rank.items():
        if t[0] == "new":
            arrivals[p].append(t[1])
    for p in arrivals:
        arrivals[p].sort()
    nb, C = {}, defaultdict(lambda: 1)
    for d, t in tgt.items():
        t = ("old", t[1]) if t[0] == "old" else ("new", t[1])
        p, k = rank[t]
        arrived = cold[p] + int(np.searchsorted(arrivals[p], d))
        nb[d] = arrived - k - 1
        C[p] = max(C[p], nb[d] + 1, cold[p])
    # ---- the serial plan over aggregates
    depth = defaultdict(int)
    side = {}
    R = defaultdict(int)
    ring = {}   # (price, rank) -> [end, v, xv]
    for p, fifo in old_fifo.items():
        e = 0
        for pos, (oid, sd, rem) in enumerate(fifo):
            if ("old", oid) in rank:
                ring[rank[("old", oid)]] = [e + rem, rem, 0]
            e += rem
        depth[p] = e
        R[p] = e
        if fifo:
            side[p] = fifo[0][1]
    r_of = {}
    for i, r in enumerate(seg):
        a, p, v = int(r["action"]), int(r["price_fx"]), int(r["volume_fx"])
        if a == 1:
            t = ("new", i)
            if t in rank:
                ring[rank[t]] = [0, 0, 0]  # cleared at the ADD (slot reuse)
            sale = r["side"] == 1
            T = v
            # sweep the opposite side, best first (GetReverseDepth + Match)
            opp = sorted((q for q in depth if depth[q] > 0 and side.get(q) == (0 if sale else 1)
                          and (q >= p if sale else q <= p)), reverse=sale)
            crossed = False
            for q in opp:
                crossed = True
                take = min(T, depth[q])
                depth[q] -= take
                T -= take
                if T <= 0:
                    break
            if crossed and T <= 0:
                continue
            E = R[p]
            R[p] += T
            depth[p] += T
            side[p] = 1 if sale else 0
            if t in rank:
                ring[rank[t]] = [E + T, T, 0]
        elif a == 2 and i in tgt:
            t = tgt[i]
            pk = rank[t]
            p0 = pk[0]
            end, vm, _ = ring[pk]
            xb = sum(ring[(p0, pk[1] + 1 + l)][2] for l in range(nb[i]))
            G = R[p0] - depth[p0]
            rr = min(max(end - G + xb, 0), vm)
            ring[pk][2] = vm  # DELed: behind-makers' windows see v
            r_of[i] = rr
            if rr > 0:
                depth[p0] -= rr
    return r_of, depth, side, sum(1 << int(np.ceil(np.log2(c))) for c in C.values())


def check(n_sym=50, batch=20000, nbatch=4, seed=1, del_frac=0.5, aggr=0.1, zipf=1.0):
    g = wl.NativeStream(n_sym, zipf, seed=seed, del_frac=del_frac, aggressive_frac=aggr)
    orc = Oracle(n_sym)
    worst = 0
    for bi in range(nbatch):
        b = g.batch(batch).copy()
        for s in range(n_sym):
            old = {}
            for lv in orc.levels(s):
                f = orc.fifo(s, int(lv["price_fx"]))
                if len(f):
                    old[int(lv["price_fx"])] = [(int(x["oid_id"]), int(x["side"]), int(x["volume_fx"])) for x in f]
            seg = b[b["symbol_id"] == s]
            r_of, depth, side, ringsum = plan_book(old, seg)
            worst = max(worst, ringsum)
            idx = np.nonzero(b["symbol_id"] == s)[0]
            ev = orc_events_for(orc, b, s) if False else None
            s_r = {int(k): v for k, v in r_of.items()}
            # oracle truth: apply the batch later; compare cancels per DEL via events
            seg_truth[s] = (idx, s_r, depth, side)
        ev = orc.submit(b)
        canc = ev[ev["kind"] == 2]
        got = {}
        for s, (idx, s_r, depth, side) in seg_truth.items():
            for li, rr in s_r.items():
                if rr > 0:
                    got[int(idx[li])] = rr
        exp = {int(e["taker_seq"]): int(e["maker_volume_fx"]) for e in canc}
        assert got == exp, f"batch {bi}: {len(got)} vs {len(exp)} cancels; " \
            f"diff {[k for k in set(got) | set(exp) if got.get(k) != exp.get(k)][:5]}"
        for s, (idx, s_r, depth, side) in seg_truth.items():
            lv = {int(x["price_fx"]): x for x in orc.levels(s)}
            for p, d in depth.items():
                od = int(lv[p]["depth_fx"]) if p in lv else 0
                assert d == od, (bi, s, p, d, od)
                if d > 0:
                    assert bool(lv[p]["in_sale"]) == (side[p] == 1) and bool(lv[p]["in_buy"]) == (side[p] == 0)
        seg_truth.clear()
        print(f"batch {bi}: {len(exp)} cancels exact, depths exact; max ring slots {worst}")


seg_truth = {}

if __name__ == "__main__":
    check()
    check(n_sym=3, batch=30000, nbatch=3, seed=7)
    check(n_sym=200, batch=40000, nbatch=3, seed=3, aggr=0.02)
