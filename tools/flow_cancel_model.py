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


def plan_book_q(old_fifo, seg):
    """The W32C plan as built (gen_plan_asm.py, match_flow_cancel.h): per level and side only the
    depth; a DEL of maker m (level p, side s) at index i carries
        Q = VA_s,p(i) - END(m) - C,   VA = volume of the segment's side-s ADDs at p before i,
        END(m) = VA(m) + v_m (new m) or oend - D0 (old m: the old volume behind it counts),
        C = volume of side-s targets ranked behind m whose DEL comes before i,
    removes r = clamp(depth_s,p - Q, 0, v_m) (v_m: the target's full volume).  While m is live the
    makers behind it are untouched (Q of them) and, if m was partly consumed, nothing is live
    ahead of it; once m is gone the side's depth is at most Q.  Returns (r per DEL index, final
    depth per price, final side per price).""" 
    old_of = {}
    for p, fifo in old_fifo.items():
        for pos, (oid, side, rem) in enumerate(fifo):
            old_of[oid] = (p, pos, side, rem)
    add_at, tgt = {}, {}
    for i, r in enumerate(seg):
        oid = int(r["oid_id"])
        if r["action"] == 1:
            add_at[oid] = i
        elif r["action"] == 2:
            if oid in add_at and int(seg[add_at[oid]]["price_fx"]) == int(r["price_fx"]):
                if all(d[1] != add_at[oid] for d in tgt.values() if d[0] == "new"):
                    tgt[i] = ("new", add_at[oid])
            elif oid in old_of and old_of[oid][0] == int(r["price_fx"]) and oid not in add_at:
                if ("old", oid) not in tgt.values():
                    tgt[i] = ("old", oid)
    lvl_t = defaultdict(list)
    for d, (kind, x) in tgt.items():
        if kind == "old":
            lvl_t[old_of[x][0]].append(((0, old_of[x][1]), (kind, x), d))
        else:
            lvl_t[int(seg[x]["price_fx"])].append(((1, x), (kind, x), d))
    rank, tv, dt = {}, {}, {}
    for p, lst in lvl_t.items():
        lst.sort()
        for k, (_, t, d) in enumerate(lst):
            rank[t] = k
            dt[(p, k)] = d
            if t[0] == "old":
                tv[(p, k)] = (old_of[t[1]][2], old_of[t[1]][3])
            else:
                tv[(p, k)] = (int(seg[t[1]]["side"]), int(seg[t[1]]["volume_fx"]))
    d0 = {p: sum(x[2] for x in f) for p, f in old_fifo.items()}
    oend = {}
    for p, f in old_fifo.items():
        e = 0
        for oid, sd, rem in f:
            e += rem
            oend[oid] = e
    # prep: Q per DEL
    Q = {}
    for i, t in tgt.items():
        r = seg[i]
        p, s = int(r["price_fx"]), int(r["side"])
        va = sum(int(x["volume_fx"]) for x in seg[:i] if x["action"] == 1 and int(x["price_fx"]) == p and int(x["side"]) == s)
        if t[0] == "new":
            m = t[1]
            end = sum(int(x["volume_fx"]) for x in seg[:m] if x["action"] == 1 and int(x["price_fx"]) == p
                      and int(x["side"]) == s) + int(seg[m]["volume_fx"])
        else:
            end = oend[t[1]] - d0[p]
        k = rank[t]
        c = sum(v for (pp, kk), (sd, v) in tv.items() if pp == p and kk > k and sd == s and dt[(pp, kk)] < i)
        Q[i] = (va - end - c, tv[(p, k)][1])
    # the plan over side depths
    dep = defaultdict(int)   # (price, side) -> depth
    for p, fifo in old_fifo.items():
        if fifo:
            dep[(p, fifo[0][1])] = sum(x[2] for x in fifo)
    r_of = {}
    for i, r in enumerate(seg):
        a, p, v, sd = int(r["action"]), int(r["price_fx"]), int(r["volume_fx"]), int(r["side"])
        if a == 1:
            T = v
            opp = sorted((q for (q, s2), d in dep.items() if d > 0 and s2 == 1 - sd and (q >= p if sd == 1 else q <= p)),
                         reverse=(sd == 1))
            crossed = False
            for q in opp:
                crossed = True
                take = min(T, dep[(q, 1 - sd)])
                dep[(q, 1 - sd)] -= take
                T -= take
                if T <= 0:
                    break
            if crossed and T <= 0:
                continue
            dep[(p, sd)] += T
        elif a == 2 and i in tgt:
            d = dep[(p, sd)]
            q, vm = Q[i]
            rr = min(max(d - q, 0), vm)
            dep[(p, sd)] = d - rr
            r_of[i] = rr
    depth, side = defaultdict(int), {}
    for (p, s2), d in dep.items():
        if d > 0:
            depth[p] += d
            side[p] = s2
        else:
            depth.setdefault(p, 0)
    return r_of, depth, side, 0


def check(n_sym=50, batch=20000, nbatch=4, seed=1, del_frac=0.5, aggr=0.1, zipf=1.0, plan=None):
    plan = plan or plan_book
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
            r_of, depth, side, ringsum = plan(old, seg)
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
    for pl in (plan_book_q, plan_book):
        print(pl.__name__)
        check(n_sym=20, batch=6000, nbatch=3, plan=pl)
        check(n_sym=3, batch=8000, nbatch=3, seed=7, plan=pl)
    check()
    check(n_sym=3, batch=30000, nbatch=3, seed=7)
    check(n_sym=200, batch=40000, nbatch=3, seed=3, aggr=0.02)
