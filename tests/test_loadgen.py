"""Native load generator (include/gome/gome_loadgen.h): the doorder.go / delorder.go
distributions at bench scale.  CPU only (host code of libgome.so)."""
import numpy as np

from gome_amd import workload as wl


def test_deterministic_and_doorder_distribution():
    a = wl.NativeStream(1000, 1.0, seed=5).batch(200000).copy()
    b = wl.NativeStream(1000, 1.0, seed=5).batch(200000).copy()
    assert a.tobytes() == b.tobytes()
    fx = 10**8
    assert set(np.unique(a["price_fx"] // 10**6)) <= set(range(1, 101))   # 2-dp prices in (0, 1]
    assert (a["price_fx"] % 10**6 == 0).all() and (a["volume_fx"] % 10**6 == 0).all()
    assert a["volume_fx"].min() >= fx // 100 and a["volume_fx"].max() <= fx
    assert (a["action"] == 1).all() and (a["uuid_id"] == 2).all()
    assert len(np.unique(a["oid_id"])) == len(a)
    assert abs(a["side"].mean() - 0.5) < 0.01
    hot = wl.ZipfSymbols(1000, 1.0).rank_to_id[0]
    share = (a["symbol_id"] == hot).mean()
    assert abs(share - wl.ZipfSymbols(1000, 1.0).share_of_top()) < 0.005


def test_cancel_mix_resends_earlier_adds_once():
    g = wl.NativeStream(200, 1.0, seed=9, del_frac=0.5, aggressive_frac=0.1)
    rec = np.concatenate([g.batch(50000).copy() for _ in range(3)])
    adds = {int(r["oid_id"]): (i, r) for i, r in enumerate(rec) if r["action"] == 1}
    dels = rec[rec["action"] == 2]
    assert abs(len(dels) / len(rec) - 0.5) < 0.02
    seen = set()
    for i in np.nonzero(rec["action"] == 2)[0][:20000]:
        d = rec[i]
        j, a = adds[int(d["oid_id"])]
        assert j < i and int(d["oid_id"]) not in seen
        seen.add(int(d["oid_id"]))
        for f in ("price_fx", "volume_fx", "symbol_id", "uuid_id", "side"):
            assert d[f] == a[f]
    a = rec[rec["action"] == 1]
    aggr = (a["volume_fx"] >= 10 * 10**8)
    assert abs(aggr.mean() - 0.1) < 0.01
    assert set(a["price_fx"][aggr & (a["side"] == 0)]) == {10**8}
    assert set(a["price_fx"][aggr & (a["side"] == 1)]) == {10**6}
    assert set(a["volume_fx"][aggr] // (10 * 10**8)) <= set(range(1, 17))


def test_rank_partition_and_deep_grid():
    z = wl.ZipfSymbols(5000, 1.0)
    shares = 0.0
    for r in range(4):
        g = wl.NativeStream(5000, 1.0, seed=1, price_decimals=4, rank=r, world=4)
        b = g.batch(20000)
        assert (z.id_to_rank[b["symbol_id"]] % 4 == r).all()
        shares += g.owned_share
        assert (b["price_fx"] % 10**4 == 0).all() and len(np.unique(b["price_fx"])) > 5000
    assert abs(shares - 1.0) < 1e-9
