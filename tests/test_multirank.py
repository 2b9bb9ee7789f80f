"""N>1 path on CPU: symbol sharding and the cross-rank reductions of bench.py
over a world-size-2 gloo process group.

Books never interact (ordernode.go:89-116: every key is prefixed by the symbol), so a
GPU that owns a subset of the symbols must produce exactly the events the single engine
produces for those symbols.  That is checked here with the C oracle as the engine on
each "rank" (the GPU engine is checked against the same oracle in test_gpu_parity.py)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

import bench
from gome_amd import workload as wl
from gome_amd.publisher import SUMMARY_FIELDS, SUMMARY_WORDS, SummaryPublisher
from oracle.pyoracle import Oracle


def test_shard_stream_partitions_symbols():
    world, n_sym = 4, 1000
    z = wl.ZipfSymbols(n_sym, 1.0)
    seen = []
    shares = 0.0
    for r in range(world):
        gen, share, top = bench.shard_stream(n_sym, 1.0, r, world, seed=3)
        b = gen(20000)
        ranks = z.id_to_rank[b["symbol_id"]]
        assert np.all(ranks % world == r)
        assert len(np.unique(b["oid_id"])) == len(b)
        seen.append(set(b["symbol_id"].tolist()))
        shares += share
    assert abs(shares - 1.0) < 1e-9
    for i in range(world):
        for j in range(i + 1, world):
            assert not (seen[i] & seen[j])


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_books_equal_global(world):
    """Union over ranks of per-rank events (taker_seq mapped back) == global events."""
    n_sym, seed, batch = 300, 11, 6000
    g = wl.Stream(n_sym, zipf_s=1.0, seed=seed)
    z = g.zipf
    glob = [g.batch(batch) for _ in range(3)]
    o = Oracle(n_sym)
    ev_glob = [o.submit(b) for b in glob]
    per_rank = [Oracle(n_sym) for _ in range(world)]
    for bi, b in enumerate(glob):
        ranks = z.id_to_rank[b["symbol_id"]]
        parts = []
        for r in range(world):
            idx = np.nonzero(ranks % world == r)[0]
            ev = per_rank[r].submit(b[idx])
            ev = ev.copy()
            ev["taker_seq"] = idx[ev["taker_seq"]]
            parts.append(ev)
        u = np.concatenate(parts)
        u = u[np.lexsort((u["fill_idx"], u["taker_seq"]))]
        assert len(u) == len(ev_glob[bi])
        assert u.tobytes() == ev_glob[bi].tobytes()
    assert sum(p.resting() for p in per_rank) == o.resting()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o, f, e, el, lat = bench.combine_ranks(100.0 * (rank + 1), 10.0 * (rank + 1), 7.0,
                                               1.5 + rank, [1.0 + rank, 5.0 - rank], "cpu")
        st = {"n_orders": 1000 + rank, "n_fills": 10 * rank, "n_events": 20 * rank,
              "n_resting": 5 + rank, "max_segment": 77 + rank}
        summary = torch.zeros(SUMMARY_WORDS, dtype=torch.int64)
        gathered = torch.zeros(SUMMARY_WORDS * world, dtype=torch.int64)
        pub = SummaryPublisher(world)
        for step in range(3):  # the rank-0 publisher consumes every step's gathered summaries
            bench.gather_summary(st, summary, gathered, rank, step)
            pub.consume(gathered)
        ok = pub.check(3 * (2000 + 1), 3 * 10, 3 * 20)
        p99 = bench.per_rank_values(10.0 + rank, rank, world, "cpu")  # (each rank's own p99)
        np.save(os.path.join(out_dir, f"r{rank}.npy"),
                np.array([o, f, e, el] + lat + gathered.tolist() + [float(ok), float(pub.steps)] + p99,
                         dtype=np.float64))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_reductions():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        res = [np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)]
    idx = {f: i for i, f in enumerate(SUMMARY_FIELDS)}
    for r in res:
        o, f, e, el = r[:4]
        assert o == 300.0 and f == 30.0 and e == 14.0   # sums over ranks
        assert el == 2.5                                 # max elapsed
        assert list(r[4:6]) == [2.0, 5.0]                # per-step max latency
        g = r[6:6 + SUMMARY_WORDS * world].reshape(world, SUMMARY_WORDS)
        for rk in range(world):
            row = [g[rk, idx[k]] for k in ("n_orders", "n_fills", "n_events", "n_resting", "max_segment", "rank", "step")]
            assert row == [1000 + rk, 10 * rk, 20 * rk, 5 + rk, 77 + rk, rk, 2]
        assert r[-4] == 1.0 and r[-3] == 3.0             # publisher totals == job totals
        assert list(r[-2:]) == [10.0, 11.0]              # every rank's p99, in rank order
    assert res[0].tobytes() == res[1].tobytes()


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_strong_and_weak_rank_batches(world):
    """Strong scaling splits --batch over the ranks by their symbols' share (the ranks' records
    sum to the global batch); weak scaling gives each rank its share of world x batch."""
    batch = 1 << 22
    strong = [bench.rank_batch(batch, world, bench.shard_stream(100000, 1.0, r, world, 42)[1], "strong")
              for r in range(world)]
    weak = [bench.rank_batch(batch, world, bench.shard_stream(100000, 1.0, r, world, 42)[1], "weak")
            for r in range(world)]
    assert abs(sum(strong) - batch) <= world and abs(sum(weak) - world * batch) <= world
    assert strong[0] == max(strong)  # (rank 0 owns the hottest symbol: Zipf rank 0)


def _scaling_worker(rank, world, port, out_dir, mode, batch, steps):
    """bench.py's rank code for the stream: this rank's batches at `mode`, the hottest book's orders
    per step (the serial plan that bounds the rank's batch on the GPU), every rank's p99 of it."""
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        gen, share, _ = bench.make_stream("config3", rank, world, 42)
        n = bench.rank_batch(batch, world, share, mode)
        hot = [bench.hottest_book_orders(gen(n)) for _ in range(steps)]
        p99 = bench.per_rank_values(bench.pctl(hot, 0.99), rank, world, "cpu")
        _, _, _, _, step_max = bench.combine_ranks(float(n), 0.0, 0.0, 0.0, [float(h) for h in hot], "cpu")
        np.save(os.path.join(out_dir, f"s{rank}.npy"), np.array(p99 + step_max, dtype=np.float64))
    finally:
        dist.destroy_process_group()


def _hot_p99(world, mode, batch=1 << 19, steps=6):
    if world == 1:
        gen, share, _ = bench.make_stream("config3", 0, 1, 42)
        n = bench.rank_batch(batch, 1, share, mode)
        return [bench.pctl([bench.hottest_book_orders(gen(n)) for _ in range(steps)], 0.99)]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_scaling_worker, args=(world, _free_port(), d, mode, batch, steps), nprocs=world, join=True)
        res = [np.load(os.path.join(d, f"s{r}.npy")) for r in range(world)]
    assert res[0].tobytes() == res[1].tobytes()
    return list(res[0][:world])


def test_strong_scaling_keeps_the_hottest_book_flat_in_n():
    """bench.py's default (--scaling strong) at world 2 over gloo: rank 0 still owns the hottest
    symbol, and its hottest book gets the same orders per step as one GPU's (the plan that sets the
    p99 batch latency), while weak scaling doubles it."""
    one = _hot_p99(1, "strong")[0]
    strong = _hot_p99(2, "strong")
    weak = _hot_p99(2, "weak")
    assert abs(strong[0] / one - 1.0) < 0.03, (one, strong)
    assert strong[1] < strong[0]  # (rank 1's hottest is the Zipf rank-1 symbol)
    assert abs(weak[0] / one - 2.0) < 0.06, (one, weak)
