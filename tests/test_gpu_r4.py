"""HIP engine (MI355X) — round-4 boundary coverage: top-of-book digests read behind batches in
flight (gome_top_of_book_enqueue / _collect), the u32 oid watermark of the fresh-batch fast path
crossed and wrapped, the duplicate-oid rule (queue order) on the flow / cold / legacy routing, the
consumer leg of bench.py, and a Router over handles on different devices when the box has them."""
import numpy as np
import pytest

import bench
from gome_amd import workload as wl
from gome_amd.abi import Engine, GomeError, GOME_E_NOTFOUND, GOME_E_STATE
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books

pytestmark = pytest.mark.gpu


def test_top_of_book_enqueue_reads_behind_the_batches_in_flight():
    """Digests enqueued between two pipelined device batches describe the books after the first
    and before the second: equal to the synchronous gome_top_of_book taken at that point on a
    twin engine, for the 64 hottest books."""
    import torch
    n = 1 << 18
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
    bs = [gen(n).copy() for _ in range(4)]
    dev = [torch.from_numpy(b.view(np.uint8)).cuda() for b in bs]
    z = wl.ZipfSymbols(100000, 1.0)
    hot = z.rank_to_id[:64]
    a = Engine(max_symbols=100000, max_batch=n, max_nodes=8 * n, max_levels=1 << 22)
    b = Engine(max_symbols=100000, max_batch=n, max_nodes=8 * n, max_levels=1 << 22)
    with pytest.raises(GomeError) as ei:
        a.top_of_book_collect()
    assert ei.value.status == GOME_E_NOTFOUND
    got, want = [], []
    a.submit_device_async(dev[0].data_ptr(), n, seq_base=0)
    for k in range(1, 4):
        a.top_of_book_enqueue(hot)  # behind batch k-1
        with pytest.raises(GomeError) as ei:
            a.top_of_book_enqueue(hot)
        assert ei.value.status == GOME_E_STATE
        a.submit_device_async(dev[k].data_ptr(), n, seq_base=k * n)
        a.collect_device()
        a.release_device_events()
        got.append(a.top_of_book_collect())
        b.submit_device(dev[k - 1].data_ptr(), n, seq_base=(k - 1) * n)
        b.release_device_events()
        want.append(b.top_of_book(hot))
    a.collect_device()
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    assert (got[-1]["flags"] == 3).all()


def test_oid_watermark_crossed_and_wrapped_stays_exact():
    """the fresh-batch fast path (k_adm_pre: oids increasing and above a watermark)
    across the u32 oid range: fresh batches just below 2^32, a batch whose oids wrap to small
    values mid-batch (not fresh: the tables decide), wrapped batches, then fresh ones again, some
    of whose oids name nodes still resting from before the wrap (the duplicate-oid rule rejects
    exactly those).  Every event, the rejected records and the books against the C oracle."""
    n = 60000
    g = wl.Stream(64, seed=8)
    eng = Engine(max_symbols=64, max_batch=n, max_nodes=1 << 21, max_levels=1 << 16)
    orc = Oracle(64)
    nxt = (1 << 32) - 3 * n - 1000
    dups = 0
    for i in range(7):
        b = g.batch(n)
        o = (np.arange(nxt, nxt + n, dtype=np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        b["oid_id"] = o
        nxt += n
        if i == 5:
            nxt = 1  # the interner starts over: low ids again, some still resting
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"batch {i}")
        d = orc.dup_records()
        assert np.array_equal(eng.dup_records(), d), f"batch {i}"
        dups += len(d)
    assert dups > 0
    _cmp_books(eng, orc, range(64), "oid wrap")
    assert eng.stats()["n_resting"] == orc.resting()


def test_consumer_leg_runs():
    out = bench.consumer_leg("config3", 100000, 1 << 13, 42, batch=1 << 11, threads=2)
    assert out["messages"] == 1 << 13 and out["messages_per_s"] > 0 and out["matchresults"] > 1000
    assert out["render_events_per_s"]["1"] > 0 and out["render_events_per_s"]["2"] > 0


def test_router_on_two_devices_matches_one_engine():
    """a Router over handles on devices 0 and 1, driven from pool threads (the device
    guard at every C-ABI entry point switches each call to its handle's device)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU on this box: cross-device Router use is untested here (INTEGRATION.md)")
    from gome_amd.router import Router, owner_table
    rec = wl.cancel_mix(40000, 16, seed=3)
    r = Router([Engine(max_symbols=16, max_batch=40000, device=d) for d in (0, 1)], owner_table(16, 2))
    one = Engine(max_symbols=16, max_batch=40000)
    for b in wl.split_batches(rec, 10000):
        r.submit(b)
        one.submit(b)
        _cmp(r.drain(), one.drain(), "router on two devices")
    r.close()
