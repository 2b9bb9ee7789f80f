"""HIP engine (MI355X) — the hottest book planned early (match_early.h).

Pipelined device batches (three in flight) of bench.py's config-3 stream: from the second
finished batch on, each batch's hottest book is prepared and planned on the copy stream as soon as
the previous batch's plan ends.  Every batch's events are compared with the C oracle, and the
books' levels and FIFOs at the end; gome_stats.n_early counts the batches whose plan was the early
one, n_early_miss the early plans that were ready but not taken (it must stay 0).  The second test
breaks the early plan's assumptions in single batches (a DEL, oids out of order, another symbol
hottest, a zero-volume ADD) and checks that the engine stays exact and goes back to early plans
afterwards; host-resolved verdicts (one refused) keep it."""
import numpy as np
import pytest

import bench
from gome_amd import workload as wl
from gome_amd.abi import GOME_E_INVAL, GOME_FLAG_NO_EARLY, GOME_ORD_ADM_HOST, GOME_ORD_ADMITTED, Engine, GomeError
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books, _hot_and_random

pytestmark = pytest.mark.gpu

N = 1 << 18


def _run(batches, nsym, label, levels=1 << 22, **kw):
    """Submit every batch with three in flight, collect in order; per-batch stats.  kw: more
    Engine arguments (layout flags, hw_queues, plan_cus)."""
    import torch
    eng = Engine(max_symbols=nsym, max_batch=N, max_nodes=(len(batches) + 4) * N, max_levels=levels, **kw)
    orc = Oracle(nsym)
    dev = [torch.from_numpy(b.view(np.uint8).copy()).cuda() for b in batches]
    torch.cuda.synchronize()
    exp = [orc.submit(b) for b in batches]
    stats = []
    nxt = 0
    for k in range(len(batches)):
        while nxt < len(batches) and nxt < k + 3:
            eng.submit_device_async(dev[nxt].data_ptr(), N, 0)
            nxt += 1
        _, n, st = eng.collect_device()  # (its events move to the host queue at the next collect)
        assert n == len(exp[k]), f"{label} batch {k}: {n} events vs oracle {len(exp[k])}"
        stats.append(st)
    _cmp(eng.drain(), np.concatenate(exp), label)
    return eng, orc, stats


def test_early_plans_on_the_config3_stream_are_exact():
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
    batches = [gen(N).copy() for _ in range(8)]
    eng, orc, stats = _run(batches, 100000, "early")
    early = [int(s["n_early"]) for s in stats]
    assert sum(int(s["n_early_miss"]) for s in stats) == 0, early
    assert sum(early[3:]) >= 4, early  # (the first batches have no finished predecessor to go by)
    z = wl.ZipfSymbols(100000, 1.0)
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=50), "early")
    assert eng.stats()["n_resting"] == orc.resting()


def test_early_plan_declines_keep_the_engine_exact():
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 7)
    z = wl.ZipfSymbols(100000, 1.0)
    hot, second = int(z.rank_to_id[0]), int(z.rank_to_id[1])
    batches = [gen(N).copy() for _ in range(13)]
    rng = np.random.default_rng(5)

    def hot_rows(b, sym=hot):
        return np.flatnonzero(b["symbol_id"] == sym)

    # 4: a DEL of a maker of the hot book (an oid of batch 0) in its segment
    b = batches[4]
    r = hot_rows(b)[100]
    b0 = batches[0]
    b["action"][r] = wl.DEL
    b["oid_id"][r] = b0["oid_id"][hot_rows(b0)[5]]
    b["side"][r] = b0["side"][hot_rows(b0)[5]]
    # 6: two of the hot book's oids swapped (out of batch order; still unique)
    b = batches[6]
    r = hot_rows(b)
    b["oid_id"][r[10]], b["oid_id"][r[20]] = b["oid_id"][r[20]], b["oid_id"][r[10]]
    # 8: another symbol is the hottest this batch (9: the hot book again, after another)
    b = batches[8]
    r = rng.choice(np.flatnonzero(b["symbol_id"] != hot), size=len(hot_rows(b)) + 5000, replace=False)
    b["symbol_id"][r] = second
    # 10: host-resolved admission on the hot book, one record refused
    b = batches[10]
    r = hot_rows(b)
    b["flags"][r] = GOME_ORD_ADM_HOST | GOME_ORD_ADMITTED
    b["flags"][r[30]] = GOME_ORD_ADM_HOST
    # 12: a zero-volume ADD (Q6) in the hot book
    batches[12]["volume_fx"][hot_rows(batches[12])[50]] = 0
    eng, orc, stats = _run(batches, 100000, "declines")
    early = [int(s["n_early"]) for s in stats]
    assert sum(int(s["n_early_miss"]) for s in stats) == 0, early
    for k in (4, 5, 6, 8, 9):  # (12: a zero-volume ADD may plan early since round 5: Q6 on the flow path)
        assert early[k] == 0, (k, early)
    # 7: the batch after a declined early plan (6) is early-eligible; its early chain reads the book
    # state batch 6's fallback plan wrote, which runs on the plan stream right behind k_x_take so the
    # chain is ordered after it (it ran on the flow stream beside that chain)
    for k in (3, 7, 10, 11):
        assert early[k] == 1, (k, early)
    _cmp_books(eng, orc, list(_hot_and_random(z, 100000, k_rand=50)) + [second], "declines")
    assert eng.stats()["n_resting"] == orc.resting()


def test_early_plans_of_a_deep_book_are_exact():
    """Config 5 (1M symbols, 4-dp prices): the hottest book has thousands of levels, so its plans
    are the deep ones (W32DV), and so is its early plan (k_xd_prep_a / k_xd_sort_new / k_xd_prep_b:
    the previous plan's live levels merged with the batch's sorted prices)."""
    gen, _, _ = bench.make_stream("config5", 0, 1, 42)
    batches = [gen(N).copy() for _ in range(8)]
    eng, orc, stats = _run(batches, 1000000, "deep early", levels=1 << 25)  # (16-level blocks per book)
    early = [int(s["n_early"]) for s in stats]
    assert sum(int(s["n_early_miss"]) for s in stats) == 0, early
    assert sum(early[3:]) >= 4, early
    assert all(int(s["chains"]) & 1 for s in stats[2:])  # (the deep chain: the book is deep)
    z = wl.ZipfSymbols(1000000, 1.0)
    _cmp_books(eng, orc, _hot_and_random(z, 1000000, k_hot=2, k_rand=20), "deep early")
    assert eng.stats()["n_resting"] == orc.resting()


def test_early_plans_of_pipelined_host_batches_are_exact():
    """The host path (gome_submit_batch_async / gome_collect: records copied in on the copy stream,
    events copied out): the early record work runs behind each batch's H2D on the copy stream and
    the plan on the early stream."""
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 21)
    batches = [gen(N).copy() for _ in range(8)]
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=12 * N, max_levels=1 << 22)
    orc = Oracle(100000)
    bufs = [eng.host_buffer(N) for _ in batches]
    for b, buf in zip(batches, bufs):
        buf[:] = b
    stats, nxt = [], 0
    for k in range(len(batches)):
        while nxt < len(batches) and nxt < k + 3:
            eng.submit_async(bufs[nxt], 0)
            nxt += 1
        ev, st = eng.collect()
        _cmp(ev, orc.submit(batches[k]), f"host early batch {k}")
        stats.append(st)
    early = [int(s["n_early"]) for s in stats]
    assert sum(int(s["n_early_miss"]) for s in stats) == 0, early
    assert sum(early[3:]) >= 4, early
    z = wl.ZipfSymbols(100000, 1.0)
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=30), "host early")


def test_rejected_batch_between_early_plans():
    """A batch the engine rejects (a record outside the domain: nothing of it is applied) while the
    next batch's early plan is already being prepared from it: that plan must not be taken, and
    the batches after it are exact and planned early again."""
    import torch
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 33)
    batches = [gen(N).copy() for _ in range(9)]
    batches[4]["symbol_id"][777] = 100000  # (>= max_symbols: the whole batch is rejected)
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=13 * N, max_levels=1 << 22)
    orc = Oracle(100000)
    dev = [torch.from_numpy(b.view(np.uint8).copy()).cuda() for b in batches]
    torch.cuda.synchronize()
    exp = [None if k == 4 else orc.submit(b) for k, b in enumerate(batches)]
    early, got, nxt = [], [], 0
    for k in range(len(batches)):
        while nxt < len(batches) and nxt < k + 3:
            eng.submit_device_async(dev[nxt].data_ptr(), N, 0)
            nxt += 1
        if k == 4:
            with pytest.raises(GomeError) as ei:
                eng.collect_device()
            assert ei.value.status == GOME_E_INVAL
            early.append(0)
            continue
        _, n, st = eng.collect_device()
        assert n == len(exp[k]), f"batch {k}"
        early.append(int(st["n_early"]))
        assert int(st["n_early_miss"]) == 0, k
    _cmp(eng.drain(), np.concatenate([e for e in exp if e is not None]), "around a rejected batch")
    assert early[5] == 0 and sum(early[6:]) >= 2, early
    z = wl.ZipfSymbols(100000, 1.0)
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=30), "around a rejected batch")


def test_early_plan_off_is_the_same_engine():
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 11)
    batches = [gen(N).copy() for _ in range(6)]
    _, _, stats = _run(batches, 100000, "early off", flags=GOME_FLAG_NO_EARLY)
    assert all(int(s["n_early"]) == 0 for s in stats)
