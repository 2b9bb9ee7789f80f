"""HIP engine (MI355X) — admission ahead of the batch (pipeline.h k_adm_verify).

Pipelined device batches of a stream one book dominates and that does not plan early (config 4:
half the records DELs): each batch's admission passes run on the early stream while the batch
before is in its hottest plan, without the resting probe; at the batch's own time k_adm_verify
checks that no ADD's key could rest (oid at or below its book's oid_max, the book not empty) and
runs the passes again with the probe where one could.  gome_stats.n_adm_ahead / n_adm_redo count
both.  Every batch's events are compared with the C oracle, and the books at the end."""
import numpy as np
import pytest

import bench
from gome_amd import workload as wl
from gome_amd.abi import GOME_E_INVAL, GOME_FLAG_NO_ADM_AHEAD, Engine, GomeError
from oracle.pyoracle import Oracle
from tests.test_gpu_early import N, _run
from tests.test_gpu_v4 import _cmp, _cmp_books, _hot_and_random

pytestmark = pytest.mark.gpu


def _config4(k, seed):
    gen, _, _ = bench.make_stream("config4", 0, 1, seed)
    return [gen(N).copy() for _ in range(k)]


def test_admission_ahead_on_the_config4_stream_is_exact():
    batches = _config4(8, 42)
    eng, orc, stats = _run(batches, 100000, "adm ahead")
    ahead = [int(s["n_adm_ahead"]) for s in stats]
    assert sum(ahead[2:]) >= 4, ahead
    assert all(int(s["n_adm_redo"]) == 0 for s in stats), ahead  # (fresh oids: no key can rest)
    z = wl.ZipfSymbols(100000, 1.0)
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=50), "adm ahead")
    assert eng.stats()["n_resting"] == orc.resting()


def test_admission_ahead_redone_where_a_key_may_rest():
    """ADDs carrying oids of earlier ADDs of their book (the duplicate-oid rule, Q7: rejected while
    the first still rests): the ahead verdicts cannot stand, the batch's own admission runs again
    with the probe, and the events are the oracle's."""
    batches = _config4(9, 7)
    z = wl.ZipfSymbols(100000, 1.0)
    hot = int(z.rank_to_id[0])
    for k, src in ((5, 1), (7, 6)):
        b, b0 = batches[k], batches[src]
        rows = np.flatnonzero((b["symbol_id"] == hot) & (b["action"] == wl.ADD))
        old = np.flatnonzero((b0["symbol_id"] == hot) & (b0["action"] == wl.ADD))
        for j in range(8):  # (some of them still rest, some were filled or cancelled)
            b["oid_id"][rows[100 + 7 * j]] = b0["oid_id"][old[40 * j]]
    eng, orc, stats = _run(batches, 100000, "adm redo")
    ahead = [int(s["n_adm_ahead"]) for s in stats]
    redo = [int(s["n_adm_redo"]) for s in stats]
    assert ahead[5] == 1 and ahead[7] == 1, ahead
    assert redo[5] == 1 and redo[7] == 1, redo
    assert redo[6] == 0 and redo[8] == 0, redo
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=30), "adm redo")
    assert eng.stats()["n_resting"] == orc.resting()


def test_rejected_batch_with_admission_ahead():
    """A record outside the domain in a batch whose admission ran ahead: the ahead pass's input
    error reaches the batch (rejected whole), and the batches around it are exact."""
    import torch
    batches = _config4(8, 33)
    batches[4]["symbol_id"][999] = 100000
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=12 * N, max_levels=1 << 22)
    orc = Oracle(100000)
    dev = [torch.from_numpy(b.view(np.uint8).copy()).cuda() for b in batches]
    torch.cuda.synchronize()
    exp = [None if k == 4 else orc.submit(b) for k, b in enumerate(batches)]
    nxt, ahead = 0, []
    for k in range(len(batches)):
        while nxt < len(batches) and nxt < k + 3:
            eng.submit_device_async(dev[nxt].data_ptr(), N, 0)
            nxt += 1
        if k == 4:
            with pytest.raises(GomeError) as ei:
                eng.collect_device()
            assert ei.value.status == GOME_E_INVAL
            continue
        _, n, st = eng.collect_device()
        assert n == len(exp[k]), f"batch {k}"
        ahead.append(int(st["n_adm_ahead"]))
    _cmp(eng.drain(), np.concatenate([e for e in exp if e is not None]), "around a rejected batch")
    assert sum(ahead[2:]) >= 3, ahead
    z = wl.ZipfSymbols(100000, 1.0)
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=30), "around a rejected batch")


def test_admission_ahead_off():
    _, _, stats = _run(_config4(5, 11), 100000, "adm ahead off", flags=GOME_FLAG_NO_ADM_AHEAD)
    assert all(int(s["n_adm_ahead"]) == 0 for s in stats)


def test_admission_ahead_soak():
    """32 pipelined config-4 batches: every one after the first admits ahead, none redoes it, and
    the events and books stay the oracle's."""
    batches = _config4(32, 101)
    eng, orc, stats = _run(batches, 100000, "adm ahead soak")
    ahead = [int(s["n_adm_ahead"]) for s in stats]
    assert sum(ahead) >= 30 and all(int(s["n_adm_redo"]) == 0 for s in stats), ahead
    z = wl.ZipfSymbols(100000, 1.0)
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=50), "adm ahead soak")
    assert eng.stats()["n_resting"] == orc.resting()


def test_config5c_pipelined_exact():
    """Config 5c's stream (deep books with DELs) pipelined three deep at 1 Mi orders per batch:
    admission ahead, the head's busy levels' cancel ranks a block each (k_fd_crank_big) and the
    hottest book's reconstruction by level (k_deep_level_hot) together, against the C oracle."""
    import torch
    n = 1 << 20
    gen, _, _ = bench.make_stream("config5c", 0, 1, 42)
    batches = [gen(n).copy() for _ in range(6)]
    eng = Engine(max_symbols=1_000_000, max_batch=n, max_nodes=8 * n, max_levels=(64 << 20) + 2 * n)
    orc = Oracle(1_000_000)
    dev = [torch.from_numpy(b.view(np.uint8).copy()).cuda() for b in batches]
    torch.cuda.synchronize()
    exp = [orc.submit(b) for b in batches]
    ahead, nxt = [], 0
    for k in range(len(batches)):
        while nxt < len(batches) and nxt < k + 3:
            eng.submit_device_async(dev[nxt].data_ptr(), n, 0)
            nxt += 1
        _, cnt, st = eng.collect_device()
        assert cnt == len(exp[k]), f"5c batch {k}: {cnt} events vs oracle {len(exp[k])}"
        ahead.append(int(st["n_adm_ahead"]))
    _cmp(eng.drain(), np.concatenate(exp), "5c pipelined")
    assert sum(ahead[1:]) >= 4, ahead
    z = wl.ZipfSymbols(1_000_000, 1.0)
    _cmp_books(eng, orc, _hot_and_random(z, 1_000_000, k_hot=4, k_rand=30), "5c pipelined")
    assert eng.stats()["n_resting"] == orc.resting()
