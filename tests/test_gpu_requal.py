"""HIP engine (MI355X) — quirk books back on the flow path.

A wrong-side cancel (Q2) or a zero-volume maker (Q6) puts a book in a state the aggregate plans
cannot express (BOOK_QUIRK), so the legacy kernel (~23x slower) applies it.  The reference's state
heals (nodepool.go:76-83, engine.go:145-175); k_requalify (match_requal.h) clears the flag once it
has.  On bench.py's config-3 stream, the hottest book gets both quirks injected in batch 1
(workload.inject_quirks, through the engine's own snapshot of the book), and every batch is
compared event for event with the C oracle; the books' levels and FIFOs at the end too."""
import numpy as np
import pytest

import bench
from gome_amd import workload as wl
from gome_amd.abi import Engine
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books, _hot_and_random

pytestmark = pytest.mark.gpu

N = 1 << 20


def _run(mode, batches=5):
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
    z = wl.ZipfSymbols(100000, 1.0)
    hot = int(z.rank_to_id[0])
    eng = Engine(max_symbols=100000, max_batch=N, max_nodes=batches * N, max_levels=1 << 22)
    orc = Oracle(100000)
    kinds, req = [], []
    for i in range(batches):
        b = gen(N).copy()
        if i == 1:
            info = wl.inject_quirks(b, hot, eng.levels(hot), lambda p: eng.fifo(hot, p), mode)
            assert info["q2_cancels"] >= 1
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"{mode} batch {i}")
        st = eng.stats()
        fl = eng.debug_flow_books()
        assert int(fl["symbol_id"][0]) == hot
        kinds.append(int(fl["kind"][0]))
        req.append((st["n_quirk_checked"], st["n_requalified"]))
    _cmp_books(eng, orc, _hot_and_random(z, 100000, k_rand=50), mode)
    assert eng.stats()["n_resting"] == orc.resting()
    return kinds, req


def test_quirks_heal_and_the_hottest_book_returns_to_the_flow_path():
    kinds, req = _run("heal")
    assert kinds[0] != 0 and kinds[1] == 0, kinds        # flow, then legacy for the injected batch
    healed = [i for i, (c, r) in enumerate(req) if r]
    assert healed and healed[0] <= 2, req                 # healed within two batches
    assert all(k != 0 for k in kinds[healed[0] + 1:]), (kinds, req)


def test_quirk_that_does_not_heal_stays_on_legacy_and_exact():
    kinds, req = _run("stuck", batches=4)
    assert kinds[0] != 0 and all(k == 0 for k in kinds[1:]), kinds
    assert all(r == 0 for _, r in req) and all(c >= 1 for c, _ in req[1:]), req
