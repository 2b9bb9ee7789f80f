"""HIP engine (MI355X) — the flow path's deep-book and cancel chains are enqueued only while recent
batches needed them (gome_abi.h GOME_CHAIN_QUIET).  A batch whose candidates ask for a chain the
host did not enqueue declines those books to the legacy / cold kernels: the results must not
change, only the path.  Every batch here is checked event for event against the C oracle."""
import numpy as np
import pytest

from gome_amd import workload as wl
from gome_amd.abi import GOME_FLAG_CHAINS_ALWAYS, GOME_FLAG_CHAINS_NEVER, GOME_FLAG_POISON, Engine
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books

pytestmark = pytest.mark.gpu

NSYM = 2000
CH_DEEP, CH_CANC = 1, 2


def _zipf_syms(k=8):
    z = wl.ZipfSymbols(NSYM, 1.0)
    return [int(z.rank_to_id[r]) for r in range(k)]


def _cancel_batch(n, seed, oid_off):
    """config 4's mix over the same symbols, oids moved out of the ADD streams' range."""
    b = wl.cancel_mix(n, NSYM, seed=seed, zipf_s=1.0)
    b["oid_id"] += oid_off
    return b


def _deep_batch(st4, n, oid_off):
    b = st4.batch(n)
    b["oid_id"] += oid_off
    return b


def test_chain_transitions_keep_parity():
    """ADD-only batches until both chains are dropped, then a batch with DELs (its cancel books
    declined: the chain was not enqueued), then DEL batches on the flow path again, then 4-dp
    books deep enough for the deep plan (declined once, then on it)."""
    n = 1 << 17
    eng = Engine(max_symbols=NSYM, max_batch=n, max_nodes=1 << 22, max_levels=1 << 22)
    orc = Oracle(NSYM)
    st2 = wl.Stream(NSYM, 1.0, seed=11)
    st4 = wl.Stream(NSYM, 1.0, seed=12, price_decimals=4)
    log = []

    def run(b, tag):
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), tag)
        s = eng.stats()
        log.append((tag, s["chains"], s["chains_wanted"], s["n_flow_cancels"], s["n_flow_books"]))
        return s

    for i in range(6):
        s = run(st2.batch(n), f"add {i}")
        assert s["chains_wanted"] == 0
    assert log[-1][1] == 0, log  # both chains dropped after GOME_CHAIN_QUIET quiet batches
    s = run(_cancel_batch(n, 5, 10_000_000), "dels 0")
    assert s["chains"] == 0 and s["chains_wanted"] & CH_CANC and s["n_flow_cancels"] == 0, log
    s = run(_cancel_batch(n, 6, 20_000_000), "dels 1")
    assert s["chains"] & CH_CANC and s["n_flow_cancels"] > 0, log
    for i in range(2):
        s = run(_deep_batch(st4, n, 30_000_000), f"deep {i}")
    deep = [x for x in log if x[0].startswith("deep")]
    assert deep[0][2] & CH_DEEP, log
    assert deep[-1][1] & CH_DEEP, log
    fl = eng.debug_flow_books()
    assert (fl["kind"] == 3).any(), "a 4-dp book on the deep plan once the chain is back"
    _cmp_books(eng, orc, _zipf_syms() + list(range(0, NSYM, 97)), "after transitions")
    assert eng.stats()["n_resting"] == orc.resting()


@pytest.mark.parametrize("flags", [GOME_FLAG_CHAINS_NEVER, GOME_FLAG_CHAINS_ALWAYS])
def test_chains_never_and_always(flags):
    """Deep books with DELs (config 5c's mix at a small scale): with the chains never enqueued
    every such book takes the legacy / cold kernels; always enqueued, the flow path."""
    _chains_case(flags)


def test_chains_always_after_early_plans():
    """The always-enqueued case in a process whose earlier engine ran early plans: its device memory
    comes back to the new engine as it was left.  This order faulted (an illegal access) in round 5:
    the deep level pass walked the bid sentinel's row 0 of a deep book's level table, which no prep
    writes, as a level (fc_level_lane: its FIFO head and target count came from the recycled memory;
    profiles/evidence/r05bg-r05bm)."""
    import bench
    from tests.test_gpu_early import _run as early_run
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 11)
    early_run([gen(1 << 18).copy() for _ in range(4)], 100000, "early, then chains")
    _chains_case(GOME_FLAG_CHAINS_ALWAYS)


def test_chains_always_on_poisoned_memory():
    """The same deep books with DELs on an engine whose every buffer starts 0xA5-filled
    (GOME_FLAG_POISON): before the fix, row 0's node count read 0xA5A5A5A5 and the batch failed
    with ERR_CHUNKS (the gather's claim overflowed) -- deterministically, not by the luck of what
    an earlier engine left."""
    _chains_case(GOME_FLAG_CHAINS_ALWAYS | GOME_FLAG_POISON)


def _chains_case(flags):
    n = 1 << 16
    gen_syms = 500
    eng = Engine(max_symbols=gen_syms, max_batch=n, max_nodes=1 << 21, max_levels=1 << 21, flags=flags)
    orc = Oracle(gen_syms)
    for i in range(3):
        b = wl.cancel_mix(n, gen_syms, seed=40 + i, zipf_s=1.0, price_decimals=4)
        b["oid_id"] += i * 1_000_000
        eng.submit(b)
        _cmp(eng.drain(), orc.submit(b), f"flags {flags} batch {i}")
        s = eng.stats()
        if flags & GOME_FLAG_CHAINS_NEVER:
            assert s["chains"] == 0 and s["n_flow_cancels"] == 0
        else:
            assert s["chains"] == CH_DEEP | CH_CANC
    if flags & GOME_FLAG_CHAINS_ALWAYS:
        assert eng.stats()["n_flow_cancels"] > 0
    z = wl.ZipfSymbols(gen_syms, 1.0)
    _cmp_books(eng, orc, [int(z.rank_to_id[r]) for r in range(8)] + list(range(0, gen_syms, 41)), f"flags {flags}")
