"""What the reference does in the quirk batches the GPU tests hand over (CPU, the C oracle).

tests/test_gpu_requal.py's `heal` stream hands its injected batch to the legacy kernel with the
hazard bit HZ_STALE.  The reason is a reference behaviour outside any aggregate plan:
a wrong-side cancel (Q2) leaves the best bid a member of S:BUY with no FIFO; a SALE later rests at
that price (depth and FIFO are keyed by price, nodepool.go:61-83), and a later SALE taker reads
S:BUY at or above its price (GetReverseDepth, nodepool.go:86-99), meets that price and fills
against the resting SALE.  This pins it: the oracle publishes exactly such a same-side fill in
batch 1, at the stale price, and none in the batch before (and none without the injection)."""
import numpy as np

import bench
from gome_amd import workload as wl
from oracle.pyoracle import Oracle

N = 1 << 20


def _same_side_fills(mode):
    gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
    hot = int(wl.ZipfSymbols(100000, 1.0).rank_to_id[0])
    orc = Oracle(100000)
    out, info = [], None
    for i in range(2):
        b = gen(N).copy()
        if i == 1 and mode != "none":
            info = wl.inject_quirks(b, hot, orc.levels(hot), lambda p: orc.fifo(hot, p), mode)
        ev = orc.submit(b)
        tk = b[ev["taker_seq"]]
        fills = (ev["kind"] == 1) & (tk["symbol_id"] == hot)
        out.append(ev[fills & (ev["maker_side"] == tk["side"])])
    return out, info


def test_heal_batch_holds_a_same_side_fill_at_the_stale_price():
    (b0, b1), info = _same_side_fills("heal")
    assert len(b0) == 0
    assert len(b1) == 1 and int(b1["price_fx"][0]) == info["q2_price"], b1
    assert int(b1["maker_side"][0]) == 1  # (GOME_SALE: a SALE maker filled by a SALE taker)


def test_q2heal_alone_does_the_same_and_the_clean_stream_never_does():
    (_, b1), info = _same_side_fills("q2heal")
    assert len(b1) >= 1 and set(b1["price_fx"].tolist()) == {info["q2_price"]}, b1
    (c0, c1), _ = _same_side_fills("none")
    assert len(c0) == 0 and len(c1) == 0
