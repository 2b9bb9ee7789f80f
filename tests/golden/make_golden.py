"""Generate the golden fixtures under tests/golden/ from oracle/literal.py (the line-faithful
transliteration of the Go engine).  Run in the build container:

    python tests/golden/make_golden.py

The reference ships no tests or vectors, so these fixtures are outputs of
the transliteration, not of the Go binary: parity is pinned to the literal oracle only.
Each fixture: {"name", "doc", "batches": [[[action, OrderRequest], ...], ...],
"results": [MatchResult JSON strings in publish order], "state": {symbol: book}} where
book = {price_fx: [depth_fx, in_BUY, in_SALE, [[oid, uuid, transaction, volume_fx]...]]}.
"""
import gzip
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.literal import run_batches  # noqa: E402
from tests.helpers import literal_state_to_levels, random_batches  # noqa: E402

S = "eth2usdt"


def req(oid, side, price, vol, uuid="2", sym=S):
    return dict(uuid=uuid, oid=str(oid), symbol=sym, transaction=side, price=price, volume=vol)


A, D = 1, 2
KATS = [
    ("simple_partial_then_full", "partial fill reports the maker's remaining volume; a full "
     "fill reports its pre-fill volume (engine.go:145-194)",
     [[(A, req(1, 0, 0.5, 1.0)), (A, req(2, 1, 0.4, 0.3)), (A, req(3, 1, 0.5, 0.9))]]),
    ("multi_level_sweep", "a SALE sweeps bids best-first across levels, then rests the rest",
     [[(A, req(1, 0, 0.5, 1.0)), (A, req(2, 0, 0.6, 0.5)), (A, req(3, 0, 0.4, 2.0)),
       (A, req(4, 0, 0.6, 0.25)), (A, req(5, 1, 0.45, 2.0))]]),
    ("q1_cancel_middle", "Q1: cancel of a middle FIFO node unlinks it; a second cancel of the "
     "same oid publishes nothing",
     [[(A, req(1, 0, 0.5, 1.0)), (A, req(2, 0, 0.5, 1.0)), (A, req(3, 0, 0.5, 1.0))],
      [(D, req(2, 0, 0.5, 1.0))],
      [(D, req(2, 0, 0.5, 1.0)), (A, req(4, 1, 0.5, 3.0))]]),
    ("q2_wrong_side_cancel", "Q2: a wrong-side cancel empties the FIFO but ZREMs the other "
     "side; the stale BUY level later matches a SALE against a resting SALE",
     [[(A, req(1, 0, 0.5, 1.0))], [(D, req(1, 1, 0.5, 1.0))],
      [(A, req(2, 1, 0.5, 0.7))], [(A, req(3, 1, 0.4, 0.2))]]),
    ("q3_wrong_price_cancel", "Q3: a cancel at the wrong price finds nothing",
     [[(A, req(1, 0, 0.5, 1.0))], [(D, req(1, 0, 0.6, 1.0))], [(A, req(2, 1, 0.5, 1.0))]]),
    ("q4_admission", "Q4: DEL consumed before its ADD in the same batch drops the ADD; a "
     "duplicate ADD of the same (S, uuid, oid) in one batch is dropped",
     [[(D, req(1, 0, 0.5, 1.0)), (A, req(1, 0, 0.5, 1.0)), (A, req(2, 1, 0.6, 1.0)),
       (A, req(2, 1, 0.6, 1.0)), (A, req(3, 0, 0.7, 0.5))]]),
    ("q6_zero_volumes", "Q6: zero-volume maker yields a 0-fill and is popped; a zero-volume "
     "taker crossing yields one 0-fill event; a non-crossing zero ADD rests",
     [[(A, req(1, 0, 0.5, 0.0)), (A, req(2, 0, 0.5, 1.0))], [(A, req(3, 1, 0.5, 0.5))],
      [(A, req(4, 1, 0.5, 0.0))], [(A, req(5, 1, 0.9, 0.0))], [(A, req(6, 0, 0.95, 0.3))]]),
    ("q6_exact_fill_leaves_zero_node", "an exact fill stops (diff == 0) before a zero-volume "
     "maker behind it; depth 0 removes the level from the side set",
     [[(A, req(1, 0, 0.5, 1.0)), (A, req(2, 0, 0.5, 0.0))], [(A, req(3, 1, 0.5, 1.0))],
      [(A, req(4, 0, 0.5, 0.5))], [(A, req(5, 1, 0.3, 2.0))]]),
    ("q8_transaction_other", "Q8: Transaction outside {0,1} is treated as BUY and echoed raw",
     [[(A, req(1, 5, 0.5, 1.0)), (A, req(2, 1, 0.5, 0.4)), (A, req(3, 2, 0.6, 1.0))],
      [(A, req(4, 1, 0.55, 2.0))]]),
    ("q9_partial_then_cancel", "Q9: a cancel after a partial fill publishes and removes the "
     "remaining volume",
     [[(A, req(1, 1, 0.5, 1.0)), (A, req(2, 0, 0.5, 0.35))], [(D, req(1, 1, 0.5, 1.0))],
      [(A, req(3, 0, 0.6, 1.0))]]),
    ("uuid_not_checked_on_cancel", "the cancel lookup ignores uuid (engine.go:92-93)",
     [[(A, req(1, 0, 0.5, 1.0, uuid="alice"))], [(D, req(1, 0, 0.5, 1.0, uuid="mallory"))]]),
    ("ignored_action", "a message with Action outside {1,2} is consumed and ignored",
     [[(7, req(1, 0, 0.5, 1.0)), (A, req(2, 1, 0.5, 1.0))]]),
    ("json_escaping", "symbols/uuids with characters Go's encoder escapes (<, >, &, quotes)",
     [[(A, req(1, 0, 0.5, 1.0, uuid='a<b>&"c', sym="x&y")),
       (A, req(2, 1, 0.5, 0.5, uuid="z", sym="x&y"))]]),
]


def state_of(eng, batches):
    syms = sorted({r["symbol"] for b in batches for _, r in b})
    out = {}
    for s in syms:
        lv = literal_state_to_levels(eng.book_state(s))
        out[s] = {str(p): [d, ib, isl, [list(x) for x in fifo]] for p, (d, ib, isl, fifo) in sorted(lv.items())}
    return out


def fixture(name, doc, batches):
    eng, res = run_batches(batches)
    return {"name": name, "doc": doc,
            "batches": [[[a, r] for a, r in b] for b in batches],
            "results": res, "state": state_of(eng, batches)}


def dump(obj, name):
    with gzip.open(os.path.join(HERE, name + ".json.gz"), "wt") as f:
        json.dump(obj, f)


def load(name):
    with gzip.open(os.path.join(HERE, name + ".json.gz"), "rt") as f:
        return json.load(f)


def main():
    kats = [fixture(n, d, b) for n, d, b in KATS]
    dump(kats, "kat")
    # doorder.go-distribution stream (config-1 shape, reduced): 1 symbol, uuid 2
    rng = np.random.default_rng(20201015)
    reqs = []
    for i in range(1, 3001):
        p = round(float(rng.random()), 2) or 0.1
        v = round(float(rng.random()), 2) or 1.0
        reqs.append((A, req(i, int(rng.integers(2)), p, v)))
    b = [reqs[i:i + 750] for i in range(0, len(reqs), 750)]
    dump(fixture("doorder_3k", "doorder.go distribution, 1 symbol, 4 batches of 750", b), "doorder_3k")
    # randomized quirk mix over 3 symbols, including one hot-size batch (>= 2048 per symbol)
    rng = np.random.default_rng(77)
    b = random_batches(rng, 3, 400, symbols=("eth2usdt", "btc2usdt", "ltc2usdt"), del_frac=0.3)
    b += random_batches(rng, 1, 2600, symbols=("eth2usdt",), del_frac=0.25, oid_base=100000)
    dump(fixture("quirk_mix", "random Appendix-A quirk mix, 3 symbols + one 2600-order "
                 "single-symbol batch", b), "quirk_mix")
    print("wrote", len(kats), "KATs + 2 streams")


if __name__ == "__main__":
    main()
