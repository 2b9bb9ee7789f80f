"""Pin the C restatement (oracle/gome_oracle.c) to the literal transliteration of the Go
engine (oracle/literal.py): identical MatchResult JSON byte streams (rendered by the
product's C++ renderer) and identical Redis-schema book state, on randomized streams
that exercise every Appendix-A quirk.  CPU only.

PARITY UNPINNED against the reference itself (no Go toolchain, no reference fixtures)."""
import numpy as np
import pytest

from oracle.literal import run_batches
from oracle.pyoracle import Oracle
from tests.helpers import (Interner, engine_state_to_levels, literal_state_to_levels,
                           random_batches, render_events, requests_to_records)


def _run_both(batches, symbols):
    eng, lit = run_batches(batches)
    names = Interner()
    for s in symbols:
        names.id("sym", s)
    orc = Oracle(max_symbols=len(symbols))
    got = []
    for b in batches:
        rec = requests_to_records(b, names)
        got += render_events(orc.submit(rec), rec, names)
    return eng, lit, orc, names, got


def _first_diff(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i, x, y
    return min(len(a), len(b)), None, None


@pytest.mark.parametrize("seed", range(40))
def test_literal_equals_c_oracle(seed):
    symbols = ("eth2usdt", "btc2usdt")
    rng = np.random.default_rng(1000 + seed)
    batches = random_batches(rng, n_batches=4, batch=50, symbols=symbols,
                             del_frac=0.15 + 0.4 * (seed % 3) / 2)
    eng, lit, orc, names, got = _run_both(batches, symbols)
    assert len(got) == len(lit), _first_diff(got, lit)
    assert got == lit, _first_diff(got, lit)
    for s in symbols:
        assert engine_state_to_levels(orc, names.id("sym", s), names) == \
            literal_state_to_levels(eng.book_state(s))


def test_doorder_distribution_single_symbol():
    """Config-1 shape (doorder.go): 1 symbol, uuid 2, fresh oids, 2-dp prices/volumes."""
    rng = np.random.default_rng(42)
    reqs = []
    for i in range(1, 1500):
        p = round(float(rng.random()), 2) or 0.1
        v = round(float(rng.random()), 2) or 1.0
        reqs.append((1, dict(uuid="2", oid=str(i), symbol="eth2usdt",
                             transaction=int(rng.integers(2)), price=p, volume=v)))
    batches = [reqs[i:i + 250] for i in range(0, len(reqs), 250)]
    eng, lit, orc, names, got = _run_both(batches, ("eth2usdt",))
    assert len(lit) > 500
    assert got == lit, _first_diff(got, lit)
    assert engine_state_to_levels(orc, 0, names) == literal_state_to_levels(eng.book_state("eth2usdt"))
