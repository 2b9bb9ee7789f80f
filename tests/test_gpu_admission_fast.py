"""HIP engine (MI355X) — the fresh-batch admission path (pipeline.h k_adm_pre / k_adm_ctl): a batch
with no DEL whose oids strictly increase and lie above the watermark of every earlier batch takes
its verdicts without the admission tables.  Batches just outside that domain must take the table
passes (duplicate-oid probe, batch rule); every batch here is checked against the C oracle."""
import numpy as np
import pytest

from gome_amd import workload as wl
from gome_amd.abi import Engine
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books

pytestmark = pytest.mark.gpu

NSYM = 64


def _run(eng, orc, b, tag):
    eng.submit(b)
    _cmp(eng.drain(), orc.submit(b), tag)
    return eng.stats()


def test_watermark_and_monotonicity_route_to_the_tables():
    st = wl.Stream(NSYM, 1.0, seed=21)
    eng = Engine(max_symbols=NSYM, max_batch=1 << 14)
    orc = Oracle(NSYM)
    a = st.batch(8000)                      # fresh: oids 1..8000
    s = _run(eng, orc, a, "fresh")
    assert s["n_dup_oid"] == 0
    # increasing oids that start below the watermark: some still rest -> the duplicate rule drops
    # them (the tables' resting probe), exactly as the oracle does
    b = st.batch(8000)
    b["oid_id"] = np.arange(4001, 12001, dtype=np.uint32)
    s = _run(eng, orc, b, "below watermark")
    assert s["n_dup_oid"] > 0
    # fresh again above the new watermark
    c = st.batch(8000)
    c["oid_id"] = np.arange(20001, 28001, dtype=np.uint32)
    _run(eng, orc, c, "fresh above")
    # one repeated oid in an otherwise increasing batch (not strictly increasing): the batch rule
    d = st.batch(8000)
    d["oid_id"] = np.arange(30001, 38001, dtype=np.uint32)
    d["oid_id"][5000] = d["oid_id"][4999]
    d["uuid_id"][5000] = 7
    _run(eng, orc, d, "one repeat")
    # host-resolved admission inside a fresh batch: the host's verdicts stand
    e = st.batch(8000)
    e["oid_id"] = np.arange(40001, 48001, dtype=np.uint32)
    e["flags"] = 1 | 2                      # GOME_ORD_ADM_HOST | GOME_ORD_ADMITTED
    e["flags"][::3] = 1                     # every third ADD without its marker
    s = _run(eng, orc, e, "host verdicts")
    assert s["n_dropped"] >= 8000 // 3
    _cmp_books(eng, orc, range(NSYM), "after")
    assert eng.stats()["n_resting"] == orc.resting()
