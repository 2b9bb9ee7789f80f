"""HIP engine (MI355X) -- the pipelined device path (gome_submit_batch_device_async /
gome_collect_device): batch k+1 is enqueued before batch k is collected, the records and the
events stay in HBM.  Every batch's events must equal the C oracle's, in publish order, whether
they are read through the device pointer's count, drained after a later batch was queued, or
moved to the host queue by the next collect."""
import numpy as np
import pytest
import torch

from gome_amd import workload as wl
from gome_amd.abi import Engine, GomeError
from oracle.pyoracle import Oracle
from tests.test_gpu_v4 import _cmp, _cmp_books

pytestmark = pytest.mark.gpu

NSYM = 300


def _dev(b):
    return torch.from_numpy(b.view(np.uint8).copy()).cuda()


def test_device_pipeline_matches_oracle():
    st = wl.Stream(NSYM, 1.0, seed=31)
    n = 1 << 15
    eng = Engine(max_symbols=NSYM, max_batch=n, max_nodes=1 << 20, max_levels=1 << 20)
    orc = Oracle(NSYM)
    host = [st.batch(n) for _ in range(6)]
    dev = [_dev(b) for b in host]
    torch.cuda.synchronize()
    exp = [orc.submit(b) for b in host]
    seq = [0] * 6  # (the oracle numbers each batch from 0)
    # three in flight (GOME_MAX_INFLIGHT), then collect the oldest: its count is the oracle's
    host.append(st.batch(n))
    dev.append(_dev(host[-1]))
    torch.cuda.synchronize()
    exp.append(orc.submit(host[-1]))
    seq.append(0)
    for k in range(3):
        eng.submit_device_async(dev[k].data_ptr(), n, seq[k])
    with pytest.raises(GomeError):
        eng.submit_device_async(dev[3].data_ptr(), n, seq[3])  # (GOME_MAX_INFLIGHT)
    p0, n0, s0 = eng.collect_device()
    assert p0 and n0 == len(exp[0]) and s0["n_orders"] == n
    # a drain now: batch 0's device events first, then batches 1 and 2 (collected into the queue)
    got = eng.drain()
    _cmp(got, np.concatenate([exp[0], exp[1], exp[2]]), "drain after collect")
    # steady state: submit k+1, collect k, the consumer releases k's events on the device
    eng.submit_device_async(dev[3].data_ptr(), n, seq[3])
    eng.submit_device_async(dev[4].data_ptr(), n, seq[4])
    _, n3, _ = eng.collect_device()
    assert n3 == len(exp[3])
    eng.release_device_events()
    eng.submit_device_async(dev[5].data_ptr(), n, seq[5])
    _, n4, _ = eng.collect_device()  # (batch 4's events; 5 in flight)
    assert n4 == len(exp[4])
    _, n5, _ = eng.collect_device()  # batch 4's events move to the host queue first
    assert n5 == len(exp[5])
    got = eng.drain()
    _cmp(got, np.concatenate([exp[4], exp[5]]), "spilled then device")
    eng.submit_device_async(dev[6].data_ptr(), n, seq[6])
    eng.collect_device()
    _cmp(eng.drain(), exp[6], "last")
    _cmp_books(eng, orc, range(0, NSYM, 7), "after")
    assert eng.stats()["n_resting"] == orc.resting()


def test_collect_device_rejects_host_batches():
    st = wl.Stream(NSYM, 1.0, seed=32)
    eng = Engine(max_symbols=NSYM, max_batch=4096)
    buf = eng.host_buffer(4096)
    buf[:] = st.batch(4096)
    eng.submit_async(buf)
    with pytest.raises(GomeError):
        eng.collect_device()
    eng.collect()
