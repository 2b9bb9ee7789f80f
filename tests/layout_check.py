"""The stream layouts real hosts get, checked against the C oracle at bench size.

The engine picks its stream layout from gome_config (hw_queues, plan_cus, GOME_FLAG_NO_EARLY /
_NO_ADM_AHEAD):

* >= 8 hardware queues (what gome_amd asks HIP for): cold books beside the tail's chain, the hottest
  book planned early (§4.8), admission ahead (§4.9), 8 CUs reserved for the hottest plan;
* < 8 (HIP's default 4, e.g. a Go host that does not set GPU_MAX_HW_QUEUES): the four-stream layout,
  cold books on the caller's stream, no early plan, no admission ahead, no plan stream;
* plan_cus < 0 (a host that keeps every CU shared, e.g. beside RCCL): no CU-masked plan stream.

check_layout() runs bench.py's config-3 and config-4 streams (five 4 Mi-order batches each: early
plans and admission ahead need finished batches before them) through the pipelined device path
(three batches in flight) and config 3 through the pipelined host path (two in flight), every event
against the C oracle, and the books of the 8 hottest and 50 random symbols at the end.  Run as a script it does the same in a fresh
process (tests/test_a_layouts_gpu.py starts it with GPU_MAX_HW_QUEUES=4 before the test process
touches the GPU) and prints one JSON line.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import gome_amd  # noqa: E402,F401  (before torch: the hardware-queue request)
import numpy as np  # noqa: E402

N = 1 << 22
_EXP: dict = {}


def _cmp(got, exp, tag):
    assert len(got) == len(exp), f"{tag}: {len(got)} events vs oracle {len(exp)}"
    if len(got) and not np.array_equal(got, exp):
        bad = int(np.nonzero(got != exp)[0][0])
        raise AssertionError(f"{tag}: first mismatch at event {bad}:\n gpu={got[bad]}\n orc={exp[bad]}")


def _cmp_books(eng, orc, syms, tag):
    for s in syms:
        lv_g, lv_o = eng.levels(int(s)), orc.levels(int(s))
        assert np.array_equal(lv_g, lv_o), f"{tag}: levels of symbol {s}"
        for p in lv_o["price_fx"]:
            assert np.array_equal(eng.fifo(int(s), int(p)), orc.fifo(int(s), int(p))), f"{tag}: fifo {s}@{p}"


def _stream(workload, k=5):
    import bench
    from gome_amd import workload as wl
    from oracle.pyoracle import Oracle
    if workload not in _EXP:
        gen, _, _ = bench.make_stream(workload, 0, 1, 42)
        batches = [gen(N).copy() for _ in range(k)]
        orc = Oracle(100000)
        exp = [orc.submit(b) for b in batches]
        z = wl.ZipfSymbols(100000, 1.0)
        syms = [int(z.rank_to_id[r]) for r in range(8)]
        syms += [int(x) for x in np.random.default_rng(0).choice(100000, 50, replace=False)]
        _EXP[workload] = (batches, exp, orc, syms)
    return _EXP[workload]


def _engine(nb, kw):
    from gome_amd.abi import Engine
    return Engine(max_symbols=100000, max_batch=N, max_nodes=(nb + 4) * N, max_levels=(nb + 4) * N, **kw)


def run_device(workload, kw, label):
    """Three batches in flight on the device path; per-batch stats."""
    import torch
    batches, exp, orc, syms = _stream(workload)
    eng = _engine(len(batches), kw)
    dev = [torch.from_numpy(b.view(np.uint8).copy()).cuda() for b in batches]
    torch.cuda.synchronize()
    stats, nxt = [], 0
    for k in range(len(batches)):
        while nxt < len(batches) and nxt < k + 3:
            eng.submit_device_async(dev[nxt].data_ptr(), N, 0)
            nxt += 1
        _, n, st = eng.collect_device()
        assert n == len(exp[k]), f"{label} batch {k}: {n} events vs oracle {len(exp[k])}"
        stats.append(st)
    _cmp(eng.drain(), np.concatenate(exp), label)
    _cmp_books(eng, orc, syms, label)
    assert eng.stats()["n_resting"] == orc.resting(), label
    eng.close()
    return stats


def run_host(workload, kw, label):
    """Two batches in flight on the host path (H2D and D2H on the copy stream)."""
    batches, exp, orc, syms = _stream(workload)
    eng = _engine(len(batches), kw)
    bufs = []
    for b in batches:
        hb = eng.host_buffer(len(b))
        hb[:] = b
        bufs.append(hb)
    stats, nxt = [], 0
    for k in range(len(batches)):
        while nxt < len(batches) and nxt < k + 2:
            eng.submit_async(bufs[nxt], 0)
            nxt += 1
        ev, st = eng.collect()
        _cmp(ev, exp[k], f"{label} batch {k}")
        stats.append(st)
    _cmp_books(eng, orc, syms, label)
    eng.close()
    return stats


def check_layout(kw: dict, tag: str) -> dict:
    """Every leg exact; returns the layout's per-batch early / admission-ahead counts."""
    out = {}
    for wk in ("config3", "config4"):
        st = run_device(wk, kw, f"{tag} {wk} device")
        out[f"{wk}_device"] = dict(early=[int(s["n_early"]) for s in st],
                                   adm_ahead=[int(s["n_adm_ahead"]) for s in st],
                                   flow_cancels=[int(s["n_flow_cancels"]) for s in st])
    st = run_host("config3", kw, f"{tag} config3 host")
    out["config3_host"] = dict(early=[int(s["n_early"]) for s in st])
    return out


if __name__ == "__main__":
    kw = json.loads(sys.argv[1]) if len(sys.argv) > 1 else {}
    res = check_layout(kw, "child")
    res["hw_queues"] = gome_amd.hw_queues()
    res["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES")
    print(json.dumps(res))
