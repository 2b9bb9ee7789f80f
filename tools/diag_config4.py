"""Diagnostics: the config-4 hot book's DEL windows and plan time (gome_debug_peek)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gome_amd import workload as wl  # noqa: E402
from gome_amd.abi import Engine  # noqa: E402
from tools.debug_fc_tail import FCDEL, HDR  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
ns = wl.NativeStream(100000, 1.0, seed=int(os.environ.get('SEED', '42')), price_decimals=2, del_frac=0.5, aggressive_frac=0.1)
eng = Engine(max_symbols=100000, max_batch=N, max_nodes=1 << 24, max_levels=1 << 25)
for bi in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
    b = ns.batch(N)
    eng.submit(b)
    eng.release_device_events() if False else eng.drain()
    st = eng.stats()
    allb = eng.debug_flow_books()
    bad = allb[allb["kind"] == 0]
    print(f"   declined candidates: {len(bad)} of {len(allb)}; orders {int(bad['orders'].sum())}; "
          f"reasons {np.unique(bad['decline'], return_counts=True)}; biggest {bad[np.argsort(-bad['orders'].astype(np.int64))][:3][['orders','dels','levels','wsum','window','w32','decline']].tolist()}")
    fb = allb[:8]
    hdr = np.frombuffer(eng.debug_peek(0, 0, HDR.itemsize * len(fb)), HDR)
    x = hdr[0]
    beg, end = int(x["beg"]), int(x["end"])
    d = np.frombuffer(eng.debug_peek(2, FCDEL.itemsize * beg, FCDEL.itemsize * (end - beg)), FCDEL)
    sym = int(x["sym"])
    seg = b[b["symbol_id"] == sym]
    isdel = seg["action"] == wl.DEL
    dd = d[isdel]
    eff = dd[dd["kind"] != 0]
    nb = eff["nb"].astype(np.int64)
    print(f"batch {bi}: plan {st['ms_flow_plan']:.2f} ms, hot n={end - beg} dels={int(isdel.sum())} "
          f"effective={len(eff)} (new {int((eff['kind'] == 1).sum())}, old {int((eff['kind'] == 2).sum())}) "
          f"cancels={int((eff['ct'] != 0xFFFFFFFF).sum())} levels={x['nl']} wsum={x['nbsum']} maxwin={x['ncancel']}")
    if len(nb):
        q = np.percentile(nb, [50, 90, 99, 100])
        print(f"   window n_b p50 {q[0]:.0f} p90 {q[1]:.0f} p99 {q[2]:.0f} max {q[3]:.0f}; >63: {float((nb > 63).mean()):.3f}"
              f"  mean chunks {float(np.ceil(nb / 63).mean()):.2f}")
    print("   head routes (kind, decline, window sum, window):", [(int(x["kind"]), int(x["decline"]), int(x["wsum"]), int(x["window"])) for x in fb])
