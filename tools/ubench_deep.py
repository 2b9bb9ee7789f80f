"""Deep plan cost per record (ms_flow_plan of a one-symbol 4-dp book, W32D)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gome_amd import workload as wl  # noqa: E402
from gome_amd.abi import Engine  # noqa: E402

N = 1 << 18
for dec in (4, 3):
    st = wl.Stream(1, seed=7, price_decimals=dec)
    eng = Engine(max_symbols=1, max_batch=N, max_nodes=1 << 23, max_levels=1 << 20)
    t = []
    for i in range(6):
        b = st.batch(N)
        eng.submit(b)
        eng.drain()
        s = eng.stats()
        if i >= 2:
            t.append(s["ms_flow_plan"] * 1e6 / N)
    fb = eng.debug_flow_books(1)
    print(f"{dec}-dp: plan ns/record {np.mean(t):6.1f}  kind {int(fb['kind'][0])} levels {int(fb['levels'][0])} "
          f"touches/order {s['n_flow_touches'] / N:.2f} batch ms {s['ms_total']:.1f}")
