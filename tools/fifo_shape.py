"""FIFO shape of the hottest books after a few bench batches (gome_debug_fifo_shape): live
nodes, dead slots still linked (cancelled or consumed makers behind the head) and chunks per
level.  usage: python tools/fifo_shape.py [workload] [batches] [books]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from gome_amd import workload as wl  # noqa: E402
from gome_amd.abi import Engine  # noqa: E402


def main(workload="config5c", batches=8, books=2):
    W = bench.WORKLOADS[workload]
    n = 1 << 22
    gen, _, _ = bench.make_stream(workload, 0, 1, 42)
    eng = Engine(max_symbols=W["symbols"], max_batch=n, max_nodes=3 * n + (1 << 20),
                 max_levels=(64 << 20) + 2 * n)
    g = wl.NativeStream(W["symbols"], W["zipf"], seed=42, price_decimals=W["decimals"])
    syms = [int(g.zipf.rank_to_id[r]) for r in range(books)]
    for i in range(batches):
        eng.submit(gen(n).copy())
        eng.drain()
        for s in syms:
            sh = eng.debug_fifo_shape(s)
            live, dead, nch = sh[:, 1], sh[:, 2], sh[:, 3]
            top = np.argsort(-nch)[:5]
            print(f"batch {i} sym {s}: levels {len(sh)} live {live.sum()} dead {dead.sum()} chunks {nch.sum()} "
                  f"max chunks {nch.max() if len(sh) else 0}; top levels (live, dead, chunks): "
                  f"{[tuple(int(v) for v in sh[k, 1:]) for k in top]}", flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "config5c", int(a[1]) if len(a) > 1 else 8, int(a[2]) if len(a) > 2 else 2)
