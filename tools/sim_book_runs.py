"""How much parallelism hides in one book's serial plan?  

Simulates one book under the doorder distribution (doorder.go:37-49: side U{0,1}, 2-dp price and
volume in (0, 1]) at the aggregate level the flow plan works on, and counts, per order, whether
it crosses and whether it empties a level.  A run of orders between two emptied levels could in
principle be applied with wave-wide scans (rests and partial fills at a fixed top of book); the
mean run length bounds what such a scheme could gain over the serial plan.

Measured (700k orders): 43% of orders cross, 24% empty a level, 1.32 level touches per order,
mean run between emptied levels 4.1 orders.
"""
import sys

import numpy as np


def main(n=700000, seed=1):
    rng = np.random.default_rng(seed)
    p = np.rint(rng.random(n) * 100).astype(int)
    p[p == 0] = 10
    v = np.rint(rng.random(n) * 100).astype(int)
    v[v == 0] = 100
    s = rng.integers(0, 2, n)
    bid, ask = [0] * 102, [0] * 102
    cross = exh = touches = 0
    runs, last = [], 0
    for i in range(n):
        pi, vi, ex = p[i], v[i], False
        book, own, rng_ = (ask, bid, range(1, pi + 1)) if s[i] == 0 else (bid, ask, range(100, pi - 1, -1))
        for k in rng_:
            if vi <= 0:
                break
            if book[k] > 0:
                touches += 1
                t = min(vi, book[k])
                book[k] -= t
                vi -= t
                ex |= book[k] == 0
        if vi > 0:
            own[pi] += vi
            touches += 1
        cross += vi < v[i]
        if ex:
            exh += 1
            runs.append(i - last)
            last = i
    print(f"cross {cross / n:.3f}  empties a level {exh / n:.3f}  touches/order {touches / n:.3f}  "
          f"mean run {np.mean(runs):.2f}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 700000)
