"""ctypes wrapper of oracle/gome_oracle.c (TEST INFRASTRUCTURE ONLY; see that file).

PARITY UNPINNED: pinned only against oracle/literal.py and the fixtures it generated.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from gome_amd.abi import Stats as _Stats  # noqa: E402  (the gome_stats layout; no library load)
from gome_amd.workload import EVENT_DTYPE, LEVEL_DTYPE, NODE_DTYPE, ORDER_DTYPE  # noqa: E402

LIB = os.path.join(_ROOT, "oracle", "build", "liboracle.so")


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            from gome_amd.build import build_oracle
            build_oracle()
        L = C.CDLL(LIB)
        VP = C.c_void_p
        L.oracle_create.argtypes = [C.c_uint32]
        L.oracle_create.restype = VP
        L.oracle_destroy.argtypes = [VP]
        L.oracle_submit.argtypes = [VP, VP, C.c_uint64]
        L.oracle_submit.restype = C.c_int
        L.oracle_num_events.argtypes = [VP]
        L.oracle_num_events.restype = C.c_uint64
        L.oracle_events.argtypes = [VP]
        L.oracle_events.restype = VP
        L.oracle_clear_events.argtypes = [VP]
        L.oracle_get_stats.argtypes = [VP, C.POINTER(_Stats)]
        L.oracle_resting.argtypes = [VP]
        L.oracle_resting.restype = C.c_uint64
        L.oracle_snapshot_levels.argtypes = [VP, C.c_uint32, VP, C.c_uint64]
        L.oracle_snapshot_levels.restype = C.c_uint64
        L.oracle_snapshot_fifo.argtypes = [VP, C.c_uint32, C.c_int64, VP, C.c_uint64]
        L.oracle_snapshot_fifo.restype = C.c_uint64
        L.oracle_levels_total.argtypes = [VP]
        L.oracle_levels_total.restype = C.c_uint64
        L.oracle_dup_records.argtypes = [VP, VP, C.c_uint64]
        L.oracle_dup_records.restype = C.c_uint64
        _lib = L
    return _lib


class Oracle:
    def __init__(self, max_symbols: int):
        self.L = lib()
        self.h = self.L.oracle_create(max_symbols)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.oracle_destroy(self.h)
            self.h = None

    def submit(self, rec: np.ndarray) -> np.ndarray:
        """Apply one batch; return its events (publish order)."""
        rec = np.ascontiguousarray(rec, dtype=ORDER_DTYPE)
        self.L.oracle_clear_events(self.h)
        if self.L.oracle_submit(self.h, rec.ctypes.data, len(rec)) != 0:
            raise ValueError("symbol_id out of range")
        n = self.L.oracle_num_events(self.h)
        if n == 0:
            return np.zeros(0, EVENT_DTYPE)
        buf = (C.c_char * (n * EVENT_DTYPE.itemsize)).from_address(self.L.oracle_events(self.h))
        return np.frombuffer(bytes(buf), dtype=EVENT_DTYPE).copy()

    def stats(self) -> dict:
        s = _Stats()
        self.L.oracle_get_stats(self.h, C.byref(s))
        return {n: getattr(s, n) for n, _ in s._fields_}

    def dup_records(self) -> np.ndarray:
        """Batch indices of the last batch's ADDs rejected by the duplicate-oid rule (Q7)."""
        n = self.L.oracle_dup_records(self.h, None, 0)
        out = np.zeros(n, np.uint32)
        if n:
            self.L.oracle_dup_records(self.h, out.ctypes.data, n)
        return out

    def levels_total(self) -> int:
        return self.L.oracle_levels_total(self.h)

    def resting(self) -> int:
        return self.L.oracle_resting(self.h)

    def levels(self, sym: int) -> np.ndarray:
        n = self.L.oracle_snapshot_levels(self.h, sym, None, 0)
        out = np.zeros(n, LEVEL_DTYPE)
        self.L.oracle_snapshot_levels(self.h, sym, out.ctypes.data, n)
        return out

    def fifo(self, sym: int, price: int) -> np.ndarray:
        n = self.L.oracle_snapshot_fifo(self.h, sym, price, None, 0)
        out = np.zeros(n, NODE_DTYPE)
        self.L.oracle_snapshot_fifo(self.h, sym, price, out.ctypes.data, n)
        return out
