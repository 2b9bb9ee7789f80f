"""ctypes bindings of include/gome/gome_abi.h (libgome.so).

The library is the product: HIP kernels for gfx950 behind a C-ABI.  There is no
CPU fallback — if libgome.so is missing or no GPU is present, the calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

from .workload import EVENT_DTYPE, LEVEL_DTYPE, NODE_DTYPE, ORDER_DTYPE

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GOME_LIB") or os.path.join(_HERE, "libgome.so")  # GOME_LIB: variant builds (tools/)
HEADER = os.path.join(os.path.dirname(_HERE), "include", "gome", "gome_abi.h")
HEADERS = [HEADER, os.path.join(os.path.dirname(_HERE), "include", "gome", "gome_loadgen.h"),
           os.path.join(os.path.dirname(_HERE), "include", "gome", "gome_host.h")]

GOME_FLAG_LEGACY_HOT = 1  # gome_config.flags: hot books on the legacy FIFO kernel
GOME_FLAG_NO_HEADROOM = 2  # gome_config.flags: no pool-headroom check before a submit
GOME_FLAG_CHAINS_ALWAYS = 4  # gome_config.flags: enqueue the deep / cancel chains on every batch
GOME_FLAG_CHAINS_NEVER = 8  # gome_config.flags: never (deep books and books with DELs: legacy / cold)
GOME_FLAG_PHASES = 16  # gome_config.flags: record the per-phase timing events (gome_stats.ms_phase)
GOME_FLAG_NO_EARLY = 32  # gome_config.flags: never plan the hottest book early
GOME_FLAG_NO_ADM_AHEAD = 64  # gome_config.flags: never run admission ahead of the batch
GOME_FLAG_POISON = 128  # gome_config.flags: test builds: device buffers start 0xA5-filled (reads of unwritten scratch show)
GOME_ABI_VERSION = 12
GOME_ORD_ADM_HOST, GOME_ORD_ADMITTED = 1, 2  # gome_order.flags: host-resolved admission (ABI 4)
GOME_MAX_INFLIGHT = 3

TOB_DTYPE = np.dtype([("symbol_id", "<u4"), ("n_levels", "<u4"), ("bid_price_fx", "<i8"), ("bid_depth_fx", "<i8"),
                      ("ask_price_fx", "<i8"), ("ask_depth_fx", "<i8"), ("bid_nodes", "<u4"), ("ask_nodes", "<u4"),
                      ("flags", "<u4"), ("pad", "<u4")])
assert TOB_DTYPE.itemsize == 56

# gome_stats.ms_phase indices (GOME_PH_*, gome_abi.h)
PHASES = ["admission", "sort", "head_prep", "head_recon", "records", "tail_prep", "tail_plan", "tail_sort",
          "tail_level", "tail_count", "tail_write", "tail_events", "near", "publish"]

GOME_OK, GOME_E_INVAL, GOME_E_CAPACITY, GOME_E_DEVICE, GOME_E_STATE, GOME_E_NOTFOUND = range(6)
STATUS_NAMES = {0: "OK", 1: "E_INVAL", 2: "E_CAPACITY", 3: "E_DEVICE", 4: "E_STATE", 5: "E_NOTFOUND"}


class GomeError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class Config(C.Structure):
    _fields_ = [("accuracy", C.c_uint32), ("device", C.c_int32), ("max_symbols", C.c_uint32),
                ("max_batch", C.c_uint32), ("max_nodes", C.c_uint64), ("max_levels", C.c_uint64),
                ("max_events", C.c_uint64), ("flags", C.c_uint32), ("abi_version", C.c_uint32),
                ("hw_queues", C.c_uint32), ("plan_cus", C.c_int32)]


assert C.sizeof(Config) == 56


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "n_orders", "n_add", "n_del", "n_dropped", "n_fills", "n_cancels", "n_rests",
        "n_events", "n_resting", "n_levels", "max_segment", "n_segments")] + [
        ("ms_total", C.c_double), ("ms_match", C.c_double), ("ms_hot", C.c_double),
        ("n_hot", C.c_uint64), ("n_hot_orders", C.c_uint64), ("n_hot_fills", C.c_uint64),
        ("n_hot_rests", C.c_uint64), ("n_hot_cancels", C.c_uint64),
        ("n_flow_books", C.c_uint64), ("n_flow_orders", C.c_uint64), ("n_flow_touches", C.c_uint64),
        ("ms_flow_plan", C.c_double), ("n_flow_head_orders", C.c_uint64),
        ("n_flow_head_touches", C.c_uint64), ("n_index_rebuilds", C.c_uint64),
        ("idx_tombstones", C.c_uint64), ("n_flow_cancels", C.c_uint64), ("ms_cold", C.c_double),
        ("lvl_used", C.c_uint64), ("n_dup_oid", C.c_uint64), ("n_flow_tail_fills", C.c_uint64),
        ("ms_phase", C.c_double * 16),
        ("ms_host_enqueue", C.c_double), ("chains", C.c_uint32), ("chains_wanted", C.c_uint32),
        ("n_quirk_checked", C.c_uint64), ("n_requalified", C.c_uint64), ("chunk_bytes", C.c_uint64),
        ("n_early", C.c_uint64), ("n_early_miss", C.c_uint64),
        ("n_adm_ahead", C.c_uint64), ("n_adm_redo", C.c_uint64),
        ("n_flow_stale", C.c_uint64), ("n_flow_bail", C.c_uint64), ("n_flow_zero", C.c_uint64),
        ("n_flow_wrong", C.c_uint64)]

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_}
        d["ms_phase"] = list(self.ms_phase)
        return d


_lib = None


def load_library(path: str = LIB_PATH) -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"libgome.so not found at {path}: build it with `python -m gome_amd.build` "
            "(the engine has no CPU fallback)")
    lib = C.CDLL(path)
    P, VP = C.POINTER, C.c_void_p
    # a host-layer-only build (host.cpp, consume.cpp, loadgen.cpp: the sanitizer build of
    # tests/test_host_sanitizers.py) has no engine entry points
    engine = hasattr(lib, "gome_create")
    if engine:
        lib.gome_create.argtypes = [P(Config), P(VP)]
        lib.gome_destroy.argtypes = [VP]
        lib.gome_destroy.restype = None
        lib.gome_last_error.argtypes = [VP]
        lib.gome_last_error.restype = C.c_char_p
        lib.gome_abi_version.restype = C.c_uint32
        lib.gome_submit_batch.argtypes = [VP, VP, C.c_size_t, C.c_uint64]
        lib.gome_submit_batch_device.argtypes = [VP, VP, C.c_size_t, C.c_uint64, VP]
        lib.gome_submit_batch_async.argtypes = [VP, VP, C.c_size_t, C.c_uint64]
        lib.gome_collect.argtypes = [VP, P(VP), P(C.c_size_t), P(Stats)]
        lib.gome_submit_batch_device_async.argtypes = [VP, VP, C.c_size_t, C.c_uint64]
        lib.gome_collect_device.argtypes = [VP, P(VP), P(C.c_size_t), P(Stats)]
        lib.gome_inflight.argtypes = [VP]
        lib.gome_inflight.restype = C.c_size_t
        lib.gome_host_alloc.argtypes = [VP, C.c_size_t, P(VP)]
        lib.gome_host_free.argtypes = [VP, VP]
        lib.gome_host_free.restype = None
        lib.gome_drain_events.argtypes = [VP, VP, C.c_size_t, P(C.c_size_t)]
        lib.gome_pending_events.argtypes = [VP]
        lib.gome_pending_events.restype = C.c_size_t
        lib.gome_device_events.argtypes = [VP, P(VP), P(C.c_size_t)]
        lib.gome_release_device_events.argtypes = [VP]
        lib.gome_debug_flow_books.argtypes = [VP, C.POINTER(C.c_uint32), C.c_size_t, C.POINTER(C.c_size_t)]
        lib.gome_debug_flow_books.restype = C.c_int32
        lib.gome_debug_peek.argtypes = [VP, C.c_uint32, C.c_uint64, C.c_uint64, VP]
        lib.gome_debug_peek.restype = C.c_int32
        if hasattr(lib, "gome_debug_fifo_shape"):  # (diagnostics; variant builds of older trees lack it)
            lib.gome_debug_fifo_shape.argtypes = [VP, C.c_uint32, VP, C.c_size_t, C.POINTER(C.c_size_t)]
            lib.gome_debug_fifo_shape.restype = C.c_int32
        lib.gome_release_device_events.restype = C.c_int32
        lib.gome_get_stats.argtypes = [VP, P(Stats)]
        lib.gome_dup_records.argtypes = [VP, P(C.c_uint32), C.c_size_t, P(C.c_size_t)]
        lib.gome_take_deferred.argtypes = [VP]
        lib.gome_top_of_book.argtypes = [VP, VP, C.c_size_t, VP]
        lib.gome_top_of_book_enqueue.argtypes = [VP, VP, C.c_size_t]
        lib.gome_top_of_book_collect.argtypes = [VP, VP, C.c_size_t, P(C.c_size_t)]
        lib.gome_snapshot_levels.argtypes = [VP, C.c_uint32, VP, C.c_size_t, P(C.c_size_t)]
        lib.gome_snapshot_fifo.argtypes = [VP, C.c_uint32, C.c_int64, VP, C.c_size_t, P(C.c_size_t)]
        lib.gome_load_books.argtypes = [VP, C.c_size_t, VP, VP, VP, VP, C.c_size_t]
    lib.gome_fixed_from_double.argtypes = [C.c_double, C.c_uint32, P(C.c_int64)]
    lib.gome_render_match_result.argtypes = [VP, VP, C.c_int64, C.c_uint32] + [C.c_char_p] * 6 + [
        VP, C.c_char_p, C.c_size_t]
    lib.gome_render_match_result.restype = C.c_int64
    lib.gome_render_link_node.argtypes = [C.c_char_p, C.c_int64, C.c_int32, C.c_int64, C.c_uint32] + [
        C.c_char_p] * 5 + [C.c_size_t]
    lib.gome_render_link_node.restype = C.c_int64
    lib.gome_render_events.argtypes = [VP, C.c_size_t, VP, C.c_size_t, C.c_uint64, C.c_uint32, VP, C.c_size_t,
                                       VP, C.c_size_t, VP, C.c_size_t, VP, VP, C.c_size_t]
    lib.gome_render_events.restype = C.c_int64
    lib.gome_render_events_mt.argtypes = [VP, C.c_size_t, VP, C.c_size_t, C.c_uint64, C.c_uint32, VP, C.c_size_t,
                                          VP, C.c_size_t, VP, C.c_size_t, VP, C.c_uint32, VP, C.c_size_t]
    lib.gome_render_events_mt.restype = C.c_int64
    lib.gome_render_events_names.argtypes = [VP, C.c_size_t, VP, C.c_size_t, C.c_uint64, C.c_uint32, VP, C.c_uint32,
                                             VP, C.c_size_t]
    lib.gome_render_events_names.restype = C.c_int64
    # gome_host.h: interning, pre-pool markers, the native OrderNode consumer
    SZ, CP = C.c_size_t, C.c_char_p
    lib.gome_names_create.restype = VP
    lib.gome_names_destroy.argtypes = [VP]
    lib.gome_names_destroy.restype = None
    lib.gome_names_intern.argtypes = [VP, C.c_int, CP, SZ]
    lib.gome_names_intern.restype = C.c_int64
    lib.gome_names_find.argtypes = [VP, C.c_int, CP, SZ]
    lib.gome_names_find.restype = C.c_int64
    lib.gome_names_count.argtypes = [VP, C.c_int]
    lib.gome_names_count.restype = SZ
    lib.gome_names_get.argtypes = [VP, C.c_int, C.c_uint32, P(SZ)]
    lib.gome_names_get.restype = VP
    lib.gome_names_table.argtypes = [VP, C.c_int]
    lib.gome_names_table.restype = VP
    lib.gome_names_tx_code.argtypes = [VP, C.c_int32]
    lib.gome_names_tx_code.restype = C.c_int32
    lib.gome_names_tx_table.argtypes = [VP]
    lib.gome_names_tx_table.restype = P(C.c_int32)
    lib.gome_names_tx_count.argtypes = [VP]
    lib.gome_names_tx_count.restype = SZ
    lib.gome_prepool_create.restype = VP
    lib.gome_prepool_destroy.argtypes = [VP]
    lib.gome_prepool_destroy.restype = None
    lib.gome_prepool_set.argtypes = [VP, CP, SZ, CP, SZ, CP, SZ]
    lib.gome_prepool_set.restype = None
    lib.gome_prepool_take.argtypes = [VP, CP, SZ, CP, SZ, CP, SZ]
    lib.gome_prepool_take.restype = C.c_int32
    lib.gome_prepool_size.argtypes = [VP]
    lib.gome_prepool_size.restype = SZ
    lib.gome_prepool_commit.argtypes = [VP]
    lib.gome_prepool_commit.restype = None
    lib.gome_prepool_abort.argtypes = [VP]
    lib.gome_prepool_abort.restype = None
    lib.gome_decode_order_nodes.argtypes = [VP, VP, SZ, C.c_uint32, VP, VP, SZ]
    lib.gome_decode_order_nodes.restype = C.c_int64
    lib.gome_consume_order_nodes.argtypes = [VP, VP, VP, VP, SZ, C.c_uint32, C.c_uint32, VP, VP, P(SZ), VP]
    lib.gome_consume_order_nodes.restype = C.c_int32
    lib.gome_consume_last_steps.argtypes = [VP, VP, SZ]
    lib.gome_consume_last_steps.restype = SZ
    lib.gome_gen_create.argtypes = [VP, P(VP)]
    lib.gome_gen_batch.argtypes = [VP, VP, C.c_size_t]
    lib.gome_gen_shares.argtypes = [VP, P(C.c_double), P(C.c_double)]
    lib.gome_gen_destroy.argtypes = [VP]
    lib.gome_gen_destroy.restype = None
    for f in ("gome_gen_create", "gome_gen_batch", "gome_gen_shares"):
        getattr(lib, f).restype = C.c_int32
    lib.gome_fixed_from_scaled.argtypes = [C.c_double, P(C.c_int64)]
    for f in ("gome_fixed_from_double", "gome_fixed_from_scaled"):
        getattr(lib, f).restype = C.c_int32
    if engine:
        for f in ("gome_create", "gome_submit_batch", "gome_submit_batch_device", "gome_drain_events",
                  "gome_device_events", "gome_get_stats", "gome_snapshot_levels", "gome_snapshot_fifo",
                  "gome_submit_batch_async", "gome_collect", "gome_host_alloc", "gome_load_books",
                  "gome_dup_records", "gome_take_deferred", "gome_top_of_book", "gome_submit_batch_device_async",
                  "gome_top_of_book_enqueue", "gome_top_of_book_collect", "gome_collect_device"):
            getattr(lib, f).restype = C.c_int32
    _lib = lib
    return lib


def declared_functions(headers=None) -> list[str]:
    """Every function the C-ABI headers (include/gome/*.h) declare."""
    txt = "".join(open(h).read() for h in (headers or HEADERS))
    return sorted(set(re.findall(r"\b(gome_[a-z_]+)\s*\(", txt)) - {"gome_status"})


def fixed_from_double(x: float, accuracy: int = 8) -> int:
    lib = load_library()
    out = C.c_int64()
    s = lib.gome_fixed_from_double(float(x), accuracy, C.byref(out))
    if s != GOME_OK:
        raise GomeError(s, f"{x!r} is outside the exact fixed-point domain at accuracy {accuracy}")
    return out.value


def fixed_from_scaled(v: float) -> int:
    """An OrderNode Price / Volume as consumed from the doOrder queue (already scaled by
    10^accuracy at gRPC time, main.go:41): exact integer below 2^53 or GomeError."""
    lib = load_library()
    out = C.c_int64()
    s = lib.gome_fixed_from_scaled(float(v), C.byref(out))
    if s != GOME_OK:
        raise GomeError(s, f"{v!r} is not an exact scaled value (integer below 2^53)")
    return out.value


def tx_table_array(table) -> np.ndarray | None:
    """Transaction code -> raw int32 table for the renderers (None = identity)."""
    if table is None:
        return None
    a = np.arange(256, dtype=np.int32)
    for code, raw in (table.items() if isinstance(table, dict) else enumerate(table)):
        a[int(code)] = int(raw)
    return a


def render_match_result(ev: np.void, taker: np.void, taker_remaining: int, symbol: str, taker_uuid: str,
                        taker_oid: str, maker_uuid: str | None, maker_oid: str | None,
                        maker_next_oid: str | None, accuracy: int = 8, tx_table=None) -> str:
    """One MatchResult line; taker_remaining = Node.Volume (workload.taker_remaining)."""
    lib = load_library()
    e = np.array([ev], dtype=EVENT_DTYPE)
    t = np.array([taker], dtype=ORDER_DTYPE)
    enc = lambda s: None if s is None else s.encode()
    tt = tx_table if isinstance(tx_table, np.ndarray) else tx_table_array(tx_table)
    size = 8192
    while True:  # a short buffer returns -(bytes needed)
        buf = C.create_string_buffer(size)
        n = lib.gome_render_match_result(e.ctypes.data, t.ctypes.data, int(taker_remaining), accuracy, symbol.encode(),
                                         taker_uuid.encode(), taker_oid.encode(), enc(maker_uuid),
                                         enc(maker_oid), enc(maker_next_oid),
                                         None if tt is None else tt.ctypes.data, buf, len(buf))
        if n >= 0:
            return buf.raw[:n].decode()
        if n == -(1 << 63):
            raise GomeError(GOME_E_INVAL, "render failed (missing argument)")
        size = -n


def render_link_node(symbol: str, price_fx: int, side: int, volume_fx: int, uuid: str, oid: str,
                     prev_oid: str | None, next_oid: str | None, accuracy: int = 8) -> str:
    """A resting node's JSON as the reference stores it in S:link:<price> (nodelink.go:119-122).
    `side` is the raw int32 Transaction value."""
    lib = load_library()
    enc = lambda s: None if s is None else s.encode()
    size = 4096
    while True:  # a short buffer returns -(bytes needed)
        buf = C.create_string_buffer(size)
        n = lib.gome_render_link_node(symbol.encode(), int(price_fx), int(side), int(volume_fx), accuracy,
                                      uuid.encode(), oid.encode(), enc(prev_oid), enc(next_oid), buf, len(buf))
        if n >= 0:
            return buf.raw[:n].decode()
        if n == -(1 << 63):
            raise GomeError(GOME_E_INVAL, "render failed (missing argument)")
        size = -n


class Engine:
    """One engine handle per GPU (include/gome/gome_abi.h)."""

    def __init__(self, max_symbols: int, max_batch: int, max_nodes: int = 1 << 20,
                 max_levels: int = 1 << 20, accuracy: int = 8, device: int = 0,
                 max_events: int = 0, flags: int = 0, hw_queues: int | None = None, plan_cus: int = 0):
        """hw_queues: the hardware queues this process's HIP runtime started with (the stream
        layout, gome_config.hw_queues); None = what gome_amd recorded at import (gome_amd.hw_queues()).
        plan_cus: CUs reserved for the hottest book's plan (0 = default, < 0 = none)."""
        from . import hw_queues as _hw_queues
        self.lib = load_library()
        if hw_queues is None:
            hw_queues = _hw_queues()
        cfg = Config(accuracy=accuracy, device=device, max_symbols=max_symbols,
                     max_batch=max_batch, max_nodes=max_nodes, max_levels=max_levels,
                     max_events=max_events, flags=flags, abi_version=GOME_ABI_VERSION,
                     hw_queues=hw_queues, plan_cus=plan_cus)
        h = C.c_void_p()
        s = self.lib.gome_create(C.byref(cfg), C.byref(h))
        if s != GOME_OK:
            raise GomeError(s, self.lib.gome_last_error(None).decode())
        self.h = h
        self.max_batch = max_batch
        self.max_symbols = max_symbols
        self.cfg_kwargs = dict(max_symbols=max_symbols, max_batch=max_batch, max_nodes=max_nodes,
                               max_levels=max_levels, accuracy=accuracy, device=device,
                               max_events=max_events, flags=flags, hw_queues=hw_queues, plan_cus=plan_cus)

    def close(self):
        if getattr(self, "h", None):
            self.lib.gome_destroy(self.h)
            self.h = None

    __del__ = close

    def _check(self, s):
        if s != GOME_OK:
            raise GomeError(s, self.lib.gome_last_error(self.h).decode())

    def submit(self, rec: np.ndarray, seq_base: int = 0):
        rec = np.ascontiguousarray(rec, dtype=ORDER_DTYPE)
        self._check(self.lib.gome_submit_batch(self.h, rec.ctypes.data, len(rec), seq_base))

    def submit_device(self, dev_ptr: int, n: int, seq_base: int = 0, stream: int | None = None):
        self._check(self.lib.gome_submit_batch_device(self.h, C.c_void_p(dev_ptr), n, seq_base,
                                                      C.c_void_p(stream or 0)))

    # ---- pipelined device path (gome_submit_batch_device_async / gome_collect_device)
    def submit_device_async(self, dev_ptr: int, n: int, seq_base: int = 0):
        """Queue a batch already in HBM (it must stay unchanged until collected)."""
        self._check(self.lib.gome_submit_batch_device_async(self.h, C.c_void_p(dev_ptr), n, seq_base))

    def collect_device(self):
        """(device pointer, count) of the oldest in-flight device batch's events and its stats."""
        p, n, st = C.c_void_p(), C.c_size_t(), Stats()
        self._check(self.lib.gome_collect_device(self.h, C.byref(p), C.byref(n), C.byref(st)))
        return (p.value or 0), n.value, st.as_dict()

    # ---- pipelined host path (gome_submit_batch_async / gome_collect)
    def host_buffer(self, n: int) -> np.ndarray:
        """Page-locked record buffer of n gome_orders (gome_host_alloc), freed with the engine."""
        p = C.c_void_p()
        self._check(self.lib.gome_host_alloc(self.h, max(n, 1) * ORDER_DTYPE.itemsize, C.byref(p)))
        buf = (C.c_char * (max(n, 1) * ORDER_DTYPE.itemsize)).from_address(p.value)
        return np.frombuffer(buf, dtype=ORDER_DTYPE)[:n]

    def submit_async(self, rec: np.ndarray, seq_base: int = 0):
        """Queue a batch (rec must stay alive and unchanged until collected)."""
        assert rec.dtype == ORDER_DTYPE and rec.flags["C_CONTIGUOUS"]
        self._check(self.lib.gome_submit_batch_async(self.h, rec.ctypes.data, len(rec), seq_base))

    def collect(self, copy: bool = True):
        """Events of the oldest in-flight batch (publish order) and its stats dict.  copy=False
        returns a view of the engine's page-locked buffer (valid until the next collect)."""
        p, n, st = C.c_void_p(), C.c_size_t(), Stats()
        self._check(self.lib.gome_collect(self.h, C.byref(p), C.byref(n), C.byref(st)))
        if n.value == 0:
            return np.zeros(0, EVENT_DTYPE), st.as_dict()
        buf = (C.c_char * (n.value * EVENT_DTYPE.itemsize)).from_address(p.value)
        ev = np.frombuffer(buf, dtype=EVENT_DTYPE)
        return (ev.copy() if copy else ev), st.as_dict()

    def inflight(self) -> int:
        return self.lib.gome_inflight(self.h)

    def drain(self) -> np.ndarray:
        got = C.c_size_t()
        self._check(self.lib.gome_drain_events(self.h, None, 0, C.byref(got)))  # collects in-flight batches
        n = self.lib.gome_pending_events(self.h)
        out = np.zeros(n, EVENT_DTYPE)
        self._check(self.lib.gome_drain_events(self.h, out.ctypes.data, n, C.byref(got)))
        return out[:got.value]

    def device_events(self):
        p, n = C.c_void_p(), C.c_size_t()
        self._check(self.lib.gome_device_events(self.h, C.byref(p), C.byref(n)))
        return p.value, n.value

    def release_device_events(self):
        """The caller consumed the last device batch's events on the device."""
        self._check(self.lib.gome_release_device_events(self.h))

    FLOW_BOOK_DTYPE = np.dtype([("kind", "<u4"), ("decline", "<u4"), ("symbol_id", "<u4"), ("orders", "<u4"),
                                ("dels", "<u4"), ("levels", "<u4"), ("w32", "<u4"), ("wsum", "<u4"),
                                ("window", "<u4"), ("deep", "<u4")])

    def debug_flow_books(self, cap: int = 4096) -> np.ndarray:
        """The last batch's hot-book routing (gome_debug_flow_books; diagnostics)."""
        out = np.zeros(cap, self.FLOW_BOOK_DTYPE)
        n = C.c_size_t()
        self._check(self.lib.gome_debug_flow_books(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), cap,
                                                   C.byref(n)))
        return out[:n.value]

    def debug_peek(self, which: int, offset: int, nbytes: int) -> bytes:
        """Raw bytes of a flow-path scratch array after the last batch (gome_debug_peek)."""
        buf = C.create_string_buffer(max(nbytes, 1))
        self._check(self.lib.gome_debug_peek(self.h, which, offset, nbytes, buf))
        return buf.raw[:nbytes]

    def debug_fifo_shape(self, symbol_id: int) -> np.ndarray:
        """Per level of a book: (price_fx, live nodes, dead slots, chunks) (gome_debug_fifo_shape)."""
        n = C.c_size_t()
        self._check(self.lib.gome_debug_fifo_shape(self.h, symbol_id, None, 0, C.byref(n)))
        out = np.zeros((n.value, 4), np.int64)
        self._check(self.lib.gome_debug_fifo_shape(self.h, symbol_id, out.ctypes.data, n.value, C.byref(n)))
        return out

    def stats(self) -> dict:
        st = Stats()
        self._check(self.lib.gome_get_stats(self.h, C.byref(st)))
        return st.as_dict()

    def dup_records(self) -> np.ndarray:
        """Batch indices of the last finished batch's ADDs rejected by the duplicate-oid rule."""
        n = C.c_size_t()
        self._check(self.lib.gome_dup_records(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, np.uint32)
        if n.value:
            self._check(self.lib.gome_dup_records(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), n.value,
                                                  C.byref(n)))
        return out

    def top_of_book(self, symbols) -> np.ndarray:
        """gome_top_of_book: best bid / ask, their depths and FIFO lengths per symbol (TOB_DTYPE)."""
        syms = np.ascontiguousarray(symbols, dtype=np.uint32)
        out = np.zeros(len(syms), TOB_DTYPE)
        self._check(self.lib.gome_top_of_book(self.h, syms.ctypes.data, len(syms), out.ctypes.data))
        return out

    def top_of_book_enqueue(self, symbols):
        """gome_top_of_book_enqueue: digests of the books as the last submitted batch leaves them,
        read on the device behind the batches in flight (collect with top_of_book_collect)."""
        syms = np.ascontiguousarray(symbols, dtype=np.uint32)
        self._check(self.lib.gome_top_of_book_enqueue(self.h, syms.ctypes.data, len(syms)))
        self._tob_n = len(syms)

    def top_of_book_collect(self) -> np.ndarray:
        n = C.c_size_t()
        out = np.zeros(getattr(self, "_tob_n", 0), TOB_DTYPE)
        self._check(self.lib.gome_top_of_book_collect(self.h, out.ctypes.data, len(out), C.byref(n)))
        return out[:n.value]

    def take_deferred(self) -> tuple[int, str]:
        """(status, message) of the first in-flight batch failure a synchronous call collected."""
        s = self.lib.gome_take_deferred(self.h)
        return s, (self.lib.gome_last_error(self.h).decode() if s != GOME_OK else "")

    def load_books(self, books) -> None:
        """gome_load_books: `books` = [(symbol_id, levels LEVEL_DTYPE ascending by price,
        nodes NODE_DTYPE in FIFO order, level by level)] into this fresh engine."""
        sym = np.array([b[0] for b in books], np.uint32)
        nlv = np.array([len(b[1]) for b in books], np.uint32)
        lv = np.concatenate([b[1] for b in books]) if books else np.zeros(0, LEVEL_DTYPE)
        nd = np.concatenate([b[2] for b in books]) if books else np.zeros(0, NODE_DTYPE)
        lv = np.ascontiguousarray(lv, LEVEL_DTYPE)
        nd = np.ascontiguousarray(nd, NODE_DTYPE)
        self._check(self.lib.gome_load_books(self.h, len(sym), sym.ctypes.data, nlv.ctypes.data, lv.ctypes.data,
                                             nd.ctypes.data, len(nd)))

    def levels(self, symbol_id: int) -> np.ndarray:
        n = C.c_size_t()
        self._check(self.lib.gome_snapshot_levels(self.h, symbol_id, None, 0, C.byref(n)))
        out = np.zeros(n.value, LEVEL_DTYPE)
        self._check(self.lib.gome_snapshot_levels(self.h, symbol_id, out.ctypes.data, n.value,
                                                  C.byref(n)))
        return out

    def fifo(self, symbol_id: int, price_fx: int) -> np.ndarray:
        n = C.c_size_t()
        self._check(self.lib.gome_snapshot_fifo(self.h, symbol_id, price_fx, None, 0, C.byref(n)))
        out = np.zeros(n.value, NODE_DTYPE)
        self._check(self.lib.gome_snapshot_fifo(self.h, symbol_id, price_fx, out.ctypes.data,
                                                n.value, C.byref(n)))
        return out
