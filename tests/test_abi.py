"""CPU checks of the C-ABI boundary: libgome.so loads and exports every function the
header declares; host helpers (fixed-point conversion, MatchResult rendering) behave
as the reference; gome_create fails loudly (no CPU fallback) when no GPU is present."""
import ctypes as C
import math

import numpy as np
import pytest

from gome_amd import abi
from oracle.literal import scale


def test_library_exports_every_declared_symbol():
    lib = abi.load_library()
    names = abi.declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(lib, n), n
    assert lib.gome_abi_version() == abi.GOME_ABI_VERSION == 12


def test_record_layouts_match_header():
    from gome_amd.workload import EVENT_DTYPE, LEVEL_DTYPE, NODE_DTYPE, ORDER_DTYPE
    assert ORDER_DTYPE.itemsize == 32 and EVENT_DTYPE.itemsize == 48
    assert LEVEL_DTYPE.itemsize == 24 and NODE_DTYPE.itemsize == 24
    assert C.sizeof(abi.Config) == 56


@pytest.mark.parametrize("x", [0.0, 0.1, 0.29, 0.57, 1.0, 12.34, 0.00000001, 123456.12345678,
                               -0.5, 90071992.54740991, 3.0e7, 1e-8])
def test_fixed_point_matches_decimal_path(x):
    """ordernode.go:76-87 via shopspring/decimal: exact where the product is an integer."""
    v = scale(x, 8)
    assert v == int(v)
    assert abi.fixed_from_double(x, 8) == int(v)


def test_fixed_point_random_two_decimals():
    rng = np.random.default_rng(0)
    for k in rng.integers(0, 10**6, 2000):
        x = round(float(k) / 100, 2)
        assert abi.fixed_from_double(x, 8) == int(scale(x, 8))


@pytest.mark.parametrize("x", [0.123456789, 1e-9, 2.0 ** 53, 1e300, math.nan, math.inf, 0.1 + 0.2])
def test_fixed_point_rejects_outside_domain(x):
    """Q5: more than `accuracy` decimals (or >= 2^53 scaled) is outside the exact domain."""
    with pytest.raises(abi.GomeError):
        abi.fixed_from_double(x, 8)


def test_fixed_point_other_accuracy():
    assert abi.fixed_from_double(0.5, 2) == 50
    with pytest.raises(abi.GomeError):
        abi.fixed_from_double(12.5, 0)
    assert abi.fixed_from_double(7.0, 0) == 7


def test_create_without_gpu_fails_loudly():
    pytest.importorskip("torch")
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(abi.GomeError) as ei:
        abi.Engine(max_symbols=4, max_batch=16)
    assert ei.value.status == abi.GOME_E_DEVICE


def test_create_refuses_a_stale_abi_version():
    """gome_config.abi_version sits where ABI <= 10 had a zero pad word: a caller built against an
    older header is refused before anything else (no silent argument shift)."""
    lib = abi.load_library()
    for v in (0, 11, 13):
        cfg = abi.Config(max_symbols=4, max_batch=16, max_nodes=64, max_levels=64, abi_version=v)
        h = C.c_void_p()
        assert lib.gome_create(C.byref(cfg), C.byref(h)) == abi.GOME_E_INVAL
        msg = lib.gome_last_error(None).decode()
        assert f"abi_version is {v}" in msg and f"ABI {abi.GOME_ABI_VERSION}" in msg, msg


def test_hw_queue_count_parsing():
    """gome_amd records the hardware queues HIP will have; odd values of the variable read as
    unset (HIP's default 4) instead of raising at import."""
    import gome_amd
    assert gome_amd._parse_queues("16") == 16 and gome_amd._parse_queues(" 8 ") == 8
    for bad in ("", "abc", "0", "-3", None, "4.5"):
        assert gome_amd._parse_queues(bad) is None
    assert gome_amd.hw_queues() >= 4


# ---- ABI v4 boundary fixes ------------------------------------------------------------
@pytest.mark.parametrize("v", [0.0, 1.0, 50000000.0, 29000000.0, 2.0 ** 53 - 1, -12345.0, 1e15])
def test_fixed_from_scaled_accepts_exact_integers(v):
    """doOrder-queue OrderNodes carry Price / Volume already scaled at gRPC time (main.go:41,
    ordernode.go:76-87): the consumer checks, it does not re-scale."""
    assert abi.fixed_from_scaled(v) == int(v)


@pytest.mark.parametrize("v", [0.5, 28999999.999999996, 2.0 ** 53, -(2.0 ** 53), math.nan, math.inf, 1e300])
def test_fixed_from_scaled_rejects_non_integers(v):
    with pytest.raises(abi.GomeError):
        abi.fixed_from_scaled(v)


def test_scaled_path_equals_decimal_path():
    """NewOrderNode's scaling (literal.scale) then gome_fixed_from_scaled == the decimal path."""
    rng = np.random.default_rng(3)
    for k in rng.integers(1, 10**6, 500):
        x = round(float(k) / 100, 2)
        assert abi.fixed_from_scaled(scale(x, 8)) == abi.fixed_from_double(x, 8)


def test_q8_transaction_257_kat_vs_literal():
    """Q8: Transaction values outside {0,1} (257, -3, 2^31-1) are BUY and echoed raw
    (ordernode.go:95, nodepool.go:89).  Records carry interned codes; the renderer maps them
    back through the tx table.  JSON byte-identical to the literal transliteration."""
    from oracle.literal import run_batches
    from oracle.pyoracle import Oracle
    from tests.helpers import Interner, render_events, requests_to_records
    req = lambda a, oid, tx, p, v: (a, dict(uuid="u1", oid=str(oid), symbol="eth2usdt",
                                            transaction=tx, price=p, volume=v))
    batches = [[req(1, 1, 1, 0.5, 1.0), req(1, 2, 257, 0.6, 0.25), req(1, 3, -3, 0.5, 0.5),
                req(1, 4, 2**31 - 1, 0.4, 0.3)],
               [req(1, 5, 1, 0.3, 2.0), req(2, 4, 2**31 - 1, 0.4, 0.3), req(1, 6, 257, 0.7, 0.1)]]
    _, lit = run_batches(batches)
    names = Interner()
    names.id("sym", "eth2usdt")
    orc = Oracle(1)
    got = []
    for b in batches:
        rec = requests_to_records(b, names)
        assert set(rec["side"]) <= set(range(5))
        got += render_events(orc.submit(rec), rec, names)
    assert got == lit
    assert any('"Transaction":257' in j for j in got)
    assert any('"Transaction":2147483647' in j for j in got)
