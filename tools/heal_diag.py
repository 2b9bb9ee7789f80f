"""Which hazard hands the hottest book over in a quirk batch (FlowHdr::haz's HZ_* bits, read back
through gome_debug_peek).  Replays tests/test_gpu_requal.py's `_run(mode)` stream for two batches
(the quirks injected in batch 1) and prints the bits after each batch, with the oracle's verdict.
  python tools/heal_diag.py [mode] [test|bench]"""
import struct
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402
from gome_amd import workload as wl  # noqa: E402
from gome_amd.abi import Engine  # noqa: E402

HZ = {1: "ZREST0", 2: "ZCONS0", 4: "ZSTOP", 8: "ZTAKER", 16: "ZDELEMPTY", 32: "ZDEL", 64: "STALE"}
HAZ_OFF = 144  # FlowHdr::haz (match_flow.h)


def main(mode="heal", where="test"):
    """where: "test" (tests/test_gpu_requal.py's stream, 1 Mi orders, quirks in batch 1) or "bench"
    (bench.py's config-3 stream, 4 Mi orders, quirks in batch 3, the first timed one)."""
    if where == "bench":
        gen, _, _ = bench.make_stream("config3", 0, 1, 42)
        n, at = 1 << 22, 3
    else:
        gen, _, _ = bench.shard_stream(100000, 1.0, 0, 1, 42)
        n, at = 1 << 20, 1
    hot = int(wl.ZipfSymbols(100000, 1.0).rank_to_id[0])
    eng = Engine(max_symbols=100000, max_batch=n, max_nodes=(at + 4) * n, max_levels=1 << 23)
    for i in range(at + 1):
        b = gen(n).copy()
        if i == at:
            print(wl.inject_quirks(b, hot, eng.levels(hot), lambda p: eng.fifo(hot, p), mode))
        eng.submit(b)
        eng.drain()
        haz = struct.unpack("<I", eng.debug_peek(0, HAZ_OFF, 4))[0]
        st = eng.stats()
        print(f"batch {i}: haz {haz:#x} {[v for k, v in HZ.items() if haz & k]} bail {int(st['n_flow_bail'])} "
              f"zero {int(st['n_flow_zero'])} wrong {int(st['n_flow_wrong'])} kind {int(eng.debug_flow_books()['kind'][0])}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
