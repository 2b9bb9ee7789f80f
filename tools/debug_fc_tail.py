"""Diagnostics for the flow path's cancel prep (match_flow_cancel.h): run a fuzz stream and, for
books the prep declined, dump the DEL records behind the decline (gome_debug_peek)."""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from gome_amd.abi import Engine  # noqa: E402
from tests.test_gpu_flow_cancel import _Fuzz  # noqa: E402

HDR = np.dtype([("ok", "<u4"), ("nl", "<u4"), ("sym", "<u4"), ("ntouch", "<u4"), ("beg", "<u4"), ("end", "<u4"),
                ("nold", "<u4"), ("adds", "<u4"), ("dropped", "<u4"), ("rests", "<u4"), ("obase", "<u4"),
                ("w32", "<u4"), ("amask", "<u8", 2), ("bmask", "<u8", 2), ("g", "<u8"),
                ("ndel", "<u4"), ("ncancel", "<u4"), ("fc_bad", "<u4"),
                ("deep", "<u4"), ("dslot", "<u4"), ("nbsum", "<u4"), ("pad3", "<u4", 4)])
FCDEL = np.dtype([("kind", "<u4"), ("li", "<u4"), ("tgt", "<u4"), ("rank", "<u4"), ("nb", "<u4"), ("ixs", "<u4"),
                  ("oend", "<u4"), ("ov", "<u4"), ("r", "<i8"), ("ct", "<u4"), ("va", "<u4")])
assert HDR.itemsize == 128 and FCDEL.itemsize == 48


def main():
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    fz = _Fuzz(200, ns=ns, nprice=5)
    eng = Engine(max_symbols=ns, max_batch=20000, max_nodes=1 << 20, max_levels=1 << 20)
    for bi in range(3):
        b = fz.batch(20000)
        eng.submit(b)
        eng.drain()
        fb = eng.debug_flow_books()
        hdr = np.frombuffer(eng.debug_peek(0, 0, HDR.itemsize * len(fb)), HDR)
        print(f"batch {bi}: books {len(fb)} declined {int((fb['decline'] != 0).sum())}")
        shown = 0
        for h in range(len(fb)):
            if not fb[h]["decline"] or shown >= 2:
                continue
            shown += 1
            x = hdr[h]
            beg, end = int(x["beg"]), int(x["end"])
            d = np.frombuffer(eng.debug_peek(2, FCDEL.itemsize * beg, FCDEL.itemsize * (end - beg)), FCDEL)
            rk = np.frombuffer(eng.debug_peek(3, 4 * beg, 4 * (end - beg)), "<u4")
            tg = np.frombuffer(eng.debug_peek(4, 4 * beg, 4 * (end - beg)), "<u4")
            seg = b[b["symbol_id"] == x["sym"]]
            print(f"  book h={h} sym={x['sym']} n={end - beg} ndel={x['ndel']} bad={x['fc_bad']} wsum={x['nbsum']} "
                  f"win={x['ncancel']} g={x['g']}")
            isdel = seg["action"] == 2
            for i in np.nonzero(isdel & (d["kind"] != 0))[0][:400]:
                nb = int(d[i]["nb"])
                if nb > 1000:
                    t = int(d[i]["tgt"])
                    print(f"    pos {i} kind {d[i]['kind']} li {d[i]['li']} tgt {t} rank {d[i]['rank']} nb {nb}"
                          f" rank_of_tgt {rk[t - beg] if d[i]['kind'] == 1 and beg <= t < end else '-'}"
                          f" tg_of_tgt {tg[t - beg] if d[i]['kind'] == 1 and beg <= t < end else '-'}")
            print("    kinds:", np.bincount(d["kind"][isdel], minlength=3), "ranks>=1e6:", int((d['rank'][isdel] > 10**6).sum()))


if __name__ == "__main__":
    main()
