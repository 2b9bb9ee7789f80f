"""Generator of flow_plan_asm.inc: the serial loop of k_flow_plan as one GCN asm block.

The plan (match_flow.h) is the batch's critical path: one wavefront per book applies every
order to the level aggregates one after another, so its cost is the latency of the
instruction stream per order.  The loop is written out here instruction by instruction
(generated, 8 orders per double-buffered SMEM group pair) so that:
  * the best ask / best bid levels and their depths live in SGPRs (top-of-book cache): a
    partial fill at the top or a rest at/inside the spread is pure SALU;
  * other levels' depths live in lane registers (level k: lane k % 64 of set k / 64) and are
    read / written with v_readlane / v_writelane only when the sweep leaves the top;
  * membership S:SALE / S:BUY are 128-bit SGPR masks with sentinel levels 0 (bid) and 127
    (ask), so the next level of a sweep is one bit scan;
  * orders stream through the scalar cache in groups of 4 (s_load_dwordx8), the next group in
    flight while the current one is applied;
  * touches are staged in three lane registers and stored 64 at a time from inside the loop
    (the common path is straight-line: every rare case branches out of line).

Run: python gome_amd/csrc/gen_plan_asm.py   (writes flow_plan_asm.inc next to this file)
Semantics follow engine.go:56-136 / nodepool.go:61-115 at the aggregate level; see the
comments of k_flow_plan in match_flow.h.
"""
from __future__ import annotations

import os

# fixed registers (declared as clobbers of the asm statement)
BUF = [(60, 61), (62, 63), (64, 65), (66, 67), (68, 69), (70, 71), (72, 73), (74, 75)]
BA, BB = "s76", "s77"            # best ask / best bid level
BAD, BBD = ("s78", "s79"), ("s80", "s81")  # their depths (authoritative while cached)
M = "s[84:85]"                   # 64-bit temp (mask word)
LI, K, T0, JJS = "s86", "s87", "s88", "s89"
O = ["s90", "s91", "s92", "s93"]
D = ("s94", "s95")               # 64-bit temp (T - depth)
HC = "s97"                       # half-groups left
ADDR = "s[98:99]"                # SMEM address of the next half-group
CLOBBERS = [f"s{i}" for i in range(60, 101)]

out: list[str] = []
uid = [0]


def e(line: str):
    out.append(line)


def lab(name: str) -> str:
    return f"{name}_%="


def fresh(name: str) -> str:
    uid[0] += 1
    return lab(f"{name}{uid[0]}")


def read(k: str, dlo: str, dhi: str):
    """dlo:dhi = depth of level k from the lane registers."""
    e(f"s_and_b32 {T0}, {k}, 63")
    e(f"v_readlane_b32 {O[0]}, %[dl0], {T0}")
    e(f"v_readlane_b32 {O[1]}, %[dh0], {T0}")
    e(f"v_readlane_b32 {O[2]}, %[dl1], {T0}")
    e(f"v_readlane_b32 {O[3]}, %[dh1], {T0}")
    e(f"s_cmp_lt_u32 {k}, 64")
    e(f"s_cselect_b32 {dlo}, {O[0]}, {O[2]}")
    e(f"s_cselect_b32 {dhi}, {O[1]}, {O[3]}")


def setbit(mask: str, k: str, op: str):
    """op = s_bitset1_b64 / s_bitset0_b64 on bit k of the 128-bit mask A or B."""
    m0, m1 = f"%[{mask}0]", f"%[{mask}1]"
    e(f"s_cmp_lt_u32 {k}, 64")
    e(f"s_cselect_b64 {M}, {m0}, {m1}")
    e(f"{op} {M}, {k}")
    e(f"s_cmp_lt_u32 {k}, 64")
    e(f"s_cselect_b64 {m0}, {M}, {m0}")
    e(f"s_cselect_b64 {m1}, {m1}, {M}")


def lowest_ask():
    e(f"s_ff1_i32_b64 {BA}, %[A0]")
    e(f"s_ff1_i32_b64 {T0}, %[A1]")
    e(f"s_add_u32 {T0}, {T0}, 64")
    e(f"s_cmp_lg_u64 %[A0], 0")
    e(f"s_cselect_b32 {BA}, {BA}, {T0}")


def highest_bid():
    e(f"s_flbit_i32_b64 {BB}, %[B0]")
    e(f"s_sub_u32 {BB}, 63, {BB}")
    e(f"s_flbit_i32_b64 {T0}, %[B1]")
    e(f"s_sub_u32 {T0}, 127, {T0}")
    e(f"s_cmp_lg_u64 %[B1], 0")
    e(f"s_cselect_b32 {BB}, {T0}, {BB}")


flushes: list[tuple[str, str]] = []  # (flush label, return label), emitted out of line

# M0 holds the staging count (lane of the next touch) for the whole loop; the rare paths that
# need M0 as a lane select save it in SAVE and restore it.
SAVE = "s100"
ADD_VIA_READ = False


def write(k: str, lo: str, hi: str):
    """Level k := lo:hi in the lane registers.  The other set's lane written is a sentinel
    lane (level 0: set 0 lane 0, level 127: set 1 lane 63), whose value is never used."""
    e(f"s_mov_b32 {SAVE}, m0")
    e(f"s_and_b32 {T0}, {k}, 63")
    e(f"s_cmp_lt_u32 {k}, 64")
    e(f"s_cselect_b32 {O[0]}, {T0}, 0")
    e(f"s_cselect_b32 {O[1]}, 63, {T0}")
    e(f"s_mov_b32 m0, {O[0]}")
    e(f"v_writelane_b32 %[dl0], {lo}, m0")
    e(f"v_writelane_b32 %[dh0], {hi}, m0")
    e(f"s_mov_b32 m0, {O[1]}")
    e(f"v_writelane_b32 %[dl1], {lo}, m0")
    e(f"v_writelane_b32 %[dh1], {hi}, m0")
    e(f"s_mov_b32 m0, {SAVE}")


def add_lane(k: str, tlo: str, thi: str):
    """Level k += tlo:thi, in the lane registers."""
    if ADD_VIA_READ:
        read(k, D[0], D[1])
        e(f"s_add_u32 {D[0]}, {D[0]}, {tlo}")
        e(f"s_addc_u32 {D[1]}, {D[1]}, {thi}")
        write(k, D[0], D[1])
        return
    e(f"v_mov_b32 %[vt], {thi}")                # before exec narrows (set 1 needs it too)
    e(f"s_lshl_b64 {M}, 1, {k}")
    e(f"s_cmp_lt_u32 {k}, 64")
    e(f"s_cselect_b64 exec, {M}, 0")
    e(f"v_add_co_u32_e32 %[dl0], vcc, {tlo}, %[dl0]")
    e(f"v_addc_co_u32_e32 %[dh0], vcc, %[vt], %[dh0], vcc")
    e(f"s_cmp_lt_u32 {k}, 64")
    e(f"s_cselect_b64 exec, 0, {M}")
    e(f"v_add_co_u32_e32 %[dl1], vcc, {tlo}, %[dl1]")
    e(f"v_addc_co_u32_e32 %[dh1], vcc, %[vt], %[dh1], vcc")
    e("s_mov_b64 exec, -1")


def log(kr: str, lo: str, hi: str, check: bool):
    """Stage one touch {kr, amount} in lane M0.  With check: store the staging when full (the
    touches an order logs before its last one); the last touch of an order needs no check
    (the staging is flushed at half-group boundaries once 60 touches are staged)."""
    e(f"v_writelane_b32 %[lk], {kr}, m0")
    e(f"v_writelane_b32 %[la], {lo}, m0")
    e(f"v_writelane_b32 %[lb], {hi}, m0")
    e("s_add_u32 m0, m0, 1")
    if check:
        fl, back = fresh("FL"), fresh("FB")
        e("s_cmp_ge_u32 m0, 60")                # keeps room for the <= 4 unchecked last
        e(f"s_cbranch_scc1 {fl}")               # touches of the half-group
        e(f"{back}:")
        flushes.append((fl, back))


def emit_flush(fl: str, back: str):
    """Store all 64 staging lanes at lpos, advance lpos by the staged count (M0).  Lanes past
    the count are garbage and are overwritten by the next store (the log has slack)."""
    skip = fresh("FS")
    e(f"{fl}:")
    e(f"s_add_u32 {T0}, %[lpos], 64")
    e(f"s_cmp_gt_u32 {T0}, %[lcap]")
    e(f"s_cbranch_scc1 {skip}")
    e(f"s_lshl_b32 {T0}, %[lpos], 4")
    e(f"v_add_u32 %[voff], {T0}, %[vl16]")
    e("global_store_dword %[voff], %[lk], %[logp]")
    e("global_store_dword %[voff], %[la], %[logp] offset:8")
    e("global_store_dword %[voff], %[lb], %[logp] offset:12")
    e(f"{skip}:")
    e("s_add_u32 %[lpos], %[lpos], m0")
    e("s_mov_b32 m0, 0")
    e(f"s_branch {back}")


def order(r: tuple[int, int]):
    """Apply one packed record s[r] (SetOrder, engine.go:56-85, at the aggregate level).
    The record's registers become the taker's remaining volume T in place.  Layout: rests
    (the most common outcome) fall through; crossing branches out; every path ends with one
    jump to the next order.  Lane values of non-member levels are don't-care (a level that
    empties is only dropped from its mask; a rest onto a non-member level writes instead of
    adds; k_flow_plan zeroes non-member lanes once at the end)."""
    lo, hi = f"s{r[0]}", f"s{r[1]}"
    T = (lo, hi)
    TT = f"s[{r[0]}:{r[1]}]"
    nxt = fresh("NX")
    for side in ("B", "S"):
        if side == "B":
            own, opp = "B", "A"            # rests into S:BUY, crosses S:SALE
            top, topd, otop, otopd = BB, BBD, BA, BAD
        else:
            own, opp = "A", "B"
            top, topd, otop, otopd = BA, BAD, BB, BBD
        loop, cross, full, notdeep, newtop, istop, dnew = (fresh(side + x) for x in ("L", "C", "F", "N", "W", "T", "D"))
        if side == "B":
            e(f"s_add_u32 {JJS}, {JJS}, 256")           # (order index + 1) << 8
            e(f"s_bfe_u32 {LI}, {hi}, 0x70015")
            e(f"s_bitcmp1_b32 {hi}, 28")
            sell = fresh("SE")
            e(f"s_cbranch_scc1 {sell}")
        else:
            e(f"{sell}:")
        e(f"s_and_b32 {hi}, {hi}, 0x1fffff")            # T = volume
        e(f"{loop}:")
        # crossing opposite level? BUY: best ask <= li; SALE: best bid >= li
        e(f"s_cmp_{'le' if side == 'B' else 'ge'}_u32 {otop}, {LI}")
        e(f"s_cbranch_scc1 {cross}")
        # ---- rest at li (engine.go:80-82): depth += T, ZADD own side
        e(f"s_cmp_{'lt' if side == 'B' else 'gt'}_u32 {LI}, {top}")   # strictly behind own top
        e(f"s_cbranch_scc0 {notdeep}")
        e(f"s_cmp_lt_u32 {LI}, 64")
        e(f"s_cselect_b64 {M}, %[{own}0], %[{own}1]")
        e(f"s_bitcmp1_b64 {M}, {LI}")
        e(f"s_cbranch_scc0 {dnew}")
        add_lane(LI, T[0], T[1])                          # existing level: lane += T
        e(f"s_or_b32 {K}, {JJS}, {LI}")
        e(f"s_bitset1_b32 {K}, 7")
        log(K, T[0], T[1], False)
        e(f"s_branch {nxt}")
        e(f"{dnew}:")                                     # new level behind the top: lane = T
        e(f"s_bitset1_b64 {M}, {LI}")
        e(f"s_cmp_lt_u32 {LI}, 64")
        e(f"s_cselect_b64 %[{own}0], {M}, %[{own}0]")
        e(f"s_cselect_b64 %[{own}1], %[{own}1], {M}")
        write(LI, T[0], T[1])
        e(f"s_or_b32 {K}, {JJS}, {LI}")
        e(f"s_bitset1_b32 {K}, 7")
        log(K, T[0], T[1], False)
        e(f"s_branch {nxt}")
        e(f"{notdeep}:")
        e(f"s_cmp_eq_u32 {LI}, {top}")
        e(f"s_cbranch_scc1 {istop}")
        # new own top inside the spread: evict the cached top to its lane
        write(top, topd[0], topd[1])
        e(f"s_mov_b32 {top}, {LI}")
        e(f"s_mov_b64 s[{topd[0][1:]}:{topd[1][1:]}], {TT}")
        setbit(own, LI, "s_bitset1_b64")
        e(f"s_or_b32 {K}, {JJS}, {LI}")
        e(f"s_bitset1_b32 {K}, 7")
        log(K, T[0], T[1], False)
        e(f"s_branch {nxt}")
        e(f"{istop}:")
        e(f"s_add_u32 {topd[0]}, {topd[0]}, {T[0]}")
        e(f"s_addc_u32 {topd[1]}, {topd[1]}, {T[1]}")
        e(f"s_or_b32 {K}, {JJS}, {LI}")
        e(f"s_bitset1_b32 {K}, 7")
        log(K, T[0], T[1], False)
        e(f"s_branch {nxt}")
        # ---- cross the best opposite level (MatchOrder, engine.go:138-198)
        e(f"{cross}:")
        e(f"s_sub_u32 {D[0]}, {T[0]}, {otopd[0]}")
        e(f"s_subb_u32 {D[1]}, {T[1]}, {otopd[1]}")
        e(f"s_cbranch_scc0 {full}")
        # partial: the level keeps depth - T (engine.go:176-194)
        e(f"s_sub_u32 {otopd[0]}, {otopd[0]}, {T[0]}")
        e(f"s_subb_u32 {otopd[1]}, {otopd[1]}, {T[1]}")
        e(f"s_or_b32 {K}, {JJS}, {otop}")
        log(K, T[0], T[1], False)
        e(f"s_branch {nxt}")
        # full: the level empties (engine.go:145-175), ZREM (nodepool.go:76-83), next level
        e(f"{full}:")
        e(f"s_or_b32 {K}, {JJS}, {otop}")
        log(K, otopd[0], otopd[1], True)
        e(f"s_mov_b64 {TT}, s[{D[0][1:]}:{D[1][1:]}]")
        setbit(opp, otop, "s_bitset0_b64")
        if side == "B":
            lowest_ask()
        else:
            highest_bid()
        read(otop, otopd[0], otopd[1])
        e(f"s_or_b32 {T0}, {T[0]}, {T[1]}")
        e(f"s_cbranch_scc0 {nxt}")                      # diff == 0: stop (engine.go:162-175)
        e(f"s_branch {loop}")
    e(f"{nxt}:")


def main():
    done = lab("DONE")
    loop = lab("HALF")
    e("s_waitcnt vmcnt(0)")
    e(f"s_mov_b64 {ADDR}, %[ob]")
    e(f"s_mov_b32 {HC}, %[nh]")
    e(f"s_mov_b32 {JJS}, 0xffffff00")          # (-1) << 8: the first record is order 0
    e("s_mov_b32 m0, %[nacc]")
    lowest_ask()
    read(BA, BAD[0], BAD[1])
    highest_bid()
    read(BB, BBD[0], BBD[1])
    e(f"s_cmp_eq_u32 {HC}, 0")
    e(f"s_cbranch_scc1 {done}")
    e(f"s_load_dwordx8 s[60:67], {ADDR}, 0x0")
    e(f"{loop}:")
    for half in range(2):
        other = 68 - 8 * half
        fl, back = fresh("HF"), fresh("HB")
        e("s_waitcnt lgkmcnt(0)")
        e(f"s_add_u32 s98, s98, 32")
        e(f"s_addc_u32 s99, s99, 0")
        e(f"s_load_dwordx8 s[{other}:{other + 7}], {ADDR}, 0x0")   # prefetch the next half
        e("s_cmp_ge_u32 m0, 60")                # room for this half's 4 last touches
        e(f"s_cbranch_scc1 {fl}")
        e(f"{back}:")
        flushes.append((fl, back))
        for u in range(4):
            order(BUF[4 * half + u])
        e(f"s_sub_u32 {HC}, {HC}, 1")
        e(f"s_cmp_eq_u32 {HC}, 0")
        e(f"s_cbranch_scc1 {done}")
    e(f"s_branch {loop}")
    for fl, back in flushes:
        emit_flush(fl, back)
    e(f"{done}:")
    e("s_waitcnt lgkmcnt(0)")
    write(BA, BAD[0], BAD[1])
    write(BB, BBD[0], BBD[1])
    e("s_mov_b32 %[nacc], m0")

    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "flow_plan_asm.inc"), "w") as f:
        f.write("// Generated by gen_plan_asm.py — do not edit.\n")
        f.write("#define FL_PLAN_ASM \\\n")
        for line in out:
            f.write(f'  "{line}\\n\\t" \\\n')
        f.write('  ""\n')
        f.write("#define FL_PLAN_CLOBBERS " + ", ".join(f'"{c}"' for c in CLOBBERS) + "\n")


if __name__ == "__main__":
    main()
