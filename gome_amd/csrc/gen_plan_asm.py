"""Generator of flow_plan_asm.inc: the serial loop of k_flow_plan as one GCN asm block.

The plan (match_flow.h) is the batch's critical path: one wavefront per book applies every
order to the level aggregates one after another, so its cost is the latency of the
instruction stream per order.  Lone-wave costs on gfx950 (tools/ubench_lone_wave.hip):
4 cycles per SALU / VALU instruction, ~13 per conditional branch even when not taken, ~26
taken, 20 per s_branch, ~20 from v_readlane to its SALU consumer.  So the loop is written
out instruction by instruction (generated, 8 orders per double-buffered SMEM group pair):
  * the best ask / best bid levels and their depths live in SGPRs (top-of-book cache): a
    partial fill at the top or a rest at the top is pure SALU;
  * other levels' depths live in lane registers (level k: lane k % 64 of set k / 64): a rest
    behind the top is an exec-masked VALU add (no readback), a new top evicts the old one
    with v_writelane, only a sweep past the top reads a lane;
  * membership S:SALE / S:BUY are 128-bit SGPR masks with sentinel levels 0 (bid) and 127
    (ask), so the next level of a sweep is one bit scan;
  * orders stream through the scalar cache in groups of 4 (s_load_dwordx8), the next group in
    flight while the current one is applied; the record registers become T in place;
  * touches are staged in lane registers (lane = M0, the staging count) and stored 64 at a
    time from inside the loop; rests (the most common outcome) fall through.

Two variants: W=64 (volumes and depths as 64-bit SGPR pairs / two lane registers per set)
and W=32 (the book's volumes divided by their GCD fit 32 bits: one register each, half the
lane traffic and no carry chains).  k_flow_prep picks the variant per book.

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
M = "s[84:85]"                   # 64-bit temp (mask word / one-hot)
LI, K, T0, JJS = "s86", "s87", "s88", "s89"
O = ["s90", "s91", "s92", "s93"]
D = ("s94", "s95")               # temp (T - depth)
HC = "s97"                       # half-groups left
ADDR = "s[98:99]"                # SMEM address of the next half-group
SAVE = "s100"                    # M0 (staging count) saved around lane writes
CLOBBERS = [f"s{i}" for i in range(60, 101)]


class Gen:
    def __init__(self, width: int):
        self.w = width
        self.out: list[str] = []
        self.uid = 0
        self.flushes: list[tuple[str, str]] = []

    def e(self, line: str):
        self.out.append(line)

    @staticmethod
    def lab(name: str) -> str:
        return f"{name}_%="

    def fresh(self, name: str) -> str:
        self.uid += 1
        return self.lab(f"{name}{self.uid}")

    # ---- lane registers -------------------------------------------------------------
    def read(self, k: str, d: tuple[str, str]):
        """d = depth of level k from the lane registers."""
        e = self.e
        e(f"s_and_b32 {T0}, {k}, 63")
        e(f"v_readlane_b32 {O[0]}, %[dl0], {T0}")
        e(f"v_readlane_b32 {O[2]}, %[dl1], {T0}")
        if self.w == 64:
            e(f"v_readlane_b32 {O[1]}, %[dh0], {T0}")
            e(f"v_readlane_b32 {O[3]}, %[dh1], {T0}")
        e(f"s_cmp_lt_u32 {k}, 64")
        e(f"s_cselect_b32 {d[0]}, {O[0]}, {O[2]}")
        if self.w == 64:
            e(f"s_cselect_b32 {d[1]}, {O[1]}, {O[3]}")

    def write(self, k: str, v: tuple[str, str]):
        """Level k := v.  The other set's lane written is a sentinel lane (level 0: set 0
        lane 0, level 127: set 1 lane 63), whose value is never used."""
        e = self.e
        e(f"s_mov_b32 {SAVE}, m0")
        e(f"s_and_b32 {T0}, {k}, 63")
        e(f"s_cmp_lt_u32 {k}, 64")
        e(f"s_cselect_b32 {O[0]}, {T0}, 0")
        e(f"s_cselect_b32 {O[1]}, 63, {T0}")
        e(f"s_mov_b32 m0, {O[0]}")
        e(f"v_writelane_b32 %[dl0], {v[0]}, m0")
        if self.w == 64:
            e(f"v_writelane_b32 %[dh0], {v[1]}, m0")
        e(f"s_mov_b32 m0, {O[1]}")
        e(f"v_writelane_b32 %[dl1], {v[0]}, m0")
        if self.w == 64:
            e(f"v_writelane_b32 %[dh1], {v[1]}, m0")
        e(f"s_mov_b32 m0, {SAVE}")

    def add_lane(self, k: str, t: tuple[str, str]):
        """Level k += t in the lane registers (exec-masked VALU add, no readback)."""
        e = self.e
        if self.w == 64:
            e(f"v_mov_b32 %[vt], {t[1]}")               # before exec narrows (set 1 needs it too)
        e(f"s_lshl_b64 {M}, 1, {k}")
        e(f"s_cmp_lt_u32 {k}, 64")
        e(f"s_cselect_b64 exec, {M}, 0")
        if self.w == 64:
            e(f"v_add_co_u32_e32 %[dl0], vcc, {t[0]}, %[dl0]")
            e(f"v_addc_co_u32_e32 %[dh0], vcc, %[vt], %[dh0], vcc")
        else:
            e(f"v_add_u32_e32 %[dl0], {t[0]}, %[dl0]")
        e(f"s_cmp_lt_u32 {k}, 64")
        e(f"s_cselect_b64 exec, 0, {M}")
        if self.w == 64:
            e(f"v_add_co_u32_e32 %[dl1], vcc, {t[0]}, %[dl1]")
            e(f"v_addc_co_u32_e32 %[dh1], vcc, %[vt], %[dh1], vcc")
        else:
            e(f"v_add_u32_e32 %[dl1], {t[0]}, %[dl1]")
        e("s_mov_b64 exec, -1")

    # ---- scalar state ---------------------------------------------------------------
    def setbit(self, mask: str, k: str, op: str):
        """op = s_bitset1_b64 / s_bitset0_b64 on bit k of the 128-bit mask A or B."""
        e = self.e
        m0, m1 = f"%[{mask}0]", f"%[{mask}1]"
        e(f"s_cmp_lt_u32 {k}, 64")
        e(f"s_cselect_b64 {M}, {m0}, {m1}")
        e(f"{op} {M}, {k}")
        e(f"s_cmp_lt_u32 {k}, 64")
        e(f"s_cselect_b64 {m0}, {M}, {m0}")
        e(f"s_cselect_b64 {m1}, {m1}, {M}")

    def lowest_ask(self):
        e = self.e
        e(f"s_ff1_i32_b64 {BA}, %[A0]")
        e(f"s_ff1_i32_b64 {T0}, %[A1]")
        e(f"s_add_u32 {T0}, {T0}, 64")
        e(f"s_cmp_lg_u64 %[A0], 0")
        e(f"s_cselect_b32 {BA}, {BA}, {T0}")

    def highest_bid(self):
        e = self.e
        e(f"s_flbit_i32_b64 {BB}, %[B0]")
        e(f"s_sub_u32 {BB}, 63, {BB}")
        e(f"s_flbit_i32_b64 {T0}, %[B1]")
        e(f"s_sub_u32 {T0}, 127, {T0}")
        e(f"s_cmp_lg_u64 %[B1], 0")
        e(f"s_cselect_b32 {BB}, {T0}, {BB}")

    # 64/32-bit scalar arithmetic on (lo, hi) pairs
    def sub(self, r, a, b):  # r = a - b, SCC = borrow
        self.e(f"s_sub_u32 {r[0]}, {a[0]}, {b[0]}")
        if self.w == 64:
            self.e(f"s_subb_u32 {r[1]}, {a[1]}, {b[1]}")

    def add(self, r, a, b):
        self.e(f"s_add_u32 {r[0]}, {a[0]}, {b[0]}")
        if self.w == 64:
            self.e(f"s_addc_u32 {r[1]}, {a[1]}, {b[1]}")

    def mov(self, r, a):
        if self.w == 64:
            self.e(f"s_mov_b64 s[{r[0][1:]}:{r[1][1:]}], s[{a[0][1:]}:{a[1][1:]}]")
        else:
            self.e(f"s_mov_b32 {r[0]}, {a[0]}")

    def is_zero_scc(self, t):  # SCC = (t == 0)
        if self.w == 64:
            self.e(f"s_or_b32 {T0}, {t[0]}, {t[1]}")
            self.e(f"s_cmp_eq_u32 {T0}, 0")
        else:
            self.e(f"s_cmp_eq_u32 {t[0]}, 0")

    # ---- touch staging --------------------------------------------------------------
    def log(self, kr: str, a, check: bool):
        """Stage one touch {kr, amount} in lane M0.  With check: store the staging once 60
        touches are staged (the touches an order logs before its last one); the last touch of
        an order needs no check (the staging is also flushed at half-group boundaries)."""
        e = self.e
        e(f"v_writelane_b32 %[lk], {kr}, m0")
        e(f"v_writelane_b32 %[la], {a[0]}, m0")
        if self.w == 64:
            e(f"v_writelane_b32 %[lb], {a[1]}, m0")
        e("s_add_u32 m0, m0, 1")
        if check:
            fl, back = self.fresh("FL"), self.fresh("FB")
            e("s_cmp_ge_u32 m0, 60")
            e(f"s_cbranch_scc1 {fl}")
            e(f"{back}:")
            self.flushes.append((fl, back))

    def emit_flush(self, fl: str, back: str):
        """Store all 64 staging lanes at lpos, advance lpos by the staged count (M0).  Lanes past
        the count are garbage and are overwritten by the next store (the log has slack).  In
        the 32-bit variant %[lb] stays 0: the amount's high word."""
        e = self.e
        skip = self.fresh("FS")
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

    # ---- one order --------------------------------------------------------------------
    def order(self, r: tuple[int, int]):
        """Apply one packed record s[r] (SetOrder, engine.go:56-85, at the aggregate level).
        Layout: rests fall through; crossing branches out; every path ends with one jump to
        the next order.  Lane values of non-member levels are don't-care (a level that
        empties only leaves its mask; a rest onto a non-member level writes instead of adds;
        k_flow_plan zeroes non-member lanes once at the end)."""
        e = self.e
        lo, hi = f"s{r[0]}", f"s{r[1]}"
        T = (lo, hi)          # 32-bit: T is lo; hi keeps the flags
        Dd = D
        bad, bbd = BAD, BBD
        nxt = self.fresh("NX")
        sell = self.fresh("SE")
        for side in ("B", "S"):
            if side == "B":
                own, opp = "B", "A"            # rests into S:BUY, crosses S:SALE
                top, topd, otop, otopd = BB, bbd, BA, bad
            else:
                own, opp = "A", "B"
                top, topd, otop, otopd = BA, bad, BB, bbd
            loop, cross, full, notdeep, istop, dnew = (self.fresh(side + x) for x in ("L", "C", "F", "N", "T", "D"))
            if side == "B":
                e(f"s_add_u32 {JJS}, {JJS}, 256")           # (order index + 1) << 8
                e(f"s_bfe_u32 {LI}, {hi}, 0x70015")
                e(f"s_bitcmp1_b32 {hi}, 28")
                e(f"s_cbranch_scc1 {sell}")
            else:
                e(f"{sell}:")
            if self.w == 64:
                e(f"s_and_b32 {hi}, {hi}, 0x1fffff")        # T = volume
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
            self.add_lane(LI, T)                              # existing level: lane += T
            e(f"s_or_b32 {K}, {JJS}, {LI}")
            e(f"s_bitset1_b32 {K}, 7")
            self.log(K, T, False)
            e(f"s_branch {nxt}")
            e(f"{dnew}:")                                     # new level behind the top: lane = T
            e(f"s_bitset1_b64 {M}, {LI}")
            e(f"s_cmp_lt_u32 {LI}, 64")
            e(f"s_cselect_b64 %[{own}0], {M}, %[{own}0]")
            e(f"s_cselect_b64 %[{own}1], %[{own}1], {M}")
            self.write(LI, T)
            e(f"s_or_b32 {K}, {JJS}, {LI}")
            e(f"s_bitset1_b32 {K}, 7")
            self.log(K, T, False)
            e(f"s_branch {nxt}")
            e(f"{notdeep}:")
            e(f"s_cmp_eq_u32 {LI}, {top}")
            e(f"s_cbranch_scc1 {istop}")
            # new own top inside the spread: evict the cached top to its lane
            self.write(top, topd)
            e(f"s_mov_b32 {top}, {LI}")
            self.mov(topd, T)
            self.setbit(own, LI, "s_bitset1_b64")
            e(f"s_or_b32 {K}, {JJS}, {LI}")
            e(f"s_bitset1_b32 {K}, 7")
            self.log(K, T, False)
            e(f"s_branch {nxt}")
            e(f"{istop}:")
            self.add(topd, topd, T)
            e(f"s_or_b32 {K}, {JJS}, {LI}")
            e(f"s_bitset1_b32 {K}, 7")
            self.log(K, T, False)
            e(f"s_branch {nxt}")
            # ---- cross the best opposite level (MatchOrder, engine.go:138-198)
            e(f"{cross}:")
            self.sub(Dd, T, otopd)
            e(f"s_cbranch_scc0 {full}")
            # partial: the level keeps depth - T (engine.go:176-194)
            self.sub(otopd, otopd, T)
            e(f"s_or_b32 {K}, {JJS}, {otop}")
            self.log(K, T, False)
            e(f"s_branch {nxt}")
            # full: the level empties (engine.go:145-175), ZREM (nodepool.go:76-83), next level
            e(f"{full}:")
            e(f"s_or_b32 {K}, {JJS}, {otop}")
            self.log(K, otopd, True)
            self.mov(T, Dd)
            self.setbit(opp, otop, "s_bitset0_b64")
            if side == "B":
                self.lowest_ask()
            else:
                self.highest_bid()
            self.read(otop, otopd)
            self.is_zero_scc(T)
            e(f"s_cbranch_scc1 {nxt}")                      # diff == 0: stop (engine.go:162-175)
            e(f"s_branch {loop}")
        e(f"{nxt}:")

    def build(self) -> list[str]:
        e = self.e
        done = self.lab("DONE")
        loop = self.lab("HALF")
        e("s_waitcnt vmcnt(0)")
        e(f"s_mov_b64 {ADDR}, %[ob]")
        e(f"s_mov_b32 {HC}, %[nh]")
        e(f"s_mov_b32 {JJS}, 0xffffff00")          # (-1) << 8: the first record is order 0
        e("s_mov_b32 m0, %[nacc]")
        self.lowest_ask()
        self.read(BA, BAD)
        self.highest_bid()
        self.read(BB, BBD)
        e(f"s_cmp_eq_u32 {HC}, 0")
        e(f"s_cbranch_scc1 {done}")
        e(f"s_load_dwordx8 s[60:67], {ADDR}, 0x0")
        e(f"{loop}:")
        for half in range(2):
            other = 68 - 8 * half
            fl, back = self.fresh("HF"), self.fresh("HB")
            e("s_waitcnt lgkmcnt(0)")
            e("s_add_u32 s98, s98, 32")
            e("s_addc_u32 s99, s99, 0")
            e(f"s_load_dwordx8 s[{other}:{other + 7}], {ADDR}, 0x0")   # prefetch the next half
            e("s_cmp_ge_u32 m0, 60")                # room for this half's 4 last touches
            e(f"s_cbranch_scc1 {fl}")
            e(f"{back}:")
            self.flushes.append((fl, back))
            for u in range(4):
                self.order(BUF[4 * half + u])
            e(f"s_sub_u32 {HC}, {HC}, 1")
            e(f"s_cmp_eq_u32 {HC}, 0")
            e(f"s_cbranch_scc1 {done}")
        e(f"s_branch {loop}")
        for fl, back in self.flushes:
            self.emit_flush(fl, back)
        e(f"{done}:")
        e("s_waitcnt lgkmcnt(0)")
        self.write(BA, BAD)
        self.write(BB, BBD)
        e("s_mov_b32 %[nacc], m0")
        return self.out


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, "flow_plan_asm.inc"), "w") as f:
        f.write("// Generated by gen_plan_asm.py — do not edit.\n")
        for w in (64, 32):
            f.write(f"#define FL_PLAN_ASM{w} \\\n")
            for line in Gen(w).build():
                f.write(f'  "{line}\\n\\t" \\\n')
            f.write('  ""\n')
        f.write("#define FL_PLAN_CLOBBERS " + ", ".join(f'"{c}"' for c in CLOBBERS) + "\n")


if __name__ == "__main__":
    main()
