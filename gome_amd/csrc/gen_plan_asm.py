"""Generator of flow_plan_asm.inc: the serial loop of k_flow_plan as one GCN asm block.

The plan (match_flow.h) is the batch's critical path: one wavefront per book applies every
order to the level aggregates one after another, so its cost is the latency of the
instruction stream per order.  Lone-wave costs on gfx950 (tools/ubench_lone_wave.hip,
tools/ubench_branch3.hip, shader cycles): 4 per SALU / VALU instruction, ~12 per conditional
branch not taken, ~24 taken, ~20 per s_branch, ~20 per v_readlane or per VALU write of an
SGPR whatever the distance to the consumer.  Branches are the dominant cost, so:
  * the best ask / best bid levels and their depths live in SGPRs (top-of-book cache): a
    partial fill is pure SALU;
  * other levels' depths live in lane registers (level k: lane k % 64 of set k / 64), with the
    invariant "a lane that is not a resting level behind the cached top holds 0" (the cached
    tops' lanes included).  A rest is then ONE branchless sequence whatever the level is
    (deep / at the top / a new top that evicts the cached one into its lane): selects decide
    the lane, the amount and the cached depth, and an exec-masked VALU add applies it;
  * bids and asks have lane registers of their own, so side-set membership (S:BUY / S:SALE)
    is "the lane is not 0": rests maintain no mask, and the next level of a sweep is two VALU
    compares and a bit scan (sentinel levels 0 (bid) and 127 (ask) are nonzero lanes); a
    promoted level's lane is read and zeroed;
  * every path ends with the next order's side dispatch (decode, one conditional branch) instead
    of a jump to a common head, and the most frequent path falls through into the next slot;
  * orders stream through the scalar cache in half-groups of 8 (s_load_dwordx16), the next one in
    flight while the current one is applied; the record registers become T in place;
  * touches are staged in lane registers (lane = M0, the staging count) and stored 64 at a
    time from inside the loop.

Two variants: W=64 (volumes and depths as 64-bit SGPR pairs / two lane registers per set)
and W=32 (the book's volumes divided by their GCD fit 32 bits: one register each, half the
lane traffic and no carry chains).  k_flow_prep picks the variant per book.

Run: python gome_amd/csrc/gen_plan_asm.py [--out PATH]   (default: flow_plan_asm.inc next to this file)
Semantics follow engine.go:56-136 / nodepool.go:61-115 at the aggregate level; see the
comments of k_flow_plan in match_flow.h.
"""
from __future__ import annotations

import os

# fixed registers (declared as clobbers of the asm statement)
HG = 8                           # records per half-group (one s_load_dwordx16)
NS = 2 * HG                      # order slots: two half-groups, double-buffered
BUF = [(44 + 2 * i, 45 + 2 * i) for i in range(HG)] + [(60 + 2 * i, 61 + 2 * i) for i in range(HG)]
BA, BB = "s76", "s77"            # best ask / best bid level
BAD, BBD = ("s78", "s79"), ("s80", "s81")  # their depths (authoritative; their lanes hold 0)
L = "s82"                        # lane target of a rest
M = "s[84:85]"                   # 64-bit temp (mask word / one-hot)
LI, K, T0, JJS = "s86", "s87", "s88", "s89"
O = ["s90", "s91", "s92", "s93"]
A, A1 = ("s90", "s91"), ("s92", "s93")     # lane amounts (set 0 / set 1) of a rest
D = ("s94", "s95")               # T - depth of a crossed level; X (cached-depth amount) in rests
X = D
HC = "s97"                       # half-groups left + 1
ADDR = "s[98:99]"                # SMEM address of the next half-group
SAVE = "s97"                     # M0 saved around the final lane writes (HC is dead by then)
CLOBBERS = [f"s{i}" for i in range(44, 100)] + ["v32", "v33", "v34", "v35"]
# W32 depth layout: one 64-bit lane pair per side, lane j = levels 2j (low word) and 2j+1 (high
# word): asks in v[32:33], bids in v[34:35] (fixed registers: the pair must be consecutive).
PAIR = {"A": (32, 33), "B": (34, 35)}
ZERO = "s91"                     # W32: stays 0, the high word of the rest amount s[90:91]
COPY_REST = os.environ.get("GOME_PLAN_COPY", "1") == "1"   # measured at a pinned placement: -2% cycles
LOOP_OFS = int(os.environ.get("GOME_PLAN_OFS", "0"))  # 4-byte words after the 256-B alignment
# timing experiment only (tools/build_variant.py): wait for each half-group's records right
# after issuing them
SYNC_SMEM = os.environ.get("GOME_PLAN_SYNC_SMEM", "0") == "1"
PF_DIST = int(os.environ.get("GOME_PLAN_PF", "0"))  # L2 prefetch distance in bytes (0: off);
# k_flow_prep pads ord8 by FL_ORD8_PAD records, which must cover it
PF_DEEP = int(os.environ.get("GOME_PLAN_PFD", "0"))  # the same for the deep plans (GenD, GenDC)


class Gen:
    pf = PF_DIST

    def __init__(self, width: int):
        self.w = width
        self.out: list[str] = []
        self.uid = 0
        self.flushes: list[tuple[str, str]] = []
        self.slow: list[list[str]] = []      # out-of-line blocks, emitted after the loop

    def e(self, line: str):
        self.out.append(line)

    @staticmethod
    def lab(name: str) -> str:
        return f"{name}_%="

    def fresh(self, name: str) -> str:
        self.uid += 1
        return self.lab(f"{name}{self.uid}")

    # ---- 64/32-bit scalar helpers on (lo, hi) pairs ------------------------------------
    def pair(self, r) -> str:
        return f"s[{r[0][1:]}:{r[1][1:]}]"

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
            self.e(f"s_mov_b64 {self.pair(r)}, {self.pair(a)}")
        else:
            self.e(f"s_mov_b32 {r[0]}, {a[0]}")

    def csel(self, r, a, b):
        """r = SCC ? a : b; a / b are pairs or the literal 0."""
        def op(x):
            return "0" if x == 0 else (self.pair(x) if self.w == 64 else x[0])
        if self.w == 64:
            self.e(f"s_cselect_b64 {self.pair(r)}, {op(a)}, {op(b)}")
        else:
            self.e(f"s_cselect_b32 {r[0]}, {op(a)}, {op(b)}")

    def is_zero_scc(self, t):  # SCC = (t == 0)
        if self.w == 64:
            self.e(f"s_cmp_eq_u64 {self.pair(t)}, 0")
        else:
            self.e(f"s_cmp_eq_u32 {t[0]}, 0")

    # ---- lane registers -------------------------------------------------------------
    @staticmethod
    def ln(sd: str, which: str) -> str:
        """Lane register of side sd ("A": asks, "B": bids): l0 / l1 = low words of sets 0 / 1,
        h0 / h1 = high words (W64)."""
        return f"%[{sd.lower()}{which}]"

    def promote(self, k: str, d, sd: str):
        """d = depth of level k from side sd's lane registers, and the lane is zeroed (level k
        becomes a cached top).  Sentinel lanes may hold garbage; their depth is never used."""
        e = self.e
        ln = self.ln
        if self.w == 32:
            ev, od = PAIR[sd]
            e(f"s_lshr_b32 {T0}, {k}, 1")
            e(f"v_readlane_b32 {O[0]}, v{ev}, {T0}")
            e(f"v_readlane_b32 {O[2]}, v{od}, {T0}")
            e(f"s_bfm_b64 {M}, 1, {T0}")
            e(f"s_bitcmp1_b32 {k}, 0")
            e(f"s_cselect_b32 {d[0]}, {O[2]}, {O[0]}")
            self.zero_half(ev, od)
            return
        e(f"s_and_b32 {T0}, {k}, 63")
        e(f"v_readlane_b32 {O[0]}, {ln(sd, 'l0')}, {T0}")
        e(f"v_readlane_b32 {O[2]}, {ln(sd, 'l1')}, {T0}")
        if self.w == 64:
            e(f"v_readlane_b32 {O[1]}, {ln(sd, 'h0')}, {T0}")
            e(f"v_readlane_b32 {O[3]}, {ln(sd, 'h1')}, {T0}")
        e(f"s_cmp_lt_u32 {k}, 64")
        e(f"s_cselect_b32 {d[0]}, {O[0]}, {O[2]}")
        if self.w == 64:
            e(f"s_cselect_b32 {d[1]}, {O[1]}, {O[3]}")
        e(f"s_bfm_b64 {M}, 1, {k}")
        e(f"s_cselect_b64 exec, {M}, 0")
        e(f"v_mov_b32 {ln(sd, 'l0')}, 0")
        if self.w == 64:
            e(f"v_mov_b32 {ln(sd, 'h0')}, 0")
        e(f"s_cselect_b64 exec, 0, {M}")
        e(f"v_mov_b32 {ln(sd, 'l1')}, 0")
        if self.w == 64:
            e(f"v_mov_b32 {ln(sd, 'h1')}, 0")

    def zero_half(self, ev: int, od: int):
        """W32: zero the word of lane M (one-hot) selected by SCC (1: odd level)."""
        e = self.e
        e(f"s_cselect_b64 exec, {M}, 0")
        e(f"v_mov_b32 v{od}, 0")
        e(f"s_cselect_b64 exec, 0, {M}")
        e(f"v_mov_b32 v{ev}, 0")

    def next_top(self, sd: str):
        """W32, after the cached top of side sd emptied: the next level of that side (asks: the
        lowest resting one, bids: the highest; the sentinels 127 / 0 are nonzero words) becomes
        the cached top: one 64-bit compare finds its lane pair, the pair's words pick the level."""
        e = self.e
        ev, od = PAIR[sd]
        top, topd = (BA, BAD) if sd == "A" else (BB, BBD)
        e("s_mov_b64 exec, -1")
        e(f"v_cmp_ne_u64_e64 {M}, 0, v[{ev}:{od}]")
        if sd == "A":
            e(f"s_ff1_i32_b64 {T0}, {M}")
        else:
            e(f"s_flbit_i32_b64 {T0}, {M}")
            e(f"s_sub_u32 {T0}, 63, {T0}")
        e(f"v_readlane_b32 {O[0]}, v{ev}, {T0}")
        e(f"v_readlane_b32 {O[2]}, v{od}, {T0}")
        e(f"s_lshl_b32 {top}, {T0}, 1")
        e(f"s_bfm_b64 {M}, 1, {T0}")
        if sd == "A":   # lowest: the even level unless it is empty
            e(f"s_cmp_eq_u32 {O[0]}, 0")
        else:           # highest: the odd level unless it is empty
            e(f"s_cmp_lg_u32 {O[2]}, 0")
        e(f"s_cselect_b32 {topd[0]}, {O[2]}, {O[0]}")
        e(f"s_cselect_b32 {T0}, 1, 0")
        self.zero_half(ev, od)
        e(f"s_add_u32 {top}, {top}, {T0}")

    def write(self, k: str, v, sd: str):
        """Level k := v (end of the loop: the cached tops go back to their lanes).  The other
        set's lane written is a sentinel lane (level 0: set 0 lane 0, level 127: set 1 lane
        63), whose value is never used."""
        e = self.e
        if self.w == 32:
            ev, od = PAIR[sd]
            e(f"s_lshr_b32 {T0}, {k}, 1")
            e(f"s_bfm_b64 {M}, 1, {T0}")
            e(f"s_bitcmp1_b32 {k}, 0")
            e(f"s_cselect_b64 exec, {M}, 0")
            e(f"v_mov_b32 v{od}, {v[0]}")
            e(f"s_cselect_b64 exec, 0, {M}")
            e(f"v_mov_b32 v{ev}, {v[0]}")
            e("s_mov_b64 exec, -1")
            return
        e(f"s_mov_b32 {SAVE}, m0")
        e(f"s_and_b32 {T0}, {k}, 63")
        e(f"s_cmp_lt_u32 {k}, 64")
        e(f"s_cselect_b32 {O[0]}, {T0}, 0")
        e(f"s_cselect_b32 {O[1]}, 63, {T0}")
        e(f"s_mov_b32 m0, {O[0]}")
        ln = self.ln
        e(f"v_writelane_b32 {ln(sd, 'l0')}, {v[0]}, m0")
        if self.w == 64:
            e(f"v_writelane_b32 {ln(sd, 'h0')}, {v[1]}, m0")
        e(f"s_mov_b32 m0, {O[1]}")
        e(f"v_writelane_b32 {ln(sd, 'l1')}, {v[0]}, m0")
        if self.w == 64:
            e(f"v_writelane_b32 {ln(sd, 'h1')}, {v[1]}, m0")
        e(f"s_mov_b32 m0, {SAVE}")

    def add_lane(self, sd: str):
        """Level L += A in the lane registers: the amount goes to the set of L, the other set's
        lane L % 64 gets 0.  exec is left narrowed (only lane-select ops follow).  W32: one 64-bit
        add of A << (32 * (L & 1)) to lane pair L >> 1."""
        e = self.e
        if self.w == 32:
            ev, od = PAIR[sd]
            e(f"s_lshr_b32 {T0}, {L}, 1")
            e(f"s_bfm_b64 exec, 1, {T0}")
            e(f"s_lshl_b32 {T0}, {L}, 5")            # (L & 1) << 5 in the low 6 bits
            e(f"s_lshl_b64 s[92:93], s[90:91], {T0}")  # s91 = 0
            e(f"v_lshl_add_u64 v[{ev}:{od}], s[92:93], 0, v[{ev}:{od}]")
            return
        e(f"s_cmp_lt_u32 {L}, 64")
        self.csel(A1, 0, A)
        self.csel(A, A, 0)
        e(f"s_bfm_b64 exec, 1, {L}")
        ln = self.ln
        l0, l1, h0, h1 = ln(sd, "l0"), ln(sd, "l1"), ln(sd, "h0"), ln(sd, "h1")
        if self.w == 64:
            e(f"v_mov_b32 %[vt], {A[1]}")
            e(f"v_add_co_u32_e32 {l0}, vcc, {A[0]}, {l0}")
            e(f"v_addc_co_u32_e32 {h0}, vcc, %[vt], {h0}, vcc")
            e(f"v_mov_b32 %[vt], {A1[1]}")
            e(f"v_add_co_u32_e32 {l1}, vcc, {A1[0]}, {l1}")
            e(f"v_addc_co_u32_e32 {h1}, vcc, %[vt], {h1}, vcc")
        else:
            e(f"v_add_u32_e32 {l0}, {A[0]}, {l0}")
            e(f"v_add_u32_e32 {l1}, {A1[0]}, {l1}")

    # ---- scalar state ---------------------------------------------------------------
    def members(self, sd: str):
        """M = lanes of set 0 of side sd holding a resting level (depth != 0), s[90:91] = set 1.
        (A VALU compare writes 0 for inactive lanes: exec is widened first.)"""
        e = self.e
        ln = self.ln
        e("s_mov_b64 exec, -1")
        for st, dst in (("0", M), ("1", "s[90:91]")):
            if self.w == 64:
                e(f"v_or_b32 %[vt], {ln(sd, 'l' + st)}, {ln(sd, 'h' + st)}")
                e(f"v_cmp_ne_u32_e64 {dst}, 0, %[vt]")
            else:
                e(f"v_cmp_ne_u32_e64 {dst}, 0, {ln(sd, 'l' + st)}")

    def lowest_ask(self):
        """BA = lowest resting ask level (ff1 gives -1 = UINT_MAX on an empty word; the ask
        sentinel 127 is a nonzero lane)."""
        e = self.e
        self.members("A")
        e(f"s_ff1_i32_b64 {BA}, {M}")
        e(f"s_ff1_i32_b64 {T0}, s[90:91]")
        e(f"s_add_u32 {T0}, {T0}, 64")
        e(f"s_min_u32 {BA}, {BA}, {T0}")

    def highest_bid(self):
        """BB = highest resting bid level (the bid sentinel 0 is a nonzero lane; an empty set 1
        gives 128 & 127 = 0)."""
        e = self.e
        self.members("B")
        e(f"s_flbit_i32_b64 {BB}, {M}")
        e(f"s_sub_u32 {BB}, 63, {BB}")
        e(f"s_flbit_i32_b64 {T0}, s[90:91]")
        e(f"s_sub_u32 {T0}, 127, {T0}")
        e(f"s_and_b32 {T0}, {T0}, 127")
        e(f"s_max_u32 {BB}, {BB}, {T0}")

    # ---- touch staging --------------------------------------------------------------
    def log(self, kr: str, a, check: bool):
        """Stage one touch {kr, amount} in lane M0.  With check: store the staging once 60
        touches are staged (touches an order logs before its last one); the last touch of
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
        e("s_mov_b64 exec, -1")
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

    # ---- one order slot ---------------------------------------------------------------
    def dispatch(self, j: int, fall: bool, copy: bool = COPY_REST):
        """Enter slot j (the next order): decode it and branch on its side.  Slots 0 and 4 open a
        half-group: jump to its head (or fall into it).  With copy, a BUY rest of slot j (the
        most frequent transition that cannot fall through) runs from a private copy of the
        rest body here instead of jumping to BR_j."""
        e = self.e
        if j % HG == 0:
            if not fall:
                e(f"s_branch {self.lab(f'H{j}')}")
            return
        self.decode(j)
        e(f"s_cbranch_scc1 {self.lab(f'S{j}')}")
        if not fall:                               # slot j's BUY entry, inline
            if self.w == 64:
                e(f"s_and_b32 s{BUF[j][1]}, s{BUF[j][1]}, 0x1fffff")
            e(f"s_cmp_le_u32 {BA}, {LI}")
            e(f"s_cbranch_scc1 {self.lab(f'BXE{j}')}")
            if copy:
                self.rest("B", (f"s{BUF[j][0]}", f"s{BUF[j][1]}"))
                self.dispatch((j + 1) % NS, False, False)
            else:
                e(f"s_branch {self.lab(f'BR{j}')}")

    def decode(self, j: int):
        """LI of record j and SCC = its side is SALE.  W64 record hi: volume bits 32..52 in
        [0, 21), LI in [21, 28), SALE at 28; the touch key is JJS | level (| 128 for a rest),
        JJS = order index << 8.  W32 record hi: LI in [0, 7), 1 << 7, the order index in
        [8, 31), SALE at 31, i.e. the rest touch key itself (k_flow_* mask the index)."""
        e = self.e
        hi = f"s{BUF[j][1]}"
        if self.w == 64:
            e(f"s_add_u32 {JJS}, {JJS}, 256")      # (order index + 1) << 8
            e(f"s_bfe_u32 {LI}, {hi}, 0x70015")
            e(f"s_bitcmp1_b32 {hi}, 28")
        else:
            e(f"s_and_b32 {LI}, {hi}, 127")
            e(f"s_bitcmp1_b32 {hi}, 31")

    def rest(self, side: str, T):
        """Rest T at LI (SetOrder engine.go:80-82: depth += T, ZADD own side), branchless.
        BUY: own top BB, beyond = LI > BB.  SALE: own top BA, beyond = LI < BA.
          at or beyond the top: the cached depth takes T (after a new top resets it);
          beyond (a new top): the old top's depth goes to its lane, the new top is LI;
          behind: the lane of LI takes T (its lane is 0 if the level is new)."""
        e = self.e
        buy = side == "B"
        top, topd = (BB, BBD) if buy else (BA, BAD)
        ge, gt = ("ge", "gt") if buy else ("le", "lt")
        e(f"s_cmp_{ge}_u32 {LI}, {top}")
        self.csel(X, T, 0)
        self.csel(A, 0, T)
        e(f"s_cmp_{gt}_u32 {LI}, {top}")
        self.csel(A, topd, A)
        e(f"s_cselect_b32 {L}, {top}, {LI}")
        self.csel(topd, 0, topd)
        e(f"s_{'max' if buy else 'min'}_u32 {top}, {top}, {LI}")
        self.add(topd, topd, X)
        self.add_lane("B" if buy else "A")
        if self.w == 64:
            e(f"s_or_b32 {K}, {JJS}, {LI}")
            e(f"s_bitset1_b32 {K}, 7")
            self.log(K, T, False)
        else:
            self.log(self.hi_of(T), T, False)

    def hi_of(self, T) -> str:
        return T[1]

    def cross_entry(self, T):
        """First crossing of an order (W32): the consume key base, order index << 8."""
        if self.w == 32:
            self.e(f"s_and_b32 {JJS}, {self.hi_of(T)}, 0xffffff00")

    def partial(self, side: str, T):
        """The crossed level keeps depth - T (MatchOrder diff < 0, engine.go:176-194)."""
        e = self.e
        otop, otopd = (BA, BAD) if side == "B" else (BB, BBD)
        self.sub(otopd, otopd, T)
        e(f"s_or_b32 {K}, {JJS}, {otop}")
        self.log(K, T, False)

    def full(self, side: str, T, i: int):
        """The crossed level empties (engine.go:145-175; ZREM nodepool.go:76-83); T -= depth;
        the next opposite level is promoted.  diff == 0 stops the order (engine.go:162-175)."""
        e = self.e
        buy = side == "B"
        otop, otopd = (BA, BAD) if buy else (BB, BBD)
        e(f"s_or_b32 {K}, {JJS}, {otop}")
        self.log(K, otopd, False)        # (the staging check is folded into the test below)
        self.mov(T, D)              # (the emptied level's lane is 0: it leaves the side)
        if self.w == 32:
            self.next_top("A" if buy else "B")
        else:
            if buy:
                self.lowest_ask()
            else:
                self.highest_bid()
            self.promote(otop, otopd, "A" if buy else "B")
        # one branch for the common case "T > 0, room in the staging, the next level crosses
        # too": T == 0 or a full staging make the limit a level that cannot cross
        never = "0" if buy else "127"
        cmp = "le" if buy else "ge"
        slow, cont = self.lab(f"{side}SL{i}"), self.lab(f"{side}CN{i}")
        self.is_zero_scc(T)
        e(f"s_cselect_b32 {T0}, {never}, {LI}")
        e(f"s_cmp_ge_u32 m0, {64 - HG}")          # (room for the half's HG final touches)
        e(f"s_cselect_b32 {T0}, {never}, {T0}")
        e(f"s_cmp_{cmp}_u32 {otop}, {T0}")
        e(f"s_cbranch_scc0 {slow}")
        fl = self.fresh("FL")
        self.flushes.append((fl, slow))
        blk = [f"{slow}:", f"s_cmp_ge_u32 m0, {64 - HG}", f"s_cbranch_scc1 {fl}"]
        blk += ([f"s_cmp_eq_u64 {self.pair(T)}, 0"] if self.w == 64 else [f"s_cmp_eq_u32 {T[0]}, 0"])
        blk += [f"s_cbranch_scc1 {self.lab(f'DN{i}')}",     # diff == 0: stop (engine.go:162-175)
                f"s_cmp_{cmp}_u32 {otop}, {LI}", f"s_cbranch_scc1 {cont}",
                f"s_branch {self.lab(f'{side}R{i}')}"]
        self.slow.append(blk)
        e(f"{cont}:")
        self.sub(D, T, otopd)                                 # the next level, inline
        e(f"s_cbranch_scc0 {self.lab(f'{side}F{i}')}")
        self.partial(side, T)
        self.dispatch((i + 1) % NS, False)

    def slot(self, i: int):
        """Order slot i (record BUF[i]); its side was decoded by the previous path.  Layout:
        B entry, BUY rest, BUY partial, BUY full, SALE partial, SALE full, exact-fill exit,
        S entry, SALE rest (falls into the next slot)."""
        e = self.e
        lo, hi = f"s{BUF[i][0]}", f"s{BUF[i][1]}"
        T = (lo, hi)          # 32-bit: T is lo; hi keeps the flags
        j = (i + 1) % NS
        lab = self.lab
        # --- BUY
        e(f"{lab(f'B{i}')}:")
        if self.w == 64:
            e(f"s_and_b32 {hi}, {hi}, 0x1fffff")     # T = volume
        e(f"s_cmp_le_u32 {BA}, {LI}")                # crossing the best ask?
        e(f"s_cbranch_scc1 {lab(f'BXE{i}')}")
        e(f"{lab(f'BR{i}')}:")
        self.rest("B", T)
        self.dispatch(j, False)
        e(f"{lab(f'BXE{i}')}:")
        self.cross_entry(T)
        self.sub(D, T, BAD)
        e(f"s_cbranch_scc0 {lab(f'BF{i}')}")
        self.partial("B", T)
        self.dispatch(j, False)
        e(f"{lab(f'BF{i}')}:")
        self.full("B", T, i)
        # --- SALE crossing paths
        e(f"{lab(f'SXE{i}')}:")
        self.cross_entry(T)
        self.sub(D, T, BBD)
        e(f"s_cbranch_scc0 {lab(f'SF{i}')}")
        self.partial("S", T)
        self.dispatch(j, False)
        e(f"{lab(f'SF{i}')}:")
        self.full("S", T, i)
        e(f"{lab(f'DN{i}')}:")
        self.dispatch(j, False)
        # --- SALE entry and rest
        e(f"{lab(f'S{i}')}:")
        if self.w == 64:
            e(f"s_and_b32 {hi}, {hi}, 0x1fffff")
        e(f"s_cmp_ge_u32 {BB}, {LI}")                # crossing the best bid?
        e(f"s_cbranch_scc1 {lab(f'SXE{i}')}")
        e(f"{lab(f'SR{i}')}:")
        self.rest("S", T)
        self.dispatch(j, j != 0)                     # falls into slot j (or the half head H4)

    def head(self, j: int):
        """Half-group head before slot j: count the half done, wait for this half's records,
        prefetch the next half, make room for its touches, dispatch slot j."""
        e = self.e
        other = 60 if j == 0 else 44
        fl, back = self.fresh("HF"), self.fresh("HB")
        hi = f"s{BUF[j][1]}"
        # one branch for "the book is done or the staging needs room for this half's HG last
        # touches"; the out-of-line block tells them apart
        e(f"{self.lab(f'H{j}')}:")
        e(f"s_sub_u32 {HC}, {HC}, 1")
        e(f"s_cmp_eq_u32 {HC}, 0")
        e(f"s_cselect_b32 {T0}, 99, m0")
        e(f"s_cmp_ge_u32 {T0}, {64 - HG}")
        hs = self.fresh("HS")
        e(f"s_cbranch_scc1 {hs}")
        e(f"{back}:")
        self.slow.append([f"{hs}:", f"s_cmp_eq_u32 {HC}, 0", f"s_cbranch_scc1 {self.lab('DONE')}", f"s_branch {fl}"])
        self.flushes.append((fl, back))
        e("s_waitcnt lgkmcnt(0)")
        e(f"s_add_u32 s98, s98, {8 * HG}")
        e("s_addc_u32 s99, s99, 0")
        e(f"s_load_dwordx16 s[{other}:{other + 15}], {ADDR}, 0x0")   # prefetch the next half
        if SYNC_SMEM:
            e("s_waitcnt lgkmcnt(0)")
        if self.pf:  # warm L2 further ahead with a vector load (never waited for in the loop)
            e("s_mov_b64 exec, 1")
            e(f"global_load_dword %[vpf], %[vzero], {ADDR} offset:{self.pf}")
        self.decode(j)
        e(f"s_cbranch_scc1 {self.lab(f'S{j}')}")

    def build(self) -> list[str]:
        e = self.e
        done = self.lab("DONE")
        e("s_waitcnt vmcnt(0)")
        e(f"s_mov_b64 {ADDR}, %[ob]")
        e(f"s_add_u32 {HC}, %[nh], 1")
        e(f"s_mov_b32 {JJS}, 0xffffff00")          # (-1) << 8: the first record is order 0
        e("s_mov_b32 m0, %[nacc]")
        if self.w == 32:   # operands -> fixed lane pairs; s91 = 0
            e("s_mov_b64 exec, -1")
            for sd, nm in (("A", "a"), ("B", "b")):
                ev, od = PAIR[sd]
                e(f"v_mov_b32 v{ev}, %[{nm}l0]")
                e(f"v_mov_b32 v{od}, %[{nm}l1]")
            e(f"s_mov_b32 {ZERO}, 0")
            self.next_top("A")
            self.next_top("B")
        else:
            self.lowest_ask()
            self.promote(BA, BAD, "A")
            self.highest_bid()
            self.promote(BB, BBD, "B")
        e(f"s_load_dwordx16 s[44:59], {ADDR}, 0x0")
        # pin the loop's placement: the lone-wave fetch is sensitive to where the hand-made
        # stream sits (a shift of the same code by a few bytes moved the hottest book's plan
        # from 80 to 101 ns per order), so align it and pad to the measured best offset
        e(".p2align 8")
        for _ in range(LOOP_OFS):
            e("s_nop 0")
        if self.pf:
            e("s_mov_b64 exec, 1")
            for off in range(64, self.pf, 64):
                e(f"global_load_dword %[vpf], %[vzero], {ADDR} offset:{off}")
        for i in range(NS):
            if i % HG == 0:
                self.head(i)
            self.slot(i)
        for blk in self.slow:
            for line in blk:
                e(line)
        for fl, back in self.flushes:
            self.emit_flush(fl, back)
        e(f"{done}:")
        e("s_waitcnt vmcnt(0) lgkmcnt(0)")      # (vpf is an asm output: no load may land later)
        e("s_mov_b64 exec, -1")
        self.write(BA, BAD, "A")
        self.write(BB, BBD, "B")
        if self.w == 32:   # fixed lane pairs -> operands
            e("s_mov_b64 exec, -1")
            for sd, nm in (("A", "a"), ("B", "b")):
                ev, od = PAIR[sd]
                e(f"v_mov_b32 %[{nm}l0], v{ev}")
                e(f"v_mov_b32 %[{nm}l1], v{od}")
        e("s_mov_b32 %[nacc], m0")
        return self.out


# ---- W32C: the 32-bit plan of a book whose segment holds DELs -------------
# ADD records are the W32 records (hi = level | 1 << 7 | j << 8 | SALE << 31, lo = volume in
# units of g; j < 2^22 in these books, so bit 30 is clear).  A DEL record: hi = level | v << 7 |
# 1 << 30 | maker SALE << 31 (v < 2^22: the target's volume), lo = Q, the volume of the makers of
# the target's side that arrived at the level after the target and before the DEL and were not
# cancelled before it (computed by the cancel prep, match_flow_cancel.h).  While the target m is
# live those makers are untouched (only the FIFO head is ever partly consumed, and a same-side
# ADD at m's level cannot cross) and, if m itself was partly consumed, nothing ahead of it is
# live; once m is gone (or never rested) the side's depth of the level is at most Q.  So
# DeleteOrder (engine.go:87-116) removes r = clamp(depth - Q, 0, v): no per-maker state in the
# plan.  A DEL that finds nothing (r = 0) logs no touch (M0 advances by r != 0).  Touch keys of
# DELs and consumes come from an order counter (JJS = j << 8, no side bit).
VE = 40                      # a DEL's depth word, then r (lane level >> 1)
CLOBBERS_C = [f"v{VE}", f"v{VE + 1}"]


class GenC(Gen):
    def __init__(self):
        super().__init__(32)

    def decode(self, j: int):
        """The order counter advances; LI of record j; a DEL branches to its path first, then
        SCC = SALE."""
        e = self.e
        hi = f"s{BUF[j][1]}"
        e(f"s_add_u32 {JJS}, {JJS}, 256")
        e(f"s_and_b32 {LI}, {hi}, 127")
        e(f"s_bitcmp1_b32 {hi}, 30")
        e(f"s_cbranch_scc1 {self.lab(f'D{j}')}")
        e(f"s_bitcmp1_b32 {hi}, 31")

    def cross_entry(self, T):
        """(The consume key base is the order counter.)"""

    def del_log(self, r: str):
        """The cancel touch {JJS | level | 1 << 30 | SALE << 31, r}; M0 advances only when r != 0
        (SCC = r != 0 on entry)."""
        e = self.e
        e(f"v_writelane_b32 %[lk], {K}, m0")
        e(f"v_writelane_b32 %[la], {r}, m0")
        e("s_addc_u32 m0, m0, 0")

    def del_path(self, i: int):
        """DeleteOrder (engine.go:87-116) of a maker of side sd at level LI: r = clamp(depth - Q,
        0, v), depth -= r.  A level behind the cached top: the depth word of lane LI >> 1 in VALU
        (no branch on r; a word that reaches 0 leaves the side set by itself); the cached top:
        SALU, and the next level of the side is promoted when it empties (ZREM)."""
        e = self.e
        lo, hi = f"s{BUF[i][0]}", f"s{BUF[i][1]}"
        lab = self.lab
        j = (i + 1) % NS
        X1, XV, SH = "s94", "s95", "s96"
        e(f"{lab(f'D{i}')}:")
        e(f"s_bfe_u32 {XV}, {hi}, 0x160007")                   # v
        e(f"s_and_b32 {K}, {hi}, 0xc000007f")
        e(f"s_or_b32 {K}, {K}, {JJS}")                          # the cancel touch key
        e(f"s_bitcmp1_b32 {hi}, 31")
        e(f"s_cbranch_scc1 {lab(f'DA{i}')}")
        for sd in ("B", "A"):
            if sd == "A":
                e(f"{lab(f'DA{i}')}:")
            top, topd = (BB, BBD) if sd == "B" else (BA, BAD)
            ev, od = PAIR[sd]
            e(f"s_cmp_eq_u32 {LI}, {top}")
            e(f"s_cbranch_scc1 {lab(f'DT{sd}{i}')}")
            e(f"s_lshr_b32 {T0}, {LI}, 1")
            e(f"s_bfm_b64 {M}, 1, {T0}")
            e(f"s_lshl_b32 {SH}, {LI}, 5")                      # (LI & 1) << 5 in the low 6 bits
            e(f"s_mov_b64 exec, {M}")
            e(f"v_lshrrev_b64 v[{VE}:{VE + 1}], {SH}, v[{ev}:{od}]")  # v40 = the level's depth word
            e(f"v_subrev_u32 v{VE}, {lo}, v{VE}")
            e(f"v_max_i32 v{VE}, 0, v{VE}")                     # (depth, Q < 2^31)
            e(f"v_min_u32 v{VE}, {XV}, v{VE}")                  # r
            e(f"v_readlane_b32 {X1}, v{VE}, {T0}")
            e(f"s_bitcmp1_b32 {LI}, 0")
            e(f"s_cselect_b64 exec, {M}, 0")
            e(f"v_sub_u32 v{od}, v{od}, v{VE}")
            e(f"s_cselect_b64 exec, 0, {M}")
            e(f"v_sub_u32 v{ev}, v{ev}, v{VE}")
            e(f"s_cmp_lg_u32 {X1}, 0")
            self.del_log(X1)
            self.dispatch(j, False)
            # the cached top
            e(f"{lab(f'DT{sd}{i}')}:")
            e(f"s_sub_u32 {X1}, {topd[0]}, {lo}")              # SCC = borrow
            e(f"s_cselect_b32 {X1}, 0, {X1}")
            e(f"s_min_u32 {X1}, {X1}, {XV}")                    # r
            e(f"s_sub_u32 {topd[0]}, {topd[0]}, {X1}")
            e(f"s_cmp_lg_u32 {X1}, 0")
            self.del_log(X1)
            e(f"s_cmp_lg_u32 {topd[0]}, 0")
            e(f"s_cbranch_scc1 {lab(f'DN{i}')}")
            self.next_top(sd)
            self.dispatch(j, False)

    def slot(self, i: int):
        """Gen.slot (W32), the DEL paths placed before the SALE entry."""
        sv = self.out
        self.out = []
        super().slot(i)
        body = self.out
        self.out = sv
        k = body.index(f"{self.lab(f'S{i}')}:")
        self.out.extend(body[:k])
        self.del_path(i)
        self.out.extend(body[k:])


# ---- W32D: the 32-bit plan of a deep book (more levels than lanes) -----------
# Depths live in LDS instead of lane registers: level k's bid depth at byte 8k, its ask depth at
# 8k + 4 (DEEP_CAP levels, 128 KiB), with the same invariant as the lanes: a slot holds 0 unless
# its level rests on that side behind the cached top.  Sentinels: level 0 is a permanent bid,
# level DEEP_CAP - 1 a permanent ask.  A per-side occupancy bitmap mirrors "slot != 0" (bit k of
# dword k >> 5; bids at DEEP_BM, asks at DEEP_BM + DEEP_CAP / 8): a rest is one ds_add plus one
# ds_or of its bit, and the next level after the top empties is one 64-lane read of 64 bitmap
# dwords (2048 levels) and two bit scans, then the level's slot (read and zeroed, its bit
# cleared).  Records: lo = volume in units of g, hi = level [0, 14) | SALE bit 31 (no-op: 0, a
# rest of 0 at the bid sentinel).  Touch keys come from the order counter (JJS | 1 << 7 for a
# rest); the level goes to the touch's second word (Touch::pos, read by the deep sort).
DEEP_CAP = 16384
DEEP_BM = DEEP_CAP * 8                       # byte offset of the bid bitmap (asks follow)
DEEP_BM_BYTES = 2 * DEEP_CAP // 8
VDA, VDD, VSA, VSD, VSL, VZD = 36, 37, 38, 39, 40, 41   # slot address / data, group read address /
VSUM_B, VSUM_A, VBASE_A, VBASE_B = 42, 43, 44, 45       # data, lane id, zero; group summaries;
CLOBBERS_D = [f"v{i}" for i in range(36, 46)]            # per-lane slot offsets (8 * lane + side)
VSUM = {"B": VSUM_B, "A": VSUM_A}
BM = {"B": DEEP_BM, "A": DEEP_BM + DEEP_CAP // 8}


class GenD(Gen):
    pf = PF_DEEP

    def __init__(self):
        super().__init__(32)

    def decode(self, j: int):
        e = self.e
        hi = f"s{BUF[j][1]}"
        e(f"s_add_u32 {JJS}, {JJS}, 256")
        e(f"s_and_b32 {LI}, {hi}, 0x3fff")
        e(f"s_bitcmp1_b32 {hi}, 31")

    def cross_entry(self, T):
        pass  # JJS is the order counter

    def logd(self, kr: str, a: str, lvl: str):
        e = self.e
        e(f"v_writelane_b32 %[lk], {kr}, m0")
        e(f"v_writelane_b32 %[la], {a}, m0")
        e(f"v_writelane_b32 %[lb], {lvl}, m0")
        e("s_add_u32 m0, m0, 1")

    def emit_flush(self, fl: str, back: str):
        """As the lane plans, with the touch's level (%[lb]) in its second word."""
        e = self.e
        skip = self.fresh("FS")
        e(f"{fl}:")
        e("s_mov_b64 exec, -1")
        e(f"s_add_u32 {T0}, %[lpos], 64")
        e(f"s_cmp_gt_u32 {T0}, %[lcap]")
        e(f"s_cbranch_scc1 {skip}")
        e(f"s_lshl_b32 {T0}, %[lpos], 4")
        e(f"v_add_u32 %[voff], {T0}, %[vl16]")
        e("global_store_dword %[voff], %[lk], %[logp]")
        e("global_store_dword %[voff], %[lb], %[logp] offset:4")
        e("global_store_dword %[voff], %[la], %[logp] offset:8")
        e("global_store_dword %[voff], %[vzero], %[logp] offset:12")
        e(f"{skip}:")
        e("s_add_u32 %[lpos], %[lpos], m0")
        e("s_mov_b32 m0, 0")
        e(f"s_branch {back}")

    @staticmethod
    def side_off(sd: str) -> int:
        return 4 if sd == "A" else 0

    def lds_add(self, lvl: str, amt: str, sd: str):
        """Slot (lvl, sd) += amt (the amount may be 0)."""
        e = self.e
        e(f"s_lshl_b32 {T0}, {lvl}, 3")
        e("s_mov_b64 exec, 1")
        e(f"v_mov_b32 v{VDA}, {T0}")
        e(f"v_mov_b32 v{VDD}, {amt}")
        e(f"ds_add_u32 v{VDA}, v{VDD} offset:{self.side_off(sd)}")

    def next_top(self, sd: str):
        """After the cached top of side sd emptied: the next level of that side (asks: the lowest
        nonzero slot above BA, bids: the highest below BB; the sentinels' slots are nonzero).  A
        per-side summary register (lane i bit j: group 32i + j of 32 levels holds a nonzero
        slot; 16 lanes cover the 16384 levels) gives the group without touching LDS: the
        candidate's own summary word first, else a compare over the lanes beyond it.  One
        32-lane read of the group's slots gives the level and its depth; the slot is zeroed and
        the group's summary bit cleared when it was the group's only nonzero slot."""
        e = self.e
        top, topd = (BA, BAD) if sd == "A" else (BB, BBD)
        asks = sd == "A"
        vs = VSUM[sd]
        base = VBASE_A if asks else VBASE_B
        more, cont = self.fresh("NM"), self.fresh("NC")
        G, W, MK, LN = O[0], O[2], O[3], "s81"
        if asks:
            e(f"s_add_u32 {T0}, {BA}, 1")                    # the first candidate level
        else:
            e(f"s_sub_u32 {T0}, {BB}, 1")
        e(f"s_lshr_b32 s79, {T0}, 5")                       # its group
        e(f"s_lshr_b32 {LN}, {T0}, 10")                     # the group's summary lane
        e(f"v_readlane_b32 {W}, v{vs}, {LN}")
        if asks:
            e(f"s_lshl_b32 {MK}, -1, s79")                  # groups >= the candidate's
        else:
            e(f"s_lshl_b32 {MK}, -2, s79")
            e(f"s_not_b32 {MK}, {MK}")                      # groups <= the candidate's
        e(f"s_and_b32 {W}, {W}, {MK}")
        e(f"s_cbranch_scc0 {more}")
        blk = [f"{more}:", "s_mov_b64 exec, -1", f"v_cmp_ne_u32_e64 {M}, 0, v{vs}"]
        if asks:   # lanes above LN
            blk += ["s_mov_b64 s[92:93], -1", f"s_add_u32 {LN}, {LN}, 1", f"s_lshl_b64 s[92:93], s[92:93], {LN}",
                    f"s_and_b64 {M}, {M}, s[92:93]", f"s_ff1_i32_b64 {LN}, {M}"]
        else:      # lanes below LN
            blk += [f"s_bfm_b64 s[92:93], {LN}, 0", f"s_and_b64 {M}, {M}, s[92:93]",
                    f"s_flbit_i32_b64 {LN}, {M}", f"s_sub_u32 {LN}, 63, {LN}"]
        blk += [f"v_readlane_b32 {W}, v{vs}, {LN}", f"s_branch {cont}"]
        self.slow.append(blk)
        e(f"{cont}:")
        if asks:
            e(f"s_ff1_i32_b32 {G}, {W}")
        else:
            e(f"s_flbit_i32_b32 {G}, {W}")
            e(f"s_sub_u32 {G}, 31, {G}")
        e(f"s_lshl_b32 {LN}, {LN}, 5")
        e(f"s_add_u32 {G}, {G}, {LN}")                      # the group
        e(f"s_lshl_b32 {W}, {G}, 8")                        # its first slot's byte offset
        e("s_mov_b64 exec, 0xffffffff")
        e(f"v_add_u32 v{VSA}, {W}, v{base}")
        e(f"ds_read_b32 v{VSD}, v{VSA}")
        e(f"s_lshl_b32 s79, 1, {G}")                        # the group's summary bit
        e(f"s_lshr_b32 {LN}, {G}, 5")
        e(f"s_lshl_b32 {top}, {G}, 5")
        e("s_waitcnt lgkmcnt(0)")
        e(f"v_cmp_ne_u32_e64 {M}, 0, v{VSD}")
        if asks:
            e(f"s_ff1_i32_b64 {MK}, {M}")
        else:
            e(f"s_flbit_i32_b64 {MK}, {M}")
            e(f"s_sub_u32 {MK}, 63, {MK}")
        e(f"v_readlane_b32 {topd[0]}, v{VSD}, {MK}")
        e(f"s_add_u32 {top}, {top}, {MK}")
        e(f"s_bfm_b64 exec, 1, {MK}")
        e(f"ds_write_b32 v{VSA}, v{VZD}")                   # the slot := 0
        e(f"s_bcnt1_i32_b64 {W}, {M}")
        e(f"s_cmp_eq_u32 {W}, 1")
        e(f"s_cselect_b32 s79, s79, 0")
        e(f"s_bfm_b64 exec, 1, {LN}")
        e(f"v_xor_b32 v{vs}, s79, v{vs}")                   # the group emptied: its bit cleared

    def rest(self, side: str, T):
        """As the 32-bit rest, with the lane add replaced by an LDS add at slot (L, side)."""
        e = self.e
        buy = side == "B"
        top, topd = (BB, BBD) if buy else (BA, BAD)
        ge, gt = ("ge", "gt") if buy else ("le", "lt")
        e(f"s_cmp_{ge}_u32 {LI}, {top}")
        self.csel(X, T, 0)
        self.csel(A, 0, T)
        e(f"s_cmp_{gt}_u32 {LI}, {top}")
        self.csel(A, topd, A)
        e(f"s_cselect_b32 {L}, {top}, {LI}")
        self.csel(topd, 0, topd)
        e(f"s_{'max' if buy else 'min'}_u32 {top}, {top}, {LI}")
        self.add(topd, topd, X)
        self.lds_add(L, A[0], "B" if buy else "A")
        # slot L is nonzero now iff A > 0 (A == 0: L is the cached top, whose slot stays 0): its
        # group's summary bit
        e(f"s_min_u32 s79, {A[0]}, 1")
        e(f"s_lshr_b32 s81, {L}, 5")
        e(f"s_lshl_b32 s79, s79, s81")
        e(f"s_lshr_b32 s81, {L}, 10")
        e(f"s_bfm_b64 exec, 1, s81")
        e(f"v_or_b32 v{VSUM['B' if buy else 'A']}, s79, v{VSUM['B' if buy else 'A']}")
        e(f"s_or_b32 {K}, {JJS}, 0x80")
        self.logd(K, T[0], LI)

    def partial(self, side: str, T):
        otop, otopd = (BA, BAD) if side == "B" else (BB, BBD)
        self.sub(otopd, otopd, T)
        self.logd(JJS, T[0], otop)

    def full(self, side: str, T, i: int):
        e = self.e
        buy = side == "B"
        otop, otopd = (BA, BAD) if buy else (BB, BBD)
        self.logd(JJS, otopd[0], otop)
        self.mov(T, D)
        self.next_top("A" if buy else "B")
        never = "0" if buy else str(DEEP_CAP - 1)
        cmp = "le" if buy else "ge"
        slow, cont = self.lab(f"{side}SL{i}"), self.lab(f"{side}CN{i}")
        self.is_zero_scc(T)
        e(f"s_cselect_b32 {T0}, {never}, {LI}")
        e(f"s_cmp_ge_u32 m0, {64 - HG}")
        e(f"s_cselect_b32 {T0}, {never}, {T0}")
        e(f"s_cmp_{cmp}_u32 {otop}, {T0}")
        e(f"s_cbranch_scc0 {slow}")
        fl = self.fresh("FL")
        self.flushes.append((fl, slow))
        blk = [f"{slow}:", f"s_cmp_ge_u32 m0, {64 - HG}", f"s_cbranch_scc1 {fl}",
               f"s_cmp_eq_u32 {T[0]}, 0", f"s_cbranch_scc1 {self.lab(f'DN{i}')}",
               f"s_cmp_{cmp}_u32 {otop}, {LI}", f"s_cbranch_scc1 {cont}",
               f"s_branch {self.lab(f'{side}R{i}')}"]
        self.slow.append(blk)
        e(f"{cont}:")
        self.sub(D, T, otopd)
        e(f"s_cbranch_scc0 {self.lab(f'{side}F{i}')}")
        self.partial(side, T)
        self.dispatch((i + 1) % NS, False)

    def write(self, k: str, v, sd: str):
        e = self.e
        e(f"s_lshl_b32 {T0}, {k}, 3")
        e("s_mov_b64 exec, 1")
        e(f"v_mov_b32 v{VDA}, {T0}")
        e(f"v_mov_b32 v{VDD}, {v[0]}")
        e(f"ds_write_b32 v{VDA}, v{VDD} offset:{self.side_off(sd)}")

    def build(self) -> list[str]:
        e = self.e
        done = self.lab("DONE")
        e("s_waitcnt vmcnt(0)")
        e(f"s_mov_b64 {ADDR}, %[ob]")
        e(f"s_add_u32 {HC}, %[nh], 1")
        e(f"s_mov_b32 {JJS}, 0xffffff00")
        e("s_mov_b32 m0, %[nacc]")
        e("s_mov_b64 exec, -1")
        e(f"v_mbcnt_lo_u32_b32 v{VSL}, -1, 0")
        e(f"v_mbcnt_hi_u32_b32 v{VSL}, -1, v{VSL}")
        e(f"v_mov_b32 v{VZD}, 0")
        e(f"v_lshlrev_b32 v{VBASE_B}, 3, v{VSL}")                 # lane l: slot l of a group (bid)
        e(f"v_add_u32 v{VBASE_A}, 4, v{VBASE_B}")                 # (ask)
        e(f"v_mov_b32 v{VSUM_B}, %[sb]")
        e(f"v_mov_b32 v{VSUM_A}, %[sa]")
        e(f"s_mov_b32 {ZERO}, 0")
        e(f"s_mov_b32 {BA}, 0")
        self.next_top("A")
        e(f"s_mov_b32 {BB}, {DEEP_CAP - 1}")
        self.next_top("B")
        e(f"s_load_dwordx16 s[44:59], {ADDR}, 0x0")
        e(".p2align 8")
        if self.pf:
            e("s_mov_b64 exec, 1")
            for off in range(64, self.pf, 64):
                e(f"global_load_dword %[vpf], %[vzero], {ADDR} offset:{off}")
        for i in range(NS):
            if i % HG == 0:
                self.head(i)
            self.slot(i)
        for blk in self.slow:
            for line in blk:
                e(line)
        for fl, back in self.flushes:
            self.emit_flush(fl, back)
        e(f"{done}:")
        e("s_waitcnt vmcnt(0) lgkmcnt(0)")
        self.write(BA, BAD, "A")
        self.write(BB, BBD, "B")
        e("s_waitcnt lgkmcnt(0)")
        e("s_mov_b64 exec, -1")
        e("s_mov_b32 %[nacc], m0")
        return self.out


# ---- W32DC: the deep plan of a book whose segment holds DELs ---------------
# ADD records are the W32D records.  A DEL record: hi = level [0, 14) | v << 14 (v < 2^16: the
# target's volume) | 1 << 30 | maker SALE << 31, lo = Q (as W32C: match_flow_cancel.h).  It removes
# r = clamp(depth - Q, 0, v) from the maker side's depth of the level: the cached top in SALU (the
# next level is promoted when it empties), any other level through its LDS slot (one round trip).
# A slot a DEL empties keeps its group's summary bit: next_top clears a bit whose group it finds
# empty and searches on.  A DEL that finds nothing logs no touch; its touch key is JJS | 1 << 30 |
# SALE << 31 (k_fc_* read it as a cancel), its level in the touch's second word.
class GenDC(GenD):
    def decode(self, j: int):
        e = self.e
        hi = f"s{BUF[j][1]}"
        e(f"s_add_u32 {JJS}, {JJS}, 256")
        e(f"s_and_b32 {LI}, {hi}, 0x3fff")
        e(f"s_bitcmp1_b32 {hi}, 30")
        e(f"s_cbranch_scc1 {self.lab(f'D{j}')}")
        e(f"s_bitcmp1_b32 {hi}, 31")

    def del_log(self, r: str):
        """The cancel touch {K, level, r}; M0 advances only when r != 0 (SCC = r != 0 on entry)."""
        e = self.e
        e(f"v_writelane_b32 %[lk], {K}, m0")
        e(f"v_writelane_b32 %[la], {r}, m0")
        e(f"v_writelane_b32 %[lb], {LI}, m0")
        e("s_addc_u32 m0, m0, 0")

    def del_path(self, i: int):
        e = self.e
        lo, hi = f"s{BUF[i][0]}", f"s{BUF[i][1]}"
        lab = self.lab
        j = (i + 1) % NS
        X1, XV, X2 = "s94", "s95", "s96"
        e(f"{lab(f'D{i}')}:")
        e(f"s_bfe_u32 {XV}, {hi}, 0x10000e")                 # v (bits 14..29)
        e(f"s_and_b32 {K}, {hi}, 0xc0000000")
        e(f"s_or_b32 {K}, {K}, {JJS}")                        # the cancel touch key
        e(f"s_bitcmp1_b32 {hi}, 31")
        e(f"s_cbranch_scc1 {lab(f'DA{i}')}")
        for sd in ("B", "A"):
            if sd == "A":
                e(f"{lab(f'DA{i}')}:")
            top, topd = (BB, BBD) if sd == "B" else (BA, BAD)
            e(f"s_cmp_eq_u32 {LI}, {top}")
            e(f"s_cbranch_scc1 {lab(f'DT{sd}{i}')}")
            # a level behind the top: its slot, read, reduced, written back
            e(f"s_lshl_b32 {T0}, {LI}, 3")
            e("s_mov_b64 exec, 1")
            e(f"v_mov_b32 v{VDA}, {T0}")
            e(f"ds_read_b32 v{VDD}, v{VDA} offset:{self.side_off(sd)}")
            e("s_waitcnt lgkmcnt(0)")
            e(f"v_readfirstlane_b32 {X1}, v{VDD}")            # depth
            e(f"s_sub_u32 {X2}, {X1}, {lo}")                  # SCC = borrow
            e(f"s_cselect_b32 {X2}, 0, {X2}")
            e(f"s_min_u32 {X2}, {X2}, {XV}")                  # r
            e(f"s_sub_u32 {X1}, {X1}, {X2}")
            e(f"v_mov_b32 v{VDD}, {X1}")
            e(f"ds_write_b32 v{VDA}, v{VDD} offset:{self.side_off(sd)}")
            e(f"s_cmp_lg_u32 {X2}, 0")
            self.del_log(X2)
            self.dispatch(j, False)
            # the cached top
            e(f"{lab(f'DT{sd}{i}')}:")
            e(f"s_sub_u32 {X1}, {topd[0]}, {lo}")
            e(f"s_cselect_b32 {X1}, 0, {X1}")
            e(f"s_min_u32 {X1}, {X1}, {XV}")                  # r
            e(f"s_sub_u32 {topd[0]}, {topd[0]}, {X1}")
            e(f"s_cmp_lg_u32 {X1}, 0")
            self.del_log(X1)
            e(f"s_cmp_lg_u32 {topd[0]}, 0")
            e(f"s_cbranch_scc1 {lab(f'DN{i}')}")
            self.next_top(sd)
            self.dispatch(j, False)

    def slot(self, i: int):
        """GenD's slot, the DEL paths placed before the SALE entry."""
        sv = self.out
        self.out = []
        super().slot(i)
        body = self.out
        self.out = sv
        k = body.index(f"{self.lab(f'S{i}')}:")
        self.out.extend(body[:k])
        self.del_path(i)
        self.out.extend(body[k:])

    def next_top(self, sd: str):
        """GenD.next_top, restarted after clearing the summary bit of a group it finds empty (a
        DEL emptied its last slot)."""
        start, stale = self.fresh("NT"), self.fresh("NS")
        self.e(f"{start}:")
        sv = self.out
        self.out = []
        super().next_top(sd)
        body = self.out
        self.out = sv
        vs = VSUM[sd]
        M_ = M
        k = body.index(f"v_cmp_ne_u32_e64 {M_}, 0, v{VSD}") + 1
        self.out.extend(body[:k])
        self.e(f"s_cmp_eq_u64 {M_}, 0")
        self.e(f"s_cbranch_scc1 {stale}")
        self.out.extend(body[k:])
        # s79 = the group's summary bit, s81 = its summary lane (set before the group read)
        self.slow.append([f"{stale}:", "s_bfm_b64 exec, 1, s81", f"v_xor_b32 v{vs}, s79, v{vs}", f"s_branch {start}"])


# ---- W32DV: the deep plan with the depths in VGPRs --------------------------
# A clean book's bids all lie below its asks, so one depth word per level suffices (its side is
# where it lies relative to the cached tops): level k's word is lane k & 63 of v[VB + (k >> 6)],
# NVR registers, NVL = 64 * NVR levels (the ask sentinel is level NVL - 1, the bid sentinel level
# 0).  The same invariant as the lane plans (a word is 0 unless its level rests behind the cached
# top of its side).  Words are read and written through the GPR index mode (s_set_gpr_idx_on:
# one SALU instruction, no memory round trip, no lgkmcnt wait behind the record stream's scalar
# loads); the staging count moves from M0 (which the index mode overwrites) to SGPR MC.  One
# summary VGPR: lane i bit j = register 32i + j holds a nonzero word (set by every rest, cleared
# by the promotion that takes a register's last word; a DEL that empties a word leaves it set and
# the promotion clears it when it finds the register empty).  The promotion after the top empties
# is: one summary lane read, one register copy, one compare across its lanes, one lane read.  The
# words come from and go back to a compact LDS array (word k at byte 4k), the cached tops are
# handed in and out as operands.
VB, NVR = 64, 192
NVL = 64 * NVR
MC = "s83"
VLB, VAM, VTR, VSM = 36, 37, 39, 42    # lane * 4 (LDS base); amount; register copy; summary
CLOBBERS_DV = [f"v{i}" for i in (VLB, VAM, VTR, VSM)] + [f"v{i}" for i in range(VB, VB + NVR)]


class GenDV(GenD):
    def logd(self, kr: str, a: str, lvl: str):
        """(v_writelane takes its lane from M0: an SGPR lane select beside an SGPR source breaks
        gfx9's one-SGPR constant bus limit.)"""
        e = self.e
        e(f"s_mov_b32 M0LANE, {MC}")
        e(f"v_writelane_b32 %[lk], {kr}, M0LANE")
        e(f"v_writelane_b32 %[la], {a}, M0LANE")
        e(f"v_writelane_b32 %[lb], {lvl}, M0LANE")
        e(f"s_add_u32 {MC}, {MC}, 1")

    def word_add(self, lvl: str, amt: str):
        """Word lvl += amt (the amount may be 0); exec is left narrowed.  (The 64-bit shift takes
        its count mod 64: lane lvl & 63 without a mask; the SGPR amount is the add's src0, the
        indexed word its src1 and destination.)"""
        e = self.e
        e(f"s_lshr_b32 {T0}, {lvl}, 6")
        e(f"s_lshl_b64 exec, 1, {lvl}")
        e(f"s_set_gpr_idx_on {T0}, gpr_idx(SRC1,DST)")
        e(f"v_add_u32 v{VB}, {amt}, v{VB}")
        e("s_set_gpr_idx_off")

    def word_set(self, lvl: str, val: str):
        e = self.e
        e(f"s_lshr_b32 {T0}, {lvl}, 6")
        e(f"s_lshl_b64 exec, 1, {lvl}")
        e(f"s_set_gpr_idx_on {T0}, gpr_idx(DST)")
        e(f"v_mov_b32 v{VB}, {val}")
        e("s_set_gpr_idx_off")

    def next_top(self, sd: str):
        """After the cached top of side sd emptied: asks, the lowest nonzero word above BA; bids,
        the highest below BB (the sentinels are nonzero words).  T0 = the candidate level c; the
        first register at or beyond c's (R) whose summary bit is set is G; its nonzero words beyond
        c give the level.  (G == R with none beyond c: search on from the next register; G != R with
        none at all: a stale bit, cleared, and the search restarts.)"""
        e = self.e
        top, topd = (BA, BAD) if sd == "A" else (BB, BBD)
        asks = sd == "A"
        start, more, cont, nxt = self.fresh("NT"), self.fresh("NM"), self.fresh("NC"), self.fresh("NX")
        G, W, MK, LN, R = O[0], O[2], O[3], "s81", "s79"
        MS = "s[94:95]"
        if asks:
            e(f"s_add_u32 {T0}, {BA}, 1")
        else:
            e(f"s_sub_u32 {T0}, {BB}, 1")
        e(f"{start}:")
        e(f"s_lshr_b32 {R}, {T0}, 6")                        # c's register
        e(f"s_lshr_b32 {LN}, {T0}, 11")                      # its summary lane
        e(f"v_readlane_b32 {W}, v{VSM}, {LN}")
        if asks:
            e(f"s_lshl_b32 {MK}, -1, {R}")                   # registers >= R (bit R & 31)
        else:
            e(f"s_lshl_b32 {MK}, -2, {R}")
            e(f"s_not_b32 {MK}, {MK}")                       # registers <= R
        e(f"s_and_b32 {W}, {W}, {MK}")
        e(f"s_cbranch_scc0 {more}")
        blk = [f"{more}:", "s_mov_b64 exec, -1", f"v_cmp_ne_u32_e64 {M}, 0, v{VSM}"]
        if asks:   # summary lanes above LN
            blk += [f"s_mov_b64 {MS}, -1", f"s_add_u32 {LN}, {LN}, 1", f"s_lshl_b64 {MS}, {MS}, {LN}",
                    f"s_and_b64 {M}, {M}, {MS}", f"s_ff1_i32_b64 {LN}, {M}"]
        else:      # below LN
            blk += [f"s_bfm_b64 {MS}, {LN}, 0", f"s_and_b64 {M}, {M}, {MS}",
                    f"s_flbit_i32_b64 {LN}, {M}", f"s_sub_u32 {LN}, 63, {LN}"]
        blk += [f"v_readlane_b32 {W}, v{VSM}, {LN}", f"s_branch {cont}"]
        self.slow.append(blk)
        e(f"{cont}:")
        if asks:
            e(f"s_ff1_i32_b32 {G}, {W}")
        else:
            e(f"s_flbit_i32_b32 {G}, {W}")
            e(f"s_sub_u32 {G}, 31, {G}")
        e(f"s_lshl_b32 {LN}, {LN}, 5")
        e(f"s_add_u32 {G}, {G}, {LN}")                      # the register
        e("s_mov_b64 exec, -1")
        e(f"s_set_gpr_idx_on {G}, gpr_idx(SRC0)")          # (on until the word's read below)
        e(f"v_cmp_ne_u32_e64 {M}, v{VB}, 0")
        if asks:   # lanes >= c & 63 when G == R
            e(f"s_lshl_b64 {MS}, -1, {T0}")
        else:      # lanes <= c & 63
            e(f"s_lshl_b64 {MS}, -2, {T0}")
            e(f"s_not_b64 {MS}, {MS}")
        e(f"s_cmp_eq_u32 {G}, {R}")
        e(f"s_cselect_b64 {MS}, {MS}, -1")
        e(f"s_and_b64 {MS}, {MS}, {M}")
        e(f"s_cbranch_scc0 {nxt}")
        stale = self.fresh("NS")
        blk = [f"{nxt}:", "s_set_gpr_idx_off", f"s_cmp_eq_u32 {G}, {R}", f"s_cbranch_scc0 {stale}"]
        if asks:   # on from the next register
            blk += [f"s_add_u32 {T0}, {R}, 1", f"s_lshl_b32 {T0}, {T0}, 6"]
        else:      # (R > 0: the bid sentinel is word 0 of register 0)
            blk += [f"s_lshl_b32 {T0}, {R}, 6", f"s_sub_u32 {T0}, {T0}, 1"]
        blk += [f"s_branch {start}",
                f"{stale}:", f"s_lshl_b32 {W}, 1, {G}", f"s_lshr_b32 {LN}, {G}, 5", f"s_lshl_b64 exec, 1, {LN}",
                f"v_xor_b32 v{VSM}, {W}, v{VSM}", f"s_branch {start}"]
        self.slow.append(blk)
        if asks:
            e(f"s_ff1_i32_b64 {MK}, {MS}")
        else:
            e(f"s_flbit_i32_b64 {MK}, {MS}")
            e(f"s_sub_u32 {MK}, 63, {MK}")
        e(f"v_readlane_b32 {topd[0]}, v{VB}, {MK}")
        e("s_set_gpr_idx_off")
        e(f"s_lshl_b32 {top}, {G}, 6")
        e(f"s_add_u32 {top}, {top}, {MK}")
        e(f"s_lshl_b64 exec, 1, {MK}")
        e(f"s_set_gpr_idx_on {G}, gpr_idx(DST)")
        e(f"v_mov_b32 v{VB}, 0")                            # the word := 0 (a cached top)
        e("s_set_gpr_idx_off")
        e(f"s_bcnt1_i32_b64 {W}, {M}")
        e(f"s_cmp_eq_u32 {W}, 1")
        e(f"s_cselect_b32 {W}, 1, 0")
        e(f"s_lshl_b32 {W}, {W}, {G}")                      # the register emptied: its bit
        e(f"s_lshr_b32 {LN}, {G}, 5")
        e(f"s_lshl_b64 exec, 1, {LN}")
        e(f"v_xor_b32 v{VSM}, {W}, v{VSM}")

    def rest(self, side: str, T):
        """As GenD.rest, the amount added to word L and its register's summary bit set."""
        e = self.e
        buy = side == "B"
        top, topd = (BB, BBD) if buy else (BA, BAD)
        ge, gt = ("ge", "gt") if buy else ("le", "lt")
        e(f"s_cmp_{ge}_u32 {LI}, {top}")
        self.csel(X, T, 0)
        self.csel(A, 0, T)
        e(f"s_cmp_{gt}_u32 {LI}, {top}")
        self.csel(A, topd, A)
        e(f"s_cselect_b32 {L}, {top}, {LI}")
        self.csel(topd, 0, topd)
        e(f"s_{'max' if buy else 'min'}_u32 {top}, {top}, {LI}")
        self.add(topd, topd, X)
        self.word_add(L, A[0])
        # word L's register's summary bit, set even when A == 0 (L is the cached top, whose word
        # stays 0): a bit over an all-zero register is stale, which next_top tolerates (it
        # searches on, or clears the bit), and a rest at the top is rare enough to pay for it
        e(f"s_lshl_b32 s79, 1, {T0}")                       # T0 = L >> 6: bit (L >> 6) & 31
        e(f"s_lshr_b32 s81, {T0}, 5")
        e("s_lshl_b64 exec, 1, s81")
        e(f"v_or_b32 v{VSM}, s79, v{VSM}")
        e(f"s_or_b32 {K}, {JJS}, 0x80")
        self.logd(K, T[0], LI)

    def full(self, side: str, T, i: int):
        sv = self.out
        self.out = []
        super().full(side, T, i)
        body = self.out
        self.out = sv
        # the sell side's "never crosses" limit is the ask sentinel's level
        self.out.extend(x.replace(f", {DEEP_CAP - 1}", f", {NVL - 1}") if x.startswith("s_cselect_b32") else x
                        for x in body)

    def write(self, k: str, v, sd: str):
        self.word_set(k, v[0])

    def build(self) -> list[str]:
        e = self.e
        done = self.lab("DONE")
        e("s_waitcnt vmcnt(0)")
        e(f"s_mov_b64 {ADDR}, %[ob]")
        e(f"s_add_u32 {HC}, %[nh], 1")
        e(f"s_mov_b32 {JJS}, 0xffffff00")
        e("s_mov_b32 m0, %[nacc]")
        e("s_mov_b64 exec, -1")
        e(f"v_mbcnt_lo_u32_b32 v{VLB}, -1, 0")
        e(f"v_mbcnt_hi_u32_b32 v{VLB}, -1, v{VLB}")
        e(f"v_lshlrev_b32 v{VLB}, 2, v{VLB}")
        for r in range(NVR):                                   # the words from the compact array
            e(f"ds_read_b32 v{VB + r}, v{VLB} offset:{256 * r}")
        e(f"v_mov_b32 v{VSM}, %[sv]")
        e(f"s_mov_b32 {BA}, %[ba]")
        e(f"s_mov_b32 {BB}, %[bb]")
        e(f"s_mov_b32 {BAD[0]}, %[bad]")
        e(f"s_mov_b32 {BBD[0]}, %[bbd]")
        e(f"s_mov_b32 {ZERO}, 0")
        e("s_waitcnt lgkmcnt(0)")
        e(f"s_load_dwordx16 s[44:59], {ADDR}, 0x0")
        e(".p2align 8")
        for i in range(NS):
            if i % HG == 0:
                self.head(i)
            self.slot(i)
        for blk in self.slow:
            for line in blk:
                e(line)
        for fl, back in self.flushes:
            self.emit_flush(fl, back)
        e(f"{done}:")
        e("s_waitcnt vmcnt(0) lgkmcnt(0)")
        self.write(BA, BAD, "A")
        self.write(BB, BBD, "B")
        e("s_mov_b64 exec, -1")
        for r in range(NVR):
            e(f"ds_write_b32 v{VLB}, v{VB + r} offset:{256 * r}")
        e("s_waitcnt lgkmcnt(0)")
        e(f"s_mov_b32 %[oba], {BA}")
        e(f"s_mov_b32 %[obb], {BB}")
        e("s_mov_b32 %[nacc], m0")
        # the staging count lives in MC (the index mode overwrites M0); M0 is loaded from it for
        # the lane writes only
        import re
        return [re.sub(r"\bm0\b", MC, x).replace("M0LANE", "m0") for x in self.out]


# ---- W32DVC: W32DV with DELs (W32DC's records and Q formula on the VGPR words) --------------
# One word per level has no side: a DEL of a maker on side sd at a level that now rests on the
# other side (or is the other side's cached top) finds nothing there (its side's depth is 0), so
# its v is zeroed first (r = clamp(d - Q, 0, 0) = 0, the word written back unchanged).
class GenDVC(GenDV):
    def decode(self, j: int):
        GenDC.decode(self, j)

    def del_log(self, r: str):
        """The cancel touch {K, level, r}; the count advances only when r != 0 (SCC on entry)."""
        e = self.e
        e(f"s_mov_b32 M0LANE, {MC}")
        e(f"v_writelane_b32 %[lk], {K}, M0LANE")
        e(f"v_writelane_b32 %[la], {r}, M0LANE")
        e(f"v_writelane_b32 %[lb], {LI}, M0LANE")
        e(f"s_addc_u32 {MC}, {MC}, 0")

    def del_path(self, i: int):
        e = self.e
        lo, hi = f"s{BUF[i][0]}", f"s{BUF[i][1]}"
        lab = self.lab
        j = (i + 1) % NS
        X1, XV, X2 = "s94", "s95", "s96"
        e(f"{lab(f'D{i}')}:")
        e(f"s_bfe_u32 {XV}, {hi}, 0x10000e")                 # v (bits 14..29)
        e(f"s_and_b32 {K}, {hi}, 0xc0000000")
        e(f"s_or_b32 {K}, {K}, {JJS}")                        # the cancel touch key
        e(f"s_bitcmp1_b32 {hi}, 31")
        e(f"s_cbranch_scc1 {lab(f'DA{i}')}")
        for sd in ("B", "A"):
            if sd == "A":
                e(f"{lab(f'DA{i}')}:")
            top, topd = (BB, BBD) if sd == "B" else (BA, BAD)
            e(f"s_cmp_eq_u32 {LI}, {top}")
            e(f"s_cbranch_scc1 {lab(f'DT{sd}{i}')}")
            # a level on the other side's half of the book: nothing of side sd rests there
            if sd == "B":
                e(f"s_cmp_ge_u32 {LI}, {BA}")
            else:
                e(f"s_cmp_le_u32 {LI}, {BB}")
            e(f"s_cselect_b32 {XV}, 0, {XV}")
            # a level behind the top: its word, reduced, written back
            e(f"s_lshr_b32 {T0}, {LI}, 6")
            e(f"s_and_b32 s79, {LI}, 63")
            e("s_lshl_b64 exec, 1, s79")
            e(f"s_set_gpr_idx_on {T0}, gpr_idx(SRC0)")
            e(f"v_mov_b32 v{VTR}, v{VB}")
            e("s_set_gpr_idx_off")
            e(f"v_readlane_b32 {X1}, v{VTR}, s79")             # depth
            e(f"s_sub_u32 {X2}, {X1}, {lo}")                  # SCC = borrow
            e(f"s_cselect_b32 {X2}, 0, {X2}")
            e(f"s_min_u32 {X2}, {X2}, {XV}")                  # r
            e(f"s_sub_u32 {X1}, {X1}, {X2}")
            e(f"v_mov_b32 v{VAM}, {X1}")
            e(f"s_set_gpr_idx_on {T0}, gpr_idx(DST)")
            e(f"v_mov_b32 v{VB}, v{VAM}")
            e("s_set_gpr_idx_off")
            e(f"s_cmp_lg_u32 {X2}, 0")
            self.del_log(X2)
            self.dispatch(j, False)
            # the cached top
            e(f"{lab(f'DT{sd}{i}')}:")
            e(f"s_sub_u32 {X1}, {topd[0]}, {lo}")
            e(f"s_cselect_b32 {X1}, 0, {X1}")
            e(f"s_min_u32 {X1}, {X1}, {XV}")                  # r
            e(f"s_sub_u32 {topd[0]}, {topd[0]}, {X1}")
            e(f"s_cmp_lg_u32 {X1}, 0")
            self.del_log(X1)
            e(f"s_cmp_lg_u32 {topd[0]}, 0")
            e(f"s_cbranch_scc1 {lab(f'DN{i}')}")
            self.next_top(sd)
            self.dispatch(j, False)

    def slot(self, i: int):
        """GenDV's slot, the DEL paths placed before the SALE entry."""
        sv = self.out
        self.out = []
        super().slot(i)
        body = self.out
        self.out = sv
        k = body.index(f"{self.lab(f'S{i}')}:")
        self.out.extend(body[:k])
        self.del_path(i)
        self.out.extend(body[k:])


ALIGN = int(os.environ.get("GOME_PLAN_ALIGN", "0"))   # log2 byte alignment of branch targets


def aligned(lines: list[str]) -> list[str]:
    if not ALIGN:
        return lines
    out = []
    for line in lines:
        if line.endswith(":"):
            out.append(f".p2align {ALIGN}")
        out.append(line)
    return out


def main():
    import argparse
    here = os.path.dirname(os.path.abspath(__file__))
    ap = argparse.ArgumentParser(description="Generate the flow plans' asm loops (flow_plan_asm.inc). "
                                             "Tuning knobs come from GOME_PLAN_* environment variables.")
    ap.add_argument("--out", default=os.path.join(here, "flow_plan_asm.inc"),
                    help="output path (default: flow_plan_asm.inc next to this script)")
    out = ap.parse_args().out
    with open(out, "w") as f:
        f.write("// Generated by gen_plan_asm.py — do not edit.\n")
        for w, g in ((64, Gen(64)), (32, Gen(32)), ("32C", GenC()), ("32D", GenD()), ("32DC", GenDC()),
                     ("32DV", GenDV()), ("32DVC", GenDVC())):
            f.write(f"#define FL_PLAN_ASM{w} \\\n")
            for line in aligned(g.build()):
                f.write(f'  "{line}\\n\\t" \\\n')
            f.write('  ""\n')
        f.write("#define FL_PLAN_CLOBBERS " + ", ".join(f'"{c}"' for c in CLOBBERS) + "\n")
        f.write("#define FL_PLAN_CLOBBERS_C " + ", ".join(f'"{c}"' for c in CLOBBERS_C) + "\n")
        f.write("#define FL_PLAN_CLOBBERS_D " + ", ".join(f'"{c}"' for c in CLOBBERS_D) + "\n")
        f.write("#define FL_PLAN_CLOBBERS_DV " + ", ".join(f'"{c}"' for c in CLOBBERS_DV) + "\n")
        f.write(f"#define FL_DEEP_NVL {NVL}\n")
        f.write(f"#define FL_DEEP_CAP {DEEP_CAP}\n")
        f.write(f"#define FL_DEEP_BM {DEEP_BM}\n")
        f.write(f"#define FL_DEEP_LDS {DEEP_BM + DEEP_BM_BYTES}\n")


if __name__ == "__main__":
    main()
