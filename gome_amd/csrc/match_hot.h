// match_hot.h — match_books for hot books (the Zipf head of the batch).
//
// A book whose segment holds >= 2^HOT_MIN_LOG2 orders is applied by k_match_hot: one
// wavefront per book, one workgroup per CU (~142 KiB of LDS), s_setprio 3.
//
// A single wavefront executes one order at a time (the reference's serial consumer,
// rabbitmq.go:116), so what bounds a hot book is the instruction stream and the dependent
// LDS round trips per order, not memory bandwidth.  The design therefore keeps the book's
// level array in registers across lanes and touches LDS only for FIFO node data:
//   * level i (ascending price) lives in lane i % 64 of register set i / 64 (up to
//     LRB_CAP = 128 levels): price, depth, side membership, FIFO head/tail chunk and slots,
//     live count, cache slot, the head chunk's next pointer and the NextNode look-ahead;
//   * crossing levels (GetReverseDepth, nodepool.go:86-115) = compare + ballot per register
//     set, iterated best-first with bit scans; the level to rest in = compare + ballot;
//     level updates = predicated VALU selects into the owning lane;
//   * the head chunk of each touched level is cached in LDS (1 KiB per level, written back
//     once at the end); one chunk step = one LDS round trip, then a single-maker fast path or
//     a DPP prefix scan over the 32 slots;
//   * events are staged in LDS and written 64 at a time with 16-B stores; per-order event
//     counts are kept in a VGPR (lane j = order j of the block) and stored once per block.
// Global loads remain only for: 64 Prep records per 64 orders (double-buffered), a head
// chunk on first touch and once per 32 consumed makers, the NextNode look-ahead into the
// chunk after the head (cached per level), and cancels (index probe).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "match_cold.h"
#include "wave.h"

namespace gome {

// Diagnostic build only (-DGOME_STAMPS): per-phase s_memtime cycle sums of each hot
// wave, read back with gome_debug_stamps.  The product build compiles these away.
#ifdef GOME_STAMPS
constexpr int NSTAMP = 16;
__device__ unsigned long long g_stamps[256 * NSTAMP];
#define ST_DECL unsigned long long st_acc[NSTAMP] = {0};
#define ST_T0(v) const unsigned long long v = __builtin_amdgcn_s_memtime();
#define ST_ADD(i, v) H.st_acc[i] += __builtin_amdgcn_s_memtime() - (v);
#define ST_CNT(i) H.st_acc[i] += 1;
#else
#define ST_DECL
#define ST_T0(v)
#define ST_ADD(i, v)
#define ST_CNT(i)
#endif

constexpr uint32_t HOT_MIN_LOG2 = 11;
constexpr uint32_t MAX_HOT = 256;
constexpr uint32_t LRB_CAP = 128;  // levels held in lanes (2 register sets)
constexpr uint32_t NCS = LRB_CAP;  // one head-chunk cache slot per level: never evicts
constexpr uint32_t ESTAGE = 64;    // staged events
constexpr uint32_t CS_NONE = 0xFFu;
constexpr uint32_t PEND = 0x80000000u;  // Node::ixs flag: index insert still pending
enum : uint32_t { LA_UNKNOWN = 0, LA_OID = 1, LA_NONE = 2 };

struct HotLds {
  Node cs[NCS][CH];              // cached head chunks (authoritative; written back at the end)
  gome_event ev[ESTAGE];         // staged events (publish order)
  Level tmp[LRB_CAP + 1];        // level array staging (insert / GC / load / write-back)
  uint32_t aux[3 * (LRB_CAP + 1)];  // hn, la, look-ahead state of the staged levels
  alignas(16) uint32_t cs_chunk[NCS];  // chunk id held by the slot (NIL = free)
  uint8_t freeslot[NCS];         // free cache slots (stack)
};
constexpr size_t HOT_LDS_BYTES = sizeof(HotLds);
static_assert(HOT_LDS_BYTES <= 160 * 1024, "hot book LDS budget");

// Deferred (S, oid) -> loc index insert of a node rested by a hot book (one 16-B store).
// Entry i of segment [beg, end) lives at pend[beg + i]; resolved in-kernel (flush, before a
// cancel lookup) or by k_pend_apply after the kernel.
struct PendEnt {
  uint32_t oid, loc, ix;
  uint8_t used, ins, dead, pad;
};
static_assert(sizeof(PendEnt) == 16, "PendEnt is stored as one uint4");

// A hot book that must continue on the HBM path (deep book, or lane array full):
// k_match_resume rests the spilled order's remainder and applies orders [next, end).
struct ResumeRec {
  uint32_t valid, next;
  uint32_t rest, oid, uuid, side;
  int64_t price, vol;
};

// One register set of the lane-resident level array (lane l = level 64*set + l).
// mf packs member [0,2), look-ahead state [2,4), hslot [8,16), tslot [16,24),
// cache slot [24,32) (CS_NONE: none).  hn caches ChunkHdr::next of the head chunk, la the
// oid of the first live node after the head chunk (valid per the look-ahead state).
struct LvSet {
  int64_t pr, dp;
  uint32_t hd, tl, hn, nv, mf, la;
};

// One level, extracted to wave-uniform scalars.
struct LvS {
  int64_t pr, dp;
  uint32_t hd, tl, hn, nv, mf, la;
};

struct HotCtx {
  WaveCtx W;         // device pointers, counters, arena block (W.L unused in lane mode)
  HotLds* S;
  LvSet L0, L1;      // levels [0, 64) and [64, 128)
  uint32_t nl;
  uint32_t nfree;    // free cache slots
  PendEnt* pend;
  uint32_t npend, nflushed;
  uint32_t esc;      // staged events
  ST_DECL
};

__device__ __forceinline__ uint32_t mf_member(uint32_t mf) { return mf & 3u; }
__device__ __forceinline__ uint32_t mf_lav(uint32_t mf) { return (mf >> 2) & 3u; }
__device__ __forceinline__ uint32_t mf_hslot(uint32_t mf) { return (mf >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t mf_tslot(uint32_t mf) { return (mf >> 16) & 0xFFu; }
__device__ __forceinline__ uint32_t mf_cs(uint32_t mf) { return mf >> 24; }
__device__ __forceinline__ uint32_t mf_make(uint32_t member, uint32_t lav, uint32_t hslot, uint32_t tslot,
                                           uint32_t cs) {
  return member | (lav << 2) | (hslot << 8) | (tslot << 16) | (cs << 24);
}
__device__ __forceinline__ uint32_t mf_with_lav(uint32_t mf, uint32_t lav) { return (mf & ~0xCu) | (lav << 2); }

__device__ __forceinline__ LvS lv_get(const HotCtx& H, uint32_t k) {
  const LvSet& s = (k < 64) ? H.L0 : H.L1;
  const uint32_t l = k & 63u;
  LvS v;
  v.pr = rl64(s.pr, l);
  v.dp = rl64(s.dp, l);
  v.hd = rl(s.hd, l);
  v.tl = rl(s.tl, l);
  v.hn = rl(s.hn, l);
  v.nv = rl(s.nv, l);
  v.mf = rl(s.mf, l);
  v.la = rl(s.la, l);
  return v;
}

__device__ __forceinline__ void lvset_put(LvSet& s, bool me, const LvS& v) {
  s.dp = me ? v.dp : s.dp;
  s.hd = me ? v.hd : s.hd;
  s.tl = me ? v.tl : s.tl;
  s.hn = me ? v.hn : s.hn;
  s.nv = me ? v.nv : s.nv;
  s.mf = me ? v.mf : s.mf;
  s.la = me ? v.la : s.la;
}

// Write back the mutable fields of level k (price never changes in place).
__device__ __forceinline__ void lv_put(HotCtx& H, uint32_t k, const LvS& v) {
  const uint32_t l = lane_id();
  lvset_put(H.L0, l == k, v);
  lvset_put(H.L1, l + 64 == k, v);
}

__device__ __forceinline__ bool lv_valid0(const HotCtx& H) { return lane_id() < H.nl; }
__device__ __forceinline__ bool lv_valid1(const HotCtx& H) { return lane_id() + 64 < H.nl; }

// Level index holding price p (found) or its insertion position.
__device__ __forceinline__ bool lv_find(const HotCtx& H, int64_t p, uint32_t& k) {
  const bool v0 = lv_valid0(H), v1 = lv_valid1(H);
  const unsigned long long e0 = __ballot(v0 && H.L0.pr == p), e1 = __ballot(v1 && H.L1.pr == p);
  if (e0 | e1) {
    k = e0 ? static_cast<uint32_t>(__builtin_ctzll(e0)) : 64u + static_cast<uint32_t>(__builtin_ctzll(e1));
    return true;
  }
  k = __popcll(__ballot(v0 && H.L0.pr < p)) + __popcll(__ballot(v1 && H.L1.pr < p));
  return false;
}

// ---- level array <-> LDS staging (insert shift, GC, load, write-back) ----------------
__device__ __forceinline__ Level lv_rec(const LvSet& s) {
  Level x;
  x.price = s.pr;
  x.depth = s.dp;
  x.head = s.hd;
  x.tail = s.tl;
  x.hslot = static_cast<uint8_t>(mf_hslot(s.mf));
  x.tslot = static_cast<uint8_t>(mf_tslot(s.mf));
  x.member = static_cast<uint8_t>(mf_member(s.mf));
  x.pad = static_cast<uint8_t>(mf_cs(s.mf));  // cache slot travels with the level
  x.nlive = s.nv;
  return x;
}

__device__ __forceinline__ void lv_stage(HotCtx& H, const LvSet& s, uint32_t at) {
  H.S->tmp[at] = lv_rec(s);
  H.S->aux[3 * at] = s.hn;
  H.S->aux[3 * at + 1] = s.la;
  H.S->aux[3 * at + 2] = mf_lav(s.mf);
}

__device__ __forceinline__ void lv_unstage(const HotCtx& H, LvSet& s, uint32_t at, bool valid) {
  Level x{};
  x.head = x.tail = NIL;
  x.pad = CS_NONE;
  uint32_t hn = NIL, la = 0, lav = LA_UNKNOWN;
  if (valid) {
    x = H.S->tmp[at];
    hn = H.S->aux[3 * at];
    la = H.S->aux[3 * at + 1];
    lav = H.S->aux[3 * at + 2];
  }
  s.pr = x.price;
  s.dp = x.depth;
  s.hd = x.head;
  s.tl = x.tail;
  s.hn = hn;
  s.nv = x.nlive;
  s.mf = mf_make(x.member, lav, x.hslot, x.tslot, x.pad);
  s.la = la;
}

__device__ __forceinline__ void lv_load_tmp(HotCtx& H) {
  const uint32_t lane = lane_id();
  lv_unstage(H, H.L0, lane, lane < H.nl);
  lv_unstage(H, H.L1, lane + 64, lane + 64 < H.nl);
}

// Insert an empty level for price p at position pos (shift [pos, nl) up by one).
// Returns false if the lane array is full even after dropping empty levels (spill).
__device__ __forceinline__ bool lv_insert(HotCtx& H, int64_t p, uint32_t& pos) {
  const uint32_t lane = lane_id();
  if (H.nl == LRB_CAP) {  // drop levels with no observable state (never-touched prices)
    const bool k0 = lv_valid0(H) && (H.L0.nv || H.L0.dp || mf_member(H.L0.mf));
    const bool k1 = lv_valid1(H) && (H.L1.nv || H.L1.dp || mf_member(H.L1.mf));
    const unsigned long long m0 = __ballot(k0), m1 = __ballot(k1), ltm = lt_mask();
    if (k0) lv_stage(H, H.L0, __popcll(m0 & ltm));
    if (k1) lv_stage(H, H.L1, __popcll(m0) + __popcll(m1 & ltm));
    const uint32_t out = __popcll(m0) + __popcll(m1);
    H.W.levels_delta -= static_cast<long long>(H.nl - out);
    H.nl = out;
    lv_load_tmp(H);
    lv_find(H, p, pos);
    if (H.nl == LRB_CAP) return false;
  }
  if (lane < H.nl) lv_stage(H, H.L0, lane + (lane >= pos ? 1 : 0));
  if (lane + 64 < H.nl) lv_stage(H, H.L1, lane + 64 + (lane + 64 >= pos ? 1 : 0));
  if (lane == 0) {
    Level z{};
    z.price = p;
    z.head = z.tail = NIL;
    z.pad = CS_NONE;
    H.S->tmp[pos] = z;
    H.S->aux[3 * pos] = NIL;
    H.S->aux[3 * pos + 1] = 0;
    H.S->aux[3 * pos + 2] = LA_UNKNOWN;
  }
  H.nl++;
  H.W.levels_delta++;
  lv_load_tmp(H);
  return true;
}

// ---- event staging -----------------------------------------------------------------
__device__ __forceinline__ void hot_ev_flush(HotCtx& H) {
  if (H.esc == 0) return;
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  ev_make_room(W, H.esc);
  if (W.ev_ok && lane < H.esc) {
    const uint4* src = reinterpret_cast<const uint4*>(&H.S->ev[lane]);
    uint4* dst = reinterpret_cast<uint4*>(&W.B.arena[W.ev_base + W.ev_used + lane]);
    const uint4 a = src[0], b = src[1], c = src[2], d = src[3];
    dst[0] = a;
    dst[1] = b;
    dst[2] = c;
    dst[3] = d;
  }
  W.ev_used += H.esc;
  H.esc = 0;
}

__device__ __forceinline__ void hot_ev_put(HotCtx& H, uint32_t at, int64_t price, int64_t qty,
                                           int64_t mvol, int64_t tvol, uint32_t seq, uint32_t fidx,
                                           uint32_t moid, uint32_t muuid, uint32_t mnext,
                                           uint32_t kind, uint32_t mside, uint32_t mlast) {
  uint4* e = reinterpret_cast<uint4*>(&H.S->ev[at]);
  e[0] = make_uint4(static_cast<uint32_t>(price), static_cast<uint32_t>(static_cast<uint64_t>(price) >> 32),
                    static_cast<uint32_t>(qty), static_cast<uint32_t>(static_cast<uint64_t>(qty) >> 32));
  e[1] = make_uint4(static_cast<uint32_t>(mvol), static_cast<uint32_t>(static_cast<uint64_t>(mvol) >> 32),
                    static_cast<uint32_t>(tvol), static_cast<uint32_t>(static_cast<uint64_t>(tvol) >> 32));
  e[2] = make_uint4(seq, fidx, H.W.sym, moid);
  e[3] = make_uint4(muuid, mnext, kind | (mside << 8) | (mlast << 16), 0u);
}

// ---- head-chunk cache --------------------------------------------------------------
__device__ __forceinline__ uint32_t hot_slot_alloc(HotCtx& H) {
  H.nfree--;
  return H.S->freeslot[H.nfree];
}

__device__ __forceinline__ void hot_slot_free(HotCtx& H, uint32_t cs) {
  if (lane_id() == 0) {
    H.S->freeslot[H.nfree] = static_cast<uint8_t>(cs);
    H.S->cs_chunk[cs] = NIL;
  }
  H.nfree++;
}

// Load HBM chunk `chunk` into cache slot cs; returns its next pointer.
__device__ __forceinline__ uint32_t hot_slot_fill(HotCtx& H, uint32_t cs, uint32_t chunk) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id();
  ST_CNT(10)
  if (lane < CH) {
    const uint4* src = reinterpret_cast<const uint4*>(&H.W.D.nodes[chunk * CH + lane]);
    uint4* dst = reinterpret_cast<uint4*>(&S->cs[cs][lane]);
    const uint4 a = src[0], b = src[1];
    dst[0] = a;
    dst[1] = b;
  }
  if (lane == 0) S->cs_chunk[cs] = chunk;
  return uni(H.W.D.chdr[chunk].next);
}

__device__ __forceinline__ void hot_slot_writeback(HotCtx& H, uint32_t cs) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id();
  if (lane < CH) {
    const uint4* src = reinterpret_cast<const uint4*>(&S->cs[cs][lane]);
    uint4* dst = reinterpret_cast<uint4*>(&H.W.D.nodes[S->cs_chunk[cs] * CH + lane]);
    const uint4 a = src[0], b = src[1];
    dst[0] = a;
    dst[1] = b;
  }
}

// First live node after the head chunk of level v (MatchNode.NextNode of the head chunk's
// last live maker); cached in the level's look-ahead fields until the FIFO after the head
// chunk changes.
__device__ __forceinline__ bool hot_lookahead(HotCtx& H, LvS& v, uint32_t tslot, uint32_t& oid) {
  const uint32_t lane = lane_id();
  const uint32_t st = mf_lav(v.mf);
  if (st == LA_OID) { oid = v.la; return true; }
  if (st == LA_NONE) return false;
  ST_CNT(11)
  bool found = false;
  uint32_t c2 = v.hn;
  for (uint32_t g = 0; c2 != NIL && g <= H.W.D.ch_cap; ++g) {
    const uint32_t lim = (c2 == v.tl) ? tslot : CH;
    const bool l2 = lane < lim && H.W.D.nodes[c2 * CH + (lane < CH ? lane : 0)].rem >= 0;
    const unsigned long long m2 = __ballot(l2);
    if (m2) {
      oid = uni(H.W.D.nodes[c2 * CH + __builtin_ctzll(m2)].oid);
      found = true;
      break;
    }
    c2 = (c2 == v.tl) ? NIL : uni(H.W.D.chdr[c2].next);
  }
  v.mf = mf_with_lav(v.mf, found ? LA_OID : LA_NONE);
  v.la = found ? oid : 0u;
  return found;
}

// Index bookkeeping of a node leaving the book (fill).
__device__ __forceinline__ void hot_drop_index(HotCtx& H, uint32_t ixs) {
  if (ixs & PEND) H.pend[ixs & ~PEND].dead = 1;
  else idx_erase(H.W, ixs);
}

// ---- MatchOrder (engine.go:138-198) against level k ------------------------------------
__device__ __forceinline__ int64_t hot_match_level(HotCtx& H, uint32_t k, int64_t T, uint32_t seq,
                                                   uint32_t& fidx) {
  HotLds* S = H.S;
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id(), s = lane & 31u;
  const bool hi = lane >= 32;
  LvS v = lv_get(H, k);
  uint32_t member = mf_member(v.mf), hslot = mf_hslot(v.mf), tslot = mf_tslot(v.mf), cs = mf_cs(v.mf);
  bool first = true, loaded = cs != CS_NONE;  // invariant: a level's slot holds its head chunk
  for (uint32_t guard = 0; v.hd != NIL && !W.fatal; ++guard) {
    if (guard > W.D.ch_cap) { set_err(W, ERR_CORRUPT); break; }
    if (H.esc + CH > ESTAGE) hot_ev_flush(H);  // room for one chunk step's events
    const uint32_t head = v.hd;
    if (!loaded) {
      if (cs == CS_NONE) cs = hot_slot_alloc(H);
      v.hn = hot_slot_fill(H, cs, head);
      v.mf = mf_with_lav(v.mf, LA_UNKNOWN);
      loaded = true;
    }
    const Node nd = S->cs[cs][s];
    const uint32_t lim = (head == v.tl) ? tslot : CH;
    const bool inr = !hi && s >= hslot && s < lim;
    const int64_t r = inr ? nd.rem : -1;
    const bool live = inr && r >= 0;
    const uint32_t mlo = static_cast<uint32_t>(__ballot(live));
    if (mlo == 0) {  // head chunk exhausted (consumed/cancelled slots only)
      if (head == v.tl) { set_err(W, ERR_CORRUPT); break; }
      free_chunk(W, head);
      v.hd = v.hn;
      hslot = 0;
      loaded = false;
      continue;
    }
    const uint32_t fl = __builtin_ctz(mlo), ll = 31 - __clz(mlo);
    const int64_t rf = rl64(r, fl);
    ST_CNT(13)
    if (T < rf) {
      // fast path: the taker ends inside the first live maker (diff < 0, engine.go:176-194)
      ST_CNT(14)
      const uint32_t after = (fl < 31) ? (mlo & (~0u << (fl + 1))) : 0u;
      uint32_t nx = 0;
      bool last = true;
      if (after) { nx = rl(nd.oid, __builtin_ctz(after)); last = false; }
      else if (hot_lookahead(H, v, tslot, nx)) last = false;
      const uint32_t tf = rl(nd.tx, fl);
      if (lane == 0) {
        hot_ev_put(H, H.esc, v.pr, T, rf - T, 0, seq, fidx, rl(nd.oid, fl), rl(nd.uuid, fl),
                   last ? 0u : nx, GOME_EV_FILL, tf, last ? 1u : 0u);
        S->cs[cs][fl].rem = rf - T;
      }
      H.esc += 1;
      fidx += 1;
      W.fills += 1;
      v.dp -= T;
      if (v.dp <= 0) member &= ~((tf == GOME_SALE) ? M_SALE : M_BUY);  // ZREM maker's side
      hslot = fl;
      T = 0;
      break;
    }
    // general path: prefix scan of live volumes decides reached / filled / partial makers
    const int64_t x = live ? r : 0;
    const int64_t incl = scan32_i64(x);
    const int64_t excl = incl - x;
    const bool arr = live && (excl < T || (first && T == 0 && s == fl));
    const bool pop = arr && incl <= T;
    const int64_t f = pop ? r : (T - excl);
    const unsigned long long am = __ballot(arr), pm = __ballot(pop);
    const uint32_t narr = __popcll(am), npop = __popcll(pm);
    const uint32_t la = 63 - __builtin_clzll(am);
    const uint32_t after = (s < 31) ? (mlo & (~0u << (s + 1))) : 0u;
    uint32_t nx_oid = __shfl(nd.oid, after ? static_cast<int>(__builtin_ctz(after)) : 0);
    bool is_last = after == 0;
    if ((am >> ll) & 1ull) {
      uint32_t la_oid = 0;
      if (hot_lookahead(H, v, tslot, la_oid) && lane == ll) { nx_oid = la_oid; is_last = false; }
    }
    const int64_t tafter = T - excl - f;
    const int64_t dafter = v.dp - excl - f;
    const bool clr = arr && dafter <= 0;
    const unsigned long long clr_s = __ballot(clr && nd.tx == GOME_SALE), clr_b = __ballot(clr && nd.tx != GOME_SALE);
    if (arr) {
      const uint32_t rank = __popcll(am & lt_mask());
      hot_ev_put(H, H.esc + rank, v.pr, f, pop ? r : r - f, tafter, seq, fidx + rank, nd.oid, nd.uuid,
                 is_last ? 0u : nx_oid, GOME_EV_FILL, nd.tx, is_last ? 1u : 0u);
    }
    H.esc += narr;
    fidx += narr;
    W.fills += narr;
    const int64_t Tn = rl64(tafter, la);
    v.dp -= (T - Tn);
    if (clr_s) member &= ~M_SALE;
    if (clr_b) member &= ~M_BUY;
    if (pop) hot_drop_index(H, nd.ixs);
    v.nv -= npop;
    W.resting_delta -= npop;
    first = false;
    if (!((pm >> la) & 1ull)) {  // partial fill of maker la: it keeps its FIFO position
      if (lane == la) S->cs[cs][s].rem = r - f;
      hslot = la;
      T = 0;
      break;
    }
    T = Tn;
    hslot = la + 1;
    if (v.nv == 0) {
      free_chain(W, v.hd, v.tl);
      hot_slot_free(H, cs);
      cs = CS_NONE;
      v.hd = v.tl = v.hn = NIL;
      hslot = tslot = 0;
      break;
    }
    if (T <= 0) break;  // diff == 0: stop (engine.go:162-175)
    free_chunk(W, head);  // every live maker of the head chunk consumed, T > 0
    v.hd = v.hn;
    hslot = 0;
    loaded = false;
  }
  v.mf = mf_make(member, mf_lav(v.mf), hslot, tslot, cs);
  lv_put(H, k, v);
  return T;
}

// ---- rest the remaining volume (engine.go:80-82) ---------------------------------------
__device__ __forceinline__ bool hot_rest(HotCtx& H, int64_t p, int64_t T, uint32_t oid, uint32_t uuid,
                                         uint32_t side) {
  HotLds* S = H.S;
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  uint32_t k;
  if (!lv_find(H, p, k) && !lv_insert(H, p, k)) return false;
  LvS v = lv_get(H, k);
  const uint32_t member = mf_member(v.mf) | ((side == GOME_SALE) ? M_SALE : M_BUY);  // SetPoolDepth
  uint32_t hslot = mf_hslot(v.mf), tslot = mf_tslot(v.mf), cs = mf_cs(v.mf), lav = mf_lav(v.mf);
  v.dp += T;                                                                          // SetPoolDepthVolume
  if (v.tl == NIL || tslot == CH) {  // SetDepthLink: new tail chunk
    const uint32_t c = alloc_chunk(W);
    if (c == NIL) return true;
    if (lane == 0) {
      ChunkHdr h;
      h.next = NIL;
      h.pad = 0;
      h.price = p;
      W.D.chdr[c] = h;
      if (v.tl != NIL) W.D.chdr[v.tl].next = c;
    }
    if (v.tl == NIL) {  // FIFO was empty: the new chunk is the head, cache it (nothing to load)
      v.hd = c;
      v.hn = NIL;
      hslot = 0;
      cs = hot_slot_alloc(H);
      if (lane == 0) S->cs_chunk[cs] = c;
      lav = LA_NONE;
    } else if (v.hd == v.tl) {
      v.hn = c;
    }
    v.tl = c;
    tslot = 0;
  }
  const uint32_t loc = v.tl * CH + tslot;
  const uint32_t pidx = H.npend++;
  const bool in_cache = cs != CS_NONE && v.hd == v.tl;  // the tail is the cached head chunk
  if (!in_cache && lav == LA_NONE) lav = LA_UNKNOWN;     // a live node now follows the head chunk
  if (lane == 0) {
    // PendEnt {oid, loc, ix = NIL, used = 1, ins = dead = 0}
    st16_glb(&H.pend[pidx], v4(oid, loc, NIL, 1u));
    const v4u a = v4(lo32(T), hi32(T), oid, uuid), b = v4(PEND | pidx, side & 0xFFu, 0u, 0u);
    if (in_cache) {
      Node* d = &S->cs[cs][tslot];
      st16_lds(d, a);
      st16_lds(reinterpret_cast<char*>(d) + 16, b);
    } else {
      Node* d = &W.D.nodes[loc];
      st16_glb(d, a);
      st16_glb(reinterpret_cast<char*>(d) + 16, b);
    }
  }
  v.nv++;
  v.mf = mf_make(member, lav, hslot, tslot + 1, cs);
  lv_put(H, k, v);
  W.rests++;
  W.resting_delta++;
  return true;
}

// ---- SetOrder (engine.go:56-85) ---------------------------------------------------------
// Returns false when the order has been matched but cannot rest because the lane array is
// full (spill): the caller hands `trest` to the HBM path.
__device__ __forceinline__ bool hot_add(HotCtx& H, int64_t p, int64_t vol, uint32_t oid, uint32_t uuid,
                                        uint32_t side, uint32_t seq, uint32_t& nev, int64_t& trest) {
  int64_t T = vol;
  uint32_t fidx = 0;
  ST_T0(t_m)
  // GetReverseDepth (nodepool.go:86-115): opposite-side levels crossing p, best first
  // (asks ascending for a BUY, bids descending for a SALE; Transaction != 1 is BUY).
  const bool buy = side != GOME_SALE;
  const uint32_t bit = buy ? M_SALE : M_BUY;
  const bool v0 = lv_valid0(H), v1 = lv_valid1(H);
  const bool c0 = v0 && (H.L0.mf & bit) && (buy ? H.L0.pr <= p : H.L0.pr >= p);
  const bool c1 = v1 && (H.L1.mf & bit) && (buy ? H.L1.pr <= p : H.L1.pr >= p);
  unsigned long long m0 = __ballot(c0), m1 = __ballot(c1);
  const bool crossed = (m0 | m1) != 0;
  // crossing levels in priority order: bits of (m1:m0) upward for a BUY, downward for a SALE
  while ((m0 | m1) && !H.W.fatal) {
    uint32_t k;
    if (buy) {
      if (m0) { k = __builtin_ctzll(m0); m0 &= m0 - 1; }
      else { k = 64 + __builtin_ctzll(m1); m1 &= m1 - 1; }
    } else {
      if (m1) { const uint32_t b = 63 - __builtin_clzll(m1); m1 &= ~(1ull << b); k = 64 + b; }
      else { const uint32_t b = 63 - __builtin_clzll(m0); m0 &= ~(1ull << b); k = b; }
    }
    T = hot_match_level(H, k, T, seq, fidx);  // Match (engine.go:118-136)
    if (T <= 0) break;
  }
  ST_ADD(1, t_m)
  nev = fidx;
  trest = T;
  if ((!crossed || T > 0) && !H.W.fatal) {
    ST_T0(t_r)
    const bool ok = hot_rest(H, p, T, oid, uuid, side);
    ST_ADD(3, t_r)
    return ok;
  }
  return true;
}

// Insert this segment's pending entries [nflushed, npend) into the global index (needed
// before a cancel lookup) and store each node's real slot into its chunk slot (LDS cache or
// HBM), so later fills and cancels erase directly.
__device__ __forceinline__ void hot_flush(HotCtx& H) {
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  const unsigned long long mask = W.D.idx_mask;
  bool full = false;
  for (uint32_t b = H.nflushed; b < H.npend; b += 64) {
    const uint32_t i = b + lane;
    PendEnt e{};
    bool ok = false;
    unsigned long long h = 0;
    if (i < H.npend) {
      e = H.pend[i];
      if (!e.dead) {
        const unsigned long long key = idx_key(W.sym, e.oid);
        h = mix64(key) & mask;
        unsigned long long probe = 0;
        for (; probe <= mask; ++probe, h = (h + 1) & mask) {
          const unsigned long long kv =
              __hip_atomic_load(&W.D.idx[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((kv == KEY_EMPTY || kv == KEY_TOMB) && atomicCAS(&W.D.idx[h].key, kv, key) == kv) break;
        }
        if (probe > mask) {
          full = true;
        } else {
          ok = true;
          W.D.idx[h].loc = e.loc;
          H.pend[i].ix = static_cast<uint32_t>(h);
          H.pend[i].ins = 1;
        }
      }
    }
    // write each node's real slot through the cache when its chunk is a cached head:
    // every lane scans the slot table (broadcast 16-B LDS reads) for its own chunk
    if (__ballot(ok)) {
      const uint32_t cid = ok ? e.loc / CH : NIL - 1;
      uint32_t cs = CS_NONE;
      const uint4* tab = reinterpret_cast<const uint4*>(H.S->cs_chunk);
#pragma unroll 8
      for (uint32_t c = 0; c < NCS / 4; ++c) {
        const uint4 w = tab[c];
        cs = (w.x == cid) ? 4 * c : cs;
        cs = (w.y == cid) ? 4 * c + 1 : cs;
        cs = (w.z == cid) ? 4 * c + 2 : cs;
        cs = (w.w == cid) ? 4 * c + 3 : cs;
      }
      if (ok) {
        if (cs != CS_NONE) *as_lds(&H.S->cs[cs][e.loc % CH].ixs) = static_cast<uint32_t>(h);
        else *as_glb(&W.D.nodes[e.loc].ixs) = static_cast<uint32_t>(h);
      }
    }
  }
  if (__ballot(full)) set_err(W, ERR_INDEX);
  H.nflushed = H.npend;
}

// ---- DeleteOrder (engine.go:87-116) ------------------------------------------------------
__device__ __forceinline__ uint32_t hot_cancel(HotCtx& H, int64_t p, uint32_t oid, uint32_t uuid,
                                               uint32_t side, uint32_t seq) {
  HotLds* S = H.S;
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  if (H.nflushed < H.npend) hot_flush(H);
  uint32_t ixslot, loc;
  if (!idx_lookup(W, oid, ixslot, loc)) return 0;                       // no event
  const uint32_t cid = loc / CH, sl = loc % CH;
  if (uni(static_cast<uint32_t>(W.D.chdr[cid].price != p))) return 0;  // Q3
  uint32_t k;
  if (!lv_find(H, p, k)) { set_err(W, ERR_CORRUPT); return 0; }
  LvS v = lv_get(H, k);
  uint32_t member = mf_member(v.mf), hslot = mf_hslot(v.mf), tslot = mf_tslot(v.mf), cs = mf_cs(v.mf);
  const bool cached = cs != CS_NONE && v.hd == cid;
  const int64_t r = cached ? rl64(*as_lds(&S->cs[cs][sl].rem), 0) : rl64(*as_glb(&W.D.nodes[loc].rem), 0);
  if (r < 0) { set_err(W, ERR_CORRUPT); return 0; }
  v.dp -= r;  // DeletePoolDepthVolume with the stored remaining volume
  if (v.dp <= 0) member &= ~((side == GOME_SALE) ? M_SALE : M_BUY);  // the REQUEST's side (Q2)
  if (lane == 0) {
    if (cached) *as_lds(&S->cs[cs][sl].rem) = -1;
    else *as_glb(&W.D.nodes[loc].rem) = -1;
    idx_erase(W, ixslot);
  }
  v.nv--;
  W.resting_delta--;
  if (v.nv == 0) {
    free_chain(W, v.hd, v.tl);
    if (cs != CS_NONE) hot_slot_free(H, cs);
    cs = CS_NONE;
    v.hd = v.tl = v.hn = NIL;
    hslot = tslot = 0;
  }
  v.mf = mf_make(member, LA_UNKNOWN, hslot, tslot, cs);
  lv_put(H, k, v);
  if (H.esc + 1 > ESTAGE) hot_ev_flush(H);
  if (lane == 0) hot_ev_put(H, H.esc, p, 0, r, r, seq, 0, oid, uuid, 0u, GOME_EV_CANCEL, side, 1u);
  H.esc += 1;
  W.cancels++;
  return 1;
}

// Write the lane book back to HBM: every cached chunk, then the level array (growing the
// book's HBM level block if needed).  Afterwards W.L/nl/cap/base describe the HBM book.
__device__ __forceinline__ void hot_writeback(HotCtx& H) {
  HotLds* S = H.S;
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  for (uint32_t cs = 0; cs < NCS; ++cs)
    if (S->cs_chunk[cs] != NIL) hot_slot_writeback(H, cs);
  if (H.nl > W.cap) {
    uint32_t ncap = 16;
    while (ncap < H.nl) ncap <<= 1;
    uint32_t nb = 0;
    if (lane == 0) nb = atomicAdd(W.D.lvl_bump, ncap);
    nb = uni(nb);
    if (static_cast<unsigned long long>(nb) + ncap > W.D.lvl_cap_total) { set_err(W, ERR_LEVELS); return; }
    W.base = nb;
    W.cap = ncap;
    W.L = W.D.lvl + nb;
  }
  Level a = lv_rec(H.L0), b = lv_rec(H.L1);
  a.pad = b.pad = 0;  // cache slots are kernel-local
  if (lane < H.nl) W.L[lane] = a;
  if (lane + 64 < H.nl) W.L[lane + 64] = b;
  W.nl = H.nl;
}

// Spill path only: complete every pending entry inline (flush) so that every resting node
// carries its real index slot, as the HBM path expects; must run before hot_writeback.
__device__ __forceinline__ void hot_resolve_pending(HotCtx& H) {
  hot_flush(H);
  for (uint32_t i = lane_id(); i < H.npend; i += 64) H.pend[i].used = 0;
}

__global__ __launch_bounds__(64) void k_match_hot(Dev D, BatchArgs B, PendEnt* pend_arena,
                                                   ResumeRec* resume) {
  extern __shared__ __align__(16) unsigned char smem[];
  if (blockIdx.x >= D.st->nhot || (D.st->err & ERR_INPUT)) return;
  __builtin_amdgcn_s_setprio(3);  // the hottest books are the batch's critical path
  const uint32_t lane = lane_id();
  const uint32_t seg = B.seg_order[blockIdx.x];
  const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
  HotCtx H;
  WaveCtx& W = H.W;
  wave_init(W, D, B, uni(B.ord[B.prep[beg].idx].symbol_id), EVB_HOT);
  ResumeRec rr{};
  if (W.nl > LRB_CAP - 16) {  // deep book: the HBM path applies the whole segment
    if (lane == 0) {
      rr.valid = 1;
      rr.next = beg;
      resume[blockIdx.x] = rr;
    }
    return;
  }
  HotLds* S = reinterpret_cast<HotLds*>(smem);
  H.S = S;
  H.nl = W.nl;
  H.pend = pend_arena + beg;
  H.npend = H.nflushed = 0;
  H.esc = 0;
  H.nfree = NCS;
  for (uint32_t c = lane; c < NCS; c += 64) {
    S->freeslot[c] = static_cast<uint8_t>(c);
    S->cs_chunk[c] = NIL;
  }
  for (uint32_t k = lane; k < H.nl; k += 64) {
    Level x = W.L[k];
    x.pad = CS_NONE;  // no cache slot yet
    S->tmp[k] = x;
    S->aux[3 * k] = NIL;
    S->aux[3 * k + 1] = 0;
    S->aux[3 * k + 2] = LA_UNKNOWN;
  }
  lv_load_tmp(H);

  bool spilled = false;
  Prep qn{};
  if (lane < min(64u, end - beg)) qn = B.prep[beg + lane];
  for (uint32_t b0 = beg; b0 < end && !W.fatal && !spilled; b0 += 64) {
    ST_T0(t_b)
    const uint32_t cnt = min(64u, end - b0);
    const Prep q = qn;
    if (b0 + 64 < end && lane < min(64u, end - b0 - 64)) qn = B.prep[b0 + 64 + lane];  // prefetch
    uint32_t evc = 0;  // lane j: events of order j of this block
    uint32_t j = 0;
    ST_ADD(6, t_b)
    for (; j < cnt && !W.fatal; ++j) {
      ST_T0(t_o)
      const uint32_t idx = rl(q.idx, j), a = rl(q.action, j);
      uint32_t nev = 0;
      if (a == GOME_ADD) {
        W.adds++;
        if (rl(q.adm, j)) {
          int64_t trest = 0;
          const int64_t p = rl64(q.price, j);
          const uint32_t oid = rl(q.oid, j), uuid = rl(q.uuid, j), side = rl(q.side, j);
          if (!hot_add(H, p, rl64(q.vol, j), oid, uuid, side, idx, nev, trest)) {
            spilled = true;  // lane array full: the HBM path rests it and continues
            rr.valid = 1;
            rr.next = b0 + j + 1;
            rr.rest = 1;
            rr.price = p;
            rr.vol = trest;
            rr.oid = oid;
            rr.uuid = uuid;
            rr.side = side;
          }
        } else {
          W.dropped++;  // marker already consumed (engine.go:58-60)
        }
      } else if (a == GOME_DEL) {
        W.dels++;
        nev = hot_cancel(H, rl64(q.price, j), rl(q.oid, j), rl(q.uuid, j), rl(q.side, j), idx);
      }
      evc = (lane == j) ? nev : evc;
      ST_ADD(0, t_o)
      ST_CNT(9)
      if (spilled) { ++j; break; }
    }
    if (lane < j) B.ev_count[q.idx] = evc;
  }
  hot_ev_flush(H);
  if (spilled) hot_resolve_pending(H);  // the HBM path expects real index slots
  hot_writeback(H);
  if (lane == 0) {
    resume[blockIdx.x] = rr;
    unsigned long long* c = W.D.st->ctr;
    atomicAdd(&c[C_HOT_ORDERS], static_cast<unsigned long long>((spilled ? rr.next : end) - beg));
    atomicAdd(&c[C_HOT_FILLS], W.fills);
    atomicAdd(&c[C_HOT_RESTS], W.rests);
    atomicAdd(&c[C_HOT_CANCELS], W.cancels);
  }
  wave_finish(W);
#ifdef GOME_STAMPS
  if (lane == 0 && blockIdx.x < 256)
    for (int i = 0; i < NSTAMP; ++i) g_stamps[blockIdx.x * NSTAMP + i] = H.st_acc[i];
#endif
}

// Continue hot books that left the lane path (see ResumeRec) on the HBM path.
__global__ __launch_bounds__(64) void k_match_resume(Dev D, BatchArgs B, const ResumeRec* resume) {
  if (blockIdx.x >= D.st->nhot || (D.st->err & ERR_INPUT)) return;
  const ResumeRec rr = resume[blockIdx.x];
  if (!rr.valid) return;
  const uint32_t seg = B.seg_order[blockIdx.x];
  const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
  WaveCtx W;
  wave_init(W, D, B, uni(B.ord[B.prep[beg].idx].symbol_id), EVB_HOT);
  if (rr.rest) do_rest(W, rr.price, rr.vol, rr.oid, rr.uuid, rr.side);
  process_global(W, rr.next, end);
  wave_finish(W);
}

// Resolve the deferred index inserts of all hot books (after k_match_hot): insert every
// entry that is still live and was not flushed in-kernel, and store the node's real index
// slot into its chunk (HBM; the kernel has written its LDS caches back).
__global__ void k_pend_apply(const Dev D, PendEnt* pend, const uint32_t* seg_start,
                             const uint32_t* seg_order, const BatchArgs B) {
  const uint32_t nhot = D.st->nhot;
  const unsigned long long mask = D.idx_mask;
  for (uint32_t h = blockIdx.y; h < nhot; h += gridDim.y) {
    const uint32_t seg = seg_order[h];
    const uint32_t beg = seg_start[seg], end = seg_start[seg + 1];
    const uint32_t sym = B.ord[B.prep[beg].idx].symbol_id;
    for (uint32_t i = beg + blockIdx.x * blockDim.x + threadIdx.x; i < end; i += gridDim.x * blockDim.x) {
      const PendEnt e = pend[i];
      if (!e.used) continue;
      pend[i].used = 0;
      if (e.dead || e.ins) continue;  // filled before insertion / completed in-kernel
      const unsigned long long key = (static_cast<unsigned long long>(sym + 1) << 32) | e.oid;
      unsigned long long hh = mix64(key) & mask, probe = 0;
      for (; probe <= mask; ++probe, hh = (hh + 1) & mask) {
        const unsigned long long kv = __hip_atomic_load(&D.idx[hh].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((kv == KEY_EMPTY || kv == KEY_TOMB) && atomicCAS(&D.idx[hh].key, kv, key) == kv) break;
      }
      if (probe > mask) { atomicOr(&D.st->err, ERR_INDEX); continue; }
      D.idx[hh].loc = e.loc;
      D.nodes[e.loc].ixs = static_cast<uint32_t>(hh);
    }
  }
}

}  // namespace gome
