// match_flow_cancel.h — cancels on the flow path: hot books whose segment holds DELs.
//
// DeleteOrder (engine.go:87-116) removes a maker's *remaining* volume from its level (depth -=
// stored remaining, ZREM when the level empties) and unlinks it (nodelink.go:124-166).  What a
// cancel removes depends on how much of the maker was consumed before it, i.e. on FIFO order,
// which the aggregate plan (match_flow.h) does not track.  It does not have to.  For a DEL of
// maker m (level k, side s, volume v_m) let Q be the volume of the side-s makers that arrived at
// level k after m and before the DEL and were not cancelled before it.  While m is live those
// makers are untouched (only the FIFO head is ever partly consumed, and a same-side ADD at m's
// level cannot cross), and if m was partly consumed nothing ahead of it is live; once m is gone
// (or never rested) every live side-s maker of the level arrived after it.  So
//
//     r_m = clamp(depth_s,k - Q, 0, v_m)
//
// and Q needs nothing from the plan: it is a sum over the segment's records (volumes of the
// same-side ADDs at the level between m and the DEL, minus the targets among them cancelled
// before the DEL).  The prep computes it per DEL and writes it into the DEL's W32C record; the
// plan (gen_plan_asm.py) keeps only the per-side depths.  tools/flow_cancel_model.py
// (plan_book_q) checks the formula against the oracle.
//
// Prep (after the book's ordinary prep, which builds the level set and the 32-bit records):
//   k_fc_hash_claim / k_fc_hash_count   (symbol, oid) table of the books' ADD / DEL records
//   k_fc_resolve    each DEL's target: an earlier admitted ADD of the segment (new maker) or a
//                   resting node (old maker, the cancel index); Q3 (wrong price) and DELs whose
//                   oid is not resting are no-ops; duplicate oids decline; Q2 (wrong side:
//                   the depth and FIFO change as for the maker's side, only the ZREM misses,
//                   engine.go:87-116) is taken by the head books' lane plans, which then
//                   compute with the maker's side (fc_del_sale) and leave the membership to
//                   k_fc_stale_level; every other book declines
//   k_fc_oldwalk    old targets' FIFO ranks, arrival ends and volumes (a walk of their level)
//   head books, tile-parallel: k_fc_pcnt / k_fc_pscan / k_fc_prank   targeted ADDs' ranks per
//                   level, each DEL's count of targets that arrived before it, and the (level,
//                   side) ADD volume before every targeted ADD and DEL; k_fc_pwin   windows, DEL
//                   times and volumes by rank; k_fc_precs   Q and the DEL records
//   tail books: k_fc_pass, the same in one block per book
// Reconstruction (after the plan and the level sort of its touches):
//   k_fc_level      per level: cancels -> their DEL's record; the consumption-space layout of
//                   the makers (a cancelled maker only spans what was consumed before its
//                   cancel), the gathered old makers, the new makers
//   k_fc_count_nf / _run, k_fc_events   fills as interval intersections (zero-length makers skipped,
//                   MatchNode.NextNode skips makers cancelled before the fill), cancel events,
//                   tombstones of cancelled old makers
//   k_fc_write      surviving new makers appended, the level records; k_fc_fin the book.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "match_cold.h"
#include "match_flow.h"
#include "pipeline.h"
#include "wave.h"

namespace gome {

struct FcHash {
  unsigned long long key;  // gen << 53 | (symbol + 1) << 32 | oid; another generation = empty
  uint32_t add_pos;        // first admitted ADD of the key (segment position), NIL none
  uint32_t cnt;            // admitted ADDs
  uint32_t del_first;      // the DEL that can find the maker: the first after the ADD (or the
                           // first at all, for a resting maker); later ones find nothing
  uint32_t pad[3];
};
static_assert(sizeof(FcHash) == 32, "FcHash layout");

struct FcDel {
  uint32_t kind;     // FC_NONE (no-op), FC_NEW, FC_OLD
  uint32_t li;       // the target's level
  uint32_t tgt;      // FC_NEW: the ADD's segment position; FC_OLD: the node (chunk * CH + slot)
  uint32_t rank;     // the target's rank among the level's targets (arrival order)
  uint32_t nb;       // window: targets that arrived behind the target before this DEL (the
                     // candidates of Q's cancelled part)
  uint32_t ixs;      // FC_OLD: the node's cancel-index slot
  uint32_t oend, ov; // the target's arrival end / volume (plan units; FC_NEW: counted over the
                     // segment's ADDs only)
  int64_t r;         // recon: volume cancelled (fixed point), 0 if the DEL found nothing
  uint32_t ct;       // recon: touch index of the cancel, NIL if none
  uint32_t va;       // volume of the segment's side-s ADDs at the level before the DEL
};
static_assert(sizeof(FcDel) == 48, "FcDel layout");
enum : uint32_t { FC_NONE = 0, FC_NEW = 1, FC_OLD = 2 };

constexpr uint32_t FC_MAXKEY_SYM = (1u << 21) - 1;  // symbol + 1 fits 21 bits of the key

// A book whose segment holds DELs: a lane book (FL_OK_CANCEL) or a deep one (FL_OK_DEEP, dc).
__device__ __forceinline__ bool fc_dels(const FlowArgs& F, uint32_t h) {
  return F.hdr[h].ok == FL_OK_CANCEL || (F.hdr[h].ok == FL_OK_DEEP && F.hdr[h].dc);
}
__device__ __forceinline__ bool fc_book(const FlowArgs& F, uint32_t h) { return fc_dels(F, h) && !F.hdr[h].fc_bad; }
// the lane books only (the kernels whose per-level state is FL_CAP wide)
__device__ __forceinline__ bool fc_lane(const FlowArgs& F, uint32_t h) {
  return F.hdr[h].ok == FL_OK_CANCEL && !F.hdr[h].fc_bad;
}
__device__ __forceinline__ bool fc_deep(const FlowArgs& F, uint32_t h) {
  return F.hdr[h].ok == FL_OK_DEEP && F.hdr[h].dc && !F.hdr[h].fc_bad;
}
constexpr uint32_t FD_MAX_V = 1u << 16;  // a deep book's DEL target volume (plan units): 16 bits of its record
__device__ __forceinline__ void fc_decline(const FlowArgs& F, uint32_t h, uint32_t why) {
  atomicOr(&F.hdr[h].fc_bad, why);
}
__device__ __forceinline__ unsigned long long fc_key(const FlowArgs& F, uint32_t sym, uint32_t oid) {
  return (static_cast<unsigned long long>(F.fc_gen & FC_GEN_MASK) << 53) |
         (static_cast<unsigned long long>(sym + 1) << 32) | oid;
}

// The side of the target of the DEL at segment position b (the maker's: a wrong-side cancel's
// request says the other, Q2), which k_fc_resolve keeps in FlowArgs::fc_rank (a DEL position's
// entry is free: ranks are the targeted ADDs').  (Read back from there rather than reloaded from
// the node or the ADD: the dual-source load miscompiled beside the window code, gfx950.)
__device__ __forceinline__ bool fc_del_sale(const FlowArgs& F, uint32_t b) { return F.fc_rank[b] != 0u; }

// Book h's list of long-window DELs (k_fc_precs -> k_fc_precs_long): its touch-fill scratch
// (FlowArgs::tfc, free until the reconstruction), as 32-bit positions.
__device__ __forceinline__ uint32_t* fc_long_list(const FlowArgs& F, const FlowHdr& hd) {
  return reinterpret_cast<uint32_t*>(F.tfc + static_cast<size_t>(FL_TOUCH_MUL) * hd.beg);
}

// Slice [b0, b1) of book h's segment for block x of `nx`.
__device__ __forceinline__ void fc_slice(const FlowHdr& hd, uint32_t x, uint32_t nx, uint32_t& b0, uint32_t& b1) {
  const uint64_t len = hd.end - hd.beg;
  b0 = hd.beg + static_cast<uint32_t>(len * x / nx);
  b1 = hd.beg + static_cast<uint32_t>(len * (x + 1) / nx);
}

__device__ __forceinline__ uint32_t fc_hash_find(const FlowArgs& F, unsigned long long key, bool claim) {
  const unsigned long long gen_mask = static_cast<unsigned long long>(FC_GEN_MASK) << 53;
  unsigned long long s = mix64(key) & F.fc_hmask;
  for (unsigned long long probe = 0; probe <= F.fc_hmask; ++probe, s = (s + 1) & F.fc_hmask) {
    unsigned long long cur = __hip_atomic_load(&F.fc_hash[s].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return static_cast<uint32_t>(s);
    const bool stale = cur == 0ull || (cur & gen_mask) != (key & gen_mask);
    if (!stale) continue;
    if (!claim) return NIL;
    const unsigned long long prev = atomicCAS(&F.fc_hash[s].key, cur, key);
    if (prev == cur) {
      F.fc_hash[s].add_pos = NIL;
      F.fc_hash[s].cnt = 0;
      F.fc_hash[s].del_first = NIL;
      return static_cast<uint32_t>(s);
    }
    if (prev == key) return static_cast<uint32_t>(s);
  }
  return NIL;
}

// Resting node of (sym, oid) through the cancel index (HGET S:link:<p> S:node:<oid>,
// engine.go:92-93); NIL if none.
__device__ __forceinline__ uint32_t fc_old_lookup(const Dev& D, uint32_t sym, uint32_t oid, uint32_t& ixs) {
  const unsigned long long key = (static_cast<unsigned long long>(sym + 1) << 32) | oid;
  unsigned long long s = mix64(key) & D.idx_mask;
  for (unsigned long long probe = 0; probe <= D.idx_mask; ++probe, s = (s + 1) & D.idx_mask) {
    const unsigned long long kv = __hip_atomic_load(&D.idx[s].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kv == key) {
      ixs = static_cast<uint32_t>(s);
      return D.idx[s].loc;
    }
    if (kv == KEY_EMPTY) return NIL;
  }
  return NIL;
}

// ---- prep 1: claim a table entry per key, reset the books' per-position scratch ----------
// (The scratch of every book with DELs is reset, declined or not: k_fc_unmark reads it.)
__global__ __launch_bounds__(256) void k_fc_hash_claim(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F) || !fc_dels(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  uint32_t b0, b1;
  fc_slice(hd, blockIdx.x, gridDim.x, b0, b1);
  const bool claim = hd.sym < FC_MAXKEY_SYM;
  if (!claim && threadIdx.x == 0) fc_decline(F, h, FC_BAD_SYM);
  if (blockIdx.x == 0 && threadIdx.x == 0) F.hdr[h].nlong = 0;  // (k_fc_precs' long-window list)
  if (hd.end - hd.beg + 8 > FC_MAX_ORDERS && blockIdx.x == 0 && threadIdx.x == 0) fc_decline(F, h, FC_BAD_RING);
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
    F.fc_tg[b] = 0;
    F.fc_rank[b] = NIL;
    const Prep q = prep_at(B, b);
    if (q.action == GOME_DEL) {
      FcDel z{};
      z.ct = NIL;
      F.fc_del[b] = z;
    }
    if (claim && (q.action == GOME_DEL || (q.action == GOME_ADD && q.adm)))
      if (fc_hash_find(F, fc_key(F, hd.sym, q.oid), true) == NIL) fc_decline(F, h, FC_BAD_TABLE);
  }
}

// ---- prep 2: first admitted ADD and the counts of each key -------------------------------
__global__ __launch_bounds__(256) void k_fc_hash_count(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F) || !fc_book(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  uint32_t b0, b1;
  fc_slice(hd, blockIdx.x, gridDim.x, b0, b1);
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
    const Prep q = prep_at(B, b);
    const bool add = q.action == GOME_ADD && q.adm;
    if (!add && q.action != GOME_DEL) continue;
    const uint32_t s = fc_hash_find(F, fc_key(F, hd.sym, q.oid), false);
    if (s == NIL) continue;  // (declined in prep 1)
    if (add) {
      atomicMin(&F.fc_hash[s].add_pos, b);
      atomicAdd(&F.fc_hash[s].cnt, 1u);
    }
  }
}

// ---- prep 2b: the DEL of each key that can find its maker ----------------------------------
__global__ __launch_bounds__(256) void k_fc_hash_first(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F) || !fc_book(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  uint32_t b0, b1;
  fc_slice(hd, blockIdx.x, gridDim.x, b0, b1);
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
    const Prep q = prep_at(B, b);
    if (q.action != GOME_DEL) continue;
    const uint32_t s = fc_hash_find(F, fc_key(F, hd.sym, q.oid), false);
    if (s == NIL) continue;
    // a DEL with another price misses S:link:<price> (Q3) and finds nothing either way
    const uint32_t ap = F.fc_hash[s].add_pos;
    bool finds = false;
    if (ap == NIL) {
      uint32_t ixs;
      const uint32_t loc = fc_old_lookup(D, hd.sym, q.oid, ixs);
      finds = loc != NIL && D.chdr[loc / CH].price == q.price;
    } else {
      finds = ap < b && prep_at(B, ap).price == q.price;
    }
    if (finds) atomicMin(&F.fc_hash[s].del_first, b);
  }
}

// Level of price p in book h's level table (1..nl, ascending), 0 if absent.
__device__ __forceinline__ uint32_t fc_level_of(const FlowLvl* LV, uint32_t nl, int64_t p) {
  uint32_t lo = 1, hi = nl + 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (LV[mid].price < p) lo = mid + 1; else hi = mid;
  }
  return (lo <= nl && LV[lo].price == p) ? lo : 0u;
}

// ---- prep 3: each DEL's target -------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fc_resolve(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F) || !fc_book(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  FlowLvl* LV = fl_lvls(F, h);
  const uint32_t lmask = hd.ok == FL_OK_DEEP ? 0x3FFFu : 127u;  // a record's level bits
  // wrong-side cancels (Q2): the head books' lane plans, which k_fc_stale_level checks and hands
  // to the legacy kernel when the stale member they make is observable
  const bool q2_ok = hd.ok == FL_OK_CANCEL && h < FL_HEAD && hd.end - hd.beg >= LEGACY_HOT_MIN;
  uint32_t b0, b1;
  fc_slice(hd, blockIdx.x, gridDim.x, b0, b1);
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
    const Prep q = prep_at(B, b);
    if (q.action != GOME_DEL) continue;
    const uint32_t s = fc_hash_find(F, fc_key(F, hd.sym, q.oid), false);
    if (s == NIL) continue;
    const FcHash e = F.fc_hash[s];
    const uint32_t nadd = e.cnt;
    if (nadd > 1) { fc_decline(F, h, FC_BAD_Q7); continue; }  // a reused oid (Q7)
    const bool sale = q.side == GOME_SALE;
    FcDel d{};
    d.ct = NIL;
    uint32_t ixs = 0;
    const uint32_t loc = fc_old_lookup(D, hd.sym, q.oid, ixs);
    if (b != e.del_first) {  // the maker is gone by then (or its ADD comes later)
      if (nadd == 1 && loc != NIL) fc_decline(F, h, FC_BAD_Q7);  // the oid rests already: duplicate (Q7)
      continue;
    }
    if (nadd == 1) {
      if (loc != NIL) { fc_decline(F, h, FC_BAD_Q7); continue; }  // the oid rests already: duplicate (Q7)
      const Prep a = prep_at(B, e.add_pos);
      if (a.price != q.price) continue;                 // S:link:<request price> misses (Q3)
      const bool wrong = (a.side == GOME_SALE) != sale;  // wrong side (Q2)
      if (wrong && !q2_ok) { fc_decline(F, h, FC_BAD_Q2); continue; }
      if (a.vol == 0) atomicOr(&F.hdr[h].haz, HZ_ZDEL);  // a zero-volume maker's cancel (Q6): k_flow_stale_check
      d.kind = FC_NEW;
      d.tgt = e.add_pos;
      F.fc_rank[b] = a.side == GOME_SALE ? 1u : 0u;
      d.li = static_cast<uint32_t>(F.ord8[hd.obase + (e.add_pos - hd.beg)] >> 32) & lmask;
      if (wrong) {
        atomicAdd(&F.hdr[h].nwrong, 1u);
        atomicAdd(&LV[d.li].c_wrong, 1u);
      }
      F.fc_del[b] = d;
      F.fc_tg[e.add_pos] = b + 1;
      continue;
    }
    if (loc == NIL) continue;                                             // not resting
    if (D.chdr[loc / CH].price != q.price) continue;                     // Q3
    const Node nd = D.nodes[loc];
    if (nd.rem < 0) continue;
    const bool wrong = (nd.tx == GOME_SALE) != sale;  // Q2
    if (wrong && !q2_ok) { fc_decline(F, h, FC_BAD_Q2); continue; }
    if (nd.rem == 0) atomicOr(&F.hdr[h].haz, HZ_ZDEL);  // a zero-volume maker's cancel (Q6): k_flow_stale_check
    const uint32_t li = fc_level_of(LV, hd.nl, q.price);
    if (li == 0) { fc_decline(F, h, FC_BAD_LEVEL); continue; }
    if (wrong) {
      atomicAdd(&F.hdr[h].nwrong, 1u);
      atomicAdd(&LV[li].c_wrong, 1u);
    }
    d.kind = FC_OLD;
    d.tgt = loc;
    F.fc_rank[b] = nd.tx == GOME_SALE ? 1u : 0u;
    d.ixs = ixs;
    d.li = li;
    F.fc_del[b] = d;
    D.nodes[loc].pad = b + 1;  // marks the target for the walks (cleared when it is cancelled)
    atomicAdd(&LV[li].c_old, 1u);
  }
}

// ---- prep 4: old targets' FIFO ranks and arrival coordinates (one wave per level) -----------
__device__ __forceinline__ void fc_oldwalk_level(const Dev& D, const FlowArgs& F, uint32_t h, uint32_t q) {
  const FlowHdr& hd = F.hdr[h];
  FlowLvl* Lq = fl_lvls(F, h) + q;
  const uint32_t cold = uni(Lq->c_old);
  if (!cold) return;
  const uint32_t lane = lane_id();
  const unsigned long long g = hd.g;
  const uint32_t tail = uni(Lq->tail), tslot = uni(Lq->tslot);
  uint32_t c = uni(Lq->head), s0 = uni(Lq->hslot), seen = 0;
  int64_t E = 0;
  for (uint32_t guard = 0; c != NIL && seen < cold; ++guard) {
    if (guard > D.ch_cap) { if (lane == 0) atomicOr(&D.st->err, ERR_CORRUPT); return; }
    const uint32_t lim = (c == tail) ? tslot : CH;
    const bool inr = lane < CH && lane >= s0 && lane < lim;
    Node nd{};
    if (inr) nd = D.nodes[c * CH + lane];
    const bool live = inr && nd.rem >= 0;
    const int64_t x = live ? nd.rem : 0;
    const int64_t em = E + wave_incl_scan(x) - x;
    const bool mk = live && nd.pad != 0;
    const unsigned long long mm = __ballot(mk);
    if (mk) {
      FcDel* d = &F.fc_del[static_cast<uint32_t>(nd.pad) - 1u];
      const uint64_t end = static_cast<uint64_t>(em + nd.rem);
      if (end % g || static_cast<uint64_t>(nd.rem) % g) fc_decline(F, h, FC_BAD_UNIT);  // not in plan units
      d->rank = seen + __popcll(mm & lt_mask());
      d->oend = static_cast<uint32_t>(end / g);
      d->ov = static_cast<uint32_t>(static_cast<uint64_t>(nd.rem) / g);
    }
    seen += __popcll(mm);
    E += rl64(wave_incl_scan(x), 63);
    c = (c == tail) ? NIL : uni(D.chdr[c].next);
    s0 = 0;
  }
  if (seen != cold && lane == 0) fc_decline(F, h, FC_BAD_WALK);
}

__global__ __launch_bounds__(64) void k_fc_oldwalk_wide(Dev D, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y, q = blockIdx.x;
  if (h >= fl_hend(D, F) || !fc_lane(F, h) || q == 0 || q > F.hdr[h].nl) return;
  fc_oldwalk_level(D, F, h, q);
}

__global__ __launch_bounds__(1024) void k_fc_oldwalk_book(Dev D, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.x;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  for (uint32_t q = 1 + (threadIdx.x >> 6); q <= F.hdr[h].nl; q += blockDim.x / 64) fc_oldwalk_level(D, F, h, uni(q));
}

// ---- the DEL records' Q -----------------------------------------------------------------------
// A DEL of maker m (level k, side s) at segment position b removes r = clamp(depth_s,k - Q, 0,
// v_m) (gen_plan_asm.py, W32C; v_m = m's volume), where Q = the volume of the side-s makers that
// arrived at level k after m and before b and were not cancelled before b
// (tools/flow_cancel_model.py, plan_book_q, checks this against the oracle):
//   Q = VA(b) - END(m) - C,   VA(x) = volume of the segment's admitted side-s ADDs at level k
//                              before position x (the old makers: END(m) = oend - D0 for an old m,
//                              i.e. the old volume behind m counts);
//                              END(m) = VA(m) + v_m for a new m;
//                              C = volume of the level's side-s targets ranked behind m (arrived
//                              after it) whose DEL comes before b: they were untouched while m
//                              was live, so each removed exactly its v.
// Those targets are among the nb that arrived behind m before b (the DEL's window), so C is a
// loop over ranks rank+1 .. rank+nb of the level's DEL times (DT) and volumes (TV).

// Per level: its targets' count and their first entry of the book's DEL-time array (an exclusive
// scan over the book's levels; `tot` = 0 for threads that are not levels).  Every thread of the
// block calls it (threads k >= FL_CAP take no part).
__device__ __forceinline__ void fc_time_bases(FlowLvl* LV, uint32_t k, uint32_t tot) {
  __shared__ uint32_t wsum[FL_CAP / 64];
  const bool in = k < FL_CAP;
  const uint32_t inc = wave_incl_scan_u32(in ? tot : 0u), w = k >> 6;
  if (in && (k & 63u) == 63u) wsum[w] = inc;
  __syncthreads();
  if (in && k >= 1) {
    uint32_t base = inc - tot;
    for (uint32_t ww = 0; ww < w; ++ww) base += wsum[ww];
    LV[k].ttot = tot;
    LV[k].tbase = base;
  }
  __syncthreads();
}

constexpr uint32_t FC_KEYS = 2 * FL_CAP;     // (level, side) keys of the volume sums: level | SALE << 7
constexpr uint32_t FC_NB_MAX = 0xFFFFu;     // a longer DEL window declines the book (FC_BAD_RING)
constexpr uint32_t FC_MAX_V = 1u << 22;     // a target's volume (plan units) fits 22 bits of its DEL record
// so does a segment whose windows add up past FC_NBSUM_MUL per record (+ FC_NBSUM_ADD): the
// records' C loops stay a small multiple of the segment
constexpr uint32_t FC_NBSUM_MUL = 256, FC_NBSUM_ADD = 1u << 24;

// Record i of book h (segment position b = beg + i): an admitted ADD's (level, side) key and
// volume (plan units), from its W32 record; NIL key for anything else.
__device__ __forceinline__ uint32_t fc_add_key(const FlowArgs& F, const FlowHdr& hd, uint32_t i, uint32_t& v) {
  const unsigned long long r = F.ord8[hd.obase + i];
  const uint32_t hi = static_cast<uint32_t>(r >> 32), k = hi & 127u;
  v = static_cast<uint32_t>(r);
  return k ? (k | ((hi >> 31) << 7)) : NIL;
}

// Volume of the lanes of this wave before this one whose ADD key equals `q` (akey: this lane's
// ADD key or NIL).
__device__ __forceinline__ uint32_t fc_wave_vol_before(uint32_t akey, uint32_t v, uint32_t q) {
  const uint32_t lane = lane_id();
  uint32_t s = 0;
  for (uint32_t l = 0; l < 63; ++l) {
    const uint32_t kl = __shfl(akey, l), vl = __shfl(v, l);
    if (l < lane && kl == q) s += vl;
  }
  return s;
}

// The tile's per-wave ADD volumes per key -> exclusive offsets from base[key] (LDS wv[FL_TILE_W]
// [FC_KEYS], every thread of a FL_TILE block calls it); base[key] advances by the tile's total
// when `advance`.
__device__ __forceinline__ void fc_tile_vol(uint32_t (*wv)[FC_KEYS], uint32_t* base, uint32_t akey, uint32_t v,
                                            bool advance) {
  const uint32_t tid = threadIdx.x, w = tid >> 6;
  for (uint32_t x = tid; x < FL_TILE_W * FC_KEYS; x += blockDim.x) wv[x / FC_KEYS][x % FC_KEYS] = 0;
  __syncthreads();
  if (akey != NIL) atomicAdd(&wv[w][akey], v);
  __syncthreads();
  for (uint32_t key = tid; key < FC_KEYS; key += blockDim.x) {
    uint32_t r = base[key];
    for (uint32_t ww = 0; ww < FL_TILE_W; ++ww) {
      const uint32_t c = wv[ww][key];
      wv[ww][key] = r;
      r += c;
    }
    if (advance) base[key] = r;
  }
  __syncthreads();
}

// A targeted ADD's arrival end (VA + v) and volume go to its DEL's record; a DEL gets VA.
__device__ __forceinline__ void fc_put_va(const FlowArgs& F, uint32_t b, bool tgt_add, bool del, uint32_t va,
                                          uint32_t v) {
  if (tgt_add) {
    FcDel* d = &F.fc_del[F.fc_tg[b] - 1u];
    d->oend = va + v;
    d->ov = v;
  }
  if (del) F.fc_del[b].va = va;
}

// C of the DEL at b: the volume of its window's side-s targets cancelled before it.
__device__ __forceinline__ uint32_t fc_del_c(const FlowArgs& F, const FlowHdr& hd, const FlowLvl* LV, uint32_t b,
                                             const FcDel& d, bool sale, uint32_t x0 = 1, uint32_t dx = 1) {
  const uint32_t* dt = F.fc_dt + hd.beg + LV[d.li].tbase;
  const uint32_t* tv = F.fc_tv + hd.beg + LV[d.li].tbase;
  uint32_t c = 0;
  for (uint32_t x = d.rank + x0; x <= d.rank + d.nb; x += dx) {
    const uint32_t t = tv[x];
    if ((t >> 31) == (sale ? 1u : 0u) && dt[x] < b) c += t & 0x7FFFFFFFu;
  }
  return c;
}

// Q of the DEL at b (see above, C given) and its W32C record.
__device__ __forceinline__ unsigned long long fc_del_rec_c(const FlowHdr& hd, const FlowLvl* LV, const FcDel& d,
                                                           bool sale, uint32_t c) {
  const uint32_t k = d.li;
  const uint32_t d0 = static_cast<uint32_t>(static_cast<unsigned long long>(LV[k].d0) / hd.g);
  const uint32_t q = (d.kind == FC_OLD ? d0 - d.oend : 0u - d.oend) + d.va - c;
  const uint32_t hi = (hd.ok == FL_OK_DEEP ? k | (d.ov << 14) : k | (d.ov << 7)) | (1u << 30) | (sale ? 0x80000000u : 0u);
  return (static_cast<unsigned long long>(hi) << 32) | q;
}

__device__ __forceinline__ unsigned long long fc_del_rec(const FlowArgs& F, const FlowHdr& hd, const FlowLvl* LV,
                                                         uint32_t b, const FcDel& d, bool sale) {
  return fc_del_rec_c(hd, LV, d, sale, fc_del_c(F, hd, LV, b, d, sale));
}

// A DEL's window and its target's DEL time / volume by rank (both prep paths).
__device__ __forceinline__ uint32_t fc_window(const FlowArgs& F, const FlowHdr& hd, const FlowLvl* LV, uint32_t b,
                                              const FcDel& d, uint32_t rk, uint32_t arrived, bool sale) {
  const uint32_t nb = arrived - rk - 1u;
  F.fc_del[b].rank = rk;
  F.fc_del[b].nb = nb;
  const uint32_t x = hd.beg + LV[d.li].tbase + rk;
  F.fc_dt[x] = b;
  F.fc_tv[x] = d.ov | (sale ? 0x80000000u : 0u);
  return nb;
}

// ---- prep 5: ranks, windows, Q and the W32C DEL records (one block per book) ----------------
constexpr uint32_t FC_PASS_T = FL_TILE, FC_PASS_W = FC_PASS_T / 64;

__global__ __launch_bounds__(FC_PASS_T) void k_fc_pass(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ uint32_t cnt[FL_CAP], wc[FC_PASS_W][FL_CAP], cvol[FC_KEYS], wv[FC_PASS_W][FC_KEYS];
  __shared__ uint32_t bad_s, mw_s, sum_s;
  const uint32_t h = F.h0 + blockIdx.x, tid = threadIdx.x, w = tid >> 6;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  FlowLvl* LV = F.lvl + h * FL_CAP;
  const uint32_t n = hd.end - hd.beg;
  if (tid < FL_CAP) cnt[tid] = 0;
  for (uint32_t x = tid; x < FC_KEYS; x += FC_PASS_T) cvol[x] = 0;
  if (tid == 0) { bad_s = 0; mw_s = 0; sum_s = 0; }
  for (uint32_t x = tid; x < FC_PASS_W * FL_CAP; x += FC_PASS_T) wc[x / FL_CAP][x % FL_CAP] = 0;
  __syncthreads();
  const unsigned long long ltm = lt_mask();
  // in segment order, tile by tile: a targeted ADD's rank = old targets of its level + targeted
  // ADDs before it; a DEL's window = targets of the level that arrived before it - its target's
  // rank - 1 (stable per-level counting across the waves of a tile); the (level, side) ADD
  // volumes before each targeted ADD and DEL
  for (uint32_t t0 = 0; t0 < n; t0 += FC_PASS_T) {
    const uint32_t i = t0 + tid;
    const uint32_t b = hd.beg + i;
    bool isa = false, isd = false, sale = false;
    uint32_t k = 0, v = 0, akey = NIL, qkey = NIL;
    FcDel d{};
    if (i < n) {
      akey = fc_add_key(F, hd, i, v);
      if (F.fc_tg[b]) {
        isa = true;
        k = akey & 127u;
        qkey = akey;
      } else if (akey == NIL && prep_at(B, b).action == GOME_DEL) {
        d = F.fc_del[b];
        if (d.kind != FC_NONE) {
          isd = true;
          k = d.li;
          sale = fc_del_sale(F, b);
          qkey = k | (sale ? 128u : 0u);
        }
      }
    }
    fc_tile_vol(wv, cvol, akey, v, true);
    const uint32_t pre = fc_wave_vol_before(akey, v, qkey);
    if (isa || isd) fc_put_va(F, b, isa, isd, wv[w][qkey] + pre, v);
    unsigned long long same = __ballot(isa);
#pragma unroll
    for (uint32_t bit = 0; bit < 7; ++bit) {
      const unsigned long long bb = __ballot((k >> bit) & 1u);
      same &= ((k >> bit) & 1u) ? bb : ~bb;
    }
    // same: the wave's targeted ADDs at level k (valid for every lane with that k)
    const uint32_t before_w = __popcll(same & ltm);
    if (isa && before_w == 0) wc[w][k] = __popcll(same);
    __syncthreads();
    if (tid < FL_CAP) {  // waves' counts -> exclusive offsets (from the tile's running count)
      uint32_t r = cnt[tid];
      for (uint32_t ww = 0; ww < FC_PASS_W; ++ww) {
        const uint32_t c = wc[ww][tid];
        wc[ww][tid] = r;
        r += c;
      }
      cnt[tid] = r;
    }
    __syncthreads();
    // wc[w][k] now = targeted ADDs at level k before wave w's first lane (all earlier tiles too)
    const uint32_t before = (isa || isd) ? wc[w][k] + before_w : 0u;
    if (isa) F.fc_rank[b] = LV[k].c_old + before;
    __syncthreads();  // (a DEL may target an ADD of the same tile)
    if (isd) {  // (arrived before it, kept in nb until the level bases are known)
      const uint32_t rk = d.kind == FC_NEW ? F.fc_rank[d.tgt] : d.rank;
      F.fc_del[b].rank = rk;
      F.fc_del[b].nb = LV[k].c_old + before;
    }
    for (uint32_t x = tid; x < FC_PASS_W * FL_CAP; x += FC_PASS_T) wc[x / FL_CAP][x % FL_CAP] = 0;
    __syncthreads();
  }
  // per level the targets' DEL times and volumes by rank
  fc_time_bases(LV, tid, (tid >= 1 && tid <= hd.nl) ? LV[tid].c_old + cnt[tid] : 0u);
  uint32_t nbsum = 0;
  for (uint32_t i = tid; i < n; i += FC_PASS_T) {
    const uint32_t b = hd.beg + i;
    if (prep_at(B, b).action != GOME_DEL) continue;
    const FcDel d = F.fc_del[b];
    if (d.kind == FC_NONE) continue;
    const uint32_t nb = fc_window(F, hd, LV, b, d, d.rank, d.nb, fc_del_sale(F, b));
    nbsum += nb;
    atomicMax(&mw_s, nb + 1u);
    if (nb >= FC_NB_MAX) atomicOr(&bad_s, FC_BAD_RING);
    if (d.ov >= FC_MAX_V) atomicOr(&bad_s, FC_BAD_UNIT);
  }
  if (nbsum) atomicAdd(&sum_s, nbsum);
  __syncthreads();
  if (tid == 0) {
    F.hdr[h].ncancel = mw_s;
    F.hdr[h].nbsum = sum_s;
    if (sum_s > FC_NBSUM_MUL * n + FC_NBSUM_ADD) bad_s |= FC_BAD_RING;
  }
  __syncthreads();
  if (bad_s) {
    if (tid == 0) fc_decline(F, h, bad_s);
    return;
  }
  for (uint32_t i = tid; i < n; i += FC_PASS_T) {
    const uint32_t b = hd.beg + i;
    if (prep_at(B, b).action != GOME_DEL) continue;
    const FcDel d = F.fc_del[b];
    if (d.kind != FC_NONE) F.ord8[hd.obase + i] = fc_del_rec(F, hd, LV, b, d, fc_del_sale(F, b));
  }
}

// ---- prep 5, tile-parallel (the head books, whose segments hold up to ~10^6 records) --------
// The same quantities as k_fc_pass, computed as a stable counting pass over 1024-record tiles:
// per tile the targeted ADDs of each level and the ADD volume of each (level, side) key (F.tcnt
// / F.tvol, free before the plan), exclusive scans over the tiles, then every targeted ADD's rank
// and every DEL's count of targets that arrived before it with the volumes before both; the
// windows (which need the ranks of targets in other tiles) and the DEL records follow as
// separate launches.
__device__ __forceinline__ bool fc_targeted_add(const FlowArgs& F, const FlowHdr& hd, uint32_t i, uint32_t& k) {
  if (!F.fc_tg[hd.beg + i]) return false;
  k = static_cast<uint32_t>(F.ord8[hd.obase + i] >> 32) & 127u;
  return true;
}

__global__ __launch_bounds__(FL_TILE) void k_fc_pcnt(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ uint32_t wc[FL_TILE_W][FL_CAP], tv[FC_KEYS];
  const uint32_t h = F.h0 + blockIdx.y, tid = threadIdx.x, w = tid >> 6;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  const uint32_t n = hd.end - hd.beg, ntile = (n + FL_TILE - 1) / FL_TILE;
  for (uint32_t tl = blockIdx.x; tl < ntile; tl += gridDim.x) {
    for (uint32_t i = tid; i < FL_TILE_W * FL_CAP; i += FL_TILE) wc[i / FL_CAP][i % FL_CAP] = 0;
    for (uint32_t i = tid; i < FC_KEYS; i += FL_TILE) tv[i] = 0;
    __syncthreads();
    const uint32_t i = tl * FL_TILE + tid;
    uint32_t k = 0, cnt, v = 0, akey = NIL;
    const bool isa = i < n && fc_targeted_add(F, hd, i, k);
    if (i < n) akey = fc_add_key(F, hd, i, v);
    if (akey != NIL) atomicAdd(&tv[akey], v);
    const uint32_t rank = fl_tile_rank(k, isa, cnt);
    if (isa && rank == 0) wc[w][k] = cnt;
    __syncthreads();
    if (tid < FL_CAP) {
      uint32_t c = 0;
      for (uint32_t ww = 0; ww < FL_TILE_W; ++ww) c += wc[ww][tid];
      F.tcnt[(static_cast<size_t>(h) * F.maxt + tl) * FL_CAP + tid] = c;
    }
    for (uint32_t key = tid; key < FC_KEYS; key += FL_TILE)
      F.tvol[(static_cast<size_t>(h) * F.maxt + tl) * FC_KEYS + key] = tv[key];
    __syncthreads();
  }
}

// Per book: tile offsets per level from its old targets, per key from 0 (in place); the level
// bases of the DEL-time arrays.  FC_PSCAN_G groups of FL_CAP threads take a contiguous range of the
// tiles each: their sums, the groups' prefixes, then the offsets written.  (One group walked the
// hottest book's ~340 tiles eight at a time: 43 dependent round trips, 59 us on config 4's critical
// path, gpurun_out/prof_r06ac_config4.)
constexpr uint32_t FC_PSCAN_G = 8;
__global__ __launch_bounds__(FL_CAP * FC_PSCAN_G) void k_fc_pscan(Dev D, FlowArgs F) {
  __shared__ uint32_t sv[FC_PSCAN_G][FL_CAP], sb[FC_PSCAN_G][FL_CAP], ss[FC_PSCAN_G][FL_CAP];
  const uint32_t h = F.h0 + blockIdx.x, k = threadIdx.x % FL_CAP, grp = threadIdx.x / FL_CAP;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  const FlowHdr& hd = F.hdr[h];
  FlowLvl* LV = F.lvl + h * FL_CAP;
  const uint32_t ntile = (hd.end - hd.beg + FL_TILE - 1) / FL_TILE;
  const uint32_t per = (ntile + FC_PSCAN_G - 1) / FC_PSCAN_G;
  const uint32_t t_beg = min(ntile, grp * per), t_end = min(ntile, t_beg + per);
  const bool lv = k >= 1 && k <= hd.nl;
  uint32_t* tc = F.tcnt + static_cast<size_t>(h) * F.maxt * FL_CAP;
  uint32_t* tvv = F.tvol + static_cast<size_t>(h) * F.maxt * FC_KEYS;
  constexpr uint32_t U = 8;  // (eight tiles' loads in flight together)
  uint32_t a = 0, ab = 0, as = 0;
  for (uint32_t t0 = t_beg; t0 < t_end; t0 += U) {
    uint32_t v[U], vb[U], vs[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t tl = t0 + u;
      const bool in = tl < t_end;
      v[u] = in ? tc[tl * FL_CAP + k] : 0u;
      vb[u] = in ? tvv[tl * FC_KEYS + k] : 0u;
      vs[u] = in ? tvv[tl * FC_KEYS + FL_CAP + k] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      a += v[u];
      ab += vb[u];
      as += vs[u];
    }
  }
  sv[grp][k] = a;
  sb[grp][k] = ab;
  ss[grp][k] = as;
  __syncthreads();
  uint32_t run = lv ? LV[k].c_old : 0u, rb = 0, rs = 0, tot = run;
  for (uint32_t g = 0; g < FC_PSCAN_G; ++g) {
    const uint32_t x = sv[g][k];
    tot += x;
    if (g < grp) {
      run += x;
      rb += sb[g][k];
      rs += ss[g][k];
    }
  }
  for (uint32_t t0 = t_beg; t0 < t_end; t0 += U) {
    uint32_t v[U], vb[U], vs[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t tl = t0 + u;
      if (tl < t_end) {
        v[u] = tc[tl * FL_CAP + k];
        vb[u] = tvv[tl * FC_KEYS + k];
        vs[u] = tvv[tl * FC_KEYS + FL_CAP + k];
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t tl = t0 + u;
      if (tl >= t_end) break;
      tc[tl * FL_CAP + k] = run;
      run += v[u];
      tvv[tl * FC_KEYS + k] = rb;
      tvv[tl * FC_KEYS + FL_CAP + k] = rs;
      rb += vb[u];
      rs += vs[u];
    }
  }
  fc_time_bases(LV, threadIdx.x, lv && grp == 0 ? tot : 0u);  // (threads >= FL_CAP: nothing)
}

// Targeted ADDs' ranks; a DEL's count of its level's targets that arrived before it (in nb); the
// (level, side) volumes before both.
__global__ __launch_bounds__(FL_TILE) void k_fc_prank(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ uint32_t wc[FL_TILE_W][FL_CAP], wv[FL_TILE_W][FC_KEYS], vb[FC_KEYS];
  const uint32_t h = F.h0 + blockIdx.y, tid = threadIdx.x, w = tid >> 6;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  const uint32_t n = hd.end - hd.beg, ntile = (n + FL_TILE - 1) / FL_TILE;
  const uint32_t* tc = F.tcnt + static_cast<size_t>(h) * F.maxt * FL_CAP;
  const uint32_t* tvv = F.tvol + static_cast<size_t>(h) * F.maxt * FC_KEYS;
  for (uint32_t tl = blockIdx.x; tl < ntile; tl += gridDim.x) {
    for (uint32_t i = tid; i < FL_TILE_W * FL_CAP; i += FL_TILE) wc[i / FL_CAP][i % FL_CAP] = 0;
    for (uint32_t i = tid; i < FC_KEYS; i += FL_TILE) vb[i] = tvv[tl * FC_KEYS + i];
    __syncthreads();
    const uint32_t i = tl * FL_TILE + tid, b = hd.beg + i;
    uint32_t k = 0, v = 0, akey = NIL, qkey = NIL;
    bool isa = false, isd = false;
    if (i < n) {
      akey = fc_add_key(F, hd, i, v);
      isa = fc_targeted_add(F, hd, i, k);
      if (isa) qkey = akey;
      if (!isa && akey == NIL && prep_at(B, b).action == GOME_DEL) {
        const FcDel d = F.fc_del[b];
        if (d.kind != FC_NONE) {
          isd = true;
          k = d.li;
          qkey = k | (fc_del_sale(F, b) ? 128u : 0u);
        }
      }
    }
    fc_tile_vol(wv, vb, akey, v, false);
    const uint32_t pre = fc_wave_vol_before(akey, v, qkey);
    if (isa || isd) fc_put_va(F, b, isa, isd, wv[w][qkey] + pre, v);
    // ballot of the wave's targeted ADDs at this lane's level (DEL lanes take part in the
    // level bits only)
    unsigned long long same = __ballot(isa);
#pragma unroll
    for (uint32_t bit = 0; bit < 7; ++bit) {
      const unsigned long long bb = __ballot((k >> bit) & 1u);
      same &= ((k >> bit) & 1u) ? bb : ~bb;
    }
    const uint32_t before_w = __popcll(same & lt_mask());
    if (isa && before_w == 0) wc[w][k] = __popcll(same);
    __syncthreads();
    if (tid < FL_CAP) {  // waves' counts -> offsets from the tile's offset of the level
      uint32_t r = tc[tl * FL_CAP + tid];
      for (uint32_t ww = 0; ww < FL_TILE_W; ++ww) {
        const uint32_t c = wc[ww][tid];
        wc[ww][tid] = r;
        r += c;
      }
    }
    __syncthreads();
    if (isa) F.fc_rank[b] = wc[w][k] + before_w;
    if (isd) F.fc_del[b].nb = wc[w][k] + before_w;  // (arrived; k_fc_pwin turns it into the window)
    __syncthreads();
  }
}

// Windows: nb = arrived - rank of the target - 1; DEL times and volumes by rank.
// only_deep: the deep books alone (the tail's lane books take k_fc_pass)
__global__ __launch_bounds__(256) void k_fc_pwin(Dev D, BatchArgs B, FlowArgs F, uint32_t only_deep) {
  __shared__ uint32_t sum_s, mw_s;
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F) || !fc_book(F, h) || (only_deep && F.hdr[h].ok != FL_OK_DEEP)) return;
  const FlowHdr hd = F.hdr[h];
  FlowLvl* LV = fl_lvls(F, h);
  const uint32_t vmax = hd.ok == FL_OK_DEEP ? FD_MAX_V : FC_MAX_V;
  if (threadIdx.x == 0) { sum_s = 0; mw_s = 0; }
  __syncthreads();
  uint32_t b0, b1, bad = 0, nbsum = 0;
  fc_slice(hd, blockIdx.x, gridDim.x, b0, b1);
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
    if (prep_at(B, b).action != GOME_DEL) continue;
    const FcDel d = F.fc_del[b];
    if (d.kind == FC_NONE) continue;
    const uint32_t rk = d.kind == FC_NEW ? F.fc_rank[d.tgt] : d.rank;
    const uint32_t nb = fc_window(F, hd, LV, b, d, rk, d.nb, fc_del_sale(F, b));
    nbsum += nb;
    atomicMax(&mw_s, nb + 1u);
    if (nb >= FC_NB_MAX) bad |= FC_BAD_RING;
    if (d.ov >= vmax) bad |= FC_BAD_UNIT;
  }
  if (nbsum) atomicAdd(&sum_s, nbsum);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (sum_s) atomicAdd(&F.hdr[h].nbsum, sum_s);
    if (mw_s) atomicMax(&F.hdr[h].ncancel, mw_s);
  }
  if (bad) fc_decline(F, h, bad);
}

// The W32C DEL records (Q), tile-parallel; a book whose windows sum past the budget is declined.
__global__ __launch_bounds__(256) void k_fc_precs(Dev D, BatchArgs B, FlowArgs F, uint32_t only_deep) {
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F) || !fc_book(F, h) || (only_deep && F.hdr[h].ok != FL_OK_DEEP)) return;
  const FlowHdr hd = F.hdr[h];
  const uint32_t n = hd.end - hd.beg;
  if (hd.nbsum > FC_NBSUM_MUL * n + FC_NBSUM_ADD) {
    if (blockIdx.x == 0 && threadIdx.x == 0) fc_decline(F, h, FC_BAD_RING);
    return;
  }
  const FlowLvl* LV = fl_lvls(F, h);
  uint32_t b0, b1;
  fc_slice(hd, blockIdx.x, gridDim.x, b0, b1);
  const uint32_t lane = lane_id();
  // a DEL with a short window loops over it alone; the long ones (the hottest books' busiest
  // levels hold thousands of targets) go to a list that k_fc_precs_long deals out one per wave:
  // as one wave's serial loop here, a run of consecutive long-window DELs (e.g. 453 wrong-side
  // cancels of one level's makers, one after another) took 11.4 ms
  uint32_t* longl = fc_long_list(F, hd);
  for (uint32_t bw = b0 + (threadIdx.x & ~63u); bw < b1; bw += blockDim.x) {
    const uint32_t b = bw + lane;
    FcDel d{};
    bool isd = false, sale = false;
    if (b < b1) {
      const Prep q = prep_at(B, b);
      if (q.action == GOME_DEL) {
        d = F.fc_del[b];
        isd = d.kind != FC_NONE;
        sale = isd && fc_del_sale(F, b);
      }
    }
    const bool longw = isd && d.nb > 32;
    if (isd && !longw) F.ord8[hd.obase + (b - hd.beg)] = fc_del_rec(F, hd, LV, b, d, sale);
    if (longw) longl[atomicAdd(&F.hdr[h].nlong, 1u)] = b;
  }
}

// The long-window DELs of k_fc_precs, one wave each (lanes stride the window).
__global__ __launch_bounds__(256) void k_fc_precs_long(Dev D, BatchArgs B, FlowArgs F, uint32_t only_deep) {
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F) || !fc_book(F, h) || (only_deep && F.hdr[h].ok != FL_OK_DEEP)) return;
  const FlowHdr hd = F.hdr[h];
  if (hd.nbsum > FC_NBSUM_MUL * (hd.end - hd.beg) + FC_NBSUM_ADD) return;  // (declined by k_fc_precs)
  const FlowLvl* LV = fl_lvls(F, h);
  const uint32_t* longl = fc_long_list(F, hd);
  const uint32_t lane = lane_id();
  const uint32_t W = gridDim.x * (blockDim.x >> 6);
  for (uint32_t i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); i < hd.nlong; i += W) {
    const uint32_t b = uni(longl[i]);
    const FcDel d = F.fc_del[b];
    const bool sale = fc_del_sale(F, b);
    uint32_t c = fc_del_c(F, hd, LV, b, d, sale, 1u + lane, 64u);
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if (lane == 0) F.ord8[hd.obase + (b - hd.beg)] = fc_del_rec_c(hd, LV, d, sale, c);
  }
}

// ---- prep 6: books declined by the cancel prep go to the legacy hot / cold kernels: drop
// their old targets' marks and route them there (FlowHdr::ok = 0)
__global__ __launch_bounds__(256) void k_fc_unmark(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F) || !fc_dels(F, h) || !F.hdr[h].fc_bad) return;
  const FlowHdr hd = F.hdr[h];
  uint32_t b0, b1;
  fc_slice(hd, blockIdx.x, gridDim.x, b0, b1);
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
    if (prep_at(B, b).action != GOME_DEL) continue;
    const FcDel d = F.fc_del[b];
    if (d.kind == FC_OLD) D.nodes[d.tgt].pad = 0;
  }
}

__global__ void k_fc_route(Dev D, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.x * blockDim.x + threadIdx.x;
  if (h < fl_hend(D, F) && fc_dels(F, h) && F.hdr[h].fc_bad) {
    F.hdr[h].ok = 0;  // (a declined deep book's price set was cleared by k_fd_decline)
    F.hdr[h].deep = 0;
  }
}

// ---- after the plan and the level sort: stale members of the head books with DELs (Q2) ------
// A level's side-set membership follows its last state-setting event in time order: a REST of side
// s makes it a member of s (ZADD, engine.go:80); a fill or a cancel that leaves depth 0 ZREMs the
// maker's set (DeletePoolMatchOrder / DeletePoolDepth, nodepool.go:76-83), except that a wrong-side
// cancel ZREMs the request's set, which leaves the level a stale member of s (no FIFO, depth 0).
// Takers pass a stale member by (MatchOrder returns at an empty FIFO) and the plan, seeing depth 0,
// passes it too; a same-side REST heals it.  A REST on the other side while the level is stale would
// put the price in both sets: hazard, the book goes to the legacy kernel (k_flow_stale_check).  One
// block per (book, level) with a stale member at batch start or a wrong-side cancel, the run in
// time order with block scans: the depth after each touch, then the last state before each
// (codes ST_*, max-scan of (index, code)); FlowLvl::mfin gets the level's stale membership after
// the batch (fc_write_level keeps it).
enum : uint32_t { ST_BUY = 1, ST_SALE = 2, ST_NONE = 3, ST_STALE_BUY = 4, ST_STALE_SALE = 5 };

__global__ __launch_bounds__(64) void k_fc_stale_level(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y, q = blockIdx.x, lane = lane_id();
  if (h >= fl_hend(D, F)) return;
  FlowHdr* hd = &F.hdr[h];
  if (hd->ok != FL_OK_CANCEL || hd->fc_bad || (hd->nstale == 0 && hd->nwrong == 0) || q == 0 || q > hd->nl) return;
  FlowLvl* Lq = F.lvl + h * FL_CAP + q;
  const bool st0 = fl_stale0(*Lq);
  if (!st0 && Lq->c_wrong == 0) return;
  const uint32_t cnt = Lq->cnt, beg = hd->beg;
  const SEnt* R = F.srt + FL_TOUCH_MUL * beg + Lq->base;
  uint32_t state = st0 ? (Lq->mem0 == M_SALE ? ST_STALE_SALE : ST_STALE_BUY)
                       : Lq->d0 > 0 ? (Lq->mem0 == M_SALE ? ST_SALE : ST_BUY) : ST_NONE;
  int64_t carry = -1;      // (index + 1) << 3 | code of the last state-setting touch of earlier chunks
  int64_t run = Lq->d0;    // the level's depth before the chunk
  bool haz = false;
  for (uint32_t c0 = 0; c0 < cnt; c0 += 64) {
    const uint32_t i = c0 + lane;
    const bool valid = i < cnt;
    SEnt e{};
    if (valid) e = R[i];
    const bool isr = valid && e.kind == TK_REST, isc = valid && e.kind == TK_CONS, isx = valid && e.kind == TK_CANC;
    const int64_t delta = isr ? e.amt : (isc || isx) ? -e.amt : 0;
    int64_t tot;
    const int64_t after = run + fl_wave_excl(delta, &tot) + delta;
    bool rsale = false;
    uint32_t code = 0;
    if (isr) {
      rsale = prep_at(B, beg + e.j).side == GOME_SALE;
      code = rsale ? ST_SALE : ST_BUY;
    } else if ((isc || isx) && e.amt > 0 && after == 0) {
      code = ST_NONE;
      if (isx) {
        const bool msale = fc_del_sale(F, beg + e.j);
        if ((prep_at(B, beg + e.j).side == GOME_SALE) != msale) code = msale ? ST_STALE_SALE : ST_STALE_BUY;
      }
    }
    int64_t mtot;
    const int64_t key = code ? (static_cast<int64_t>(i + 1) << 3) | code : -1;
    const int64_t prev_key = max(carry, fl_wave_max_excl(key, &mtot));
    const uint32_t prev = prev_key >= 0 ? static_cast<uint32_t>(prev_key & 7) : state;
    if (isr && (prev == (rsale ? ST_STALE_BUY : ST_STALE_SALE))) haz = true;  // the other side's stale price
    carry = max(carry, mtot);
    run += tot;
  }
  if (__ballot(haz) && lane == 0) atomicOr(&hd->haz, HZ_STALE);
  if (lane == 0) {
    const uint32_t fin = carry >= 0 ? static_cast<uint32_t>(carry & 7) : state;
    Lq->mfin = fin == ST_STALE_BUY ? M_BUY : fin == ST_STALE_SALE ? M_SALE : 0u;
  }
}

// A head book with DELs handed to the legacy kernel after its plan (k_flow_stale_check): its old
// targets' marks go (as k_fc_unmark's for a declined book).
__global__ __launch_bounds__(256) void k_fc_unmark_bailed(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y;
  if (h >= fl_hend(D, F)) return;
  const FlowHdr hd = F.hdr[h];
  if (!hd.bail || !hd.ndel) return;
  uint32_t b0, b1;
  fc_slice(hd, blockIdx.x, gridDim.x, b0, b1);
  for (uint32_t b = b0 + threadIdx.x; b < b1; b += blockDim.x) {
    if (prep_at(B, b).action != GOME_DEL) continue;
    const FcDel d = F.fc_del[b];
    if (d.kind == FC_OLD) D.nodes[d.tgt].pad = 0;
  }
}

// ============================================================== reconstruction
// Makers of a cancel book's level in FIFO order: the gathered old ones IG[0, ig_n) (IgEnt: e =
// start in consumption space, v, oid, uuid, tx, pad = touch of its cancel or NIL), then the new
// ones RS[0, nrest) (RsEnt: e = start, v = volume rested, j = order, t = touch of the rest,
// pad0 = touch of its cancel or NIL).  Consumption space: a maker spans the volume consumed from
// it — all of it, or what was consumed before its cancel — so consecutive makers abut and
// a maker's length is the next one's start minus its own.
struct FcLvlView {
  const IgEnt* IG;
  const RsEnt* RS;
  uint32_t ig_n, nrest, ig_all;
  int64_t base_new;  // start of the new makers (old live volume minus its cancelled part)
  int64_t qend;      // end of the last new maker
};

__device__ __forceinline__ FcLvlView fc_view(const FlowArgs& F, uint32_t h, const FlowLvl& Lq) {
  FcLvlView V;
  V.IG = F.ig + Lq.ig_base;
  V.RS = F.rs + FL_TOUCH_MUL * F.hdr[h].beg + Lq.base;
  V.ig_n = Lq.ig_n;
  V.nrest = Lq.nrest;
  V.ig_all = Lq.ig_all;
  V.base_new = Lq.d0 - static_cast<int64_t>(static_cast<uint64_t>(Lq.ocan) * F.hdr[h].g);
  V.qend = static_cast<int64_t>((static_cast<uint64_t>(Lq.pad1) << 32) | Lq.pad0);
  return V;
}

__device__ __forceinline__ int64_t fc_start(const FcLvlView& V, uint32_t m) {
  return m < V.ig_n ? V.IG[m].e : V.RS[m - V.ig_n].e;
}
__device__ __forceinline__ int64_t fc_len(const FcLvlView& V, uint32_t m) {
  if (m + 1 < V.ig_n) return V.IG[m + 1].e - V.IG[m].e;
  // the last gathered old maker: the new makers follow it, or (not all gathered) it is an
  // untargeted one, never cancelled
  if (m + 1 == V.ig_n) return V.ig_all ? V.base_new - V.IG[m].e : V.IG[m].v;
  if (m + 1 < V.ig_n + V.nrest) return V.RS[m + 1 - V.ig_n].e - V.RS[m - V.ig_n].e;
  return V.qend - V.RS[m - V.ig_n].e;
}
__device__ __forceinline__ int64_t fc_vol(const FcLvlView& V, uint32_t m) {
  return m < V.ig_n ? V.IG[m].v : V.RS[m - V.ig_n].v;
}
__device__ __forceinline__ uint32_t fc_ct(const FcLvlView& V, uint32_t m) {
  return m < V.ig_n ? V.IG[m].pad : V.RS[m - V.ig_n].pad0;
}
// The maker spanning consumption point x: the last whose start <= x (a zero-length maker shares
// its successor's start, so the search lands on the one with volume there).
__device__ __forceinline__ uint32_t fc_find(const FcLvlView& V, int64_t x) {
  if (x < V.base_new) {
    uint32_t lo = 0, hi = V.ig_n;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (V.IG[mid].e <= x) lo = mid; else hi = mid;
    }
    return lo;
  }
  uint32_t lo = 0, hi = V.nrest;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (V.RS[mid].e <= x) lo = mid; else hi = mid;
  }
  return V.ig_n + lo;
}

#ifdef GOME_PROBE_LEVEL
// (tuning builds: the level passes' time split, summed over a batch; k_ctr_fold prints and clears)
__device__ unsigned long long g_probe[32];
#define GOME_PROBE_T(k, t0) do { if (threadIdx.x == 0) atomicAdd(&g_probe[k], wall_clock64() - (t0)); } while (0)
#else
#define GOME_PROBE_T(k, t0) do { } while (0)
#endif

// ---- k_fc_level: one wave per (book, level) ----------------------------------------------
__device__ __forceinline__ void fc_level_one(const Dev& D, const FlowArgs& F, uint32_t h, uint32_t q) {
  const FlowHdr* hd = &F.hdr[h];
  const uint32_t lane = lane_id();
  const unsigned long long ltm = lt_mask();
  FlowLvl* Lq = fl_lvls(F, h) + q;
  const uint32_t beg = uni(hd->beg);
  const uint32_t L = FL_TOUCH_MUL * beg;
  const unsigned long long g = static_cast<unsigned long long>(uni64(static_cast<int64_t>(hd->g)));
  const uint32_t base = uni(Lq->base), cnt = uni(Lq->cnt);
  const int64_t d0 = uni64(Lq->d0);
  SEnt* R = F.srt + L + base;
  RsEnt* RS = F.rs + L + base;
#ifdef GOME_PROBE_LEVEL  // (tuning builds, tools/build_variant.py: slow levels on stdout)
  const uint64_t pt0 = wall_clock64();
  uint32_t pwalk = 0;
#endif
  // 1. each cancel -> its DEL's record (r, touch); the consumption cursor before each consume
  int64_t cc = 0, ocan = 0;
  uint32_t nr = 0, ncan_old = 0, ncons = 0;
  for (uint32_t c0 = 0; c0 < cnt; c0 += 64) {
    const uint32_t i = c0 + lane;
    const bool valid = i < cnt;
    SEnt e{};
    if (valid) e = R[i];
    const bool isc = valid && e.kind == TK_CONS, isx = valid && e.kind == TK_CANC;
    if (isx) {
      FcDel* d = &F.fc_del[beg + e.j];
      d->r = e.amt;
      d->ct = e.t;
      if (d->kind == FC_OLD) { ocan += e.amt; ncan_old++; }
    }
    const int64_t ac = isc ? e.amt : 0;
    const int64_t ic = wave_incl_scan(ac);
    if (isc) R[i].coord = cc + ic - ac;
    cc += rl64(ic, 63);
    nr += __popcll(__ballot(valid && e.kind == TK_REST));
    ncons += __popcll(__ballot(isc));
  }
  for (int off = 32; off > 0; off >>= 1) {
    ocan += __shfl_xor(ocan, off);
    ncan_old += __shfl_xor(ncan_old, off);
  }
  __threadfence();  // the DEL records are read back below (by other lanes)
  const int64_t cfin = cc;
  const int64_t base_new = d0 - ocan;
  // (a level that may hold zero-volume makers: the level-end continuation, fl_cont)
  const bool zl = Lq->z0 || hd->nzero;
  const bool lcont = zl && cfin > 0 && fl_run_cont(F, L, uni(hd->ntouch), R, cnt, true);
  // 2. the new makers in FIFO (rest) order, their consumption-space starts and cancels
  int64_t acc = base_new;
  uint32_t k = 0;
  for (uint32_t c0 = 0; c0 < cnt; c0 += 64) {
    const uint32_t i = c0 + lane;
    const bool valid = i < cnt;
    SEnt e{};
    if (valid) e = R[i];
    const bool isr = valid && e.kind == TK_REST;
    uint32_t ct = NIL;
    int64_t len = 0;
    if (isr) {
      len = e.amt;
      const uint32_t tg = F.fc_tg[beg + e.j];
      if (tg) {
        const FcDel d = F.fc_del[tg - 1u];
        if (d.ct != NIL) { ct = d.ct; len = e.amt - d.r; }
      }
    }
    const int64_t il = wave_incl_scan(len);
    const unsigned long long rm = __ballot(isr);
    if (isr) {
      RsEnt x;
      x.e = acc + il - len;
      x.v = e.amt;
      x.j = e.j;
      x.t = e.t;
      x.pad0 = ct;
      x.pad1 = 0;
      RS[k + __popcll(rm & ltm)] = x;
    }
    acc += rl64(il, 63);
    k += __popcll(rm);
  }
  const int64_t qend = acc;
#ifdef GOME_PROBE_LEVEL
  const uint64_t pt1 = wall_clock64();
#endif
  // 3. the old FIFO, gathered through the consumption end, then on through targeted makers (a
  //    later cancel may remove them) to the first untargeted one (never cancelled, so a
  //    MatchNode.NextNode search stops there)
  const uint32_t nv0 = uni(Lq->nv0), tail = uni(Lq->tail), tslot = uni(Lq->tslot);
  uint32_t head = uni(Lq->head), hslot = uni(Lq->hslot);
  uint32_t ttail = tail, ttslot = tslot;
  uint32_t ig_base = 0, ng = 0, consumed = 0, zpopped = 0;
  bool ig_all = true;
  // (a CONS of 0 -- a zero-volume taker -- reads the head even when nothing was consumed)
  if (nv0 > 0 && (cfin > 0 || uni(Lq->c_old) || ncons)) {
    uint32_t bb = 0;
    if (lane == 0) bb = atomicAdd(F.ig_bump, nv0);
    ig_base = uni(bb);
    if (static_cast<unsigned long long>(ig_base) + nv0 > F.ig_cap) {
      if (lane == 0) atomicOr(&D.st->err, ERR_CHUNKS);
      return;
    }
    IgEnt* IG = F.ig + ig_base;
    int64_t E = 0;
    bool have_surv = false, stop = false;
    uint32_t c = head, s0 = hslot, nh = NIL, nhs = 0;
    for (uint32_t guard = 0; c != NIL && !stop; ++guard) {
      if (guard > D.ch_cap) { if (lane == 0) atomicOr(&D.st->err, ERR_CORRUPT); return; }
      const uint32_t lim = (c == tail) ? tslot : CH;
      const bool inr = lane < CH && lane >= s0 && lane < lim;
      const uint32_t nxt = (c == tail) ? NIL : D.chdr[c].next;  // (in flight beside the nodes)
      Node nd{};
      if (inr) nd = D.nodes[c * CH + lane];
      const bool live = inr && nd.rem >= 0;
      const bool targ = live && nd.pad != 0;
      uint32_t ct = NIL;
      int64_t len = live ? nd.rem : 0;
      if (targ) {
        const FcDel d = F.fc_del[static_cast<uint32_t>(nd.pad) - 1u];
        if (d.ct != NIL) { ct = d.ct; len = nd.rem - d.r; }
      }
      const int64_t inc = wave_incl_scan(len);
      const int64_t em = E + inc - len;
      const bool zend = lcont && live && !targ && nd.rem == 0 && em == cfin;  // (popped: the last consume went on)
      const unsigned long long after = __ballot(live && em >= cfin && !targ && !zend);
      const uint32_t fb = after ? static_cast<uint32_t>(__builtin_ctzll(after)) : 64u;
      const bool take = live && lane <= fb;
      const unsigned long long tm = __ballot(take);
      if (take) {
        IgEnt gq;
        gq.e = em;
        gq.v = nd.rem;
        gq.oid = nd.oid;
        gq.uuid = nd.uuid;
        gq.tx = nd.tx;
        gq.pad = ct;
        IG[ng + __popcll(tm & ltm)] = gq;
      }
      ng += __popcll(tm);
      // fully consumed (uncancelled) makers leave with their index entries
      // (a zero-volume maker (Q6) is popped strictly before the consumption end, or at it when the
      // last consume went on, as the ADD path's gather: engine.go:145-161 pops it with a 0-fill
      // when the taker goes on)
      const bool cons = live && ct == NIL && em + nd.rem <= cfin && (nd.rem > 0 || em < cfin || zend);
      if (cons) __hip_atomic_store(&D.idx[nd.ixs].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      consumed += __popcll(__ballot(cons));
      zpopped += __popcll(__ballot(cons && nd.rem == 0));
      if (!have_surv) {
        const unsigned long long sv = __ballot(live && ct == NIL && !cons);
        if (sv) {
          have_surv = true;
          nh = c;
          nhs = static_cast<uint32_t>(__builtin_ctzll(sv));
          if (lane == nhs && em < cfin) D.nodes[c * CH + lane].rem = em + nd.rem - cfin;  // partial head
        } else {
          // nothing survives in this chunk: consumed / cancelled makers only (k_fc_events
          // tombstones the cancelled ones; the chunk goes back to the pool)
          if (lane == 0) D.freed_ids[atomicAdd(&D.st->freed_top, 1u)] = c;
        }
      }
      if (after) { stop = true; ig_all = false; }
      E += rl64(inc, 63);
      c = uni(nxt);
      s0 = 0;
#ifdef GOME_PROBE_LEVEL
      ++pwalk;
#endif
    }
    if (!have_surv && ig_all) {
      head = ttail = NIL;
      hslot = ttslot = 0;
    } else if (have_surv) {
      head = nh;
      hslot = nhs;
    }
    // (!have_surv && !ig_all cannot happen: the untargeted stop maker survives)
  }
#ifdef GOME_PROBE_LEVEL
  {
    const uint64_t pt2 = wall_clock64();
    if (lane == 0) {
      atomicAdd(&g_probe[0], pt1 - pt0);
      atomicAdd(&g_probe[1], pt2 - pt1);
      atomicAdd(&g_probe[2], 1ull);
      atomicAdd(&g_probe[3], static_cast<unsigned long long>(pwalk));
      atomicMax(&g_probe[4], pt2 - pt0);
      atomicAdd(&g_probe[5], static_cast<unsigned long long>(cnt));
      if (pt2 - pt0 > GOME_PROBE_LEVEL) atomicAdd(&g_probe[6], 1ull);
      atomicMax(&g_probe[7], static_cast<unsigned long long>(cnt));
    }
  }
#endif
  if (lane == 0) {
    Lq->cfin = cfin;
    Lq->nrest = nr;
    Lq->ig_base = ig_base;
    Lq->ig_n = ng;
    Lq->ig_all = ig_all ? 1u : 0u;
    Lq->head = head;
    Lq->tail = ttail;
    Lq->hslot = hslot;
    Lq->tslot = ttslot;
    Lq->nlive0 = nv0 - consumed - ncan_old;
    Lq->zpop = zpopped;
    Lq->zcont = lcont ? 1u : 0u;
    Lq->ocan = static_cast<uint32_t>(static_cast<uint64_t>(ocan) / g);
    Lq->pad0 = static_cast<uint32_t>(static_cast<uint64_t>(qend));
    Lq->pad1 = static_cast<uint32_t>(static_cast<uint64_t>(qend) >> 32);
  }
}

// fc_level_one by ONE lane, for a level of at most FC_LANE_MAX touches (the same outputs; the
// DEL records it writes in step 1 are the ones it reads back in steps 2 and 3, a level's own
// cancels, so no fence).  The tail's deep books hold ~600k levels per batch with ~3 touches each
// (config 5c, GOME_PROBE_LEVEL): one wave took them one after another, each a chain of dependent
// loads, and k_deep_level ran 15 ms.  Lanes take their levels side by side.
constexpr uint32_t FC_LANE_MAX = 16;
__device__ __forceinline__ void fc_level_lane(const Dev& D, const FlowArgs& F, uint32_t h, uint32_t q, uint32_t cnt) {
  const FlowHdr* hd = &F.hdr[h];
  FlowLvl* Lq = fl_lvls(F, h) + q;
  const uint32_t beg = hd->beg;
  const uint32_t L = FL_TOUCH_MUL * beg;
  const unsigned long long g = static_cast<unsigned long long>(hd->g);
  const uint32_t base = Lq->base;
  const int64_t d0 = Lq->d0;
  SEnt* R = F.srt + L + base;
  RsEnt* RS = F.rs + L + base;
  // 1. cancels -> their DEL records; the consumption cursor before each consume
  int64_t cc = 0, ocan = 0;
  uint32_t nr = 0, ncan_old = 0, ncons = 0;
  for (uint32_t i = 0; i < cnt; ++i) {
    const SEnt e = R[i];
    if (e.kind == TK_CANC) {
      FcDel* d = &F.fc_del[beg + e.j];
      d->r = e.amt;
      d->ct = e.t;
      if (d->kind == FC_OLD) { ocan += e.amt; ncan_old++; }
    } else if (e.kind == TK_CONS) {
      R[i].coord = cc;
      cc += e.amt;
      ++ncons;
    } else if (e.kind == TK_REST) {
      nr++;
    }
  }
  const int64_t cfin = cc;
  const bool lcont = (Lq->z0 || hd->nzero) && cfin > 0 && fl_run_cont(F, L, hd->ntouch, R, cnt, true);  // (fc_level_one)
  // 2. the new makers in FIFO order
  int64_t acc = d0 - ocan;
  uint32_t k = 0;
  for (uint32_t i = 0; i < cnt; ++i) {
    const SEnt e = R[i];
    if (e.kind != TK_REST) continue;
    uint32_t ct = NIL;
    int64_t len = e.amt;
    const uint32_t tg = F.fc_tg[beg + e.j];
    if (tg) {
      const FcDel d = F.fc_del[tg - 1u];
      if (d.ct != NIL) { ct = d.ct; len = e.amt - d.r; }
    }
    RsEnt x;
    x.e = acc;
    x.v = e.amt;
    x.j = e.j;
    x.t = e.t;
    x.pad0 = ct;
    x.pad1 = 0;
    RS[k++] = x;
    acc += len;
  }
  const int64_t qend = acc;
  // 3. the old FIFO (fc_level_one's walk, a chunk's slots in order)
  const uint32_t nv0 = Lq->nv0, tail = Lq->tail, tslot = Lq->tslot;
  uint32_t head = Lq->head, hslot = Lq->hslot;
  uint32_t ttail = tail, ttslot = tslot;
  uint32_t ig_base = 0, ng = 0, consumed = 0, zpopped = 0;
  bool ig_all = true;
  if (nv0 > 0 && (cfin > 0 || Lq->c_old || ncons)) {  // (fc_level_one)
    ig_base = atomicAdd(F.ig_bump, nv0);
    if (static_cast<unsigned long long>(ig_base) + nv0 > F.ig_cap) {
      atomicOr(&D.st->err, ERR_CHUNKS);
      return;
    }
    IgEnt* IG = F.ig + ig_base;
    int64_t E = 0;
    bool have_surv = false, stop = false;
    uint32_t c = head, s0 = hslot, nh = NIL, nhs = 0;
    for (uint32_t guard = 0; c != NIL && !stop; ++guard) {
      if (guard > D.ch_cap) { atomicOr(&D.st->err, ERR_CORRUPT); return; }
      const uint32_t lim = (c == tail) ? tslot : CH;
      const uint32_t nxt = (c == tail) ? NIL : D.chdr[c].next;
      Node nd[CH];
#pragma unroll
      for (uint32_t s = 0; s < CH; ++s) {
        nd[s] = Node{};
        if (s >= s0 && s < lim) nd[s] = D.nodes[c * CH + s];
      }
      bool taking = true, surv_here = false;
#pragma unroll
      for (uint32_t s = 0; s < CH; ++s) {
        const bool live = s >= s0 && s < lim && nd[s].rem >= 0;
        if (!live) continue;
        const bool targ = nd[s].pad != 0;
        uint32_t ct = NIL;
        int64_t len = nd[s].rem;
        if (targ) {
          const FcDel d = F.fc_del[static_cast<uint32_t>(nd[s].pad) - 1u];
          if (d.ct != NIL) { ct = d.ct; len = nd[s].rem - d.r; }
        }
        const int64_t em = E;
        E += len;
        const bool zend = lcont && !targ && nd[s].rem == 0 && em == cfin;
        if (taking) {  // (every live maker through the first untargeted one at or past the consumption end)
          IgEnt gq;
          gq.e = em;
          gq.v = nd[s].rem;
          gq.oid = nd[s].oid;
          gq.uuid = nd[s].uuid;
          gq.tx = nd[s].tx;
          gq.pad = ct;
          IG[ng++] = gq;
          if (em >= cfin && !targ && !zend) { taking = false; stop = true; ig_all = false; }
        }
        const bool cons = ct == NIL && em + nd[s].rem <= cfin && (nd[s].rem > 0 || em < cfin || zend);  // (Q6 as above)
        if (cons) {
          __hip_atomic_store(&D.idx[nd[s].ixs].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          consumed++;
          if (nd[s].rem == 0) zpopped++;
        }
        if (!have_surv && !surv_here && ct == NIL && !cons) {
          surv_here = true;
          nh = c;
          nhs = s;
          if (em < cfin) D.nodes[c * CH + s].rem = em + nd[s].rem - cfin;  // partial head
        }
      }
      if (!have_surv) {
        if (surv_here) have_surv = true;
        else D.freed_ids[atomicAdd(&D.st->freed_top, 1u)] = c;
      }
      c = nxt;
      s0 = 0;
    }
    if (!have_surv && ig_all) {
      head = ttail = NIL;
      hslot = ttslot = 0;
    } else if (have_surv) {
      head = nh;
      hslot = nhs;
    }
  }
  Lq->cnt = cnt;
  Lq->cfin = cfin;
  Lq->nrest = nr;
  Lq->ig_base = ig_base;
  Lq->ig_n = ng;
  Lq->ig_all = ig_all ? 1u : 0u;
  Lq->head = head;
  Lq->tail = ttail;
  Lq->hslot = hslot;
  Lq->tslot = ttslot;
  Lq->nlive0 = nv0 - consumed - ncan_old;
  Lq->zpop = zpopped;
  Lq->zcont = lcont ? 1u : 0u;
  Lq->ocan = static_cast<uint32_t>(static_cast<uint64_t>(ocan) / g);
  Lq->pad0 = static_cast<uint32_t>(static_cast<uint64_t>(qend));
  Lq->pad1 = static_cast<uint32_t>(static_cast<uint64_t>(qend) >> 32);
}

constexpr uint32_t FC_LVB_T = FL_LVB_T, FC_K = 4;
// a level of FC_BIG touches or more takes a whole block (fc_level_blk), smaller ones a wave
constexpr uint32_t FC_BIG = 1024;

// A big level's pass, step 3 (one wave): its old FIFO gathered (the makers the batch reaches, their
// consumption-space starts), the consumed ones tombstoned, the partial head cut, and the level's
// results; cfin / ncons / nrest / ncan_old / ocan_t / qend from steps 1-2 (fc_level_blk, or the
// chunked pass of a huge level, k_fcb_*).
__device__ __forceinline__ void fc_level_fifo(const Dev& D, const FlowArgs& F, const FlowHdr* hd, FlowLvl* Lq,
                                              const SEnt* R, uint32_t cnt, uint32_t L, int64_t cfin, uint32_t ncons_s,
                                              uint32_t nr_s, uint32_t ncan_s, int64_t ocan_t, int64_t qend) {
  const uint32_t lane = lane_id();
  const unsigned long long g = static_cast<unsigned long long>(hd->g);
  const bool lcont = (Lq->z0 || hd->nzero) && cfin > 0 && fl_run_cont(F, L, hd->ntouch, R, cnt, true);
  const unsigned long long ltm = lt_mask();
  const uint32_t nv0 = Lq->nv0, tail = Lq->tail, tslot = Lq->tslot;
  uint32_t head = Lq->head, hslot = Lq->hslot;
  uint32_t ttail = tail, ttslot = tslot;
  uint32_t ig_base = 0, ng = 0, consumed = 0, zpopped = 0;
  bool ig_all = true;
  if (nv0 > 0 && (cfin > 0 || Lq->c_old || ncons_s)) {  // (fc_level_one)
    uint32_t bb = 0;
    if (lane == 0) bb = atomicAdd(F.ig_bump, nv0);
    ig_base = uni(bb);
    if (static_cast<unsigned long long>(ig_base) + nv0 > F.ig_cap) {
      if (lane == 0) atomicOr(&D.st->err, ERR_CHUNKS);
      return;
    }
    IgEnt* IG = F.ig + ig_base;
    int64_t E = 0;
    bool have_surv = false, stop = false;
    uint32_t c = head, s0 = hslot, nh = NIL, nhs = 0;
    for (uint32_t guard = 0; c != NIL && !stop; ++guard) {
      if (guard > D.ch_cap) { if (lane == 0) atomicOr(&D.st->err, ERR_CORRUPT); return; }
      const uint32_t lim = (c == tail) ? tslot : CH;
      const bool inr = lane < CH && lane >= s0 && lane < lim;
      const uint32_t nxt = (c == tail) ? NIL : D.chdr[c].next;  // (in flight beside the nodes)
      Node nd{};
      if (inr) nd = D.nodes[c * CH + lane];
      const bool live = inr && nd.rem >= 0;
      const bool targ = live && nd.pad != 0;
      uint32_t ct = NIL;
      int64_t len = live ? nd.rem : 0;
      if (targ) {
        const FcDel d = F.fc_del[static_cast<uint32_t>(nd.pad) - 1u];
        if (d.ct != NIL) { ct = d.ct; len = nd.rem - d.r; }
      }
      const int64_t inc = wave_incl_scan(len);
      const int64_t em = E + inc - len;
      const bool zend = lcont && live && !targ && nd.rem == 0 && em == cfin;
      const unsigned long long after = __ballot(live && em >= cfin && !targ && !zend);
      const uint32_t fb = after ? static_cast<uint32_t>(__builtin_ctzll(after)) : 64u;
      const bool take = live && lane <= fb;
      const unsigned long long tm = __ballot(take);
      if (take) {
        IgEnt gq;
        gq.e = em;
        gq.v = nd.rem;
        gq.oid = nd.oid;
        gq.uuid = nd.uuid;
        gq.tx = nd.tx;
        gq.pad = ct;
        IG[ng + __popcll(tm & ltm)] = gq;
      }
      ng += __popcll(tm);
      // (a zero-volume maker (Q6) is popped strictly before the consumption end, or at it when the
      // last consume went on: fc_level_one)
      const bool cons = live && ct == NIL && em + nd.rem <= cfin && (nd.rem > 0 || em < cfin || zend);
      if (cons) __hip_atomic_store(&D.idx[nd.ixs].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      consumed += __popcll(__ballot(cons));
      zpopped += __popcll(__ballot(cons && nd.rem == 0));
      if (!have_surv) {
        const unsigned long long sv = __ballot(live && ct == NIL && !cons);
        if (sv) {
          have_surv = true;
          nh = c;
          nhs = static_cast<uint32_t>(__builtin_ctzll(sv));
          if (lane == nhs && em < cfin) D.nodes[c * CH + lane].rem = em + nd.rem - cfin;  // partial head
        } else {
          if (lane == 0) D.freed_ids[atomicAdd(&D.st->freed_top, 1u)] = c;
        }
      }
      if (after) { stop = true; ig_all = false; }
      E += rl64(inc, 63);
      c = uni(nxt);
      s0 = 0;
    }
    if (!have_surv && ig_all) {
      head = ttail = NIL;
      hslot = ttslot = 0;
    } else if (have_surv) {
      head = nh;
      hslot = nhs;
    }
  }
  if (lane == 0) {
    Lq->cfin = cfin;
    Lq->nrest = nr_s;
    Lq->ig_base = ig_base;
    Lq->ig_n = ng;
    Lq->ig_all = ig_all ? 1u : 0u;
    Lq->head = head;
    Lq->tail = ttail;
    Lq->hslot = hslot;
    Lq->tslot = ttslot;
    Lq->nlive0 = nv0 - consumed - ncan_s;
    Lq->zpop = zpopped;
    Lq->zcont = lcont ? 1u : 0u;
    Lq->ocan = static_cast<uint32_t>(static_cast<uint64_t>(ocan_t) / g);
    Lq->pad0 = static_cast<uint32_t>(static_cast<uint64_t>(qend));
    Lq->pad1 = static_cast<uint32_t>(static_cast<uint64_t>(qend) >> 32);
  }
}


// fc_level_one with a whole block (FC_LVB_T threads) on one level: the level's touches in
// block-wide chunks (the long levels of the hottest books hold tens of thousands of touches,
// which one wave walks 64 at a time); the old FIFO's gather stays with wave 0.
__device__ __forceinline__ void fc_level_blk(const Dev& D, const FlowArgs& F, uint32_t h, uint32_t q) {
  __shared__ int64_t red_s[2];
  __shared__ uint32_t nr_s, ncan_s, ncons_s;
  const FlowHdr* hd = &F.hdr[h];
  const uint32_t tid = threadIdx.x;
  FlowLvl* Lq = fl_lvls(F, h) + q;  // (a lane book's F.lvl row, or a deep book's level table)
  const uint32_t beg = hd->beg;
  const uint32_t L = FL_TOUCH_MUL * beg;
  const uint32_t base = Lq->base, cnt = Lq->cnt;
  const int64_t d0 = Lq->d0;
  SEnt* R = F.srt + L + base;
  RsEnt* RS = F.rs + L + base;
  if (tid == 0) { red_s[0] = 0; nr_s = 0; ncan_s = 0; ncons_s = 0; }
  __syncthreads();
  // 1. each cancel -> its DEL's record (r, touch); the consumption cursor before each consume.
  //    FC_K consecutive touches per thread: their loads in flight together, a quarter of the
  //    block scans (a busy level is tens of thousands of touches)
  int64_t cc = 0, ocan = 0;
  uint32_t nr = 0, ncan_old = 0, nc = 0;
  for (uint32_t c0 = 0; c0 < cnt; c0 += FC_LVB_T * FC_K) {
    const uint32_t i0 = c0 + tid * FC_K;
    SEnt e[FC_K];
#pragma unroll
    for (uint32_t u = 0; u < FC_K; ++u)
      if (i0 + u < cnt) e[u] = R[i0 + u];
    int64_t sum = 0;
#pragma unroll
    for (uint32_t u = 0; u < FC_K; ++u) {
      if (i0 + u >= cnt) continue;
      if (e[u].kind == TK_CANC) {
        FcDel* d = &F.fc_del[beg + e[u].j];
        d->r = e[u].amt;
        d->ct = e[u].t;
        if (d->kind == FC_OLD) { ocan += e[u].amt; ncan_old++; }
      }
      sum += e[u].kind == TK_CONS ? e[u].amt : 0;
      nr += e[u].kind == TK_REST ? 1u : 0u;
      nc += e[u].kind == TK_CONS ? 1u : 0u;
    }
    int64_t tot;
    int64_t run = cc + fl_blk_excl(sum, &tot);
#pragma unroll
    for (uint32_t u = 0; u < FC_K; ++u) {
      if (i0 + u >= cnt || e[u].kind != TK_CONS) continue;
      R[i0 + u].coord = run;
      run += e[u].amt;
    }
    cc += tot;
  }
  if (ocan) atomicAdd(reinterpret_cast<unsigned long long*>(&red_s[0]), static_cast<unsigned long long>(ocan));
  if (nr) atomicAdd(&nr_s, nr);
  if (ncan_old) atomicAdd(&ncan_s, ncan_old);
  if (nc) atomicAdd(&ncons_s, nc);
  __threadfence();  // the DEL records are read back below (by other threads)
  __syncthreads();
  const int64_t ocan_t = red_s[0];
  const int64_t cfin = cc;
  const int64_t base_new = d0 - ocan_t;
  // 2. the new makers in FIFO (rest) order, their consumption-space starts and cancels
  int64_t acc = base_new;
  uint32_t k = 0;
  for (uint32_t c0 = 0; c0 < cnt; c0 += FC_LVB_T * FC_K) {
    const uint32_t i0 = c0 + tid * FC_K;
    SEnt e[FC_K];
    uint32_t tg[FC_K];
#pragma unroll
    for (uint32_t u = 0; u < FC_K; ++u) {
      tg[u] = 0;
      if (i0 + u < cnt) e[u] = R[i0 + u];
    }
#pragma unroll
    for (uint32_t u = 0; u < FC_K; ++u)
      if (i0 + u < cnt && e[u].kind == TK_REST) tg[u] = F.fc_tg[beg + e[u].j];
    uint32_t ct[FC_K];
    int64_t len[FC_K], sum = 0, nsum = 0;
#pragma unroll
    for (uint32_t u = 0; u < FC_K; ++u) {
      const bool isr = i0 + u < cnt && e[u].kind == TK_REST;
      ct[u] = NIL;
      len[u] = isr ? e[u].amt : 0;
      if (isr && tg[u]) {
        const FcDel d = F.fc_del[tg[u] - 1u];
        if (d.ct != NIL) { ct[u] = d.ct; len[u] = e[u].amt - d.r; }
      }
      sum += len[u];
      nsum += isr ? 1 : 0;
    }
    int64_t tot, ntot;
    int64_t run = acc + fl_blk_excl(sum, &tot);
    uint32_t rk = k + static_cast<uint32_t>(fl_blk_excl(nsum, &ntot));
#pragma unroll
    for (uint32_t u = 0; u < FC_K; ++u) {
      if (i0 + u >= cnt || e[u].kind != TK_REST) continue;
      RsEnt x;
      x.e = run;
      x.v = e[u].amt;
      x.j = e[u].j;
      x.t = e[u].t;
      x.pad0 = ct[u];
      x.pad1 = 0;
      RS[rk++] = x;
      run += len[u];
    }
    acc += tot;
    k += static_cast<uint32_t>(ntot);
  }
  const int64_t qend = acc;
  // 3. the old FIFO (wave 0), as fc_level_one
  if (tid >= 64) return;
  fc_level_fifo(D, F, hd, Lq, R, cnt, L, cfin, ncons_s, nr_s, ncan_s, ocan_t, qend);
}

// The head books' levels: a block per (book, level).  huge: the hottest book's launch, after
// k_fcb_list marked its huge levels (their chunked pass, match_flow_deep.h)
__global__ __launch_bounds__(FC_LVB_T) void k_fc_level_blk(Dev D, FlowArgs F, uint32_t huge) {
  const uint32_t h = F.h0 + blockIdx.y, q = blockIdx.x;
  if (h >= fl_hend(D, F) || !fc_lane(F, h) || q == 0 || q > F.hdr[h].nl) return;
  if (huge && fl_lvls(F, h)[q].pad6) return;
  fc_level_blk(D, F, h, q);
}

__global__ __launch_bounds__(64) void k_fc_level_wide(Dev D, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y, q = blockIdx.x;
  if (h >= fl_hend(D, F) || !fc_lane(F, h) || q == 0 || q > F.hdr[h].nl) return;
  fc_level_one(D, F, h, q);
}

// The tail's books: a block per book.  Its busiest levels first, each with the whole block (the
// aggressive orders' remainders rest at 1.00 / 0.01 and the other side's orders consume there: one
// wave took 64 of those touches at a time, and config 4's tail level pass took 5.8 ms), then the
// others a wave each.
__global__ __launch_bounds__(FC_LVB_T) void k_fc_level_book(Dev D, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.x;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  const uint32_t nl = F.hdr[h].nl;
  const FlowLvl* LV = fl_lvls(F, h);
  for (uint32_t q = 1 + threadIdx.x; q <= nl; q += blockDim.x) {  // small levels: a lane each
    const uint32_t cnt = LV[q].cnt;
    if (cnt <= FC_LANE_MAX) fc_level_lane(D, F, h, q, cnt);
  }
  for (uint32_t q = 1; q <= nl; ++q) {
    if (LV[q].cnt < FC_BIG) continue;
    fc_level_blk(D, F, h, q);
    __syncthreads();  // (fc_level_blk's shared words, before the next level's)
  }
  for (uint32_t q = 1 + (threadIdx.x >> 6); q <= nl; q += blockDim.x / 64) {
    const uint32_t cnt = uni(LV[q].cnt);
    if (cnt > FC_LANE_MAX && cnt < FC_BIG) fc_level_one(D, F, h, uni(q));
  }
}

// ---- fills of one consume touch ----------------------------------------------------------
struct FcTouch {
  FcLvlView V;
  const FlowLvl* Lq;
  int64_t c, a;           // cursor before the touch, amount
  uint32_t first, last;   // makers spanned
  bool cont;              // the consume went on past the level (fl_cont; levels with zero-volume makers)
};

// The head of a level's FIFO when the consume at cursor c, log index t, came (a zero-volume taker:
// MatchOrder fills its first node, engine.go:138-198).  f = fc_find(c).  A maker spanning c is
// partly consumed, so live: the head.  Makers starting at c with length 0 were cancelled before any
// consumption -- after t some of them, which were live at t and ahead of the one with volume: the
// first of those that had arrived and was not yet cancelled at t is the head.  (A zero-volume maker
// there is a hazard, k_flow_zero_check: diff == 0 pops it.)
__device__ __forceinline__ uint32_t fc_head_at(const FcLvlView& V, uint32_t f, int64_t c, uint32_t t) {
  if (fc_start(V, f) != c) return f;
  uint32_t m = f;
  while (m > 0 && fc_start(V, m - 1) == c) --m;
  for (; m < f; ++m) {
    const bool arrived = m < V.ig_n || V.RS[m - V.ig_n].t < t;
    const uint32_t ct = fc_ct(V, m);
    if (arrived && (ct == NIL || ct > t)) return m;
  }
  return f;
}

// t: the touch's log index (book-local)
__device__ __forceinline__ FcTouch fc_touch(const FlowArgs& F, uint32_t h, uint32_t L, const Touch& x, uint32_t t) {
  FcTouch T;
  const uint32_t k = F.hdr[h].ok == FL_OK_DEEP ? F.srt[L + x.pos].lvl : (x.kr & 127u);
  T.Lq = fl_lvls(F, h) + k;
  T.V = fc_view(F, h, *T.Lq);
  T.c = F.srt[L + x.pos].coord;
  T.a = x.amt;
  T.first = fc_find(T.V, T.c);
  T.cont = false;
  if (T.a == 0) {  // a zero-volume taker (Q6): one 0-fill, of the FIFO's head at its time
    T.first = T.last = fc_head_at(T.V, T.first, T.c, t);
    return T;
  }
  // a level that may hold zero-volume makers (Q6): the ones starting at the cursor are popped by
  // this consume too (they share the start of the maker fc_find lands on; fl_first_back), unless
  // the consume before it went on and popped them; a consume that goes on pops the ones at its end
  // (fl_cont)
  const bool zl = (T.Lq->z0 || F.hdr[h].nzero) && T.a > 0;
  if (zl) {
    const uint32_t nt = F.hdr[h].ntouch;
    T.cont = fl_cont(F, L, nt, t, true);
    const uint32_t base = T.Lq->base;
    if (!fl_prev_cont(F, L, nt, F.srt + L + base, x.pos - base, true))
      while (T.first > 0 && fc_start(T.V, T.first - 1) == T.c) --T.first;
  }
  // the last maker: a touch spans a few makers, so step on from the first (neighbouring entries,
  // one cache line) before a second binary search (~16 dependent loads on a busy level); the
  // starts rise through the old makers into the new ones, so both give the last start <= x
  const int64_t xl = T.c + T.a - 1;
  const uint32_t nm = T.V.ig_n + T.V.nrest;
  uint32_t m = T.first, st = 0;
  for (; st < 8 && m + 1 < nm && fc_start(T.V, m + 1) <= xl; ++st) ++m;
  T.last = st < 8 ? m : fc_find(T.V, xl);
  // (going on: over the zero-length makers at the end, the zero-volume ones among them filled)
  if (T.cont)
    while (T.last + 1 < nm && fc_len(T.V, T.last + 1) == 0 && fc_start(T.V, T.last + 1) == T.c + T.a) ++T.last;
  return T;
}

// A maker of zero length in consumption space fills nothing (cancelled before any consumption),
// except a zero-volume maker (Q6: volume 0, never cancelled in a flow batch -- its DEL is a hazard,
// k_fc_resolve) that starts inside the consume [c, c + a), or at its end c + a when the consume
// goes on (cont): MatchOrder pops it with a 0-fill and goes on (engine.go:145-161).
__device__ __forceinline__ bool fc_fills(const FcLvlView& V, uint32_t m, int64_t c, int64_t a, bool cont) {
  if (fc_len(V, m) > 0) return true;
  const int64_t e = fc_start(V, m);
  return fc_vol(V, m) == 0 && e >= c && (e < c + a || (cont && e == c + a));
}

// Fills of a consume touch: makers of [first, last] with volume in consumption space.
__device__ __forceinline__ uint32_t fc_nfills(const FcTouch& T, uint32_t& pops) {
  uint32_t nf = 0;
  pops = 0;
  if (T.a == 0) return 1;  // (a zero-volume taker: one 0-fill, nothing popped)
  for (uint32_t m = T.first; m <= T.last; ++m) {
    if (!fc_fills(T.V, m, T.c, T.a, T.cont)) continue;
    ++nf;
    if (fc_start(T.V, m) + fc_vol(T.V, m) <= T.c + T.a) ++pops;  // filled to its whole volume
  }
  return nf;
}

// ---- k_fc_count_nf / k_fc_count_run: events per touch and per order -----------------------
// A touch's fills cost a binary search of its level's makers (fc_touch: ~16 dependent loads on a
// busy level), so they are counted a thread per touch (k_fc_count_nf, into fbase), and only then
// summed per order (k_fc_count_run: the order's first touch walks its touches' counts, a few cache
// lines).  One pass that walked each order's touches from its first (round 5) ran as long as the
// longest sweep's chain of searches: 0.32 ms on config 4's hottest book (orders of 74 levels).
__global__ void k_fc_count_nf(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t hend = fl_hend(D, F), nb = hend > F.h0 ? hend - F.h0 : 0u;
  const uint32_t total = nb ? F.toff[F.tb + nb] : 0u;
  unsigned long long fills = 0, pops = 0, cancels = 0;
  for (uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x; gt < total; gt += gridDim.x * blockDim.x) {
    const uint32_t hb = fl_book_of_wave(F, nb, gt - lane_id(), gt), h = F.h0 + hb, t = gt - F.toff[F.tb + hb];
    const uint32_t L = FL_TOUCH_MUL * F.hdr[h].beg;
    const Touch x = F.log[L + t];
    const uint32_t kind = tk_kind(x.kr, true);
    uint32_t nf = 0;
    if (kind == TK_CONS) {
      uint32_t pp;
      nf = fc_nfills(fc_touch(F, h, L, x, t), pp);
      fills += nf;
      pops += pp;
    } else if (kind == TK_CANC) {
      nf = 1;
      cancels += 1;
    }
    F.fbase[L + t] = nf;
  }
  for (int off = 32; off > 0; off >>= 1) {
    fills += __shfl_xor(fills, off);
    pops += __shfl_xor(pops, off);
    cancels += __shfl_xor(cancels, off);
  }
  if (lane_id() == 0 && (fills || cancels)) {
    ctr_add(D, C_FILLS, fills);
    ctr_add(D, C_HOT_FILLS, fills);
    ctr_add(D, C_CANCELS, cancels);
    ctr_add(D, C_HOT_CANCELS, cancels);
    ctr_add(D, C_FLOW_CANCELS, cancels);
    ctr_add(D, C_RESTING_DELTA, static_cast<unsigned long long>(-static_cast<long long>(pops + cancels)));
  }
}

// fbase: each touch's count -> the order's events before it; the order's total -> ev_count
__global__ void k_fc_count_run(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t hend = fl_hend(D, F), nb = hend > F.h0 ? hend - F.h0 : 0u;
  const uint32_t total = nb ? F.toff[F.tb + nb] : 0u;
  for (uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x; gt < total; gt += gridDim.x * blockDim.x) {
    const uint32_t hb = fl_book_of_wave(F, nb, gt - lane_id(), gt), h = F.h0 + hb, t = gt - F.toff[F.tb + hb];
    const uint32_t nt = F.hdr[h].ntouch, beg = F.hdr[h].beg, L = FL_TOUCH_MUL * beg;
    const uint32_t j = tk_jc(F.log[L + t]);
    if (t > 0 && tk_jc(F.log[L + t - 1]) == j) continue;
    uint32_t acc = 0;
    for (uint32_t u = t; u < nt && (u == t || tk_jc(F.log[L + u]) == j); ++u) {
      const uint32_t v = F.fbase[L + u];
      F.fbase[L + u] = acc;
      acc += v;
    }
    if (j < F.hdr[h].end - beg) B.ev_count[prep_at(B, beg + j).idx] = acc;  // not padding
  }
}

// ---- k_fc_events: every MatchResult of the range's books, into the event arena -------------
__global__ __launch_bounds__(256) void k_fc_events(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t hend = fl_hend(D, F), nb = hend > F.h0 ? hend - F.h0 : 0u;
  const uint32_t total = nb ? F.toff[F.tb + nb] : 0u;
  const uint32_t lane = lane_id(), stride = gridDim.x * blockDim.x;
  const uint32_t w = threadIdx.x >> 6;
  __shared__ uint32_t wtot[FL_EV_T / 64], bbase;
  // block tiles (every wave of the block iterates together: the arena is claimed once per tile)
  for (uint32_t b0 = blockIdx.x * blockDim.x; b0 < total; b0 += stride) {
    const uint32_t gt = b0 + threadIdx.x, g0w = b0 + (threadIdx.x & ~63u);
    uint32_t h = 0, L = 0, t = 0, cnt = 0, kind = TK_REST;
    Touch x{};
    FcTouch T{};
    uint32_t hbw = 0;
    if (g0w < total) hbw = fl_book_of_wave(F, nb, g0w, gt < total ? gt : g0w);
    if (gt < total) {
      const uint32_t hb = hbw;
      h = F.h0 + hb;
      t = gt - F.toff[F.tb + hb];
      L = FL_TOUCH_MUL * F.hdr[h].beg;
      x = F.log[L + t];
      kind = tk_kind(x.kr, true);
      if (kind == TK_CONS) {
        uint32_t pp;
        T = fc_touch(F, h, L, x, t);
        cnt = fc_nfills(T, pp);
      } else if (kind == TK_CANC) {
        cnt = 1;
      }
    }
    uint32_t inc = cnt;
    for (uint32_t off = 1; off < 64; off <<= 1) {
      const uint32_t v = __shfl_up(inc, off);
      if (lane >= off) inc += v;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t tt = 0;
      for (uint32_t k = 0; k < FL_EV_T / 64; ++k) { const uint32_t v = wtot[k]; wtot[k] = tt; tt += v; }
      bbase = tt ? atomicAdd(&D.st->ev_bump, tt) : 0u;
      if (tt && static_cast<unsigned long long>(bbase) + tt > B.arena_cap) {
        atomicOr(&D.st->err, ERR_EVENTS);
        bbase = NIL;
      }
    }
    __syncthreads();
    const uint32_t base = bbase, wb = wtot[w];
    __syncthreads();  // (wtot / bbase are rewritten by the next tile)
    if (base == NIL || !cnt) continue;
    gome_event* dst = B.arena + base + wb + (inc - cnt);
    const uint32_t beg = F.hdr[h].beg, sym = F.hdr[h].sym;
    const Prep tk = prep_at(B, beg + tk_jc(x));
    if (kind == TK_CANC) {  // DeleteOrder's MatchResult (engine.go:109-113)
      const FcDel d = F.fc_del[beg + tk_jc(x)];
      gome_event ev;
      ev.price_fx = tk.price;
      ev.match_volume_fx = 0;
      ev.maker_volume_fx = x.amt;
      ev.taker_seq = tk.idx;
      ev.fill_idx = 0;
      ev.maker_oid_id = tk.oid;
      ev.maker_uuid_id = tk.uuid;
      ev.maker_next_oid_id = 0;
      ev.kind = GOME_EV_CANCEL;
      ev.maker_side = tk.side;
      ev.maker_is_last = 1;
      ev.pad0 = 0;
      dst[0] = ev;
      if (d.kind == FC_OLD) {  // unlink (nodelink.go:124-166): a tombstone, the index entry erased
        Node* nd = &D.nodes[d.tgt];
        nd->rem = -1;
        nd->pad = 0;
        __hip_atomic_store(&D.idx[d.ixs].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      continue;
    }
    // taker remaining before this level: volume minus what its better levels took
    int64_t tb = tk.vol;
    for (uint32_t u = t; u > 0; --u) {
      const Touch y = F.log[L + u - 1];
      if (tk_jc(y) != tk_jc(x)) break;
      tb -= y.amt;
    }
    const FcLvlView& V = T.V;
    const int64_t price = T.Lq->price;
    const uint32_t fb = F.fbase[L + t];
    uint32_t k = 0;
    for (uint32_t m = T.first; m <= T.last; ++m) {
      if (T.a > 0 && !fc_fills(V, m, T.c, T.a, T.cont)) continue;  // (a zero-volume taker: its head)
      const int64_t len = fc_len(V, m);
      const int64_t e = fc_start(V, m), v = fc_vol(V, m);
      uint32_t oid, uuid, tx;
      if (m < V.ig_n) {
        const IgEnt gq = V.IG[m];
        oid = gq.oid; uuid = gq.uuid; tx = gq.tx;
      } else {
        const Prep mk = prep_at(B, beg + V.RS[m - V.ig_n].j);
        oid = mk.oid; uuid = mk.uuid; tx = mk.side;
      }
      const int64_t lo = e > T.c ? e : T.c;
      const int64_t hi = (e + len < T.c + T.a) ? e + len : T.c + T.a;
      const int64_t qty = hi - lo, pre = e + v - lo;  // remaining before this fill
      const bool full = e + v <= T.c + T.a;
      // MatchNode.NextNode: the next maker of the FIFO at the time of this fill — arrived
      // before it, not cancelled before it (engine.go:138-198 reads the head node's link)
      uint32_t nx = 0, last = 1;
      for (uint32_t m2 = m + 1; m2 < V.ig_n + V.nrest; ++m2) {
        if (m2 >= V.ig_n && V.RS[m2 - V.ig_n].t > t) break;  // not rested yet
        const uint32_t ct = fc_ct(V, m2);
        if (ct != NIL && ct < t) continue;                     // cancelled before
        nx = m2 < V.ig_n ? V.IG[m2].oid : prep_at(B, beg + V.RS[m2 - V.ig_n].j).oid;
        last = 0;
        break;
      }
      gome_event ev;
      ev.price_fx = price;
      ev.match_volume_fx = qty;
      ev.maker_volume_fx = full ? pre : pre - qty;
      ev.taker_seq = tk.idx;
      ev.fill_idx = fb + k;
      ev.maker_oid_id = oid;
      ev.maker_uuid_id = uuid;
      ev.maker_next_oid_id = nx;
      ev.kind = GOME_EV_FILL;
      ev.maker_side = static_cast<uint8_t>(tx);
      ev.maker_is_last = static_cast<uint8_t>(last);
      ev.pad0 = 0;
      dst[k] = ev;
      ++k;
    }
  }
}

// ---- k_fc_write: surviving new makers appended, the final level record (wave per level) ----
__device__ __forceinline__ Level fc_write_level(const Dev& D, const BatchArgs& B, const FlowArgs& F,
                                                const FlowHdr& hd, uint32_t h, uint32_t q) {
  const uint32_t lane = lane_id();
  const unsigned long long ltm = lt_mask();
  const unsigned long long mask = D.idx_mask;
  const FlowLvl f = fl_lvls(F, h)[q];
  const FcLvlView V = fc_view(F, h, f);
  Level x{};
  x.price = f.price;
  x.head = x.tail = NIL;
  // survivors among the new makers: not cancelled, not filled to the end (in FIFO order); a
  // maker starting before the consumption end keeps e + v - cfin
  uint32_t S = 0;
  uint32_t zadd = 0;  // zero-volume makers appended (Q6; the old ones the batch popped: FlowLvl::zpop)
  const bool zc = f.cfin > 0 && f.zcont;
  for (uint32_t c0 = 0; c0 < V.nrest; c0 += 64) {
    const uint32_t i = c0 + lane;
    bool sv = false;
    if (i < V.nrest) {
      const RsEnt r = V.RS[i];
      // (Q6: as the gather; one at the consumption end is popped when the last consume went on)
      sv = r.pad0 == NIL && (r.e + r.v > f.cfin || (r.v == 0 && r.e >= f.cfin && !(r.e == f.cfin && zc)));
    }
    S += __popcll(__ballot(sv));
    zadd += __popcll(__ballot(sv && i < V.nrest && V.RS[i].v == 0));
  }
  const bool fresh = f.nlive0 == 0;
  const uint32_t s0 = fresh ? 0u : f.tslot;
  const uint32_t room = fresh ? 0u : CH - s0;
  const uint32_t need = S > room ? (S - room + CH - 1) / CH : 0u;
  int t = 0;
  uint32_t nst = 0, bb = 0;
  if (need) {
    if (lane == 0) t = atomicSub(&D.st->free_top, static_cast<int>(need));
    t = static_cast<int>(uni(static_cast<uint32_t>(t)));
    nst = static_cast<uint32_t>(min(max(t, 0), static_cast<int>(need)));
    if (lane == 0 && nst < need) bb = atomicAdd(D.ch_bump, need - nst);
    bb = uni(bb);
    if (bb + (need - nst) > D.ch_cap) {
      if (lane == 0) atomicOr(&D.st->err, ERR_CHUNKS);
      return x;
    }
  }
  auto chunk_id = [&](uint32_t i) -> uint32_t {
    return i < nst ? D.free_ids[t - static_cast<int>(nst) + static_cast<int>(i)] : bb + (i - nst);
  };
  for (uint32_t i = lane; i < need; i += 64) {
    ChunkHdr c;
    c.next = (i + 1 < need) ? chunk_id(i + 1) : NIL;
    c.pad = 0;
    c.price = f.price;
    D.chdr[chunk_id(i)] = c;
  }
  if (need && !fresh && lane == 0) D.chdr[f.tail].next = chunk_id(0);
  uint32_t w = 0;
  for (uint32_t c0 = 0; c0 < V.nrest; c0 += 64) {
    const uint32_t i = c0 + lane;
    RsEnt r{};
    bool sv = false;
    if (i < V.nrest) {
      r = V.RS[i];
      sv = r.pad0 == NIL && (r.e + r.v > f.cfin || (r.v == 0 && r.e >= f.cfin && !(r.e == f.cfin && zc)));
    }
    const unsigned long long sm = __ballot(sv);
    if (sv) {
      const uint32_t gi = w + __popcll(sm & ltm);
      const Prep mk = prep_at(B, hd.beg + r.j);
      const int64_t rem = (r.e < f.cfin) ? r.e + r.v - f.cfin : r.v;
      uint32_t cid, slot;
      if (!fresh && s0 + gi < CH) {
        cid = f.tail;
        slot = s0 + gi;
      } else {
        const uint32_t gg = fresh ? gi : gi - room;
        cid = chunk_id(gg / CH);
        slot = gg % CH;
      }
      const uint32_t loc = cid * CH + slot;
      const unsigned long long key = (static_cast<unsigned long long>(hd.sym + 1) << 32) | mk.oid;
      unsigned long long hh = mix64(key) & mask, probe = 0;
      for (; probe <= mask; ++probe, hh = (hh + 1) & mask) {
        const unsigned long long kv = __hip_atomic_load(&D.idx[hh].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((kv == KEY_EMPTY || kv == KEY_TOMB) && atomicCAS(&D.idx[hh].key, kv, key) == kv) break;
      }
      if (probe > mask) {
        atomicOr(&D.st->err, ERR_INDEX);
      } else {
        D.idx[hh].loc = loc;
        Node nd{};
        nd.rem = rem;
        nd.oid = mk.oid;
        nd.uuid = mk.uuid;
        nd.ixs = static_cast<uint32_t>(hh);
        nd.tx = mk.side;
        D.nodes[loc] = nd;
      }
    }
    w += __popcll(sm);
  }
  x.depth = f.dfin;
  x.nlive = f.nlive0 + S;
  x.pad = x.nlive ? l_zero_count(f.z0, f.zpop, zadd) : 0u;
  uint32_t mem = 0;
  if (hd.ok == FL_OK_DEEP) {
    mem = f.memf;
  } else {
    if (((q < 64 ? hd.amask[0] : hd.amask[1]) >> (q & 63)) & 1ull) mem |= M_SALE;
    if (((q < 64 ? hd.bmask[0] : hd.bmask[1]) >> (q & 63)) & 1ull) mem |= M_BUY;
  }
  // a level that ends without makers: no member, or a stale one (Q2, k_fc_stale_level)
  const bool mem_ok = x.nlive > 0 || mem == 0 || mem == f.mfin;
  if (x.nlive == 0) mem = f.mfin;
  x.member = static_cast<uint8_t>(mem);
  if (x.nlive == 0) {
    x.hslot = x.tslot = 0;
  } else if (fresh) {
    x.head = chunk_id(0);
    x.hslot = 0;
    x.tail = chunk_id(need - 1);
    x.tslot = static_cast<uint8_t>(S - (need - 1) * CH);
  } else {
    x.head = f.head;
    x.hslot = static_cast<uint8_t>(f.hslot);
    x.tail = need ? chunk_id(need - 1) : f.tail;
    x.tslot = static_cast<uint8_t>(need ? (S - room) - (need - 1) * CH : s0 + S);
  }
  const bool ok = (x.nlive > 0) == (x.depth > 0) && (x.nlive == 0 || mem == M_BUY || mem == M_SALE) && mem_ok;
  if (!ok && lane == 0) atomicOr(&D.st->err, ERR_CORRUPT);
  return x;
}

__global__ __launch_bounds__(64) void k_fc_write_lv(Dev D, BatchArgs B, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y, q = blockIdx.x;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  if (q == 0 || q > hd.nl) return;
  const Level x = fc_write_level(D, B, F, hd, h, q);
  if (lane_id() == 0) F.lvout[h * FL_CAP + q] = x;
}

// The book: level array compaction and counters (as k_flow_write_fin), DELs and their stats.
__global__ __launch_bounds__(128) void k_fc_fin(Dev D, FlowArgs F) {
  __shared__ Level lv[FL_CAP];
  __shared__ uint32_t keep[FL_CAP];
  __shared__ uint32_t nout_s, base_s, cap_s;
  const uint32_t h = F.h0 + blockIdx.x;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  for (uint32_t q = 1 + threadIdx.x; q <= hd.nl; q += blockDim.x) lv[q] = F.lvout[h * FL_CAP + q];
  __syncthreads();
  fl_write_finish(D, hd, lv, keep, base_s, cap_s, nout_s);
  if (threadIdx.x == 0) {
    ctr_add(D, C_DEL, static_cast<unsigned long long>(hd.ndel));
    if (F.h0 == 0) {
      ctr_add(D, C_FLOW_HEAD_ORDERS, static_cast<unsigned long long>(hd.end - hd.beg));
      ctr_add(D, C_FLOW_HEAD_TOUCHES, static_cast<unsigned long long>(hd.ntouch));
    }
  }
}

// Tail books: one workgroup per book (waves take its levels), then the compaction.
__global__ __launch_bounds__(FL_WRITE_T) void k_fc_write_book(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ Level lv[FL_CAP];
  __shared__ uint32_t keep[FL_CAP];
  __shared__ uint32_t nout_s, base_s, cap_s;
  const uint32_t h = F.h0 + blockIdx.x;
  if (h >= fl_hend(D, F) || !fc_lane(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  const uint32_t w = threadIdx.x >> 6, nw = FL_WRITE_T / 64;
  for (uint32_t q = 1 + w; q <= hd.nl; q += nw) {
    const Level x = fc_write_level(D, B, F, hd, h, uni(q));
    if (lane_id() == 0) lv[q] = x;
  }
  __syncthreads();
  fl_write_finish(D, hd, lv, keep, base_s, cap_s, nout_s);
  if (threadIdx.x == 0) ctr_add(D, C_DEL, static_cast<unsigned long long>(hd.ndel));
}

}  // namespace gome
