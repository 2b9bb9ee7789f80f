// match_cold.h — match_books for cold books: one wavefront per book, book state in HBM.
// Also the HBM path a hot book falls back to when it outgrows the LDS level array.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "pipeline.h"
#include "wave.h"

namespace gome {

// ============================================================== match_books
struct BatchArgs {
  const Prep* prep;           // segment-ordered records
  const gome_order* ord;
  uint32_t n;
  const uint32_t* seg_start;  // [nseg + 1]
  const uint32_t* seg_order;  // launch order (longest first; the first nhot are hot books)
  gome_event* arena;          // per-wave event blocks, compacted afterwards
  uint32_t arena_cap;
  uint32_t* ev_count;         // events per batch index
  const uint32_t* sidx;       // segment position -> batch index (the radix sort's permutation)
  const uint32_t* adm_flag;   // per batch index: admitted ADD (k_adm_flag)
  unsigned long long seq_base;  // sequence number of batch index 0 (published events)
  uint32_t* dup_list;         // batch indices of the ADDs the duplicate-oid rule rejected (Q7)
};

// The Prep record of segment position b built from the input (what k_prep writes to
// prep[b]), for the head's prep which runs before k_prep finishes.
__device__ __forceinline__ Prep prep_at(const BatchArgs& B, uint32_t b) {
  const uint32_t j = B.sidx[b];
  const gome_order o = B.ord[j];
  Prep q;
  q.price = o.price_fx;
  q.vol = o.volume_fx;
  q.oid = o.oid_id;
  q.uuid = o.uuid_id;
  q.idx = j;
  q.side = o.side;
  q.action = o.action;
  q.adm = static_cast<uint8_t>(B.adm_flag[j]);
  q.pad = 0;
  return q;
}

constexpr uint32_t EVB = 32;      // events per arena block (cold books)

// Routing of a batch's books (seg_order is longest first).  The first nhot segments
// (>= 2^FLOW_MIN_LOG2 orders, at most MAX_FLOW) are flow candidates (match_flow.h); a
// candidate the flow path declines goes to the legacy LDS kernel when it has at least
// LEGACY_HOT_MIN orders (match_hot.h), else to the cold kernel below, like every other book.
constexpr uint32_t FLOW_MIN_LOG2 = 7;
constexpr uint32_t MAX_FLOW = 4096;
constexpr uint32_t LEGACY_HOT_MIN = 2048;
constexpr uint32_t MAX_LEGACY = 256;
#ifndef GOME_COLD_BLOCKS
#define GOME_COLD_BLOCKS 128  // half the CUs: the rest stay free for the flow path (plans own whole CUs)
#endif
constexpr uint32_t COLD_BLOCKS = GOME_COLD_BLOCKS;  // persistent cold-kernel blocks
constexpr uint32_t EVB_HOT = 256; // events per arena block (hot books)

// Wave-uniform context of the book being matched.
struct WaveCtx {
  Dev D;
  BatchArgs B;
  uint32_t sym;
  Level* L;          // the book's sorted level array: HBM, or the wave's LDS copy (in_lds)
  uint32_t nl, cap, base;  // cap: entries of L; base / hcap: the book's HBM level block
  uint32_t hcap;
  Level* lds;        // the wave's LDS level slots (COLD_LDS_LVLS), or nullptr
  bool in_lds;
  uint32_t ev_base, ev_used, evb;
  uint32_t flags;    // Book flags (BOOK_QUIRK)
  bool ev_ok, fatal;
  unsigned long long fills, cancels, rests, dropped, adds, dels;
  long long resting_delta, levels_delta;
  // the wave's chunk pool: lane i < npool holds a free chunk id.  Allocations and frees go
  // through it, so the shared free stack / bump pointer / freed list (one cache line of Status
  // that every wave of the grid would otherwise hit once per allocation and per free) see one
  // atomic per CPOOL chunks; the rest goes to the freed list at wave_flush.
  uint32_t cpool, npool;
};
constexpr uint32_t CPOOL = 32;
constexpr uint32_t COLD_SCAN_FROM = 256;  // levels above which do_add's scan starts at the spread

__device__ __forceinline__ void set_err(WaveCtx& W, uint32_t e) {
  if (lane_id() == 0) atomicOr(&W.D.st->err, e);
  W.fatal = true;
}

// Mark the unused tail of the current event block invalid (taker_seq = NIL).
__device__ __forceinline__ void ev_close(WaveCtx& W) {
  if (W.ev_base == NIL || !W.ev_ok) return;
  for (uint32_t j = W.ev_used + lane_id(); j < W.evb; j += 64) W.B.arena[W.ev_base + j].taker_seq = NIL;
}

__device__ __forceinline__ void ev_make_room(WaveCtx& W, uint32_t k) {
  if (W.ev_base != NIL && W.ev_used + k <= W.evb) return;
  const uint32_t lane = lane_id();
  ev_close(W);
  uint32_t b = 0;
  if (lane == 0) b = atomicAdd(&W.D.st->ev_bump, W.evb);
  b = uni(b);
  if (b + W.evb > W.B.arena_cap) {
    W.ev_ok = false;
    if (lane == 0) atomicOr(&W.D.st->err, ERR_EVENTS);
  }
  W.ev_base = b;
  W.ev_used = 0;
}

__device__ __forceinline__ uint32_t alloc_chunk(WaveCtx& W) {
  const uint32_t lane = lane_id();
  if (W.npool == 0) {  // claim CPOOL ids: the free stack first, then the bump pointer
    int t = 0;
    if (lane == 0) t = atomicSub(&W.D.st->free_top, static_cast<int>(CPOOL));
    t = static_cast<int>(uni(static_cast<uint32_t>(t)));
    const uint32_t nst = static_cast<uint32_t>(min(max(t, 0), static_cast<int>(CPOOL)));
    uint32_t b = 0;
    if (lane == 0 && nst < CPOOL) b = atomicAdd(W.D.ch_bump, CPOOL - nst);
    b = uni(b);
    if (lane < CPOOL)
      W.cpool = (lane < nst) ? W.D.free_ids[t - static_cast<int>(nst) + static_cast<int>(lane)] : b + (lane - nst);
    W.npool = CPOOL;
  }
  W.npool--;
  const uint32_t c = rl(W.cpool, W.npool);
  if (c >= W.D.ch_cap) { set_err(W, ERR_CHUNKS); return NIL; }
  return c;
}

// Pool ids lanes [lo, hi) -> the batch's freed list (recycled after the batch by k_recycle_*);
// ids past the pool's capacity (a bump claim that overshot it) are dropped.
__device__ __forceinline__ void pool_publish(WaveCtx& W, uint32_t lo, uint32_t hi) {
  const uint32_t lane = lane_id();
  const bool ok = lane >= lo && lane < hi && W.cpool < W.D.ch_cap;
  const unsigned long long m = __ballot(ok);
  if (!m) return;
  uint32_t b = 0;
  if (lane == 0) b = atomicAdd(&W.D.st->freed_top, static_cast<uint32_t>(__popcll(m)));
  b = uni(b);
  if (ok) W.D.freed_ids[b + __popcll(m & lt_mask())] = W.cpool;
}

// A chunk no FIFO references any more (its nodes are consumed, cancelled or erased from the
// index): back to the wave's pool, reused by its next allocation.
__device__ __forceinline__ void free_chunk(WaveCtx& W, uint32_t c) {
  if (W.npool == 64) {
    pool_publish(W, 32, 64);
    W.npool = 32;
  }
  if (lane_id() == W.npool) W.cpool = c;
  W.npool++;
}

__device__ __forceinline__ void free_chain(WaveCtx& W, uint32_t head, uint32_t tail) {
  uint32_t c = head;
  for (uint32_t guard = 0; c != NIL; ++guard) {
    if (guard > W.D.ch_cap) { set_err(W, ERR_CORRUPT); return; }
    uint32_t nx = (c == tail) ? NIL : uni(W.D.chdr[c].next);
    free_chunk(W, c);
    c = nx;
  }
}

// ---- level array (sorted by price) --------------------------
// Lower bound of p with a 64-ary wave search; returns true iff L[pos].price == p.
__device__ __forceinline__ bool level_search_in(const Level* L, uint32_t nl, int64_t p, uint32_t& pos) {
  const uint32_t lane = lane_id();
  uint32_t lo = 0, hi = nl;
  while (hi - lo > 64) {
    uint32_t step = (hi - lo + 63) / 64;
    uint32_t q = lo + lane * step;
    bool v = q < hi;
    int64_t pr = v ? L[q].price : 0;
    uint32_t ns = __popcll(__ballot(v));
    uint32_t cnt = __popcll(__ballot(v && pr < p));
    uint32_t nlo = cnt ? lo + (cnt - 1) * step + 1 : lo;
    uint32_t nhi = (cnt < ns) ? lo + cnt * step + 1 : hi;
    lo = nlo;
    hi = nhi;
  }
  uint32_t q = lo + lane;
  bool v = q < hi;
  int64_t pr = v ? L[q].price : 0;
  pos = lo + __popcll(__ballot(v && pr < p));
  return __ballot(v && pr == p) != 0;
}

__device__ __forceinline__ bool level_search(const WaveCtx& W, int64_t p, uint32_t& pos) {
  return level_search_in(W.L, W.nl, p, pos);
}

// Drop levels with no observable state (no nodes, zero depth, no side membership);
// equivalent to a never-touched price in the Redis schema.
__device__ __forceinline__ void level_gc(WaveCtx& W) {
  const uint32_t lane = lane_id();
  const unsigned long long ltm = lt_mask();
  uint32_t out = 0;
  for (uint32_t w0 = 0; w0 < W.nl; w0 += 64) {
    uint32_t k = w0 + lane;
    bool keep = false;
    Level x{};
    if (k < W.nl) {
      x = W.L[k];
      keep = x.nlive != 0 || x.depth != 0 || x.member != 0;
    }
    unsigned long long m = __ballot(keep);
    if (keep) W.L[out + __popcll(m & ltm)] = x;
    out += __popcll(m);
  }
  W.levels_delta -= static_cast<long long>(W.nl - out);
  W.nl = out;
}

// The book's levels held in LDS go (back) to an HBM block of at least `need` entries.
__device__ __forceinline__ bool level_spill(WaveCtx& W, uint32_t need) {
  const uint32_t lane = lane_id();
  uint32_t base = W.base, cap = W.hcap;
  if (need > cap) {
    uint32_t ncap = 16;
    while (ncap < need) ncap <<= 1;
    uint32_t nb = 0;
    if (lane == 0) nb = lvl_block_alloc(W.D, ncap);
    nb = uni(nb);
    if (nb == NIL) {
      set_err(W, ERR_LEVELS);
      return false;
    }
    if (lane == 0) lvl_block_release(W.D, W.base, W.hcap);  // reusable from the next batch on
    base = nb;
    cap = ncap;
  }
  Level* H = W.D.lvl + base;
  for (uint32_t k = lane; k < W.nl; k += 64) H[k] = W.L[k];
  W.base = base;
  W.hcap = cap;
  W.L = H;
  W.cap = cap;
  W.in_lds = false;
  return true;
}

__device__ __forceinline__ bool level_grow(WaveCtx& W) {
  if (W.in_lds) return level_spill(W, 2 * W.nl);
  const uint32_t lane = lane_id();
  uint32_t ncap = W.cap ? W.cap * 2 : 16;
  uint32_t nb = 0;
  if (lane == 0) nb = lvl_block_alloc(W.D, ncap);
  nb = uni(nb);
  if (nb == NIL) {
    set_err(W, ERR_LEVELS);
    return false;
  }
  Level* NL = W.D.lvl + nb;
  for (uint32_t w0 = 0; w0 < W.nl; w0 += 64) {
    uint32_t k = w0 + lane;
    if (k < W.nl) NL[k] = W.L[k];
  }
  if (lane == 0) lvl_block_release(W.D, W.base, W.cap);  // reusable from the next batch on
  W.L = NL;
  W.cap = ncap;
  W.hcap = ncap;
  W.base = nb;
  return true;
}

// Insert an empty level for price p at lower-bound position pos (updated on GC).
__device__ __forceinline__ bool level_insert(WaveCtx& W, int64_t p, uint32_t& pos) {
  const uint32_t lane = lane_id();
  if (W.nl == W.cap) {
    if (W.nl) {
      level_gc(W);
      level_search(W, p, pos);
    }
    if (W.nl == W.cap && !level_grow(W)) return false;
  }
  for (int32_t top = static_cast<int32_t>(W.nl); top > static_cast<int32_t>(pos); top -= 64) {
    int32_t lo = max(top - 64, static_cast<int32_t>(pos));
    int32_t k = lo + static_cast<int32_t>(lane);
    if (k < top) {
      Level x = W.L[k];
      W.L[k + 1] = x;
    }
  }
  if (lane == 0) {
    Level z{};
    z.price = p;
    z.head = z.tail = NIL;
    W.L[pos] = z;
  }
  W.nl++;
  W.levels_delta++;
  return true;
}

// ---- (S, oid) -> node index (stands in for HGET S:link:<p> S:node:<oid>) -------
__device__ __forceinline__ unsigned long long idx_key(uint32_t sym, uint32_t oid) {
  return (static_cast<unsigned long long>(sym + 1) << 32) | oid;
}

__device__ __forceinline__ uint32_t idx_insert(WaveCtx& W, uint32_t oid, uint32_t loc) {
  const uint32_t lane = lane_id();
  const unsigned long long key = idx_key(W.sym, oid), mask = W.D.idx_mask;
  unsigned long long h = mix64(key) & mask;
  for (unsigned long long probe = 0; probe <= mask; probe += 64) {
    const unsigned long long slot = (h + lane) & mask;
    unsigned long long kv =
        __hip_atomic_load(&W.D.idx[slot].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long cand = __ballot(kv == KEY_EMPTY || kv == KEY_TOMB);
    while (cand) {
      uint32_t b = __builtin_ctzll(cand);
      bool ok = false;
      if (lane == b) {
        unsigned long long exp = kv;
        ok = atomicCAS(&W.D.idx[slot].key, exp, key) == exp;
        if (ok) W.D.idx[slot].loc = loc;
      }
      if (__ballot(ok)) return static_cast<uint32_t>((h + b) & mask);
      cand &= cand - 1;
    }
    h = (h + 64) & mask;
  }
  set_err(W, ERR_INDEX);
  return NIL;
}

__device__ __forceinline__ bool idx_lookup(const WaveCtx& W, uint32_t oid, uint32_t& ixslot, uint32_t& loc) {
  const uint32_t lane = lane_id();
  const unsigned long long key = idx_key(W.sym, oid), mask = W.D.idx_mask;
  unsigned long long h = mix64(key) & mask;
  for (unsigned long long probe = 0; probe <= mask; probe += 64) {
    const unsigned long long slot = (h + lane) & mask;
    unsigned long long kv =
        __hip_atomic_load(&W.D.idx[slot].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long hit = __ballot(kv == key), emp = __ballot(kv == KEY_EMPTY);
    unsigned long long any = hit | emp;
    if (any) {
      uint32_t b = __builtin_ctzll(any);
      if (!((hit >> b) & 1ull)) return false;
      uint32_t lc = (lane == b) ? W.D.idx[slot].loc : 0;
      loc = __shfl(lc, b);
      ixslot = static_cast<uint32_t>((h + b) & mask);
      return true;
    }
    h = (h + 64) & mask;
  }
  return false;
}

__device__ __forceinline__ void idx_erase(WaveCtx& W, uint32_t ixslot) {
  __hip_atomic_store(&W.D.idx[ixslot].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- MatchOrder at one level (engine.go:138-198) --------------------------------
// Consumes the FIFO head of level k for a taker with remaining T.  Lanes 0..31 hold the
// head chunk, lanes 32..63 the next chunk (for MatchNode.NextNode).  Per chunk, a prefix
// scan over live volumes decides which makers are reached (reference recursion continues
// while diff > 0), fully filled (diff >= 0) or partially filled (diff < 0).
__device__ __forceinline__ int64_t match_level(WaveCtx& W, uint32_t k, int64_t T, uint32_t seq, uint32_t& fidx) {
  const uint32_t lane = lane_id(), s = lane & 31u;
  const bool hi = lane >= 32;
  Level lv = W.L[k];
  bool first = true;
  for (uint32_t guard = 0; lv.head != NIL && !W.fatal; ++guard) {
    if (guard > W.D.ch_cap) { set_err(W, ERR_CORRUPT); break; }
    const uint32_t head = lv.head;
    const uint32_t nxt = uni(W.D.chdr[head].next);
    const uint32_t cid = hi ? nxt : head;
    int64_t r = -1;
    uint32_t o = 0, u = 0, ix = 0, t = 0;
    bool inr = false;
    if (cid != NIL) {
      uint32_t lim = (cid == lv.tail) ? lv.tslot : CH;
      uint32_t lo = hi ? 0u : lv.hslot;
      inr = s >= lo && s < lim;
    }
    if (inr) {
      const Node nd = W.D.nodes[cid * CH + s];
      r = nd.rem;
      o = nd.oid;
      u = nd.uuid;
      ix = nd.ixs;
      t = nd.tx;
    }
    const bool live = inr && r >= 0;
    const unsigned long long lm = __ballot(live);
    const uint32_t mlo = static_cast<uint32_t>(lm), mhi = static_cast<uint32_t>(lm >> 32);
    if (mlo == 0) {  // head chunk exhausted (consumed/cancelled slots only)
      if (head == lv.tail) { set_err(W, ERR_CORRUPT); break; }
      free_chunk(W, head);
      lv.head = nxt;
      lv.hslot = 0;
      continue;
    }
    const int64_t x = (!hi && live) ? r : 0;
    const int64_t incl = wave_incl_scan(x);
    const int64_t excl = incl - x;
    const uint32_t fl = __builtin_ctz(mlo);
    const bool arr = !hi && live && (excl < T || (first && T == 0 && s == fl));
    const bool pop = arr && incl <= T;
    const int64_t f = pop ? r : (T - excl);
    const unsigned long long am = __ballot(arr), pm = __ballot(pop);
    const uint32_t narr = __popcll(am), npop = __popcll(pm);
    const uint32_t la = 63 - __builtin_clzll(am);
    // MatchNode.NextNode / IsLast: next live node after s in FIFO order.
    const uint32_t after = (s < 31) ? (mlo & (~0u << (s + 1))) : 0u;
    int src = after ? static_cast<int>(__builtin_ctz(after))
                    : (mhi ? 32 + static_cast<int>(__builtin_ctz(mhi)) : -1);
    uint32_t nx_oid = __shfl(o, src < 0 ? 0 : src);
    bool is_last = src < 0;
    const uint32_t ll = 31 - __clz(mlo);  // last live slot of the head chunk
    if (!mhi && nxt != NIL && ((am >> ll) & 1ull)) {
      // next chunk is all tombstones: search further down the chain
      uint32_t c2 = uni(W.D.chdr[nxt].next);
      for (uint32_t guard = 0; c2 != NIL && guard <= W.D.ch_cap; ++guard) {
        uint32_t lim = (c2 == lv.tail) ? lv.tslot : CH;
        bool l2 = lane < lim && W.D.nodes[c2 * CH + (lane < CH ? lane : 0)].rem >= 0;
        unsigned long long m2 = __ballot(l2);
        if (m2) {
          uint32_t b = __builtin_ctzll(m2);
          uint32_t oo = W.D.nodes[c2 * CH + b].oid;
          if (lane == ll) { nx_oid = oo; is_last = false; }
          break;
        }
        c2 = (c2 == lv.tail) ? NIL : uni(W.D.chdr[c2].next);
      }
    }
    const int64_t tafter = T - excl - f;
    const int64_t dafter = lv.depth - excl - f;
    const bool clr = arr && dafter <= 0;  // DeletePoolDepth: ZREM maker's side (nodepool.go:76-83)
    const unsigned long long clr_s = __ballot(clr && t == GOME_SALE), clr_b = __ballot(clr && t != GOME_SALE);
    // publish (engine.go:154,171,190)
    ev_make_room(W, narr);
    if (arr && W.ev_ok) {
      uint32_t rank = __popcll(am & lt_mask());
      gome_event e;
      e.price_fx = lv.price;
      e.match_volume_fx = f;
      e.maker_volume_fx = pop ? r : r - f;
      e.taker_seq = seq;
      e.fill_idx = fidx + rank;
      e.maker_oid_id = o;
      e.maker_uuid_id = u;
      e.maker_next_oid_id = is_last ? 0u : nx_oid;
      e.kind = GOME_EV_FILL;
      e.maker_side = static_cast<uint8_t>(t);
      e.maker_is_last = is_last ? 1 : 0;
      e.pad0 = 0;
      W.B.arena[W.ev_base + W.ev_used + rank] = e;
    }
    W.ev_used += narr;
    fidx += narr;
    W.fills += narr;
    const int64_t Tn = rl64(tafter, la);
    lv.depth -= (T - Tn);
    if (clr_s) lv.member &= static_cast<uint8_t>(~M_SALE);
    if (clr_b) lv.member &= static_cast<uint8_t>(~M_BUY);
    if (pop) idx_erase(W, ix);
    lv.nlive -= npop;
    W.resting_delta -= npop;
    first = false;
    if (!((pm >> la) & 1ull)) {  // partial fill of maker la: it keeps its FIFO position
      if (lane == la) W.D.nodes[head * CH + s].rem = r - f;
      lv.hslot = static_cast<uint8_t>(la);
      T = 0;
      break;
    }
    T = Tn;
    lv.hslot = static_cast<uint8_t>(la + 1);
    if (lv.nlive == 0) {
      free_chain(W, lv.head, lv.tail);
      lv.head = lv.tail = NIL;
      lv.hslot = lv.tslot = 0;
      break;
    }
    if (T <= 0) break;  // diff == 0: stop (engine.go:162-175)
    // every live maker of the head chunk consumed, T > 0: continue down the FIFO
    free_chunk(W, head);
    lv.head = nxt;
    lv.hslot = 0;
  }
  if (lane == 0) W.L[k] = lv;
  return T;
}

// ---- rest the remaining volume (engine.go:80-82) ----------------------------------
__device__ __forceinline__ void do_rest(WaveCtx& W, int64_t p, int64_t T, uint32_t oid, uint32_t uuid,
                        uint32_t side) {
  const uint32_t lane = lane_id();
  uint32_t pos;
  if (!level_search(W, p, pos) && !level_insert(W, p, pos)) return;
  Level lv = W.L[pos];
  lv.member |= (side == GOME_SALE) ? M_SALE : M_BUY;  // SetPoolDepth (ZADD own side)
  lv.depth += T;                                       // SetPoolDepthVolume
  if (lv.tail == NIL || lv.tslot == CH) {              // SetDepthLink: append at the tail
    uint32_t c = alloc_chunk(W);
    if (c == NIL) return;
    if (lane == 0) {
      W.D.chdr[c].next = NIL;
      W.D.chdr[c].price = p;
      if (lv.tail != NIL) W.D.chdr[lv.tail].next = c;
    }
    if (lv.tail == NIL) { lv.head = c; lv.hslot = 0; }
    lv.tail = c;
    lv.tslot = 0;
  }
  const uint32_t slot = lv.tslot, loc = lv.tail * CH + slot;
  if (T == 0) W.flags |= BOOK_QUIRK;  // zero-volume maker (Q6)
  const uint32_t ix = idx_insert(W, oid, loc);
  if (lane == 0) {
    Node* d = &W.D.nodes[loc];
    st16_glb(d, v4(lo32(T), hi32(T), oid, uuid));
    st16_glb(reinterpret_cast<char*>(d) + 16, v4(ix, side & 0xFFu, 0u, 0u));
  }
  lv.tslot = static_cast<uint8_t>(slot + 1);
  lv.nlive++;
  if (lane == 0) W.L[pos] = lv;
  W.rests++;
  W.resting_delta++;
}

// ---- SetOrder (engine.go:56-85) -------------------------------------------------
__device__ __forceinline__ uint32_t do_add(WaveCtx& W, int64_t p, int64_t vol, uint32_t oid, uint32_t uuid,
                           uint32_t side, uint32_t seq) {
  const uint32_t lane = lane_id();
  const bool sale = side == GOME_SALE;
  const uint8_t opp = sale ? M_BUY : M_SALE;
  int64_t T = vol;
  bool crossed = false;
  uint32_t fidx = 0;
  // GetReverseDepth (nodepool.go:86-115): opposite-side levels crossing p, best first.  In a
  // book without quirks or stale members every bid is below every ask (a rest follows a complete sweep), so on a
  // deep book the scan starts just above the highest bid <= p (BUY) or just below the lowest
  // ask >= p (SALE) instead of walking the book's other side from its far end.
  uint32_t up0 = 0;
  int32_t dn0 = static_cast<int32_t>(W.nl);
  if (!(W.flags & (BOOK_QUIRK | BOOK_STALE)) && W.nl > COLD_SCAN_FROM) {
    uint32_t pos;
    const bool at = level_search(W, p, pos);
    if (!sale) {
      for (int32_t hi = static_cast<int32_t>(pos + (at ? 1u : 0u)); hi > 0; hi -= 64) {
        const int32_t lo = max(hi - 64, 0), k = lo + static_cast<int32_t>(lane);
        const bool v = k < hi;
        const unsigned long long bm = __ballot(v && (W.L[v ? k : 0].member & M_BUY));
        if (bm) {
          up0 = static_cast<uint32_t>(lo) + 64u - static_cast<uint32_t>(__builtin_clzll(bm));
          break;
        }
      }
    } else {
      for (uint32_t w0 = pos; w0 < W.nl; w0 += 64) {
        const uint32_t k = w0 + lane;
        const bool v = k < W.nl;
        const unsigned long long am = __ballot(v && (W.L[v ? k : 0].member & M_SALE));
        if (am) {
          dn0 = static_cast<int32_t>(w0 + static_cast<uint32_t>(__builtin_ctzll(am)));
          break;
        }
      }
    }
  }
  if (!sale) {
    for (uint32_t w0 = up0; w0 < W.nl && !W.fatal; w0 += 64) {
      const uint32_t k = w0 + lane;
      const bool v = k < W.nl;
      int64_t lp = 0;
      uint8_t mem = 0;
      if (v) { lp = W.L[k].price; mem = W.L[k].member; }
      unsigned long long cm = __ballot(v && (mem & opp) && lp <= p);
      const bool beyond = __ballot(v && lp > p) != 0;
      while (cm && !W.fatal) {
        const uint32_t kk = w0 + __builtin_ctzll(cm);
        cm &= cm - 1;
        crossed = true;
        T = match_level(W, kk, T, seq, fidx);  // Match (engine.go:118-136)
        if (T <= 0) goto matched;
      }
      if (beyond) break;
    }
  } else {
    for (int32_t top = dn0; top > 0 && !W.fatal; top -= 64) {
      const int32_t lo = top - 64, k = lo + static_cast<int32_t>(lane);
      const bool v = k >= 0;
      int64_t lp = 0;
      uint8_t mem = 0;
      if (v) { lp = W.L[k].price; mem = W.L[k].member; }
      unsigned long long cm = __ballot(v && (mem & opp) && lp >= p);
      const bool beyond = __ballot(v && lp < p) != 0;
      while (cm && !W.fatal) {
        const uint32_t b = 63 - __builtin_clzll(cm);
        cm &= ~(1ull << b);
        crossed = true;
        T = match_level(W, static_cast<uint32_t>(lo + static_cast<int32_t>(b)), T, seq, fidx);
        if (T <= 0) goto matched;
      }
      if (beyond) break;
    }
  }
matched:
  if ((!crossed || T > 0) && !W.fatal) do_rest(W, p, T, oid, uuid, side);
  return fidx;
}

// ---- DeleteOrder (engine.go:87-116) ---------------------------------------------
__device__ __forceinline__ uint32_t do_cancel(WaveCtx& W, int64_t p, uint32_t oid, uint32_t uuid, uint32_t side,
                              uint32_t seq) {
  const uint32_t lane = lane_id();
  uint32_t ixslot, loc;
  if (!idx_lookup(W, oid, ixslot, loc)) return 0;    // not in any FIFO: no event
  const uint32_t cid = loc / CH, s = loc % CH;
  if (uni(static_cast<uint32_t>(W.D.chdr[cid].price != p))) return 0;  // wrong price (Q3)
  const int64_t r = rl64(W.D.nodes[cid * CH + s].rem, 0);
  const uint32_t ntx = uni(static_cast<uint32_t>(W.D.nodes[cid * CH + s].tx));
  if ((ntx == GOME_SALE) != (side == GOME_SALE)) W.flags |= BOOK_QUIRK;  // wrong-side cancel (Q2)
  uint32_t pos;
  if (r < 0 || !level_search(W, p, pos)) { set_err(W, ERR_CORRUPT); return 0; }
  Level lv = W.L[pos];
  lv.depth -= r;  // DeletePoolDepthVolume with the stored remaining volume
  if (lv.depth <= 0) lv.member &= static_cast<uint8_t>(~((side == GOME_SALE) ? M_SALE : M_BUY));
  if (lane == 0) W.D.nodes[cid * CH + s].rem = -1;
  if (lane == 0) idx_erase(W, ixslot);
  lv.nlive--;
  W.resting_delta--;
  if (lv.nlive == 0) {
    free_chain(W, lv.head, lv.tail);
    lv.head = lv.tail = NIL;
    lv.hslot = lv.tslot = 0;
  }
  if (lane == 0) W.L[pos] = lv;
  ev_make_room(W, 1);
  if (lane == 0 && W.ev_ok) {
    gome_event e;
    e.price_fx = p;
    e.match_volume_fx = 0;
    e.maker_volume_fx = r;
    e.taker_seq = seq;
    e.fill_idx = 0;
    e.maker_oid_id = oid;
    e.maker_uuid_id = uuid;
    e.maker_next_oid_id = 0;
    e.kind = GOME_EV_CANCEL;
    e.maker_side = static_cast<uint8_t>(side);
    e.maker_is_last = 1;
    e.pad0 = 0;
    W.B.arena[W.ev_base + W.ev_used] = e;
  }
  W.ev_used += 1;
  W.cancels++;
  return 1;
}

// Apply orders [b0, end) of the book in W (HBM-resident level array).
__device__ __forceinline__ void process_global(WaveCtx& W, uint32_t b0, uint32_t end) {
  const uint32_t lane = lane_id();
  for (; b0 < end && !W.fatal; b0 += 64) {
    const uint32_t cnt = min(64u, end - b0);
    Prep q{};
    if (lane < cnt) q = W.B.prep[b0 + lane];  // 64 records of this book, one per lane
    for (uint32_t j = 0; j < cnt && !W.fatal; ++j) {
      const uint32_t idx = rl(q.idx, j), a = rl(q.action, j);
      uint32_t nev = 0;
      if (a == GOME_ADD) {
        W.adds++;
        const uint32_t adm = rl(q.adm, j);
        uint32_t ixs, loc;
        if (adm == ADM_V_CHECK && idx_lookup(W, rl(q.oid, j), ixs, loc)) {
          W.dropped++;  // (S, oid) names a live node: the duplicate-oid rule (Q7, pipeline.h)
          if (lane == 0) dup_note(W.D.st, W.B.dup_list, idx);
        } else if (adm != ADM_V_NO) {
          nev = do_add(W, rl64(q.price, j), rl64(q.vol, j), rl(q.oid, j), rl(q.uuid, j), rl(q.side, j), idx);
        } else {
          W.dropped++;  // marker already consumed (engine.go:58-60)
        }
      } else if (a == GOME_DEL) {
        W.dels++;
        nev = do_cancel(W, rl64(q.price, j), rl(q.oid, j), rl(q.uuid, j), rl(q.side, j), idx);
      }
      if (lane == 0) W.B.ev_count[idx] = nev;
    }
  }
}

__device__ __forceinline__ void wave_flush(WaveCtx& W);

// The book's record; with `flush` also the wave's counters (a persistent cold wave keeps them
// across its books and flushes once, see k_match).
__device__ __forceinline__ void wave_finish(WaveCtx& W, bool flush = true) {
  const uint32_t lane = lane_id();
  if (W.in_lds) level_spill(W, W.nl);
  if (lane == 0) {
    Book nb;
    nb.lvl_base = W.base;
    nb.n_lvl = W.nl;
    nb.lvl_cap = W.hcap;
    nb.pad = W.flags;
    W.D.books[W.sym] = nb;
    if (W.flags & BOOK_QUIRK) quirk_note(W.D, W.sym);  // (k_requalify)
  }
  if (flush) wave_flush(W);
}

__device__ __forceinline__ void wave_flush(WaveCtx& W) {
  ev_close(W);
  pool_publish(W, 0, W.npool);
  W.npool = 0;
  if (lane_id() == 0) {
    if (W.fills) ctr_add(W.D, C_FILLS, W.fills);
    if (W.cancels) ctr_add(W.D, C_CANCELS, W.cancels);
    if (W.rests) ctr_add(W.D, C_RESTS, W.rests);
    if (W.dropped) ctr_add(W.D, C_DROPPED, W.dropped);
    if (W.adds) ctr_add(W.D, C_ADD, W.adds);
    if (W.dels) ctr_add(W.D, C_DEL, W.dels);
    if (W.resting_delta) ctr_add(W.D, C_RESTING_DELTA, static_cast<unsigned long long>(W.resting_delta));
    if (W.levels_delta) ctr_add(W.D, C_LEVELS_DELTA, static_cast<unsigned long long>(W.levels_delta));
  }
}

// The next book of a wave: its state, the event block continues (a persistent cold wave keeps
// one partly filled block and its counters across books).
// Cold books with few levels work on an LDS copy of their level array (every level search,
// insert and update is then an LDS access instead of an HBM round trip); written back by
// wave_finish.
#ifndef GOME_COLD_LDS_LVLS
#define GOME_COLD_LDS_LVLS 128
#endif
constexpr uint32_t COLD_LDS_LVLS = GOME_COLD_LDS_LVLS;

__device__ __forceinline__ void wave_next_book(WaveCtx& W, uint32_t sym) {
  W.sym = sym;
  const Book bk = W.D.books[sym];
  W.base = uni(bk.lvl_base);
  W.nl = uni(bk.n_lvl);
  W.cap = W.hcap = uni(bk.lvl_cap);
  W.flags = uni(bk.pad);
  if (W.flags & BOOK_ZERO) W.flags |= BOOK_QUIRK;  // (its levels' L_ZERO marks: k_requalify's to redo)
  W.L = W.D.lvl + W.base;
  W.in_lds = W.lds != nullptr && W.nl <= COLD_LDS_LVLS;
  if (W.in_lds) {
    for (uint32_t k = lane_id(); k < W.nl; k += 64) W.lds[k] = W.L[k];
    W.L = W.lds;
    W.cap = COLD_LDS_LVLS;
  }
}

__device__ __forceinline__ void wave_init(WaveCtx& W, const Dev& D, const BatchArgs& B, uint32_t sym, uint32_t evb,
                                          Level* lds = nullptr) {
  W.D = D;
  W.B = B;
  W.lds = lds;
  wave_next_book(W, sym);
  W.ev_base = NIL;
  W.ev_used = 0;
  W.evb = evb;
  W.ev_ok = true;
  W.fatal = false;
  W.fills = W.cancels = W.rests = W.dropped = W.adds = W.dels = 0;
  W.resting_delta = W.levels_delta = 0;
  W.cpool = NIL;
  W.npool = 0;
}

// Cold books: one wavefront per book, state in HBM.  Wave w of the grid takes books
// seg_order[w], seg_order[w + waves], ...; flow candidates are skipped unless the flow path
// declined them and they are too short for the legacy hot kernel (`flow_ok[i]`: FlowHdr::ok
// of candidate i).  Every step of a cold book is a dependent HBM round trip, so the kernel
// needs many waves in flight: COLD_WAVES per workgroup on at most COLD_BLOCKS workgroups
// (fewer workgroups than CUs leaves whole CUs free for the flow plans' one-block-per-CU
// kernels, launched later).  A wave keeps its event block and its counters across books.
#ifndef GOME_COLD_WAVES
#define GOME_COLD_WAVES 8
#endif
constexpr uint32_t COLD_WAVES = GOME_COLD_WAVES;
constexpr uint32_t COLD_LDS_BYTES = COLD_WAVES * COLD_LDS_LVLS * sizeof(Level);
__global__ __launch_bounds__(64 * COLD_WAVES) void k_match(Dev D, BatchArgs B, const uint32_t* flow_ok, uint32_t ok_stride) {
  if (D.st->err & ERR_INPUT) return;
  const uint32_t nseg = D.st->nseg, nhot = D.st->nhot;
  const uint32_t nw = blockDim.x >> 6, stride = gridDim.x * nw;
  extern __shared__ Level lvl_lds[];  // COLD_WAVES x COLD_LDS_LVLS (dynamic: COLD_LDS_BYTES)
  WaveCtx W;
  bool started = false;
  for (uint32_t i = blockIdx.x * nw + (threadIdx.x >> 6); i < nseg; i += stride) {
    const uint32_t seg = B.seg_order[i];
    const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
    if (i < nhot && (flow_ok[i * ok_stride] || (end - beg >= LEGACY_HOT_MIN && i < MAX_LEGACY))) continue;
    const uint32_t sym = uni(B.ord[B.prep[beg].idx].symbol_id);
    if (!started) {
      wave_init(W, D, B, sym, EVB, lvl_lds + (threadIdx.x >> 6) * COLD_LDS_LVLS);
      started = true;
    } else {
      wave_next_book(W, sym);
    }
    process_global(W, beg, end);
    wave_finish(W, false);
    if (W.fatal) break;
  }
  if (started) wave_flush(W);
}


}  // namespace gome
