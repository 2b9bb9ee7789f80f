// match_hot.h — match_books for hot books (the Zipf head of the batch).
//
// A book whose segment holds >= 2^HOT_MIN_LOG2 orders is applied by k_match_hot: one
// wavefront per book, one workgroup per CU (~142 KiB of LDS), s_setprio 3.  A hot book
// is the batch's critical path: one wavefront must apply its orders one after another
// (the reference's serial consumer, rabbitmq.go:116), so what bounds it is the LATENCY of
// one lone wave per order.  Measured lone-wave costs on gfx950: ~4-5 cycles
// per instruction, +20 per VALU->SALU hand-off, 20 per taken branch, 60 per LDS round
// trip, ~730 per returning global atomic.  The design follows from those numbers:
//
//  * Level i (ascending price, up to LRB_CAP = 128) lives in lane i % 64 of register set
//    i / 64: price, depth, FIFO head/tail chunk, slots, live count, and — once the level is
//    "resident" — its HEAD NODE (remaining volume, oid, uuid, index slot, side), the oid of
//    the next live node (MatchNode.NextNode) and the live-slot mask of the head chunk,
//    whose 1 KiB is cached in LDS.  Side-set membership (S:BUY / S:SALE) is kept as 64-bit
//    SGPR masks.
//  * GetReverseDepth (nodepool.go:86-115) = one 64-bit compare per register set ANDed with
//    a membership mask; levels are visited best-first by bit scans.
//  * MatchOrder (engine.go:138-198) works on the head registers: a partial fill
//    (diff < 0) touches no memory but the event store; a full fill (diff >= 0) pops the
//    head and fetches the next one from the cached chunk with one LDS round trip.
//  * Level updates are v_writelane (no exec masking); single-lane stores (events, nodes)
//    are asm blocks that set exec to lane 0 (no branch, no hand-off).
//  * Chunk allocation and release go through wave-local pools in LDS, refilled / flushed
//    32 at a time, so no returning atomic sits on the per-order path.
//  * Cancel-index inserts of rested nodes are deferred (one 16-B PendEnt per rest):
//    flushed lane-parallel before a cancel's lookup, otherwise applied by k_pend_apply.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "match_cold.h"
#include "match_flow.h"
#include "wave.h"

namespace gome {

// Diagnostic build only (-DGOME_STAMPS): s_memtime cycle sums per phase, accumulated in
// LDS by lane 0 (no SGPR cost), copied to g_stamps at the end; read with gome_debug_stamps.
#ifndef GOME_EXPERIMENT
#define GOME_EXPERIMENT 0
#endif
#ifdef GOME_STAMPS
constexpr int NSTAMP = 16;
__device__ unsigned long long g_stamps[256 * NSTAMP];
#define ST_T0(v) const unsigned long long v = __builtin_amdgcn_s_memtime();
#define ST_ADD(i, v) st_add(H.S, i, __builtin_amdgcn_s_memtime() - (v));
#else
#define ST_T0(v)
#define ST_ADD(i, v)
#endif

constexpr uint32_t MAX_HOT = MAX_LEGACY;  // legacy hot kernel grid (see match_cold.h)
constexpr uint32_t LRB_CAP = 128;  // levels held in lanes (2 register sets)
constexpr uint32_t NCS = LRB_CAP;  // one head-chunk cache slot per resident level
constexpr uint32_t CS_NONE = 0xFFu;
constexpr uint32_t PEND = 0x80000000u;  // Node::ixs flag: index insert still pending
constexpr uint32_t POOL = 32;           // chunk ids claimed per refill
constexpr uint32_t FREED = 64;          // freed chunk ids buffered before a flush
constexpr int64_t PR_NONE = 0x7FFFFFFFFFFFFFFFll;  // price of an unused lane (never matches)
enum : uint32_t { HN_UNKNOWN = 0, HN_OID = 1, HN_NONE = 2 };

// One price level of a hot book, resident in LDS (80 B = five 16-B quads, written back
// quad by quad).  Only price and side-set membership are mirrored in lane registers (the
// crossing and find ballots); everything else is read with one broadcast LDS load.
//   sl packs hslot [0,8) (head node slot when resident, else first unconsumed slot),
//   tslot [8,16), cache slot [16,24) (CS_NONE: not resident), next-node state [24,26).
//   hrem/hoid/huuid/hix/hx describe the head node and hnx its successor (MatchNode.NextNode)
//   while the level is resident (its head chunk cached in LDS).
struct LvRec {
  int64_t pr, dp;                  // q0
  int64_t hrem;                    // q1
  uint32_t hoid, huuid;
  uint32_t hd, tl, hn, nv;         // q2
  uint32_t sl, live, hix, hx;      // q3
  uint32_t hnx, mem, pad1, pad2;   // q4 (mem: membership, only while staging)
};
static_assert(sizeof(LvRec) == 80, "LvRec is five 16-B quads");

// A hot book that continues on the HBM path (deep book, or lane array full).
struct ResumeRec {
  uint32_t valid, next;
  uint32_t rest, oid, uuid, side, pad0, pad1;
  int64_t price, vol;
};
static_assert(sizeof(ResumeRec) == 48, "ResumeRec is written as three 16-B stores");

// Pointers and sizes the per-order path needs only rarely: kept in LDS (read uniformly
// when used) instead of SGPRs, so the per-order state fits the SGPR file without spills.
struct HotEnv {
  Status* st;
  IdxEnt* idx;
  unsigned long long idx_mask;
  uint32_t* free_ids;
  uint32_t* freed_ids;
  uint32_t* ch_bump;
  const Prep* prep;
  uint32_t* ev_count;
  Book* books;
  Level* lvl;
  uint32_t* lvl_bump;
  ResumeRec* resume;
  LvlPool lpool;
  uint32_t* dup_list;  // (BatchArgs::dup_list)
  uint32_t ch_cap, arena_cap, lvl_cap_total, lvl_base, lvl_cap, beg, end, pad;
};

struct HotLds {
  Node cs[NCS][CH];                 // cached head chunks (authoritative while cached)
  LvRec lv[LRB_CAP];
  alignas(16) uint32_t cs_chunk[NCS];  // chunk held by each cache slot (NIL = free)
  uint32_t pool[POOL];              // claimed, unused chunk ids
  uint32_t freed[FREED];            // released chunk ids not yet published
  HotEnv env;
  uint32_t nfree, npool, nfreed, nflushed;  // pool / cache-slot / flush counters (rare paths)
  uint32_t bflags;                          // Book flags (BOOK_QUIRK), rare-path writes
  ResumeRec rr;                             // written only when the lane book spills
#ifdef GOME_STAMPS
  unsigned long long st[16];
#endif
  uint8_t freeslot[NCS];            // free cache slots (stack)
};
constexpr size_t HOT_LDS_BYTES = sizeof(HotLds);
static_assert(HOT_LDS_BYTES <= 160 * 1024, "hot book LDS budget");

// Deferred (S, oid) -> loc index insert of a node rested by a hot book (one 16-B store).
struct PendEnt {
  uint32_t oid, loc, ix;
  uint8_t used, ins, dead, pad;
};
static_assert(sizeof(PendEnt) == 16, "PendEnt is stored as one 16-B write");


struct HotCtx {
  HotLds* S;
  int64_t P0, P1;   // lane l: price of level l / l + 64 (PR_NONE when unused)
  uint32_t M0, M1;  // lane l: S:BUY / S:SALE membership bits of level l / l + 64
  Node* nodes;
  ChunkHdr* chdr;
  gome_event* arena;
  PendEnt* pend;
  uint32_t sym, nl, npend;
  uint32_t ev_base, ev_used;
  uint32_t fills, pops, rests, cancels, adds, dels, dropped;
  int32_t lvd;  // levels created - dropped
  bool fatal;
};

// Environment pointers are global memory: the explicit address space keeps every access
// through them a global_* instruction (a generic pointer read back from LDS would compile
// to FLAT, see wave.h).
template <class T>
__device__ __forceinline__ GOME_GLB T* gp(T* const& f) {
  return (GOME_GLB T*)(reinterpret_cast<T*>(uni64(reinterpret_cast<int64_t>(f))));
}
#define G_ADD(p, v) __hip_atomic_fetch_add((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define G_OR(p, v) __hip_atomic_fetch_or((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)

__device__ __forceinline__ void hot_err(HotCtx& H, uint32_t e) {
  if (lane_id() == 0) G_OR(&gp(H.S->env.st)->err, e);
  H.fatal = true;
}

__device__ __forceinline__ uint32_t sl_make(uint32_t hs, uint32_t ts, uint32_t cs, uint32_t nxs) {
  return hs | (ts << 8) | (cs << 16) | (nxs << 24);
}
__device__ __forceinline__ uint32_t sl_hs(uint32_t sl) { return sl & 0xFFu; }
__device__ __forceinline__ uint32_t sl_ts(uint32_t sl) { return (sl >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t sl_cs(uint32_t sl) { return (sl >> 16) & 0xFFu; }
__device__ __forceinline__ uint32_t sl_nxs(uint32_t sl) { return (sl >> 24) & 3u; }
// Side-set bit of a raw Transaction value: SALE iff 1, anything else BUY (ordernode.go:95).
__device__ __forceinline__ uint32_t side_bit(uint32_t tx) { return tx == GOME_SALE ? M_SALE : M_BUY; }

__device__ __forceinline__ uint32_t wl(uint32_t reg, uint32_t v, uint32_t l) { return wl_u32(reg, v, l); }
__device__ __forceinline__ int64_t wl64(int64_t reg, int64_t v, uint32_t l) {
  const uint32_t lo = wl(lo32(reg), lo32(v), l), hi = wl(hi32(reg), hi32(v), l);
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}

// ---- single-lane stores without exec branches ------------------------------------------
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<size_t>(as_lds(const_cast<void*>(p))));
}
__device__ __forceinline__ void l0_glb16(void* p, v4u a) {
  unsigned long long sv;
  const unsigned long long ad = reinterpret_cast<unsigned long long>(p);
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "global_store_dwordx4 %1, %2, off\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(ad), "v"(a) : "memory");
}
__device__ __forceinline__ void l0_glb32(void* p, v4u a, v4u b) {
  unsigned long long sv;
  const unsigned long long ad = reinterpret_cast<unsigned long long>(p);
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "global_store_dwordx4 %1, %2, off\n\t"
               "global_store_dwordx4 %1, %3, off offset:16\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(ad), "v"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void l0_glb64(void* p, v4u a, v4u b, v4u c, v4u d) {
  unsigned long long sv;
  const unsigned long long ad = reinterpret_cast<unsigned long long>(p);
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "global_store_dwordx4 %1, %2, off\n\t"
               "global_store_dwordx4 %1, %3, off offset:16\n\t"
               "global_store_dwordx4 %1, %4, off offset:32\n\t"
               "global_store_dwordx4 %1, %5, off offset:48\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(ad), "v"(a), "v"(b), "v"(c), "v"(d) : "memory");
}
__device__ __forceinline__ void l0_glb48(void* p, v4u a, v4u b, v4u c) {
  unsigned long long sv;
  const unsigned long long ad = reinterpret_cast<unsigned long long>(p);
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "global_store_dwordx4 %1, %2, off\n\t"
               "global_store_dwordx4 %1, %3, off offset:16\n\t"
               "global_store_dwordx4 %1, %4, off offset:32\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(ad), "v"(a), "v"(b), "v"(c) : "memory");
}
__device__ __forceinline__ void l0_glb8(void* p, int64_t v) {
  unsigned long long sv;
  const unsigned long long ad = reinterpret_cast<unsigned long long>(p);
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "global_store_dwordx2 %1, %2, off\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(ad), "v"(v) : "memory");
}
__device__ __forceinline__ void l0_glb4(void* p, uint32_t v) {
  unsigned long long sv;
  const unsigned long long ad = reinterpret_cast<unsigned long long>(p);
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "global_store_dword %1, %2, off\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(ad), "v"(v) : "memory");
}
__device__ __forceinline__ void l0_glb1(void* p, uint32_t v) {
  unsigned long long sv;
  const unsigned long long ad = reinterpret_cast<unsigned long long>(p);
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "global_store_byte %1, %2, off\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(ad), "v"(v) : "memory");
}
__device__ __forceinline__ void l0_lds32(void* p, v4u a, v4u b) {
  unsigned long long sv;
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "ds_write_b128 %1, %2\n\tds_write_b128 %1, %3 offset:16\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(lds_addr(p)), "v"(a), "v"(b) : "memory");
}
__device__ __forceinline__ void l0_lds8(void* p, int64_t v) {
  unsigned long long sv;
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "ds_write_b64 %1, %2\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void l0_lds4(void* p, uint32_t v) {
  unsigned long long sv;
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "ds_write_b32 %1, %2\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void l0_lds1(void* p, uint32_t v) {
  unsigned long long sv;
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "ds_write_b8 %1, %2\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(lds_addr(p)), "v"(v) : "memory");
}

#ifdef GOME_STAMPS
__device__ __forceinline__ void st_add(HotLds* S, int i, unsigned long long dt) {
  unsigned long long sv;
  asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\t"
               "ds_add_u64 %1, %2\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(lds_addr(&S->st[i])), "v"(dt) : "memory");
}
#endif

// Counters kept in LDS (used on rare paths only).
__device__ __forceinline__ uint32_t lds_get(const uint32_t& c) { return uni(c); }
__device__ __forceinline__ void lds_set(uint32_t& c, uint32_t v) { l0_lds4(&c, v); }

// ---- events --------------------------------------------------------------------------
// Events go to per-wave blocks of EVB_HOT in the batch's arena (k_publish compacts
// them into publish order); unused tails are marked taker_seq = NIL.
__device__ __forceinline__ void hot_ev_close(HotCtx& H) {
  if (H.ev_base == NIL || H.fatal) return;
  for (uint32_t j = H.ev_used + lane_id(); j < EVB_HOT; j += 64) H.arena[H.ev_base + j].taker_seq = NIL;
}

__device__ __forceinline__ void hot_ev_block(HotCtx& H) {
  uint32_t b = 0;
  if (lane_id() == 0) b = G_ADD(&gp(H.S->env.st)->ev_bump, EVB_HOT);
  b = uni(b);
  if (b + EVB_HOT > uni(H.S->env.arena_cap)) {
    hot_err(H, ERR_EVENTS);
  }
  H.ev_base = b;
  H.ev_used = 0;
}

// One MatchResult (engine.go:24-28) as a 64-B gome_event, written by lane 0.
__device__ __forceinline__ void hot_emit(HotCtx& H, int64_t price, int64_t qty, int64_t mvol, int64_t tvol,
                                         uint32_t seq, uint32_t fidx, uint32_t moid, uint32_t muuid,
                                         uint32_t mnext, uint32_t kind, uint32_t mside, uint32_t mlast) {
  ST_T0(t_e)
  if (H.ev_used == EVB_HOT) hot_ev_block(H);  // ev_base starts NIL with ev_used = EVB_HOT
  if (!H.fatal)
    l0_glb48(&H.arena[H.ev_base + H.ev_used], v4(lo32(price), hi32(price), lo32(qty), hi32(qty)),
             v4(lo32(mvol), hi32(mvol), seq, fidx), v4(moid, muuid, mnext, kind | (mside << 8) | (mlast << 16)));
  H.ev_used++;
  ST_ADD(5, t_e)
}

// ---- chunk pools (no returning atomics on the per-order path) -------------------------
__device__ __forceinline__ uint32_t hot_alloc_chunk(HotCtx& H) {
  HotEnv& E = H.S->env;
  uint32_t npool = lds_get(H.S->npool);
  if (npool == 0) {  // claim POOL ids: free stack first, then the bump pointer
    const uint32_t lane = lane_id();
    int t = 0;
    if (lane == 0) t = G_ADD(&gp(E.st)->free_top, -static_cast<int>(POOL));
    t = static_cast<int>(uni(static_cast<uint32_t>(t)));
    const uint32_t nst = static_cast<uint32_t>(min(max(t, 0), static_cast<int>(POOL)));
    uint32_t b = 0;
    if (lane == 0 && nst < POOL) b = G_ADD(gp(E.ch_bump), POOL - nst);
    b = uni(b);
    if (lane < POOL) {
      const uint32_t id = (lane < nst) ? gp(E.free_ids)[t - static_cast<int>(nst) + static_cast<int>(lane)]
                                       : b + (lane - nst);
      H.S->pool[lane] = id;
    }
    npool = POOL;
  }
  npool--;
  lds_set(H.S->npool, npool);
  const uint32_t c = uni(H.S->pool[npool]);
  if (c >= uni(E.ch_cap)) { hot_err(H, ERR_CHUNKS); return NIL; }
  return c;
}

// Publish n chunk ids from LDS buffer `buf` to the batch's freed list (recycled after the
// batch by k_recycle_*).
__device__ __forceinline__ void hot_publish_ids(HotCtx& H, const uint32_t* buf, uint32_t n) {
  if (n == 0) return;
  const uint32_t lane = lane_id();
  uint32_t b = 0;
  if (lane == 0) b = G_ADD(&gp(H.S->env.st)->freed_top, n);
  b = uni(b);
  if (lane < n) gp(H.S->env.freed_ids)[b + lane] = buf[lane];
}

__device__ __forceinline__ void hot_free_chunk(HotCtx& H, uint32_t c) {
  uint32_t nf = lds_get(H.S->nfreed);
  if (nf == FREED) {
    hot_publish_ids(H, H.S->freed, FREED);
    nf = 0;
  }
  l0_lds4(&H.S->freed[nf], c);
  lds_set(H.S->nfreed, nf + 1);
}

__device__ __forceinline__ void hot_free_chain(HotCtx& H, uint32_t head, uint32_t tail) {
  uint32_t c = head;
  for (uint32_t guard = 0; c != NIL; ++guard) {
    if (guard > uni(H.S->env.ch_cap)) { hot_err(H, ERR_CORRUPT); return; }
    const uint32_t nx = (c == tail) ? NIL : uni(H.chdr[c].next);
    hot_free_chunk(H, c);
    c = nx;
  }
}

__device__ __forceinline__ uint32_t hot_slot_alloc(HotCtx& H) {
  const uint32_t n = lds_get(H.S->nfree) - 1;
  lds_set(H.S->nfree, n);
  return uni(H.S->freeslot[n]);
}

__device__ __forceinline__ void hot_slot_free(HotCtx& H, uint32_t cs) {
  const uint32_t n = lds_get(H.S->nfree);
  l0_lds1(&H.S->freeslot[n], cs);
  l0_lds4(&H.S->cs_chunk[cs], NIL);
  lds_set(H.S->nfree, n + 1);
}

// ---- cancel index (engine.go:92-93: HGET S:link:<p> S:node:<oid>) -------------------------
__device__ __forceinline__ bool hot_idx_lookup(HotCtx& H, uint32_t oid, uint32_t& ixslot, uint32_t& loc) {
  const uint32_t lane = lane_id();
  GOME_GLB IdxEnt* idx = gp(H.S->env.idx);
  const unsigned long long key = idx_key(H.sym, oid), mask = static_cast<unsigned long long>(uni64(static_cast<int64_t>(H.S->env.idx_mask)));
  unsigned long long h = mix64(key) & mask;
  for (unsigned long long probe = 0; probe <= mask; probe += 64) {
    const unsigned long long slot = (h + lane) & mask;
    const unsigned long long kv = __hip_atomic_load(&idx[slot].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hit = __ballot(kv == key), emp = __ballot(kv == KEY_EMPTY);
    const unsigned long long any = hit | emp;
    if (any) {
      const uint32_t b = __builtin_ctzll(any);
      if (!((hit >> b) & 1ull)) return false;
      const uint32_t lc = (lane == b) ? idx[slot].loc : 0u;
      loc = rl(lc, b);
      ixslot = static_cast<uint32_t>((h + b) & mask);
      return true;
    }
    h = (h + 64) & mask;
  }
  return false;
}

__device__ __forceinline__ void hot_idx_erase(HotCtx& H, uint32_t ixslot) {
  GOME_GLB IdxEnt* idx = gp(H.S->env.idx);
  __hip_atomic_store(&idx[ixslot].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// ---- resident head ----------------------------------------------------------------------
struct Head {
  int64_t rem;
  uint32_t oid, uuid, ix, tx;
  uint32_t slot, live, hd, hn, nx, nxs;
};

// Load the FIFO's first live node from HBM into cache slot cs, starting at chunk h.hd,
// slot h.slot (first unconsumed); skips (and frees) exhausted chunks.
__device__ __forceinline__ void hot_fill_head(HotCtx& H, uint32_t cs, uint32_t tl, uint32_t tslot,
                                              uint32_t nv, Head& h) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id(), s = lane & 31u;
  for (uint32_t guard = 0;; ++guard) {
    if (guard > uni(S->env.ch_cap) || h.hd == NIL) { hot_err(H, ERR_CORRUPT); h.live = 0; return; }
    const uint4* src = reinterpret_cast<const uint4*>(&H.nodes[h.hd * CH + s]);
    const uint4 a = src[0], b = src[1];
    h.hn = uni(H.chdr[h.hd].next);
    if (lane < CH) {
      st16_lds(&S->cs[cs][lane], v4(a.x, a.y, a.z, a.w));
      st16_lds(reinterpret_cast<char*>(&S->cs[cs][lane]) + 16, v4(b.x, b.y, b.z, b.w));
    }
    const int64_t rem = static_cast<int64_t>((static_cast<uint64_t>(a.y) << 32) | a.x);
    const uint32_t lim = (h.hd == tl) ? tslot : CH;
    const uint32_t live = static_cast<uint32_t>(__ballot(lane < lim && lane >= h.slot && rem >= 0));
    if (live) {
      l0_lds4(&S->cs_chunk[cs], h.hd);
      const uint32_t f = __builtin_ctz(live), rest = live & (live - 1);
      h.slot = f;
      h.live = live;
      h.rem = rl64(rem, f);
      h.oid = rl(a.z, f);
      h.uuid = rl(a.w, f);
      h.ix = rl(b.x, f);
      h.tx = rl(b.y, f) & 0xFFu;
      h.nx = rest ? rl(a.z, __builtin_ctz(rest)) : 0u;
      h.nxs = rest ? HN_OID : (static_cast<uint32_t>(__popc(live)) < nv ? HN_UNKNOWN : HN_NONE);
      return;
    }
    if (h.hd == tl) { hot_err(H, ERR_CORRUPT); h.live = 0; return; }
    hot_free_chunk(H, h.hd);
    h.hd = h.hn;
    h.slot = 0;
  }
}

// After the head node left (fill or cancel) and nv > 0 nodes remain: next head.
__device__ __forceinline__ void hot_next_head(HotCtx& H, uint32_t cs, uint32_t tl, uint32_t tslot,
                                              uint32_t nv, Head& h) {
  HotLds* S = H.S;
  if (h.live) {
    const uint32_t f = __builtin_ctz(h.live), rest = h.live & (h.live - 1);
    const Node nd = S->cs[cs][f];
    const uint32_t nxo = rest ? S->cs[cs][__builtin_ctz(rest)].oid : 0u;
    h.slot = f;
    h.rem = uni64(nd.rem);
    h.oid = uni(nd.oid);
    h.uuid = uni(nd.uuid);
    h.ix = uni(nd.ixs);
    h.tx = uni(nd.tx);
    h.nx = uni(nxo);
    h.nxs = rest ? HN_OID : (static_cast<uint32_t>(__popc(h.live)) < nv ? HN_UNKNOWN : HN_NONE);
    return;
  }
  hot_free_chunk(H, h.hd);  // head chunk exhausted: continue in the next chunk
  h.hd = h.hn;
  h.slot = 0;
  hot_fill_head(H, cs, tl, tslot, nv, h);
}

// MatchNode.NextNode of the head when unknown: the next live node in the head chunk, or
// the first live node of the chunks after it (HBM).
__device__ __forceinline__ void hot_resolve_next(HotCtx& H, uint32_t cs, uint32_t tl, uint32_t tslot, Head& h) {
  const uint32_t lane = lane_id();
  const uint32_t after = h.live & ~((2u << h.slot) - 1u);
  if (after) {
    h.nx = uni(H.S->cs[cs][__builtin_ctz(after)].oid);
    h.nxs = HN_OID;
    return;
  }
  h.nxs = HN_NONE;
  const uint32_t cap = uni(H.S->env.ch_cap);
  uint32_t c2 = h.hn;
  for (uint32_t g = 0; c2 != NIL && g <= cap; ++g) {
    const uint32_t lim = (c2 == tl) ? tslot : CH;
    const bool l2 = lane < lim && H.nodes[c2 * CH + (lane & 31u)].rem >= 0;
    const unsigned long long m2 = __ballot(l2);
    if (m2) {
      h.nx = uni(H.nodes[c2 * CH + __builtin_ctzll(m2)].oid);
      h.nxs = HN_OID;
      return;
    }
    c2 = (c2 == tl) ? NIL : uni(H.chdr[c2].next);
  }
}

__device__ __forceinline__ void hot_drop_index(HotCtx& H, uint32_t ixs) {
  if (ixs & PEND) l0_glb1(&H.pend[ixs & ~PEND].dead, 1u);
  else hot_idx_erase(H, ixs);
}

// ---- level records --------------------------------------------------------------------------
// Uniform (broadcast) read of record k: five 16-B LDS loads issued together.
__device__ __forceinline__ LvRec rec_load(const HotCtx& H, uint32_t k) {
  const v4u* q = reinterpret_cast<const v4u*>(&H.S->lv[k]);
  const v4u a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
  LvRec r;
  r.pr = static_cast<int64_t>((static_cast<uint64_t>(uni(a.y)) << 32) | uni(a.x));
  r.dp = static_cast<int64_t>((static_cast<uint64_t>(uni(a.w)) << 32) | uni(a.z));
  r.hrem = static_cast<int64_t>((static_cast<uint64_t>(uni(b.y)) << 32) | uni(b.x));
  r.hoid = uni(b.z);
  r.huuid = uni(b.w);
  r.hd = uni(c.x);
  r.tl = uni(c.y);
  r.hn = uni(c.z);
  r.nv = uni(c.w);
  r.sl = uni(d.x);
  r.live = uni(d.y);
  r.hix = uni(d.z);
  r.hx = uni(d.w);
  r.hnx = uni(e.x);
  r.mem = 0;
  r.pad1 = r.pad2 = 0;
  return r;
}

enum : uint32_t { Q0 = 1, Q1 = 2, Q2 = 4, Q3 = 8, Q4 = 16, QALL = 31 };

// Write the quads of record k selected by `mask` (lane 0, one asm block per quad).
__device__ __forceinline__ void rec_store(HotCtx& H, uint32_t k, const LvRec& r, uint32_t mask) {
  LvRec* d = &H.S->lv[k];
  char* b = reinterpret_cast<char*>(d);
  unsigned long long sv;
  const uint32_t a = lds_addr(b);
  if (mask & Q0) {
    const v4u q = v4(lo32(r.pr), hi32(r.pr), lo32(r.dp), hi32(r.dp));
    asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\tds_write_b128 %1, %2\n\ts_mov_b64 exec, %0"
                 : "=&s"(sv) : "v"(a), "v"(q) : "memory");
  }
  if (mask & Q1) {
    const v4u q = v4(lo32(r.hrem), hi32(r.hrem), r.hoid, r.huuid);
    asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\tds_write_b128 %1, %2 offset:16\n\ts_mov_b64 exec, %0"
                 : "=&s"(sv) : "v"(a), "v"(q) : "memory");
  }
  if (mask & Q2) {
    const v4u q = v4(r.hd, r.tl, r.hn, r.nv);
    asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\tds_write_b128 %1, %2 offset:32\n\ts_mov_b64 exec, %0"
                 : "=&s"(sv) : "v"(a), "v"(q) : "memory");
  }
  if (mask & Q3) {
    const v4u q = v4(r.sl, r.live, r.hix, r.hx);
    asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\tds_write_b128 %1, %2 offset:48\n\ts_mov_b64 exec, %0"
                 : "=&s"(sv) : "v"(a), "v"(q) : "memory");
  }
  if (mask & Q4) {
    const v4u q = v4(r.hnx, 0u, 0u, 0u);
    asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 exec, 1\n\tds_write_b128 %1, %2 offset:64\n\ts_mov_b64 exec, %0"
                 : "=&s"(sv) : "v"(a), "v"(q) : "memory");
  }
}

// Side-set membership of level k (lane register mirror, S:BUY / S:SALE).
__device__ __forceinline__ uint32_t mem_get(const HotCtx& H, uint32_t k) {
  return k < 64 ? rl(H.M0, k) : rl(H.M1, k - 64);
}
__device__ __forceinline__ void mem_put(HotCtx& H, uint32_t k, uint32_t m) {
  if (k < 64) H.M0 = wl(H.M0, m, k);
  else H.M1 = wl(H.M1, m, k - 64);
}

__device__ __forceinline__ Head head_of(const LvRec& r) {
  Head h;
  h.rem = r.hrem;
  h.oid = r.hoid;
  h.uuid = r.huuid;
  h.ix = r.hix;
  h.tx = r.hx;
  h.slot = sl_hs(r.sl);
  h.live = r.live;
  h.hd = r.hd;
  h.hn = r.hn;
  h.nx = r.hnx;
  h.nxs = sl_nxs(r.sl);
  return h;
}

__device__ __forceinline__ void head_into(LvRec& r, const Head& h) {
  r.hrem = h.rem;
  r.hoid = h.oid;
  r.huuid = h.uuid;
  r.hix = h.ix;
  r.hx = h.tx;
  r.live = h.live;
  r.hd = h.hd;
  r.hn = h.hn;
  r.hnx = h.nx;
}

// ---- MatchOrder (engine.go:138-198) at level k, general case ------------------------------
__device__ __forceinline__ int64_t hot_visit_gen(HotCtx& H, uint32_t k, LvRec r, int64_t T, uint32_t seq, uint32_t& fidx) {
  uint32_t nv = r.nv;
  if (nv == 0) return T;  // membership without nodes (Q2): GetFirstNode finds nothing
  const uint32_t sl = r.sl, tl = r.tl, tslot = sl_ts(sl);
  uint32_t cs = sl_cs(sl);
  uint32_t mem = mem_get(H, k);
  Head h;
  if (cs == CS_NONE) {  // first touch in this kernel: make the level resident
    cs = hot_slot_alloc(H);
    h.hd = r.hd;
    h.slot = sl_hs(sl);
    hot_fill_head(H, cs, tl, tslot, nv, h);
  } else {
    h = head_of(r);
  }
  int64_t dp = r.dp;
  bool empty = false;
  while (!H.fatal) {
    if (h.nxs == HN_UNKNOWN) hot_resolve_next(H, cs, tl, tslot, h);
    const uint32_t last = (h.nxs == HN_OID) ? 0u : 1u;
    const uint32_t nxo = last ? 0u : h.nx;
    if (T < h.rem) {  // diff < 0: the maker keeps its FIFO position (engine.go:176-194)
      hot_emit(H, r.pr, T, h.rem - T, 0, seq, fidx++, h.oid, h.uuid, nxo, GOME_EV_FILL, h.tx, last);
      h.rem -= T;
      dp -= T;
      T = 0;
      if (dp <= 0) mem &= ~side_bit(h.tx);  // ZREM from the maker's side set
      H.fills++;
      break;
    }
    // diff >= 0: the maker is filled completely and leaves the FIFO (engine.go:145-175)
    hot_emit(H, r.pr, h.rem, h.rem, T - h.rem, seq, fidx++, h.oid, h.uuid, nxo, GOME_EV_FILL, h.tx, last);
    T -= h.rem;
    dp -= h.rem;
    if (dp <= 0) mem &= ~side_bit(h.tx);
    H.fills++;
    H.pops++;
    hot_drop_index(H, h.ix);
    h.live &= ~(1u << h.slot);
    nv--;
    if (nv == 0) {
      hot_free_chain(H, h.hd, tl);
      hot_slot_free(H, cs);
      empty = true;
      break;
    }
    hot_next_head(H, cs, tl, tslot, nv, h);
    if (T <= 0) break;  // diff == 0: stop (engine.go:162-175)
  }
  r.dp = dp;
  r.nv = nv;
  if (empty) {
    r.hd = r.tl = r.hn = NIL;
    r.live = 0;
    r.sl = sl_make(0, 0, CS_NONE, HN_UNKNOWN);
  } else {
    head_into(r, h);
    r.sl = sl_make(h.slot, tslot, cs, h.nxs);
  }
  rec_store(H, k, r, QALL);
  mem_put(H, k, mem);
  return T;
}

// ---- rest the remaining volume at level k (engine.go:80-82, nodepool.go:31-83), general ------
__device__ __forceinline__ void hot_rest_gen(HotCtx& H, uint32_t k, LvRec r, int64_t p, int64_t T, uint32_t oid, uint32_t uuid,
                             uint32_t side) {
  HotLds* S = H.S;
  uint32_t cs = sl_cs(r.sl), tslot = sl_ts(r.sl), nxs = sl_nxs(r.sl);
  const uint32_t pidx = H.npend++;
  const v4u na = v4(lo32(T), hi32(T), oid, uuid), nb = v4(PEND | pidx, side & 0xFFu, 0u, 0u);
  if (T == 0) l0_lds4(&S->bflags, BOOK_QUIRK);  // zero-volume maker (Q6)
  uint32_t loc;
  if (r.tl == NIL) {  // empty FIFO (InitOrderLink, nodelink.go:12): new chunk = head = tail
    const uint32_t c = hot_alloc_chunk(H);
    if (c == NIL) return;
    l0_glb16(&H.chdr[c], v4(NIL, 0u, lo32(p), hi32(p)));
    cs = hot_slot_alloc(H);
    l0_lds4(&S->cs_chunk[cs], c);
    l0_lds32(&S->cs[cs][0], na, nb);
    loc = c * CH;
    r.hrem = T;
    r.hoid = oid;
    r.huuid = uuid;
    r.hix = PEND | pidx;
    r.hx = side & 0xFFu;
    r.live = 1u;
    r.hd = r.tl = c;
    r.hn = NIL;
    r.hnx = 0;
    r.sl = sl_make(0, 1, cs, HN_NONE);
  } else {
    const bool res = cs != CS_NONE;
    if (tslot == CH) {  // SetLast with a full tail chunk: link a new one
      const uint32_t c = hot_alloc_chunk(H);
      if (c == NIL) return;
      l0_glb16(&H.chdr[c], v4(NIL, 0u, lo32(p), hi32(p)));
      l0_glb4(&H.chdr[r.tl].next, c);
      if (res && r.hd == r.tl) r.hn = c;
      r.tl = c;
      tslot = 0;
    }
    loc = r.tl * CH + tslot;
    if (res && r.hd == r.tl) {
      l0_lds32(&S->cs[cs][tslot], na, nb);
      r.live |= 1u << tslot;
    } else {
      l0_glb32(&H.nodes[loc], na, nb);
    }
    if (res && nxs == HN_NONE) {  // the head had no successor: this node is MatchNode.NextNode
      r.hnx = oid;
      nxs = HN_OID;
    }
    r.sl = sl_make(sl_hs(r.sl), tslot + 1, cs, nxs);
  }
  r.nv += 1;
  r.dp += T;  // SetPoolDepthVolume
  rec_store(H, k, r, QALL);
  mem_put(H, k, mem_get(H, k) | side_bit(side));  // SetPoolDepth (ZADD own side)
  l0_glb16(&H.pend[pidx], v4(oid, loc, NIL, 1u));
  H.rests++;
}

// ---- fast paths ------------------------------------------------------------------------------
// Rest at existing level k whose tail chunk has room.
__device__ __forceinline__ void hot_rest_fast(HotCtx& H, uint32_t k, int64_t p, int64_t T, uint32_t oid,
                                              uint32_t uuid, uint32_t side) {
  LvRec r = rec_load(H, k);
  const uint32_t ts = sl_ts(r.sl), cs = sl_cs(r.sl);
  if (r.tl == NIL || ts >= CH) {
    hot_rest_gen(H, k, r, p, T, oid, uuid, side);
    return;
  }
  const uint32_t pidx = H.npend++;
  const uint32_t loc = r.tl * CH + ts;
  if (T == 0) l0_lds4(&H.S->bflags, BOOK_QUIRK);  // zero-volume maker (Q6)
  const v4u na = v4(lo32(T), hi32(T), oid, uuid), nb = v4(PEND | pidx, side & 0xFFu, 0u, 0u);
  uint32_t mask = Q0 | Q2 | Q3;
  if (cs != CS_NONE && r.hd == r.tl) {  // tail == cached head chunk
    l0_lds32(&H.S->cs[cs][ts], na, nb);
    r.live |= 1u << ts;
  } else {
    l0_glb32(&H.nodes[loc], na, nb);
  }
  uint32_t sl = r.sl + (1u << 8);  // tslot + 1
  if (cs != CS_NONE && sl_nxs(r.sl) == HN_NONE) {  // the head had no successor
    r.hnx = oid;
    sl = (sl & ~(3u << 24)) | (HN_OID << 24);
    mask |= Q4;
  }
  r.sl = sl;
  r.nv += 1;
  r.dp += T;  // SetPoolDepthVolume
  rec_store(H, k, r, mask);
  mem_put(H, k, mem_get(H, k) | side_bit(side));  // SetPoolDepth (ZADD own side)
  l0_glb16(&H.pend[pidx], v4(oid, loc, NIL, 1u));
  H.rests++;
}

// MatchOrder at level k: partial fill of the head and pops of a head that has a live
// successor in the cached chunk are handled here; everything else in hot_visit_gen.
__device__ __forceinline__ int64_t hot_visit_fast(HotCtx& H, uint32_t k, int64_t T, uint32_t seq, uint32_t& fidx) {
  LvRec r = rec_load(H, k);
  if (r.nv == 0) return T;
  const uint32_t cs = sl_cs(r.sl);
  if (cs == CS_NONE) return hot_visit_gen(H, k, r, T, seq, fidx);
  uint32_t mask = 0;
  for (;;) {
    const uint32_t nxs = sl_nxs(r.sl);
    if (nxs == HN_UNKNOWN || H.fatal) break;
    const uint32_t last = nxs == HN_OID ? 0u : 1u;
    const uint32_t nxo = last ? 0u : r.hnx;
    if (T < r.hrem) {  // diff < 0: the maker keeps its FIFO position (engine.go:176-194)
      hot_emit(H, r.pr, T, r.hrem - T, 0, seq, fidx++, r.hoid, r.huuid, nxo, GOME_EV_FILL, r.hx, last);
      r.hrem -= T;
      r.dp -= T;
      if (r.dp <= 0) mem_put(H, k, mem_get(H, k) & ~side_bit(r.hx));  // ZREM maker's side
      H.fills++;
      rec_store(H, k, r, mask | Q0 | Q1);
      return 0;
    }
    const uint32_t live = r.live & ~(1u << sl_hs(r.sl));
    if (r.nv == 1 || live == 0) break;  // level empties / head chunk exhausted
    // diff >= 0: the head leaves the FIFO (engine.go:145-175); the next live node of the
    // cached chunk becomes the head (one LDS round trip)
    hot_emit(H, r.pr, r.hrem, r.hrem, T - r.hrem, seq, fidx++, r.hoid, r.huuid, nxo, GOME_EV_FILL, r.hx, last);
    T -= r.hrem;
    r.dp -= r.hrem;
    if (r.dp <= 0) mem_put(H, k, mem_get(H, k) & ~side_bit(r.hx));
    H.fills++;
    H.pops++;
    hot_drop_index(H, r.hix);
    r.nv -= 1;
    const uint32_t s1 = __builtin_ctz(live), rest = live & (live - 1);
    const Node* c = H.S->cs[cs];
    const v4u* n1 = reinterpret_cast<const v4u*>(&c[s1]);
    const v4u a = n1[0], b = n1[1];
    const uint32_t nxo2 = c[rest ? __builtin_ctz(rest) : s1].oid;
    r.hrem = static_cast<int64_t>((static_cast<uint64_t>(uni(a.y)) << 32) | uni(a.x));
    r.hoid = uni(a.z);
    r.huuid = uni(a.w);
    r.hix = uni(b.x);
    r.hx = uni(b.y) & 0xFFu;
    r.hnx = uni(nxo2);
    r.live = live;
    const uint32_t nn = rest ? HN_OID : (static_cast<uint32_t>(__popc(live)) < r.nv ? HN_UNKNOWN : HN_NONE);
    r.sl = (r.sl & ~0x030000FFu) | s1 | (nn << 24);
    mask = QALL;
    if (T <= 0) {  // diff == 0: stop (engine.go:162-175)
      rec_store(H, k, r, mask);
      return T;
    }
  }
  return hot_visit_gen(H, k, r, T, seq, fidx);  // r carries the fast path's updates
}

// ---- level array: insert / GC ----------------------------------------------------------------
__device__ __forceinline__ void lv_regs_from_lds(HotCtx& H) {
  const uint32_t lane = lane_id();
  H.P0 = lane < H.nl ? H.S->lv[lane].pr : PR_NONE;
  H.P1 = lane + 64 < H.nl ? H.S->lv[lane + 64].pr : PR_NONE;
  H.M0 = lane < H.nl ? H.S->lv[lane].mem : 0u;
  H.M1 = lane + 64 < H.nl ? H.S->lv[lane + 64].mem : 0u;
}

// Level index of price p, or its insertion position.
__device__ __forceinline__ bool lv_find(const HotCtx& H, int64_t p, uint32_t& k) {
  const unsigned long long e0 = __ballot(H.P0 == p), e1 = __ballot(H.P1 == p);
  if (e0 | e1) {
    k = e0 ? static_cast<uint32_t>(__builtin_ctzll(e0)) : 64u + static_cast<uint32_t>(__builtin_ctzll(e1));
    return true;
  }
  k = __popcll(__ballot(H.P0 < p)) + __popcll(__ballot(H.P1 < p));
  return false;
}

// A record as five 16-B vectors (record moves without struct copies through scratch).
struct RecQ {
  v4u q[5];
};
__device__ __forceinline__ RecQ recq_load(const HotLds* S, uint32_t k) {
  const v4u* src = reinterpret_cast<const v4u*>(&S->lv[k]);
  RecQ r;
#pragma unroll
  for (int i = 0; i < 5; ++i) r.q[i] = src[i];
  return r;
}
__device__ __forceinline__ void recq_store(HotLds* S, uint32_t k, const RecQ& r) {
  v4u* dst = reinterpret_cast<v4u*>(&S->lv[k]);
#pragma unroll
  for (int i = 0; i < 5; ++i) dst[i] = r.q[i];
}

// Insert an empty level for price p at position pos (records move in LDS; lane registers
// are rebuilt).  When the array is full, levels with no observable state are dropped
// first; false if it is still full (spill).
__device__ __forceinline__ bool lv_insert(HotCtx& H, int64_t p, uint32_t& pos) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id();
  // every lane holds its two records while the array is rewritten; membership travels in
  // the record's `mem` word (q4.y)
  const bool v0 = lane < H.nl, v1 = lane + 64 < H.nl;
  RecQ r0, r1;
  r0 = v0 ? recq_load(S, lane) : RecQ{};
  r1 = v1 ? recq_load(S, lane + 64) : RecQ{};
  r0.q[4].y = H.M0;
  r1.q[4].y = H.M1;
  if (H.nl == LRB_CAP) {
    // keep levels with nodes, depth or a side-set membership
    const bool k0 = v0 && (r0.q[2].w || r0.q[0].z || r0.q[0].w || r0.q[4].y);
    const bool k1 = v1 && (r1.q[2].w || r1.q[0].z || r1.q[0].w || r1.q[4].y);
    const unsigned long long a0 = __ballot(k0), a1 = __ballot(k1), ltm = lt_mask();
    if (k0) recq_store(S, __popcll(a0 & ltm), r0);
    if (k1) recq_store(S, __popcll(a0) + __popcll(a1 & ltm), r1);
    const uint32_t out = __popcll(a0) + __popcll(a1);
    H.lvd -= static_cast<int32_t>(H.nl - out);
    H.nl = out;
    lv_regs_from_lds(H);
    lv_find(H, p, pos);
    if (H.nl == LRB_CAP) return false;
    r0 = lane < H.nl ? recq_load(S, lane) : RecQ{};  // compacted records carry `mem`
    r1 = lane + 64 < H.nl ? recq_load(S, lane + 64) : RecQ{};
  }
  // every record is rewritten (not only the shifted ones): the staged membership word must
  // reach all of them before the lane registers are rebuilt from LDS
  if (lane < H.nl) recq_store(S, lane + (lane >= pos ? 1 : 0), r0);
  if (lane + 64 < H.nl) recq_store(S, lane + 64 + (lane + 64 >= pos ? 1 : 0), r1);
  if (lane == 0) {
    RecQ z;
    z.q[0] = v4(lo32(p), hi32(p), 0u, 0u);                     // pr, dp
    z.q[1] = v4(0u, 0u, 0u, 0u);                               // hrem, hoid, huuid
    z.q[2] = v4(NIL, NIL, NIL, 0u);                            // hd, tl, hn, nv
    z.q[3] = v4(sl_make(0, 0, CS_NONE, HN_UNKNOWN), 0u, 0u, 0u);  // sl, live, hix, hx
    z.q[4] = v4(0u, 0u, 0u, 0u);                               // hnx, mem
    recq_store(S, pos, z);
  }
  H.nl++;
  H.lvd++;
  lv_regs_from_lds(H);
  return true;
}

// ---- SetOrder (engine.go:56-85) -------------------------------------------------------------
// Returns false when the order was matched but cannot rest (lane array full): the caller
// hands `trest` to the HBM path.
__device__ __forceinline__ bool hot_add(HotCtx& H, int64_t p, int64_t vol, uint32_t oid, uint32_t uuid,
                                        uint32_t side, uint32_t seq, uint32_t& nev, int64_t& trest) {
  int64_t T = vol;
  uint32_t fidx = 0;
  // GetReverseDepth (nodepool.go:86-115): opposite-side levels crossing p, best first
  // (asks ascending for a BUY, bids descending for a SALE; Transaction != 1 is BUY).
  const bool buy = side != GOME_SALE;
  const uint32_t opp = buy ? M_SALE : M_BUY;
  unsigned long long m0, m1;
  if (buy) {
    m0 = __ballot((H.M0 & opp) && H.P0 <= p);
    m1 = __ballot((H.M1 & opp) && H.P1 <= p);
  } else {
    m0 = __ballot((H.M0 & opp) && H.P0 >= p);
    m1 = __ballot((H.M1 & opp) && H.P1 >= p);
  }
  const unsigned long long q0 = __ballot(H.P0 == p), q1 = __ballot(H.P1 == p);  // rest level
  const bool crossed = (m0 | m1) != 0;
  while (m0 | m1) {  // Match (engine.go:118-136)
    uint32_t k;
    if (buy) {
      if (m0) {
        k = __builtin_ctzll(m0);
        m0 &= m0 - 1;
      } else {
        k = 64 + __builtin_ctzll(m1);
        m1 &= m1 - 1;
      }
    } else {
      if (m1) {
        const uint32_t b = 63 - __builtin_clzll(m1);
        m1 &= ~(1ull << b);
        k = 64 + b;
      } else {
        const uint32_t b = 63 - __builtin_clzll(m0);
        m0 &= ~(1ull << b);
        k = b;
      }
    }
    T = hot_visit_fast(H, k, T, seq, fidx);
    if (T <= 0 || H.fatal) break;
  }
  nev = fidx;
  trest = T;
  if ((crossed && T <= 0) || H.fatal) return true;
  if (q0 | q1) {  // the level exists (levels never move while an order is matched)
    hot_rest_fast(H, q0 ? static_cast<uint32_t>(__builtin_ctzll(q0)) : 64u + static_cast<uint32_t>(__builtin_ctzll(q1)),
                  p, T, oid, uuid, side);
    return true;
  }
  uint32_t k;
  if (!lv_find(H, p, k) && !lv_insert(H, p, k)) return false;
  hot_rest_gen(H, k, rec_load(H, k), p, T, oid, uuid, side);
  return true;
}

// Insert this segment's pending entries [nflushed, npend) into the cancel index (needed
// before a lookup), store each node's real slot into the node (LDS cache or HBM), and
// refresh the records' head index slots.
__device__ __forceinline__ void hot_flush(HotCtx& H) {
  const uint32_t lane = lane_id();
  GOME_GLB IdxEnt* idx = gp(H.S->env.idx);
  const unsigned long long mask = static_cast<unsigned long long>(uni64(static_cast<int64_t>(H.S->env.idx_mask)));
  bool full = false;
  for (uint32_t b = lds_get(H.S->nflushed); b < H.npend; b += 64) {
    const uint32_t i = b + lane;
    PendEnt e{};
    bool ok = false;
    unsigned long long h = 0;
    if (i < H.npend) {
      e = H.pend[i];
      if (!e.dead) {
        const unsigned long long key = idx_key(H.sym, e.oid);
        h = mix64(key) & mask;
        unsigned long long probe = 0;
        for (; probe <= mask; ++probe, h = (h + 1) & mask) {
          const unsigned long long kv = __hip_atomic_load(&idx[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          unsigned long long exp = kv;
          if ((kv == KEY_EMPTY || kv == KEY_TOMB) &&
              __hip_atomic_compare_exchange_strong(&idx[h].key, &exp, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT))
            break;
        }
        if (probe > mask) {
          full = true;
        } else {
          ok = true;
          idx[h].loc = e.loc;
          H.pend[i].ix = static_cast<uint32_t>(h);
          H.pend[i].ins = 1;
        }
      }
    }
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
        else *as_glb(&H.nodes[e.loc].ixs) = static_cast<uint32_t>(h);
      }
    }
  }
  if (__ballot(full)) hot_err(H, ERR_INDEX);
  lds_set(H.S->nflushed, H.npend);
  // the records cache their head node's index slot
  for (uint32_t k = lane; k < H.nl; k += 64) {
    const uint32_t sl = H.S->lv[k].sl, cs = sl_cs(sl);
    if (cs != CS_NONE) H.S->lv[k].hix = H.S->cs[cs][sl_hs(sl)].ixs;
  }
}

// ---- DeleteOrder (engine.go:87-116) -----------------------------------------------------------
__device__ __forceinline__ void hot_cancel_at(HotCtx& H, uint32_t k, uint32_t loc, uint32_t ixslot, int64_t p, uint32_t oid,
                              uint32_t uuid, uint32_t side, uint32_t seq) {
  HotLds* S = H.S;
  LvRec r = rec_load(H, k);
  const uint32_t cid = loc / CH, s = loc % CH;
  const uint32_t cs = sl_cs(r.sl), tslot = sl_ts(r.sl);
  Head h = head_of(r);
  const bool inhead = cs != CS_NONE && cid == r.hd;
  const bool ishead = inhead && s == h.slot;
  const int64_t rem = ishead ? r.hrem : inhead ? uni64(*as_lds(&S->cs[cs][s].rem)) : uni64(*as_glb(&H.nodes[loc].rem));
  const uint32_t ntx = ishead ? r.hx : inhead ? uni(*as_lds(&S->cs[cs][s].tx)) : uni(*as_glb(&H.nodes[loc].tx));
  if ((ntx == GOME_SALE) != (side == GOME_SALE)) l0_lds4(&S->bflags, BOOK_QUIRK);  // wrong-side cancel (Q2)
  if (rem < 0) { hot_err(H, ERR_CORRUPT); return; }
  r.dp -= rem;  // DeletePoolDepthVolume with the stored remaining volume
  if (r.dp <= 0) mem_put(H, k, mem_get(H, k) & ~side_bit(side));  // ZREM from the REQUEST's side set (Q2)
  if (inhead) l0_lds8(&S->cs[cs][s].rem, -1);
  else l0_glb8(&H.nodes[loc].rem, -1);
  hot_idx_erase(H, ixslot);
  r.nv -= 1;
  if (r.nv == 0) {
    hot_free_chain(H, r.hd, r.tl);
    if (cs != CS_NONE) hot_slot_free(H, cs);
    r.hd = r.tl = r.hn = NIL;
    r.live = 0;
    r.sl = sl_make(0, 0, CS_NONE, HN_UNKNOWN);
  } else if (cs != CS_NONE) {
    if (ishead) {
      h.live &= ~(1u << s);
      hot_next_head(H, cs, r.tl, tslot, r.nv, h);
    } else {
      if (inhead) h.live &= ~(1u << s);
      if (h.nxs == HN_OID && h.nx == oid) h.nxs = HN_UNKNOWN;
    }
    head_into(r, h);
    r.sl = sl_make(h.slot, tslot, cs, h.nxs);
  }
  rec_store(H, k, r, QALL);
  hot_emit(H, p, 0, rem, rem, seq, 0, oid, uuid, 0u, GOME_EV_CANCEL, side, 1u);
  H.cancels++;
}

// Cancel: index lookup (by oid, engine.go:92-93), price check (Q3), then the level.
__device__ __forceinline__ uint32_t hot_cancel(HotCtx& H, int64_t p, uint32_t oid, uint32_t uuid,
                                               uint32_t side, uint32_t seq) {
  if (lds_get(H.S->nflushed) < H.npend) hot_flush(H);
  uint32_t ixslot, loc;
  if (!hot_idx_lookup(H, oid, ixslot, loc)) return 0;                     // no event
  if (uni(static_cast<uint32_t>(H.chdr[loc / CH].price != p))) return 0;  // wrong price (Q3)
  uint32_t k;
  if (!lv_find(H, p, k)) { hot_err(H, ERR_CORRUPT); return 0; }
  hot_cancel_at(H, k, loc, ixslot, p, oid, uuid, side, seq);
  return H.fatal ? 0u : 1u;
}

// Duplicate-oid rule (Q7): does (S, oid) name a live node now?  The index after the pending
// inserts of this segment's rests (the deferred inserts of nodes consumed since are dead).
__device__ __forceinline__ bool hot_oid_live(HotCtx& H, uint32_t oid) {
  if (lds_get(H.S->nflushed) < H.npend) hot_flush(H);
  uint32_t ixslot, loc;
  return hot_idx_lookup(H, oid, ixslot, loc);
}

// Write the book back to HBM: head volumes into their cached chunks, every cached chunk,
// then the level array into the book's level block.
__device__ __forceinline__ void hot_writeback(HotCtx& H, GOME_GLB Level* Lv) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id();
  for (uint32_t k = lane; k < H.nl; k += 64) {
    const LvRec r = S->lv[k];
    const uint32_t cs = sl_cs(r.sl);
    if (cs != CS_NONE) *as_lds(&S->cs[cs][sl_hs(r.sl)].rem) = r.hrem;
  }
  for (uint32_t cs = 0; cs < NCS; ++cs) {
    const uint32_t c = uni(S->cs_chunk[cs]);
    if (c != NIL && lane < CH) {
      const uint4* src = reinterpret_cast<const uint4*>(&S->cs[cs][lane]);
      uint4* dst = reinterpret_cast<uint4*>(&H.nodes[c * CH + lane]);
      const uint4 a = src[0], b = src[1];
      dst[0] = a;
      dst[1] = b;
    }
  }
  hot_publish_ids(H, S->freed, lds_get(S->nfreed));  // released chunks
  hot_publish_ids(H, S->pool, lds_get(S->npool));    // claimed but unused chunks go back too
  // Level {price, depth, head, tail, hslot, tslot, member, pad, nlive} as two 16-B stores
  auto put = [&](uint32_t k, uint32_t m) {
    const LvRec r = S->lv[k];
    GOME_GLB v4u* d = (GOME_GLB v4u*)(&Lv[k]);
    d[0] = v4(lo32(r.pr), hi32(r.pr), lo32(r.dp), hi32(r.dp));
    d[1] = v4(r.hd, r.tl, sl_hs(r.sl) | (sl_ts(r.sl) << 8) | (m << 16), r.nv);
  };
  if (lane < H.nl) put(lane, H.M0);
  if (lane + 64 < H.nl) put(lane + 64, H.M1);
}

// Spill path: resolve every pending entry inline so that resting nodes carry real index
// slots, as the HBM path expects; must run before hot_writeback.
__device__ __forceinline__ void hot_resolve_pending(HotCtx& H) {
  hot_flush(H);
  for (uint32_t i = lane_id(); i < H.npend; i += 64) H.pend[i].used = 0;
}

// A head book the flow path planned and then handed over (FlowHdr::bail, k_flow_stale_check): the
// check stores bail, then ok = 0 (release), so a reader that sees ok == 0 from it sees bail too.
__device__ __forceinline__ bool hot_bailed(const FlowHdr* flow, uint32_t h, bool* ok) {
  *ok = __hip_atomic_load(const_cast<uint32_t*>(&flow[h].ok), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0;
  return !*ok && __hip_atomic_load(const_cast<uint32_t*>(&flow[h].bail), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// mode 0: the candidates the flow path declined at its prep (the main launch); mode 1: the books of
// candidates [h0, h1) it handed over after their plan (bail), on the stream of their reconstruction.
__global__ __launch_bounds__(64) void k_match_hot(Dev D, BatchArgs B, PendEnt* pend_arena,
                                                   ResumeRec* resume, const FlowHdr* flow, uint32_t mode = 0,
                                                   uint32_t h0 = 0, uint32_t h1 = 0) {
  extern __shared__ __align__(16) unsigned char smem[];
  if (blockIdx.x >= D.st->nhot || (D.st->err & ERR_INPUT)) return;
  bool fok;
  const bool bailed = hot_bailed(flow, blockIdx.x, &fok);
  if (mode == 1 && (blockIdx.x < h0 || blockIdx.x >= h1 || !bailed)) return;
  if (mode == 0 && (fok || bailed ||  // applied by the flow path (match_flow.h), or handed over later
      B.seg_start[B.seg_order[blockIdx.x] + 1] - B.seg_start[B.seg_order[blockIdx.x]] < LEGACY_HOT_MIN)) {
    if (lane_id() == 0) resume[blockIdx.x].valid = 0;  // declined and short: the cold kernel
    return;
  }
  __builtin_amdgcn_s_setprio(3);  // the hottest books are the batch's critical path
  const uint32_t lane = lane_id();
  const uint32_t seg = B.seg_order[blockIdx.x];
  const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
  const uint32_t sym = uni(B.ord[B.prep[beg].idx].symbol_id);
  const Book bk = D.books[sym];
  const uint32_t nl0 = uni(bk.n_lvl);
  if (nl0 > LRB_CAP - 16) {  // deep book: the HBM path applies the whole segment
    if (lane == 0) {
      ResumeRec rr{};
      rr.valid = 1;
      rr.next = beg;
      resume[blockIdx.x] = rr;
    }
    return;
  }
  HotLds* S = reinterpret_cast<HotLds*>(smem);
  if (lane == 0) {
    HotEnv e;
    e.st = D.st;
    e.idx = D.idx;
    e.idx_mask = D.idx_mask;
    e.free_ids = D.free_ids;
    e.freed_ids = D.freed_ids;
    e.ch_bump = D.ch_bump;
    e.prep = B.prep;
    e.ev_count = B.ev_count;
    e.books = D.books;
    e.lvl = D.lvl;
    e.lvl_bump = D.lvl_bump;
    e.resume = resume;
    e.lpool = lvl_pool(D);
    e.dup_list = B.dup_list;
    e.ch_cap = D.ch_cap;
    e.arena_cap = B.arena_cap;
    e.lvl_cap_total = D.lvl_cap_total;
    e.lvl_base = bk.lvl_base;
    e.lvl_cap = bk.lvl_cap;
    e.beg = beg;
    e.end = end;
    e.pad = 0;
    S->env = e;
    S->nfree = NCS;
    S->npool = S->nfreed = S->nflushed = 0;
    S->bflags = bk.pad | ((bk.pad & BOOK_ZERO) ? BOOK_QUIRK : 0u);  // (L_ZERO marks: k_requalify redoes them)
    S->rr = ResumeRec{};
  }
#ifdef GOME_STAMPS
  if (lane < 16) S->st[lane] = 0;
#endif
  HotCtx H;
  H.S = S;
  H.nodes = D.nodes;
  H.chdr = D.chdr;
  H.arena = B.arena;
  H.pend = pend_arena + beg;
  H.sym = vreg(sym);
  H.nl = nl0;
  H.npend = 0;
  H.ev_base = NIL;
  H.ev_used = EVB_HOT;
  H.fills = vreg(0u);  // counters never feed scalar control flow
  H.pops = vreg(0u);
  H.rests = vreg(0u);
  H.cancels = vreg(0u);
  H.adds = vreg(0u);
  H.dels = vreg(0u);
  H.dropped = vreg(0u);
  H.lvd = vreg(0);
  H.fatal = false;
  const Level* L0 = D.lvl + uni(bk.lvl_base);
  for (uint32_t c = lane; c < NCS; c += 64) {
    S->freeslot[c] = static_cast<uint8_t>(c);
    S->cs_chunk[c] = NIL;
  }
  for (uint32_t k = lane; k < H.nl; k += 64) {
    const Level x = L0[k];
    LvRec r{};
    r.pr = x.price;
    r.dp = x.depth;
    r.hd = x.head;
    r.tl = x.tail;
    r.hn = NIL;
    r.nv = x.nlive;
    r.sl = sl_make(x.hslot, x.tslot, CS_NONE, HN_UNKNOWN);
    r.mem = x.member;
    S->lv[k] = r;
  }
  lv_regs_from_lds(H);

  bool spilled = false;
  for (uint32_t b0 = beg; b0 < end && !H.fatal && !spilled; b0 += 64) {
    const uint32_t cnt = min(64u, end - b0);
    // This block's records, loaded synchronously and laundered through asm so that the
    // wait sits here and not inside the order loop (where vmcnt(0) would also wait for
    // the previous order's stores).
    v4u qa = v4(0u, 0u, 0u, 0u), qb = v4(0u, 0u, 0u, 0u);
    if (b0 + lane < end) {
      const GOME_GLB v4u* src = (const GOME_GLB v4u*)(&gp(S->env.prep)[b0 + lane]);
      qa = src[0];
      qb = src[1];
    }
    const uint4 x = make_uint4(vreg(qa.x), vreg(qa.y), vreg(qa.z), vreg(qa.w));
    const uint4 y = make_uint4(vreg(qb.x), vreg(qb.y), vreg(qb.z), vreg(qb.w));
    // Prep {price, vol | oid, uuid, idx, side|action<<8|adm<<16}
    uint32_t evc = 0;  // lane j: events of order j of this block
    uint32_t j = 0;
    for (; j < cnt && !H.fatal; ++j) {
      ST_T0(t_o)
      const uint32_t fl = rl(y.w, j), a = (fl >> 8) & 0xFFu;
      uint32_t nev = 0;
      if (a == GOME_ADD) {
        const uint32_t admv = (fl >> 16) & 0xFFu;
        if (admv == ADM_V_CHECK && hot_oid_live(H, rl(y.x, j))) {
          // (S, oid) names a live node: the duplicate-oid rule (Q7, pipeline.h)
          H.dropped += 1u;
          if (lane == 0) dup_note(S->env.st, S->env.dup_list, rl(y.z, j));
        } else if (admv != ADM_V_NO) {
          int64_t trest = 0;
          const int64_t p = static_cast<int64_t>((static_cast<uint64_t>(rl(x.y, j)) << 32) | rl(x.x, j));
          const int64_t v = static_cast<int64_t>((static_cast<uint64_t>(rl(x.w, j)) << 32) | rl(x.z, j));
          const uint32_t oid = rl(y.x, j), uuid = rl(y.y, j), side = fl & 0xFFu;
          // The most common case (no crossing level, the rest level exists) is decided
          // here and handled without entering hot_add.
          const uint32_t opp = side != GOME_SALE ? M_SALE : M_BUY;
          const bool c0 = (H.M0 & opp) && (side != GOME_SALE ? H.P0 <= p : H.P0 >= p);
          const bool c1 = (H.M1 & opp) && (side != GOME_SALE ? H.P1 <= p : H.P1 >= p);
          const unsigned long long cr = __ballot(c0) | __ballot(c1);
          const unsigned long long q0 = __ballot(H.P0 == p), q1 = __ballot(H.P1 == p);
          if (cr == 0 && (q0 | q1)) {
            hot_rest_fast(H, q0 ? static_cast<uint32_t>(__builtin_ctzll(q0)) : 64u + static_cast<uint32_t>(__builtin_ctzll(q1)),
                          p, v, oid, uuid, side);
          } else if (!hot_add(H, p, v, oid, uuid, side, rl(y.z, j), nev, trest)) {
            spilled = true;  // lane array full: the HBM path rests it and continues
            if (lane == 0) {
              ResumeRec r{};
              r.valid = 1;
              r.next = b0 + j + 1;
              r.rest = 1;
              r.price = p;
              r.vol = trest;
              r.oid = oid;
              r.uuid = uuid;
              r.side = side;
              S->rr = r;
            }
          }
        }
      } else if (a == GOME_DEL) {
        const int64_t p = static_cast<int64_t>((static_cast<uint64_t>(rl(x.y, j)) << 32) | rl(x.x, j));
        nev = hot_cancel(H, p, rl(y.x, j), rl(y.y, j), fl & 0xFFu, rl(y.z, j));
      }
      evc = wl(evc, nev, j);
      ST_ADD(0, t_o)
      if (spilled) { ++j; break; }
    }
    const uint32_t act = (y.w >> 8) & 0xFFu;
    const bool mine = lane < j;
    H.adds += __popcll(__ballot(mine && act == GOME_ADD));
    H.dels += __popcll(__ballot(mine && act == GOME_DEL));
    H.dropped += __popcll(__ballot(mine && act == GOME_ADD && ((y.w >> 16) & 0xFFu) == ADM_V_NO));
    if (mine) gp(S->env.ev_count)[y.z] = evc;
  }
  if (spilled) hot_resolve_pending(H);  // the HBM path expects real index slots
  hot_ev_close(H);
#ifdef GOME_STAMPS
  if (lane < 16 && blockIdx.x < 256) g_stamps[blockIdx.x * NSTAMP + lane] = S->st[lane];
#endif
  // everything below reads the environment from LDS, not the kernel arguments, so the
  // compiler need not keep those live in SGPRs across the order loop
  const HotEnv& E = S->env;
  const uint32_t beg2 = uni(E.beg), end2 = uni(E.end);
  uint32_t base = uni(E.lvl_base), cap = uni(E.lvl_cap);
  if (H.nl > cap) {  // level block of the book, grown if the lane book outgrew it
    uint32_t ncap = 16;
    while (ncap < H.nl) ncap <<= 1;
    uint32_t nb = 0;
    if (lane == 0) {
      const LvlPool P = S->env.lpool;
      nb = lvl_block_alloc(P, ncap);
      if (nb != NIL) lvl_block_release(P, base, cap);  // the book's old block
    }
    nb = uni(nb);
    if (nb == NIL) hot_err(H, ERR_LEVELS);
    else { base = nb; cap = ncap; }
  }
  if (H.nl <= cap) hot_writeback(H, gp(E.lvl) + base);
  if (lane == 0) {
    GOME_GLB v4u* rp = (GOME_GLB v4u*)(&gp(E.resume)[blockIdx.x]);
    const ResumeRec rr = S->rr;
    rp[0] = v4(rr.valid, rr.next, rr.rest, rr.oid);
    rp[1] = v4(rr.uuid, rr.side, 0u, 0u);  // pad0, pad1
    rp[2] = v4(lo32(rr.price), hi32(rr.price), lo32(rr.vol), hi32(rr.vol));
    *(GOME_GLB v4u*)(&gp(E.books)[H.sym]) = v4(base, H.nl, cap, S->bflags);
    GOME_GLB unsigned long long* c = gp(E.st)->ctr;
    const long long resting = static_cast<long long>(H.rests) - H.pops - H.cancels;
    auto add = [&](int i, long long v) { if (v) G_ADD(&c[i], static_cast<unsigned long long>(v)); };
    add(C_FILLS, H.fills);
    add(C_CANCELS, H.cancels);
    add(C_RESTS, H.rests);
    add(C_DROPPED, H.dropped);
    add(C_ADD, H.adds);
    add(C_DEL, H.dels);
    add(C_RESTING_DELTA, resting);
    add(C_LEVELS_DELTA, H.lvd);
    add(C_HOT_ORDERS, static_cast<long long>((spilled ? rr.next : end2) - beg2));
    add(C_HOT_FILLS, H.fills);
    add(C_HOT_RESTS, H.rests);
    add(C_HOT_CANCELS, H.cancels);
  }
}

// Continue hot books that left the lane path (see ResumeRec) on the HBM path.
__global__ __launch_bounds__(64) void k_match_resume(Dev D, BatchArgs B, const ResumeRec* resume,
                                                      const FlowHdr* flow = nullptr, uint32_t h0 = 0,
                                                      uint32_t h1 = 0) {
  if (blockIdx.x >= D.st->nhot || (D.st->err & ERR_INPUT)) return;
  if (flow) {  // (mode 1: the handed-over books of [h0, h1) only)
    bool fok;
    if (blockIdx.x < h0 || blockIdx.x >= h1 || !hot_bailed(flow, blockIdx.x, &fok)) return;
  }
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
                             const uint32_t* seg_order, const BatchArgs B, const FlowHdr* flow = nullptr,
                             uint32_t h0 = 0, uint32_t h1 = 0) {
  const uint32_t nhot = min(D.st->nhot, MAX_HOT);
  const unsigned long long mask = D.idx_mask;
  for (uint32_t h = blockIdx.y; h < nhot; h += gridDim.y) {
    bool fok;
    if (flow && (h < h0 || h >= h1 || !hot_bailed(flow, h, &fok))) continue;  // (mode 1)
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
