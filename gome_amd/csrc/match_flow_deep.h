// match_flow_deep.h — the flow path for deep head books: more price levels than the lane plans
// hold (FL_MAX), up to DEEP_CAP - 2 (config 5's 4-dp price grid: ~10k levels per book).
//
// The matching semantics are the flow path's (match_flow.h): a serial aggregate plan over level
// depths, then the parallel reconstruction of fills and FIFOs.  What changes with the level
// count:
//   k_deep_prep_a/b/c   the price set in a global-memory hash per book (DEEP_HASH slots), sorted
//                       in LDS (bitonic, one workgroup), old levels merged; FlowLvl in F.dlvl;
//                       32-bit records with a 14-bit level index (hi = level | SALE << 31)
//   plan                gen_plan_asm.py W32D: depths in LDS (fl_deep_load / fl_deep_store),
//                       the next level after an emptied top by 64-slot reads; a touch carries
//                       its level in Touch::pos
//   k_deep_sort_*       stable LSD sort of the touches by level, two 7-bit passes through
//                       F.tlog (each pass the head sort's tile count / scan / scatter)
//   k_deep_runs/level   the run of each touched level in the sorted touches, then fl_level_one
//                       on the touched levels only (the prep leaves an untouched level final);
//                       count and events are the ADD-only kernels (fl_touch_ctx reads a deep
//                       touch's level from its sorted entry)
//   k_deep_write_*      FIFO appends per touched level (untouched ones copied lane-parallel),
//                       the book's level array compacted by a scan.
// Declines (the book goes to the legacy kernel, bit-exact as before): DELs in the segment,
// zero-volume ADDs (Q6), quirk books, more than DEEP_CAP - 2 levels, volumes beyond the 32-bit
// plan.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "match_cold.h"
#include "match_flow.h"
#include "match_flow_cancel.h"
#include "pipeline.h"
#include "wave.h"

namespace gome {

__device__ __forceinline__ uint32_t fd_hash(unsigned long long key) {
  return static_cast<uint32_t>(mix64(key) >> 16) & (DEEP_HASH - 1);
}

// Insert key (nonzero) into a book's price set; the slot, or NIL when full.
__device__ __forceinline__ uint32_t fd_put(unsigned long long* keys, unsigned long long key, bool* fresh) {
  uint32_t s = fd_hash(key);
  *fresh = false;
  for (uint32_t probe = 0; probe < DEEP_HASH; ++probe) {
    const unsigned long long cur = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return s;
    if (cur == 0ull) {
      const unsigned long long prev = atomicCAS(&keys[s], 0ull, key);
      if (prev == 0ull) {
        *fresh = true;
        return s;
      }
      if (prev == key) return s;
    }
    s = (s + 1) & (DEEP_HASH - 1);
  }
  return NIL;
}

__device__ __forceinline__ uint32_t fd_find(const unsigned long long* keys, unsigned long long key) {
  uint32_t s = fd_hash(key);
  for (uint32_t probe = 0; probe < DEEP_HASH; ++probe) {
    const unsigned long long cur = keys[s];
    if (cur == key) return s;
    if (cur == 0ull) return NIL;
    s = (s + 1) & (DEEP_HASH - 1);
  }
  return NIL;
}

// The book of deep slot ds (launches cover the slots [ds0, ds1) of their range), NIL if none.
__device__ __forceinline__ uint32_t fd_book(const Dev& D, const FlowArgs& F, uint32_t i) {
  const uint32_t ds = F.ds0 + i;
  if (ds >= F.ds1) return NIL;
  const uint32_t h = F.dslot_h[ds];
  return (h != NIL && h < fl_hend(D, F) && F.hdr[h].dslot == ds) ? h : NIL;
}

// Deep slots a launch of this range walks: the head's are fixed (slot = candidate), the tail's
// are handed out by its prep in the order it finds deep books (F.dslot_n).
__device__ __forceinline__ uint32_t fd_nslots(const FlowArgs& F) {
  return F.ds0 >= FL_HEAD ? min(F.ds1 - F.ds0, *F.dslot_n) : F.ds1 - F.ds0;
}

// A deep slot's sort tile counts (seg_order is longest first: candidate h has at most
// 1 / (h + 1) of the batch, so a tail slot needs at most an eighth of the head's tiles).
__device__ __forceinline__ uint32_t* fd_tcnt(const FlowArgs& F, uint32_t ds) {
  const size_t t = ds < FL_HEAD ? static_cast<size_t>(ds) * F.dmaxt
                                : static_cast<size_t>(FL_HEAD) * F.dmaxt + static_cast<size_t>(ds - FL_HEAD) * F.dtmaxt;
  return F.dtcnt + t * FL_CAP;
}
__device__ __forceinline__ uint32_t fd_tiles(const FlowArgs& F, uint32_t ds) { return ds < FL_HEAD ? F.dmaxt : F.dtmaxt; }

// A slot's price set back to empty (kept clean between batches instead of a per-batch memset).
__device__ __forceinline__ void fd_clear(const FlowArgs& F, uint32_t ds) {
  unsigned long long* keys = F.dh_key + static_cast<size_t>(ds) * DEEP_HASH;
  uint32_t* vals = F.dh_val + static_cast<size_t>(ds) * DEEP_HASH;
  for (uint32_t i = threadIdx.x; i < DEEP_HASH; i += blockDim.x) {
    keys[i] = 0ull;
    vals[i] = NIL;
  }
}

__device__ __forceinline__ bool fd_candidate(const Dev& D, const FlowArgs& F, uint32_t h) {
  return h != NIL && F.hdr[h].deep && !F.hdr[h].ok;
}

__device__ __forceinline__ bool fd_deep(const FlowArgs& F, uint32_t h) {
  return h != NIL && F.hdr[h].ok == FL_OK_DEEP;
}

// Slice x of nx of [beg, end).
__device__ __forceinline__ void fd_slice(uint32_t beg, uint32_t end, uint32_t x, uint32_t nx, uint32_t& b0, uint32_t& b1) {
  const uint64_t len = end - beg;
  b0 = beg + static_cast<uint32_t>(len * x / nx);
  b1 = beg + static_cast<uint32_t>(len * (x + 1) / nx);
}

// ---- prep a: per slice, the batch's prices into the set, gcd / sum, counts ----------------
__device__ __forceinline__ void k_deep_prep_a_one(Dev D, BatchArgs B, FlowArgs F, uint32_t slot_i) {
  __shared__ uint32_t adds, dropped, dels, bad, nd;
  __shared__ unsigned long long wg[FL_PREP_T / 64], ws[FL_PREP_T / 64];
  const uint32_t h = fd_book(D, F, slot_i), tid = threadIdx.x;
  if (!fd_candidate(D, F, h)) return;
  const uint32_t ds = F.hdr[h].dslot;
  FlPrepScr* P = F.dscr + ds;
  unsigned long long* keys = F.dh_key + static_cast<size_t>(ds) * DEEP_HASH;
  const uint32_t seg = B.seg_order[h];
  uint32_t b0, b1;
  fd_slice(B.seg_start[seg], B.seg_start[seg + 1], blockIdx.x, gridDim.x, b0, b1);
  if (tid == 0) adds = dropped = dels = bad = nd = 0;
  __syncthreads();
  unsigned long long mg = 0, msum = 0;
  uint32_t my_adds = 0, my_drop = 0, my_dels = 0, my_bad = 0, my_nd = 0;
  for (uint32_t b = b0 + tid; b < b1; b += FL_PREP_T) {
    const Prep q = prep_at(B, b);
    if (q.action == GOME_DEL) { my_dels++; continue; }
    if (q.action != GOME_ADD) continue;
    my_adds++;
    if (!q.adm) { my_drop++; continue; }
    if (q.vol == 0 || q.adm == ADM_V_CHECK) { my_bad = 1; continue; }  // a zero-volume maker (Q6), a Q7 candidate
    const unsigned long long v = static_cast<unsigned long long>(q.vol);
    mg = fl_gcd(mg, v);
    msum = min(msum + v, FL_SUM_CAP);
    bool fresh;
    if (fd_put(keys, static_cast<unsigned long long>(q.price) + FL_KEY_OFF, &fresh) == NIL) my_bad = 1;
    my_nd += fresh ? 1u : 0u;
  }
  if (my_adds) atomicAdd(&adds, my_adds);
  if (my_drop) atomicAdd(&dropped, my_drop);
  if (my_dels) atomicAdd(&dels, my_dels);
  if (my_bad) bad = 1;
  if (my_nd) atomicAdd(&nd, my_nd);
  fl_block_gcd_sum(mg, msum, wg, ws);  // (synchronises the block)
  if (tid == 0) {
    P->pg[blockIdx.x] = mg;
    P->ps[blockIdx.x] = msum;
    if (adds) atomicAdd(&P->d_adds, adds);
    if (dropped) atomicAdd(&P->d_dropped, dropped);
    if (dels) atomicAdd(&P->d_dels, dels);
    if (bad) atomicOr(&P->d_bad, 1u);
    if (nd) atomicAdd(&P->d_ndist, nd);
  }
}
__global__ __launch_bounds__(FL_PREP_T) void k_deep_prep_a(Dev D, BatchArgs B, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) {
    k_deep_prep_a_one(D, B, F, i);
    __syncthreads();
  }
}

// ---- prep b: old levels into the set, the sorted level table, the header -----------------
// Dynamic LDS: DEEP_CAP keys (the sort).
// Ranks of a deep book's price set (keys in its DEEP_HASH slots, n of them) by a bitmap over the
// grid the keys lie on: slot[r] = the hash slot of the r-th key (LDS).  False (nothing done) when
// the keys span 2^32 or more, or their offsets from the lowest key over their gcd more than
// FD_RANK_BITS.  The whole block; the bitmap, its word prefix and slot[] in the dynamic LDS.
constexpr uint32_t FD_RANK_BITS = 1u << 17, FD_RANK_WORDS = FD_RANK_BITS / 32;
__device__ __forceinline__ uint32_t fd_gcd32(uint32_t a, uint32_t b) {  // (binary: no divisions)
  if (!a) return b;
  if (!b) return a;
  const int sh = __builtin_ctz(a | b);
  a >>= __builtin_ctz(a);
  do {
    b >>= __builtin_ctz(b);
    if (a > b) { const uint32_t t = a; a = b; b = t; }
    b -= a;
  } while (b);
  return a << sh;
}
__device__ __forceinline__ bool fd_rank_grid(const unsigned long long* keys, uint32_t n, uint32_t** slot_out) {
  __shared__ unsigned long long kmin_s, kmax_s;
  __shared__ uint32_t g_s[FL_PREP_T / 64], part_s[FL_PREP_T / 64];
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
#ifdef GOME_PROBE_LEVEL
  const bool pr = blockIdx.x == 0 && n > 4096;
  uint64_t pt = wall_clock64();
#define PR(k) do { if (pr) { GOME_PROBE_T(k, pt); pt = wall_clock64(); } } while (0)
#else
#define PR(k) do { } while (0)
#endif
  // one pass for the bounds and the grid (two passes over the 2^16 slots until round 6): a thread
  // takes the offsets of its keys from its first one, and the gcd of those and of the threads' first
  // keys' offsets from the lowest key is the grid (the offsets from any one key of the set generate
  // the same lattice as the offsets from the lowest)
  if (tid == 0) { kmin_s = ~0ull; kmax_s = 0; }
  __syncthreads();
  unsigned long long mn = ~0ull, mx = 0, r = 0;
  uint32_t g = 0;
  constexpr uint32_t U = 4;  // (four loads in flight a thread)
  for (uint32_t s0 = tid; s0 < DEEP_HASH; s0 += U * FL_PREP_T) {
    unsigned long long kk[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) kk[u] = s0 + u * FL_PREP_T < DEEP_HASH ? keys[s0 + u * FL_PREP_T] : 0ull;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const unsigned long long k = kk[u];
      if (!k) continue;
      mn = min(mn, k);
      mx = max(mx, k);
      if (!r) r = k;
      else g = fd_gcd32(g, static_cast<uint32_t>(k >= r ? k - r : r - k));  // (garbage past 2^32: refused below)
    }
  }
  atomicMin(&kmin_s, mn);
  atomicMax(&kmax_s, mx);
  __syncthreads();
  PR(20);
  const unsigned long long kmin = kmin_s, kmax = kmax_s;
  if (n == 0 || kmax < kmin || kmax - kmin >= (1ull << 32)) return false;  // (uniform)
  if (r) g = fd_gcd32(g, static_cast<uint32_t>(r - kmin));
  for (int off = 32; off > 0; off >>= 1) g = fd_gcd32(g, __shfl_xor(g, off));
  if (lane == 0) g_s[w] = g;
  __syncthreads();
  g = 0;
  for (uint32_t k = 0; k < FL_PREP_T / 64; ++k) g = fd_gcd32(g, g_s[k]);
  if (!g) g = 1;  // (one key)
  PR(21);
  if (static_cast<uint32_t>(kmax - kmin) / g >= FD_RANK_BITS) return false;
  uint32_t* bm = reinterpret_cast<uint32_t*>(fl_ring);
  uint32_t* pre = bm + FD_RANK_WORDS;
  uint32_t* slot = pre + FD_RANK_WORDS;  // [DEEP_CAP]
  for (uint32_t i = tid; i < FD_RANK_WORDS; i += FL_PREP_T) bm[i] = 0;
  __syncthreads();
  for (uint32_t s0 = tid; s0 < DEEP_HASH; s0 += U * FL_PREP_T) {
    unsigned long long kk[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) kk[u] = s0 + u * FL_PREP_T < DEEP_HASH ? keys[s0 + u * FL_PREP_T] : 0ull;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      if (!kk[u]) continue;
      const uint32_t x = static_cast<uint32_t>(kk[u] - kmin) / g;
      atomicOr(&bm[x >> 5], 1u << (x & 31));
    }
  }
  __syncthreads();
  PR(22);
  // exclusive prefix of the words' popcounts: FD_RANK_WORDS / FL_PREP_T consecutive words a thread
  constexpr uint32_t PW = FD_RANK_WORDS / FL_PREP_T;
  static_assert(FD_RANK_WORDS % FL_PREP_T == 0, "whole words per thread");
  static_assert(2 * FD_RANK_WORDS * 4 + DEEP_CAP * 4 <= DEEP_CAP * 8, "bitmap, prefix and slots in the sort's LDS");
  uint32_t loc[PW], s = 0;
#pragma unroll
  for (uint32_t k = 0; k < PW; ++k) {
    loc[k] = s;
    s += __popc(bm[tid * PW + k]);
  }
  const uint32_t inc = wave_incl_scan_u32(s);
  if (lane == 63) part_s[w] = inc;
  __syncthreads();
  uint32_t before = 0, tot = 0;
  for (uint32_t k = 0; k < FL_PREP_T / 64; ++k) {
    before += k < w ? part_s[k] : 0u;
    tot += part_s[k];
  }
  const uint32_t ex = before + inc - s;
#pragma unroll
  for (uint32_t k = 0; k < PW; ++k) pre[tid * PW + k] = ex + loc[k];
  __syncthreads();
  PR(23);
  if (tot != n || n > DEEP_CAP) return false;  // (uniform: every key set its own bit)
  for (uint32_t s0 = tid; s0 < DEEP_HASH; s0 += U * FL_PREP_T) {
    unsigned long long kk[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) kk[u] = s0 + u * FL_PREP_T < DEEP_HASH ? keys[s0 + u * FL_PREP_T] : 0ull;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      if (!kk[u]) continue;
      const uint32_t x = static_cast<uint32_t>(kk[u] - kmin) / g;
      slot[pre[x >> 5] + __popc(bm[x >> 5] & ((1u << (x & 31)) - 1u))] = s0 + u * FL_PREP_T;
    }
  }
  __syncthreads();
  PR(24);
#undef PR
  *slot_out = slot;
  return true;
}

__device__ __forceinline__ void k_deep_prep_b_one(Dev D, BatchArgs B, FlowArgs F, uint32_t slot_i) {
  __shared__ uint32_t bad, ndist, nc;
  __shared__ unsigned long long wg[FL_PREP_T / 64], ws[FL_PREP_T / 64];
  const uint32_t h = fd_book(D, F, slot_i), tid = threadIdx.x;
  if (!fd_candidate(D, F, h)) return;
  FlowHdr* hd = &F.hdr[h];
  const uint32_t ds = hd->dslot;
  FlPrepScr* P = F.dscr + ds;
  unsigned long long* keys = F.dh_key + static_cast<size_t>(ds) * DEEP_HASH;
  uint32_t* vals = F.dh_val + static_cast<size_t>(ds) * DEEP_HASH;
  const uint32_t seg = B.seg_order[h];
  const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
  const uint32_t sym = B.ord[B.sidx[beg]].symbol_id;
  const Book bk = D.books[sym];
  if (tid == 0) {
    // (a segment with DELs takes the W32DC plan after the cancel prep)
    const uint64_t tiles = (static_cast<uint64_t>(FL_TOUCH_MUL) * (end - beg) + FL_TILE - 1) / FL_TILE;
    bad = (P->d_bad || (bk.pad & (BOOK_QUIRK | BOOK_ZERO | BOOK_STALE)) || bk.n_lvl > DEEP_CAP - 2 || tiles > fd_tiles(F, ds)) ? 1u : 0u;
    if (!bad && P->d_dels) {  // the W32DC plan needs the cancel chain
      ctr_add(D, C_WANT_CANC, 1ull);
      if (!(F.chains & FL_CH_CANCEL)) bad = 1;
    }
    ndist = P->d_ndist;
    nc = 0;
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) hd->deep = 0;
    fd_clear(F, ds);
    return;
  }
  const Level* L0 = D.lvl + bk.lvl_base;
#ifdef GOME_PROBE_LEVEL
  const bool pr = slot_i == 0;
  uint64_t pt = wall_clock64();
#define PB(k) do { if (pr) { GOME_PROBE_T(k, pt); pt = wall_clock64(); } } while (0)
#else
#define PB(k) do { } while (0)
#endif
  unsigned long long mg = 0, msum = 0;
  if (tid < FL_PG) {
    mg = P->pg[tid];
    msum = P->ps[tid];
  }
  for (uint32_t k = tid; k < bk.n_lvl; k += FL_PREP_T) {
    const Level x = L0[k];
    const uint32_t nm = (x.member & M_BUY ? 1u : 0u) + (x.member & M_SALE ? 1u : 0u);
    if (x.nlive == 0) {
      if (x.depth != 0 || x.member != 0) bad = 1;
      continue;
    }
    if (x.depth <= 0 || nm != 1) { bad = 1; continue; }
    mg = fl_gcd(mg, static_cast<unsigned long long>(x.depth));
    msum = min(msum + static_cast<unsigned long long>(x.depth), FL_SUM_CAP);
    bool fresh;
    const uint32_t sl = fd_put(keys, static_cast<unsigned long long>(x.price) + FL_KEY_OFF, &fresh);
    if (sl == NIL) { bad = 1; continue; }
    vals[sl] = k;  // the old level (vals start NIL)
    if (fresh) atomicAdd(&ndist, 1u);
  }
  __syncthreads();
  PB(16);
  fl_block_gcd_sum(mg, msum, wg, ws);  // (synchronises the block)
  PB(17);
  const unsigned long long g = mg ? mg : 1;
  const bool w32 = msum < FL_SUM_CAP && msum / g < (1ull << 32);
  if (bad || ndist > DEEP_CAP - 2 || !w32) {
    if (tid == 0) hd->deep = 0;
    fd_clear(F, ds);
    return;
  }
  const uint32_t n = ndist;
  FlowLvl* LV = F.dlvl + static_cast<size_t>(ds) * DEEP_CAP;
  auto put_level = [&](uint32_t r, unsigned long long key, uint32_t sl) {  // level r + 1 = the r-th price
    const uint32_t old = vals[sl];
    FlowLvl f{};
    f.price = static_cast<int64_t>(key - FL_KEY_OFF);
    f.old = old;
    f.head = f.tail = NIL;
    f.ig_all = 1;  // (what k_deep_level leaves on a level the batch does not touch: it skips them)
    if (old != NIL) {
      const Level x = L0[old];
      f.d0 = x.depth;
      f.nv0 = x.nlive;
      f.head = x.head;
      f.tail = x.tail;
      f.hslot = x.hslot;
      f.tslot = x.tslot;
      f.mem0 = x.member;
      f.nlive0 = x.nlive;
    }
    LV[r + 1] = f;
    vals[sl] = r + 1;  // (the set maps price -> level from here on)
  };
  // The keys' ranks.  Prices on a grid (a book's prices are multiples of its tick): the offsets
  // from the lowest key over their gcd index a bitmap of FD_RANK_BITS in LDS, and a key's rank is
  // the bits below its own (popcounts and a scan of the words); a bitonic sort of up to DEEP_CAP
  // keys in LDS took ~250 us of the hottest book's prep (config 5c).  Other sets: the sort.
  uint32_t* slot = nullptr;
  if (fd_rank_grid(keys, n, &slot)) {
    // each rank's hash slot into its level row; k_deep_prep_put fills the rows, many blocks a book
    // (one block took ~0.2 ms of the hottest book's prep here, three dependent loads per level)
    for (uint32_t r = tid; r < n; r += FL_PREP_T) LV[r + 1].pad4 = slot[r];
    if (tid == 0) P->d_put = 1;
    __syncthreads();
    PB(18);
    goto fd_prep_b_hdr;
  }
  {
  // the set's keys, sorted (bitonic over the next power of two)
  uint32_t np = 1024;
  while (np < n) np <<= 1;
  unsigned long long* sk = reinterpret_cast<unsigned long long*>(fl_ring);
  for (uint32_t sl = tid; sl < DEEP_HASH; sl += FL_PREP_T) {
    const unsigned long long key = keys[sl];
    if (key) sk[atomicAdd(&nc, 1u)] = key;
  }
  __syncthreads();
  for (uint32_t i = n + tid; i < np; i += FL_PREP_T) sk[i] = ~0ull;
  __syncthreads();
  for (uint32_t k = 2; k <= np; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = tid; i < np; i += FL_PREP_T) {
        const uint32_t p = i ^ j;
        if (p > i) {
          const unsigned long long a = sk[i], b = sk[p];
          if ((a > b) == ((i & k) == 0)) {
            sk[i] = b;
            sk[p] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t r = tid; r < n; r += FL_PREP_T) {
    const unsigned long long key = sk[r];
    put_level(r, key, fd_find(keys, key));
  }
  }
fd_prep_b_hdr:
  const uint32_t obase = fl_obase(beg, seg);
#undef PB
  if (tid < ((8u - ((end - beg) & 7u)) & 7u)) F.ord8[obase + (end - beg) + tid] = 0ull;  // no-op padding
  if (tid == 0) {
    // the bid sentinel's row: no old level, no FIFO (no level pass reads it; a clean row all the same)
    FlowLvl z{};
    z.old = NIL;
    z.head = z.tail = NIL;
    LV[0] = z;
    FlowHdr x{};
    x.ok = FL_OK_DEEP;
    x.nl = n;
    x.sym = sym;
    x.beg = beg;
    x.end = end;
    x.nold = bk.n_lvl;
    x.adds = P->d_adds;
    x.dropped = P->d_dropped;
    x.obase = obase;
    x.w32 = 1;
    x.g = g;
    x.deep = 1;
    x.dslot = ds;
    x.ndel = P->d_dels;
    x.dc = P->d_dels ? 1u : 0u;
    x.bid = F.bid;
    *hd = x;
  }
}
// The level table of a set k_deep_prep_b ranked by its grid: row r + 1 from the r-th key's hash
// slot (FlowLvl::pad4): its price, its old level's FIFO and depth; the set maps price -> level.
__device__ __forceinline__ void k_deep_prep_put_one(Dev D, FlowArgs F, uint32_t slot_i) {
  const uint32_t h = fd_book(D, F, slot_i);
  if (!fd_deep(F, h)) return;
  const FlowHdr& hd = F.hdr[h];
  const uint32_t ds = hd.dslot;
  if (!F.dscr[ds].d_put) return;
  const unsigned long long* keys = F.dh_key + static_cast<size_t>(ds) * DEEP_HASH;
  uint32_t* vals = F.dh_val + static_cast<size_t>(ds) * DEEP_HASH;
  FlowLvl* LV = F.dlvl + static_cast<size_t>(ds) * DEEP_CAP;
  const Level* L0 = D.lvl + D.books[hd.sym].lvl_base;
  const uint32_t n = hd.nl;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
    const uint32_t sl = LV[r + 1].pad4;
    const unsigned long long key = keys[sl];
    const uint32_t old = vals[sl];
    FlowLvl f{};
    f.price = static_cast<int64_t>(key - FL_KEY_OFF);
    f.old = old;
    f.head = f.tail = NIL;
    f.ig_all = 1;  // (what k_deep_level leaves on a level the batch does not touch: it skips them)
    if (old != NIL) {
      const Level x = L0[old];
      f.d0 = x.depth;
      f.nv0 = x.nlive;
      f.head = x.head;
      f.tail = x.tail;
      f.hslot = x.hslot;
      f.tslot = x.tslot;
      f.mem0 = x.member;
      f.nlive0 = x.nlive;
    }
    LV[r + 1] = f;
    vals[sl] = r + 1;
  }
}
__global__ __launch_bounds__(FL_PREP_T) void k_deep_prep_put(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) k_deep_prep_put_one(D, F, i);
}

__global__ __launch_bounds__(FL_PREP_T) void k_deep_prep_b(Dev D, BatchArgs B, FlowArgs F) {
  for (uint32_t i = blockIdx.x; i < fd_nslots(F); i += gridDim.x) {
    k_deep_prep_b_one(D, B, F, i);
    __syncthreads();
  }
}

// ---- prep c: the 32-bit records (level index from the set) ---------------------------------
__device__ __forceinline__ void k_deep_prep_c_one(Dev D, BatchArgs B, FlowArgs F, uint32_t slot_i) {
  const uint32_t h = fd_book(D, F, slot_i), tid = threadIdx.x;
  if (!fd_deep(F, h)) return;
  const FlowHdr* hd = &F.hdr[h];
  const unsigned long long* keys = F.dh_key + static_cast<size_t>(hd->dslot) * DEEP_HASH;
  const uint32_t* vals = F.dh_val + static_cast<size_t>(hd->dslot) * DEEP_HASH;
  const uint32_t beg = hd->beg, obase = hd->obase;
  const unsigned long long g = hd->g;
  uint32_t b0, b1;
  fd_slice(beg, hd->end, blockIdx.x, gridDim.x, b0, b1);
  for (uint32_t b = b0 + tid; b < b1; b += FL_PREP_T) {
    const Prep q = prep_at(B, b);
    unsigned long long rec = 0ull;  // no-op: a rest of 0 at the bid sentinel
    if (q.action == GOME_ADD && q.adm) {
      const uint32_t li = vals[fd_find(keys, static_cast<unsigned long long>(q.price) + FL_KEY_OFF)];
      const unsigned long long v = static_cast<unsigned long long>(static_cast<double>(q.vol) / static_cast<double>(g));
      rec = (static_cast<unsigned long long>(li | (q.side == GOME_SALE ? 0x80000000u : 0u)) << 32) | v;
    }
    F.ord8[obase + (b - beg)] = rec;
    B.ev_count[q.idx] = 0;
  }
}
__global__ __launch_bounds__(FL_PREP_T) void k_deep_prep_c(Dev D, BatchArgs B, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) {
    k_deep_prep_c_one(D, B, F, i);
    __syncthreads();
  }
}

// ---- sort: two stable 7-bit passes by level (tile counts, per-book scan, scatter) ---------
// PASS 1 reads the plan's log (level in Touch::pos) and writes F.tlog in low-7-bit order, the
// touch's log index in the amount's high word; PASS 2 writes the level-ordered SEnt runs.
template <int PASS>
__device__ __forceinline__ uint32_t fd_key(const FlowArgs& F, uint32_t L, uint32_t t, Touch& x) {
  x = (PASS == 1 ? F.log : F.tlog)[L + t];
  return PASS == 1 ? (x.pos & 127u) : (x.pos >> 7);
}

template <int PASS>
__device__ __forceinline__ void k_deep_sort_cnt_one(Dev D, FlowArgs F, uint32_t slot_i) {
  __shared__ uint32_t wc[FL_TILE_W][FL_CAP];
  __shared__ uint32_t nrest;
  const uint32_t h = fd_book(D, F, slot_i), tid = threadIdx.x, w = tid >> 6;
  if (!fd_deep(F, h)) return;
  const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg;
  const uint32_t ntile = (nt + FL_TILE - 1) / FL_TILE;
  for (uint32_t tl = blockIdx.x; tl < ntile; tl += gridDim.x) {
    for (uint32_t i = tid; i < FL_TILE_W * FL_CAP; i += FL_TILE) wc[i / FL_CAP][i % FL_CAP] = 0;
    if (tid == 0) nrest = 0;
    __syncthreads();
    const uint32_t t = tl * FL_TILE + tid;
    const bool valid = t < nt;
    Touch x{};
    const uint32_t k = valid ? fd_key<PASS>(F, L, t, x) : 0u;
    uint32_t cnt;
    const uint32_t rank = fl_tile_rank(k, valid, cnt);
    if (valid && rank == 0) wc[w][k] = cnt;
    if (PASS == 1) {
      const unsigned long long rm = __ballot(valid && ((x.kr >> 7) & 1u) == TK_REST && x.pos != 0);
      if (lane_id() == 0 && rm) atomicAdd(&nrest, static_cast<uint32_t>(__popcll(rm)));
    }
    __syncthreads();
    if (tid < FL_CAP) {
      uint32_t c = 0;
      for (uint32_t ww = 0; ww < FL_TILE_W; ++ww) c += wc[ww][tid];
      fd_tcnt(F, F.hdr[h].dslot)[static_cast<size_t>(tl) * FL_CAP + tid] = c;
    }
    if (PASS == 1 && tid == 0 && nrest) atomicAdd(&F.hdr[h].rests, nrest);
    __syncthreads();
  }
}
template <int PASS>
__global__ __launch_bounds__(FL_TILE) void k_deep_sort_cnt(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) {
    k_deep_sort_cnt_one<PASS>(D, F, i);
    __syncthreads();
  }
}

__device__ __forceinline__ void k_deep_sort_scan_one(Dev D, FlowArgs F, uint32_t slot_i) {
  __shared__ uint32_t tot[FL_CAP];
  const uint32_t h = fd_book(D, F, slot_i), k = threadIdx.x;
  if (!fd_deep(F, h)) return;
  const uint32_t nt = F.hdr[h].ntouch;
  const uint32_t ntile = (nt + FL_TILE - 1) / FL_TILE;
  uint32_t* tc = fd_tcnt(F, F.hdr[h].dslot);
  uint32_t s = 0;
  constexpr uint32_t U = 8;  // (eight tiles' loads in flight: the hottest book's ~600 tiles after its plan)
  for (uint32_t t0 = 0; t0 < ntile; t0 += U) {
    uint32_t v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) v[u] = t0 + u < ntile ? tc[(t0 + u) * FL_CAP + k] : 0u;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) s += v[u];
  }
  tot[k] = s;
  __syncthreads();
  if (k == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < FL_CAP; ++i) { const uint32_t v = tot[i]; tot[i] = acc; acc += v; }
  }
  __syncthreads();
  uint32_t run = tot[k];  // (eight tiles' loads in flight before their stores, as k_fc_pscan)
  for (uint32_t t0 = 0; t0 < ntile; t0 += U) {
    uint32_t v[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u)
      if (t0 + u < ntile) v[u] = tc[(t0 + u) * FL_CAP + k];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      if (t0 + u >= ntile) break;
      tc[(t0 + u) * FL_CAP + k] = run;
      run += v[u];
    }
  }
}
__global__ __launch_bounds__(FL_CAP) void k_deep_sort_scan(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.x; i < fd_nslots(F); i += gridDim.x) {
    k_deep_sort_scan_one(D, F, i);
    __syncthreads();
  }
}

template <int PASS>
__device__ __forceinline__ void k_deep_sort_scatter_one(Dev D, FlowArgs F, uint32_t slot_i) {
  __shared__ uint32_t wc[FL_TILE_W][FL_CAP];
  const uint32_t h = fd_book(D, F, slot_i), tid = threadIdx.x, w = tid >> 6;
  if (!fd_deep(F, h)) return;
  const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg;
  const unsigned long long g = F.hdr[h].g;
  const bool dc = F.hdr[h].dc != 0;
  const uint32_t ntile = (nt + FL_TILE - 1) / FL_TILE;
  const uint32_t* tc = fd_tcnt(F, F.hdr[h].dslot);
  for (uint32_t i = tid; i < FL_TILE_W * FL_CAP; i += FL_TILE) wc[i / FL_CAP][i % FL_CAP] = 0;
  __syncthreads();
  for (uint32_t tl = blockIdx.x; tl < ntile; tl += gridDim.x) {
    const uint32_t t = tl * FL_TILE + tid;
    const bool valid = t < nt;
    Touch x{};
    const uint32_t k = valid ? fd_key<PASS>(F, L, t, x) : 0u;
    uint32_t cnt;
    const uint32_t rank = fl_tile_rank(k, valid, cnt);
    if (valid && rank == 0) wc[w][k] = cnt;
    __syncthreads();
    if (tid < FL_CAP) {
      uint32_t r = tc[tl * FL_CAP + tid];
      for (uint32_t ww = 0; ww < FL_TILE_W; ++ww) {
        const uint32_t c = wc[ww][tid];
        wc[ww][tid] = r;
        r += c;
      }
    }
    __syncthreads();
    if (valid) {
      const uint32_t pos = wc[w][k] + rank;
      const unsigned long long a = static_cast<unsigned long long>(x.amt);
      if (PASS == 1) {
        Touch y = x;
        y.amt = static_cast<int64_t>((a & 0xFFFFFFFFull) | (static_cast<unsigned long long>(t) << 32));
        F.tlog[L + pos] = y;
      } else {
        const uint32_t t0 = static_cast<uint32_t>(a >> 32);  // the touch's log index
        SEnt e;
        e.j = dc ? tk_jc(x) : tk_j(x);
        e.kind = tk_kind(x.kr, dc);
        e.amt = static_cast<int64_t>((a & 0xFFFFFFFFull) * g);  // plan units -> fixed point
        e.coord = 0;
        e.t = t0;
        e.lvl = x.pos;
        F.srt[L + pos] = e;
        F.log[L + t0].pos = pos;
        F.log[L + t0].amt = e.amt;
      }
    }
    __syncthreads();
    for (uint32_t i = tid; i < FL_TILE_W * FL_CAP; i += FL_TILE) wc[i / FL_CAP][i % FL_CAP] = 0;
    __syncthreads();
  }
}
template <int PASS>
__global__ __launch_bounds__(FL_TILE) void k_deep_sort_scatter(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) {
    k_deep_sort_scatter_one<PASS>(D, F, i);
    __syncthreads();
  }
}

// ---- levels: the run of each level, then the ADD-only level reconstruction -----------------
// First index in srt[L, L + nt) whose level is >= q (wave-wide 64-ary search).
__device__ __forceinline__ uint32_t fd_lower(const SEnt* R, uint32_t nt, uint32_t q) {
  const uint32_t lane = lane_id();
  uint32_t lo = 0, hi = nt;
  while (hi - lo > 64) {
    const uint32_t step = (hi - lo + 63) / 64;
    const uint32_t i = lo + lane * step;
    const bool v = i < hi;
    const bool below = v && R[i].lvl < q;
    const uint32_t ns = __popcll(__ballot(v)), c = __popcll(__ballot(below));
    const uint32_t nlo = c ? lo + (c - 1) * step + 1 : lo;
    const uint32_t nhi = c < ns ? lo + c * step + 1 : hi;
    lo = nlo;
    hi = min(nhi, hi);
  }
  const uint32_t i = lo + lane;
  return lo + __popcll(__ballot(i < hi && R[i].lvl < q));
}

constexpr uint32_t DEEP_GRID = 1024;  // workgroups per deep book in the per-level kernels

// The run of each level in the sorted touches: FlowLvl::base = its first, ::pad1 = its end
// (0 for a level without touches; the deep prep zeroed both).
__device__ __forceinline__ void k_deep_runs_one(Dev D, FlowArgs F, uint32_t slot_i) {
  const uint32_t h = fd_book(D, F, slot_i);
  if (!fd_deep(F, h)) return;
  const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg;
  const SEnt* R = F.srt + L;
  FlowLvl* LV = fl_lvls(F, h);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nt; i += gridDim.x * blockDim.x) {
    const uint32_t q = R[i].lvl;
    if (i == 0 || R[i - 1].lvl != q) LV[q].base = i;
    if (i + 1 == nt || R[i + 1].lvl != q) LV[q].pad1 = i + 1;
  }
}
__global__ __launch_bounds__(256) void k_deep_runs(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) k_deep_runs_one(D, F, i);
}

// Only the levels the batch touched: a deep book holds thousands of levels (config 5's grow to
// ~10k) and most see no touch in a batch; the prep left those in the state fl_level_one would give
// them (nothing consumed or rested, every old node live, ig_all).  A wave takes the levels whose
// run starts in its 64 sorted touches.
__device__ __forceinline__ void k_deep_level_one(Dev D, FlowArgs F, uint32_t slot_i, uint32_t skip_dc) {
  const uint32_t h = fd_book(D, F, slot_i);
  if (!fd_deep(F, h) || (skip_dc && F.hdr[h].dc)) return;
  const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg;
  FlowLvl* LV = fl_lvls(F, h);
  const SEnt* R = F.srt + L;
  const uint32_t lane = lane_id();
  const bool dc = F.hdr[h].dc != 0;
  for (uint32_t i0 = blockIdx.x * 64u; i0 < nt; i0 += gridDim.x * 64u) {
    const uint32_t i = i0 + lane;
    const uint32_t lv = i < nt ? R[i].lvl : 0u;
    // (not the bid sentinel's run, level 0: it holds only the no-op rests of 0 of dropped ADDs,
    // DELs that find nothing and the padding, and nothing is rebuilt there -- as every lane level
    // pass skips q == 0.  Until round 6 it was walked as a level: fc_level_lane read row 0's FIFO
    // and target count, which no prep writes, and a fresh engine on recycled memory faulted.)
    bool head = i < nt && lv != 0 && (i == 0 || R[i - 1].lvl != lv);
    if (head) {  // a level of few touches: its lane (fc_level_lane, fl_level_lane)
      const uint32_t b = LV[lv].base, n = LV[lv].pad1 - b;
      if (dc && n <= FC_LANE_MAX) {
        fc_level_lane(D, F, h, lv, n);
        head = false;
      } else if (!dc && n <= FL_LANE_MAX) {
        fl_level_lane(D, F, h, lv, b, n);
        head = false;
      }
    }
    for (unsigned long long hm = __ballot(head); hm; hm &= hm - 1) {
      const uint32_t q = uni(rl(lv, static_cast<uint32_t>(__builtin_ctzll(hm))));
      const uint32_t e = uni(LV[q].pad1), b = uni(LV[q].base);  // (k_deep_runs)
      if (dc && e - b >= FC_BIG) continue;  // (k_deep_level_big)
      if (lane == 0) LV[q].cnt = e - b;
      if (dc) {
        __threadfence_block();  // (fc_level_one reads the count back)
        fc_level_one(D, F, h, q);
      } else {
        fl_level_one(D, F, h, q, b, e - b);
      }
    }
  }
}
// skip_dc: books with DELs are k_deep_level_hot's (the hottest book's launch); otherwise a book
// with DELs leaves its levels of FC_BIG touches or more to k_deep_level_big
__global__ __launch_bounds__(64) void k_deep_level(Dev D, FlowArgs F, uint32_t skip_dc) {
#ifdef GOME_PROBE_LEVEL
  const uint64_t t0 = wall_clock64();
#endif
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) {
    k_deep_level_one(D, F, i, skip_dc);
    __syncthreads();
  }
#ifdef GOME_PROBE_LEVEL
  if (threadIdx.x == 0) {
    const uint64_t t = wall_clock64() - t0;
    atomicAdd(&g_probe[8], 1ull);
    atomicAdd(&g_probe[9], t);
    atomicMax(&g_probe[10], t);
    if (t > 1000) atomicAdd(&g_probe[11], 1ull);
    atomicMin(&g_probe[12], t0);
    atomicMax(&g_probe[13], t0 + t);
  }
#endif
}

// The tail's deep books with DELs: their levels of FC_BIG touches or more, a block each (the
// tail's level pass took 15 ms on config 5c, one wave per level; gpurun_out/r05ar).
__device__ __forceinline__ uint32_t fd_run(const FlowLvl* LV, const SEnt* R, uint32_t nt, uint32_t q);
constexpr uint32_t DEEP_BIG_GRID = 8;  // blocks per deep book
__global__ __launch_bounds__(FC_LVB_T) void k_deep_level_big(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) {
    const uint32_t h = fd_book(D, F, i);
    if (!fd_deep(F, h) || !F.hdr[h].dc) continue;
    const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg, nl = F.hdr[h].nl;
    FlowLvl* LV = fl_lvls(F, h);
    const SEnt* R = F.srt + L;
    for (uint32_t q = 1 + blockIdx.x; q <= nl; q += gridDim.x) {
      const uint32_t cnt = fd_run(LV, R, nt, q);
      if (cnt < FC_BIG) continue;
      if (threadIdx.x == 0) LV[q].cnt = cnt;
      __syncthreads();
      fc_level_blk(D, F, h, q);
      __syncthreads();
    }
  }
}

// The hottest book's levels after its plan when it has DELs (the batch's critical path).  Its
// busiest levels carry tens of thousands of touches: on config 5c's streams the aggressive orders'
// remainders rest at 1.00 / 0.01 and every ordinary order of the other side consumes there, and
// one wave took 64 of those touches at a time (1.7 ms of k_deep_level).  Here a block takes each
// level of FC_BIG touches or more (fc_level_blk), then its waves the others, one level each.
// A level's run counts only where the sorted touches hold exactly it: base / pad1 of a level the
// cancel prep's key sort gave a run that no touch reached are still that sort's.
__device__ __forceinline__ uint32_t fd_run(const FlowLvl* LV, const SEnt* R, uint32_t nt, uint32_t q) {
  const uint32_t e = LV[q].pad1, b = LV[q].base;
  const bool ok = e != 0 && e <= nt && b < e && R[b].lvl == q && R[e - 1].lvl == q && (b == 0 || R[b - 1].lvl != q) &&
                  (e == nt || R[e].lvl != q);
  return ok ? e - b : 0u;
}

// ---- huge levels: one level's steps 1-2 over many blocks (the hottest book's) ----------------
// Config 4's and 5c's hottest books hold two levels of ~50k touches each per batch (the aggressive
// orders' remainders at 1.00 / 0.01, consumed there by every ordinary order of the other side).
// fc_level_blk took such a level FC_LVB_T * FC_K touches at a time, each chunk a chain of dependent
// loads and block scans: 0.34 ms (config 4, k_fc_level_blk) and 0.57 ms (config 5c,
// k_deep_level_hot) on the batch's critical path.  A level of FC_HUGE touches or more instead goes
// by chunks of FCB_CK touches, a block each: per-chunk sums (k_fcb_sum1: the cancels' DEL records,
// the consumed volume, the counts; k_fcb_sum2: the new makers' lengths, which read those records),
// their prefixes per level (k_fcb_scan), the consume cursors and the new makers written per chunk
// (k_fcb_write), then fc_level_fifo per level (k_fcb_fifo).  k_fcb_list / _off pick the levels first and
// mark them (FlowLvl::pad6 = 1): k_fc_level_blk and k_deep_level_hot skip them.
constexpr uint32_t FCB_T = 256, FCB_K = 4, FCB_CK = FCB_T * FCB_K;
constexpr uint32_t FC_HUGE = 16384;
constexpr uint32_t FCB_HCAP = 512;  // huge levels per pass (beyond: fc_level_blk, unmarked)
constexpr uint32_t FCB_GRID = 512;
struct FcbChunk {
  int64_t cons, ocan, rlen;      // consumed volume, cancelled old volume, new makers' lengths
  int64_t pcons, prlen;          // their exclusive prefixes within the level (k_fcb_scan)
  uint32_t nr, nc, ncan, pnr;    // rests, consumes, cancels of old makers; the rests before the chunk
};
struct FcbCtl {
  uint32_t n, total, h, pad;
  uint32_t q[FCB_HCAP];
  uint32_t off[FCB_HCAP + 1];    // each listed level's first chunk; off[n] = total
  int64_t cfin[FCB_HCAP], ocan[FCB_HCAP], qend[FCB_HCAP];
  uint32_t nr[FCB_HCAP], nc[FCB_HCAP], ncan[FCB_HCAP];
};
static_assert(sizeof(FcbCtl) == 22552, "tests/test_gpu_huge_levels.py reads the control blocks by this size");

// the hottest book of the pass, or NIL: a lane book with DELs (k_fc_level_blk's) or a deep one
// (k_deep_level_hot's), by the same tests as those kernels
__device__ __forceinline__ uint32_t fcb_book(const Dev& D, const FlowArgs& F, uint32_t deep) {
  if (deep) {
    const uint32_t h = fd_nslots(F) ? fd_book(D, F, 0) : NIL;
    return (fd_deep(F, h) && F.hdr[h].dc) ? h : NIL;
  }
  const uint32_t h = F.h0;
  return (h < fl_hend(D, F) && fc_lane(F, h)) ? h : NIL;
}

// (many blocks: a deep book has up to DEEP_CAP levels, and one block sized them 1024 at a time, 67 us
// on config 5c's; C->n was zeroed before the launch)
constexpr uint32_t FCB_LIST_GRID = 16;
__global__ __launch_bounds__(1024) void k_fcb_list(Dev D, FlowArgs F, uint32_t deep) {
  FcbCtl* C = F.fcb_ctl + deep;
  const uint32_t h = fcb_book(D, F, deep);
  if (h == NIL) return;
  const uint32_t nl = F.hdr[h].nl, nt = F.hdr[h].ntouch;
  FlowLvl* LV = fl_lvls(F, h);
  const SEnt* R = F.srt + FL_TOUCH_MUL * F.hdr[h].beg;
  for (uint32_t q = 1 + blockIdx.x * blockDim.x + threadIdx.x; q <= nl; q += gridDim.x * blockDim.x) {
    const uint32_t cnt = deep ? fd_run(LV, R, nt, q) : LV[q].cnt;
    uint32_t mark = 0;
    if (cnt >= FC_HUGE) {
      const uint32_t k = atomicAdd(&C->n, 1u);
      if (k < FCB_HCAP) {
        C->q[k] = q;
        mark = 1;
        if (deep) LV[q].cnt = cnt;  // (as k_deep_level_hot sets it for fc_level_blk)
      }
    }
    LV[q].pad6 = mark;
  }
}

// the listed levels' first chunks (one thread)
__global__ void k_fcb_off(Dev D, FlowArgs F, uint32_t deep) {
  FcbCtl* C = F.fcb_ctl + deep;
  const uint32_t h = fcb_book(D, F, deep);
  if (threadIdx.x != 0) return;
  const uint32_t n = h == NIL ? 0u : min(C->n, FCB_HCAP);
  uint32_t off = 0;
  for (uint32_t k = 0; k < n; ++k) {
    C->off[k] = off;
    off += (fl_lvls(F, h)[C->q[k]].cnt + FCB_CK - 1) / FCB_CK;
  }
  C->off[n] = off;
  C->n = n;
  C->total = off;
  C->h = h;
}

// the listed level whose chunks hold chunk g: off[k] <= g < off[k + 1]
__device__ __forceinline__ uint32_t fcb_slot(const FcbCtl* C, uint32_t g) {
  uint32_t lo = 0, hi = C->n;
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (C->off[m] <= g) lo = m;
    else hi = m;
  }
  return lo;
}

// block totals of up to 5 values (FCB_T threads); every thread gets them
__device__ __forceinline__ void fcb_totals(int64_t (&v)[5]) {
  __shared__ int64_t ws[5][FCB_T / 64];
  const uint32_t w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    int64_t x = v[k];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    if ((threadIdx.x & 63u) == 0) ws[k][w] = x;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    int64_t t = 0;
    for (uint32_t j = 0; j < FCB_T / 64; ++j) t += ws[k][j];
    v[k] = t;
  }
  __syncthreads();  // (ws is reused by the next chunk)
}

// exclusive block prefixes of 3 values (FCB_T threads)
__device__ __forceinline__ void fcb_excl(int64_t (&v)[3]) {
  __shared__ int64_t ws[3][FCB_T / 64];
  const uint32_t w = threadIdx.x >> 6;
  int64_t inc[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    inc[k] = wave_incl_scan(v[k]);
    if ((threadIdx.x & 63u) == 63u) ws[k][w] = inc[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    int64_t before = 0;
    for (uint32_t j = 0; j < w; ++j) before += ws[k][j];
    v[k] = before + inc[k] - v[k];
  }
  __syncthreads();
}

struct FcbView {  // a chunk's level
  uint32_t sl, q, c, beg, cnt;
  FlowLvl* Lq;
  SEnt* R;
  RsEnt* RS;
};
__device__ __forceinline__ FcbView fcb_view(const FlowArgs& F, const FcbCtl* C, uint32_t g) {
  FcbView v;
  v.sl = fcb_slot(C, g);
  v.q = C->q[v.sl];
  v.c = g - C->off[v.sl];
  const FlowHdr* hd = &F.hdr[C->h];
  v.beg = hd->beg;
  v.Lq = fl_lvls(F, C->h) + v.q;
  v.cnt = v.Lq->cnt;
  const uint32_t L = FL_TOUCH_MUL * v.beg;
  v.R = F.srt + L + v.Lq->base;
  v.RS = F.rs + L + v.Lq->base;
  return v;
}

// step 1 of fc_level_blk per chunk: each cancel -> its DEL's record (r, touch); the chunk's sums
__global__ __launch_bounds__(FCB_T) void k_fcb_sum1(Dev D, FlowArgs F, uint32_t deep) {
  const FcbCtl* C = F.fcb_ctl + deep;
  FcbChunk* K = F.fcb + static_cast<size_t>(deep) * F.fcb_cap;
  const uint32_t total = C->total;
  for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
    const FcbView V = fcb_view(F, C, g);
    const uint32_t i0 = V.c * FCB_CK + threadIdx.x * FCB_K;
    SEnt e[FCB_K];
#pragma unroll
    for (uint32_t u = 0; u < FCB_K; ++u)
      if (i0 + u < V.cnt) e[u] = V.R[i0 + u];
    int64_t v[5] = {0, 0, 0, 0, 0};  // cons, ocan, nr, nc, ncan
#pragma unroll
    for (uint32_t u = 0; u < FCB_K; ++u) {
      if (i0 + u >= V.cnt) continue;
      if (e[u].kind == TK_CANC) {
        FcDel* d = &F.fc_del[V.beg + e[u].j];
        d->r = e[u].amt;
        d->ct = e[u].t;
        if (d->kind == FC_OLD) { v[1] += e[u].amt; v[4] += 1; }
      }
      v[0] += e[u].kind == TK_CONS ? e[u].amt : 0;
      v[2] += e[u].kind == TK_REST ? 1 : 0;
      v[3] += e[u].kind == TK_CONS ? 1 : 0;
    }
    fcb_totals(v);
    if (threadIdx.x == 0) {
      K[g].cons = v[0];
      K[g].ocan = v[1];
      K[g].nr = static_cast<uint32_t>(v[2]);
      K[g].nc = static_cast<uint32_t>(v[3]);
      K[g].ncan = static_cast<uint32_t>(v[4]);
    }
  }
}

// a rest touch's length in consumption space: its volume, less what its DEL (if it came) removed
__device__ __forceinline__ int64_t fcb_rest_len(const FlowArgs& F, uint32_t beg, const SEnt& e, uint32_t& ct) {
  ct = NIL;
  const uint32_t tg = F.fc_tg[beg + e.j];
  if (tg) {
    const FcDel d = F.fc_del[tg - 1u];
    if (d.ct != NIL) {
      ct = d.ct;
      return e.amt - d.r;
    }
  }
  return e.amt;
}

// step 2's sums per chunk: the new makers' lengths
__global__ __launch_bounds__(FCB_T) void k_fcb_sum2(Dev D, FlowArgs F, uint32_t deep) {
  const FcbCtl* C = F.fcb_ctl + deep;
  FcbChunk* K = F.fcb + static_cast<size_t>(deep) * F.fcb_cap;
  const uint32_t total = C->total;
  for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
    const FcbView V = fcb_view(F, C, g);
    const uint32_t i0 = V.c * FCB_CK + threadIdx.x * FCB_K;
    SEnt e[FCB_K];
#pragma unroll
    for (uint32_t u = 0; u < FCB_K; ++u)
      if (i0 + u < V.cnt) e[u] = V.R[i0 + u];
    int64_t v[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (uint32_t u = 0; u < FCB_K; ++u) {
      if (i0 + u >= V.cnt || e[u].kind != TK_REST) continue;
      uint32_t ct;
      v[0] += fcb_rest_len(F, V.beg, e[u], ct);
    }
    fcb_totals(v);
    if (threadIdx.x == 0) K[g].rlen = v[0];
  }
}

// per listed level (a wave each): the chunks' exclusive prefixes and the level's totals
__global__ __launch_bounds__(64) void k_fcb_scan(Dev D, FlowArgs F, uint32_t deep) {
  FcbCtl* C = F.fcb_ctl + deep;
  FcbChunk* K = F.fcb + static_cast<size_t>(deep) * F.fcb_cap;
  const uint32_t lane = lane_id();
  for (uint32_t sl = blockIdx.x; sl < C->n; sl += gridDim.x) {
    const uint32_t a = C->off[sl], b = C->off[sl + 1];
    int64_t cons = 0, ocan = 0, rlen = 0, nr = 0, nc = 0, ncan = 0;
    for (uint32_t g0 = a; g0 < b; g0 += 64) {
      const uint32_t g = g0 + lane;
      const bool in = g < b;
      const int64_t xc = in ? K[g].cons : 0, xr = in ? K[g].rlen : 0, xn = in ? K[g].nr : 0;
      const int64_t ic = wave_incl_scan(xc), ir = wave_incl_scan(xr), in_ = wave_incl_scan(xn);
      if (in) {
        K[g].pcons = cons + ic - xc;
        K[g].prlen = rlen + ir - xr;
        K[g].pnr = static_cast<uint32_t>(nr + in_ - xn);
      }
      cons += rl64(ic, 63);
      rlen += rl64(ir, 63);
      nr += rl64(in_, 63);
      int64_t xo = in ? K[g].ocan : 0, xq = in ? K[g].nc : 0, xk = in ? K[g].ncan : 0;
      for (int off = 32; off > 0; off >>= 1) {
        xo += __shfl_xor(xo, off);
        xq += __shfl_xor(xq, off);
        xk += __shfl_xor(xk, off);
      }
      ocan += xo;
      nc += xq;
      ncan += xk;
    }
    if (lane == 0) {
      const FlowLvl* Lq = fl_lvls(F, C->h) + C->q[sl];
      C->cfin[sl] = cons;
      C->ocan[sl] = ocan;
      C->qend[sl] = Lq->d0 - ocan + rlen;
      C->nr[sl] = static_cast<uint32_t>(nr);
      C->nc[sl] = static_cast<uint32_t>(nc);
      C->ncan[sl] = static_cast<uint32_t>(ncan);
    }
  }
}

// per chunk: each consume's cursor before it, each new maker (its start, volume, order, touch and
// cancel touch) at its rest rank -- fc_level_blk's writes of steps 1 and 2
__global__ __launch_bounds__(FCB_T) void k_fcb_write(Dev D, FlowArgs F, uint32_t deep) {
  const FcbCtl* C = F.fcb_ctl + deep;
  const FcbChunk* K = F.fcb + static_cast<size_t>(deep) * F.fcb_cap;
  const uint32_t total = C->total;
  for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
    const FcbView V = fcb_view(F, C, g);
    const uint32_t i0 = V.c * FCB_CK + threadIdx.x * FCB_K;
    SEnt e[FCB_K];
#pragma unroll
    for (uint32_t u = 0; u < FCB_K; ++u)
      if (i0 + u < V.cnt) e[u] = V.R[i0 + u];
    uint32_t ct[FCB_K];
    int64_t len[FCB_K];
    int64_t v[3] = {0, 0, 0};  // consumed volume, new makers' lengths, rests
#pragma unroll
    for (uint32_t u = 0; u < FCB_K; ++u) {
      ct[u] = NIL;
      len[u] = 0;
      if (i0 + u >= V.cnt) continue;
      if (e[u].kind == TK_CONS) v[0] += e[u].amt;
      if (e[u].kind == TK_REST) {
        len[u] = fcb_rest_len(F, V.beg, e[u], ct[u]);
        v[1] += len[u];
        v[2] += 1;
      }
    }
    fcb_excl(v);
    int64_t cc = K[g].pcons + v[0];
    int64_t run = V.Lq->d0 - C->ocan[V.sl] + K[g].prlen + v[1];
    uint32_t rk = K[g].pnr + static_cast<uint32_t>(v[2]);
#pragma unroll
    for (uint32_t u = 0; u < FCB_K; ++u) {
      if (i0 + u >= V.cnt) continue;
      if (e[u].kind == TK_CONS) {
        V.R[i0 + u].coord = cc;
        cc += e[u].amt;
      } else if (e[u].kind == TK_REST) {
        RsEnt x;
        x.e = run;
        x.v = e[u].amt;
        x.j = e[u].j;
        x.t = e[u].t;
        x.pad0 = ct[u];
        x.pad1 = 0;
        V.RS[rk++] = x;
        run += len[u];
      }
    }
  }
}

// per listed level (a wave each): the old FIFO step with the level's totals
__global__ __launch_bounds__(64) void k_fcb_fifo(Dev D, FlowArgs F, uint32_t deep) {
  const FcbCtl* C = F.fcb_ctl + deep;
  for (uint32_t sl = blockIdx.x; sl < C->n; sl += gridDim.x) {
    const FlowHdr* hd = &F.hdr[C->h];
    FlowLvl* Lq = fl_lvls(F, C->h) + C->q[sl];
    const uint32_t L = FL_TOUCH_MUL * hd->beg;
    fc_level_fifo(D, F, hd, Lq, F.srt + L + Lq->base, Lq->cnt, L, C->cfin[sl], C->nc[sl], C->nr[sl], C->ncan[sl],
                  C->ocan[sl], C->qend[sl]);
  }
}

// The block's levels (q = 1 + blockIdx.x mod gridDim.x) are sized all at once, a thread each, before
// any of them is rebuilt (a level's pass rewrites its run end, FlowLvl::pad1, which fd_run checks):
// the small ones rebuilt there by their thread (fc_level_lane), the big ones listed for the whole
// block (fc_level_blk) and the others for a wave each (fc_level_one).  (Until round 6 each block
// walked its levels one after another to find the big ones, two dependent loads a level: 0.42 ms
// of config 5c's critical path for its ~16k levels, gpurun_out/prof_r06ae_config5c.)
constexpr uint32_t DLH_GRID = DEEP_GRID / 16, DLH_CAP = 512;
static_assert(DEEP_CAP <= DLH_GRID * DLH_CAP, "k_deep_level_hot's per-block level lists");
__global__ __launch_bounds__(FC_LVB_T) void k_deep_level_hot(Dev D, FlowArgs F) {
  __shared__ uint32_t big_q[DLH_CAP], big_c[DLH_CAP], mid_q[DLH_CAP], mid_c[DLH_CAP];
  __shared__ uint32_t nbig, nmid;
  const uint32_t h = fd_nslots(F) ? fd_book(D, F, 0) : NIL;  // (the hottest book's range: one slot)
  if (!fd_deep(F, h) || !F.hdr[h].dc) return;
  const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg, nl = F.hdr[h].nl;
  FlowLvl* LV = fl_lvls(F, h);
  const SEnt* R = F.srt + L;
  if (threadIdx.x == 0) nbig = nmid = 0;
  __syncthreads();
  // (the huge levels went by chunks, k_fcb_*: marked, and their run ends already rewritten)
  for (uint32_t q = 1 + blockIdx.x + gridDim.x * threadIdx.x; q <= nl; q += gridDim.x * blockDim.x) {
    const uint32_t cnt = LV[q].pad6 ? 0u : fd_run(LV, R, nt, q);
    if (cnt >= FC_BIG) {
      const uint32_t k = atomicAdd(&nbig, 1u);
      big_q[k] = q;
      big_c[k] = cnt;
    } else if (cnt > FC_LANE_MAX) {
      const uint32_t k = atomicAdd(&nmid, 1u);
      mid_q[k] = q;
      mid_c[k] = cnt;
    } else if (cnt != 0) {
      fc_level_lane(D, F, h, q, cnt);
    }
  }
  __syncthreads();
  for (uint32_t k = 0; k < nbig; ++k) {
    const uint32_t q = big_q[k];
    if (threadIdx.x == 0) LV[q].cnt = big_c[k];
    __syncthreads();
    fc_level_blk(D, F, h, q);
    __syncthreads();  // (fc_level_blk's shared words, before the next level's)
  }
  const uint32_t nw = blockDim.x >> 6, lane = lane_id();
  for (uint32_t k = threadIdx.x >> 6; k < nmid; k += nw) {
    const uint32_t q = mid_q[k];
    if (lane == 0) LV[q].cnt = mid_c[k];
    __threadfence_block();  // (fc_level_one reads the count back)
    fc_level_one(D, F, h, q);
  }
}

// ---- write: FIFO appends per level, then the level array ------------------------------------
// ---- FIFO chunks of all the book's appends, claimed at once --------------------------------
// (a level claiming its own is two atomics on one shared line of Status; a deep book has
// thousands of levels).  FlowLvl::pad0 := the level's first id in the book's claim.
constexpr uint32_t DEEP_CLAIM_T = 1024;
__device__ __forceinline__ void k_deep_claim_one(Dev D, BatchArgs B, FlowArgs F, uint32_t slot_i) {
  __shared__ uint32_t part[DEEP_CLAIM_T];
  __shared__ uint32_t tot_s;
  const uint32_t h = fd_book(D, F, slot_i), tid = threadIdx.x;
  if (!fd_deep(F, h) || F.hdr[h].dc) return;  // (a book with DELs claims per level: fc_write_level)
  const FlowHdr hd = F.hdr[h];
  FlowLvl* LV = fl_lvls(F, h);
  const RsEnt* RS = F.rs + FL_TOUCH_MUL * hd.beg;
  const uint32_t per = (hd.nl + DEEP_CLAIM_T - 1) / DEEP_CLAIM_T;
  const uint32_t q0 = 1 + tid * per, q1 = min(hd.nl + 1, q0 + per);
  uint32_t sum = 0;
  for (uint32_t q = q0; q < q1; ++q) sum += fl_wplan(LV[q], RS + LV[q].base).need;
  part[tid] = sum;
  __syncthreads();
  if (tid < 64) {  // exclusive scan of the 1024 partial sums by one wave
    uint32_t v[DEEP_CLAIM_T / 64], acc = 0;
#pragma unroll
    for (uint32_t u = 0; u < DEEP_CLAIM_T / 64; ++u) { v[u] = part[tid * (DEEP_CLAIM_T / 64) + u]; acc += v[u]; }
    const uint32_t incl = wave_incl_scan_u32(acc);
    uint32_t run = incl - acc;
#pragma unroll
    for (uint32_t u = 0; u < DEEP_CLAIM_T / 64; ++u) { part[tid * (DEEP_CLAIM_T / 64) + u] = run; run += v[u]; }
    if (tid == 63) tot_s = incl;
  }
  __syncthreads();
  uint32_t off = part[tid];
  for (uint32_t q = q0; q < q1; ++q) {
    LV[q].pad0 = off;
    off += fl_wplan(LV[q], RS + LV[q].base).need;
  }
  if (tid == 0) {
    FlPrepScr* P = F.dscr + hd.dslot;
    const FlClaim c = fl_claim_chunks(D, tot_s);
    P->c_t = c.c_t;
    P->c_nst = c.c_nst;
    P->c_bb = c.c_bb;
    P->c_ok = c.c_ok;
  }
}
__global__ __launch_bounds__(DEEP_CLAIM_T) void k_deep_claim(Dev D, BatchArgs B, FlowArgs F) {
  for (uint32_t i = blockIdx.x; i < fd_nslots(F); i += gridDim.x) {
    k_deep_claim_one(D, B, F, i);
    __syncthreads();
  }
}

__device__ __forceinline__ void k_deep_write_lv_one(Dev D, BatchArgs B, FlowArgs F, uint32_t slot_i) {
  const uint32_t h = fd_book(D, F, slot_i);
  if (!fd_deep(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  const FlPrepScr* P = F.dscr + hd.dslot;
  const FlClaim cl{P->c_t, P->c_nst, P->c_bb, P->c_ok};
  const FlClaim* claim = &cl;
  const FlowLvl* LV = fl_lvls(F, h);
  Level* out = F.dlvout + static_cast<size_t>(hd.dslot) * DEEP_CAP;
  const uint32_t lane = lane_id();
  uint32_t pops = 0;  // (ADD books: fl_level_pops; books with DELs count theirs in k_fc_count_nf)
  // A wave takes 64 consecutive levels: the untouched ones (no touch, so no append and nothing
  // consumed: the prep's FlowLvl is final) one per lane, then the touched ones one at a time.
  for (uint32_t q0 = 1 + blockIdx.x * 64u; q0 <= hd.nl; q0 += gridDim.x * 64u) {
    const uint32_t q = q0 + lane;
    const bool v = q <= hd.nl;
    const bool touched = v && LV[q].cnt != 0;
    if (v && !touched) {
      const FlowLvl& f = LV[q];
      Level x{};
      x.price = f.price;
      x.depth = f.dfin;
      x.nlive = f.nlive0;
      x.member = static_cast<uint8_t>(f.memf);
      x.head = x.tail = NIL;
      if (x.nlive > 0) {
        x.head = f.head;
        x.hslot = static_cast<uint8_t>(f.hslot);
        x.tail = f.tail;
        x.tslot = static_cast<uint8_t>(f.tslot);
      }
      const bool ok = (x.nlive > 0) == (x.depth > 0) && (x.nlive > 0) == (f.memf == M_BUY || f.memf == M_SALE) &&
                      (x.nlive > 0 || f.memf == 0);
      if (!ok) atomicOr(&D.st->err, ERR_CORRUPT);
      out[q] = x;
    }
    for (unsigned long long tm = __ballot(touched); tm; tm &= tm - 1) {
      const uint32_t qq = q0 + static_cast<uint32_t>(__builtin_ctzll(tm));
      const Level x = hd.dc ? fc_write_level(D, B, F, hd, h, qq) : fl_write_level(D, B, F, hd, h, qq, claim, &pops);
      if (lane == 0) out[qq] = x;
    }
  }
  if (lane == 0) ctr_pops(D, pops);
}
__global__ __launch_bounds__(64) void k_deep_write_lv(Dev D, BatchArgs B, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) {
    k_deep_write_lv_one(D, B, F, i);
    __syncthreads();
  }
}

constexpr uint32_t DEEP_FIN_T = 1024, DEEP_FIN_PER = DEEP_CAP / DEEP_FIN_T;

__device__ __forceinline__ void k_deep_write_fin_one(Dev D, FlowArgs F, uint32_t slot_i) {
  __shared__ uint32_t part[DEEP_FIN_T];
  __shared__ uint32_t base_s, cap_s, nout_s;
  const uint32_t h = fd_book(D, F, slot_i), tid = threadIdx.x;
  if (!fd_deep(F, h)) return;
  const FlowHdr hd = F.hdr[h];
  const Level* lv = F.dlvout + static_cast<size_t>(hd.dslot) * DEEP_CAP;
  // levels q0 .. q0 + DEEP_FIN_PER - 1 per thread (1-based)
  const uint32_t q0 = 1 + tid * DEEP_FIN_PER;
  uint32_t c = 0;
  for (uint32_t u = 0; u < DEEP_FIN_PER; ++u) {
    const uint32_t q = q0 + u;
    if (q <= hd.nl && lv[q].nlive > 0) ++c;
  }
  part[tid] = c;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < DEEP_FIN_T; ++i) { const uint32_t v = part[i]; part[i] = acc; acc += v; }
    const uint32_t nout = acc;
    nout_s = nout;
    const Book bk = D.books[hd.sym];
    uint32_t base = bk.lvl_base, cap = bk.lvl_cap;
    if (nout > cap) {
      uint32_t ncap = 16;
      while (ncap < nout) ncap <<= 1;
      const uint32_t nb = lvl_block_alloc(D, ncap);
      if (nb == NIL) {
        atomicOr(&D.st->err, ERR_LEVELS);
        cap = 0;
      } else {
        lvl_block_release(D, base, cap);
        base = nb;
        cap = ncap;
      }
    }
    base_s = base;
    cap_s = cap;
    if (nout <= cap) {
      Book nb;
      nb.lvl_base = base;
      nb.n_lvl = nout;
      nb.lvl_cap = cap;
      nb.pad = 0;
      D.books[hd.sym] = nb;
    }
    ctr_add(D, C_RESTS, static_cast<unsigned long long>(hd.rests));
    ctr_add(D, C_HOT_RESTS, static_cast<unsigned long long>(hd.rests));
    ctr_add(D, C_RESTING_DELTA, static_cast<unsigned long long>(hd.rests));
    ctr_add(D, C_ADD, static_cast<unsigned long long>(hd.adds));
    ctr_add(D, C_DROPPED, static_cast<unsigned long long>(hd.dropped));
    ctr_add(D, C_LEVELS_DELTA, static_cast<unsigned long long>(static_cast<long long>(nout) - hd.nold));
    ctr_add(D, C_HOT_ORDERS, static_cast<unsigned long long>(hd.end - hd.beg));
    ctr_add(D, C_FLOW_BOOKS, 1ull);
    ctr_add(D, C_FLOW_ORDERS, static_cast<unsigned long long>(hd.end - hd.beg));
    ctr_add(D, C_FLOW_TOUCHES, static_cast<unsigned long long>(hd.ntouch));
    if (hd.dc) ctr_add(D, C_DEL, static_cast<unsigned long long>(hd.ndel));
    if (hd.dslot == 0) {  // the hottest book (k_flow_plan_head's work)
      ctr_add(D, C_FLOW_HEAD_ORDERS, static_cast<unsigned long long>(hd.end - hd.beg));
      ctr_add(D, C_FLOW_HEAD_TOUCHES, static_cast<unsigned long long>(hd.ntouch));
      if (!hd.dc) ctr_add(D, C_HEAD_ADD, 1ull);
    }
  }
  __syncthreads();
  fd_clear(F, hd.dslot);  // (the records were built in prep c)
  if (nout_s > cap_s) return;  // (ERR_LEVELS)
  uint32_t o = part[tid];
  for (uint32_t u = 0; u < DEEP_FIN_PER; ++u) {
    const uint32_t q = q0 + u;
    if (q <= hd.nl && lv[q].nlive > 0) D.lvl[base_s + o++] = lv[q];
  }
}
__global__ __launch_bounds__(DEEP_FIN_T) void k_deep_write_fin(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.x; i < fd_nslots(F); i += gridDim.x) {
    k_deep_write_fin_one(D, F, i);
    __syncthreads();
  }
}

// ============================================================== deep books with DELs: cancel prep
// The quantities k_fc_pass computes for a lane book with per-level LDS counters (every targeted
// ADD's rank and arrival end, every DEL's count of its level's targets that arrived before it and
// its side's ADD volume before it; match_flow_cancel.h), for a book with up to DEEP_CAP levels:
// the segment's records sorted stably by level (the deep touch sort, on a key log written over
// F.log before the plan needs it), then one wave per level walks its run in segment order.

// Old targets' FIFO ranks and arrival ends: a wave per level that holds old targets.
__device__ __forceinline__ void k_fd_oldwalk_one(Dev D, FlowArgs F, uint32_t slot_i) {
  const uint32_t h = fd_book(D, F, slot_i);
  if (h == NIL || !fc_deep(F, h)) return;
  const uint32_t nl = F.hdr[h].nl;
  const FlowLvl* LV = fl_lvls(F, h);
  for (uint32_t q = 1 + blockIdx.x; q <= nl; q += gridDim.x)
    if (uni(LV[q].c_old)) fc_oldwalk_level(D, F, h, q);
}
__global__ __launch_bounds__(64) void k_fd_oldwalk(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) k_fd_oldwalk_one(D, F, i);
}

// The key log: record i of the segment at its level (an admitted ADD's, or a DEL's target's;
// level 0 for the rest), kr = i << 8 (no kind bits).  FlowHdr::ntouch = the segment's length
// until the plan sets the touch count.
__device__ __forceinline__ void k_fd_ckeys_one(Dev D, BatchArgs B, FlowArgs F, uint32_t slot_i) {
  const uint32_t h = fd_book(D, F, slot_i);
  if (h == NIL || !fc_deep(F, h)) return;
  const FlowHdr& hd = F.hdr[h];
  const uint32_t n = hd.end - hd.beg, L = FL_TOUCH_MUL * hd.beg;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t b = hd.beg + i;
    const unsigned long long r = F.ord8[hd.obase + i];  // (DEL records are still no-ops)
    uint32_t lvl = static_cast<uint32_t>(r >> 32) & 0x3FFFu;
    if (!r && prep_at(B, b).action == GOME_DEL) {
      const FcDel d = F.fc_del[b];
      if (d.kind != FC_NONE) lvl = d.li;
    }
    Touch x;
    x.kr = i << 8;
    x.pos = lvl;
    x.amt = 0;
    F.log[L + i] = x;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) F.hdr[h].ntouch = n;
}
__global__ __launch_bounds__(256) void k_fd_ckeys(Dev D, BatchArgs B, FlowArgs F) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) k_fd_ckeys_one(D, B, F, i);
}

// One level's run R[b, e) of sorted keys, in segment order: running ADD volumes per side and the
// count of targeted ADDs (from the level's old targets).
__device__ __forceinline__ void fd_crank_level(const BatchArgs& B, const FlowArgs& F, const FlowHdr& hd, FlowLvl* LV,
                                               const SEnt* R, uint32_t q, uint32_t b, uint32_t e) {
  const uint32_t lane = lane_id();
  int64_t sb = 0, sa = 0;
  uint32_t tc = uni(LV[q].c_old);
  for (uint32_t c0 = b; c0 < e; c0 += 64) {
    const uint32_t i = c0 + lane;
    const bool valid = i < e;
    const uint32_t j = valid ? R[i].j : 0u, bs = hd.beg + j;
    bool isadd = false, targ = false, isdel = false, sale = false;
    uint32_t v = 0;
    if (valid) {
      const unsigned long long r = F.ord8[hd.obase + j];
      if (r) {
        isadd = true;
        v = static_cast<uint32_t>(r);
        sale = (r >> 63) != 0;
        targ = F.fc_tg[bs] != 0;
      } else {
        isdel = true;  // (a DEL with a target: the only other records with a level)
        sale = prep_at(B, bs).side == GOME_SALE;
      }
    }
    const int64_t ab = (isadd && !sale) ? v : 0, aa = (isadd && sale) ? v : 0;
    const uint32_t t1 = targ ? 1u : 0u;
    const int64_t ib = wave_incl_scan(ab), ia = wave_incl_scan(aa);
    const uint32_t it = wave_incl_scan_u32(t1);
    const uint32_t before_t = tc + it - t1;
    const uint32_t before_v = static_cast<uint32_t>(sale ? sa + ia - aa : sb + ib - ab);
    if (targ) {  // (k_fc_pass: fc_put_va and the rank)
      FcDel* d = &F.fc_del[F.fc_tg[bs] - 1u];
      d->oend = before_v + v;
      d->ov = v;
      F.fc_rank[bs] = before_t;
    }
    if (isdel) {  // (arrived: k_fc_pwin turns it into the window)
      F.fc_del[bs].nb = before_t;
      F.fc_del[bs].va = before_v;
    }
    sb += rl64(ib, 63);
    sa += rl64(ia, 63);
    tc += rl(it, 63);
  }
  if (lane == 0) LV[q].ttot = tc;
}

// fd_crank_level with a whole block (FC_LVB_T threads) on a level of FC_CRANK_BIG keys or more:
// on config 5c's streams the aggressive remainders' levels (1.00 / 0.01) hold tens of thousands of
// the hottest book's records, and one wave walked them 64 at a time (0.5 ms of the head's prep,
// before the plan).  The two sides' ADD volumes scan as one word (each side's sum is below 2^32 in
// a W32 book: FlowHdr::w32).
constexpr uint32_t FC_CRANK_BIG = 2048;
__device__ __forceinline__ void fd_crank_level_blk(const BatchArgs& B, const FlowArgs& F, const FlowHdr& hd,
                                                   FlowLvl* LV, const SEnt* R, uint32_t q, uint32_t b, uint32_t e) {
  // FD_CK consecutive keys per thread: their three dependent loads (key, record, target link) in
  // flight together, a quarter of the block scans
  constexpr uint32_t FD_CK = 4;
  int64_t vv = 0, tc = LV[q].c_old;
  for (uint32_t c0 = b; c0 < e; c0 += blockDim.x * FD_CK) {
    const uint32_t i0 = c0 + threadIdx.x * FD_CK;
    uint32_t j[FD_CK], tg[FD_CK], v[FD_CK];
    unsigned long long r[FD_CK];
    bool sale[FD_CK];
#pragma unroll
    for (uint32_t u = 0; u < FD_CK; ++u) j[u] = i0 + u < e ? R[i0 + u].j : 0u;
#pragma unroll
    for (uint32_t u = 0; u < FD_CK; ++u) r[u] = i0 + u < e ? F.ord8[hd.obase + j[u]] : 0ull;
    int64_t sv = 0, st = 0;
#pragma unroll
    for (uint32_t u = 0; u < FD_CK; ++u) {
      const uint32_t bs = hd.beg + j[u];
      tg[u] = 0;
      v[u] = static_cast<uint32_t>(r[u]);
      sale[u] = (r[u] >> 63) != 0;
      if (i0 + u < e) {
        if (r[u]) tg[u] = F.fc_tg[bs];
        else sale[u] = prep_at(B, bs).side == GOME_SALE;  // (a DEL with a target: the only other keys)
      }
      sv += r[u] ? (sale[u] ? static_cast<int64_t>(v[u]) << 32 : static_cast<int64_t>(v[u])) : 0;
      st += tg[u] ? 1 : 0;
    }
    int64_t tv, tt;
    int64_t xv = vv + fl_blk_excl(sv, &tv), xt = tc + fl_blk_excl(st, &tt);
#pragma unroll
    for (uint32_t u = 0; u < FD_CK; ++u) {
      if (i0 + u >= e) continue;
      const uint32_t bs = hd.beg + j[u];
      const uint32_t before_t = static_cast<uint32_t>(xt);
      const uint32_t before_v = static_cast<uint32_t>(sale[u] ? static_cast<uint64_t>(xv) >> 32 : static_cast<uint64_t>(xv));
      if (tg[u]) {
        FcDel* d = &F.fc_del[tg[u] - 1u];
        d->oend = before_v + v[u];
        d->ov = v[u];
        F.fc_rank[bs] = before_t;
        xt += 1;
      }
      if (r[u]) {
        xv += sale[u] ? static_cast<int64_t>(v[u]) << 32 : static_cast<int64_t>(v[u]);
      } else {
        F.fc_del[bs].nb = before_t;
        F.fc_del[bs].va = before_v;
      }
    }
    vv += tv;
    tc += tt;
  }
  if (threadIdx.x == 0) LV[q].ttot = static_cast<uint32_t>(tc);
}

// big: 0 = every level a wave; 1 = only the levels below FC_CRANK_BIG keys (k_fd_crank_big takes
// the others)
__device__ __forceinline__ void k_fd_crank_one(Dev D, BatchArgs B, FlowArgs F, uint32_t slot_i, uint32_t big) {
  const uint32_t h = fd_book(D, F, slot_i);
  if (h == NIL || !fc_deep(F, h)) return;
  const FlowHdr& hd = F.hdr[h];
  const uint32_t nt = hd.ntouch, L = FL_TOUCH_MUL * hd.beg;
  FlowLvl* LV = fl_lvls(F, h);
  const SEnt* R = F.srt + L;
  const uint32_t lane = lane_id();
  for (uint32_t i0 = blockIdx.x * 64u; i0 < nt; i0 += gridDim.x * 64u) {
    const uint32_t i = i0 + lane;
    const uint32_t lv = i < nt ? R[i].lvl : 0u;
    const bool head = i < nt && lv != 0 && (i == 0 || R[i - 1].lvl != lv);
    for (unsigned long long hm = __ballot(head); hm; hm &= hm - 1) {
      const uint32_t q = uni(rl(lv, static_cast<uint32_t>(__builtin_ctzll(hm))));
      const uint32_t b = uni(LV[q].base), e = uni(LV[q].pad1);  // (k_deep_runs)
      if (big && e - b >= FC_CRANK_BIG) continue;
      fd_crank_level(B, F, hd, LV, R, q, b, e);
    }
  }
}
__global__ __launch_bounds__(64) void k_fd_crank(Dev D, BatchArgs B, FlowArgs F, uint32_t big) {
  for (uint32_t i = blockIdx.y; i < fd_nslots(F); i += gridDim.y) k_fd_crank_one(D, B, F, i, big);
}
// The levels of FC_CRANK_BIG keys or more, a block each (found from the sorted keys: a run's head).
constexpr uint32_t FD_CRANK_GRID = 16, FD_CRANK_CAP = DEEP_CAP / FD_CRANK_GRID;
__global__ __launch_bounds__(FC_LVB_T) void k_fd_crank_big(Dev D, BatchArgs B, FlowArgs F) {
  for (uint32_t si = blockIdx.y; si < fd_nslots(F); si += gridDim.y) {
    const uint32_t h = fd_book(D, F, si);
    if (h == NIL || !fc_deep(F, h)) continue;
    const FlowHdr& hd = F.hdr[h];
    const uint32_t nt = hd.ntouch, L = FL_TOUCH_MUL * hd.beg, nl = hd.nl;
    FlowLvl* LV = fl_lvls(F, h);
    const SEnt* R = F.srt + L;
    // the block's big levels found a thread per level first (one after another, two dependent
    // loads each, the 16 blocks took 0.28 ms over config 5c's ~16k levels), then ranked a block each
    __shared__ uint32_t big_q[FD_CRANK_CAP], nbig;
    if (threadIdx.x == 0) nbig = 0;
    __syncthreads();
    for (uint32_t q = 1 + blockIdx.x + gridDim.x * threadIdx.x; q <= nl; q += gridDim.x * blockDim.x) {
      const uint32_t b = LV[q].base, e = LV[q].pad1;
      // (a run of the current sort: this prep's k_deep_runs wrote base / pad1 of every level with keys)
      if (e < b + FC_CRANK_BIG || e > nt || R[b].lvl != q || R[e - 1].lvl != q) continue;
      big_q[atomicAdd(&nbig, 1u)] = q;
    }
    __syncthreads();
    for (uint32_t k = 0; k < nbig; ++k) {
      const uint32_t q = big_q[k];
      fd_crank_level_blk(B, F, hd, LV, R, q, LV[q].base, LV[q].pad1);
      __syncthreads();
    }
    __syncthreads();  // (nbig, before the next slot's list)
  }
}

// Per level the first entry of the book's DEL-time array (an exclusive scan of the levels'
// target counts; one block per book).
__device__ __forceinline__ void k_fd_tbase_one(Dev D, FlowArgs F, uint32_t slot_i) {
  __shared__ uint32_t part[DEEP_CLAIM_T];
  const uint32_t h = fd_book(D, F, slot_i), tid = threadIdx.x;
  if (h == NIL || !fc_deep(F, h)) return;
  const uint32_t nl = F.hdr[h].nl;
  FlowLvl* LV = fl_lvls(F, h);
  const uint32_t per = (nl + DEEP_CLAIM_T - 1) / DEEP_CLAIM_T;
  const uint32_t q0 = 1 + tid * per, q1 = min(nl + 1, q0 + per);
  uint32_t sum = 0;
  for (uint32_t q = q0; q < q1; ++q) sum += LV[q].ttot;
  part[tid] = sum;
  __syncthreads();
  if (tid < 64) {
    uint32_t v[DEEP_CLAIM_T / 64], acc = 0;
#pragma unroll
    for (uint32_t u = 0; u < DEEP_CLAIM_T / 64; ++u) { v[u] = part[tid * (DEEP_CLAIM_T / 64) + u]; acc += v[u]; }
    uint32_t run = wave_incl_scan_u32(acc) - acc;
#pragma unroll
    for (uint32_t u = 0; u < DEEP_CLAIM_T / 64; ++u) { part[tid * (DEEP_CLAIM_T / 64) + u] = run; run += v[u]; }
  }
  __syncthreads();
  uint32_t off = part[tid];
  for (uint32_t q = q0; q < q1; ++q) {
    LV[q].tbase = off;
    off += LV[q].ttot;
  }
}
__global__ __launch_bounds__(DEEP_CLAIM_T) void k_fd_tbase(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.x; i < fd_nslots(F); i += gridDim.x) {
    k_fd_tbase_one(D, F, i);
    __syncthreads();
  }
}

// A deep book the cancel prep declined goes to the legacy kernels: its price set back to empty
// (before k_fc_route takes it off the deep path).
__global__ __launch_bounds__(256) void k_fd_decline(Dev D, FlowArgs F) {
  for (uint32_t i = blockIdx.x; i < fd_nslots(F); i += gridDim.x) {
    const uint32_t h = fd_book(D, F, i);
    if (h != NIL && F.hdr[h].ok == FL_OK_DEEP && F.hdr[h].dc && F.hdr[h].fc_bad) fd_clear(F, F.hdr[h].dslot);
    __syncthreads();
  }
}

}  // namespace gome
