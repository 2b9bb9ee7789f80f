// engine.hip — MI355X (gfx950) batch matching engine: kernels + C-ABI host runtime.
//
// Replaces the reference's serial consumer (gomengine/engine/rabbitmq.go:116-125
// calling engine.DoOrder, engine.go:46) with a per-batch device pipeline:
//
//   k_validate        domain check of the 32-B records (symbol range, volume >= 0, |v| < 2^53)
//   k_radix_hist/     stable LSD radix sort of (symbol_id, seq) -> per-symbol segments in
//   k_radix_scatter   consume order (the reference is serial, so per-symbol order = arrival)
//   k_seg_*           segment starts + longest-first launch order (hottest book starts first)
//   k_adm             admission markers S:comparison (nodepool.go:14-28, Q4), batch model
//   k_match           match_books: ONE WAVEFRONT PER BOOK applies its segment in order:
//                     SetOrder / Match / MatchOrder / DeleteOrder (engine.go:56-206) with
//                     64-lane ballots over the level array and a 32-lane prefix scan over
//                     FIFO volumes to find how far a taker sweeps
//   k_scan_* + k_ev_scatter   event compaction into publish order (taker_seq, fill_idx)
//   k_recycle         freed FIFO chunks back to the free pool
//
// Everything is integer / byte work (no MFMA).  See DESIGN.md for layout and rooflines.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gome/gome_abi.h"
#include "device.h"

using namespace gome;

// ============================================================== wave helpers
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ unsigned long long lt_mask() {
  uint32_t l = lane_id();
  return l ? (~0ull >> (64 - l)) : 0ull;
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t j) {
  return __builtin_amdgcn_readlane(v, j);
}
__device__ __forceinline__ int64_t rl64(int64_t v, uint32_t j) {
  uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), j);
  uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32), j);
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}
__device__ __forceinline__ int64_t wave_incl_scan(int64_t x) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int64_t y = __shfl_up(x, off);
    if (lane >= static_cast<uint32_t>(off)) x += y;
  }
  return x;
}
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t x) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t y = __shfl_up(x, off);
    if (lane >= static_cast<uint32_t>(off)) x += y;
  }
  return x;
}
__host__ __device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}

// ============================================================== scan (u32, exclusive)
constexpr int SCAN_T = 256, SCAN_IPT = 8, SCAN_TILE = SCAN_T * SCAN_IPT;

// Exclusive block scan of one value per thread (256 threads); returns prefix, sets total.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds4, uint32_t& total) {
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan_u32(v);
  if (lane == 63) lds4[w] = inc;
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t i = 0; i < w; ++i) off += lds4[i];
  total = lds4[0] + lds4[1] + lds4[2] + lds4[3];
  __syncthreads();
  return off + inc - v;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_reduce(const uint32_t* in, uint32_t m,
                                                        uint32_t* bsum) {
  __shared__ uint32_t lds4[4];
  const uint32_t base = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_IPT;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_IPT; ++i)
    if (base + i < m) s += in[base + i];
  uint32_t tot;
  block_excl_scan(s, lds4, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_spine(uint32_t* bsum, uint32_t nb,
                                                       uint32_t* total) {
  __shared__ uint32_t lds4[4];
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < nb; c0 += SCAN_TILE) {
    const uint32_t base = c0 + threadIdx.x * SCAN_IPT;
    uint32_t v[SCAN_IPT], s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_IPT; ++i) {
      v[i] = (base + i < nb) ? bsum[base + i] : 0;
      s += v[i];
    }
    uint32_t tot;
    uint32_t pre = block_excl_scan(s, lds4, tot) + carry;
#pragma unroll
    for (int i = 0; i < SCAN_IPT; ++i)
      if (base + i < nb) { bsum[base + i] = pre; pre += v[i]; }
    carry += tot;
  }
  if (threadIdx.x == 0 && total) *total = carry;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_down(const uint32_t* in, uint32_t m,
                                                      const uint32_t* bsum, uint32_t* out) {
  __shared__ uint32_t lds4[4];
  const uint32_t base = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_IPT;
  uint32_t v[SCAN_IPT], s = 0;
#pragma unroll
  for (int i = 0; i < SCAN_IPT; ++i) {
    v[i] = (base + i < m) ? in[base + i] : 0;
    s += v[i];
  }
  uint32_t tot;
  uint32_t pre = block_excl_scan(s, lds4, tot) + bsum[blockIdx.x];
#pragma unroll
  for (int i = 0; i < SCAN_IPT; ++i)
    if (base + i < m) { out[base + i] = pre; pre += v[i]; }
}

// ============================================================== radix sort by symbol
constexpr int RS_T = 256, RS_IPT = 8, RS_TILE = RS_T * RS_IPT, RS_MAXBITS = 11;
constexpr int RS_WAVE_ITEMS = RS_TILE / 4;  // contiguous items per wave

template <bool FROM_ORD>
__device__ __forceinline__ uint32_t rs_key(const gome_order* ord, const uint32_t* keys, uint32_t i) {
  return FROM_ORD ? ord[i].symbol_id : keys[i];
}

template <bool FROM_ORD>
__global__ __launch_bounds__(RS_T) void k_radix_hist(const gome_order* ord, const uint32_t* keys,
                                                     uint32_t n, uint32_t shift, uint32_t bits,
                                                     uint32_t* hist, uint32_t nblk) {
  __shared__ uint32_t h[1 << RS_MAXBITS];
  const uint32_t nb = 1u << bits, mask = nb - 1;
  for (uint32_t i = threadIdx.x; i < nb; i += RS_T) h[i] = 0;
  __syncthreads();
  const uint32_t tile = blockIdx.x * RS_TILE;
#pragma unroll
  for (int it = 0; it < RS_IPT; ++it) {
    uint32_t i = tile + it * RS_T + threadIdx.x;
    if (i < n) atomicAdd(&h[(rs_key<FROM_ORD>(ord, keys, i) >> shift) & mask], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < nb; d += RS_T) hist[d * nblk + blockIdx.x] = h[d];
}

// Stable scatter: wave w of the block owns items [w*512, (w+1)*512) of the tile and ranks
// them in rounds of 64 with a ballot-based match of equal digits (multi-split).
template <bool FROM_ORD>
__global__ __launch_bounds__(RS_T) void k_radix_scatter(const gome_order* ord,
                                                        const uint32_t* keys_in,
                                                        const uint32_t* vals_in, uint32_t n,
                                                        uint32_t shift, uint32_t bits,
                                                        const uint32_t* hist_scanned,
                                                        uint32_t* keys_out, uint32_t* vals_out,
                                                        uint32_t nblk) {
  __shared__ uint32_t cnt[4][1 << RS_MAXBITS];
  const uint32_t nb = 1u << bits, mask = nb - 1;
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  for (uint32_t i = threadIdx.x; i < 4 * nb; i += RS_T) cnt[i / nb][i % nb] = 0;
  __syncthreads();
  const uint32_t base = blockIdx.x * RS_TILE + w * RS_WAVE_ITEMS;
  uint32_t kk[RS_WAVE_ITEMS / 64], vv[RS_WAVE_ITEMS / 64], off[RS_WAVE_ITEMS / 64];
  const unsigned long long ltm = lt_mask();
#pragma unroll
  for (int r = 0; r < RS_WAVE_ITEMS / 64; ++r) {
    const uint32_t i = base + r * 64 + lane;
    const bool valid = i < n;
    uint32_t k = valid ? rs_key<FROM_ORD>(ord, keys_in, i) : 0;
    uint32_t v = valid ? (FROM_ORD ? i : vals_in[i]) : 0;
    uint32_t d = (k >> shift) & mask;
    unsigned long long m = __ballot(valid);
    for (uint32_t b = 0; b < bits; ++b) {
      unsigned long long bb = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bb : ~bb;
    }
    uint32_t rank = __popcll(m & ltm);
    uint32_t c = valid ? cnt[w][d] : 0;
    off[r] = c + rank;
    if (valid && rank == 0) cnt[w][d] = c + __popcll(m);
    kk[r] = k;
    vv[r] = v;
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < nb; d += RS_T) {
    uint32_t run = hist_scanned[d * nblk + blockIdx.x];
    for (int ww = 0; ww < 4; ++ww) {
      uint32_t t = cnt[ww][d];
      cnt[ww][d] = run;
      run += t;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < RS_WAVE_ITEMS / 64; ++r) {
    const uint32_t i = base + r * 64 + lane;
    if (i < n) {
      uint32_t pos = cnt[w][(kk[r] >> shift) & mask] + off[r];
      keys_out[pos] = kk[r];
      vals_out[pos] = vv[r];
    }
  }
}

// ============================================================== validation
__global__ void k_validate(const gome_order* ord, uint32_t n, uint32_t max_symbols, Status* st) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const gome_order o = ord[i];
  const int64_t lim = 1ll << 53;
  bool bad = o.symbol_id >= max_symbols || o.volume_fx < 0 || o.volume_fx >= lim ||
             o.price_fx <= -lim || o.price_fx >= lim;
  if (bad) atomicOr(&st->err, ERR_INPUT);
}

// ============================================================== segments
__global__ void k_seg_flags(const uint32_t* skeys, uint32_t n, uint32_t* flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = (i == 0 || skeys[i] != skeys[i - 1]) ? 1u : 0u;
}

__global__ void k_seg_write(const uint32_t* skeys, uint32_t n, const uint32_t* segpos,
                            uint32_t* seg_start, const Status* st) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (i == 0 || skeys[i] != skeys[i - 1])) seg_start[segpos[i]] = i;
  if (i == 0) seg_start[st->nseg] = n;
}

// Longest-first launch order by floor(log2(len)) buckets (hot books start first).
__global__ void k_seg_count(const uint32_t* seg_start, const Status* st, uint32_t* bcnt,
                            unsigned long long* maxseg) {
  __shared__ uint32_t h[32];
  __shared__ uint32_t mx;
  if (threadIdx.x < 32) h[threadIdx.x] = 0;
  if (threadIdx.x == 0) mx = 0;
  __syncthreads();
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < st->nseg) {
    uint32_t len = seg_start[s + 1] - seg_start[s];
    atomicAdd(&h[31 - __clz(len)], 1u);
    atomicMax(&mx, len);
  }
  __syncthreads();
  if (threadIdx.x < 32 && h[threadIdx.x]) atomicAdd(&bcnt[threadIdx.x], h[threadIdx.x]);
  if (threadIdx.x == 0 && mx) atomicMax(maxseg, (unsigned long long)mx);
}

__global__ void k_seg_bscan(uint32_t* bcnt, uint32_t* boff, Status* st, uint32_t hot_log2,
                            uint32_t max_hot) {
  if (threadIdx.x == 0) {
    uint32_t off = 0, hot = 0;
    for (int b = 31; b >= 0; --b) {
      boff[b] = off;
      off += bcnt[b];
      if (static_cast<uint32_t>(b) >= hot_log2) hot += bcnt[b];
    }
    st->nhot = min(hot, max_hot);
  }
}

// Block-aggregated bucket scatter (one global atomic per bucket per block).
__global__ void k_seg_scatter(const uint32_t* seg_start, const Status* st, uint32_t* boff,
                              uint32_t* seg_order) {
  __shared__ uint32_t cnt[32], base[32];
  if (threadIdx.x < 32) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t b = 0, local = 0;
  const bool v = s < st->nseg;
  if (v) {
    b = 31 - __clz(seg_start[s + 1] - seg_start[s]);
    local = atomicAdd(&cnt[b], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 32 && cnt[threadIdx.x]) base[threadIdx.x] = atomicAdd(&boff[threadIdx.x], cnt[threadIdx.x]);
  __syncthreads();
  if (v) seg_order[base[b] + local] = s;
}

// ============================================================== admission (Q4)
// Markers S:comparison[S:uuid:oid] are set at gRPC time for every ADD of the batch
// (main.go:44-45) and tested+cleared at consume time (engine.go:58-62,90).  Under the
// batch ingress model an ADD is admitted iff no earlier ADD/DEL of the batch carries
// the same (S, uuid, oid).  claim[] holds the first claimant (seq+1) of a key's slot;
// amin[] the smallest seq of the key.
__global__ void k_adm(const gome_order* ord, uint32_t n, uint32_t* claim, uint32_t* amin,
                      uint32_t* slot, uint32_t mask) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const gome_order g = ord[i];
  if (g.action != GOME_ADD && g.action != GOME_DEL) { slot[i] = NIL; return; }
  uint32_t h = static_cast<uint32_t>(
      mix64((static_cast<unsigned long long>(g.symbol_id) << 40) ^
            (static_cast<unsigned long long>(g.uuid_id) << 20) ^ mix64(g.oid_id))) & mask;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    uint32_t c = atomicCAS(&claim[h], 0u, i + 1);
    if (c == 0) break;
    const gome_order q = ord[c - 1];
    if (q.symbol_id == g.symbol_id && q.uuid_id == g.uuid_id && q.oid_id == g.oid_id) break;
    h = (h + 1) & mask;
  }
  atomicMin(&amin[h], i);
  slot[i] = h;
}

// ============================================================== prepared records
// One 32-B record per order in segment (symbol-sorted, stable) order, admission resolved:
// the match kernels fetch 64 orders with one coalesced load instead of a chain of
// dependent gathers (sorted index -> record -> admission slot -> admission min).
struct Prep {
  int64_t price;
  int64_t vol;
  uint32_t oid, uuid, idx;
  uint8_t side, action, adm, pad;
};
static_assert(sizeof(Prep) == 32, "Prep layout");

__global__ void k_prep(const gome_order* ord, uint32_t n, const uint32_t* sidx,
                       const uint32_t* adm_slot, const uint32_t* amin, Prep* prep) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = sidx[i];
  const gome_order o = ord[j];
  Prep q;
  q.price = o.price_fx;
  q.vol = o.volume_fx;
  q.oid = o.oid_id;
  q.uuid = o.uuid_id;
  q.idx = j;
  q.side = o.side;
  q.action = o.action;
  q.adm = (o.action == GOME_ADD && amin[adm_slot[j]] == j) ? 1 : 0;
  q.pad = 0;
  prep[i] = q;
}

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
};

constexpr uint32_t EVB = 32;      // events per arena block (cold books)
constexpr uint32_t EVB_HOT = 256; // events per arena block (hot books)

// Wave-uniform context of the book being matched.
struct WaveCtx {
  Dev D;
  BatchArgs B;
  uint32_t sym;
  Level* L;          // the book's sorted level array (HBM)
  uint32_t nl, cap, base;
  uint32_t ev_base, ev_used, evb;
  bool ev_ok, fatal;
  unsigned long long fills, cancels, rests, dropped, adds, dels;
  long long resting_delta, levels_delta;
};

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
  uint32_t c = 0;
  if (lane_id() == 0) {
    int t = atomicSub(&W.D.st->free_top, 1);
    c = (t > 0) ? W.D.free_ids[t - 1] : atomicAdd(W.D.ch_bump, 1u);
  }
  c = uni(c);
  if (c >= W.D.ch_cap) { set_err(W, ERR_CHUNKS); return NIL; }
  return c;
}

__device__ __forceinline__ void free_chunk(WaveCtx& W, uint32_t c) {
  if (lane_id() == 0) W.D.freed_ids[atomicAdd(&W.D.st->freed_top, 1u)] = c;
}

__device__ __forceinline__ void free_chain(WaveCtx& W, uint32_t head, uint32_t tail) {
  uint32_t c = head;
  for (uint32_t guard = 0; c != NIL; ++guard) {
    if (guard > W.D.ch_cap) { set_err(W, ERR_CORRUPT); return; }
    uint32_t nx = (c == tail) ? NIL : uni(W.D.ch[c].next);
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

__device__ __forceinline__ bool level_grow(WaveCtx& W) {
  const uint32_t lane = lane_id();
  uint32_t ncap = W.cap ? W.cap * 2 : 16;
  uint32_t nb = 0;
  if (lane == 0) nb = atomicAdd(W.D.lvl_bump, ncap);
  nb = uni(nb);
  if (static_cast<unsigned long long>(nb) + ncap > W.D.lvl_cap_total) {
    set_err(W, ERR_LEVELS);
    return false;
  }
  Level* NL = W.D.lvl + nb;
  for (uint32_t w0 = 0; w0 < W.nl; w0 += 64) {
    uint32_t k = w0 + lane;
    if (k < W.nl) NL[k] = W.L[k];
  }
  W.L = NL;
  W.cap = ncap;
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
    const uint32_t nxt = uni(W.D.ch[head].next);
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
      const Chunk* c = &W.D.ch[cid];
      r = c->rem[s];
      o = c->oid[s];
      u = c->uuid[s];
      ix = c->ixs[s];
      t = c->tx[s];
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
      uint32_t c2 = uni(W.D.ch[nxt].next);
      for (uint32_t guard = 0; c2 != NIL && guard <= W.D.ch_cap; ++guard) {
        uint32_t lim = (c2 == lv.tail) ? lv.tslot : CH;
        bool l2 = lane < lim && W.D.ch[c2].rem[lane < CH ? lane : 0] >= 0;
        unsigned long long m2 = __ballot(l2);
        if (m2) {
          uint32_t b = __builtin_ctzll(m2);
          uint32_t oo = W.D.ch[c2].oid[b];
          if (lane == ll) { nx_oid = oo; is_last = false; }
          break;
        }
        c2 = (c2 == lv.tail) ? NIL : uni(W.D.ch[c2].next);
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
      e.taker_volume_fx = tafter;
      e.taker_seq = seq;
      e.fill_idx = fidx + rank;
      e.symbol_id = W.sym;
      e.maker_oid_id = o;
      e.maker_uuid_id = u;
      e.maker_next_oid_id = is_last ? 0u : nx_oid;
      e.kind = GOME_EV_FILL;
      e.maker_side = static_cast<uint8_t>(t);
      e.maker_is_last = is_last ? 1 : 0;
      e.pad0 = 0;
      e.pad1 = 0;
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
      if (lane == la) W.D.ch[head].rem[s] = r - f;
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
      W.D.ch[c].next = NIL;
      W.D.ch[c].price = p;
      if (lv.tail != NIL) W.D.ch[lv.tail].next = c;
    }
    if (lv.tail == NIL) { lv.head = c; lv.hslot = 0; }
    lv.tail = c;
    lv.tslot = 0;
  }
  const uint32_t slot = lv.tslot, loc = lv.tail * CH + slot;
  const uint32_t ix = idx_insert(W, oid, loc);
  if (lane == 0) {
    Chunk* c = &W.D.ch[lv.tail];
    c->rem[slot] = T;
    c->oid[slot] = oid;
    c->uuid[slot] = uuid;
    c->tx[slot] = static_cast<uint8_t>(side);
    c->ixs[slot] = ix;
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
  // GetReverseDepth (nodepool.go:86-115): opposite-side levels crossing p, best first.
  if (!sale) {
    for (uint32_t w0 = 0; w0 < W.nl && !W.fatal; w0 += 64) {
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
    for (int32_t top = static_cast<int32_t>(W.nl); top > 0 && !W.fatal; top -= 64) {
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
  if (uni(static_cast<uint32_t>(W.D.ch[cid].price != p))) return 0;  // wrong price (Q3)
  const int64_t r = rl64(W.D.ch[cid].rem[s], 0);
  uint32_t pos;
  if (r < 0 || !level_search(W, p, pos)) { set_err(W, ERR_CORRUPT); return 0; }
  Level lv = W.L[pos];
  lv.depth -= r;  // DeletePoolDepthVolume with the stored remaining volume
  if (lv.depth <= 0) lv.member &= static_cast<uint8_t>(~((side == GOME_SALE) ? M_SALE : M_BUY));
  if (lane == 0) W.D.ch[cid].rem[s] = -1;
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
    e.taker_volume_fx = r;
    e.taker_seq = seq;
    e.fill_idx = 0;
    e.symbol_id = W.sym;
    e.maker_oid_id = oid;
    e.maker_uuid_id = uuid;
    e.maker_next_oid_id = 0;
    e.kind = GOME_EV_CANCEL;
    e.maker_side = static_cast<uint8_t>(side);
    e.maker_is_last = 1;
    e.pad0 = 0;
    e.pad1 = 0;
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
        if (rl(q.adm, j)) {
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

__device__ __forceinline__ void wave_finish(WaveCtx& W) {
  const uint32_t lane = lane_id();
  ev_close(W);
  if (lane == 0) {
    Book nb;
    nb.lvl_base = W.base;
    nb.n_lvl = W.nl;
    nb.lvl_cap = W.cap;
    nb.pad = 0;
    W.D.books[W.sym] = nb;
    unsigned long long* c = W.D.st->ctr;
    if (W.fills) atomicAdd(&c[C_FILLS], W.fills);
    if (W.cancels) atomicAdd(&c[C_CANCELS], W.cancels);
    if (W.rests) atomicAdd(&c[C_RESTS], W.rests);
    if (W.dropped) atomicAdd(&c[C_DROPPED], W.dropped);
    if (W.adds) atomicAdd(&c[C_ADD], W.adds);
    if (W.dels) atomicAdd(&c[C_DEL], W.dels);
    if (W.resting_delta) atomicAdd(&c[C_RESTING_DELTA], static_cast<unsigned long long>(W.resting_delta));
    if (W.levels_delta) atomicAdd(&c[C_LEVELS_DELTA], static_cast<unsigned long long>(W.levels_delta));
  }
}

__device__ __forceinline__ void wave_init(WaveCtx& W, const Dev& D, const BatchArgs& B, uint32_t sym, uint32_t evb) {
  W.D = D;
  W.B = B;
  W.sym = sym;
  const Book bk = D.books[sym];
  W.base = uni(bk.lvl_base);
  W.nl = uni(bk.n_lvl);
  W.cap = uni(bk.lvl_cap);
  W.L = D.lvl + W.base;
  W.ev_base = NIL;
  W.ev_used = 0;
  W.evb = evb;
  W.ev_ok = true;
  W.fatal = false;
  W.fills = W.cancels = W.rests = W.dropped = W.adds = W.dels = 0;
  W.resting_delta = W.levels_delta = 0;
}

// Cold books: one 64-thread workgroup (one wavefront) per book, state in HBM.
__global__ __launch_bounds__(64) void k_match(Dev D, BatchArgs B) {
  const uint32_t nhot = D.st->nhot;
  if (blockIdx.x + nhot >= D.st->nseg || (D.st->err & ERR_INPUT)) return;
  const uint32_t seg = B.seg_order[nhot + blockIdx.x];
  const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
  WaveCtx W;
  wave_init(W, D, B, uni(B.ord[B.prep[beg].idx].symbol_id), EVB);
  process_global(W, beg, end);
  wave_finish(W);
}

// ============================================================== match_books, hot books
// Books whose segment holds >= 2^HOT_MIN_LOG2 orders of the batch (the Zipf head) are
// applied by k_match_hot: one wavefront per book with the whole level array and the head
// chunk of every crossed level resident in LDS, so the per-order critical path issues no
// dependent global-memory load.  Global memory is only written on that path (events,
// index tombstones, appended nodes, deferred index inserts), and read once per 64 orders
// (coalesced Prep records) and once per exhausted head chunk.
constexpr uint32_t HOT_MIN_LOG2 = 11;
constexpr uint32_t MAX_HOT = 256;
constexpr uint32_t LCAP = 1024;   // levels resident in LDS
constexpr uint32_t NCS = 144;     // cached head chunks
constexpr uint16_t NONE16 = 0xFFFF;
constexpr uint32_t PEND = 0x80000000u;  // Chunk::ixs flag: index insert still pending

struct CSlot {
  int64_t rem[CH];
  uint32_t oid[CH];
  uint32_t uuid[CH];
  uint32_t ixs[CH];
  uint8_t tx[CH];
};
struct HotLds {
  Level lv[LCAP];
  CSlot cs[NCS];
  int64_t cs_owner[NCS];   // price of the level whose head chunk the slot holds
  uint32_t cs_chunk[NCS];  // chunk id held (NIL = free)
  uint32_t cs_next[NCS];   // cached Chunk::next
  uint16_t lcs[LCAP];      // level -> cache slot
  uint8_t cs_dirty[NCS];
};
constexpr size_t HOT_LDS_BYTES = sizeof(HotLds);

// Deferred (S, oid) -> loc index insert of a node rested by a hot book.  Entry i of
// segment [beg, end) lives at pend[beg + i]; resolved by k_pend_apply after the kernel.
struct PendEnt {
  uint32_t oid, loc, ix;
  uint8_t used, ins, dead, pad;
};

struct HotCtx {
  WaveCtx W;        // device pointers, counters, event writer (W.L unused in LDS mode)
  HotLds* S;
  uint32_t nl;
  PendEnt* pend;    // this segment's pending inserts
  uint32_t npend, nflushed;
  uint32_t clock;   // eviction clock
};

__device__ __forceinline__ void hot_slot_writeback(HotCtx& H, uint32_t cs) {
  HotLds* S = H.S;
  if (!S->cs_dirty[cs]) return;
  const uint32_t lane = lane_id();
  Chunk* c = &H.W.D.ch[S->cs_chunk[cs]];
  if (lane < CH) {
    c->rem[lane] = S->cs[cs].rem[lane];
    c->oid[lane] = S->cs[cs].oid[lane];
    c->uuid[lane] = S->cs[cs].uuid[lane];
    c->ixs[lane] = S->cs[cs].ixs[lane];
    c->tx[lane] = S->cs[cs].tx[lane];
  }
  if (lane == 0) S->cs_dirty[cs] = 0;
}

__device__ __forceinline__ uint32_t hot_slot_alloc(HotCtx& H) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id();
  for (uint32_t w0 = 0; w0 < NCS; w0 += 64) {
    const uint32_t k = w0 + lane;
    unsigned long long m = __ballot(k < NCS && S->cs_chunk[k] == NIL);
    if (m) return w0 + static_cast<uint32_t>(__builtin_ctzll(m));
  }
  const uint32_t v = H.clock;  // evict round-robin
  H.clock = (H.clock + 1) % NCS;
  hot_slot_writeback(H, v);
  uint32_t pos;
  if (level_search_in(S->lv, H.nl, S->cs_owner[v], pos) && S->lcs[pos] == v) {
    if (lane == 0) S->lcs[pos] = NONE16;
  }
  if (lane == 0) S->cs_chunk[v] = NIL;
  return v;
}

__device__ __forceinline__ void hot_slot_release(HotCtx& H, uint32_t k) {
  const uint16_t cs = H.S->lcs[k];
  if (cs != NONE16 && lane_id() == 0) {
    H.S->cs_chunk[cs] = NIL;
    H.S->cs_dirty[cs] = 0;
    H.S->lcs[k] = NONE16;
  }
}

// Slot holding the head chunk `chunk` of level k (loaded from HBM on a miss).
__device__ __forceinline__ uint32_t hot_head_slot(HotCtx& H, uint32_t k, uint32_t chunk, int64_t price) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id();
  uint32_t cs = S->lcs[k];
  if (cs != NONE16 && S->cs_chunk[cs] == chunk) return cs;
  if (cs == NONE16) {
    cs = hot_slot_alloc(H);
    if (lane == 0) S->lcs[k] = static_cast<uint16_t>(cs);
  }
  const Chunk* c = &H.W.D.ch[chunk];
  if (lane < CH) {
    S->cs[cs].rem[lane] = c->rem[lane];
    S->cs[cs].oid[lane] = c->oid[lane];
    S->cs[cs].uuid[lane] = c->uuid[lane];
    S->cs[cs].ixs[lane] = c->ixs[lane];
    S->cs[cs].tx[lane] = c->tx[lane];
  }
  const uint32_t nx = uni(c->next);
  if (lane == 0) {
    S->cs_chunk[cs] = chunk;
    S->cs_next[cs] = nx;
    S->cs_owner[cs] = price;
    S->cs_dirty[cs] = 0;
  }
  return cs;
}

// Index bookkeeping of a node leaving the book (fill or cancel).
__device__ __forceinline__ void hot_drop_index(HotCtx& H, uint32_t ixs) {
  if (ixs & PEND) H.pend[ixs & ~PEND].dead = 1;
  else idx_erase(H.W, ixs);
}

__device__ __forceinline__ bool hot_level_insert(HotCtx& H, int64_t p, uint32_t& pos) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id();
  if (H.nl == LCAP) {  // drop levels with no observable state, keeping lcs[] aligned
    const unsigned long long ltm = lt_mask();
    uint32_t out = 0;
    for (uint32_t w0 = 0; w0 < H.nl; w0 += 64) {
      const uint32_t k = w0 + lane;
      bool keep = false;
      Level x{};
      uint16_t c = NONE16;
      if (k < H.nl) {
        x = S->lv[k];
        c = S->lcs[k];
        keep = x.nlive != 0 || x.depth != 0 || x.member != 0;
      }
      unsigned long long m = __ballot(keep);
      if (keep) {
        S->lv[out + __popcll(m & ltm)] = x;
        S->lcs[out + __popcll(m & ltm)] = c;
      }
      out += __popcll(m);
    }
    H.W.levels_delta -= static_cast<long long>(H.nl - out);
    H.nl = out;
    level_search_in(S->lv, H.nl, p, pos);
    if (H.nl == LCAP) return false;  // spill to the HBM path
  }
  for (int32_t top = static_cast<int32_t>(H.nl); top > static_cast<int32_t>(pos); top -= 64) {
    const int32_t lo = max(top - 64, static_cast<int32_t>(pos));
    const int32_t k = lo + static_cast<int32_t>(lane);
    if (k < top) {
      Level x = S->lv[k];
      uint16_t c = S->lcs[k];
      S->lv[k + 1] = x;
      S->lcs[k + 1] = c;
    }
  }
  if (lane == 0) {
    Level z{};
    z.price = p;
    z.head = z.tail = NIL;
    S->lv[pos] = z;
    S->lcs[pos] = NONE16;
  }
  H.nl++;
  H.W.levels_delta++;
  return true;
}

// MatchOrder (engine.go:138-198) against the LDS-cached head chunk of level k.
__device__ __forceinline__ int64_t hot_match_level(HotCtx& H, uint32_t k, int64_t T, uint32_t seq, uint32_t& fidx) {
  HotLds* S = H.S;
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id(), s = lane & 31u;
  const bool hi = lane >= 32;
  Level lv = S->lv[k];
  bool first = true;
  for (uint32_t guard = 0; lv.head != NIL && !W.fatal; ++guard) {
    if (guard > W.D.ch_cap) { set_err(W, ERR_CORRUPT); break; }
    const uint32_t head = lv.head;
    const uint32_t cs = hot_head_slot(H, k, head, lv.price);
    const uint32_t nxt = S->cs_next[cs];
    int64_t r = -1;
    uint32_t o = 0, u = 0, ix = 0, t = 0;
    const uint32_t lim = (head == lv.tail) ? lv.tslot : CH;
    const bool inr = !hi && s >= lv.hslot && s < lim;
    if (inr) {
      r = S->cs[cs].rem[s];
      o = S->cs[cs].oid[s];
      u = S->cs[cs].uuid[s];
      ix = S->cs[cs].ixs[s];
      t = S->cs[cs].tx[s];
    }
    const bool live = inr && r >= 0;
    const uint32_t mlo = static_cast<uint32_t>(__ballot(live));
    if (mlo == 0) {
      if (head == lv.tail) { set_err(W, ERR_CORRUPT); break; }
      free_chunk(W, head);
      lv.head = nxt;
      lv.hslot = 0;
      continue;
    }
    const int64_t x = live ? r : 0;
    const int64_t incl = wave_incl_scan(x);
    const int64_t excl = incl - x;
    const uint32_t fl = __builtin_ctz(mlo);
    const bool arr = live && (excl < T || (first && T == 0 && s == fl));
    const bool pop = arr && incl <= T;
    const int64_t f = pop ? r : (T - excl);
    const unsigned long long am = __ballot(arr), pm = __ballot(pop);
    const uint32_t narr = __popcll(am), npop = __popcll(pm);
    const uint32_t la = 63 - __builtin_clzll(am);
    const uint32_t after = (s < 31) ? (mlo & (~0u << (s + 1))) : 0u;
    uint32_t nx_oid = __shfl(o, after ? static_cast<int>(__builtin_ctz(after)) : 0);
    bool is_last = after == 0;
    const uint32_t ll = 31 - __clz(mlo);
    if (nxt != NIL && ((am >> ll) & 1ull)) {
      // the head chunk's last live maker is reached: its NextNode is the first live node
      // of the following chunks (HBM-resident: only head chunks are cached)
      uint32_t c2 = nxt;
      for (uint32_t g2 = 0; c2 != NIL && g2 <= W.D.ch_cap; ++g2) {
        const uint32_t lim2 = (c2 == lv.tail) ? lv.tslot : CH;
        const bool l2 = lane < lim2 && W.D.ch[c2].rem[lane < CH ? lane : 0] >= 0;
        const unsigned long long m2 = __ballot(l2);
        if (m2) {
          const uint32_t oo = W.D.ch[c2].oid[__builtin_ctzll(m2)];
          if (lane == ll) { nx_oid = oo; is_last = false; }
          break;
        }
        c2 = (c2 == lv.tail) ? NIL : uni(W.D.ch[c2].next);
      }
    }
    const int64_t tafter = T - excl - f;
    const int64_t dafter = lv.depth - excl - f;
    const bool clr = arr && dafter <= 0;
    const unsigned long long clr_s = __ballot(clr && t == GOME_SALE), clr_b = __ballot(clr && t != GOME_SALE);
    ev_make_room(W, narr);
    if (arr && W.ev_ok) {
      const uint32_t rank = __popcll(am & lt_mask());
      gome_event e;
      e.price_fx = lv.price;
      e.match_volume_fx = f;
      e.maker_volume_fx = pop ? r : r - f;
      e.taker_volume_fx = tafter;
      e.taker_seq = seq;
      e.fill_idx = fidx + rank;
      e.symbol_id = W.sym;
      e.maker_oid_id = o;
      e.maker_uuid_id = u;
      e.maker_next_oid_id = is_last ? 0u : nx_oid;
      e.kind = GOME_EV_FILL;
      e.maker_side = static_cast<uint8_t>(t);
      e.maker_is_last = is_last ? 1 : 0;
      e.pad0 = 0;
      e.pad1 = 0;
      W.B.arena[W.ev_base + W.ev_used + rank] = e;
    }
    W.ev_used += narr;
    fidx += narr;
    W.fills += narr;
    const int64_t Tn = rl64(tafter, la);
    lv.depth -= (T - Tn);
    if (clr_s) lv.member &= static_cast<uint8_t>(~M_SALE);
    if (clr_b) lv.member &= static_cast<uint8_t>(~M_BUY);
    if (pop) hot_drop_index(H, ix);
    lv.nlive -= npop;
    W.resting_delta -= npop;
    first = false;
    if (!((pm >> la) & 1ull)) {  // partial fill: maker keeps its FIFO position
      if (lane == la) S->cs[cs].rem[s] = r - f;
      if (lane == 0) S->cs_dirty[cs] = 1;
      lv.hslot = static_cast<uint8_t>(la);
      T = 0;
      break;
    }
    T = Tn;
    lv.hslot = static_cast<uint8_t>(la + 1);
    if (lv.nlive == 0) {
      free_chain(W, lv.head, lv.tail);
      hot_slot_release(H, k);
      lv.head = lv.tail = NIL;
      lv.hslot = lv.tslot = 0;
      break;
    }
    if (T <= 0) break;
    free_chunk(W, head);  // every live maker of the head chunk consumed
    lv.head = nxt;
    lv.hslot = 0;
  }
  if (lane == 0) S->lv[k] = lv;
  return T;
}

__device__ __forceinline__ bool hot_rest(HotCtx& H, int64_t p, int64_t T, uint32_t oid, uint32_t uuid, uint32_t side) {
  HotLds* S = H.S;
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  uint32_t pos;
  if (!level_search_in(S->lv, H.nl, p, pos) && !hot_level_insert(H, p, pos)) return false;
  Level lv = S->lv[pos];
  lv.member |= (side == GOME_SALE) ? M_SALE : M_BUY;
  lv.depth += T;
  if (lv.tail == NIL || lv.tslot == CH) {
    const uint32_t c = alloc_chunk(W);  // one allocation per 32 appended nodes
    if (c == NIL) return true;
    if (lane == 0) {
      W.D.ch[c].next = NIL;
      W.D.ch[c].price = p;
      if (lv.tail != NIL) W.D.ch[lv.tail].next = c;
    }
    if (lv.tail != NIL) {
      const uint16_t cs = S->lcs[pos];
      if (cs != NONE16 && S->cs_chunk[cs] == lv.tail && lane == 0) S->cs_next[cs] = c;
    } else {  // FIFO was empty: the new chunk is the head, cache it (nothing to load)
      lv.head = c;
      lv.hslot = 0;
      uint32_t cs = S->lcs[pos];
      if (cs == NONE16) {
        cs = hot_slot_alloc(H);
        if (lane == 0) S->lcs[pos] = static_cast<uint16_t>(cs);
      }
      if (lane == 0) {
        S->cs_chunk[cs] = c;
        S->cs_next[cs] = NIL;
        S->cs_owner[cs] = p;
        S->cs_dirty[cs] = 1;
      }
    }
    lv.tail = c;
    lv.tslot = 0;
  }
  const uint32_t slot = lv.tslot, loc = lv.tail * CH + slot;
  const uint32_t pidx = H.npend++;
  const uint32_t ixs = PEND | pidx;
  if (lane == 0) {
    PendEnt e;
    e.oid = oid;
    e.loc = loc;
    e.ix = NIL;
    e.used = 1;
    e.ins = 0;
    e.dead = 0;
    e.pad = 0;
    H.pend[pidx] = e;
    const uint16_t cs = S->lcs[pos];
    if (cs != NONE16 && S->cs_chunk[cs] == lv.tail) {
      S->cs[cs].rem[slot] = T;
      S->cs[cs].oid[slot] = oid;
      S->cs[cs].uuid[slot] = uuid;
      S->cs[cs].ixs[slot] = ixs;
      S->cs[cs].tx[slot] = static_cast<uint8_t>(side);
      S->cs_dirty[cs] = 1;
    } else {
      Chunk* c = &W.D.ch[lv.tail];
      c->rem[slot] = T;
      c->oid[slot] = oid;
      c->uuid[slot] = uuid;
      c->ixs[slot] = ixs;
      c->tx[slot] = static_cast<uint8_t>(side);
    }
  }
  lv.tslot = static_cast<uint8_t>(slot + 1);
  lv.nlive++;
  if (lane == 0) S->lv[pos] = lv;
  W.rests++;
  W.resting_delta++;
  return true;
}

// SetOrder (engine.go:56-85) on the LDS-resident book.  Returns false when the order has
// been matched but cannot rest because the LDS level array is full (spill): the caller
// rests `trest` on the HBM path.
__device__ __forceinline__ bool hot_add(HotCtx& H, int64_t p, int64_t vol, uint32_t oid, uint32_t uuid,
                        uint32_t side, uint32_t seq, uint32_t& nev, int64_t& trest) {
  HotLds* S = H.S;
  const uint32_t lane = lane_id();
  const bool sale = side == GOME_SALE;
  const uint8_t opp = sale ? M_BUY : M_SALE;
  int64_t T = vol;
  bool crossed = false;
  uint32_t fidx = 0;
  if (!sale) {
    for (uint32_t w0 = 0; w0 < H.nl && !H.W.fatal; w0 += 64) {
      const uint32_t k = w0 + lane;
      const bool v = k < H.nl;
      int64_t lp = 0;
      uint8_t mem = 0;
      if (v) { lp = S->lv[k].price; mem = S->lv[k].member; }
      unsigned long long cm = __ballot(v && (mem & opp) && lp <= p);
      const bool beyond = __ballot(v && lp > p) != 0;
      while (cm && !H.W.fatal) {
        const uint32_t kk = w0 + __builtin_ctzll(cm);
        cm &= cm - 1;
        crossed = true;
        T = hot_match_level(H, kk, T, seq, fidx);
        if (T <= 0) goto matched;
      }
      if (beyond) break;
    }
  } else {
    for (int32_t top = static_cast<int32_t>(H.nl); top > 0 && !H.W.fatal; top -= 64) {
      const int32_t lo = top - 64, k = lo + static_cast<int32_t>(lane);
      const bool v = k >= 0;
      int64_t lp = 0;
      uint8_t mem = 0;
      if (v) { lp = S->lv[k].price; mem = S->lv[k].member; }
      unsigned long long cm = __ballot(v && (mem & opp) && lp >= p);
      const bool beyond = __ballot(v && lp < p) != 0;
      while (cm && !H.W.fatal) {
        const uint32_t b = 63 - __builtin_clzll(cm);
        cm &= ~(1ull << b);
        crossed = true;
        T = hot_match_level(H, static_cast<uint32_t>(lo + static_cast<int32_t>(b)), T, seq, fidx);
        if (T <= 0) goto matched;
      }
      if (beyond) break;
    }
  }
matched:
  nev = fidx;
  trest = T;
  if ((!crossed || T > 0) && !H.W.fatal) return hot_rest(H, p, T, oid, uuid, side);
  return true;
}

// Insert this segment's pending entries [nflushed, npend) into the global index (needed
// before a cancel lookup).  Lane-parallel, one entry per lane.
__device__ __forceinline__ void hot_flush(HotCtx& H) {
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  const unsigned long long mask = W.D.idx_mask;
  bool full = false;
  for (uint32_t b = H.nflushed; b < H.npend; b += 64) {
    const uint32_t i = b + lane;
    if (i < H.npend) {
      PendEnt e = H.pend[i];
      if (!e.dead) {
        const unsigned long long key = idx_key(W.sym, e.oid);
        unsigned long long h = mix64(key) & mask;
        unsigned long long probe = 0;
        for (; probe <= mask; ++probe, h = (h + 1) & mask) {
          unsigned long long kv = __hip_atomic_load(&W.D.idx[h].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((kv == KEY_EMPTY || kv == KEY_TOMB) && atomicCAS(&W.D.idx[h].key, kv, key) == kv) break;
        }
        if (probe > mask) {
          full = true;
        } else {
          W.D.idx[h].loc = e.loc;
          H.pend[i].ix = static_cast<uint32_t>(h);
          H.pend[i].ins = 1;
        }
      }
    }
  }
  if (__ballot(full)) set_err(W, ERR_INDEX);
  H.nflushed = H.npend;
}

// DeleteOrder (engine.go:87-116) on the LDS-resident book.
__device__ __forceinline__ uint32_t hot_cancel(HotCtx& H, int64_t p, uint32_t oid, uint32_t uuid, uint32_t side,
                               uint32_t seq) {
  HotLds* S = H.S;
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  if (H.nflushed < H.npend) hot_flush(H);
  uint32_t ixslot, loc;
  if (!idx_lookup(W, oid, ixslot, loc)) return 0;
  const uint32_t cid = loc / CH, sl = loc % CH;
  if (uni(static_cast<uint32_t>(W.D.ch[cid].price != p))) return 0;  // Q3
  uint32_t pos;
  if (!level_search_in(S->lv, H.nl, p, pos)) { set_err(W, ERR_CORRUPT); return 0; }
  Level lv = S->lv[pos];
  const uint16_t cs = S->lcs[pos];
  const bool cached = cs != NONE16 && S->cs_chunk[cs] == cid;
  const int64_t r = cached ? rl64(S->cs[cs].rem[sl], 0) : rl64(W.D.ch[cid].rem[sl], 0);
  const uint32_t nixs = cached ? S->cs[cs].ixs[sl] : W.D.ch[cid].ixs[sl];
  if (r < 0) { set_err(W, ERR_CORRUPT); return 0; }
  lv.depth -= r;
  if (lv.depth <= 0) lv.member &= static_cast<uint8_t>(~((side == GOME_SALE) ? M_SALE : M_BUY));
  if (lane == 0) {
    if (cached) { S->cs[cs].rem[sl] = -1; S->cs_dirty[cs] = 1; }
    else W.D.ch[cid].rem[sl] = -1;
    idx_erase(W, ixslot);
    if (nixs & PEND) {  // tombstoned here: k_pend_apply must neither insert nor erase it
      H.pend[nixs & ~PEND].dead = 1;
      H.pend[nixs & ~PEND].ins = 0;
    }
  }
  lv.nlive--;
  W.resting_delta--;
  if (lv.nlive == 0) {
    free_chain(W, lv.head, lv.tail);
    hot_slot_release(H, pos);
    lv.head = lv.tail = NIL;
    lv.hslot = lv.tslot = 0;
  }
  if (lane == 0) S->lv[pos] = lv;
  ev_make_room(W, 1);
  if (lane == 0 && W.ev_ok) {
    gome_event e;
    e.price_fx = p;
    e.match_volume_fx = 0;
    e.maker_volume_fx = r;
    e.taker_volume_fx = r;
    e.taker_seq = seq;
    e.fill_idx = 0;
    e.symbol_id = W.sym;
    e.maker_oid_id = oid;
    e.maker_uuid_id = uuid;
    e.maker_next_oid_id = 0;
    e.kind = GOME_EV_CANCEL;
    e.maker_side = static_cast<uint8_t>(side);
    e.maker_is_last = 1;
    e.pad0 = 0;
    e.pad1 = 0;
    W.B.arena[W.ev_base + W.ev_used] = e;
  }
  W.ev_used += 1;
  W.cancels++;
  return 1;
}

// Write the LDS book back to HBM: dirty cached chunks, then the level array (growing the
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
  for (uint32_t k = lane; k < H.nl; k += 64) W.L[k] = S->lv[k];
  W.nl = H.nl;
}

// Resolve every pending entry of this segment inline (spill path only): afterwards every
// resting node carries its real index slot, as the HBM path expects.
__device__ __forceinline__ void hot_resolve_pending(HotCtx& H) {
  hot_flush(H);
  WaveCtx& W = H.W;
  const uint32_t lane = lane_id();
  for (uint32_t i = lane; i < H.npend; i += 64) {
    PendEnt e = H.pend[i];
    if (e.dead) {
      if (e.ins) idx_erase(W, e.ix);
    } else if (e.ins) {
      W.D.ch[e.loc / CH].ixs[e.loc % CH] = e.ix;
    }
    H.pend[i].used = 0;
  }
}

__global__ __launch_bounds__(64) void k_match_hot(Dev D, BatchArgs B, PendEnt* pend_arena) {
  extern __shared__ __align__(16) unsigned char smem[];
  if (blockIdx.x >= D.st->nhot || (D.st->err & ERR_INPUT)) return;
  __builtin_amdgcn_s_setprio(3);  // the hottest books are the batch's critical path
  const uint32_t lane = lane_id();
  const uint32_t seg = B.seg_order[blockIdx.x];
  const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
  HotCtx H;
  WaveCtx& W = H.W;
  wave_init(W, D, B, uni(B.ord[B.prep[beg].idx].symbol_id), EVB_HOT);
  if (W.nl > LCAP / 2) {  // deep book: HBM path from the start
    process_global(W, beg, end);
    wave_finish(W);
    return;
  }
  HotLds* S = reinterpret_cast<HotLds*>(smem);
  H.S = S;
  H.nl = W.nl;
  H.pend = pend_arena + beg;
  H.npend = H.nflushed = 0;
  H.clock = 0;
  for (uint32_t k = lane; k < H.nl; k += 64) { S->lv[k] = W.L[k]; S->lcs[k] = NONE16; }
  for (uint32_t c = lane; c < NCS; c += 64) { S->cs_chunk[c] = NIL; S->cs_dirty[c] = 0; }

  uint32_t next = end;  // first order left for the HBM path after a spill
  bool spilled = false;
  for (uint32_t b0 = beg; b0 < end && !W.fatal && !spilled; b0 += 64) {
    const uint32_t cnt = min(64u, end - b0);
    Prep q{};
    if (lane < cnt) q = B.prep[b0 + lane];
    for (uint32_t j = 0; j < cnt && !W.fatal; ++j) {
      const uint32_t idx = rl(q.idx, j), a = rl(q.action, j);
      uint32_t nev = 0;
      if (a == GOME_ADD) {
        W.adds++;
        if (rl(q.adm, j)) {
          int64_t trest = 0;
          const int64_t p = rl64(q.price, j);
          const uint32_t oid = rl(q.oid, j), uuid = rl(q.uuid, j), side = rl(q.side, j);
          if (!hot_add(H, p, rl64(q.vol, j), oid, uuid, side, idx, nev, trest)) {
            spilled = true;  // LDS level array full: move the book to HBM and rest there
            hot_writeback(H);
            hot_resolve_pending(H);
            if (!W.fatal) do_rest(W, p, trest, oid, uuid, side);
          }
        } else {
          W.dropped++;  // marker already consumed (engine.go:58-60)
        }
      } else if (a == GOME_DEL) {
        W.dels++;
        nev = hot_cancel(H, rl64(q.price, j), rl(q.oid, j), rl(q.uuid, j), rl(q.side, j), idx);
      }
      if (lane == 0) B.ev_count[idx] = nev;
      if (spilled) { next = b0 + j + 1; break; }
    }
  }
  if (spilled) process_global(W, next, end);
  else hot_writeback(H);
  wave_finish(W);
}

// Resolve the deferred index inserts of all hot books (after k_match_hot): insert live
// entries, tombstone entries flushed then filled, and store each live node's real index
// slot into its chunk.
__global__ void k_pend_apply(const Dev D, PendEnt* pend, const uint32_t* seg_start,
                             const uint32_t* seg_order, const BatchArgs B) {
  const uint32_t nhot = D.st->nhot;
  const unsigned long long mask = D.idx_mask;
  for (uint32_t h = blockIdx.y; h < nhot; h += gridDim.y) {
    const uint32_t seg = seg_order[h];
    const uint32_t beg = seg_start[seg], end = seg_start[seg + 1];
    const uint32_t sym = B.ord[B.prep[beg].idx].symbol_id;
    for (uint32_t i = beg + blockIdx.x * blockDim.x + threadIdx.x; i < end; i += gridDim.x * blockDim.x) {
      PendEnt e = pend[i];
      if (!e.used) continue;
      pend[i].used = 0;
      if (e.dead) {
        if (e.ins) __hip_atomic_store(&D.idx[e.ix].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      uint32_t ix = e.ix;
      if (!e.ins) {
        const unsigned long long key = (static_cast<unsigned long long>(sym + 1) << 32) | e.oid;
        unsigned long long hh = mix64(key) & mask, probe = 0;
        for (; probe <= mask; ++probe, hh = (hh + 1) & mask) {
          unsigned long long kv = __hip_atomic_load(&D.idx[hh].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((kv == KEY_EMPTY || kv == KEY_TOMB) && atomicCAS(&D.idx[hh].key, kv, key) == kv) break;
        }
        if (probe > mask) { atomicOr(&D.st->err, ERR_INDEX); continue; }
        D.idx[hh].loc = e.loc;
        ix = static_cast<uint32_t>(hh);
      }
      D.ch[e.loc / CH].ixs[e.loc % CH] = ix;
    }
  }
}

// ============================================================== event compaction
__global__ void k_ev_scatter(const gome_event* arena, uint32_t cap, const Status* st,
                             const uint32_t* ev_off, gome_event* out) {
  const uint32_t used = min(st->ev_bump, cap);
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < used; j += gridDim.x * blockDim.x) {
    const gome_event e = arena[j];
    if (e.taker_seq != NIL) out[ev_off[e.taker_seq] + e.fill_idx] = e;
  }
}

// Freed FIFO chunks of this batch -> free pool (two kernels: copy, then counters).
__global__ void k_recycle_copy(Dev D) {
  const int top = max(D.st->free_top, 0);
  const uint32_t nf = D.st->freed_top;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += gridDim.x * blockDim.x)
    D.free_ids[top + i] = D.freed_ids[i];
}

__global__ void k_recycle_fin(Dev D) {
  if (threadIdx.x == 0) {
    D.st->free_top = max(D.st->free_top, 0) + static_cast<int>(D.st->freed_top);
    D.st->freed_top = 0;
  }
}

// ============================================================== host runtime
namespace {

thread_local std::string g_create_err;

uint32_t ceil_div(uint64_t a, uint64_t b) { return static_cast<uint32_t>((a + b - 1) / b); }
uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

struct gome_engine {
  gome_config cfg{};
  hipStream_t stream = nullptr;
  hipStream_t hot_stream = nullptr;
  bool own_stream = false;
  hipEvent_t fork{}, join{}, evh0{}, evh1{};
  Prep* d_prep = nullptr;
  PendEnt* d_pend = nullptr;
  Dev D{};
  Status* d_st = nullptr;
  Status* h_st = nullptr;
  // capacities
  uint32_t max_batch = 0, key_bits = 1, passes = 1, dbits = 1;
  uint32_t hist_cap = 0, bsum_cap = 0;
  // batch buffers
  gome_order* d_orders = nullptr;
  uint32_t *d_k0 = nullptr, *d_v0 = nullptr, *d_k1 = nullptr, *d_v1 = nullptr;
  uint32_t* d_hist = nullptr;
  uint32_t* d_bsum = nullptr;
  uint32_t* d_tmp = nullptr;  // flags / segpos (n)
  uint32_t* d_seg_start = nullptr;
  uint32_t* d_seg_order = nullptr;
  uint32_t* d_bcnt = nullptr;  // 32 counts + 32 offsets
  uint32_t* d_claim = nullptr;
  uint32_t* d_amin = nullptr;
  uint32_t* d_adm_slot = nullptr;
  uint32_t adm_mask = 0;
  uint32_t* d_ev_count = nullptr;
  uint32_t* d_ev_off = nullptr;
  gome_event* d_arena = nullptr;
  gome_event* d_events = nullptr;
  uint32_t arena_cap = 0;
  hipEvent_t ev0{}, ev1{}, evm0{}, evm1{};
  // host-side state
  std::vector<gome_event> pending;
  size_t pending_pos = 0;
  size_t dev_events = 0, dev_events_pos = 0;
  gome_stats stats{};
  unsigned long long resting = 0, levels = 0;
  bool poisoned = false;
  std::string err;
  std::vector<void*> allocs;

  gome_status fail(gome_status s, const std::string& m) {
    err = m;
    return s;
  }
  template <class T>
  bool alloc(T** p, size_t count, const char* what) {
    void* q = nullptr;
    size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
    if (hipMalloc(&q, bytes) != hipSuccess) {
      err = std::string("hipMalloc failed for ") + what + " (" + std::to_string(bytes) + " B)";
      return false;
    }
    allocs.push_back(q);
    *p = static_cast<T*>(q);
    return true;
  }
  ~gome_engine() {
    for (void* p : allocs) (void)hipFree(p);
    if (h_st) (void)hipHostFree(h_st);
    if (ev0) { (void)hipEventDestroy(ev0); (void)hipEventDestroy(ev1); }
    if (evm0) { (void)hipEventDestroy(evm0); (void)hipEventDestroy(evm1); }
    if (fork) { (void)hipEventDestroy(fork); (void)hipEventDestroy(join); }
    if (evh0) { (void)hipEventDestroy(evh0); (void)hipEventDestroy(evh1); }
    if (hot_stream) (void)hipStreamDestroy(hot_stream);
    if (own_stream && stream) (void)hipStreamDestroy(stream);
  }

  gome_status init(const gome_config& c);
  void scan(const uint32_t* in, uint32_t m, uint32_t* out, uint32_t* total, hipStream_t s);
  gome_status run(const gome_order* d_ord, uint32_t n, hipStream_t s);
};

#define HIPCHK(x)                                                                    \
  do {                                                                               \
    hipError_t _e = (x);                                                             \
    if (_e != hipSuccess)                                                            \
      return fail(GOME_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e));    \
  } while (0)

gome_status gome_engine::init(const gome_config& c) {
  cfg = c;
  if (cfg.accuracy == 0) cfg.accuracy = 8;
  if (!cfg.max_symbols || !cfg.max_batch || !cfg.max_nodes || !cfg.max_levels)
    return fail(GOME_E_INVAL, "gome_config: max_symbols, max_batch, max_nodes, max_levels must be > 0");
  if (cfg.max_batch > (1u << 30) || cfg.max_levels > 0xF0000000ull)
    return fail(GOME_E_INVAL, "gome_config: capacity out of range");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(GOME_E_DEVICE, "no HIP device available (the engine has no CPU fallback)");
  if (cfg.device < 0 || cfg.device >= ndev) return fail(GOME_E_INVAL, "gome_config.device out of range");
  HIPCHK(hipSetDevice(cfg.device));
  HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  own_stream = true;
  HIPCHK(hipEventCreate(&ev0));
  HIPCHK(hipEventCreate(&ev1));
  HIPCHK(hipEventCreate(&evm0));
  HIPCHK(hipEventCreate(&evm1));
  HIPCHK(hipStreamCreateWithFlags(&hot_stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  HIPCHK(hipEventCreate(&evh0));
  HIPCHK(hipEventCreate(&evh1));
  HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_match_hot),
                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(HOT_LDS_BYTES)));

  max_batch = cfg.max_batch;
  uint32_t ms = cfg.max_symbols;
  key_bits = (ms <= 1) ? 1 : 32 - __builtin_clz(ms - 1);
  passes = (key_bits + RS_MAXBITS - 1) / RS_MAXBITS;
  dbits = (key_bits + passes - 1) / passes;
  const uint32_t nblk_max = ceil_div(max_batch, RS_TILE);
  hist_cap = (1u << dbits) * nblk_max;
  uint32_t scan_max = std::max(hist_cap, max_batch);
  bsum_cap = ceil_div(scan_max, SCAN_TILE) + 1;

  // ---- persistent book state
  // chunks: every non-empty level holds >= 1 (plus head/tail chunks partly consumed),
  // and every 32 resting nodes fill one more
  const unsigned long long nchunks = std::min<unsigned long long>(
      cfg.max_nodes / 8 + 2 * std::min<unsigned long long>(cfg.max_levels, cfg.max_nodes) + 1024,
      0xF0000000ull);
  const unsigned long long idx_cap = next_pow2(std::max<unsigned long long>(2 * cfg.max_nodes, 1024));
  if (!alloc(&D.books, ms, "books") || !alloc(&D.lvl, cfg.max_levels, "levels") ||
      !alloc(&D.lvl_bump, 1, "lvl_bump") || !alloc(&D.ch, nchunks, "chunks") ||
      !alloc(&D.ch_bump, 1, "ch_bump") || !alloc(&D.free_ids, nchunks, "free_ids") ||
      !alloc(&D.freed_ids, nchunks, "freed_ids") || !alloc(&D.idx, idx_cap, "index") ||
      !alloc(&d_st, 1, "status"))
    return GOME_E_CAPACITY;
  D.max_symbols = ms;
  D.lvl_cap_total = static_cast<uint32_t>(cfg.max_levels);
  D.ch_cap = static_cast<uint32_t>(nchunks);
  D.idx_mask = idx_cap - 1;
  D.st = d_st;
  HIPCHK(hipMemsetAsync(D.books, 0, sizeof(Book) * ms, stream));
  HIPCHK(hipMemsetAsync(D.lvl_bump, 0, 4, stream));
  HIPCHK(hipMemsetAsync(D.ch_bump, 0, 4, stream));
  HIPCHK(hipMemsetAsync(D.idx, 0, sizeof(IdxEnt) * idx_cap, stream));
  HIPCHK(hipMemsetAsync(d_st, 0, sizeof(Status), stream));
  HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h_st), sizeof(Status), hipHostMallocDefault));

  // ---- per-batch buffers
  const uint32_t nb = max_batch;
  adm_mask = static_cast<uint32_t>(next_pow2(2ull * nb + 16) - 1);
  uint64_t evcap = cfg.max_events ? cfg.max_events
                                  : 2ull * nb + EVB * std::min<uint64_t>(nb, ms) + 1024;
  if (evcap > 0xF0000000ull) evcap = 0xF0000000ull;
  arena_cap = static_cast<uint32_t>(evcap);
  if (!alloc(&d_orders, nb, "orders") || !alloc(&d_k0, nb, "keys0") || !alloc(&d_v0, nb, "vals0") ||
      !alloc(&d_k1, nb, "keys1") || !alloc(&d_v1, nb, "vals1") || !alloc(&d_hist, hist_cap, "hist") ||
      !alloc(&d_bsum, bsum_cap, "scan") || !alloc(&d_tmp, nb, "segflags") ||
      !alloc(&d_seg_start, nb + 1, "seg_start") || !alloc(&d_seg_order, nb, "seg_order") ||
      !alloc(&d_bcnt, 64, "buckets") || !alloc(&d_claim, adm_mask + 1ull, "adm_claim") ||
      !alloc(&d_amin, adm_mask + 1ull, "adm_min") || !alloc(&d_adm_slot, nb, "adm_slot") ||
      !alloc(&d_ev_count, nb, "ev_count") || !alloc(&d_ev_off, nb, "ev_off") ||
      !alloc(&d_prep, nb, "prep") || !alloc(&d_pend, nb, "pending inserts") ||
      !alloc(&d_arena, arena_cap, "event arena") || !alloc(&d_events, arena_cap, "events"))
    return GOME_E_CAPACITY;
  HIPCHK(hipMemsetAsync(d_pend, 0, sizeof(PendEnt) * nb, stream));
  if (D.idx_mask >= PEND) return fail(GOME_E_INVAL, "gome_config.max_nodes too large (index > 2^31 slots)");
  HIPCHK(hipStreamSynchronize(stream));
  return GOME_OK;
}

void gome_engine::scan(const uint32_t* in, uint32_t m, uint32_t* out, uint32_t* total,
                       hipStream_t s) {
  const uint32_t nb = ceil_div(m, SCAN_TILE);
  k_scan_reduce<<<nb, SCAN_T, 0, s>>>(in, m, d_bsum);
  k_scan_spine<<<1, SCAN_T, 0, s>>>(d_bsum, nb, total);
  k_scan_down<<<nb, SCAN_T, 0, s>>>(in, m, d_bsum, out);
}

gome_status gome_engine::run(const gome_order* d_ord, uint32_t n, hipStream_t s) {
  // conservative event bound: one partial per ADD + one event per DEL + one per popped
  // maker (<= resting + ADDs) + block padding
  const unsigned long long bound =
      2ull * n + resting + EVB * static_cast<unsigned long long>(std::min(n, cfg.max_symbols)) + EVB;
  if (bound > arena_cap) {
    if (bound > 0xF0000000ull) return fail(GOME_E_CAPACITY, "event bound exceeds 2^32");
    HIPCHK(hipStreamSynchronize(s));
    for (auto it = allocs.begin(); it != allocs.end();) {
      if (*it == d_arena || *it == d_events) { (void)hipFree(*it); it = allocs.erase(it); }
      else ++it;
    }
    arena_cap = static_cast<uint32_t>(std::min<unsigned long long>(bound + bound / 2, 0xF0000000ull));
    if (!alloc(&d_arena, arena_cap, "event arena") || !alloc(&d_events, arena_cap, "events")) {
      poisoned = true;
      return GOME_E_CAPACITY;
    }
  }
  HIPCHK(hipEventRecord(ev0, s));
  // per-batch status reset (free_top / freed_top persist)
  HIPCHK(hipMemsetAsync(d_st, 0, offsetof(Status, free_top), s));
  const uint32_t T256 = 256, gN = ceil_div(n, T256);
  k_validate<<<gN, T256, 0, s>>>(d_ord, n, cfg.max_symbols, d_st);

  // ---- stable radix sort of (symbol_id, seq)
  const uint32_t nblk = ceil_div(n, RS_TILE);
  const uint32_t nbins = 1u << dbits;
  uint32_t *kin = nullptr, *vin = nullptr, *kout = d_k0, *vout = d_v0;
  for (uint32_t p = 0; p < passes; ++p) {
    const uint32_t shift = p * dbits;
    const uint32_t bits = std::min(dbits, key_bits - shift);
    if (p == 0) {
      k_radix_hist<true><<<nblk, RS_T, 0, s>>>(d_ord, nullptr, n, shift, bits, d_hist, nblk);
      scan(d_hist, (1u << bits) * nblk, d_hist, nullptr, s);
      k_radix_scatter<true><<<nblk, RS_T, 0, s>>>(d_ord, nullptr, nullptr, n, shift, bits, d_hist,
                                                  kout, vout, nblk);
    } else {
      k_radix_hist<false><<<nblk, RS_T, 0, s>>>(nullptr, kin, n, shift, bits, d_hist, nblk);
      scan(d_hist, (1u << bits) * nblk, d_hist, nullptr, s);
      k_radix_scatter<false><<<nblk, RS_T, 0, s>>>(nullptr, kin, vin, n, shift, bits, d_hist, kout,
                                                   vout, nblk);
    }
    (void)nbins;
    kin = kout;
    vin = vout;
    kout = (kin == d_k0) ? d_k1 : d_k0;
    vout = (vin == d_v0) ? d_v1 : d_v0;
  }
  const uint32_t* skeys = kin;
  const uint32_t* sidx = vin;

  // ---- segments (one per symbol present), longest first
  k_seg_flags<<<gN, T256, 0, s>>>(skeys, n, d_tmp);
  scan(d_tmp, n, d_tmp, &d_st->nseg, s);
  k_seg_write<<<gN, T256, 0, s>>>(skeys, n, d_tmp, d_seg_start, d_st);
  HIPCHK(hipMemsetAsync(d_bcnt, 0, 64 * sizeof(uint32_t), s));
  k_seg_count<<<gN, T256, 0, s>>>(d_seg_start, d_st, d_bcnt, &d_st->ctr[C_MAXSEG]);
  k_seg_bscan<<<1, 64, 0, s>>>(d_bcnt, d_bcnt + 32, d_st, HOT_MIN_LOG2, MAX_HOT);
  k_seg_scatter<<<gN, T256, 0, s>>>(d_seg_start, d_st, d_bcnt + 32, d_seg_order);

  // ---- admission markers
  HIPCHK(hipMemsetAsync(d_claim, 0, (adm_mask + 1ull) * 4, s));
  HIPCHK(hipMemsetAsync(d_amin, 0xFF, (adm_mask + 1ull) * 4, s));
  k_adm<<<gN, T256, 0, s>>>(d_ord, n, d_claim, d_amin, d_adm_slot, adm_mask);

  k_prep<<<gN, T256, 0, s>>>(d_ord, n, sidx, d_adm_slot, d_amin, d_prep);

  // ---- match_books: one wavefront per book; hot books (LDS) on a second stream,
  //      concurrently with the cold books (HBM)
  BatchArgs B;
  B.prep = d_prep;
  B.ord = d_ord;
  B.n = n;
  B.seg_start = d_seg_start;
  B.seg_order = d_seg_order;
  B.arena = d_arena;
  B.arena_cap = arena_cap;
  B.ev_count = d_ev_count;
  const uint32_t grid = std::min<uint32_t>(n, cfg.max_symbols);
  HIPCHK(hipEventRecord(evm0, s));
  HIPCHK(hipEventRecord(fork, s));
  HIPCHK(hipStreamWaitEvent(hot_stream, fork, 0));
  HIPCHK(hipEventRecord(evh0, hot_stream));
  k_match_hot<<<std::min<uint32_t>(MAX_HOT, grid), 64, HOT_LDS_BYTES, hot_stream>>>(D, B, d_pend);
  HIPCHK(hipEventRecord(evh1, hot_stream));
  k_pend_apply<<<dim3(8, 64), 256, 0, hot_stream>>>(D, d_pend, d_seg_start, d_seg_order, B);
  HIPCHK(hipEventRecord(join, hot_stream));
  k_match<<<grid, 64, 0, s>>>(D, B);
  HIPCHK(hipStreamWaitEvent(s, join, 0));
  HIPCHK(hipEventRecord(evm1, s));

  // ---- event compaction into publish order
  scan(d_ev_count, n, d_ev_off, &d_st->n_events, s);
  k_ev_scatter<<<2048, T256, 0, s>>>(d_arena, arena_cap, d_st, d_ev_off, d_events);
  k_recycle_copy<<<256, 256, 0, s>>>(D);
  k_recycle_fin<<<1, 64, 0, s>>>(D);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(ev1, s));
  HIPCHK(hipMemcpyAsync(h_st, d_st, sizeof(Status), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));

  const Status& st = *h_st;
  if (st.err & ERR_INPUT)
    return fail(GOME_E_INVAL, "batch rejected: a record is outside the exact domain "
                              "(symbol_id >= max_symbols, volume < 0, or |value| >= 2^53)");
  if (st.err) {
    poisoned = true;
    return fail((st.err & ERR_CORRUPT) ? GOME_E_STATE : GOME_E_CAPACITY,
                "device pool exhausted or invariant violated (err bits " + std::to_string(st.err) +
                    "); engine state is no longer usable");
  }
  resting += st.ctr[C_RESTING_DELTA];
  levels += st.ctr[C_LEVELS_DELTA];
  float ms_total = 0, ms_match = 0, ms_hot = 0;
  (void)hipEventElapsedTime(&ms_total, ev0, ev1);
  (void)hipEventElapsedTime(&ms_match, evm0, evm1);
  (void)hipEventElapsedTime(&ms_hot, evh0, evh1);
  stats.ms_hot = ms_hot;
  stats.n_hot = st.nhot;
  stats.n_orders = n;
  stats.n_add = st.ctr[C_ADD];
  stats.n_del = st.ctr[C_DEL];
  stats.n_dropped = st.ctr[C_DROPPED];
  stats.n_fills = st.ctr[C_FILLS];
  stats.n_cancels = st.ctr[C_CANCELS];
  stats.n_rests = st.ctr[C_RESTS];
  stats.n_events = st.n_events;
  stats.n_resting = resting;
  stats.n_levels = levels;
  stats.max_segment = st.ctr[C_MAXSEG];
  stats.n_segments = st.nseg;
  stats.ms_total = ms_total;
  stats.ms_match = ms_match;
  dev_events = st.n_events;
  dev_events_pos = 0;
  return GOME_OK;
}

// ============================================================== C-ABI
extern "C" {

uint32_t gome_abi_version(void) { return GOME_ABI_VERSION; }

gome_status gome_create(const gome_config* cfg, gome_engine** out) {
  if (!cfg || !out) { g_create_err = "gome_create: NULL argument"; return GOME_E_INVAL; }
  *out = nullptr;
  gome_engine* e = new (std::nothrow) gome_engine();
  if (!e) { g_create_err = "gome_create: out of host memory"; return GOME_E_CAPACITY; }
  gome_status s = e->init(*cfg);
  if (s != GOME_OK) {
    g_create_err = e->err;
    delete e;
    return s;
  }
  *out = e;
  return GOME_OK;
}

void gome_destroy(gome_engine* e) { delete e; }

const char* gome_last_error(const gome_engine* e) {
  return e ? e->err.c_str() : g_create_err.c_str();
}

gome_status gome_submit_batch(gome_engine* e, const gome_order* orders, size_t n, uint64_t) {
  if (!e) return GOME_E_INVAL;
  if (e->poisoned) return e->fail(GOME_E_STATE, "engine poisoned by an earlier fatal error");
  if (n == 0) { e->dev_events = 0; return GOME_OK; }
  if (!orders || n > e->max_batch) return e->fail(GOME_E_INVAL, "batch larger than max_batch");
  for (size_t i = 0; i < n; ++i)
    if (orders[i].flags != 0) return e->fail(GOME_E_INVAL, "gome_order.flags must be 0");
  hipError_t he = hipMemcpyAsync(e->d_orders, orders, n * sizeof(gome_order),
                                 hipMemcpyHostToDevice, e->stream);
  if (he != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
  gome_status s = e->run(e->d_orders, static_cast<uint32_t>(n), e->stream);
  if (s != GOME_OK) return s;
  // queue the batch's events on the host in publish order
  const size_t old = e->pending.size() - e->pending_pos;
  if (e->pending_pos) {
    e->pending.erase(e->pending.begin(), e->pending.begin() + static_cast<long>(e->pending_pos));
    e->pending_pos = 0;
  }
  e->pending.resize(old + e->dev_events);
  if (e->dev_events) {
    he = hipMemcpy(e->pending.data() + old, e->d_events, e->dev_events * sizeof(gome_event),
                   hipMemcpyDeviceToHost);
    if (he != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
  }
  e->dev_events = 0;
  return GOME_OK;
}

gome_status gome_submit_batch_device(gome_engine* e, const gome_order* dev_orders, size_t n,
                                     uint64_t, void* stream) {
  if (!e) return GOME_E_INVAL;
  if (e->poisoned) return e->fail(GOME_E_STATE, "engine poisoned by an earlier fatal error");
  if (n == 0) { e->dev_events = 0; return GOME_OK; }
  if (!dev_orders || n > e->max_batch) return e->fail(GOME_E_INVAL, "batch larger than max_batch");
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  return e->run(dev_orders, static_cast<uint32_t>(n), s);
}

size_t gome_pending_events(const gome_engine* e) {
  if (!e) return 0;
  return (e->pending.size() - e->pending_pos) + (e->dev_events - e->dev_events_pos);
}

gome_status gome_drain_events(gome_engine* e, gome_event* out, size_t cap, size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  size_t c = 0;
  size_t hp = e->pending.size() - e->pending_pos;
  if (hp) {
    c = std::min(cap, hp);
    std::memcpy(out, e->pending.data() + e->pending_pos, c * sizeof(gome_event));
    e->pending_pos += c;
    if (e->pending_pos == e->pending.size()) { e->pending.clear(); e->pending_pos = 0; }
  }
  size_t dp = e->dev_events - e->dev_events_pos;
  if (c < cap && dp) {
    size_t k = std::min(cap - c, dp);
    hipError_t he = hipMemcpy(out + c, e->d_events + e->dev_events_pos, k * sizeof(gome_event),
                              hipMemcpyDeviceToHost);
    if (he != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
    e->dev_events_pos += k;
    c += k;
  }
  *n_out = c;
  return GOME_OK;
}

gome_status gome_device_events(gome_engine* e, const gome_event** dev_ptr, size_t* n) {
  if (!e || !dev_ptr || !n) return GOME_E_INVAL;
  *dev_ptr = e->d_events;
  *n = e->dev_events;
  return GOME_OK;
}

gome_status gome_get_stats(const gome_engine* e, gome_stats* out) {
  if (!e || !out) return GOME_E_INVAL;
  *out = e->stats;
  return GOME_OK;
}

gome_status gome_snapshot_levels(gome_engine* e, uint32_t sym, gome_level* out, size_t cap,
                                 size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  if (sym >= e->cfg.max_symbols) return e->fail(GOME_E_NOTFOUND, "symbol_id out of range");
  Book bk;
  if (hipMemcpy(&bk, e->D.books + sym, sizeof bk, hipMemcpyDeviceToHost) != hipSuccess)
    return e->fail(GOME_E_DEVICE, "snapshot copy failed");
  std::vector<Level> lv(bk.n_lvl);
  if (bk.n_lvl && hipMemcpy(lv.data(), e->D.lvl + bk.lvl_base, bk.n_lvl * sizeof(Level),
                            hipMemcpyDeviceToHost) != hipSuccess)
    return e->fail(GOME_E_DEVICE, "snapshot copy failed");
  size_t c = 0;
  for (const Level& L : lv) {
    if (!L.nlive && !L.depth && !L.member) continue;
    if (c < cap) {
      out[c].price_fx = L.price;
      out[c].depth_fx = L.depth;
      out[c].n_nodes = L.nlive;
      out[c].in_buy = (L.member & M_BUY) ? 1 : 0;
      out[c].in_sale = (L.member & M_SALE) ? 1 : 0;
      out[c].pad = 0;
    }
    ++c;
  }
  *n_out = c;
  return GOME_OK;
}

gome_status gome_snapshot_fifo(gome_engine* e, uint32_t sym, int64_t price, gome_node* out,
                               size_t cap, size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  if (sym >= e->cfg.max_symbols) return e->fail(GOME_E_NOTFOUND, "symbol_id out of range");
  Book bk;
  if (hipMemcpy(&bk, e->D.books + sym, sizeof bk, hipMemcpyDeviceToHost) != hipSuccess)
    return e->fail(GOME_E_DEVICE, "snapshot copy failed");
  std::vector<Level> lv(bk.n_lvl);
  if (bk.n_lvl && hipMemcpy(lv.data(), e->D.lvl + bk.lvl_base, bk.n_lvl * sizeof(Level),
                            hipMemcpyDeviceToHost) != hipSuccess)
    return e->fail(GOME_E_DEVICE, "snapshot copy failed");
  size_t c = 0;
  for (const Level& L : lv) {
    if (L.price != price) continue;
    uint32_t cid = L.head;
    bool firstc = true;
    while (cid != NIL) {
      Chunk ch;
      if (hipMemcpy(&ch, e->D.ch + cid, sizeof ch, hipMemcpyDeviceToHost) != hipSuccess)
        return e->fail(GOME_E_DEVICE, "snapshot copy failed");
      uint32_t lo = firstc ? L.hslot : 0, hi = (cid == L.tail) ? L.tslot : CH;
      for (uint32_t sl = lo; sl < hi; ++sl) {
        if (ch.rem[sl] < 0) continue;
        if (c < cap) {
          std::memset(&out[c], 0, sizeof(gome_node));
          out[c].volume_fx = ch.rem[sl];
          out[c].oid_id = ch.oid[sl];
          out[c].uuid_id = ch.uuid[sl];
          out[c].side = ch.tx[sl];
        }
        ++c;
      }
      firstc = false;
      cid = (cid == L.tail) ? NIL : ch.next;
    }
  }
  *n_out = c;
  return GOME_OK;
}

}  // extern "C"
