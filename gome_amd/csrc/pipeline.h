// pipeline.h — batch-preparation kernels: exclusive scan, stable LSD radix sort by symbol,
// validation, per-symbol segments (longest first), admission markers, prepared records.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "wave.h"

namespace gome {

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
#ifndef GOME_RS_MAXBITS
#define GOME_RS_MAXBITS 8  // (digits of up to 8 bits: 11 measured 0.16 ms slower on config 2's 10-bit keys)
#endif
constexpr int RS_T = 256, RS_IPT = 8, RS_TILE = RS_T * RS_IPT, RS_MAXBITS = GOME_RS_MAXBITS;
constexpr int RS_WAVE_ITEMS = RS_TILE / 4;  // contiguous items per wave

template <bool FROM_ORD>
__device__ __forceinline__ uint32_t rs_key(const gome_order* ord, const uint32_t* keys, uint32_t i) {
  return FROM_ORD ? ord[i].symbol_id : keys[i];
}

// FROM_ORD (the first pass): the keys come from the records, and the kernel also writes
// them to keys_out, so the first scatter reads 4 B per order instead of the 32-B record.
template <bool FROM_ORD>
__global__ __launch_bounds__(RS_T) void k_radix_hist(const gome_order* ord, const uint32_t* keys,
                                                     uint32_t* keys_out, uint32_t n, uint32_t shift,
                                                     uint32_t bits, uint32_t* hist, uint32_t nblk) {
  __shared__ uint32_t h[1 << RS_MAXBITS];
  const uint32_t nb = 1u << bits, mask = nb - 1;
  for (uint32_t i = threadIdx.x; i < nb; i += RS_T) h[i] = 0;
  __syncthreads();
  const uint32_t tile = blockIdx.x * RS_TILE;
#pragma unroll
  for (int it = 0; it < RS_IPT; ++it) {
    uint32_t i = tile + it * RS_T + threadIdx.x;
    if (i < n) {
      const uint32_t k = rs_key<FROM_ORD>(ord, keys, i);
      if (FROM_ORD) keys_out[i] = k;
      atomicAdd(&h[(k >> shift) & mask], 1u);
    }
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < nb; d += RS_T) hist[d * nblk + blockIdx.x] = h[d];
}

// Stable scatter: wave w of the block owns items [w*512, (w+1)*512) of the tile and ranks
// them in rounds of 64 with a ballot-based match of equal digits (multi-split).
// IDV (the first pass): the values are the record indices themselves.
template <bool IDV>
__global__ __launch_bounds__(RS_T) void k_radix_scatter(const uint32_t* keys_in,
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
    uint32_t k = valid ? keys_in[i] : 0;
    uint32_t v = valid ? (IDV ? i : vals_in[i]) : 0;
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

// ============================================================== admission (Q4, Q7)
// Markers S:comparison[S:uuid:oid] are set at gRPC time for every ADD of the batch
// (main.go:44-45) and tested+cleared at consume time (engine.go:58-62,90).  Under the
// batch ingress model an ADD is admitted iff no earlier ADD/DEL of the batch carries
// the same (S, uuid, oid).  A record whose admission the host resolved (GOME_ORD_ADM_HOST: the
// consumer keeps the reference's pre-pool markers itself) carries the verdict in
// GOME_ORD_ADMITTED.
//
// Duplicate oids.  The reference names a resting node S:node:<oid> with
// no uuid (ordernode.go:110-112, nodelink.go:119-122) and assumes oids unique per symbol
// (README.md:27); a second live node with the same name corrupts its FIFO.  The boundary rule,
// the same on every path and in the oracle: an admitted ADD whose (S, oid) names a live node when
// the ADD is applied is not applied (dropped like an ADD without a marker), counted
// (gome_stats.n_dup_oid) and its batch index reported (gome_dup_records).  Whether the node is
// still live depends on the matching before it in the batch, so admission only marks the
// candidates: an admitted ADD whose (S, oid) rests at batch start, or was carried by an earlier
// admitted ADD of the batch, gets verdict ADM_V_CHECK (2).  The flow preps decline a book with
// one; the serial kernels (match_cold.h, match_hot.h) probe the cancel index as they reach it.
// Every ADD the rule rejects is a candidate, so the rule depends on the queue order only.
//
// Both rules key on (S, oid) first.  k_adm puts every ADD / DEL into one open-addressing table
// of 64-bit words keyed (S, oid): a key's slot holds its fingerprint (high half, never 0) and
// the smallest batch index of the key seen so far (low half): a new key claims an empty slot
// with one CAS, a repeat lowers the index with one 64-bit atomicMin and marks the slot `multi`.
// A record alone with its (S, oid) in the batch (every record of a stream with fresh oids)
// needs nothing else: an ADD is admitted (batch rule) or takes the host's verdict, and is a
// duplicate only if its oid rests at batch start.  Only keys seen more than once take the
// second table, keyed (S, uuid, oid) for the batch rule, and the first admitted ADD per (S, oid)
// (k_adm_multi, k_adm_res, k_adm_dup); k_adm_clean leaves those tables empty for the next batch.
//
// "Rests at batch start" is a read-only probe of the (S, oid) cancel index, and only for an ADD
// whose oid is not above the highest oid any ADD of its book ever carried (oid_max, kept by
// k_oid_max): fresh, increasing oids (interned in arrival order) never probe.
constexpr uint32_t ADM_RESTING = 0x80000000u, ADM_MULTI = 0x40000000u, ADM_OK = 0x20000000u;
constexpr uint32_t ADM_SLOT = 0x1FFFFFFFu;  // (table slots < 2^29)
// final verdicts (Prep::adm): not admitted, admitted, admitted but its (S, oid) may be live (Q7)
constexpr uint32_t ADM_V_NO = 0u, ADM_V_YES = 1u, ADM_V_CHECK = 2u;

// Read-only probe of the (S, oid) cancel index: does a live node carry this key?
__device__ __forceinline__ bool idx_live(const IdxEnt* idx, unsigned long long mask, unsigned long long key) {
  unsigned long long h = mix64(key) & mask;
  for (unsigned long long probe = 0; probe <= mask; ++probe, h = (h + 1) & mask) {
    const unsigned long long k = idx[h].key;
    if (k == key) return true;
    if (k == KEY_EMPTY) return false;
  }
  return false;
}

// Insert `key` (its record index i) into a fingerprint / min-index table; returns the slot and
// whether the key was there before.  same(c): the record of index c carries the same key.
template <class Same>
__device__ __forceinline__ uint32_t adm_insert(unsigned long long* tab, uint32_t mask, unsigned long long km, uint32_t i,
                                               Same same, bool& repeat) {
  const unsigned long long mine = ((km >> 32) | 0x80000000ull) << 32 | i;
  uint32_t h = static_cast<uint32_t>(km) & mask;
  repeat = false;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long c = atomicCAS(&tab[h], 0ull, mine);
    if (c == 0) break;
    if ((c >> 32) == (mine >> 32) && same(static_cast<uint32_t>(c))) {
      repeat = true;
      if (c > mine) atomicMin(&tab[h], mine);
      break;
    }
    h = (h + 1) & mask;
  }
  return h;
}

__device__ __forceinline__ unsigned long long key_so(const gome_order& g) {
  return (static_cast<unsigned long long>(g.symbol_id) + 1) << 32 | g.oid_id;
}

// Pass 1 (every record): validation (k_validate's check, folded in), the (S, oid) table, the
// resting probe.  slot[i] := its (S, oid) slot | ADM_RESTING, or NIL (not an ADD / DEL).
// Fresh batches (k_adm_pre): every record an ADD or an ignored action, oids strictly increasing
// in batch order and above every oid an admitted ADD ever carried (or a loaded node holds).  No
// (S, oid) repeats in such a batch and none rests, so each ADD's verdict is its own (admitted by
// the batch rule, or the host's) and the tables are not touched.  Any other batch sets *notfast.
// ctl: [0] the watermark (no oid of an earlier batch is above it), [1] not fresh, [2] this batch's
// highest oid (folded into [0] by the next batch's k_adm_ctl: an upper bound of every oid an
// admitted ADD ever carried, so "above it" is safe).  Launch with at most a few thousand blocks.
__global__ void k_adm_ctl(uint32_t* ctl, uint32_t fast) {
  ctl[0] = max(ctl[0], ctl[2]);
  ctl[2] = 0;
  ctl[1] = fast ? 0u : 1u;
}
__global__ void k_adm_pre(const gome_order* ord, uint32_t n, uint32_t* ctl) {
  __shared__ uint32_t bmax;
  if (threadIdx.x == 0) bmax = 0;
  __syncthreads();
  bool bad = false;
  uint32_t mx = 0;
  const uint32_t g0 = ctl[0];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t oid = ord[i].oid_id, prev = i ? ord[i - 1].oid_id : g0;
    if (ord[i].action == GOME_DEL || oid <= prev) bad = true;
    mx = max(mx, oid);
  }
  for (int off = 32; off > 0; off >>= 1) mx = max(mx, static_cast<uint32_t>(__shfl_xor(mx, off)));
  if (__any(bad) && lane_id() == 0) atomicOr(&ctl[1], 1u);
  if (lane_id() == 0) atomicMax(&bmax, mx);
  __syncthreads();
  if (threadIdx.x == 0 && bmax) atomicMax(&ctl[2], bmax);  // (one device atomic per block)
}

// noprobe (admission ahead of the batch, see k_adm_verify): no resting probe, every verdict as if
// the key did not rest.  gate (the batch's own admission after an ahead pass that cannot stand):
// the kernel runs only when *gate is set.
__global__ void k_adm(const gome_order* ord, uint32_t n, unsigned long long* tab, uint32_t* slot, uint32_t mask,
                      uint32_t max_symbols, Status* st, const Book* books, const IdxEnt* idx,
                      unsigned long long idx_mask, const uint32_t* oid_max, uint8_t* multi, const uint32_t* notfast,
                      bool noprobe = false, const uint32_t* gate = nullptr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (gate && !*gate)) return;
  if (i == 0 && gate) atomicAdd(&st->ctr[C_ADM_REDO], 1ull);
  const gome_order g = ord[i];
  {
    const int64_t lim = 1ll << 53;
    if (g.symbol_id >= max_symbols || g.volume_fx < 0 || g.volume_fx >= lim || g.price_fx <= -lim ||
        g.price_fx >= lim || (g.flags & ~GOME_ORD_FLAGS_MASK) != 0) {
      atomicOr(&st->err, ERR_INPUT);
      slot[i] = NIL;
      return;  // (the batch is rejected; nothing below may index by symbol_id)
    }
  }
  if (!*notfast) {  // a fresh batch: the final verdict at once (k_adm_flag .. k_adm_clean return)
    slot[i] = g.action == GOME_ADD && (!(g.flags & GOME_ORD_ADM_HOST) || (g.flags & GOME_ORD_ADMITTED)) ? 1u : 0u;
    return;
  }
  if (g.action != GOME_ADD && g.action != GOME_DEL) { slot[i] = NIL; return; }
  const bool resting = !noprobe && g.action == GOME_ADD && g.oid_id <= oid_max[g.symbol_id] &&
                       books[g.symbol_id].n_lvl != 0 && idx_live(idx, idx_mask, key_so(g));
  bool repeat;
  const uint32_t h = adm_insert(tab, mask, mix64(key_so(g)), i, [&](uint32_t c) {
    const gome_order q = ord[c];
    return q.symbol_id == g.symbol_id && q.oid_id == g.oid_id;
  }, repeat);
  if (repeat) multi[h] = 1;
  slot[i] = h | (resting ? ADM_RESTING : 0u);
}

// Pass 2: records alone with their (S, oid) get their final verdict (ADM_V_CHECK when the key
// rests at batch start); the others enter the (S, uuid, oid) table (slot2) and keep
// slot | ADM_MULTI.  aux[i] = the (S, oid) slot of a shared key's record, else NIL (k_adm_clean).
__global__ void k_adm_flag(const gome_order* ord, uint32_t n, uint32_t* slot, const uint8_t* multi,
                           unsigned long long* tab2, uint32_t* slot2, uint32_t* aux, uint32_t mask,
                           unsigned long long* tab, const uint32_t* notfast, const uint32_t* gate = nullptr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !*notfast || (gate && !*gate)) return;
  const uint32_t s = slot[i];
  const bool shared = s != NIL && multi[s & ADM_SLOT];
  if (s != NIL) tab[s & ADM_SLOT] = 0ull;  // (k_adm's probes are over: the table is left empty)
  aux[i] = shared ? (s & ADM_SLOT) : NIL;
  if (s == NIL) { slot[i] = 0; return; }
  const gome_order g = ord[i];
  if (!shared) {
    if (g.action != GOME_ADD) { slot[i] = 0; return; }
    const bool adm = (g.flags & GOME_ORD_ADM_HOST) ? (g.flags & GOME_ORD_ADMITTED) != 0 : true;
    slot[i] = !adm ? ADM_V_NO : (s & ADM_RESTING) ? ADM_V_CHECK : ADM_V_YES;
    return;
  }
  const unsigned long long km = mix64((static_cast<unsigned long long>(g.symbol_id) << 40) ^
                                      (static_cast<unsigned long long>(g.uuid_id) << 20) ^ mix64(g.oid_id));
  bool repeat;
  slot2[i] = adm_insert(tab2, mask, km, i, [&](uint32_t c) {
    const gome_order q = ord[c];
    return q.symbol_id == g.symbol_id && q.uuid_id == g.uuid_id && q.oid_id == g.oid_id;
  }, repeat);
  slot[i] = s | ADM_MULTI;
}

// Pass 3 (shared keys): the batch rule / host verdict; an admitted ADD offers its index as the
// key's first admitted ADD (first[] is NIL between batches).
__global__ void k_adm_res(const gome_order* ord, uint32_t n, uint32_t* slot, const unsigned long long* tab2,
                          const uint32_t* slot2, uint32_t* first, const uint32_t* notfast,
                          const uint32_t* gate = nullptr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !*notfast || (gate && !*gate)) return;
  const uint32_t s = slot[i];
  if (!(s & ADM_MULTI)) return;
  const gome_order g = ord[i];
  if (g.action != GOME_ADD) return;
  const bool adm = (g.flags & GOME_ORD_ADM_HOST) ? (g.flags & GOME_ORD_ADMITTED) != 0
                                                 : static_cast<uint32_t>(tab2[slot2[i]]) == i;
  if (!adm) return;
  atomicMin(&first[s & ADM_SLOT], i);
  slot[i] = s | ADM_OK;
}

// Pass 4 (shared keys): final verdicts; an admitted ADD that is not its key's first admitted ADD,
// or whose oid rests at batch start, is a candidate of the duplicate-oid rule (ADM_V_CHECK).
__global__ void k_adm_dup(uint32_t n, uint32_t* slot, const uint32_t* first, const uint32_t* notfast,
                          const uint32_t* gate = nullptr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !*notfast || (gate && !*gate)) return;
  const uint32_t s = slot[i];
  if (!(s & ADM_MULTI)) return;
  const bool adm = (s & ADM_OK) != 0;
  const bool check = adm && ((s & ADM_RESTING) || first[s & ADM_SLOT] != i);
  slot[i] = !adm ? ADM_V_NO : check ? ADM_V_CHECK : ADM_V_YES;
}

// Admission ahead of the batch (pipelined batches while the one before is in its hottest plan):
// the same passes on another stream, without the resting probe (the books are still changing), into
// the batch slot's own verdicts.  The probe is the only input of the verdicts beyond the records,
// and at the batch's own time (the books final) it can only find a key where an ADD's oid is at or
// below its book's oid_max and the book is not empty; where none is, every ahead verdict is the
// one the batch's own admission would give.  Else *redo is set and the passes run again, with the
// probe (gated on *redo; the ahead pass left the tables empty).  The ahead pass's input errors (its
// own Status, ast) join the batch's.
__global__ void k_adm_verify(const gome_order* ord, uint32_t n, const Book* books, const uint32_t* oid_max,
                             uint32_t max_symbols, uint32_t* redo, Status* st, const Status* ast) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    if (ast->err) atomicOr(&st->err, ast->err);
    atomicAdd(&st->ctr[C_ADM_AHEAD], 1ull);
  }
  bool cand = false;
  if (i < n) {
    const gome_order g = ord[i];
    cand = g.action == GOME_ADD && g.symbol_id < max_symbols && g.oid_id <= oid_max[g.symbol_id] &&
           books[g.symbol_id].n_lvl != 0;
  }
  if (__any(cand) && lane_id() == 0) atomicOr(redo, 1u);
}

// An ADD with verdict ADM_V_CHECK that the serial kernels found live: rejected (one thread).
__device__ __forceinline__ void dup_note(Status* st, uint32_t* list, uint32_t i) {
  list[atomicAdd(&st->ctr[C_DUP], 1ull)] = i;
}

// Pass 5 (shared keys): their entries of the second table, first[] and multi[] back to empty.
__global__ void k_adm_clean(uint32_t n, const uint32_t* aux, const uint32_t* slot2, unsigned long long* tab2,
                            uint32_t* first, uint8_t* multi, const uint32_t* notfast,
                            const uint32_t* gate = nullptr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !*notfast || (gate && !*gate)) return;
  const uint32_t h = aux[i];
  if (h == NIL) return;
  tab2[slot2[i]] = 0ull;
  first[h] = NIL;
  multi[h] = 0;
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

// oid_max[S] = the highest oid any applied ADD of book S carried (the resting probe's filter).
// Over the symbol-sorted records (Prep: oid and the final admission verdict), one atomicMax per
// symbol run of a wave.
__global__ void k_oid_max(uint32_t n, const uint32_t* skeys, const Prep* prep, uint32_t* oid_max) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = lane_id();
  const bool v = i < n;
  const uint32_t sym = v ? skeys[i] : NIL;
  uint32_t o = 0;
  if (v) {
    const Prep q = prep[i];
    if (q.action == GOME_ADD && q.adm) o = q.oid;
  }
  // a run = lanes of one symbol; the run's last lane takes the run's max
  const uint32_t prev = __shfl_up(sym, 1), next = __shfl_down(sym, 1);
  const bool head = lane == 0 || prev != sym, tail = lane == 63 || next != sym;
  const unsigned long long heads = __ballot(head);
  const uint32_t start = 63u - __clzll(heads & ((2ull << lane) - 1));  // this lane's run start
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(o, off);
    if (lane >= static_cast<uint32_t>(off) && lane - off >= start) o = max(o, y);
  }
  if (v && tail && o > 0) atomicMax(&oid_max[sym], o);
}


__global__ void k_prep(const gome_order* ord, uint32_t n, const uint32_t* sidx,
                       const uint32_t* adm_flag, Prep* prep) {
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
  q.adm = static_cast<uint8_t>(adm_flag[j]);
  q.pad = 0;
  prep[i] = q;
}


}  // namespace gome
