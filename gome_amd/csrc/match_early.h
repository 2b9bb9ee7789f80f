// match_early.h — the hottest book's plan started right after the previous batch's plan.
//
// One wavefront plans the hottest book (k_flow_plan_head) and bounds the batch; everything else
// runs beside it.  But between two batches' plans the pipeline put ~1.1 ms of serial work on
// config 3: the previous batch's reconstruction and publish, then the next batch's sort,
// admission and head prep.  The plan needs none of it: a book's plan reads only its level
// aggregates (price, depth, side: the plan's own final state, FlowHdr / FlowLvl) and the batch's
// packed records of that book.  So for a pipelined batch (gome_submit_batch_device_async or
// gome_submit_batch_async) whose hottest book was also the previous batch's hottest book on an ADD
// plan (lane or deep), the engine prepares and plans that book as soon as the previous plan ends
// (device batches: the record work on the early stream, the rest on the copy stream; host batches:
// the record work behind the H2D on the copy stream, the rest on the early stream):
//
//   k_x_count / k_x_scan / k_x_scatter  the records of the previous batch's hottest symbol, in
//                batch order, at the positions the batch's stable sort will give them (the sort
//                itself stays on the caller's stream, off the critical path)
//   k_x_adm      their admission verdicts as k_adm will give them (an ADD alone with its (S, oid)
//                in the batch, oid above the book's oid_max: its own verdict, pipeline.h); any
//                DEL, ignored action or oid out of order declines the early plan
//   k_flow_prep_a  the batch's prices and volume gcd / sum of the book (the head prep's own kernel)
//   -- the previous batch's plan ends (plan_done) --
//   k_x_prep_b   the price set: the previous plan's final levels (F.hdr[0] / F.lvl, that batch's
//                header: FlowHdr::bid) plus the batch's prices; rank, the 32-bit test, XH / XL
//   k_flow_prep_c  the packed records (into X.ord8), k_flow_plan_early (k_flow_plan_head's code
//                under its own name, for the profiles; X.log, FlowArgs::xlog)
// Deep books take k_xd_prep_a / k_xd_sort_new (beside the previous plan) and k_xd_prep_b /
// k_deep_prep_c after it instead of the lane preps (below).
//
// The batch's own pipeline still prepares the book as before (k_flow_prep_a/b/c into F).  Then
// k_x_cmp checks that the early inputs equal the normal ones (header, levels, every packed record:
// the verdicts were predicted, the prices taken from the plan's state instead of the level pool),
// and k_x_take, once the early plan is done, copies its outputs (final depths, side masks, touch
// count) into F and marks the header `pre`, so k_flow_plan_head leaves the book alone; the log
// follows (k_x_logcopy) and the reconstruction runs unchanged.  Anything that differs, or an early
// plan that was declined, leaves the normal plan to run: the early plan can cost time, never
// change a result.  gome_stats.n_early_miss counts early plans that were ready but not taken.
#pragma once
#include <hip/hip_runtime.h>

#include "match_flow.h"
#include "match_flow_deep.h"

namespace gome {

struct XCtl {
  uint32_t ok;     // k_x_prep_b accepted: XH / XL / X.ord8 describe the batch's hottest book
  uint32_t bad;    // k_x_adm: a record the prediction does not cover
  uint32_t mism;   // k_x_cmp: the early inputs differ from the batch's own prep
  uint32_t used;   // k_x_take: the early plan is the book's plan
  uint32_t kind;   // the previous plan of the book: FL_OK_ADD (lane plans) or FL_OK_DEEP
  uint32_t nnew;   // deep books: the batch's distinct prices (X.dnew, sorted)
  uint32_t pad[2];
  Status st;       // the early kernels' Dev::st (nhot: 1 = plan the hottest segment, 0 = skip; err)
};

// k_xd_prep_b's two prefix arrays, then every XD_S-th key of the old levels and of the batch's
// prices (the binary searches' first steps in LDS)
constexpr uint32_t XD_S = 16, XD_NS = DEEP_CAP / XD_S;
constexpr uint32_t XD_PREP_LDS = (2 * DEEP_CAP + 2) * 4 + 2 * XD_NS * 8;
constexpr uint32_t X_FIND_T = 256, X_FIND_B = 1024;  // k_x_count / k_x_scatter: blocks of contiguous records

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) { return rl(wave_incl_scan_u32(x), 63); }

// The previous batch's hottest book (its header: an ADD plan of batch bid_prev, lane or deep), or NIL.
__device__ __forceinline__ uint32_t x_hot_sym(const FlowHdr* hdr, uint32_t bid_prev) {
  const FlowHdr h = hdr[0];
  const bool add = h.ok == FL_OK_ADD || (h.ok == FL_OK_DEEP && !h.dc && h.ndel == 0 && h.dslot == 0);
  return (add && h.bid == bid_prev) ? h.sym : NIL;
}

__device__ __forceinline__ void x_range(uint32_t n, uint32_t& r0, uint32_t& r1) {
  const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
  r0 = min(n, blockIdx.x * per);
  r1 = min(n, r0 + per);
}

// Per block: records of the hot symbol, and records of lower symbols (the segment's start).
__global__ __launch_bounds__(X_FIND_T) void k_x_count(const gome_order* ord, uint32_t n, const FlowHdr* hdr,
                                                      uint32_t bid_prev, uint32_t* cnt) {
  const uint32_t hs = x_hot_sym(hdr, bid_prev);
  uint32_t r0, r1;
  x_range(n, r0, r1);
  uint32_t c = 0, lt = 0;
  if (hs != NIL)
    for (uint32_t i = r0 + threadIdx.x; i < r1; i += X_FIND_T) {
      const uint32_t sy = ord[i].symbol_id;
      c += sy == hs ? 1u : 0u;
      lt += sy < hs ? 1u : 0u;
    }
  c = wave_sum_u32(c);
  lt = wave_sum_u32(lt);
  __shared__ uint32_t sc[X_FIND_T / 64], sl[X_FIND_T / 64];
  if (lane_id() == 0) { sc[threadIdx.x >> 6] = c; sl[threadIdx.x >> 6] = lt; }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0, b = 0;
    for (uint32_t w = 0; w < X_FIND_T / 64; ++w) { a += sc[w]; b += sl[w]; }
    cnt[blockIdx.x] = a;
    cnt[gridDim.x + blockIdx.x] = b;
  }
}

// Exclusive scan of the blocks' counts; the segment [beg, end) the stable sort will give the hot
// symbol (xseg = {0, beg, end}: seg_order / seg_start of a one-segment batch), and st.nhot = 1 when
// it is a flow candidate.  One block of X_FIND_B threads.
__global__ __launch_bounds__(X_FIND_B) void k_x_scan(const FlowHdr* hdr, uint32_t bid_prev, uint32_t* cnt,
                                                     uint32_t nblk, uint32_t* xseg, XCtl* X) {
  __shared__ uint32_t part[X_FIND_B / 64], lts[X_FIND_B / 64];
  const uint32_t t = threadIdx.x;
  const uint32_t c = t < nblk ? cnt[t] : 0u, lt = t < nblk ? cnt[nblk + t] : 0u;
  const uint32_t inc = wave_incl_scan_u32(c), ls = wave_sum_u32(lt);
  if (lane_id() == 63) part[t >> 6] = inc;
  if (lane_id() == 0) lts[t >> 6] = ls;
  __syncthreads();
  uint32_t before = 0, beg = 0, tot = 0;
  for (uint32_t w = 0; w < X_FIND_B / 64; ++w) {
    if (w < (t >> 6)) before += part[w];
    beg += lts[w];
    tot += part[w];
  }
  if (t < nblk) cnt[t] = before + inc - c;
  if (t == 0) {
    xseg[0] = 0;
    xseg[1] = beg;
    xseg[2] = beg + tot;
    X->st.nhot = (x_hot_sym(hdr, bid_prev) != NIL && tot >= (1u << FLOW_MIN_LOG2)) ? 1u : 0u;
    X->kind = hdr[0].ok;
  }
}

// xsidx[beg + rank] = batch index of the hot symbol's rank-th record (batch order): the slice of
// the stable sort's permutation that covers the segment.
__global__ __launch_bounds__(X_FIND_T) void k_x_scatter(const gome_order* ord, uint32_t n, const FlowHdr* hdr,
                                                        uint32_t bid_prev, const uint32_t* cnt, const uint32_t* xseg,
                                                        const XCtl* X, uint32_t* xsidx) {
  if (X->st.nhot == 0) return;
  const uint32_t hs = x_hot_sym(hdr, bid_prev);
  uint32_t r0, r1;
  x_range(n, r0, r1);
  __shared__ uint32_t wc[X_FIND_T / 64];
  uint32_t base = xseg[1] + cnt[blockIdx.x];
  const uint32_t w = threadIdx.x >> 6;
  for (uint32_t c0 = r0; c0 < r1; c0 += X_FIND_T) {
    const uint32_t i = c0 + threadIdx.x;
    const bool m = i < r1 && ord[i].symbol_id == hs;
    const unsigned long long bm = __ballot(m);
    if (lane_id() == 0) wc[w] = __popcll(bm);
    __syncthreads();
    uint32_t off = 0, all = 0;
    for (uint32_t k = 0; k < X_FIND_T / 64; ++k) {
      off += k < w ? wc[k] : 0u;
      all += wc[k];
    }
    if (m) xsidx[base + off + __popcll(bm & lt_mask())] = i;
    base += all;
    __syncthreads();
  }
}

// The verdicts k_adm will give the hottest segment's records, when they are all ADDs whose oids
// rise in batch order above the book's oid_max: such a key is alone in the batch and rests
// nowhere, so on both admission paths (fresh batch or the tables) its verdict is its own.
__global__ void k_x_adm(BatchArgs Bx, XCtl* X, const uint32_t* oid_max, uint32_t max_symbols, uint32_t* xadm) {
  if (X->st.nhot == 0) return;
  const uint32_t seg = Bx.seg_order[0];
  const uint32_t beg = Bx.seg_start[seg], end = Bx.seg_start[seg + 1];
  const uint32_t sym = Bx.ord[Bx.sidx[beg]].symbol_id;
  if (sym >= max_symbols) {
    if (blockIdx.x == 0 && threadIdx.x == 0) X->bad = 1;
    return;
  }
  const uint32_t om = oid_max[sym];
  bool bad = false;
  for (uint32_t b = beg + blockIdx.x * blockDim.x + threadIdx.x; b < end; b += gridDim.x * blockDim.x) {
    const uint32_t j = Bx.sidx[b];
    const gome_order o = Bx.ord[j];
    const uint32_t prev = b == beg ? om : Bx.ord[Bx.sidx[b - 1]].oid_id;
    if (o.action != GOME_ADD || o.oid_id <= prev) bad = true;
    xadm[j] = (!(o.flags & GOME_ORD_ADM_HOST) || (o.flags & GOME_ORD_ADMITTED)) ? ADM_V_YES : ADM_V_NO;
  }
  if (__any(bad) && lane_id() == 0) atomicOr(&X->bad, 1u);
}

// The lane plan's records in two halves around the last plan's end.  Before it (early stream),
// k_x_gather reads each of the segment's records through the permutation (the dependent loads)
// into a compact 16-B entry in segment order: the price key, and for an admitted ADD its volume
// with bit 63 set and bit 62 for a SALE.  After it (plan stream, on the plan's CUs), k_x_prep_c
// maps the key to its level and writes the record, k_flow_prep_c's output: reading the compact
// entries in order took the early chain's k_flow_prep_c 109 us -> (config 3, gpurun_out/r05bx).
struct XComp {
  unsigned long long key, v;
};
__global__ __launch_bounds__(256) void k_x_gather(BatchArgs Bx, const uint32_t* __restrict__ xseg, XComp* __restrict__ out) {
  const uint32_t beg = xseg[1], end = xseg[2];
  for (uint32_t b = beg + blockIdx.x * blockDim.x + threadIdx.x; b < end; b += gridDim.x * blockDim.x) {
    const Prep q = prep_at(Bx, b);
    XComp c;
    c.key = static_cast<unsigned long long>(q.price) + FL_KEY_OFF;
    c.v = (q.action == GOME_ADD && q.adm)
              ? static_cast<unsigned long long>(q.vol) | (1ull << 63) | (q.side == GOME_SALE ? 1ull << 62 : 0ull)
              : 0ull;
    out[b - beg] = c;
  }
}
constexpr uint32_t X_PREPC_U = 4;
__global__ __launch_bounds__(FL_PREP_T) void k_x_prep_c(Dev D, FlowArgs F, const XComp* __restrict__ comp) {
  __shared__ unsigned long long hkey[FL_HASH];
  __shared__ uint32_t hval[FL_HASH];
  const uint32_t h = F.h0, tid = threadIdx.x;
  if (h >= fl_hend(D, F) || !uni(F.hdr[h].ok)) return;
  const FlPrepScr* P = F.pscr;
  const FlowHdr* hd = &F.hdr[h];
  const uint32_t n = hd->end - hd->beg, obase = hd->obase;
  const bool w32 = hd->w32 != 0;
  const unsigned long long g = hd->g;
  for (uint32_t i = tid; i < FL_HASH; i += FL_PREP_T) {
    hkey[i] = P->key[i];
    hval[i] = P->val[i];
  }
  __syncthreads();
  const uint32_t stride = gridDim.x * FL_PREP_T;
  for (uint32_t i0 = blockIdx.x * FL_PREP_T + tid; i0 < n; i0 += X_PREPC_U * stride) {
    XComp c[X_PREPC_U];
#pragma unroll
    for (uint32_t u = 0; u < X_PREPC_U; ++u)
      if (i0 + u * stride < n) c[u] = comp[i0 + u * stride];
#pragma unroll
    for (uint32_t u = 0; u < X_PREPC_U; ++u) {
      const uint32_t i = i0 + u * stride;
      if (i >= n) break;
      unsigned long long rec = fl_rec(false, 0, 0, false, i, w32);
      if (c[u].v >> 63) {
        const unsigned long long key = c[u].key;
        uint32_t s = fl_hash(key);
        while (hkey[s] != key) s = (s + 1) & (FL_HASH - 1);
        const unsigned long long vol = c[u].v & ((1ull << 62) - 1ull);
        const unsigned long long v = w32 ? static_cast<unsigned long long>(static_cast<double>(vol) / static_cast<double>(g)) : vol;
        rec = fl_rec(true, hval[s], v, ((c[u].v >> 62) & 1ull) != 0, i, w32);
      }
      F.ord8[obase + i] = rec;
    }
  }
}

// The early head prep's price set and header (k_flow_prep_b's, with the book's live levels taken
// from the previous batch's plan instead of the level pool).  F: the pipeline's own flow args
// (F.hdr[0] / F.lvl: the previous batch's hottest book after its plan, header of batch bid_prev).
__global__ __launch_bounds__(FL_PREP_T) void k_x_prep_b(BatchArgs Bx, FlowArgs FX, FlowArgs F, XCtl* X,
                                                        uint32_t bid_prev) {
  __shared__ unsigned long long hkey[FL_HASH];
  __shared__ uint32_t hval[FL_HASH];
  __shared__ unsigned long long ckey[FL_CAP + FL_PREP_T];
  __shared__ uint32_t cslot[FL_CAP + FL_PREP_T];
  __shared__ uint32_t ndist, nc, bad;
  __shared__ unsigned long long wg[FL_PREP_T / 64], ws[FL_PREP_T / 64];
  const uint32_t tid = threadIdx.x;
  FlowHdr* hd = &FX.hdr[0];
  FlPrepScr* P = FX.pscr;
  const FlowHdr ph = F.hdr[0];
  const uint32_t seg = Bx.seg_order[0];
  const uint32_t beg = Bx.seg_start[seg], end = Bx.seg_start[seg + 1];
  if (X->kind != FL_OK_ADD) return;  // (a deep book: k_xd_prep_b)
  if (tid == 0) {
    ndist = nc = 0;
    bad = (X->st.nhot == 0 || X->bad || P->bad || P->many || P->dels || ph.ok != FL_OK_ADD || ph.bid != bid_prev ||
           ph.sym != Bx.ord[Bx.sidx[beg]].symbol_id || (end - beg) >= FL_MAX_ORDERS || ph.nl > FL_MAX)
              ? 1u : 0u;
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) { hd->ok = 0; X->st.nhot = 0; }
    return;
  }
  uint32_t my_n = 0;
  for (uint32_t i = tid; i < FL_HASH; i += FL_PREP_T) {
    hkey[i] = P->key[i];
    hval[i] = NIL;
    my_n += hkey[i] ? 1u : 0u;
  }
  if (my_n) atomicAdd(&ndist, my_n);
  __syncthreads();
  // the previous plan's live levels: side from its final masks, depth from dfin
  const FlowLvl* LP = F.lvl;
  unsigned long long mg = 0, msum = 0;
  if (tid < FL_PG) {
    mg = P->pg[tid];
    msum = P->ps[tid];
  }
  for (uint32_t q = 1 + tid; q <= ph.nl; q += FL_PREP_T) {
    const bool sa = ((q < 64 ? ph.amask[0] >> q : ph.amask[1] >> (q - 64)) & 1ull) != 0;
    const bool sb = ((q < 64 ? ph.bmask[0] >> q : ph.bmask[1] >> (q - 64)) & 1ull) != 0;
    const int64_t d = LP[q].dfin;
    if (!sa && !sb) {
      if (d != 0) bad = 1;
      continue;
    }
    if ((sa && sb) || d <= 0) { bad = 1; continue; }
    mg = fl_gcd(mg, static_cast<unsigned long long>(d));
    msum = min(msum + static_cast<unsigned long long>(d), FL_SUM_CAP);
    bool fresh;
    const uint32_t sl = fl_set_put(hkey, static_cast<unsigned long long>(LP[q].price) + FL_KEY_OFF, &fresh);
    if (sl == FL_HASH) { bad = 1; continue; }
    hval[sl] = q;
    if (fresh) atomicAdd(&ndist, 1u);
  }
  fl_block_gcd_sum(mg, msum, wg, ws);  // (synchronises the block)
  if (bad || ndist > FL_MAX) {
    if (tid == 0) { hd->ok = 0; X->st.nhot = 0; }
    return;
  }
  for (uint32_t sl = tid; sl < FL_HASH; sl += FL_PREP_T) {
    if (hkey[sl]) {
      const uint32_t i = atomicAdd(&nc, 1u);
      ckey[i] = hkey[sl];
      cslot[i] = sl;
    }
  }
  __syncthreads();
  const uint32_t n = nc;
  FlowLvl* LV = FX.lvl;
  if (tid < n) {
    const unsigned long long key = ckey[tid];
    uint32_t r = 0;
    for (uint32_t i = 0; i < n; ++i) r += ckey[i] < key ? 1u : 0u;
    const uint32_t sl = cslot[tid], q = hval[sl];
    FlowLvl f{};
    f.price = static_cast<int64_t>(key - FL_KEY_OFF);
    f.old = q;  // (the previous plan's level index: informational)
    f.head = f.tail = NIL;
    if (q != NIL) {
      const bool sa = ((q < 64 ? ph.amask[0] >> q : ph.amask[1] >> (q - 64)) & 1ull) != 0;
      f.d0 = LP[q].dfin;
      f.mem0 = sa ? M_SALE : M_BUY;
    }
    LV[r + 1] = f;
    hval[sl] = r + 1;
  }
  __syncthreads();
  for (uint32_t i = tid; i < FL_HASH; i += FL_PREP_T) {
    P->key[i] = hkey[i];
    P->val[i] = hval[i];
  }
  unsigned long long g = mg ? mg : 1;
  const bool w32 = msum < FL_SUM_CAP && msum / g < (1ull << 32);
  if (!w32) g = 1;
  if (tid < ((8u - ((end - beg) & 7u)) & 7u))  // padding to whole half-groups (8 records)
    FX.ord8[(end - beg) + tid] = fl_rec(false, 0, 0, false, end - beg + tid, w32);
  if (tid == 0) {
    FlowHdr x{};
    x.ok = FL_OK_ADD;
    x.nl = n;
    x.sym = ph.sym;
    x.beg = beg;
    x.end = end;
    x.adds = P->adds;
    x.dropped = P->dropped;
    x.obase = 0;
    x.w32 = w32 ? 1u : 0u;
    x.g = g;
    *hd = x;
    X->ok = 1;
  }
}

// ---- deep books (W32D / W32DV, match_flow_deep.h) -------------------------------------------
// The batch's prices of the book into the early price set (FX.dh_key, emptied per batch), the
// volumes' gcd / sum per slice and the counts (k_deep_prep_a's, into the early scratch).
__global__ __launch_bounds__(FL_PREP_T) void k_xd_prep_a(BatchArgs Bx, FlowArgs FX, XCtl* X) {
  __shared__ uint32_t adds, dropped, bad, nd;
  __shared__ unsigned long long wg[FL_PREP_T / 64], ws[FL_PREP_T / 64];
  if (X->kind != FL_OK_DEEP || X->st.nhot == 0) return;
  const uint32_t tid = threadIdx.x;
  FlPrepScr* P = FX.dscr;
  uint32_t b0, b1;
  fd_slice(Bx.seg_start[0], Bx.seg_start[1], blockIdx.x, gridDim.x, b0, b1);
  if (tid == 0) adds = dropped = bad = nd = 0;
  __syncthreads();
  unsigned long long mg = 0, msum = 0;
  uint32_t my_adds = 0, my_drop = 0, my_bad = 0, my_nd = 0;
  for (uint32_t b = b0 + tid; b < b1; b += FL_PREP_T) {
    const Prep q = prep_at(Bx, b);
    if (q.action != GOME_ADD) { my_bad = 1; continue; }
    my_adds++;
    if (!q.adm) { my_drop++; continue; }
    if (q.vol == 0 || q.adm == ADM_V_CHECK) { my_bad = 1; continue; }
    const unsigned long long v = static_cast<unsigned long long>(q.vol);
    mg = fl_gcd(mg, v);
    msum = min(msum + v, FL_SUM_CAP);
    bool fresh;
    if (fd_put(FX.dh_key, static_cast<unsigned long long>(q.price) + FL_KEY_OFF, &fresh) == NIL) my_bad = 1;
    my_nd += fresh ? 1u : 0u;
  }
  if (my_adds) atomicAdd(&adds, my_adds);
  if (my_drop) atomicAdd(&dropped, my_drop);
  if (my_bad) bad = 1;
  if (my_nd) atomicAdd(&nd, my_nd);
  fl_block_gcd_sum(mg, msum, wg, ws);  // (synchronises the block)
  if (tid == 0) {
    P->pg[blockIdx.x] = mg;
    P->ps[blockIdx.x] = msum;
    if (adds) atomicAdd(&P->d_adds, adds);
    if (dropped) atomicAdd(&P->d_dropped, dropped);
    if (bad) atomicOr(&P->d_bad, 1u);
    if (nd) atomicAdd(&P->d_ndist, nd);
  }
}

// The batch's distinct prices of the book, sorted (bitonic in LDS, one workgroup), into dnew:
// this runs beside the previous plan, so only a merge is left after it.
// Dynamic LDS: DEEP_CAP keys.
__global__ __launch_bounds__(FL_PREP_T) void k_xd_sort_new(FlowArgs FX, XCtl* X, unsigned long long* dnew) {
  __shared__ uint32_t nc;
  if (X->kind != FL_OK_DEEP || X->st.nhot == 0) return;
  const uint32_t tid = threadIdx.x;
  const FlPrepScr* P = FX.dscr;
  const uint32_t n = P->d_ndist;
  if (P->d_bad || n > DEEP_CAP - 2) {
    if (tid == 0) X->bad = 1;
    return;
  }
  unsigned long long* sk = reinterpret_cast<unsigned long long*>(fl_ring);
  if (tid == 0) nc = 0;
  __syncthreads();
  for (uint32_t sl = tid; sl < DEEP_HASH; sl += FL_PREP_T) {
    const unsigned long long key = FX.dh_key[sl];
    if (key) sk[atomicAdd(&nc, 1u)] = key;
  }
  __syncthreads();
  uint32_t np = 1024;
  while (np < n) np <<= 1;
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
  for (uint32_t i = tid; i < n; i += FL_PREP_T) dnew[i] = sk[i];
  if (tid == 0) X->nnew = n;
}

// Exclusive block scan of flags f[0..n) in place (FL_PREP_T threads, chunks of FL_PREP_T);
// f[n] = the total.
__device__ __forceinline__ void x_block_scan(uint32_t* f, uint32_t n, uint32_t* wsum) {
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < n; c0 += FL_PREP_T) {
    const uint32_t i = c0 + threadIdx.x;
    const uint32_t v = i < n ? f[i] : 0u;
    const uint32_t inc = wave_incl_scan_u32(v);
    if (lane_id() == 63) wsum[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t w = 0; w < FL_PREP_T / 64; ++w) {
      before += w < (threadIdx.x >> 6) ? wsum[w] : 0u;
      all += wsum[w];
    }
    if (i < n) f[i] = carry + before + inc - v;
    carry += all;
    __syncthreads();
  }
  if (threadIdx.x == 0) f[n] = carry;
  __syncthreads();
}

// First index in [0, n) whose key is >= x (keys ascending), n if none.
template <class Key>
__device__ __forceinline__ uint32_t x_lower(Key key, uint32_t n, unsigned long long x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (key(mid) < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// x_lower through a sample s[k] = key(k * XD_S), k < ns, in LDS: the sample's search leaves a
// window of at most XD_S keys, searched in global memory (the hottest deep book's ~10k levels
// and prices: 14 dependent global loads per search before, ~4 now).
template <class Key>
__device__ __forceinline__ uint32_t xs_lower(const unsigned long long* smp, uint32_t ns, Key key, uint32_t n,
                                             unsigned long long x) {
  uint32_t lo = 0, hi = ns;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (smp[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  // key((lo - 1) * XD_S) < x <= key(lo * XD_S): the answer is in ((lo - 1) * XD_S, lo * XD_S]
  uint32_t a = lo ? (lo - 1) * XD_S + 1 : 0u, b = min(lo * XD_S, n);
  while (a < b) {
    const uint32_t mid = (a + b) >> 1;
    if (key(mid) < x) a = mid + 1;
    else b = mid;
  }
  return a;
}

// The early deep prep after the previous plan: its live levels (F.dlvl of deep slot 0: price,
// dfin, memf; sorted by price) merged with the batch's sorted prices into the level table
// (FX.dlvl), each batch price's level into the early set's values, the header.  A merge by
// ranks (scans and binary searches) instead of k_deep_prep_b's sort of the whole set.
// Dynamic LDS: two DEEP_CAP + 1 flag / prefix arrays.
__global__ __launch_bounds__(FL_PREP_T) void k_xd_prep_b(BatchArgs Bx, FlowArgs FX, FlowArgs F, XCtl* X,
                                                         const unsigned long long* dnew, uint32_t bid_prev) {
  __shared__ uint32_t bad, wsum[FL_PREP_T / 64];
  __shared__ unsigned long long wg[FL_PREP_T / 64], ws[FL_PREP_T / 64];
  if (X->kind != FL_OK_DEEP) return;
  const uint32_t tid = threadIdx.x;
  FlowHdr* hd = &FX.hdr[0];
  const FlPrepScr* P = FX.dscr;
  const FlowHdr ph = F.hdr[0];
  const uint32_t beg = Bx.seg_start[0], end = Bx.seg_start[1];
  const uint32_t nlp = ph.nl, nn = X->nnew;
  if (tid == 0) {
    const uint64_t tiles = (static_cast<uint64_t>(FL_TOUCH_MUL) * (end - beg) + FL_TILE - 1) / FL_TILE;
    bad = (X->st.nhot == 0 || X->bad || P->d_bad || ph.ok != FL_OK_DEEP || ph.dc || ph.ndel || ph.dslot != 0 ||
           ph.bid != bid_prev || ph.sym != Bx.ord[Bx.sidx[beg]].symbol_id || nlp > DEEP_CAP - 2 || tiles > F.dmaxt)
              ? 1u : 0u;
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) X->st.nhot = 0;
    return;
  }
  const FlowLvl* LP = F.dlvl;  // (deep slot 0: the hottest book's)
  uint32_t* lpre = reinterpret_cast<uint32_t*>(fl_ring);  // [nlp + 1]: live old levels before
  uint32_t* mpre = lpre + DEEP_CAP + 1;                     // [nn + 1]: batch prices on a live old level before
  unsigned long long* so = reinterpret_cast<unsigned long long*>(mpre + DEEP_CAP + 1);  // samples: old keys
  unsigned long long* sn = so + XD_NS;                                                // ... batch prices
  auto oldkey = [&](uint32_t i) { return static_cast<unsigned long long>(LP[i + 1].price) + FL_KEY_OFF; };
  auto newkey = [&](uint32_t k) { return dnew[k]; };
  const uint32_t nso = (nlp + XD_S - 1) / XD_S, nsn = (nn + XD_S - 1) / XD_S;
  for (uint32_t k = tid; k < nso; k += FL_PREP_T) so[k] = oldkey(k * XD_S);
  for (uint32_t k = tid; k < nsn; k += FL_PREP_T) sn[k] = dnew[k * XD_S];
  __syncthreads();
  unsigned long long mg = 0, msum = 0;
  if (tid < FL_PG) {
    mg = P->pg[tid];
    msum = P->ps[tid];
  }
  for (uint32_t i = tid; i < nlp; i += FL_PREP_T) {
    const FlowLvl& f = LP[i + 1];
    const bool live = f.memf != 0;
    if (live != (f.dfin > 0) || f.memf == (M_BUY | M_SALE)) bad = 1;
    if (live) {
      mg = fl_gcd(mg, static_cast<unsigned long long>(f.dfin));
      msum = min(msum + static_cast<unsigned long long>(f.dfin), FL_SUM_CAP);
    }
    lpre[i] = live ? 1u : 0u;
  }
  for (uint32_t i = tid; i < nn; i += FL_PREP_T) {
    const uint32_t q = xs_lower(so, nso, oldkey, nlp, dnew[i]);
    mpre[i] = (q < nlp && oldkey(q) == dnew[i] && LP[q + 1].memf != 0) ? 1u : 0u;
  }
  fl_block_gcd_sum(mg, msum, wg, ws);  // (synchronises the block)
  x_block_scan(lpre, nlp, wsum);
  x_block_scan(mpre, nn, wsum);
  const uint32_t n = lpre[nlp] + nn - mpre[nn];
  const unsigned long long g = mg ? mg : 1;
  const bool w32 = msum < FL_SUM_CAP && msum / g < (1ull << 32);
  if (bad || n > DEEP_CAP - 2 || !w32) {
    if (tid == 0) X->st.nhot = 0;
    return;
  }
  FlowLvl* LV = FX.dlvl;
  // live old levels: rank = live ones before + batch-only prices below
  for (uint32_t i = tid; i < nlp; i += FL_PREP_T) {
    const FlowLvl& o = LP[i + 1];
    if (!o.memf) continue;
    const uint32_t pos = xs_lower(sn, nsn, newkey, nn, oldkey(i));
    FlowLvl f{};
    f.price = o.price;
    f.d0 = o.dfin;
    f.mem0 = o.memf;
    f.old = i + 1;  // (the previous plan's level: informational)
    f.head = f.tail = NIL;
    f.ig_all = 1;
    LV[lpre[i] + (pos - mpre[pos]) + 1] = f;
  }
  // the batch's prices: a new level unless a live old level has it; each one's level in the set
  for (uint32_t i = tid; i < nn; i += FL_PREP_T) {
    const unsigned long long key = dnew[i];
    const uint32_t q = xs_lower(so, nso, oldkey, nlp, key);  // (live old levels below: lpre[q])
    const bool on_old = mpre[i + 1] != mpre[i];
    const uint32_t r = lpre[q] + (i - mpre[i]) + 1;
    if (!on_old) {
      FlowLvl f{};
      f.price = static_cast<int64_t>(key - FL_KEY_OFF);
      f.old = NIL;
      f.head = f.tail = NIL;
      f.ig_all = 1;
      LV[r] = f;
    }
    FX.dh_val[fd_find(FX.dh_key, key)] = r;
  }
  if (tid < ((8u - ((end - beg) & 7u)) & 7u)) FX.ord8[(end - beg) + tid] = 0ull;  // no-op padding
  if (tid == 0) {
    FlowLvl z{};  // the bid sentinel's row, clean (as k_deep_prep_b)
    z.old = NIL;
    z.head = z.tail = NIL;
    LV[0] = z;
    FlowHdr x{};
    x.ok = FL_OK_DEEP;
    x.nl = n;
    x.sym = ph.sym;
    x.beg = beg;
    x.end = end;
    x.adds = P->d_adds;
    x.dropped = P->d_dropped;
    x.obase = 0;
    x.w32 = 1;
    x.g = g;
    x.deep = 1;
    x.dslot = 0;
    *hd = x;
    X->ok = 1;
  }
}

// The early inputs against the batch's own head prep of the same book: header, levels, every
// packed record (a grid of blocks; block 0 also takes the header and the levels).
__global__ void k_x_cmp(Dev D, FlowArgs F, FlowArgs FX, XCtl* X) {
  if (!X->ok) return;
  const FlowHdr hd = F.hdr[0], xh = FX.hdr[0];
  const bool kind = (hd.ok == FL_OK_ADD || (hd.ok == FL_OK_DEEP && !hd.dc && hd.dslot == 0)) && xh.ok == hd.ok;
  bool diff = D.st->nhot == 0 || !kind || hd.bid != F.bid || hd.nl != xh.nl || hd.sym != xh.sym ||
              hd.beg != xh.beg || hd.end != xh.end || hd.adds != xh.adds || hd.dropped != xh.dropped ||
              hd.w32 != xh.w32 || hd.g != xh.g || hd.ndel != 0;
  if (!diff) {
    const FlowLvl* A = fl_lvls(F, 0);
    const FlowLvl* B = fl_lvls(FX, 0);
    for (uint32_t q = 1 + blockIdx.x * blockDim.x + threadIdx.x; q <= hd.nl; q += gridDim.x * blockDim.x)
      if (A[q].price != B[q].price || A[q].d0 != B[q].d0 || A[q].mem0 != B[q].mem0) diff = true;
    const uint32_t m = ((hd.end - hd.beg) + 7u) & ~7u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
      if (F.ord8[hd.obase + i] != FX.ord8[i]) diff = true;
  }
  if (__any(diff) && lane_id() == 0) atomicOr(&X->mism, 1u);
}

// After the early plan: take it (its final depths and sides, touch count into F, the header
// marked `pre`) when its inputs matched and it ran clean.
// (a grid: a deep book's ~10k levels took one block 45 us, on the early chain's critical path;
// every block decides alike, block 0 writes the header)
__global__ void k_x_take(Dev D, FlowArgs F, FlowArgs FX, XCtl* X) {
  __shared__ uint32_t use;
  const FlowHdr xh = FX.hdr[0];
  if (threadIdx.x == 0) {
    const uint32_t ok = F.hdr[0].ok;
    const bool normal = D.st->nhot != 0 && (ok == FL_OK_ADD || ok == FL_OK_DEEP) && ok == xh.ok;
    use = (X->ok && !X->mism && X->st.err == 0 && normal) ? 1u : 0u;
    // (a batch whose hottest book is another symbol than the last one's plans it normally)
    if (blockIdx.x == 0 && !use && normal && X->ok && F.hdr[0].sym == xh.sym) ctr_add(D, C_EARLY_MISS, 1ull);
  }
  __syncthreads();
  if (!use) return;
  FlowLvl* A = fl_lvls(F, 0);
  const FlowLvl* B = fl_lvls(FX, 0);
  for (uint32_t q = 1 + blockIdx.x * blockDim.x + threadIdx.x; q <= xh.nl; q += gridDim.x * blockDim.x) {
    A[q].dfin = B[q].dfin;
    A[q].memf = B[q].memf;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    FlowHdr* w = &F.hdr[0];
    w->ntouch = xh.ntouch;
    w->amask[0] = xh.amask[0];
    w->amask[1] = xh.amask[1];
    w->bmask[0] = xh.bmask[0];
    w->bmask[1] = xh.bmask[1];
    w->dv_ba = xh.dv_ba;
    w->pre = 1;
    X->used = 1;
    ctr_add(D, C_EARLY, 1ull);
  }
}

// The early plan's touch log to where the reconstruction reads the book's log.
__global__ void k_x_logcopy(FlowArgs F, FlowArgs FX, const XCtl* X) {
  if (!X->used) return;
  const FlowHdr xh = FX.hdr[0];
  const uint4* src = reinterpret_cast<const uint4*>(FX.log);
  uint4* dst = reinterpret_cast<uint4*>(F.log + static_cast<size_t>(FL_TOUCH_MUL) * xh.beg);
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < xh.ntouch; t += gridDim.x * blockDim.x) dst[t] = src[t];
}

}  // namespace gome
