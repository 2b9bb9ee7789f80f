// engine.hip — MI355X (gfx950) batch matching engine: kernels + C-ABI host runtime.
//
// Replaces the reference's serial consumer (gomengine/engine/rabbitmq.go:116-125
// calling engine.DoOrder, engine.go:46) with a per-batch device pipeline:
//
//   (input domain check of the 32-B records — symbol range, volume >= 0, |v| < 2^53 — is
//    done by k_adm, beside the radix sort)
//   k_radix_hist/     stable LSD radix sort of (symbol_id, seq) -> per-symbol segments in
//   k_radix_scatter   consume order (the reference is serial, so per-symbol order = arrival)
//   k_seg_*           segment starts + longest-first launch order (hottest book starts first)
//   k_adm             admission markers S:comparison (nodepool.go:14-28, Q4), batch model
//   k_match           match_books: ONE WAVEFRONT PER BOOK applies its segment in order:
//                     SetOrder / Match / MatchOrder / DeleteOrder (engine.go:56-206) with
//                     64-lane ballots over the level array and a 32-lane prefix scan over
//                     FIFO volumes to find how far a taker sweeps
//   k_flow_*          hot books on the flow path (match_flow.h): a serial plan over level
//                     aggregates, then parallel fills / FIFO rebuild (the batch's critical path)
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
#include "match_cold.h"
#include "match_flow.h"
#include "match_hot.h"
#include "pipeline.h"
#include "wave.h"

using namespace gome;

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
  hipStream_t flow_stream = nullptr;
  bool own_stream = false;
  hipEvent_t fork{}, join{}, evh0{}, evh1{};
  hipEvent_t joinf{}, prep_h{}, prep_t{}, evf0{}, evf1{}, fork_adm{}, adm_done{}, seg_done{}, ev_scan{}, ev_hot{};
  FlowArgs F{};
  Prep* d_prep = nullptr;
  PendEnt* d_pend = nullptr;
  ResumeRec* d_resume = nullptr;
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
    if (evf0) {
      (void)hipEventDestroy(evf0); (void)hipEventDestroy(evf1); (void)hipEventDestroy(joinf);
      (void)hipEventDestroy(prep_h); (void)hipEventDestroy(prep_t);
      (void)hipEventDestroy(fork_adm); (void)hipEventDestroy(adm_done); (void)hipEventDestroy(seg_done);
      (void)hipEventDestroy(ev_scan); (void)hipEventDestroy(ev_hot);
    }
    if (hot_stream) (void)hipStreamDestroy(hot_stream);
    if (flow_stream) (void)hipStreamDestroy(flow_stream);
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
  HIPCHK(hipStreamCreateWithFlags(&flow_stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&joinf, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&prep_h, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&prep_t, hipEventDisableTiming));
  HIPCHK(hipEventCreate(&evf0));
  HIPCHK(hipEventCreate(&evf1));
  HIPCHK(hipEventCreateWithFlags(&fork_adm, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&adm_done, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&seg_done, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&ev_scan, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&ev_hot, hipEventDisableTiming));
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
      !alloc(&D.lvl_bump, 1, "lvl_bump") || !alloc(&D.nodes, nchunks * CH, "chunks") ||
      !alloc(&D.chdr, nchunks, "chunk headers") ||
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
      !alloc(&d_resume, MAX_HOT, "resume records") ||
      !alloc(&d_arena, arena_cap, "event arena") || !alloc(&d_events, arena_cap, "events"))
    return GOME_E_CAPACITY;
  // flow path (match_flow.h): per-hot-book headers and level slots, packed records, the
  // touch log and its per-level views (FL_TOUCH_MUL entries per order), gathered makers
  const uint64_t ntouch = static_cast<uint64_t>(FL_TOUCH_MUL) * nb;
  F.ig_cap = static_cast<uint32_t>(std::min<uint64_t>(std::max<uint64_t>(cfg.max_nodes, 1u << 16), 0xF0000000ull));
  F.enabled = (cfg.flags & GOME_FLAG_LEGACY_HOT) ? 0u : 1u;
  if (!alloc(&F.hdr, MAX_FLOW, "flow headers") || !alloc(&F.lvl, MAX_FLOW * FL_CAP, "flow levels") ||
      !alloc(&F.ord8, static_cast<uint64_t>(FL_ORD8_MUL) * nb + FL_ORD8_PAD, "flow records") || !alloc(&F.log, ntouch, "flow touch log") ||
      !alloc(&F.srt, ntouch, "flow level runs") || !alloc(&F.rs, ntouch, "flow new makers") ||
      !alloc(&F.fbase, ntouch, "flow fill bases") || !alloc(&F.ig, F.ig_cap, "flow gathered makers") ||
      !alloc(&F.ig_bump, 1, "flow gather bump") || !alloc(&F.toff, MAX_FLOW + 16, "flow touch offsets") ||
      !alloc(&F.lvout, static_cast<size_t>(MAX_FLOW) * FL_CAP, "flow final levels"))
    return GOME_E_CAPACITY;
  F.maxt = ceil_div(ntouch, FL_TILE);
  if (!alloc(&F.tcnt, static_cast<size_t>(FL_HEAD) * F.maxt * FL_CAP, "flow head tile counts") ||
      !alloc(&F.pscr, FL_HEAD, "flow head prep scratch"))
    return GOME_E_CAPACITY;
  HIPCHK(hipMemsetAsync(F.hdr, 0, sizeof(FlowHdr) * MAX_FLOW, stream));
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
  // admission markers depend on the input records only: they run on the flow stream beside
  // the validation, the radix sort and the segmentation (the batch's critical path)
  HIPCHK(hipEventRecord(fork_adm, s));
  HIPCHK(hipStreamWaitEvent(flow_stream, fork_adm, 0));
  HIPCHK(hipMemsetAsync(d_claim, 0, (adm_mask + 1ull) * 4, flow_stream));
  HIPCHK(hipMemsetAsync(d_amin, 0xFF, (adm_mask + 1ull) * 4, flow_stream));
  k_adm<<<gN, T256, 0, flow_stream>>>(d_ord, n, d_claim, d_amin, d_adm_slot, adm_mask, cfg.max_symbols, d_st);
  k_adm_flag<<<gN, T256, 0, flow_stream>>>(d_ord, n, d_adm_slot, d_amin);
  HIPCHK(hipEventRecord(adm_done, flow_stream));

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
  k_seg_bscan<<<1, 64, 0, s>>>(d_bcnt, d_bcnt + 32, d_st, FLOW_MIN_LOG2, MAX_FLOW);
  k_seg_scatter<<<gN, T256, 0, s>>>(d_seg_start, d_st, d_bcnt + 32, d_seg_order);

  BatchArgs B;
  B.prep = d_prep;
  B.ord = d_ord;
  B.n = n;
  B.seg_start = d_seg_start;
  B.seg_order = d_seg_order;
  B.arena = d_arena;
  B.arena_cap = arena_cap;
  B.ev_count = d_ev_count;
  B.sidx = sidx;
  B.adm_flag = d_adm_slot;
  const uint32_t grid = std::min<uint32_t>(n, cfg.max_symbols);
  const uint32_t nhot_max = std::min<uint32_t>(MAX_FLOW, grid);
  // flow path: the head (longest FL_HEAD candidates, the batch's critical path) and the tail
  // each run prep -> serial plan -> parallel reconstruction on their own stream, so the
  // hottest book's plan starts after its own prep and the tail overlaps it
  // FH: the head's prep; FH0: the hottest book (plan + reconstruction on the flow stream,
  // the batch's critical path); FH1: the other head books (on the tail's stream, done long
  // before the hottest); FT: the tail.  tb: each range's slice of toff.
  FlowArgs FH = F, FH0 = F, FH1 = F, FT = F;
  FH.h0 = 0; FH.h1 = FL_HEAD; FH.tb = 0;
  FH0.h0 = 0; FH0.h1 = 1; FH0.tb = 0;
  FH1.h0 = 1; FH1.h1 = FL_HEAD; FH1.tb = 2;
  FT.h0 = FL_HEAD; FT.h1 = MAX_FLOW; FT.tb = FL_HEAD + 3;
  const uint32_t nh_head = std::min<uint32_t>(FL_HEAD, nhot_max);
  const uint32_t nh_near = nh_head > 1 ? nh_head - 1 : 0;
  const uint32_t nh_tail = nhot_max > FL_HEAD ? nhot_max - FL_HEAD : 0;
  // the head's prep gathers through the sort permutation (prep_at): it starts right after
  // segmentation, beside k_prep
  HIPCHK(hipEventRecord(seg_done, s));
  HIPCHK(hipStreamWaitEvent(flow_stream, seg_done, 0));
  HIPCHK(hipMemsetAsync(F.pscr, 0, sizeof(FlPrepScr) * FL_HEAD, flow_stream));
  k_flow_prep_a<<<dim3(FL_PG, nh_head), FL_PREP_T, 0, flow_stream>>>(D, B, FH);
  k_flow_prep_b<<<nh_head, FL_PREP_T, 0, flow_stream>>>(D, B, FH);
  k_flow_prep_c<<<dim3(FL_PG, nh_head), FL_PREP_T, 0, flow_stream>>>(D, B, FH);
  HIPCHK(hipEventRecord(prep_h, flow_stream));
  HIPCHK(hipEventRecord(evf0, flow_stream));
  k_flow_plan_head<<<1, 256, 0, flow_stream>>>(D, FH0);
  HIPCHK(hipEventRecord(evf1, flow_stream));
  // ---- admission markers (k_adm, launched above on the flow stream)
  HIPCHK(hipStreamWaitEvent(s, adm_done, 0));
  // k_prep gathers the same records as the head's prep: let the head's prep (the critical
  // path) have the memory system first; the cold books have slack
  HIPCHK(hipStreamWaitEvent(s, prep_h, 0));

  // ---- match_books: one wavefront per book; hot books (LDS) on a second stream,
  //      concurrently with the cold books (HBM)
  k_prep<<<gN, T256, 0, s>>>(d_ord, n, sidx, d_adm_slot, d_prep);
  HIPCHK(hipEventRecord(evm0, s));
  HIPCHK(hipMemsetAsync(F.ig_bump, 0, 4, s));
  HIPCHK(hipEventRecord(fork, s));
  HIPCHK(hipStreamWaitEvent(flow_stream, fork, 0));  // (k_prep, the gather bump)
  // the hottest book's reconstruction: wide kernels (tile-parallel sort, one wave per level)
  auto head_recon = [&](const FlowArgs& R, uint32_t nb, hipStream_t st) {
    k_flow_sort_cnt<<<dim3(FL_SORT_GRID, nb), FL_TILE, 0, st>>>(D, R);
    k_flow_sort_scan<<<nb, FL_CAP, 0, st>>>(D, R);
    k_flow_sort_scatter<<<dim3(FL_SORT_GRID, nb), FL_TILE, 0, st>>>(D, R);
    k_flow_level_wide<<<dim3(FL_CAP, nb), 64, 0, st>>>(D, R);
    k_flow_toff<<<1, 1024, 0, st>>>(D, R);
    k_flow_count<<<1024, 256, 0, st>>>(D, B, R);
    k_flow_write_lv<<<dim3(FL_CAP, nb), 64, 0, st>>>(D, B, R);
    k_flow_write_fin<<<nb, 128, 0, st>>>(D, R);
  };
  head_recon(FH0, 1, flow_stream);
  HIPCHK(hipEventRecord(joinf, flow_stream));
  // The tail's chain and the legacy hot kernels share the third stream: HIP maps more
  // streams than hardware queues (4 per process, one taken by the caller) onto shared
  // queues, which would serialise them behind the head.
  HIPCHK(hipStreamWaitEvent(hot_stream, fork, 0));
  if (nh_tail) {
    k_flow_prep<<<nh_tail, FL_PREP_T, 0, hot_stream>>>(D, B, FT);
    HIPCHK(hipEventRecord(prep_t, hot_stream));
    k_flow_plan_tail<<<nh_tail, 64, 0, hot_stream>>>(D, FT);
    k_flow_sort<<<nh_tail, FL_SORT_T, 0, hot_stream>>>(D, FT);
    k_flow_level<<<nh_tail, FL_LEVEL_T, 0, hot_stream>>>(D, FT);
    k_flow_toff<<<1, 1024, 0, hot_stream>>>(D, FT);
    k_flow_count<<<1024, 256, 0, hot_stream>>>(D, B, FT);
    k_flow_write<<<nh_tail, FL_WRITE_T, 0, hot_stream>>>(D, B, FT);
    // the tail's events into the arena now (k_ev_scatter places them after the scan)
    k_flow_events_arena<<<1024, 256, 0, hot_stream>>>(D, B, FT);
  } else {
    HIPCHK(hipEventRecord(prep_t, hot_stream));
  }
  // the other head books: plan, reconstruction and events (into the arena) after the tail
  HIPCHK(hipStreamWaitEvent(hot_stream, prep_h, 0));
  if (nh_near) {
    k_flow_plan_near<<<nh_near, 256, 0, hot_stream>>>(D, FH1);
    head_recon(FH1, nh_near, hot_stream);
    k_flow_events_arena<<<1024, 256, 0, hot_stream>>>(D, B, FH1);
  }
  // legacy hot path (books the flow path declined); it and the cold kernel read the preps'
  // routing decisions (FlowHdr::ok)
  HIPCHK(hipEventRecord(evh0, hot_stream));
  const uint32_t nleg = std::min<uint32_t>(MAX_HOT, grid);
  k_match_hot<<<nleg, 64, HOT_LDS_BYTES, hot_stream>>>(D, B, d_pend, d_resume, F.hdr);
  HIPCHK(hipEventRecord(evh1, hot_stream));
  k_match_resume<<<nleg, 64, 0, hot_stream>>>(D, B, d_resume);
  k_pend_apply<<<dim3(8, 64), 256, 0, hot_stream>>>(D, d_pend, d_seg_start, d_seg_order, B);
  HIPCHK(hipEventRecord(join, hot_stream));
  HIPCHK(hipStreamWaitEvent(s, prep_h, 0));
  HIPCHK(hipStreamWaitEvent(s, prep_t, 0));
  k_match<<<std::min<uint32_t>(grid, COLD_BLOCKS), 64, 0, s>>>(D, B, &F.hdr[0].ok, sizeof(FlowHdr) / sizeof(uint32_t));
  HIPCHK(hipStreamWaitEvent(s, join, 0));
  HIPCHK(hipStreamWaitEvent(s, joinf, 0));

  HIPCHK(hipEventRecord(evm1, s));

  // ---- event compaction into publish order
  scan(d_ev_count, n, d_ev_off, &d_st->n_events, s);
  // the hottest book's events and the arena scatter fill disjoint slots: run them side by side
  HIPCHK(hipEventRecord(ev_scan, s));
  HIPCHK(hipStreamWaitEvent(flow_stream, ev_scan, 0));
  k_flow_events<<<1024, 256, 0, flow_stream>>>(D, B, FH0, d_ev_off, d_events);
  HIPCHK(hipEventRecord(ev_hot, flow_stream));
  k_ev_scatter<<<2048, T256, 0, s>>>(d_arena, arena_cap, d_st, d_ev_off, d_events);
  HIPCHK(hipStreamWaitEvent(s, ev_hot, 0));
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
  float ms_total = 0, ms_match = 0, ms_hot = 0, ms_flow = 0;
  (void)hipEventElapsedTime(&ms_total, ev0, ev1);
  (void)hipEventElapsedTime(&ms_match, evm0, evm1);
  (void)hipEventElapsedTime(&ms_hot, evh0, evh1);
  (void)hipEventElapsedTime(&ms_flow, evf0, evf1);
  stats.ms_hot = ms_hot;
  stats.ms_flow_plan = ms_flow;
  stats.n_flow_books = st.ctr[C_FLOW_BOOKS];
  stats.n_flow_orders = st.ctr[C_FLOW_ORDERS];
  stats.n_flow_touches = st.ctr[C_FLOW_TOUCHES];
  stats.n_flow_head_orders = st.ctr[C_FLOW_HEAD_ORDERS];
  stats.n_flow_head_touches = st.ctr[C_FLOW_HEAD_TOUCHES];
  stats.n_hot = st.nhot;
  stats.n_hot_orders = st.ctr[C_HOT_ORDERS];
  stats.n_hot_fills = st.ctr[C_HOT_FILLS];
  stats.n_hot_rests = st.ctr[C_HOT_RESTS];
  stats.n_hot_cancels = st.ctr[C_HOT_CANCELS];
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

#ifdef GOME_STAMPS
// Diagnostic builds only: per-hot-wave phase cycle sums (see match_hot.h).
int gome_debug_stamps(unsigned long long* out, size_t n) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gome::g_stamps), std::min<size_t>(n, 256 * NSTAMP) * 8, 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (n <= 256 * NSTAMP) return 0;  // then the plan stamps of the head books
  return hipMemcpyFromSymbol(out + 256 * NSTAMP, HIP_SYMBOL(gome::g_pstamps),
                             std::min<size_t>(n - 256 * NSTAMP, gome::FL_HEAD * 4) * 8, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

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
      Node nd[CH];
      ChunkHdr hd;
      if (hipMemcpy(nd, e->D.nodes + static_cast<size_t>(cid) * CH, sizeof nd, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(&hd, e->D.chdr + cid, sizeof hd, hipMemcpyDeviceToHost) != hipSuccess)
        return e->fail(GOME_E_DEVICE, "snapshot copy failed");
      uint32_t lo = firstc ? L.hslot : 0, hi = (cid == L.tail) ? L.tslot : CH;
      for (uint32_t sl = lo; sl < hi; ++sl) {
        if (nd[sl].rem < 0) continue;
        if (c < cap) {
          std::memset(&out[c], 0, sizeof(gome_node));
          out[c].volume_fx = nd[sl].rem;
          out[c].oid_id = nd[sl].oid;
          out[c].uuid_id = nd[sl].uuid;
          out[c].side = nd[sl].tx;
        }
        ++c;
      }
      firstc = false;
      cid = (cid == L.tail) ? NIL : hd.next;
    }
  }
  *n_out = c;
  return GOME_OK;
}

}  // extern "C"
