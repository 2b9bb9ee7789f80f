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
//   k_scan_* + k_publish      event compaction into publish order (taker_seq, fill_idx)
//   k_recycle         freed FIFO chunks back to the free pool
//
// Everything is integer / byte work (no MFMA).  See DESIGN.md for layout and rooflines.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <set>
#include <thread>
#include <unordered_set>
#include <string>
#include <vector>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "match_cold.h"
#include "match_flow.h"
#include "match_flow_cancel.h"
#include "match_flow_deep.h"
#include "match_early.h"
#include "match_hot.h"
#include "match_requal.h"
#include "pipeline.h"
#include "wave.h"

using namespace gome;

// ============================================================== event compaction
// Arena events -> publish positions; the sequence number is seq_base + the batch index
// (gome_event.taker_seq: its low 32 bits).  Three lanes per 48-B event, 16 B each (a wave moves 21
// events: 1008 B of the arena per load instruction, each event written as whole 16-B pieces); part
// 1 holds taker_seq (.z) and fill_idx (.w).
__device__ __forceinline__ void ev_scatter(const gome_event* arena, uint32_t cap, const Status* st,
                                           const uint32_t* ev_off, gome_event* out, unsigned long long seq_base,
                                           uint32_t bid, uint32_t nblk) {
  const uint32_t used = min(st->ev_bump, cap);
  const uint32_t lane = lane_id(), part = lane % 3u, src = lane - part + 1u;
  const uint32_t waves = (nblk * blockDim.x) >> 6;
  const uint4* ain = reinterpret_cast<const uint4*>(arena);
  uint4* dst = reinterpret_cast<uint4*>(out);
  for (uint32_t w = (bid * blockDim.x + threadIdx.x) >> 6;; w += waves) {
    const uint32_t j0 = w * 21u;
    if (j0 >= used) break;  // (wave-uniform)
    const uint32_t j = j0 + lane / 3u;
    const bool ok = lane < 63u && j < used;
    uint4 v = ok ? ain[3ull * j + part] : make_uint4(0u, 0u, NIL, 0u);
    const uint32_t idx = __shfl(v.z, static_cast<int>(min(src, 63u)));  // taker_seq
    const uint32_t fi = __shfl(v.w, static_cast<int>(min(src, 63u)));   // fill_idx
    if (!ok || idx == NIL) continue;
    if (part == 1) v.z = static_cast<uint32_t>(seq_base + idx);
    dst[3ull * (ev_off[idx] + fi) + part] = v;
  }
}
static_assert(offsetof(gome_event, taker_seq) == 24 && offsetof(gome_event, fill_idx) == 28 &&
              sizeof(gome_event) == 48, "ev_scatter's parts");

// After the publish-order scan, in one launch (no hop to a second stream and back): blocks
// [0, nscat) place the arena's events, the rest write the hottest book's events (fl_events_hot).
constexpr uint32_t PUB_SCAT = 2048, PUB_HOT = 1024;
__global__ __launch_bounds__(256) void k_publish(Dev D, BatchArgs B, FlowArgs F, const gome_event* arena,
                                                 uint32_t cap, const uint32_t* ev_off, gome_event* out,
                                                 unsigned long long seq_base) {
  if (blockIdx.x < PUB_SCAT) ev_scatter(arena, cap, D.st, ev_off, out, seq_base, blockIdx.x, PUB_SCAT);
  else fl_events_hot(D, B, F, ev_off, out, blockIdx.x - PUB_SCAT, gridDim.x - PUB_SCAT);
}

// Freed FIFO chunks of this batch -> free pool (two kernels: copy, then counters).
// The stream-layout probe (four hardware queues): a ~2 ms spin on one stream, an empty kernel on the
// other; the empty one finishing late means the two streams share a hardware queue.
__global__ void k_probe_spin(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) {
  }
}
__global__ void k_probe_nop() {}

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

// Level blocks released this batch -> their class's free stack (block c = class c).
// The slot's segmentation results into the batch's Status (after its per-batch reset).
__global__ void k_sort_status(Status* st, const Status* sst) {
  st->nseg = sst->nseg;
  st->nhot = sst->nhot;
  st->ctr[C_MAXSEG] = sst->ctr[C_MAXSEG];
}

// Batch end: the striped counters (ctr_add) into Status::ctr, the stripes zeroed for the next batch.
__global__ void k_ctr_fold(Dev D) {
  const uint32_t c = threadIdx.x;
  if (c >= C_NCTR) return;
  unsigned long long v = 0;
  for (uint32_t k = 0; k < CTR_STRIPES; ++k) {
    v += D.ctr_s[k * CTR_STRIDE + c];
    D.ctr_s[k * CTR_STRIDE + c] = 0;
  }
  D.st->ctr[c] += v;
#ifdef GOME_PROBE_LEVEL
  if (c == 0) {
    printf("PROBE levels %llu t12 %llu t3 %llu walk %llu max %llu cnt %llu slow %llu maxcnt %llu | waves %llu wsum %llu wmax %llu w>10us %llu span %llu\n",
           g_probe[2], g_probe[0], g_probe[1], g_probe[3], g_probe[4], g_probe[5], g_probe[6], g_probe[7], g_probe[8],
           g_probe[9], g_probe[10], g_probe[11], g_probe[13] - g_probe[12]);
    printf("PROBE prep_b old %llu gcd %llu rank %llu hdr %llu | rank: minmax %llu gcd %llu bits %llu scan %llu put %llu\n",
           g_probe[16], g_probe[17], g_probe[18], g_probe[19], g_probe[20], g_probe[21], g_probe[22], g_probe[23], g_probe[24]);
    for (int k = 0; k < 32; ++k) g_probe[k] = 0;
    g_probe[12] = ~0ull;
  }
#endif
}

__global__ __launch_bounds__(256) void k_lvl_recycle(Dev D) {
  const uint32_t c = blockIdx.x;
  const int top = max(D.st->lvl_free_top[c], 0);
  const uint32_t off = D.lvl_cls_off[c], room = D.lvl_cls_off[c + 1] - off;
  const uint32_t nf = min(D.st->lvl_freed_top[c], room - min(room, static_cast<uint32_t>(top)));
  for (uint32_t i = threadIdx.x; i < nf; i += blockDim.x) D.lvl_free[off + top + i] = D.lvl_freed[off + i];
  __syncthreads();
  if (threadIdx.x == 0) {
    D.st->lvl_free_top[c] = top + static_cast<int>(nf);
    D.st->lvl_freed_top[c] = 0;
    if (c == 0) {
      D.st->lvl_used = min(*D.lvl_bump, D.lvl_cap_total);
      D.st->ch_used = min(*D.ch_bump, D.ch_cap);
    }
  }
}

// Rebuild the (S, oid) cancel index from the live FIFO nodes (the table was zeroed): bounds
// the probe length of lookups that miss (a cancel of a filled or unknown oid scans to the
// first EMPTY slot, and erases only leave tombstones).  One wave per book, a lane per slot.
// One wave per (symbol, level): the hottest book's FIFOs hold millions of nodes, so its levels
// are walked side by side (blockIdx.y strides over a book's levels).
__global__ __launch_bounds__(64) void k_idx_rebuild(Dev D) {
  const uint32_t lane = lane_id();
  const unsigned long long mask = D.idx_mask;
  for (uint32_t sym = blockIdx.x; sym < D.max_symbols; sym += gridDim.x) {
    const Book bk = D.books[sym];
    const Level* L = D.lvl + bk.lvl_base;
    for (uint32_t k = blockIdx.y; k < bk.n_lvl; k += gridDim.y) {
      const Level x = L[k];
      uint32_t c = x.head, s0 = x.hslot;
      for (uint32_t guard = 0; c != NIL && guard <= D.ch_cap; ++guard) {
        const uint32_t lim = (c == x.tail) ? x.tslot : CH;
        if (lane < CH && lane >= s0 && lane < lim) {
          Node* nd = &D.nodes[c * CH + lane];
          if (nd->rem >= 0) {
            const unsigned long long key = (static_cast<unsigned long long>(sym + 1) << 32) | nd->oid;
            unsigned long long hh = mix64(key) & mask;
            for (unsigned long long probe = 0; probe <= mask; ++probe, hh = (hh + 1) & mask)
              if (atomicCAS(&D.idx[hh].key, KEY_EMPTY, key) == KEY_EMPTY) break;
            D.idx[hh].loc = c * CH + lane;
            nd->ixs = static_cast<uint32_t>(hh);
          }
        }
        c = (c == x.tail) ? NIL : D.chdr[c].next;
        s0 = 0;
      }
    }
  }
}

// Top-of-book digests (the publisher's depth summary): per requested symbol, the
// best bid (highest S:BUY member) and best ask (lowest S:SALE member) with their S:depth fields
// and FIFO lengths, as GetReverseDepth's first level would report them (nodepool.go:86-115).
// A thread per symbol walks the book's sorted level block.
__global__ void k_tob(Dev D, const uint32_t* syms, uint32_t n, gome_tob* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  gome_tob t{};
  t.symbol_id = syms[i];
  if (t.symbol_id < D.max_symbols) {
    const Book bk = D.books[t.symbol_id];
    const Level* L = D.lvl + bk.lvl_base;
    bool bid = false, ask = false;
    for (uint32_t k = 0; k < bk.n_lvl; ++k) {
      const Level x = L[k];
      if (!x.nlive && !x.depth && !x.member) continue;
      ++t.n_levels;
      if (!ask && (x.member & M_SALE)) {
        ask = true;
        t.ask_price_fx = x.price;
        t.ask_depth_fx = x.depth;
        t.ask_nodes = x.nlive;
      }
      if (x.member & M_BUY) {
        bid = true;
        t.bid_price_fx = x.price;
        t.bid_depth_fx = x.depth;
        t.bid_nodes = x.nlive;
      }
    }
    t.flags = (bid ? 1u : 0u) | (ask ? 2u : 0u);
  }
  out[i] = t;
}

// ============================================================== host runtime
namespace {

thread_local std::string g_create_err;

constexpr uint32_t QUIRK_CAP = 1u << 16;  // quirk books checked per batch (Dev::quirk)

uint32_t ceil_div(uint64_t a, uint64_t b) { return static_cast<uint32_t>((a + b - 1) / b); }
uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// One of the two batch slots: a batch's device records, its published events, its
// status copy and its timing events.  Batch k uses slot k % 2, so batch k+1's H2D and
// batch k-1's D2H never touch the buffers batch k's pipeline works on.
struct Slot {
  gome_order* d_orders = nullptr;
  gome_event* d_events = nullptr;
  uint32_t ev_cap = 0;
  Status* h_st = nullptr;          // page-locked copy of the batch's Status
  gome_event* h_events = nullptr;  // page-locked event copy (gome_collect)
  // async host batches: the event copy, issued by the engine's copy thread the moment the batch
  // is done (gome_engine::d2h_loop); d2h_state: 0 none, 1 queued, 2 issued (d2h recorded), 3 failed
  int d2h_state = 0;
  hipError_t d2h_err = hipSuccess;
  hipEvent_t d2h{};
  uint32_t* d_dup = nullptr;       // batch indices of the ADDs rejected as duplicate oids (Q7)
  size_t h_cap = 0;
  hipEvent_t ev0{}, ev1{}, evm0{}, evm1{}, evh0{}, evh1{}, evf0{}, evf1{}, evc0{}, evc1{};
  hipEvent_t evx0{}, evx1{};  // the early plan (match_early.h), when the batch enqueued one
  bool early = false;
  uint32_t* adm_v = nullptr;  // the batch's verdicts when its admission ran ahead (k_adm_verify)
  hipEvent_t h2d{}, done{};
  hipEvent_t ph[GOME_NPHASE][2]{};  // GOME_PH_* phase brackets (ph_on: recorded this batch)
  bool ph_on[GOME_NPHASE]{};
  double ms_enqueue = 0;  // host wall time of enqueue()
  uint32_t chains = 0;    // the flow chains (FL_CH_*) the batch enqueued
  // the batch's radix sort and segments (per slot: with two batches in flight the next
  // batch's sort runs during this one's hottest plan, see enqueue)
  uint32_t *k0 = nullptr, *v0 = nullptr, *k1 = nullptr, *v1 = nullptr, *hist = nullptr, *bsum = nullptr;
  uint32_t* tmp = nullptr;        // flags / segpos (n)
  uint32_t* seg_start = nullptr;
  uint32_t* seg_order = nullptr;
  uint32_t* bcnt = nullptr;       // 32 counts + 32 offsets
  Status* sst = nullptr;          // the segmentation's nseg / nhot / C_MAXSEG, copied to Status by k_sort_status
};

struct Flight {
  uint32_t slot, n;
  uint64_t seq_base;
  bool dev;  // records in the caller's HBM (gome_submit_batch_device_async)
};

}  // namespace

struct gome_engine {
  gome_config cfg{};
  hipStream_t stream = nullptr;       // the pipeline's main stream
  hipStream_t hot_stream = nullptr;   // tail / near-head flow books, legacy hot kernel
  hipStream_t flow_stream = nullptr;  // the hottest book's plan (critical path)
  hipStream_t copy_stream = nullptr;  // H2D of records, D2H of events (pipelined path)
  hipStream_t early_stream = nullptr; // the early plan's record work (match_early.h), beside the plan before it
  hipStream_t d2h_stream = nullptr;   // event copies (gome_collect), beside the next batch's H2D and pipeline
  hipStream_t h2d_stream = nullptr;   // async host batches' record copies: nothing else on it, so the next
                                      // batch's H2D never waits behind this batch's work
  // The hottest book's plans on a stream of their own restricted to CUs [0, k), every other engine
  // stream to the rest: the plan wave alone with its CU's instruction cache and L1, and no other
  // kernel's code or data beside it (gome_config.plan_cus, default 8; none below 8 queues)
  hipStream_t plan_stream = nullptr;
  hipEvent_t pl_fork{}, pl_join{};
  uint32_t plan_cus = 0;
  uint32_t hw_queues = 4;  // the process's hardware queues (gome_config.hw_queues; layout)
  std::vector<uint32_t> cu_rest;  // every CU but the plan's
  hipError_t new_stream(hipStream_t* st) {
    return plan_cus ? hipExtStreamCreateWithCUMask(st, static_cast<uint32_t>(cu_rest.size()), cu_rest.data())
                    : hipStreamCreateWithFlags(st, hipStreamNonBlocking);
  }
  // Whether stream b waits for work on stream a: they share a hardware queue (tools/queue_map.hip).
  hipError_t shares_queue(hipStream_t a, hipStream_t b, bool* shared) {
    int khz = 0;
    hipError_t he = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, cfg.device);
    hipEvent_t ev{};
    if (he == hipSuccess) he = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (he == hipSuccess) he = hipStreamSynchronize(a);
    if (he == hipSuccess) he = hipStreamSynchronize(b);
    if (he != hipSuccess) return he;
    k_probe_spin<<<1, 64, 0, a>>>(2ull * static_cast<unsigned long long>(khz));  // (~2 ms)
    k_probe_nop<<<1, 64, 0, b>>>();
    he = hipEventRecord(ev, b);
    const auto t0 = std::chrono::steady_clock::now();
    if (he == hipSuccess) he = hipEventSynchronize(ev);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const hipError_t h2 = hipStreamSynchronize(a);
    (void)hipEventDestroy(ev);
    *shared = ms > 1.0;
    return he != hipSuccess ? he : h2;
  }
  // Four hardware queues: a stream for the early plan whose queue is none of the caller's, flow and
  // hot streams'.  HIP hands queues to new streams by how many streams each already carries, so which
  // stream gets which queue depends on what the host created before the engine (torch's null-stream
  // work, RCCL's streams): the first of up to 6 new streams the probe finds alone is the early stream,
  // the others become the copy streams (work only on the host path).  None alone: the last one
  // (exact either way; only slower).  Round 6's first 4-queue layout relied on creation order and
  // its early plan shared the hot stream's queue under torch: 99M orders/s instead of 146.6M.
  hipError_t q4_early_stream() {
    std::vector<hipStream_t> spare;
    for (int k = 0; k < 6 && !early_stream; ++k) {
      hipStream_t c{};
      hipError_t he = new_stream(&c);
      if (he != hipSuccess) return he;
      bool any = false;
      for (hipStream_t x : {stream, flow_stream, hot_stream}) {
        bool sh = false;
        if ((he = shares_queue(x, c, &sh)) != hipSuccess) return he;
        any = any || sh;
      }
      if (any) spare.push_back(c);
      else early_stream = c;
    }
    if (!early_stream) {
      early_stream = spare.back();
      spare.pop_back();
    }
    for (hipStream_t* st : {&copy_stream, &d2h_stream, &h2d_stream}) {
      if (spare.empty()) break;
      *st = spare.back();
      spare.pop_back();
    }
    for (hipStream_t c : spare) (void)hipStreamDestroy(c);
    return hipSuccess;
  }
  // The engine's streams on every CU, for batches after one no book dominated: there the tail's
  // chain is the critical path, and on the masked queues config 2 ran 5% slower.  set_masked
  // swaps the two sets (the new streams wait for the old ones' work first).
  static constexpr int NSET = 5;
  hipStream_t alt[NSET]{};
  hipEvent_t sw_ev[NSET]{};
  bool masked = false, alt_made = false;
  hipStream_t* live_streams(int i) {
    hipStream_t* v[NSET] = {&stream, &hot_stream, &flow_stream, &copy_stream, &early_stream};
    return v[i];
  }
  hipError_t make_sets() {
    masked = plan_cus != 0;
    return hipSuccess;
  }
  hipError_t set_masked(bool want) {
    if (!plan_cus || want == masked) return hipSuccess;
    // (the other set on first use: idle streams still take hardware queues, which RCCL and torch
    // need too; with both sets made up front the RCCL line lost 5%)
    for (int i = 0; i < NSET && !alt_made; ++i) {
      if (!*live_streams(i)) continue;
      hipError_t he = hipStreamCreateWithFlags(&alt[i], hipStreamNonBlocking);
      if (he == hipSuccess) he = hipEventCreateWithFlags(&sw_ev[i], hipEventDisableTiming);
      if (he != hipSuccess) return he;
    }
    alt_made = true;
    for (int i = 0; i < NSET; ++i) {
      hipStream_t* cur = live_streams(i);
      if (!*cur) continue;
      hipError_t he = hipEventRecord(sw_ev[i], *cur);
      if (he == hipSuccess) he = hipStreamWaitEvent(alt[i], sw_ev[i], 0);
      if (he != hipSuccess) return he;
      std::swap(*cur, alt[i]);
    }
    masked = want;
    ++n_set_switch;
    return hipSuccess;
  }
  uint64_t n_set_switch = 0;
  // before a batch's first stream use: the masked set while the last finished batch had a
  // dominant book (enqueue's `dominant`), every CU otherwise
  gome_status pick_streams() {
    const hipError_t he = set_masked(!(last_maxseg * 16 < last_n));
    return he == hipSuccess ? GOME_OK : fail(GOME_E_DEVICE, hipGetErrorString(he));
  }
  hipEvent_t fork{}, join{}, joinf{}, prep_h{}, prep_t{}, fork_adm{}, adm_done{}, seg_done{};
  hipEvent_t ho_fork{};  // the hottest book's post-plan checks done (its hand-over kernels fork there)
  hipEvent_t tfc_fork{}, tfc_done{};  // the tail's sort done / its cancel books' level pass done
  hipEvent_t sort_done{};  // a batch's radix sort and segments, sorted ahead on the copy stream
  hipEvent_t dp_fork{}, cnt_fork{}, cnt_done{}, dw_done{}, dl_done{}, tl_done{};  // the hottest book's deep chain, k_flow_count beside its writes
  // the early plan of the hottest book (match_early.h): the last batch's plan done (flow stream),
  // its oid watermarks folded (hot stream), this batch's early prep and plan done (copy stream)
  hipEvent_t plan_done{}, oidmax_done{}, xpre_done{}, xprep_done{}, xplan_done{};
  hipEvent_t xcmp_done{};  // k_x_cmp done (flow stream)
  // the last enqueued batch's final F.hdr[0] / F.lvl writers (its plan, or its early plan's k_x_take and
  // the fallback plan behind it) ran on the plan stream: the next early chain there needs no plan_done
  // (device batches only)
  bool f_on_plan = false;
  struct XBuf {
    XCtl* ctl = nullptr;
    FlowHdr* hdr = nullptr;
    FlowLvl* lvl = nullptr;
    unsigned long long* ord8 = nullptr;
    Touch* log = nullptr;
    FlowLvl* dlvl = nullptr;       // deep books' level table (DEEP_CAP)
  } xb[2];                         // by batch parity (the next batch's chain runs beside this one's take)
  FlPrepScr* x_pscr = nullptr;
  uint32_t *x_adm = nullptr, *x_evc = nullptr;  // predicted verdicts; the early prep_c's ev_count sink
  uint32_t *x_cnt = nullptr, *x_seg = nullptr, *x_sidx = nullptr;  // the hot symbol's records (k_x_*)
  FlPrepScr* x_dscr = nullptr;                 // deep books: prep scratch, price set, sorted prices
  unsigned long long *x_dkey = nullptr, *x_dnew = nullptr;
  uint32_t *x_dval = nullptr, *x_dslot = nullptr;
  XComp* x_comp = nullptr;  // the early lane plan's records, gathered before the last plan's end
  bool early_on = true;            // (GOME_FLAG_NO_EARLY: never)
  // pipelined device batches of a dominated stream that plan late: admission ahead, on the early
  // stream beside the last batch's plan (k_adm_verify; GOME_FLAG_NO_ADM_AHEAD: never)
  bool adm_ahead_on = true;
  hipEvent_t adm_pre_done{};
  Status* d_adm_st = nullptr;      // the ahead pass's input errors
  uint32_t* d_adm_redo = nullptr;  // k_adm_verify: the batch's own admission runs again
  uint32_t head_add = 0;           // bit 0 / 1: the last / the one before finished batch's hottest book took an ADD plan
  uint32_t bid = 0;                // batches enqueued (FlowArgs::bid)
  Slot slots[GOME_MAX_INFLIGHT];
  uint32_t next_slot = 0;
  std::deque<Flight> flights;
  FlowArgs F{};
  Prep* d_prep = nullptr;
  PendEnt* d_pend = nullptr;
  ResumeRec* d_resume = nullptr;
  Dev D{};
  Status* d_st = nullptr;
  // capacities
  uint32_t max_batch = 0, key_bits = 1, passes = 1, dbits = 1;
  // blocks of the tail's per-touch kernels (4096 measured 5% faster than 1024 on config 2)
  static constexpr uint32_t tail_grid = 4096;
  bool cold_main = false;  // k_match on the caller's stream (fewer than 8 hardware queues; default: the copy stream)
  bool q4 = false;         // 4 to 7 hardware queues: cold_main, and the early plan on a fourth stream
  bool copy_busy = false;  // the batch being enqueued came by gome_submit_batch_async (H2D / D2H on the copy stream)
  // GOME_PH_* timing events (gome_stats.ms_phase): ~24 event records per batch, 0.12 ms on config 2's
  // critical path, so only on request (GOME_FLAG_PHASES)
  bool phases = false;
  uint64_t last_maxseg = 0, last_n = 0;  // the last finished batch's hottest book / size
  uint32_t hist_cap = 0, bsum_cap = 0;
  unsigned long long idx_cap = 0;
  // batch buffers (the sort's and the segments' are per slot: Slot)
  uint32_t* d_bsum = nullptr;
  unsigned long long* d_adm = nullptr;  // admission table (k_adm)
  unsigned long long* d_dup = nullptr;  // (S, uuid, oid) table of the records whose (S, oid) repeats
  uint8_t* d_multi = nullptr;           // per (S, oid) slot: the key repeats in the batch
  uint32_t* d_first = nullptr;          // per (S, oid) slot: its first admitted ADD (NIL between batches)
  uint32_t *d_adm_slot2 = nullptr, *d_adm_aux = nullptr;  // per record: (S, uuid, oid) / (S, oid) slot
  uint32_t* d_oid_max = nullptr;        // per symbol: the highest oid an admitted ADD carried
  uint32_t* d_adm_ctl = nullptr;        // k_adm_ctl / k_adm_pre: oid watermark, not-fresh flag, batch max oid
  uint32_t oid_gmax_load = 0;           // (gome_load_books' copy source)
  uint32_t* d_adm_slot = nullptr;
  uint32_t adm_mask = 0;
  uint32_t* d_ev_count = nullptr;
  uint32_t* d_ev_off = nullptr;
  gome_event* d_arena = nullptr;
  uint32_t arena_cap = 0;
  // host-side state
  std::vector<gome_event> pending;
  std::vector<uint32_t> dup_idx;  // the last finished batch's duplicate-oid rejections (sorted)
  uint32_t* d_tob_syms = nullptr;  // gome_top_of_book's device buffers
  gome_tob* d_tob = nullptr;
  size_t tob_cap = 0;
  // gome_top_of_book_enqueue: page-locked staging (symbols in, digests out), its completion event
  uint32_t* h_tob_syms = nullptr;
  gome_tob* h_tob = nullptr;
  size_t h_tob_cap = 0, tob_pending = 0;
  bool tob_queued = false;
  hipEvent_t tob_done{};
  gome_status tob_buffers(size_t n);
  size_t pending_pos = 0;
  size_t dev_events = 0, dev_events_pos = 0;  // events of the last device submit
  uint32_t dev_slot = 0;
  gome_stats stats{};
  unsigned long long resting = 0, levels = 0;
  unsigned long long idx_tomb = 0, n_rebuilds = 0;  // tombstones (upper bound) since the last rebuild
  uint32_t fc_gen = 0;            // batch generation of the cancel books' (symbol, oid) table
  static constexpr uint32_t plan_lds = FL_DEEP_LDS;  // dynamic LDS of the head / deep plans
  unsigned long long fc_hcap = 0;  // its entries
  bool poisoned = false;
  std::string err;
  gome_status deferred = GOME_OK;  // an in-flight batch's failure collected by a synchronous call
  std::string deferred_msg;
  std::vector<void*> allocs;
  std::set<void*> host_allocs;

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
    // Every buffer starts zeroed (defence: the allocator hands memory back as an earlier engine in
    // the process left it).  No kernel may depend on it: a buffer a batch reads is written first,
    // by a per-batch reset or by init's own memsets.  GOME_FLAG_POISON (test hosts) fills 0xA5
    // instead, so a read of scratch nobody wrote shows as an out-of-range value.  (Round 5's fault,
    // the deep level pass read its sentinel row 0, which no prep wrote.)
    // The fill goes on the engine's own stream, ahead of init's explicit memsets and copies on it:
    // a plain hipMemset runs on the legacy null stream, which the engine's non-blocking streams do
    // not wait for, so it could land after them (round 6: a 0xA5 fill over the zeroed headers
    // faulted; a zero fill can clobber d_first / dh_val's 0xFF and the level-class table).
    if (hipMemsetAsync(q, (cfg.flags & GOME_FLAG_POISON) ? 0xA5 : 0, bytes, stream) != hipSuccess) {
      (void)hipFree(q);
      err = std::string("hipMemset failed for ") + what;
      return false;
    }
    allocs.push_back(q);
    *p = static_cast<T*>(q);
    return true;
  }
  void release(void* p) {
    for (auto it = allocs.begin(); it != allocs.end(); ++it)
      if (*it == p) { (void)hipFree(p); allocs.erase(it); return; }
  }
  ~gome_engine() {
    if (d2h_thr.joinable()) {
      {
        std::lock_guard<std::mutex> lk(d2h_mu);
        d2h_stop = true;
      }
      d2h_cv.notify_all();
      d2h_thr.join();
    }
    if (stream) (void)hipStreamSynchronize(stream);
    if (copy_stream) (void)hipStreamSynchronize(copy_stream);
    if (early_stream) (void)hipStreamSynchronize(early_stream);
    if (d2h_stream) (void)hipStreamSynchronize(d2h_stream);
    if (h2d_stream) (void)hipStreamSynchronize(h2d_stream);
    for (void* p : allocs) (void)hipFree(p);
    for (void* p : host_allocs) (void)hipHostFree(p);
    for (Slot& S : slots) {
      if (S.h_st) (void)hipHostFree(S.h_st);
      if (S.h_events) (void)hipHostFree(S.h_events);
      for (hipEvent_t ev : {S.ev0, S.ev1, S.evm0, S.evm1, S.evh0, S.evh1, S.evf0, S.evf1, S.evc0, S.evc1, S.h2d, S.done,
                            S.evx0, S.evx1, S.d2h})
        if (ev) (void)hipEventDestroy(ev);
      for (auto& pr : S.ph)
        for (hipEvent_t ev : pr)
          if (ev) (void)hipEventDestroy(ev);
    }
    for (hipEvent_t ev : {fork, join, joinf, prep_h, prep_t, fork_adm, adm_done, seg_done, ho_fork, tfc_fork, tfc_done, sort_done, dp_fork, cnt_fork, cnt_done,
                          dw_done, dl_done, tl_done, tob_done, plan_done, oidmax_done, xpre_done, xprep_done,
                          xplan_done, xcmp_done, adm_pre_done})
      if (ev) (void)hipEventDestroy(ev);
    if (h_tob_syms) (void)hipHostFree(h_tob_syms);
    if (h_tob) (void)hipHostFree(h_tob);
    if (hot_stream) (void)hipStreamDestroy(hot_stream);
    if (plan_stream) (void)hipStreamDestroy(plan_stream);
    for (int i = 0; i < NSET; ++i) {
      if (alt[i]) (void)hipStreamDestroy(alt[i]);
      if (sw_ev[i]) (void)hipEventDestroy(sw_ev[i]);
    }
    if (pl_fork) (void)hipEventDestroy(pl_fork);
    if (pl_join) (void)hipEventDestroy(pl_join);
    if (flow_stream) (void)hipStreamDestroy(flow_stream);
    if (copy_stream) (void)hipStreamDestroy(copy_stream);
    if (d2h_stream) (void)hipStreamDestroy(d2h_stream);
    if (h2d_stream) (void)hipStreamDestroy(h2d_stream);
    if (early_stream) (void)hipStreamDestroy(early_stream);
    if (stream) (void)hipStreamDestroy(stream);
  }

  gome_status init(const gome_config& c);
  void scan(const uint32_t* in, uint32_t m, uint32_t* out, uint32_t* total, hipStream_t s, uint32_t* bsum = nullptr);
  gome_status enqueue(const gome_order* d_ord, uint32_t n, hipStream_t s, uint32_t slot, uint64_t seq_base,
                      uint64_t inflight_n, bool ahead = false);
  gome_status finish(uint32_t slot, uint32_t n);
  gome_status check_submit(size_t n, const void* p);
  gome_status load_books(size_t nb, const uint32_t* bsym, const uint32_t* bnlv, const gome_level* lv,
                         const gome_node* nd, size_t nn);
  bool used = false;  // a batch was submitted or books were loaded (gome_load_books needs a fresh engine)
  // finished batches in a row whose flow candidates asked for no deep / cancel chain
  uint32_t deep_quiet = 0, canc_quiet = 0;
  uint32_t pick_chains() const {
    if (cfg.flags & GOME_FLAG_CHAINS_NEVER) return 0u;
    const bool all = (cfg.flags & GOME_FLAG_CHAINS_ALWAYS) != 0;
    return ((all || deep_quiet < GOME_CHAIN_QUIET) ? FL_CH_DEEP : 0u) |
           ((all || canc_quiet < GOME_CHAIN_QUIET) ? FL_CH_CANCEL : 0u);
  }
  gome_status check_capacity(unsigned long long adds, unsigned long long inflight_n);
  gome_status check_capacity_host(const gome_order* o, size_t n, unsigned long long inflight_n);
  uint32_t take_slot() {
    const uint32_t k = next_slot;
    next_slot = (next_slot + 1) % GOME_MAX_INFLIGHT;
    return k;
  }
  gome_status collect(const gome_event** evs, size_t* nev);
  // The copy thread: async host batches' event copies, issued the moment each batch is done (its
  // count is known then), so they run beside the next batch's H2D and pipeline instead of waiting
  // for gome_collect.  (Round 5, config 2 e2e: a copy issued at submit behind a wait on the batch
  // held the copy engine and the next H2D behind it, 8.2 ms a step; a kernel writing the events to
  // mapped host memory slowed the next batch's pipeline 2.4x; a copy issued at gome_collect kept
  // the host from the next submit for its whole length, 5.2 ms.)
  std::thread d2h_thr;
  std::mutex d2h_mu;
  std::condition_variable d2h_cv;
  std::deque<uint32_t> d2h_q;
  bool d2h_stop = false;
  void d2h_queue(uint32_t sl) {
    {
      std::lock_guard<std::mutex> lk(d2h_mu);
      if (!d2h_thr.joinable()) d2h_thr = std::thread([this] { d2h_loop(); });
      slots[sl].d2h_state = 1;
      d2h_q.push_back(sl);
    }
    d2h_cv.notify_all();
  }
  void d2h_loop() {
    (void)hipSetDevice(cfg.device);
    for (;;) {
      uint32_t sl;
      {
        std::unique_lock<std::mutex> lk(d2h_mu);
        d2h_cv.wait(lk, [&] { return d2h_stop || !d2h_q.empty(); });
        if (d2h_q.empty()) return;  // (stop, nothing queued)
        sl = d2h_q.front();
        d2h_q.pop_front();
      }
      Slot& S = slots[sl];
      hipError_t he = hipEventSynchronize(S.done);
      const size_t n = he == hipSuccess ? S.h_st->n_events : 0;
      if (he == hipSuccess && n > S.h_cap) {  // (the caller touches the buffer only after state 2)
        if (S.h_events) (void)hipHostFree(S.h_events);
        S.h_events = nullptr;
        S.h_cap = 0;
        he = hipHostMalloc(reinterpret_cast<void**>(&S.h_events), (n + n / 4 + 1024) * sizeof(gome_event),
                           hipHostMallocDefault);
        if (he == hipSuccess) S.h_cap = n + n / 4 + 1024;
      }
      if (he == hipSuccess && n)
        he = hipMemcpyAsync(S.h_events, S.d_events, n * sizeof(gome_event), hipMemcpyDeviceToHost, d2h_stream);
      if (he == hipSuccess) he = hipEventRecord(S.d2h, d2h_stream);
      {
        std::lock_guard<std::mutex> lk(d2h_mu);
        S.d2h_err = he;
        S.d2h_state = he == hipSuccess ? 2 : 3;
      }
      d2h_cv.notify_all();
    }
  }
  // slot S's page-locked event buffer with room for `cap` events (none in flight)
  gome_status host_events(Slot& S, size_t cap) {
    if (S.h_events) (void)hipHostFree(S.h_events);
    S.h_events = nullptr;
    S.h_cap = 0;
    hipError_t he = hipHostMalloc(reinterpret_cast<void**>(&S.h_events), cap * sizeof(gome_event), hipHostMallocDefault);
    if (he != hipSuccess) return fail(GOME_E_DEVICE, std::string("event buffer: ") + hipGetErrorString(he));
    S.h_cap = cap;
    return GOME_OK;
  }
  gome_status collect_all();
  gome_status spill_device_events();
  gome_status queue_events(uint32_t slot, size_t n, hipStream_t s);
};

#define HIPCHK_E(e, x)                                                               \
  do {                                                                               \
    hipError_t _e = (x);                                                             \
    if (_e != hipSuccess)                                                            \
      return (e)->fail(GOME_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

#define HIPCHK(x)                                                                    \
  do {                                                                               \
    hipError_t _e = (x);                                                             \
    if (_e != hipSuccess)                                                            \
      return fail(GOME_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e));    \
  } while (0)

// GPU_MAX_HW_QUEUES as set now (HIP's default 4 if unset or not a number): the layout's fallback
// when the host does not say how many queues its runtime started with (gome_config.hw_queues)
static uint32_t env_hw_queues() {
  const char* q = std::getenv("GPU_MAX_HW_QUEUES");
  if (!q || !*q) return 4;
  char* end = nullptr;
  const long v = std::strtol(q, &end, 10);
  return (end && *end == 0 && v > 0 && v < 1024) ? static_cast<uint32_t>(v) : 4u;
}

gome_status gome_engine::init(const gome_config& c) {
  cfg = c;
  if (cfg.abi_version != GOME_ABI_VERSION)
    return fail(GOME_E_INVAL, "gome_config.abi_version is " + std::to_string(cfg.abi_version) +
                                  ", this library is ABI " + std::to_string(GOME_ABI_VERSION) +
                                  " (rebuild the caller against include/gome/gome_abi.h)");
  if (cfg.accuracy == 0) cfg.accuracy = 8;
  if (!cfg.max_symbols || !cfg.max_batch || !cfg.max_nodes || !cfg.max_levels)
    return fail(GOME_E_INVAL, "gome_config: max_symbols, max_batch, max_nodes, max_levels must be > 0");
  // (max_batch <= 2^28 keeps the admission tables' slots below 2^30: k_adm flags bit 31)
  if (cfg.max_batch > (1u << 28) || cfg.max_levels > 0xF0000000ull)
    return fail(GOME_E_INVAL, "gome_config: capacity out of range");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(GOME_E_DEVICE, "no HIP device available (the engine has no CPU fallback)");
  if (cfg.device < 0 || cfg.device >= ndev) return fail(GOME_E_INVAL, "gome_config.device out of range");
  HIPCHK(hipSetDevice(cfg.device));
  // ---- stream layout: with fewer than 8 hardware queues the engine's streams would
  // share them (the copy stream with the hottest plan's: +6 ms per config-3 batch), so the cold books
  // stay on the caller's stream and there is no early plan, no admission ahead and no plan stream
  hw_queues = cfg.hw_queues ? cfg.hw_queues : env_hw_queues();
  cold_main = hw_queues < 8;
  // four hardware queues (HIP's default, a host that does not raise GPU_MAX_HW_QUEUES): the caller's,
  // flow and hot streams, and the early plan on a fourth stream created right after them, so it
  // takes the fourth queue (streams beyond the count share queues, tools/queue_map.hip; the later
  // copy streams share with these, and carry work only on the host path).  Its record work and the
  // plan go on that one stream, the cold books on the caller's.
  q4 = cold_main && hw_queues >= 4;
  early_on = (!cold_main || q4) && !(cfg.flags & GOME_FLAG_NO_EARLY);
  adm_ahead_on = !cold_main && !(cfg.flags & GOME_FLAG_NO_ADM_AHEAD);
  {
    int ncu = 0;
    HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cfg.device));
    plan_cus = cfg.plan_cus < 0 ? 0u : cfg.plan_cus > 0 ? static_cast<uint32_t>(cfg.plan_cus) : cold_main ? 0u : 8u;
    if (plan_cus >= static_cast<uint32_t>(ncu)) plan_cus = 0;
    const uint32_t words = (static_cast<uint32_t>(ncu) + 31) / 32;
    cu_rest.assign(words, 0u);
    std::vector<uint32_t> cu_plan(words, 0u);
    for (uint32_t c = 0; c < static_cast<uint32_t>(ncu); ++c) (c < plan_cus ? cu_plan : cu_rest)[c / 32] |= 1u << (c % 32);
    if (plan_cus) {
      HIPCHK(hipExtStreamCreateWithCUMask(&plan_stream, words, cu_plan.data()));
      HIPCHK(hipEventCreateWithFlags(&pl_fork, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&pl_join, hipEventDisableTiming));
    }
  }
  HIPCHK(new_stream(&stream));
  if (q4) {
    HIPCHK(new_stream(&flow_stream));
    HIPCHK(new_stream(&hot_stream));
    if (early_on) HIPCHK(q4_early_stream());
  } else {
    HIPCHK(new_stream(&hot_stream));
    HIPCHK(new_stream(&flow_stream));
  }
  for (hipStream_t* st : {&copy_stream, &d2h_stream, &h2d_stream})
    if (!*st) HIPCHK(new_stream(st));
  for (hipEvent_t* ev : {&fork, &join, &joinf, &prep_h, &prep_t, &fork_adm, &adm_done, &seg_done, &ho_fork, &tfc_fork, &tfc_done, &sort_done,
                         &dp_fork, &cnt_fork, &cnt_done, &dw_done, &dl_done, &tl_done, &tob_done, &plan_done,
                         &oidmax_done, &xpre_done, &xprep_done, &xplan_done, &xcmp_done, &adm_pre_done})
    HIPCHK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
  for (Slot& S : slots) {
    for (hipEvent_t* ev : {&S.ev0, &S.ev1, &S.evm0, &S.evm1, &S.evh0, &S.evh1, &S.evf0, &S.evf1, &S.evc0, &S.evc1,
                           &S.evx0, &S.evx1})
      HIPCHK(hipEventCreate(ev));
    for (auto& pr : S.ph)
      for (hipEvent_t& ev : pr) HIPCHK(hipEventCreate(&ev));
    HIPCHK(hipEventCreateWithFlags(&S.h2d, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&S.done, hipEventDisableTiming));
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&S.h_st), sizeof(Status), hipHostMallocDefault));
    HIPCHK(hipEventCreateWithFlags(&S.d2h, hipEventDisableTiming));
  }
  HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_match_hot),
                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(HOT_LDS_BYTES)));
  HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_match),
                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(COLD_LDS_BYTES)));
  // the head plans (and the deep tail plans) hold a deep book's depth slots in LDS
  {
    int lds = 0;
    HIPCHK(hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, cfg.device));
    if (lds < static_cast<int>(FL_DEEP_LDS)) return fail(GOME_E_DEVICE, "device LDS per workgroup below 132 KiB");
    for (const void* k : {reinterpret_cast<const void*>(k_flow_plan_head), reinterpret_cast<const void*>(k_flow_plan_near),
                          reinterpret_cast<const void*>(k_flow_plan_early),
                          reinterpret_cast<const void*>(k_flow_plan_tail_d)})
      HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(plan_lds)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_deep_prep_b), hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(DEEP_CAP * 8)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_xd_sort_new), hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(DEEP_CAP * 8)));
    HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_xd_prep_b), hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(XD_PREP_LDS)));
  }

  max_batch = cfg.max_batch;
  phases = (cfg.flags & GOME_FLAG_PHASES) != 0;
  uint32_t ms = cfg.max_symbols;
  key_bits = (ms <= 1) ? 1 : 32 - __builtin_clz(ms - 1);
  passes = (key_bits + RS_MAXBITS - 1) / RS_MAXBITS;
  dbits = (key_bits + passes - 1) / passes;
  const uint32_t nblk_max = ceil_div(max_batch, RS_TILE);
  hist_cap = (1u << dbits) * nblk_max;
  uint32_t scan_max = std::max(hist_cap, max_batch);
  bsum_cap = ceil_div(scan_max, SCAN_TILE) + 1;

  // ---- persistent book state
  // chunks: every non-empty level holds >= 1 (plus head/tail chunks partly consumed and chunks
  // of tombstones awaiting the head), and every CH resting nodes fill one more: slots for 4x
  // max_nodes plus two chunks per possible level
  const unsigned long long nchunks = std::min<unsigned long long>(
      4 * ((cfg.max_nodes + CH - 1) / CH) + 2 * std::min<unsigned long long>(cfg.max_levels, cfg.max_nodes) + 1024,
      std::min<unsigned long long>(0xF0000000ull, 0xFFFFFFFEull / CH));
  idx_cap = next_pow2(std::max<unsigned long long>(2 * cfg.max_nodes, 1024));
  // level-block free lists: class c (16 << c levels) holds at most max_levels >> (4 + c) blocks
  std::vector<uint32_t> cls_off(LVL_NCLS + 1, 0);
  for (uint32_t k = 0; k < LVL_NCLS; ++k)
    cls_off[k + 1] = cls_off[k] + static_cast<uint32_t>((cfg.max_levels >> (4 + k)) + 1);
  uint32_t* d_cls_off = nullptr;
  if (!alloc(&D.books, ms, "books") || !alloc(&D.lvl, cfg.max_levels, "levels") ||
      !alloc(&D.lvl_bump, 1, "lvl_bump") || !alloc(&D.nodes, nchunks * CH, "chunks") ||
      !alloc(&D.chdr, nchunks, "chunk headers") ||
      !alloc(&D.ch_bump, 1, "ch_bump") || !alloc(&D.free_ids, nchunks, "free_ids") ||
      !alloc(&D.freed_ids, nchunks, "freed_ids") || !alloc(&D.idx, idx_cap, "index") ||
      !alloc(&d_st, 1, "status") || !alloc(&D.lvl_free, cls_off[LVL_NCLS], "level-block free lists") ||
      !alloc(&D.lvl_freed, cls_off[LVL_NCLS], "level-block release lists") ||
      !alloc(&d_cls_off, LVL_NCLS + 1, "level-block classes") ||
      !alloc(&D.ctr_s, CTR_STRIPES * CTR_STRIDE, "counter stripes") ||
      !alloc(&D.quirk, QUIRK_CAP, "quirk book list"))
    return GOME_E_CAPACITY;
  D.quirk_cap = QUIRK_CAP;
  D.lvl_cls_off = d_cls_off;
  D.max_symbols = ms;
  D.lvl_cap_total = static_cast<uint32_t>(cfg.max_levels);
  D.ch_cap = static_cast<uint32_t>(nchunks);
  D.idx_mask = idx_cap - 1;
  D.st = d_st;
  HIPCHK(hipMemcpyAsync(d_cls_off, cls_off.data(), cls_off.size() * 4, hipMemcpyHostToDevice, stream));
  HIPCHK(hipMemsetAsync(D.books, 0, sizeof(Book) * ms, stream));
  HIPCHK(hipMemsetAsync(D.lvl_bump, 0, 4, stream));
  HIPCHK(hipMemsetAsync(D.ch_bump, 0, 4, stream));
  HIPCHK(hipMemsetAsync(D.idx, 0, sizeof(IdxEnt) * idx_cap, stream));
  HIPCHK(hipMemsetAsync(d_st, 0, sizeof(Status), stream));
  HIPCHK(hipMemsetAsync(D.ctr_s, 0, 8ull * CTR_STRIPES * CTR_STRIDE, stream));

  // ---- per-batch buffers
  const uint32_t nb = max_batch;
  adm_mask = static_cast<uint32_t>(std::min<uint64_t>(next_pow2(2ull * nb + 16), 1ull << 29) - 1);  // (ADM_SLOT)
  // events of one batch <= one partial per ADD + one per DEL + one per popped maker (<= the
  // resting capacity + the batch's rests) + block padding: sized once, so a pipelined
  // submit never waits to regrow it (HBM is plentiful; the regrowth path stays as a fallback)
  uint64_t evcap = cfg.max_events ? cfg.max_events
                                  : 2ull * nb + cfg.max_nodes + EVB * std::min<uint64_t>(nb, ms) + 1024;
  if (evcap > 0xF0000000ull) evcap = 0xF0000000ull;
  arena_cap = static_cast<uint32_t>(evcap);
  for (Slot& S : slots)
    if (!alloc(&S.k0, nb, "keys0") || !alloc(&S.v0, nb, "vals0") || !alloc(&S.k1, nb, "keys1") ||
        !alloc(&S.v1, nb, "vals1") || !alloc(&S.hist, hist_cap, "hist") || !alloc(&S.bsum, bsum_cap, "sort scan") ||
        !alloc(&S.tmp, nb, "segflags") || !alloc(&S.seg_start, nb + 1, "seg_start") ||
        !alloc(&S.seg_order, nb, "seg_order") || !alloc(&S.bcnt, 64, "buckets") || !alloc(&S.sst, 1, "sort status"))
      return GOME_E_CAPACITY;
  if (!alloc(&d_bsum, bsum_cap, "scan") || !alloc(&d_adm, adm_mask + 1ull, "adm_table") ||
      !alloc(&d_dup, adm_mask + 1ull, "admission key table") ||
      !alloc(&d_multi, adm_mask + 1ull, "admission repeat flags") ||
      !alloc(&d_first, adm_mask + 1ull, "first admitted ADDs") ||
      !alloc(&d_adm_slot2, nb, "admission key slots") || !alloc(&d_adm_aux, nb, "admission shared slots") ||
      !alloc(&d_oid_max, cfg.max_symbols, "oid watermarks") || !alloc(&d_adm_ctl, 3, "admission control") ||
      !alloc(&d_adm_slot, nb, "adm_slot") ||
      !alloc(&d_ev_count, nb, "ev_count") || !alloc(&d_ev_off, nb, "ev_off") ||
      !alloc(&d_prep, nb, "prep") || !alloc(&d_pend, nb, "pending inserts") ||
      !alloc(&d_resume, MAX_HOT, "resume records") || !alloc(&d_arena, arena_cap, "event arena"))
    return GOME_E_CAPACITY;
  if (!alloc(&d_adm_st, 1, "ahead admission status") || !alloc(&d_adm_redo, 1, "ahead admission redo"))
    return GOME_E_CAPACITY;
  for (Slot& S : slots) {
    if (!alloc(&S.d_orders, nb, "orders") || !alloc(&S.d_events, arena_cap, "events") ||
        !alloc(&S.d_dup, nb, "duplicate-oid list") || !alloc(&S.adm_v, nb, "ahead verdicts"))
      return GOME_E_CAPACITY;
    S.ev_cap = arena_cap;
  }
  // flow path (match_flow.h): per-hot-book headers and level slots, packed records, the
  // touch log and its per-level views (FL_TOUCH_MUL entries per order), gathered makers
  const uint64_t ntouch = static_cast<uint64_t>(FL_TOUCH_MUL) * nb;
  F.ig_cap = static_cast<uint32_t>(std::min<uint64_t>(std::max<uint64_t>(cfg.max_nodes, 1u << 16), 0xF0000000ull));
  F.enabled = (cfg.flags & GOME_FLAG_LEGACY_HOT) ? 0u : 1u;
  if (!alloc(&F.hdr, MAX_FLOW, "flow headers") || !alloc(&F.lvl, MAX_FLOW * FL_CAP, "flow levels") ||
      !alloc(&F.ord8, static_cast<uint64_t>(FL_ORD8_MUL) * nb + FL_ORD8_PAD, "flow records") || !alloc(&F.log, ntouch, "flow touch log") ||
      !alloc(&F.srt, ntouch, "flow level runs") || !alloc(&F.rs, ntouch, "flow new makers") ||
      !alloc(&F.fbase, ntouch, "flow fill bases") || !alloc(&F.tfc, ntouch, "flow touch fills") || !alloc(&F.ig, F.ig_cap, "flow gathered makers") ||
      !alloc(&F.ig_bump, 1, "flow gather bump") || !alloc(&F.toff, 2 * FC_TOFF, "flow touch offsets") ||
      !alloc(&F.tmap, 6ull * (ntouch / 64 + 2), "flow touch-group books") ||
      !alloc(&F.lvout, static_cast<size_t>(MAX_FLOW) * FL_CAP, "flow final levels"))
    return GOME_E_CAPACITY;
  F.maxt = ceil_div(ntouch, FL_TILE);
  F.tmap_stride = static_cast<uint32_t>(ntouch / 64 + 2);
  if (!alloc(&F.tcnt, static_cast<size_t>(FL_HEAD) * F.maxt * FL_CAP, "flow head tile counts") ||
      !alloc(&F.pscr, FL_HEAD, "flow head prep scratch"))
    return GOME_E_CAPACITY;
  // the early plan's buffers (match_early.h): by batch parity the control block, header, levels,
  // packed records and log of one book; shared its prep scratch and verdicts
  for (XBuf& X : xb)
    if (!alloc(&X.ctl, 1, "early control") || !alloc(&X.hdr, 1, "early header") ||
        !alloc(&X.lvl, FL_CAP, "early levels") || !alloc(&X.ord8, nb + FL_ORD8_PAD, "early records") ||
        !alloc(&X.log, ntouch, "early touch log") || !alloc(&X.dlvl, DEEP_CAP, "early deep levels"))
      return GOME_E_CAPACITY;
  if (!alloc(&x_pscr, 1, "early prep scratch") || !alloc(&x_adm, nb, "early verdicts") ||
      !alloc(&x_evc, nb, "early event counts") || !alloc(&x_comp, nb, "early gathered records") || !alloc(&x_cnt, 2 * X_FIND_B, "early block counts") ||
      !alloc(&x_seg, 3, "early segment") || !alloc(&x_sidx, nb, "early permutation") ||
      !alloc(&x_dscr, 1, "early deep scratch") || !alloc(&x_dkey, DEEP_HASH, "early deep prices") ||
      !alloc(&x_dval, DEEP_HASH, "early deep levels of prices") || !alloc(&x_dnew, DEEP_CAP, "early deep sorted prices") ||
      !alloc(&x_dslot, 1, "early deep slot"))
    return GOME_E_CAPACITY;
  for (XBuf& X : xb) HIPCHK(hipMemsetAsync(X.ctl, 0, sizeof(XCtl), stream));
  HIPCHK(hipMemsetAsync(x_dslot, 0, 4, stream));  // (the early deep book is deep slot 0's)
  if ((early_on || adm_ahead_on) && !early_stream) HIPCHK(new_stream(&early_stream));
  // books with DELs (match_flow_cancel.h): per-position scratch, the (symbol, oid)
  // table (generation-tagged: cleared once per 2048 batches)
  fc_hcap = next_pow2(std::max<unsigned long long>(2ull * nb, 1024));
  F.fc_hmask = fc_hcap - 1;
  if (!alloc(&F.fc_del, nb, "flow cancel records") ||
      !alloc(&F.fc_tg, nb, "flow cancel targets") || !alloc(&F.fc_rank, nb, "flow cancel ranks") ||
      !alloc(&F.fc_dt, nb, "flow cancel DEL times") || !alloc(&F.fc_tv, nb, "flow cancel target volumes") ||
      !alloc(&F.tvol, static_cast<size_t>(FL_HEAD) * F.maxt * FC_KEYS, "flow head tile volumes") ||
      !alloc(&F.fc_hash, fc_hcap, "flow cancel table"))
    return GOME_E_CAPACITY;
  F.fcb_cap = static_cast<uint32_t>(ceil_div(ntouch, FCB_CK) + FCB_HCAP);
  if (!alloc(&F.fcb_ctl, 2, "huge level passes") || !alloc(&F.fcb, 2ull * F.fcb_cap, "huge level chunks"))
    return GOME_E_CAPACITY;
  HIPCHK(hipMemsetAsync(F.fc_hash, 0, sizeof(FcHash) * fc_hcap, stream));
  // deep books (match_flow_deep.h): per deep slot
  F.dmaxt = F.maxt;
  F.dtmaxt = ceil_div(F.maxt, 8);
  // one deep slot per possible candidate (a book with >= 2^FLOW_MIN_LOG2 orders), at most MAX_FLOW
  F.dslots = static_cast<uint32_t>(std::min<uint64_t>(MAX_FLOW, std::max<uint64_t>(FL_HEAD + 1, (nb >> FLOW_MIN_LOG2) + FL_HEAD)));
  const size_t ds = F.dslots;
  if (!alloc(&F.dlvl, ds * DEEP_CAP, "deep level tables") ||
      !alloc(&F.dlvout, ds * DEEP_CAP, "deep final levels") ||
      !alloc(&F.dh_key, ds * DEEP_HASH, "deep price sets") ||
      !alloc(&F.dh_val, ds * DEEP_HASH, "deep price levels") ||
      !alloc(&F.dscr, ds, "deep prep scratch") || !alloc(&F.dslot_n, 1, "deep slot count") ||
      !alloc(&F.dtcnt, (static_cast<size_t>(FL_HEAD) * F.dmaxt + (ds - FL_HEAD) * F.dtmaxt) * FL_CAP,
             "deep sort tile counts") ||
      !alloc(&F.dslot_h, ds, "deep slot books") ||
      !alloc(&F.tlog, ntouch, "deep sort pass"))
    return GOME_E_CAPACITY;
  // the price sets start empty; each batch's deep books clear theirs when done
  HIPCHK(hipMemsetAsync(F.dh_key, 0, sizeof(unsigned long long) * ds * DEEP_HASH, stream));
  HIPCHK(hipMemsetAsync(F.dh_val, 0xFF, sizeof(uint32_t) * ds * DEEP_HASH, stream));
  HIPCHK(hipMemsetAsync(F.hdr, 0, sizeof(FlowHdr) * MAX_FLOW, stream));
  // the admission tables that k_adm_clean keeps empty between batches
  HIPCHK(hipMemsetAsync(d_dup, 0, (adm_mask + 1ull) * 8, stream));
  HIPCHK(hipMemsetAsync(d_multi, 0, adm_mask + 1ull, stream));
  HIPCHK(hipMemsetAsync(d_first, 0xFF, (adm_mask + 1ull) * 4, stream));
  HIPCHK(hipMemsetAsync(d_oid_max, 0, 4ull * cfg.max_symbols, stream));
  HIPCHK(hipMemsetAsync(d_adm_ctl, 0, 12, stream));
  HIPCHK(hipMemsetAsync(d_adm, 0, (adm_mask + 1ull) * 8, stream));  // (k_adm_flag leaves it empty)
  HIPCHK(hipMemsetAsync(d_pend, 0, sizeof(PendEnt) * nb, stream));
  if (D.idx_mask >= PEND) return fail(GOME_E_INVAL, "gome_config.max_nodes too large (index > 2^31 slots)");
  HIPCHK(make_sets());
  HIPCHK(hipStreamSynchronize(stream));
  return GOME_OK;
}

void gome_engine::scan(const uint32_t* in, uint32_t m, uint32_t* out, uint32_t* total,
                       hipStream_t s, uint32_t* bsum) {
  const uint32_t nb = ceil_div(m, SCAN_TILE);
  if (!bsum) bsum = d_bsum;  // (the sorts' scans have their slot's: they may run beside a batch's)
  k_scan_reduce<<<nb, SCAN_T, 0, s>>>(in, m, bsum);
  k_scan_spine<<<1, SCAN_T, 0, s>>>(bsum, nb, total);
  k_scan_down<<<nb, SCAN_T, 0, s>>>(in, m, bsum, out);
}

// Enqueue batch `n` records at d_ord through the whole device pipeline on stream s (plus the
// flow / hot streams it forks), publishing into slot `sl`.  Ends with the Status copy to the
// slot's page-locked status and the slot's `done` event; finish() reads them.
gome_status gome_engine::enqueue(const gome_order* d_ord, uint32_t n, hipStream_t s, uint32_t sl,
                                 uint64_t seq_base, uint64_t inflight_n, bool ahead) {
  Slot& S = slots[sl];
  const auto t_enq = std::chrono::steady_clock::now();
  // conservative event bound: one partial per ADD + one event per DEL + one per popped
  // maker (<= resting + ADDs) + block padding; batches still in flight may add to resting
  const unsigned long long rest_ub = resting + inflight_n;
  const unsigned long long bound =
      2ull * n + rest_ub + EVB * static_cast<unsigned long long>(std::min(n, cfg.max_symbols)) + EVB;
  if (bound > 0xF0000000ull) return fail(GOME_E_CAPACITY, "event bound exceeds 2^32");
  if (bound > arena_cap || bound > S.ev_cap) {
    // the arena only lives within one batch, and this slot's events were collected: wait for
    // the batches in flight and grow both (the other slot keeps its events)
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipStreamSynchronize(stream));
    const uint32_t ncap = static_cast<uint32_t>(std::min<unsigned long long>(bound + bound / 2, 0xF0000000ull));
    if (bound > arena_cap) {
      release(d_arena);
      arena_cap = ncap;
      if (!alloc(&d_arena, arena_cap, "event arena")) { poisoned = true; return GOME_E_CAPACITY; }
    }
    if (bound > S.ev_cap) {
      release(S.d_events);
      S.ev_cap = ncap;
      if (!alloc(&S.d_events, S.ev_cap, "events")) { poisoned = true; return GOME_E_CAPACITY; }
    }
    HIPCHK(hipStreamSynchronize(stream));  // (alloc's fill, before the batch's streams use them)
  }
  // cancel-index hygiene: erases leave tombstones and lookups that miss stop only at an EMPTY
  // slot, so rebuild the table from the live nodes before it fills up (70%)
  if ((rest_ub + idx_tomb + 2 * inflight_n) * 10 > idx_cap * 7) {
    HIPCHK(hipMemsetAsync(D.idx, 0, sizeof(IdxEnt) * idx_cap, s));
    k_idx_rebuild<<<dim3(2048, 128), 64, 0, s>>>(D);
    idx_tomb = 0;
    ++n_rebuilds;
  }
  HIPCHK(hipEventRecord(S.ev0, s));
  for (bool& on : S.ph_on) on = false;
  // GOME_PH_* brackets (gome_stats.ms_phase): one event pair per phase on its stream
  auto mark = [&](int ph, int end, hipStream_t st) -> hipError_t {
    if (!phases) return hipSuccess;
    S.ph_on[ph] = true;
    return hipEventRecord(S.ph[ph][end], st);
  };
  // ---- stable radix sort of (symbol_id, seq) and the segments, into the slot's buffers, on the
  // caller's stream.  (Sorting a pipelined batch on the copy stream during the last batch's plan was
  // measured in round 3 and dropped: its record reads slowed the concurrent plan)
  const bool dominant = !(last_maxseg * 16 < last_n);
  hipStream_t ss = s;
  // the hottest book planned early on the copy stream (match_early.h): pipelined device batches
  // after a batch whose hottest book took an ADD plan (the device checks the rest)
  const bool early = early_on && (ahead || copy_busy) && dominant && head_add != 0 && bid > 0 && F.enabled;
  S.early = early;
  const bool adm_ahead = adm_ahead_on && ahead && dominant && !early && early_stream != nullptr;
  const uint32_t bid_prev = bid;
  F.bid = ++bid;
  // per-batch status reset (free_top / freed_top and the level pools persist); admission
  // (flow stream) starts from fork_adm, beside the sort when both are on the caller's stream
  auto status_reset = [&]() -> hipError_t {
    hipError_t he = hipMemsetAsync(d_st, 0, offsetof(Status, free_top), s);
    return he == hipSuccess ? hipEventRecord(fork_adm, s) : he;
  };
  HIPCHK(status_reset());
  const uint32_t T256 = 256, gN = ceil_div(n, T256);
  // A pipelined device batch whose hottest book plans late (no early plan: books with DELs): its
  // sort on the copy stream as soon as the slot's buffers are free (the slot's last batch ended),
  // beside the last batch's plan, so that only the last batch's reconstruction and publish stand
  // between two plans (the sort needs only this batch's records).  Round 3 measured a sort beside
  // the plan slowing it (its record reads); with the plan's CUs reserved (plan_cus) it does not:
  // 78.0 ns per order either way, config 4 +1.2%, config 5c +0.2% against the sort from the last
  // plan's end (same-box A/B, gpurun_out/r06ac; before the chunked huge levels and the split event
  // count shortened the reconstruction, the sort was not on the critical path: r06x, even).
  const bool sort_ahead = ahead && !early && !copy_busy && !cold_main && dominant && bid_prev > 0;
  if (sort_ahead) {
    HIPCHK(hipStreamWaitEvent(copy_stream, S.done, 0));
    ss = copy_stream;
  }
  HIPCHK(mark(GOME_PH_SORT, 0, ss));
  HIPCHK(hipMemsetAsync(S.sst, 0, sizeof(Status), ss));
  const uint32_t nblk = ceil_div(n, RS_TILE);
  uint32_t *kin = nullptr, *vin = nullptr, *kout = S.k0, *vout = S.v0;
  for (uint32_t p = 0; p < passes; ++p) {
    const uint32_t shift = p * dbits;
    const uint32_t bits = std::min(dbits, key_bits - shift);
    if (p == 0) {  // the keys out of the records into k1 (the second pass's output) first
      k_radix_hist<true><<<nblk, RS_T, 0, ss>>>(d_ord, nullptr, S.k1, n, shift, bits, S.hist, nblk);
      scan(S.hist, (1u << bits) * nblk, S.hist, nullptr, ss, S.bsum);
      k_radix_scatter<true><<<nblk, RS_T, 0, ss>>>(S.k1, nullptr, n, shift, bits, S.hist, kout, vout, nblk);
    } else {
      k_radix_hist<false><<<nblk, RS_T, 0, ss>>>(nullptr, kin, nullptr, n, shift, bits, S.hist, nblk);
      scan(S.hist, (1u << bits) * nblk, S.hist, nullptr, ss, S.bsum);
      k_radix_scatter<false><<<nblk, RS_T, 0, ss>>>(kin, vin, n, shift, bits, S.hist, kout, vout, nblk);
    }
    kin = kout;
    vin = vout;
    kout = (kin == S.k0) ? S.k1 : S.k0;
    vout = (vin == S.v0) ? S.v1 : S.v0;
  }
  const uint32_t* skeys = kin;
  const uint32_t* sidx = vin;
  // segments (one per symbol present), longest first
  k_seg_flags<<<gN, T256, 0, ss>>>(skeys, n, S.tmp);
  scan(S.tmp, n, S.tmp, &S.sst->nseg, ss, S.bsum);
  k_seg_write<<<gN, T256, 0, ss>>>(skeys, n, S.tmp, S.seg_start, S.sst);
  HIPCHK(hipMemsetAsync(S.bcnt, 0, 64 * sizeof(uint32_t), ss));
  k_seg_count<<<gN, T256, 0, ss>>>(S.seg_start, S.sst, S.bcnt, &S.sst->ctr[C_MAXSEG]);
  k_seg_bscan<<<1, 64, 0, ss>>>(S.bcnt, S.bcnt + 32, S.sst, FLOW_MIN_LOG2, MAX_FLOW);
  k_seg_scatter<<<gN, T256, 0, ss>>>(S.seg_start, S.sst, S.bcnt + 32, S.seg_order);
  HIPCHK(mark(GOME_PH_SORT, 1, ss));
  if (ss != s) {
    HIPCHK(hipEventRecord(sort_done, ss));
    HIPCHK(hipStreamWaitEvent(s, sort_done, 0));
  }
  k_sort_status<<<1, 1, 0, s>>>(d_st, S.sst);

  // ---- the early plan of the hottest book (match_early.h), on the copy stream: its records and
  // verdicts and the batch's prices of it now, the price set, records and plan as soon as the last
  // batch's plan is done (plan_done)
  XBuf& X = xb[bid & 1];
  FlowArgs FX = F;
  FX.hdr = X.hdr; FX.lvl = X.lvl; FX.ord8 = X.ord8; FX.log = X.log; FX.pscr = x_pscr;
  FX.xlog = 1; FX.h0 = 0; FX.h1 = 1; FX.tb = 0; FX.mb = 0; FX.chains = 0;
  FX.dlvl = X.dlvl; FX.dh_key = x_dkey; FX.dh_val = x_dval; FX.dscr = x_dscr; FX.dslot_h = x_dslot;
  FX.ds0 = 0; FX.ds1 = 1;
  if (early) {
    // the records, verdicts and prices on the early stream (the copy stream is still running the
    // last batch's early plan), the rest after both on the copy stream
    // (pipelined host batches: the record work on the copy stream right behind the batch's H2D, the
    // plan on the early stream, so the copy stream stays free for the copies)
    // (GOME_PLAN_CUS: the part after plan_done on the plan's own stream, which then needs no hop)
    hipStream_t es = (copy_busy && !q4) ? copy_stream : early_stream;
    hipStream_t ps = plan_stream ? plan_stream : (copy_busy || q4) ? early_stream : copy_stream;
    Dev Dx = D;
    Dx.st = reinterpret_cast<Status*>(reinterpret_cast<char*>(X.ctl) + offsetof(XCtl, st));
    BatchArgs Bx{};
    Bx.ord = d_ord; Bx.n = n; Bx.seg_order = x_seg; Bx.seg_start = x_seg + 1; Bx.sidx = x_sidx;
    Bx.adm_flag = x_adm; Bx.ev_count = x_evc; Bx.seq_base = seq_base;
    const uint32_t xn = std::min<uint32_t>(X_FIND_B, std::max<uint32_t>(1u, ceil_div(n, 4096u)));
    HIPCHK(hipStreamWaitEvent(es, prep_h, 0));  // (the last batch's head prep: F.hdr[0] names its book)
    // a host batch's records arrive by the H2D stream: the record work waits for them (until round 6
    // it read the slot's previous records, which k_x_cmp then refused; a poisoned fresh slot faulted)
    if (copy_busy) HIPCHK(hipStreamWaitEvent(es, S.h2d, 0));
    HIPCHK(hipMemsetAsync(X.ctl, 0, sizeof(XCtl), es));
    HIPCHK(hipMemsetAsync(x_pscr, 0, sizeof(FlPrepScr), es));
    HIPCHK(hipMemsetAsync(X.hdr, 0, sizeof(FlowHdr), es));
    HIPCHK(hipMemsetAsync(x_dscr, 0, sizeof(FlPrepScr), es));
    HIPCHK(hipMemsetAsync(x_dkey, 0, sizeof(unsigned long long) * DEEP_HASH, es));
    k_x_count<<<xn, X_FIND_T, 0, es>>>(d_ord, n, F.hdr, bid_prev, x_cnt);
    k_x_scan<<<1, X_FIND_B, 0, es>>>(F.hdr, bid_prev, x_cnt, xn, x_seg, X.ctl);
    k_x_scatter<<<xn, X_FIND_T, 0, es>>>(d_ord, n, F.hdr, bid_prev, x_cnt, x_seg, X.ctl, x_sidx);
    HIPCHK(hipStreamWaitEvent(es, oidmax_done, 0));  // (the last batch's oid watermarks)
    k_x_adm<<<256, 256, 0, es>>>(Bx, X.ctl, d_oid_max, cfg.max_symbols, x_adm);
    k_x_gather<<<1024, 256, 0, es>>>(Bx, x_seg, x_comp);
    k_flow_prep_a<<<dim3(FL_PG, 1), FL_PREP_T, 0, es>>>(Dx, Bx, FX);        // (lane plans)
    k_xd_prep_a<<<FL_PG, FL_PREP_T, 0, es>>>(Bx, FX, X.ctl);                 // (deep plans)
    k_xd_sort_new<<<1, FL_PREP_T, DEEP_CAP * 8, es>>>(FX, X.ctl, x_dnew);
    HIPCHK(hipEventRecord(xpre_done, es));
    HIPCHK(hipStreamWaitEvent(ps, xpre_done, 0));
    // On the plan's own stream the last batch's plan, or its early plan's k_x_take (and the fallback
    // plan when that early plan was not taken), wrote F.hdr[0] / F.lvl on this stream before: no hop
    // through the flow stream (plan_done) between two plans.
    // (Device batches only: on the host path, three batches in flight, every other batch's early
    // plan came 13 ms late without this wait, config 3's e2e 147.7 -> 120.7M, gpurun_out/r05cb.)
    if (!(ps == plan_stream && f_on_plan && !copy_busy)) HIPCHK(hipStreamWaitEvent(ps, plan_done, 0));
    k_x_prep_b<<<1, FL_PREP_T, 0, ps>>>(Bx, FX, F, X.ctl, bid_prev);
    k_x_prep_c<<<ps == plan_stream ? 2 * plan_cus : FL_PG, FL_PREP_T, 0, ps>>>(Dx, FX, x_comp);
    k_xd_prep_b<<<1, FL_PREP_T, XD_PREP_LDS, ps>>>(Bx, FX, F, X.ctl, x_dnew, bid_prev);
    k_deep_prep_c<<<dim3(FL_PG, 1), FL_PREP_T, 0, ps>>>(Dx, Bx, FX);
    HIPCHK(hipEventRecord(xprep_done, ps));
    hipStream_t pst = ps;
    HIPCHK(hipEventRecord(S.evx0, pst));
    k_flow_plan_early<<<1, 256, plan_lds, pst>>>(Dx, FX);
    HIPCHK(hipEventRecord(S.evx1, pst));
    HIPCHK(hipEventRecord(xplan_done, pst));
  }

  // admission markers depend on the input records only: they run on the flow stream beside
  // the validation, the radix sort and the segmentation (the batch's critical path), enqueued
  // after the sort so that the main stream's first kernels reach the GPU first.  Ahead (the batch
  // before it in its hottest plan): on the early stream as soon as that batch's admission is done,
  // without the resting probe; the flow stream then checks that no probe could find a key
  // (k_adm_verify) and runs the passes again, with it, where one could.
  uint32_t* const adm_v = adm_ahead ? S.adm_v : d_adm_slot;
  auto admission = [&](hipStream_t as, Status* ast, bool noprobe, const uint32_t* gate) {
    k_adm<<<gN, T256, 0, as>>>(d_ord, n, d_adm, adm_v, adm_mask, cfg.max_symbols, ast, D.books, D.idx, D.idx_mask,
                               d_oid_max, d_multi, d_adm_ctl + 1, noprobe, gate);
    k_adm_flag<<<gN, T256, 0, as>>>(d_ord, n, adm_v, d_multi, d_dup, d_adm_slot2, d_adm_aux, adm_mask, d_adm,
                                    d_adm_ctl + 1, gate);
    k_adm_res<<<gN, T256, 0, as>>>(d_ord, n, adm_v, d_dup, d_adm_slot2, d_first, d_adm_ctl + 1, gate);
    k_adm_dup<<<gN, T256, 0, as>>>(n, adm_v, d_first, d_adm_ctl + 1, gate);
    k_adm_clean<<<gN, T256, 0, as>>>(n, d_adm_aux, d_adm_slot2, d_dup, d_first, d_multi, d_adm_ctl + 1, gate);
  };
  if (adm_ahead) {
    HIPCHK(hipStreamWaitEvent(early_stream, adm_done, 0));  // (the tables, the watermark: the last batch's admission)
    HIPCHK(hipStreamWaitEvent(early_stream, prep_h, 0));    // (after the last batch's head prep: its plan runs)
    HIPCHK(hipMemsetAsync(d_adm_st, 0, offsetof(Status, free_top), early_stream));
    HIPCHK(hipMemsetAsync(d_adm_redo, 0, 4, early_stream));
    k_adm_ctl<<<1, 1, 0, early_stream>>>(d_adm_ctl, 1u);
    k_adm_pre<<<std::min<uint32_t>(gN, 1024), T256, 0, early_stream>>>(d_ord, n, d_adm_ctl);
    admission(early_stream, d_adm_st, true, nullptr);
    HIPCHK(hipEventRecord(adm_pre_done, early_stream));
  }
  HIPCHK(hipStreamWaitEvent(flow_stream, fork_adm, 0));
  if (!adm_ahead) {
    k_adm_ctl<<<1, 1, 0, flow_stream>>>(d_adm_ctl, 1u);
    k_adm_pre<<<std::min<uint32_t>(gN, 1024), T256, 0, flow_stream>>>(d_ord, n, d_adm_ctl);
  }
  if ((++fc_gen & FC_GEN_MASK) == 0) HIPCHK(hipMemsetAsync(F.fc_hash, 0, sizeof(FcHash) * fc_hcap, flow_stream));
  F.fc_gen = fc_gen;
  HIPCHK(mark(GOME_PH_ADMISSION, 0, flow_stream));
  if (adm_ahead) {
    HIPCHK(hipStreamWaitEvent(flow_stream, adm_pre_done, 0));
    k_adm_verify<<<gN, T256, 0, flow_stream>>>(d_ord, n, D.books, d_oid_max, cfg.max_symbols, d_adm_redo, d_st,
                                               d_adm_st);
    admission(flow_stream, d_st, false, d_adm_redo);
  } else {
    admission(flow_stream, d_st, false, nullptr);
  }
  HIPCHK(mark(GOME_PH_ADMISSION, 1, flow_stream));
  HIPCHK(hipEventRecord(adm_done, flow_stream));


  BatchArgs B;
  B.prep = d_prep;
  B.ord = d_ord;
  B.n = n;
  B.seg_start = S.seg_start;
  B.seg_order = S.seg_order;
  B.arena = d_arena;
  B.arena_cap = arena_cap;
  B.ev_count = d_ev_count;
  B.sidx = sidx;
  B.adm_flag = adm_v;
  B.seq_base = seq_base;
  B.dup_list = S.d_dup;
  const uint32_t grid = std::min<uint32_t>(n, cfg.max_symbols);
  const uint32_t nhot_max = std::min<uint32_t>(MAX_FLOW, grid);
  // flow path: the head (longest FL_HEAD candidates, the batch's critical path) and the tail
  // each run prep -> serial plan -> parallel reconstruction on their own stream, so the
  // hottest book's plan starts after its own prep and the tail overlaps it
  // FH: the head's prep; FH0: the hottest book (plan + reconstruction on the flow stream,
  // the batch's critical path); FH1: the other head books (on the tail's stream, done long
  // before the hottest); FT: the tail.  tb: each range's slice of toff.
  // the deep / cancel chains only while recent batches needed them (GOME_CHAIN_QUIET)
  const uint32_t ch = pick_chains();
  const bool c_deep = (ch & FL_CH_DEEP) != 0, c_canc = (ch & FL_CH_CANCEL) != 0;
  S.chains = ch;
  F.chains = ch;
  // the tail's writes (caller's stream) and events (hot stream, after the near books and the legacy
  // kernels) as two kernels side by side when the last batch had no dominant book: 0.07 ms faster on
  // config 2, but the split events kernel's traffic slows a concurrent hottest-book plan (config 3:
  // +0.2 ms), so with a hot book one fused launch
  const bool split_tail = !dominant;
  FlowArgs FH = F, FH0 = F, FH1 = F, FT = F;
  FH.h0 = 0; FH.h1 = FL_HEAD; FH.tb = 0;
  FH0.h0 = 0; FH0.h1 = 1; FH0.tb = 0; FH0.mb = 0;
  FH1.h0 = 1; FH1.h1 = FL_HEAD; FH1.tb = 2; FH1.mb = 1;
  FT.h0 = FL_HEAD; FT.h1 = MAX_FLOW; FT.tb = FL_HEAD + 3; FT.mb = 2;
  FH.ds0 = 0; FH.ds1 = FL_HEAD; FH0.ds0 = 0; FH0.ds1 = 1; FH1.ds0 = 1; FH1.ds1 = FL_HEAD;
  FT.ds0 = FL_HEAD; FT.ds1 = F.dslots;
  // the ranges' books with DELs count and place their events through a second toff region
  FlowArgs FH0c = FH0, FH1c = FH1, FTc = FT;
  FH0c.tb += FC_TOFF; FH1c.tb += FC_TOFF; FTc.tb += FC_TOFF;
  FH0c.mb += 3; FH1c.mb += 3; FTc.mb += 3;
  // a range's touch offsets, then its group map
  auto toff = [&](const FlowArgs& R, bool cancel, hipStream_t st) {
    if (cancel) k_flow_toff<FL_OK_CANCEL><<<1, 1024, 0, st>>>(D, R);
    else k_flow_toff<FL_OK_ADD><<<1, 1024, 0, st>>>(D, R);
    k_flow_tmap<<<std::min<uint32_t>(ceil_div(R.h1 - R.h0, 4), 1024), 256, 0, st>>>(D, R);
  };
  const uint32_t nh_head = std::min<uint32_t>(FL_HEAD, nhot_max);
  const uint32_t nh_near = nh_head > 1 ? nh_head - 1 : 0;
  const uint32_t nh_tail = nhot_max > FL_HEAD ? nhot_max - FL_HEAD : 0;
  // the head's prep gathers through the sort permutation (prep_at): it starts right after
  // segmentation, beside k_prep
  // deep books: slots, price sets and prep scratch of both ranges
  if (c_deep) {
    HIPCHK(hipMemsetAsync(F.dslot_h, 0xFF, 4ull * F.dslots, s));
    HIPCHK(hipMemsetAsync(F.dslot_n, 0, 4, s));
    HIPCHK(hipMemsetAsync(F.dscr, 0, sizeof(FlPrepScr) * F.dslots, s));
  }
  HIPCHK(hipEventRecord(seg_done, s));
  HIPCHK(hipStreamWaitEvent(flow_stream, seg_done, 0));
  if (early) HIPCHK(hipStreamWaitEvent(flow_stream, xprep_done, 0));  // (it read F.hdr[0] / F.lvl)
  HIPCHK(hipMemsetAsync(F.pscr, 0, sizeof(FlPrepScr) * FL_HEAD, flow_stream));
  HIPCHK(mark(GOME_PH_HEAD_PREP, 0, flow_stream));
  k_flow_prep_a<<<dim3(FL_PG, nh_head), FL_PREP_T, 0, flow_stream>>>(D, B, FH);
  k_flow_prep_b<<<nh_head, FL_PREP_T, 0, flow_stream>>>(D, B, FH);
  k_flow_prep_c<<<dim3(FL_PG, nh_head), FL_PREP_T, 0, flow_stream>>>(D, B, FH);
  // head books with more levels than lanes: the deep prep (match_flow_deep.h)
  auto deep_prep = [&](const FlowArgs& R, uint32_t px, hipStream_t st) {
    const uint32_t ns = std::min<uint32_t>(R.ds1 - R.ds0, DEEP_GRID_T);  // (blocks walk the slots)
    k_deep_prep_a<<<dim3(px, ns), FL_PREP_T, 0, st>>>(D, B, R);
    k_deep_prep_b<<<ns, FL_PREP_T, DEEP_CAP * 8, st>>>(D, B, R);
    k_deep_prep_put<<<dim3(px, ns), FL_PREP_T, 0, st>>>(D, R);
    k_deep_prep_c<<<dim3(px, ns), FL_PREP_T, 0, st>>>(D, B, R);
  };
  if (c_deep) deep_prep(FH, FL_PG, flow_stream);
  // deep books: the two-pass stable sort of a log by level (touches, or the cancel prep's keys)
  // and each level's run
  auto deep_sort = [&](const FlowArgs& R, uint32_t tiles, hipStream_t st) {
    const uint32_t ns = std::min<uint32_t>(R.ds1 - R.ds0, DEEP_GRID_T);  // (blocks walk the slots)
    k_deep_sort_cnt<1><<<dim3(tiles, ns), FL_TILE, 0, st>>>(D, R);
    k_deep_sort_scan<<<ns, FL_CAP, 0, st>>>(D, R);
    k_deep_sort_scatter<1><<<dim3(tiles, ns), FL_TILE, 0, st>>>(D, R);
    k_deep_sort_cnt<2><<<dim3(tiles, ns), FL_TILE, 0, st>>>(D, R);
    k_deep_sort_scan<<<ns, FL_CAP, 0, st>>>(D, R);
    k_deep_sort_scatter<2><<<dim3(tiles, ns), FL_TILE, 0, st>>>(D, R);
    k_deep_runs<<<dim3(64, ns), 256, 0, st>>>(D, R);
  };
  // books with DELs: targets, windows, Q and the W32C / W32DC DEL records (or back to the legacy
  // path).  The deep books' ranks come from a sort of their records by level (match_flow_deep.h).
  auto cancel_prep = [&](const FlowArgs& R, uint32_t nb, uint32_t px, bool wide, hipStream_t st) {
    const uint32_t ns = std::min<uint32_t>(R.ds1 - R.ds0, DEEP_GRID_T);
    k_fc_hash_claim<<<dim3(px, nb), 256, 0, st>>>(D, B, R);
    k_fc_hash_count<<<dim3(px, nb), 256, 0, st>>>(D, B, R);
    k_fc_hash_first<<<dim3(px, nb), 256, 0, st>>>(D, B, R);
    k_fc_resolve<<<dim3(px, nb), 256, 0, st>>>(D, B, R);
    if (c_deep) {  // deep books with DELs (W32DC)
      k_fd_oldwalk<<<dim3(DEEP_GRID, ns), 64, 0, st>>>(D, R);
      k_fd_ckeys<<<dim3(wide ? 256 : 16, ns), 256, 0, st>>>(D, B, R);
      deep_sort(R, wide ? FL_SORT_GRID : 32, st);
      const bool big = wide;  // (the head's busiest levels a block each)
      k_fd_crank<<<dim3(DEEP_GRID, ns), 64, 0, st>>>(D, B, R, big ? 1u : 0u);
      if (big) k_fd_crank_big<<<dim3(FD_CRANK_GRID, ns), FC_LVB_T, 0, st>>>(D, B, R);
      k_fd_tbase<<<ns, DEEP_CLAIM_T, 0, st>>>(D, R);
    }
    if (wide) {  // the head: tile-parallel ranks, windows, layout and records
      k_fc_oldwalk_wide<<<dim3(FL_CAP, nb), 64, 0, st>>>(D, R);
      k_fc_pcnt<<<dim3(FL_SORT_GRID, nb), FL_TILE, 0, st>>>(D, B, R);
      k_fc_pscan<<<nb, FL_CAP * FC_PSCAN_G, 0, st>>>(D, R);
      k_fc_prank<<<dim3(FL_SORT_GRID, nb), FL_TILE, 0, st>>>(D, B, R);
      k_fc_pwin<<<dim3(px, nb), 256, 0, st>>>(D, B, R, 0u);
      k_fc_precs<<<dim3(px, nb), 256, 0, st>>>(D, B, R, 0u);
      k_fc_precs_long<<<dim3(64, nb), 256, 0, st>>>(D, B, R, 0u);
    } else {
      k_fc_oldwalk_book<<<nb, 1024, 0, st>>>(D, R);
      k_fc_pass<<<nb, FC_PASS_T, 0, st>>>(D, B, R);
      k_fc_pwin<<<dim3(px, nb), 256, 0, st>>>(D, B, R, 1u);
      k_fc_precs<<<dim3(px, nb), 256, 0, st>>>(D, B, R, 1u);
      k_fc_precs_long<<<dim3(16, nb), 256, 0, st>>>(D, B, R, 1u);
    }
    if (c_deep) k_fd_decline<<<ns, 256, 0, st>>>(D, R);
    k_fc_unmark<<<dim3(px, nb), 256, 0, st>>>(D, B, R);
    k_fc_route<<<ceil_div(nb, 256), 256, 0, st>>>(D, R);
  };
  // (the head's per-record cancel prep kernels: 512 blocks a book, each a short slice of the hottest
  // book's records, whose loops are chains of hash and index probes: config 4 +1.5% over 64,
  // gpurun_out/r05br, r05bs)
  if (c_canc) cancel_prep(FH, nh_head, 8 * FL_PG, true, flow_stream);
  HIPCHK(mark(GOME_PH_HEAD_PREP, 1, flow_stream));
  HIPCHK(hipEventRecord(prep_h, flow_stream));
  if (early) {  // the early inputs against this prep's, then the early plan taken (or not)
    k_x_cmp<<<256, 256, 0, flow_stream>>>(D, F, FX, X.ctl);
    if (plan_stream && !copy_busy) {  // (right behind the early plan: the next early chain follows it there)
      HIPCHK(hipEventRecord(xcmp_done, flow_stream));
      HIPCHK(hipStreamWaitEvent(plan_stream, xcmp_done, 0));
      k_x_take<<<32, 256, 0, plan_stream>>>(D, F, FX, X.ctl);
    } else {
      HIPCHK(hipStreamWaitEvent(flow_stream, xplan_done, 0));
      k_x_take<<<32, 256, 0, flow_stream>>>(D, F, FX, X.ctl);
    }
  }
  {
    hipStream_t pst = flow_stream;
    // (with no dominant book the batch's critical path is the tail's chain: no hops for it.  A book
    // planned early skips this launch; one whose early plan was not taken is planned here, on the
    // plan stream right behind k_x_take, so whatever writes F.hdr[0] / F.lvl last — the take or this
    // fallback — runs there before the next early chain reads them: ADVICE r5, the fallback used to
    // run on the flow stream beside that chain.)
    // (the plan on the flow stream instead, on every CU but the plan's, skipping this hop: the plan
    // 78 -> 81 ns per order, config 4 -2.3%, 5c -3.1%, gpurun_out/r06ag)
    if (plan_stream && !early && dominant) {
      HIPCHK(hipEventRecord(pl_fork, flow_stream));
      HIPCHK(hipStreamWaitEvent(plan_stream, pl_fork, 0));
      pst = plan_stream;
    } else if (plan_stream && early && !copy_busy) {
      pst = plan_stream;  // (behind k_x_take, which waited for k_x_cmp and so for the head prep)
    }
    HIPCHK(hipEventRecord(S.evf0, pst));
    k_flow_plan_head<<<1, 256, plan_lds, pst>>>(D, FH0);  // (a book planned early: nothing)
    HIPCHK(hipEventRecord(S.evf1, pst));
    if (pst == plan_stream) {
      HIPCHK(hipEventRecord(pl_join, plan_stream));
      HIPCHK(hipStreamWaitEvent(flow_stream, pl_join, 0));
    }
    f_on_plan = plan_stream && pst == plan_stream;
  }
  HIPCHK(hipEventRecord(plan_done, flow_stream));
  if (early) k_x_logcopy<<<1024, 256, 0, flow_stream>>>(F, FX, X.ctl);
  // the other head books' plans need only the head's prep: each takes a whole CU, so they go
  // first, before the tail's prep and plans spread their waves over every CU
  HIPCHK(hipStreamWaitEvent(hot_stream, prep_h, 0));
  if (nh_near) {
    HIPCHK(mark(GOME_PH_NEAR, 0, hot_stream));
    k_flow_plan_near<<<nh_near, 256, plan_lds, hot_stream>>>(D, FH1);
  }
  // ---- admission markers (k_adm, launched above on the flow stream)
  HIPCHK(hipStreamWaitEvent(s, adm_done, 0));
  // k_prep gathers the same records as the head's prep: let the head's prep (the critical
  // path) have the memory system first; the cold books have slack
  // (only when one book dominates the batch, the split_tail test: A/B r3j, without the wait
  // config 2 -0.14 ms, config 3 +0.2 ms; with no dominant book the tail's chain is the critical path)
  if (!split_tail) HIPCHK(hipStreamWaitEvent(s, prep_h, 0));

  // ---- match_books: one wavefront per book; hot books (LDS) on a second stream,
  //      concurrently with the cold books (HBM)
  HIPCHK(mark(GOME_PH_RECORDS, 0, s));
  k_prep<<<gN, T256, 0, s>>>(d_ord, n, sidx, adm_v, d_prep);
  HIPCHK(mark(GOME_PH_RECORDS, 1, s));
  HIPCHK(hipEventRecord(S.evm0, s));
  HIPCHK(hipMemsetAsync(F.ig_bump, 0, 4, s));
  HIPCHK(hipEventRecord(fork, s));
  HIPCHK(hipStreamWaitEvent(flow_stream, fork, 0));  // (k_prep, the gather bump)
  // deep books: the two-pass level sort and the per-level reconstruction, then the writes
  // (per_level: the hottest book's; with DELs its levels go to k_deep_level_hot)
  // the hottest book's levels of FC_HUGE touches or more, by chunks (match_flow_deep.h, k_fcb_*;
  // deep: 0 for a lane book, 1 for a deep one), before the block / wave passes of its other levels
  auto huge_levels = [&](const FlowArgs& R, uint32_t deep, hipStream_t st) {
    (void)hipMemsetAsync(&R.fcb_ctl[deep].n, 0, 4, st);  // (an error is sticky: the next checked call reports it)
    k_fcb_list<<<FCB_LIST_GRID, 1024, 0, st>>>(D, R, deep);
    k_fcb_off<<<1, 64, 0, st>>>(D, R, deep);
    k_fcb_sum1<<<FCB_GRID, FCB_T, 0, st>>>(D, R, deep);
    k_fcb_sum2<<<FCB_GRID, FCB_T, 0, st>>>(D, R, deep);
    k_fcb_scan<<<64, 64, 0, st>>>(D, R, deep);
    k_fcb_write<<<FCB_GRID, FCB_T, 0, st>>>(D, R, deep);
    k_fcb_fifo<<<64, 64, 0, st>>>(D, R, deep);
  };
  auto deep_sort_level = [&](const FlowArgs& R, uint32_t tiles, hipStream_t st, bool per_level) {
    const uint32_t ns = std::min<uint32_t>(R.ds1 - R.ds0, DEEP_GRID_T);  // (blocks walk the slots)
    deep_sort(R, tiles, st);
    const bool hot = per_level && c_canc;
    k_deep_level<<<dim3(DEEP_GRID, ns), 64, 0, st>>>(D, R, hot ? 1u : 0u);
    // (after k_deep_level: a level pass overwrites its level's run end, FlowLvl::pad1, which
    // k_deep_level reads and fd_run checks)
    if (!hot && c_canc) k_deep_level_big<<<dim3(DEEP_BIG_GRID, ns), FC_LVB_T, 0, st>>>(D, R);
    if (hot) {
      huge_levels(R, 1u, st);
      k_deep_level_hot<<<DLH_GRID, FC_LVB_T, 0, st>>>(D, R);
    }
  };
  auto deep_write = [&](const FlowArgs& R, hipStream_t st) {
    const uint32_t ns = std::min<uint32_t>(R.ds1 - R.ds0, DEEP_GRID_T);  // (blocks walk the slots)
    k_deep_claim<<<ns, DEEP_CLAIM_T, 0, st>>>(D, B, R);
    k_deep_write_lv<<<dim3(DEEP_CAP / 64, ns), 64, 0, st>>>(D, B, R);
    k_deep_write_fin<<<ns, DEEP_FIN_T, 0, st>>>(D, R);
  };
  // the hottest book's reconstruction: wide kernels (tile-parallel sort, one wave per level).
  // cs: the stream of the deep books' chain and of k_flow_count.  The deep kernels work on
  // other books than the flow sort / level / write kernels, and k_flow_count reads the plan's
  // log and the level records, which the writes neither read from it nor change, so with
  // cs != st they run beside the writes; k_flow_count still comes after both level passes.
  // fused: the books' events go to the arena, and k_flow_events_fused counts them there (no
  // k_flow_count).
  // pl: the hottest book (a wave per level of a deep book with DELs)
  auto head_recon = [&](const FlowArgs& R, uint32_t nb, hipStream_t st, hipStream_t cs, bool fused,
                        bool pl, bool hand_wait) -> gome_status {
    const bool split = cs != st;
    if (split) {  // the deep books' level sort (other books than the ones below) beside it
      HIPCHK(hipEventRecord(dp_fork, st));
      HIPCHK(hipStreamWaitEvent(cs, dp_fork, 0));
      if (c_deep) deep_sort_level(R, FL_SORT_GRID, cs, pl);
      HIPCHK(hipEventRecord(dl_done, cs));  // (a deep book with DELs: k_fc_count_* / events wait)
    }
    k_flow_sort_cnt<<<dim3(FL_SORT_GRID, nb), FL_TILE, 0, st>>>(D, R);
    k_flow_sort_scan<<<nb, FL_CAP * FL_SCAN_P, 0, st>>>(D, R);
    k_flow_sort_scatter<<<dim3(FL_SORT_GRID, nb), FL_TILE, 0, st>>>(D, R);
    // books planned with stale members (Q2) or zero-volume ADDs (Q6): an order that rested on the
    // other side of a stale price, or a zero-volume maker, hands its book to the legacy kernel
    // (k_flow_zero_check, k_flow_stale_check), on this stream, before any of the book is written;
    // for the hottest book after the hot stream's main legacy launch and its index inserts
    // (hand_wait), which the near books' stream has behind it anyway
    // (books with DELs: stale members and wrong-side cancels, k_fc_stale_level; a bailed one's
    // old targets unmarked)
    k_flow_zero_check<<<dim3(FL_CAP, nb), 64, 0, st>>>(D, R);
    if (c_canc) k_fc_stale_level<<<dim3(FL_CAP, nb), 64, 0, st>>>(D, B, R);
    k_flow_stale_check<<<nb, FL_CAP, 0, st>>>(D, B, R);
    if (c_canc) k_fc_unmark_bailed<<<dim3(FL_PG, nb), 256, 0, st>>>(D, B, R);
    // the hand-over kernels (the legacy kernel in mode 1 for a bailed book, almost always a launch
    // with nothing to do): for the hottest book on the other stream, off its critical path (they
    // took 0.1 ms each on config 5c's, waiting for room on busy CUs); the batch's join waits for
    // that stream before the publish.  The flow kernels after the checks skip a bailed book.
    hipStream_t hs = st;
    if (hand_wait && split) {
      HIPCHK(hipEventRecord(ho_fork, st));
      HIPCHK(hipStreamWaitEvent(cs, ho_fork, 0));
      hs = cs;
    }
    if (hand_wait) HIPCHK(hipStreamWaitEvent(hs, oidmax_done, 0));
    k_match_hot<<<R.h0 + nb, 64, HOT_LDS_BYTES, hs>>>(D, B, d_pend, d_resume, F.hdr, 1u, R.h0, R.h0 + nb);
    k_match_resume<<<R.h0 + nb, 64, 0, hs>>>(D, B, d_resume, F.hdr, R.h0, R.h0 + nb);
    k_pend_apply<<<dim3(8, R.h0 + nb), 256, 0, hs>>>(D, d_pend, S.seg_start, S.seg_order, B, F.hdr, R.h0, R.h0 + nb);
    if (!split && c_deep) deep_sort_level(R, FL_SORT_GRID, st, pl);
    k_flow_level_wide<<<dim3(FL_CAP, nb), FL_LVB_T, 0, st>>>(D, R);
    toff(R, false, st);
    if (split) {
      HIPCHK(hipEventRecord(cnt_fork, st));
      HIPCHK(hipStreamWaitEvent(cs, cnt_fork, 0));
    }
    if (!fused) k_flow_count_fused<<<1024, FL_EV_T, 0, cs>>>(D, B, R);
    if (split) {  // (the publish scan waits for the count, the batch's end for the deep writes)
      HIPCHK(hipEventRecord(cnt_done, cs));
      if (c_deep) deep_write(R, cs);  // (after the count, which reads neither the claims nor the writes)
      HIPCHK(hipEventRecord(dw_done, cs));
    }
    k_flow_write_lv_blk<<<dim3(FL_CAP, nb), FL_LVB_T, 0, st>>>(D, B, R);
    k_flow_write_fin<<<nb, 128, 0, st>>>(D, R);
    if (!split && c_deep) deep_write(R, st);
    return GOME_OK;
  };
  // books with DELs (match_flow_cancel.h); their events go to the arena
  auto head_recon_c = [&](const FlowArgs& R, const FlowArgs& Rc, uint32_t nb, hipStream_t st, bool split) -> gome_status {
    if (!c_canc) return GOME_OK;
    if (split) huge_levels(R, 0u, st);  // (the hottest book's call: nb == 1)
    k_fc_level_blk<<<dim3(FL_CAP, nb), FC_LVB_T, 0, st>>>(D, R, split ? 1u : 0u);
    if (split) HIPCHK(hipStreamWaitEvent(st, dl_done, 0));  // (the deep books' level pass ran on cs)
    toff(Rc, true, st);
    k_fc_count_nf<<<1024, 256, 0, st>>>(D, B, Rc);
    k_fc_count_run<<<1024, 256, 0, st>>>(D, B, Rc);
    k_fc_write_lv<<<dim3(FL_CAP, nb), 64, 0, st>>>(D, B, Rc);
    k_fc_fin<<<nb, 128, 0, st>>>(D, Rc);
    k_fc_events<<<1024, 256, 0, st>>>(D, B, Rc);
    return GOME_OK;
  };
  // Streams (HIP maps more streams than its 4 hardware queues per process onto shared queues,
  // which would serialise them): the hottest book on the flow stream; the other head books'
  // plans (whole CUs, from the head's prep on) and then the legacy hot kernels on the hot
  // stream; the tail's prep, the cold books and the tail's plans and reconstruction on the
  // caller's stream.  Each chain ends well before the hottest book's.  The host enqueues in
  // order of need (a launch costs microseconds of host time, and a hundred of them would
  // otherwise starve the caller's stream): the tail's chain first, then the other head
  // books', then the hottest book's reconstruction (needed only when its plan ends).
  if (nh_tail) {
    HIPCHK(mark(GOME_PH_TAIL_PREP, 0, s));
    k_flow_prep<<<nh_tail, FL_PREP_T, 0, s>>>(D, B, FT);
    if (c_deep) deep_prep(FT, 8, s);
    if (c_canc) cancel_prep(FT, nh_tail, 1, false, s);
    HIPCHK(mark(GOME_PH_TAIL_PREP, 1, s));
  }
  HIPCHK(hipEventRecord(prep_t, s));
  // the cold books (k_match) beside the tail's chain instead of before it: they share no book, only
  // the pools' atomics, and on deep books the cold kernel alone grew to 20 ms per batch (config 5 at
  // step 200), which put the tail's plans and reconstruction behind it on the critical path.  On the
  // copy stream, idle during device and synchronous batches.  Pipelined host batches keep the
  // caller's stream: there the copy stream carries the next batch's H2D, which waited for the cold
  // kernel (config-2 e2e 5.24 -> 6.9 ms per batch).  A stream of its own measured slower at 4, 8
  // and 16 hardware queues (config 2: 2.3 -> 3.6 ms per batch).  A batch with an early
  // plan keeps the copy stream for it and runs the cold books on the early stream (A/B: config 3
  // +0.3..0.7%, config 5 even).  Fewer than 8 hardware queues (cold_main): the caller's stream
  hipStream_t cst = cold_main ? s : (early && !copy_busy) ? early_stream : (copy_busy || early) ? s : copy_stream;
  if (cst != s) HIPCHK(hipStreamWaitEvent(cst, prep_t, 0));
  HIPCHK(hipEventRecord(S.evc0, cst));
  k_match<<<std::min<uint32_t>(ceil_div(grid, COLD_WAVES), COLD_BLOCKS), 64 * COLD_WAVES, COLD_LDS_BYTES, cst>>>(
      D, B, &F.hdr[0].ok, sizeof(FlowHdr) / sizeof(uint32_t));
  HIPCHK(hipEventRecord(S.evc1, cst));
  if (nh_tail) {  // the tail's plans and reconstruction
    HIPCHK(mark(GOME_PH_TAIL_PLAN, 0, s));
    k_flow_plan_tail<<<nh_tail, 64, 0, s>>>(D, FT);
    if (c_canc) k_flow_plan_tail_c<<<nh_tail, 64, 0, s>>>(D, FT);
    // (its blocks walk the tail's deep slots: at most DEEP_GRID_T whole-CU blocks)
    if (c_deep) k_flow_plan_tail_d<<<std::min<uint32_t>(nh_tail, DEEP_GRID_T), 256, FL_DEEP_LDS, s>>>(D, FT);
    HIPCHK(mark(GOME_PH_TAIL_PLAN, 1, s));
    HIPCHK(mark(GOME_PH_TAIL_SORT, 0, s));
    k_flow_sort<<<nh_tail, FL_SORT_T, 0, s>>>(D, FT);
    HIPCHK(mark(GOME_PH_TAIL_SORT, 1, s));
    // the level pass of the tail's lane books with DELs needs only their sorted touches: on the
    // cold books' stream (idle by the time the tail's plans end), beside the deep books' sort and
    // level pass, which took 15 ms on config 5c's tail and had it behind them, 2.8 ms after the
    // hottest book's plan ended, where it slowed that book's reconstruction (gpurun_out/r05ap)
    const bool tfc_split = c_canc && cst != s;
    if (tfc_split) {
      HIPCHK(hipEventRecord(tfc_fork, s));
      HIPCHK(hipStreamWaitEvent(cst, tfc_fork, 0));
      k_fc_level_book<<<nh_tail, 1024, 0, cst>>>(D, FT);
      HIPCHK(hipEventRecord(tfc_done, cst));
    }
    HIPCHK(mark(GOME_PH_TAIL_LEVEL, 0, s));
    k_flow_level<<<nh_tail, FL_LEVEL_T, 0, s>>>(D, FT);
    if (c_deep) deep_sort_level(FT, 32, s, false);
    HIPCHK(mark(GOME_PH_TAIL_LEVEL, 1, s));
    HIPCHK(mark(GOME_PH_TAIL_COUNT, 0, s));
    toff(FT, false, s);
    HIPCHK(mark(GOME_PH_TAIL_COUNT, 1, s));
    // the flow books' writes beside their events (into the arena: k_publish places them
    // after the publish scan), then the deep books' writes
    HIPCHK(mark(GOME_PH_TAIL_WRITE, 0, s));
    if (split_tail) {
      HIPCHK(hipEventRecord(tl_done, s));  // (the events run on the hot stream, below)
      k_flow_write<<<nh_tail, FL_WRITE_T, 0, s>>>(D, B, FT);
    } else {
      k_flow_write_events<<<nh_tail + ceil_div(tail_grid * FL_EV_T, FL_WRITE_T), FL_WRITE_T, 0, s>>>(D, B, FT, nh_tail);
    }
    HIPCHK(mark(GOME_PH_TAIL_WRITE, 1, s));
    HIPCHK(mark(GOME_PH_TAIL_EVENTS, 0, s));
    if (c_deep) deep_write(FT, s);
    if (c_canc) {
      if (tfc_split) HIPCHK(hipStreamWaitEvent(s, tfc_done, 0));
      else k_fc_level_book<<<nh_tail, 1024, 0, s>>>(D, FT);
      toff(FTc, true, s);
      k_fc_count_nf<<<1024, 256, 0, s>>>(D, B, FTc);
      k_fc_count_run<<<1024, 256, 0, s>>>(D, B, FTc);
      k_fc_write_book<<<nh_tail, FL_WRITE_T, 0, s>>>(D, B, FTc);
      k_fc_events<<<1024, 256, 0, s>>>(D, B, FTc);
    }
    HIPCHK(mark(GOME_PH_TAIL_EVENTS, 1, s));
  }
  HIPCHK(hipStreamWaitEvent(hot_stream, fork, 0));  // (their reconstruction reads k_prep's records)
  if (nh_near) {
    if (head_recon(FH1, nh_near, hot_stream, hot_stream, true, false, false) != GOME_OK) return GOME_E_DEVICE;
    if (head_recon_c(FH1, FH1c, nh_near, hot_stream, false) != GOME_OK) return GOME_E_DEVICE;
    k_flow_events_fused<<<1024, FL_EV_T, 0, hot_stream>>>(D, B, FH1);
    HIPCHK(mark(GOME_PH_NEAR, 1, hot_stream));
  }
  // legacy hot path (books the flow path declined); it and the cold kernel read the preps'
  // routing decisions (FlowHdr::ok)
  HIPCHK(hipStreamWaitEvent(hot_stream, prep_t, 0));
  HIPCHK(hipEventRecord(S.evh0, hot_stream));
  const uint32_t nleg = std::min<uint32_t>(MAX_HOT, grid);
  k_match_hot<<<nleg, 64, HOT_LDS_BYTES, hot_stream>>>(D, B, d_pend, d_resume, F.hdr);
  HIPCHK(hipEventRecord(S.evh1, hot_stream));
  k_match_resume<<<nleg, 64, 0, hot_stream>>>(D, B, d_resume);
  k_pend_apply<<<dim3(8, 64), 256, 0, hot_stream>>>(D, d_pend, S.seg_start, S.seg_order, B);
  // oid watermarks for the next batches' duplicate-oid probe (the hot stream has slack here)
  k_oid_max<<<gN, T256, 0, hot_stream>>>(n, skeys, d_prep, d_oid_max);
  HIPCHK(hipEventRecord(oidmax_done, hot_stream));
  if (nh_tail && split_tail) {  // the tail's events beside its writes (arena; k_publish places them)
    HIPCHK(hipStreamWaitEvent(hot_stream, tl_done, 0));
    k_flow_events_fused_w<<<ceil_div(tail_grid * FL_EV_T, FL_WRITE_T), FL_WRITE_T, 0, hot_stream>>>(D, B, FT);
  }
  HIPCHK(hipEventRecord(join, hot_stream));
  // (the hot stream's own work ended long before the hottest book's plan does)
  HIPCHK(mark(GOME_PH_HEAD_RECON, 0, flow_stream));
  if (head_recon(FH0, 1, flow_stream, hot_stream, false, true, true) != GOME_OK) return GOME_E_DEVICE;
  if (head_recon_c(FH0, FH0c, 1, flow_stream, true) != GOME_OK) return GOME_E_DEVICE;
  HIPCHK(mark(GOME_PH_HEAD_RECON, 1, flow_stream));
  HIPCHK(hipEventRecord(joinf, flow_stream));
  HIPCHK(hipStreamWaitEvent(s, join, 0));
  HIPCHK(hipStreamWaitEvent(s, joinf, 0));
  HIPCHK(hipStreamWaitEvent(s, cnt_done, 0));
  if (cst != s) HIPCHK(hipStreamWaitEvent(s, S.evc1, 0));  // (the cold books' events and index)

  HIPCHK(hipEventRecord(S.evm1, s));

  // ---- event compaction into publish order
  HIPCHK(mark(GOME_PH_PUBLISH, 0, s));
  scan(d_ev_count, n, d_ev_off, &d_st->n_events, s);
  // the hottest book's events and the arena scatter fill disjoint slots: run them side by side
  k_publish<<<PUB_SCAT + PUB_HOT, T256, 0, s>>>(D, B, FH0, d_arena, arena_cap, d_ev_off, S.d_events, seq_base);
  HIPCHK(mark(GOME_PH_PUBLISH, 1, s));
  HIPCHK(hipStreamWaitEvent(s, dw_done, 0));
  // quirk books whose state healed go back to the flow path from the next batch on
  k_requalify<<<64, 256, 0, s>>>(D, B, F.hdr, d_resume);
  k_recycle_copy<<<256, 256, 0, s>>>(D);
  k_recycle_fin<<<1, 64, 0, s>>>(D);
  k_lvl_recycle<<<LVL_NCLS, 256, 0, s>>>(D);
  k_ctr_fold<<<1, 64, 0, s>>>(D);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(S.ev1, s));
  HIPCHK(hipMemcpyAsync(S.h_st, d_st, sizeof(Status), hipMemcpyDeviceToHost, s));
  HIPCHK(hipEventRecord(S.done, s));
  S.ms_enqueue = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_enq).count();
  return GOME_OK;
}

// After slot `sl`'s done event: the batch's outcome, counters and timings.
gome_status gome_engine::finish(uint32_t sl, uint32_t n) {
  Slot& S = slots[sl];
  const Status& st = *S.h_st;
  dup_idx.clear();
  if (st.err & ERR_INPUT)
    return fail(GOME_E_INVAL, "batch rejected: a record is outside the exact domain "
                              "(symbol_id >= max_symbols, volume < 0, |value| >= 2^53, or unknown flags)");
  if (st.err) {
    poisoned = true;
    return fail((st.err & ERR_CORRUPT) ? GOME_E_STATE : GOME_E_CAPACITY,
                "device pool exhausted or invariant violated (err bits " + std::to_string(st.err) +
                    "); engine state is no longer usable");
  }
  resting += st.ctr[C_RESTING_DELTA];
  levels += st.ctr[C_LEVELS_DELTA];
  // index entries erased this batch (each leaves a tombstone): rests - net resting change
  idx_tomb += st.ctr[C_RESTS] - st.ctr[C_RESTING_DELTA];
  float ms_total = 0, ms_match = 0, ms_hot = 0, ms_flow = 0, ms_cold = 0;
  (void)hipEventElapsedTime(&ms_cold, S.evc0, S.evc1);
  stats.ms_cold = ms_cold;
  (void)hipEventElapsedTime(&ms_total, S.ev0, S.ev1);
  (void)hipEventElapsedTime(&ms_match, S.evm0, S.evm1);
  (void)hipEventElapsedTime(&ms_hot, S.evh0, S.evh1);
  if (S.early && st.ctr[C_EARLY]) (void)hipEventElapsedTime(&ms_flow, S.evx0, S.evx1);
  else (void)hipEventElapsedTime(&ms_flow, S.evf0, S.evf1);
  head_add = ((head_add << 1) | (st.ctr[C_HEAD_ADD] != 0 ? 1u : 0u)) & 3u;
  stats.n_early = st.ctr[C_EARLY];
  stats.n_early_miss = st.ctr[C_EARLY_MISS];
  stats.n_adm_ahead = st.ctr[C_ADM_AHEAD];
  stats.n_adm_redo = st.ctr[C_ADM_REDO];
  stats.n_flow_stale = st.ctr[C_FLOW_STALE];
  stats.n_flow_bail = st.ctr[C_FLOW_BAIL];
  stats.n_flow_zero = st.ctr[C_FLOW_ZERO];
  stats.n_flow_wrong = st.ctr[C_FLOW_WRONG];
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
  stats.n_index_rebuilds = n_rebuilds;
  stats.idx_tombstones = idx_tomb;
  stats.n_flow_cancels = st.ctr[C_FLOW_CANCELS];
  stats.lvl_used = st.lvl_used;
  stats.n_dup_oid = st.ctr[C_DUP];
  stats.n_flow_tail_fills = st.ctr[C_FLOW_TAIL_FILLS];
  for (int k = 0; k < GOME_NPHASE; ++k) {
    float ms = 0;
    if (S.ph_on[k]) (void)hipEventElapsedTime(&ms, S.ph[k][0], S.ph[k][1]);
    stats.ms_phase[k] = ms;
  }
  stats.ms_host_enqueue = S.ms_enqueue;
  const bool want_deep = st.ctr[C_WANT_DEEP] != 0, want_canc = st.ctr[C_WANT_CANC] != 0;
  deep_quiet = want_deep ? 0u : std::min<uint32_t>(deep_quiet + 1u, GOME_CHAIN_QUIET);
  canc_quiet = want_canc ? 0u : std::min<uint32_t>(canc_quiet + 1u, GOME_CHAIN_QUIET);
  stats.chains = S.chains;
  last_maxseg = st.ctr[C_MAXSEG];
  last_n = n;
  stats.chains_wanted = (want_deep ? FL_CH_DEEP : 0u) | (want_canc ? FL_CH_CANCEL : 0u);
  // FIFO chunks holding nodes (carved from the pool and not on the free stack), with headers
  stats.chunk_bytes = static_cast<uint64_t>(st.ch_used - std::min<uint32_t>(st.ch_used, static_cast<uint32_t>(std::max(st.free_top, 0)))) *
                      (CH * sizeof(Node) + sizeof(ChunkHdr));
  stats.n_quirk_checked = st.ctr[C_QUIRK_CHECKED];
  stats.n_requalified = st.ctr[C_REQUAL];
  if (const uint64_t nd = std::min<uint64_t>(st.ctr[C_DUP], n)) {
    dup_idx.resize(nd);
    HIPCHK(hipMemcpy(dup_idx.data(), S.d_dup, nd * sizeof(uint32_t), hipMemcpyDeviceToHost));
    std::sort(dup_idx.begin(), dup_idx.end());
  }
  return GOME_OK;
}

// (`used`, which gome_load_books checks, is set only when a batch is actually enqueued)
gome_status gome_engine::check_submit(size_t n, const void* p) {
  if (poisoned) return fail(GOME_E_STATE, "engine poisoned by an earlier fatal error");
  if (n > max_batch) return fail(GOME_E_INVAL, "batch larger than max_batch");
  if (n && !p) return fail(GOME_E_INVAL, "NULL records");
  return GOME_OK;
}

// Pool headroom before anything is applied (a device-side capacity error poisons the handle):
// every ADD may rest as a new maker on a new level.  `adds` is the batch's ADD count, or its
// record count when the records are not readable here (device records); batches still in
// flight count in full.  The FIFO chunk pool is sized from max_nodes / max_levels with slack
// and level blocks can fragment, so a device-side error stays possible at the very edge of
// the pools.  GOME_FLAG_NO_HEADROOM turns the check off.
gome_status gome_engine::check_capacity(unsigned long long adds, unsigned long long inflight_n) {
  if (cfg.flags & GOME_FLAG_NO_HEADROOM) return GOME_OK;
  const unsigned long long add = adds + inflight_n, rest = resting + add, lv = levels + add;
  if (rest > cfg.max_nodes || lv > cfg.max_levels)
    return fail(GOME_E_CAPACITY,
                "batch rejected before it was applied (book unchanged): up to " + std::to_string(add) +
                    " new makers on top of " + std::to_string(resting) + " resting / " + std::to_string(levels) +
                    " levels could exceed gome_config.max_nodes / max_levels; submit fewer ADDs or raise them");
  return GOME_OK;
}

// ADD records of a host batch (counted only when the record count alone fails the check).
static unsigned long long count_adds(const gome_order* o, size_t n) {
  unsigned long long a = 0;
  for (size_t i = 0; i < n; ++i) a += o[i].action == GOME_ADD ? 1u : 0u;
  return a;
}

gome_status gome_engine::check_capacity_host(const gome_order* o, size_t n, unsigned long long inflight_n) {
  if (check_capacity(n, inflight_n) == GOME_OK) return GOME_OK;
  return check_capacity(count_adds(o, n), inflight_n);
}

// Copy `n` events of slot `sl` (device) to the host drain queue.
gome_status gome_engine::queue_events(uint32_t sl, size_t n, hipStream_t s) {
  if (pending_pos) {
    pending.erase(pending.begin(), pending.begin() + static_cast<long>(pending_pos));
    pending_pos = 0;
  }
  const size_t old = pending.size();
  pending.resize(old + n);
  if (n) {
    HIPCHK(hipMemcpyAsync(pending.data() + old, slots[sl].d_events, n * sizeof(gome_event),
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  return GOME_OK;
}

// Events of the last device submit that were not drained yet go to the host queue before
// anything reuses their slot (never dropped).
gome_status gome_engine::spill_device_events() {
  if (dev_events_pos < dev_events) {
    Slot& S = slots[dev_slot];
    const size_t k = dev_events - dev_events_pos;
    if (pending_pos) {
      pending.erase(pending.begin(), pending.begin() + static_cast<long>(pending_pos));
      pending_pos = 0;
    }
    const size_t old = pending.size();
    pending.resize(old + k);
    HIPCHK(hipMemcpy(pending.data() + old, S.d_events + dev_events_pos, k * sizeof(gome_event),
                     hipMemcpyDeviceToHost));
  }
  dev_events = dev_events_pos = 0;
  return GOME_OK;
}

gome_status gome_engine::collect(const gome_event** evs, size_t* nev) {
  if (flights.empty()) return fail(GOME_E_NOTFOUND, "no batch in flight");
  const Flight f = flights.front();
  flights.pop_front();
  *evs = nullptr;
  *nev = 0;
  if (f.n == 0) return GOME_OK;
  Slot& S = slots[f.slot];
  HIPCHK(hipEventSynchronize(S.done));
  bool copied = false;
  int ds = 0;
  {  // an async host batch: the copy thread issued its event copy at its end
    std::unique_lock<std::mutex> lk(d2h_mu);
    if (S.d2h_state) {
      d2h_cv.wait(lk, [&] { return S.d2h_state >= 2; });
      ds = S.d2h_state;
      S.d2h_state = 0;
    }
  }
  if (ds) {
    if (ds == 3) return fail(GOME_E_DEVICE, std::string("event copy: ") + hipGetErrorString(S.d2h_err));
    HIPCHK(hipEventSynchronize(S.d2h));
    copied = true;
  }
  gome_status st = finish(f.slot, f.n);
  if (st != GOME_OK) return st;
  const size_t n = S.h_st->n_events;
  if (!copied && n) {
    if (n > S.h_cap && (st = host_events(S, n + n / 4 + 1024)) != GOME_OK) return st;
    HIPCHK(hipMemcpyAsync(S.h_events, S.d_events, n * sizeof(gome_event), hipMemcpyDeviceToHost, d2h_stream));
    HIPCHK(hipStreamSynchronize(d2h_stream));
  }
  *evs = S.h_events;
  *nev = n;
  return GOME_OK;
}

// Every batch still in flight -> the drain queue (before a synchronous call).  A batch that
// was rejected (GOME_E_INVAL: nothing applied) does not fail the synchronous call that collected
// it: its status and message are kept as the deferred failure (gome_take_deferred) and the call
// goes on.  Only a failure that leaves the engine unusable (poisoned, or a HIP error) is returned.
gome_status gome_engine::collect_all() {
  gome_status fatal = GOME_OK;
  // (a device batch collected by gome_collect_device is older than those still in flight)
  if (!flights.empty()) {
    if (gome_status st = spill_device_events()) return st;
  }
  while (!flights.empty()) {
    const gome_event* evs = nullptr;
    size_t n = 0;
    const uint64_t base = flights.front().seq_base;
    gome_status st = collect(&evs, &n);
    if (st != GOME_OK) {
      if (!poisoned && st == GOME_E_INVAL) {
        if (deferred == GOME_OK) {
          deferred = st;
          deferred_msg = "in-flight batch (seq_base " + std::to_string(base) + ") rejected: " + err;
        }
      } else if (fatal == GOME_OK) {
        fatal = st;
      }
      continue;
    }
    if (pending_pos) {
      pending.erase(pending.begin(), pending.begin() + static_cast<long>(pending_pos));
      pending_pos = 0;
    }
    pending.insert(pending.end(), evs, evs + n);
  }
  return fatal;
}

// ============================================================== C-ABI
// Every entry point that touches the device switches to the handle's device first and restores
// the caller's on return: a host thread may drive handles on several GPUs (gome_amd/router.py),
// and allocations, copies and launches go to the thread's current device.
struct DevGuard {
  int prev = -1, dev;
  explicit DevGuard(int d) : dev(d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
  }
};

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
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  gome_status s = e->init(*cfg);  // (switches to cfg->device; the caller's device is restored below)
  if (s != GOME_OK) {
    g_create_err = e->err;
    delete e;
  } else {
    *out = e;
  }
  if (prev >= 0) (void)hipSetDevice(prev);
  return s;
}

void gome_destroy(gome_engine* e) {
  if (!e) return;
  DevGuard dg(e->cfg.device);
  delete e;
}

const char* gome_last_error(const gome_engine* e) {
  return e ? e->err.c_str() : g_create_err.c_str();
}

gome_status gome_submit_batch(gome_engine* e, const gome_order* orders, size_t n, uint64_t seq_base) {
  if (!e) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (e->pick_streams() != GOME_OK) return GOME_E_DEVICE;
  gome_status st = e->collect_all();
  if (st != GOME_OK) return st;
  if ((st = e->spill_device_events()) != GOME_OK) return st;
  if ((st = e->check_submit(n, orders)) != GOME_OK) return st;
  if (n == 0) return GOME_OK;
  if ((st = e->check_capacity_host(orders, n, 0)) != GOME_OK) return st;
  const uint32_t sl = e->take_slot();
  Slot& S = e->slots[sl];
  e->used = true;
  hipError_t he = hipMemcpyAsync(S.d_orders, orders, n * sizeof(gome_order), hipMemcpyHostToDevice, e->stream);
  if (he != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
  if ((st = e->enqueue(S.d_orders, static_cast<uint32_t>(n), e->stream, sl, seq_base, 0)) != GOME_OK) return st;
  if ((he = hipEventSynchronize(S.done)) != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
  if ((st = e->finish(sl, static_cast<uint32_t>(n))) != GOME_OK) return st;
  return e->queue_events(sl, S.h_st->n_events, e->stream);
}

gome_status gome_submit_batch_device(gome_engine* e, const gome_order* dev_orders, size_t n,
                                     uint64_t seq_base, void* stream) {
  if (!e) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (e->pick_streams() != GOME_OK) return GOME_E_DEVICE;
  gome_status st = e->collect_all();
  if (st != GOME_OK) return st;
  if ((st = e->spill_device_events()) != GOME_OK) return st;
  if ((st = e->check_submit(n, dev_orders)) != GOME_OK) return st;
  if (n == 0) return GOME_OK;
  if ((st = e->check_capacity(n, 0)) != GOME_OK) return st;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  const uint32_t sl = e->take_slot();
  Slot& S = e->slots[sl];
  e->used = true;
  if ((st = e->enqueue(dev_orders, static_cast<uint32_t>(n), s, sl, seq_base, 0)) != GOME_OK) return st;
  hipError_t he = hipEventSynchronize(S.done);
  if (he != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
  if ((st = e->finish(sl, static_cast<uint32_t>(n))) != GOME_OK) return st;
  e->dev_slot = sl;
  e->dev_events = S.h_st->n_events;
  e->dev_events_pos = 0;
  return GOME_OK;
}

gome_status gome_submit_batch_async(gome_engine* e, const gome_order* orders, size_t n, uint64_t seq_base) {
  if (!e) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (e->pick_streams() != GOME_OK) return GOME_E_DEVICE;
  if (e->flights.size() >= GOME_MAX_INFLIGHT)
    return e->fail(GOME_E_STATE, "GOME_MAX_INFLIGHT batches in flight: gome_collect first");
  gome_status st = e->spill_device_events();
  if (st != GOME_OK) return st;
  if ((st = e->check_submit(n, orders)) != GOME_OK) return st;
  uint64_t inflight_n = 0;
  for (const Flight& f : e->flights) inflight_n += f.n;
  if (n && (st = e->check_capacity_host(orders, n, inflight_n)) != GOME_OK) return st;
  const uint32_t sl = e->take_slot();
  if (n) {
    Slot& S = e->slots[sl];
    e->used = true;
    // the records travel on the H2D stream (beside the batch in flight and the last one's event
    // copy); the pipeline waits.  (On the copy stream, which the pipeline also uses, batch k+2's
    // H2D queued behind batch k+1's early work: e2e 5.6 ms per config-2 step, round 5.)
    hipError_t he = hipMemcpyAsync(S.d_orders, orders, n * sizeof(gome_order), hipMemcpyHostToDevice,
                                   e->h2d_stream);
    if (he == hipSuccess) he = hipEventRecord(S.h2d, e->h2d_stream);
    if (he == hipSuccess) he = hipStreamWaitEvent(e->stream, S.h2d, 0);
    if (he != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
    // (no sort ahead here: on the copy stream it delayed the event copies; e2e +2 ms per config-3 batch)
    e->copy_busy = true;
    st = e->enqueue(S.d_orders, static_cast<uint32_t>(n), e->stream, sl, seq_base, inflight_n);
    e->copy_busy = false;
    if (st != GOME_OK) return st;
    e->d2h_queue(sl);
  }
  e->flights.push_back(Flight{sl, static_cast<uint32_t>(n), seq_base, false});
  return GOME_OK;
}

gome_status gome_submit_batch_device_async(gome_engine* e, const gome_order* dev_orders, size_t n,
                                           uint64_t seq_base) {
  if (!e) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (e->pick_streams() != GOME_OK) return GOME_E_DEVICE;
  if (e->flights.size() >= GOME_MAX_INFLIGHT)
    return e->fail(GOME_E_STATE, "GOME_MAX_INFLIGHT batches in flight: gome_collect first");
  gome_status st = e->spill_device_events();
  if (st != GOME_OK) return st;
  if ((st = e->check_submit(n, dev_orders)) != GOME_OK) return st;
  uint64_t inflight_n = 0;
  for (const Flight& f : e->flights) inflight_n += f.n;
  if (n && (st = e->check_capacity(n, inflight_n)) != GOME_OK) return st;
  const uint32_t sl = e->take_slot();
  if (n) {
    e->used = true;
    if ((st = e->enqueue(dev_orders, static_cast<uint32_t>(n), e->stream, sl, seq_base, inflight_n, true)) != GOME_OK)
      return st;
  }
  e->flights.push_back(Flight{sl, static_cast<uint32_t>(n), seq_base, true});
  return GOME_OK;
}

gome_status gome_collect_device(gome_engine* e, const gome_event** dev_events, size_t* n_events,
                                gome_stats* stats) {
  if (!e || !dev_events || !n_events) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  *dev_events = nullptr;
  *n_events = 0;
  if (e->flights.empty()) return e->fail(GOME_E_NOTFOUND, "no batch in flight");
  const Flight f = e->flights.front();
  if (!f.dev) return e->fail(GOME_E_STATE, "the oldest batch in flight is a host batch: gome_collect");
  e->flights.pop_front();
  gome_status st = e->spill_device_events();
  if (st != GOME_OK) return st;
  if (f.n) {
    Slot& S = e->slots[f.slot];
    hipError_t he = hipEventSynchronize(S.done);
    if (he != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
    if ((st = e->finish(f.slot, f.n)) != GOME_OK) return st;
    e->dev_slot = f.slot;
    e->dev_events = S.h_st->n_events;
    e->dev_events_pos = 0;
    *dev_events = S.d_events;
    *n_events = e->dev_events;
  }
  if (stats) *stats = e->stats;
  return GOME_OK;
}

gome_status gome_collect(gome_engine* e, const gome_event** events, size_t* n_events, gome_stats* stats) {
  if (!e || !events || !n_events) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  gome_status st = e->collect(events, n_events);
  if (st == GOME_OK && stats) *stats = e->stats;
  return st;
}

size_t gome_inflight(const gome_engine* e) { return e ? e->flights.size() : 0; }

gome_status gome_host_alloc(gome_engine* e, size_t bytes, void** out) {
  if (!e || !out) return GOME_E_INVAL;
  *out = nullptr;
  void* p = nullptr;
  if (hipHostMalloc(&p, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess)
    return e->fail(GOME_E_CAPACITY, "hipHostMalloc failed (" + std::to_string(bytes) + " B)");
  e->host_allocs.insert(p);
  *out = p;
  return GOME_OK;
}

void gome_host_free(gome_engine* e, void* p) {
  if (!e || !p) return;
  auto it = e->host_allocs.find(p);
  if (it == e->host_allocs.end()) return;
  (void)hipHostFree(p);
  e->host_allocs.erase(it);
}

size_t gome_pending_events(const gome_engine* e) {
  if (!e) return 0;
  return (e->pending.size() - e->pending_pos) + (e->dev_events - e->dev_events_pos);
}

gome_status gome_drain_events(gome_engine* e, gome_event* out, size_t cap, size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (gome_status s = e->collect_all()) return s;
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
    hipError_t he = hipMemcpy(out + c, e->slots[e->dev_slot].d_events + e->dev_events_pos,
                              k * sizeof(gome_event), hipMemcpyDeviceToHost);
    if (he != hipSuccess) return e->fail(GOME_E_DEVICE, hipGetErrorString(he));
    e->dev_events_pos += k;
    c += k;
  }
  *n_out = c;
  return GOME_OK;
}

gome_status gome_device_events(gome_engine* e, const gome_event** dev_ptr, size_t* n) {
  if (!e || !dev_ptr || !n) return GOME_E_INVAL;
  *dev_ptr = e->slots[e->dev_slot].d_events;
  *n = e->dev_events;
  return GOME_OK;
}

gome_status gome_release_device_events(gome_engine* e) {
  if (!e) return GOME_E_INVAL;
  e->dev_events = e->dev_events_pos = 0;
  return GOME_OK;
}

gome_status gome_debug_flow_books(gome_engine* e, uint32_t* out, size_t cap, size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  gome_status s = e->collect_all();
  if (s != GOME_OK) return s;
  const size_t n = std::min<size_t>({cap, static_cast<size_t>(e->stats.n_hot), static_cast<size_t>(gome::MAX_FLOW)});
  std::vector<gome::FlowHdr> h(n);
  if (n && hipMemcpy(h.data(), e->F.hdr, n * sizeof(gome::FlowHdr), hipMemcpyDeviceToHost) != hipSuccess)
    return e->fail(GOME_E_DEVICE, "gome_debug_flow_books: copy failed");
  for (size_t i = 0; i < n; ++i) {
    const gome::FlowHdr& x = h[i];
    const uint32_t w[GOME_DEBUG_FLOW_WORDS] = {x.ok, x.fc_bad, x.sym, x.end - x.beg, x.ndel, x.nl, x.w32, x.nbsum,
                                               x.ncancel, x.deep};
    std::copy(w, w + GOME_DEBUG_FLOW_WORDS, out + i * GOME_DEBUG_FLOW_WORDS);
  }
  *n_out = n;
  return GOME_OK;
}

gome_status gome_debug_peek(gome_engine* e, uint32_t which, uint64_t offset, uint64_t bytes, void* out) {
  if (!e || (bytes && !out)) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  gome_status s = e->collect_all();
  if (s != GOME_OK) return s;
  const uint64_t nb = e->max_batch;
  const void* base = nullptr;
  uint64_t size = 0;
  switch (which) {
    case 0: base = e->F.hdr; size = sizeof(gome::FlowHdr) * gome::MAX_FLOW; break;
    case 1: base = e->F.lvl; size = sizeof(gome::FlowLvl) * gome::MAX_FLOW * gome::FL_CAP; break;
    case 2: base = e->F.fc_del; size = sizeof(gome::FcDel) * nb; break;
    case 3: base = e->F.fc_rank; size = 4 * nb; break;
    case 4: base = e->F.fc_tg; size = 4 * nb; break;
    case 5: base = e->F.ord8; size = 8 * (static_cast<uint64_t>(gome::FL_ORD8_MUL) * nb + gome::FL_ORD8_PAD); break;
    case 6: base = e->F.fcb_ctl; size = 2 * sizeof(gome::FcbCtl); break;
    default: return GOME_E_INVAL;
  }
  if (offset > size || bytes > size - offset) return GOME_E_INVAL;
  if (bytes && hipMemcpy(out, static_cast<const char*>(base) + offset, bytes, hipMemcpyDeviceToHost) != hipSuccess)
    return e->fail(GOME_E_DEVICE, "gome_debug_peek: copy failed");
  return GOME_OK;
}

gome_status gome_debug_fifo_shape(gome_engine* e, uint32_t sym, int64_t* out, size_t cap, size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (gome_status st = e->collect_all()) return st;
  if (sym >= e->cfg.max_symbols) return e->fail(GOME_E_NOTFOUND, "symbol_id out of range");
  Book bk;
  if (hipMemcpy(&bk, e->D.books + sym, sizeof bk, hipMemcpyDeviceToHost) != hipSuccess)
    return e->fail(GOME_E_DEVICE, "fifo shape copy failed");
  std::vector<Level> lv(bk.n_lvl);
  std::vector<ChunkHdr> ch(e->D.ch_cap);
  std::vector<Node> nd(static_cast<size_t>(e->D.ch_cap) * CH);
  if ((bk.n_lvl && hipMemcpy(lv.data(), e->D.lvl + bk.lvl_base, bk.n_lvl * sizeof(Level), hipMemcpyDeviceToHost) != hipSuccess) ||
      hipMemcpy(ch.data(), e->D.chdr, ch.size() * sizeof(ChunkHdr), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(nd.data(), e->D.nodes, nd.size() * sizeof(Node), hipMemcpyDeviceToHost) != hipSuccess)
    return e->fail(GOME_E_DEVICE, "fifo shape copy failed");
  for (size_t k = 0; k < lv.size() && k < cap; ++k) {
    const Level& L = lv[k];
    int64_t live = 0, dead = 0, nch = 0;
    uint32_t c = L.head;
    for (uint32_t s0 = L.hslot; c != NIL && nch <= e->D.ch_cap; s0 = 0) {
      const uint32_t hi = (c == L.tail) ? L.tslot : CH;
      for (uint32_t sl = s0; sl < hi; ++sl) (nd[static_cast<size_t>(c) * CH + sl].rem < 0 ? dead : live)++;
      ++nch;
      c = (c == L.tail) ? NIL : ch[c].next;
    }
    out[4 * k] = L.price;
    out[4 * k + 1] = live;
    out[4 * k + 2] = dead;
    out[4 * k + 3] = nch;
  }
  *n_out = lv.size();
  return GOME_OK;
}

gome_status gome_get_stats(const gome_engine* e, gome_stats* out) {
  if (!e || !out) return GOME_E_INVAL;
  *out = e->stats;
  return GOME_OK;
}

gome_status gome_engine::tob_buffers(size_t n) {
  if (n <= tob_cap) return GOME_OK;  // (kept between calls: the publisher asks every batch)
  if (d_tob_syms) release(d_tob_syms);
  if (d_tob) release(d_tob);
  d_tob_syms = nullptr;
  d_tob = nullptr;
  tob_cap = 0;
  const size_t cap = std::max<size_t>(n, 64);
  if (!alloc(&d_tob_syms, cap, "tob symbols") || !alloc(&d_tob, cap, "tob digests")) return GOME_E_CAPACITY;
  tob_cap = cap;
  return GOME_OK;
}

gome_status gome_top_of_book(gome_engine* e, const uint32_t* symbols, size_t n, gome_tob* out) {
  if (!e || (n && (!symbols || !out))) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (gome_status s = e->collect_all()) return s;
  if (n == 0) return GOME_OK;
  if (n > (1u << 20)) return e->fail(GOME_E_INVAL, "gome_top_of_book: more than 2^20 symbols");
  if (gome_status s = e->tob_buffers(n)) return s;
  uint32_t* d_syms = e->d_tob_syms;
  gome_tob* d_out = e->d_tob;
  hipStream_t s = e->stream;
  gome_status st = GOME_OK;
  if (hipMemcpyAsync(d_syms, symbols, n * 4, hipMemcpyHostToDevice, s) != hipSuccess) st = GOME_E_DEVICE;
  if (st == GOME_OK) {
    k_tob<<<static_cast<uint32_t>((n + 63) / 64), 64, 0, s>>>(e->D, d_syms, static_cast<uint32_t>(n), d_out);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(out, d_out, n * sizeof(gome_tob), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      st = GOME_E_DEVICE;
  }
  return st == GOME_OK ? GOME_OK : e->fail(st, "gome_top_of_book: device error");
}

// The same digests without waiting: k_tob goes on the pipeline's stream behind the batches
// already submitted (in flight or not), so it reads the books as the last of them leaves them
// and before any later submit touches them; gome_top_of_book_collect waits for it alone.
gome_status gome_top_of_book_enqueue(gome_engine* e, const uint32_t* symbols, size_t n) {
  if (!e || (n && !symbols)) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (e->tob_queued) return e->fail(GOME_E_STATE, "gome_top_of_book_enqueue: collect the pending digests first");
  if (n > (1u << 20)) return e->fail(GOME_E_INVAL, "gome_top_of_book_enqueue: more than 2^20 symbols");
  if (e->poisoned) return e->fail(GOME_E_STATE, "engine poisoned by an earlier fatal error");
  if (gome_status s = e->tob_buffers(n)) return s;
  if (n > e->h_tob_cap) {
    if (e->h_tob_syms) (void)hipHostFree(e->h_tob_syms);
    if (e->h_tob) (void)hipHostFree(e->h_tob);
    e->h_tob_syms = nullptr;
    e->h_tob = nullptr;
    e->h_tob_cap = 0;
    const size_t cap = std::max<size_t>(n, 64);
    HIPCHK_E(e, hipHostMalloc(reinterpret_cast<void**>(&e->h_tob_syms), cap * 4, hipHostMallocDefault));
    HIPCHK_E(e, hipHostMalloc(reinterpret_cast<void**>(&e->h_tob), cap * sizeof(gome_tob), hipHostMallocDefault));
    e->h_tob_cap = cap;
  }
  if (n) {
    std::memcpy(e->h_tob_syms, symbols, n * 4);
    hipStream_t s = e->stream;
    HIPCHK_E(e, hipMemcpyAsync(e->d_tob_syms, e->h_tob_syms, n * 4, hipMemcpyHostToDevice, s));
    k_tob<<<static_cast<uint32_t>((n + 63) / 64), 64, 0, s>>>(e->D, e->d_tob_syms, static_cast<uint32_t>(n), e->d_tob);
    HIPCHK_E(e, hipGetLastError());
    HIPCHK_E(e, hipMemcpyAsync(e->h_tob, e->d_tob, n * sizeof(gome_tob), hipMemcpyDeviceToHost, s));
    HIPCHK_E(e, hipEventRecord(e->tob_done, s));
  }
  e->tob_pending = n;
  e->tob_queued = true;
  return GOME_OK;
}

gome_status gome_top_of_book_collect(gome_engine* e, gome_tob* out, size_t cap, size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (!e->tob_queued) return e->fail(GOME_E_NOTFOUND, "gome_top_of_book_collect: nothing enqueued");
  const size_t n = e->tob_pending;
  if (n) HIPCHK_E(e, hipEventSynchronize(e->tob_done));
  std::memcpy(out, e->h_tob, std::min(cap, n) * sizeof(gome_tob));
  *n_out = n;
  e->tob_queued = false;
  e->tob_pending = 0;
  return GOME_OK;
}

gome_status gome_dup_records(const gome_engine* e, uint32_t* out, size_t cap, size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  const size_t n = e->dup_idx.size();
  std::copy(e->dup_idx.begin(), e->dup_idx.begin() + static_cast<long>(std::min(cap, n)), out);
  *n_out = n;
  return GOME_OK;
}

gome_status gome_take_deferred(gome_engine* e) {
  if (!e) return GOME_E_INVAL;
  const gome_status s = e->deferred;
  if (s != GOME_OK) e->err = e->deferred_msg;
  e->deferred = GOME_OK;
  e->deferred_msg.clear();
  return s;
}

// ---- gome_load_books: a Redis-schema book image straight into the pools of a fresh engine
__global__ void k_load_index(IdxEnt* idx, const unsigned long long* slot, const IdxEnt* ent, size_t n) {
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += gridDim.x * static_cast<size_t>(blockDim.x))
    idx[slot[i]] = ent[i];
}

gome_status gome_engine::load_books(size_t nb, const uint32_t* bsym, const uint32_t* bnlv, const gome_level* lv,
                                    const gome_node* nd, size_t nn) {
  if (poisoned) return fail(GOME_E_STATE, "engine poisoned by an earlier fatal error");
  if (used) return fail(GOME_E_STATE, "gome_load_books: load into a fresh engine (no batch submitted, nothing loaded)");
  if ((nb && (!bsym || !bnlv)) || (nn && !nd)) return fail(GOME_E_INVAL, "gome_load_books: NULL arrays");
  size_t nlv = 0;
  for (size_t b = 0; b < nb; ++b) nlv += bnlv[b];
  if (nlv && !lv) return fail(GOME_E_INVAL, "gome_load_books: NULL levels");
  if (nn > cfg.max_nodes) return fail(GOME_E_CAPACITY, "gome_load_books: more nodes than max_nodes");
  const uint32_t ms = D.max_symbols;
  std::vector<Book> books(ms, Book{0, 0, 0, 0});
  std::vector<uint8_t> seen(ms, 0);
  std::vector<uint32_t> oid_max(ms, 0);  // the duplicate-oid rule's probe filter (k_adm)
  std::vector<Level> lvl;
  std::vector<Node> nodes;
  std::vector<ChunkHdr> chdr;
  std::vector<unsigned long long> islot;
  std::vector<IdxEnt> ient;
  std::unordered_set<unsigned long long> occ;
  const unsigned long long mask = idx_cap - 1;
  size_t li = 0, ni = 0;
  for (size_t b = 0; b < nb; ++b) {
    const uint32_t sym = bsym[b], n = bnlv[b];
    if (sym >= ms || seen[sym]) return fail(GOME_E_INVAL, "gome_load_books: symbol out of range or repeated");
    seen[sym] = 1;
    uint32_t cap = 16;
    while (cap < n) cap <<= 1;
    if (cap > (16u << (LVL_NCLS - 1))) return fail(GOME_E_CAPACITY, "gome_load_books: book with too many levels");
    const size_t base = lvl.size();
    if (base + cap > cfg.max_levels) return fail(GOME_E_CAPACITY, "gome_load_books: levels exceed max_levels");
    lvl.resize(base + cap, Level{});
    bool quirk = false;
    int64_t best_bid = INT64_MIN, best_ask = INT64_MAX;
    for (uint32_t k = 0; k < n; ++k, ++li) {
      const gome_level& g = lv[li];
      if (k && g.price_fx <= lv[li - 1].price_fx) return fail(GOME_E_INVAL, "gome_load_books: prices not ascending");
      if (ni + g.n_nodes > nn) return fail(GOME_E_INVAL, "gome_load_books: level node counts exceed n_nodes");
      Level L{};
      L.price = g.price_fx;
      L.depth = g.depth_fx;
      L.member = static_cast<uint8_t>((g.in_buy ? M_BUY : 0) | (g.in_sale ? M_SALE : 0));
      L.head = L.tail = NIL;
      L.nlive = g.n_nodes;
      int64_t sum = 0;
      uint32_t sides = 0, prev = NIL;
      for (uint32_t j = 0; j < g.n_nodes; ++j, ++ni) {
        const gome_node& x = nd[ni];
        if (x.volume_fx < 0) return fail(GOME_E_INVAL, "gome_load_books: negative node volume");
        if (j % CH == 0) {
          const uint32_t c = static_cast<uint32_t>(chdr.size());
          if (c >= D.ch_cap) return fail(GOME_E_CAPACITY, "gome_load_books: FIFO chunks exceed the pool");
          chdr.push_back(ChunkHdr{NIL, 0, g.price_fx});
          nodes.resize(static_cast<size_t>(c + 1) * CH, Node{});
          if (prev != NIL) chdr[prev].next = c;
          else L.head = c;
          prev = c;
        }
        const uint32_t loc = prev * CH + j % CH;
        Node& N = nodes[loc];
        N.rem = x.volume_fx;
        N.oid = x.oid_id;
        N.uuid = x.uuid_id;
        N.tx = x.side;
        oid_max[sym] = std::max(oid_max[sym], x.oid_id);
        const unsigned long long key = (static_cast<unsigned long long>(sym + 1) << 32) | x.oid_id;
        unsigned long long h = mix64(key) & mask;
        while (occ.count(h)) h = (h + 1) & mask;
        occ.insert(h);
        N.ixs = static_cast<uint32_t>(h);
        islot.push_back(h);
        ient.push_back(IdxEnt{key, loc, 0});
        sum += x.volume_fx;
        sides |= x.side == GOME_SALE ? 2u : 1u;
        if (x.volume_fx == 0) quirk = true;  // a zero-volume maker (Q6)
      }
      if (g.n_nodes) {
        L.tail = prev;
        L.tslot = static_cast<uint8_t>((g.n_nodes - 1) % CH + 1);
      }
      // the flow plans' invariant: a live level has nodes of one side, its depth is their sum
      // and it is a member of exactly that side's set
      const uint32_t want = sides == 1u ? M_BUY : (sides == 2u ? M_SALE : 0u);
      if (!g.n_nodes || sum != g.depth_fx || sides == 3u || L.member != want) quirk = true;
      if (L.member & M_BUY) best_bid = std::max(best_bid, g.price_fx);
      if (L.member & M_SALE) best_ask = std::min(best_ask, g.price_fx);
      lvl[base + k] = L;
    }
    if (best_bid >= best_ask) quirk = true;  // a crossed book (only reachable through quirks)
    books[sym] = Book{static_cast<uint32_t>(base), n, cap, quirk ? BOOK_QUIRK : 0u};
  }
  if (ni != nn) return fail(GOME_E_INVAL, "gome_load_books: n_nodes differs from the levels' node counts");
  if (occ.size() > idx_cap / 2) return fail(GOME_E_CAPACITY, "gome_load_books: cancel index over half full");
  used = true;  // (from here on the pools are written: no second attempt on this engine)
  hipStream_t s = stream;
  const uint32_t nch = static_cast<uint32_t>(chdr.size()), nl = static_cast<uint32_t>(lvl.size());
  if (nl) HIPCHK(hipMemcpyAsync(D.lvl, lvl.data(), nl * sizeof(Level), hipMemcpyHostToDevice, s));
  if (nch) {
    HIPCHK(hipMemcpyAsync(D.nodes, nodes.data(), static_cast<size_t>(nch) * CH * sizeof(Node), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(D.chdr, chdr.data(), nch * sizeof(ChunkHdr), hipMemcpyHostToDevice, s));
  }
  HIPCHK(hipMemcpyAsync(D.books, books.data(), static_cast<size_t>(ms) * sizeof(Book), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(d_oid_max, oid_max.data(), static_cast<size_t>(ms) * 4, hipMemcpyHostToDevice, s));
  oid_gmax_load = *std::max_element(oid_max.begin(), oid_max.end());  // (k_adm_pre's watermark)
  HIPCHK(hipMemcpyAsync(d_adm_ctl, &oid_gmax_load, 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(D.lvl_bump, &nl, 4, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(D.ch_bump, &nch, 4, hipMemcpyHostToDevice, s));
  if (!islot.empty()) {
    unsigned long long* d_slot = nullptr;
    IdxEnt* d_ent = nullptr;
    if (!alloc(&d_slot, islot.size(), "load index slots") || !alloc(&d_ent, ient.size(), "load index entries"))
      return GOME_E_CAPACITY;
    HIPCHK(hipMemcpyAsync(d_slot, islot.data(), islot.size() * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_ent, ient.data(), ient.size() * sizeof(IdxEnt), hipMemcpyHostToDevice, s));
    k_load_index<<<ceil_div(static_cast<uint32_t>(std::min<size_t>(islot.size(), 1u << 24)), 256), 256, 0, s>>>(
        D.idx, d_slot, d_ent, islot.size());
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    release(d_slot);
    release(d_ent);
  }
  HIPCHK(hipStreamSynchronize(s));
  resting = nn;
  levels = nlv;
  stats.n_resting = resting;
  stats.n_levels = levels;
  used = true;
  return GOME_OK;
}

gome_status gome_load_books(gome_engine* e, size_t n_books, const uint32_t* book_sym, const uint32_t* book_nlv,
                            const gome_level* levels, const gome_node* nodes, size_t n_nodes) {
  if (!e) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (gome_status st = e->collect_all()) return st;
  return e->load_books(n_books, book_sym, book_nlv, levels, nodes, n_nodes);
}

gome_status gome_snapshot_levels(gome_engine* e, uint32_t sym, gome_level* out, size_t cap,
                                 size_t* n_out) {
  if (!e || !n_out || (cap && !out)) return GOME_E_INVAL;
  DevGuard dg(e->cfg.device);
  if (gome_status st = e->collect_all()) return st;
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
  DevGuard dg(e->cfg.device);
  if (gome_status st = e->collect_all()) return st;
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
