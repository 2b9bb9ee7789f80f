// match_requal.h — requalification of quirk books for the flow path.
//
// BOOK_QUIRK sends a book to the legacy / cold kernels, which reproduce the reference's
// behaviour on any state.  The flag is set by the states the aggregate plans cannot express:
// a wrong-side cancel (Q2: engine.go:87-116 ZREMs the request's side set, so a level emptied
// that way stays a member of its true side with no FIFO), a zero-volume maker (Q6), or a load
// of such a state.  The reference's state heals: a stale member level leaves its set once a
// later same-side maker there is consumed or cancelled (DeletePoolDepth, nodepool.go:76-83),
// and a zero-volume maker leaves the FIFO when a taker reaches it (MatchOrder, engine.go:145-175).
// After every batch, each book a legacy or cold wave finished with the flag is checked against
// the flow plans' precondition (eligibility) and the flag is cleared when it holds,
// so one legal message no longer keeps a hot book on the ~23x slower legacy kernel for good.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "match_cold.h"
#include "match_flow.h"
#include "match_hot.h"
#include "wave.h"

namespace gome {

// The flow plans' precondition on one book (a whole wave, wave-uniform result):
//  * every level in S:BUY or S:SALE is in exactly one of them, has live FIFO nodes and depth > 0,
//    or is a stale member (Q2: no node, depth 0: the head books' lane plans take it, k_flow_prep_b,
//    every other prep declines it); every other level has no node and depth 0;
//  * every bid lies below every ask (levels are sorted by price; stale members aside);
//  * every live node of a member level has the level's side, or a zero remaining volume (a Q6
//    maker, any side: the head books' lane plans take the book while no order reaches it, marked
//    L_ZERO on its level and BOOK_ZERO on the book), and the level's FIFO holds exactly nlive nodes
//    summing to its depth.
// The level checks come first: a book that is still stale fails them without a FIFO walk.
// Returns -1 (no), else the book's flags after it: BOOK_ZERO (zero-volume makers), BOOK_STALE (stale
// members); sets the levels' L_ZERO.
__device__ __forceinline__ int book_requalifies(const Dev& D, uint32_t sym) {
  const uint32_t lane = lane_id();
  const Book bk = D.books[sym];
  const uint32_t nl = uni(bk.n_lvl);
  Level* L = D.lvl + uni(bk.lvl_base);
  int32_t last_bid = -1;
  uint32_t first_ask = NIL;
  bool anys = false;
  for (uint32_t w0 = 0; w0 < nl; w0 += 64) {
    const uint32_t k = w0 + lane;
    bool bad = false, bid = false, ask = false;
    if (k < nl) {
      const Level x = L[k];
      const bool stale = x.member && x.member != (M_BUY | M_SALE) && x.nlive == 0 && x.depth == 0 && x.head == NIL;
      bid = x.member == M_BUY && !stale;
      ask = x.member == M_SALE && !stale;
      if (x.member == (M_BUY | M_SALE)) bad = true;
      else if (x.member) bad = !stale && (x.nlive == 0 || x.depth <= 0 || x.head == NIL);
      else bad = x.nlive != 0 || x.depth != 0 || x.head != NIL;
    }
    if (__ballot(bad)) return -1;
    if (__ballot(k < nl && L[k].member && !bid && !ask)) anys = true;
    const unsigned long long bm = __ballot(bid), am = __ballot(ask);
    if (bm) last_bid = static_cast<int32_t>(w0 + 63u - static_cast<uint32_t>(__builtin_clzll(bm)));
    if (am && first_ask == NIL) first_ask = w0 + static_cast<uint32_t>(__builtin_ctzll(am));
  }
  if (last_bid >= 0 && first_ask != NIL && static_cast<uint32_t>(last_bid) > first_ask) return -1;
  bool anyz = false;
  for (uint32_t k = 0; k < nl; ++k) {
    const Level x = L[k];
    if (lane == 0 && x.pad) L[k].pad = 0;  // (set below where zero-volume makers rest: their count)
    if (!x.member || x.head == NIL) continue;  // (a stale member: checked above)
    const bool sale = x.member == M_SALE;
    uint32_t c = uni(x.head), s0 = uni(x.hslot), cnt = 0;
    const uint32_t tail = uni(x.tail), tslot = uni(x.tslot);
    int64_t sum = 0;
    bool bad = false;
    uint32_t zc = 0;
    for (uint32_t guard = 0; c != NIL; ++guard) {
      if (guard > D.ch_cap) return -1;
      const uint32_t lim = (c == tail) ? tslot : CH;
      int64_t r = -1;
      uint32_t tx = 0;
      if (lane >= s0 && lane < lim) {
        const Node nd = D.nodes[static_cast<size_t>(c) * CH + lane];
        r = nd.rem;
        tx = nd.tx;
      }
      const bool live = r >= 0;
      bad = bad || (live && r > 0 && ((tx == GOME_SALE) != sale));
      zc += static_cast<uint32_t>(__popcll(__ballot(live && r == 0)));
      cnt += static_cast<uint32_t>(__popcll(__ballot(live)));
      sum += rl64(wave_incl_scan(live ? r : 0), 63);
      c = (c == tail) ? NIL : uni(D.chdr[c].next);
      s0 = 0;
    }
    if (__ballot(bad) || cnt != x.nlive || sum != x.depth) return -1;
    if (zc) {
      anyz = true;
      if (lane == 0) L[k].pad = l_zero_count(zc, 0u, 0u);
    }
  }
  return static_cast<int>((anyz ? BOOK_ZERO : 0u) | (anys ? BOOK_STALE : 0u));
}

// After a batch's book kernels: the books the cold / resume waves listed (Dev::quirk) and the
// legacy kernel's books (hot candidates the flow path declined, at least LEGACY_HOT_MIN orders,
// not handed to k_match_resume, which lists its own), one wave per book.
__global__ __launch_bounds__(256) void k_requalify(Dev D, BatchArgs B, const FlowHdr* flow, const ResumeRec* resume) {
  if (D.st->err) return;  // (a rejected batch applied nothing; a poisoned one is not trusted)
  const uint32_t nw = blockDim.x >> 6;
  const uint32_t nlist = min(D.st->nquirk, D.quirk_cap), nh = min(D.st->nhot, MAX_HOT);
  for (uint32_t i = blockIdx.x * nw + (threadIdx.x >> 6); i < nlist + nh; i += gridDim.x * nw) {
    uint32_t sym;
    if (i < nlist) {
      sym = uni(D.quirk[i]);
    } else {
      const uint32_t h = i - nlist;
      if (flow[h].ok || resume[h].valid) continue;
      const uint32_t seg = B.seg_order[h], beg = B.seg_start[seg];
      if (B.seg_start[seg + 1] - beg < LEGACY_HOT_MIN) continue;  // (the cold kernel's: listed)
      sym = uni(B.ord[B.prep[beg].idx].symbol_id);
    }
    if (!(uni(D.books[sym].pad) & BOOK_QUIRK)) continue;
    const int ok = book_requalifies(D, sym);
    if (lane_id() == 0) {
      ctr_add(D, C_QUIRK_CHECKED, 1);
      if (ok >= 0) {
        D.books[sym].pad = static_cast<uint32_t>(ok);
        ctr_add(D, C_REQUAL, 1);
      }
    }
  }
}

}  // namespace gome
