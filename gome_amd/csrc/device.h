// device.h — device-side data layout of the MI355X matching engine.
//
// Book state lives in HBM and mirrors the reference's Redis key schema
//  per symbol S:
//   Level    <- S:depth field (depth), S:BUY / S:SALE membership (member bits),
//               S:link:<price> "f"/"l" pointers (head/tail chunk + slot)
//   Node     <- one JSON node of S:link:<price> (32 B, two 16-B halves)
//   chunks   <- CH consecutive Nodes of one FIFO (CH x 32 B) + a ChunkHdr
//   IdxEnt   <- HGET S:link:<p> S:node:<oid> (engine.go:92-93) as an (S, oid) index
#pragma once
#include <stdint.h>

namespace gome {

constexpr int WAVE = 64;
// FIFO slots per chunk.  A level's FIFO is a chain of chunks, so every non-empty level holds at
// least one: deep books (config 5: ~1.2 makers per level) paid 1 KiB per level with 32-slot
// chunks; 4-slot chunks (128 B + a 16-B header) hold them at ~110-140 B per resting order for
// 0-2.6% of batch time on the deep-FIFO workloads (same-box A/B, round 4).
#ifndef GOME_CH
#define GOME_CH 4
#endif
constexpr int CH = GOME_CH;
constexpr uint32_t NIL = 0xFFFFFFFFu;
constexpr uint8_t M_BUY = 1, M_SALE = 2;  // side-set membership bits
constexpr unsigned long long KEY_EMPTY = 0ull, KEY_TOMB = ~0ull;

// One price level (32 B).  Levels of a book form an array sorted by price.
struct Level {
  int64_t price;
  int64_t depth;     // == sum of live FIFO volumes (S:depth:<price>)
  uint32_t head;     // head chunk id or NIL (FIFO empty)
  uint32_t tail;     // tail chunk id or NIL
  uint8_t hslot;     // first not-yet-consumed slot of the head chunk
  uint8_t tslot;     // next free slot of the tail chunk
  uint8_t member;    // M_BUY | M_SALE
  uint8_t pad;
  uint32_t nlive;    // live FIFO nodes
};
static_assert(sizeof(Level) == 32, "Level layout");

// One FIFO slot (32 B).  rem < 0 marks a cancelled slot (tombstone).
struct alignas(16) Node {
  int64_t rem;       // remaining volume
  uint32_t oid;
  uint32_t uuid;
  uint32_t ixs;      // cancel-index slot of the node (O(1) erase on fill)
  uint8_t tx;        // raw Transaction of the resting order
  uint8_t p0, p1, p2;
  uint64_t pad;
};
static_assert(sizeof(Node) == 32, "Node layout");

struct ChunkHdr {
  uint32_t next;     // next chunk of the FIFO or NIL
  uint32_t pad;
  int64_t price;     // level price (Q3 check on cancel)
};

struct Book {
  uint32_t lvl_base, n_lvl, lvl_cap, pad;  // pad: BOOK_* flags
};
// The book holds (or may hold) state the aggregate (flow) plan cannot express: set by a cancel
// whose request side differs from the node's side (Q2), a zero-volume maker (Q6), or a load of
// such a state.  Cleared after a batch by k_requalify (match_requal.h) once the book's state
// is again one the flow plans assume (the reference's state heals: nodepool.go:76-83).
constexpr uint32_t BOOK_QUIRK = 1u;
// Book::pad: the book may hold zero-volume makers (Q6), and Level::pad counts the zero-volume makers
// in each level's FIFO (L_ZERO_SAT: that many or more; k_requalify sets both, the head books' flow
// writes keep them, match_flow.h; any other kernel that applies such a book sets BOOK_QUIRK, so
// k_requalify recounts after it).
constexpr uint32_t BOOK_ZERO = 2u;
constexpr uint8_t L_ZERO_SAT = 255u;
// a level's zero-volume maker count after `popped` of `before` left and `added` joined
__host__ __device__ constexpr uint8_t l_zero_count(uint32_t before, uint32_t popped, uint32_t added) {
  return before >= L_ZERO_SAT ? L_ZERO_SAT
                              : static_cast<uint8_t>(before - popped + added < L_ZERO_SAT ? before - popped + added : L_ZERO_SAT);
}
// Book::pad: the book may hold stale side-set members (Q2: member, no FIFO, depth 0), so a bid
// may lie above an ask (a stale one) and the cold kernel's bid/ask split scan does not hold
// (set by k_requalify and the flow writes that keep such a level; cleared by a later requalify).
constexpr uint32_t BOOK_STALE = 4u;

struct IdxEnt {
  unsigned long long key;  // ((S+1) << 32) | oid ; 0 empty, ~0 tombstone
  uint32_t loc;            // chunk * CH + slot
  uint32_t pad;
};

// error bits
enum : uint32_t {
  ERR_INPUT = 1u,        // record outside the domain (symbol range, volume, price)
  ERR_LEVELS = 2u,       // level pool exhausted
  ERR_CHUNKS = 4u,       // chunk pool exhausted
  ERR_EVENTS = 8u,       // event arena exhausted
  ERR_INDEX = 16u,       // cancel index full
  ERR_CORRUPT = 32u,     // internal invariant violated
};

// counters (u64), per batch unless noted
enum {
  C_FILLS = 0, C_CANCELS, C_RESTS, C_DROPPED, C_ADD, C_DEL, C_EVENTS,
  C_RESTING_DELTA, C_LEVELS_DELTA, C_MAXSEG, C_NSEG,
  C_HOT_ORDERS, C_HOT_FILLS, C_HOT_RESTS, C_HOT_CANCELS,  // hot books (flow + legacy)
  C_FLOW_BOOKS, C_FLOW_ORDERS, C_FLOW_TOUCHES,            // hot books on the flow path
  C_FLOW_HEAD_ORDERS, C_FLOW_HEAD_TOUCHES,                // ... of which the head (k_flow_plan_head)
  C_FLOW_CANCELS,                                         // cancels applied on the flow path
  C_DUP,                                                  // ADDs rejected as duplicate oids (Q7)
  C_FLOW_TAIL_FILLS,                                      // fills of the tail's flow books
  C_WANT_DEEP, C_WANT_CANC,                               // flow candidates that asked for the deep /
                                                          // cancel chain (enqueued or not)
  C_QUIRK_CHECKED, C_REQUAL,                              // quirk books checked / requalified (k_requalify)
  C_HEAD_ADD,                                             // the hottest book went through an ADD plan
  C_EARLY, C_EARLY_MISS,                                  // its plan was the early one / could not be (match_early.h)
  C_ADM_AHEAD, C_ADM_REDO,                                // admission ran ahead / ran again (k_adm_verify)
  C_FLOW_STALE, C_FLOW_BAIL,                              // head books planned with stale members (Q2) /
                                                          // handed to the legacy kernel after their plan
  C_FLOW_ZERO,                                            // head books planned with zero-volume ADDs (Q6)
  C_FLOW_WRONG,                                           // head books with wrong-side cancels (Q2) on the cancel path
  C_NCTR = 40
};

// Level blocks (a book's sorted level array) come in power-of-two capacities 16 << c.  A
// block a book outgrows is released to its class (a `freed` list during the batch, merged
// into the class's free stack by k_lvl_recycle at batch end, so no block is reused within
// the batch that released it); allocations pop the free stack before the bump pointer.
constexpr uint32_t LVL_NCLS = 24;

struct Status {
  unsigned long long ctr[C_NCTR];
  uint32_t err;
  uint32_t nseg;
  uint32_t ev_bump;
  uint32_t n_events;
  uint32_t nhot;       // segments handled by k_match_hot (first nhot of seg_order)
  uint32_t lvl_used;   // level slots ever carved from the pool (lvl_bump at batch end)
  uint32_t nquirk;     // books the cold / resume waves finished with BOOK_QUIRK (Dev::quirk)
  uint32_t ch_used;    // FIFO chunks ever carved from the pool (ch_bump at batch end)
  // ---- everything below persists across batches (the per-batch reset stops here)
  int32_t free_top;
  uint32_t freed_top;
  int32_t lvl_free_top[LVL_NCLS];
  uint32_t lvl_freed_top[LVL_NCLS];
};

struct Dev {
  Book* books;
  uint32_t max_symbols;
  Level* lvl;
  uint32_t lvl_cap_total;
  uint32_t* lvl_bump;
  Node* nodes;         // chunk c, slot s -> nodes[c * CH + s]
  ChunkHdr* chdr;
  uint32_t ch_cap;
  uint32_t* ch_bump;
  uint32_t* free_ids;
  uint32_t* freed_ids;
  IdxEnt* idx;
  unsigned long long idx_mask;
  Status* st;
  uint32_t* lvl_free;        // per class c: free stack at lvl_cls_off[c] (level-block bases)
  uint32_t* lvl_freed;       // per class c: blocks released this batch
  const uint32_t* lvl_cls_off;  // [LVL_NCLS + 1] offsets; class c holds lvl_cls_off[c+1]-off[c]
  unsigned long long* ctr_s;    // [CTR_STRIPES][CTR_STRIDE] striped batch counters (ctr_add)
  uint32_t* quirk;              // [quirk_cap] symbols of this batch's quirk books (k_requalify's input)
  uint32_t quirk_cap;
};

// The batch counters are added by thousands of waves.  Device-scope atomics on one address (or
// one cache line) serialise -- 64k of them cost ~0.3 ms on the tail's event pass -- so the adds
// go to one of CTR_STRIPES stripes (by workgroup) and k_ctr_fold sums the stripes into
// Status::ctr at the batch's end (and zeroes them).  Counters a kernel reads back during the
// batch (C_DUP: a list index; C_MAXSEG: atomicMax) stay on Status.
constexpr uint32_t CTR_STRIPES = 64, CTR_STRIDE = 48;  // (384-B stripes: three 128-B lines)
static_assert(C_NCTR <= CTR_STRIDE, "one stripe holds every counter");
__device__ __forceinline__ void ctr_add(const Dev& D, uint32_t c, unsigned long long v) {
  const uint32_t s = (blockIdx.x + 13u * blockIdx.y) & (CTR_STRIPES - 1);
  atomicAdd(&D.ctr_s[s * CTR_STRIDE + c], v);
}

// A book a wave finished with BOOK_QUIRK set: k_requalify checks it after the batch (one
// thread; a list that overflows leaves the book flagged until a later batch lists it).
__device__ __forceinline__ void quirk_note(const Dev& D, uint32_t sym) {
  const uint32_t i = atomicAdd(&D.st->nquirk, 1u);
  if (i < D.quirk_cap) D.quirk[i] = sym;
}

__device__ __forceinline__ uint32_t lvl_cls(uint32_t cap) { return (31u - __clz(cap)) - 4u; }

// A level block of `cap` (16 << c) levels: the class's free stack, else the bump pointer.
// Single-thread; NIL when the level pool is exhausted.
struct LvlPool {
  Status* st;
  uint32_t* lvl_free;
  uint32_t* lvl_freed;
  const uint32_t* lvl_cls_off;
  uint32_t* lvl_bump;
  uint32_t lvl_cap_total;
};
__device__ __forceinline__ LvlPool lvl_pool(const Dev& D) {
  return LvlPool{D.st, D.lvl_free, D.lvl_freed, D.lvl_cls_off, D.lvl_bump, D.lvl_cap_total};
}

__device__ __forceinline__ uint32_t lvl_block_alloc(const LvlPool& P, uint32_t cap) {
  const uint32_t c = lvl_cls(cap);
  const int t = atomicSub(&P.st->lvl_free_top[c], 1);
  if (t > 0) return P.lvl_free[P.lvl_cls_off[c] + static_cast<uint32_t>(t) - 1u];
  const uint32_t nb = atomicAdd(P.lvl_bump, cap);
  if (static_cast<unsigned long long>(nb) + cap > P.lvl_cap_total) return NIL;
  return nb;
}
__device__ __forceinline__ uint32_t lvl_block_alloc(const Dev& D, uint32_t cap) {
  return lvl_block_alloc(lvl_pool(D), cap);
}

// Give back the block a book moved out of (single-thread).  A class holds at most
// lvl_cap_total / cap blocks, which is its list's capacity.
__device__ __forceinline__ void lvl_block_release(const LvlPool& P, uint32_t base, uint32_t cap) {
  if (cap < 16u) return;
  const uint32_t c = lvl_cls(cap);
  const uint32_t i = atomicAdd(&P.st->lvl_freed_top[c], 1u);
  if (P.lvl_cls_off[c] + i < P.lvl_cls_off[c + 1]) P.lvl_freed[P.lvl_cls_off[c] + i] = base;
}
__device__ __forceinline__ void lvl_block_release(const Dev& D, uint32_t base, uint32_t cap) {
  lvl_block_release(lvl_pool(D), base, cap);
}

}  // namespace gome
