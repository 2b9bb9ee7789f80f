// match_flow.h — the "flow" path for hot books: match_books split into a minimal serial
// plan over level aggregates and a fully parallel reconstruction of fills and FIFOs.
//
// Why.  Matching within one book is sequential (the reference's single consumer,
// rabbitmq.go:116), so a Zipf-hot book is the batch's critical path and what bounds
// throughput is the per-order latency of ONE wavefront.  The legacy hot kernel
// (match_hot.h) carries the whole FIFO machinery on that serial path (head nodes, chunk
// caches, event stores, index probes): ~1.8 us per order.  But the only state the ORDER
// of operations really flows through is the per-level aggregate S:depth:<p> plus the
// S:BUY / S:SALE membership (nodepool.go:61-115): which levels a taker sweeps and how much
// it takes from each (engine.go:118-136) depend on nothing else.  Given those per-level
// amounts, the individual fills follow from FIFO order alone (engine.go:138-198): the makers
// of one level form a queue in "volume coordinates" — maker m occupies [E_m, E_m + v_m),
// the level's consumption advances a cursor — so every fill is an interval intersection.
//
//   k_flow_prep    (parallel, one workgroup per hot book) eligibility, the book's sorted
//                  price set (<= FL_CAP levels) and one packed 8-B record per order
//                  {volume, level index, side}.
//   k_flow_plan    (SERIAL, one wave per book) the aggregate state machine: depths in lane
//                  registers, membership as scalar bit masks, orders read through the
//                  scalar cache; per order it logs one 16-B "touch" per level it rests at /
//                  consumes from.  Nothing else is on the serial path.
//   k_flow_sort    (one workgroup per book) stable counting sort of the touches by level
//                  -> per-level runs in time order.
//   k_flow_level   (one wave per level) segmented scans -> volume coordinates of each
//                  consumption and each new maker; gathers the consumed prefix of the
//                  level's resting FIFO (chunk chain), frees consumed chunks, erases their
//                  cancel-index entries, writes the partially filled head back.
//   k_flow_count   (parallel) events per touch by binary search -> ev_count[], fill_idx base.
//   k_flow_events  (parallel, after the global publish-order scan) writes every MatchResult
//                  directly at its final position (taker_seq, fill_idx).
//   k_flow_write   (one workgroup per book) appends the surviving new makers to the FIFOs,
//                  inserts them into the cancel index, rewrites the level array.
//
// Eligibility (else the book takes the legacy hot path, bit-exact as before): no
// duplicate-oid candidate (Q7) in the segment and no BOOK_QUIRK state (a state only the legacy /
// cold kernels apply).  A segment with DELs takes the cancel plans (match_flow_cancel.h, W32C /
// W32DC); more levels than FL_CAP lanes the deep plans (match_flow_deep.h).  Every live level
// then has nodes, positive depth and exactly one side-set membership, which is what makes the
// aggregate plan exact -- except the states the head books of at least LEGACY_HOT_MIN orders may
// carry: stale side-set members (Q2), zero-volume takers and makers (Q6, BOOK_ZERO)
// and wrong-side cancels, each checked after the plan (k_flow_zero_check, k_flow_stale_check,
// k_fc_stale_level), which hand the book to the legacy kernel before any of it is written where
// the aggregate view cannot say what the reference does.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gome/gome_abi.h"
#include "device.h"
#include "match_cold.h"
#include "pipeline.h"
#include "wave.h"

namespace gome {

constexpr uint32_t FL_CAP = 128;          // level slots per flow book (two lane sets)
constexpr uint32_t FL_MAX = FL_CAP - 2;   // usable levels 1..126: slot 0 is the bid sentinel,
                                          // slot 127 the ask sentinel (bit scans never miss)
constexpr uint32_t FL_HASH = 1024;        // LDS price-set slots in k_flow_prep
constexpr uint32_t FL_PREP_T = 1024;
constexpr uint32_t FL_HEAD = 8;           // longest candidates on the critical-path stream
constexpr uint32_t FL_TOUCH_MUL = 5;      // log capacity per order (touches <= 3n + L0, plus
                                          // 64 entries of staging slack, n >= 128)
constexpr unsigned long long FL_KEY_OFF = 1ull << 62;
// Packed records of book `seg` start at the 8-aligned index at or above beg + 8 * seg and are
// followed by no-op records up to a multiple of 8: every book's stream is whole half-groups
// (ceil8(x) + ceil8(n) <= ceil8(x + n + 8): books never overlap).
__host__ __device__ constexpr uint32_t fl_obase(uint32_t beg, uint32_t seg) { return (beg + 8u * seg + 7u) & ~7u; }
constexpr uint32_t FL_ORD8_MUL = 9, FL_ORD8_PAD = 512;  // ord8 capacity: 9 * max_batch + 512 (>= the plan loop's L2 prefetch distance + 2 half-groups)

// packed order record of the plan (8 B): volume [0,53), level [53,60), SALE bit 60.  A record
// that must not touch the book (dropped ADD, ignored action, padding) is 0: a zero-volume BUY
// rest at sentinel level 0, which changes nothing and whose touch no later kernel reads.
constexpr uint32_t OR_LI_SHIFT = 21, OR_SELL = 1u << 28;
constexpr uint32_t FL_MAX_ORDERS = (1u << 23) - 8;  // order index (padding included) fits [8, 31) of a touch key
constexpr unsigned long long OR_NOP = 0ull;

enum : uint32_t { TK_CONS = 0, TK_REST = 1, TK_CANC = 2 };
// kind of a logged touch key (W32C cancel touches carry bit 30: the order index of a book with
// DELs is below 2^22; bit 31 is the SALE bit of W32 rest keys and of cancel keys)
constexpr uint32_t FC_MAX_ORDERS = (1u << 22) - 8;  // order index (padding included) of a W32C book
__device__ __forceinline__ uint32_t tk_kind(uint32_t kr, bool cancel_book) {
  return (cancel_book && ((kr >> 30) & 1u)) ? TK_CANC : ((kr >> 7) & 1u);
}

struct Touch {       // one level visited by one order (16 B)
  uint32_t kr;       // level [0,7) | kind << 7 | order index within the segment << 8
  uint32_t pos;      // position in the level-sorted runs (set by k_flow_sort)
  int64_t amt;       // volume taken from the level (CONS) or rested at it (REST)
};
__device__ __forceinline__ uint32_t tk_j(const Touch& x) { return (x.kr >> 8) & 0x7FFFFFu; }  // bit 31: W32 records' side
// the order index of a touch of a book with DELs (bit 30: cancel)
__device__ __forceinline__ uint32_t tk_jc(const Touch& x) { return (x.kr >> 8) & 0x3FFFFFu; }
__device__ __forceinline__ uint32_t tk_jb(const Touch& x, bool cancel_book) { return cancel_book ? tk_jc(x) : tk_j(x); }
static_assert(sizeof(Touch) == 16, "Touch layout");

struct SEnt {        // a touch in its level's run (32 B)
  uint32_t j, kind;
  int64_t amt;
  int64_t coord;     // CONS: cursor before; REST: maker start E (volume coordinates)
  uint32_t t;        // log index
  uint32_t lvl;      // the level (deep books read a touch's level here)
};
static_assert(sizeof(SEnt) == 32, "SEnt layout");

struct RsEnt {       // a new maker of the level, in FIFO order (32 B)
  int64_t e;         // start coordinate
  int64_t v;         // volume rested
  uint32_t j;        // order index within the segment
  uint32_t t;        // log index of the rest (existence test for MatchNode.NextNode)
  uint32_t pad0, pad1;
};
static_assert(sizeof(RsEnt) == 32, "RsEnt layout");

struct FlTouchFc {   // the makers a CONS touch fills (set by the level pass, read by the event passes)
  uint32_t first, last;  // FIFO-order maker indices (old makers IG[0, ig_n), then new ones)
  uint32_t lvl, pad;     // its level
  int64_t coord;         // the consumption cursor before it (volume coordinates)
};
static_assert(sizeof(FlTouchFc) == 24, "FlTouchFc layout");

struct IgEnt {       // a resting maker from before the batch, gathered in FIFO order (32 B)
  int64_t e, v;
  uint32_t oid, uuid;
  uint32_t tx, pad;
};
static_assert(sizeof(IgEnt) == 32, "IgEnt layout");

struct FlowHdr {
  uint32_t ok, nl, sym, ntouch;
  uint32_t beg, end, nold, adds;
  uint32_t dropped, rests, obase, w32;   // obase: first packed record (4-aligned, padded);
                                        // w32: the 32-bit plan (volumes / depths in units of g)
  unsigned long long amask[2], bmask[2];  // final S:SALE / S:BUY membership of the levels
  unsigned long long g;                   // volume unit of the book's plan (1 for the 64-bit plan)
  // books whose segment holds DELs (ok == FL_OK_CANCEL, match_flow_cancel.h)
  uint32_t ndel;       // DEL records of the segment
  uint32_t ncancel;    // the cancel prep's longest window + 1 (diagnostics)
  uint32_t fc_bad;     // set by the cancel prep: decline the book (legacy / cold kernels)
  uint32_t deep;       // the lane prep found more levels than FL_MAX: a deep-book candidate
  uint32_t dslot;      // its deep slot (head: = h; tail: handed out by k_flow_prep)
  uint32_t nbsum;      // books with DELs: the DEL windows' total (the cancel prep's C loops)
  uint32_t dc;         // a deep book whose segment holds DELs (the W32DC plan)
  uint32_t dv_ba;      // W32DV: the best ask after the plan (asks lie at or above it)
  uint32_t pre;        // planned early (match_early.h): k_flow_plan_head leaves the book alone
  uint32_t bid;        // the batch whose prep wrote the header (FlowArgs::bid)
  uint32_t nstale;     // stale side-set members in the level table (Q2, k_flow_stale_check)
  uint32_t bail;       // set with ok = 0 by k_flow_stale_check: the legacy kernel applies the book
  uint32_t nzero;      // admitted zero-volume ADDs of the segment (Q6, k_flow_zero_check)
  uint32_t nzlev;      // levels that may hold zero-volume makers at batch start (FlowLvl::z0)
  uint32_t haz;        // k_flow_zero_check / k_fc_stale_level / k_fc_resolve: a state the reconstruction
                       // cannot take (HZ_* bits: which check found it; diagnostics read them)
  uint32_t nwrong;     // books with DELs: wrong-side cancels that find their maker (Q2, k_fc_resolve)
  uint32_t nlong;      // books with DELs: DELs with a long window (k_fc_precs -> k_fc_precs_long)
};
static_assert(offsetof(FlowHdr, haz) == 144, "FlowHdr::haz offset (tools/heal_diag.py reads it)");
// FlowHdr::ok: 0 declined, FL_OK_ADD an ADD-only flow book, FL_OK_CANCEL a book with DELs,
// FL_OK_DEEP an ADD-only head book with more levels than the lane plans hold (match_flow_deep.h)
constexpr uint32_t FL_OK_ADD = 1, FL_OK_CANCEL = 2, FL_OK_DEEP = 3;
// FlowHdr::haz: a REST of 0 at depth 0, a CONS of 0 on the cancel path, a consume that empties a level
// and stops beside a zero-volume maker, a zero-volume taker meeting one (ADD path), a cancel that
// empties a level beside one, a cancel of one, a rest across a stale price (Q2)
enum : uint32_t {
  HZ_ZREST0 = 1, HZ_ZCONS0 = 2, HZ_ZSTOP = 4, HZ_ZTAKER = 8, HZ_ZDELEMPTY = 16, HZ_ZDEL = 32, HZ_STALE = 64
};
constexpr uint32_t FL_CH_DEEP = 1, FL_CH_CANCEL = 2;  // FlowArgs::chains
constexpr uint32_t DEEP_CAP = 16384;     // level slots of a deep book (0 and DEEP_CAP - 1: sentinels)
constexpr uint32_t DEEP_HASH = 1u << 16; // price-set slots of a deep book (global memory)
constexpr uint32_t DEEP_GRID_T = 128;    // blocks (per dimension) of the tail's deep launches
// Deep slots: the head's FL_HEAD candidates own slots 0..FL_HEAD-1; every other candidate whose
// levels exceed the lanes takes the next free slot (FlowArgs::dslot_n) while FlowArgs::dslots
// lasts (sized at gome_create: one per possible candidate, at most MAX_FLOW).
// FlowHdr::fc_bad: why the cancel prep declined a book (bits; diagnostics read them)
enum : uint32_t {
  FC_BAD_SYM = 1, FC_BAD_TABLE = 2, FC_BAD_Q7 = 4, FC_BAD_Q2 = 8, FC_BAD_LEVEL = 16, FC_BAD_UNIT = 32,
  FC_BAD_WALK = 64, FC_BAD_RING = 128   // FC_BAD_RING: a DEL window / the windows' sum / the segment too long
};

struct FlowLvl {
  int64_t price;
  int64_t d0;        // depth at batch start (== sum of live FIFO volumes)
  int64_t dfin;      // depth after the batch (plan)
  int64_t cfin;      // volume consumed from the level this batch
  uint32_t old;      // index in the book's old level array, NIL if new
  uint32_t nv0;      // live nodes at batch start
  uint32_t cnt;      // touches
  uint32_t base;     // start of the level's run (book-local)
  uint32_t nrest;    // new makers (REST touches)
  uint32_t ig_base, ig_n, ig_all;  // gathered old makers; ig_all: no live node beyond them
  uint32_t head, tail;             // FIFO chunk chain (after the gather)
  uint32_t hslot, tslot;
  uint32_t nlive0;   // old makers surviving the batch
  uint32_t mem0;     // membership at batch start
  uint32_t pad0, pad1;
  // books with DELs (match_flow_cancel.h): the targets of the level's DELs
  uint32_t c_old;    // old (pre-batch) makers targeted by a DEL of the batch
  uint32_t z0;       // zero-volume makers in the level's FIFO at batch start (Level::pad; L_ZERO_SAT: or more)
  uint32_t c_wrong;  // wrong-side DELs (Q2) whose maker rests at this level (k_fc_resolve)
  uint32_t ocan;     // cancelled volume of old makers (plan units), set by the recon
  uint32_t memf;     // deep books: membership after the batch (M_BUY / M_SALE)
  uint32_t ttot;     // targets of the level (old + new): ranks 0 .. ttot - 1
  uint32_t tbase;    // first entry of the level's DEL-time array in FlowArgs::fc_dt (book-local)
  uint32_t mfin;     // books with DELs: the level ends a stale member of this set (M_BUY / M_SALE;
                     // k_fc_stale_level), 0 if not
  uint32_t zpop;     // ADD books: old zero-volume makers the batch popped (fl_level_one's gather)
  uint32_t pad4;
  uint32_t zcont;    // levels that may hold zero-volume makers: the last consume went on (fl_run_cont)
  uint32_t pad6;
};
static_assert(sizeof(FlowLvl) % 16 == 0, "FlowLvl alignment");

// A level that is a stale member at batch start (Q2: one side's set, no FIFO, depth 0; k_flow_prep_b).
__device__ __forceinline__ bool fl_stale0(const FlowLvl& f) {
  return f.old != NIL && f.nv0 == 0 && f.d0 == 0 && (f.mem0 == M_BUY || f.mem0 == M_SALE);
}

constexpr uint32_t FC_TOFF = MAX_FLOW + 16;  // second toff region for books with DELs
constexpr uint32_t FC_GEN_MASK = 0x7FF;   // generation bits of an FcHash key

struct FcDel;  // a DEL record's target (match_flow_cancel.h)
struct FcHash;
struct FcbChunk;  // the chunked pass of a huge level (match_flow_deep.h)
struct FcbCtl;

struct FlowArgs {
  FlowHdr* hdr;        // [MAX_HOT]
  FlowLvl* lvl;        // [MAX_HOT * FL_CAP]
  unsigned long long* ord8;  // [max_batch] packed records, segment order
  Touch* log;          // [FL_TOUCH_MUL * max_batch], book h at FL_TOUCH_MUL * beg
  SEnt* srt;           // same index space
  RsEnt* rs;           // same index space
  uint32_t* fbase;     // same index space: fill_idx of a touch's first event
  FlTouchFc* tfc;      // same index space (log order): a CONS touch's makers (fl_level_fc)
  IgEnt* ig;
  uint32_t ig_cap;
  uint32_t* ig_bump;
  uint32_t* toff;      // [MAX_FLOW + 16] per range (at tb): exclusive scan of the books' touch counts
  uint32_t* tcnt;      // head sort: [FL_HEAD][maxt][FL_CAP] per-tile level counts, then offsets
  Level* lvout;        // head write: [MAX_FLOW * FL_CAP] final level records
  uint32_t maxt;       // tiles per head book (log capacity / FL_TILE)
  struct FlPrepScr* pscr;  // head prep scratch [FL_HEAD] (k_flow_prep_a/b/c)
  uint32_t enabled;
  // the chains this batch enqueued (FL_CH_*): a candidate that needs one that is not there is
  // declined to the legacy / cold kernels (and counted in C_WANT_*, which re-enables it)
  uint32_t chains;
  // the candidates [h0, min(h1, nhot)) this launch covers (head and tail run on their own
  // streams), and the range's offset in toff
  uint32_t h0, h1, tb;
  // books with DELs (match_flow_cancel.h)
  FcDel* fc_del;       // [max_batch] per segment position: the DEL's target
  uint32_t* fc_tg;     // [max_batch] per segment position: ADD targeted by the DEL at (value - 1)
  uint32_t* fc_rank;   // [max_batch] per segment position: a targeted ADD's rank in its level
  uint32_t* fc_dt;     // [max_batch] per book, per level, per target rank: its DEL's segment position
  uint32_t* fc_tv;     // [max_batch] same index: the target's volume (plan units) | SALE << 31
  uint32_t* tvol;      // head prep: [FL_HEAD][maxt][2 * FL_CAP] per-tile ADD volume per (level, side)
  FcHash* fc_hash;     // (symbol, oid) table of the cancel books' records
  uint64_t fc_hmask;
  // deep books (match_flow_deep.h), per deep slot: level tables, final level records, price
  // sets, prep scratch, sort tile counts
  FlowLvl* dlvl;       // [dslots * DEEP_CAP]
  Level* dlvout;       // [dslots * DEEP_CAP]
  unsigned long long* dh_key;  // [dslots * DEEP_HASH]
  uint32_t* dh_val;    // [dslots * DEEP_HASH] level index (after the prep), else old index
  struct FlPrepScr* dscr;  // [dslots]
  uint32_t* dtcnt;     // sort tile counts: FL_CAP per tile, dmaxt tiles per head slot, dtmaxt per tail slot
  uint32_t dmaxt, dtmaxt;
  uint32_t* dslot_h;   // [dslots] the book of each deep slot this batch (NIL: none)
  uint32_t* dslot_n;   // tail deep slots handed out this batch
  uint32_t dslots;     // deep slots (head included)
  uint32_t ds0, ds1;   // the deep slots a launch covers (the range's)
  Touch* tlog;         // the first sort pass's output (the log's index space)
  uint32_t fc_gen;     // batch generation (FcHash entries of older batches are empty)
  // per range (region mb): the book of each 64-touch group of the range's flattened touches
  // (k_flow_tmap), so a wave finds its book with one load instead of a search of toff
  uint32_t* tmap;
  uint32_t tmap_stride, mb;
  uint32_t bid;        // batch number (FlowHdr::bid)
  uint32_t xlog;       // the early plan's arguments (match_early.h): the book's log at F.log + 0
  // the hottest book's huge levels (k_fcb_*): a control block and fcb_cap chunks for a lane book
  // ([0]) and a deep book ([1])
  FcbCtl* fcb_ctl;     // [2]
  FcbChunk* fcb;       // [2 * fcb_cap]
  uint32_t fcb_cap;
};

__device__ __forceinline__ uint32_t fl_hend(const Dev& D, const FlowArgs& F) { return min(F.h1, D.st->nhot); }

// The level table of book h (a deep book's is DEEP_CAP slots in F.dlvl).
__device__ __forceinline__ FlowLvl* fl_lvls(const FlowArgs& F, uint32_t h) {
  return F.hdr[h].ok == FL_OK_DEEP ? F.dlvl + static_cast<size_t>(F.hdr[h].dslot) * DEEP_CAP
                                   : F.lvl + static_cast<size_t>(h) * FL_CAP;
}

__device__ __forceinline__ uint32_t fl_hash(unsigned long long key) {
  return static_cast<uint32_t>(mix64(key) >> 20) & (FL_HASH - 1);
}

// Binary GCD (Stein) of two 64-bit values; gcd(0, x) = x.
__device__ __forceinline__ unsigned long long fl_gcd(unsigned long long a, unsigned long long b) {
  if (a == 0) return b;
  if (b == 0) return a;
  const int sh = __builtin_ctzll(a | b);
  a >>= __builtin_ctzll(a);
  do {
    b >>= __builtin_ctzll(b);
    if (a > b) { const unsigned long long t = a; a = b; b = t; }
    b -= a;
  } while (b);
  return a << sh;
}

constexpr unsigned long long FL_SUM_CAP = 1ull << 62;  // saturation of the volume sum

// Packed plan record of order j of a book.  W64: hi = volume bits 32..52 | li << 21 |
// SALE << 28 (no-op: 0).  W32 (volume in units of g < 2^32): hi = li | 1 << 7 | j << 8 |
// SALE << 31, the key of the touch the order logs when it rests; a no-op (dropped / ignored
// order, padding) rests 0 at the bid sentinel level 0: hi = 1 << 7 | j << 8.
__device__ __forceinline__ unsigned long long fl_rec(bool live, uint32_t li, unsigned long long v, bool sell,
                                                     uint32_t j, bool w32) {
  if (w32) {
    const uint32_t hi = (live ? li | (sell ? 0x80000000u : 0u) : 0u) | 0x80u | (j << 8);
    return (static_cast<unsigned long long>(hi) << 32) | (live ? static_cast<uint32_t>(v) : 0u);
  }
  if (!live) return OR_NOP;
  const uint32_t hi = static_cast<uint32_t>(v >> 32) | (li << OR_LI_SHIFT) | (sell ? OR_SELL : 0u);
  return (static_cast<unsigned long long>(hi) << 32) | static_cast<uint32_t>(v);
}

// ============================================================== k_flow_prep
__global__ __launch_bounds__(FL_PREP_T) void k_flow_prep(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ unsigned long long hkey[FL_HASH];
  __shared__ uint32_t hval[FL_HASH];
  __shared__ unsigned long long ckey[FL_CAP + FL_PREP_T];
  __shared__ uint32_t cslot[FL_CAP + FL_PREP_T];
  __shared__ uint32_t ndist, nc, bad, adds, dropped, dels, many;
  __shared__ unsigned long long wg[FL_PREP_T / 64], ws[FL_PREP_T / 64];
  const uint32_t h = F.h0 + blockIdx.x, tid = threadIdx.x;
  if (h >= fl_hend(D, F)) return;
  FlowHdr* hd = &F.hdr[h];
  const uint32_t seg = B.seg_order[h];
  const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
  const uint32_t sym = B.ord[B.prep[beg].idx].symbol_id;
  if (D.st->err & ERR_INPUT) {  // (the batch is rejected; sym may be out of range)
    if (tid == 0) { hd->ok = 0; hd->deep = 0; hd->bail = 0; }
    return;
  }
  const Book bk = D.books[sym];
  for (uint32_t i = tid; i < FL_HASH; i += FL_PREP_T) { hkey[i] = 0; hval[i] = NIL; }
  if (tid == 0) {
    ndist = nc = adds = dropped = dels = 0;
    bad = (!F.enabled || (bk.pad & (BOOK_QUIRK | BOOK_ZERO)) || (D.st->err & ERR_INPUT) || (end - beg) >= FL_MAX_ORDERS) ? 1u : 0u;
    many = bk.n_lvl > FL_MAX ? 1u : 0u;  // more levels than lanes: a deep candidate
  }
  __syncthreads();
  auto insert = [&](unsigned long long key, uint32_t val) {
    uint32_t s = fl_hash(key);
    for (uint32_t probe = 0; probe < FL_HASH; ++probe) {
      // a hot book hits a few dozen prices: read first, CAS only on a miss (no LDS atomic
      // contention on the hot slots)
      const unsigned long long cur = *reinterpret_cast<volatile unsigned long long*>(&hkey[s]);
      if (cur == key && val == NIL) return;
      if (cur != 0ull && cur != key) {
        s = (s + 1) & (FL_HASH - 1);
        continue;
      }
      const unsigned long long prev = atomicCAS(&hkey[s], 0ull, key);
      if (prev == 0ull) {
        if (val != NIL) hval[s] = val;
        if (atomicAdd(&ndist, 1u) >= FL_MAX) many = 1;
        return;
      }
      if (prev == key) {
        if (val != NIL) hval[s] = val;
        return;
      }
      s = (s + 1) & (FL_HASH - 1);
    }
    many = 1;
  };
  // live levels of the book (clean invariant: live <=> nodes, positive depth, one side)
  const Level* L0 = D.lvl + bk.lvl_base;
  unsigned long long mg = 0, msum = 0;  // gcd and (saturating) sum of every volume the plan sees
  if (!bad && !many) {
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
      insert(static_cast<unsigned long long>(x.price) + FL_KEY_OFF, k);
    }
  }
  __syncthreads();
  // the segment's orders
  uint32_t my_adds = 0, my_drop = 0, my_dels = 0;
  if (!bad && !many) {
    // 4 independent record loads in flight per thread (one block per book is latency-bound)
    for (uint32_t b0 = beg + tid; b0 < end && !bad && !many; b0 += 4 * FL_PREP_T) {
      Prep qs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t b = b0 + u * FL_PREP_T;
        if (b < end) qs[u] = B.prep[b];
        else qs[u].action = 0;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
      const Prep q = qs[u];
      if (q.action == GOME_DEL) { my_dels++; continue; }  // the cancel path (match_flow_cancel.h)
      if (q.action != GOME_ADD) continue;
      my_adds++;
      if (!q.adm) { my_drop++; continue; }
      if (q.vol == 0 || q.adm == ADM_V_CHECK) { bad = 1; break; }  // (Q6; Q7 candidates: serial kernels)
      {  // gcd, with a cheap divisibility test first (exact: integers < 2^53 as doubles)
        const unsigned long long v = static_cast<unsigned long long>(q.vol);
        const double qd = static_cast<double>(v) / static_cast<double>(mg ? mg : 1);
        if (mg == 0 || static_cast<unsigned long long>(qd) * mg != v) mg = fl_gcd(mg, v);
      }
      msum = min(msum + static_cast<unsigned long long>(q.vol), FL_SUM_CAP);
      insert(static_cast<unsigned long long>(q.price) + FL_KEY_OFF, NIL);
      if (bad || many) break;
      }
    }
  }
  if (my_adds) atomicAdd(&adds, my_adds);
  if (my_drop) atomicAdd(&dropped, my_drop);
  if (my_dels) atomicAdd(&dels, my_dels);
  for (int off = 32; off > 0; off >>= 1) {
    mg = fl_gcd(mg, __shfl_xor(mg, off));
    msum = min(msum + __shfl_xor(msum, off), FL_SUM_CAP);
  }
  if (lane_id() == 0) { wg[tid >> 6] = mg; ws[tid >> 6] = msum; }
  __syncthreads();
  if (bad || many || ndist > FL_MAX) {
    if (tid == 0) {
      hd->ok = 0;
      // too many levels for the lanes: a deep book if a deep slot is free (match_flow_deep.h)
      uint32_t slot = NIL;
      const bool want = !bad && bk.n_lvl <= DEEP_CAP - 2;
      if (want) ctr_add(D, C_WANT_DEEP, 1ull);
      if (want && (F.chains & FL_CH_DEEP)) {
        const uint32_t t = atomicAdd(F.dslot_n, 1u);
        if (t < F.dslots - FL_HEAD) slot = FL_HEAD + t;
      }
      hd->deep = slot != NIL ? 1u : 0u;
      hd->dslot = slot;
      if (slot != NIL) F.dslot_h[slot] = h;
    }
    return;
  }
  // compact the set, rank-sort it (<= FL_CAP keys)
  for (uint32_t s = tid; s < FL_HASH; s += FL_PREP_T) {
    if (hkey[s]) {
      const uint32_t i = atomicAdd(&nc, 1u);
      ckey[i] = hkey[s];
      cslot[i] = s;
    }
  }
  __syncthreads();
  const uint32_t n = nc;
  FlowLvl* LV = F.lvl + h * FL_CAP;
  if (tid < n) {
    const unsigned long long key = ckey[tid];
    uint32_t r = 0;
    for (uint32_t i = 0; i < n; ++i) r += ckey[i] < key ? 1u : 0u;
    const uint32_t s = cslot[tid], old = hval[s];
    FlowLvl f{};
    f.price = static_cast<int64_t>(key - FL_KEY_OFF);
    f.old = old;
    f.head = f.tail = NIL;
    f.ig_base = 0;
    if (old != NIL) {
      const Level x = L0[old];
      f.d0 = x.depth;
      f.nv0 = x.nlive;
      f.head = x.head;
      f.tail = x.tail;
      f.hslot = x.hslot;
      f.tslot = x.tslot;
      f.mem0 = x.member;
    }
    LV[r + 1] = f;
    hval[s] = r + 1;  // the slot now maps price -> level index (each slot has one owner thread)
  }
  __syncthreads();
  const uint32_t obase = fl_obase(beg, seg);
  // volume unit of the plan: the 32-bit plan runs when every depth the book can reach,
  // counted in units of the gcd of all its volumes, fits 32 bits
  unsigned long long g = 0, sum = 0;
  for (uint32_t w = 0; w < FL_PREP_T / 64; ++w) {
    g = fl_gcd(g, wg[w]);
    sum = min(sum + ws[w], FL_SUM_CAP);
  }
  if (g == 0) g = 1;
  // (the cancel plan needs every depth and Q < 2^31: its DEL path clamps with signed arithmetic)
  const bool w32 = sum < FL_SUM_CAP && sum / g < (dels ? (1ull << 31) : (1ull << 32));
  if (!w32) g = 1;
  if (dels && !w32) {  // the cancel plan is 32-bit only
    if (tid == 0) { hd->ok = 0; hd->deep = 0; hd->bail = 0; }
    return;
  }
  if (tid < ((8u - ((end - beg) & 7u)) & 7u))  // padding to whole half-groups (8 records)
    F.ord8[obase + (end - beg) + tid] = fl_rec(false, 0, 0, false, end - beg + tid, w32);
  for (uint32_t b0 = beg + tid; b0 < end; b0 += 4 * FL_PREP_T) {
    Prep qs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t b = b0 + u * FL_PREP_T;
      if (b < end) qs[u] = B.prep[b];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
    const uint32_t b = b0 + u * FL_PREP_T;
    if (b >= end) break;
    const Prep q = qs[u];
    unsigned long long rec = fl_rec(false, 0, 0, false, b - beg, w32);
    if (q.action == GOME_ADD && q.adm) {
      const unsigned long long key = static_cast<unsigned long long>(q.price) + FL_KEY_OFF;
      uint32_t s = fl_hash(key);
      while (hkey[s] != key) s = (s + 1) & (FL_HASH - 1);
      const uint32_t li = hval[s];
      // w32: the volume in units of g (exact: an integer quotient < 2^32 of doubles < 2^53)
      const unsigned long long v = w32 ? static_cast<unsigned long long>(static_cast<double>(q.vol) / static_cast<double>(g))
                                       : static_cast<unsigned long long>(q.vol);
      rec = fl_rec(true, li, v, q.side == GOME_SALE, b - beg, w32);
    }
    F.ord8[obase + (b - beg)] = rec;
    B.ev_count[q.idx] = 0;
    }
  }
  if (tid == 0) {
    FlowHdr x{};
    if (dels) ctr_add(D, C_WANT_CANC, 1ull);
    x.ok = dels ? ((F.chains & FL_CH_CANCEL) ? FL_OK_CANCEL : 0u) : FL_OK_ADD;
    x.nl = n;
    x.sym = sym;
    x.beg = beg;
    x.end = end;
    x.nold = bk.n_lvl;
    x.adds = adds;
    x.dropped = dropped;
    x.obase = obase;
    x.w32 = w32 ? 1u : 0u;
    x.g = g;
    x.ndel = dels;
    *hd = x;
  }
}

// ============================================================== head prep, wide
// The head's books are long (the hottest holds ~8% of a batch): one workgroup per book is
// latency-bound on its record loads, so the head preps in three launches.
//   k_flow_prep_a  (FL_PG blocks per book) a slice of the orders each: distinct prices into the
//                  book's global set, slice gcd / sum, counts, order-level ineligibility;
//   k_flow_prep_b  (one block per book) live levels, eligibility, the sorted level table (same
//                  as k_flow_prep), the price -> level map back to the global set;
//   k_flow_prep_c  (FL_PG blocks per book) the packed records of the slice.
constexpr uint32_t FL_PG = 64;
struct FlPrepScr {
  unsigned long long key[FL_HASH];  // price set (open addressing, fl_hash, linear probing)
  uint32_t val[FL_HASH];            // after k_flow_prep_b: level index of each key
  unsigned long long pg[FL_PG], ps[FL_PG];  // per-slice gcd and saturated sum of volumes
  uint32_t adds, dropped, bad, dels;
  uint32_t many;       // more distinct prices than the lane plans hold: a deep-book candidate
  uint32_t zeros;      // admitted zero-volume ADDs (Q6): k_flow_prep_b takes them on long head books
  // the deep prep's own totals (match_flow_deep.h)
  uint32_t d_adds, d_dropped, d_dels, d_bad, d_ndist;
  // a deep tail book's chunk ids for its FIFO appends, claimed once for all its levels
  // (k_deep_claim; see FlClaim)
  int32_t c_t;
  uint32_t c_nst, c_bb, c_ok;
  uint32_t d_put;      // k_deep_prep_b ranked the set by its grid: k_deep_prep_put fills the level table
};

// A book's chunk ids for all its levels' FIFO appends, claimed at once: id j = j < c_nst ?
// free_ids[c_t - c_nst + j] : c_bb + (j - c_nst); FlowLvl::pad0 = a level's first j.
struct FlClaim {
  int32_t c_t;
  uint32_t c_nst, c_bb, c_ok;
};

// Claim `need` chunk ids (free stack first, then the bump pointer); single thread.
__device__ __forceinline__ FlClaim fl_claim_chunks(const Dev& D, uint32_t need) {
  FlClaim c{0, 0u, 0u, 1u};
  if (!need) return c;
  c.c_t = atomicSub(&D.st->free_top, static_cast<int>(need));
  c.c_nst = static_cast<uint32_t>(min(max(c.c_t, 0), static_cast<int>(need)));
  if (c.c_nst < need) c.c_bb = atomicAdd(D.ch_bump, need - c.c_nst);
  if (static_cast<unsigned long long>(c.c_bb) + (need - c.c_nst) > D.ch_cap) {
    atomicOr(&D.st->err, ERR_CHUNKS);
    c.c_ok = 0;
  }
  return c;
}

__device__ __forceinline__ void fl_slice(uint32_t beg, uint32_t end, uint32_t x, uint32_t& b0, uint32_t& b1) {
  const uint64_t len = end - beg;
  b0 = beg + static_cast<uint32_t>(len * x / FL_PG);
  b1 = beg + static_cast<uint32_t>(len * (x + 1) / FL_PG);
}

// Insert key into an open-addressed set of FL_HASH slots (read first, CAS only on an empty
// slot).  Returns the slot, or FL_HASH when the set is full.  *fresh = this call added it.
template <typename KeyPtr>
__device__ __forceinline__ uint32_t fl_set_put(KeyPtr keys, unsigned long long key, bool* fresh) {
  uint32_t s = fl_hash(key);
  *fresh = false;
  for (uint32_t probe = 0; probe < FL_HASH; ++probe) {
    const unsigned long long cur = *reinterpret_cast<volatile unsigned long long*>(&keys[s]);
    if (cur == key) return s;
    if (cur == 0ull) {
      const unsigned long long prev = atomicCAS(&keys[s], 0ull, key);
      if (prev == 0ull) {
        *fresh = true;
        return s;
      }
      if (prev == key) return s;
    }
    s = (s + 1) & (FL_HASH - 1);
  }
  return FL_HASH;
}

// fl_set_put for k_flow_prep_a's per-block sets, which only ever need FL_MAX + 1 keys: a probe
// chain longer than FL_PUT_PROBES counts as an overflow (FL_HASH), as does a block whose distinct
// count already passed FL_MAX.  A deep book fills the table with ~FL_HASH keys in its first
// round of inserts, and unbounded linear probing in that full table cost ~0.7 ms per batch.
// (A false overflow only sends a shallow book to the deep candidates: still exact.)
constexpr uint32_t FL_PUT_PROBES = 32;
__device__ __forceinline__ uint32_t fl_set_put_small(unsigned long long* keys, const uint32_t* ndist,
                                                     unsigned long long key, bool* fresh) {
  uint32_t s = fl_hash(key);
  *fresh = false;
  for (uint32_t probe = 0; probe < FL_PUT_PROBES; ++probe) {
    if (*reinterpret_cast<const volatile uint32_t*>(ndist) > FL_MAX) return FL_HASH;
    const unsigned long long cur = *reinterpret_cast<volatile unsigned long long*>(&keys[s]);
    if (cur == key) return s;
    if (cur == 0ull) {
      const unsigned long long prev = atomicCAS(&keys[s], 0ull, key);
      if (prev == 0ull) {
        *fresh = true;
        return s;
      }
      if (prev == key) return s;
    }
    s = (s + 1) & (FL_HASH - 1);
  }
  return FL_HASH;
}

__device__ __forceinline__ void fl_block_gcd_sum(unsigned long long& mg, unsigned long long& msum,
                                                 unsigned long long* wg, unsigned long long* ws) {
  for (int off = 32; off > 0; off >>= 1) {
    mg = fl_gcd(mg, __shfl_xor(mg, off));
    msum = min(msum + __shfl_xor(msum, off), FL_SUM_CAP);
  }
  if (lane_id() == 0) { wg[threadIdx.x >> 6] = mg; ws[threadIdx.x >> 6] = msum; }
  __syncthreads();
  mg = msum = 0;
  for (uint32_t w = 0; w < FL_PREP_T / 64; ++w) {
    mg = fl_gcd(mg, wg[w]);
    msum = min(msum + ws[w], FL_SUM_CAP);
  }
}

__global__ __launch_bounds__(FL_PREP_T) void k_flow_prep_a(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ unsigned long long hkey[FL_HASH];
  __shared__ uint32_t ndist, bad, adds, dropped, dels, many;
  __shared__ unsigned long long wg[FL_PREP_T / 64], ws[FL_PREP_T / 64];
  const uint32_t hb = blockIdx.y, h = F.h0 + hb, tid = threadIdx.x;
  if (h >= fl_hend(D, F) || !F.enabled) return;
  FlPrepScr* P = F.pscr + hb;
  const uint32_t seg = B.seg_order[h];
  uint32_t b0, b1;
  fl_slice(B.seg_start[seg], B.seg_start[seg + 1], blockIdx.x, b0, b1);
  for (uint32_t i = tid; i < FL_HASH; i += FL_PREP_T) hkey[i] = 0;
  if (tid == 0) ndist = bad = adds = dropped = dels = many = 0;
  __syncthreads();
  unsigned long long mg = 0, msum = 0;
  uint32_t my_adds = 0, my_drop = 0, my_bad = 0, my_dels = 0, my_many = 0, my_zero = 0;
  // (every thread stops once the block's distinct prices overflowed: a deep candidate, whose
  // own prep starts over)
  for (uint32_t c0 = b0 + tid; c0 < b1 && !my_bad && !my_many && *reinterpret_cast<volatile uint32_t*>(&ndist) <= FL_MAX;
       c0 += 4 * FL_PREP_T) {
    Prep qs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t b = c0 + u * FL_PREP_T;
      if (b < b1) qs[u] = prep_at(B, b);
      else qs[u].action = 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const Prep q = qs[u];
      if (q.action == GOME_DEL) { my_dels++; continue; }
      if (q.action != GOME_ADD) continue;
      my_adds++;
      if (!q.adm) { my_drop++; continue; }
      if (q.adm == ADM_V_CHECK) { my_bad = 1; break; }  // (Q7 candidates: serial kernels)
      my_zero += q.vol == 0 ? 1u : 0u;  // (Q6: k_flow_prep_b decides; gcd(g, 0) = g, the sum unchanged)
      const unsigned long long v = static_cast<unsigned long long>(q.vol);
      const double qd = static_cast<double>(v) / static_cast<double>(mg ? mg : 1);
      if (mg == 0 || static_cast<unsigned long long>(qd) * mg != v) mg = fl_gcd(mg, v);
      msum = min(msum + v, FL_SUM_CAP);
      bool fresh;
      const uint32_t sl = fl_set_put_small(hkey, &ndist, static_cast<unsigned long long>(q.price) + FL_KEY_OFF, &fresh);
      if (sl == FL_HASH || (fresh && atomicAdd(&ndist, 1u) >= FL_MAX)) { my_many = 1; break; }
    }
  }
  if (my_adds) atomicAdd(&adds, my_adds);
  if (my_drop) atomicAdd(&dropped, my_drop);
  if (my_dels) atomicAdd(&dels, my_dels);
  if (my_zero) atomicAdd(&P->zeros, my_zero);
  if (my_bad) bad = 1;
  if (my_many) many = 1;
  fl_block_gcd_sum(mg, msum, wg, ws);  // (synchronises the block)
  if (tid == 0) {
    P->pg[blockIdx.x] = mg;
    P->ps[blockIdx.x] = msum;
    if (adds) atomicAdd(&P->adds, adds);
    if (dropped) atomicAdd(&P->dropped, dropped);
    if (dels) atomicAdd(&P->dels, dels);
    if (bad) atomicOr(&P->bad, 1u);
    if (many) atomicOr(&P->many, 1u);
  }
  if (bad || many) return;
  for (uint32_t i = tid; i < FL_HASH; i += FL_PREP_T) {
    if (hkey[i]) {
      bool fresh;
      if (fl_set_put(P->key, hkey[i], &fresh) == FL_HASH) atomicOr(&P->many, 1u);  // (a deep candidate)
    }
  }
}

__global__ __launch_bounds__(FL_PREP_T) void k_flow_prep_b(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ unsigned long long hkey[FL_HASH];
  __shared__ uint32_t hval[FL_HASH];
  __shared__ unsigned long long ckey[FL_CAP + FL_PREP_T];
  __shared__ uint32_t cslot[FL_CAP + FL_PREP_T];
  __shared__ uint32_t ndist, nc, bad, deepc, nstale, nzlev;
  __shared__ unsigned long long wg[FL_PREP_T / 64], ws[FL_PREP_T / 64];
  const uint32_t hb = blockIdx.x, h = F.h0 + hb, tid = threadIdx.x;
  if (h >= fl_hend(D, F)) return;
  FlowHdr* hd = &F.hdr[h];
  FlPrepScr* P = F.pscr + hb;
  const uint32_t seg = B.seg_order[h];
  const uint32_t beg = B.seg_start[seg], end = B.seg_start[seg + 1];
  const uint32_t sym = B.ord[B.sidx[beg]].symbol_id;
  if (D.st->err & ERR_INPUT) {  // (the batch is rejected; sym may be out of range)
    if (tid == 0) { hd->ok = 0; hd->deep = 0; hd->bail = 0; }
    return;
  }
  const Book bk = D.books[sym];
  // Stale side-set members (Q2): a wrong-side cancel that empties a level ZREMs the
  // request's side set, so the level stays in its true side's set with no FIFO and depth 0.  A
  // taker that reaches it in the reference finds no node and moves on (MatchOrder returns at an
  // empty FIFO, engine.go:139-142), and a same-side rest there is an ordinary rest: the plans,
  // which see a depth of 0 as "no level", are exact for both.  Only an order resting on the OTHER
  // side at that price is not (the level would be a member of both sets), which
  // k_flow_stale_check finds after the plan: the book then goes to the legacy kernel
  // (k_match_hot mode 1).  Head books of at least LEGACY_HOT_MIN orders only (the cold kernel
  // never takes such a book, so a late hand-over cannot race with it); with DELs, the cancel path
  // also takes wrong-side cancels that make such a level (k_fc_resolve, k_fc_stale_level).
  // Zero-volume ADDs (Q6) under the same conditions: one that crosses takes 0 at the best opposite
  // level, the reference's one 0-fill with the maker unchanged (engine.go:176-194), which the plans
  // log as a CONS touch of 0; one that rests leaves a zero-volume maker in the FIFO, which the
  // reconstruction does not model: k_flow_zero_check finds its REST of 0 and hands the book over.
  // With DELs (the cancel path) a zero-volume taker or a DEL of a zero-volume maker hands it over
  // too (k_flow_zero_check, k_fc_resolve).
  const bool stale_ok = (end - beg) >= LEGACY_HOT_MIN, zero_ok = stale_ok;
  if (tid == 0) {
    ndist = nc = nstale = nzlev = 0;
    const bool base_bad = !F.enabled || P->bad || (bk.pad & BOOK_QUIRK) || (D.st->err & ERR_INPUT) ||
                          ((P->zeros || (bk.pad & BOOK_ZERO)) && !zero_ok) ||
                          (end - beg) >= FL_MAX_ORDERS;
    const bool many = P->many || bk.n_lvl > FL_MAX;
    // more levels than lanes: the deep plan's candidate (match_flow_deep.h re-checks the rest)
    deepc = (!base_bad && many && bk.n_lvl <= DEEP_CAP - 2) ? 1u : 0u;
    if (deepc) ctr_add(D, C_WANT_DEEP, 1ull);
    if (!(F.chains & FL_CH_DEEP)) deepc = 0;
    bad = (base_bad || many) ? 1u : 0u;
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) {
      hd->ok = 0;
      hd->bail = 0;
      hd->deep = deepc;
      hd->dslot = h;
      if (deepc) F.dslot_h[h] = h;
    }
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
  // live levels of the book (as k_flow_prep)
  const Level* L0 = D.lvl + bk.lvl_base;
  unsigned long long mg = 0, msum = 0;
  if (tid < FL_PG) {
    mg = P->pg[tid];
    msum = P->ps[tid];
  }
  for (uint32_t k = tid; k < bk.n_lvl; k += FL_PREP_T) {
    const Level x = L0[k];
    const uint32_t nm = (x.member & M_BUY ? 1u : 0u) + (x.member & M_SALE ? 1u : 0u);
    if (x.nlive == 0) {
      const bool stale = stale_ok && x.depth == 0 && nm == 1 && x.head == NIL;
      if (!stale) {
        if (x.depth != 0 || x.member != 0) bad = 1;
        continue;
      }
      atomicAdd(&nstale, 1u);  // (in the table, so a rest at its price lands in this level)
    } else {
      if (x.depth <= 0 || nm != 1) { bad = 1; continue; }
      mg = fl_gcd(mg, static_cast<unsigned long long>(x.depth));
      msum = min(msum + static_cast<unsigned long long>(x.depth), FL_SUM_CAP);
    }
    bool fresh;
    const uint32_t sl = fl_set_put(hkey, static_cast<unsigned long long>(x.price) + FL_KEY_OFF, &fresh);
    if (sl == FL_HASH) { bad = 1; continue; }
    hval[sl] = k;
    if (fresh) atomicAdd(&ndist, 1u);
  }
  fl_block_gcd_sum(mg, msum, wg, ws);  // (synchronises the block)
  if (bad || ndist > FL_MAX) {
    if (tid == 0) {
      hd->ok = 0;
      hd->bail = 0;
      hd->deep = (!bad && ndist <= DEEP_CAP - 2) ? 1u : 0u;
      if (hd->deep) ctr_add(D, C_WANT_DEEP, 1ull);
      if (!(F.chains & FL_CH_DEEP)) hd->deep = 0;
      hd->dslot = h;
      if (hd->deep) F.dslot_h[h] = h;
    }
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
  FlowLvl* LV = F.lvl + h * FL_CAP;
  if (tid < n) {
    const unsigned long long key = ckey[tid];
    uint32_t r = 0;
    for (uint32_t i = 0; i < n; ++i) r += ckey[i] < key ? 1u : 0u;
    const uint32_t sl = cslot[tid], old = hval[sl];
    FlowLvl f{};
    f.price = static_cast<int64_t>(key - FL_KEY_OFF);
    f.old = old;
    f.head = f.tail = NIL;
    f.ig_base = 0;
    if (old != NIL) {
      const Level x = L0[old];
      f.d0 = x.depth;
      f.nv0 = x.nlive;
      f.head = x.head;
      f.tail = x.tail;
      f.hslot = x.hslot;
      f.tslot = x.tslot;
      f.mem0 = x.member;
      f.z0 = (bk.pad & BOOK_ZERO) ? x.pad : 0u;
      if (f.z0) atomicAdd(&nzlev, 1u);
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
  const uint32_t dels = P->dels;
  // (the cancel plan needs every depth and Q < 2^31: its DEL path clamps with signed arithmetic)
  const bool w32 = msum < FL_SUM_CAP && msum / g < (dels ? (1ull << 31) : (1ull << 32));
  if (!w32) g = 1;
  if (dels && !w32) {  // the cancel plan is 32-bit only
    if (tid == 0) { hd->ok = 0; hd->deep = 0; hd->bail = 0; }
    return;
  }
  const uint32_t obase = fl_obase(beg, seg);
  if (tid < ((8u - ((end - beg) & 7u)) & 7u))  // padding to whole half-groups (8 records)
    F.ord8[obase + (end - beg) + tid] = fl_rec(false, 0, 0, false, end - beg + tid, w32);
  if (tid == 0) {
    FlowHdr x{};
    if (dels) ctr_add(D, C_WANT_CANC, 1ull);
    x.ok = dels ? ((F.chains & FL_CH_CANCEL) ? FL_OK_CANCEL : 0u) : FL_OK_ADD;
    x.nl = n;
    x.sym = sym;
    x.beg = beg;
    x.end = end;
    x.nold = bk.n_lvl;
    x.adds = P->adds;
    x.dropped = P->dropped;
    x.obase = obase;
    x.w32 = w32 ? 1u : 0u;
    x.g = g;
    x.ndel = dels;
    x.bid = F.bid;
    x.nstale = nstale;
    x.nzero = P->zeros;
    x.nzlev = nzlev;
    if (nstale) ctr_add(D, C_FLOW_STALE, 1ull);
    if (x.nzero || nzlev) ctr_add(D, C_FLOW_ZERO, 1ull);
    *hd = x;
  }
}

__global__ __launch_bounds__(FL_PREP_T) void k_flow_prep_c(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ unsigned long long hkey[FL_HASH];
  __shared__ uint32_t hval[FL_HASH];
  const uint32_t hb = blockIdx.y, h = F.h0 + hb, tid = threadIdx.x;
  if (h >= fl_hend(D, F) || !uni(F.hdr[h].ok)) return;
  const FlPrepScr* P = F.pscr + hb;
  const FlowHdr* hd = &F.hdr[h];
  const uint32_t beg = hd->beg, obase = hd->obase;
  const bool w32 = hd->w32 != 0;
  const unsigned long long g = hd->g;
  uint32_t b0, b1;
  fl_slice(beg, hd->end, blockIdx.x, b0, b1);
  for (uint32_t i = tid; i < FL_HASH; i += FL_PREP_T) {
    hkey[i] = P->key[i];
    hval[i] = P->val[i];
  }
  __syncthreads();
  for (uint32_t c0 = b0 + tid; c0 < b1; c0 += 4 * FL_PREP_T) {
    Prep qs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t b = c0 + u * FL_PREP_T;
      if (b < b1) qs[u] = prep_at(B, b);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t b = c0 + u * FL_PREP_T;
      if (b >= b1) break;
      const Prep q = qs[u];
      unsigned long long rec = fl_rec(false, 0, 0, false, b - beg, w32);
      if (q.action == GOME_ADD && q.adm) {
        const unsigned long long key = static_cast<unsigned long long>(q.price) + FL_KEY_OFF;
        uint32_t s = fl_hash(key);
        while (hkey[s] != key) s = (s + 1) & (FL_HASH - 1);
        const uint32_t li = hval[s];
        const unsigned long long v = w32 ? static_cast<unsigned long long>(static_cast<double>(q.vol) / static_cast<double>(g))
                                         : static_cast<unsigned long long>(q.vol);
        rec = fl_rec(true, li, v, q.side == GOME_SALE, b - beg, w32);
      }
      F.ord8[obase + (b - beg)] = rec;
      B.ev_count[q.idx] = 0;
    }
  }
}

// ============================================================== k_flow_plan (serial)
// One wave per flow book; everything per order is wave-uniform (SALU + lane reads/writes):
//   * depth of level k: lane k % 64 of the 64-bit lane pair D[k / 64] (two register sets);
//   * S:SALE / S:BUY membership: 128-bit scalar masks A, Bm.  Slot 127 is a permanent ask
//     and slot 0 a permanent bid (sentinels), so "best opposite level" is one bit scan and
//     "does it cross" one compare, with no emptiness test;
//   * orders: 8-B packed records read 8 at a time through the scalar cache (s_load_dwordx16,
//     prefetched one group ahead), so no vector-memory wait sits on the order path;
//   * the log: lane `nacc` of four staging VGPRs per touch (v_writelane), stored 64 touches
//     at a time (fire and forget: nothing on the path ever waits for vector memory).
typedef const __attribute__((address_space(4))) unsigned long long* fl_cptr;
struct alignas(64) FlGroup {
  unsigned long long o[8];
};

// r = a - b on 64-bit scalars; returns the borrow (a < b, unsigned) from SCC.
__device__ __forceinline__ uint32_t fl_sub64(uint32_t alo, uint32_t ahi, uint32_t blo, uint32_t bhi,
                                             uint32_t& rlo, uint32_t& rhi) {
  uint32_t br;
  asm volatile("s_sub_u32 %0, %3, %5\n\ts_subb_u32 %1, %4, %6\n\ts_cselect_b32 %2, 1, 0"
               : "=&s"(rlo), "=&s"(rhi), "=&s"(br)
               : "s"(alo), "s"(ahi), "s"(blo), "s"(bhi)
               : "scc");
  return br;
}

// r = a + b on 64-bit scalars.
__device__ __forceinline__ void fl_add64(uint32_t alo, uint32_t ahi, uint32_t blo, uint32_t bhi,
                                         uint32_t& rlo, uint32_t& rhi) {
  asm volatile("s_add_u32 %0, %2, %4\n\ts_addc_u32 %1, %3, %5"
               : "=&s"(rlo), "=&s"(rhi)
               : "s"(alo), "s"(ahi), "s"(blo), "s"(bhi)
               : "scc");
}

struct FlDepth {  // depths of levels 0..127 as four 32-bit lane registers
  uint32_t l0, h0, l1, h1;
};

// Read level k; old values of lane k % 64 of both sets are returned for the write-back.
__device__ __forceinline__ void fl_dget(const FlDepth& D, uint32_t k, uint32_t& lo, uint32_t& hi, uint32_t (&o)[4]) {
  const uint32_t kl = k & 63u;
  o[0] = rl(D.l0, kl);
  o[1] = rl(D.h0, kl);
  o[2] = rl(D.l1, kl);
  o[3] = rl(D.h1, kl);
  lo = k < 64 ? o[0] : o[2];
  hi = k < 64 ? o[1] : o[3];
}

// Write level k (the other set's lane gets its old value back: no branch, no exec mask).
__device__ __forceinline__ void fl_dset(FlDepth& D, uint32_t k, uint32_t lo, uint32_t hi, const uint32_t (&o)[4]) {
  const uint32_t kl = k & 63u;
  const bool s0 = k < 64;
  D.l0 = wl_u32(D.l0, s0 ? lo : o[0], kl);
  D.h0 = wl_u32(D.h0, s0 ? hi : o[1], kl);
  D.l1 = wl_u32(D.l1, s0 ? o[2] : lo, kl);
  D.h1 = wl_u32(D.h1, s0 ? o[3] : hi, kl);
}

__device__ __forceinline__ uint32_t fl_lowest(unsigned long long m0, unsigned long long m1) {
  return m0 ? static_cast<uint32_t>(__builtin_ctzll(m0)) : 64u + static_cast<uint32_t>(__builtin_ctzll(m1));
}
__device__ __forceinline__ uint32_t fl_highest(unsigned long long m0, unsigned long long m1) {
  return m1 ? 127u - static_cast<uint32_t>(__builtin_clzll(m1)) : 63u - static_cast<uint32_t>(__builtin_clzll(m0));
}

struct FlLog {
  uint32_t lk, la, lb, pad;  // staging lanes
  uint32_t nacc, lpos, lcap;
  GOME_GLB v4u* p;
};

#include "flow_plan_asm.inc"
static_assert(FL_DEEP_CAP == DEEP_CAP, "deep plan generated for another DEEP_CAP");
static_assert(FL_DEEP_BM == DEEP_CAP * 8 && FL_DEEP_LDS <= 160 * 1024, "deep plan LDS layout");
// W32DV's LDS: the words (word k at 4k), then FL_DV_HDR words: the cached tops and their depths
// (ask, bid, ask depth, bid depth) and the summary (FL_DEEP_NVL / 64 / 32 lanes)
constexpr uint32_t FL_DV_HDR = 4 + FL_DEEP_NVL / 2048;
static_assert((FL_DEEP_NVL + FL_DV_HDR) * 4 <= FL_DEEP_LDS && FL_DEEP_NVL <= DEEP_CAP, "VGPR deep plan's word array");
#ifndef GOME_DEEP_LDS_ONLY
constexpr bool FL_DEEP_VGPR = true;   // W32DV (depths in VGPRs) for ADD-only deep books that fit
#else
constexpr bool FL_DEEP_VGPR = false;  // (variant build: every deep book on the LDS plan)
#endif

// Does deep book h take the VGPR plan (gen_plan_asm.py W32DV, W32DVC with DELs)?  Its levels and
// the two sentinels within the FL_DEEP_NVL words.
__device__ __forceinline__ bool fl_deep_vgpr(const FlowHdr& hd) {
  return FL_DEEP_VGPR && hd.nl + 2 <= FL_DEEP_NVL;
}



__device__ __forceinline__ void fl_plan_book(const Dev& D, const FlowArgs& F, uint32_t h);
#ifdef GOME_STAMPS
// Diagnostic build only: per head book {shader cycles, 100 MHz ticks, orders, touches} of the
// plan loop (read with gome_debug_stamps after the hot-kernel stamps).
__device__ unsigned long long g_pstamps[FL_HEAD * 4];
#endif

// EXCL: the block is 4 waves that each hold the whole register file of their SIMD (all 512
// VGPR+AGPR), so no other wave can share the CU — in particular not its scalar unit, which
// every instruction of the plan's critical path uses.  Waves 1-3 park at the barrier.
extern __shared__ uint4 fl_ring[];  // the deep plan's depth slots and bitmaps (dynamic LDS)

// Deep books: the depth slots (W32 units; bid of level k at byte 8k, ask at 8k + 4) -> LDS by
// every thread of the block, with the sentinels; back to FlowLvl (dfin, memf) after the plan.
__device__ __forceinline__ void fl_deep_load(const FlowArgs& F, uint32_t h) {
  uint32_t* dep = reinterpret_cast<uint32_t*>(fl_ring);
  const FlowHdr& hd = F.hdr[h];
  const FlowLvl* LV = fl_lvls(F, h);
  const unsigned long long g = hd.g;
  if (fl_deep_vgpr(hd)) {  // W32DV: one word per level (a clean book's bids lie below its asks)
    uint32_t* hw = dep + FL_DEEP_NVL;
    if (threadIdx.x < FL_DV_HDR) hw[threadIdx.x] = threadIdx.x == 0 ? FL_DEEP_NVL - 1 : 0u;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < FL_DEEP_NVL; k += blockDim.x) {
      uint32_t w = (k == 0 || k == FL_DEEP_NVL - 1) ? 1u : 0u;  // the sentinels
      if (k >= 1 && k <= hd.nl) {
        const FlowLvl& f = LV[k];
        if (f.mem0 & (M_SALE | M_BUY)) w = static_cast<uint32_t>(static_cast<unsigned long long>(f.d0) / g);
        if (w && (f.mem0 & M_SALE)) atomicMin(&hw[0], k);  // the best ask / bid: the cached tops
        if (w && (f.mem0 & M_BUY)) atomicMax(&hw[1], k);
      }
      dep[k] = w;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // the tops' depths leave their words (the plan's invariant)
      hw[2] = dep[hw[0]];
      hw[3] = dep[hw[1]];
      dep[hw[0]] = 0;
      dep[hw[1]] = 0;
    }
    __syncthreads();
    // the summary: bit r % 32 of word r / 32 = register r (words 64r .. 64r + 63) is nonzero
    for (uint32_t r = threadIdx.x; r < FL_DEEP_NVL / 64; r += blockDim.x) {
      uint32_t nz = 0;
      for (uint32_t i = 0; i < 64; ++i) nz |= dep[64 * r + i];
      if (nz) atomicOr(&hw[4 + r / 32], 1u << (r % 32));
    }
    return;
  }
  for (uint32_t k = threadIdx.x; k < DEEP_CAP; k += blockDim.x) {
    uint32_t a = 0, b = 0;
    if (k >= 1 && k <= hd.nl) {
      const FlowLvl& f = LV[k];
      const uint32_t d = static_cast<uint32_t>(static_cast<unsigned long long>(f.d0) / g);
      if (f.mem0 & M_SALE) a = d;
      if (f.mem0 & M_BUY) b = d;
    }
    if (k == 0) b = 1;
    if (k == DEEP_CAP - 1) a = 1;
    dep[2 * k] = b;
    dep[2 * k + 1] = a;
  }
  // the plan's occupancy bitmaps (bit k of dword k >> 5: slot k != 0), bids then asks
  __syncthreads();
  uint32_t* bm = dep + FL_DEEP_BM / 4;
  const uint32_t lane = lane_id();
  for (uint32_t k0 = (threadIdx.x & ~63u); k0 < DEEP_CAP; k0 += blockDim.x) {
    const unsigned long long mb = __ballot(dep[2 * (k0 + lane)] != 0);
    const unsigned long long ma = __ballot(dep[2 * (k0 + lane) + 1] != 0);
    if (lane < 2) {
      bm[(k0 >> 5) + lane] = static_cast<uint32_t>(mb >> (32 * lane));
      bm[DEEP_CAP / 32 + (k0 >> 5) + lane] = static_cast<uint32_t>(ma >> (32 * lane));
    }
  }
}

__device__ __forceinline__ void fl_deep_store(const FlowArgs& F, uint32_t h) {
  const uint32_t* dep = reinterpret_cast<const uint32_t*>(fl_ring);
  const FlowHdr& hd = F.hdr[h];
  FlowLvl* LV = fl_lvls(F, h);
  const unsigned long long g = hd.g;
  if (fl_deep_vgpr(hd)) {  // W32DV: asks lie at or above the final best ask
    const uint32_t ba = hd.dv_ba;
    for (uint32_t k = 1 + threadIdx.x; k <= hd.nl; k += blockDim.x) {
      const uint32_t w = dep[k];
      LV[k].dfin = static_cast<int64_t>(static_cast<unsigned long long>(w) * g);
      LV[k].memf = w ? (k >= ba ? M_SALE : M_BUY) : 0u;
    }
    return;
  }
  for (uint32_t k = 1 + threadIdx.x; k <= hd.nl; k += blockDim.x) {
    const uint32_t b = dep[2 * k], a = dep[2 * k + 1];
    LV[k].dfin = static_cast<int64_t>(static_cast<unsigned long long>(a + b) * g);  // (one side is 0)
    LV[k].memf = (a ? M_SALE : 0u) | (b ? M_BUY : 0u);
  }
}

template <bool EXCL>
__device__ __forceinline__ void fl_plan_kernel(const Dev& D, const FlowArgs& F, uint32_t kind) {
  const uint32_t h = F.h0 + blockIdx.x;
  const bool mine = h < fl_hend(D, F) && uni(F.hdr[h].ok) == kind && !uni(F.hdr[h].pre);
  if (mine && kind == FL_OK_DEEP) fl_deep_load(F, h);
  if (EXCL) {
    asm volatile("" ::: "v255", "a255");
    __syncthreads();
    if (threadIdx.x < 64 && mine) fl_plan_book(D, F, h);
    __syncthreads();
    if (mine && kind == FL_OK_DEEP) fl_deep_store(F, h);
    return;
  }
  if (mine) fl_plan_book(D, F, h);
}

// The head's plan (the batch's critical path) and the tail's: distinct names for the profiles.
// (The head kernels plan either kind of book: their block owns the CU and its LDS anyway.)
__global__ __launch_bounds__(256) void k_flow_plan_head(Dev D, FlowArgs F) {
  fl_plan_kernel<true>(D, F, uni(F.hdr[F.h0 + blockIdx.x < fl_hend(D, F) ? F.h0 + blockIdx.x : 0].ok));
}
// the hottest book planned early (match_early.h: right after the batch before's plan)
__global__ __launch_bounds__(256) void k_flow_plan_early(Dev D, FlowArgs F) {
  fl_plan_kernel<true>(D, F, uni(F.hdr[F.h0 + blockIdx.x < fl_hend(D, F) ? F.h0 + blockIdx.x : 0].ok));
}
// the other head books (planned on the tail's stream, beside the hottest)
__global__ __launch_bounds__(256) void k_flow_plan_near(Dev D, FlowArgs F) {
  fl_plan_kernel<true>(D, F, uni(F.hdr[F.h0 + blockIdx.x < fl_hend(D, F) ? F.h0 + blockIdx.x : 0].ok));
}
__global__ __launch_bounds__(64) void k_flow_plan_tail(Dev D, FlowArgs F) { fl_plan_kernel<false>(D, F, FL_OK_ADD); }
// tail books with DELs
__global__ __launch_bounds__(64) void k_flow_plan_tail_c(Dev D, FlowArgs F) { fl_plan_kernel<false>(D, F, FL_OK_CANCEL); }
// deep tail books (depths in LDS: a whole CU each, like the head): each block walks the tail's
// deep slots (handed out by k_flow_prep) in turn
__global__ __launch_bounds__(256) void k_flow_plan_tail_d(Dev D, FlowArgs F) {
  const uint32_t n = min(F.ds1 - F.ds0, *F.dslot_n);
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t h = F.dslot_h[F.ds0 + i];
    const bool mine = h != NIL && h < fl_hend(D, F) && F.hdr[h].ok == FL_OK_DEEP && F.hdr[h].dslot == F.ds0 + i;
    if (mine) fl_deep_load(F, h);
    asm volatile("" ::: "v255", "a255");
    __syncthreads();
    if (threadIdx.x < 64 && mine) fl_plan_book(D, F, h);
    __syncthreads();
    if (mine) fl_deep_store(F, h);
    __syncthreads();
  }
}

__device__ __forceinline__ void fl_plan_deep(const Dev& D, const FlowArgs& F, uint32_t h);

__device__ __forceinline__ void fl_plan_book(const Dev& D, const FlowArgs& F, uint32_t h) {
  const FlowHdr* hd = &F.hdr[h];
  if (uni(hd->ok) == FL_OK_DEEP) {
    fl_plan_deep(D, F, h);
    return;
  }
  __builtin_amdgcn_s_setprio(3);
  const uint32_t lane = lane_id();
  const uint32_t nl = uni(hd->nl), beg = uni(hd->beg), end = uni(hd->end), n = end - beg;
  FlowLvl* LV = F.lvl + h * FL_CAP;
  const bool v0 = lane >= 1 && lane <= nl, v1 = lane + 64 <= nl;
  const bool w32 = uni(hd->w32) != 0;
  const unsigned long long g = static_cast<unsigned long long>(uni64(static_cast<int64_t>(hd->g)));
  const uint32_t m0 = v0 ? LV[lane].mem0 : 0u, m1 = v1 ? LV[lane + 64].mem0 : 0u;
  // Bids and asks have lane registers of their own, and the loop's invariant is that a lane
  // holds 0 unless its level rests on that side (membership = nonzero lane).  The sentinel
  // levels 0 (bid) and 127 (ask) are nonzero lanes.
  int64_t d0 = v0 ? LV[lane].d0 : 0, d1 = v1 ? LV[lane + 64].d0 : 0;
  if (w32) {  // depths in units of g (exact: g divides every volume and depth of the book)
    d0 = static_cast<int64_t>(static_cast<unsigned long long>(d0) / g);
    d1 = static_cast<int64_t>(static_cast<unsigned long long>(d1) / g);
  }
  const int64_t a0 = (m0 & M_SALE) ? d0 : 0, a1 = (m1 & M_SALE) ? d1 : (lane == 63 ? 1 : 0);
  const int64_t b0 = (m0 & M_BUY) ? d0 : (lane == 0 ? 1 : 0), b1 = (m1 & M_BUY) ? d1 : 0;
  FlDepth Da{lo32(a0), hi32(a0), lo32(a1), hi32(a1)}, Db{lo32(b0), hi32(b0), lo32(b1), hi32(b1)};
  if (w32) {  // the 32-bit plan's layout: lane j holds levels 2j (l0) and 2j + 1 (l1)
    const uint32_t se = (2u * lane) & 63u, so = (2u * lane + 1u) & 63u;
    const bool hiset = lane >= 32;
    auto pick = [&](uint32_t x0, uint32_t x1, uint32_t src) {
      const uint32_t v0 = __shfl(x0, src), v1 = __shfl(x1, src);
      return hiset ? v1 : v0;
    };
    Da = FlDepth{pick(Da.l0, Da.l1, se), 0u, pick(Da.l0, Da.l1, so), 0u};
    Db = FlDepth{pick(Db.l0, Db.l1, se), 0u, pick(Db.l0, Db.l1, so), 0u};
  }

  const uint32_t lb = F.xlog ? 0u : FL_TOUCH_MUL * beg;  // (the early plan logs into a buffer of its own)
  FlLog lg{vreg(0u), vreg(0u), vreg(0u), 0u, 0u, 0u, FL_TOUCH_MUL * n, (GOME_GLB v4u*)(F.log + lb)};
  // records are read in half-groups of 8 (the book's stream is padded to whole groups)
  const uint32_t nh = (n + 7) / 8;
  const unsigned long long ob = reinterpret_cast<unsigned long long>(F.ord8 + uni(hd->obase));
  const unsigned long long logp = reinterpret_cast<unsigned long long>(F.log + lb);
  const uint32_t vl16 = lane * 16u;
  uint32_t voff, vt, vpf;
  const uint32_t vzero = 0;
#define FL_PLAN_OPERANDS                                                                          \
  : [al0] "+v"(Da.l0), [ah0] "+v"(Da.h0), [al1] "+v"(Da.l1), [ah1] "+v"(Da.h1), [bl0] "+v"(Db.l0),     \
    [bh0] "+v"(Db.h0), [bl1] "+v"(Db.l1), [bh1] "+v"(Db.h1), [lk] "+v"(lg.lk), [la] "+v"(lg.la),         \
    [lb] "+v"(lg.lb),                                                                                 \
    [nacc] "+s"(lg.nacc), [lpos] "+s"(lg.lpos), [voff] "=&v"(voff), [vt] "=&v"(vt), [vpf] "=&v"(vpf)    \
  : [ob] "s"(ob), [nh] "s"(nh), [logp] "s"(logp), [lcap] "s"(lg.lcap), [vl16] "v"(vl16),              \
    [vzero] "v"(vzero)                                                                                  \
  : FL_PLAN_CLOBBERS, "scc", "vcc", "memory"
#ifdef GOME_STAMPS
  const unsigned long long sc0 = __builtin_amdgcn_s_memtime(), sr0 = __builtin_amdgcn_s_memrealtime();
#endif
  if (uni(hd->ok) == FL_OK_CANCEL) {
    asm volatile(FL_PLAN_ASM32C
      : [al0] "+v"(Da.l0), [ah0] "+v"(Da.h0), [al1] "+v"(Da.l1), [ah1] "+v"(Da.h1), [bl0] "+v"(Db.l0),
        [bh0] "+v"(Db.h0), [bl1] "+v"(Db.l1), [bh1] "+v"(Db.h1), [lk] "+v"(lg.lk), [la] "+v"(lg.la),
        [lb] "+v"(lg.lb), [nacc] "+s"(lg.nacc), [lpos] "+s"(lg.lpos), [voff] "=&v"(voff), [vt] "=&v"(vt),
        [vpf] "=&v"(vpf)
      : [ob] "s"(ob), [nh] "s"(nh), [logp] "s"(logp), [lcap] "s"(lg.lcap), [vl16] "v"(vl16),
        [vzero] "v"(vzero)
      : FL_PLAN_CLOBBERS, FL_PLAN_CLOBBERS_C, "scc", "vcc", "memory");
  } else if (w32) {
    asm volatile(FL_PLAN_ASM32 FL_PLAN_OPERANDS);
  } else {
    asm volatile(FL_PLAN_ASM64 FL_PLAN_OPERANDS);
  }
#undef FL_PLAN_OPERANDS
#ifdef GOME_STAMPS
  const unsigned long long sc1 = __builtin_amdgcn_s_memtime(), sr1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && h < FL_HEAD) {
    g_pstamps[h * 4 + 0] = sc1 - sc0;
    g_pstamps[h * 4 + 1] = sr1 - sr0;
    g_pstamps[h * 4 + 2] = n;
    g_pstamps[h * 4 + 3] = lg.lpos + lg.nacc;
  }
#endif
  if (lg.nacc) {
    if (lane < lg.nacc && lg.lpos + lg.nacc <= lg.lcap) lg.p[lg.lpos + lane] = v4(lg.lk, 0u, lg.la, lg.lb);
    lg.lpos += lg.nacc;
  }
  if (lg.lpos > lg.lcap) {  // cannot happen (touch bound); never read past the log
    if (lane == 0) atomicOr(&D.st->err, ERR_CORRUPT);
    lg.lpos = 0;
  }
  // side sets from the nonzero lanes (the sentinel bits 127 / 0 are set, as the write kernels
  // expect); a level rests on at most one side, so its final depth is the sum of its lanes
  auto u64of = [&](uint32_t lo, uint32_t hi) -> uint64_t {
    return w32 ? static_cast<uint64_t>(lo) * g : (static_cast<uint64_t>(hi) << 32) | lo;
  };
  if (w32) {  // back to level k -> lane k % 64 of set k / 64
    auto level = [&](uint32_t ev, uint32_t od, uint32_t k) {
      const uint32_t e = __shfl(ev, (k >> 1) & 63u), o = __shfl(od, (k >> 1) & 63u);
      return (k & 1u) ? o : e;
    };
    const uint32_t a_lo = level(Da.l0, Da.l1, lane), a_hi = level(Da.l0, Da.l1, lane + 64);
    const uint32_t b_lo = level(Db.l0, Db.l1, lane), b_hi = level(Db.l0, Db.l1, lane + 64);
    Da = FlDepth{a_lo, 0u, a_hi, 0u};
    Db = FlDepth{b_lo, 0u, b_hi, 0u};
  }
  const uint64_t ua0 = u64of(Da.l0, Da.h0), ua1 = u64of(Da.l1, Da.h1);
  const uint64_t ub0 = u64of(Db.l0, Db.h0), ub1 = u64of(Db.l1, Db.h1);
  const unsigned long long A0 = __ballot(ua0 != 0) & ~1ull, A1 = __ballot(ua1 != 0) | (1ull << 63);
  const unsigned long long B0 = __ballot(ub0 != 0) | 1ull, B1 = __ballot(ub1 != 0) & ~(1ull << 63);
  const int64_t f0 = lane == 0 ? 0 : static_cast<int64_t>(ua0 + ub0);
  const int64_t f1 = lane == 63 ? 0 : static_cast<int64_t>(ua1 + ub1);
  if (v0) LV[lane].dfin = f0;
  if (v1) LV[lane + 64].dfin = f1;
  if (lane == 0) {
    FlowHdr* w = &F.hdr[h];
    w->ntouch = lg.lpos;
    w->amask[0] = A0;
    w->amask[1] = A1;
    w->bmask[0] = B0;
    w->bmask[1] = B1;
  }
}

// The deep plan (gen_plan_asm.py, W32D): depths in LDS (fl_deep_load), touches carry their level
// in the second word.
__device__ __forceinline__ void fl_plan_deep(const Dev& D, const FlowArgs& F, uint32_t h) {
  const FlowHdr* hd = &F.hdr[h];
  __builtin_amdgcn_s_setprio(3);
  const uint32_t lane = lane_id();
  const uint32_t beg = uni(hd->beg), end = uni(hd->end), n = end - beg;
  const uint32_t lb = F.xlog ? 0u : FL_TOUCH_MUL * beg;  // (the early plan logs into a buffer of its own)
  FlLog lg{vreg(0u), vreg(0u), vreg(0u), 0u, 0u, 0u, FL_TOUCH_MUL * n, (GOME_GLB v4u*)(F.log + lb)};
  const uint32_t nh = (n + 7) / 8;
  const unsigned long long ob = reinterpret_cast<unsigned long long>(F.ord8 + uni(hd->obase));
  const unsigned long long logp = reinterpret_cast<unsigned long long>(F.log + lb);
  const uint32_t vl16 = lane * 16u;
  uint32_t voff, vpf;
  const uint32_t vzero = 0;
  // the plan's group summaries (lane i bit j: group 32i + j of 32 levels holds a nonzero slot of
  // that side), from the bitmaps fl_deep_load built
  const uint32_t* bm = reinterpret_cast<const uint32_t*>(fl_ring) + FL_DEEP_BM / 4;
  uint32_t sb = 0, sa = 0;
  if (lane < DEEP_CAP / 1024)
    for (uint32_t j = 0; j < 32; ++j) {
      sb |= (bm[32 * lane + j] != 0 ? 1u : 0u) << j;
      sa |= (bm[DEEP_CAP / 32 + 32 * lane + j] != 0 ? 1u : 0u) << j;
    }
  if (fl_deep_vgpr(*hd)) {  // W32DV: the words from LDS into VGPRs inside the asm, tops as operands
    // the cached tops, their depths and the summary, from fl_deep_load
    const uint32_t* hw = reinterpret_cast<const uint32_t*>(fl_ring) + FL_DEEP_NVL;
    const uint32_t ba = uni(hw[0]), bb = uni(hw[1]), bad = uni(hw[2]), bbd = uni(hw[3]);
    const uint32_t sv = lane < FL_DEEP_NVL / 2048 ? hw[4 + lane] : 0u;
    uint32_t oba, obb;
#define FL_DV_OPERANDS                                                                                        \
  : [lk] "+v"(lg.lk), [la] "+v"(lg.la), [lb] "+v"(lg.lb), [nacc] "+s"(lg.nacc), [lpos] "+s"(lg.lpos),         \
    [voff] "=&v"(voff), [vpf] "=&v"(vpf), [oba] "=s"(oba), [obb] "=s"(obb)                                     \
  : [ob] "s"(ob), [nh] "s"(nh), [logp] "s"(logp), [lcap] "s"(lg.lcap), [vl16] "v"(vl16), [vzero] "v"(vzero), \
    [sv] "v"(sv), [ba] "s"(ba), [bb] "s"(bb), [bad] "s"(bad), [bbd] "s"(bbd)                                   \
  : FL_PLAN_CLOBBERS, FL_PLAN_CLOBBERS_DV, "scc", "vcc", "memory"
    if (uni(hd->dc)) {
      asm volatile(FL_PLAN_ASM32DVC FL_DV_OPERANDS);
    } else {
      asm volatile(FL_PLAN_ASM32DV FL_DV_OPERANDS);
    }
#undef FL_DV_OPERANDS
    if (lane == 0) F.hdr[h].dv_ba = oba;  // (fl_deep_store: asks lie at or above it)
    (void)obb;
  } else if (uni(hd->dc)) {  // DELs in the segment (gen_plan_asm.py W32DC)
    asm volatile(FL_PLAN_ASM32DC
                 : [lk] "+v"(lg.lk), [la] "+v"(lg.la), [lb] "+v"(lg.lb), [nacc] "+s"(lg.nacc), [lpos] "+s"(lg.lpos),
                   [voff] "=&v"(voff), [vpf] "=&v"(vpf)
                 : [ob] "s"(ob), [nh] "s"(nh), [logp] "s"(logp), [lcap] "s"(lg.lcap), [vl16] "v"(vl16),
                   [vzero] "v"(vzero), [sb] "v"(sb), [sa] "v"(sa)
                 : FL_PLAN_CLOBBERS, FL_PLAN_CLOBBERS_D, "scc", "vcc", "memory");
  } else {
    asm volatile(FL_PLAN_ASM32D
                 : [lk] "+v"(lg.lk), [la] "+v"(lg.la), [lb] "+v"(lg.lb), [nacc] "+s"(lg.nacc), [lpos] "+s"(lg.lpos),
                   [voff] "=&v"(voff), [vpf] "=&v"(vpf)
                 : [ob] "s"(ob), [nh] "s"(nh), [logp] "s"(logp), [lcap] "s"(lg.lcap), [vl16] "v"(vl16),
                   [vzero] "v"(vzero), [sb] "v"(sb), [sa] "v"(sa)
                 : FL_PLAN_CLOBBERS, FL_PLAN_CLOBBERS_D, "scc", "vcc", "memory");
  }
  if (lg.nacc) {  // {key, level, amount, 0}
    if (lane < lg.nacc && lg.lpos + lg.nacc <= lg.lcap) lg.p[lg.lpos + lane] = v4(lg.lk, lg.lb, lg.la, 0u);
    lg.lpos += lg.nacc;
  }
  if (lg.lpos > lg.lcap) {
    if (lane == 0) atomicOr(&D.st->err, ERR_CORRUPT);
    lg.lpos = 0;
  }
  if (lane == 0) F.hdr[h].ntouch = lg.lpos;
}

// ============================================================== k_flow_sort
// Stable counting sort of one book's touches by level: histogram -> run bases, then tiles of
// FL_SORT_T touches ranked within each wave by a 7-bit ballot match (equal levels) and
// across waves through LDS counters, so every level's run keeps log (= time) order.
constexpr uint32_t FL_SORT_T = 1024, FL_SORT_W = FL_SORT_T / 64;

__global__ __launch_bounds__(FL_SORT_T) void k_flow_sort(Dev D, FlowArgs F) {
  __shared__ uint32_t hist[FL_CAP], run[FL_CAP];
  __shared__ uint32_t wc[FL_SORT_W][FL_CAP];
  __shared__ uint32_t nrest;
  const uint32_t h = F.h0 + blockIdx.x, tid = threadIdx.x, w = tid >> 6;
  if (h >= fl_hend(D, F) || !F.hdr[h].ok || F.hdr[h].ok == FL_OK_DEEP) return;
  const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg, nl = F.hdr[h].nl;
  const unsigned long long g = F.hdr[h].g;
  const bool cb = F.hdr[h].ok == FL_OK_CANCEL;
  FlowLvl* LV = F.lvl + h * FL_CAP;
  if (tid < FL_CAP) hist[tid] = 0;
  if (tid == 0) nrest = 0;
  for (uint32_t i = tid; i < FL_SORT_W * FL_CAP; i += FL_SORT_T) wc[i / FL_CAP][i % FL_CAP] = 0;
  __syncthreads();
  uint32_t myr = 0;
  for (uint32_t t = tid; t < nt; t += FL_SORT_T) {
    const uint32_t kr = F.log[L + t].kr;
    atomicAdd(&hist[kr & 127u], 1u);
    myr += tk_kind(kr, cb) == TK_REST && (kr & 127u) ? 1u : 0u;  // level-0 touches are no-op records
  }
  if (myr) atomicAdd(&nrest, myr);
  __syncthreads();
  if (tid == 0) F.hdr[h].rests = nrest;
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < FL_CAP; ++k) {
      run[k] = acc;
      acc += hist[k];
    }
  }
  __syncthreads();
  if (tid >= 1 && tid <= nl) {
    LV[tid].cnt = hist[tid];
    LV[tid].base = run[tid];
  }
  const unsigned long long ltm = lt_mask();
  for (uint32_t t0 = 0; t0 < nt; t0 += FL_SORT_T) {
    const uint32_t t = t0 + tid;
    const bool valid = t < nt;
    Touch x{};
    if (valid) x = F.log[L + t];
    const uint32_t k = valid ? (x.kr & 127u) : 0u;
    unsigned long long same = __ballot(valid);
#pragma unroll
    for (uint32_t b = 0; b < 7; ++b) {
      const unsigned long long bb = __ballot((k >> b) & 1u);
      same &= ((k >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t rank = __popcll(same & ltm);
    if (valid && rank == 0) wc[w][k] = __popcll(same);
    __syncthreads();
    if (tid < FL_CAP) {
      uint32_t r = run[tid];
      for (uint32_t ww = 0; ww < FL_SORT_W; ++ww) {
        const uint32_t c = wc[ww][tid];
        wc[ww][tid] = r;
        r += c;
      }
      run[tid] = r;
    }
    __syncthreads();
    if (valid) {
      SEnt e;
      e.j = tk_jb(x, cb);
      e.kind = tk_kind(x.kr, cb);
      e.amt = x.amt;
      e.coord = 0;
      e.t = t;
      e.lvl = k;
      const uint32_t pos = wc[w][k] + rank;
      e.amt = static_cast<int64_t>(static_cast<unsigned long long>(x.amt) * g);  // plan units -> fixed point
      F.srt[L + pos] = e;
      if (cb) {  // (the cancel kernels read the run position and fixed-point amounts from the log;
                 // the ADD books' event kernels scale the plan units themselves: fl_amt_unit)
        F.log[L + t].pos = pos;
        if (g != 1) F.log[L + t].amt = e.amt;
      }
    }
    __syncthreads();
    for (uint32_t i = tid; i < FL_SORT_W * FL_CAP; i += FL_SORT_T) wc[i / FL_CAP][i % FL_CAP] = 0;
    __syncthreads();
  }
}

// ============================================================== k_flow_level
// One wave per level (waves of a per-book workgroup take the book's levels in turn):
// volume coordinates of the level's run, then the gather of the consumed prefix of its
// resting FIFO.
// (run_base / run_cnt: the level's run when the caller found it, deep books; else FlowLvl's.
// ig_pre: the level's gathered-maker space when the caller claimed it, else claimed here.)
// Block-wide exclusive scan of one int64 per thread (FL_LVB_T threads); *total = the block's sum.
constexpr uint32_t FL_LVB_T = 1024, FL_LVB_W = FL_LVB_T / 64;
__device__ __forceinline__ int64_t fl_blk_excl(int64_t x, int64_t* total) {
  __shared__ int64_t ws[FL_LVB_W];
  const uint32_t w = threadIdx.x >> 6;
  const int64_t inc = wave_incl_scan(x);
  if ((threadIdx.x & 63u) == 63u) ws[w] = inc;
  __syncthreads();
  int64_t before = 0, tot = 0;
  for (uint32_t k = 0; k < FL_LVB_W; ++k) {
    const int64_t v = ws[k];
    before += k < w ? v : 0;
    tot += v;
  }
  __syncthreads();  // (ws is reused by the next call)
  *total = tot;
  return before + inc - x;
}

// fl_level_one's touch scan with a whole block (FL_LVB_T threads) on one level: the level's
// touches in block-wide chunks (the hottest book's levels hold thousands of touches).
__device__ __forceinline__ void fl_level_scan_blk(const FlowArgs& F, uint32_t h, uint32_t q, int64_t& cfin,
                                                  uint32_t& nr, uint32_t* ncons = nullptr) {
  const FlowHdr* hd = &F.hdr[h];
  FlowLvl* Lq = fl_lvls(F, h) + q;
  const uint32_t L = FL_TOUCH_MUL * hd->beg, base = Lq->base, cnt = Lq->cnt;
  SEnt* R = F.srt + L + base;
  RsEnt* RS = F.rs + L + base;
  int64_t cc = 0, rr = Lq->d0;
  uint32_t n = 0, nc = 0;
  for (uint32_t c0 = 0; c0 < cnt; c0 += FL_LVB_T) {
    const uint32_t i = c0 + threadIdx.x;
    const bool valid = i < cnt;
    SEnt e{};
    if (valid) e = R[i];
    const bool isc = valid && e.kind == TK_CONS, isr = valid && e.kind == TK_REST;
    int64_t tc, tr, tn;
    const int64_t xc = fl_blk_excl(isc ? e.amt : 0, &tc);
    const int64_t xr = fl_blk_excl(isr ? e.amt : 0, &tr);
    const int64_t xn = fl_blk_excl(isr ? 1 : 0, &tn);
    nc += static_cast<uint32_t>(__syncthreads_count(isc));
    if (isc) R[i].coord = cc + xc;
    if (isr) {
      const int64_t e0 = rr + xr;
      R[i].coord = e0;
      RsEnt x;
      x.e = e0;
      x.v = e.amt;
      x.j = e.j;
      x.t = e.t;
      x.pad0 = x.pad1 = 0;
      RS[n + static_cast<uint32_t>(xn)] = x;
    }
    cc += tc;
    rr += tr;
    n += static_cast<uint32_t>(tn);
  }
  cfin = cc;
  nr = n;
  if (ncons) *ncons = nc;
}

// ============================================================== events of one touch
// Makers of level q in FIFO order: the gathered old makers IG[0, ig_n) (coordinates from 0),
// then the new makers RS[0, nrest) (from d0).  Index of the maker covering coordinate x.
__device__ __forceinline__ uint32_t fl_find(const IgEnt* IG, uint32_t ig_n, const RsEnt* RS, uint32_t nrest,
                                            int64_t d0, int64_t x) {
  if (x < d0) {
    uint32_t lo = 0, hi = ig_n;  // last e <= x
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (IG[mid].e <= x) lo = mid; else hi = mid;
    }
    return lo;
  }
  uint32_t lo = 0, hi = nrest;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (RS[mid].e <= x) lo = mid; else hi = mid;
  }
  return ig_n + lo;
}

// Zero-volume makers (Q6) share their successor's start.  A consume whose cursor is c fills first
// the zero-volume makers starting at c (the FIFO head: everything before them is gone, and the
// consume before stopped at c with diff == 0, engine.go:162-175), so its first maker steps back
// from fl_find's (the last start <= c) over those: a maker before the found one with start c has
// length 0 (k_flow_zero_check hands over a book where a consume leaves depth 0 beside one, or a
// zero-volume taker meets one).
__device__ __forceinline__ uint32_t fl_first_back(const IgEnt* IG, uint32_t ig_n, const RsEnt* RS, uint32_t f, int64_t c) {
  while (f > 0 && (f - 1 < ig_n ? IG[f - 1].e : RS[f - 1 - ig_n].e) == c) --f;
  return f;
}

// The level-end continuation (Q6).  A consume that takes a level's whole depth with volume to spare
// goes on (MatchOrder's diff > 0 branch recurses, engine.go:145-161): it pops the zero-volume makers
// still at the level's end with 0-fills before Match moves to the next level or the taker rests
// (engine.go:129-131).  A taker that stopped there (diff == 0) leaves them.  It went on exactly when
// its next touch in the log (in time order, an order's touches consecutive) is its own.  cb: a book
// with DELs (tk_jc).
__device__ __forceinline__ bool fl_cont(const FlowArgs& F, uint32_t L, uint32_t nt, uint32_t t, bool cb) {
  return t + 1 < nt && tk_jb(F.log[L + t], cb) == tk_jb(F.log[L + t + 1], cb);
}
// ... of the consume before run entry i (the level's previous CONS in time order, which ended at this
// one's cursor): the zero-volume makers starting at the cursor are then gone, not this consume's
// first fills (fl_first_back).  Walked back one entry at a time: levels that may hold zero-volume
// makers only (a run's CONS gaps add up to its length).
__device__ __forceinline__ bool fl_prev_cont(const FlowArgs& F, uint32_t L, uint32_t nt, const SEnt* R, uint32_t i,
                                             bool cb) {
  while (i-- > 0)
    if (R[i].kind == TK_CONS) return R[i].amt > 0 && fl_cont(F, L, nt, R[i].t, cb);
  return false;
}
// ... of the level's last consume (FlowLvl::zcont): the zero-volume makers at the consumption end
// are popped, not survivors.
__device__ __forceinline__ bool fl_run_cont(const FlowArgs& F, uint32_t L, uint32_t nt, const SEnt* R, uint32_t cnt,
                                            bool cb) {
  return fl_prev_cont(F, L, nt, R, cnt, cb);
}
// A continuing consume's last maker steps on over the zero-volume makers starting at its end x
// (the mirror of fl_first_back; a maker that rested there after it has volume, or starts later).
__device__ __forceinline__ uint32_t fl_last_fwd(const IgEnt* IG, uint32_t ig_n, const RsEnt* RS, uint32_t nrest,
                                                uint32_t l, int64_t x) {
  for (uint32_t m = l + 1; m < ig_n + nrest; ++m) {
    const bool old = m < ig_n;
    if ((old ? IG[m].v : RS[m - ig_n].v) != 0 || (old ? IG[m].e : RS[m - ig_n].e) != x) break;
    l = m;
  }
  return l;
}

// Wave-cooperative fl_find: every lane's query q (lanes with !valid ignored), b a maker at or
// before every valid query's.  Windows of 64 consecutive makers from b (one coalesced read into
// the lanes) searched by shuffles; a query beyond FL_FC_WIN windows searches alone.  Makers'
// starts ascend (strictly but for zero-volume makers, which share their successor's), IG then RS,
// from 0.
constexpr int FL_FC_WIN = 3;
__device__ __forceinline__ uint32_t fl_wave_find(const IgEnt* IG, uint32_t ig_n, const RsEnt* RS, uint32_t nrest,
                                                 int64_t d0, bool valid, int64_t q, uint32_t b) {
  const uint32_t nm = ig_n + nrest, lane = lane_id();
  uint32_t res = NIL;
  bool done = !valid;
  for (int w = 0; w < FL_FC_WIN && !__all(done); ++w) {
    const uint32_t m = b + lane;
    const int64_t st = m < nm ? (m < ig_n ? IG[m].e : RS[m - ig_n].e) : INT64_MAX;
    const int64_t last = __shfl(st, 63);
    const bool here = !done && (q < last || b + 63 >= nm);
    // (every lane takes part in the shuffles; the count of the window's starts <= q)
    const int64_t qq = here ? q : INT64_MIN;
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1) {
      const int64_t sv = __shfl(st, static_cast<int>(pos + step - 1));
      if (sv <= qq) pos += step;
    }
    if (here) {
      res = b + pos - 1;
      done = true;
    }
    b += 63;  // (the window's last maker opens the next one)
  }
  if (!done) res = fl_find(IG, ig_n, RS, nrest, d0, q);
  return res;
}

// The makers every CONS touch of level q fills (first / last in FIFO order), with its cursor and
// level, into F.tfc at the touch's log index, where the level's maker arrays were just written
// (L2-hot), so the event passes read one entry per touch instead of searching.  Waves w, w + nw,
// ... of the caller take the level's touches 64 at a time.  The consumption starts at coordinate
// 0 (maker 0) and advances, so a lone wave (nw == 1) starts each chunk's windows where the last
// chunk's ended; interleaved waves find their chunk's first maker by one search.
__device__ __forceinline__ void fl_level_fc(const FlowArgs& F, uint32_t L, uint32_t q, uint32_t base, uint32_t cnt,
                                            const IgEnt* IG, uint32_t ig_n, uint32_t nrest, int64_t d0, uint32_t w,
                                            uint32_t nw, bool zl = false, uint32_t nt = 0) {
  const SEnt* R = F.srt + L + base;
  const RsEnt* RS = F.rs + L + base;
  const uint32_t lane = lane_id();
  uint32_t carry = 0;  // (nw == 1) the maker the next chunk's windows start at
  for (uint32_t i0 = w * 64; i0 < cnt; i0 += nw * 64) {
    const uint32_t i = i0 + lane;
    SEnt e{};
    if (i < cnt) e = R[i];
    const bool cons = i < cnt && e.kind == TK_CONS;
    const unsigned long long cm = __ballot(cons);
    if (!cm) continue;
    // (a CONS of 0, a zero-volume taker (Q6): the one maker at its cursor, MatchVolume 0)
    const int64_t x = e.coord + (e.amt ? e.amt : 1) - 1;
    const int l0 = static_cast<int>(__builtin_ctzll(cm)), l1 = 63 - static_cast<int>(__builtin_clzll(cm));
    const uint32_t b = nw == 1 ? carry : fl_find(IG, ig_n, RS, nrest, d0, __shfl(e.coord, l0));
    const uint32_t f0 = fl_wave_find(IG, ig_n, RS, nrest, d0, cons, e.coord, b);
    const uint32_t l = fl_wave_find(IG, ig_n, RS, nrest, d0, cons, x, __shfl(f0, l0));
    carry = __shfl(l, l1);
    if (cons) {
      uint32_t f = f0, ll = l;
      if (zl && e.amt) {  // (zero-volume makers at the cursor, and at the end of a consume that went on)
        if (!fl_prev_cont(F, L, nt, R, i, false)) f = fl_first_back(IG, ig_n, RS, f0, e.coord);
        if (fl_cont(F, L, nt, e.t, false)) ll = fl_last_fwd(IG, ig_n, RS, nrest, l, e.coord + e.amt);
      }
      FlTouchFc y;
      y.first = f;
      y.last = ll;
      y.lvl = q;
      y.pad = 0;
      y.coord = e.coord;
      F.tfc[L + e.t] = y;
    }
  }
}

// A workgroup's fully consumed chunk ids, staged in LDS and published with one claim on
// Status::freed_top at the workgroup's end (fl_freed_flush): a device-scope atomic per level on
// that one word serialised the tail's level pass.  Ids beyond the stage go straight out.
constexpr uint32_t FL_FREED_LDS = 1024;
struct FlFreed {
  uint32_t n;
  uint32_t ids[FL_FREED_LDS];
};
__device__ __forceinline__ void fl_freed_flush(const Dev& D, FlFreed* stg) {
  __shared__ uint32_t fb_s;
  const uint32_t n = min(stg->n, FL_FREED_LDS);
  if (threadIdx.x == 0) fb_s = n ? atomicAdd(&D.st->freed_top, n) : 0u;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) D.freed_ids[fb_s + i] = stg->ids[i];
}

__device__ __forceinline__ void fl_level_one(const Dev& D, const FlowArgs& F, uint32_t h, uint32_t q,
                                             uint32_t run_base = NIL, uint32_t run_cnt = 0,
                                             uint32_t ig_pre = NIL, int64_t pre_cfin = -1, uint32_t pre_nr = 0,
                                             bool fc_here = true, FlFreed* stg = nullptr, bool gather0 = false) {
  const FlowHdr* hd = &F.hdr[h];
  const uint32_t lane = lane_id();
  FlowLvl* Lq = fl_lvls(F, h) + q;
  const uint32_t L = FL_TOUCH_MUL * uni(hd->beg);
  const uint32_t base = run_base != NIL ? run_base : uni(Lq->base), cnt = run_base != NIL ? run_cnt : uni(Lq->cnt);
  const int64_t d0 = uni64(Lq->d0);
  SEnt* R = F.srt + L + base;
  RsEnt* RS = F.rs + L + base;
  int64_t cc = 0, rr = d0;
  uint32_t nr = 0;
  const unsigned long long ltm = lt_mask();
  const bool zl = Lq->z0 || hd->nzero;  // (the level may hold zero-volume makers: fl_first_back)
  if (pre_cfin >= 0) {  // (the touch scan ran block-wide: fl_level_scan_blk)
    cc = pre_cfin;
    nr = pre_nr;
  }
  // a lone wave with the fill contexts (fl_level_fc) to make: the level's total consumption first
  // (the old makers' gather needs it), then one scan that writes the new makers and the contexts
  // from registers (no cursor round trip through the sorted runs)
  const bool fused_fc = fc_here && pre_cfin < 0;
  if (fused_fc) {
    int64_t sc = 0;
    for (uint32_t c0 = 0; c0 < cnt; c0 += 64) {
      const uint32_t i = c0 + lane;
      if (i < cnt && R[i].kind == TK_CONS) sc += R[i].amt;
    }
    for (int off = 32; off > 0; off >>= 1) sc += __shfl_xor(sc, off);
    cc = sc;
  }
  for (uint32_t c0 = 0; pre_cfin < 0 && !fused_fc && c0 < cnt; c0 += 64) {
    const uint32_t i = c0 + lane;
    const bool valid = i < cnt;
    SEnt e{};
    if (valid) e = R[i];
    const bool isc = valid && e.kind == TK_CONS, isr = valid && e.kind == TK_REST;
    const int64_t ac = isc ? e.amt : 0, ar = isr ? e.amt : 0;
    const int64_t ic = wave_incl_scan(ac), ir = wave_incl_scan(ar);
    const unsigned long long rm = __ballot(isr);
    if (isc) R[i].coord = cc + ic - ac;
    if (isr) {
      const int64_t e0 = rr + ir - ar;
      R[i].coord = e0;
      RsEnt x;
      x.e = e0;
      x.v = e.amt;
      x.j = e.j;
      x.t = e.t;
      x.pad0 = x.pad1 = 0;
      RS[nr + __popcll(rm & ltm)] = x;
    }
    cc += rl64(ic, 63);
    rr += rl64(ir, 63);
    nr += __popcll(rm);
  }
  const int64_t cfin = cc;
  // (a level that may hold zero-volume makers: the level-end continuation, fl_cont)
  const uint32_t nt = zl ? uni(hd->ntouch) : 0u;
  const bool lcont = zl && cfin > 0 && fl_run_cont(F, L, nt, R, cnt, false);
  uint32_t nv0 = uni(Lq->nv0), head = uni(Lq->head), tail = uni(Lq->tail);
  uint32_t hslot = uni(Lq->hslot), tslot = uni(Lq->tslot);
  uint32_t ig_base = 0, ng = 0, consumed = 0, zpopped = 0;
  bool have_extra = false;
  // (gather0: a CONS of 0 reads the maker at the cursor even when nothing was consumed)
  if (nv0 > 0 && (cfin > 0 || gather0)) {
    uint32_t b = ig_pre;
    if (ig_pre == NIL) {
      if (lane == 0) b = atomicAdd(F.ig_bump, nv0);
      b = uni(b);
    }
    ig_base = b;
    if (static_cast<unsigned long long>(ig_base) + nv0 > F.ig_cap) {
      if (lane == 0) atomicOr(&D.st->err, ERR_CHUNKS);
      return;
    }
    IgEnt* IG = F.ig + ig_base;
    int64_t E = 0;
    bool have_surv = false;
    uint32_t c = head, s0 = hslot, nh = NIL, nhs = 0;
    uint32_t nfr = 0, fid = 0;  // fully consumed chunks, published 64 at a time
    auto publish = [&]() {
      uint32_t fb = 0;
      if (stg) {  // the workgroup's stage first; what does not fit goes out
        if (lane == 0) fb = atomicAdd(&stg->n, nfr);
        fb = uni(fb);
        const uint32_t fit = fb < FL_FREED_LDS ? min(nfr, FL_FREED_LDS - fb) : 0u;
        if (lane < fit) stg->ids[fb + lane] = fid;
        if (fit < nfr) {
          uint32_t gb = 0;
          if (lane == 0) gb = atomicAdd(&D.st->freed_top, nfr - fit);
          gb = uni(gb);
          if (lane >= fit && lane < nfr) D.freed_ids[gb + lane - fit] = fid;
        }
      } else {
        if (lane == 0) fb = atomicAdd(&D.st->freed_top, nfr);
        fb = uni(fb);
        if (lane < nfr) D.freed_ids[fb + lane] = fid;
      }
      nfr = 0;
    };
    for (uint32_t guard = 0; c != NIL && !have_extra; ++guard) {
      if (guard > D.ch_cap) { if (lane == 0) atomicOr(&D.st->err, ERR_CORRUPT); return; }
      const uint32_t lim = (c == tail) ? tslot : CH;
      const bool inr = lane < CH && lane >= s0 && lane < lim;
      const uint32_t nxt = (c == tail) ? NIL : D.chdr[c].next;  // (in flight beside the nodes)
      Node nd{};
      if (inr) nd = D.nodes[c * CH + lane];
      const bool live = inr && nd.rem >= 0;
      const int64_t x = live ? nd.rem : 0;
      const int64_t inc = wave_incl_scan(x);
      const int64_t em = E + inc - x;
      const bool zend = lcont && live && nd.rem == 0 && em == cfin;  // (popped by the last consume, going on)
      const unsigned long long beyond = __ballot(live && em >= cfin && !zend);
      const uint32_t fb = beyond ? static_cast<uint32_t>(__builtin_ctzll(beyond)) : 64u;
      const bool take = live && (em < cfin || zend || lane == fb);
      const unsigned long long tm = __ballot(take);
      if (take) {
        IgEnt g;
        g.e = em;
        g.v = nd.rem;
        g.oid = nd.oid;
        g.uuid = nd.uuid;
        g.tx = nd.tx;
        g.pad = 0;
        IG[ng + __popcll(tm & ltm)] = g;
      }
      ng += __popcll(tm);
      // (a zero-volume maker is consumed, popped, strictly before the consumption end, or at it when
      // the last consume went on: one at the end was not reached by a taker that stopped there,
      // engine.go:162-175)
      const bool cons = live && em + nd.rem <= cfin && (nd.rem > 0 || em < cfin || zend);
      if (cons) __hip_atomic_store(&D.idx[nd.ixs].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      consumed += __popcll(__ballot(cons));
      zpopped += __popcll(__ballot(cons && nd.rem == 0));
      if (!have_surv) {
        const unsigned long long sv = __ballot(live && !cons);
        if (sv) {
          have_surv = true;
          nh = c;
          nhs = static_cast<uint32_t>(__builtin_ctzll(sv));
          if (lane == nhs && em < cfin) D.nodes[c * CH + lane].rem = em + nd.rem - cfin;  // partial head
        } else {  // a fully consumed chunk
          if (lane == nfr) fid = c;
          if (++nfr == 64) publish();
        }
      }
      if (beyond) have_extra = true;
      E += rl64(inc, 63);
      c = uni(nxt);
      s0 = 0;
    }
    if (nfr) publish();
    if (!have_surv) {
      head = tail = NIL;
      hslot = tslot = 0;
    } else {
      head = nh;
      hslot = nhs;
    }
  }
  if (fused_fc) {  // the scan: new makers, and each CONS touch's makers (old ones: IG, complete)
    const IgEnt* IG = F.ig + ig_base;
    int64_t c1 = 0;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < cnt; c0 += 64) {
      const uint32_t i = c0 + lane;
      const bool valid = i < cnt;
      SEnt e{};
      if (valid) e = R[i];
      const bool isc = valid && e.kind == TK_CONS, isr = valid && e.kind == TK_REST;
      const int64_t ac = isc ? e.amt : 0, ar = isr ? e.amt : 0;
      const int64_t ic = wave_incl_scan(ac), ir = wave_incl_scan(ar);
      const unsigned long long rm = __ballot(isr), cm = __ballot(isc);
      if (isr) {
        RsEnt x;
        x.e = rr + ir - ar;
        x.v = e.amt;
        x.j = e.j;
        x.t = e.t;
        x.pad0 = x.pad1 = 0;
        RS[nr + __popcll(rm & ltm)] = x;
      }
      nr += __popcll(rm);
      rr += rl64(ir, 63);
      if (cm) {  // (a consume fills makers that rested before it: up to this chunk's, written above)
        __threadfence_block();
        const int64_t c = c1 + ic - ac, x = c + (ac ? ac : 1) - 1;  // (a CONS of 0: fl_level_fc)
        const int l0 = static_cast<int>(__builtin_ctzll(cm)), l1 = 63 - static_cast<int>(__builtin_clzll(cm));
        const uint32_t f0 = fl_wave_find(IG, ng, RS, nr, d0, isc, c, carry);
        const uint32_t l = fl_wave_find(IG, ng, RS, nr, d0, isc, x, __shfl(f0, l0));
        carry = __shfl(l, l1);
        if (isc) {
          uint32_t f = f0, ll = l;
          if (zl && ac) {  // (as fl_level_fc)
            if (!fl_prev_cont(F, L, nt, R, i, false)) f = fl_first_back(IG, ng, RS, f0, c);
            if (fl_cont(F, L, nt, e.t, false)) ll = fl_last_fwd(IG, ng, RS, nr, l, c + ac);
          }
          FlTouchFc y;
          y.first = f;
          y.last = ll;
          y.lvl = q;
          y.pad = 0;
          y.coord = c;
          F.tfc[L + e.t] = y;
        }
      }
      c1 += rl64(ic, 63);
    }
  }
  if (lane == 0) {
    Lq->cfin = cfin;
    Lq->nrest = nr;
    Lq->ig_base = ig_base;
    Lq->ig_n = ng;
    Lq->ig_all = have_extra ? 0u : 1u;
    Lq->head = head;
    Lq->tail = tail;
    Lq->hslot = hslot;
    Lq->tslot = tslot;
    Lq->nlive0 = nv0 - consumed;
    Lq->zpop = zpopped;
    Lq->zcont = lcont ? 1u : 0u;
  }
}

// fl_level_one (its fused path: no pre-scan, contexts made here) by ONE lane, for a level of at
// most FL_LANE_MAX touches, with the same outputs: the level's consumption, the old FIFO's gather
// (a chunk's slots in order), the new makers, then each CONS touch's makers (fl_find_all over the
// gathered and the new makers, as fl_wave_find).  Deep books hold thousands of touched levels of a
// few touches each per batch, which one wave took one after another (k_deep_level).
constexpr uint32_t FL_LANE_MAX = 16;
__device__ __forceinline__ uint32_t fl_find_all(const IgEnt* IG, uint32_t ig_n, const RsEnt* RS, uint32_t nrest, int64_t x) {
  uint32_t lo = 0, hi = ig_n + nrest;  // the last maker whose start <= x (starts ascend, IG then RS)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((mid < ig_n ? IG[mid].e : RS[mid - ig_n].e) <= x) lo = mid; else hi = mid;
  }
  return lo;
}
// ig_pre / stg: as fl_level_one's (the gather's claimed space, the workgroup's freed-chunk stage).
__device__ __forceinline__ void fl_level_lane(const Dev& D, const FlowArgs& F, uint32_t h, uint32_t q, uint32_t base,
                                              uint32_t cnt, uint32_t ig_pre = NIL, FlFreed* stg = nullptr) {
  const FlowHdr* hd = &F.hdr[h];
  FlowLvl* Lq = fl_lvls(F, h) + q;
  const uint32_t L = FL_TOUCH_MUL * hd->beg;
  const int64_t d0 = Lq->d0;
  const SEnt* R = F.srt + L + base;
  RsEnt* RS = F.rs + L + base;
  const bool zl = Lq->z0 || hd->nzero;
  int64_t cfin = 0;
  for (uint32_t i = 0; i < cnt; ++i)
    if (R[i].kind == TK_CONS) cfin += R[i].amt;
  const uint32_t nt = zl ? hd->ntouch : 0u;
  const bool lcont = zl && cfin > 0 && fl_run_cont(F, L, nt, R, cnt, false);  // (fl_level_one)
  uint32_t nv0 = Lq->nv0, head = Lq->head, tail = Lq->tail;
  uint32_t hslot = Lq->hslot, tslot = Lq->tslot;
  uint32_t ig_base = 0, ng = 0, consumed = 0, zpopped = 0;
  bool have_extra = false;
  if (nv0 > 0 && cfin > 0) {
    ig_base = ig_pre != NIL ? ig_pre : atomicAdd(F.ig_bump, nv0);
    if (static_cast<unsigned long long>(ig_base) + nv0 > F.ig_cap) {
      atomicOr(&D.st->err, ERR_CHUNKS);
      return;
    }
    IgEnt* IG = F.ig + ig_base;
    int64_t E = 0;
    bool have_surv = false;
    uint32_t c = head, s0 = hslot, nh = NIL, nhs = 0;
    for (uint32_t guard = 0; c != NIL && !have_extra; ++guard) {
      if (guard > D.ch_cap) { atomicOr(&D.st->err, ERR_CORRUPT); return; }
      const uint32_t lim = (c == tail) ? tslot : CH;
      const uint32_t nxt = (c == tail) ? NIL : D.chdr[c].next;
      Node nd[CH];
#pragma unroll
      for (uint32_t s = 0; s < CH; ++s) {
        nd[s] = Node{};
        if (s >= s0 && s < lim) nd[s] = D.nodes[c * CH + s];
      }
      bool surv_here = false;
#pragma unroll
      for (uint32_t s = 0; s < CH; ++s) {
        if (!(s >= s0 && s < lim && nd[s].rem >= 0)) continue;  // (live makers only)
        const int64_t em = E;
        E += nd[s].rem;
        const bool zend = lcont && nd[s].rem == 0 && em == cfin;
        if (!have_extra) {  // every maker before the consumption end, then the first at or past it
          IgEnt g;
          g.e = em;
          g.v = nd[s].rem;
          g.oid = nd[s].oid;
          g.uuid = nd[s].uuid;
          g.tx = nd[s].tx;
          g.pad = 0;
          IG[ng++] = g;
          if (em >= cfin && !zend) have_extra = true;
        }
        const bool cons = em + nd[s].rem <= cfin && (nd[s].rem > 0 || em < cfin || zend);
        if (cons) {
          __hip_atomic_store(&D.idx[nd[s].ixs].key, KEY_TOMB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          consumed++;
          if (nd[s].rem == 0) zpopped++;
        }
        if (!have_surv && !surv_here && !cons) {
          surv_here = true;
          nh = c;
          nhs = s;
          if (em < cfin) D.nodes[c * CH + s].rem = em + nd[s].rem - cfin;  // partial head
        }
      }
      if (!have_surv) {
        if (surv_here) {
          have_surv = true;
        } else {  // a fully consumed chunk
          const uint32_t k = stg ? atomicAdd(&stg->n, 1u) : FL_FREED_LDS;
          if (k < FL_FREED_LDS) stg->ids[k] = c;
          else D.freed_ids[atomicAdd(&D.st->freed_top, 1u)] = c;
        }
      }
      c = nxt;
      s0 = 0;
    }
    if (!have_surv) {
      head = tail = NIL;
      hslot = tslot = 0;
    } else {
      head = nh;
      hslot = nhs;
    }
  }
  // the new makers, then each CONS touch's makers (every new maker of the level written first, as
  // fl_level_one's 64-touch chunk)
  int64_t rr = d0;
  uint32_t nr = 0;
  for (uint32_t i = 0; i < cnt; ++i) {
    const SEnt e = R[i];
    if (e.kind != TK_REST) continue;
    RsEnt x;
    x.e = rr;
    x.v = e.amt;
    x.j = e.j;
    x.t = e.t;
    x.pad0 = x.pad1 = 0;
    RS[nr++] = x;
    rr += e.amt;
  }
  const IgEnt* IG = F.ig + ig_base;
  int64_t c1 = 0;
  for (uint32_t i = 0; i < cnt; ++i) {
    const SEnt e = R[i];
    if (e.kind != TK_CONS) continue;
    const int64_t c = c1, x = c + (e.amt ? e.amt : 1) - 1;
    const uint32_t f0 = fl_find_all(IG, ng, RS, nr, c);
    const uint32_t l = fl_find_all(IG, ng, RS, nr, x);
    FlTouchFc y;
    y.first = zl && e.amt && !fl_prev_cont(F, L, nt, R, i, false) ? fl_first_back(IG, ng, RS, f0, c) : f0;
    y.last = zl && e.amt && fl_cont(F, L, nt, e.t, false) ? fl_last_fwd(IG, ng, RS, nr, l, c + e.amt) : l;
    y.lvl = q;
    y.pad = 0;
    y.coord = c;
    F.tfc[L + e.t] = y;
    c1 += e.amt;
  }
  Lq->cfin = cfin;
  Lq->nrest = nr;
  Lq->ig_base = ig_base;
  Lq->ig_n = ng;
  Lq->ig_all = have_extra ? 0u : 1u;
  Lq->head = head;
  Lq->tail = tail;
  Lq->hslot = hslot;
  Lq->tslot = tslot;
  Lq->nlive0 = nv0 - consumed;
  Lq->zpop = zpopped;
  Lq->zcont = lcont ? 1u : 0u;
  Lq->cnt = cnt;
}

constexpr uint32_t FL_LEVEL_T = 1024;
// Tail books: one workgroup per book, its waves take the levels in turn.  The book's gathered-
// maker space is claimed once (every touched level with old makers: a superset of the levels
// that gather, within F.ig_cap since their makers are live nodes), and its freed chunks are
// published once (FlFreed): per-level claims on those two words serialised the pass.
__global__ __launch_bounds__(FL_LEVEL_T) void k_flow_level(Dev D, FlowArgs F) {
  static_assert(FL_CAP <= 128, "one wave scans a book's levels, two per lane");
  __shared__ uint32_t igo[FL_CAP];
  __shared__ FlFreed stg;
  const uint32_t h = F.h0 + blockIdx.x;
  if (h >= fl_hend(D, F) || F.hdr[h].ok != FL_OK_ADD) return;
  const uint32_t nl = F.hdr[h].nl, tid = threadIdx.x;
  const FlowLvl* LV = fl_lvls(F, h);
  if (tid < 64) {
    uint32_t v0 = 0, v1 = 0;
    const uint32_t q0 = 2 * tid + 1, q1 = 2 * tid + 2;
    if (q0 <= nl && LV[q0].cnt) v0 = LV[q0].nv0;
    if (q1 <= nl && LV[q1].cnt) v1 = LV[q1].nv0;
    const uint32_t x = v0 + v1;
    uint32_t inc = x;
    for (uint32_t off = 1; off < 64; off <<= 1) {
      const uint32_t u = __shfl_up(inc, off);
      if (tid >= off) inc += u;
    }
    const uint32_t tot = __shfl(inc, 63);
    uint32_t b = 0;
    if (tid == 0) b = tot ? atomicAdd(F.ig_bump, tot) : 0u;
    b = __shfl(b, 0);
    const uint32_t ex = b + inc - x;
    if (q0 < FL_CAP) igo[q0] = v0 ? ex : NIL;
    if (q1 < FL_CAP) igo[q1] = v1 ? ex + v0 : NIL;
    if (tid == 0) stg.n = 0;
  }
  __syncthreads();
  // (the lane pass, fl_level_lane, measured 1.5% slower on config 2 here: its tail books' levels
  // hold tens of touches, r05ba)
  for (uint32_t q = 1 + (tid >> 6); q <= nl; q += FL_LEVEL_T / 64)
    fl_level_one(D, F, h, uni(q), NIL, 0, igo[q], -1, 0, true, &stg);
  __syncthreads();
  fl_freed_flush(D, &stg);
}

struct FlTouchCtx {
  const FlowLvl* Lq;
  const IgEnt* IG;
  const RsEnt* RS;
  int64_t c, a;
  uint32_t first, last;
};

// The fixed-point value of one plan unit in book h's log: a lane ADD book's log keeps the plan's
// units (its sort leaves the log alone); deep and cancel books' logs were converted.
__device__ __forceinline__ int64_t fl_amt_unit(const FlowArgs& F, uint32_t h) {
  return F.hdr[h].ok == FL_OK_ADD ? static_cast<int64_t>(F.hdr[h].g) : 1;
}

// CONS touch t (log index) of book h: its level and the makers it fills (fl_level_fc).
__device__ __forceinline__ FlTouchCtx fl_touch_ctx(const FlowArgs& F, uint32_t h, uint32_t L, const Touch& x, uint32_t t) {
  FlTouchCtx c;
  const FlTouchFc tf = F.tfc[L + t];
  c.Lq = fl_lvls(F, h) + tf.lvl;
  c.IG = F.ig + c.Lq->ig_base;
  c.RS = F.rs + L + c.Lq->base;
  c.c = tf.coord;
  c.a = x.amt * fl_amt_unit(F, h);
  c.first = tf.first;
  c.last = tf.last;
  return c;
}

// The same for every lane of a wave whose touches are consecutive from g0 (lane 0's, a multiple
// of 64): the book of g0's group from the range's map, then each lane steps over the (at most
// few) book boundaries after g0.  Called by every lane whose gt < total (lane 0 among them).
__device__ __forceinline__ uint32_t fl_book_of_wave(const FlowArgs& F, uint32_t nb, uint32_t g0, uint32_t gt) {
  uint32_t hb = F.tmap[static_cast<size_t>(F.mb) * F.tmap_stride + (g0 >> 6)];
  const uint32_t* to = F.toff + F.tb;
  while (hb + 1 < nb && to[hb + 1] <= gt) ++hb;
  return hb;
}

// Exclusive scan of the flow books' touch counts (declined candidates count 0).  KIND: the books
// the range's count / event kernels cover (FL_OK_ADD: k_flow_*, FL_OK_CANCEL: k_fc_*).
template <uint32_t KIND>
__global__ __launch_bounds__(1024) void k_flow_toff(Dev D, FlowArgs F) {
  __shared__ uint32_t part[1024];
  const uint32_t hend = fl_hend(D, F), nb = hend > F.h0 ? hend - F.h0 : 0u, tid = threadIdx.x;
  const FlowHdr* hdr = F.hdr + F.h0;
  uint32_t* toff = F.toff + F.tb;
  const uint32_t per = (nb + 1023) / 1024, b0 = tid * per;
  uint32_t s = 0;
  // (deep books with DELs count with the books with DELs: k_fc_count_nf / k_fc_events)
  auto mine = [&](const FlowHdr& x) {
    return x.ok == FL_OK_DEEP ? (KIND == (x.dc ? FL_OK_CANCEL : FL_OK_ADD)) : x.ok == KIND;
  };
  for (uint32_t i = b0; i < b0 + per && i < nb; ++i) s += mine(hdr[i]) ? hdr[i].ntouch : 0u;
  part[tid] = s;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < 1024; ++i) { const uint32_t v = part[i]; part[i] = acc; acc += v; }
    toff[nb] = acc;
  }
  __syncthreads();
  uint32_t acc = part[tid];
  for (uint32_t i = b0; i < b0 + per && i < nb; ++i) {
    toff[i] = acc;
    acc += mine(hdr[i]) ? hdr[i].ntouch : 0u;
  }
}

// The range's group map (FlowArgs::tmap), one wave per book: group g (touches [64g, 64g + 64))
// belongs to the book holding touch 64g.
__global__ __launch_bounds__(256) void k_flow_tmap(Dev D, FlowArgs F) {
  const uint32_t hend = fl_hend(D, F), nb = hend > F.h0 ? hend - F.h0 : 0u;
  const uint32_t* to = F.toff + F.tb;
  uint32_t* map = F.tmap + static_cast<size_t>(F.mb) * F.tmap_stride;
  for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < nb; i += gridDim.x * 4) {
    const uint32_t g0 = (to[i] + 63) >> 6, g1 = (to[i + 1] + 63) >> 6;
    for (uint32_t g = g0 + lane_id(); g < g1; g += 64) map[g] = i;
  }
}

// ============================================================== k_flow_events
// Lane-per-event emission.  A CONS touch fills makers first..last of its level; the touches of a
// wave hold very different counts (one taker sweeping a level of hundreds of makers beside takers
// filling one), so the events are not written by their touch's lane: each lane keeps its touch's
// context (FlEvLane, cnt == 0 for none), and the wave enumerates its events 64 at a time, every
// lane finding its touch by a binary search over the wave's inclusive counts (shuffles, no LDS).
// A lane's maker is usually the next lane's MatchNode.NextNode: taken by a shuffle, not reloaded.
// Stores of consecutive events are consecutive 64-B slots (coalesced).
struct FlEvLane {
  uint32_t inc;        // events of the wave's lanes <= this one
  uint32_t mb;         // maker index of wave event e: e + mb
  uint32_t dbase;      // its slot: dst[dbase + m]
  uint32_t fbm;        // its fill_idx: fbm + m
  uint32_t ig_n, nra;  // nra: new makers | ig_all << 31
  uint32_t igb, rsb, beg, t, idx, sym;
  int64_t c, ca, tbc, price;  // cursor before the touch, cursor after, taker volume + c, level price
};

__device__ __forceinline__ void fl_ev_lane(FlEvLane& r, const FlTouchCtx& c, uint32_t L, uint32_t beg, uint32_t t,
                                           uint32_t idx, uint32_t sym, int64_t tb) {
  r.ig_n = c.Lq->ig_n;
  r.nra = c.Lq->nrest | (c.Lq->ig_all ? 0x80000000u : 0u);
  r.igb = c.Lq->ig_base;
  r.rsb = L + c.Lq->base;
  r.beg = beg;
  r.t = t;
  r.idx = idx;
  r.sym = sym;
  r.c = c.c;
  r.ca = c.c + c.a;
  r.tbc = tb + c.c;
  r.price = c.Lq->price;
}

template <bool ARENA>
__device__ __forceinline__ void fl_emit_wave(const BatchArgs& B, const FlowArgs& F, gome_event* dst, const FlEvLane& x) {
  const uint32_t lane = lane_id();
  const uint32_t tot = __shfl(x.inc, 63);
  for (uint32_t e0 = 0; e0 < tot; e0 += 64) {
    const uint32_t e = e0 + lane;
    const bool v = e < tot;
    uint32_t lo = 0, hi = 63;  // the first lane k with inc[k] > e (inc[63] == tot)
#pragma unroll
    for (int it = 0; it < 6; ++it) {
      const uint32_t mid = (lo + hi) >> 1;
      if (__shfl(x.inc, static_cast<int>(mid)) > e) hi = mid; else lo = mid + 1;
    }
    const int k = static_cast<int>(lo);
    const uint32_t m = e + __shfl(x.mb, k);
    const uint32_t ig_n = __shfl(x.ig_n, k), nra = __shfl(x.nra, k), igb = __shfl(x.igb, k);
    const uint32_t rsb = __shfl(x.rsb, k), beg = __shfl(x.beg, k), t = __shfl(x.t, k);
    // (every shuffle before any lane leaves: a shuffle reads 0 from an inactive lane)
    const int64_t c = __shfl(x.c, k), ca = __shfl(x.ca, k), tbc = __shfl(x.tbc, k), price = __shfl(x.price, k);
    const uint32_t idx = __shfl(x.idx, k), fbm = __shfl(x.fbm, k), sym = __shfl(x.sym, k), dbase = __shfl(x.dbase, k);
    int64_t me = 0, mv = 0;
    uint32_t oid = 0, uuid = 0, tx = 0, rt = 0;
    if (v) {
      if (m < ig_n) {
        const IgEnt g = F.ig[igb + m];
        me = g.e; mv = g.v; oid = g.oid; uuid = g.uuid; tx = g.tx;
      } else {
        const RsEnt r = F.rs[rsb + m - ig_n];
        const Prep mk = B.prep[beg + r.j];
        me = r.e; mv = r.v; oid = mk.oid; uuid = mk.uuid; tx = mk.side; rt = r.t;
      }
    }
    // MatchNode.NextNode at the time of this fill: maker m + 1 of the same touch is the next lane's
    const uint32_t kn = __shfl_down(static_cast<uint32_t>(k), 1), oidn = __shfl_down(oid, 1), rtn = __shfl_down(rt, 1);
    if (!v) continue;
    const bool nbr = lane < 63 && e + 1 < tot && kn == static_cast<uint32_t>(k);
    const uint32_t nrest = nra & 0x7FFFFFFFu;
    uint32_t nx = 0, lst = 1;
    if (m + 1 < ig_n) {
      nx = nbr ? oidn : F.ig[igb + m + 1].oid;
      lst = 0;
    } else if ((nra >> 31) || m + 1 > ig_n) {
      const uint32_t r = m + 1 - ig_n;
      if (nbr) {
        if (rtn < t) { nx = oidn; lst = 0; }
      } else if (r < nrest) {
        const RsEnt rr = F.rs[rsb + r];
        if (rr.t < t) { nx = B.prep[beg + rr.j].oid; lst = 0; }
      }
    }
    const int64_t lo_ = me > c ? me : c;
    const int64_t hi_ = (me + mv < ca) ? me + mv : ca;
    const int64_t qty = hi_ - lo_, pre = me + mv - lo_;
    const bool full = me + mv <= ca;
    const unsigned long long sq = ARENA ? idx : B.seq_base + idx;  // arena: the batch index (k_publish)
    gome_event ev;
    ev.price_fx = price;
    ev.match_volume_fx = qty;
    ev.maker_volume_fx = full ? pre : pre - qty;
    ev.taker_seq = static_cast<uint32_t>(sq);
    ev.fill_idx = fbm + m;
    ev.maker_oid_id = oid;
    ev.maker_uuid_id = uuid;
    ev.maker_next_oid_id = nx;
    ev.kind = GOME_EV_FILL;
    ev.maker_side = static_cast<uint8_t>(tx);
    ev.maker_is_last = static_cast<uint8_t>(lst);
    ev.pad0 = 0;
    dst[dbase + m] = ev;
  }
}

// After the publish-order scan: every fill event of the hottest book at out[ev_off[taker] + fill_idx]
// (fill_idx bases from the count pass, F.fbase).
constexpr uint32_t FL_EV_T = 256;  // threads of the event kernels' blocks
constexpr uint32_t FL_WRITE_T = 1024;  // ... of the tail's (and of k_flow_write's)
// (blocks bid of nblk; k_publish runs it beside the arena scatter in one launch)
__device__ __forceinline__ void fl_events_hot(const Dev& D, const BatchArgs& B, const FlowArgs& F,
                                              const uint32_t* ev_off, gome_event* out, uint32_t bid, uint32_t nblk) {
  const uint32_t hend = fl_hend(D, F), nb = hend > F.h0 ? hend - F.h0 : 0u;
  const uint32_t total = nb ? F.toff[F.tb + nb] : 0u;
  const uint32_t lane = lane_id(), stride = nblk * blockDim.x;
  for (uint32_t b0 = bid * blockDim.x + (threadIdx.x & ~63u); b0 < total; b0 += stride) {
    const uint32_t gt = b0 + lane;
    uint32_t cnt = 0, first = 0;
    FlEvLane r{};
    const uint32_t hb = fl_book_of_wave(F, nb, b0, gt < total ? gt : b0);
    if (gt < total) {
      const uint32_t h = F.h0 + hb, t = gt - F.toff[F.tb + hb], beg = F.hdr[h].beg, L = FL_TOUCH_MUL * beg;
      const Touch x = F.log[L + t];
      if (((x.kr >> 7) & 1u) == TK_CONS) {
        const FlTouchCtx c = fl_touch_ctx(F, h, L, x, t);
        cnt = c.last - c.first + 1;
        first = c.first;
        const Prep tk = B.prep[beg + tk_j(x)];
        int64_t tb = tk.vol;  // taker remaining before this level: volume minus its better levels
        const int64_t gm = fl_amt_unit(F, h);
        for (uint32_t u = t; u > 0; --u) {
          const Touch y = F.log[L + u - 1];
          if (tk_j(y) != tk_j(x)) break;
          tb -= y.amt * gm;
        }
        fl_ev_lane(r, c, L, beg, t, tk.idx, F.hdr[h].sym, tb);
        const uint32_t fb = F.fbase[L + t];
        r.fbm = fb - c.first;
        r.dbase = ev_off[tk.idx] + fb - c.first;
      }
    }
    uint32_t inc = cnt;
    for (uint32_t off = 1; off < 64; off <<= 1) {
      const uint32_t v = __shfl_up(inc, off);
      if (lane >= off) inc += v;
    }
    r.inc = inc;
    r.mb = first - (inc - cnt);
    fl_emit_wave<false>(B, F, out, r);
  }
}
__global__ __launch_bounds__(256) void k_flow_events(Dev D, BatchArgs B, FlowArgs F, const uint32_t* ev_off,
                                                     gome_event* out) {
  fl_events_hot(D, B, F, ev_off, out, blockIdx.x, gridDim.x);
}

// Segmented inclusive wave scan: lane i sums lanes s..i, s = the last lane <= i with `head` set
// (lane 0 always starts a segment).
template <typename T>
__device__ __forceinline__ T wave_seg_incl(T v, unsigned long long heads) {
  const uint32_t lane = lane_id();
  const unsigned long long le = heads | 1ull;
  const uint32_t s = 63u - static_cast<uint32_t>(__builtin_clzll(le & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull))));
#pragma unroll
  for (uint32_t off = 1; off < 64; off <<= 1) {
    const T u = __shfl_up(v, off);
    if (lane >= off && lane - off >= s) v += u;
  }
  return v;
}

// ============================================================== k_flow_events_fused
// The books whose events go to the arena (the tail, the near head books): k_flow_count and
// the arena event writes in one pass over the touches.  An order's touches are consecutive in its
// book's log, so its fill_idx bases and the volume its better levels took are segmented scans
// over the touches (a wave's first lane walks back into an order begun before the wave); the
// order's last touch writes ev_count[taker].
// Blocks bid of nblk, T threads each.
// COUNT: the hottest book's count pass (its events are written after the publish scan, straight to
// their positions, by k_flow_events): each touch's fill_idx base to F.fbase, ev_count, no arena.
template <uint32_t T, bool COUNT = false>
__device__ __forceinline__ void fl_events_fused(const Dev& D, const BatchArgs& B, const FlowArgs& F, uint32_t bid,
                                                uint32_t nblk) {
  const uint32_t hend = fl_hend(D, F), nb = hend > F.h0 ? hend - F.h0 : 0u;
  const uint32_t total = nb ? F.toff[F.tb + nb] : 0u;
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6, stride = nblk * T;
  __shared__ uint32_t wtot[T / 64], bbase;
  unsigned long long fills = 0;
  for (uint32_t b0 = bid * T; b0 < total; b0 += stride) {
    const uint32_t gt = b0 + threadIdx.x, g0w = b0 + (threadIdx.x & ~63u);
    const bool valid = gt < total;
    uint32_t h = 0, L = 0, t = 0, beg = 0, j = 0, cnt = 0, hend_j = 0, sym = 0;
    int64_t gm = 1;
    Touch x{};
    FlTouchFc tf{};
    Prep tk{};
    const FlowLvl* Lq = nullptr;
    bool first = true, last = true;
    // (loads issued in dependence order, each stage's together: book -> header -> the touch, its
    // neighbours and its fill context -> the taker's record and the level)
    if (g0w < total) {
      const uint32_t hb = fl_book_of_wave(F, nb, g0w, valid ? gt : g0w);
      if (valid) {
        h = F.h0 + hb;
        t = gt - F.toff[F.tb + hb];
        const FlowHdr& H = F.hdr[h];
        gm = H.ok == FL_OK_ADD ? static_cast<int64_t>(H.g) : 1;  // (fl_amt_unit)
        const uint32_t nt = H.ntouch;
        beg = H.beg;
        hend_j = H.end - beg;
        sym = H.sym;
        L = FL_TOUCH_MUL * beg;
        x = F.log[L + t];
        const uint32_t jm = t > 0 ? tk_j(F.log[L + t - 1]) : NIL, jp = t + 1 < nt ? tk_j(F.log[L + t + 1]) : NIL;
        if (!COUNT) tf = F.tfc[L + t];  // (a CONS touch's; read before its kind is known)
        j = tk_j(x);
        first = jm != j;
        last = jp != j;
        const bool cons = ((x.kr >> 7) & 1u) == TK_CONS;
        if (COUNT) {
          if (cons) tf = F.tfc[L + t];
        } else if (j < hend_j) {
          tk = B.prep[beg + j];  // (padding records are never CONS and rest nowhere)
        }
        if (cons) {
          if (!COUNT) Lq = fl_lvls(F, h) + tf.lvl;
          cnt = tf.last - tf.first + 1;
          fills += cnt;
        }
      }
    }
    // the order's events and volume before this touch: segmented scans, plus lane 0's carry
    const unsigned long long heads = __ballot(first);
    uint32_t carry_n = 0;
    int64_t carry_a = 0;
    if (lane == 0 && !first) {
      for (uint32_t u = t; u > 0; --u) {
        const Touch y = F.log[L + u - 1];
        if (tk_j(y) != j) break;
        carry_a += y.amt * gm;
        if (((y.kr >> 7) & 1u) == TK_CONS) {
          const FlTouchFc ty = F.tfc[L + u - 1];
          carry_n += ty.last - ty.first + 1;
        }
      }
    }
    const bool in_first_seg = !(heads & 1ull) && ((heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull))) == 0ull);
    carry_n = __shfl(carry_n, 0);
    carry_a = __shfl(carry_a, 0);
    const uint32_t n_incl = wave_seg_incl<uint32_t>(cnt, heads) + (in_first_seg ? carry_n : 0u);
    const int64_t xa = valid ? x.amt * gm : 0;  // (plan units -> fixed point: fl_amt_unit)
    const int64_t a_incl = wave_seg_incl<int64_t>(xa, heads) + (in_first_seg ? carry_a : 0);
    const uint32_t fb = n_incl - cnt;  // the touch's fill_idx base within its order
    const int64_t a_before = a_incl - xa;
    if (COUNT) {
      if (valid && last && j < hend_j) B.ev_count[B.prep[beg + j].idx] = n_incl;  // (not padding)
      if (valid) F.fbase[L + t] = fb;
      continue;
    }
    if (valid && last && j < hend_j) B.ev_count[tk.idx] = n_incl;
    // arena slots: one bump allocation per block tile
    uint32_t inc = cnt;
    for (uint32_t off = 1; off < 64; off <<= 1) {
      const uint32_t v = __shfl_up(inc, off);
      if (lane >= off) inc += v;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t s = 0;
      for (uint32_t k = 0; k < T / 64; ++k) { const uint32_t v = wtot[k]; wtot[k] = s; s += v; }
      bbase = s ? atomicAdd(&D.st->ev_bump, s) : 0u;
      if (s && static_cast<unsigned long long>(bbase) + s > B.arena_cap) {
        atomicOr(&D.st->err, ERR_EVENTS);
        bbase = NIL;
      }
    }
    __syncthreads();
    const uint32_t base = bbase, wb = wtot[w];
    __syncthreads();  // (wtot / bbase are rewritten by the next tile)
    if (base == NIL) continue;
    FlEvLane r{};
    r.inc = inc;
    if (cnt) {
      r.ig_n = Lq->ig_n;
      r.nra = Lq->nrest | (Lq->ig_all ? 0x80000000u : 0u);
      r.igb = Lq->ig_base;
      r.rsb = L + Lq->base;
      r.price = Lq->price;
      r.beg = beg;
      r.t = t;
      r.idx = tk.idx;
      r.sym = sym;
      r.c = tf.coord;
      r.ca = tf.coord + x.amt * gm;
      r.tbc = tk.vol - a_before + tf.coord;  // (taker remaining before the level, + c)
      r.mb = tf.first - (inc - cnt);
      r.dbase = base + wb + (inc - cnt) - tf.first;
      r.fbm = fb - tf.first;
    }
    fl_emit_wave<true>(B, F, B.arena, r);
  }
  // the block's fills, then one stripe add per counter (ctr_add).  (The makers the fills pop are
  // counted by the writes, per level: fl_level_pops.)
  for (int off = 32; off > 0; off >>= 1) fills += __shfl_xor(fills, off);
  __shared__ unsigned long long wf[T / 64];
  if (lane == 0) wf[w] = fills;
  __syncthreads();
  if (threadIdx.x == 0) {
    fills = 0;
    for (uint32_t k = 0; k < T / 64; ++k) fills += wf[k];
    if (fills) {
      ctr_add(D, C_FILLS, fills);
      ctr_add(D, C_HOT_FILLS, fills);
      if (F.h0 >= FL_HEAD) ctr_add(D, C_FLOW_TAIL_FILLS, fills);
    }
  }
}
__global__ __launch_bounds__(FL_EV_T) void k_flow_events_fused(Dev D, BatchArgs B, FlowArgs F) {
  fl_events_fused<FL_EV_T>(D, B, F, blockIdx.x, gridDim.x);
}
// The tail's events: one arena claim per 1024 touches (a claim is a device-scope atomic on one
// address: 256-touch tiles made 22k of them on config 2's tail).
__global__ __launch_bounds__(FL_WRITE_T) void k_flow_events_fused_w(Dev D, BatchArgs B, FlowArgs F) {
  fl_events_fused<FL_WRITE_T>(D, B, F, blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(FL_EV_T) void k_flow_count_fused(Dev D, BatchArgs B, FlowArgs F) {
  fl_events_fused<FL_EV_T, true>(D, B, F, blockIdx.x, gridDim.x);
}

// ============================================================== k_flow_write
// One workgroup per flow book: append the surviving new makers to their FIFOs (chunks from
// the free stack / bump pool), insert them into the cancel index, rewrite the level array.

// Append level q's surviving new makers to its FIFO, insert them into the cancel index, and
// return (on every lane) the level's final record.
// New makers of level q that survive the batch (from rf on) and the FIFO chunks their append
// needs beyond the tail chunk's room.
struct FlWPlan {
  uint32_t rf, S, s0, room, need;
  bool fresh;
};
__device__ __forceinline__ FlWPlan fl_wplan(const FlowLvl& f, const RsEnt* RS) {
  FlWPlan w;
  w.rf = 0;
  // (zcont: the last consume went on and popped the zero-volume makers at the consumption end)
  const bool zc = f.cfin > 0 && f.zcont;
  if (f.cfin > f.d0 || (zc && f.cfin == f.d0)) {
    uint32_t lo = 0, hi = f.nrest;  // first r with e + v > cfin
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      // (a zero-volume maker (Q6) survives at the cursor: width 1, unless the last consume went on,
      // fl_cont; it rests after every consume of its level, k_flow_zero_check)
      if (RS[mid].e + (RS[mid].v ? RS[mid].v : (zc ? 0 : 1)) > f.cfin) hi = mid; else lo = mid + 1;
    }
    w.rf = lo;
  }
  w.S = f.nrest - w.rf;
  w.fresh = f.nlive0 == 0;
  w.s0 = w.fresh ? 0u : f.tslot;
  w.room = w.fresh ? 0u : CH - w.s0;
  w.need = w.S > w.room ? (w.S - w.room + CH - 1) / CH : 0u;
  return w;
}

// Makers of level f the batch's fills popped (filled to their whole volume): its consumed old
// makers and its new makers wholly inside the consumption (fl_wplan's rf).  Counted here, per
// level, rather than per fill by the event passes (where it cost a dependent load per touch).
__device__ __forceinline__ uint32_t fl_level_pops(const FlowLvl& f, uint32_t rf) { return f.nv0 - f.nlive0 + rf; }
__device__ __forceinline__ void ctr_pops(const Dev& D, uint32_t pops) {
  if (pops) ctr_add(D, C_RESTING_DELTA, static_cast<unsigned long long>(-static_cast<long long>(pops)));
}

// claim: a deep tail book's pre-claimed chunk ids (k_deep_claim; FlowLvl::pad0 = the level's
// first), else the level claims its own.
__device__ __forceinline__ Level fl_write_level(const Dev& D, const BatchArgs& B, const FlowArgs& F,
                                                const FlowHdr& hd, uint32_t h, uint32_t q,
                                                const FlClaim* claim = nullptr, uint32_t* pops = nullptr) {
  const uint32_t lane = lane_id();
  const uint32_t L = FL_TOUCH_MUL * hd.beg;
  const unsigned long long mask = D.idx_mask;
  const FlowLvl f = fl_lvls(F, h)[q];
  const RsEnt* RS = F.rs + L + f.base;
  Level x{};
  x.price = f.price;
  x.head = x.tail = NIL;
  const FlWPlan wp = fl_wplan(f, RS);
  const uint32_t rf = wp.rf, S = wp.S, s0 = wp.s0, room = wp.room, need = wp.need;
  const bool fresh = wp.fresh;
  if (pops) *pops += fl_level_pops(f, rf);
  // claim `need` chunk ids: free stack first, then the bump pointer
  int t = 0;
  uint32_t nst = 0, bb = 0;
  if (need && claim) {  // ids [pad0, pad0 + need) of the book's claim
    if (!claim->c_ok) return x;  // (ERR_CHUNKS set by the claim)
    const uint32_t j0 = f.pad0, cn = claim->c_nst;
    nst = j0 < cn ? min(cn - j0, need) : 0u;
    t = claim->c_t - static_cast<int>(cn) + static_cast<int>(j0) + static_cast<int>(nst);
    bb = claim->c_bb + (j0 + nst - cn);
  } else if (need) {
    if (lane == 0) t = atomicSub(&D.st->free_top, static_cast<int>(need));
    t = static_cast<int>(uni(static_cast<uint32_t>(t)));
    nst = static_cast<uint32_t>(min(max(t, 0), static_cast<int>(need)));
    if (lane == 0 && nst < need) bb = atomicAdd(D.ch_bump, need - nst);
    bb = uni(bb);
    if (bb + (need - nst) > D.ch_cap) {
      if (lane == 0) atomicOr(&D.st->err, ERR_CHUNKS);
      return x;
    }
  }
  auto chunk_id = [&](uint32_t i) -> uint32_t {
    return i < nst ? D.free_ids[t - static_cast<int>(nst) + static_cast<int>(i)] : bb + (i - nst);
  };
  for (uint32_t i = lane; i < need; i += 64) {
    ChunkHdr c;
    c.next = (i + 1 < need) ? chunk_id(i + 1) : NIL;
    c.pad = 0;
    c.price = f.price;
    D.chdr[chunk_id(i)] = c;
  }
  if (need && !fresh && lane == 0) D.chdr[f.tail].next = chunk_id(0);
  for (uint32_t i = lane; i < S; i += 64) {
    const RsEnt r = RS[rf + i];
    const Prep mk = B.prep[hd.beg + r.j];
    const int64_t rem = (r.e < f.cfin) ? r.e + r.v - f.cfin : r.v;
    uint32_t cid, slot;
    if (!fresh && s0 + i < CH) {
      cid = f.tail;
      slot = s0 + i;
    } else {
      const uint32_t g = fresh ? i : i - room;
      cid = chunk_id(g / CH);
      slot = g % CH;
    }
    const uint32_t loc = cid * CH + slot;
    const unsigned long long key = (static_cast<unsigned long long>(hd.sym + 1) << 32) | mk.oid;
    unsigned long long hh = mix64(key) & mask, probe = 0;
    for (; probe <= mask; ++probe, hh = (hh + 1) & mask) {
      const unsigned long long kv = __hip_atomic_load(&D.idx[hh].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((kv == KEY_EMPTY || kv == KEY_TOMB) && atomicCAS(&D.idx[hh].key, kv, key) == kv) break;
    }
    if (probe > mask) { atomicOr(&D.st->err, ERR_INDEX); continue; }
    D.idx[hh].loc = loc;
    Node nd{};
    nd.rem = rem;
    nd.oid = mk.oid;
    nd.uuid = mk.uuid;
    nd.ixs = static_cast<uint32_t>(hh);
    nd.tx = mk.side;
    D.nodes[loc] = nd;
  }
  x.depth = f.dfin;
  x.nlive = f.nlive0 + S;
  uint32_t mem = 0;
  if (hd.ok == FL_OK_DEEP) {
    mem = f.memf;
  } else {
    if (((q < 64 ? hd.amask[0] : hd.amask[1]) >> (q & 63)) & 1ull) mem |= M_SALE;
    if (((q < 64 ? hd.bmask[0] : hd.bmask[1]) >> (q & 63)) & 1ull) mem |= M_BUY;
  }
  x.member = static_cast<uint8_t>(mem);
  if (x.nlive == 0) {
    x.hslot = x.tslot = 0;
  } else if (fresh) {
    x.head = chunk_id(0);
    x.hslot = 0;
    x.tail = chunk_id(need - 1);
    x.tslot = static_cast<uint8_t>(S - (need - 1) * CH);
  } else {
    x.head = f.head;
    x.hslot = static_cast<uint8_t>(f.hslot);
    x.tail = need ? chunk_id(need - 1) : f.tail;
    x.tslot = static_cast<uint8_t>(need ? (S - room) - (need - 1) * CH : s0 + S);
  }
  // clean-book invariant: nodes <=> positive depth <=> one side-set membership
  const bool ok = (x.nlive > 0) == (x.depth > 0) && (x.nlive > 0) == (mem == M_BUY || mem == M_SALE) &&
                  (x.nlive > 0 || mem == 0);
  if (!ok && lane == 0) atomicOr(&D.st->err, ERR_CORRUPT);
  return x;
}

// Compact the book's final levels (lv[1..nl], LDS) into its level block, write the Book and
// the batch counters.  Called by every thread of the block after lv is complete.
__device__ __forceinline__ void fl_write_finish(const Dev& D, const FlowHdr& hd, Level* lv, uint32_t* keep,
                                                uint32_t& base_s, uint32_t& cap_s, uint32_t& nout_s) {
  __shared__ uint32_t zflag_s;
  if (threadIdx.x == 0) {
    uint32_t c = 0;
    for (uint32_t q = 1; q <= hd.nl; ++q) {
      const uint32_t k = (lv[q].nlive > 0 || lv[q].member != 0) ? 1u : 0u;  // (member, no node: stale)
      keep[q] = k ? c : NIL;
      c += k;
    }
    nout_s = c;
    uint32_t fl = 0;  // levels that may hold zero-volume makers (BOOK_ZERO); stale members (BOOK_STALE)
    for (uint32_t q = 1; q <= hd.nl; ++q) {
      if (keep[q] == NIL) continue;
      if (lv[q].pad) fl |= BOOK_ZERO;
      if (lv[q].nlive == 0) fl |= BOOK_STALE;
    }
    zflag_s = fl;
    const Book bk = D.books[hd.sym];
    uint32_t base = bk.lvl_base, cap = bk.lvl_cap;
    if (c > cap) {
      uint32_t ncap = 16;
      while (ncap < c) ncap <<= 1;
      const uint32_t nb = lvl_block_alloc(D, ncap);
      if (nb == NIL) {
        atomicOr(&D.st->err, ERR_LEVELS);
        cap = 0;
      } else {
        lvl_block_release(D, base, cap);  // the book's old block (reusable from the next batch)
        base = nb;
        cap = ncap;
      }
    }
    base_s = base;
    cap_s = cap;
  }
  __syncthreads();
  const uint32_t nout = nout_s;
  if (nout > cap_s) return;
  for (uint32_t q = 1 + threadIdx.x; q <= hd.nl; q += blockDim.x)
    if (keep[q] != NIL) D.lvl[base_s + keep[q]] = lv[q];
  if (threadIdx.x == 0) {
    Book nb;
    nb.lvl_base = base_s;
    nb.n_lvl = nout;
    nb.lvl_cap = cap_s;
    nb.pad = zflag_s;
    D.books[hd.sym] = nb;
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
  }
}

// Tail books: one workgroup per book.  Thread i plans level i + 1 (fl_wplan); one block scan
// of the levels' surviving new makers and new chunks, one chunk claim for the book; then every
// thread takes surviving makers of the whole book (its level by a binary search over the scan),
// so the book's FIFO appends and index inserts are all in flight at once instead of one level
// per wave in turn (a tail book's level holds a few new makers: most of a wave idled); the
// chunk headers the same way; then the level records and the finish.
__device__ __forceinline__ void fl_write_book(const Dev& D, const BatchArgs& B, const FlowArgs& F, uint32_t h) {
  static_assert(FL_CAP <= 128, "one wave plans a book's levels, two per lane");
  __shared__ Level lv[FL_CAP];
  __shared__ uint32_t keep[FL_CAP];
  __shared__ uint32_t nout_s, base_s, cap_s;
  __shared__ uint32_t rof[FL_CAP + 1], cof[FL_CAP + 1];  // exclusive scans: surviving makers, new chunks
  __shared__ uint32_t wrf[FL_CAP], wtl[FL_CAP], wbs[FL_CAP], ws0[FL_CAP];  // ws0: s0 | fresh << 31
  __shared__ int64_t wcf[FL_CAP];
  __shared__ FlClaim claim_s;
  __shared__ uint32_t pops_s;
  if (h >= fl_hend(D, F) || F.hdr[h].ok != FL_OK_ADD) return;
  const FlowHdr hd = F.hdr[h];
  const uint32_t tid = threadIdx.x, lane = lane_id(), nl = hd.nl;
  const FlowLvl* LV = F.lvl + h * FL_CAP;
  const uint32_t L = FL_TOUCH_MUL * hd.beg;
  const unsigned long long mask = D.idx_mask;
  if (tid < 64) {  // wave 0: levels 2 lane + 1 and 2 lane + 2
    int64_t x = 0, x0 = 0;  // (S, need) packed: need < 2^32 over a book
#pragma unroll
    for (uint32_t u = 0; u < 2; ++u) {
      const uint32_t i = 2 * tid + u;
      if (i < nl) {
        const FlowLvl& f = LV[i + 1];
        const FlWPlan wp = fl_wplan(f, F.rs + L + f.base);
        wrf[i] = wp.rf;
        wtl[i] = f.tail;
        wbs[i] = f.base;
        ws0[i] = wp.s0 | (wp.fresh ? 0x80000000u : 0u);
        wcf[i] = f.cfin;
        const int64_t v = (static_cast<int64_t>(wp.S) << 32) | wp.need;
        if (u == 0) x0 = v;
        x += v;
      }
    }
    const int64_t ex = wave_incl_scan(x) - x;
    rof[2 * tid] = static_cast<uint32_t>(ex >> 32);
    cof[2 * tid] = static_cast<uint32_t>(ex);
    rof[2 * tid + 1] = static_cast<uint32_t>((ex + x0) >> 32);
    cof[2 * tid + 1] = static_cast<uint32_t>(ex + x0);
    if (tid == 0) pops_s = 0;
    if (tid == 63) {
      const int64_t tot = ex + x;
      rof[128] = static_cast<uint32_t>(tot >> 32);
      cof[128] = static_cast<uint32_t>(tot);
      claim_s = fl_claim_chunks(D, static_cast<uint32_t>(tot));
    }
  }
  __syncthreads();
  const FlClaim cl = claim_s;
  auto cid = [&](uint32_t c) -> uint32_t {  // the book's c-th new chunk
    return c < cl.c_nst ? D.free_ids[cl.c_t - static_cast<int>(cl.c_nst) + static_cast<int>(c)] : cl.c_bb + (c - cl.c_nst);
  };
  // the last level i (0-based) with off[i] <= g (off[0] = 0 <= g; nl >= 1)
  auto level_of = [&](const uint32_t* off, uint32_t g) -> uint32_t {
    uint32_t lo = 0, hi = nl - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (off[mid] <= g) lo = mid; else hi = mid - 1;
    }
    return lo;
  };
  const uint32_t nch = cof[nl], nsv = rof[nl];
  if (cl.c_ok) {
    for (uint32_t c = tid; c < nch; c += FL_WRITE_T) {
      const uint32_t i = level_of(cof, c);
      ChunkHdr ch;
      ch.next = c + 1 < cof[i + 1] ? cid(c + 1) : NIL;
      ch.pad = 0;
      ch.price = LV[i + 1].price;
      D.chdr[cid(c)] = ch;
    }
  }
  for (uint32_t g = tid; g < nsv; g += FL_WRITE_T) {
    const uint32_t i = level_of(rof, g), k = g - rof[i];
    const bool needs = cof[i + 1] > cof[i];
    if (needs && !cl.c_ok) continue;  // (ERR_CHUNKS set by the claim)
    const RsEnt r = F.rs[L + wbs[i] + wrf[i] + k];
    const Prep mk = B.prep[hd.beg + r.j];
    const int64_t cfin = wcf[i];
    const int64_t rem = (r.e < cfin) ? r.e + r.v - cfin : r.v;
    const uint32_t s0 = ws0[i] & 0x7FFFFFFFu;
    const bool fresh = ws0[i] >> 31;
    const uint32_t room = fresh ? 0u : CH - s0;
    uint32_t c, slot;
    if (!fresh && s0 + k < CH) {
      c = wtl[i];
      slot = s0 + k;
    } else {
      const uint32_t gg = fresh ? k : k - room;
      c = cid(cof[i] + gg / CH);
      slot = gg % CH;
    }
    const uint32_t loc = c * CH + slot;
    const unsigned long long key = (static_cast<unsigned long long>(hd.sym + 1) << 32) | mk.oid;
    unsigned long long hh = mix64(key) & mask, probe = 0;
    for (; probe <= mask; ++probe, hh = (hh + 1) & mask) {
      const unsigned long long kv = __hip_atomic_load(&D.idx[hh].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((kv == KEY_EMPTY || kv == KEY_TOMB) && atomicCAS(&D.idx[hh].key, kv, key) == kv) break;
    }
    if (probe > mask) { atomicOr(&D.st->err, ERR_INDEX); continue; }
    D.idx[hh].loc = loc;
    Node nd{};
    nd.rem = rem;
    nd.oid = mk.oid;
    nd.uuid = mk.uuid;
    nd.ixs = static_cast<uint32_t>(hh);
    nd.tx = mk.side;
    D.nodes[loc] = nd;
  }
  if (tid < nl) {  // the level's final record
    const FlowLvl& f = LV[tid + 1];
    if (const uint32_t p = fl_level_pops(f, wrf[tid])) atomicAdd(&pops_s, p);
    const uint32_t q = tid + 1, S = rof[tid + 1] - rof[tid], need = cof[tid + 1] - cof[tid];
    const uint32_t s0 = ws0[tid] & 0x7FFFFFFFu;
    const bool fresh = ws0[tid] >> 31;
    const uint32_t room = fresh ? 0u : CH - s0;
    Level x{};
    x.price = f.price;
    x.head = x.tail = NIL;
    if (need && !cl.c_ok) {
      lv[q] = x;
    } else {
      if (need && !fresh) D.chdr[f.tail].next = cid(cof[tid]);
      x.depth = f.dfin;
      x.nlive = f.nlive0 + S;
      uint32_t mem = 0;
      if (((q < 64 ? hd.amask[0] : hd.amask[1]) >> (q & 63)) & 1ull) mem |= M_SALE;
      if (((q < 64 ? hd.bmask[0] : hd.bmask[1]) >> (q & 63)) & 1ull) mem |= M_BUY;
      x.member = static_cast<uint8_t>(mem);
      if (x.nlive == 0) {
        x.hslot = x.tslot = 0;
      } else if (fresh) {
        x.head = cid(cof[tid]);
        x.hslot = 0;
        x.tail = cid(cof[tid] + need - 1);
        x.tslot = static_cast<uint8_t>(S - (need - 1) * CH);
      } else {
        x.head = f.head;
        x.hslot = static_cast<uint8_t>(f.hslot);
        x.tail = need ? cid(cof[tid] + need - 1) : f.tail;
        x.tslot = static_cast<uint8_t>(need ? (S - room) - (need - 1) * CH : s0 + S);
      }
      // clean-book invariant: nodes <=> positive depth <=> one side-set membership
      const bool ok = (x.nlive > 0) == (x.depth > 0) && (x.nlive > 0) == (mem == M_BUY || mem == M_SALE) &&
                      (x.nlive > 0 || mem == 0);
      if (!ok) atomicOr(&D.st->err, ERR_CORRUPT);
      lv[q] = x;
    }
  }
  __syncthreads();
  if (tid == 0) ctr_pops(D, pops_s);
  fl_write_finish(D, hd, lv, keep, base_s, cap_s, nout_s);
}
__global__ __launch_bounds__(FL_WRITE_T) void k_flow_write(Dev D, BatchArgs B, FlowArgs F) {
  fl_write_book(D, B, F, F.h0 + blockIdx.x);
}

// The tail's writes and events in one launch (both need only the level pass, and both wait on
// memory latency, so they overlap): blocks [0, nwb) write book h0 + blockIdx.x, the rest run the
// fused event pass in FL_WRITE_T-thread tiles.
__global__ __launch_bounds__(FL_WRITE_T) void k_flow_write_events(Dev D, BatchArgs B, FlowArgs F, uint32_t nwb) {
  if (blockIdx.x < nwb) {
    fl_write_book(D, B, F, F.h0 + blockIdx.x);
    return;
  }
  fl_events_fused<FL_WRITE_T>(D, B, F, blockIdx.x - nwb, gridDim.x - nwb);
}

// Head books: fl_write_level with a whole block (FL_LVB_T threads) per (book, level) -- the chunk
// headers and the surviving new makers (thousands on the hottest book's levels) in block-wide
// strides -- storing the level's final record ...
__global__ __launch_bounds__(FL_LVB_T) void k_flow_write_lv_blk(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ int t_s;
  __shared__ uint32_t nst_s, bb_s, bad_s;
  const uint32_t h = F.h0 + blockIdx.y, q = blockIdx.x, tid = threadIdx.x;
  if (h >= fl_hend(D, F) || F.hdr[h].ok != FL_OK_ADD) return;
  const FlowHdr hd = F.hdr[h];
  if (q == 0 || q > hd.nl) return;
  const uint32_t L = FL_TOUCH_MUL * hd.beg;
  const unsigned long long mask = D.idx_mask;
  const FlowLvl f = fl_lvls(F, h)[q];
  const RsEnt* RS = F.rs + L + f.base;
  const FlWPlan wp = fl_wplan(f, RS);
  const uint32_t rf = wp.rf, S = wp.S, s0 = wp.s0, room = wp.room, need = wp.need;
  const bool fresh = wp.fresh;
  __shared__ uint32_t zadd_s;
  uint32_t zs = 0;
  if (tid == 0) {  // claim `need` chunk ids: free stack first, then the bump pointer
    zadd_s = 0;
    int t = 0;
    uint32_t nst = 0, bb = 0;
    if (need) {
      t = atomicSub(&D.st->free_top, static_cast<int>(need));
      nst = static_cast<uint32_t>(min(max(t, 0), static_cast<int>(need)));
      if (nst < need) bb = atomicAdd(D.ch_bump, need - nst);
    }
    t_s = t;
    nst_s = nst;
    bb_s = bb;
    bad_s = need && bb + (need - nst) > D.ch_cap ? 1u : 0u;
    if (bad_s) atomicOr(&D.st->err, ERR_CHUNKS);
  }
  __syncthreads();
  if (bad_s) {
    if (tid == 0) {
      Level x{};
      x.price = f.price;
      x.head = x.tail = NIL;
      F.lvout[h * FL_CAP + q] = x;
    }
    return;
  }
  const int t = t_s;
  const uint32_t nst = nst_s, bb = bb_s;
  auto chunk_id = [&](uint32_t i) -> uint32_t {
    return i < nst ? D.free_ids[t - static_cast<int>(nst) + static_cast<int>(i)] : bb + (i - nst);
  };
  for (uint32_t i = tid; i < need; i += FL_LVB_T) {
    ChunkHdr c;
    c.next = (i + 1 < need) ? chunk_id(i + 1) : NIL;
    c.pad = 0;
    c.price = f.price;
    D.chdr[chunk_id(i)] = c;
  }
  if (need && !fresh && tid == 0) D.chdr[f.tail].next = chunk_id(0);
  for (uint32_t i = tid; i < S; i += FL_LVB_T) {
    const RsEnt r = RS[rf + i];
    const Prep mk = B.prep[hd.beg + r.j];
    const int64_t rem = (r.e < f.cfin) ? r.e + r.v - f.cfin : r.v;
    uint32_t cid, slot;
    if (!fresh && s0 + i < CH) {
      cid = f.tail;
      slot = s0 + i;
    } else {
      const uint32_t g = fresh ? i : i - room;
      cid = chunk_id(g / CH);
      slot = g % CH;
    }
    const uint32_t loc = cid * CH + slot;
    const unsigned long long key = (static_cast<unsigned long long>(hd.sym + 1) << 32) | mk.oid;
    unsigned long long hh = mix64(key) & mask, probe = 0;
    for (; probe <= mask; ++probe, hh = (hh + 1) & mask) {
      const unsigned long long kv = __hip_atomic_load(&D.idx[hh].key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((kv == KEY_EMPTY || kv == KEY_TOMB) && atomicCAS(&D.idx[hh].key, kv, key) == kv) break;
    }
    if (probe > mask) { atomicOr(&D.st->err, ERR_INDEX); continue; }
    D.idx[hh].loc = loc;
    Node nd{};
    nd.rem = rem;
    nd.oid = mk.oid;
    nd.uuid = mk.uuid;
    nd.ixs = static_cast<uint32_t>(hh);
    nd.tx = mk.side;
    D.nodes[loc] = nd;
    zs += r.v == 0 ? 1u : 0u;
  }
  // zero-volume makers in the level's FIFO after the batch (Q6): the old ones the batch did not pop
  // and the ones appended now (Level::pad)
  if (zs) atomicAdd(&zadd_s, zs);
  __syncthreads();
  const uint32_t zadd = zadd_s;
  if (tid != 0) return;
  ctr_pops(D, fl_level_pops(f, rf));
  Level x{};
  x.price = f.price;
  x.head = x.tail = NIL;
  x.depth = f.dfin;
  x.nlive = f.nlive0 + S;
  uint32_t mem = 0;
  if (((q < 64 ? hd.amask[0] : hd.amask[1]) >> (q & 63)) & 1ull) mem |= M_SALE;
  if (((q < 64 ? hd.bmask[0] : hd.bmask[1]) >> (q & 63)) & 1ull) mem |= M_BUY;
  // a stale member no order touched stays one (a touch of it heals or, k_flow_stale_check, bails)
  const bool stale = fl_stale0(f) && f.cnt == 0;
  if (stale) mem = f.mem0;
  x.member = static_cast<uint8_t>(mem);
  if (x.nlive == 0) {
    x.hslot = x.tslot = 0;
  } else if (fresh) {
    x.head = chunk_id(0);
    x.hslot = 0;
    x.tail = chunk_id(need - 1);
    x.tslot = static_cast<uint8_t>(S - (need - 1) * CH);
  } else {
    x.head = f.head;
    x.hslot = static_cast<uint8_t>(f.hslot);
    x.tail = need ? chunk_id(need - 1) : f.tail;
    x.tslot = static_cast<uint8_t>(need ? (S - room) - (need - 1) * CH : s0 + S);
  }
  // clean-book invariant: nodes <=> positive depth <=> one side-set membership (or an untouched
  // stale member: no nodes, depth 0, one side)
  const bool ok = stale ? (x.nlive == 0 && x.depth == 0)
                        : (x.nlive > 0) == (x.depth > 0) && (x.nlive > 0) == (mem == M_BUY || mem == M_SALE) &&
                              (x.nlive > 0 || mem == 0);
  if (!ok) atomicOr(&D.st->err, ERR_CORRUPT);
  x.pad = x.nlive ? l_zero_count(f.z0, f.zpop, zadd) : 0u;
  F.lvout[h * FL_CAP + q] = x;
}

// ... then one workgroup per head book compacts the level array.
__global__ __launch_bounds__(128) void k_flow_write_fin(Dev D, FlowArgs F) {
  __shared__ Level lv[FL_CAP];
  __shared__ uint32_t keep[FL_CAP];
  __shared__ uint32_t nout_s, base_s, cap_s;
  const uint32_t h = F.h0 + blockIdx.x;
  if (h >= fl_hend(D, F) || F.hdr[h].ok != FL_OK_ADD) return;
  const FlowHdr hd = F.hdr[h];
  for (uint32_t q = 1 + threadIdx.x; q <= hd.nl; q += blockDim.x) lv[q] = F.lvout[h * FL_CAP + q];
  __syncthreads();
  fl_write_finish(D, hd, lv, keep, base_s, cap_s, nout_s);
  if (threadIdx.x == 0 && F.h0 == 0) {  // k_flow_plan_head's work (its roofline numerator)
    ctr_add(D, C_FLOW_HEAD_ORDERS, static_cast<unsigned long long>(hd.end - hd.beg));
    ctr_add(D, C_FLOW_HEAD_TOUCHES, static_cast<unsigned long long>(hd.ntouch));
    ctr_add(D, C_HEAD_ADD, 1ull);
  }
}

// ============================================================== head: wide sort and levels
// The head books' touch logs are long (the hottest book: ~450k touches): sort them with one
// workgroup per 1024-touch tile (count -> per-book scan -> scatter) instead of one per book,
// and their levels with one wave per (book, level).
constexpr uint32_t FL_TILE = 1024, FL_TILE_W = FL_TILE / 64, FL_SORT_GRID = 512;

// stable in-tile rank of a touch among the tile's touches of the same level
__device__ __forceinline__ uint32_t fl_tile_rank(uint32_t k, bool valid, uint32_t& cnt) {
  unsigned long long same = __ballot(valid);
#pragma unroll
  for (uint32_t b = 0; b < 7; ++b) {
    const unsigned long long bb = __ballot((k >> b) & 1u);
    same &= ((k >> b) & 1u) ? bb : ~bb;
  }
  cnt = __popcll(same);
  return __popcll(same & lt_mask());
}

__global__ __launch_bounds__(FL_TILE) void k_flow_sort_cnt(Dev D, FlowArgs F) {
  __shared__ uint32_t wc[FL_TILE_W][FL_CAP];
  __shared__ uint32_t nrest;
  const uint32_t hb = blockIdx.y, h = F.h0 + hb, tid = threadIdx.x, w = tid >> 6;
  if (h >= fl_hend(D, F) || !F.hdr[h].ok || F.hdr[h].ok == FL_OK_DEEP) return;
  const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg;
  const uint32_t ntile = (nt + FL_TILE - 1) / FL_TILE;
  const bool cb = F.hdr[h].ok == FL_OK_CANCEL;
  for (uint32_t tl = blockIdx.x; tl < ntile; tl += gridDim.x) {
    for (uint32_t i = tid; i < FL_TILE_W * FL_CAP; i += FL_TILE) wc[i / FL_CAP][i % FL_CAP] = 0;
    if (tid == 0) nrest = 0;
    __syncthreads();
    const uint32_t t = tl * FL_TILE + tid;
    const bool valid = t < nt;
    const uint32_t kr = valid ? F.log[L + t].kr : 0u, k = kr & 127u;
    uint32_t cnt;
    const uint32_t rank = fl_tile_rank(k, valid, cnt);
    if (valid && rank == 0) wc[w][k] = cnt;
    const unsigned long long rm = __ballot(valid && tk_kind(kr, cb) == TK_REST && k);
    if (lane_id() == 0 && rm) atomicAdd(&nrest, static_cast<uint32_t>(__popcll(rm)));
    __syncthreads();
    if (tid < FL_CAP) {
      uint32_t c = 0;
      for (uint32_t ww = 0; ww < FL_TILE_W; ++ww) c += wc[ww][tid];
      F.tcnt[(static_cast<size_t>(h) * F.maxt + tl) * FL_CAP + tid] = c;  // (head books: h < FL_HEAD)
    }
    if (tid == 0 && nrest) atomicAdd(&F.hdr[h].rests, nrest);
    __syncthreads();
  }
}

// Per head book: level totals -> run bases (FlowLvl::cnt/base), then each tile's offset per
// level (in place over the counts).
// FL_SCAN_P threads per level, each over a contiguous range of the tiles (the hottest book has
// ~450 tiles: one thread per level walking them all twice took 26 us on the critical path).
constexpr uint32_t FL_SCAN_P = 8;
__global__ __launch_bounds__(FL_CAP * FL_SCAN_P) void k_flow_sort_scan(Dev D, FlowArgs F) {
  __shared__ uint32_t part[FL_SCAN_P][FL_CAP];
  __shared__ uint32_t tot[FL_CAP], cnt[FL_CAP];
  const uint32_t hb = blockIdx.x, h = F.h0 + hb, k = threadIdx.x % FL_CAP, p = threadIdx.x / FL_CAP;
  if (h >= fl_hend(D, F) || !F.hdr[h].ok || F.hdr[h].ok == FL_OK_DEEP) return;
  const uint32_t nt = F.hdr[h].ntouch, nl = F.hdr[h].nl;
  const uint32_t ntile = (nt + FL_TILE - 1) / FL_TILE;
  const uint32_t per = (ntile + FL_SCAN_P - 1) / FL_SCAN_P, t0 = min(p * per, ntile), t1 = min(t0 + per, ntile);
  uint32_t* tc = F.tcnt + static_cast<size_t>(h) * F.maxt * FL_CAP;
  uint32_t s = 0;
  uint32_t tl = t0;
  for (; tl + 8 <= t1; tl += 8) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = tc[(tl + u) * FL_CAP + k];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; tl < t1; ++tl) s += tc[tl * FL_CAP + k];
  part[p][k] = s;
  __syncthreads();
  if (p == 0) {  // the level's parts -> their offsets within the level, and its total
    uint32_t acc = 0;
    for (uint32_t q = 0; q < FL_SCAN_P; ++q) {
      const uint32_t v = part[q][k];
      part[q][k] = acc;
      acc += v;
    }
    cnt[k] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (uint32_t i = 0; i < FL_CAP; ++i) { tot[i] = acc; acc += cnt[i]; }
  }
  __syncthreads();
  const uint32_t base = tot[k];
  if (p == 0 && k >= 1 && k <= nl) {
    F.lvl[h * FL_CAP + k].cnt = cnt[k];
    F.lvl[h * FL_CAP + k].base = base;
  }
  uint32_t run = base + part[p][k];
  for (tl = t0; tl + 8 <= t1; tl += 8) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = tc[(tl + u) * FL_CAP + k];
#pragma unroll
    for (int u = 0; u < 8; ++u) { tc[(tl + u) * FL_CAP + k] = run; run += v[u]; }
  }
  for (; tl < t1; ++tl) {
    const uint32_t v = tc[tl * FL_CAP + k];
    tc[tl * FL_CAP + k] = run;
    run += v;
  }
}

__global__ __launch_bounds__(FL_TILE) void k_flow_sort_scatter(Dev D, FlowArgs F) {
  __shared__ uint32_t wc[FL_TILE_W][FL_CAP];
  const uint32_t hb = blockIdx.y, h = F.h0 + hb, tid = threadIdx.x, w = tid >> 6;
  if (h >= fl_hend(D, F) || !F.hdr[h].ok || F.hdr[h].ok == FL_OK_DEEP) return;
  const uint32_t nt = F.hdr[h].ntouch, L = FL_TOUCH_MUL * F.hdr[h].beg;
  const unsigned long long g = F.hdr[h].g;
  const bool cb = F.hdr[h].ok == FL_OK_CANCEL;
  const uint32_t ntile = (nt + FL_TILE - 1) / FL_TILE;
  const uint32_t* tc = F.tcnt + static_cast<size_t>(h) * F.maxt * FL_CAP;
  for (uint32_t i = tid; i < FL_TILE_W * FL_CAP; i += FL_TILE) wc[i / FL_CAP][i % FL_CAP] = 0;
  __syncthreads();
  for (uint32_t tl = blockIdx.x; tl < ntile; tl += gridDim.x) {
    const uint32_t t = tl * FL_TILE + tid;
    const bool valid = t < nt;
    Touch x{};
    if (valid) x = F.log[L + t];
    const uint32_t k = valid ? (x.kr & 127u) : 0u;
    uint32_t cnt;
    const uint32_t rank = fl_tile_rank(k, valid, cnt);
    if (valid && rank == 0) wc[w][k] = cnt;
    __syncthreads();
    if (tid < FL_CAP) {  // prefix over the waves, from the tile's offset of each level
      uint32_t r = tc[tl * FL_CAP + tid];
      for (uint32_t ww = 0; ww < FL_TILE_W; ++ww) {
        const uint32_t c = wc[ww][tid];
        wc[ww][tid] = r;
        r += c;
      }
    }
    __syncthreads();
    if (valid) {
      SEnt e;
      e.j = tk_jb(x, cb);
      e.kind = tk_kind(x.kr, cb);
      e.amt = static_cast<int64_t>(static_cast<unsigned long long>(x.amt) * g);
      e.coord = 0;
      e.t = t;
      e.lvl = k;
      const uint32_t pos = wc[w][k] + rank;
      F.srt[L + pos] = e;
      if (cb) {  // (as k_flow_sort)
        F.log[L + t].pos = pos;
        if (g != 1) F.log[L + t].amt = e.amt;
      }
    }
    __syncthreads();
    // stale wc entries of levels absent from the next tile are never read: only a wave's
    // present levels are written before the prefix, and the prefix reads every level, so clear
    for (uint32_t i = tid; i < FL_TILE_W * FL_CAP; i += FL_TILE) wc[i / FL_CAP][i % FL_CAP] = 0;
    __syncthreads();
  }
}

// Books planned with zero-volume ADDs (Q6, k_flow_prep_b) or holding zero-volume makers (FlowLvl::z0):
// the reconstruction takes a zero-volume maker where no order reaches it, and where a consume passes
// it or goes on past the level's end (it pops it with a 0-fill, engine.go:145-161).  One block
// per (book, level), the level's run in time order with block scans; hazards (FlowHdr::haz, handed
// over by k_flow_stale_check):
//  * a REST of 0 while the level's depth is 0: the reference makes it a side-set member of depth 0
//    (SetPoolDepth, engine.go:78-80), which the plans, seeing depth 0 as "no level", would not visit;
//  * after a zero-volume maker may be in the FIFO (z0, or a REST of 0 earlier in the run): a CONS that
//    empties the level and stops there, or a CONS of 0 (ADD books: it meets the maker; cancel books:
//    the maker may be its head).
// A REST of 0 with depth > 0 is an ordinary FIFO append (fl_wplan), popped by the first consume
// that passes it (fl_first_back; the gather in fl_level_one).  Books with DELs (the cancel path): a
// cancel lowers the depth like a CONS, and one that empties the level beside a zero-volume maker is a
// hazard too.
// Wave-wide exclusive scans (one wave per level: the checks run in the rare batches that need them,
// and a launch of small blocks gets onto busy CUs at once; 1024-thread blocks waited ~0.8 ms for
// room on config 5c's critical path even when every block had nothing to do).
__device__ __forceinline__ int64_t fl_wave_excl(int64_t x, int64_t* total) {
  const int64_t inc = wave_incl_scan(x);
  *total = rl64(inc, 63);
  return inc - x;
}
__device__ __forceinline__ int64_t fl_wave_max_excl(int64_t x, int64_t* total) {
  const uint32_t lane = lane_id();
  int64_t inc = x;
  for (uint32_t off = 1; off < 64; off <<= 1) {
    const int64_t v = __shfl_up(inc, off);
    if (lane >= off) inc = max(inc, v);
  }
  *total = rl64(inc, 63);
  const int64_t ex = __shfl_up(inc, 1);
  return lane ? ex : static_cast<int64_t>(-1);
}

__global__ __launch_bounds__(64) void k_flow_zero_check(Dev D, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y, q = blockIdx.x, lane = lane_id();
  if (h >= fl_hend(D, F)) return;
  FlowHdr* hd = &F.hdr[h];
  const bool canc = hd->ok == FL_OK_CANCEL && !hd->fc_bad;
  if ((hd->ok != FL_OK_ADD && !canc) || (hd->nzero == 0 && hd->nzlev == 0) || q == 0 || q > hd->nl) return;
  const FlowLvl* Lq = F.lvl + h * FL_CAP + q;
  const uint32_t cnt = Lq->cnt;
  if (!cnt) return;
  const uint32_t L = FL_TOUCH_MUL * hd->beg, nt = hd->ntouch;
  const SEnt* R = F.srt + L + Lq->base;
  const int64_t d0 = Lq->d0;
  int64_t run = d0;          // the level's depth before the chunk
  int64_t rr = d0, cc = 0;   // arrival end and consumption cursor before the chunk (volume coordinates)
  int64_t zlast = -1;        // start of the latest zero-volume maker rested before the chunk (-1: none)
  int64_t wlast = -1;        // cancel books: the latest reach point of a zero-volume maker (below)
  uint32_t hz = 0;           // HZ_* found by this lane
  for (uint32_t c0 = 0; c0 < cnt; c0 += 64) {
    const uint32_t i = c0 + lane;
    const bool valid = i < cnt;
    SEnt e{};
    if (valid) e = R[i];
    const bool isr = valid && e.kind == TK_REST, isc = valid && e.kind == TK_CONS, zr = isr && e.amt == 0;
    const bool isx = valid && e.kind == TK_CANC;
    int64_t tot, tr, tc, tzm;
    const int64_t before = run + fl_wave_excl(isr ? e.amt : (isc || isx) ? -e.amt : 0, &tot);
    const int64_t rb = rr + fl_wave_excl(isr ? e.amt : 0, &tr);  // this REST's start
    const int64_t cb = cc + fl_wave_excl(isc ? e.amt : 0, &tc);  // this CONS's cursor
    const int64_t zm = max(zlast, fl_wave_max_excl(zr ? rb : -1, &tzm));
    // a consume that empties the level and goes on pops the zero-volume makers at its end (fl_cont)
    const bool cont = isc && e.amt > 0 && before - e.amt == 0 && fl_cont(F, L, nt, e.t, canc);
    if (canc) {
      // Cancel books (round 6: their reconstruction pops zero-volume makers, fc_fills).  A
      // zero-volume maker rested at depth D after C of the level was consumed is reached once the
      // consumption passes W = C + D: exactly in consumption space when no cancel removes volume
      // ahead of it, an upper bound otherwise (a cancel may hit a maker behind it).  A consume or
      // cancel that empties the level while some W >= the consumption after it (the maker may still
      // be in the FIFO, which the reference leaves in place, its level out of its set) is a hazard,
      // unless it is a consume that goes on and pops them (fl_cont); so are a REST of 0 at depth 0 and a
      // CONS of 0 (a zero-volume taker) where a zero-volume maker may be its head.  Old zero-volume
      // makers: W = d0.
      int64_t twm;
      const int64_t wm = max(wlast, fl_wave_max_excl(zr ? before + cb : -1, &twm));
      const int64_t cend = cb + (isc ? e.amt : 0);
      const bool present = (Lq->z0 && d0 >= cend) || wm >= cend;
      const bool empt = before - e.amt == 0 && present;
      // (a CONS of 0 fills the head of the FIFO, fc_head_at; if that may be a zero-volume maker,
      // diff == 0 pops it: the hazard)
      hz |= (zr && before == 0 ? HZ_ZREST0 : 0u) | (isc && e.amt == 0 && (Lq->z0 || wm >= 0) ? HZ_ZCONS0 : 0u) |
            (isc && !cont && empt ? HZ_ZSTOP : 0u) | (isx && empt ? HZ_ZDELEMPTY : 0u);
      wlast = max(wlast, twm);
    } else {
      // ADD books: a zero-volume maker is in the FIFO until a consume passes its start (an old
      // one: until the cursor passes the old FIFO's end).  A consume that leaves depth > 0 pops the
      // ones it passes (fl_first_back, the intervals), and one that empties the level and goes on
      // the ones at its end too (fl_cont); one that empties the level and stops there (it leaves
      // them in a FIFO whose level left its set) or a zero-volume taker meeting one (diff == 0 pops
      // it and the cursor stays) is a hazard, and so is a REST of 0 at depth 0.
      const bool zp = (Lq->z0 && cb <= d0) || zm >= cb;
      hz |= (zr && before == 0 ? HZ_ZREST0 : 0u) | (isc && zp && e.amt == 0 ? HZ_ZTAKER : 0u) |
            (isc && zp && e.amt > 0 && before - e.amt == 0 && !cont ? HZ_ZSTOP : 0u);
    }
    run += tot;
    rr += tr;
    cc += tc;
    zlast = max(zlast, tzm);
  }
  for (int off = 32; off > 0; off >>= 1) hz |= __shfl_xor(hz, off);
  if (hz && lane == 0) atomicOr(&hd->haz, hz);
}

// After the head's level sort: a book planned with stale members is exact unless an order rested
// at a stale price on the side opposite its membership before a same-side rest healed it (the
// reference would then hold the price in both side sets, and a later taker of the resting side
// could meet its own side's maker there: SURVEY Appendix A Q2).  The plan never consumes at a
// stale level before a rest there (its depth is 0), so the first touch of the level's run, in time
// order, decides.  Such a book is handed to the legacy kernel: bail, then ok = 0, so every later
// flow kernel skips it and k_match_hot (mode 1) applies it from its unchanged state (nothing of the
// book has been written yet: the plan and the sort write scratch only).  One thread per level.
__global__ __launch_bounds__(FL_CAP) void k_flow_stale_check(Dev D, BatchArgs B, FlowArgs F) {
  __shared__ uint32_t haz;
  const uint32_t h = F.h0 + blockIdx.x, q = threadIdx.x;
  if (h >= fl_hend(D, F)) return;
  FlowHdr* hd = &F.hdr[h];
  const bool canc = hd->ok == FL_OK_CANCEL;  // (its levels: k_fc_stale_level, which ran before)
  if ((hd->ok != FL_OK_ADD && !canc) || (hd->nstale == 0 && hd->haz == 0 && hd->nwrong == 0)) return;
  if (q == 0) {
    haz = hd->haz;
    if (hd->nwrong) ctr_add(D, C_FLOW_WRONG, 1ull);
  }
  __syncthreads();
  if (!canc && q >= 1 && q <= hd->nl) {
    const FlowLvl f = F.lvl[h * FL_CAP + q];
    if (fl_stale0(f) && f.cnt) {
      const SEnt e = F.srt[FL_TOUCH_MUL * hd->beg + f.base];
      const bool sale = B.prep[hd->beg + e.j].side == GOME_SALE;
      if (e.kind != TK_REST || sale != (f.mem0 == M_SALE)) atomicOr(&haz, 1u);
    }
  }
  __syncthreads();
  if (q == 0 && haz) {
    __hip_atomic_store(&hd->bail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence();
    __hip_atomic_store(&hd->ok, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    ctr_add(D, C_FLOW_BAIL, 1ull);
  }
}

__global__ __launch_bounds__(FL_LVB_T) void k_flow_level_wide(Dev D, FlowArgs F) {
  const uint32_t h = F.h0 + blockIdx.y, q = blockIdx.x;
  if (h >= fl_hend(D, F) || F.hdr[h].ok != FL_OK_ADD) return;
  if (q == 0 || q > F.hdr[h].nl) return;
  int64_t cfin;
  uint32_t nr, ncons;
  fl_level_scan_blk(F, h, q, cfin, nr, &ncons);
  const bool z0 = cfin == 0 && ncons > 0;  // (only CONS touches of 0: zero-volume takers, Q6)
  if (threadIdx.x < 64) fl_level_one(D, F, h, q, NIL, 0, NIL, cfin, nr, false, nullptr, z0);
  __syncthreads();  // (wave 0's level record, then the whole block searches)
  const FlowLvl* Lq = F.lvl + h * FL_CAP + q;
  if (cfin > 0 || z0)
    fl_level_fc(F, FL_TOUCH_MUL * F.hdr[h].beg, q, Lq->base, Lq->cnt, F.ig + Lq->ig_base, Lq->ig_n, Lq->nrest, Lq->d0,
                threadIdx.x >> 6, FL_LVB_T / 64, Lq->z0 || F.hdr[h].nzero, F.hdr[h].ntouch);
}

}  // namespace gome
