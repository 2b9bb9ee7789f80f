/*
 * gome_abi.h — C-ABI of the MI355X batch matching engine (drop-in for gome's
 * order-matching hot path).
 *
 * The reference engine entry point is the Go function
 *     func DoOrder(node OrderNode) bool              gomengine/engine/engine.go:46
 * called once per message by the serial consumer loop
 *     for d := range msgs { ... DoOrder(order) }      gomengine/engine/rabbitmq.go:116-125
 * with book state in Redis (nodepool.go, nodelink.go) and one MatchResult JSON
 * published per fill/cancel (engine.go:24-28,109-113,154-158,171-175,190-194).
 *
 * This header replaces that per-message call with a per-batch call: the caller
 * (batching consumer, cgo backend) converts OrderNode messages to
 * 32-byte gome_order records and submits them in consume order; the engine
 * applies them with exactly the reference's sequential semantics per symbol and
 * returns 48-byte gome_event records in the reference's publish order.
 *
 * Conventions: plain C types only, no exceptions or panics across the ABI,
 * every call returns a gome_status, the handle is not thread-safe (one host
 * thread per handle, as the reference has one consumer goroutine,
 * rabbitmq.go:116).  The caller owns all host buffers for the call's duration;
 * no pointer is retained across calls.
 */
#ifndef GOME_ABI_H
#define GOME_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GOME_ABI_VERSION 12u

/* ---- status codes (replace the reference's swallowed errors / panics,
 *      rabbitmq.go:44-49,70-72,120-122; nodelink.go:132,142,157) ---------- */
typedef int32_t gome_status;
enum {
  GOME_OK = 0,
  GOME_E_INVAL = 1,     /* input outside the exact parity domain (Q5), bad args      */
  GOME_E_CAPACITY = 2,  /* a device pool (levels, nodes, index, events) is full    */
  GOME_E_DEVICE = 3,    /* HIP runtime error / no device                           */
  GOME_E_STATE = 4,     /* engine poisoned by an earlier fatal error                */
  GOME_E_NOTFOUND = 5,  /* lookup miss (snapshot of an unknown symbol, ...)         */
};

/* ---- actions and sides ---------------------------------------------------- */
enum { GOME_ADD = 1, GOME_DEL = 2 };      /* engine.go:14-18, main.go:14-18 */
enum { GOME_BUY = 0, GOME_SALE = 1 };     /* api/order.proto:4-7            */
/* Transaction codes.  OrderRequest.transaction is an int32 (order.proto:13,
 * ordernode.go:14); the reference treats 1 as SALE and ANY other value as BUY
 * (ordernode.go:95, nodepool.go:89; quirk Q8) and echoes the raw value in every
 * MatchResult it publishes.  A record carries a one-byte code:
 *   0 = BUY (Transaction 0), 1 = SALE (Transaction 1),
 *   2..255 = a host-interned Transaction value outside {0, 1} (BUY semantics).
 * The engine echoes the code in events (gome_event.maker_side); the renderers map
 * codes back to the raw int32 through the caller's table (gome_tx_table). */
#define GOME_TX_CODES 256

/* ---- records ------------------------------------------------------------- */

/* gome_order.flags (ABI >= 4).  By default admission (S:comparison, nodepool.go:14-28,
 * engine.go:58-62,90; quirk Q4) follows the batch model: an ADD is admitted iff no
 * earlier ADD or DEL of the same batch carries the same (symbol, uuid, oid).  A host
 * that keeps the reference's pre-pool markers itself (set at gRPC time, main.go:44-45;
 * gome_amd/consumer.py PrePool) resolves admission per record instead: */
#define GOME_ORD_ADM_HOST 1u   /* admission decided by the host (ignore the batch rule) */
#define GOME_ORD_ADMITTED 2u   /* ... and this ADD is admitted (its marker existed)      */
#define GOME_ORD_FLAGS_MASK (GOME_ORD_ADM_HOST | GOME_ORD_ADMITTED)

/* One consumed OrderNode message (ordernode.go:9-36) in fixed point.
 * price_fx / volume_fx = value * 10^accuracy exactly (ordernode.go:76-87, see
 * gome_fixed_from_double / gome_fixed_from_scaled).  The sequence number of a record
 * is seq_base + its index in the submitted batch (gome_event.taker_seq: its low 32 bits). */
typedef struct gome_order {
  int64_t price_fx;   /* OrderNode.Price  (limit price; request price for DEL)  */
  int64_t volume_fx;  /* OrderNode.Volume (>= 0)                                */
  uint32_t symbol_id; /* interned OrderNode.Symbol, < gome_config.max_symbols    */
  uint32_t oid_id;    /* interned OrderNode.Oid (unique per symbol, README:27; see
                         the duplicate-oid rule below)                            */
  uint32_t uuid_id;   /* interned OrderNode.Uuid                                 */
  uint8_t side;       /* Transaction code (see above): 1 SALE, anything else BUY */
  uint8_t action;     /* OrderNode.Action: 1 ADD, 2 DEL, anything else ignored   */
  uint16_t flags;     /* GOME_ORD_* (0: batch admission model); other bits E_INVAL */
} gome_order;

enum { GOME_EV_FILL = 1, GOME_EV_CANCEL = 2 };

/* One published MatchResult (engine.go:24-28), 48 bytes (ABI >= 8; SURVEY §8's EventRec).
 *   FILL   (engine.go:154,171,190): Node = taker after the fill, MatchNode = maker
 *          as read from the FIFO head (IsFirst=true, PrevNode=""), MatchVolume = qty.
 *   CANCEL (engine.go:109): Node = MatchNode = the DEL request with Volume = the
 *          stored remaining volume; MatchVolume = 0.
 * The taker's record (symbol, uuid, oid, Transaction, limit price) is the submitted record of
 * sequence number seq; Node.Volume of a FILL is the taker's remaining volume after it: its
 * record's volume minus the MatchVolumes of its fills so far (a taker's events are consecutive
 * in publish order; gome_render_events keeps that running sum).
 * Sequence number of the taker (the ADD / DEL record) = seq_base + its index in the batch;
 * taker_seq holds its low 32 bits (the caller knows seq_base: with seq_base = 0, taker_seq IS
 * the batch index).  Events of one batch are returned in the reference publish order, i.e.
 * sorted by (sequence number, fill_idx). */
typedef struct gome_event {
  int64_t price_fx;         /* level price (= MatchNode.Price); DEL: request price  */
  int64_t match_volume_fx;  /* MatchVolume                                           */
  int64_t maker_volume_fx;  /* MatchNode.Volume: pre-fill if fully filled, else the
                               maker's remaining volume; DEL: stored remaining       */
  uint32_t taker_seq;       /* low 32 bits of seq_base + batch index                 */
  uint32_t fill_idx;        /* 0,1,2... within one taker                             */
  uint32_t maker_oid_id;    /* MatchNode.Oid                                         */
  uint32_t maker_uuid_id;   /* MatchNode.Uuid                                        */
  uint32_t maker_next_oid_id; /* MatchNode.NextNode = S:node:<this> unless is_last   */
  uint8_t kind;             /* GOME_EV_FILL / GOME_EV_CANCEL                         */
  uint8_t maker_side;       /* MatchNode.Transaction code                            */
  uint8_t maker_is_last;    /* MatchNode.IsLast (NextNode == "")                     */
  uint8_t pad0;
} gome_event;

/* One price level of a book in the reference key schema (nodepool.go:61-115):
 * bid/ask membership = presence of the price in S:BUY / S:SALE, depth = the
 * S:depth:<price> field, nodes = length of the S:link:<price> FIFO. */
typedef struct gome_level {
  int64_t price_fx;
  int64_t depth_fx;
  uint32_t n_nodes;
  uint8_t in_buy;   /* member of S:BUY  */
  uint8_t in_sale;  /* member of S:SALE */
  uint16_t pad;
} gome_level;

/* One resting node of a FIFO, in link order (nodelink.go, S:link:<price>). */
typedef struct gome_node {
  int64_t volume_fx;
  uint32_t oid_id;
  uint32_t uuid_id;
  uint8_t side;
  uint8_t pad[7];
} gome_node;

/* gome_config.flags: GOME_FLAG_LEGACY_HOT applies every hot book with the legacy one-wave FIFO
 * kernel instead of the flow path (same results; for A/B measurement and parity checks). */
#define GOME_FLAG_LEGACY_HOT 1u
/* By default a submit whose ADDs could push the resting makers past max_nodes or the level
 * records past max_levels (every ADD resting on a new level; batches in flight counted in
 * full) is rejected with GOME_E_CAPACITY before anything is applied: the book is unchanged
 * and the handle stays usable (size max_nodes >= the resting makers + GOME_MAX_INFLIGHT
 * batches).  This flag turns the check off (pools sized tightly on purpose). */
#define GOME_FLAG_NO_HEADROOM 2u
/* The flow path's deep-book and cancel chains (match_flow_deep.h, match_flow_cancel.h: ~70
 * kernel launches per batch) are enqueued only while recent batches needed them: a chain is
 * dropped after GOME_CHAIN_QUIET finished batches in which no flow candidate asked for it, and
 * comes back on the next submit after one did (a host submit whose records hold a DEL enqueues
 * the cancel chain at once).  A candidate that asks for a chain the batch did not enqueue is
 * applied by the legacy / cold kernels instead (same results, slower for that batch).
 * GOME_FLAG_CHAINS_ALWAYS enqueues both chains on every batch; GOME_FLAG_CHAINS_NEVER never
 * (every deep book and every book with DELs on the legacy / cold kernels; A/B and tests). */
#define GOME_FLAG_CHAINS_ALWAYS 4u
#define GOME_FLAG_CHAINS_NEVER 8u
#define GOME_CHAIN_QUIET 4u
/* gome_stats.ms_phase (per-phase device times) needs ~24 timing-event records per batch on the
 * pipeline's streams (0.12 ms per config-2 batch); they are recorded only with this flag. */
#define GOME_FLAG_PHASES 16u
/* Stream layout (ABI >= 11).  The early plan of the hottest book (§4.8) and
 * admission ahead of the batch (§4.9) are on by default when the process has at least 8 hardware
 * queues (gome_config.hw_queues); these flags turn them off (A/B and tests: same results). */
#define GOME_FLAG_NO_EARLY 32u
#define GOME_FLAG_NO_ADM_AHEAD 64u
/* Test builds of a host (ABI >= 12): every device buffer of the handle starts filled with 0xA5
 * bytes instead of zeros, so a kernel that reads scratch it never wrote sees an out-of-range
 * index or an absurd count (an error or a fault) instead of a benign zero.  Same results as
 * the default when no such read exists; never for production. */
#define GOME_FLAG_POISON 128u

typedef struct gome_config {
  uint32_t accuracy;       /* gomengine.accuracy (config.yaml.example:23-24), default 8 */
  int32_t device;          /* HIP device ordinal (one handle per GPU)                    */
  uint32_t max_symbols;    /* symbol_id range                                            */
  uint32_t max_batch;      /* max records per submit                                     */
  uint64_t max_nodes;      /* resting-order capacity (node pool)                         */
  uint64_t max_levels;     /* level-record capacity (all books)                          */
  uint64_t max_events;     /* event capacity per batch (0: derived from max_batch)       */
  uint32_t flags;          /* GOME_FLAG_* (0 = defaults)                                 */
  uint32_t abi_version;    /* must be GOME_ABI_VERSION: gome_create refuses any other value,
                              so a caller built against another ABI fails loudly (ABI <= 10
                              had a zero pad word here)                                 */
  /* Hardware queues the process's HIP runtime has: GPU_MAX_HW_QUEUES as the runtime read it
   * when it started (HIP's default is 4).  Streams beyond that share queues and run one after
   * another, so the engine picks its stream layout from this count: with >= 8 the cold books
   * run beside the tail's chain, the hottest book is planned early and admission runs ahead;
   * below 8, the four-stream layout.  0: the variable's value at gome_create (4 if unset or
   * not a number) -- correct only when nothing started HIP before the variable was set. */
  uint32_t hw_queues;
  /* CUs reserved for the hottest book's plan (a CU-masked stream, every other stream masked off
   * them): 0 = the default (8 with >= 8 hardware queues, else none), < 0 = none,
   * k > 0 = k. */
  int32_t plan_cus;
} gome_config;

/* gome_stats.ms_phase (ABI >= 5): device time of the pipeline's phases in the last batch, each
 * timed on the stream it runs on (phases on different streams overlap). */
enum {
  GOME_PH_ADMISSION = 0, /* admission markers and the duplicate-oid rule (Q4, Q7)         */
  GOME_PH_SORT,          /* radix sort by symbol, segments                                */
  GOME_PH_HEAD_PREP,     /* the head books' preps (lane, deep, cancel)                     */
  GOME_PH_HEAD_RECON,    /* the hottest book's reconstruction after its plan              */
  GOME_PH_RECORDS,       /* k_prep: the symbol-sorted 32-B records                        */
  GOME_PH_TAIL_PREP,     /* tail books: prep (k_flow_prep, deep and cancel preps)          */
  GOME_PH_TAIL_PLAN,     /* tail books: serial plans (k_flow_plan_tail, _c, _d)           */
  GOME_PH_TAIL_SORT,     /* tail books: touches sorted by level (k_flow_sort)             */
  GOME_PH_TAIL_LEVEL,    /* tail books: level reconstruction (k_flow_level, deep levels)  */
  GOME_PH_TAIL_COUNT,    /* tail books: the touch offsets and group map (k_flow_toff/tmap) */
  GOME_PH_TAIL_WRITE,    /* tail books: FIFO appends, level arrays, events and ev_count
                            in one launch (k_flow_write_events)                         */
  GOME_PH_TAIL_EVENTS,   /* tail books: the deep books' writes, the DEL books' chain      */
  GOME_PH_NEAR,          /* the other head books: plans and reconstruction               */
  GOME_PH_PUBLISH,       /* publish-order scan, the hottest book's events, arena scatter  */
  GOME_NPHASE = 16
};

/* Per-batch counters of the last submit (and running totals). */
typedef struct gome_stats {
  uint64_t n_orders, n_add, n_del, n_dropped; /* dropped = ADD without admission marker */
  uint64_t n_fills, n_cancels, n_rests, n_events;
  uint64_t n_resting;                         /* resting nodes after the batch (total)  */
  uint64_t n_levels;                          /* level records in use (total)           */
  uint64_t max_segment;                       /* orders of the hottest book this batch  */
  uint64_t n_segments;                        /* books touched this batch               */
  double ms_total;                            /* device time of the batch pipeline      */
  double ms_match;                            /* device time of the match phase (hot and
                                                 cold books, concurrent)                 */
  double ms_hot;                              /* device time of k_match_hot (hot books)  */
  uint64_t n_hot;                             /* books applied by k_match_hot            */
  uint64_t n_hot_orders, n_hot_fills;         /* work done inside k_match_hot (roofline   */
  uint64_t n_hot_rests, n_hot_cancels;        /* numerator of the hot kernel)             */
  uint64_t n_flow_books;                      /* hot books applied by the flow path       */
  uint64_t n_flow_orders, n_flow_touches;     /* their orders / level touches (plan log)  */
  double ms_flow_plan;                        /* device time of k_flow_plan_head (the
                                                 serial plan of the longest flow books,
                                                 the batch's critical path)               */
  uint64_t n_flow_head_orders;                /* orders / touches of the books that        */
  uint64_t n_flow_head_touches;               /* k_flow_plan_head planned (ABI >= 3)      */
  uint64_t n_index_rebuilds;                  /* cancel-index rebuilds so far (ABI >= 4)   */
  uint64_t idx_tombstones;                    /* index tombstones since (upper bound)     */
  uint64_t n_flow_cancels;                    /* DELs applied on the flow path this batch */
  double ms_cold;                             /* device time of k_match (cold books)      */
  uint64_t lvl_used;                          /* level slots carved from the pool so far
                                                 (released blocks are reused first)      */
  uint64_t n_dup_oid;                         /* ADDs of the batch rejected by the
                                                 duplicate-oid rule (ABI >= 5; also counted
                                                 in n_dropped)                           */
  uint64_t n_flow_tail_fills;                 /* fills of the tail's flow books (ABI >= 5) */
  double ms_phase[GOME_NPHASE];               /* GOME_PH_* device times (ABI >= 5; 0 unless
                                                 GOME_FLAG_PHASES, ABI >= 6)              */
  double ms_host_enqueue;                     /* host wall time the batch's launches took
                                                 (ABI >= 5): the GPU cannot finish before
                                                 the last one is issued                  */
  uint32_t chains;                            /* flow chains this batch enqueued (ABI >= 6):
                                                 1 = deep books, 2 = books with DELs     */
  uint32_t chains_wanted;                     /* chains its candidates asked for (same bits;
                                                 wanted and not enqueued: legacy / cold)  */
  uint64_t n_quirk_checked;                   /* books in a quirk state (wrong-side cancel Q2,
                                                 zero-volume maker Q6) the legacy / cold
                                                 kernels applied this batch (ABI >= 8)    */
  uint64_t n_requalified;                     /* ... of which healed: back on the flow path
                                                 from the next batch on (ABI >= 8)        */
  uint64_t chunk_bytes;                       /* HBM held by FIFO chunks in use (node slots plus
                                                 chunk headers) after the batch (ABI >= 8):
                                                 / n_resting = bytes per resting order     */
  uint64_t n_early;                           /* 1 when the batch's hottest book was planned
                                                 early, right after the previous batch's plan
                                                 (pipelined device batches, ABI >= 9)      */
  uint64_t n_early_miss;                      /* an early plan the batch could not take although
                                                 its hottest book went through the same plan
                                                 (0 unless something is wrong; ABI >= 9)   */
  uint64_t n_adm_ahead;                       /* 1 when the batch's admission ran ahead, beside
                                                 the previous batch's plan (pipelined device
                                                 batches, ABI >= 10)                       */
  uint64_t n_adm_redo;                        /* ... and ran again at the batch's own time: an
                                                 ADD's key might rest (ABI >= 10)           */
  uint64_t n_flow_stale;                      /* head books planned on the flow path with stale
                                                 side-set members (Q2: a member level with no
                                                 FIFO, left by a wrong-side cancel; ABI >= 11) */
  uint64_t n_flow_bail;                       /* head books the legacy kernel applied after their
                                                 plan: an order rested on the other side of a
                                                 stale price, or a zero-volume maker an order
                                                 reaches (ABI >= 11)                        */
  uint64_t n_flow_zero;                       /* head books planned on the flow path with
                                                 zero-volume ADDs or zero-volume makers (Q6;
                                                 ABI >= 11)                                 */
  uint64_t n_flow_wrong;                      /* head books whose wrong-side cancels (Q2)
                                                 the flow cancel path applied (ABI >= 11)   */
} gome_stats;

typedef struct gome_engine gome_engine;

/* ---- lifecycle ----------------------------------------------------------- */
gome_status gome_create(const gome_config* cfg, gome_engine** out);
void gome_destroy(gome_engine* e);
const char* gome_last_error(const gome_engine* e); /* handle-local message, never NULL */
uint32_t gome_abi_version(void);

/* ---- hot path ------------------------------------------------------------ */
/* Every submit applies its batch after every earlier one (per symbol in record order, as
 * the reference's single consumer, rabbitmq.go:116).  Events of a batch are published in
 * (sequence number, fill_idx) order.  A batch rejected with GOME_E_INVAL (a record outside
 * the exact domain) leaves the book unchanged.
 *
 * Duplicate oids (ABI >= 5).  The reference names a resting node
 * S:node:<oid> without the uuid (ordernode.go:110-112, nodelink.go:119-122) and assumes oids
 * unique per symbol (README.md:27): a second live node of the same name corrupts the FIFO.
 * Rule, on every path: an ADD that admission lets through (batch rule or GOME_ORD_ADMITTED)
 * is NOT applied when its (symbol, oid) rests in the book at the start of its batch, or was
 * carried by an earlier admitted ADD of the same batch.  It publishes nothing, as an ADD
 * without an admission marker (engine.go:58); gome_stats.n_dup_oid counts the batch's
 * rejections and gome_dup_records lists their batch indices.  (Reusing an oid once its node
 * is gone, in a later batch, is an ordinary ADD.) */

/* Apply one batch of host records (replaces n calls of DoOrder, engine.go:46).
 * Synchronous: on return the events are queued for gome_drain_events. */
gome_status gome_submit_batch(gome_engine* e, const gome_order* orders, size_t n,
                              uint64_t seq_base);
/* Same, with the records already resident in device memory (HBM); `stream` is a
 * hipStream_t or NULL.  Events stay on the device: read them with
 * gome_device_events or copy them out with gome_drain_events (events of an earlier
 * device batch not yet drained are moved to the host queue first, never dropped). */
gome_status gome_submit_batch_device(gome_engine* e, const gome_order* dev_orders,
                                     size_t n, uint64_t seq_base, void* stream);
/* Copy out up to cap pending events in publish order; *n_out = copied.  Batches still in
 * flight (gome_submit_batch_async) are collected into the queue first. */
gome_status gome_drain_events(gome_engine* e, gome_event* out, size_t cap,
                              size_t* n_out);
/* Events waiting in the drain queue (in-flight batches not included: collect them first, or
 * call gome_drain_events, which does). */
size_t gome_pending_events(const gome_engine* e);
/* Device pointer + count of the last gome_submit_batch_device batch's events (valid until the
 * next submit; host batches, synchronous or in flight, are not among them). */
gome_status gome_device_events(gome_engine* e, const gome_event** dev_ptr,
                               size_t* n);
/* A device-side consumer has taken the last device batch's events (read through
 * gome_device_events): the next submit need not move them to the host drain queue. */
gome_status gome_release_device_events(gome_engine* e);
/* Counters of the last batch that finished (gome_submit_batch*, gome_collect or a synchronous
 * call's collection); batches still in flight are not included. */
gome_status gome_get_stats(const gome_engine* e, gome_stats* out);
/* Batch indices (ascending) of the ADDs the duplicate-oid rule rejected in the last finished
 * batch (ABI >= 5); *n_out = their number (only cap are written). */
gome_status gome_dup_records(const gome_engine* e, uint32_t* out, size_t cap, size_t* n_out);
/* Diagnostics (tests, tuning): the last batch's hot-book routing, GOME_DEBUG_FLOW_WORDS words
 * per candidate book, longest segment first: {flow kind (0 legacy / cold, 1 ADD-only flow,
 * 2 flow with cancels), cancel-prep decline bits, symbol, orders, DELs, levels, 32-bit plan,
 * ring entries needed, longest cancel window + 1, deep-book candidate}.  *n_out = candidates written (<= cap). */
#define GOME_DEBUG_FLOW_WORDS 10
gome_status gome_debug_flow_books(gome_engine* e, uint32_t* out, size_t cap, size_t* n_out);
/* Diagnostics: raw bytes [offset, offset + bytes) of one of the flow path's device scratch
 * arrays after the last batch (0 headers, 1 level slots, 2 DEL records, 3 targeted-ADD ranks,
 * 4 DEL-of-ADD links, 5 packed records, 6 the hottest book's huge-level passes: two control blocks,
 * lane book then deep book, each starting {levels taken, chunks, book, 0} as uint32). */
gome_status gome_debug_peek(gome_engine* e, uint32_t which, uint64_t offset, uint64_t bytes, void* out);
/* Diagnostics: the shape of one book's FIFOs, 4 words per level in the book's level order
 * {price_fx, live nodes, dead slots (cancelled / consumed, still linked), chunks}.  *n_out =
 * levels (only cap are written). */
gome_status gome_debug_fifo_shape(gome_engine* e, uint32_t symbol_id, int64_t* out, size_t cap, size_t* n_out);

/* ---- pipelined host path (ABI >= 4) ---------------------------------------- */
/* The batching consumer's loop: submit batch k+1, then collect batch k.
 * The copy of batch k+1's records to HBM and of batch k's events to the host run on two
 * copy streams while the device applies the other batch, so PCIe hides under matching (with
 * three batches in flight, batch k+2's H2D and batch k's D2H also overlap each other).
 * At most GOME_MAX_INFLIGHT batches are in flight; `orders` must stay valid and
 * unchanged until the batch is collected (memory from gome_host_alloc is page-locked,
 * which makes the copy asynchronous).  gome_submit_batch, gome_submit_batch_device,
 * gome_drain_events, gome_snapshot_*, gome_load_books and gome_debug_* first collect every
 * in-flight batch into the drain queue.  A batch collected that way that was rejected
 * (GOME_E_INVAL, nothing applied) does not fail that call: the call goes on and the failure
 * is kept for gome_take_deferred. */
#define GOME_MAX_INFLIGHT 3u  /* (2 before ABI v8) */
gome_status gome_submit_batch_async(gome_engine* e, const gome_order* orders, size_t n,
                                    uint64_t seq_base);
/* Wait for the oldest in-flight batch and copy its events to engine-owned page-locked
 * memory: *events (publish order) stays valid until the next gome_collect or
 * synchronous call.  stats (optional) = that batch's counters.  GOME_E_NOTFOUND when no
 * batch is in flight; the batch's own status otherwise (E_INVAL: rejected, no events). */
gome_status gome_collect(gome_engine* e, const gome_event** events, size_t* n_events,
                         gome_stats* stats);
size_t gome_inflight(const gome_engine* e);
/* The same pipeline with the records already in HBM (ABI >= 7): submit device batch k+1, then
 * collect device batch k, so the host's enqueue of one batch hides under the device's work on
 * the other.  `dev_orders` must stay valid and unchanged until the batch is collected.  The
 * collect returns the batch's events in device memory (publish order, as gome_device_events):
 * valid until the next submit or collect, which first moves them to the host drain queue
 * unless gome_release_device_events said a device-side consumer took them.  GOME_E_STATE when the
 * oldest batch in flight is a host batch (gome_collect takes those). */
gome_status gome_submit_batch_device_async(gome_engine* e, const gome_order* dev_orders, size_t n,
                                           uint64_t seq_base);
gome_status gome_collect_device(gome_engine* e, const gome_event** dev_events, size_t* n_events,
                                gome_stats* stats);
/* The first failure of an in-flight batch that a synchronous call collected since the last
 * gome_take_deferred (its message then in gome_last_error), or GOME_OK; clears it. */
gome_status gome_take_deferred(gome_engine* e);
gome_status gome_host_alloc(gome_engine* e, size_t bytes, void** out);
void gome_host_free(gome_engine* e, void* p);

/* ---- book state (Redis-schema view; snapshot / parity) ------ */
/* Levels of one book in ascending price order, including empty levels that
 * still carry a side-set membership (Q2).  *n_out = number of levels; when
 * cap < *n_out only cap are written. */
gome_status gome_snapshot_levels(gome_engine* e, uint32_t symbol_id,
                                 gome_level* out, size_t cap, size_t* n_out);
/* Nodes of the FIFO at one price, head first. */
gome_status gome_snapshot_fifo(gome_engine* e, uint32_t symbol_id, int64_t price_fx,
                               gome_node* out, size_t cap, size_t* n_out);

/* Top-of-book digest of one book (ABI >= 5): what GetReverseDepth's first level reports for a
 * taker of either side (nodepool.go:86-115) — the highest S:BUY member and the lowest S:SALE
 * member with their S:depth fields and FIFO lengths.  flags bit 0: a bid exists, bit 1: an
 * ask exists (prices and depths are 0 otherwise).  n_levels = the book's observable levels
 * (as gome_snapshot_levels counts them).  The publisher's per-GPU depth summary. */
typedef struct gome_tob {
  uint32_t symbol_id;
  uint32_t n_levels;
  int64_t bid_price_fx, bid_depth_fx;
  int64_t ask_price_fx, ask_depth_fx;
  uint32_t bid_nodes, ask_nodes;
  uint32_t flags, pad;
} gome_tob;
gome_status gome_top_of_book(gome_engine* e, const uint32_t* symbols, size_t n, gome_tob* out);
/* The same digests without collecting the batches in flight (ABI >= 8): enqueued on the pipeline's
 * stream behind every batch submitted so far, so they describe the books as the last submitted
 * batch leaves them (a later submit waits for them).  One request at a time; symbols are copied.
 * gome_top_of_book_collect waits for that request alone and copies min(cap, n) digests
 * (*n_out = n); GOME_E_NOTFOUND when nothing is enqueued.  With two batches in flight, enqueue
 * before submitting batch k+1 and collect after collecting batch k: the digests of batch k. */
gome_status gome_top_of_book_enqueue(gome_engine* e, const uint32_t* symbols, size_t n);
gome_status gome_top_of_book_collect(gome_engine* e, gome_tob* out, size_t cap, size_t* n_out);

/* ---- book state load (restart from Redis) ------------------- */
/* The reference restarts from whatever its Redis holds (nodepool.go:14-115,
 * nodelink.go:12-166, ordernode.go:89-116).  gome_load_books writes such books straight
 * into the device pools of a fresh engine (no batch submitted and nothing loaded before;
 * otherwise GOME_E_STATE): the inverse of gome_snapshot_levels / gome_snapshot_fifo.
 * Book b is symbol book_sym[b] (distinct, < max_symbols) with book_nlv[b] levels; the
 * levels follow book by book in ascending price, and each level's n_nodes nodes follow in
 * `nodes` in FIFO order (head first, side = Transaction code).  Every state the reference
 * can hold loads as it is, quirk states included (a depth that differs from the FIFO's
 * sum, a side-set member without nodes (Q2), a zero-volume maker (Q6), a FIFO of mixed
 * sides); books in such a state are applied by the legacy kernels from then on.  Duplicate
 * (symbol, oid) keys: lookups find the first in load order.  GOME_E_CAPACITY when the
 * pools (max_levels, max_nodes) cannot hold the image. */
gome_status gome_load_books(gome_engine* e, size_t n_books, const uint32_t* book_sym,
                            const uint32_t* book_nlv, const gome_level* levels,
                            const gome_node* nodes, size_t n_nodes);

/* ---- host helpers (no device work) --------------------------------------- */
/* ordernode.go:76-87: Float64(decimal.NewFromFloat(x) * decimal.NewFromFloat(10^acc)).
 * Succeeds iff that product is an integer with |v| < 2^53 (the domain on which the
 * reference's float64 / Redis long-double arithmetic is exact integer arithmetic);
 * otherwise GOME_E_INVAL (e.g. 0.123456789 at acc 8).  Use it on a
 * gRPC OrderRequest (main.go:41 -> NewOrderNode). */
gome_status gome_fixed_from_double(double x, uint32_t accuracy, int64_t* out);
/* An OrderNode consumed from the doOrder queue already carries the scaled value
 * (NewOrderNode ran at gRPC time, main.go:41, ordernode.go:76-87): accept it iff it is
 * an integer-valued float64 with |v| < 2^53 (the exact domain), else GOME_E_INVAL. */
gome_status gome_fixed_from_scaled(double scaled, int64_t* out);
/* Render one event as the reference's MatchResult JSON (Go encoding/json of
 * engine.MatchResult, byte-identical).  Strings are the host's interned names;
 * `taker` is the record of the event's taker, taker_remaining_fx its remaining volume after
 * this fill (Node.Volume; ignored for a CANCEL).  tx_table maps Transaction codes
 * (gome_order.side, gome_event.maker_side) to the raw int32 Transaction values to echo;
 * NULL = identity (codes 0..255 are the values).  Returns bytes written (excl. NUL), or
 * -(bytes needed incl. NUL) when cap is too small, or INT64_MIN on a NULL argument. */
int64_t gome_render_match_result(const gome_event* ev, const gome_order* taker,
                                 int64_t taker_remaining_fx, uint32_t accuracy, const char* symbol,
                                 const char* taker_uuid, const char* taker_oid,
                                 const char* maker_uuid, const char* maker_oid,
                                 const char* maker_next_oid, const int32_t* tx_table,
                                 char* buf, size_t cap);
/* Render a batch's events (publish order) as newline-terminated MatchResult JSON lines, the
 * bytes the reference publishes to matchOrder (engine.go:109-113,154-194), for the batching
 * consumer's sink.  `batch` / seq_base: the submitted records and the batch's seq_base (the
 * taker of an event is batch[seq - seq_base]).  Names are the host's interned strings indexed
 * by id (sym_names[symbol_id], ...; n_* = table sizes).  Returns bytes written, or
 * -(bytes needed) when cap is too small, or INT64_MIN on a bad id. */
int64_t gome_render_events(const gome_event* ev, size_t n, const gome_order* batch, size_t batch_n,
                           uint64_t seq_base, uint32_t accuracy, const char* const* sym_names,
                           size_t n_sym, const char* const* uuid_names, size_t n_uuid,
                           const char* const* oid_names, size_t n_oid, const int32_t* tx_table,
                           char* buf, size_t cap);
/* Render one resting node as the reference stores it in S:link:<price> under
 * S:node:<oid> (nodelink.go:119-122; Go encoding/json of engine.OrderNode, byte-identical):
 * the ADD that rested with its remaining volume, IsFirst / IsLast / PrevNode / NextNode from
 * its FIFO neighbours (NULL = none).  `transaction` is the raw int32 value.  Used by the
 * snapshot writer (gome_amd/snapshot.py).  Returns bytes written (excl.
 * NUL), or -(bytes needed incl. NUL) when cap is too small, or INT64_MIN on a NULL argument. */
int64_t gome_render_link_node(const char* symbol, int64_t price_fx, int32_t transaction, int64_t volume_fx,
                              uint32_t accuracy, const char* uuid, const char* oid,
                              const char* prev_oid, const char* next_oid, char* buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* GOME_ABI_H */
