/*
 * gome_host.h — the host side of the drop-in in native code: the consumer
 * loop of the reference, minus the queue client.
 *
 * The reference's consumer (gomengine/engine/rabbitmq.go:116-125) does, per doOrder message:
 *     json.Unmarshal(d.Body, &order)      // errors printed, DoOrder still runs
 *     DoOrder(order)                      // engine.go:46: admission (S:comparison), match
 * and the gRPC handlers set the admission marker before enqueueing (main.go:39-52,
 * nodepool.go:14-16).  The batching consumer replaces that with one call per drained batch:
 *
 *   gome_consume_order_nodes  decodes every OrderNode JSON body with Go's encoding/json
 *                             semantics (on several threads), converts the already-scaled
 *                             Price / Volume (gome_fixed_from_scaled), interns Symbol / Uuid /
 *                             Oid and Transaction codes, and resolves admission against the
 *                             pre-pool markers in queue order -> gome_order records for
 *                             gome_submit_batch (GOME_ORD_ADM_HOST verdicts);
 *   gome_render_events_mt     renders the batch's events as MatchResult JSON lines
 *                             (gome_render_events, split over threads at taker boundaries).
 *
 * Go json.Unmarshal(body, &OrderNode{}) semantics (go encoding/json decode.go, ordernode.go:9-36):
 *   - the whole body must be valid JSON (nesting depth <= 10000), else nothing is decoded: a
 *     zero OrderNode, Action 0, which DoOrder ignores (engine.go:46-54);
 *   - a top-level value that is not an object decodes nothing either;
 *   - object keys match a field exactly, else case-insensitively (Go's foldName: ASCII case,
 *     U+017F ~ 's', U+212A ~ 'k'); a later duplicate key wins;
 *   - Action (int8) / Transaction (int32) take an integer literal within their width, Price /
 *     Volume (float64) any number literal that parses finite (strconv.ParseFloat, round to
 *     nearest), Uuid / Oid / Symbol a string; null, a wrong type or an overflow leaves the field
 *     unchanged;
 *   - strings: escapes decoded, a lone UTF-16 surrogate escape -> U+FFFD, every byte that does
 *     not start a valid UTF-8 encoding -> U+FFFD.
 *
 * Thread safety: a gome_names is interned by one consumer thread, and rendered from by
 * gome_render_events_names on another at the same time (the pipelined consumer renders batch k
 * while it decodes batch k + 1); a gome_prepool may take markers (gome_prepool_set) from any thread
 * while one consumer consumes.
 */
#ifndef GOME_HOST_H
#define GOME_HOST_H

#include "gome_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- interning: OrderNode strings <-> the u32 ids gome_order carries ------------------------ */
enum { GOME_NAME_SYMBOL = 0, GOME_NAME_UUID = 1, GOME_NAME_OID = 2 };
typedef struct gome_names gome_names;
gome_names* gome_names_create(void);
void gome_names_destroy(gome_names* nm);
/* The id of the string (a new one, in first-seen order, if unseen); -1 on a bad argument. */
int64_t gome_names_intern(gome_names* nm, int kind, const char* s, size_t len);
/* The id of the string, or -1 if it was never interned. */
int64_t gome_names_find(const gome_names* nm, int kind, const char* s, size_t len);
size_t gome_names_count(const gome_names* nm, int kind);
/* The string of an id (NUL-terminated; *len = its length), or NULL. */
const char* gome_names_get(const gome_names* nm, int kind, uint32_t id, size_t* len);
/* Every string of a kind by id, NUL-terminated: the tables gome_render_events takes.  Valid
 * until the next intern of that kind (gome_render_events_names reads them safely beside one). */
const char* const* gome_names_table(gome_names* nm, int kind);
/* Transaction int32 -> one-byte code (0 / 1 for 0 / 1, then first-seen order: gome_abi.h);
 * -1 once 256 codes exist. */
int32_t gome_names_tx_code(gome_names* nm, int32_t raw);
/* The raw Transaction of every code (256 entries; unused codes map to themselves). */
const int32_t* gome_names_tx_table(const gome_names* nm);
size_t gome_names_tx_count(const gome_names* nm);

/* ---- pre-pool markers S:comparison (nodepool.go:14-28), keyed (Symbol, Uuid, Oid) ------------ */
typedef struct gome_prepool gome_prepool;
gome_prepool* gome_prepool_create(void);
void gome_prepool_destroy(gome_prepool* pp);
/* SetPrePool (main.go:44-45). */
void gome_prepool_set(gome_prepool* pp, const char* sym, size_t sym_len, const char* uuid, size_t uuid_len,
                      const char* oid, size_t oid_len);
/* ExistsPrePool + DeletePrePool at once (engine.go:58-62): 1 if the marker existed. */
int32_t gome_prepool_take(gome_prepool* pp, const char* sym, size_t sym_len, const char* uuid, size_t uuid_len,
                          const char* oid, size_t oid_len);
size_t gome_prepool_size(const gome_prepool* pp);
/* gome_consume_order_nodes consumes markers provisionally (staged): commit removes them once the
 * engine took the batch; abort forgets them (the batch can be consumed again with the same
 * verdicts). */
void gome_prepool_commit(gome_prepool* pp);
void gome_prepool_abort(gome_prepool* pp);

/* ---- the decoder alone (Go json.Unmarshal into OrderNode, the fields the engine reads) -------- */
typedef struct gome_decoded_node {
  double price;           /* OrderNode.Price as decoded (the gRPC side scaled it)            */
  double volume;          /* OrderNode.Volume                                                */
  int32_t transaction;
  int8_t action;
  uint8_t is_object;      /* 0: syntax error or not an object (a zero OrderNode)             */
  uint16_t pad;
  uint32_t sym_off, sym_len, uuid_off, uuid_len, oid_off, oid_len;  /* strings in strbuf      */
} gome_decoded_node;
/* Message i is buf[off[i], off[i + 1]).  The decoded strings go to strbuf (at most 3 bytes per
 * body byte).  Returns the bytes of strbuf used, or -(bytes needed) if strcap is short, or
 * INT64_MIN on a bad argument.  threads: 0 = the machine's cores (at most 16). */
int64_t gome_decode_order_nodes(const char* buf, const uint64_t* off, size_t n, uint32_t threads,
                                gome_decoded_node* out, char* strbuf, size_t strcap);

/* ---- one drained batch -> records ------------------------------------------------------------ */
typedef struct gome_consume_stats {
  uint64_t messages;       /* bodies consumed                                                  */
  uint64_t records;        /* records written (an ignored Action still takes a record: DoOrder
                              sees it, engine.go:46-54, and it takes a sequence number)       */
  uint64_t rejected;       /* outside the engine's domain, not submitted: Price / Volume not an
                              exact scaled integer below 2^53 (Q5), a negative Volume, a Symbol
                              beyond max_symbols distinct symbols, a 257th Transaction code    */
  uint64_t ignored;        /* Action not ADD / DEL (syntax errors included)                    */
  uint64_t not_objects;    /* bodies that decoded nothing (syntax error / not an object)       */
  uint64_t admitted;       /* ADDs whose marker existed                                        */
  uint64_t ns_decode;      /* wall time of the parallel decode                                 */
  uint64_t ns_prepare;     /* ... of the parallel pass that hashes and builds the marker keys  */
  uint64_t ns_queue;       /* ... of the queue-order work (interning, markers, records)        */
  uint64_t queue_parallel; /* 1: that work ran shard by shard on the pool; 0: message by message
                              (a Transaction outside 0 / 1, or a Symbol range the batch could
                              fill, keeps it serial; so does a batch below 2048 messages)      */
} gome_consume_stats;
/* Decode, convert and admit messages buf[off[i], off[i + 1]) in queue order.  out[] receives
 * *n_out <= n records (the rejected messages are dropped), msg_index[] (optional) each record's
 * message.  Markers are consumed staged on pp (gome_prepool_commit / _abort).  max_symbols: the
 * engine's symbol range (a Symbol whose id would reach it is rejected; 0: no limit). */
gome_status gome_consume_order_nodes(gome_names* nm, gome_prepool* pp, const char* buf, const uint64_t* off, size_t n,
                                     uint32_t max_symbols, uint32_t threads, gome_order* out, uint32_t* msg_index,
                                     size_t* n_out, gome_consume_stats* st);

/* Diagnostics: the wall time (ns) of each step of the last gome_consume_order_nodes call on nm
 * (its parallel queue-order path: 0 lookups, 1 bucket by shard, 2 new symbols, 3 new uuids / oids
 * and markers, 4 id order, 5 new names stored, 6 their slots, 7 positions, 8 records, 9 the rest;
 * zeros where the call took the serial pass).  Copies min(n, GOME_CONSUME_STEPS) values into ns
 * and returns GOME_CONSUME_STEPS (0 for a null nm). */
#define GOME_CONSUME_STEPS 10
size_t gome_consume_last_steps(const gome_names* nm, uint64_t* ns, size_t n);

/* gome_render_events (gome_abi.h) on several threads: the events are split at taker boundaries
 * and the pieces concatenated in publish order (the same bytes).  Returns the bytes written, or
 * -(bytes needed) when cap is short, or INT64_MIN on a bad argument / unknown id. */
int64_t gome_render_events_mt(const gome_event* ev, size_t n, const gome_order* batch, size_t batch_n,
                              uint64_t seq_base, uint32_t accuracy, const char* const* sym_names, size_t n_sym,
                              const char* const* uuid_names, size_t n_uuid, const char* const* oid_names,
                              size_t n_oid, const int32_t* tx_table, uint32_t threads, char* buf, size_t cap);

/* gome_render_events_mt with the name tables of nm, read under its lock: safe beside
 * gome_consume_order_nodes interning into nm on another thread (an intern that moves a table
 * waits for the render).  The events may only name ids interned before the call. */
int64_t gome_render_events_names(const gome_event* ev, size_t n, const gome_order* batch, size_t batch_n,
                                 uint64_t seq_base, uint32_t accuracy, gome_names* nm, uint32_t threads, char* buf,
                                 size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* GOME_HOST_H */
