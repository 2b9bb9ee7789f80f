/*
 * gome_oracle.c — CPU restatement of gome's matching semantics (clean model).
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/ as the parity checker, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg.  The product
 * (gome_amd/, libgome.so) never links or calls it.
 *
 * PARITY UNPINNED (no reference golden vectors exist; no Go
 * toolchain here).  This file is checked event-for-event and state-for-state
 * against oracle/literal.py, a line-faithful transliteration of the Go engine
 * on a fake Redis (tests/test_oracle_parity.py), and against the committed
 * fixtures under tests/golden/ that literal.py generated.
 *
 * ABI v4 record flags: GOME_ORD_ADM_HOST records take their admission verdict from
 * GOME_ORD_ADMITTED (the consumer's pre-pool markers, gome_amd/consumer.py) instead of the
 * batch rule, exactly as the engine's k_adm_flag does.
 *
 * Model, per symbol S:
 *   - a price-keyed level table shared by both sides: depth (S:depth field,
 *     nodepool.go:61-68) and one FIFO (S:link:<price>, nodelink.go), plus one
 *     membership bit per side set (S:BUY / S:SALE ZSETs, nodepool.go:71-83);
 *   - an (S, oid) -> node index standing in for HGET S:link:<p> S:node:<oid>
 *     (engine.go:92-93), with the price compared explicitly (Q3);
 *   - per-batch admission markers (S:comparison, nodepool.go:14-28) under the
 *     deterministic ingress model of literal.run_batches (Q4);
 *   - the boundary's duplicate-oid rule (Q7, gome_abi.h): an admitted ADD whose (S, oid)
 *     names a live node when the ADD is applied is not applied (literal.py's
 *     consume_boundary applies the same rule before DoOrder).  It depends on the queue order
 *     only, not on where batches start and end.
 * All arithmetic is int64 on value*10^accuracy (exact on the parity domain).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gome/gome_abi.h"

#define MEM_BUY 1u
#define MEM_SALE 2u

typedef struct onode {
  int64_t rem;
  int64_t price;
  uint32_t oid, uuid;
  uint8_t side;
  int32_t prev, next; /* node indices, -1 = none */
} onode;

typedef struct olevel {
  int64_t price, depth;
  int32_t head, tail; /* FIFO "f" / "l" pointers (nodelink.go:34,66) */
  uint32_t nnodes;
  uint32_t member;
} olevel;

typedef struct obook {
  olevel* lv; /* ascending price */
  uint32_t n, cap;
} obook;

typedef struct { uint64_t key; int32_t node; } oidx_ent; /* key 0 empty, ~0 tomb */

typedef struct oracle {
  uint32_t max_symbols;
  obook* books;
  onode* nodes;
  uint32_t nnodes, capnodes;
  int32_t freelist;
  oidx_ent* idx;
  uint64_t idxcap, idxused;
  /* admission (per batch) */
  uint64_t* adm; /* stores hashed (sym,uuid,oid) triple as two words */
  uint32_t* adm3;
  uint64_t admcap;
  uint32_t* dups;   /* batch indices rejected by the Q7 rule */
  uint64_t ndups, dupcap;
  /* events */
  gome_event* ev;
  uint64_t nev, capev;
  gome_stats st;
} oracle;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33; return x;
}

/* ---------------------------------------------------------------- index */
static void idx_put(oracle* o, uint64_t key, int32_t node);
static void idx_grow(oracle* o) {
  oidx_ent* old = o->idx; uint64_t oc = o->idxcap;
  o->idxcap = oc ? oc * 2 : 1024;
  o->idx = (oidx_ent*)calloc(o->idxcap, sizeof(oidx_ent));
  o->idxused = 0;
  for (uint64_t i = 0; i < oc; ++i)
    if (old[i].key && old[i].key != ~0ULL) idx_put(o, old[i].key, old[i].node);
  free(old);
}
static void idx_put(oracle* o, uint64_t key, int32_t node) {
  if ((o->idxused + 1) * 2 > o->idxcap) idx_grow(o);
  uint64_t m = o->idxcap - 1, h = mix64(key) & m;
  while (o->idx[h].key && o->idx[h].key != ~0ULL) h = (h + 1) & m;
  if (!o->idx[h].key) o->idxused++;
  o->idx[h].key = key; o->idx[h].node = node;
}
static int64_t idx_find(const oracle* o, uint64_t key) {
  if (!o->idxcap) return -1;
  uint64_t m = o->idxcap - 1, h = mix64(key) & m;
  while (o->idx[h].key) {
    if (o->idx[h].key == key) return (int64_t)h;
    h = (h + 1) & m;
  }
  return -1;
}
static uint64_t okey(uint32_t sym, uint32_t oid) { return ((uint64_t)(sym + 1) << 32) | oid; }

/* ---------------------------------------------------------------- nodes */
static int32_t node_alloc(oracle* o) {
  if (o->freelist >= 0) { int32_t i = o->freelist; o->freelist = o->nodes[i].next; return i; }
  if (o->nnodes == o->capnodes) {
    o->capnodes = o->capnodes ? o->capnodes * 2 : 4096;
    o->nodes = (onode*)realloc(o->nodes, (size_t)o->capnodes * sizeof(onode));
  }
  return (int32_t)o->nnodes++;
}
static void node_free(oracle* o, int32_t i) { o->nodes[i].next = o->freelist; o->freelist = i; }

/* ---------------------------------------------------------------- levels */
static uint32_t lower_bound(const obook* b, int64_t p) {
  uint32_t lo = 0, hi = b->n;
  while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (b->lv[mid].price < p) lo = mid + 1; else hi = mid; }
  return lo;
}
static olevel* level_find(obook* b, int64_t p) {
  uint32_t k = lower_bound(b, p);
  return (k < b->n && b->lv[k].price == p) ? &b->lv[k] : NULL;
}
static olevel* level_get(obook* b, int64_t p) {
  uint32_t k = lower_bound(b, p);
  if (k < b->n && b->lv[k].price == p) return &b->lv[k];
  if (b->n == b->cap) {
    b->cap = b->cap ? b->cap * 2 : 16;
    b->lv = (olevel*)realloc(b->lv, (size_t)b->cap * sizeof(olevel));
  }
  memmove(&b->lv[k + 1], &b->lv[k], (size_t)(b->n - k) * sizeof(olevel));
  b->n++;
  olevel* L = &b->lv[k];
  L->price = p; L->depth = 0; L->head = L->tail = -1; L->nnodes = 0; L->member = 0;
  return L;
}
static uint32_t side_bit(uint8_t side) { return side == GOME_SALE ? MEM_SALE : MEM_BUY; }

/* ---------------------------------------------------------------- events */
static gome_event* ev_push(oracle* o) {
  if (o->nev == o->capev) {
    o->capev = o->capev ? o->capev * 2 : 4096;
    o->ev = (gome_event*)realloc(o->ev, (size_t)o->capev * sizeof(gome_event));
  }
  gome_event* e = &o->ev[o->nev++];
  memset(e, 0, sizeof *e);
  return e;
}

/* FIFO unlink (nodelink.go:124-166: only / head / tail / middle cases). */
static void fifo_unlink(oracle* o, olevel* L, int32_t i) {
  onode* n = &o->nodes[i];
  if (n->prev >= 0) o->nodes[n->prev].next = n->next; else L->head = n->next;
  if (n->next >= 0) o->nodes[n->next].prev = n->prev; else L->tail = n->prev;
  L->nnodes--;
}

/* MatchOrder, engine.go:138-198, at one level; returns taker remaining. */
static int64_t match_level(oracle* o, uint32_t sym, olevel* L, int64_t T, uint32_t seq,
                           uint32_t* fill_idx) {
  for (;;) {
    int32_t mi = L->head; /* GetFirstNode, nodelink.go:38 */
    if (mi < 0) return T;
    onode* m = &o->nodes[mi];
    int64_t diff = T - m->rem; /* engine.go:143 */
    gome_event* e = ev_push(o);
    e->kind = GOME_EV_FILL; e->taker_seq = seq; e->fill_idx = (*fill_idx)++;
    e->price_fx = L->price;
    e->maker_oid_id = m->oid; e->maker_uuid_id = m->uuid; e->maker_side = m->side;
    e->maker_is_last = m->next < 0;
    e->maker_next_oid_id = m->next >= 0 ? o->nodes[m->next].oid : 0;
    o->st.n_fills++;
    if (diff >= 0) { /* :145-175 maker fully filled (pre-fill volume reported) */
      int64_t mv = m->rem;
      T -= mv;
      e->match_volume_fx = mv; e->maker_volume_fx = mv;
      fifo_unlink(o, L, mi);
      int64_t k = idx_find(o, okey(sym, m->oid));
      if (k >= 0 && o->idx[k].node == mi) o->idx[k].key = ~0ULL;
      L->depth -= mv; /* DeletePoolMatchOrder, engine.go:200-206 */
      if (L->depth <= 0) L->member &= ~side_bit(m->side);
      node_free(o, mi);
      if (diff == 0) return T;
      continue; /* recursion, engine.go:161 */
    }
    /* :176-194 maker partially filled: remaining volume reported, keeps position */
    int64_t fill = T;
    m->rem -= fill;
    e->match_volume_fx = fill; e->maker_volume_fx = m->rem;
    L->depth -= fill;
    if (L->depth <= 0) L->member &= ~side_bit(m->side);
    return 0;
  }
}

static void do_add(oracle* o, const gome_order* r, uint32_t seq) {
  obook* b = &o->books[r->symbol_id];
  int64_t p = r->price_fx, T = r->volume_fx;
  int sale = r->side == GOME_SALE;
  uint32_t opp = sale ? MEM_BUY : MEM_SALE;
  int crossed = 0;
  uint32_t fill_idx = 0;
  /* GetReverseDepth (nodepool.go:86-115) + Match (engine.go:118-136) */
  if (!sale) {
    for (uint32_t k = 0; k < b->n && b->lv[k].price <= p; ++k) {
      if (!(b->lv[k].member & opp)) continue;
      crossed = 1;
      T = match_level(o, r->symbol_id, &b->lv[k], T, seq, &fill_idx);
      if (T <= 0) break;
    }
  } else {
    for (uint32_t k = b->n; k-- > 0 && b->lv[k].price >= p;) {
      if (!(b->lv[k].member & opp)) continue;
      crossed = 1;
      T = match_level(o, r->symbol_id, &b->lv[k], T, seq, &fill_idx);
      if (T <= 0) break;
    }
  }
  if (crossed && T <= 0) return; /* engine.go:69-75 */
  /* rest: SetPoolDepth / SetPoolDepthVolume / SetDepthLink (engine.go:80-82) */
  olevel* L = level_get(b, p);
  L->member |= sale ? MEM_SALE : MEM_BUY;
  L->depth += T;
  int32_t ni = node_alloc(o);
  onode* n = &o->nodes[ni];
  n->rem = T; n->price = p; n->oid = r->oid_id; n->uuid = r->uuid_id; n->side = r->side;
  n->next = -1; n->prev = L->tail;
  if (L->tail >= 0) o->nodes[L->tail].next = ni; else L->head = ni;
  L->tail = ni; L->nnodes++;
  idx_put(o, okey(r->symbol_id, r->oid_id), ni);
  o->st.n_rests++;
}

static void do_del(oracle* o, const gome_order* r, uint32_t seq) {
  /* DeleteOrder, engine.go:87-116 */
  int64_t k = idx_find(o, okey(r->symbol_id, r->oid_id));
  if (k < 0) return;
  int32_t ni = o->idx[k].node;
  onode* n = &o->nodes[ni];
  if (n->price != r->price_fx) return; /* lookup is in S:link:<request price> (Q3) */
  obook* b = &o->books[r->symbol_id];
  olevel* L = level_find(b, n->price);
  int64_t rem = n->rem;
  L->depth -= rem;
  if (L->depth <= 0) L->member &= ~side_bit(r->side); /* request's side set (Q2) */
  fifo_unlink(o, L, ni);
  o->idx[k].key = ~0ULL;
  node_free(o, ni);
  gome_event* e = ev_push(o);
  e->kind = GOME_EV_CANCEL; e->taker_seq = seq; e->fill_idx = 0;
  e->price_fx = r->price_fx; e->match_volume_fx = 0; e->maker_volume_fx = rem;
  e->maker_oid_id = r->oid_id; e->maker_uuid_id = r->uuid_id;
  e->maker_side = r->side; e->maker_is_last = 1; e->maker_next_oid_id = 0;
  o->st.n_cancels++;
}

/* ---------------------------------------------------------------- admission */
/* Marker key (S, uuid, oid) of S:comparison (ordernode.go:89-92). */
static int adm_first(oracle* o, const gome_order* r) {
  uint64_t m = o->admcap - 1;
  uint64_t h = mix64(((uint64_t)r->symbol_id << 40) ^ ((uint64_t)r->uuid_id << 20) ^
                     mix64(r->oid_id)) & m;
  for (;;) {
    uint32_t* s = &o->adm3[3 * h];
    if (!o->adm[h]) {
      o->adm[h] = 1; s[0] = r->symbol_id; s[1] = r->uuid_id; s[2] = r->oid_id;
      return 1;
    }
    if (s[0] == r->symbol_id && s[1] == r->uuid_id && s[2] == r->oid_id) return 0;
    h = (h + 1) & m;
  }
}

/* ---------------------------------------------------------------- API */
oracle* oracle_create(uint32_t max_symbols) {
  oracle* o = (oracle*)calloc(1, sizeof(oracle));
  o->max_symbols = max_symbols;
  o->books = (obook*)calloc(max_symbols, sizeof(obook));
  o->freelist = -1;
  return o;
}

void oracle_destroy(oracle* o) {
  if (!o) return;
  for (uint32_t s = 0; s < o->max_symbols; ++s) free(o->books[s].lv);
  free(o->books); free(o->nodes); free(o->idx); free(o->adm); free(o->adm3); free(o->ev);
  free(o->dups);
  free(o);
}

/* Apply one batch in consume order (rabbitmq.go:116-125).  Events are appended
 * to the oracle's event buffer (taker_seq = index in this batch).  Returns 0, or
 * 1 if a record has symbol_id out of range. */
int oracle_submit(oracle* o, const gome_order* r, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i)
    if (r[i].symbol_id >= o->max_symbols) return 1;
  uint64_t need = 16;
  while (need < 2 * n) need <<= 1;
  if (need > o->admcap) {
    free(o->adm); free(o->adm3);
    o->admcap = need;
    o->adm = (uint64_t*)malloc(need * sizeof(uint64_t));
    o->adm3 = (uint32_t*)malloc(need * 3 * sizeof(uint32_t));
  }
  if (n > o->dupcap) {
    free(o->dups);
    o->dupcap = n;
    o->dups = (uint32_t*)malloc(n * sizeof(uint32_t));
  }
  memset(o->adm, 0, o->admcap * sizeof(uint64_t));
  o->ndups = 0;
  o->st.n_dup_oid = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const gome_order* q = &r[i];
    o->st.n_orders++;
    if (q->action == GOME_ADD) {
      o->st.n_add++;
      int adm = adm_first(o, q); /* engine.go:58-62 (batch model) */
      if (q->flags & GOME_ORD_ADM_HOST) adm = (q->flags & GOME_ORD_ADMITTED) != 0; /* host markers */
      if (!adm) { o->st.n_dropped++; continue; }
      if (idx_find(o, okey(q->symbol_id, q->oid_id)) >= 0) { /* Q7: (S, oid) names a live node */
        o->st.n_dropped++;
        o->st.n_dup_oid++;
        o->dups[o->ndups++] = (uint32_t)i;
        continue;
      }
      do_add(o, q, (uint32_t)i);
    } else if (q->action == GOME_DEL) {
      o->st.n_del++;
      adm_first(o, q); /* DeletePrePool, engine.go:90 */
      do_del(o, q, (uint32_t)i);
    }
  }
  o->st.n_events = o->nev;
  return 0;
}

uint64_t oracle_num_events(const oracle* o) { return o->nev; }
/* Batch indices (ascending) of the last batch's Q7 rejections. */
uint64_t oracle_dup_records(const oracle* o, uint32_t* out, uint64_t cap) {
  for (uint64_t i = 0; i < o->ndups && i < cap; ++i) out[i] = o->dups[i];
  return o->ndups;
}
const gome_event* oracle_events(const oracle* o) { return o->ev; }
void oracle_clear_events(oracle* o) { o->nev = 0; }
void oracle_get_stats(const oracle* o, gome_stats* s) { *s = o->st; }

uint64_t oracle_resting(const oracle* o) {
  uint64_t t = 0;
  for (uint32_t s = 0; s < o->max_symbols; ++s)
    for (uint32_t k = 0; k < o->books[s].n; ++k) t += o->books[s].lv[k].nnodes;
  return t;
}

/* Observable levels over all books (sizing studies). */
uint64_t oracle_levels_total(const oracle* o) {
  uint64_t t = 0;
  for (uint32_t s = 0; s < o->max_symbols; ++s)
    for (uint32_t k = 0; k < o->books[s].n; ++k) {
      const olevel* L = &o->books[s].lv[k];
      t += (L->nnodes || L->depth || L->member) ? 1u : 0u;
    }
  return t;
}

/* Levels with any observable state (nodes, depth or membership), ascending. */
uint64_t oracle_snapshot_levels(const oracle* o, uint32_t sym, gome_level* out, uint64_t cap) {
  if (sym >= o->max_symbols) return 0;
  const obook* b = &o->books[sym];
  uint64_t c = 0;
  for (uint32_t k = 0; k < b->n; ++k) {
    const olevel* L = &b->lv[k];
    if (!L->nnodes && !L->depth && !L->member) continue;
    if (c < cap) {
      out[c].price_fx = L->price; out[c].depth_fx = L->depth; out[c].n_nodes = L->nnodes;
      out[c].in_buy = (L->member & MEM_BUY) != 0; out[c].in_sale = (L->member & MEM_SALE) != 0;
      out[c].pad = 0;
    }
    c++;
  }
  return c;
}

uint64_t oracle_snapshot_fifo(const oracle* o, uint32_t sym, int64_t price, gome_node* out,
                              uint64_t cap) {
  if (sym >= o->max_symbols) return 0;
  olevel* L = level_find(&o->books[sym], price);
  if (!L) return 0;
  uint64_t c = 0;
  for (int32_t i = L->head; i >= 0; i = o->nodes[i].next) {
    if (c < cap) {
      memset(&out[c], 0, sizeof(gome_node));
      out[c].volume_fx = o->nodes[i].rem; out[c].oid_id = o->nodes[i].oid;
      out[c].uuid_id = o->nodes[i].uuid; out[c].side = o->nodes[i].side;
    }
    c++;
  }
  return c;
}
