/*
 * gome_loadgen.h — seeded synthetic order streams for BASELINE.json configs 1-5 (the
 * doorder.go / delorder.go counterparts).
 *
 * The reference's only load generators send 1,999 time-seeded random limit orders
 * (gomengine/doorder.go:34-49: side U{0,1}, price = round2(U[0,1)) with 0 -> 0.10, volume =
 * round2(U[0,1)) with 0 -> 1.00, uuid "2", fresh oids) and one fixed cancel
 * (gomengine/delorder.go:30).  This generator reproduces that distribution at bench scale,
 * plus the configs' symbol laws (uniform / Zipf(s) over symbol rank, rank -> id through the
 * caller's permutation), config 4's cancel mix (each DEL re-sends a uniformly chosen earlier
 * ADD that no DEL targeted yet, with its symbol / side / price / uuid; a share of ADDs are
 * aggressive: BUY @ 1.00 or SALE @ 0.01 with volume k * 10.00, k ~ U{1..16}) and config 5's
 * 4-dp price grid.  `rank / world` keeps the symbols whose Zipf rank % world == rank
 * (the multi-GPU ownership map), sampled conditionally.
 *
 * Host-only (no device work), deterministic for a given config.  Records use gome_abi.h.
 */
#ifndef GOME_LOADGEN_H
#define GOME_LOADGEN_H

#include "gome_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gome_gen_config {
  uint32_t n_symbols;
  uint32_t price_decimals;     /* 2 (doorder) or 4 (config 5)                           */
  double zipf_s;               /* 0: uniform symbols                                    */
  double del_frac;             /* share of records that are DELs (config 4: 0.5)        */
  double aggressive_frac;      /* share of ADDs that sweep (config 4: 0.1)              */
  uint64_t seed;
  uint64_t first_oid;          /* oids are fresh, counting up from here                */
  const uint32_t* rank_to_id;  /* [n_symbols] symbol id of Zipf rank r (NULL: identity) */
  uint32_t rank, world;        /* keep symbols with rank % world == this rank           */
  uint32_t uuid;               /* uuid_id of every ADD (doorder.go: "2")                */
  uint32_t accuracy;           /* fixed-point digits (8)                                */
} gome_gen_config;

typedef struct gome_gen gome_gen;

gome_status gome_gen_create(const gome_gen_config* cfg, gome_gen** out);
/* The next n records of the stream. */
gome_status gome_gen_batch(gome_gen* g, gome_order* out, size_t n);
/* Probability mass of the owned symbols and of the hottest owned symbol. */
gome_status gome_gen_shares(const gome_gen* g, double* owned_share, double* top_share);
void gome_gen_destroy(gome_gen* g);

#ifdef __cplusplus
}
#endif
#endif /* GOME_LOADGEN_H */
