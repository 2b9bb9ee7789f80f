// loadgen.cpp — seeded synthetic order streams (include/gome/gome_loadgen.h).
//
// Distribution of gomengine/doorder.go:34-49 (side, price, volume) and delorder.go:30 (a
// cancel re-sends its target's fields), scaled to BASELINE configs 1-5.  xoshiro256** RNG.
#include "../../include/gome/gome_loadgen.h"

#include <algorithm>
#include <cmath>
#include <new>
#include <vector>

namespace {

struct Rng {
  uint64_t s[4];
  explicit Rng(uint64_t seed) {
    for (auto& w : s) {  // splitmix64 seeding
      seed += 0x9e3779b97f4a7c15ull;
      uint64_t z = seed;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      w = z ^ (z >> 31);
    }
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  double uni() { return static_cast<double>(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0, 1)
};

int64_t pow10i(uint32_t k) {
  int64_t v = 1;
  while (k--) v *= 10;
  return v;
}

}  // namespace

struct gome_gen {
  gome_gen_config cfg{};
  Rng rng{0};
  std::vector<double> cdf;       // over the owned ranks
  std::vector<uint32_t> ids;     // symbol id of each owned rank
  double owned = 1.0, top = 0.0;
  uint64_t next_oid = 1;
  std::vector<gome_order> live;  // ADDs no DEL targeted yet (config 4)
  int64_t fx = 100000000;
};

extern "C" {

gome_status gome_gen_create(const gome_gen_config* c, gome_gen** out) {
  if (!c || !out || !c->n_symbols || !c->world || c->rank >= c->world) return GOME_E_INVAL;
  gome_gen* g = new (std::nothrow) gome_gen();
  if (!g) return GOME_E_CAPACITY;
  g->cfg = *c;
  g->rng = Rng(c->seed * 0x100000001b3ull + 1000003ull * c->rank + 17);
  g->next_oid = c->first_oid ? c->first_oid : 1;
  g->fx = pow10i(c->accuracy ? c->accuracy : 8);
  // symbol law over ranks, restricted to the owned ranks (conditional sampling)
  std::vector<double> w(c->n_symbols);
  double tot = 0;
  for (uint32_t r = 0; r < c->n_symbols; ++r) {
    w[r] = c->zipf_s > 0 ? 1.0 / std::pow(static_cast<double>(r + 1), c->zipf_s) : 1.0;
    tot += w[r];
  }
  double acc = 0, own = 0;
  for (uint32_t r = c->rank; r < c->n_symbols; r += c->world) own += w[r];
  g->owned = own / tot;
  for (uint32_t r = c->rank; r < c->n_symbols; r += c->world) {
    acc += w[r] / own;
    g->cdf.push_back(acc);
    g->ids.push_back(c->rank_to_id ? c->rank_to_id[r] : r);
  }
  if (g->cdf.empty()) { delete g; return GOME_E_INVAL; }
  g->cdf.back() = 1.0;
  g->top = w[c->rank] / tot;
  *out = g;
  return GOME_OK;
}

gome_status gome_gen_batch(gome_gen* g, gome_order* out, size_t n) {
  if (!g || (n && !out)) return GOME_E_INVAL;
  const gome_gen_config& c = g->cfg;
  const int64_t q = pow10i(c.price_decimals);
  const int64_t pstep = g->fx / q, vstep = g->fx / 100;
  for (size_t i = 0; i < n; ++i) {
    gome_order& o = out[i];
    if (c.del_frac > 0 && !g->live.empty() && g->rng.uni() < c.del_frac) {
      // delorder.go: a cancel re-sends the target's symbol / oid / uuid / side / price
      const size_t j = static_cast<size_t>(g->rng.uni() * static_cast<double>(g->live.size()));
      o = g->live[j];
      o.action = GOME_DEL;
      g->live[j] = g->live.back();
      g->live.pop_back();
      continue;
    }
    const double u = g->rng.uni();
    const size_t r = static_cast<size_t>(std::upper_bound(g->cdf.begin(), g->cdf.end(), u) - g->cdf.begin());
    o.symbol_id = g->ids[std::min(r, g->ids.size() - 1)];
    o.side = static_cast<uint8_t>(g->rng.next() >> 63);  // doorder.go:37
    int64_t pk = static_cast<int64_t>(std::nearbyint(g->rng.uni() * static_cast<double>(q)));
    if (pk == 0) pk = q / 10;                               // doorder.go:38-41, :63-67
    int64_t vk = static_cast<int64_t>(std::nearbyint(g->rng.uni() * 100.0));
    if (vk == 0) vk = 100;                                  // doorder.go:43-47
    o.price_fx = pk * pstep;
    o.volume_fx = vk * vstep;
    if (c.aggressive_frac > 0 && g->rng.uni() < c.aggressive_frac) {
      o.price_fx = o.side == GOME_SALE ? g->fx / 100 : g->fx;  // SALE @ 0.01, BUY @ 1.00
      o.volume_fx = static_cast<int64_t>(1 + (g->rng.next() >> 60)) * 10 * g->fx;  // k * 10.00
    }
    o.uuid_id = c.uuid;
    o.oid_id = static_cast<uint32_t>(g->next_oid++);
    o.action = GOME_ADD;
    o.flags = 0;
    if (c.del_frac > 0) g->live.push_back(o);
  }
  return GOME_OK;
}

gome_status gome_gen_shares(const gome_gen* g, double* owned_share, double* top_share) {
  if (!g) return GOME_E_INVAL;
  if (owned_share) *owned_share = g->owned;
  if (top_share) *top_share = g->top;
  return GOME_OK;
}

void gome_gen_destroy(gome_gen* g) { delete g; }

}  // extern "C"
