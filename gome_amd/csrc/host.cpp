// host.cpp — host-side pieces of the drop-in boundary that do no device work:
//   * exact fixed-point conversion (ordernode.go:76-87 via shopspring/decimal v1.2.0)
//   * MatchResult JSON rendering byte-identical to Go encoding/json of
//     engine.MatchResult (engine.go:24-28) / engine.OrderNode (ordernode.go:9-36)
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gome/gome_abi.h"
#include "../../include/gome/gome_host.h"
#include "host_pool.h"

namespace {

// shopspring decimal.NewFromFloat keeps the shortest round-trip decimal of x;
// Mul by NewFromFloat(10^acc) is exact; Float64() rounds the exact product to the
// nearest float64.  The product is an integer iff the shortest decimal has at most
// `acc` fractional digits; then the float64 is that integer whenever |v| < 2^53.
gome_status fixed_from_double(double x, uint32_t acc, int64_t* out) {
  if (!out || !std::isfinite(x) || acc > 18) return GOME_E_INVAL;
  if (x == 0.0) { *out = 0; return GOME_OK; }
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::scientific);
  if (r.ec != std::errc()) return GOME_E_INVAL;
  *r.ptr = 0;
  // buf = [-]d[.ddd]e[+-]XX
  const char* p = buf;
  bool neg = false;
  if (*p == '-') { neg = true; ++p; }
  char digits[40];
  int nd = 0;
  for (; *p && *p != 'e'; ++p)
    if (*p != '.') digits[nd++] = *p;
  if (*p != 'e') return GOME_E_INVAL;
  int e10 = std::atoi(p + 1) - (nd - 1);  // x = digits * 10^e10
  while (nd > 1 && digits[nd - 1] == '0') { --nd; ++e10; }
  int shift = e10 + static_cast<int>(acc);
  if (shift < 0) return GOME_E_INVAL;  // more than acc decimals: non-integer product (Q5)
  const uint64_t lim = 1ULL << 53;
  uint64_t v = 0;
  for (int i = 0; i < nd; ++i) {
    v = v * 10 + static_cast<uint64_t>(digits[i] - '0');
    if (v >= lim) return GOME_E_INVAL;
  }
  for (int i = 0; i < shift; ++i) {
    v *= 10;
    if (v >= lim) return GOME_E_INVAL;
  }
  *out = neg ? -static_cast<int64_t>(v) : static_cast<int64_t>(v);
  return GOME_OK;
}

// ---- Go encoding/json pieces -------------------------------------------------
// Output cursor: writes while the bytes (plus a NUL) fit in cap, and counts every byte either
// way, so a caller whose buffer is short learns the size it needs (n + 1).
struct Out {
  char* buf;
  size_t cap, n = 0;
  bool ok = true;
  void put(const char* s, size_t k) {
    if (ok && n + k < cap) std::memcpy(buf + n, s, k);
    else ok = false;
    n += k;
  }
  void put(const char* s) { put(s, std::strlen(s)); }
  void putc(char c) { put(&c, 1); }
};

// encoding/json string encoder with HTML escaping (the default for json.Marshal), without the
// quotes: the key strings are concatenations (S + ":node:" + oid), and escaping is per character,
// so each piece is escaped in turn between one pair of quotes.
void json_escape(Out& o, const char* s) {
  static const char hex[] = "0123456789abcdef";
  const unsigned char* p = reinterpret_cast<const unsigned char*>(s);
  for (;;) {  // runs of bytes that need no escape in one copy
    const unsigned char* q = p;
    while (*q >= 0x20 && *q != '"' && *q != '\\' && *q != '<' && *q != '>' && *q != '&' && *q != 0xE2) ++q;
    if (q != p) o.put(reinterpret_cast<const char*>(p), static_cast<size_t>(q - p));
    p = q;
    if (!*p) return;
    const unsigned char c = *p;
    if (c == '"') o.put("\\\"");
    else if (c == '\\') o.put("\\\\");
    else if (c == '\n') o.put("\\n");
    else if (c == '\r') o.put("\\r");
    else if (c == '\t') o.put("\\t");
    else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      char u[7] = {'\\', 'u', '0', '0', hex[c >> 4], hex[c & 15], 0};
      o.put(u, 6);
    } else if (c == 0xE2 && p[1] == 0x80 && (p[2] == 0xA8 || p[2] == 0xA9)) {
      o.put(p[2] == 0xA8 ? "\\u2028" : "\\u2029");
      p += 2;
    } else {
      o.putc(static_cast<char>(c));
    }
    ++p;
  }
}

void json_string(Out& o, const char* s) {
  o.putc('"');
  json_escape(o, s);
  o.putc('"');
}

// "a" + "b" + ... as one JSON string
void json_cat(Out& o, std::initializer_list<const char*> parts) {
  o.putc('"');
  for (const char* x : parts) json_escape(o, x);
  o.putc('"');
}

// encoding/json float64: strconv 'f' -1, or 'e' -1 outside [1e-6, 1e21) with the
// exponent cleaned from e-09 to e-9.
void json_float(Out& o, double f) {
  char b[64];
  double a = std::fabs(f);
  if (a != 0 && (a < 1e-6 || a >= 1e21)) {
    auto r = std::to_chars(b, b + sizeof b, f, std::chars_format::scientific);
    size_t n = static_cast<size_t>(r.ptr - b);
    if (n >= 4 && b[n - 4] == 'e' && b[n - 3] == '-' && b[n - 2] == '0') {
      b[n - 2] = b[n - 1];
      --n;
    }
    o.put(b, n);
    return;
  }
  if (f == 0) { o.put(std::signbit(f) ? "-0" : "0"); return; }
  auto r = std::to_chars(b, b + sizeof b, f, std::chars_format::fixed);
  o.put(b, static_cast<size_t>(r.ptr - b));
}

void json_int(Out& o, long long v) {
  char b[32];
  auto r = std::to_chars(b, b + sizeof b, v);
  o.put(b, static_cast<size_t>(r.ptr - b));
}

struct NodeView {
  int action;
  const char* uuid;
  const char* oid;
  const char* symbol;
  int transaction;
  int64_t price, volume;
  uint32_t accuracy;
  bool is_first, is_last;
  const char* next_oid;  // nullptr => NextNode ""
  const char* prev_oid = nullptr;  // nullptr => PrevNode ""
};

// encoding/json of OrderNode, fields in declaration order (ordernode.go:9-36), keys
// built as SetOrderHashKey/SetListZsetKey/SetDepthHashKey/SetNodeName/SetNodeLink.
void render_node(Out& o, const NodeView& v) {
  // decimal.NewFromFloat(price).String() for an integer-valued price (ordernode.go:106,115)
  char P[32];
  *std::to_chars(P, P + sizeof P - 1, static_cast<long long>(v.price)).ptr = 0;
  const char* S = v.symbol;
  bool sale = v.transaction == GOME_SALE;
  o.put("{\"Action\":"); json_int(o, v.action);
  o.put(",\"Uuid\":"); json_string(o, v.uuid);
  o.put(",\"Oid\":"); json_string(o, v.oid);
  o.put(",\"Symbol\":"); json_string(o, v.symbol);
  o.put(",\"Transaction\":"); json_int(o, v.transaction);
  o.put(",\"Price\":"); json_float(o, static_cast<double>(v.price));
  o.put(",\"Volume\":"); json_float(o, static_cast<double>(v.volume));
  o.put(",\"Accuracy\":"); json_int(o, v.accuracy);
  o.put(",\"NodeName\":"); json_cat(o, {S, ":node:", v.oid});
  o.put(",\"IsFirst\":"); o.put(v.is_first ? "true" : "false");
  o.put(",\"IsLast\":"); o.put(v.is_last ? "true" : "false");
  o.put(",\"PrevNode\":");
  if (v.prev_oid) json_cat(o, {S, ":node:", v.prev_oid});
  else o.put("\"\"");
  o.put(",\"NextNode\":");
  if (v.next_oid) json_cat(o, {S, ":node:", v.next_oid});
  else o.put("\"\"");
  o.put(",\"NodeLink\":"); json_cat(o, {S, ":link:", P});
  o.put(",\"OrderHashKey\":"); json_cat(o, {S, ":comparison"});
  o.put(",\"OrderHashField\":"); json_cat(o, {S, ":", v.uuid, ":", v.oid});
  o.put(",\"OrderListZsetKey\":"); json_cat(o, {S, sale ? ":SALE" : ":BUY"});
  o.put(",\"OrderListZsetRKey\":"); json_cat(o, {S, sale ? ":BUY" : ":SALE"});
  o.put(",\"OrderDepthHashKey\":"); json_cat(o, {S, ":depth"});
  o.put(",\"OrderDepthHashField\":"); json_cat(o, {S, ":depth:", P});
  o.putc('}');
}

}  // namespace

extern "C" int64_t gome_render_link_node(const char* symbol, int64_t price_fx, int32_t transaction, int64_t volume_fx,
                                         uint32_t accuracy, const char* uuid, const char* oid,
                                         const char* prev_oid, const char* next_oid, char* buf, size_t cap) {
  if (!symbol || !uuid || !oid || (!buf && cap)) return INT64_MIN;
  Out o{buf, cap};
  // a resting node as nodelink.go stores it (SetLinkNode, :119-122): the ADD that rested,
  // its remaining volume, and the FIFO flags / neighbours kept by InitOrderLink, SetLast and
  // DeleteLinkNode (:12-19, :53-64, :124-166)
  NodeView v{GOME_ADD, uuid, oid, symbol, transaction, price_fx, volume_fx, accuracy,
             prev_oid == nullptr, next_oid == nullptr, next_oid, prev_oid};
  render_node(o, v);
  if (!o.ok) return -static_cast<int64_t>(o.n + 1);
  buf[o.n] = 0;
  return static_cast<int64_t>(o.n);
}

extern "C" gome_status gome_fixed_from_double(double x, uint32_t accuracy, int64_t* out) {
  return fixed_from_double(x, accuracy, out);
}

// The doOrder queue carries OrderNodes whose Price / Volume were scaled at gRPC time
// (main.go:41 -> ordernode.go:76-87): exact iff integer-valued and below 2^53.
extern "C" gome_status gome_fixed_from_scaled(double v, int64_t* out) {
  if (!out || !std::isfinite(v)) return GOME_E_INVAL;
  const double lim = 9007199254740992.0;  // 2^53
  if (!(std::fabs(v) < lim) || std::trunc(v) != v) return GOME_E_INVAL;
  *out = static_cast<int64_t>(v);
  return GOME_OK;
}

extern "C" int64_t gome_render_match_result(const gome_event* ev, const gome_order* taker,
                                            int64_t taker_remaining_fx, uint32_t accuracy, const char* symbol,
                                            const char* taker_uuid, const char* taker_oid,
                                            const char* maker_uuid, const char* maker_oid,
                                            const char* maker_next_oid, const int32_t* tx_table,
                                            char* buf, size_t cap);

extern "C" int64_t gome_render_events(const gome_event* ev, size_t n, const gome_order* batch, size_t batch_n,
                                      uint64_t seq_base, uint32_t accuracy, const char* const* sym_names,
                                      size_t n_sym, const char* const* uuid_names, size_t n_uuid,
                                      const char* const* oid_names, size_t n_oid, const int32_t* tx_table,
                                      char* buf, size_t cap) {
  if ((n && (!ev || !batch)) || !sym_names || !uuid_names || !oid_names) return INT64_MIN;
  size_t used = 0;
  bool fits = buf != nullptr;
  char none[1];
  size_t cur = SIZE_MAX;  // the taker whose fills are being rendered, and its remaining volume
  int64_t rem = 0;
  for (size_t i = 0; i < n; ++i) {
    const gome_event& e = ev[i];
    // (taker_seq: the low 32 bits of seq_base + batch index)
    const size_t bi = static_cast<uint32_t>(e.taker_seq - static_cast<uint32_t>(seq_base));
    if (bi >= batch_n) return INT64_MIN;
    const gome_order& t = batch[bi];
    if (bi != cur) {  // Node.Volume: the taker's volume minus its fills so far (engine.go:147,164,184)
      cur = bi;
      rem = t.volume_fx;
    }
    if (e.kind == GOME_EV_FILL) rem -= e.match_volume_fx;
    if (t.symbol_id >= n_sym || t.uuid_id >= n_uuid || t.oid_id >= n_oid) return INT64_MIN;
    const bool fill = e.kind == GOME_EV_FILL;
    if (fill && (e.maker_uuid_id >= n_uuid || e.maker_oid_id >= n_oid ||
                 (!e.maker_is_last && e.maker_next_oid_id >= n_oid)))
      return INT64_MIN;
    // straight into the caller's buffer while it fits (the line, its '\n' and the renderer's
    // NUL), else a sizing pass (cap 0) that only counts
    const size_t room = fits && cap > used ? cap - used : 0;
    int64_t k = gome_render_match_result(
        &e, &t, rem, accuracy, sym_names[t.symbol_id], uuid_names[t.uuid_id], oid_names[t.oid_id],
        fill ? uuid_names[e.maker_uuid_id] : nullptr, fill ? oid_names[e.maker_oid_id] : nullptr,
        (fill && !e.maker_is_last) ? oid_names[e.maker_next_oid_id] : nullptr, tx_table,
        room ? buf + used : none, room);
    if (k == INT64_MIN) return INT64_MIN;
    size_t len;
    if (k >= 0) {  // (it fit with its NUL, so its '\n' fits too)
      len = static_cast<size_t>(k);
      buf[used + len] = '\n';
    } else {
      fits = false;
      len = k >= 0 ? static_cast<size_t>(k) : static_cast<size_t>(-k) - 1;
    }
    used += len + 1;
  }
  return fits ? static_cast<int64_t>(used) : -static_cast<int64_t>(used);
}

extern "C" int64_t gome_render_match_result(const gome_event* ev, const gome_order* taker,
                                            int64_t taker_remaining_fx, uint32_t accuracy, const char* symbol,
                                            const char* taker_uuid, const char* taker_oid,
                                            const char* maker_uuid, const char* maker_oid,
                                            const char* maker_next_oid, const int32_t* tx_table,
                                            char* buf, size_t cap) {
  if (!ev || !taker || !symbol || !taker_uuid || !taker_oid || (!buf && cap)) return INT64_MIN;
  // Transaction codes -> the raw int32 values the reference echoes (Q8, gome_abi.h)
  const int taker_tx = tx_table ? tx_table[taker->side] : taker->side;
  const int maker_tx = tx_table ? tx_table[ev->maker_side] : ev->maker_side;
  Out o{buf, cap};
  o.put("{\"Node\":");
  if (ev->kind == GOME_EV_CANCEL) {
    // engine.go:109 — MatchResult{Node: node, MatchNode: node, MatchVolume: 0}, with
    // node.Volume overwritten by the stored remaining volume (engine.go:89,100).
    NodeView n{taker->action, taker_uuid, taker_oid, symbol, taker_tx, taker->price_fx,
               ev->maker_volume_fx, accuracy, false, false, nullptr};
    render_node(o, n);
    o.put(",\"MatchNode\":");
    render_node(o, n);
  } else {
    if (!maker_uuid || !maker_oid) return INT64_MIN;
    // Node: the taker after this fill (engine.go:154,171,190).
    NodeView t{taker->action, taker_uuid, taker_oid, symbol, taker_tx, taker->price_fx,
               taker_remaining_fx, accuracy, false, false, nullptr};
    render_node(o, t);
    // MatchNode: the FIFO head as stored (IsFirst, PrevNode "", Action ADD).
    NodeView m{GOME_ADD, maker_uuid, maker_oid, symbol, maker_tx, ev->price_fx,
               ev->maker_volume_fx, accuracy, true, ev->maker_is_last != 0,
               ev->maker_is_last ? nullptr : maker_next_oid};
    if (!ev->maker_is_last && !maker_next_oid) return INT64_MIN;
    o.put(",\"MatchNode\":");
    render_node(o, m);
  }
  o.put(",\"MatchVolume\":");
  json_float(o, static_cast<double>(ev->match_volume_fx));
  o.putc('}');
  if (!o.ok) return -static_cast<int64_t>(o.n + 1);  // the buffer size it needs
  buf[o.n] = 0;
  return static_cast<int64_t>(o.n);
}

// gome_render_events over `threads` pieces cut at taker boundaries (a taker's Node.Volume is a
// running sum over its consecutive events): each piece rendered into a buffer of its own, then the
// pieces copied into the caller's buffer at their offsets, both on the host worker pool (host_pool.h).
// The piece buffers are kept from call to call (no per-call allocation, zero fill or thread start:
// ADVICE r5; one call at a time takes them).
namespace {
struct RenderPiece {
  std::unique_ptr<char[]> b;
  size_t cap = 0;
  int64_t got = 0;
};
std::mutex g_render_mu;
std::vector<RenderPiece> g_pieces;
}  // namespace

extern "C" int64_t gome_render_events_mt(const gome_event* ev, size_t n, const gome_order* batch, size_t batch_n,
                                         uint64_t seq_base, uint32_t accuracy, const char* const* sym_names,
                                         size_t n_sym, const char* const* uuid_names, size_t n_uuid,
                                         const char* const* oid_names, size_t n_oid, const int32_t* tx_table,
                                         uint32_t threads, char* buf, size_t cap) {
  if ((n && (!ev || !batch)) || !sym_names || !uuid_names || !oid_names || (!buf && cap)) return INT64_MIN;
  uint32_t t = threads ? threads : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  t = static_cast<uint32_t>(std::max<size_t>(1, std::min<size_t>({t, 64, (n + 255) / 256})));
  std::vector<size_t> cut(t + 1, n);
  cut[0] = 0;
  for (uint32_t k = 1; k < t; ++k) {
    size_t i = std::max(cut[k - 1], n * k / t);
    while (i > cut[k - 1] && i < n && ev[i].taker_seq == ev[i - 1].taker_seq) ++i;
    cut[k] = i;
  }
  std::lock_guard<std::mutex> one(g_render_mu);
  if (g_pieces.size() < t) g_pieces.resize(t);
  auto render = [&](uint32_t k) {
    const size_t a = cut[k], b = cut[k + 1];
    RenderPiece& pc = g_pieces[k];
    size_t want = std::max<size_t>(4096, (b - a) * 1400);
    for (;;) {
      if (pc.cap < want) {
        pc.b.reset(new char[want]);  // (not zero-filled)
        pc.cap = want;
      }
      const int64_t r = gome_render_events(ev + a, b - a, batch, batch_n, seq_base, accuracy, sym_names, n_sym,
                                           uuid_names, n_uuid, oid_names, n_oid, tx_table, pc.b.get(), pc.cap);
      if (r == INT64_MIN || r >= 0) {
        pc.got = r;
        return;
      }
      want = static_cast<size_t>(-r) + 1;
    }
  };
  gome_host::Pool::get(1).run(t, render);
  std::vector<size_t> at(t + 1, 0);
  for (uint32_t k = 0; k < t; ++k) {
    if (g_pieces[k].got == INT64_MIN) return INT64_MIN;
    at[k + 1] = at[k] + static_cast<size_t>(g_pieces[k].got);
  }
  const size_t total = at[t];
  if (total + 1 > cap) return -static_cast<int64_t>(total + 1);
  gome_host::Pool::get(1).run(t, [&](uint32_t k) {
    std::memcpy(buf + at[k], g_pieces[k].b.get(), static_cast<size_t>(g_pieces[k].got));
  });
  buf[total] = 0;
  return static_cast<int64_t>(total);
}
