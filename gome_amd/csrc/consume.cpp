// consume.cpp — the batching consumer's per-message work in native code (include/gome/gome_host.h):
// Go encoding/json decoding of the doOrder OrderNode bodies (rabbitmq.go:118-121), interning,
// fixed-point conversion and the pre-pool admission markers (engine.go:58-62,90;
// nodepool.go:14-28), one call per drained batch.  Host-only: no device work.
#include <algorithm>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gome/gome_host.h"
#include "host_pool.h"

extern "C" gome_status gome_fixed_from_scaled(double v, int64_t* out);

namespace {

constexpr int MAX_DEPTH = 10000;  // encoding/json scanner.go maxNestingDepth

// ---- UTF-8 (Go unicode/utf8) -------------------------------------------------------------------
// utf8.DecodeRune: (rune, size), (U+FFFD, 1) for a byte that does not start a valid encoding
// (bad lead, truncated, overlong, surrogate, beyond U+10FFFF).
inline uint32_t decode_rune(const unsigned char* p, const unsigned char* e, int* size) {
  const unsigned c = p[0];
  *size = 1;
  if (c < 0x80) return c;
  auto cont = [&](int k, unsigned lo, unsigned hi) { return p + k < e && p[k] >= lo && p[k] <= hi; };
  if (c >= 0xC2 && c <= 0xDF) {
    if (!cont(1, 0x80, 0xBF)) return 0xFFFD;
    *size = 2;
    return ((c & 0x1F) << 6) | (p[1] & 0x3F);
  }
  if (c >= 0xE0 && c <= 0xEF) {
    const unsigned lo = c == 0xE0 ? 0xA0 : 0x80, hi = c == 0xED ? 0x9F : 0xBF;
    if (!cont(1, lo, hi) || !cont(2, 0x80, 0xBF)) return 0xFFFD;
    *size = 3;
    return ((c & 0x0F) << 12) | ((p[1] & 0x3F) << 6) | (p[2] & 0x3F);
  }
  if (c >= 0xF0 && c <= 0xF4) {
    const unsigned lo = c == 0xF0 ? 0x90 : 0x80, hi = c == 0xF4 ? 0x8F : 0xBF;
    if (!cont(1, lo, hi) || !cont(2, 0x80, 0xBF) || !cont(3, 0x80, 0xBF)) return 0xFFFD;
    *size = 4;
    return ((c & 0x07) << 18) | ((p[1] & 0x3F) << 12) | ((p[2] & 0x3F) << 6) | (p[3] & 0x3F);
  }
  return 0xFFFD;
}

inline void put_rune(std::string& o, uint32_t r) {
  if (r < 0x80) {
    o.push_back(static_cast<char>(r));
  } else if (r < 0x800) {
    o.push_back(static_cast<char>(0xC0 | (r >> 6)));
    o.push_back(static_cast<char>(0x80 | (r & 0x3F)));
  } else if (r < 0x10000) {
    o.push_back(static_cast<char>(0xE0 | (r >> 12)));
    o.push_back(static_cast<char>(0x80 | ((r >> 6) & 0x3F)));
    o.push_back(static_cast<char>(0x80 | (r & 0x3F)));
  } else {
    o.push_back(static_cast<char>(0xF0 | (r >> 18)));
    o.push_back(static_cast<char>(0x80 | ((r >> 12) & 0x3F)));
    o.push_back(static_cast<char>(0x80 | ((r >> 6) & 0x3F)));
    o.push_back(static_cast<char>(0x80 | (r & 0x3F)));
  }
}

inline int hexv(unsigned c) {
  if (c >= '0' && c <= '9') return static_cast<int>(c - '0');
  if (c >= 'a' && c <= 'f') return static_cast<int>(c - 'a' + 10);
  if (c >= 'A' && c <= 'F') return static_cast<int>(c - 'A' + 10);
  return -1;
}
inline uint32_t hex4(const unsigned char* q) {
  return static_cast<uint32_t>((hexv(q[0]) << 12) | (hexv(q[1]) << 8) | (hexv(q[2]) << 4) | hexv(q[3]));
}

// ---- the decoder -------------------------------------------------------------------------------
// A decoded string: a view into the body (no escape, ASCII only) or a slice of the thread's arena.
struct Str {
  const char* p = nullptr;
  uint32_t len = 0;
  int32_t arena = -1;  // >= 0: p is unset, the bytes are arenas[arena][off, off + len)
  uint32_t off = 0;
};

enum { F_ACTION, F_UUID, F_OID, F_SYMBOL, F_TX, F_PRICE, F_VOLUME, NF };

struct Dec {
  double price = 0, volume = 0;
  int32_t tx = 0;
  int8_t action = 0;
  bool is_object = false;
  Str s[3];  // uuid, oid, symbol
};

// Field match by Go's foldName (encoding/json fold.go): ASCII letters to upper case, and the two
// non-ASCII runes whose fold orbit holds an ASCII letter (U+017F long s ~ S, U+212A Kelvin ~ K).
// An exact match is also a folded match, and the fields' folded names are distinct.
inline bool eq_fold(const unsigned char* k, const char* up, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if ((k[i] | 0x20) != (static_cast<unsigned char>(up[i]) | 0x20)) return false;  // (up: letters only)
  return true;
}

int match_field_slow(const unsigned char* k, size_t n);

// ASCII keys by length first (every field name is letters only, so a key byte matches an upper-case
// letter U iff it is U or U + 32); keys with a byte >= 0x80 take the rune-by-rune fold.
inline int match_field(const unsigned char* k, size_t n) {
  switch (n) {
    case 3: if (eq_fold(k, "OID", 3)) return F_OID; break;
    case 4: if (eq_fold(k, "UUID", 4)) return F_UUID; break;
    case 5: if (eq_fold(k, "PRICE", 5)) return F_PRICE; break;
    case 6:
      if (eq_fold(k, "ACTION", 6)) return F_ACTION;
      if (eq_fold(k, "SYMBOL", 6)) return F_SYMBOL;
      if (eq_fold(k, "VOLUME", 6)) return F_VOLUME;
      break;
    case 11: if (eq_fold(k, "TRANSACTION", 11)) return F_TX; break;
    default: break;
  }
  for (size_t i = 0; i < n; ++i)
    if (k[i] >= 0x80) return match_field_slow(k, n);
  return -1;
}

int match_field_slow(const unsigned char* k, size_t n) {
  static const char* const up[NF] = {"ACTION", "UUID", "OID", "SYMBOL", "TRANSACTION", "PRICE", "VOLUME"};
  char f[16];
  size_t m = 0;
  for (size_t i = 0; i < n;) {
    if (m >= 12) return -1;
    const unsigned c = k[i];
    if (c < 0x80) {
      f[m++] = static_cast<char>((c >= 'a' && c <= 'z') ? c - 32 : c);
      ++i;
      continue;
    }
    int sz;
    const uint32_t r = decode_rune(k + i, k + n, &sz);
    if (r == 0x17F) f[m++] = 'S';
    else if (r == 0x212A) f[m++] = 'K';
    else return -1;
    i += static_cast<size_t>(sz);
  }
  for (int j = 0; j < NF; ++j)
    if (std::strlen(up[j]) == m && std::memcmp(up[j], f, m) == 0) return j;
  return -1;
}

struct Parser {
  const unsigned char* p;
  const unsigned char* e;
  std::string* arena;
  int32_t arena_id;
  std::string key;  // a decoded key (slow path)

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }

  // A string at p ('"'): validated (scanner.go stateInString: control bytes are errors, any other
  // byte passes; escapes \" \\ \/ \b \f \n \r \t \uXXXX); [*s, *t) the raw bytes between the quotes;
  // *plain: no escape and no byte >= 0x80 (the decoded string is the raw bytes).
  bool scan_string(const unsigned char** s, const unsigned char** t, bool* plain) {
    ++p;
    *s = p;
    bool pl = true;
    for (;;) {
      while (p < e && *p != '"' && *p != '\\' && *p >= 0x20 && *p < 0x80) ++p;  // (the common bytes)
      if (p >= e) return false;
      const unsigned c = *p;
      if (c == '"') break;
      if (c == '\\') {
        pl = false;
        if (p + 1 >= e) return false;
        const unsigned x = p[1];
        if (x == 'u') {
          if (p + 6 > e) return false;
          for (int k = 2; k < 6; ++k)
            if (hexv(p[k]) < 0) return false;
          p += 6;
        } else if (x == '"' || x == '\\' || x == '/' || x == 'b' || x == 'f' || x == 'n' || x == 'r' || x == 't') {
          p += 2;
        } else {
          return false;
        }
        continue;
      }
      if (c < 0x20) return false;
      if (c >= 0x80) pl = false;
      ++p;
    }
    *t = p++;
    *plain = pl;
    return true;
  }

  // encoding/json unquote (decode.go): escapes, surrogate pairs, a lone surrogate -> U+FFFD,
  // invalid UTF-8 -> U+FFFD per byte.
  static void unquote(const unsigned char* q, const unsigned char* t, std::string& o) {
    while (q < t) {
      const unsigned c = *q;
      if (c == '\\') {
        const unsigned x = q[1];
        if (x != 'u') {
          char ch = static_cast<char>(x);
          if (x == 'b') ch = '\b';
          else if (x == 'f') ch = '\f';
          else if (x == 'n') ch = '\n';
          else if (x == 'r') ch = '\r';
          else if (x == 't') ch = '\t';
          o.push_back(ch);
          q += 2;
          continue;
        }
        uint32_t r = hex4(q + 2);
        q += 6;
        if (r >= 0xD800 && r < 0xE000) {
          // utf16.DecodeRune(r, getu4(next)): a pair only for high + \u-escaped low
          if (r < 0xDC00 && q + 6 <= t && q[0] == '\\' && q[1] == 'u') {
            const uint32_t r1 = hex4(q + 2);
            if (r1 >= 0xDC00 && r1 < 0xE000) {
              put_rune(o, 0x10000 + ((r - 0xD800) << 10) + (r1 - 0xDC00));
              q += 6;
              continue;
            }
          }
          r = 0xFFFD;
        }
        put_rune(o, r);
        continue;
      }
      if (c < 0x80) {
        o.push_back(static_cast<char>(c));
        ++q;
        continue;
      }
      int sz;
      const uint32_t r = decode_rune(q, t, &sz);
      if (r == 0xFFFD && sz == 1) put_rune(o, 0xFFFD);
      else o.append(reinterpret_cast<const char*>(q), static_cast<size_t>(sz));
      q += sz;
    }
  }

  bool string_value(Str* out) {
    const unsigned char *s, *t;
    bool plain;
    if (!scan_string(&s, &t, &plain)) return false;
    if (!out) return true;
    if (plain) {
      out->p = reinterpret_cast<const char*>(s);
      out->len = static_cast<uint32_t>(t - s);
      out->arena = -1;
    } else {
      const size_t o0 = arena->size();
      unquote(s, t, *arena);
      out->arena = arena_id;
      out->off = static_cast<uint32_t>(o0);
      out->len = static_cast<uint32_t>(arena->size() - o0);
    }
    return true;
  }

  // A number literal at p (JSON grammar); [*s, p) its text; *is_int: no fraction, no exponent.
  bool number(const unsigned char** s, bool* is_int) {
    *s = p;
    if (*p == '-') ++p;
    if (p >= e) return false;
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < e && *p >= '0' && *p <= '9') ++p;
    } else {
      return false;
    }
    *is_int = true;
    if (p < e && *p == '.') {
      ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
      *is_int = false;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      if (p >= e || *p < '0' || *p > '9') return false;
      while (p < e && *p >= '0' && *p <= '9') ++p;
      *is_int = false;
    }
    return true;
  }

  bool literal(const char* w) {
    const size_t n = std::strlen(w);
    if (static_cast<size_t>(e - p) < n || std::memcmp(p, w, n) != 0) return false;
    p += n;
    return true;
  }

  // Validate one value at p (after whitespace), nested in `depth` containers; iterative.
  bool skip_value(int depth) {
    std::vector<char> st;  // open containers below this value
    for (;;) {
      // a value
      ws();
      if (p >= e) return false;
      const unsigned c = *p;
      bool opened = false;
      if (c == '{' || c == '[') {
        if (depth + static_cast<int>(st.size()) + 1 > MAX_DEPTH) return false;
        ++p;
        ws();
        if (p < e && *p == (c == '{' ? '}' : ']')) {
          ++p;  // empty container: a complete value
        } else {
          st.push_back(static_cast<char>(c));
          opened = true;
        }
      } else if (c == '"') {
        const unsigned char *s, *t;
        bool pl;
        if (!scan_string(&s, &t, &pl)) return false;
      } else if (c == '-' || (c >= '0' && c <= '9')) {
        const unsigned char* s;
        bool ii;
        if (!number(&s, &ii)) return false;
      } else if (!(literal("true") || literal("false") || literal("null"))) {
        return false;
      }
      if (opened && st.back() == '{') {  // its first key
        if (!object_key()) return false;
        continue;
      }
      if (opened) continue;  // an array's first element
      // after a complete value: close containers, or move to the next member / element
      for (;;) {
        if (st.empty()) return true;
        ws();
        if (p >= e) return false;
        const char top = st.back();
        if (*p == ',') {
          ++p;
          if (top == '{' && !object_key()) return false;
          break;
        }
        if (*p == (top == '{' ? '}' : ']')) {
          ++p;
          st.pop_back();
          continue;
        }
        return false;
      }
    }
  }

  // a value at p whose first byte is c: scalars inline, containers through skip_value
  bool skip_scalar_or_value(unsigned c) {
    if (c == '"') {
      const unsigned char *s, *t;
      bool pl;
      return scan_string(&s, &t, &pl);
    }
    if (c == '-' || (c >= '0' && c <= '9')) {
      const unsigned char* s;
      bool ii;
      return number(&s, &ii);
    }
    if (c == 't') return lit4("true");
    if (c == 'n') return lit4("null");
    if (c == 'f') {
      if (e - p < 5 || std::memcmp(p, "false", 5) != 0) return false;
      p += 5;
      return true;
    }
    return skip_value(1);
  }
  bool lit4(const char* w) {
    if (e - p < 4 || std::memcmp(p, w, 4) != 0) return false;
    p += 4;
    return true;
  }

  // "key" ws ':' (the value follows)
  bool object_key() {
    ws();
    if (p >= e || *p != '"') return false;
    const unsigned char *s, *t;
    bool pl;
    if (!scan_string(&s, &t, &pl)) return false;
    ws();
    if (p >= e || *p != ':') return false;
    ++p;
    return true;
  }

  // json.Unmarshal(body, &OrderNode{}) for the fields the engine reads.
  bool decode(Dec& d) {
    ws();
    if (p >= e) return false;
    if (*p != '{') {  // a valid non-object decodes nothing (null: no effect; other: type error)
      if (!skip_value(0)) return false;
      ws();
      return false;
    }
    Dec t;
    ++p;
    ws();
    if (p < e && *p == '}') {
      ++p;
    } else {
      for (;;) {
        ws();
        if (p >= e || *p != '"') return false;
        const unsigned char *ks, *kt;
        bool kpl;
        if (!scan_string(&ks, &kt, &kpl)) return false;
        int f;
        if (kpl) {
          f = match_field(ks, static_cast<size_t>(kt - ks));
        } else {
          key.clear();
          unquote(ks, kt, key);
          f = match_field(reinterpret_cast<const unsigned char*>(key.data()), key.size());
        }
        ws();
        if (p >= e || *p != ':') return false;
        ++p;
        ws();
        if (p >= e) return false;
        const unsigned c = *p;
        if (f < 0) {
          if (!skip_scalar_or_value(c)) return false;
        } else if (c == '"') {
          Str* sv = f == F_UUID ? &t.s[0] : f == F_OID ? &t.s[1] : f == F_SYMBOL ? &t.s[2] : nullptr;
          if (!string_value(sv)) return false;  // (into a numeric field: a type error, skipped)
        } else if (c == '-' || (c >= '0' && c <= '9')) {
          const unsigned char* ns;
          bool is_int;
          if (!number(&ns, &is_int)) return false;
          if (f == F_PRICE || f == F_VOLUME) {
            double v;
            if (parse_float(ns, p, &v)) (f == F_PRICE ? t.price : t.volume) = v;
          } else if ((f == F_ACTION || f == F_TX) && is_int) {
            int64_t v;
            const int64_t lo = f == F_ACTION ? -128 : INT32_MIN, hi = f == F_ACTION ? 127 : INT32_MAX;
            if (parse_int(ns, p, &v) && v >= lo && v <= hi) {
              if (f == F_ACTION) t.action = static_cast<int8_t>(v);
              else t.tx = static_cast<int32_t>(v);
            }
          }
        } else {
          if (!skip_value(1)) return false;  // null, bool, object, array: no effect / type error
        }
        ws();
        if (p >= e) return false;
        if (*p == ',') {
          ++p;
          continue;
        }
        if (*p == '}') {
          ++p;
          break;
        }
        return false;
      }
    }
    ws();
    if (p != e) return false;
    t.is_object = true;
    d = t;
    return true;
  }

  // strconv.ParseInt(s, 10, 64): an error (skipped field) beyond int64
  static bool parse_int(const unsigned char* s, const unsigned char* t, int64_t* out) {
    bool neg = false;
    if (*s == '-') {
      neg = true;
      ++s;
    }
    uint64_t v = 0;
    const uint64_t lim = neg ? (1ull << 63) : (1ull << 63) - 1;
    for (; s < t; ++s) {
      const uint64_t d = static_cast<uint64_t>(*s - '0');
      if (v > (lim - d) / 10) return false;
      v = v * 10 + d;
    }
    *out = neg ? static_cast<int64_t>(0 - v) : static_cast<int64_t>(v);
    return true;
  }

  // strconv.ParseFloat(s, 64): correctly rounded; out of range (+-Inf) is an error (skipped
  // field), an underflow gives the rounded value (0 or a subnormal)
  static bool parse_float(const unsigned char* s, const unsigned char* t, double* out) {
    const char* a = reinterpret_cast<const char*>(s);
    const char* b = reinterpret_cast<const char*>(t);
    auto r = std::from_chars(a, b, *out);
    if (r.ec == std::errc() && r.ptr == b) return std::isfinite(*out);
    std::string z(a, b);  // (out of range for from_chars: strtod tells overflow from underflow)
    const double v = std::strtod(z.c_str(), nullptr);
    if (!std::isfinite(v)) return false;
    *out = v;
    return true;
  }
};

uint32_t pick_threads(uint32_t threads, size_t n) {
  uint32_t t = threads ? threads : std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
  t = std::min<uint32_t>(t, 64);
  const size_t per = 1024;  // messages per thread worth a thread
  return static_cast<uint32_t>(std::max<size_t>(1, std::min<size_t>(t, (n + per - 1) / per)));
}

// Decode messages [0, n) on `nt` threads: dec[i], arenas[thread].
void decode_all(const char* buf, const uint64_t* off, size_t n, uint32_t nt, std::vector<Dec>& dec,
                std::vector<std::string>& arenas) {
  dec.assign(n, Dec{});
  arenas.resize(nt);
  for (std::string& a : arenas) a.clear();  // (capacity kept: a consumer's scratch is reused per batch)
  auto work = [&](uint32_t k) {
    const size_t i0 = n * k / nt, i1 = n * (k + 1) / nt;
    // (the thread's own string object while it appends: the vector's neighbouring string objects
    // share cache lines, and every append writes the size)
    std::string ar;
    ar.swap(arenas[k]);
    ar.reserve(64 * (i1 - i0));
    Parser ps{nullptr, nullptr, &ar, static_cast<int32_t>(k), {}};
    for (size_t i = i0; i < i1; ++i) {
      ps.p = reinterpret_cast<const unsigned char*>(buf + off[i]);
      ps.e = reinterpret_cast<const unsigned char*>(buf + off[i + 1]);
      const size_t mark = ar.size();
      if (!ps.decode(dec[i])) {
        dec[i] = Dec{};
        ar.resize(mark);
      }
    }
    arenas[k].swap(ar);
  };
  gome_host::Pool::get().run(nt, work);
}

inline const char* str_ptr(const Str& s, const std::vector<std::string>& arenas) {
  return s.arena >= 0 ? arenas[static_cast<size_t>(s.arena)].data() + s.off : s.p;
}

// ---- interning -----------------------------------------------------------------------------------
inline uint64_t hash_bytes(const char* s, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xFF51AFD7ED558CCDull);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, s + i, 8);
    h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
    h ^= h >> 29;
  }
  uint64_t w = 0;
  std::memcpy(&w, s + i, n - i);
  h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 32;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  return h;
}

// Open addressing, in IN_SHARDS tables by the hash's top bits (so a batch's new names can be
// interned shard by shard on several threads, gome_consume_order_nodes); a slot holds (id + 1, the
// hash's high 32 bits), so a probe that is not the string reads no string.  Ids are global, handed
// out in first-seen order; strings live NUL-terminated in 1 MiB blocks (per shard) that never move.
// During a parallel intern a slot may hold a provisional entry (IN_PROV | its index in the shard's
// batch list) until the batch's new names get their ids.
constexpr uint32_t IN_SHARDS = 64, IN_PROV = 0x80000000u;
inline uint32_t in_shard(uint64_t h) { return static_cast<uint32_t>(h >> 58); }

struct Interner {
  struct Fresh {
    const char* s;
    uint32_t n;
    uint32_t first;  // the message that names it first (queue order)
    uint64_t h;
  };
  struct alignas(64) Store {  // string blocks that never move (a shard's, or a pool thread's)
    std::vector<std::unique_ptr<char[]>> blocks;
    size_t bused = 0, bcap = 0;
  };
  struct alignas(64) Shard : Store {  // (a cache line of its own: neighbouring shards are other threads')
    std::vector<uint64_t> slot;  // (id + 1 or IN_PROV | fresh index) | tag << 32; 0 = empty
    uint64_t mask = 0;
    std::vector<uint32_t> ids;   // the shard's ids (its rehash)
    std::vector<Fresh> fresh;    // a parallel intern's new names, in queue order
    std::vector<uint32_t> fresh_id;
  };
  Shard sh[IN_SHARDS];
  // by id; its reallocation (the only change a reader of older ids can see) happens under *gmu,
  // which gome_render_events_names holds shared while it renders beside the next batch's decode
  std::vector<const char*> strs;
  std::vector<uint32_t> lens;
  std::vector<uint64_t> hs;
  std::shared_mutex* gmu = nullptr;

  std::vector<Store> tstore;  // the pool threads' (a parallel intern stores its new names there)
  void reserve_stores(uint32_t nt) {
    if (tstore.size() < nt) tstore.resize(nt);
  }
  static const char* store(Store& d, const char* s, size_t n) {
    if (n + 1 > d.bcap - d.bused) {  // (blocks of 4 KiB doubling to 1 MiB: 3 x 64 shards start small)
      const size_t cap = std::max<size_t>(std::min<size_t>(size_t{4096} << d.blocks.size(), 1 << 20), n + 1);
      d.blocks.emplace_back(new char[cap]);
      d.bused = 0;
      d.bcap = cap;
    }
    char* p = d.blocks.back().get() + d.bused;
    std::memcpy(p, s, n);
    p[n] = 0;
    d.bused += n + 1;
    return p;
  }
  static void put(Shard& d, uint64_t h, uint64_t v) {
    uint64_t j = h & d.mask;
    while (d.slot[j]) j = (j + 1) & d.mask;
    d.slot[j] = v | (h >> 32 << 32);
  }
  // room for one more entry (its ids and the provisional ones, rehashed)
  void reserve1(Shard& d) {
    if ((d.ids.size() + d.fresh.size() + 1) * 2 <= d.mask + 1) return;
    const uint64_t cap = std::max<uint64_t>(1024, (d.mask + 1) * 2);
    d.slot.assign(cap, 0);
    d.mask = cap - 1;
    for (uint32_t id : d.ids) put(d, hs[id], id + 1ull);
    for (uint32_t l = 0; l < d.fresh.size(); ++l) put(d, d.fresh[l].h, IN_PROV | l);
  }
  // the slot value of the string (id + 1, or IN_PROV | fresh index during a parallel intern), or 0
  uint32_t lookup(const Shard& d, const char* s, size_t n, uint64_t h) const {
    if (d.slot.empty()) return 0;
    const uint64_t tag = h >> 32 << 32;
    for (uint64_t j = h & d.mask;; j = (j + 1) & d.mask) {
      const uint64_t v = d.slot[j];
      if (!v) return 0;
      if ((v & ~0xFFFFFFFFull) != tag) continue;
      const uint32_t x = static_cast<uint32_t>(v);
      if (x & IN_PROV) {
        const Fresh& f = d.fresh[x & ~IN_PROV];
        if (f.n == n && std::memcmp(f.s, s, n) == 0) return x;
      } else if (lens[x - 1] == n && std::memcmp(strs[x - 1], s, n) == 0) {
        return x;
      }
    }
  }
  int64_t find(const char* s, size_t n, uint64_t h) const {
    const uint32_t x = lookup(sh[in_shard(h)], s, n, h);
    return (x && !(x & IN_PROV)) ? static_cast<int64_t>(x - 1) : -1;
  }
  void prefetch(uint64_t h) const {
    const Shard& d = sh[in_shard(h)];
    if (!d.slot.empty()) __builtin_prefetch(&d.slot[h & d.mask]);
  }
  // second stage (the slot is in cache by now): the string its first probe compares against
  void prefetch2(uint64_t h) const {
    const Shard& d = sh[in_shard(h)];
    if (d.slot.empty()) return;
    const uint64_t v = d.slot[h & d.mask];
    if (v && (v & ~0xFFFFFFFFull) == (h >> 32 << 32) && !(static_cast<uint32_t>(v) & IN_PROV))
      __builtin_prefetch(strs[static_cast<uint32_t>(v) - 1]);
  }
  // room in the id tables for `more` new ids (they move: not while a render reads them)
  void grow_tables(size_t more) {
    const size_t want = strs.size() + more;
    if (want <= strs.capacity()) return;
    std::unique_lock<std::shared_mutex> lk(*gmu);
    strs.reserve(std::max<size_t>({1024, strs.capacity() * 2, want}));
  }
  // the id tables `more` longer at once (a parallel intern's new names; their entries are written
  // after, each by its shard's thread: a render never reads ids of the batch being interned)
  void extend_tables(size_t more) {
    grow_tables(more);
    std::unique_lock<std::shared_mutex> lk(*gmu);
    strs.resize(strs.size() + more);
    lens.resize(lens.size() + more);
    hs.resize(hs.size() + more);
  }
  uint32_t intern(const char* s, size_t n) { return intern_h(s, n, hash_bytes(s, n)); }
  uint32_t intern_h(const char* s, size_t n, uint64_t h) {
    Shard& d = sh[in_shard(h)];
    const uint32_t x = lookup(d, s, n, h);
    if (x) return x - 1;
    reserve1(d);
    grow_tables(1);
    const uint32_t id = static_cast<uint32_t>(strs.size());
    strs.push_back(store(d, s, n));
    lens.push_back(static_cast<uint32_t>(n));
    hs.push_back(h);
    d.ids.push_back(id);
    put(d, h, id + 1ull);
    return id;
  }
};

}  // namespace

namespace {
struct ConsumePre {  // gome_consume_order_nodes: one message's probes and values
  uint64_t hs, hu, ho, hk;
  int64_t p, v;
  uint32_t koff, klen, ka;  // the marker key: karena[ka][koff, koff + klen)
  uint8_t kind;             // 0 ignored action, 1 outside the domain (price / volume), 2 good
};
struct ConsumeScratch {
  std::vector<Dec> dec;
  std::vector<std::string> arenas, karena;
  std::vector<ConsumePre> pre;
  std::vector<uint32_t> odd_tx, cnt, kbase;
  std::vector<uint32_t> idx[4], pos[4], start[4], ref[3], first[3], newmsg[3], owner;
  std::vector<uint8_t> adm;
  std::vector<gome_consume_stats> ps;
  uint64_t step_ns[GOME_CONSUME_STEPS] = {};  // the last call's parallel queue-order steps (gome_consume_last_steps)
};
}  // namespace

struct gome_names {
  Interner in[3];
  ConsumeScratch scratch;  // (the consumer thread's, batch after batch)
  int32_t tx_raw[GOME_TX_CODES];
  uint32_t tx_n = 2;
  std::shared_mutex mu;  // the id tables' moves (Interner::gmu)
  gome_names() {
    for (int i = 0; i < GOME_TX_CODES; ++i) tx_raw[i] = i;
    for (Interner& x : in) x.gmu = &mu;
  }
  int32_t tx_code(int32_t raw) {
    if (raw == 0 || raw == 1) return raw;
    for (uint32_t c = 2; c < tx_n; ++c)
      if (tx_raw[c] == raw) return static_cast<int32_t>(c);
    if (tx_n == GOME_TX_CODES) return -1;
    tx_raw[tx_n] = raw;
    return static_cast<int32_t>(tx_n++);
  }
};

// The markers: open addressing over (hash, key bytes in an arena), in PP_SHARDS tables by the
// hash's top bits, each with its lock (the consumer stages a batch's markers shard by shard on
// several threads; the gRPC side's gome_prepool_set takes one shard's lock).  A marker the consumer
// took provisionally is STAGED until commit (-> a tombstone) or abort (-> live again).  A STAGED
// marker set again before the commit (the gRPC side's SetPrePool after the consumer's
// DeletePrePool, nodepool.go:14-28) is RESET: commit leaves it LIVE (the new marker), abort LIVE too
// (one key, one marker).
constexpr uint32_t PP_SHARDS = 64;
inline uint32_t pp_shard(uint64_t h) { return static_cast<uint32_t>(h >> 58); }

struct alignas(64) PPShard {  // (a cache line of its own: neighbouring shards are other threads')
  enum : uint8_t { EMPTY = 0, LIVE = 1, TOMB = 2, STAGED = 3, RESET = 4 };
  struct Ent {
    uint64_t h;
    uint64_t off;  // key bytes in arena
    uint32_t len;
    uint8_t state;
  };
  std::mutex mu;
  std::vector<Ent> tab;
  uint64_t mask = 0, live = 0, used = 0;  // used: live + staged + tombstones
  std::vector<char> arena;
  std::vector<uint64_t> staged;  // slots

  bool same(const Ent& x, uint64_t h, const char* k, size_t n) const {
    return x.h == h && x.len == n && std::memcmp(arena.data() + x.off, k, n) == 0;
  }
  // slot of the key (LIVE, STAGED or RESET), or -1
  int64_t find(const char* k, size_t n, uint64_t h) const {
    if (tab.empty()) return -1;
    for (uint64_t j = h & mask;; j = (j + 1) & mask) {
      const Ent& x = tab[j];
      if (x.state == EMPTY) return -1;
      if (x.state != TOMB && same(x, h, k, n)) return static_cast<int64_t>(j);
    }
  }
  void prefetch(uint64_t h) const {
    if (!tab.empty()) __builtin_prefetch(&tab[h & mask]);
  }
  void prefetch2(uint64_t h) const {  // (second stage: the key bytes of the slot's entry)
    if (tab.empty()) return;
    const Ent& x = tab[h & mask];
    if (x.state != EMPTY && x.h == h) __builtin_prefetch(arena.data() + x.off);
  }
  void rebuild(uint64_t cap) {  // (drops tombstones and their key bytes)
    std::vector<Ent> old;
    old.swap(tab);
    std::vector<char> oa;
    oa.swap(arena);
    tab.assign(cap, Ent{0, 0, 0, EMPTY});
    mask = cap - 1;
    used = 0;
    for (const Ent& x : old) {
      if (x.state != LIVE && x.state != STAGED && x.state != RESET) continue;
      uint64_t j = x.h & mask;
      while (tab[j].state != EMPTY) j = (j + 1) & mask;
      tab[j] = Ent{x.h, arena.size(), x.len, x.state};
      arena.insert(arena.end(), oa.begin() + static_cast<long>(x.off), oa.begin() + static_cast<long>(x.off + x.len));
      ++used;
    }
    staged.clear();  // (slots moved: re-list the staged ones)
    for (uint64_t j = 0; j < cap; ++j)
      if (tab[j].state == STAGED || tab[j].state == RESET) staged.push_back(j);
  }
  void set(const char* k, size_t n, uint64_t h) {
    const int64_t f = find(k, n, h);
    if (f >= 0) {  // (a staged marker set again: the commit keeps it)
      if (tab[static_cast<size_t>(f)].state == STAGED) tab[static_cast<size_t>(f)].state = RESET;
      return;
    }
    if ((used + 1) * 2 > mask + 1) rebuild(std::max<uint64_t>(1024, (live + 1) * 4 > mask + 1 ? (mask + 1) * 2 : mask + 1));
    uint64_t j = h & mask;
    while (tab[j].state == LIVE || tab[j].state == STAGED || tab[j].state == RESET) j = (j + 1) & mask;
    if (tab[j].state == EMPTY) ++used;
    tab[j] = Ent{h, arena.size(), static_cast<uint32_t>(n), LIVE};
    arena.insert(arena.end(), k, k + n);
    ++live;
  }
  bool take(const char* k, size_t n, uint64_t h) {
    const int64_t j = find(k, n, h);
    if (j < 0) return false;
    uint8_t& st = tab[static_cast<size_t>(j)].state;
    if (st == RESET) {  // (the re-set marker taken: the consumer's staged take still pending)
      st = STAGED;
      return true;
    }
    if (st != LIVE) return false;
    st = TOMB;
    --live;
    return true;
  }
  // the staged ExistsPrePool + DeletePrePool of an ADD (engine.go:58-62), and the staged
  // DeletePrePool of a DEL (engine.go:90): a LIVE marker becomes STAGED.  (The caller holds mu.)
  bool stage_locked(const char* k, size_t n, uint64_t h) {
    const int64_t j = find(k, n, h);
    if (j < 0) return false;
    uint8_t& st = tab[static_cast<size_t>(j)].state;
    if (st == RESET) {  // (the re-set marker consumed again in the same window; already listed)
      st = STAGED;
      return true;
    }
    if (st != LIVE) return false;
    st = STAGED;
    staged.push_back(static_cast<uint64_t>(j));
    return true;
  }
  void commit() {
    std::lock_guard<std::mutex> g(mu);
    for (uint64_t j : staged)
      if (tab[j].state == STAGED) {
        tab[j].state = TOMB;
        --live;
      } else if (tab[j].state == RESET) {
        tab[j].state = LIVE;
      }
    staged.clear();
  }
  void abort() {
    std::lock_guard<std::mutex> g(mu);
    for (uint64_t j : staged)
      if (tab[j].state == STAGED || tab[j].state == RESET) tab[j].state = LIVE;
    staged.clear();
  }
};

struct gome_prepool {
  PPShard sh[PP_SHARDS];
  static void key(std::string& k, const char* s, size_t sn, const char* u, size_t un, const char* o, size_t on) {
    k.clear();
    const uint32_t a = static_cast<uint32_t>(sn), b = static_cast<uint32_t>(un);
    k.append(reinterpret_cast<const char*>(&a), 4).append(s, sn);
    k.append(reinterpret_cast<const char*>(&b), 4).append(u, un);
    k.append(o, on);
  }
  PPShard& of(uint64_t h) { return sh[pp_shard(h)]; }
};

extern "C" {

gome_names* gome_names_create(void) { return new (std::nothrow) gome_names(); }
void gome_names_destroy(gome_names* nm) { delete nm; }

int64_t gome_names_intern(gome_names* nm, int kind, const char* s, size_t len) {
  if (!nm || kind < 0 || kind > 2 || (!s && len) || len > 0xFFFFFFFFu) return -1;
  return nm->in[kind].intern(s ? s : "", len);
}

int64_t gome_names_find(const gome_names* nm, int kind, const char* s, size_t len) {
  if (!nm || kind < 0 || kind > 2 || (!s && len)) return -1;
  return nm->in[kind].find(s ? s : "", len, hash_bytes(s ? s : "", len));
}

size_t gome_names_count(const gome_names* nm, int kind) {
  return (nm && kind >= 0 && kind <= 2) ? nm->in[kind].strs.size() : 0;
}

const char* gome_names_get(const gome_names* nm, int kind, uint32_t id, size_t* len) {
  if (!nm || kind < 0 || kind > 2 || id >= nm->in[kind].strs.size()) return nullptr;
  if (len) *len = nm->in[kind].lens[id];
  return nm->in[kind].strs[id];
}

const char* const* gome_names_table(gome_names* nm, int kind) {
  if (!nm || kind < 0 || kind > 2) return nullptr;
  static const char* const empty[1] = {""};
  return nm->in[kind].strs.empty() ? empty : nm->in[kind].strs.data();
}

int32_t gome_names_tx_code(gome_names* nm, int32_t raw) { return nm ? nm->tx_code(raw) : -1; }

size_t gome_consume_last_steps(const gome_names* nm, uint64_t* ns, size_t n) {
  if (!nm) return 0;
  const size_t k = std::min<size_t>(n, GOME_CONSUME_STEPS);
  for (size_t i = 0; ns && i < k; ++i) ns[i] = nm->scratch.step_ns[i];
  return GOME_CONSUME_STEPS;
}

int64_t gome_render_events_names(const gome_event* ev, size_t n, const gome_order* batch, size_t batch_n,
                                 uint64_t seq_base, uint32_t accuracy, gome_names* nm, uint32_t threads, char* buf,
                                 size_t cap) {
  if (!nm) return INT64_MIN;
  std::shared_lock<std::shared_mutex> lk(nm->mu);  // (the tables stay where they are meanwhile)
  const char* const* t[3];
  size_t c[3];
  static const char* const empty[1] = {nullptr};
  for (int k = 0; k < 3; ++k) {
    c[k] = nm->in[k].strs.size();
    t[k] = c[k] ? nm->in[k].strs.data() : empty;
  }
  return gome_render_events_mt(ev, n, batch, batch_n, seq_base, accuracy, t[0], c[0], t[1], c[1], t[2], c[2],
                               nm->tx_raw, threads, buf, cap);
}
const int32_t* gome_names_tx_table(const gome_names* nm) { return nm ? nm->tx_raw : nullptr; }
size_t gome_names_tx_count(const gome_names* nm) { return nm ? nm->tx_n : 0; }

gome_prepool* gome_prepool_create(void) { return new (std::nothrow) gome_prepool(); }
void gome_prepool_destroy(gome_prepool* pp) { delete pp; }

void gome_prepool_set(gome_prepool* pp, const char* sym, size_t sym_len, const char* uuid, size_t uuid_len,
                      const char* oid, size_t oid_len) {
  if (!pp || (!sym && sym_len) || (!uuid && uuid_len) || (!oid && oid_len)) return;
  std::string k;
  gome_prepool::key(k, sym, sym_len, uuid, uuid_len, oid, oid_len);
  const uint64_t h = hash_bytes(k.data(), k.size());
  PPShard& d = pp->of(h);
  std::lock_guard<std::mutex> g(d.mu);
  d.set(k.data(), k.size(), h);
}

int32_t gome_prepool_take(gome_prepool* pp, const char* sym, size_t sym_len, const char* uuid, size_t uuid_len,
                          const char* oid, size_t oid_len) {
  if (!pp || (!sym && sym_len) || (!uuid && uuid_len) || (!oid && oid_len)) return 0;
  std::string k;
  gome_prepool::key(k, sym, sym_len, uuid, uuid_len, oid, oid_len);
  const uint64_t h = hash_bytes(k.data(), k.size());
  PPShard& d = pp->of(h);
  std::lock_guard<std::mutex> g(d.mu);
  return d.take(k.data(), k.size(), h) ? 1 : 0;
}

size_t gome_prepool_size(const gome_prepool* pp) {
  if (!pp) return 0;
  size_t n = 0;
  for (PPShard& d : const_cast<gome_prepool*>(pp)->sh) {
    std::lock_guard<std::mutex> g(d.mu);
    n += d.live;
  }
  return n;
}

void gome_prepool_commit(gome_prepool* pp) {
  if (pp)
    for (PPShard& d : pp->sh) d.commit();
}

void gome_prepool_abort(gome_prepool* pp) {
  if (pp)
    for (PPShard& d : pp->sh) d.abort();
}

int64_t gome_decode_order_nodes(const char* buf, const uint64_t* off, size_t n, uint32_t threads,
                                gome_decoded_node* out, char* strbuf, size_t strcap) {
  if ((n && (!buf || !off || !out)) || (!strbuf && strcap)) return INT64_MIN;
  std::vector<Dec> dec;
  std::vector<std::string> arenas;
  decode_all(buf, off, n, pick_threads(threads, n), dec, arenas);
  size_t used = 0;
  for (size_t i = 0; i < n; ++i)
    for (const Str& s : dec[i].s) used += s.len;
  if (used > strcap) return -static_cast<int64_t>(used);
  size_t at = 0;
  for (size_t i = 0; i < n; ++i) {
    const Dec& d = dec[i];
    gome_decoded_node& o = out[i];
    o = gome_decoded_node{};
    o.price = d.price;
    o.volume = d.volume;
    o.transaction = d.tx;
    o.action = d.action;
    o.is_object = d.is_object ? 1 : 0;
    uint32_t* fo[3][2] = {{&o.uuid_off, &o.uuid_len}, {&o.oid_off, &o.oid_len}, {&o.sym_off, &o.sym_len}};
    for (int k = 0; k < 3; ++k) {
      const Str& s = d.s[k];
      if (s.len) std::memcpy(strbuf + at, str_ptr(s, arenas), s.len);
      *fo[k][0] = static_cast<uint32_t>(at);
      *fo[k][1] = s.len;
      at += s.len;
    }
  }
  return static_cast<int64_t>(used);
}

gome_status gome_consume_order_nodes(gome_names* nm, gome_prepool* pp, const char* buf, const uint64_t* off, size_t n,
                                     uint32_t max_symbols, uint32_t threads, gome_order* out, uint32_t* msg_index,
                                     size_t* n_out, gome_consume_stats* st) {
  if (!nm || !pp || !n_out || (n && (!buf || !off || !out))) return GOME_E_INVAL;
  // (the names' scratch, reused batch after batch: fresh multi-megabyte vectors were page-faulted in
  // by every pool thread at once, and the faults, not the work, set the parallel passes' time)
  ConsumeScratch& W = nm->scratch;
  std::vector<Dec>& dec = W.dec;
  std::vector<std::string>& arenas = W.arenas;
  const uint32_t nt = pick_threads(threads, n);
  using clk = std::chrono::steady_clock;
  const auto ns = [](clk::time_point a, clk::time_point b) {
    return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count());
  };
  gome_host::Pool& pool = gome_host::Pool::get();
  const auto t0 = clk::now();
  decode_all(buf, off, n, nt, dec, arenas);
  const auto t1 = clk::now();
  // Per message, on the pool: the hashes the queue-order work probes with (symbol, uuid, oid and the
  // marker key, built here as gome_prepool::key builds it), the fixed-point values, and whether the
  // batch can take the parallel path below.
  std::vector<ConsumePre>& pre = W.pre;
  std::vector<std::string>& karena = W.karena;
  std::vector<uint32_t>& odd_tx = W.odd_tx;
  pre.resize(n);
  karena.resize(nt);
  for (std::string& a : karena) a.clear();
  odd_tx.assign(nt, 0);
  pool.run(nt, [&](uint32_t t) {
    const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
    std::string ka;  // (the thread's own while it appends, as decode_all's arenas)
    ka.swap(karena[t]);
    ka.reserve(48 * (i1 - i0));
    uint32_t odd = 0;
    for (size_t i = i0; i < i1; ++i) {
      const Dec& d = dec[i];
      ConsumePre& q = pre[i];
      q.kind = 0;
      if (d.action != GOME_ADD && d.action != GOME_DEL) continue;
      const char* sym = str_ptr(d.s[2], arenas);
      const char* uuid = str_ptr(d.s[0], arenas);
      const char* oid = str_ptr(d.s[1], arenas);
      const size_t sl = d.s[2].len, ul = d.s[0].len, ol = d.s[1].len;
      q.hs = hash_bytes(sym ? sym : "", sl);
      q.hu = hash_bytes(uuid ? uuid : "", ul);
      q.ho = hash_bytes(oid ? oid : "", ol);
      const size_t k0 = ka.size();
      const uint32_t a = static_cast<uint32_t>(sl), b = static_cast<uint32_t>(ul);
      ka.append(reinterpret_cast<const char*>(&a), 4).append(sym ? sym : "", sl);
      ka.append(reinterpret_cast<const char*>(&b), 4).append(uuid ? uuid : "", ul);
      ka.append(oid ? oid : "", ol);
      q.koff = static_cast<uint32_t>(k0);
      q.ka = t;
      q.klen = static_cast<uint32_t>(ka.size() - k0);
      q.hk = hash_bytes(ka.data() + k0, q.klen);
      const bool bad = gome_fixed_from_scaled(d.price, &q.p) != GOME_OK ||
                       gome_fixed_from_scaled(d.volume, &q.v) != GOME_OK || q.v < 0;
      q.kind = bad ? 1 : 2;
      if (bad) continue;
      odd += (d.tx != 0 && d.tx != 1) ? 1u : 0u;  // (the parallel path's precondition)
    }
    odd_tx[t] = odd;
    karena[t].swap(ka);
  });
  const auto t2 = clk::now();
  gome_consume_stats s{};
  s.messages = n;
  // The queue-order work -- ids handed out in first-seen order, markers consumed in queue order
  // (engine.go:58-62,90) -- in parallel where the order it must respect allows: a name's id depends
  // only on which messages named a new name first, and a marker's fate only on the messages with
  // its key.  So each kind's new names are found shard by shard (a shard's messages in queue order,
  // on the pool), numbered by their first message, and the markers staged shard by shard.  Two
  // rules break that independence and take the serial pass instead: a Symbol that would reach the
  // engine's max_symbols (its message is dropped, so later names shift), and a Transaction outside
  // 0 / 1 (its code is handed out in queue order and a 257th drops the message).
  uint32_t odd = 0;
  for (uint32_t t = 0; t < nt; ++t) odd += odd_tx[t];
  bool parallel = nt > 1 && odd == 0;
  size_t k = 0;
  for (uint64_t& x : W.step_ns) x = 0;
  auto lt = clk::now();
  auto lap = [&](int i) {  // (one step of the parallel path done)
    const auto t = clk::now();
    W.step_ns[i] = ns(lt, t);
    lt = t;
  };
  if (parallel) {
    const uint32_t NS = IN_SHARDS;
    constexpr uint32_t QPF = 16;  // prefetch distance (messages)
    static_assert(PP_SHARDS == IN_SHARDS, "one pass over the shards of both kinds of table");
    auto hash_of = [&](const ConsumePre& q, int kk) { return kk == 0 ? q.hs : kk == 1 ? q.hu : q.ho; };
    auto si_of = [](int kk) { return kk == 0 ? 2 : kk == 1 ? 0 : 1; };  // (Dec::s order: uuid, oid, symbol)
    // 1. every name looked up in the tables as the batch found them, read-only, by message range
    //    (a name's messages spread over the threads however skewed the names are: the hottest
    //    symbol alone is 8% of config 3's messages): ref = id + 1, or 0 for a name not seen before
    std::vector<uint32_t>* ref = W.ref;
    for (int kk = 0; kk < 3; ++kk) ref[kk].resize(n);
    pool.run(nt, [&](uint32_t t) {
      const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
      for (size_t i = i0; i < i1; ++i) {
        if (i + QPF < i1 && pre[i + QPF].kind == 2)
          for (int kk = 0; kk < 3; ++kk) nm->in[kk].prefetch(hash_of(pre[i + QPF], kk));
        if (i + QPF / 2 < i1 && pre[i + QPF / 2].kind == 2)
          for (int kk = 0; kk < 3; ++kk) nm->in[kk].prefetch2(hash_of(pre[i + QPF / 2], kk));
        if (pre[i].kind != 2) continue;
        for (int kk = 0; kk < 3; ++kk) {
          const Str& x = dec[i].s[si_of(kk)];
          const char* str = str_ptr(x, arenas);
          const uint64_t h = hash_of(pre[i], kk);
          ref[kk][i] = nm->in[kk].lookup(nm->in[kk].sh[in_shard(h)], str ? str : "", x.len, h);
        }
      }
    });
    lap(0);
    // 2. the names not seen before and every marker, by shard: a counting sort of their messages
    //    (queue order kept), then a shard's messages in order on one thread -- the first message of
    //    a new name gives it a provisional entry, a marker is staged
    std::vector<uint32_t>* idx = W.idx;      // new names of kind 0..2 (interner shards), markers (pre-pool shards)
    std::vector<uint32_t>* start = W.start;
    std::vector<uint32_t>& cnt = W.cnt;
    cnt.assign(static_cast<size_t>(nt) * NS * 4, 0);
    auto shard_of = [&](size_t i, int kk) -> uint32_t {
      return kk < 3 ? in_shard(hash_of(pre[i], kk)) : pp_shard(pre[i].hk);
    };
    auto wanted = [&](size_t i, int kk) { return kk < 3 ? pre[i].kind == 2 && ref[kk][i] == 0 : pre[i].kind != 0; };
    pool.run(nt, [&](uint32_t t) {
      const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
      uint32_t* c = &cnt[static_cast<size_t>(t) * NS * 4];
      for (size_t i = i0; i < i1; ++i)
        for (int kk = 0; kk < 4; ++kk)
          if (wanted(i, kk)) c[kk * NS + shard_of(i, kk)]++;
    });
    for (int kk = 0; kk < 4; ++kk) {
      start[kk].assign(NS + 1, 0);
      uint32_t run = 0;
      for (uint32_t sh = 0; sh < NS; ++sh) {
        start[kk][sh] = run;
        for (uint32_t t = 0; t < nt; ++t) {
          uint32_t& c = cnt[(static_cast<size_t>(t) * 4 + kk) * NS + sh];
          const uint32_t v = c;
          c = run;
          run += v;
        }
      }
      start[kk][NS] = run;
      idx[kk].resize(run);
    }
    pool.run(nt, [&](uint32_t t) {
      const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
      uint32_t* c = &cnt[static_cast<size_t>(t) * NS * 4];
      for (size_t i = i0; i < i1; ++i)
        for (int kk = 0; kk < 4; ++kk)
          if (wanted(i, kk)) idx[kk][c[kk * NS + shard_of(i, kk)]++] = static_cast<uint32_t>(i);
    });
    lap(1);
    // (outputs by position in idx[], written by one thread each: indexed by message they would be
    // written from every thread at neighbouring addresses)
    std::vector<uint32_t>* nref = W.first;  // a new name's message: IN_PROV | its shard's fresh index
    std::vector<uint8_t>& adm = W.adm;
    for (int kk = 0; kk < 3; ++kk) nref[kk].resize(idx[kk].size());
    adm.assign(idx[3].size(), 0);
    auto names_pass = [&](uint32_t sh, int kk) {
      Interner& in = nm->in[kk];
      Interner::Shard& d = in.sh[sh];
      d.fresh.clear();
      for (uint32_t r = start[kk][sh]; r < start[kk][sh + 1]; ++r) {
        const uint32_t i = idx[kk][r];
        const uint64_t h = hash_of(pre[i], kk);
        const Str& x = dec[i].s[si_of(kk)];
        const char* str = str_ptr(x, arenas);
        uint32_t v = in.lookup(d, str ? str : "", x.len, h);  // (a provisional entry of this batch, or none)
        if (!v) {
          in.reserve1(d);
          v = IN_PROV | static_cast<uint32_t>(d.fresh.size());
          d.fresh.push_back(Interner::Fresh{str ? str : "", x.len, i, h});
          Interner::put(d, h, v);
        }
        nref[kk][r] = v;
      }
    };
    // the symbols first: the batch's new ones must fit the engine's symbol range (else the serial
    // pass, which drops the messages whose symbol would not fit; their provisional entries go)
    pool.run(nt, [&](uint32_t t) {
      for (uint32_t sh = t; sh < NS; sh += nt) names_pass(sh, 0);
    });
    lap(2);
    size_t new_syms = 0;
    for (const Interner::Shard& d : nm->in[0].sh) new_syms += d.fresh.size();
    if (max_symbols && nm->in[0].strs.size() + new_syms > max_symbols) {
      for (Interner::Shard& d : nm->in[0].sh) {
        if (d.fresh.empty()) continue;
        d.fresh.clear();
        std::fill(d.slot.begin(), d.slot.end(), 0ull);
        for (uint32_t id : d.ids) Interner::put(d, nm->in[0].hs[id], id + 1ull);
      }
      parallel = false;
    }
    if (parallel) {
      pool.run(nt, [&](uint32_t t) {
        for (uint32_t sh = t; sh < NS; sh += nt) {
          names_pass(sh, 1);
          names_pass(sh, 2);
          PPShard& d = pp->sh[sh];
          std::lock_guard<std::mutex> g(d.mu);
          const uint32_t r1 = start[3][sh + 1];
          for (uint32_t r = start[3][sh]; r < r1; ++r) {
            if (r + 2 * QPF < r1) __builtin_prefetch(&pre[idx[3][r + 2 * QPF]]);
            if (r + QPF < r1) d.prefetch(pre[idx[3][r + QPF]].hk);
            if (r + QPF / 2 < r1) d.prefetch2(pre[idx[3][r + QPF / 2]].hk);
            const ConsumePre& q = pre[idx[3][r]];
            adm[r] = d.stage_locked(karena[q.ka].data() + q.koff, q.klen, q.hk) ? 1 : 0;
          }
        }
      });
      lap(3);
      // 3. ids of each kind's new names in the order of their first messages: a shard's fresh
      //    entries are in its queue order, so a merge by first message numbers them (newmsg: the
      //    fresh entries in id order, as (shard, index))
      bool any_new = false;
      size_t base[3];
      for (int kk = 0; kk < 3; ++kk) {
        Interner& in = nm->in[kk];
        std::vector<uint32_t>& order = W.newmsg[kk];
        order.clear();
        base[kk] = in.strs.size();
        // (each message introduces at most one name of a kind: the entries by first message, then
        // read in message order)
        std::vector<uint32_t>& owner = W.owner;
        bool any = false;
        for (uint32_t sh = 0; sh < NS && !any; ++sh) any = !in.sh[sh].fresh.empty();
        if (!any) continue;
        owner.assign(n, ~0u);
        for (uint32_t sh = 0; sh < NS; ++sh)
          for (uint32_t l = 0; l < in.sh[sh].fresh.size(); ++l) owner[in.sh[sh].fresh[l].first] = sh << 24 | l;
        for (size_t i = 0; i < n; ++i)
          if (owner[i] != ~0u) order.push_back(owner[i]);
        for (Interner::Shard& d : in.sh) d.fresh_id.resize(d.fresh.size());
        in.extend_tables(order.size());
        in.reserve_stores(nt);
        any_new = true;
      }
      lap(4);
      if (any_new)
        pool.run(nt, [&](uint32_t t) {
          for (int kk = 0; kk < 3; ++kk) {
            Interner& in = nm->in[kk];
            // the new names stored and their id entries written, a range of ids per thread (by shard,
            // the threads would write neighbouring ids: the same cache lines)
            const std::vector<uint32_t>& order = W.newmsg[kk];
            const size_t a = order.size() * t / nt, b = order.size() * (t + 1) / nt;
            for (size_t r = a; r < b; ++r) {
              Interner::Shard& d = in.sh[order[r] >> 24];
              const uint32_t l = order[r] & 0xFFFFFF;
              const Interner::Fresh& f = d.fresh[l];
              const size_t id = base[kk] + r;
              in.strs[id] = Interner::store(in.tstore[t], f.s, f.n);
              in.lens[id] = f.n;
              in.hs[id] = f.h;
              d.fresh_id[l] = static_cast<uint32_t>(id);
            }
          }
        });
      lap(5);
      if (any_new)
        pool.run(nt, [&](uint32_t t) {  // (... and the shards' slots given the ids)
          for (int kk = 0; kk < 3; ++kk)
            for (uint32_t sh = t; sh < NS; sh += nt) {
              Interner::Shard& d = nm->in[kk].sh[sh];
              for (uint32_t l = 0; l < d.fresh.size(); ++l) {
                const uint32_t id = d.fresh_id[l];
                const uint64_t h = d.fresh[l].h;
                d.ids.push_back(id);
                for (uint64_t j = h & d.mask;; j = (j + 1) & d.mask)
                  if (static_cast<uint32_t>(d.slot[j]) == (IN_PROV | l)) {
                    d.slot[j] = (id + 1ull) | (h >> 32 << 32);
                    break;
                  }
              }
            }
        });
      lap(6);
      // 4. the records, in message order (the rejected ones dropped): a new name's id through its
      //    message's position in idx[] (the position of each message: counted again per range)
      std::vector<uint32_t>* pos = W.pos;
      for (int kk = 0; kk < 4; ++kk) pos[kk].resize(n);
      pool.run(nt, [&](uint32_t t) {  // (each message's position in idx[kk], by its own range)
        for (int kk = 0; kk < 4; ++kk)
          for (uint32_t sh = 0; sh < NS; ++sh) {
            // (the thread's messages of shard sh sit at [c0, c1) of the bucket, in message order)
            const uint32_t c1 = cnt[(static_cast<size_t>(t) * 4 + kk) * NS + sh];
            const uint32_t c0 = t == 0 ? start[kk][sh] : cnt[(static_cast<size_t>(t - 1) * 4 + kk) * NS + sh];
            for (uint32_t r = c0; r < c1; ++r) pos[kk][idx[kk][r]] = r;
          }
      });
      lap(7);
      std::vector<uint32_t>& kbase = W.kbase;
      kbase.assign(nt + 1, 0);
      for (uint32_t t = 0; t < nt; ++t) {
        const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
        uint32_t c = 0;
        for (size_t i = i0; i < i1; ++i) c += pre[i].kind == 1 ? 0u : 1u;
        kbase[t + 1] = kbase[t] + c;
      }
      auto id_of = [&](size_t i, int kk) -> uint32_t {
        const uint32_t x = ref[kk][i];
        if (x) return x - 1;
        const uint32_t v = nref[kk][pos[kk][i]];
        return nm->in[kk].sh[in_shard(hash_of(pre[i], kk))].fresh_id[v & ~IN_PROV];
      };
      std::vector<gome_consume_stats>& ps = W.ps;
      ps.assign(nt, gome_consume_stats{});
      pool.run(nt, [&](uint32_t t) {
        const size_t i0 = n * t / nt, i1 = n * (t + 1) / nt;
        gome_consume_stats c{};  // (the thread's own: ps[] entries share cache lines)
        size_t kk = kbase[t];
        for (size_t i = i0; i < i1; ++i) {
          const Dec& d = dec[i];
          const ConsumePre& q = pre[i];
          c.not_objects += d.is_object ? 0 : 1;
          if (q.kind == 0) {  // DoOrder ignores it (engine.go:46-54): a zero record
            out[kk] = gome_order{};
            if (msg_index) msg_index[kk] = static_cast<uint32_t>(i);
            ++kk;
            ++c.ignored;
            continue;
          }
          if (q.kind == 1) {  // outside the engine's domain: not submitted (its marker was consumed)
            ++c.rejected;
            continue;
          }
          gome_order& r = out[kk];
          r = gome_order{};
          r.price_fx = q.p;
          r.volume_fx = q.v;
          r.symbol_id = id_of(i, 0);
          r.uuid_id = id_of(i, 1);
          r.oid_id = id_of(i, 2);
          r.side = static_cast<uint8_t>(d.tx);
          r.action = static_cast<uint8_t>(d.action);
          if (d.action == GOME_ADD) {
            const uint8_t ok = adm[pos[3][i]];
            c.admitted += ok;
            r.flags = static_cast<uint16_t>(GOME_ORD_ADM_HOST | (ok ? GOME_ORD_ADMITTED : 0));
          } else {
            r.flags = GOME_ORD_ADM_HOST;
          }
          if (msg_index) msg_index[kk] = static_cast<uint32_t>(i);
          ++kk;
        }
        ps[t] = c;
      });
      lap(8);
      for (Interner& in : nm->in)
        for (Interner::Shard& d : in.sh) d.fresh.clear();
      for (const gome_consume_stats& c : ps) {
        s.not_objects += c.not_objects;
        s.ignored += c.ignored;
        s.rejected += c.rejected;
        s.admitted += c.admitted;
      }
      k = kbase[nt];
    }
  }
  if (!parallel) {
    // The serial pass: one message after another, bound by its table probes' cache misses (the oid
    // and marker tables hold millions of keys), so it prefetches the slots PF messages ahead.
    constexpr size_t PF = 16;  // messages of prefetch distance
    std::vector<std::unique_lock<std::mutex>> locks;  // (every marker shard, in shard order, once for the batch)
    locks.reserve(PP_SHARDS);
    for (PPShard& d : pp->sh) locks.emplace_back(d.mu);
    for (size_t i = 0; i < n; ++i) {
      if (i + PF < n && pre[i + PF].kind != 0) {
        const ConsumePre& q = pre[i + PF];
        nm->in[0].prefetch(q.hs);
        nm->in[1].prefetch(q.hu);
        nm->in[2].prefetch(q.ho);
        pp->of(q.hk).prefetch(q.hk);
      }
      if (i + PF / 2 < n && pre[i + PF / 2].kind != 0) {  // (the strings and keys its probes compare)
        const ConsumePre& q = pre[i + PF / 2];
        nm->in[0].prefetch2(q.hs);
        nm->in[1].prefetch2(q.hu);
        nm->in[2].prefetch2(q.ho);
        pp->of(q.hk).prefetch2(q.hk);
      }
      const Dec& d = dec[i];
      s.not_objects += d.is_object ? 0 : 1;
      const ConsumePre& q = pre[i];
      if (q.kind == 0) {  // DoOrder ignores it (engine.go:46-54): a zero record
        out[k] = gome_order{};
        if (msg_index) msg_index[k] = static_cast<uint32_t>(i);
        ++k;
        ++s.ignored;
        continue;
      }
      const char* sym = str_ptr(d.s[2], arenas);
      const char* uuid = str_ptr(d.s[0], arenas);
      const char* oid = str_ptr(d.s[1], arenas);
      const size_t sl = d.s[2].len, ul = d.s[0].len, ol = d.s[1].len;
      bool bad = q.kind == 1;
      if (!bad && max_symbols) {
        const int64_t sid = nm->in[0].find(sym ? sym : "", sl, q.hs);
        const uint64_t would = sid >= 0 ? static_cast<uint64_t>(sid) : nm->in[0].strs.size();
        bad = would >= max_symbols;
      }
      int32_t code = 0;
      if (!bad) {
        code = nm->tx_code(d.tx);
        bad = code < 0;
      }
      const char* key = karena[q.ka].data() + q.koff;
      PPShard& ps = pp->of(q.hk);
      if (bad) {  // outside the engine's domain: not submitted (its marker is consumed as DoOrder would)
        ++s.rejected;
        ps.stage_locked(key, q.klen, q.hk);
        continue;
      }
      gome_order& r = out[k];
      r = gome_order{};
      r.price_fx = q.p;
      r.volume_fx = q.v;
      r.symbol_id = nm->in[0].intern_h(sym ? sym : "", sl, q.hs);
      r.uuid_id = nm->in[1].intern_h(uuid ? uuid : "", ul, q.hu);
      r.oid_id = nm->in[2].intern_h(oid ? oid : "", ol, q.ho);
      r.side = static_cast<uint8_t>(code);
      r.action = static_cast<uint8_t>(d.action);
      if (d.action == GOME_ADD) {
        const bool ok = ps.stage_locked(key, q.klen, q.hk);
        s.admitted += ok ? 1 : 0;
        r.flags = static_cast<uint16_t>(GOME_ORD_ADM_HOST | (ok ? GOME_ORD_ADMITTED : 0));
      } else {
        ps.stage_locked(key, q.klen, q.hk);
        r.flags = GOME_ORD_ADM_HOST;
      }
      if (msg_index) msg_index[k] = static_cast<uint32_t>(i);
      ++k;
    }
  }
  if (parallel) lap(9);
  else for (uint64_t& x : W.step_ns) x = 0;  // (a batch that fell back to the serial pass)
  s.records = k;
  s.queue_parallel = parallel ? 1 : 0;
  s.ns_decode = ns(t0, t1);
  s.ns_prepare = ns(t1, t2);
  s.ns_queue = ns(t2, clk::now());
  *n_out = k;
  if (st) *st = s;
  return GOME_OK;
}

}  // extern "C"
