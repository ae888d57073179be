// format.cpp — RoaringFormatSpec (de)serialization on the host, mirroring
// RoaringArray.serialize / deserialize (RoaringArray.java:276-348, 547-629, 781-790, 851-953).
#include "format.hpp"

#include <cstring>

#include "rbgpu.h"

namespace rbg {

namespace {
constexpr uint32_t kCookie = 12347, kCookieNoRun = 12346; // SERIAL_COOKIE(_NO_RUNCONTAINER)
constexpr uint32_t kNoOffsetThreshold = 4;                // RoaringArray.NO_OFFSET_THRESHOLD

struct Cursor {
  const uint8_t *p;
  uint64_t n, pos = 0;
  bool ok = true;
  bool need(uint64_t k) {
    if (pos + k > n) ok = false;
    return ok;
  }
  template <class T> T get() {
    T v{};
    if (!need(sizeof(T))) return v;
    std::memcpy(&v, p + pos, sizeof(T));
    pos += sizeof(T);
    return v;
  }
};
inline uint64_t round16(uint64_t x) { return (x + 15) & ~15ull; }
} // namespace

int validate_container(uint16_t type, uint32_t card, uint32_t nruns, const uint8_t *payload, std::string &err) {
  if (type == RB_ARRAY) {
    if (card < 1 || card > 4096) { err = "array container cardinality out of [1,4096]"; return RB_EINVAL; }
    const uint16_t *v = reinterpret_cast<const uint16_t *>(payload);
    for (uint32_t i = 1; i < card; ++i)
      if (v[i] <= v[i - 1]) { err = "array container values not strictly increasing"; return RB_EINVAL; }
    return RB_OK;
  }
  if (type == RB_BITMAP) {
    const uint64_t *w = reinterpret_cast<const uint64_t *>(payload);
    uint32_t c = 0;
    for (int i = 0; i < 1024; ++i) c += (uint32_t)__builtin_popcountll(w[i]);
    if (c != card) { err = "bitmap container cardinality does not match its popcount"; return RB_EINVAL; }
    if (card <= 4096) { err = "bitmap container with cardinality <= 4096 (non-canonical)"; return RB_EINVAL; }
    return RB_OK;
  }
  if (type == RB_RUN) {
    if (nruns < 1) { err = "empty run container"; return RB_EINVAL; }
    const uint16_t *r = reinterpret_cast<const uint16_t *>(payload);
    int64_t prev_end = -2;
    uint64_t c = 0;
    for (uint32_t i = 0; i < nruns; ++i) {
      int64_t s = r[2 * i], e = s + r[2 * i + 1];
      if (e > 65535) { err = "run exceeds the container"; return RB_EINVAL; }
      if (s <= prev_end + 1) { err = "runs overlap, touch or are unsorted (non-canonical)"; return RB_EINVAL; }
      prev_end = e;
      c += (uint64_t)(e - s + 1);
    }
    if (c != card) { err = "run container cardinality mismatch"; return RB_EINVAL; }
    return RB_OK;
  }
  err = "unknown container type";
  return RB_EINVAL;
}

int parse_serialized(const uint8_t *buf, uint64_t len, HostSoA &out, std::string &err) {
  Cursor c{buf, len};
  const uint32_t cookie = c.get<uint32_t>();
  if (!c.ok) { err = "truncated header"; return RB_EFORMAT; }
  if ((cookie & 0xFFFF) != kCookie && cookie != kCookieNoRun) { err = "I failed to find a valid cookie."; return RB_EFORMAT; }
  const bool hasrun = (cookie & 0xFFFF) == kCookie;
  const uint32_t size = hasrun ? (cookie >> 16) + 1 : c.get<uint32_t>();
  if (!c.ok) { err = "truncated header"; return RB_EFORMAT; }
  if (size > (1u << 16)) { err = "Size too large"; return RB_EFORMAT; }
  std::vector<uint8_t> runmark;
  if (hasrun) {
    const uint64_t nbm = (size + 7) / 8;
    if (!c.need(nbm)) { err = "truncated run marker"; return RB_EFORMAT; }
    runmark.assign(buf + c.pos, buf + c.pos + nbm);
    c.pos += nbm;
  }
  std::vector<uint16_t> keys(size);
  std::vector<uint32_t> cards(size);
  for (uint32_t k = 0; k < size; ++k) {
    keys[k] = c.get<uint16_t>();
    cards[k] = 1u + c.get<uint16_t>();
  }
  if (!c.ok) { err = "truncated key/cardinality table"; return RB_EFORMAT; }
  if (!hasrun || size >= kNoOffsetThreshold) {
    if (!c.need(4ull * size)) { err = "truncated offset table"; return RB_EFORMAT; }
    c.pos += 4ull * size;
  }
  // stage into a temporary so a failure leaves `out` untouched; all format (truncation) errors
  // are reported before any canonical-form check, like the reference which only fails on EOF.
  HostSoA t;
  for (uint32_t k = 0; k < size; ++k) {
    const bool is_run = hasrun && ((runmark[k / 8] >> (k % 8)) & 1);
    const bool is_bitmap = !is_run && cards[k] > 4096;
    uint8_t ty;
    uint32_t nr = 0;
    uint64_t bytes;
    if (is_bitmap) {
      ty = RB_BITMAP;
      bytes = 8192;
    } else if (is_run) {
      ty = RB_RUN;
      nr = c.get<uint16_t>();
      if (!c.ok) { err = "truncated run container"; return RB_EFORMAT; }
      bytes = 4ull * nr;
    } else {
      ty = RB_ARRAY;
      bytes = 2ull * cards[k];
    }
    if (!c.need(bytes)) { err = "truncated container payload"; return RB_EFORMAT; }
    const uint64_t at = t.payload.size();
    t.payload.resize(at + round16(bytes), 0);
    std::memcpy(t.payload.data() + at, buf + c.pos, bytes);
    c.pos += bytes;
    t.key.push_back(keys[k]);
    t.type.push_back(ty);
    t.card.push_back(cards[k]);
    t.nruns.push_back((uint16_t)nr);
    t.off.push_back(at);
  }
  for (uint32_t k = 0; k < size; ++k) {
    if (k > 0 && t.key[k] <= t.key[k - 1]) { err = "container keys not strictly increasing"; return RB_EINVAL; }
    int rc = validate_container(t.type[k], t.card[k], t.nruns[k], t.payload.data() + t.off[k], err);
    if (rc) return rc;
  }
  // append
  const uint64_t base = out.payload.size();
  out.payload.insert(out.payload.end(), t.payload.begin(), t.payload.end());
  for (uint64_t i = 0; i < t.key.size(); ++i) {
    out.key.push_back(t.key[i]);
    out.type.push_back(t.type[i]);
    out.card.push_back(t.card[i]);
    out.nruns.push_back(t.nruns[i]);
    out.off.push_back(base + t.off[i]);
  }
  out.nb += 1;
  out.begin.push_back(out.key.size());
  return RB_OK;
}

static uint64_t container_bytes(const HostSoA &s, uint64_t i) { // Container.getArraySizeInBytes
  switch (s.type[i]) {
  case RB_ARRAY: return 2ull * s.card[i];
  case RB_BITMAP: return 8192;
  default: return 2 + 4ull * s.nruns[i];
  }
}

uint64_t serialized_size(const HostSoA &s, uint32_t b) {
  const uint64_t lo = s.begin[b], hi = s.begin[b + 1], n = hi - lo;
  bool hasrun = false;
  uint64_t bytes = 0;
  for (uint64_t i = lo; i < hi; ++i) {
    hasrun |= s.type[i] == RB_RUN;
    bytes += container_bytes(s, i);
  }
  uint64_t h = hasrun ? (n < kNoOffsetThreshold ? 4 + (n + 7) / 8 + 4 * n : 4 + (n + 7) / 8 + 8 * n) : 8 + 8 * n;
  return h + bytes;
}

void serialize_bitmap(const HostSoA &s, uint32_t b, uint8_t *dst) {
  const uint64_t lo = s.begin[b], hi = s.begin[b + 1];
  const uint32_t n = (uint32_t)(hi - lo);
  bool hasrun = false;
  for (uint64_t i = lo; i < hi; ++i) hasrun |= s.type[i] == RB_RUN;
  uint8_t *p = dst;
  auto w32 = [&](uint32_t v) { std::memcpy(p, &v, 4); p += 4; };
  auto w16 = [&](uint16_t v) { std::memcpy(p, &v, 2); p += 2; };
  uint32_t start;
  if (hasrun) {
    w32(kCookie | ((n - 1) << 16));
    const uint32_t nbm = (n + 7) / 8;
    std::memset(p, 0, nbm);
    for (uint32_t i = 0; i < n; ++i)
      if (s.type[lo + i] == RB_RUN) p[i / 8] |= (uint8_t)(1u << (i % 8));
    p += nbm;
    start = n < kNoOffsetThreshold ? 4 + 4 * n + nbm : 4 + 8 * n + nbm;
  } else {
    w32(kCookieNoRun);
    w32(n);
    start = 4 + 4 + 4 * n + 4 * n;
  }
  for (uint64_t i = lo; i < hi; ++i) {
    w16(s.key[i]);
    w16((uint16_t)(s.card[i] - 1));
  }
  if (!hasrun || n >= kNoOffsetThreshold)
    for (uint64_t i = lo; i < hi; ++i) {
      w32(start);
      start += (uint32_t)container_bytes(s, i);
    }
  for (uint64_t i = lo; i < hi; ++i) {
    const uint8_t *src = s.payload.data() + s.off[i];
    if (s.type[i] == RB_RUN) {
      w16(s.nruns[i]);
      std::memcpy(p, src, 4ull * s.nruns[i]);
      p += 4ull * s.nruns[i];
    } else {
      const uint64_t k = container_bytes(s, i);
      std::memcpy(p, src, k);
      p += k;
    }
  }
}

} // namespace rbg
