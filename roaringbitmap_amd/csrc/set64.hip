// set64.hip — the 64-bit front end (longlong/): Roaring64NavigableMap and Roaring64Bitmap over the
// 32-bit engine.
//
// A 64-bit bitmap is a list of buckets (high 32 bits, 32-bit RoaringBitmap of the low halves), in
// ascending unsigned order of the highs — Roaring64NavigableMap's own structure (highToBitmap) and
// Roaring64Bitmap's 48-bit ART keys grouped by their high 32 bits.  An rbgpu_set64 keeps every bucket's
// 32-bit bitmap in one device set and a host directory (per 64-bit bitmap: its buckets' highs and set
// indices).  A batch of 64-bit ops is one batched 32-bit pairwise call over the buckets: the host merges
// each pair's bucket lists by high and emits one bucket pair per result bucket — matched buckets
// (x1's, x2's), a bucket of one side against RB_EMPTY_BITMAP where the op keeps it (its containers
// come out as clones) — so the container algebra, the 16-bit key alignment and the result types are
// the 32-bit path's.  What differs between the two 64-bit classes is which buckets survive and how
// empty results are treated (see rbgpu.h, rb64_flavor).
#include <algorithm>
#include <cstring>
#include <vector>

#include "internal.hpp"

using namespace rbg;

struct rbgpu_set64 {
  rbgpu_ctx *ctx = nullptr;
  rbgpu_set *buckets = nullptr;   // owned: the buckets' 32-bit bitmaps
  std::vector<uint64_t> begin;    // [n + 1] CSR of each 64-bit bitmap's directory entries
  std::vector<uint32_t> high;     // per entry: the high 32 bits
  std::vector<uint32_t> idx;      // per entry: its bitmap in `buckets`
  std::vector<uint8_t> sgn;       // per bitmap: Roaring64NavigableMap signedLongs (the legacy format's
                                  // bucket order); the directory itself is always in unsigned order
  uint32_t n() const { return (uint32_t)(begin.size() - 1); }
  bool signed_longs(uint32_t i) const { return i < sgn.size() && sgn[i]; }
};

namespace {

uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
uint16_t rd16(const uint8_t *p) {
  uint16_t v;
  std::memcpy(&v, p, 2);
  return v;
}

// Byte length of the 32-bit RoaringFormatSpec bitmap at p (RoaringArray.deserialize's layout,
// RoaringArray.java:276-348), or 0 when it does not fit in `avail` bytes or the cookie is unknown.
uint64_t blob_len(const uint8_t *p, uint64_t avail) {
  if (avail < 4) return 0;
  const uint32_t cookie = rd32(p);
  uint64_t pos = 4, n;
  bool hasrun;
  if ((cookie & 0xFFFF) == 12347) {
    hasrun = true;
    n = (cookie >> 16) + 1ull;
  } else if (cookie == 12346) {
    hasrun = false;
    if (avail < 8) return 0;
    n = rd32(p + 4);
    pos = 8;
  } else {
    return 0;
  }
  if (n > 65536) return 0;
  const uint64_t runbits = hasrun ? pos : 0;
  if (hasrun) pos += (n + 7) / 8;
  const uint64_t pairs = pos;
  pos += 4 * n;
  if (!hasrun || n >= 4) pos += 4 * n;
  if (pos > avail) return 0;
  for (uint64_t i = 0; i < n; ++i) {
    const bool run = hasrun && ((p[runbits + i / 8] >> (i % 8)) & 1);
    if (run) {
      if (pos + 2 > avail) return 0;
      pos += 2 + 4ull * rd16(p + pos);
    } else {
      const uint64_t card = rd16(p + pairs + 4 * i + 2) + 1ull;
      pos += card <= 4096 ? 2 * card : 8192;
    }
    if (pos > avail) return 0;
  }
  return pos;
}

rbgpu_set *empty_set(rbgpu_ctx *ctx) {
  rbgpu_set *s = new rbgpu_set;
  if (set_alloc(ctx, s, 0, 0, 16)) {
    delete s;
    return nullptr;
  }
  const uint64_t z = 0;
  if (hipMemcpy(s->begin, &z, 8, hipMemcpyHostToDevice) != hipSuccess) {
    rbgpu_set_free(s);
    return nullptr;
  }
  s->h_begin = {0};
  return s;
}

uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
void put_be32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

// The directory entries of 64-bit bitmap i in the bucket order its map iterates: unsigned highs, or
// for a signedLongs Roaring64NavigableMap the highs as signed ints (negative ones first).
std::vector<uint64_t> map_order(const rbgpu_set64 *s, uint32_t i) {
  std::vector<uint64_t> e;
  for (uint64_t k = s->begin[i]; k < s->begin[i + 1]; ++k) e.push_back(k);
  if (s->signed_longs(i))
    std::stable_partition(e.begin(), e.end(), [&](uint64_t k) { return (int32_t)s->high[k] < 0; });
  return e;
}

// Per 64-bit pair, the bucket pairs of a static / in-place op (the merge of the two bucket lists by
// high): matched buckets, and a bucket of one side against RB_EMPTY_BITMAP where the op keeps it.
struct BucketPairs {
  std::vector<uint32_t> pa, pb, hi;
  std::vector<uint8_t> keep; // keep the result bucket even when it holds no container
  std::vector<uint64_t> obegin{0};
};
int bucket_pairs(const rbgpu_set64 *a, const rbgpu_set64 *b, int op, bool inplace, bool nav, const uint32_t *a_idx,
                 const uint32_t *b_idx, uint32_t npairs, BucketPairs &bp) {
  const bool same_set = a == b;
  for (uint32_t p = 0; p < npairs; ++p) {
    const uint32_t ai = a_idx ? a_idx[p] : p, bi = b_idx ? b_idx[p] : p;
    if (ai >= a->n() || bi >= b->n()) return fail(RB_EINVAL, "pair %u: index out of range", p);
    const uint64_t i1 = a->begin[ai + 1], j1 = b->begin[bi + 1];
    uint64_t i = a->begin[ai], j = b->begin[bi];
    if (inplace && same_set && ai == bi) {
      // x1.op(x1): `if (x2 == this)` return (and, or) / clear() (xor, andNot) — each bucket with itself
      // in the in-place 32-bit call takes the same branch; a cleared bucket goes
      if (op == RB_AND || op == RB_OR)
        for (; i < i1; ++i)
          bp.pa.push_back(a->idx[i]), bp.pb.push_back(a->idx[i]), bp.hi.push_back(a->high[i]), bp.keep.push_back(nav);
      bp.obegin.push_back(bp.pa.size());
      continue;
    }
    while (i < i1 || j < j1) {
      const bool take_a = j == j1 || (i < i1 && a->high[i] < b->high[j]);
      const bool take_b = i == i1 || (j < j1 && b->high[j] < a->high[i]);
      if (!take_a && !take_b) { // matched bucket: the op per 48-bit key / the 32-bit in-place op
        bp.pa.push_back(a->idx[i]), bp.pb.push_back(b->idx[j]), bp.hi.push_back(a->high[i]), bp.keep.push_back(nav);
        ++i, ++j;
      } else if (take_a) {      // x1's bucket alone: removed by and, otherwise kept (cloned)
        if (op != RB_AND)
          bp.pa.push_back(a->idx[i]), bp.pb.push_back(kEmptyBitmap), bp.hi.push_back(a->high[i]), bp.keep.push_back(nav);
        ++i;
      } else {                  // x2's bucket alone: cloned in by or / xor
        if (op == RB_OR || op == RB_XOR)
          bp.pa.push_back(kEmptyBitmap), bp.pb.push_back(b->idx[j]), bp.hi.push_back(b->high[j]), bp.keep.push_back(nav);
        ++j;
      }
    }
    bp.obegin.push_back(bp.pa.size());
  }
  if (bp.pa.size() >= kEmptyBitmap) return fail(RB_EINVAL, "too many result buckets");
  return RB_OK;
}

} // namespace

extern "C" {

int rbgpu_set64_from_portable(rbgpu_ctx *ctx, const uint8_t *const *bufs, const uint64_t *lens, uint32_t n,
                              rbgpu_set64 **out) {
  if (!ctx || !out || (n && (!bufs || !lens))) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  std::vector<const uint8_t *> blobs;
  std::vector<uint64_t> blens;
  rbgpu_set64 *s = new rbgpu_set64;
  s->ctx = ctx;
  s->begin.push_back(0);
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *p = bufs[i];
    const uint64_t len = lens[i];
    // Roaring64NavigableMap.deserializePortable: u64 bucket count, then (u32 high, RoaringBitmap) each
    if (len < 8 || (!p && len)) {
      delete s;
      return fail(RB_EFORMAT, "64-bit bitmap %u: truncated", i);
    }
    uint64_t nb;
    std::memcpy(&nb, p, 8);
    uint64_t pos = 8;
    for (uint64_t k = 0; k < nb; ++k) {
      if (pos + 4 > len) {
        delete s;
        return fail(RB_EFORMAT, "64-bit bitmap %u: truncated bucket %llu", i, (unsigned long long)k);
      }
      const uint32_t h = rd32(p + pos);
      pos += 4;
      const uint64_t bl = blob_len(p + pos, len - pos);
      if (!bl) {
        delete s;
        return fail(RB_EFORMAT, "64-bit bitmap %u: bucket %llu is not a RoaringBitmap", i, (unsigned long long)k);
      }
      if (s->high.size() > s->begin.back() && h <= s->high.back()) {
        delete s;
        return fail(RB_EINVAL, "64-bit bitmap %u: bucket highs not strictly increasing", i);
      }
      s->high.push_back(h);
      s->idx.push_back((uint32_t)blobs.size());
      blobs.push_back(p + pos);
      blens.push_back(bl);
      pos += bl;
    }
    if (pos != len) {
      delete s;
      return fail(RB_EFORMAT, "64-bit bitmap %u: %llu trailing bytes", i, (unsigned long long)(len - pos));
    }
    s->begin.push_back(s->high.size());
  }
  if (blobs.size() >= kEmptyBitmap) {
    delete s;
    return fail(RB_EINVAL, "too many buckets");
  }
  int rc = blobs.empty() ? ((s->buckets = empty_set(ctx)) ? RB_OK : fail(RB_ENOMEM, "empty bucket set"))
                         : rbgpu_set_from_serialized(ctx, blobs.data(), blens.data(), (uint32_t)blobs.size(),
                                                     &s->buckets);
  if (rc) {
    delete s;
    return rc;
  }
  *out = s;
  return RB_OK;
}

int rbgpu_set64_from_buckets(const rbgpu_set *buckets, const uint32_t *highs, const uint64_t *begin, uint32_t n,
                             rbgpu_set64 **out) {
  SETTLE(buckets);
  if (!buckets || !out || !begin || (begin[n] && !highs)) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  if (begin[0] != 0 || begin[n] != buckets->nb) return fail(RB_EINVAL, "begin must cover the bucket set");
  for (uint32_t i = 0; i < n; ++i) {
    if (begin[i + 1] < begin[i]) return fail(RB_EINVAL, "begin must be non-decreasing");
    for (uint64_t k = begin[i] + 1; k < begin[i + 1]; ++k)
      if (highs[k] <= highs[k - 1]) return fail(RB_EINVAL, "64-bit bitmap %u: bucket highs not strictly increasing", i);
  }
  rbgpu_set64 *s = new rbgpu_set64;
  s->ctx = buckets->ctx;
  s->begin.assign(begin, begin + n + 1);
  s->high.assign(highs, highs + begin[n]);
  s->idx.resize(begin[n]);
  for (uint64_t k = 0; k < begin[n]; ++k) s->idx[k] = (uint32_t)k;
  const int rc = buckets->nb ? rbgpu_set_extract(buckets, 0, buckets->nb, &s->buckets)
                             : ((s->buckets = empty_set(buckets->ctx)) ? RB_OK : fail(RB_ENOMEM, "empty set"));
  if (rc) {
    delete s;
    return rc;
  }
  *out = s;
  return RB_OK;
}

void rbgpu_set64_free(rbgpu_set64 *s) {
  if (!s) return;
  rbgpu_set_free(s->buckets);
  delete s;
}

uint32_t rbgpu_set64_bitmap_count(const rbgpu_set64 *s) { return s ? s->n() : 0; }

int rbgpu_set64_buckets(const rbgpu_set64 *s, uint32_t i, uint32_t *highs, uint64_t cap, uint64_t *count) {
  if (!s || !count) return fail(RB_EINVAL, "null argument");
  if (i >= s->n()) return fail(RB_EINVAL, "bitmap %u out of range", i);
  const uint64_t lo = s->begin[i], k = s->begin[i + 1] - lo;
  *count = k;
  if (highs) std::copy(s->high.begin() + lo, s->high.begin() + lo + std::min(k, cap), highs);
  return RB_OK;
}

int rbgpu_set64_bucket_set(const rbgpu_set64 *s, uint32_t i, rbgpu_set **out) {
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  if (i >= s->n()) return fail(RB_EINVAL, "bitmap %u out of range", i);
  const std::vector<uint32_t> idx(s->idx.begin() + s->begin[i], s->idx.begin() + s->begin[i + 1]);
  if (idx.empty()) return (*out = empty_set(s->ctx)) ? RB_OK : fail(RB_ENOMEM, "empty set");
  return set_gather(s->buckets, idx.data(), (uint32_t)idx.size(), out);
}

int rbgpu_set64_extract(const rbgpu_set64 *s, uint32_t first, uint32_t count, rbgpu_set64 **out) {
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  if ((uint64_t)first + count > s->n()) return fail(RB_EINVAL, "bitmap range out of bounds");
  rbgpu_set64 *r = new rbgpu_set64;
  r->ctx = s->ctx;
  r->begin.push_back(0);
  for (uint32_t i = first; i < first + count; ++i) {
    for (uint64_t k = s->begin[i]; k < s->begin[i + 1]; ++k) {
      r->high.push_back(s->high[k]);
      r->idx.push_back((uint32_t)r->idx.size());
    }
    r->begin.push_back(r->high.size());
    r->sgn.push_back(s->signed_longs(i));
  }
  const std::vector<uint32_t> idx(s->idx.begin() + s->begin[first], s->idx.begin() + s->begin[first + count]);
  const int rc = idx.empty() ? ((r->buckets = empty_set(s->ctx)) ? RB_OK : fail(RB_ENOMEM, "empty set"))
                             : set_gather(s->buckets, idx.data(), (uint32_t)idx.size(), &r->buckets);
  if (rc) {
    delete r;
    return rc;
  }
  *out = r;
  return RB_OK;
}

int rbgpu_set64_cardinalities(const rbgpu_set64 *s, uint64_t *out) {
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  std::vector<uint64_t> c(std::max<uint32_t>(s->buckets->nb, 1));
  if (s->buckets->nb) {
    const int rc = rbgpu_set_cardinalities(s->buckets, c.data());
    if (rc) return rc;
  }
  for (uint32_t i = 0; i < s->n(); ++i) {
    out[i] = 0;
    for (uint64_t k = s->begin[i]; k < s->begin[i + 1]; ++k) out[i] += c[s->idx[k]];
  }
  return RB_OK;
}

int rbgpu_set64_portable_sizes(const rbgpu_set64 *s, uint64_t *out) {
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  std::vector<uint64_t> z(std::max<uint32_t>(s->buckets->nb, 1));
  if (s->buckets->nb) {
    const int rc = rbgpu_set_serialized_sizes(s->buckets, z.data());
    if (rc) return rc;
  }
  for (uint32_t i = 0; i < s->n(); ++i) {
    out[i] = 8;
    for (uint64_t k = s->begin[i]; k < s->begin[i + 1]; ++k) out[i] += 4 + z[s->idx[k]];
  }
  return RB_OK;
}

int rbgpu_set64_serialize_portable(const rbgpu_set64 *s, uint32_t first, uint32_t count, uint8_t *dst, uint64_t cap,
                                   uint64_t *offsets) {
  if (!s || (count && !dst)) return fail(RB_EINVAL, "null argument");
  if ((uint64_t)first + count > s->n()) return fail(RB_EINVAL, "bitmap range out of bounds");
  const uint32_t nb = s->buckets->nb;
  std::vector<uint64_t> boff(nb + 1, 0), z(std::max<uint32_t>(nb, 1));
  std::vector<uint8_t> bytes;
  if (nb) {
    int rc = rbgpu_set_serialized_sizes(s->buckets, z.data());
    if (rc) return rc;
    uint64_t tot = 0;
    for (uint32_t k = 0; k < nb; ++k) tot += z[k];
    bytes.resize(std::max<uint64_t>(tot, 1));
    rc = rbgpu_set_serialize(s->buckets, 0, nb, bytes.data(), tot, boff.data());
    if (rc) return rc;
  }
  uint64_t pos = 0;
  for (uint32_t i = first; i < first + count; ++i) {
    uint64_t need = 8;
    for (uint64_t k = s->begin[i]; k < s->begin[i + 1]; ++k) need += 4 + z[s->idx[k]];
    if (pos + need > cap) return fail(RB_EINVAL, "destination buffer too small (%llu needed)", (unsigned long long)(pos + need));
    if (offsets) offsets[i - first] = pos;
    const uint64_t nk = s->begin[i + 1] - s->begin[i];
    std::memcpy(dst + pos, &nk, 8); // Roaring64NavigableMap.serializePortable (:1254-1261), little endian
    pos += 8;
    for (uint64_t k : map_order(s, i)) { // the map's own iteration order (signed highs first if signedLongs)
      std::memcpy(dst + pos, &s->high[k], 4);
      pos += 4;
      const uint32_t b = s->idx[k];
      std::memcpy(dst + pos, bytes.data() + boff[b], z[b]);
      pos += z[b];
    }
  }
  if (offsets) offsets[count] = pos;
  return RB_OK;
}

int rbgpu_pairwise64(rbgpu_ctx *ctx, int flavor, int op, int inplace, const rbgpu_set64 *a, const rbgpu_set64 *b,
                     const uint32_t *a_idx, const uint32_t *b_idx, uint32_t npairs, rbgpu_set64 **out) {
  if (!ctx || !a || !b || !out) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  if (op < RB_AND || op > RB_ANDNOT) return fail(RB_EINVAL, "bad op %d", op);
  if (flavor != RB64_BITMAP && flavor != RB64_NAVIGABLE) return fail(RB_EINVAL, "bad 64-bit flavor %d", flavor);
  if (flavor == RB64_NAVIGABLE && !inplace)
    return fail(RB_EINVAL, "Roaring64NavigableMap has in-place and/or/xor/andNot only");
  if (a->ctx != ctx || b->ctx != ctx) return fail(RB_EINVAL, "sets belong to another context");
  const bool nav = flavor == RB64_NAVIGABLE;
  BucketPairs bp;
  int rc = bucket_pairs(a, b, op, inplace != 0, nav, a_idx, b_idx, npairs, bp);
  if (rc) return rc;
  const std::vector<uint32_t> &pa = bp.pa, &pb = bp.pb, &hi = bp.hi;
  const std::vector<uint8_t> &keep = bp.keep;
  const std::vector<uint64_t> &obegin = bp.obegin;
  rbgpu_set *res = nullptr;
  if (pa.empty()) {
    res = empty_set(ctx);
    rc = res ? RB_OK : fail(RB_ENOMEM, "empty bucket set");
  } else {
    // Roaring64Bitmap keeps empty xor results (no isEmpty check, Roaring64Bitmap.java:392-460);
    // Roaring64NavigableMap's buckets are RoaringBitmaps, whose xor drops them (RoaringBitmap.java:3296-3348)
    rc = pairwise_call(ctx, op, a->buckets, b->buckets, pa.data(), pb.data(), (uint32_t)pa.size(), &res,
                       inplace != 0, !nav && op == RB_XOR);
    if (!rc) rc = ensure_h_begin(res);
  }
  if (rc) {
    rbgpu_set_free(res);
    return rc;
  }
  rbgpu_set64 *r = new rbgpu_set64;
  r->ctx = ctx;
  r->buckets = res;
  r->begin.push_back(0);
  for (uint32_t p = 0; p < npairs; ++p) {
    // an in-place result is x1's map: it keeps x1's signedLongs
    r->sgn.push_back(inplace && nav ? (uint8_t)a->signed_longs(a_idx ? a_idx[p] : p) : 0);
    for (uint64_t k = obegin[p]; k < obegin[p + 1]; ++k) {
      // Roaring64Bitmap: a bucket exists while it holds a (possibly empty) container; a
      // Roaring64NavigableMap bucket stays even when its RoaringBitmap is empty
      if (keep[k] || res->h_begin[k + 1] > res->h_begin[k]) {
        r->high.push_back(hi[k]);
        r->idx.push_back((uint32_t)k);
      }
    }
    r->begin.push_back(r->high.size());
  }
  *out = r;
  return RB_OK;
}

int rbgpu_pairwise64_cardinality(rbgpu_ctx *ctx, int op, const rbgpu_set64 *a, const rbgpu_set64 *b,
                                 const uint32_t *a_idx, const uint32_t *b_idx, uint32_t npairs, uint64_t *out) {
  if (!ctx || !a || !b || (npairs && !out)) return fail(RB_EINVAL, "null argument");
  if (op < RB_AND || op > RB_ANDNOT) return fail(RB_EINVAL, "bad op %d", op);
  if (a->ctx != ctx || b->ctx != ctx) return fail(RB_EINVAL, "sets belong to another context");
  BucketPairs bp;
  int rc = bucket_pairs(a, b, op, false, false, a_idx, b_idx, npairs, bp);
  if (rc) return rc;
  std::vector<uint64_t> c(std::max<size_t>(bp.pa.size(), 1), 0);
  if (!bp.pa.empty()) {
    rc = rbgpu_pairwise_cardinality(ctx, op, a->buckets, b->buckets, bp.pa.data(), bp.pb.data(),
                                    (uint32_t)bp.pa.size(), c.data());
    if (rc) return rc;
  }
  for (uint32_t p = 0; p < npairs; ++p) {
    out[p] = 0;
    for (uint64_t k = bp.obegin[p]; k < bp.obegin[p + 1]; ++k) out[p] += c[k];
  }
  return RB_OK;
}

int rbgpu_set64_from_legacy(rbgpu_ctx *ctx, const uint8_t *const *bufs, const uint64_t *lens, uint32_t n,
                            rbgpu_set64 **out) {
  if (!ctx || !out || (n && (!bufs || !lens))) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  std::vector<const uint8_t *> blobs;
  std::vector<uint64_t> blens;
  rbgpu_set64 *s = new rbgpu_set64;
  s->ctx = ctx;
  s->begin.push_back(0);
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *p = bufs[i];
    const uint64_t len = lens[i];
    // Roaring64NavigableMap.serializeLegacy (:1229-1240): boolean signedLongs, int bucket count, then
    // (int high, RoaringBitmap) each — DataOutput ints are big-endian, the RoaringBitmaps little-endian
    if (len < 5 || !p) {
      delete s;
      return fail(RB_EFORMAT, "64-bit bitmap %u: truncated", i);
    }
    if (p[0] > 1) {
      delete s;
      return fail(RB_EFORMAT, "64-bit bitmap %u: bad signedLongs byte", i);
    }
    const bool sgn = p[0] != 0;
    const uint32_t nb = be32(p + 1);
    uint64_t pos = 5;
    std::vector<std::pair<uint32_t, uint64_t>> ent; // (high, blob index) in the map's order
    for (uint64_t k = 0; k < nb; ++k) {
      if (pos + 4 > len) {
        delete s;
        return fail(RB_EFORMAT, "64-bit bitmap %u: truncated bucket %llu", i, (unsigned long long)k);
      }
      const uint32_t h = be32(p + pos);
      pos += 4;
      const uint64_t bl = blob_len(p + pos, len - pos);
      if (!bl) {
        delete s;
        return fail(RB_EFORMAT, "64-bit bitmap %u: bucket %llu is not a RoaringBitmap", i, (unsigned long long)k);
      }
      // the map's comparator order (signed or unsigned ints), strictly increasing (TreeMap keys)
      if (!ent.empty() && (sgn ? (int32_t)h <= (int32_t)ent.back().first : h <= ent.back().first)) {
        delete s;
        return fail(RB_EINVAL, "64-bit bitmap %u: bucket highs not strictly increasing", i);
      }
      ent.push_back({h, blobs.size()});
      blobs.push_back(p + pos);
      blens.push_back(bl);
      pos += bl;
    }
    if (pos != len) {
      delete s;
      return fail(RB_EFORMAT, "64-bit bitmap %u: %llu trailing bytes", i, (unsigned long long)(len - pos));
    }
    std::stable_sort(ent.begin(), ent.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    for (const auto &e : ent) {
      s->high.push_back(e.first);
      s->idx.push_back((uint32_t)e.second);
    }
    s->begin.push_back(s->high.size());
    s->sgn.push_back(sgn);
  }
  if (blobs.size() >= kEmptyBitmap) {
    delete s;
    return fail(RB_EINVAL, "too many buckets");
  }
  const int rc = blobs.empty() ? ((s->buckets = empty_set(ctx)) ? RB_OK : fail(RB_ENOMEM, "empty bucket set"))
                               : rbgpu_set_from_serialized(ctx, blobs.data(), blens.data(), (uint32_t)blobs.size(),
                                                           &s->buckets);
  if (rc) {
    delete s;
    return rc;
  }
  *out = s;
  return RB_OK;
}

int rbgpu_set64_set_signed_longs(rbgpu_set64 *s, uint32_t i, int signed_longs) {
  if (!s) return fail(RB_EINVAL, "null argument");
  if (i >= s->n()) return fail(RB_EINVAL, "bitmap %u out of range", i);
  s->sgn.resize(s->n(), 0);
  s->sgn[i] = signed_longs != 0;
  return RB_OK;
}

int rbgpu_set64_get_signed_longs(const rbgpu_set64 *s, uint32_t i, int *out) {
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  if (i >= s->n()) return fail(RB_EINVAL, "bitmap %u out of range", i);
  *out = s->signed_longs(i) ? 1 : 0;
  return RB_OK;
}

int rbgpu_set64_legacy_sizes(const rbgpu_set64 *s, uint64_t *out) {
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  const int rc = rbgpu_set64_portable_sizes(s, out); // 8-B count + 4 B per bucket + the buckets
  if (rc) return rc;
  for (uint32_t i = 0; i < s->n(); ++i) out[i] -= 3;  // 1-B flag + 4-B count instead of the 8-B count
  return RB_OK;
}

int rbgpu_set64_serialize_legacy(const rbgpu_set64 *s, uint32_t first, uint32_t count, uint8_t *dst, uint64_t cap,
                                 uint64_t *offsets) {
  if (!s || (count && !dst)) return fail(RB_EINVAL, "null argument");
  if ((uint64_t)first + count > s->n()) return fail(RB_EINVAL, "bitmap range out of bounds");
  const uint32_t nb = s->buckets->nb;
  std::vector<uint64_t> boff(nb + 1, 0), z(std::max<uint32_t>(nb, 1));
  std::vector<uint8_t> bytes;
  if (nb) {
    int rc = rbgpu_set_serialized_sizes(s->buckets, z.data());
    if (rc) return rc;
    uint64_t tot = 0;
    for (uint32_t k = 0; k < nb; ++k) tot += z[k];
    bytes.resize(std::max<uint64_t>(tot, 1));
    rc = rbgpu_set_serialize(s->buckets, 0, nb, bytes.data(), tot, boff.data());
    if (rc) return rc;
  }
  uint64_t pos = 0;
  for (uint32_t i = first; i < first + count; ++i) {
    uint64_t need = 5;
    for (uint64_t k = s->begin[i]; k < s->begin[i + 1]; ++k) need += 4 + z[s->idx[k]];
    if (pos + need > cap) return fail(RB_EINVAL, "destination buffer too small (%llu needed)", (unsigned long long)(pos + need));
    if (offsets) offsets[i - first] = pos;
    dst[pos] = s->signed_longs(i) ? 1 : 0;
    put_be32(dst + pos + 1, (uint32_t)(s->begin[i + 1] - s->begin[i]));
    pos += 5;
    for (uint64_t k : map_order(s, i)) {
      put_be32(dst + pos, s->high[k]);
      pos += 4;
      const uint32_t b = s->idx[k];
      std::memcpy(dst + pos, bytes.data() + boff[b], z[b]);
      pos += z[b];
    }
  }
  if (offsets) offsets[count] = pos;
  return RB_OK;
}

} // extern "C"
