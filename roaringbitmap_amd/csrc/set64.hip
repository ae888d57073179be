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
  if (hipMemcpyAsync(s->begin, &z, 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
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

// ---- ART codec (host only; tests/test_art_host.py compiles this part alone)
// Roaring64Bitmap.serialize: HighLowContainer = ART over the 6-byte high keys + Containers
// (longlong/HighLowContainer.java:230-254, art/Art.java:309-391, art/Node*.java, art/Containers.java:210-303).
// Little-endian fields (the writers reverse bytes around DataOutput), node type ordinals NODE4 / NODE16 /
// NODE48 / NODE256 / LEAF_NODE = 0..4.  Parity unpinned: no reference fixture holds this format.
constexpr uint8_t kArtLeaf = 4;
constexpr uint32_t kArtBody[4] = {4, 16, 256, 32}; // Node4 int key, Node16 2 longs, Node48 childIndex, Node256 mask
uint8_t key_byte(uint64_t k48, int d) { return (uint8_t)(k48 >> (8 * (5 - d))); }

// Writes (dst != nullptr) or measures the canonical ART of the ascending keys: the path-compressed radix
// tree with the smallest node type per child count — what inserting the keys with no removal builds
// (Node4 / 16 / 48 grow at their 5th / 17th / 49th child: Node4.java:90-108, Node16.java:140-180,
// Node48.java:180-200) — leaf i holding container index i; Node48 children in slots of key order.
struct ArtOut {
  uint8_t *dst;
  uint64_t pos = 0;
  void put(uint8_t b) {
    if (dst) dst[pos] = b;
    ++pos;
  }
  void put_le(uint64_t v, int n) {
    for (int i = 0; i < n; ++i) put((uint8_t)(v >> (8 * i)));
  }
};
void art_nodes(const std::vector<uint64_t> &k, size_t lo, size_t hi, int depth, ArtOut &o) {
  if (hi - lo == 1) { // LeafNode (art/LeafNode.java:43-47): header (no prefix), key bytes, container index
    o.put(kArtLeaf);
    o.put_le(0, 2);
    o.put(0);
    for (int d = 0; d < 6; ++d) o.put(key_byte(k[lo], d));
    o.put_le(lo, 8);
    return;
  }
  int p = 0; // the keys' common bytes from `depth`: the node's compressed prefix
  while (depth + p < 6 && key_byte(k[lo], depth + p) == key_byte(k[hi - 1], depth + p)) ++p;
  const int d = depth + p;
  std::vector<size_t> starts;
  for (size_t i = lo; i < hi; ++i)
    if (i == lo || key_byte(k[i], d) != key_byte(k[i - 1], d)) starts.push_back(i);
  const size_t n = starts.size();
  const uint8_t t = n <= 4 ? 0 : n <= 16 ? 1 : n <= 48 ? 2 : 3;
  o.put(t); // Node.serializeHeader (art/Node.java:326-335): type, count (reversed short), prefix length, prefix
  o.put_le(n, 2);
  o.put((uint8_t)p);
  for (int j = 0; j < p; ++j) o.put(key_byte(k[lo], depth + j));
  uint8_t kb[256];
  for (size_t c = 0; c < n; ++c) kb[c] = key_byte(k[starts[c]], d);
  if (t == 0) { // Node4.key: child c's byte at bits (3 - c) * 8, written as reverseBytes
    for (int c = 3; c >= 0; --c) o.put((size_t)c < n ? kb[c] : 0);
  } else if (t == 1) { // Node16.firstV / secondV: bytes 0-7 / 8-15 big-endian, each long reversed
    for (int h = 0; h < 2; ++h)
      for (int c = 7; c >= 0; --c) o.put((size_t)(8 * h + c) < n ? kb[8 * h + c] : 0);
  } else if (t == 2) { // Node48.childIndex: key byte -> child slot (0xFF empty), 8 keys per long, reversed
    uint8_t ci[256];
    std::memset(ci, 0xFF, sizeof ci);
    for (size_t c = 0; c < n; ++c) ci[kb[c]] = (uint8_t)c;
    for (int l = 0; l < 32; ++l)
      for (int j = 7; j >= 0; --j) o.put(ci[8 * l + j]);
  } else { // Node256.bitmapMask: bit k & 63 of long k >> 6, little endian
    uint64_t m[4] = {0, 0, 0, 0};
    for (size_t c = 0; c < n; ++c) m[kb[c] >> 6] |= 1ull << (kb[c] & 63);
    for (int l = 0; l < 4; ++l) o.put_le(m[l], 8);
  }
  for (size_t c = 0; c < n; ++c) art_nodes(k, starts[c], c + 1 < n ? starts[c + 1] : hi, d + 1, o);
}
// Containers.grow from a 1-slot array (ArrayList growth: old + old / 2, at least the count)
uint64_t art_capacity(uint64_t n) {
  uint64_t cap = 1;
  for (uint64_t m = 2; m <= n; ++m)
    if (m > cap) cap = std::max(cap + (cap >> 1), m);
  return cap;
}

// One 64-bit bitmap's containers in ascending 48-bit key order, from the downloaded bucket SoA.
struct ArtView {
  std::vector<uint64_t> key;
  std::vector<uint64_t> cont; // container index in the SoA
};
// Writes (dst) or measures one bitmap's stream.
uint64_t art_stream(const ArtView &v, const rb_soa &soa, uint8_t *dst) {
  ArtOut o{dst};
  if (v.key.empty()) { // HighLowContainer.serialize: EMPTY_TAG
    o.put(0);
    return o.pos;
  }
  o.put(1);
  o.put_le(v.key.size(), 8); // Art.keySize
  art_nodes(v.key, 0, v.key.size(), 0, o);
  const uint64_t n = v.key.size(), cap = art_capacity(n);
  o.put_le(1, 4);  // Containers.serialize: one first-level array,
  o.put(0xFE);     // NOT_TRIMMED_MARK
  o.put_le(cap, 4);
  for (uint64_t j = 0; j < n; ++j) {
    const uint64_t c = v.cont[j];
    const uint8_t ty = soa.type[c];
    o.put(1); // NOT_NULL_MARK, containerType (0 Run, 1 Bitmap, 2 Array), cardinality, writeArray
    o.put(ty == RB_RUN ? 0 : ty == RB_BITMAP ? 1 : 2);
    o.put_le(soa.card[c], 4);
    if (ty == RB_RUN) o.put_le(soa.nruns[c], 2);
    const uint64_t bytes = payload_bytes(ty, soa.card[c], soa.nruns[c]);
    if (dst) std::memcpy(dst + o.pos, soa.payload + soa.offset[c], bytes);
    o.pos += bytes;
  }
  for (uint64_t j = n; j < cap; ++j) o.put(0); // NULL_MARK slots of the grown array
  o.put_le(n, 8);     // containerSize
  o.put_le(0, 4);     // firstLevelIdx
  o.put_le(n - 1, 4); // secondLevelIdx
  return o.pos;
}

// One stream's containers in ascending 48-bit key order (nullptr) or what is wrong with it.  Reads any
// tree shape and container-slot layout: the preorder node walk (art/Art.java:373-391: an internal node's
// `count` children follow it), then the Containers arrays (art/Containers.java:276-303, the type codes of
// instanceContainer :352-378), each leaf's container found by its index.
struct ArtCont {
  uint64_t key; // high 48 bits
  uint8_t t;    // rb_type
  uint32_t card;
  uint16_t nr;
  const uint8_t *payload;
};
const char *art_parse(const uint8_t *p, uint64_t len, std::vector<ArtCont> &out) {
  out.clear();
  if (!p || len < 1) return "truncated";
  if (p[0] > 1) return "bad empty tag";
  if (p[0] == 0) return len == 1 ? nullptr : "trailing bytes after the empty tag"; // EMPTY_TAG
  uint64_t pos = 9; // the tag, Art.keySize
  if (len < pos) return "truncated";
  std::vector<std::pair<uint64_t, uint64_t>> leaves; // (48-bit key, container index)
  uint64_t pending = 1;
  while (pending) {
    --pending;
    if (pos + 4 > len) return "truncated ART node";
    const uint8_t t = p[pos];
    const uint32_t cnt = rd16(p + pos + 1), plen = p[pos + 3];
    pos += 4 + plen;
    if (t == kArtLeaf) {
      if (pos + 14 > len) return "truncated ART leaf";
      uint64_t k = 0, ci;
      for (int d = 0; d < 6; ++d) k = (k << 8) | p[pos + d];
      std::memcpy(&ci, p + pos + 6, 8);
      leaves.push_back({k, ci});
      pos += 14;
    } else {
      if (t > 3) return "bad ART node type";
      if (cnt < 2 || cnt > 256) return "bad ART node child count";
      pos += kArtBody[t];
      pending += cnt;
    }
  }
  if (pos + 4 > len) return "truncated containers";
  const uint32_t nfirst = rd32(p + pos);
  pos += 4;
  std::vector<std::pair<uint64_t, ArtCont>> conts; // (container index, container) in index order
  for (uint32_t f = 0; f < nfirst; ++f) {
    if (pos + 5 > len) return "truncated containers";
    const uint32_t nsecond = rd32(p + pos + 1);
    pos += 5;
    for (uint32_t j = 0; j < nsecond; ++j) {
      if (pos + 1 > len) return "truncated containers";
      const uint8_t tag = p[pos++];
      if (tag == 0) continue; // NULL_MARK
      if (tag != 1 || pos + 5 > len) return "bad container null tag";
      const uint8_t ct = p[pos];
      ArtCont c{};
      c.card = rd32(p + pos + 1);
      pos += 5;
      uint64_t bytes;
      if (ct == 0) { // Run: nbrruns, then (value, length) pairs
        if (pos + 2 > len) return "truncated run container";
        c.t = RB_RUN;
        c.nr = rd16(p + pos);
        pos += 2;
        bytes = 4ull * c.nr;
      } else if (ct == 1) {
        c.t = RB_BITMAP;
        bytes = 8192;
      } else if (ct == 2) {
        c.t = RB_ARRAY;
        if (c.card > 4096) return "array container over 4096 values";
        bytes = 2ull * c.card;
      } else {
        return "bad container type";
      }
      if (pos + bytes > len) return "truncated container payload";
      c.payload = p + pos;
      pos += bytes;
      conts.push_back({((uint64_t)f << 32) | j, c});
    }
  }
  if (pos + 16 != len) return "bad length after the containers";
  std::sort(leaves.begin(), leaves.end());
  for (size_t l = 1; l < leaves.size(); ++l)
    if (leaves[l].first == leaves[l - 1].first) return "duplicate ART key";
  for (const auto &lf : leaves) {
    const auto it = std::lower_bound(conts.begin(), conts.end(), lf.second,
                                     [](const std::pair<uint64_t, ArtCont> &x, uint64_t v) { return x.first < v; });
    if (it == conts.end() || it->first != lf.second) return "ART leaf without a container";
    ArtCont c = it->second;
    c.key = lf.first;
    out.push_back(c);
  }
  return nullptr;
}
// ---- end of the ART codec

ArtView art_view(const rbgpu_set64 *s, uint32_t i, const rb_soa &soa) {
  ArtView v;
  for (uint64_t e = s->begin[i]; e < s->begin[i + 1]; ++e) { // directory: ascending unsigned highs
    const uint32_t b = s->idx[e];
    for (uint64_t c = soa.begin[b]; c < soa.begin[b + 1]; ++c) {
      v.key.push_back(((uint64_t)s->high[e] << 16) | soa.key[c]);
      v.cont.push_back(c);
    }
  }
  return v;
}

// The bucket set downloaded as host SoA (the ART writers need every container's payload).
struct HostBuckets {
  rb_soa soa{};
  std::vector<uint64_t> begin, offset;
  std::vector<uint16_t> key, nruns;
  std::vector<uint8_t> type, payload;
  std::vector<uint32_t> card;
};
int download_buckets(const rbgpu_set64 *s, HostBuckets &h) {
  const rbgpu_set *b = s->buckets;
  h.begin.assign(b->nb + 1, 0);
  h.soa = rb_soa{};
  h.soa.begin = h.begin.data();
  if (!b->nb) return RB_OK;
  int rc = rbgpu_set_download(b, 0, b->nb, &h.soa); // sizes first (key == NULL)
  if (rc) return rc;
  h.key.resize(std::max<uint64_t>(h.soa.n_containers, 1));
  h.type.resize(h.key.size());
  h.card.resize(h.key.size());
  h.nruns.resize(h.key.size());
  h.offset.resize(h.key.size());
  h.payload.resize(std::max<uint64_t>(h.soa.payload_bytes, 16));
  h.soa.key = h.key.data();
  h.soa.type = h.type.data();
  h.soa.card = h.card.data();
  h.soa.nruns = h.nruns.data();
  h.soa.offset = h.offset.data();
  h.soa.payload = h.payload.data();
  return rbgpu_set_download(b, 0, b->nb, &h.soa);
}

} // namespace

extern "C" {

int rbgpu_set64_from_art(rbgpu_ctx *ctx, const uint8_t *const *bufs, const uint64_t *lens, uint32_t n,
                         rbgpu_set64 **out) {
  if (!ctx || !out || (n && (!bufs || !lens))) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  // every bucket's containers into one host SoA, then one upload (rbgpu_set_from_soa validates them)
  std::vector<uint64_t> begin{0}, offset;
  std::vector<uint16_t> key, nruns;
  std::vector<uint8_t> type, payload;
  std::vector<uint32_t> card;
  rbgpu_set64 *s = new rbgpu_set64;
  s->ctx = ctx;
  s->begin.push_back(0);
  auto bad = [&](uint32_t i, const char *what) {
    delete s;
    return fail(RB_EFORMAT, "64-bit bitmap %u: %s", i, what);
  };
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t *p = bufs[i];
    const uint64_t len = lens[i];
    std::vector<ArtCont> conts;
    if (const char *why = art_parse(p, len, conts)) return bad(i, why);
    // buckets: the containers grouped by their high 32 bits.  An empty container (what Roaring64Bitmap.xor
    // leaves under its key) is kept, as Containers.deserialize keeps it (art/Containers.java:276-303): it
    // holds no value, but it is serialized again and later ops see it like any other container
    int64_t cur_high = -1;
    for (const ArtCont &c : conts) {
      if (c.card == 0 && (c.t == RB_BITMAP || (c.t == RB_RUN && c.nr))) return bad(i, "non-canonical empty container");
      const uint32_t high = (uint32_t)(c.key >> 16);
      if ((int64_t)high != cur_high) {
        if (s->idx.size() + 1 >= kEmptyBitmap) return bad(i, "too many buckets");
        s->high.push_back(high);
        s->idx.push_back((uint32_t)(begin.size() - 1));
        begin.push_back(begin.back());
        cur_high = high;
      }
      key.push_back((uint16_t)(c.key & 0xFFFF));
      type.push_back(c.t);
      card.push_back(c.card);
      nruns.push_back(c.t == RB_RUN ? c.nr : 0);
      offset.push_back(payload.size());
      const uint64_t bytes = payload_bytes(c.t, c.card, c.nr);
      payload.insert(payload.end(), c.payload, c.payload + bytes);
      payload.resize((payload.size() + 15) & ~size_t(15));
      ++begin.back();
    }
    s->begin.push_back(s->high.size());
    s->sgn.push_back(0);
  }
  rb_soa soa{(uint32_t)(begin.size() - 1), key.size(), payload.size(), begin.data(), key.data(), type.data(),
             card.data(), nruns.data(), offset.data(), payload.data()};
  const int rc = soa.n_bitmaps ? set_from_soa(ctx, &soa, &s->buckets, true)
                               : ((s->buckets = empty_set(ctx)) ? RB_OK : fail(RB_ENOMEM, "empty bucket set"));
  if (rc) {
    delete s;
    return rc;
  }
  *out = s;
  return RB_OK;
}

int rbgpu_set64_art_sizes(const rbgpu_set64 *s, uint64_t *out) {
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  HostBuckets h;
  const int rc = download_buckets(s, h);
  if (rc) return rc;
  for (uint32_t i = 0; i < s->n(); ++i) out[i] = art_stream(art_view(s, i, h.soa), h.soa, nullptr);
  return RB_OK;
}

int rbgpu_set64_serialize_art(const rbgpu_set64 *s, uint32_t first, uint32_t count, uint8_t *dst, uint64_t cap,
                              uint64_t *offsets) {
  if (!s || (count && !dst)) return fail(RB_EINVAL, "null argument");
  if ((uint64_t)first + count > s->n()) return fail(RB_EINVAL, "bitmap range out of bounds");
  HostBuckets h;
  const int rc = download_buckets(s, h);
  if (rc) return rc;
  uint64_t pos = 0;
  for (uint32_t i = first; i < first + count; ++i) {
    const ArtView v = art_view(s, i, h.soa);
    const uint64_t need = art_stream(v, h.soa, nullptr);
    if (pos + need > cap) return fail(RB_EINVAL, "destination buffer too small (%llu needed)", (unsigned long long)(pos + need));
    if (offsets) offsets[i - first] = pos;
    pos += art_stream(v, h.soa, dst + pos);
  }
  if (offsets) offsets[count] = pos;
  return RB_OK;
}

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
    const bool sgn = p[0] != 0; // DataInput.readBoolean: any non-zero byte is true
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
      ent.push_back({h, blobs.size()});
      blobs.push_back(p + pos);
      blens.push_back(bl);
      pos += bl;
    }
    if (pos != len) {
      delete s;
      return fail(RB_EFORMAT, "64-bit bitmap %u: %llu trailing bytes", i, (unsigned long long)(len - pos));
    }
    // highToBitmap.put(high, bitmap) per entry (:1309-1320): the TreeMap orders the highs whatever the
    // stream's order, and a repeated high keeps the bitmap read last (kept here in unsigned order; the
    // map's signed order is applied on output)
    std::stable_sort(ent.begin(), ent.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
    for (size_t e = 0; e < ent.size(); ++e) {
      if (e + 1 < ent.size() && ent[e + 1].first == ent[e].first) continue; // replaced by a later put
      s->high.push_back(ent[e].first);
      s->idx.push_back((uint32_t)ent[e].second);
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
