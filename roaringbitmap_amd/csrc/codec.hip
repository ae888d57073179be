// codec.hip — RoaringFormatSpec (de)serialization on the device.
//
// The portable format is what the Java side hands over (RoaringBitmap.serialize / deserialize(ByteBuffer),
// RoaringArray.java:547-629 read, 851-940 write, 947-953 size).  Parsing it on the GPU takes the host
// out of the upload path: the serialized bytes go to HBM in one copy and these kernels produce the
// SoA set (Bitmaps first at 8 KiB strides, the rest 16-B aligned — the same layout upload_host builds).
// Writing it on the GPU turns a result set into the exact reference bytes without a host walk.
//
// Parse (n bitmaps at d_in + in_off[b]):
//   k_de_header    one thread per bitmap: cookie, size, header truncation -> count[b]
//   (scan count -> cbase)
//   k_de_table     one wave per bitmap: descriptive header, run markers, payload positions.  The
//                  reference reads payloads back to back and skips the offset table
//                  (RoaringArray.java:596-599); we take the table's positions and verify that every
//                  one equals header + the sizes before it (an induction: then the sequential read
//                  sees the same bytes).  A bitmap that fails the check is walked sequentially by one
//                  lane, which also finds its truncation errors.
//   (scan layout flags -> off)
//   k_de_copy      one wave per container: canonical-form checks (format.cpp validate_container) and
//                  the unaligned -> aligned payload copy.
// Errors land in one 64-bit word by atomicMin over (bitmap << 25 | class << 24 | container << 8 | reason):
// the lowest failing bitmap wins and, inside it, truncation (class 0, RB_EFORMAT) before canonical form
// (class 1, RB_EINVAL), then the lowest container — the order the host parser reports them in.
//
// Serialize (bitmaps [first, first+count) into d_out):
//   k_ser_measure  one wave per bitmap: container payload positions (wave scan), header size, total
//   (scan sizes -> out_off)
//   k_ser_header   one wave per bitmap: header bytes (cookie, run markers, descriptive, offsets)
//   k_ser_payload  one wave per container: [nruns] + payload at an arbitrary byte position
// Output positions are byte-granular, so each wave writes whole aligned dwords inside its range and
// the partial dwords at either end byte by byte (neighbouring ranges never share a written byte).
#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {
namespace {

constexpr uint32_t kCookie = 12347, kCookieNoRun = 12346; // SERIAL_COOKIE(_NO_RUNCONTAINER)
constexpr uint32_t kNoOffsetThreshold = 4;                // RoaringArray.NO_OFFSET_THRESHOLD
constexpr int kWaves = 4;                                 // waves per 256-thread block

enum Reason : uint32_t {
  kOk = 0,
  kTruncHeader,
  kBadCookie,
  kSizeTooLarge,
  kTruncRunMarker,
  kTruncTable,
  kTruncOffsets,
  kTruncRun,
  kTruncPayload,
  kKeysOrder,
  kArrayOrder,
  kBitmapCard,
  kRunEmpty,
  kRunBounds,
  kRunOrder,
  kRunCard,
  kReasons
};
const char *const kReasonText[kReasons] = {"ok",
                                           "truncated header",
                                           "I failed to find a valid cookie.",
                                           "Size too large",
                                           "truncated run marker",
                                           "truncated key/cardinality table",
                                           "truncated offset table",
                                           "truncated run container",
                                           "truncated container payload",
                                           "container keys not strictly increasing",
                                           "array container values not strictly increasing",
                                           "bitmap container cardinality does not match its popcount",
                                           "empty run container",
                                           "run exceeds the container",
                                           "runs overlap, touch or are unsorted (non-canonical)",
                                           "run container cardinality mismatch"};

__device__ __forceinline__ void report(unsigned long long *err, uint64_t b, uint32_t cls, uint32_t k, uint32_t why) {
  atomicMin(err, (unsigned long long)((b << 25) | ((uint64_t)cls << 24) | ((uint64_t)(k & 0xFFFF) << 8) | why));
}

// Input bytes: dwords are read aligned and combined; nothing at or beyond `lim` (the caller's
// readable extent, rounded up to 4) is touched.
struct InBytes {
  const uint8_t *p;
  uint64_t lim;
  __device__ __forceinline__ uint32_t dw(uint64_t a) const { // a multiple of 4
    return a < lim ? *reinterpret_cast<const uint32_t *>(p + a) : 0u;
  }
  __device__ __forceinline__ uint32_t u32(uint64_t pos) const {
    const uint64_t a = pos & ~3ull;
    const uint32_t s = (uint32_t)(pos & 3);
    const uint32_t lo = dw(a);
    return s ? __builtin_amdgcn_alignbyte(dw(a + 4), lo, s) : lo;
  }
  __device__ __forceinline__ uint32_t u16(uint64_t pos) const { return u32(pos) & 0xFFFF; }
  __device__ __forceinline__ uint32_t u8(uint64_t pos) const { return u32(pos) & 0xFF; }
};

struct DeArgs {
  InBytes in;
  const uint64_t *in_off; // [n + 1] bitmap b occupies [in_off[b], in_off[b + 1])
  uint32_t n;
  uint64_t *count;        // [n + 1] containers per bitmap (0 after a header error)
  const uint64_t *cbase;  // [n + 1] exclusive scan of count
  unsigned long long *err;
  uint8_t *bad;           // [n] bitmap has a truncation error: its containers are not copied
  // per container
  uint16_t *key;
  uint8_t *type;
  uint32_t *card;
  uint16_t *nruns;
  uint64_t *src;          // absolute input position of the payload (after a Run's count)
  uint32_t *owner;        // bitmap index
  uint64_t *bigflag, *small;
};

struct Header {
  bool hasrun, offsets;
  uint32_t n;
  uint64_t marks, desc, offtab, first; // positions relative to the bitmap start
};

// RoaringArray.deserialize(ByteBuffer) header, RoaringArray.java:547-590
__device__ __forceinline__ uint32_t parse_header(const InBytes &in, uint64_t base, uint64_t len, Header &h) {
  if (len < 4) return kTruncHeader;
  const uint32_t cookie = in.u32(base);
  if ((cookie & 0xFFFF) != kCookie && cookie != kCookieNoRun) return kBadCookie;
  h.hasrun = (cookie & 0xFFFF) == kCookie;
  uint64_t pos = 4;
  if (h.hasrun) {
    h.n = (cookie >> 16) + 1;
  } else {
    if (len < 8) return kTruncHeader;
    h.n = in.u32(base + 4);
    pos = 8;
  }
  if (h.n > (1u << 16)) return kSizeTooLarge;
  h.marks = pos;
  if (h.hasrun) {
    pos += (h.n + 7) / 8;
    if (pos > len) return kTruncRunMarker;
  }
  h.desc = pos;
  pos += 4ull * h.n;
  if (pos > len) return kTruncTable;
  h.offsets = !h.hasrun || h.n >= kNoOffsetThreshold;
  h.offtab = pos;
  if (h.offsets) {
    pos += 4ull * h.n;
    if (pos > len) return kTruncOffsets;
  }
  h.first = pos;
  return kOk;
}

__global__ __launch_bounds__(256) void k_de_header(DeArgs a) {
  for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < a.n; b += (uint64_t)gridDim.x * 256) {
    const uint64_t base = a.in_off[b], len = a.in_off[b + 1] - base;
    Header h;
    const uint32_t why = parse_header(a.in, base, len, h);
    a.bad[b] = why != kOk;
    a.count[b] = why == kOk ? h.n : 0;
    if (why != kOk) report(a.err, b, 0, 0, why);
  }
}

__device__ __forceinline__ void de_put(const DeArgs &a, uint64_t g, uint32_t b, uint32_t key, int ty, uint32_t card,
                                       uint32_t nr, uint64_t src) {
  a.key[g] = (uint16_t)key;
  a.type[g] = (uint8_t)ty;
  a.card[g] = card;
  a.nruns[g] = (uint16_t)nr;
  a.src[g] = src;
  a.owner[g] = b;
  a.bigflag[g] = ty == kBitmap;
  a.small[g] = ty == kBitmap ? 0 : round16(payload_bytes(ty, card, nr));
}

__global__ __launch_bounds__(256) void k_de_table(DeArgs a) {
  const int lane = lane_id();
  for (uint64_t b = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); b < a.n; b += (uint64_t)gridDim.x * kWaves) {
    if (a.count[b] == 0) continue;
    const uint64_t base = a.in_off[b], len = a.in_off[b + 1] - base, g0 = a.cbase[b];
    Header h;
    parse_header(a.in, base, len, h); // succeeded in k_de_header
    const uint32_t n = h.n;
    // parallel pass: positions from the offset table, verified against the sequential layout
    bool ok = h.offsets;
    uint64_t carry = h.first;
    for (uint32_t k0 = 0; ok && k0 < n; k0 += 64) {
      const uint32_t k = k0 + lane;
      const bool live = k < n;
      uint32_t key = 0, card = 0, nr = 0, size = 0;
      int ty = kArray;
      uint64_t pos = 0;
      bool good = true;
      if (live) {
        const uint32_t d = a.in.u32(base + h.desc + 4ull * k);
        key = d & 0xFFFF;
        card = (d >> 16) + 1;
        const bool run = h.hasrun && ((a.in.u8(base + h.marks + k / 8) >> (k % 8)) & 1);
        ty = run ? kRun : card > kMaxArray ? kBitmap : kArray;
        pos = a.in.u32(base + h.offtab + 4ull * k);
        if (run) {
          good = pos + 2 <= len;
          nr = good ? a.in.u16(base + pos) : 0;
          size = 2 + 4 * nr;
        } else {
          size = ty == kBitmap ? kBitmapBytes : 2 * card;
        }
      }
      const uint32_t incl = wave_scan_u32(size, lane);
      const uint64_t expect = carry + (incl - size);
      good = good && (!live || (pos == expect && expect + size <= len));
      if (__ballot(!good)) {
        ok = false;
        break;
      }
      if (live) {
        de_put(a, g0 + k, (uint32_t)b, key, ty, card, nr, base + pos + (ty == kRun ? 2 : 0));
        if (k > 0 && key <= (a.in.u32(base + h.desc + 4ull * (k - 1)) & 0xFFFF)) report(a.err, b, 1, k, kKeysOrder);
      }
      carry += readlane(incl, 63);
    }
    if (ok) continue;
    // sequential read, exactly as RoaringArray.deserialize does it (RoaringArray.java:600-625)
    if (lane == 0) {
      uint64_t pos = h.first;
      for (uint32_t k = 0; k < n; ++k) {
        const uint32_t d = a.in.u32(base + h.desc + 4ull * k);
        const uint32_t key = d & 0xFFFF, card = (d >> 16) + 1;
        const bool run = h.hasrun && ((a.in.u8(base + h.marks + k / 8) >> (k % 8)) & 1);
        const int ty = run ? kRun : card > kMaxArray ? kBitmap : kArray;
        uint32_t nr = 0;
        uint64_t size;
        if (run) {
          if (pos + 2 > len) {
            report(a.err, b, 0, k, kTruncRun);
            a.bad[b] = 1;
            break;
          }
          nr = a.in.u16(base + pos);
          pos += 2;
          size = 4ull * nr;
        } else {
          size = ty == kBitmap ? kBitmapBytes : 2ull * card;
        }
        if (pos + size > len) {
          report(a.err, b, 0, k, kTruncPayload);
          a.bad[b] = 1;
          break;
        }
        de_put(a, g0 + k, (uint32_t)b, key, ty, card, nr, base + pos);
        if (k > 0 && key <= (a.in.u32(base + h.desc + 4ull * (k - 1)) & 0xFFFF)) report(a.err, b, 1, k, kKeysOrder);
        pos += size;
      }
    }
  }
}

// canonical form (format.cpp validate_container) + copy to the aligned layout
__global__ __launch_bounds__(256) void k_de_copy(DeArgs a, uint64_t nc, const uint64_t *off, uint8_t *payload) {
  const int lane = lane_id();
  for (uint64_t g = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); g < nc; g += (uint64_t)gridDim.x * kWaves) {
    const uint32_t b = a.owner[g];
    if (a.bad[b]) continue;
    const int ty = a.type[g];
    const uint32_t card = a.card[g], nr = a.nruns[g];
    const uint64_t src = a.src[g];
    const uint32_t k = (uint32_t)(g - a.cbase[b]);
    const uint32_t bytes = (uint32_t)payload_bytes(ty, card, nr), padded = (uint32_t)round16(bytes);
    uint32_t *dst = reinterpret_cast<uint32_t *>(payload + off[g]);
    uint32_t pop = 0;
    for (uint32_t j = lane; j < padded / 4; j += 64) {
      uint32_t v = 4 * j < bytes ? a.in.u32(src + 4ull * j) : 0u;
      if (4 * j + 4 > bytes) v &= 4 * j + 2 == bytes ? 0xFFFFu : 0u;
      dst[j] = v;
      pop += __builtin_popcount(v);
    }
    uint32_t why = kOk;
    if (ty == kBitmap) {
      if (wave_sum_u32(pop) != card) why = kBitmapCard;
    } else if (ty == kArray) {
      bool bad = false;
      for (uint32_t i = lane + 1; i < card; i += 64) bad |= a.in.u16(src + 2ull * i) <= a.in.u16(src + 2ull * i - 2);
      if (__ballot(bad)) why = kArrayOrder;
    } else {
      if (nr == 0) {
        why = kRunEmpty;
      } else {
        // the host walk (format.cpp validate_container) stops at the first failing run and checks its
        // bounds before its order: the reason reported is that of the least code 2 * run + (order)
        uint32_t first = 0xFFFFFFFFu;
        uint32_t total = 0;
        for (uint32_t i = lane; i < nr; i += 64) {
          const uint32_t r = a.in.u32(src + 4ull * i), s = r & 0xFFFF, e = s + (r >> 16);
          bool order = false;
          if (i > 0) {
            const uint32_t q = a.in.u32(src + 4ull * (i - 1));
            order = s <= (q & 0xFFFF) + (q >> 16) + 1;
          }
          if (e > 65535) first = min(first, 2 * i);
          else if (order) first = min(first, 2 * i + 1);
          total += (r >> 16) + 1;
        }
        first = ~wave_max_u32(~first);
        if (first != 0xFFFFFFFFu) why = (first & 1) ? kRunOrder : kRunBounds;
        else if (wave_sum_u32(total) != card) why = kRunCard;
      }
    }
    if (why != kOk && lane == 0) report(a.err, b, 1, k, why);
  }
}

// ---------------------------------------------------------------- serialize
struct SerArgs {
  SetView s;
  uint32_t first, count;
  uint64_t *cpos;     // per container (set-global index): payload position relative to the bitmap start
  uint64_t *hdr;      // [count] header bytes | hasrun << 32
  uint64_t *size;     // [count + 1] serialized bytes per bitmap
  const uint64_t *out_off; // [count + 1] exclusive scan of size
  uint8_t *out;
};

__device__ __forceinline__ uint32_t ser_bytes(int ty, uint32_t card, uint32_t nr) { // getArraySizeInBytes
  return ty == kArray ? 2 * card : ty == kBitmap ? kBitmapBytes : 2 + 4 * nr;
}
__device__ __forceinline__ uint64_t header_bytes(bool hasrun, uint64_t n) { // RoaringArray.java:851-870
  return hasrun ? (n < kNoOffsetThreshold ? 4 + (n + 7) / 8 + 4 * n : 4 + (n + 7) / 8 + 8 * n) : 8 + 8 * n;
}

__global__ __launch_bounds__(256) void k_ser_measure(SerArgs a) {
  const int lane = lane_id();
  for (uint64_t i = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); i < a.count; i += (uint64_t)gridDim.x * kWaves) {
    const uint64_t lo = a.s.begin[a.first + i], hi = a.s.begin[a.first + i + 1];
    bool hasrun = false;
    for (uint64_t c = lo + lane; c < hi && !hasrun; c += 64) hasrun = a.s.type[c] == kRun;
    hasrun = __ballot(hasrun) != 0;
    const uint64_t h = header_bytes(hasrun, hi - lo);
    uint64_t carry = h;
    for (uint64_t c0 = lo; c0 < hi; c0 += 64) {
      const uint64_t c = c0 + lane;
      const uint32_t sz = c < hi ? ser_bytes(a.s.type[c], a.s.card[c], a.s.nruns[c]) : 0;
      const uint32_t incl = wave_scan_u32(sz, lane);
      if (c < hi) a.cpos[c] = carry + incl - sz;
      carry += readlane(incl, 63);
    }
    if (lane == 0) {
      a.hdr[i] = h | ((uint64_t)hasrun << 32);
      a.size[i] = carry;
    }
  }
}

// Writes bytes [p, p + len) of `out`; fetch(o) returns content bytes [o, o + 4) little-endian (bytes at
// or beyond len are ignored).  Lanes write the aligned dwords, lanes 0..2 the partial head / tail bytes.
template <class F>
__device__ __forceinline__ void write_stream(uint8_t *out, uint64_t p, uint64_t len, int lane, const F &fetch) {
  const uint64_t end = p + len, a0 = (p + 3) & ~3ull, a1 = end & ~3ull;
  const uint64_t head_end = a0 < end ? a0 : end;
  if (p + lane < head_end) out[p + lane] = (uint8_t)fetch(lane);
  if (a0 < a1) {
    uint32_t *o = reinterpret_cast<uint32_t *>(out);
    for (uint64_t w = a0 / 4 + lane; w < a1 / 4; w += 64) o[w] = fetch(4 * w - p);
  }
  const uint64_t tail = a1 > a0 ? a1 : a0;
  if (tail + lane < end) out[tail + lane] = (uint8_t)fetch(tail + lane - p);
}

__device__ __forceinline__ uint32_t header_byte(const SerArgs &a, uint64_t lo, uint32_t n, bool hasrun, uint64_t j) {
  auto byte_of = [](uint32_t v, uint64_t r) { return (v >> (8 * r)) & 0xFF; };
  const SetView &s = a.s;
  if (j < 4) return byte_of(hasrun ? kCookie | ((n - 1) << 16) : kCookieNoRun, j);
  uint64_t d0;
  if (hasrun) {
    const uint64_t nbm = (n + 7) / 8;
    if (j < 4 + nbm) {
      const uint64_t m = j - 4;
      uint32_t bits = 0;
      for (uint32_t t = 0; t < 8 && 8 * m + t < n; ++t) bits |= (uint32_t)(s.type[lo + 8 * m + t] == kRun) << t;
      return bits;
    }
    d0 = 4 + nbm;
  } else {
    if (j < 8) return byte_of(n, j - 4);
    d0 = 8;
  }
  if (j < d0 + 4ull * n) {
    const uint64_t c = lo + (j - d0) / 4, r = (j - d0) % 4;
    return r < 2 ? byte_of(s.key[c], r) : byte_of(s.card[c] - 1, r - 2);
  }
  const uint64_t o0 = d0 + 4ull * n, c = lo + (j - o0) / 4, r = (j - o0) % 4;
  return byte_of((uint32_t)a.cpos[c], r);
}

__global__ __launch_bounds__(256) void k_ser_header(SerArgs a) {
  const int lane = lane_id();
  for (uint64_t i = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); i < a.count; i += (uint64_t)gridDim.x * kWaves) {
    const uint64_t lo = a.s.begin[a.first + i], n = a.s.begin[a.first + i + 1] - lo;
    const uint64_t h = a.hdr[i] & 0xFFFFFFFFull;
    const bool hasrun = (a.hdr[i] >> 32) != 0;
    write_stream(a.out, a.out_off[i], h, lane, [&](uint64_t o) {
      uint32_t v = 0;
      for (uint32_t t = 0; t < 4 && o + t < h; ++t) v |= header_byte(a, lo, (uint32_t)n, hasrun, o + t) << (8 * t);
      return v;
    });
  }
}

__global__ __launch_bounds__(256) void k_ser_payload(SerArgs a, const uint32_t *owner, uint64_t nc) {
  const int lane = lane_id();
  const uint64_t c_lo = a.s.begin[a.first];
  for (uint64_t q = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); q < nc; q += (uint64_t)gridDim.x * kWaves) {
    const uint64_t c = c_lo + q;
    const uint32_t i = owner[q];
    const int ty = a.s.type[c];
    const uint32_t nr = a.s.nruns[c], bytes = ser_bytes(ty, a.s.card[c], nr);
    const uint32_t npre = ty == kRun ? 2 : 0, plen = bytes - npre, pdw = (uint32_t)round16(plen) / 4;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(a.s.payload + a.s.off[c]);
    // content = [nruns (Run)] ++ payload; dword k of the payload, k = -1 is the prefix
    auto dwk = [&](int64_t k) -> uint32_t { return k < 0 ? nr << 16 : (uint64_t)k < pdw ? src[k] : 0u; };
    write_stream(a.out, a.out_off[i] + a.cpos[c], bytes, lane, [&](uint64_t o) {
      const int64_t qq = (int64_t)o - npre;
      const int64_t k = qq >= 0 ? qq / 4 : -1;
      const uint32_t sh = (uint32_t)(qq - 4 * k);
      const uint32_t lo = dwk(k);
      return sh ? __builtin_amdgcn_alignbyte(dwk(k + 1), lo, sh) : lo;
    });
  }
}

__global__ __launch_bounds__(256) void k_ser_owner(SerArgs a, uint32_t *owner) {
  for (uint64_t i = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); i < a.count; i += (uint64_t)gridDim.x * kWaves) {
    const uint64_t lo = a.s.begin[a.first + i], hi = a.s.begin[a.first + i + 1], base = a.s.begin[a.first];
    for (uint64_t c = lo + lane_id(); c < hi; c += 64) owner[c - base] = (uint32_t)i;
  }
}

uint32_t grid_for(uint64_t waves) { return (uint32_t)std::min<uint64_t>(std::max<uint64_t>((waves + kWaves - 1) / kWaves, 1), 1u << 20); }

struct Scratch { // pool allocations released together
  DevPool &pool;
  std::vector<void *> held;
  explicit Scratch(DevPool &p) : pool(p) {}
  ~Scratch() {
    for (void *p : held) pool.release(p);
  }
  template <class T> bool get(T *&p, uint64_t n) {
    if (pool.alloc((void **)&p, std::max<uint64_t>(n, 1) * sizeof(T))) return false;
    held.push_back(p);
    return true;
  }
};

int report_error(uint64_t e) {
  const uint32_t b = (uint32_t)(e >> 25), cls = (e >> 24) & 1, k = (e >> 8) & 0xFFFF, why = e & 0xFF;
  const char *txt = why < kReasons ? kReasonText[why] : "?";
  if (cls == 0) return fail(RB_EFORMAT, "bitmap %u: %s", b, txt);
  return fail(RB_EINVAL, "bitmap %u container %u: %s", b, k, txt);
}

} // namespace

int deserialize_device(rbgpu_ctx *ctx, const uint8_t *d_in, uint64_t in_lim, const uint64_t *d_in_off, uint32_t n,
                       rbgpu_set **out) {
  hipStream_t st = ctx->stream;
  Scratch w(ctx->pool);
  DeArgs a{};
  a.in = InBytes{d_in, (in_lim + 3) & ~3ull};
  a.in_off = d_in_off;
  a.n = n;
  uint64_t *cbase, *tmp;
  unsigned long long *err;
  if (!w.get(a.count, n + 1ull) || !w.get(cbase, n + 1ull) || !w.get(err, 1) || !w.get(a.bad, n) ||
      !w.get(tmp, scan_tmp_words(n + 1ull)))
    return fail(RB_ENOMEM, "deserialize workspace for %u bitmaps", n);
  a.cbase = cbase;
  a.err = err;
  HIPCHK(hipMemsetAsync(err, 0xFF, 8, st));
  HIPCHK(hipMemsetAsync(a.count + n, 0, 8, st));
  if (n) k_de_header<<<(uint32_t)std::min<uint64_t>((n + 255) / 256, 1u << 20), 256, 0, st>>>(a);
  scan_exclusive(a.count, cbase, n + 1ull, tmp, st);
  uint64_t nc = 0;
  HIPCHK(hipMemcpyAsync(&nc, cbase + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  LAUNCHCHK();
  uint64_t *bidx, *soff, *tmp2;
  if (!w.get(a.key, nc) || !w.get(a.type, nc) || !w.get(a.card, nc) || !w.get(a.nruns, nc) || !w.get(a.src, nc) ||
      !w.get(a.owner, nc) || !w.get(a.bigflag, nc + 1) || !w.get(a.small, nc + 1) || !w.get(bidx, nc + 1) ||
      !w.get(soff, nc + 1) || !w.get(tmp2, scan_tmp_words(nc + 1)))
    return fail(RB_ENOMEM, "deserialize workspace for %llu containers", (unsigned long long)nc);
  // containers of a bitmap that fails mid-way keep zero sizes
  HIPCHK(hipMemsetAsync(a.bigflag, 0, (nc + 1) * 8, st));
  HIPCHK(hipMemsetAsync(a.small, 0, (nc + 1) * 8, st));
  HIPCHK(hipMemsetAsync(a.owner, 0, std::max<uint64_t>(nc, 1) * 4, st));
  HIPCHK(hipMemsetAsync(a.type, kArray, std::max<uint64_t>(nc, 1), st));
  HIPCHK(hipMemsetAsync(a.card, 0, std::max<uint64_t>(nc, 1) * 4, st));
  if (n) k_de_table<<<grid_for(n), 256, 0, st>>>(a);
  scan_exclusive(a.bigflag, bidx, nc + 1, tmp2, st);
  scan_exclusive(a.small, soff, nc + 1, tmp2, st);
  uint64_t tot[3] = {0, 0, 0};
  HIPCHK(hipMemcpyAsync(&tot[0], bidx + nc, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&tot[1], soff + nc, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  LAUNCHCHK();
  const uint64_t small_base = tot[0] * kBitmapBytes, total = small_base + tot[1];
  rbgpu_set *s = new rbgpu_set;
  int rc = set_alloc(ctx, s, n, nc, total);
  if (rc) {
    set_release(s);
    delete s;
    return rc;
  }
  launch_layout(a.bigflag, bidx, soff, small_base, s->off, nc, st);
  if (nc) k_de_copy<<<grid_for(nc), 256, 0, st>>>(a, nc, s->off, s->payload);
  auto cp = [&](void *dst, const void *src, size_t bytes) {
    return bytes ? hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st) : hipSuccess;
  };
  uint64_t e = ~0ull;
  if (cp(s->begin, cbase, (n + 1ull) * 8) || cp(s->key, a.key, nc * 2) || cp(s->type, a.type, nc) ||
      cp(s->card, a.card, nc * 4) || cp(s->nruns, a.nruns, nc * 2) ||
      hipMemcpyAsync(&e, err, 8, hipMemcpyDeviceToHost, st) || hipStreamSynchronize(st)) {
    set_release(s);
    delete s;
    return fail(RB_EDEVICE, "device deserialize failed");
  }
  if (e != ~0ull) {
    set_release(s);
    delete s;
    return report_error(e);
  }
  *out = s;
  return RB_OK;
}

int serialize_device(const rbgpu_set *s, uint32_t first, uint32_t count, uint8_t *d_out, uint64_t cap,
                     uint64_t *offsets, bool host_dst) {
  rbgpu_ctx *ctx = s->ctx;
  hipStream_t st = ctx->stream;
  int rc = ensure_h_begin(s);
  if (rc) return rc;
  const uint64_t c_lo = s->h_begin[first], nc = s->h_begin[first + count] - c_lo;
  Scratch w(ctx->pool);
  SerArgs a{};
  a.s = s->view();
  a.first = first;
  a.count = count;
  uint64_t *cpos_local, *out_off, *tmp;
  uint32_t *owner;
  if (!w.get(cpos_local, nc) || !w.get(a.hdr, count) || !w.get(a.size, count + 1ull) || !w.get(out_off, count + 1ull) ||
      !w.get(tmp, scan_tmp_words(count + 1ull)) || !w.get(owner, nc))
    return fail(RB_ENOMEM, "serialize workspace for %u bitmaps", count);
  a.cpos = cpos_local - c_lo; // indexed by set-global container index
  a.out_off = out_off;
  HIPCHK(hipMemsetAsync(a.size + count, 0, 8, st));
  if (count) {
    k_ser_measure<<<grid_for(count), 256, 0, st>>>(a);
    k_ser_owner<<<grid_for(count), 256, 0, st>>>(a, owner);
  }
  scan_exclusive(a.size, out_off, count + 1ull, tmp, st);
  std::vector<uint64_t> h_off(count + 1ull);
  HIPCHK(hipMemcpyAsync(h_off.data(), out_off, (count + 1ull) * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  LAUNCHCHK();
  const uint64_t total = h_off[count];
  if (total > cap) return fail(RB_EINVAL, "destination buffer too small (%llu needed)", (unsigned long long)total);
  uint8_t *dev = d_out;
  if (host_dst && !w.get(dev, total)) return fail(RB_ENOMEM, "serialize staging of %llu bytes", (unsigned long long)total);
  a.out = dev;
  if (count) k_ser_header<<<grid_for(count), 256, 0, st>>>(a);
  if (nc) k_ser_payload<<<grid_for(nc), 256, 0, st>>>(a, owner, nc);
  if (host_dst && total) HIPCHK(hipMemcpyAsync(d_out, dev, total, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  LAUNCHCHK();
  if (offsets) std::copy(h_off.begin(), h_off.end(), offsets);
  return RB_OK;
}

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_codec() {}
void warm_codec(hipStream_t st) { k_warm_codec<<<1, 64, 0, st>>>(); }

} // namespace rbg
