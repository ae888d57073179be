// comm.hip — multi-GPU exchange behind the C ABI: RCCL communicator, shard summaries, and the
// gather of a key-range-sharded result into the RoaringFormatSpec bytes of the whole bitmap.
//
// The data path never crosses GPUs: each rank aggregates its own high-key range (wide.hip, bsi.hip).
// What the result needs from the other ranks is small and exact:
//   summaries  one ncclAllGather of 5 u64 per rank (cardinality, containers, Run containers,
//              payload bytes, shard bytes) -> the whole result's size, cardinality and this rank's
//              offsets in the global bytes;
//   gather     every rank serializes its shard on its GPU (codec.hip), one grouped ncclSend /
//              ncclRecv moves the shards to the root, and one kernel there writes the global header
//              — cookie, Run-container bitmap, (key, card-1) pairs, payload offsets (RoaringArray.
//              serialize, RoaringArray.java:851-940) — around the shard payloads, which are copied
//              verbatim.  The shard headers hold everything the global one needs, so no per-container
//              metadata travels separately.
// RCCL is opened with dlopen at rbgpu_comm_init, so librbgpu has no link-time dependency on it.
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include <rccl/rccl.h>

#include "internal.hpp"

namespace rbg {
namespace {

// ---------------------------------------------------------------- RCCL entry points (dlopen)
struct Rccl {
  void *h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char *(*error_string)(ncclResult_t) = nullptr;
};
const Rccl *rccl(std::string &err) {
  static Rccl r;
  static bool tried = false, ok = false;
  static std::string why;
  if (!tried) {
    tried = true;
    // a process that already holds RCCL (torch's copy) gets that one back for the same soname
    for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.h) break;
    }
    if (!r.h) {
      why = std::string("cannot load RCCL: ") + dlerror();
    } else {
      auto sym = [&](auto &fp, const char *name) {
        fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(r.h, name));
        if (!fp && why.empty()) why = std::string("RCCL lacks ") + name;
      };
      sym(r.get_unique_id, "ncclGetUniqueId");
      sym(r.init_rank, "ncclCommInitRank");
      sym(r.destroy, "ncclCommDestroy");
      sym(r.all_gather, "ncclAllGather");
      sym(r.all_reduce, "ncclAllReduce");
      sym(r.send, "ncclSend");
      sym(r.recv, "ncclRecv");
      sym(r.group_start, "ncclGroupStart");
      sym(r.group_end, "ncclGroupEnd");
      sym(r.error_string, "ncclGetErrorString");
      ok = why.empty();
    }
  }
  if (!ok) {
    err = why;
    return nullptr;
  }
  return &r;
}

#define NCCLCHK(R, x)                                                                                  \
  do {                                                                                                 \
    ncclResult_t e_ = (x);                                                                             \
    if (e_ != ncclSuccess) return ::rbg::fail(RB_EDEVICE, "%s failed: %s", #x, (R)->error_string(e_)); \
  } while (0)

// ---------------------------------------------------------------- RoaringFormatSpec assembly
// Everything below is __host__ __device__: rbgpu_shard_assemble_host runs the same code on the CPU.
constexpr uint32_t kSerialCookie = 12347, kSerialCookieNoRun = 12346; // RoaringArray.java:42-43
constexpr uint64_t kNoOffsetThreshold = 4;                            // RoaringArray.java:44

__host__ __device__ inline uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
__host__ __device__ inline uint32_t rd32(const uint8_t *p) { return rd16(p) | (rd16(p + 2) << 16); }
__host__ __device__ inline void wr32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
  p[2] = (uint8_t)(v >> 16);
  p[3] = (uint8_t)(v >> 24);
}
// RoaringArray.headerSize (RoaringArray.java:781-790)
__host__ __device__ inline uint64_t header_bytes(uint64_t n, bool has_run) {
  if (has_run) return 4 + (n + 7) / 8 + 4 * n + (n >= kNoOffsetThreshold ? 4 * n : 0);
  return 8 + 8 * n;
}

// One shard's standalone serialization, as the assembly sees it.
struct Part {
  const uint8_t *bytes;
  uint64_t n;      // containers
  uint64_t pre;    // bytes before the (key, card-1) pairs: cookie (+ count) (+ Run bitmap)
  uint64_t lh;     // header bytes
  uint64_t body;   // payload bytes
  uint64_t cbase;  // first container index in the whole result
  uint64_t bbase;  // first payload byte, relative to the whole result's first payload byte
  uint32_t has_run, has_off;
};
// Parse a shard header (RoaringArray.deserialize's cookie logic, RoaringArray.java:276-300);
// false when the bytes are not a serialized bitmap.
__host__ __device__ inline bool parse_part(const uint8_t *b, uint64_t len, Part &p) {
  if (len < 4) return false;
  const uint32_t cookie = rd32(b);
  if ((cookie & 0xFFFF) == kSerialCookie) {
    p.has_run = 1;
    p.n = (cookie >> 16) + 1ull;
    p.pre = 4 + (p.n + 7) / 8;
  } else if (cookie == kSerialCookieNoRun) {
    if (len < 8) return false;
    p.has_run = 0;
    p.n = rd32(b + 4);
    p.pre = 8;
  } else {
    return false;
  }
  p.has_off = !p.has_run || p.n >= kNoOffsetThreshold;
  p.lh = header_bytes(p.n, p.has_run);
  if (p.lh > len) return false;
  p.bytes = b;
  p.body = len - p.lh;
  return true;
}
__host__ __device__ inline bool part_is_run(const Part &p, uint64_t j) {
  return p.has_run && ((p.bytes[4 + j / 8] >> (j % 8)) & 1);
}
// payload position of container j inside the part's payload area
__host__ __device__ inline uint64_t part_payload_pos(const Part &p, uint64_t j) {
  if (p.has_off) return rd32(p.bytes + p.pre + 4 * p.n + 4 * j) - p.lh;
  uint64_t pos = 0; // < 4 containers with Runs: walk them (RoaringArray.java:325-345)
  for (uint64_t i = 0; i < j; ++i) {
    const uint32_t card = rd16(p.bytes + p.pre + 4 * i + 2) + 1;
    if (part_is_run(p, i)) pos += 2 + 4ull * rd16(p.bytes + p.lh + pos);
    else pos += card <= 4096 ? 2ull * card : 8192ull;
  }
  return pos;
}
struct Global {
  uint64_t n, pre, h;
  uint32_t has_run, has_off;
};
__host__ __device__ inline Global global_of(uint64_t n, bool has_run) {
  Global g;
  g.n = n;
  g.has_run = has_run;
  g.pre = has_run ? 4 + (n + 7) / 8 : 8;
  g.has_off = !has_run || n >= kNoOffsetThreshold;
  g.h = header_bytes(n, has_run);
  return g;
}
__host__ __device__ inline uint32_t part_of(const Part *parts, uint32_t np, uint64_t i) {
  uint32_t lo = 0, hi = np; // last part with cbase <= i (parts may be empty)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (parts[mid].cbase <= i) lo = mid;
    else hi = mid;
  }
  while (lo + 1 < np && parts[lo + 1].cbase <= i) ++lo;
  return lo;
}
// header item t: t == 0 the cookie; t in [1, 1 + N) container t-1's pair and offset; then the
// Run-bitmap bytes
__host__ __device__ inline void assemble_item(const Part *parts, uint32_t np, const Global &g, uint64_t t,
                                              uint8_t *dst) {
  if (t == 0) {
    if (g.has_run) {
      wr32(dst, kSerialCookie | (uint32_t)((g.n - 1) << 16));
    } else {
      wr32(dst, kSerialCookieNoRun);
      wr32(dst + 4, (uint32_t)g.n);
    }
    return;
  }
  if (t <= g.n) {
    const uint64_t i = t - 1;
    const Part &p = parts[part_of(parts, np, i)];
    const uint64_t j = i - p.cbase;
    const uint8_t *kc = p.bytes + p.pre + 4 * j;
    uint8_t *o = dst + g.pre + 4 * i;
    o[0] = kc[0];
    o[1] = kc[1];
    o[2] = kc[2];
    o[3] = kc[3];
    if (g.has_off) wr32(dst + g.pre + 4 * g.n + 4 * i, (uint32_t)(g.h + p.bbase + part_payload_pos(p, j)));
    return;
  }
  const uint64_t byte = t - 1 - g.n; // Run bitmap byte: 8 containers, possibly from two shards
  if (!g.has_run || byte >= (g.n + 7) / 8) return;
  uint32_t v = 0;
  for (uint64_t k = 0; k < 8 && 8 * byte + k < g.n; ++k) {
    const uint64_t i = 8 * byte + k;
    const Part &p = parts[part_of(parts, np, i)];
    v |= (uint32_t)part_is_run(p, i - p.cbase) << k;
  }
  dst[4 + byte] = (uint8_t)v;
}
__host__ __device__ inline uint64_t assemble_items(const Global &g) { return 1 + g.n + (g.has_run ? (g.n + 7) / 8 : 0); }

__global__ __launch_bounds__(256) void k_shard_header(const Part *parts, uint32_t np, Global g, uint8_t *dst) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < assemble_items(g)) assemble_item(parts, np, g, t, dst);
}

// parts -> plan: container / payload prefixes and the global header shape
int plan_parts(std::vector<Part> &parts, Global &g) {
  uint64_t n = 0, body = 0;
  bool has_run = false;
  for (Part &p : parts) {
    p.cbase = n;
    p.bbase = body;
    n += p.n;
    body += p.body;
    has_run |= p.has_run != 0;
  }
  if (has_run && n > 65536) return fail(RB_EINVAL, "more than 65536 containers");
  g = global_of(n, has_run);
  return RB_OK;
}

// ---------------------------------------------------------------- transports
// The exchange logic below (summaries, failure agreement, the naive_and order, the shard gather and
// the header assembly) runs over a transport: RCCL on device buffers, or a caller's host transport
// (rb_host_transport: the JVM's own channel; the CPU tests' gloo group).  Every collective is entered
// by every rank whatever its own step did: a local failure travels as a flag inside the exchange.
struct Xport {
  int nranks = 1, rank = 0;
  virtual ~Xport() {}
  virtual bool on_device() const = 0; // exchange buffers (gather staging) live in device memory
  // all-gather of k u64 per rank -> out[nranks * k] (host values in, host values out)
  virtual int gather_u64(const uint64_t *mine, uint32_t k, std::vector<uint64_t> &out) = 0;
  // element-wise sum over the ranks, in place (host values)
  virtual int reduce_u64(uint64_t *v, uint32_t n) = 0;
  // shards to the root: rank r's lens[r] bytes land at recv + base[r] on the root (transport memory)
  virtual int gather_bytes(int root, const uint8_t *mine, const std::vector<uint64_t> &lens,
                           const std::vector<uint64_t> &base, uint8_t *recv) = 0;
};

constexpr uint32_t kXbufWords = 1u << 16; // RCCL exchange buffer: every u64 exchange goes through it in chunks

struct RcclXport final : Xport {
  rbgpu_ctx *ctx = nullptr;
  const Rccl *r = nullptr;
  ncclComm_t nc = nullptr;
  uint64_t *d_buf = nullptr; // kXbufWords * (nranks + 1) u64, allocated once: no allocation inside a collective
  bool on_device() const override { return true; }
  int gather_u64(const uint64_t *mine, uint32_t k, std::vector<uint64_t> &out) override {
    if (k > kXbufWords) return fail(RB_EINVAL, "exchange of %u words", k);
    hipStream_t st = ctx->stream;
    uint64_t *send = d_buf, *recv = d_buf + kXbufWords;
    int rc = hipSetDevice(ctx->device) || hipMemcpyAsync(send, mine, 8ull * k, hipMemcpyHostToDevice, st)
                 ? fail(RB_EDEVICE, "exchange upload")
                 : RB_OK;
    // the collective is entered even when the upload failed: the other ranks are already in it
    const ncclResult_t e = r->all_gather(send, recv, (size_t)k, ncclUint64, nc, st);
    if (!rc && e != ncclSuccess) rc = fail(RB_EDEVICE, "ncclAllGather: %s", r->error_string(e));
    out.assign((size_t)nranks * k, 0);
    if (!rc && (hipMemcpyAsync(out.data(), recv, 8ull * k * nranks, hipMemcpyDeviceToHost, st) ||
                hipStreamSynchronize(st)))
      rc = fail(RB_EDEVICE, "exchange read-back");
    return rc;
  }
  int reduce_u64(uint64_t *v, uint32_t n) override {
    hipStream_t st = ctx->stream;
    int rc = hipSetDevice(ctx->device) ? fail(RB_EDEVICE, "hipSetDevice") : RB_OK;
    for (uint32_t o = 0; o < n; o += kXbufWords) { // fixed chunks: the same count of collectives on every rank
      const uint32_t m = std::min(kXbufWords, n - o);
      if (!rc && hipMemcpyAsync(d_buf, v + o, 8ull * m, hipMemcpyHostToDevice, st)) rc = fail(RB_EDEVICE, "reduce upload");
      const ncclResult_t e = r->all_reduce(d_buf, d_buf, m, ncclUint64, ncclSum, nc, st);
      if (!rc && e != ncclSuccess) rc = fail(RB_EDEVICE, "ncclAllReduce: %s", r->error_string(e));
      if (!rc && (hipMemcpyAsync(v + o, d_buf, 8ull * m, hipMemcpyDeviceToHost, st) || hipStreamSynchronize(st)))
        rc = fail(RB_EDEVICE, "reduce read-back");
    }
    return rc;
  }
  int gather_bytes(int root, const uint8_t *mine, const std::vector<uint64_t> &lens, const std::vector<uint64_t> &base,
                   uint8_t *recv) override {
    hipStream_t st = ctx->stream;
    ncclResult_t e = r->group_start(); // one grouped send / recv
    if (e == ncclSuccess) {
      if (rank == root) {
        for (int q = 0; q < nranks && e == ncclSuccess; ++q)
          if (q != root && lens[q]) e = r->recv(recv + base[q], lens[q], ncclUint8, q, nc, st);
      } else if (lens[rank]) {
        e = r->send(mine, lens[rank], ncclUint8, root, nc, st);
      }
      const ncclResult_t e2 = r->group_end();
      if (e == ncclSuccess) e = e2;
    }
    if (e != ncclSuccess) return fail(RB_EDEVICE, "shard gather: %s", r->error_string(e));
    return RB_OK;
  }
  ~RcclXport() override {
    if (nc) (void)r->destroy(nc);
    if (d_buf) (void)hipFree(d_buf);
  }
};

struct HostXport final : Xport {
  rb_host_transport t{};
  bool on_device() const override { return false; }
  int gather_u64(const uint64_t *mine, uint32_t k, std::vector<uint64_t> &out) override {
    out.assign((size_t)nranks * k, 0);
    if (t.all_gather(t.user, mine, out.data(), 8ull * k)) return fail(RB_EDEVICE, "host transport all_gather failed");
    return RB_OK;
  }
  int reduce_u64(uint64_t *v, uint32_t n) override {
    if (n && t.all_reduce_sum_u64(t.user, v, n)) return fail(RB_EDEVICE, "host transport all_reduce failed");
    return RB_OK;
  }
  int gather_bytes(int root, const uint8_t *mine, const std::vector<uint64_t> &lens, const std::vector<uint64_t> &base,
                   uint8_t *recv) override {
    int rc = RB_OK;
    if (rank == root) {
      for (int q = 0; q < nranks; ++q)
        if (q != root && lens[q] && t.recv(t.user, recv + base[q], lens[q], q) && !rc)
          rc = fail(RB_EDEVICE, "host transport recv from rank %d failed", q);
    } else if (lens[rank] && t.send(t.user, mine, lens[rank], root)) {
      rc = fail(RB_EDEVICE, "host transport send failed");
    }
    return rc;
  }
};

// ---------------------------------------------------------------- a local shard as the exchange sees it
// A one-bitmap device set (the product path) or the standalone serialized bytes of one (host memory).
struct ShardSrc {
  const rbgpu_set *set = nullptr;
  const uint8_t *bytes = nullptr;
  uint64_t len = 0;
  // (cardinality, containers, Run containers, payload bytes, serialized bytes)
  int summary(uint64_t (&v)[5]) const {
    if (set) {
      rb_bitmap_summary s{};
      int rc = rbgpu_set_summaries(set, 0, 1, &s);
      uint64_t ser = 0;
      if (!rc) rc = rbgpu_set_serialized_sizes(set, &ser);
      if (rc) return rc;
      v[0] = s.cardinality, v[1] = s.n_containers, v[2] = s.n_run_containers, v[3] = s.payload_bytes, v[4] = ser;
      return RB_OK;
    }
    Part p{};
    if (!parse_part(bytes, len, p)) return fail(RB_EFORMAT, "the shard is not a serialized bitmap");
    uint64_t card = 0, runs = 0;
    for (uint64_t j = 0; j < p.n; ++j) {
      const bool run = part_is_run(p, j);
      runs += run;
      if (!run) {
        // card-1 from the header; an empty container (horizontal_xor keeps one, FastAggregation.java:278)
        // writes 0xFFFF there, so with offsets an Array's card is its payload length / 2
        uint64_t cj = rd16(p.bytes + p.pre + 4 * j + 2) + 1ull;
        if (p.has_off) {
          const uint64_t b0 = part_payload_pos(p, j), b1 = j + 1 < p.n ? part_payload_pos(p, j + 1) : p.body;
          if (b1 - b0 != 8192) cj = (b1 - b0) / 2;
        }
        card += cj;
      } else { // a Run's cardinality is its run lengths (an empty Run's header says 65536)
        const uint64_t at = p.lh + part_payload_pos(p, j);
        if (at + 2 > len) return fail(RB_EFORMAT, "truncated Run container");
        const uint32_t nr = rd16(bytes + at);
        if (at + 2 + 4ull * nr > len) return fail(RB_EFORMAT, "truncated Run container");
        for (uint32_t q = 0; q < nr; ++q) card += rd16(bytes + at + 4 + 4 * q) + 1ull;
      }
    }
    v[0] = card, v[1] = p.n, v[2] = runs, v[3] = p.body, v[4] = len;
    return RB_OK;
  }
  // the standalone serialized bytes into `dst` (device memory when on_device, else host)
  int serialize(uint8_t *dst, uint64_t cap, bool on_device, hipStream_t st) const {
    if (set) {
      uint64_t offs[2] = {0, 0};
      return on_device ? rbgpu_set_serialize_device(set, 0, 1, dst, cap, offs) : rbgpu_set_serialize(set, 0, 1, dst, cap, offs);
    }
    if (cap < len) return fail(RB_EINVAL, "shard staging holds %llu bytes", (unsigned long long)cap);
    if (!on_device) {
      if (len) std::memcpy(dst, bytes, len);
      return RB_OK;
    }
    if (len && (hipMemcpyAsync(dst, bytes, len, hipMemcpyHostToDevice, st) || hipStreamSynchronize(st)))
      return fail(RB_EDEVICE, "shard upload");
    return RB_OK;
  }
};

int agree(int local_rc, uint64_t failed_others) {
  if (local_rc) return local_rc;
  if (failed_others) return fail(RB_EDEVICE, "%llu other rank(s) failed this collective call", (unsigned long long)failed_others);
  return RB_OK;
}

} // namespace
} // namespace rbg

using namespace rbg;

struct rbgpu_comm {
  rbgpu_ctx *ctx = nullptr; // null for a host-transport communicator without a device
  Xport *x = nullptr;
  int nranks = 1, rank = 0;
};

namespace {

// summary exchange; local_rc != 0: this rank's shard could not be built (src may be null), it
// still takes part in the all-gather and every rank fails together
int summarize(rbgpu_comm *c, const ShardSrc *src, int local_rc, rb_shard_summary *out) {
  uint64_t v[5] = {0, 0, 0, 0, 0};
  if (!local_rc) local_rc = src->summary(v);
  const uint64_t mine[6] = {v[0], v[1], v[2], v[3], v[4], local_rc ? 1ull : 0ull};
  std::vector<uint64_t> g;
  int rc = c->x->gather_u64(mine, 6, g);
  if (rc) return local_rc ? local_rc : rc;
  uint64_t failed = 0;
  for (int r = 0; r < c->nranks; ++r) failed += g[6 * r + 5];
  rc = agree(local_rc, failed - (local_rc ? 1 : 0));
  if (rc) return rc;
  rb_shard_summary o{};
  uint64_t before_payload = 0, before_cont = 0;
  for (int r = 0; r < c->nranks; ++r) {
    o.cardinality += g[6 * r];
    o.n_containers += g[6 * r + 1];
    o.n_run_containers += g[6 * r + 2];
    o.payload_bytes += g[6 * r + 3];
    if (r < c->rank) {
      before_cont += g[6 * r + 1];
      before_payload += g[6 * r + 3];
    }
  }
  if (o.n_run_containers && o.n_containers > 65536) return fail(RB_EINVAL, "more than 65536 containers");
  const uint64_t h = header_bytes(o.n_containers, o.n_run_containers > 0);
  o.serialized_size = h + o.payload_bytes;
  o.payload_offset = h + before_payload;
  o.container_offset = before_cont;
  o.local_serialized = v[4];
  *out = o;
  return RB_OK;
}

// all-reduce of n member counts plus a failure flag: every rank takes part whatever its own step did;
// then naive_and's order: the globally smallest member (first on ties) first, the rest in order
// (FastAggregation.java:328-346)
int naive_and_order(rbgpu_comm *c, const uint32_t *mem, const uint64_t *counts, uint32_t n, int local_rc,
                    std::vector<uint32_t> &ord) {
  std::vector<uint64_t> cnt(n + 1, 0);
  if (!local_rc && n) std::copy(counts, counts + n, cnt.begin());
  cnt[n] = local_rc ? 1 : 0;
  int rc = c->x->reduce_u64(cnt.data(), n + 1);
  if (rc) return local_rc ? local_rc : rc;
  rc = agree(local_rc, cnt[n] - (local_rc ? 1 : 0));
  if (rc) return rc;
  ord.clear();
  if (n) {
    uint32_t sm = 0;
    for (uint32_t i = 1; i < n; ++i)
      if (cnt[i] < cnt[sm]) sm = i;
    ord.push_back(mem[sm]);
    for (uint32_t i = 0; i < n; ++i)
      if (mem[i] != mem[sm]) ord.push_back(mem[i]);
  }
  return RB_OK;
}

// The whole result's bytes on the root: shard lengths exchanged (with failure flags), every rank
// serializes its shard into transport memory, the shards travel to the root, the root assembles the
// global header around the concatenated payloads (a kernel on a device transport, the same code on the
// host otherwise) into dst (device memory when dst_device).
int gather(rbgpu_comm *c, const ShardSrc *src, const rb_shard_summary *summary, int root, uint8_t *dst, uint64_t cap,
           bool dst_device, int local_rc) {
  Xport &X = *c->x;
  const bool is_root = c->rank == root, dev = X.on_device();
  rbgpu_ctx *ctx = c->ctx;
  hipStream_t st = ctx ? ctx->stream : nullptr;
  if (!local_rc && is_root && (!dst || cap < summary->serialized_size))
    local_rc = fail(RB_EINVAL, "destination holds %llu bytes, %llu needed", (unsigned long long)cap,
                    (unsigned long long)summary->serialized_size);
  // every rank's shard size (the summary's own field, gathered again: callers may pass a summary from
  // another exchange of the same shards) and failure flag
  const uint64_t mine[2] = {local_rc ? 0 : summary->local_serialized, local_rc ? 1ull : 0ull};
  std::vector<uint64_t> g;
  int rc = X.gather_u64(mine, 2, g);
  if (rc) return local_rc ? local_rc : rc;
  uint64_t failed = 0;
  std::vector<uint64_t> lens(c->nranks), base(c->nranks + 1, 0);
  for (int r = 0; r < c->nranks; ++r) {
    lens[r] = g[2 * r];
    failed += g[2 * r + 1];
    base[r + 1] = base[r] + lens[r];
  }
  rc = agree(local_rc, failed - (local_rc ? 1 : 0));
  if (rc) return rc;
  // this rank's shard, serialized into transport memory (the root stages every shard)
  const uint64_t stage = is_root ? base[c->nranks] : lens[c->rank];
  uint8_t *d_stage = nullptr;
  std::vector<uint8_t> h_stage;
  Part *d_parts = nullptr;
  uint8_t *d_out = nullptr; // device assembly into a host dst
  if (dev) {
    if (ctx->pool.alloc((void **)&d_stage, std::max<uint64_t>(stage, 16))) {
      d_stage = nullptr;
      local_rc = fail(RB_ENOMEM, "gather staging");
    }
  } else {
    h_stage.assign(std::max<uint64_t>(stage, 16), 0);
  }
  uint8_t *stage_p = dev ? d_stage : h_stage.data();
  auto done = [&](int code) { // every pooled buffer goes back on every path
    if (st) (void)hipStreamSynchronize(st);
    for (void *p : {(void *)d_stage, (void *)d_parts, (void *)d_out})
      if (p) ctx->pool.release(p);
    return code;
  };
  uint8_t *mine_at = stage_p ? stage_p + (is_root ? base[c->rank] : 0) : nullptr;
  if (!local_rc) local_rc = src->serialize(mine_at, lens[c->rank], dev, st);
  // agree once more before the point-to-point phase
  const uint64_t flag = local_rc ? 1 : 0;
  rc = X.gather_u64(&flag, 1, g);
  if (rc) return done(local_rc ? local_rc : rc);
  failed = 0;
  for (int r = 0; r < c->nranks; ++r) failed += g[r];
  rc = agree(local_rc, failed - flag);
  if (rc) return done(rc);
  rc = X.gather_bytes(root, mine_at, lens, base, stage_p);
  if (rc || !is_root) return done(rc);
  // the root reads the shard headers (small) to plan the global header
  std::vector<Part> parts(c->nranks);
  std::vector<uint8_t> hdr;
  for (int r = 0; r < c->nranks; ++r) {
    const uint8_t *hp = stage_p + base[r];
    if (dev) { // at most 4 + 8192 + 8 * 65536 header bytes per shard
      const uint64_t take = std::min<uint64_t>(lens[r], 8 + 8192 + 8ull * 65536);
      hdr.resize(std::max<uint64_t>(take, 1));
      if (take && (hipMemcpyAsync(hdr.data(), d_stage + base[r], take, hipMemcpyDeviceToHost, st) ||
                   hipStreamSynchronize(st)))
        return done(fail(RB_EDEVICE, "shard header read-back"));
      hp = hdr.data();
    }
    Part p{};
    if (!parse_part(hp, lens[r], p)) return done(fail(RB_EFORMAT, "shard %d is not a serialized bitmap", r));
    p.bytes = stage_p + base[r]; // the assembly reads the staged copy
    parts[r] = p;
  }
  Global gl;
  rc = plan_parts(parts, gl);
  if (rc) return done(rc);
  uint64_t total = gl.h;
  for (const Part &p : parts) total += p.body;
  if (cap < total)
    return done(fail(RB_EINVAL, "destination holds %llu bytes, %llu needed", (unsigned long long)cap,
                     (unsigned long long)total));
  if (dev) {
    uint8_t *out = dst;
    if (!dst_device) {
      if (ctx->pool.alloc((void **)&d_out, std::max<uint64_t>(total, 16))) {
        d_out = nullptr;
        return done(fail(RB_ENOMEM, "assembly buffer"));
      }
      out = d_out;
    }
    if (ctx->pool.alloc((void **)&d_parts, sizeof(Part) * parts.size())) {
      d_parts = nullptr;
      return done(fail(RB_ENOMEM, "gather plan"));
    }
    if (hipMemcpyAsync(d_parts, parts.data(), sizeof(Part) * parts.size(), hipMemcpyHostToDevice, st))
      return done(fail(RB_EDEVICE, "gather plan upload"));
    const uint64_t items = assemble_items(gl);
    k_shard_header<<<(unsigned)((items + 255) / 256), 256, 0, st>>>(d_parts, (uint32_t)parts.size(), gl, out);
    for (const Part &p : parts)
      if (p.body && hipMemcpyAsync(out + gl.h + p.bbase, p.bytes + p.lh, p.body, hipMemcpyDeviceToDevice, st))
        return done(fail(RB_EDEVICE, "shard body copy"));
    if (!dst_device && hipMemcpyAsync(dst, out, total, hipMemcpyDeviceToHost, st))
      return done(fail(RB_EDEVICE, "assembly read-back"));
    if (hipStreamSynchronize(st)) return done(fail(RB_EDEVICE, "shard gather"));
    const hipError_t le = hipGetLastError();
    if (le != hipSuccess) return done(fail(RB_EDEVICE, "kernel launch failed: %s", hipGetErrorString(le)));
    return done(RB_OK);
  }
  std::vector<uint8_t> h_out;
  uint8_t *out = dst;
  if (dst_device) {
    h_out.resize(std::max<uint64_t>(total, 1));
    out = h_out.data();
  }
  for (uint64_t t = 0; t < assemble_items(gl); ++t) assemble_item(parts.data(), (uint32_t)parts.size(), gl, t, out);
  for (const Part &p : parts)
    if (p.body) std::memcpy(out + gl.h + p.bbase, p.bytes + p.lh, p.body);
  if (dst_device && total &&
      (hipMemcpyAsync(dst, out, total, hipMemcpyHostToDevice, st) || hipStreamSynchronize(st)))
    return done(fail(RB_EDEVICE, "assembly upload"));
  return done(RB_OK);
}

int need_device(const rbgpu_comm *c) {
  return c->ctx ? RB_OK : fail(RB_EINVAL, "this communicator has no device context");
}

} // namespace

extern "C" {

int rbgpu_comm_unique_id(uint8_t id[RB_COMM_ID_BYTES]) {
  if (!id) return fail(RB_EINVAL, "null id");
  std::string err;
  const Rccl *r = rccl(err);
  if (!r) return fail(RB_EDEVICE, "%s", err.c_str());
  static_assert(sizeof(ncclUniqueId) == RB_COMM_ID_BYTES, "RCCL id size");
  ncclUniqueId u;
  NCCLCHK(r, r->get_unique_id(&u));
  std::memcpy(id, &u, RB_COMM_ID_BYTES);
  return RB_OK;
}

int rbgpu_comm_init(rbgpu_ctx *ctx, const uint8_t id[RB_COMM_ID_BYTES], int nranks, int rank, rbgpu_comm **out) {
  if (!ctx || !id || !out) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(RB_EINVAL, "bad rank %d of %d", rank, nranks);
  std::string err;
  const Rccl *r = rccl(err);
  if (!r) return fail(RB_EDEVICE, "%s", err.c_str());
  HIPCHK(hipSetDevice(ctx->device));
  ncclUniqueId u;
  std::memcpy(&u, id, RB_COMM_ID_BYTES);
  RcclXport *x = new RcclXport;
  x->ctx = ctx;
  x->r = r;
  x->nranks = nranks;
  x->rank = rank;
  const ncclResult_t e = r->init_rank(&x->nc, nranks, u, rank);
  if (e != ncclSuccess) {
    x->nc = nullptr;
    delete x;
    return fail(RB_EDEVICE, "ncclCommInitRank: %s", r->error_string(e));
  }
  if (hipMalloc((void **)&x->d_buf, 8ull * kXbufWords * (size_t)(nranks + 1)) != hipSuccess) {
    x->d_buf = nullptr;
    delete x;
    return fail(RB_ENOMEM, "exchange buffer");
  }
  rbgpu_comm *c = new rbgpu_comm;
  c->ctx = ctx;
  c->x = x;
  c->nranks = nranks;
  c->rank = rank;
  ctx->refs++;
  *out = c;
  return RB_OK;
}

int rbgpu_comm_init_host(rbgpu_ctx *ctx, const rb_host_transport *t, rbgpu_comm **out) {
  if (!t || !out) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  if (!t->all_gather || !t->all_reduce_sum_u64 || !t->send || !t->recv) return fail(RB_EINVAL, "incomplete transport");
  if (t->nranks < 1 || t->rank < 0 || t->rank >= t->nranks) return fail(RB_EINVAL, "bad rank %d of %d", t->rank, t->nranks);
  if (ctx) HIPCHK(hipSetDevice(ctx->device));
  HostXport *x = new HostXport;
  x->t = *t;
  x->nranks = t->nranks;
  x->rank = t->rank;
  rbgpu_comm *c = new rbgpu_comm;
  c->ctx = ctx;
  c->x = x;
  c->nranks = t->nranks;
  c->rank = t->rank;
  if (ctx) ctx->refs++;
  *out = c;
  return RB_OK;
}

void rbgpu_comm_destroy(rbgpu_comm *c) {
  if (!c) return;
  if (c->ctx) {
    (void)hipSetDevice(c->ctx->device);
    (void)hipStreamSynchronize(c->ctx->stream);
  }
  delete c->x;
  rbgpu_ctx *ctx = c->ctx;
  delete c;
  if (ctx) ctx_unref(ctx);
}

int rbgpu_comm_allreduce_sum(rbgpu_comm *c, uint64_t *values, uint32_t n) {
  if (!c || (n && !values)) return fail(RB_EINVAL, "null argument");
  if (!n) return RB_OK;
  return c->x->reduce_u64(values, n);
}

int rbgpu_shard_summarize(rbgpu_comm *c, const rbgpu_set *local, rb_shard_summary *out) {
  SETTLE(local);
  if (!c || !out) return fail(RB_EINVAL, "null argument");
  int local_rc = need_device(c);
  if (!local_rc && !local) local_rc = fail(RB_EINVAL, "null argument");
  else if (!local_rc && local->nb != 1) local_rc = fail(RB_EINVAL, "a shard is a one-bitmap set");
  else if (!local_rc && local->ctx != c->ctx) local_rc = fail(RB_EINVAL, "the shard belongs to another context");
  ShardSrc src;
  src.set = local;
  return summarize(c, &src, local_rc, out);
}

int rbgpu_shard_summarize_serialized(rbgpu_comm *c, const uint8_t *shard, uint64_t len, rb_shard_summary *out) {
  if (!c || !out) return fail(RB_EINVAL, "null argument");
  ShardSrc src;
  src.bytes = shard;
  src.len = len;
  const int local_rc = shard ? RB_OK : fail(RB_EINVAL, "null shard");
  return summarize(c, &src, local_rc, out);
}

int rbgpu_comm_naive_and_order(rbgpu_comm *c, const uint32_t *members, const uint64_t *local_counts, uint32_t n,
                               int local_failed, uint32_t *order, uint32_t *n_order) {
  if (!c) return fail(RB_EINVAL, "null argument");
  int local_rc = local_failed ? fail(RB_EINVAL, "this rank's member counts failed") : RB_OK;
  if (!local_rc && (!n_order || (n && (!local_counts || !order)))) local_rc = fail(RB_EINVAL, "null argument");
  std::vector<uint32_t> mem(n), ord;
  for (uint32_t i = 0; i < n; ++i) mem[i] = members ? members[i] : i;
  const int rc = naive_and_order(c, mem.data(), local_counts, n, local_rc, ord);
  if (!rc) {
    std::copy(ord.begin(), ord.end(), order);
    *n_order = (uint32_t)ord.size();
  }
  return rc;
}

int rbgpu_wide_sharded(rbgpu_comm *c, int sem, const rbgpu_set *in, const uint32_t *members, uint32_t n,
                       uint32_t key_lo, uint32_t key_hi, rbgpu_set **local, rb_shard_summary *summary) {
  if (!c || !local || !summary) return fail(RB_EINVAL, "null argument");
  *local = nullptr;
  // priorityqueue_or / _xor merge in the order of intermediate result sizes, which are global: a
  // key-range shard cannot follow it.  Refused on every rank alike (the arguments agree) before any
  // collective.
  if (c->nranks > 1 && (sem == RB_PQ_OR || sem == RB_PQ_XOR || sem >= RB_BUFFER_PQ_OR))
    return fail(RB_EINVAL, "priorityqueue_or / priorityqueue_xor cannot be key-range sharded");
  int rc = need_device(c);
  if (!rc && !in) rc = fail(RB_EINVAL, "null input set");
  if (sem == RB_NAIVE_AND || (sem == RB_FAST_AND && n <= 10)) {
    // naive_and(varargs) starts from the bitmap with the fewest containers (first on ties) and skips
    // it by identity (FastAggregation.java:328-346): its container counts are global, so they are the
    // ranks' key-range counts summed; then every shard folds the same order (naive_and(Iterator))
    std::vector<uint32_t> mem(n), ord;
    for (uint32_t i = 0; i < n; ++i) mem[i] = members ? members[i] : i;
    std::vector<uint64_t> cnt(std::max<uint32_t>(n, 1), 0);
    if (!rc) rc = rbgpu_set_range_counts(in, mem.data(), n, key_lo, key_hi, cnt.data());
    rc = naive_and_order(c, mem.data(), cnt.data(), n, rc, ord);
    if (rc) return rc;
    rc = rbgpu_wide_keys(c->ctx, RB_NAIVE_AND_ITER, in, ord.data(), (uint32_t)ord.size(), key_lo, key_hi, local);
  } else if (!rc) {
    rc = rbgpu_wide_keys(c->ctx, sem, in, members, n, key_lo, key_hi, local);
  }
  if (rc) *local = nullptr;
  ShardSrc src;
  src.set = *local;
  rc = summarize(c, &src, rc, summary);
  if (rc) {
    rbgpu_set_free(*local);
    *local = nullptr;
  }
  return rc;
}

int rbgpu_bsi_compare_sharded(rbgpu_comm *c, const rbgpu_set *bsi, int op, uint64_t start_or_value, uint64_t end,
                              uint64_t min_value, uint64_t max_value, const rbgpu_set *found, uint32_t key_lo,
                              uint32_t key_hi, rbgpu_set **local, rb_shard_summary *summary) {
  if (!c || !local || !summary) return fail(RB_EINVAL, "null argument");
  *local = nullptr;
  int rc = need_device(c);
  if (!rc)
    rc = rbgpu_bsi_compare_keys(c->ctx, bsi, op, start_or_value, end, min_value, max_value, found, key_lo, key_hi,
                                local);
  if (rc) *local = nullptr;
  ShardSrc src;
  src.set = *local;
  rc = summarize(c, &src, rc, summary); // every rank joins the exchange, failed or not
  if (rc) {
    rbgpu_set_free(*local);
    *local = nullptr;
  }
  return rc;
}

int rbgpu_shard_gather_serialized(rbgpu_comm *c, const rbgpu_set *local, const rb_shard_summary *summary, int root,
                                  uint8_t *d_dst, uint64_t cap) {
  SETTLE(local);
  if (!c || !summary) return fail(RB_EINVAL, "null argument");
  if (root < 0 || root >= c->nranks) return fail(RB_EINVAL, "bad root %d", root); // the same on every rank
  // a bad argument on one rank is exchanged with the lengths, so every rank fails together instead of
  // the others waiting in the send / recv
  int local_rc = need_device(c);
  if (!local_rc && !local) local_rc = fail(RB_EINVAL, "null shard");
  ShardSrc src;
  src.set = local;
  return gather(c, &src, summary, root, d_dst, cap, true, local_rc);
}

int rbgpu_shard_gather_host(rbgpu_comm *c, const uint8_t *shard, uint64_t len, const rb_shard_summary *summary,
                            int root, uint8_t *dst, uint64_t cap) {
  if (!c || !summary) return fail(RB_EINVAL, "null argument");
  if (root < 0 || root >= c->nranks) return fail(RB_EINVAL, "bad root %d", root);
  int local_rc = shard ? RB_OK : fail(RB_EINVAL, "null shard");
  if (!local_rc && len != summary->local_serialized)
    local_rc = fail(RB_EINVAL, "shard of %llu bytes, the summary says %llu", (unsigned long long)len,
                    (unsigned long long)summary->local_serialized);
  ShardSrc src;
  src.bytes = shard;
  src.len = len;
  return gather(c, &src, summary, root, dst, cap, false, local_rc);
}

int rbgpu_shard_assemble_host(const uint8_t *const *bufs, const uint64_t *lens, uint32_t nparts, uint8_t *dst,
                              uint64_t cap, uint64_t *written) {
  if ((nparts && (!bufs || !lens)) || !written) return fail(RB_EINVAL, "null argument");
  std::vector<Part> parts(nparts);
  for (uint32_t r = 0; r < nparts; ++r)
    if (!parse_part(bufs[r], lens[r], parts[r])) return fail(RB_EFORMAT, "part %u is not a serialized bitmap", r);
  Global g;
  int rc = plan_parts(parts, g);
  if (rc) return rc;
  uint64_t total = g.h;
  for (const Part &p : parts) total += p.body;
  *written = total;
  if (!dst || cap < total) return fail(RB_EINVAL, "destination holds %llu bytes, %llu needed", (unsigned long long)cap,
                                       (unsigned long long)total);
  for (uint64_t t = 0; t < assemble_items(g); ++t) assemble_item(parts.data(), nparts, g, t, dst);
  for (const Part &p : parts)
    if (p.body) std::memcpy(dst + g.h + p.bbase, p.bytes + p.lh, p.body);
  return RB_OK;
}

} // extern "C"
