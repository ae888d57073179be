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

} // namespace
} // namespace rbg

using namespace rbg;

struct rbgpu_comm {
  rbgpu_ctx *ctx = nullptr;
  ncclComm_t nc = nullptr;
  const Rccl *r = nullptr;
  int nranks = 1, rank = 0;
  uint64_t *d_buf = nullptr; // small exchange buffer (64 u64 per rank)
};

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
  rbgpu_comm *c = new rbgpu_comm;
  c->ctx = ctx;
  c->r = r;
  c->nranks = nranks;
  c->rank = rank;
  ncclResult_t e = r->init_rank(&c->nc, nranks, u, rank);
  if (e != ncclSuccess) {
    delete c;
    return fail(RB_EDEVICE, "ncclCommInitRank: %s", r->error_string(e));
  }
  if (hipMalloc((void **)&c->d_buf, 64 * 8 * (size_t)(nranks + 1)) != hipSuccess) {
    (void)r->destroy(c->nc);
    delete c;
    return fail(RB_ENOMEM, "exchange buffer");
  }
  ctx->refs++;
  *out = c;
  return RB_OK;
}

void rbgpu_comm_destroy(rbgpu_comm *c) {
  if (!c) return;
  (void)hipSetDevice(c->ctx->device);
  (void)hipStreamSynchronize(c->ctx->stream);
  if (c->nc) (void)c->r->destroy(c->nc);
  if (c->d_buf) (void)hipFree(c->d_buf);
  rbgpu_ctx *ctx = c->ctx;
  delete c;
  ctx_unref(ctx);
}

int rbgpu_comm_allreduce_sum(rbgpu_comm *c, uint64_t *values, uint32_t n) {
  if (!c || (n && !values)) return fail(RB_EINVAL, "null argument");
  if (n > 64 * (uint32_t)(c->nranks + 1)) return fail(RB_EINVAL, "at most %d values", 64 * (c->nranks + 1));
  if (!n) return RB_OK;
  hipStream_t st = c->ctx->stream;
  HIPCHK(hipSetDevice(c->ctx->device));
  HIPCHK(hipMemcpyAsync(c->d_buf, values, 8ull * n, hipMemcpyHostToDevice, st));
  NCCLCHK(c->r, c->r->all_reduce(c->d_buf, c->d_buf, n, ncclUint64, ncclSum, c->nc, st));
  HIPCHK(hipMemcpyAsync(values, c->d_buf, 8ull * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return RB_OK;
}

// all_gather of k u64 per rank -> out[nranks * k] (host)
static int gather_u64(rbgpu_comm *c, const uint64_t *mine, int k, std::vector<uint64_t> &out) {
  hipStream_t st = c->ctx->stream;
  HIPCHK(hipSetDevice(c->ctx->device));
  uint64_t *send = c->d_buf, *recv = c->d_buf + 64;
  HIPCHK(hipMemcpyAsync(send, mine, 8ull * k, hipMemcpyHostToDevice, st));
  NCCLCHK(c->r, c->r->all_gather(send, recv, (size_t)k, ncclUint64, c->nc, st));
  out.assign((size_t)c->nranks * k, 0);
  HIPCHK(hipMemcpyAsync(out.data(), recv, 8ull * k * c->nranks, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return RB_OK;
}

// Every rank takes part in each collective even when its own step failed (a rank that returned
// early would leave the others waiting in the collective): a failure travels as a flag inside the
// exchange, and every rank then fails together.  Returns the local code, or RB_EDEVICE naming the
// failure on another rank.
static int agree(int local_rc, uint64_t failed_ranks) {
  if (local_rc) return local_rc;
  if (failed_ranks) return fail(RB_EDEVICE, "%llu other rank(s) failed this collective call", (unsigned long long)failed_ranks);
  return RB_OK;
}

// summary exchange; local_rc != 0: this rank's shard could not be built (local may be null), it
// still takes part in the all-gather and every rank fails together
static int summarize(rbgpu_comm *c, const rbgpu_set *local, int local_rc, rb_shard_summary *out) {
  rb_bitmap_summary s{};
  uint64_t ser = 0;
  if (!local_rc) local_rc = rbgpu_set_summaries(local, 0, 1, &s);
  if (!local_rc) local_rc = rbgpu_set_serialized_sizes(local, &ser);
  const uint64_t mine[6] = {s.cardinality, s.n_containers, s.n_run_containers, s.payload_bytes, ser,
                            local_rc ? 1ull : 0ull};
  std::vector<uint64_t> g;
  int rc = gather_u64(c, mine, 6, g);
  if (rc) return rc;
  uint64_t failed = 0;
  for (int r = 0; r < c->nranks; ++r) failed += g[6 * r + 5];
  rc = agree(local_rc, failed);
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
  const uint64_t h = header_bytes(o.n_containers, o.n_run_containers > 0);
  o.serialized_size = h + o.payload_bytes;
  o.payload_offset = h + before_payload;
  o.container_offset = before_cont;
  o.local_serialized = ser;
  *out = o;
  return RB_OK;
}

int rbgpu_shard_summarize(rbgpu_comm *c, const rbgpu_set *local, rb_shard_summary *out) {
  if (!c || !out) return fail(RB_EINVAL, "null argument");
  int local_rc = RB_OK;
  if (!local) local_rc = fail(RB_EINVAL, "null argument");
  else if (local->nb != 1) local_rc = fail(RB_EINVAL, "a shard is a one-bitmap set");
  else if (local->ctx != c->ctx) local_rc = fail(RB_EINVAL, "the shard belongs to another context");
  return summarize(c, local, local_rc, out);
}

// all-reduce of n member counts plus a failure flag: every rank takes part whatever its own step did
static int reduce_counts(rbgpu_comm *c, std::vector<uint64_t> &cnt, int local_rc) {
  const uint32_t n = (uint32_t)cnt.size();
  cnt.push_back(local_rc ? 1 : 0);
  uint64_t *d = nullptr;
  rbgpu_ctx *ctx = c->ctx;
  if (ctx->pool.alloc((void **)&d, 8ull * (n + 1))) return fail(RB_ENOMEM, "member counts");
  hipStream_t st = ctx->stream;
  int rc = RB_OK;
  ncclResult_t e = ncclSuccess;
  if (hipSetDevice(ctx->device) || hipMemcpyAsync(d, cnt.data(), 8ull * (n + 1), hipMemcpyHostToDevice, st))
    rc = fail(RB_EDEVICE, "member counts upload");
  if (!rc && (e = c->r->all_reduce(d, d, n + 1, ncclUint64, ncclSum, c->nc, st)) != ncclSuccess)
    rc = fail(RB_EDEVICE, "member counts all-reduce: %s", c->r->error_string(e));
  if (!rc && (hipMemcpyAsync(cnt.data(), d, 8ull * (n + 1), hipMemcpyDeviceToHost, st) || hipStreamSynchronize(st)))
    rc = fail(RB_EDEVICE, "member counts read-back");
  (void)hipStreamSynchronize(st);
  ctx->pool.release(d);
  if (rc) return rc;
  const uint64_t failed = cnt[n] - (local_rc ? 1 : 0);
  cnt.pop_back();
  return agree(local_rc, failed);
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
  int rc = in ? RB_OK : fail(RB_EINVAL, "null input set");
  std::vector<uint32_t> ord;
  if (sem == RB_NAIVE_AND || (sem == RB_FAST_AND && n <= 10)) {
    // naive_and(varargs) starts from the bitmap with the fewest containers (first on ties) and skips
    // it by identity (FastAggregation.java:328-346): its container counts are global, so they are the
    // ranks' key-range counts summed; then every shard folds the same order (naive_and(Iterator))
    std::vector<uint32_t> mem(n);
    for (uint32_t i = 0; i < n; ++i) mem[i] = members ? members[i] : i;
    std::vector<uint64_t> cnt(n, 0);
    if (!rc) rc = rbgpu_set_range_counts(in, mem.data(), n, key_lo, key_hi, cnt.data());
    if (rc) std::fill(cnt.begin(), cnt.end(), 0ull);
    rc = reduce_counts(c, cnt, rc);
    if (rc) return rc;
    if (n) {
      uint32_t sm = 0;
      for (uint32_t i = 1; i < n; ++i)
        if (cnt[i] < cnt[sm]) sm = i;
      ord.push_back(mem[sm]);
      for (uint32_t m : mem)
        if (m != mem[sm]) ord.push_back(m);
    }
    rc = rbgpu_wide_keys(c->ctx, RB_NAIVE_AND_ITER, in, ord.data(), (uint32_t)ord.size(), key_lo, key_hi, local);
  } else if (!rc) {
    rc = rbgpu_wide_keys(c->ctx, sem, in, members, n, key_lo, key_hi, local);
  }
  if (rc) *local = nullptr;
  rc = summarize(c, *local, rc, summary);
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
  int rc = rbgpu_bsi_compare_keys(c->ctx, bsi, op, start_or_value, end, min_value, max_value, found, key_lo, key_hi,
                                  local);
  if (rc) *local = nullptr;
  rc = summarize(c, *local, rc, summary); // every rank joins the exchange, failed or not
  if (rc) {
    rbgpu_set_free(*local);
    *local = nullptr;
  }
  return rc;
}

int rbgpu_shard_gather_serialized(rbgpu_comm *c, const rbgpu_set *local, const rb_shard_summary *summary, int root,
                                  uint8_t *d_dst, uint64_t cap) {
  if (!c || !summary) return fail(RB_EINVAL, "null argument");
  if (root < 0 || root >= c->nranks) return fail(RB_EINVAL, "bad root %d", root); // the same on every rank
  const bool is_root = c->rank == root;
  // a bad argument on one rank is exchanged with the lengths, so every rank fails together instead of
  // the others waiting in the send / recv
  int local_rc = RB_OK;
  if (!local) local_rc = fail(RB_EINVAL, "null shard");
  else if (is_root && (!d_dst || cap < summary->serialized_size))
    local_rc = fail(RB_EINVAL, "destination holds %llu bytes, %llu needed", (unsigned long long)cap,
                    (unsigned long long)summary->serialized_size);
  rbgpu_ctx *ctx = c->ctx;
  hipStream_t st = ctx->stream;
  // every rank's shard size (the summary's own field, gathered again: callers may pass a summary
  // from another exchange of the same shards) and failure flag
  const uint64_t mine[2] = {summary->local_serialized, local_rc ? 1ull : 0ull};
  std::vector<uint64_t> g;
  int rc = gather_u64(c, mine, 2, g);
  if (rc) return rc;
  uint64_t failed = 0;
  std::vector<uint64_t> lens(c->nranks), base(c->nranks + 1, 0);
  for (int r = 0; r < c->nranks; ++r) {
    lens[r] = g[2 * r];
    failed += g[2 * r + 1];
    base[r + 1] = base[r] + lens[r];
  }
  rc = agree(local_rc, failed - (local_rc ? 1 : 0));
  if (rc) return rc;
  // this rank's shard, serialized on its GPU
  uint8_t *d_stage = nullptr;
  Part *d_parts = nullptr;
  const uint64_t stage = is_root ? base[c->nranks] : lens[c->rank];
  if (ctx->pool.alloc((void **)&d_stage, std::max<uint64_t>(stage, 16))) {
    d_stage = nullptr;
    local_rc = fail(RB_ENOMEM, "gather staging");
  }
  auto done = [&](int code) { // every pooled buffer goes back on every path
    (void)hipStreamSynchronize(st);
    if (d_stage) ctx->pool.release(d_stage);
    if (d_parts) ctx->pool.release(d_parts);
    return code;
  };
  uint8_t *mine_at = d_stage ? d_stage + (is_root ? base[c->rank] : 0) : nullptr;
  if (!local_rc) {
    uint64_t offs[2] = {0, 0};
    local_rc = rbgpu_set_serialize_device(local, 0, 1, mine_at, lens[c->rank], offs);
  }
  // agree once more before the point-to-point phase
  const uint64_t flag = local_rc ? 1 : 0;
  rc = gather_u64(c, &flag, 1, g);
  if (rc) return done(rc);
  failed = 0;
  for (int r = 0; r < c->nranks; ++r) failed += g[r];
  rc = agree(local_rc, failed - flag);
  if (rc) return done(rc);
  // one grouped send / recv: the shards travel to the root
  ncclResult_t e = c->r->group_start();
  if (e == ncclSuccess) {
    if (is_root) {
      for (int r = 0; r < c->nranks && e == ncclSuccess; ++r)
        if (r != root && lens[r]) e = c->r->recv(d_stage + base[r], lens[r], ncclUint8, r, c->nc, st);
    } else if (lens[c->rank]) {
      e = c->r->send(mine_at, lens[c->rank], ncclUint8, root, c->nc, st);
    }
    const ncclResult_t e2 = c->r->group_end();
    if (e == ncclSuccess) e = e2;
  }
  if (e != ncclSuccess) return done(fail(RB_EDEVICE, "shard gather: %s", c->r->error_string(e)));
  if (!is_root) return done(RB_OK);
  // the root reads the shard headers (small) to plan the global header
  std::vector<Part> parts(c->nranks);
  std::vector<uint8_t> hdr;
  for (int r = 0; r < c->nranks; ++r) {
    // at most 4 + 8192 + 8 * 65536 header bytes per shard
    const uint64_t take = std::min<uint64_t>(lens[r], 8 + 8192 + 8ull * 65536);
    hdr.resize(take);
    if (take) {
      if (hipMemcpyAsync(hdr.data(), d_stage + base[r], take, hipMemcpyDeviceToHost, st) ||
          hipStreamSynchronize(st))
        return done(fail(RB_EDEVICE, "shard header read-back"));
    }
    Part p{};
    if (!parse_part(hdr.data(), lens[r], p)) return done(fail(RB_EFORMAT, "shard %d is not a serialized bitmap", r));
    p.bytes = d_stage + base[r]; // the kernel reads the device copy
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
  if (ctx->pool.alloc((void **)&d_parts, sizeof(Part) * parts.size())) {
    d_parts = nullptr;
    return done(fail(RB_ENOMEM, "gather plan"));
  }
  if (hipMemcpyAsync(d_parts, parts.data(), sizeof(Part) * parts.size(), hipMemcpyHostToDevice, st))
    return done(fail(RB_EDEVICE, "gather plan upload"));
  const uint64_t items = assemble_items(gl);
  k_shard_header<<<(unsigned)((items + 255) / 256), 256, 0, st>>>(d_parts, (uint32_t)parts.size(), gl, d_dst);
  for (const Part &p : parts)
    if (p.body && hipMemcpyAsync(d_dst + gl.h + p.bbase, p.bytes + p.lh, p.body, hipMemcpyDeviceToDevice, st))
      return done(fail(RB_EDEVICE, "shard body copy"));
  if (hipStreamSynchronize(st)) return done(fail(RB_EDEVICE, "shard gather"));
  const hipError_t le = hipGetLastError();
  if (le != hipSuccess) return done(fail(RB_EDEVICE, "kernel launch failed: %s", hipGetErrorString(le)));
  return done(RB_OK);
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
