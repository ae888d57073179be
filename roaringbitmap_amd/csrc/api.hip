// api.hip — the C ABI of librbgpu (include/rbgpu.h): contexts, device-resident sets,
// pairwise / wide set algebra orchestration, serialization, synthetic generation.
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "format.hpp"
#include "internal.hpp"
#include "kernels.hpp"

using namespace rbg;

namespace {
thread_local std::string g_err;
} // namespace

namespace rbg {
int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int set_alloc(rbgpu_ctx *ctx, rbgpu_set *s, uint32_t nb, uint64_t nc, uint64_t payload) {
  s->ctx = ctx;
  ctx->refs++;
  s->nb = nb;
  s->nc = nc;
  s->payload_bytes = payload;
  DevPool &p = ctx->pool;
  const uint64_t ncap = std::max<uint64_t>(nc, 1);
  if (p.alloc((void **)&s->begin, (nb + 1) * sizeof(uint64_t)) != hipSuccess ||
      p.alloc((void **)&s->key, ncap * 2) != hipSuccess || p.alloc((void **)&s->type, ncap) != hipSuccess ||
      p.alloc((void **)&s->card, ncap * 4) != hipSuccess || p.alloc((void **)&s->nruns, ncap * 2) != hipSuccess ||
      p.alloc((void **)&s->off, ncap * 8) != hipSuccess ||
      p.alloc((void **)&s->payload, std::max<uint64_t>(payload, 16)) != hipSuccess) {
    // give back what was taken and the context reference: callers only `delete s` on failure
    set_release(s);
    return fail(RB_ENOMEM, "device allocation of a %u-bitmap / %llu-container set failed", nb,
                (unsigned long long)nc);
  }
  return RB_OK;
}
void set_release(rbgpu_set *s) {
  if (!s || !s->ctx) return;
  (void)settle(s); // an asynchronous result's kernels may still write its buffers
  if (s->read_done) { // ... and a pending call that takes this set as an input may still read them
    (void)hipEventSynchronize(s->read_done);
    (void)hipEventDestroy(s->read_done);
    s->read_done = nullptr;
  }
  DevPool &p = s->ctx->pool;
  p.release(s->begin);
  p.release(s->key);
  p.release(s->type);
  p.release(s->card);
  p.release(s->nruns);
  p.release(s->off);
  p.release(s->payload);
  p.release(s->mrec);
  p.release(s->krec);
  p.release(s->bsi_table);
  p.release(s->bsi_klist);
  rbgpu_ctx *ctx = s->ctx;
  s->ctx = nullptr;
  ctx_unref(ctx);
}
void ctx_unref(rbgpu_ctx *ctx) {
  if (--ctx->refs > 0) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->side) (void)hipStreamSynchronize(ctx->side);
  for (auto &e : ctx->ev) (void)hipEventDestroy(e);
  for (auto &e : ctx->ev_side) (void)hipEventDestroy(e);
  (void)hipEventDestroy(ctx->ev_tot);
  if (ctx->ev_ext) (void)hipEventDestroy(ctx->ev_ext);
  (void)hipFree(ctx->d_stats);
  (void)hipHostFree(ctx->h_pinned);
  (void)hipHostFree(ctx->h_stats);
  if (ctx->h_async) (void)hipHostFree(ctx->h_async);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->h_small) (void)hipHostFree(ctx->h_small);
  if (ctx->d_small_ctr) (void)hipFree(ctx->d_small_ctr);
  if (ctx->d_small_slots) (void)hipFree(ctx->d_small_slots);
  ctx->pool.clear();
  ctx->ws_pairs.destroy();
  ctx->ws_tasks.destroy();
  ctx->ws_segs.destroy();
  (void)hipStreamDestroy(ctx->stream);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  delete ctx;
}
int settle(const rbgpu_set *cs) {
  if (cs && cs->failed) return fail(RB_EDEVICE, "the asynchronous call that produced this set failed");
  if (!cs || !cs->pending) return RB_OK;
  rbgpu_set *s = const_cast<rbgpu_set *>(cs);
  rbgpu_ctx *ctx = s->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  const hipError_t e = hipEventSynchronize(s->pending);
  (void)hipEventDestroy(s->pending);
  s->pending = nullptr;
  // the slot is only read when the call completed; a failed call leaves the set failed (sticky), not a
  // set whose container count is whatever the pinned word held
  s->nc = e == hipSuccess ? ctx->h_async[s->pend_slot] : 0;
  ctx->async_free.push_back(s->pend_slot);
  s->pend_slot = -1;
  if (e != hipSuccess) {
    s->failed = true;
    return fail(RB_EDEVICE, "asynchronous call failed: %s", hipGetErrorString(e));
  }
  return RB_OK;
}
int ensure_h_begin(const rbgpu_set *cs) {
  rbgpu_set *s = const_cast<rbgpu_set *>(cs);
  if (s->h_begin.size() == (size_t)s->nb + 1) return RB_OK;
  s->h_begin.resize((size_t)s->nb + 1);
  HIPCHK(hipSetDevice(s->ctx->device));
  HIPCHK(hipMemcpyAsync(s->h_begin.data(), s->begin, (s->nb + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost,
                        s->ctx->stream));
  HIPCHK(hipStreamSynchronize(s->ctx->stream));
  LAUNCHCHK();
  return RB_OK;
}
// Sets are immutable, so the largest per-bitmap container count is computed once (host CSR if it
// is already here, else one reduction kernel + read-back) and cached.
int ensure_max_keys(const rbgpu_set *cs) {
  rbgpu_set *s = const_cast<rbgpu_set *>(cs);
  if (s->max_keys >= 0) return RB_OK;
  uint64_t m = 0;
  if (s->h_begin.size() == (size_t)s->nb + 1) {
    for (uint32_t i = 0; i < s->nb; ++i) m = std::max<uint64_t>(m, s->h_begin[i + 1] - s->h_begin[i]);
  } else if (s->nb) {
    HIPCHK(hipSetDevice(s->ctx->device));
    uint64_t *d = nullptr;
    if (s->ctx->pool.alloc((void **)&d, 8)) return fail(RB_ENOMEM, "max-keys word");
    HIPCHK(hipMemsetAsync(d, 0, 8, s->ctx->stream));
    launch_max_span(s->begin, s->nb, d, s->ctx->stream);
    HIPCHK(hipMemcpyAsync(s->ctx->h_pinned + 7, d, 8, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipStreamSynchronize(s->ctx->stream));
    LAUNCHCHK();
    s->ctx->pool.release(d);
    m = s->ctx->h_pinned[7];
  }
  s->max_keys = (int64_t)m;
  return RB_OK;
}
int ensure_max_runs(const rbgpu_set *cs) {
  rbgpu_set *s = const_cast<rbgpu_set *>(cs);
  if (s->max_runs >= 0) return RB_OK;
  uint64_t m = 0;
  if (s->nc) {
    HIPCHK(hipSetDevice(s->ctx->device));
    uint64_t *d = nullptr;
    if (s->ctx->pool.alloc((void **)&d, 8)) return fail(RB_ENOMEM, "max-runs word");
    HIPCHK(hipMemsetAsync(d, 0, 8, s->ctx->stream));
    launch_max_runs(s->type, s->nruns, s->nc, d, s->ctx->stream);
    HIPCHK(hipMemcpyAsync(s->ctx->h_pinned + 7, d, 8, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipStreamSynchronize(s->ctx->stream));
    LAUNCHCHK();
    s->ctx->pool.release(d);
    m = s->ctx->h_pinned[7];
  }
  s->max_runs = (int64_t)m;
  return RB_OK;
}
int ensure_dense(const rbgpu_set *cs) {
  rbgpu_set *s = const_cast<rbgpu_set *>(cs);
  if (s->dense_lo != -2) return RB_OK;
  int rc = ensure_h_begin(s);
  if (rc) return rc;
  s->dense_lo = s->dense_hi = -1;
  if (!s->nb) return RB_OK;
  const uint64_t cnt = s->h_begin[1] - s->h_begin[0];
  if (!cnt) return RB_OK;
  for (uint32_t b = 1; b < s->nb; ++b)
    if (s->h_begin[b + 1] - s->h_begin[b] != cnt) return RB_OK;
  HIPCHK(hipSetDevice(s->ctx->device));
  uint16_t k0 = 0;
  uint32_t *d = nullptr;
  if (s->ctx->pool.alloc((void **)&d, 4)) return fail(RB_ENOMEM, "dense-check word");
  hipStream_t st = s->ctx->stream;
  HIPCHK(hipMemcpyAsync(&k0, s->key + s->h_begin[0], 2, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  uint32_t bad = 1;
  if ((uint64_t)k0 + cnt <= 65536) {
    {
      DeriveTimer t(s, 0);
      HIPCHK(hipMemsetAsync(d, 0, 4, st));
      launch_dense_check(s->view(), s->nb, k0, (uint32_t)cnt, d, st);
    }
    HIPCHK(hipMemcpyAsync(&bad, d, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    LAUNCHCHK();
  }
  s->ctx->pool.release(d);
  s->derive_bytes += 2ull * s->nc; // the keys
  s->part_bytes[0] += 2ull * s->nc;
  if (!bad) {
    s->dense_lo = k0;
    s->dense_hi = (int64_t)k0 + (int64_t)cnt;
  }
  return RB_OK;
}
int ensure_mrec(const rbgpu_set *cs) {
  rbgpu_set *s = const_cast<rbgpu_set *>(cs);
  if (s->mrec) return RB_OK;
  if (s->payload_bytes >= kRecMaxPayload) return fail(RB_EINVAL, "packed records hold 40-bit payload offsets");
  HIPCHK(hipSetDevice(s->ctx->device));
  uint64_t *m = nullptr;
  if (s->ctx->pool.alloc((void **)&m, std::max<uint64_t>(s->nc, 1) * 8)) return fail(RB_ENOMEM, "packed records");
  {
    DeriveTimer t(s, 1);
    launch_pack_records(s->view(), s->nc, m, s->ctx->stream);
  }
  if (hipGetLastError() != hipSuccess) {
    s->ctx->pool.release(m);
    return fail(RB_EDEVICE, "packed-record kernel failed");
  }
  s->mrec = m;
  s->derive_bytes += 24ull * s->nc; // 16 B of metadata read, an 8-B record written per container
  s->part_bytes[1] += 24ull * s->nc;
  return RB_OK;
}
// naive_xor's key-major 4-B records of keys [a, b) into k (the set's whole dense range laid out from dense_lo).
// (Round 6 also built them in two key chunks on the side stream beside the first call's kernel: the build slowed
// the kernel beside it about as much as it hid, profiles/r06/xor/krec_overlap.)
// Member m's container at key x is begin[m] + x - dense_lo: the set's own device begin array, no host table
// copied up (a pageable 32 KiB copy cost ~0.8 ms inside the timed setup).  From mrec when the set already has it
// (12 B per container), else from the SoA itself (the run count and the offset, 10 B read, a 4-B record
// written: k_records_direct).  Returns the bytes it moves.
uint64_t build_krec_range(const rbgpu_set *s, uint32_t *k, uint32_t a, uint32_t b, hipStream_t st) {
  const SetView v = s->view();
  uint32_t *dst = k + (uint64_t)(a - (uint32_t)s->dense_lo) * s->nb;
  if (s->mrec) {
    launch_records_transpose(s->mrec, v.begin, (uint64_t)s->dense_lo, s->nb, a, b, dst, st);
    return 12ull * s->nb * (b - a);
  }
  // two containers per load: member m's first container begin[m] at an even index and the arrays aligned for it
  bool even_bases = !((uintptr_t)v.nruns & 3) && !((uintptr_t)v.off & 15) && !((a - (uint32_t)s->dense_lo) & 1);
  for (uint32_t m = 0; m < s->nb && even_bases; ++m) even_bases = !(s->h_begin[m] & 1);
  // four per load: container indices begin[m] - dense_lo + a in fours, the arrays aligned for 8-B / 16-B loads
  bool quads = !((uintptr_t)v.nruns & 7) && !((uintptr_t)v.off & 15);
  for (uint32_t m = 0; m < s->nb && quads; ++m) quads = !((s->h_begin[m] - (uint64_t)s->dense_lo + a) & 3);
  launch_records_direct(v, v.begin, (uint64_t)s->dense_lo, s->nb, a, b, dst, st, even_bases, quads);
  return 14ull * s->nb * (b - a);
}
int ensure_krec(const rbgpu_set *cs) {
  rbgpu_set *s = const_cast<rbgpu_set *>(cs);
  if (s->krec) return RB_OK;
  int rc = ensure_dense(s);
  if (rc) return rc;
  if (s->dense_lo < 0) return fail(RB_EINVAL, "key-major records need a dense set");
  HIPCHK(hipSetDevice(s->ctx->device));
  uint32_t *k = nullptr;
  if (s->ctx->pool.alloc((void **)&k, std::max<uint64_t>(s->nc, 1) * 4)) return fail(RB_ENOMEM, "key-major records");
  uint64_t bytes;
  {
    DeriveTimer t(s, 2);
    bytes = build_krec_range(s, k, (uint32_t)s->dense_lo, (uint32_t)s->dense_hi, s->ctx->stream);
  }
  if (hipGetLastError() != hipSuccess) {
    s->ctx->pool.release(k);
    return fail(RB_EDEVICE, "key-major record kernel failed");
  }
  s->krec = k;
  s->derive_bytes += bytes;
  s->part_bytes[2] += bytes;
  return RB_OK;
}
} // namespace rbg

namespace {
// Upload a validated host SoA, re-laid out: Bitmaps first (8 KiB aligned), then the rest (16 B).
int upload_host(rbgpu_ctx *ctx, const HostSoA &h, rbgpu_set **out) {
  const uint64_t nc = h.nc();
  std::vector<uint64_t> off(nc);
  uint64_t nbig = 0, small = 0;
  for (uint64_t i = 0; i < nc; ++i) {
    if (h.type[i] == RB_BITMAP) ++nbig;
    else small += round16(payload_bytes(h.type[i], h.card[i], h.nruns[i]));
  }
  uint64_t bi = 0, so = nbig * kBitmapBytes;
  for (uint64_t i = 0; i < nc; ++i) {
    if (h.type[i] == RB_BITMAP) off[i] = (bi++) * kBitmapBytes;
    else {
      off[i] = so;
      so += round16(payload_bytes(h.type[i], h.card[i], h.nruns[i]));
    }
  }
  const uint64_t total = nbig * kBitmapBytes + small;
  // a run count only on Run containers: workShyAnd's SoA reads and naive_xor's records take "nruns > 0" for
  // "a Run", so an Array / Bitmap entry's count (which the format ignores) is stored as 0
  std::vector<uint16_t> nruns(h.nruns.begin(), h.nruns.begin() + nc);
  for (uint64_t i = 0; i < nc; ++i)
    if (h.type[i] != RB_RUN) nruns[i] = 0;
  std::vector<uint8_t> staged(std::max<uint64_t>(total, 16), 0);
  for (uint64_t i = 0; i < nc; ++i)
    std::memcpy(staged.data() + off[i], h.payload.data() + h.off[i], payload_bytes(h.type[i], h.card[i], h.nruns[i]));
  rbgpu_set *s = new rbgpu_set;
  int rc = set_alloc(ctx, s, h.nb, nc, total);
  if (rc) {
    delete s;
    return rc;
  }
  hipStream_t st = ctx->stream;
  auto cp = [&](void *dst, const void *src, size_t n) {
    return n ? hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st) : hipSuccess;
  };
  if (cp(s->begin, h.begin.data(), (h.nb + 1) * 8) || cp(s->key, h.key.data(), nc * 2) ||
      cp(s->type, h.type.data(), nc) || cp(s->card, h.card.data(), nc * 4) || cp(s->nruns, nruns.data(), nc * 2) ||
      cp(s->off, off.data(), nc * 8) || cp(s->payload, staged.data(), total) || hipStreamSynchronize(st)) {
    set_release(s);
    delete s;
    return fail(RB_EDEVICE, "host-to-device upload failed");
  }
  s->h_begin = h.begin;
  *out = s;
  return RB_OK;
}

// Download bitmaps [first, first+count) into a HostSoA with compact 16-B aligned payloads.
int download_host(const rbgpu_set *s, uint32_t first, uint32_t count, HostSoA &h) {
  rbgpu_ctx *ctx = s->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  int rc = ensure_h_begin(s);
  if (rc) return rc;
  const uint64_t lo = s->h_begin[first], hi = s->h_begin[first + count], n = hi - lo;
  hipStream_t st = ctx->stream;
  h.nb = count;
  h.begin.resize(count + 1);
  for (uint32_t i = 0; i <= count; ++i) h.begin[i] = s->h_begin[first + i] - lo;
  h.key.resize(n);
  h.type.resize(n);
  h.card.resize(n);
  h.nruns.resize(n);
  h.off.resize(n);
  std::vector<uint64_t> soff(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(h.key.data(), s->key + lo, n * 2, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h.type.data(), s->type + lo, n, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h.card.data(), s->card + lo, n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(h.nruns.data(), s->nruns + lo, n * 2, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(soff.data(), s->off + lo, n * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    LAUNCHCHK();
  }
  std::vector<uint64_t> bytes(n);
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) {
    bytes[i] = payload_bytes(h.type[i], h.card[i], h.nruns[i]);
    h.off[i] = total;
    total += round16(bytes[i]);
  }
  h.payload.assign(std::max<uint64_t>(total, 16), 0);
  if (n) {
    uint64_t *d_soff, *d_doff, *d_bytes;
    uint8_t *d_stage;
    if (ctx->pool.alloc((void **)&d_soff, n * 8) || ctx->pool.alloc((void **)&d_doff, n * 8) ||
        ctx->pool.alloc((void **)&d_bytes, n * 8) || ctx->pool.alloc((void **)&d_stage, std::max<uint64_t>(total, 16)))
      return fail(RB_ENOMEM, "download staging allocation failed");
    HIPCHK(hipMemcpyAsync(d_soff, soff.data(), n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_doff, h.off.data(), n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_bytes, bytes.data(), n * 8, hipMemcpyHostToDevice, st));
    launch_gather(s->payload, d_soff, d_bytes, d_stage, d_doff, n, st);
    HIPCHK(hipMemcpyAsync(h.payload.data(), d_stage, total, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    LAUNCHCHK();
    ctx->pool.release(d_soff);
    ctx->pool.release(d_doff);
    ctx->pool.release(d_bytes);
    ctx->pool.release(d_stage);
  }
  return RB_OK;
}

int check_ctx(rbgpu_ctx *ctx) {
  if (!ctx) return fail(RB_EINVAL, "null context");
  HIPCHK(hipSetDevice(ctx->device));
  (void)hipGetLastError(); // LAUNCHCHK reports only what this call launches
  return RB_OK;
}

} // namespace

namespace rbg {
// Only the min/max shortcut answers of a key-range BSI shard come here (a copy of ebM or foundSet,
// restricted); the containers stay bytes-identical.
int set_key_subset(const rbgpu_set *s, uint32_t key_lo, uint32_t key_hi, rbgpu_set **out) {
  HostSoA h;
  int rc = download_host(s, 0, 1, h);
  if (rc) return rc;
  HostSoA r;
  r.nb = 1;
  r.begin.assign(2, 0);
  for (uint64_t i = 0; i < h.nc(); ++i) {
    if (h.key[i] < key_lo || h.key[i] >= key_hi) continue;
    const uint64_t bytes = payload_bytes(h.type[i], h.card[i], h.nruns[i]);
    r.key.push_back(h.key[i]);
    r.type.push_back(h.type[i]);
    r.card.push_back(h.card[i]);
    r.nruns.push_back(h.nruns[i]);
    r.off.push_back(r.payload.size());
    r.payload.insert(r.payload.end(), h.payload.begin() + h.off[i], h.payload.begin() + h.off[i] + round16(bytes));
  }
  r.begin[1] = r.key.size();
  return upload_host(s->ctx, r, out);
}

// Bitmaps idx[0..n) of s as a new set, in that order (a device-resident copy through the host; the
// containers stay bytes-identical, empty ones included).
int set_gather(const rbgpu_set *s, const uint32_t *idx, uint32_t n, rbgpu_set **out) {
  for (uint32_t i = 0; i < n; ++i)
    if (idx[i] >= s->nb) return fail(RB_EINVAL, "bitmap %u out of range", idx[i]);
  HostSoA h;
  int rc = s->nb ? download_host(s, 0, s->nb, h) : RB_OK;
  if (rc) return rc;
  HostSoA r;
  r.nb = n;
  r.begin.assign(1, 0);
  for (uint32_t k = 0; k < n; ++k) {
    for (uint64_t i = h.begin[idx[k]]; i < h.begin[idx[k] + 1]; ++i) {
      const uint64_t bytes = payload_bytes(h.type[i], h.card[i], h.nruns[i]);
      r.key.push_back(h.key[i]);
      r.type.push_back(h.type[i]);
      r.card.push_back(h.card[i]);
      r.nruns.push_back(h.nruns[i]);
      r.off.push_back(r.payload.size());
      r.payload.insert(r.payload.end(), h.payload.begin() + h.off[i], h.payload.begin() + h.off[i] + round16(bytes));
    }
    r.begin.push_back(r.key.size());
  }
  return upload_host(s->ctx, r, out);
}

// The counters are zeroed right behind their read-back in stats_end (the memset runs while the host
// waits anyway), so the next call starts its kernels without one; a call that did not reach
// stats_end leaves them dirty and the next stats_begin zeroes them.
void stats_begin(rbgpu_ctx *ctx, bool zero) {
  ctx->stats_pending = false;
  if (zero && !ctx->stats_clean)
    (void)hipMemsetAsync(ctx->d_stats, 0, kStatWords * kStripes * sizeof(uint64_t), ctx->stream);
  ctx->stats_clean = false;
  (void)hipEventRecord(ctx->ev[0], ctx->stream);
}
int stats_end(rbgpu_ctx *ctx, uint64_t tasks, uint64_t result_containers, const KernelSpan *k, int n,
              const uint64_t *d_src) {
  HIPCHK(hipEventRecord(ctx->ev[5], ctx->stream));
  HIPCHK(hipMemcpyAsync(ctx->h_stats, d_src ? d_src : ctx->d_stats, kStatWords * kStripes * sizeof(uint64_t),
                        hipMemcpyDeviceToHost, ctx->stream));
  if (!d_src) HIPCHK(hipMemsetAsync(ctx->d_stats, 0, kStatWords * kStripes * sizeof(uint64_t), ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  LAUNCHCHK();
  if (!d_src) ctx->stats_clean = true;
  uint64_t *w = ctx->words;
  for (int i = 0; i < kStatWords; ++i) {
    w[i] = 0;
    for (int j = 0; j < kStripes; ++j) w[i] += ctx->h_stats[i * kStripes + j];
  }
  return stats_fill(ctx, tasks, result_containers, k, n);
}
int stats_fill(rbgpu_ctx *ctx, uint64_t tasks, uint64_t result_containers, const KernelSpan *k, int n, bool timed) {
  ctx->stats_pending = false;
  ctx->pend_n = 0;
  const uint64_t *w = ctx->words;
  rb_stats &s = ctx->last;
  s = rb_stats{};
  s.tasks = tasks;
  s.input_bytes = w[0];
  s.output_bytes = w[1];
  s.result_cardinality = w[7];
  s.result_containers = result_containers;
  float ms = 0;
  s.total_ms = timed && hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[5]) == hipSuccess ? ms : 0.0;
  s.n_kernels = (uint32_t)std::min(n, 4);
  int best = -1;
  for (int i = 0; i < (int)s.n_kernels; ++i) {
    std::snprintf(s.kernel_name[i], sizeof s.kernel_name[i], "%s", k[i].name);
    hipEvent_t e0 = k[i].e0 ? k[i].e0 : ctx->ev[1 + i], e1 = k[i].e1 ? k[i].e1 : ctx->ev[2 + i];
    s.kernel_ms[i] = timed && hipEventElapsedTime(&ms, e0, e1) == hipSuccess ? ms : 0.0;
    s.kernel_bytes[i] = (k[i].in_word >= 0 ? w[k[i].in_word] : 0) + (k[i].out_word >= 0 ? w[k[i].out_word] : 0) +
                        (k[i].in2 >= 0 ? w[k[i].in2] : 0) + (k[i].out2 >= 0 ? w[k[i].out2] : 0);
    s.kernel_items[i] = k[i].items;
    if (best < 0 || s.kernel_ms[i] > s.kernel_ms[best]) best = i;
  }
  if (best >= 0) {
    s.main_kernel_ms = s.kernel_ms[best];
    s.main_kernel_bytes = s.kernel_bytes[best];
    std::snprintf(s.main_kernel, sizeof s.main_kernel, "%s", s.kernel_name[best]);
  }
  return RB_OK;
}
// Host-visible result words a one-launch call's last block writes (8 words: [5] = the call's sequence
// number, written last) and the device counters it resets (pairwise_small, the fused BSI compare).
int ensure_call_words(rbgpu_ctx *ctx) {
  if (!ctx->h_small) {
    if (hipHostMalloc((void **)&ctx->h_small, 256, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return fail(RB_ENOMEM, "host-visible result words");
    if (hipHostGetDevicePointer((void **)&ctx->d_small, ctx->h_small, 0) != hipSuccess) {
      (void)hipHostFree(ctx->h_small);
      ctx->h_small = nullptr;
      return fail(RB_EDEVICE, "host-visible result words have no device address");
    }
  }
  if (!ctx->d_small_ctr) { // block tickets and counters of the one-launch kernels; each call's last block resets its own
    if (hipMalloc((void **)&ctx->d_small_ctr, 512) != hipSuccess) return fail(RB_ENOMEM, "block counters");
    if (hipMemset(ctx->d_small_ctr, 0, 512) != hipSuccess) return fail(RB_EDEVICE, "block counters");
  }
  if (!ctx->d_small_slots) { // every word kSlotUnset (all ones) between calls: each call's compaction resets its own
    if (hipMalloc((void **)&ctx->d_small_slots, 16ull * kSmallSlots) != hipSuccess) return fail(RB_ENOMEM, "slot words");
    if (hipMemset(ctx->d_small_slots, 0xFF, 16ull * kSmallSlots) != hipSuccess) return fail(RB_EDEVICE, "slot words");
  }
  return RB_OK;
}
// Spins (bounded) until the call's last block has written `seq` after its result words: the host returns
// without waiting for the kernel's end to be signalled (it has no work left by then, and later calls on the
// stream are ordered behind it).  false: not seen in time — the caller waits for the stream, which also
// reports a fault.
bool wait_call_seq(rbgpu_ctx *ctx, uint64_t seq, int word) {
  const volatile uint64_t *flag = reinterpret_cast<const volatile uint64_t *>(ctx->h_small) + word;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t it = 0;; ++it) {
    if (__atomic_load_n(const_cast<const uint64_t *>(flag), __ATOMIC_ACQUIRE) == seq) return true;
    if ((it & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) return false;
  }
}
int seq_begin(rbgpu_ctx *ctx) {
  if (ctx->seq_settled >= ctx->seq_recorded) return RB_OK;
  const hipError_t q = hipEventQuery(ctx->ev[5]);
  if (q == hipSuccess) {
    ctx->seq_settled = ctx->seq_recorded;
    return RB_OK;
  }
  if (q == hipErrorNotReady) return RB_OK; // still running: this call's work queues behind it
  (void)hipGetLastError();
  return fail(RB_EDEVICE, "an earlier one-launch call's kernel failed after the call returned: %s", hipGetErrorString(q));
}
int seq_end(rbgpu_ctx *ctx, uint64_t seq, bool poll, const char *what, bool *seen, int word) {
  *seen = false;
  ctx->seq_recorded = seq; // ctx->ev[5], recorded by the caller behind the kernel, marks its end
  const bool s = poll && wait_call_seq(ctx, seq, word);
  const hipError_t e1 = s ? hipSuccess : hipStreamSynchronize(ctx->stream), e2 = hipGetLastError();
  if (e1 != hipSuccess || e2 != hipSuccess)
    return fail(RB_EDEVICE, "%s kernel failed: %s", what, hipGetErrorString(e1 != hipSuccess ? e1 : e2));
  if (!s) {
    ctx->seq_settled = seq;
    const uint64_t got = __atomic_load_n(reinterpret_cast<const uint64_t *>(ctx->h_small) + word, __ATOMIC_ACQUIRE);
    if (got != seq) { // no block saw itself last: the counters are not this call's, and nor are the words
      (void)hipMemsetAsync(ctx->d_small_ctr, 0, 512, ctx->stream);
      if (ctx->d_small_slots) (void)hipMemsetAsync(ctx->d_small_slots, 0xFF, 16ull * kSmallSlots, ctx->stream);
      (void)hipStreamSynchronize(ctx->stream);
      return fail(RB_EDEVICE, "%s: the kernel ended without handing over call %llu's result words (found %llu)", what,
                  (unsigned long long)seq, (unsigned long long)got);
    }
  }
  *seen = s;
  return RB_OK;
}
int seq_settle(rbgpu_ctx *ctx, uint64_t seq) {
  if (!seq || seq <= ctx->seq_settled) return RB_OK;
  const hipError_t e = hipEventSynchronize(ctx->ev[5]); // recorded behind call seq or a later one
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(RB_EDEVICE, "one-launch kernel failed: %s", hipGetErrorString(e));
  }
  ctx->seq_settled = ctx->seq_recorded;
  return RB_OK;
}
} // namespace rbg

// ===================================================================== C ABI
extern "C" {

const char *rbgpu_last_error(void) { return g_err.c_str(); }

int rbgpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int rbgpu_open(int device, rbgpu_ctx **out) {
  if (!out) return fail(RB_EINVAL, "null out");
  *out = nullptr;
  int n = rbgpu_device_count();
  if (device < 0 || device >= n) return fail(RB_EDEVICE, "no HIP device %d (found %d)", device, n);
  HIPCHK(hipSetDevice(device));
  rbgpu_ctx *c = new rbgpu_ctx;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void **)&c->d_stats, kStatWords * kStripes * sizeof(uint64_t)) != hipSuccess ||
      hipHostMalloc((void **)&c->h_stats, kStatWords * kStripes * sizeof(uint64_t)) != hipSuccess ||
      hipHostMalloc((void **)&c->h_pinned, 16 * sizeof(uint64_t)) != hipSuccess) {
    delete c;
    return fail(RB_EDEVICE, "context creation failed on device %d", device);
  }
  for (auto &e : c->ev) (void)hipEventCreate(&e);
  for (auto &e : c->ev_side) (void)hipEventCreate(&e);
  (void)hipEventCreate(&c->ev_tot);
  (void)hipEventCreateWithFlags(&c->ev_ext, hipEventDisableTiming);
  // every source file's code object now, not inside the first call of each kind: HIP loads a code object at
  // the first launch of one of its kernels (~1 ms each), which otherwise lands in that call's time and in a
  // set's first-use setup (rbgpu_set_setup_parts)
  for (auto w : {warm_pairwise, warm_scan, warm_wide, warm_wide_runs, warm_wide_xor, warm_bsi, warm_codec, warm_setops,
                 warm_generate})
    w(c->stream);
  if (hipStreamSynchronize(c->stream) != hipSuccess || hipGetLastError() != hipSuccess) {
    rbgpu_close(c);
    return fail(RB_EDEVICE, "context creation failed on device %d (kernel load)", device);
  }
  *out = c;
  return RB_OK;
}

void rbgpu_close(rbgpu_ctx *ctx) {
  // sets still alive keep the context (stream, pool) alive until they are freed
  if (!ctx || ctx->closed) return;
  ctx->closed = true;
  ctx_unref(ctx);
}

int rbgpu_synchronize(rbgpu_ctx *ctx) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(ctx->stream));
  LAUNCHCHK();
  return RB_OK;
}

int rbgpu_get_stats(rbgpu_ctx *ctx, rb_stats *out) {
  if (!ctx || !out) return fail(RB_EINVAL, "null argument");
  if (ctx->stats_pending) { // a small batch returned before its end was signalled: its times now
    ctx->stats_pending = false;
    float ms = 0.f;
    const hipError_t e = hipEventSynchronize(ctx->ev[5]);
    if (e != hipSuccess) { // the kernel faulted after its last block handed the result over
      (void)hipGetLastError();
      return fail(RB_EDEVICE, "the last call's kernel failed after the call returned: %s", hipGetErrorString(e));
    }
    ctx->seq_settled = std::max(ctx->seq_settled, ctx->seq_recorded); // ev[5] follows the last one-launch kernel
    if (ctx->pend_n) { // a general-pipeline call's spans (CallTail): the same accounting as stats_end, now timed
      const rb_stats keep = ctx->last;
      KernelSpan spans[4];
      const int n = ctx->pend_n;
      for (int i = 0; i < n; ++i) spans[i] = ctx->pend_spans[i];
      (void)stats_fill(ctx, ctx->pend_tasks, keep.result_containers, spans, n, true);
      ctx->last.call_us = keep.call_us;
    } else {
      if (hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[5]) == hipSuccess) ctx->last.total_ms = ms;
      if (ctx->stats_pending_k && hipEventElapsedTime(&ms, ctx->ev[1], ctx->ev[2]) == hipSuccess)
        ctx->last.kernel_ms[0] = ctx->last.main_kernel_ms = ms;
    }
  }
  *out = ctx->last;
  return RB_OK;
}

// RBGPU_HOST_CODEC=1 selects the host parser / writer (format.cpp) instead of codec.hip — an A/B
// switch for tests; both give identical sets, bytes and error codes.
static bool host_codec() {
  const char *e = std::getenv("RBGPU_HOST_CODEC");
  return e && e[0] == '1';
}

int rbgpu_set_from_serialized(rbgpu_ctx *ctx, const uint8_t *const *bufs, const uint64_t *lens, uint32_t n,
                              rbgpu_set **out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!out || (n && (!bufs || !lens))) return fail(RB_EINVAL, "null argument");
  if (host_codec()) {
    HostSoA h;
    std::string err;
    for (uint32_t i = 0; i < n; ++i) {
      rc = parse_serialized(bufs[i], lens[i], h, err);
      if (rc) return fail(rc, "bitmap %u: %s", i, err.c_str());
    }
    return upload_host(ctx, h, out);
  }
  // one host-to-device copy of the concatenated bytes, parsed on the GPU
  std::vector<uint64_t> off(n + 1ull, 0);
  for (uint32_t i = 0; i < n; ++i) off[i + 1] = off[i] + lens[i];
  const uint64_t total = off[n];
  uint8_t *pin = nullptr, *d_in = nullptr;
  uint64_t *d_off = nullptr;
  DevPool &pool = ctx->pool;
  if (hipHostMalloc((void **)&pin, std::max<uint64_t>(total, 4) + 8 * (n + 1ull)) != hipSuccess)
    return fail(RB_ENOMEM, "pinned staging of %llu bytes", (unsigned long long)total);
  for (uint32_t i = 0; i < n; ++i)
    if (lens[i]) std::memcpy(pin + off[i], bufs[i], lens[i]);
  uint8_t *pin_off = pin + std::max<uint64_t>(total, 4);
  std::memcpy(pin_off, off.data(), 8 * (n + 1ull));
  if (pool.alloc((void **)&d_in, ((total + 3) & ~3ull) + 4) || pool.alloc((void **)&d_off, 8 * (n + 1ull))) {
    (void)hipHostFree(pin);
    pool.release(d_in);
    return fail(RB_ENOMEM, "device staging of %llu bytes", (unsigned long long)total);
  }
  hipStream_t st = ctx->stream;
  if ((total && hipMemcpyAsync(d_in, pin, total, hipMemcpyHostToDevice, st)) ||
      hipMemcpyAsync(d_off, pin_off, 8 * (n + 1ull), hipMemcpyHostToDevice, st)) {
    (void)hipStreamSynchronize(st);
    (void)hipHostFree(pin);
    pool.release(d_in);
    pool.release(d_off);
    return fail(RB_EDEVICE, "host-to-device copy failed");
  }
  rc = deserialize_device(ctx, d_in, total, d_off, n, out);
  (void)hipStreamSynchronize(st);
  (void)hipHostFree(pin);
  pool.release(d_in);
  pool.release(d_off);
  return rc;
}

int rbgpu_set_from_serialized_device(rbgpu_ctx *ctx, const uint8_t *d_bytes, const uint64_t *offsets, uint32_t n,
                                     rbgpu_set **out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!out || !offsets || (n && !d_bytes)) return fail(RB_EINVAL, "null argument");
  for (uint32_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return fail(RB_EINVAL, "offsets not monotone at %u", i);
  uint64_t *d_off = nullptr;
  if (ctx->pool.alloc((void **)&d_off, 8 * (n + 1ull))) return fail(RB_ENOMEM, "offsets");
  hipStream_t st = ctx->stream;
  if (hipMemcpyAsync(d_off, offsets, 8 * (n + 1ull), hipMemcpyHostToDevice, st)) {
    ctx->pool.release(d_off);
    return fail(RB_EDEVICE, "host-to-device copy failed");
  }
  rc = deserialize_device(ctx, d_bytes, offsets[n], d_off, n, out);
  (void)hipStreamSynchronize(st);
  ctx->pool.release(d_off);
  return rc;
}

int rbgpu_set_from_soa(rbgpu_ctx *ctx, const rb_soa *soa, rbgpu_set **out) {
  return rbg::set_from_soa(ctx, soa, out, false);
}
}  // extern "C"

namespace rbg {
// allow_empty: an empty Array (card 0, no payload) or Run (card 0, no runs) is kept — the containers a
// Roaring64Bitmap xor leaves under their keys, read back from its own serialized form (set64.hip)
int set_from_soa(rbgpu_ctx *ctx, const rb_soa *soa, rbgpu_set **out, bool allow_empty) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!soa || !out) return fail(RB_EINVAL, "null argument");
  HostSoA h;
  h.nb = soa->n_bitmaps;
  h.begin.assign(soa->begin, soa->begin + soa->n_bitmaps + 1);
  if (h.begin[0] != 0 || h.begin[h.nb] != soa->n_containers) return fail(RB_EINVAL, "bad CSR begin array");
  const uint64_t nc = soa->n_containers;
  h.key.assign(soa->key, soa->key + nc);
  h.type.assign(soa->type, soa->type + nc);
  h.card.assign(soa->card, soa->card + nc);
  h.nruns.assign(soa->nruns, soa->nruns + nc);
  h.off.resize(nc);
  std::string err;
  for (uint32_t b = 0; b < h.nb; ++b) {
    if (h.begin[b + 1] < h.begin[b]) return fail(RB_EINVAL, "bad CSR begin array");
    for (uint64_t i = h.begin[b]; i < h.begin[b + 1]; ++i)
      if (i > h.begin[b] && h.key[i] <= h.key[i - 1]) return fail(RB_EINVAL, "bitmap %u: keys not increasing", b);
  }
  for (uint64_t i = 0; i < nc; ++i) {
    const uint64_t bytes = payload_bytes(h.type[i], h.card[i], h.nruns[i]);
    if (soa->offset[i] + bytes > soa->payload_bytes) return fail(RB_EINVAL, "container %llu payload out of range", (unsigned long long)i);
    const bool empty_ok = allow_empty && h.card[i] == 0 && h.type[i] != RB_BITMAP && h.nruns[i] == 0;
    rc = empty_ok ? RB_OK : validate_container(h.type[i], h.card[i], h.nruns[i], soa->payload + soa->offset[i], err);
    if (rc) return fail(rc, "container %llu: %s", (unsigned long long)i, err.c_str());
    h.off[i] = soa->offset[i];
  }
  h.payload.assign(soa->payload, soa->payload + soa->payload_bytes);
  return upload_host(ctx, h, out);
}
}  // namespace rbg

extern "C" {

void rbgpu_set_free(rbgpu_set *set) {
  if (!set) return;
  set_release(set);
  delete set;
}
uint32_t rbgpu_set_bitmap_count(const rbgpu_set *s) { return s ? s->nb : 0; }
uint64_t rbgpu_set_container_count(const rbgpu_set *s) { return s && !settle(s) ? s->nc : 0; }
uint64_t rbgpu_set_payload_capacity(const rbgpu_set *s) { return s ? s->payload_bytes : 0; }

int rbgpu_set_cardinalities(const rbgpu_set *s, uint64_t *out) {
  SETTLE(s);
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  rbgpu_ctx *ctx = s->ctx;
  int rc = check_ctx(ctx);
  if (rc) return rc;
  uint64_t *d;
  if (ctx->pool.alloc((void **)&d, std::max<uint64_t>(s->nb, 1) * 8)) return fail(RB_ENOMEM, "alloc");
  launch_bitmap_cards(s->view(), s->nb, d, ctx->stream);
  HIPCHK(hipMemcpyAsync(out, d, s->nb * 8ull, hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  LAUNCHCHK();
  ctx->pool.release(d);
  return RB_OK;
}

int rbgpu_set_download(const rbgpu_set *s, uint32_t first, uint32_t count, rb_soa *soa) {
  SETTLE(s);
  if (!s || !soa) return fail(RB_EINVAL, "null argument");
  if ((uint64_t)first + count > s->nb) return fail(RB_EINVAL, "bitmap range out of bounds");
  HostSoA h;
  int rc = download_host(s, first, count, h);
  if (rc) return rc;
  if (!soa->key) { // size query
    soa->n_bitmaps = count;
    soa->n_containers = h.nc();
    soa->payload_bytes = h.payload.size();
    return RB_OK;
  }
  if (soa->n_containers < h.nc() || soa->payload_bytes < h.payload.size())
    return fail(RB_EINVAL, "rb_soa buffers too small");
  soa->n_bitmaps = count;
  soa->n_containers = h.nc();
  soa->payload_bytes = h.payload.size();
  std::memcpy(soa->begin, h.begin.data(), (count + 1) * 8ull);
  std::memcpy(soa->key, h.key.data(), h.nc() * 2);
  std::memcpy(soa->type, h.type.data(), h.nc());
  std::memcpy(soa->card, h.card.data(), h.nc() * 4);
  std::memcpy(soa->nruns, h.nruns.data(), h.nc() * 2);
  std::memcpy(soa->offset, h.off.data(), h.nc() * 8);
  std::memcpy(soa->payload, h.payload.data(), h.payload.size());
  return RB_OK;
}

int rbgpu_set_serialized_sizes(const rbgpu_set *s, uint64_t *out) {
  SETTLE(s);
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  int rc = check_ctx(s->ctx);
  if (rc) return rc;
  rc = ensure_h_begin(s);
  if (rc) return rc;
  // sizes need only metadata: download types / cards / nruns
  const uint64_t n = s->nc;
  std::vector<uint8_t> type(n);
  std::vector<uint16_t> nruns(n);
  std::vector<uint32_t> card(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(type.data(), s->type, n, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(nruns.data(), s->nruns, n * 2, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(card.data(), s->card, n * 4, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipStreamSynchronize(s->ctx->stream));
    LAUNCHCHK();
  }
  for (uint32_t b = 0; b < s->nb; ++b) {
    const uint64_t lo = s->h_begin[b], hi = s->h_begin[b + 1], k = hi - lo;
    bool hasrun = false;
    uint64_t bytes = 0;
    for (uint64_t i = lo; i < hi; ++i) {
      hasrun |= type[i] == RB_RUN;
      bytes += type[i] == RB_ARRAY ? 2ull * card[i] : type[i] == RB_BITMAP ? 8192 : 2 + 4ull * nruns[i];
    }
    out[b] = (hasrun ? (k < 4 ? 4 + (k + 7) / 8 + 4 * k : 4 + (k + 7) / 8 + 8 * k) : 8 + 8 * k) + bytes;
  }
  return RB_OK;
}

int rbgpu_set_summaries(const rbgpu_set *s, uint32_t first, uint32_t count, rb_bitmap_summary *out) {
  SETTLE(s);
  if (!s || (count && !out)) return fail(RB_EINVAL, "null argument");
  if ((uint64_t)first + count > s->nb) return fail(RB_EINVAL, "bitmap range out of bounds");
  int rc = check_ctx(s->ctx);
  if (rc) return rc;
  rc = ensure_h_begin(s);
  if (rc) return rc;
  const uint64_t lo = s->h_begin[first], n = s->h_begin[first + count] - lo;
  std::vector<uint16_t> nruns(n);
  std::vector<uint8_t> type(n);
  std::vector<uint32_t> card(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(type.data(), s->type + lo, n, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(nruns.data(), s->nruns + lo, n * 2, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(card.data(), s->card + lo, n * 4, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipStreamSynchronize(s->ctx->stream));
    LAUNCHCHK();
  }
  for (uint32_t b = 0; b < count; ++b) {
    rb_bitmap_summary &o = out[b];
    o = rb_bitmap_summary{};
    o.size_in_bytes = 8;
    for (uint64_t i = s->h_begin[first + b] - lo; i < s->h_begin[first + b + 1] - lo; ++i) {
      o.cardinality += card[i];
      o.n_containers += 1;
      o.n_run_containers += type[i] == RB_RUN;
      o.payload_bytes += type[i] == RB_BITMAP ? 8192ull : type[i] == RB_ARRAY ? 2ull * card[i] : 2 + 4ull * nruns[i];
      // 2 key bytes + Container.getSizeInBytes: Array 2c + 4, Bitmap 8192, Run 4r + 4
      o.size_in_bytes += 2 + (type[i] == RB_BITMAP ? 8192ull : type[i] == RB_ARRAY ? 2ull * card[i] + 4 : 4ull * nruns[i] + 4);
    }
  }
  return RB_OK;
}

int rbgpu_set_type_stats(const rbgpu_set *s, uint64_t *out) {
  SETTLE(s);
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  int rc = check_ctx(s->ctx);
  if (rc) return rc;
  const uint64_t n = s->nc;
  std::vector<uint16_t> nruns(n);
  std::vector<uint8_t> type(n);
  std::vector<uint32_t> card(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(type.data(), s->type, n, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(nruns.data(), s->nruns, n * 2, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(card.data(), s->card, n * 4, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipStreamSynchronize(s->ctx->stream));
  }
  std::fill(out, out + 6, 0ull);
  for (uint64_t i = 0; i < n; ++i) {
    const int t = type[i] <= RB_RUN ? type[i] : RB_RUN;
    out[t] += 1;
    out[3 + t] += t == RB_BITMAP ? 8192ull : t == RB_ARRAY ? 2ull * card[i] : 2 + 4ull * nruns[i];
  }
  return RB_OK;
}

// containers of each member with high key in [lo, hi): two binary searches over its sorted keys
__global__ void k_range_counts(const uint64_t *begin, const uint16_t *key, const uint32_t *members, uint32_t n,
                               uint32_t lo, uint32_t hi, uint64_t *out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t m = members ? members[i] : i;
  const uint64_t b = begin[m], e = begin[m + 1];
  auto lower = [&](uint32_t k) {
    uint64_t l = b, h = e;
    while (l < h) {
      const uint64_t mid = (l + h) >> 1;
      if (key[mid] < k) l = mid + 1;
      else h = mid;
    }
    return l;
  };
  out[i] = lower(hi) - lower(lo);
}

int rbgpu_set_range_counts(const rbgpu_set *s, const uint32_t *members, uint32_t n, uint32_t key_lo, uint32_t key_hi,
                           uint64_t *out) {
  SETTLE(s);
  if (!s || (n && !out)) return fail(RB_EINVAL, "null argument");
  if (key_lo > key_hi || key_hi > 65536u) return fail(RB_EINVAL, "key range [%u, %u) outside [0, 65536]", key_lo, key_hi);
  if (!members && n != s->nb) return fail(RB_EINVAL, "without a member list n must be the bitmap count");
  for (uint32_t i = 0; members && i < n; ++i)
    if (members[i] >= s->nb) return fail(RB_EINVAL, "member %u out of range", members[i]);
  int rc = check_ctx(s->ctx);
  if (rc) return rc;
  if (!n) return RB_OK;
  HIPCHK(hipSetDevice(s->ctx->device));
  uint32_t *d_m = nullptr;
  uint64_t *d_out = nullptr;
  if ((members && s->ctx->pool.alloc((void **)&d_m, 4ull * n)) || s->ctx->pool.alloc((void **)&d_out, 8ull * n)) {
    if (d_m) s->ctx->pool.release(d_m);
    return fail(RB_ENOMEM, "range counts");
  }
  hipStream_t st = s->ctx->stream;
  if (members) HIPCHK(hipMemcpyAsync(d_m, members, 4ull * n, hipMemcpyHostToDevice, st));
  k_range_counts<<<(n + 255) / 256, 256, 0, st>>>(s->begin, s->key, d_m, n, key_lo, key_hi, d_out);
  HIPCHK(hipMemcpyAsync(out, d_out, 8ull * n, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  LAUNCHCHK();
  if (d_m) s->ctx->pool.release(d_m);
  s->ctx->pool.release(d_out);
  return RB_OK;
}

int rbgpu_set_key_bytes(const rbgpu_set *s, uint64_t *out) {
  SETTLE(s);
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  int rc = check_ctx(s->ctx);
  if (rc) return rc;
  const uint64_t n = s->nc;
  std::vector<uint16_t> key(n), nruns(n);
  std::vector<uint8_t> type(n);
  std::vector<uint32_t> card(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(key.data(), s->key, n * 2, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(type.data(), s->type, n, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(nruns.data(), s->nruns, n * 2, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(card.data(), s->card, n * 4, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipStreamSynchronize(s->ctx->stream));
    LAUNCHCHK();
  }
  std::fill(out, out + 65536, 0ull);
  for (uint64_t i = 0; i < n; ++i)
    out[key[i]] += (type[i] == RB_BITMAP ? 8192ull : type[i] == RB_ARRAY ? 2ull * card[i] : 4ull * nruns[i] + 2) + 16;
  return RB_OK;
}

int rbgpu_set_serialize(const rbgpu_set *s, uint32_t first, uint32_t count, uint8_t *dst, uint64_t cap,
                        uint64_t *offsets) {
  SETTLE(s);
  if (!s || (count && !dst)) return fail(RB_EINVAL, "null argument");
  if ((uint64_t)first + count > s->nb) return fail(RB_EINVAL, "bitmap range out of bounds");
  int rc = check_ctx(s->ctx);
  if (rc) return rc;
  if (!host_codec()) return serialize_device(s, first, count, dst, cap, offsets, true);
  HostSoA h;
  rc = download_host(s, first, count, h);
  if (rc) return rc;
  uint64_t pos = 0;
  for (uint32_t b = 0; b < count; ++b) {
    const uint64_t k = serialized_size(h, b);
    if (pos + k > cap) return fail(RB_EINVAL, "destination buffer too small (%llu needed)", (unsigned long long)(pos + k));
    if (offsets) offsets[b] = pos;
    serialize_bitmap(h, b, dst + pos);
    pos += k;
  }
  if (offsets) offsets[count] = pos;
  return RB_OK;
}

int rbgpu_set_serialize_device(const rbgpu_set *s, uint32_t first, uint32_t count, uint8_t *d_dst, uint64_t cap,
                               uint64_t *offsets) {
  SETTLE(s);
  if (!s || (count && !d_dst)) return fail(RB_EINVAL, "null argument");
  if ((uint64_t)first + count > s->nb) return fail(RB_EINVAL, "bitmap range out of bounds");
  int rc = check_ctx(s->ctx);
  if (rc) return rc;
  return serialize_device(s, first, count, d_dst, cap, offsets, false);
}

// ---------------------------------------------------------------- pairwise
// Merge-path segment length: 256 merged keys per thread for large batches; shorter when the batch's
// expected key count would leave fewer than ~128K walking threads (the walk is latency-bound).
static uint32_t pairwise_seg_keys(const rbgpu_set *a, const rbgpu_set *b, uint64_t np) {
  const double per = (double)a->nc / std::max<uint32_t>(a->nb, 1) + (double)b->nc / std::max<uint32_t>(b->nb, 1);
  const double est = per * (double)np;
  uint32_t seg = 256;
  while (seg > 8 && est / seg < 131072.0) seg >>= 1;
  return seg;
}
// Small batches (kernels.hpp: <= kSmallPairs pairs of <= kSmallPairKeys keys, <= kSmallSlots merged
// keys, no Run container over 8 KiB to copy): two launches and one host read-back.  Returns 1 when
// the batch does not qualify (the general pipeline runs), else an rbgpu status.
// containers of bitmap i (RB_EMPTY_BITMAP: none)
static inline uint64_t bm_conts(const rbgpu_set *s, uint32_t i) {
  return i == kEmptyBitmap ? 0 : s->h_begin[i + 1] - s->h_begin[i];
}
#ifndef RBG_SMALL_POLL
#define RBG_SMALL_POLL 1 // study builds: 0 waits for the stream
#endif
static int pairwise_small(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, const uint32_t *a_idx,
                          const uint32_t *b_idx, uint32_t np, rbgpu_set **out, uint64_t *card_out, bool inplace,
                          bool keep_empty) {
  const char *dis = getenv("RBGPU_NO_SMALL_PAIRS"); // parity tests run both paths
  if ((dis && dis[0] == '1') || np == 0 || np > kSmallPairs) return 1;
  int rc = ensure_h_begin(a);
  if (!rc) rc = ensure_h_begin(b);
  if (rc) return rc;
  // per pair: first containers and counts (from the host CSR), first slot (merged keys <= na + nb), first
  // block (small_pair_nsub blocks per pair, at most ~16K blocks in all), the x1.op(x1) flag
  if (a->nc >= (1ull << 32) || b->nc >= (1ull << 32)) return 1; // 32-bit container indices in the tables
  const uint32_t cap = std::max<uint32_t>(1, std::min<uint32_t>(2048, 16384 / np));
  const bool inl = np <= kSmallInline;
  const uint64_t nid = (np + 31) / 32;
  std::vector<uint32_t> &tabv = ctx->small_tab; // [ident nid | i0 np | j0 np | nab np | slot np + 1 | blk np + 1]
  SmallTabInline *ti = inl ? &ctx->small_inline : nullptr;
  uint32_t *ident, *ti0, *tj0, *tnab, *slot, *blk;
  if (inl) {
    ident = ti->ident, ti0 = ti->i0, tj0 = ti->j0, tnab = ti->nab, slot = ti->slot, blk = nullptr;
  } else {
    tabv.assign(nid + 5ull * np + 2, 0u);
    ident = tabv.data(), ti0 = ident + nid, tj0 = ti0 + np, tnab = tj0 + np, slot = tnab + np, blk = slot + np + 1;
  }
  std::memset(ident, 0, 4 * nid);
  uint64_t acc = 0;
  uint32_t max_keys = 0;
  for (uint32_t p = 0; p < np; ++p) {
    const uint32_t ai = a_idx ? a_idx[p] : p, bi = b_idx ? b_idx[p] : p;
    const uint64_t na = bm_conts(a, ai), nb = bm_conts(b, bi), nk = na + nb;
    if (na > kSmallPairKeys || nb > kSmallPairKeys || nk > kSmallPairKeys) return 1;
    max_keys = std::max(max_keys, (uint32_t)nk);
    ti0[p] = ai == kEmptyBitmap ? 0u : (uint32_t)a->h_begin[ai];
    tj0[p] = bi == kEmptyBitmap ? 0u : (uint32_t)b->h_begin[bi];
    tnab[p] = (uint32_t)na | ((uint32_t)nb << 16);
    if (inplace && a == b && ai == bi && ai != kEmptyBitmap) ident[p >> 5] |= 1u << (p & 31);
    slot[p] = (uint32_t)acc;
    acc += nk;
    if (acc > kSmallSlots) return 1;
  }
  slot[np] = (uint32_t)acc;
  rc = ensure_max_runs(a);
  if (!rc) rc = ensure_max_runs(b);
  if (rc) return rc;
  if (a->max_runs > 2048 || b->max_runs > 2048) return 1; // a copy would not fit its 8 KiB slot
  const uint64_t E = acc;
  // merged keys per wave: 1, or doubled until the blocks fit the resident ones (one round of blocks)
  const uint64_t resident = small_resident_blocks();
  auto nsub = [&](uint32_t p, uint32_t kpw) { return small_pair_nsub(slot[p + 1] - slot[p], cap, kpw); };
  auto blocks_for = [&](uint32_t kpw) {
    uint64_t n = 0;
    for (uint32_t p = 0; p < np; ++p) n += nsub(p, kpw);
    return n;
  };
  uint32_t kpw = 1;
  uint64_t nblocks64 = blocks_for(1);
  while (nblocks64 > resident && kpw < 64) {
    kpw *= 2;
    nblocks64 = blocks_for(kpw);
  }
  const uint32_t nblocks = (uint32_t)nblocks64;
  for (uint32_t p = 0, k = 0; p <= np; ++p) {
    if (inl) ti->blk[p] = (uint16_t)k;
    else blk[p] = k;
    if (p < np) k += nsub(p, kpw);
  }
  rc = ensure_call_words(ctx);
  if (!rc) rc = seq_begin(ctx);
  if (rc) return rc;
  uint64_t *hout = reinterpret_cast<uint64_t *>(ctx->h_small);

  hipStream_t st = ctx->stream;
  const bool card_only = out == nullptr;
  const uint64_t E1 = std::max<uint64_t>(E, 1);
  const size_t tabb = inl ? 0 : 4 * tabv.size();
  const size_t need = aligned256(8ull * np) + aligned256(4 * E1) + aligned256(tabb) + 256;
  if (ctx->ws_pairs.reserve(need, st) != hipSuccess) return fail(RB_ENOMEM, "pair workspace");
  Workspace &W = ctx->ws_pairs;
  SmallPairArgs sa{};
  sa.A = a->view();
  sa.B = b->view();
  sa.np = np;
  SmallTabDev dt{};
  if (!inl) { // larger batches: the tables in device memory, one copy from pinned staging
    if (tabb > ctx->h_stage_cap) {
      if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
      ctx->h_stage = nullptr;
      ctx->h_stage_cap = 0;
      if (hipHostMalloc((void **)&ctx->h_stage, tabb) != hipSuccess) return fail(RB_ENOMEM, "pinned staging");
      ctx->h_stage_cap = tabb;
    }
    std::memcpy(ctx->h_stage, tabv.data(), tabb);
    uint32_t *d = W.take<uint32_t>(tabv.size());
    HIPCHK(hipMemcpyAsync(d, ctx->h_stage, tabb, hipMemcpyHostToDevice, st));
    dt = SmallTabDev{d, d + nid, d + nid + np, d + nid + 2ull * np, d + nid + 3ull * np, d + nid + 4ull * np + 1};
  }
  sa.pcard = card_out ? W.take<uint64_t>(np) : nullptr;
  uint32_t *xpos = W.take<uint32_t>(E1);
  sa.smeta = ctx->d_small_slots;
  sa.ctr = ctx->d_small_ctr;

  rbgpu_set *res = nullptr;
  if (!card_only) {
    res = new rbgpu_set;
    rc = set_alloc(ctx, res, np, E, E * kBitmapBytes);
    if (rc) {
      delete res;
      return rc;
    }
    sa.arena = res->payload;
  }
  // kernel events only when asked for (RBGPU_SMALL_KERNEL_TIMES=1, the bench's breakdown): the call is a
  // few tens of microseconds
  const char *kt = getenv("RBGPU_SMALL_KERNEL_TIMES");
  const bool ktimes = kt && kt[0] == '1';
  stats_begin(ctx, false);
  if (ktimes) HIPCHK(hipEventRecord(ctx->ev[1], st));
  sa.E = (uint32_t)E;
  sa.nblocks = nblocks;
  sa.xpos = xpos;
  sa.rbegin = res ? res->begin : nullptr;
  if (res) sa.out = OutView{res->key, res->type, res->card, res->nruns, res->off};
  sa.hout = reinterpret_cast<uint64_t *>(ctx->d_small);
  sa.seq = ++ctx->small_seq;
  sa.lazy = is_lazy_op(op) ? op : 0;
  sa.inplace = inplace;
  sa.keep_empty = keep_empty;
  launch_pair_small(is_lazy_op(op) ? (int)RB_OR : op, card_only, sa, ti, dt, max_keys, nblocks, st);
  if (ktimes) HIPCHK(hipEventRecord(ctx->ev[2], st));
  if (card_out) HIPCHK(hipMemcpyAsync(card_out, sa.pcard, 8ull * np, hipMemcpyDeviceToHost, st));
  HIPCHK(hipEventRecord(ctx->ev[5], st));
  // The last block writes the result words to host memory and then the call's sequence number
  // (wait_call_seq); per-pair cardinalities come back by a copy, so those calls wait for the stream.
  bool seen = false;
  rc = seq_end(ctx, sa.seq, RBG_SMALL_POLL && !card_out, "small-batch pairwise", &seen);
  if (rc) {
    if (res) rbgpu_set_free(res);
    return rc;
  }
  // the result words, written by the last block straight into host memory
  uint64_t *w = ctx->words;
  for (int i = 0; i < kStatWords; ++i) w[i] = 0;
  w[0] = hout[1];           // input bytes with key arrays
  w[6] = hout[1] - hout[2]; // container input bytes
  w[1] = hout[3];           // output bytes
  w[7] = hout[4];           // result cardinality
  const uint64_t nres = hout[0];
  const KernelSpan spans[1] = {{"k_pair_small", 6, 1, E}};
  rc = stats_fill(ctx, E, nres, spans, ktimes ? 1 : 0, !seen);
  ctx->stats_pending = seen;
  ctx->stats_pending_k = seen && ktimes;
  if (rc) {
    if (res) rbgpu_set_free(res);
    return rc;
  }
  ctx->last.result_containers = nres;
  if (res) {
    res->nc = nres;
    res->end_seq = seen ? sa.seq : 0;
    *out = res;
  }
  return RB_OK;
}

// probe: 0 = the product path; 1 / 2 = measurement probes (rbgpu_internal_probe) in place of the
// task kernel — results are not produced.
static // tasks bound up to which pairwise_impl reserves the task workspace before the totals are read back
// (58 B per task: 464 MiB at the cap; the bound a.nc + b.nc can far exceed the real count — an AND of
// mostly disjoint keys — and the workspace stays grown, so the cap is set just above config 2's 6.1M)
constexpr uint64_t kEarlyEmitTasks = 1ull << 23;

// async: return once the task kernels and the compaction are enqueued (rbgpu_pairwise_async): the result
// is pending (settle() fills its container count), the call's counters are not read back (rb_stats keeps
// the last synchronous call's), and `ext` (if any, another stream of the caller) is ordered around the call.
int pairwise_impl(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, const uint32_t *a_idx,
                         const uint32_t *b_idx, uint32_t npairs, rbgpu_set **out, uint64_t *card_out,
                         int probe = 0, bool inplace = false, bool keep_empty = false, bool async = false,
                         hipStream_t ext = nullptr) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if ((op < RB_AND || op > RB_ANDNOT) && !is_lazy_op(op)) return fail(RB_EINVAL, "bad op %d", op);
  if (!a || !b) return fail(RB_EINVAL, "null set");
  if (a->ctx != ctx || b->ctx != ctx) return fail(RB_EINVAL, "sets belong to another context");
  if (!a_idx && npairs > a->nb) return fail(RB_EINVAL, "npairs exceeds bitmaps of a");
  if (!b_idx && npairs > b->nb) return fail(RB_EINVAL, "npairs exceeds bitmaps of b");
  for (uint32_t i = 0; a_idx && i < npairs; ++i)
    if (a_idx[i] >= a->nb && a_idx[i] != kEmptyBitmap) return fail(RB_EINVAL, "a_idx[%u] out of range", i);
  for (uint32_t i = 0; b_idx && i < npairs; ++i)
    if (b_idx[i] >= b->nb && b_idx[i] != kEmptyBitmap) return fail(RB_EINVAL, "b_idx[%u] out of range", i);
  if (ext == ctx->stream) ext = nullptr;
  if (ext) { // the caller's earlier work on its stream comes first
    HIPCHK(hipEventRecord(ctx->ev_ext, ext));
    HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_ext, 0));
  }
  if (!probe) { // small batches complete before the return, asynchronous call or not
    rc = pairwise_small(ctx, op, a, b, a_idx, b_idx, npairs, out, card_out, inplace, keep_empty);
    if (rc == RB_OK && ext) {
      // the host returned on the last block's sequence word, before the kernel's end (and its L2 write-back):
      // the caller's later work on its stream waits for that end, as after the general path below
      HIPCHK(hipEventRecord(ctx->ev_ext, ctx->stream));
      HIPCHK(hipStreamWaitEvent(ext, ctx->ev_ext, 0));
    }
    if (rc != 1) return rc;
  }
  int slot = -1;
  struct SlotGuard { // an error return gives the slot back
    rbgpu_ctx *c;
    int &slot;
    ~SlotGuard() {
      if (slot >= 0) c->async_free.push_back(slot);
    }
  } slot_guard{ctx, slot};
  if (async && out) { // a pinned word for the result count; none free: the call completes synchronously
    if (!ctx->h_async) {
      if (hipHostMalloc((void **)&ctx->h_async, kAsyncSlots * sizeof(uint64_t)) != hipSuccess)
        return fail(RB_ENOMEM, "pinned result-count slots");
      for (int i = kAsyncSlots - 1; i >= 0; --i) ctx->async_free.push_back(i);
    }
    if (!ctx->async_free.empty()) {
      slot = ctx->async_free.back();
      ctx->async_free.pop_back();
    }
  }
  const bool card_only = out == nullptr;
  const int kop = is_lazy_op(op) ? (int)RB_OR : op; // the kernels' op (lazy roles run as OR, TaskMeta::lazy)
  hipStream_t st = ctx->stream;
  const uint64_t np = npairs;
  // ---- per pair: indices, merge-path segment counts and their scan, pair cardinalities
  size_t need = 2 * aligned256(np * 4) + 3 * aligned256((np + 1) * 8) + aligned256(scan_tmp_words(np + 1) * 8);
  if (ctx->ws_pairs.reserve(need, st) != hipSuccess) return fail(RB_ENOMEM, "pair workspace");
  Workspace &W = ctx->ws_pairs;
  uint32_t *d_aidx = a_idx ? W.take<uint32_t>(np) : nullptr;
  uint32_t *d_bidx = b_idx ? W.take<uint32_t>(np) : nullptr;
  uint64_t *nseg_p = W.take<uint64_t>(np + 1), *seg_begin = W.take<uint64_t>(np + 1);
  uint64_t *pcard = W.take<uint64_t>(np + 1);
  uint64_t *ptmp = W.take<uint64_t>(std::max<uint64_t>(scan_tmp_words(np + 1), 1));
  // small batches: the merge-path segment counts come from the host CSR copies (no count kernel,
  // scan and host read-back before the segment phase)
  const bool host_segs = np && np <= 4096 && !ensure_h_begin(a) && !ensure_h_begin(b);
  const uint32_t seg_keys = pairwise_seg_keys(a, b, np);
  if (d_aidx || d_bidx || host_segs) { // through pinned staging: a pageable copy would block the host
    const size_t bytes = np * 4 * ((d_aidx != nullptr) + (d_bidx != nullptr)) + (host_segs ? (np + 1) * 8 : 0);
    if (bytes > ctx->h_stage_cap) {
      if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
      ctx->h_stage = nullptr;
      ctx->h_stage_cap = 0;
      if (hipHostMalloc((void **)&ctx->h_stage, bytes) != hipSuccess) return fail(RB_ENOMEM, "pinned staging");
      ctx->h_stage_cap = bytes;
    }
    uint8_t *h = ctx->h_stage;
    if (d_aidx) {
      std::memcpy(h, a_idx, np * 4);
      HIPCHK(hipMemcpyAsync(d_aidx, h, np * 4, hipMemcpyHostToDevice, st));
      h += np * 4;
    }
    if (d_bidx) {
      std::memcpy(h, b_idx, np * 4);
      HIPCHK(hipMemcpyAsync(d_bidx, h, np * 4, hipMemcpyHostToDevice, st));
      h += np * 4;
    }
    if (host_segs) {
      uint64_t *sb = reinterpret_cast<uint64_t *>(h), acc = 0;
      for (uint64_t p = 0; p < np; ++p) { // k_seg_count's formula
        const uint32_t ai = a_idx ? a_idx[p] : (uint32_t)p, bi = b_idx ? b_idx[p] : (uint32_t)p;
        const uint64_t nk = bm_conts(a, ai) + bm_conts(b, bi);
        sb[p] = acc;
        acc += (nk + seg_keys - 1) / seg_keys + (nk == 0);
      }
      sb[np] = acc;
      HIPCHK(hipMemcpyAsync(seg_begin, sb, (np + 1) * 8, hipMemcpyHostToDevice, st));
    }
  }
  if (card_out && np) HIPCHK(hipMemsetAsync(pcard, 0, np * 8, st));

  stats_begin(ctx);
  PairArgs pa{op, a->view(), b->view(), d_aidx, d_bidx, npairs, seg_begin, nullptr, 0, seg_keys, inplace, a == b,
              a->nc, b->nc};
  uint64_t *const tot = ctx->h_pinned;
  uint64_t ns = 0;
  // one segment per pair when no pair can exceed seg_keys merged keys (config 2: <= 8 keys per
  // pair): seg_begin is the identity and the count kernel, its scan and the read-back are skipped
  const bool ident_segs = !host_segs && np && !a_idx && !b_idx && !ensure_max_keys(a) && !ensure_max_keys(b) &&
                          (uint64_t)(a->max_keys + b->max_keys) <= seg_keys;
  if (host_segs) {
    ns = reinterpret_cast<const uint64_t *>(ctx->h_stage + np * 4 * ((d_aidx != nullptr) + (d_bidx != nullptr)))[np];
  } else if (ident_segs) {
    ns = np;
  } else {
    launch_seg_count(pa, nseg_p, st);
    scan_exclusive(nseg_p, seg_begin, np, ptmp, st);
    HIPCHK(hipMemcpyAsync(tot + 6, seg_begin + np, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    LAUNCHCHK();
    ns = np ? tot[6] : 0;
  }
  // ---- per segment: counts, block totals and their scans, result counts / offsets
  const uint64_t nblk = pair_blocks(ns);
  need = aligned256(ns * 4) + 3 * aligned256((ns + 1) * 8) + 10 * aligned256((nblk + 1) * 8) + 4 * 256;
  Workspace &G = ctx->ws_segs;
  if (G.reserve(need, st) != hipSuccess) return fail(RB_ENOMEM, "segment workspace");
  uint32_t *seg_pair = G.take<uint32_t>(std::max<uint64_t>(ns, 1));
  uint64_t *cnt = G.take<uint64_t>(ns + 1); // per segment, packed (pack_seg_counts)
  PairCountArrays bt{G.take<uint64_t>(nblk + 1), G.take<uint64_t>(nblk + 1), G.take<uint64_t>(nblk + 1),
                     G.take<uint64_t>(nblk + 1)};
  PairCountArrays bs{G.take<uint64_t>(nblk + 1), G.take<uint64_t>(nblk + 1), G.take<uint64_t>(nblk + 1),
                     G.take<uint64_t>(nblk + 1)};
  uint64_t *task_begin = G.take<uint64_t>(ns + 1), *rseg = G.take<uint64_t>(ns + 1);
  uint64_t *bk = G.take<uint64_t>(nblk + 1), *bks = G.take<uint64_t>(nblk + 1);
  uint64_t *d_tot = G.take<uint64_t>(4);
  // one segment per pair: no segment maps at all (the kernels take segment p as pair p)
  if (!ident_segs) launch_seg_fill(pa, seg_begin, seg_pair, st);
  pa.seg_pair = ident_segs ? nullptr : seg_pair;
  pa.nseg = ns;
  launch_pair_count(pa, cnt, bt, ctx->d_stats, st);
  if (ns) {
    const uint64_t *scan_in[4] = {bt.task, bt.light, bt.big, bt.small};
    uint64_t *scan_out[4] = {bs.task, bs.light, bs.big, bs.small};
    scan_blocks_multi(scan_in, scan_out, 4, nblk, d_tot, st);
  }
  HIPCHK(hipMemcpyAsync(tot, d_tot, 4 * 8, hipMemcpyDeviceToHost, st));
  // Early emission: with identity pairing every container of A and of B takes at most one task, so
  // a.nc + b.nc bounds the task count before the totals are on the host.  The task workspace is then
  // sized by that bound and the emit kernel reads the totals on the device: it runs while the host
  // waits for the totals, allocates the result and launches the task kernels.  Otherwise the host
  // reads the totals first (the bound is the segments' key capacity, too loose to reserve).
  // light tasks come from a shared chunk queue (a second light launch takes over the heavy kernel's
  // CUs when it finishes)
  const uint64_t seg_cap = ns * (uint64_t)seg_keys;
  const uint64_t tbound = !d_aidx && !d_bidx ? std::min<uint64_t>(a->nc + b->nc, seg_cap) : seg_cap;
  const bool early = !probe && ns && tbound <= kEarlyEmitTasks;
  TaskMeta tm{};
  tm.lazy = is_lazy_op(op) ? op : 0;
  tm.inplace = inplace;
  tm.keep_empty = keep_empty;
  TaskRec *light = nullptr;
  unsigned long long *queue = nullptr;
  // one record array (the light records, then the heavy ones) and the per-task metadata, for nt tasks
  auto take_tasks = [&](uint64_t nt) -> int {
    const uint64_t nt1 = std::max<uint64_t>(nt, 1);
    const size_t tneed = aligned256(nt1 * sizeof(TaskRec)) + aligned256(nt1) + 2 * aligned256(nt1 * 8) +
                         aligned256(kQueueWords * 8) + 256;
    Workspace &T = ctx->ws_tasks;
    if (T.reserve(tneed, st) != hipSuccess)
      return fail(RB_ENOMEM, "task workspace (%llu tasks)", (unsigned long long)nt);
    light = T.take<TaskRec>(nt1);
    tm.type = T.take<uint8_t>(nt1);
    tm.res = T.take<uint64_t>(nt1);
    tm.slot = T.take<uint64_t>(nt1);
    queue = T.take<unsigned long long>(kQueueWords); // light-task chunk counters (<= 32, 128 B apart)
    return RB_OK;
  };
  if (early) {
    if ((rc = take_tasks(tbound))) return rc;
    HIPCHK(hipEventRecord(ctx->ev_tot, st));
    launch_pair_emit(pa, cnt, bs, 0, light, nullptr, tm, task_begin, d_tot, tbound, queue,
                     st);
    HIPCHK(hipEventSynchronize(ctx->ev_tot));
  } else {
    HIPCHK(hipStreamSynchronize(st));
  }
  LAUNCHCHK();
  if (!ns) tot[0] = tot[1] = tot[2] = tot[3] = 0;
  const uint64_t ntasks = tot[0], nlight = tot[1], nheavy = ntasks - nlight, nbig_t = tot[2], small_t = tot[3];
  const uint64_t small_base = nbig_t * kBitmapBytes;
  const uint64_t arena = card_only ? 0 : small_base + small_t;
  if (arena >= kSlotOffsetLimit) { // a task slot holds 40-bit arena offsets
    (void)hipStreamSynchronize(st);
    return fail(RB_ENOMEM, "pairwise: result arena of %llu bytes", (unsigned long long)arena);
  }
  if (early && ntasks > tbound) { // never expected: the emit dropped the records past the bound
    (void)hipStreamSynchronize(st);
    return fail(RB_EDEVICE, "pairwise: %llu tasks exceed the bound %llu", (unsigned long long)ntasks,
                (unsigned long long)tbound);
  }
  if (!early && (rc = take_tasks(ntasks))) return rc;
  TaskRec *heavy = light + nlight;

  rbgpu_set *res = nullptr;
  if (!card_only) {
    res = new rbgpu_set;
    rc = set_alloc(ctx, res, npairs, ntasks, arena);
    if (rc) {
      delete res;
      (void)hipStreamSynchronize(st); // the early emit may still write the workspace
      return rc;
    }
  }
  // the light and heavy task kernels run concurrently (heavy on the side stream, 1 block per CU;
  // light 2 blocks per CU: 2 x 128 + 256 VGPRs per SIMD)
#ifndef RBG_FORCE_SERIAL
#define RBG_FORCE_SERIAL 0 // study: light then heavy on one stream (each kernel's standalone time)
#endif
  const bool conc = !RBG_FORCE_SERIAL && !probe && nlight && nheavy && nlight + nheavy >= 65536; // small batches: the
                                                  // cross-stream waits cost more than the overlap
  // the emit zeroes the queue counters before ev[1]: the side stream waits on ev[1] before its light launch
  if (!early)
    launch_pair_emit(pa, cnt, bs, small_base, light, heavy, tm, task_begin, nullptr, 0, queue,
                     st);
  HIPCHK(hipEventRecord(ctx->ev[1], st));
  if (probe) {
    uint32_t *sink = nullptr;
    const unsigned blocks = 256 * 4;
    if (ctx->pool.alloc((void **)&sink, blocks * 256ull * 4)) return fail(RB_ENOMEM, "probe sink");
    launch_probe(op, probe, a->payload, b->payload, a->payload_bytes, light, nlight, sink, blocks, st);
    if (probe == 1) launch_probe(op, probe, a->payload, b->payload, 0, heavy, nheavy, sink, blocks, st);
    HIPCHK(hipEventRecord(ctx->ev[2], st));
    HIPCHK(hipStreamSynchronize(st));
    LAUNCHCHK();
    ctx->pool.release(sink);
    if (res) rbgpu_set_free(res);
    const KernelSpan spans[1] = {{probe == 1 ? "k_probe_tasks" : "k_probe_stream", 6, -1, ntasks}};
    rc = stats_end(ctx, ntasks, 0, spans, 1);
    if (probe == 2) ctx->last.main_kernel_bytes = ctx->last.kernel_bytes[0] = a->payload_bytes / 8192 * 8192;
    return rc;
  }
  if (conc) {
    HIPCHK(hipStreamWaitEvent(ctx->side, ctx->ev[1], 0));
    launch_pairwise_concurrent(kop, card_only, a->payload, b->payload, light, nlight, heavy, nheavy,
                               res ? res->payload : nullptr, tm, st, ctx->side, ctx->ev[2], ctx->ev_side[0],
                               ctx->ev_side[1], queue);
    HIPCHK(hipEventRecord(ctx->ev_side[2], ctx->side));
    HIPCHK(hipStreamWaitEvent(st, ctx->ev_side[2], 0));
  } else {
    launch_pairwise(kop, card_only, a->payload, b->payload, light, nlight, heavy, nheavy, res ? res->payload : nullptr,
                    tm, st, ctx->ev[2]);
  }
  HIPCHK(hipEventRecord(ctx->ev[3], st));
  launch_compact_count(task_begin, ns, tm.type, bk, st);
  // the block totals' scan total is the result container count: stats word 8, read back with the
  // counters by stats_end
  if (ns) {
    const uint64_t *kin[1] = {bk};
    uint64_t *kout[1] = {bks};
    scan_blocks_multi(kin, kout, 1, nblk, ctx->d_stats + 8 * kStripes, st);
  }
  OutView ov{};
  if (res) ov = OutView{res->key, res->type, res->card, res->nruns, res->off};
  // one segment per pair: the compaction writes the result CSR itself; else per segment, mapped below
  uint64_t *rb_direct = res && ident_segs ? res->begin : nullptr;
  // RBGPU_CALL_TAIL=1: a synchronous call whose compaction is its last kernel returns on that kernel's tail
  // (CallTail): the last block hands the summed counters to host-visible words, so no counters copy, memset or
  // stream wait.  Off by default: measured slower on config 2 (4.384 vs 4.333 ms per AND step, three interleaved
  // pairs, profiles/r06/tail) — the host phase did not shrink and the next call's light kernel ran ~35 us longer.
  const char *ct = getenv("RBGPU_CALL_TAIL"); // the parity test runs both forms
  const bool tailed = ct && ct[0] == '1' && slot < 0 && res && ident_segs && !card_out && ns;
  CallTail tail{};
  if (tailed) {
    if ((rc = ensure_call_words(ctx)) || (rc = seq_begin(ctx))) {
      (void)hipStreamSynchronize(st);
      rbgpu_set_free(res);
      return rc;
    }
    tail = CallTail{ctx->d_small_ctr + 48, reinterpret_cast<uint64_t *>(ctx->d_small) + kTailWord, ++ctx->small_seq};
  }
  launch_compact_write(task_begin, ns, tm, bks, ov, pa.seg_pair, card_out ? pcard : nullptr, ctx->d_stats,
                       res && !ident_segs ? rseg : nullptr, rb_direct, st, tail);
  if (res && np && !ident_segs) launch_pair_rbegin(seg_begin, npairs, rseg, res->begin, nullptr, st);
  else if (res && !np) HIPCHK(hipMemsetAsync(res->begin, 0, 8, st));
  if (card_out && np) HIPCHK(hipMemcpyAsync(card_out, pcard, np * 8, hipMemcpyDeviceToHost, st));
  if (slot >= 0) {
    // the result count (stats word 8, written by the compaction's scan) into the pinned slot, the
    // counters zeroed for the next call, and the completion event the result settles on
    const int prc = np ? (hipMemcpyAsync(ctx->h_async + slot, ctx->d_stats + 8 * kStripes, 8, hipMemcpyDeviceToHost, st)
                              ? RB_EDEVICE : RB_OK)
                       : (ctx->h_async[slot] = 0, RB_OK);
    hipEvent_t done = nullptr;
    if (prc || hipMemsetAsync(ctx->d_stats, 0, kStatWords * kStripes * sizeof(uint64_t), st) ||
        hipEventCreateWithFlags(&done, hipEventDisableTiming) || hipEventRecord(done, st) ||
        (ext && hipStreamWaitEvent(ext, done, 0)) ||
        hipGetLastError()) {
      if (done) (void)hipEventDestroy(done);
      (void)hipStreamSynchronize(st);
      rbgpu_set_free(res);
      return fail(RB_EDEVICE, "asynchronous pairwise: enqueue failed");
    }
    // the inputs stay allocated until the call is done with them: set_release waits for this
    for (const rbgpu_set *in : {a, b}) {
      rbgpu_set *m = const_cast<rbgpu_set *>(in);
      if ((!m->read_done && hipEventCreateWithFlags(&m->read_done, hipEventDisableTiming)) ||
          hipEventRecord(m->read_done, st)) {
        (void)hipStreamSynchronize(st);
        res->pending = done;
        res->pend_slot = slot;
        slot = -1;
        rbgpu_set_free(res);
        return fail(RB_EDEVICE, "asynchronous pairwise: enqueue failed");
      }
    }
    ctx->stats_clean = true;
    res->pending = done;
    res->pend_slot = slot;
    slot = -1; // the result owns it now
    *out = res;
    return RB_OK;
  }
  KernelSpan spans[3] = {{"k_pair_tasks<light>", 2, 4, nlight}, {"k_pair_tasks<heavy>", 3, 5, nheavy}, {"", -1, -1, 0}};
  int nspans = 2;
  if (conc) { // [0] the concurrent task phase (both kernels' bytes over the union of their spans), then each
    spans[0] = KernelSpan{"k_pair_tasks<light>||<heavy>", 2, 4, ntasks, ctx->ev[1], ctx->ev[3], 3, 5};
    spans[1] = KernelSpan{"k_pair_tasks<light>", 2, 4, nlight, ctx->ev[1], ctx->ev[2]};
    spans[2] = KernelSpan{"k_pair_tasks<heavy>", 3, 5, nheavy, ctx->ev_side[0], ctx->ev_side[1]};
    nspans = 3;
  }
  if (tailed) {
    HIPCHK(hipEventRecord(ctx->ev[5], st));
    bool seen = false;
    rc = seq_end(ctx, tail.seq, true, "pairwise compaction", &seen, kTailWord + kStatWords);
    if (rc) {
      rbgpu_set_free(res);
      return rc;
    }
    const uint64_t *hw = reinterpret_cast<const uint64_t *>(ctx->h_small) + kTailWord;
    for (int i = 0; i < kStatWords; ++i) ctx->words[i] = hw[i];
    ctx->stats_clean = true; // the tail zeroed the counters
    rc = stats_fill(ctx, ntasks, 0, spans, nspans, !seen);
    if (seen) { // the kernel times when the stats are asked for (rbgpu_get_stats)
      ctx->stats_pending = true;
      ctx->stats_pending_k = false;
      for (int i = 0; i < nspans; ++i) ctx->pend_spans[i] = spans[i];
      ctx->pend_n = nspans;
      ctx->pend_tasks = ntasks;
      res->end_seq = tail.seq;
    }
  } else {
    rc = stats_end(ctx, ntasks, 0, spans, nspans);
  }
  if (rc) {
    if (res) rbgpu_set_free(res);
    return rc;
  }
  const uint64_t nres = np ? ctx->words[8] : 0;
  ctx->last.result_containers = nres;
  if (res) {
    res->nc = nres;
    *out = res;
  }
  if (ext) { // the caller's later work on its stream comes after this call's
    HIPCHK(hipEventRecord(ctx->ev_ext, ctx->stream));
    HIPCHK(hipStreamWaitEvent(ext, ctx->ev_ext, 0));
  }
  return RB_OK;
}

static double us_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}

int rbgpu_pairwise(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, const uint32_t *a_idx,
                   const uint32_t *b_idx, uint32_t npairs, rbgpu_set **out) {
  SETTLE(a, b);
  const auto t0 = std::chrono::steady_clock::now();
  if (!out) return fail(RB_EINVAL, "null out");
  *out = nullptr;
  const int rc = pairwise_impl(ctx, op, a, b, a_idx, b_idx, npairs, out, nullptr);
  if (!rc) ctx->last.call_us = us_since(t0);
  return rc;
}

int rbgpu_pairwise_async(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, const uint32_t *a_idx,
                         const uint32_t *b_idx, uint32_t npairs, void *stream, rbgpu_set **out) {
  SETTLE(a, b);
  if (!out) return fail(RB_EINVAL, "null out");
  *out = nullptr;
  return pairwise_impl(ctx, op, a, b, a_idx, b_idx, npairs, out, nullptr, 0, false, false, true,
                       reinterpret_cast<hipStream_t>(stream));
}

int rbgpu_set_wait(const rbgpu_set *s) {
  if (!s) return fail(RB_EINVAL, "null argument");
  const int rc = settle(s);
  return rc ? rc : seq_settle(s->ctx, s->end_seq);
}

int rbgpu_set_device_view(const rbgpu_set *s, rb_device_view *out) {
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  if (s->failed) return fail(RB_EDEVICE, "the asynchronous call that produced this set failed");
  *out = rb_device_view{s->nb, s->pending ? RB_UNKNOWN_COUNT : s->nc, s->payload_bytes, s->begin, s->key, s->type,
                        s->card, s->nruns, s->off, s->payload};
  return RB_OK;
}

int rbgpu_pairwise_cardinality(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, const uint32_t *a_idx,
                               const uint32_t *b_idx, uint32_t npairs, uint64_t *out) {
  SETTLE(a, b);
  const auto t0 = std::chrono::steady_clock::now();
  if (!out && npairs) return fail(RB_EINVAL, "null out");
  const int rc = pairwise_impl(ctx, op, a, b, a_idx, b_idx, npairs, nullptr, out);
  if (!rc) ctx->last.call_us = us_since(t0);
  return rc;
}

} // extern "C"
namespace rbg {
int pairwise_call(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, const uint32_t *a_idx,
                  const uint32_t *b_idx, uint32_t npairs, rbgpu_set **out, bool inplace, bool keep_empty) {
  *out = nullptr;
  return pairwise_impl(ctx, op, a, b, a_idx, b_idx, npairs, out, nullptr, 0, inplace, keep_empty);
}
} // namespace rbg
extern "C" {

int rbgpu_set_run_optimize(const rbgpu_set *in, rbgpu_set **out, uint8_t *any_run) {
  SETTLE(in);
  if (!in || !out) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  rbgpu_ctx *ctx = in->ctx;
  int rc = check_ctx(ctx);
  if (rc) return rc;
  hipStream_t st = ctx->stream;
  rbgpu_set *res = new rbgpu_set;
  rc = set_alloc(ctx, res, in->nb, in->nc, in->payload_bytes);
  if (rc) {
    delete res;
    return rc;
  }
  uint8_t *d_any = nullptr;
  if (any_run && in->nb && ctx->pool.alloc((void **)&d_any, in->nb)) {
    rbgpu_set_free(res);
    return fail(RB_ENOMEM, "runOptimize flags");
  }
  const uint64_t n = in->nc;
  auto copy = [&](void *d, const void *s, uint64_t b) { return b ? hipMemcpyAsync(d, s, b, hipMemcpyDeviceToDevice, st) : hipSuccess; };
  if (copy(res->begin, in->begin, 8ull * (in->nb + 1)) || copy(res->key, in->key, 2 * n) ||
      copy(res->card, in->card, 4 * n) || copy(res->off, in->off, 8 * n)) {
    ctx->pool.release(d_any);
    rbgpu_set_free(res);
    return fail(RB_EDEVICE, "runOptimize metadata copy");
  }
  stats_begin(ctx);
  HIPCHK(hipEventRecord(ctx->ev[1], st));
  launch_run_optimize(in->view(), n, res->type, res->nruns, res->payload, in->nb, d_any, st);
  HIPCHK(hipEventRecord(ctx->ev[2], st));
  if (d_any) HIPCHK(hipMemcpyAsync(any_run, d_any, in->nb, hipMemcpyDeviceToHost, st));
  const KernelSpan spans[1] = {{"k_run_optimize", 0, 1, n}};
  rc = stats_end(ctx, n, n, spans, 1);
  ctx->pool.release(d_any);
  if (rc) {
    rbgpu_set_free(res);
    return rc;
  }
  res->h_begin = in->h_begin;
  *out = res;
  return RB_OK;
}

int rbgpu_pairwise_inplace(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, const uint32_t *a_idx,
                           const uint32_t *b_idx, uint32_t npairs, rbgpu_set **out) {
  SETTLE(a, b);
  const auto t0 = std::chrono::steady_clock::now();
  if (!out) return fail(RB_EINVAL, "null out");
  *out = nullptr;
  if (op < RB_AND || op > RB_ANDNOT) return fail(RB_EINVAL, "bad op %d", op);
  const int rc = pairwise_impl(ctx, op, a, b, a_idx, b_idx, npairs, out, nullptr, 0, true);
  if (!rc) ctx->last.call_us = us_since(t0);
  return rc;
}

// Measurement hook (not part of rbgpu.h): runs the pairwise setup, then a read-only probe kernel
// in place of the task kernel (mode 1: the task kernel's payload loads; 2: a streaming read of
// a's arena).  The probe's time is in rbgpu_get_stats().main_kernel_ms.
int rbgpu_internal_probe(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, uint32_t npairs, int mode) {
  SETTLE(a, b);
  if (mode != 1 && mode != 2) return fail(RB_EINVAL, "probe mode");
  rbgpu_set *res = nullptr;
  return pairwise_impl(ctx, op, a, b, nullptr, nullptr, npairs, &res, nullptr, mode);
}

// Kernel-study hook (not part of rbgpu.h): config-2 generator type mix, cumulative per mille
// {filter Array, filter Array+Bitmap, posting Array, posting Array+Bitmap}.
void rbgpu_internal_set_mix(int fa, int fab, int pa, int pab) {
  const int m[4] = {fa, fab, pa, pab};
  set_mix(m);
}

// ---------------------------------------------------------------- wide
// FastAggregation.priorityqueue_xor (FastAggregation.java:732-752): a queue of bitmaps ordered by
// getLongSizeInBytes (java.util.PriorityQueue, Collections.addAll order); the two smallest are
// replaced by their RoaringBitmap.xor — one pairwise call on the device — until one is left.
static int empty_result(rbgpu_ctx *ctx, rbgpu_set **out) {
  rbgpu_set *e = new rbgpu_set;
  int rc = set_alloc(ctx, e, 1, 0, 16);
  if (rc) {
    delete e;
    return rc;
  }
  const uint64_t hb[2] = {0, 0};
  // on the library stream (it is non-blocking: a null-stream copy would not be ordered after its kernels)
  HIPCHK(hipMemcpyAsync(e->begin, hb, 16, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  e->h_begin = {0, 0};
  *out = e;
  return RB_OK;
}
// The size a priority queue orders bitmaps by, per bitmap of s (one metadata read-back):
//   kSizeLong       RoaringBitmap.getLongSizeInBytes (RoaringBitmap.java:2212-2219): 8 + per container
//                   2 + getSizeInBytes (Array 2c + 4, Bitmap 8192 lazy or not, Run 4r + 4);
//   kSizeImmutable  ImmutableRoaringBitmap.getLongSizeInBytes (buffer/ImmutableRoaringBitmap.java:1508-1521):
//                   4 + per container 4 + (Run 2 + 4r; else getCardinality() > 4096 ? 8192 : 2 getCardinality()),
//                   a lazy Bitmap's getCardinality() being -1 (MappeableBitmapContainer.java:540-542);
//   kSizeSerialized ImmutableRoaringBitmap.serializedSizeInBytes (buffer/MutableRoaringArray.java:756-764).
// Intermediate results of priorityqueue_or carry the lazy marks in their card words (common.hpp).
enum { kSizeLong = 0, kSizeImmutable = 1, kSizeSerialized = 2 };
static int pq_sizes(const rbgpu_set *s, int kind, std::vector<int64_t> &out) {
  int rc = ensure_h_begin(s);
  if (rc) return rc;
  const uint64_t n = s->nc;
  std::vector<uint8_t> type(n);
  std::vector<uint16_t> nruns(n);
  std::vector<uint32_t> card(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(type.data(), s->type, n, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(nruns.data(), s->nruns, n * 2, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipMemcpyAsync(card.data(), s->card, n * 4, hipMemcpyDeviceToHost, s->ctx->stream));
    HIPCHK(hipStreamSynchronize(s->ctx->stream));
  }
  out.assign(s->nb, 0);
  for (uint32_t b = 0; b < s->nb; ++b) {
    const uint64_t lo = s->h_begin[b], hi = s->h_begin[b + 1], k = hi - lo;
    int64_t v = kind == kSizeLong ? 8 : kind == kSizeImmutable ? 4 : 0;
    bool hasrun = false;
    for (uint64_t i = lo; i < hi; ++i) {
      const int64_t r = nruns[i], c = card[i] & ~kCardMarks;
      const bool lazy = type[i] == RB_BITMAP && (card[i] & kLazyCard);
      hasrun |= type[i] == RB_RUN;
      if (kind == kSizeLong)
        v += 2 + (type[i] == RB_BITMAP ? 8192 : type[i] == RB_ARRAY ? 2 * c + 4 : 4 * r + 4);
      else if (kind == kSizeImmutable)
        v += 4 + (type[i] == RB_RUN ? 2 + 4 * r : lazy ? -2 : c > kMaxArray ? 8192 : 2 * c);
      else
        v += type[i] == RB_BITMAP ? 8192 : type[i] == RB_ARRAY ? 2 * c : 2 + 4 * r;
    }
    if (kind == kSizeSerialized)
      v += (int64_t)(hasrun ? (k < 4 ? 4 + (k + 7) / 8 + 4 * k : 4 + (k + 7) / 8 + 8 * k) : 8 + 8 * k);
    out[b] = v;
  }
  return RB_OK;
}

// buffered: BufferFastAggregation.priorityqueue_xor (buffer/BufferFastAggregation.java:933-958) — fewer
// than 2 bitmaps throw, the queue orders by ImmutableRoaringBitmap.getLongSizeInBytes.
static int pq_xor(rbgpu_ctx *ctx, const rbgpu_set *in, const std::vector<uint32_t> &mem, rbgpu_set **out,
                  bool buffered) {
  const size_t n = mem.size();
  if (buffered && n < 2) return fail(RB_EINVAL, "Expecting at least 2 bitmaps");
  if (n == 0) return empty_result(ctx, out);
  const int kind = buffered ? kSizeImmutable : kSizeLong;
  std::vector<int64_t> sz;
  int rc = pq_sizes(in, kind, sz);
  if (rc) return rc;
  struct Node {
    const rbgpu_set *s;
    uint32_t idx;
    int64_t size;
    rbgpu_set *owned;
  };
  std::vector<Node> nodes;
  nodes.reserve(2 * n);
  for (uint32_t m : mem) nodes.push_back(Node{in, m, sz[m], nullptr});
  auto cmp = [&](uint32_t a, uint32_t b) { return (int)(nodes[a].size - nodes[b].size); };
  JavaHeap<uint32_t, decltype(cmp)> pq(cmp);
  for (uint32_t k = 0; k < n; ++k) pq.offer(k);
  auto cleanup = [&]() {
    for (Node &x : nodes)
      if (x.owned) rbgpu_set_free(x.owned), x.owned = nullptr;
  };
  while (pq.size() > 1) {
    const uint32_t x1 = pq.poll(), x2 = pq.poll();
    const uint32_t i1 = nodes[x1].idx, i2 = nodes[x2].idx;
    rbgpu_set *r = nullptr;
    rc = rbgpu_pairwise(ctx, RB_XOR, nodes[x1].s, nodes[x2].s, &i1, &i2, 1, &r);
    std::vector<int64_t> rs;
    if (!rc) rc = pq_sizes(r, kind, rs);
    if (rc) {
      if (r) rbgpu_set_free(r);
      cleanup();
      return rc;
    }
    for (uint32_t x : {x1, x2}) // the operands are not referenced again
      if (nodes[x].owned) rbgpu_set_free(nodes[x].owned), nodes[x].owned = nullptr;
    nodes.push_back(Node{r, 0, rs[0], r});
    pq.offer((uint32_t)nodes.size() - 1);
  }
  Node &last = nodes[pq.poll()];
  if (last.owned) {
    *out = last.owned;
    last.owned = nullptr;
    cleanup();
    return RB_OK;
  }
  cleanup();
  return rbgpu_set_extract(last.s, last.idx, 1, out); // one member: the reference returns it as is
}

// FastAggregation.priorityqueue_or(RoaringBitmap...) (FastAggregation.java:675-721; oracle wide_pq_or):
// the bitmaps in a java.util.PriorityQueue by getLongSizeInBytes; the two smallest are lazily OR'd —
// RoaringBitmap.lazyor (static) when neither is a temporary, this.lazyor(other) on the temporary one,
// lazyorfromlazyinputs when both are — the result re-queued with its size; the survivor is repaired
// (repairAfterLazy).  Each step is one device pairwise call in a lazy role (pairwise.hip
// lazy_or_type); its size comes back from the result's summary.  The repair is one more call, the
// survivor with itself in the kLazyRepair role (a lazy Bitmap -> LR, an exact one kept, Run -> EFF).
// BufferFastAggregation.priorityqueue_or (buffer/BufferFastAggregation.java:810-930) runs the same merges
// ordered by serializedSizeInBytes (varargs, kind kSizeSerialized) or ImmutableRoaringBitmap.
// getLongSizeInBytes (Iterator, kSizeImmutable), and returns a lone bitmap as a copy, unrepaired.
static int pq_or(rbgpu_ctx *ctx, const rbgpu_set *in, const std::vector<uint32_t> &mem, rbgpu_set **out,
                 int kind) {
  const size_t n = mem.size();
  if (n == 0) return empty_result(ctx, out);
  if (n == 1 && kind != kSizeLong) return rbgpu_set_extract(in, mem[0], 1, out); // toMutableRoaringBitmap
  std::vector<int64_t> sz;
  int rc = pq_sizes(in, kind, sz);
  if (rc) return rc;
  struct Node {
    const rbgpu_set *s;
    uint32_t idx;
    int64_t size;
    rbgpu_set *owned;
    bool tmp; // a temporary of the queue (istmp)
  };
  std::vector<Node> nodes;
  nodes.reserve(2 * n);
  for (uint32_t m : mem) nodes.push_back(Node{in, m, sz[m], nullptr, false});
  auto cmp = [&](uint32_t a, uint32_t b) { return (int)(nodes[a].size - nodes[b].size); };
  JavaHeap<uint32_t, decltype(cmp)> pq(cmp);
  for (uint32_t k = 0; k < n; ++k) pq.offer(k);
  auto cleanup = [&]() {
    for (Node &x : nodes)
      if (x.owned) rbgpu_set_free(x.owned), x.owned = nullptr;
  };
  while (pq.size() > 1) {
    const uint32_t x1 = pq.poll(), x2 = pq.poll();
    // target (left operand) and role, FastAggregation.java:690-716
    uint32_t t = x1, o = x2;
    int role = kLazyStatic;
    if (nodes[x1].tmp && nodes[x2].tmp) role = kLazyIorBf;
    else if (nodes[x2].tmp) t = x2, o = x1, role = kLazyIor;
    else if (nodes[x1].tmp) role = kLazyIor;
    const uint32_t it = nodes[t].idx, io = nodes[o].idx;
    rbgpu_set *r = nullptr;
    rc = pairwise_impl(ctx, role, nodes[t].s, nodes[o].s, &it, &io, 1, &r, nullptr);
    std::vector<int64_t> rs;
    if (!rc) rc = pq_sizes(r, kind, rs);
    if (rc) {
      if (r) rbgpu_set_free(r);
      cleanup();
      return rc;
    }
    for (uint32_t x : {x1, x2}) // the operands are not referenced again
      if (nodes[x].owned) rbgpu_set_free(nodes[x].owned), nodes[x].owned = nullptr;
    nodes.push_back(Node{r, 0, rs[0], r, true});
    pq.offer((uint32_t)nodes.size() - 1);
  }
  const Node last = nodes[pq.poll()];
  const uint32_t il = last.idx;
  rc = pairwise_impl(ctx, kLazyRepair, last.s, last.s, &il, &il, 1, out, nullptr); // repairAfterLazy
  cleanup();
  return rc;
}

int rbgpu_wide(rbgpu_ctx *ctx, int sem, const rbgpu_set *in, const uint32_t *members, uint32_t n, rbgpu_set **out) {
  return rbgpu_wide_keys(ctx, sem, in, members, n, 0, 65536, out);
}

int rbgpu_wide_keys(rbgpu_ctx *ctx, int sem, const rbgpu_set *in, const uint32_t *members, uint32_t n,
                    uint32_t key_lo, uint32_t key_hi, rbgpu_set **out) {
  SETTLE(in);
  if (!out) return fail(RB_EINVAL, "null out");
  if (key_lo > key_hi || key_hi > 65536) return fail(RB_EINVAL, "bad key range [%u, %u)", key_lo, key_hi);
  *out = nullptr;
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!in || in->ctx != ctx) return fail(RB_EINVAL, "bad input set");
  if (sem < RB_FAST_OR || sem > RB_BUFFER_PQ_XOR) return fail(RB_EINVAL, "bad semantics %d", sem);
  rc = ensure_h_begin(in);
  if (rc) return rc;
  std::vector<uint32_t> mem;
  if (members) {
    mem.assign(members, members + n);
    for (uint32_t m : mem)
      if (m >= in->nb) return fail(RB_EINVAL, "member %u out of range", m);
  } else {
    if (n > in->nb) return fail(RB_EINVAL, "n exceeds the set");
    mem.resize(n);
    for (uint32_t i = 0; i < n; ++i) mem[i] = i;
  }
  if (sem == RB_PQ_XOR || sem == RB_PQ_OR || sem >= RB_BUFFER_PQ_OR) {
    if (key_lo != 0 || key_hi != 65536) return fail(RB_EINVAL, "priorityqueue_or/xor have no key-range shards");
    switch (sem) {
    case RB_PQ_XOR: return pq_xor(ctx, in, mem, out, false);
    case RB_BUFFER_PQ_XOR: return pq_xor(ctx, in, mem, out, true);
    case RB_PQ_OR: return pq_or(ctx, in, mem, out, kSizeLong);
    case RB_BUFFER_PQ_OR: return pq_or(ctx, in, mem, out, kSizeSerialized);
    default: return pq_or(ctx, in, mem, out, kSizeImmutable);
    }
  }
  return wide_run(ctx, sem, in, mem, key_lo, key_hi, out);
}

int rbgpu_wide_cardinality(rbgpu_ctx *ctx, int op, const rbgpu_set *in, const uint32_t *members, uint32_t n,
                           uint64_t *out) {
  SETTLE(in);
  if (!out) return fail(RB_EINVAL, "null out");
  if (op != RB_AND && op != RB_OR) return fail(RB_EINVAL, "wide cardinality supports AND and OR");
  rbgpu_set *r = nullptr;
  int rc = rbgpu_wide(ctx, op == RB_AND ? RB_WORKSHY_AND : RB_FAST_OR, in, members, n, &r);
  if (rc) return rc;
  rc = rbgpu_set_cardinalities(r, out);
  rbgpu_set_free(r);
  return rc;
}

// ---------------------------------------------------------------- bit-sliced index
int rbgpu_bsi_compare_keys(rbgpu_ctx *ctx, const rbgpu_set *bsi, int op, uint64_t start_or_value, uint64_t end,
                           uint64_t min_value, uint64_t max_value, const rbgpu_set *found, uint32_t key_lo,
                           uint32_t key_hi, rbgpu_set **out) {
  SETTLE(bsi, found);
  if (!out) return fail(RB_EINVAL, "null out");
  *out = nullptr;
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!bsi || bsi->ctx != ctx) return fail(RB_EINVAL, "bad bsi set");
  if (bsi->nb < 1 || bsi->nb > 65) return fail(RB_EINVAL, "a bsi set holds 0..64 slices and the existence bitmap");
  if (found && (found->ctx != ctx || found->nb != 1)) return fail(RB_EINVAL, "foundSet must be a one-bitmap set");
  if (op < RB_BSI_EQ || op > RB_BSI_RANGE) return fail(RB_EINVAL, "not support operation!");
  if (key_lo > key_hi || key_hi > 65536) return fail(RB_EINVAL, "bad key range [%u, %u)", key_lo, key_hi);
  rc = ensure_h_begin(bsi);
  if (rc) return rc;
  return bsi_compare(ctx, bsi, op, start_or_value, end, min_value, max_value, found, key_lo, key_hi, out);
}

int rbgpu_bsi_compare(rbgpu_ctx *ctx, const rbgpu_set *bsi, int op, uint64_t start_or_value, uint64_t end,
                      uint64_t min_value, uint64_t max_value, const rbgpu_set *found, rbgpu_set **out) {
  return rbgpu_bsi_compare_keys(ctx, bsi, op, start_or_value, end, min_value, max_value, found, 0, 65536, out);
}

int rbgpu_set_setup_stats(const rbgpu_set *s, double *ms, uint64_t *bytes) {
  if (!s || !ms || !bytes) return fail(RB_EINVAL, "null argument");
  *ms = s->derive_ms;
  *bytes = s->derive_bytes;
  return RB_OK;
}

int rbgpu_set_setup_parts(const rbgpu_set *s, double *ms, uint64_t *bytes) {
  if (!s || !ms || !bytes) return fail(RB_EINVAL, "null argument");
  for (int i = 0; i < 4; ++i) {
    ms[i] = s->part_ms[i];
    bytes[i] = s->part_bytes[i];
  }
  return RB_OK;
}

int rbgpu_set_extract(const rbgpu_set *s, uint32_t first, uint32_t count, rbgpu_set **out) {
  SETTLE(s);
  if (!s || !out) return fail(RB_EINVAL, "null argument");
  *out = nullptr;
  if ((uint64_t)first + count > s->nb) return fail(RB_EINVAL, "bitmap range out of bounds");
  HostSoA h;
  int rc = download_host(s, first, count, h);
  if (rc) return rc;
  return upload_host(s->ctx, h, out);
}

int rbgpu_generate_bsi(rbgpu_ctx *ctx, uint32_t nslices, uint64_t nrows, uint64_t seed, rbgpu_set **out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!out) return fail(RB_EINVAL, "null out");
  *out = nullptr;
  return generate_bsi(ctx, nslices, nrows, seed, 0, 65536, out);
}

int rbgpu_generate_bsi_keys(rbgpu_ctx *ctx, uint32_t nslices, uint64_t nrows, uint64_t seed, uint32_t key_lo,
                            uint32_t key_hi, rbgpu_set **out) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!out) return fail(RB_EINVAL, "null out");
  *out = nullptr;
  return generate_bsi(ctx, nslices, nrows, seed, key_lo, key_hi, out);
}

// ---------------------------------------------------------------- generator
int rbgpu_generate(rbgpu_ctx *ctx, int workload, uint32_t n, uint64_t seed, rbgpu_set **a, rbgpu_set **b) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!a) return fail(RB_EINVAL, "null out");
  *a = nullptr;
  if (b) *b = nullptr;
  if (workload == RB_WL_FILTER_POSTING && !b) return fail(RB_EINVAL, "filter/posting workload needs two outputs");
  return generate_sets(ctx, workload, n, seed, 0, 65536, a, b);
}

int rbgpu_generate_keys(rbgpu_ctx *ctx, int workload, uint32_t n, uint64_t seed, uint32_t key_lo, uint32_t key_hi,
                        rbgpu_set **a) {
  int rc = check_ctx(ctx);
  if (rc) return rc;
  if (!a) return fail(RB_EINVAL, "null out");
  *a = nullptr;
  if (workload == RB_WL_FILTER_POSTING) return fail(RB_EINVAL, "key ranges apply to the wide workloads");
  return generate_sets(ctx, workload, n, seed, key_lo, key_hi, a, nullptr);
}

} // extern "C"
