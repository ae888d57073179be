#include <algorithm>
// generate.hip — device-side synthetic container generator for the benchmark workloads
// (SURVEY §8d "rbgen"): SplitMix64 streams keyed by (seed, container id, lane), every container
// finished with runOptimize semantics like RoaringBitmapWriter(runCompress=true)
// (ContainerAppender.java:130-137).  Two passes with identical regeneration: measure, emit.
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

__device__ __forceinline__ uint64_t splitmix(uint64_t &x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

enum { kGenArray = 0, kGenBitmap = 1, kGenRuns = 2, kGenCoreRuns = 3, kGenHalfLimit = 4, kGenFullLimit = 5 };

// word mask of [a, b) restricted to container word wi
__device__ __forceinline__ uint64_t range_mask(int wi, int a, int b) {
  int lo = max(a, wi * 64), hi = min(b, wi * 64 + 64);
  if (lo >= hi) return 0;
  return (~0ull << (lo & 63)) & (~0ull >> (63 - ((hi - 1) & 63)));
}

__device__ void gen_container(const GenSpec &g, uint64_t cid, uint32_t *s, uint64_t (&w)[kW], int lane) {
  const int target = g.target[cid];
  const uint32_t param = g.param[cid];
  // content streams are keyed by the container's uid (not its position in the set), so a key-range
  // shard regenerates exactly the containers of the full dataset
  const uint64_t uid = g.uid[cid];
  uint64_t ls = g.seed ^ (uid * 0xD1B54A32D192ED03ull) ^ ((uint64_t)(lane + 1) * 0x8CB92BA72F3D8DD7ull);
  uint64_t us = g.seed ^ (uid * 0xD1B54A32D192ED03ull) ^ 0x5851F42D4C957F2Dull; // wave-uniform stream
  if (target == kGenBitmap) {
#pragma unroll
    for (int j = 0; j < kW; ++j) {
      uint64_t x = 0;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        uint64_t r = splitmix(ls);
        x = ((param >> b) & 1) ? (x | r) : (x & r);
      }
      w[j] = x;
    }
  } else if (target == kGenArray) {
    lds_zero(s, lane);
    wave_lds_sync();
    for (uint32_t i = lane; i < param; i += 64) {
      uint32_t v = (uint32_t)splitmix(ls) & 0xFFFF;
      atomicOr(&s[v >> 5], 1u << (v & 31));
    }
    wave_lds_sync();
    lds_read_words(s, w, lane);
    wave_lds_sync();
  } else if (target == kGenRuns) {
    // 2r random cut points toggled, membership = prefix-xor (same machinery as expand_runs)
    lds_zero(s, lane);
    wave_lds_sync();
    for (uint32_t i = lane; i < 2 * param; i += 64) {
      uint32_t v = (uint32_t)splitmix(ls) & 0xFFFF;
      atomicXor(&s[v >> 5], 1u << (v & 31));
    }
    wave_lds_sync();
    uint64_t t[kW];
    lds_read_words(s, t, lane);
    wave_lds_sync();
    uint32_t q = 0, p0 = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t a = __popcll(t[2 * k]) & 1, b = __popcll(t[2 * k + 1]) & 1;
      q |= (a ^ b) << k;
      p0 |= a << k;
    }
    const uint32_t incl = wave_xscan_xor(q, lane), excl = incl ^ q;
    const uint32_t tot = readlane(incl, 63);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t c0 = (__popc(tot & ((1u << k) - 1)) & 1) ^ ((excl >> k) & 1);
      uint32_t c1 = c0 ^ ((p0 >> k) & 1);
      w[2 * k] = prefix_xor64(t[2 * k]) ^ (c0 ? ~0ull : 0ull);
      w[2 * k + 1] = prefix_xor64(t[2 * k + 1]) ^ (c1 ? ~0ull : 0ull);
    }
  } else if (target == kGenHalfLimit || target == kGenFullLimit) {
    // BSI slice (random value bit per row, density 1/2) / existence bitmap, rows [0, param)
#pragma unroll
    for (int j = 0; j < kW; ++j) {
      const int wi = 128 * (j >> 1) + 2 * lane + (j & 1);
      const uint64_t m = range_mask(wi, 0, (int)param);
      w[j] = target == kGenFullLimit ? m : (splitmix(ls) & m);
    }
  } else { // kGenCoreRuns: shared core run [s_k, s_k+1024) + r-1 random runs (r ~ U[1,8], len U[1,256])
    const int core = (int)(param % 64512u);
    int ra[8], rb[8];
    ra[0] = core;
    rb[0] = core + 1024;
    const int r = 1 + (int)(splitmix(us) % 8);
    for (int i = 1; i < 8; ++i) {
      uint64_t z = splitmix(us);
      int st = (int)(z & 0xFFFF), len = 1 + (int)((z >> 16) % 256);
      ra[i] = st;
      rb[i] = i < r ? min(st + len, kSpan) : st;
    }
#pragma unroll
    for (int j = 0; j < kW; ++j) {
      const int wi = 128 * (j >> 1) + 2 * lane + (j & 1);
      uint64_t x = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) x |= range_mask(wi, ra[i], rb[i]);
      w[j] = x;
    }
  }
}

__device__ __forceinline__ void gen_finish(uint64_t (&w)[kW], int lane, int &c, int &r) {
  metrics(w, lane, true, c, r);
  if (c == 0) { // containers are never empty
    if (lane == 0) w[0] |= 1;
    metrics(w, lane, true, c, r);
  }
}

__global__ __launch_bounds__(256) void k_gen_measure(GenSpec g, uint64_t n, uint8_t *type, uint32_t *card,
                                                     uint16_t *nruns, uint64_t *big, uint64_t *small) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4][2048];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // grid-stride over containers: a launch may not exceed 2^32 work-items per dimension
  for (uint64_t cid = (uint64_t)blockIdx.x * 4 + wv; cid < n; cid += (uint64_t)gridDim.x * 4) {
    uint64_t w[kW];
    gen_container(g, cid, lds[wv], w, lane);
    int c, r;
    gen_finish(w, lane, c, r);
    const int ty = type_runopt(c, r);
    if (lane == 0) {
      type[cid] = (uint8_t)ty;
      card[cid] = (uint32_t)c;
      nruns[cid] = (uint16_t)(ty == kRun ? r : 0);
      big[cid] = ty == kBitmap;
      small[cid] = ty == kBitmap ? 0 : round16(payload_bytes(ty, c, r));
    }
    wave_lds_sync();
  }
}

__global__ __launch_bounds__(256) void k_gen_emit(GenSpec g, uint64_t n, const uint8_t *type, const uint64_t *off,
                                                  uint8_t *payload) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4][2048];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint64_t cid = (uint64_t)blockIdx.x * 4 + wv; cid < n; cid += (uint64_t)gridDim.x * 4) {
    uint64_t w[kW];
    gen_container(g, cid, lds[wv], w, lane);
    int c, r;
    gen_finish(w, lane, c, r);
    emit_container(type[cid], w, c, r, payload + off[cid], lds[wv], lane);
    wave_lds_sync();
  }
}

void launch_gen_measure(const GenSpec &g, uint64_t n, uint8_t *type, uint32_t *card, uint16_t *nruns, uint64_t *big,
                        uint64_t *small, hipStream_t st) {
  if (!n) return;
  k_gen_measure<<<(unsigned)std::min<uint64_t>((n + 3) / 4, 1u << 20), 256, 0, st>>>(g, n, type, card, nruns, big, small);
}
void launch_gen_emit(const GenSpec &g, uint64_t n, const uint8_t *type, const uint64_t *off, uint8_t *payload,
                     hipStream_t st) {
  if (!n) return;
  k_gen_emit<<<(unsigned)std::min<uint64_t>((n + 3) / 4, 1u << 20), 256, 0, st>>>(g, n, type, off, payload);
}

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_generate() {}
void warm_generate(hipStream_t st) { k_warm_generate<<<1, 64, 0, st>>>(); }

} // namespace rbg

// ===================================================================== host side
#include "internal.hpp"

namespace rbg {
namespace {
struct HostRng {
  uint64_t x;
  uint64_t next() {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint32_t below(uint32_t n) { return (uint32_t)(next() % n); }
};
struct GenStructure {
  uint32_t nb = 0;
  std::vector<uint64_t> begin{0};
  std::vector<uint16_t> key;
  std::vector<uint8_t> target;
  std::vector<uint32_t> param;
  std::vector<uint64_t> uid;
  void add(uint16_t k, uint8_t t, uint32_t p, uint64_t u = ~0ull) {
    uid.push_back(u == ~0ull ? (uint64_t)key.size() : u);
    key.push_back(k);
    target.push_back(t);
    param.push_back(p);
  }
  void close() {
    ++nb;
    begin.push_back(key.size());
  }
};
// Bitmap density U[0.07, 0.93] as a numerator over 256
uint32_t dense_num(HostRng &r) { return 18 + r.below(238 - 18 + 1); }

// Per-(bitmap, key) decision stream for the wide workloads: independent of the key range asked
// for, so shards [lo, hi) of one seed partition the same dataset.
HostRng key_rng(uint64_t seed, uint32_t i, uint32_t k) {
  HostRng r{seed * 0x2545F4914F6CDD1Dull ^ ((uint64_t)i << 20) * 0x9E3779B97F4A7C15ull ^
            ((uint64_t)k + 1) * 0xD6E8FEB86659FD93ull};
  r.next();
  return r;
}

// Config-2 type mix as cumulative per-mille cuts (filter A, filter A+B, posting A, posting A+B).
// rbgpu_internal_set_mix changes it for kernel studies (scripts/mix_study.py); the bench uses the
// SURVEY §8d defaults.
int g_mix[4] = {400, 700, 700, 800};

void structure(int workload, uint32_t n, uint64_t seed, uint32_t key_lo, uint32_t key_hi,
               std::vector<GenStructure> &out) {
  HostRng r{seed * 0x2545F4914F6CDD1Dull + 0x9E3779B97F4A7C15ull};
  if (workload == RB_WL_FILTER_POSTING) {
    out.resize(2);
    GenStructure &f = out[0], &p = out[1];
    for (uint32_t i = 0; i < n; ++i) { // filters: all 4 keys of the 2^18 universe, A/B/R = .4/.3/.3
      for (uint16_t k = 0; k < 4; ++k) {
        uint32_t u = r.below(1000);
        if (u < (uint32_t)g_mix[0]) f.add(k, kGenArray, 1 + r.below(4096));
        else if (u < (uint32_t)g_mix[1]) f.add(k, kGenBitmap, dense_num(r));
        else f.add(k, kGenRuns, 1 + r.below(1024));
      }
      f.close();
    }
    for (uint32_t i = 0; i < n; ++i) { // posting lists: key w.p. .5 (>= 1), A/B/R = .7/.1/.2
      uint32_t mask = r.below(16);
      if (!mask) mask = 1u << r.below(4);
      for (uint16_t k = 0; k < 4; ++k) {
        if (!((mask >> k) & 1)) continue;
        uint32_t u = r.below(1000);
        if (u < (uint32_t)g_mix[2]) p.add(k, kGenArray, 1 + r.below(2048));
        else if (u < (uint32_t)g_mix[3]) p.add(k, kGenBitmap, dense_num(r));
        else p.add(k, kGenRuns, 1 + r.below(1024));
      }
      p.close();
    }
    return;
  }
  out.resize(1);
  GenStructure &g = out[0];
  for (uint32_t i = 0; i < n; ++i) {
    for (uint32_t k = key_lo; k < key_hi; ++k) {
      const uint64_t uid = ((uint64_t)i << 16) | k;
      if (workload == RB_WL_WIDE_RUNS) { // every key; shared core run per key (config 4)
        uint64_t h = (uint64_t)k * 0x9E3779B97F4A7C15ull;
        h ^= h >> 29;
        g.add((uint16_t)k, kGenCoreRuns, (uint32_t)(h >> 32), uid);
        continue;
      }
      HostRng kr = key_rng(seed, i, k);
      if (kr.below(16) != 0) continue; // key present w.p. 1/16 (config 3)
      if (workload == RB_WL_WIDE_DENSE) {
        g.add((uint16_t)k, kGenBitmap, 16 + kr.below(9), uid); // d ~ U[1/16, 3/32]
      } else {
        uint32_t u = kr.below(1000);
        if (u < 700) g.add((uint16_t)k, kGenBitmap, 16 + kr.below(9), uid);
        else if (u < 900) g.add((uint16_t)k, kGenArray, 1 + kr.below(4096), uid);
        else g.add((uint16_t)k, kGenRuns, 1 + kr.below(2047), uid);
      }
    }
    g.close();
  }
}

int materialize(rbgpu_ctx *ctx, const GenStructure &gs, uint64_t seed, rbgpu_set **out) {
  hipStream_t st = ctx->stream;
  DevPool &pool = ctx->pool;
  const uint64_t n = gs.key.size();
  rbgpu_set *s = new rbgpu_set;
  int rc = set_alloc(ctx, s, gs.nb, n, 16);
  if (rc) {
    delete s;
    return rc;
  }
  uint8_t *d_target;
  uint32_t *d_param;
  uint64_t *d_uid;
  uint64_t *d_big, *d_small, *d_bidx, *d_soff, *d_tmp;
  const uint64_t tmpw = std::max<uint64_t>(scan_tmp_words(n + 1), 1);
  const uint64_t nn = std::max<uint64_t>(n, 1);
  if (pool.alloc((void **)&d_target, nn) || pool.alloc((void **)&d_param, nn * 4) ||
      pool.alloc((void **)&d_uid, nn * 8) ||
      pool.alloc((void **)&d_big, (nn + 1) * 8) || pool.alloc((void **)&d_small, (nn + 1) * 8) ||
      pool.alloc((void **)&d_bidx, (nn + 1) * 8) || pool.alloc((void **)&d_soff, (nn + 1) * 8) ||
      pool.alloc((void **)&d_tmp, tmpw * 8)) {
    set_release(s);
    delete s;
    return fail(RB_ENOMEM, "generator workspace for %llu containers", (unsigned long long)n);
  }
  HIPCHK(hipMemcpyAsync(s->begin, gs.begin.data(), (gs.nb + 1) * 8, hipMemcpyHostToDevice, st));
  if (n) {
    HIPCHK(hipMemcpyAsync(s->key, gs.key.data(), n * 2, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_target, gs.target.data(), n, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_param, gs.param.data(), n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_uid, gs.uid.data(), n * 8, hipMemcpyHostToDevice, st));
  }
  GenSpec g{s->key, d_target, d_param, d_uid, seed};
  launch_gen_measure(g, n, s->type, s->card, s->nruns, d_big, d_small, st);
  scan_exclusive(d_big, d_bidx, n, d_tmp, st);
  scan_exclusive(d_small, d_soff, n, d_tmp, st);
  uint64_t tot[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(&tot[0], d_bidx + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipMemcpyAsync(&tot[1], d_soff + n, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  LAUNCHCHK();
  const uint64_t small_base = tot[0] * kBitmapBytes, total = small_base + tot[1];
  launch_layout(d_big, d_bidx, d_soff, small_base, s->off, n, st);
  pool.release(s->payload);
  if (pool.alloc((void **)&s->payload, std::max<uint64_t>(total, 16))) {
    s->payload = nullptr;
    set_release(s);
    delete s;
    return fail(RB_ENOMEM, "generator payload of %llu bytes", (unsigned long long)total);
  }
  s->payload_bytes = total;
  launch_gen_emit(g, n, s->type, s->off, s->payload, st);
  HIPCHK(hipStreamSynchronize(st));
  LAUNCHCHK();
  for (void *p : {(void *)d_target, (void *)d_param, (void *)d_uid, (void *)d_big, (void *)d_small, (void *)d_bidx, (void *)d_soff,
                  (void *)d_tmp})
    pool.release(p);
  s->h_begin = gs.begin;
  *out = s;
  return RB_OK;
}
} // namespace

void set_mix(const int *m) {
  for (int i = 0; i < 4; ++i) g_mix[i] = m[i];
}

// Containers are a function of (seed, slice, key) alone, so a key-range shard holds exactly the
// whole index's containers for its keys.
int generate_bsi(rbgpu_ctx *ctx, uint32_t nslices, uint64_t nrows, uint64_t seed, uint32_t key_lo, uint32_t key_hi,
                 rbgpu_set **out) {
  if (nslices > 64 || nrows > (1ull << 32)) return fail(RB_EINVAL, "bsi: at most 64 slices over 2^32 rows");
  if (key_lo > key_hi || key_hi > 65536) return fail(RB_EINVAL, "bad key range [%u, %u)", key_lo, key_hi);
  GenStructure g;
  const uint64_t nkeys = std::min<uint64_t>((nrows + 65535) / 65536, key_hi);
  for (uint32_t b = 0; b <= nslices; ++b) { // slices 0..nslices-1, then the existence bitmap
    for (uint64_t k = key_lo; k < nkeys; ++k) {
      const uint32_t limit = (uint32_t)std::min<uint64_t>(65536, nrows - k * 65536);
      g.add((uint16_t)k, b < nslices ? kGenHalfLimit : kGenFullLimit, limit, ((uint64_t)b << 16) | k);
    }
    g.close();
  }
  return materialize(ctx, g, seed * 31 + 5, out);
}

int generate_sets(rbgpu_ctx *ctx, int workload, uint32_t n, uint64_t seed, uint32_t key_lo, uint32_t key_hi,
                  rbgpu_set **a, rbgpu_set **b) {
  if (workload < RB_WL_FILTER_POSTING || workload > RB_WL_WIDE_RUNS) return fail(RB_EINVAL, "bad workload %d", workload);
  if (key_lo > key_hi || key_hi > 65536) return fail(RB_EINVAL, "bad key range [%u, %u)", key_lo, key_hi);
  std::vector<GenStructure> gs;
  structure(workload, n, seed, key_lo, key_hi, gs);
  int rc = materialize(ctx, gs[0], seed * 31 + 1, a);
  if (rc) return rc;
  if (gs.size() > 1) {
    rc = materialize(ctx, gs[1], seed * 31 + 2, b);
    if (rc) {
      rbgpu_set_free(*a);
      *a = nullptr;
      return rc;
    }
  }
  return RB_OK;
}

} // namespace rbg
