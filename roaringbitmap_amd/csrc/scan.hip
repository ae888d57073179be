// scan.hip — device exclusive prefix sums (u64) used to lay out variable-size outputs.
#include "kernels.hpp"

namespace rbg {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 4; // per thread -> 1024 per block

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *sh, uint64_t &total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t t = (uint64_t)__shfl_up((unsigned long long)incl, d);
    if (lane >= d) incl += t;
  }
  if (lane == 63) sh[wave] = incl;
  __syncthreads();
  uint64_t woff = 0;
  for (int i = 0; i < wave; ++i) woff += sh[i];
  total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return woff + incl - v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_partials(const uint64_t *in, uint64_t n, uint64_t *partials) {
  __shared__ uint64_t sh[4];
  const uint64_t base = (uint64_t)blockIdx.x * kScanThreads * kScanItems + threadIdx.x * kScanItems;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i)
    if (base + i < n) s += in[base + i];
  uint64_t total;
  block_excl_scan(s, sh, total);
  if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const uint64_t *in, uint64_t n, const uint64_t *offs,
                                                             uint64_t *out) {
  __shared__ uint64_t sh[4];
  const uint64_t base = (uint64_t)blockIdx.x * kScanThreads * kScanItems + threadIdx.x * kScanItems;
  uint64_t v[kScanItems], s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = base + i < n ? in[base + i] : 0;
    s += v[i];
  }
  uint64_t total;
  uint64_t run = block_excl_scan(s, sh, total) + (offs ? offs[blockIdx.x] : 0);
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kScanThreads - 1)
    out[n] = (offs ? offs[blockIdx.x] : 0) + total;
}

// out[i] = sum(in[0..i)), out[n] = total.  `tmp` must hold scan_tmp_words(n) words.
uint64_t scan_tmp_words(uint64_t n) {
  const uint64_t per = kScanThreads * kScanItems;
  uint64_t nb = (n + per - 1) / per;
  if (nb <= 1) return 0;
  return 2 * (nb + 1) + scan_tmp_words(nb);
}

// tmp words for scan_exclusive_multi over k arrays of n
uint64_t scan_multi_tmp_words(uint64_t n, int k) {
  const uint64_t per = kScanThreads * kScanItems, nb = (n + per - 1) / per;
  return std::max<uint64_t>(scan_tmp_words(n), 2 * (uint64_t)k * (nb + 1));
}

void scan_exclusive(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *tmp, hipStream_t st) {
  const uint64_t per = kScanThreads * kScanItems;
  uint64_t nb = (n + per - 1) / per;
  if (nb == 0) {
    (void)hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    return;
  }
  if (nb == 1) {
    k_scan_apply<<<1, kScanThreads, 0, st>>>(in, n, nullptr, out);
    return;
  }
  uint64_t *partials = tmp, *poffs = tmp + (nb + 1);
  k_scan_partials<<<(unsigned)nb, kScanThreads, 0, st>>>(in, n, partials);
  scan_exclusive(partials, poffs, nb, tmp + 2 * (nb + 1), st);
  k_scan_apply<<<(unsigned)nb, kScanThreads, 0, st>>>(in, n, poffs, out);
}

struct Multi {
  const uint64_t *in[4];
  uint64_t *out[4];
};
__global__ __launch_bounds__(kScanThreads) void k_scan_multi(Multi m, uint64_t n, uint64_t *totals) {
  __shared__ uint64_t sh[4];
  const uint64_t *in = m.in[blockIdx.y];
  uint64_t *out = m.out[blockIdx.y];
  const uint64_t base = threadIdx.x * kScanItems;
  uint64_t v[kScanItems], s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = base + i < n ? in[base + i] : 0;
    s += v[i];
  }
  uint64_t total;
  uint64_t run = block_excl_scan(s, sh, total);
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (threadIdx.x == 0) {
    out[n] = total;
    totals[blockIdx.y] = total;
  }
}
// partials of array blockIdx.y at tmp + y * stride
__global__ __launch_bounds__(kScanThreads) void k_scan_partials_multi(Multi m, uint64_t n, uint64_t *tmp,
                                                                      uint64_t stride) {
  __shared__ uint64_t sh[4];
  const uint64_t *in = m.in[blockIdx.y];
  const uint64_t base = (uint64_t)blockIdx.x * kScanThreads * kScanItems + threadIdx.x * kScanItems;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i)
    if (base + i < n) s += in[base + i];
  uint64_t total;
  block_excl_scan(s, sh, total);
  if (threadIdx.x == 0) tmp[blockIdx.y * stride + blockIdx.x] = total;
}
// out[y][i] = scanned block offset + in-block exclusive scan; the last block writes out[y][n] from
// the array's total (pm.out[y][nb], written by k_scan_multi)
__global__ __launch_bounds__(kScanThreads) void k_scan_apply_multi(Multi m, uint64_t n, Multi pm,
                                                                   const uint64_t *totals) {
  __shared__ uint64_t sh[4];
  const uint64_t *in = m.in[blockIdx.y];
  uint64_t *out = m.out[blockIdx.y];
  const uint64_t off = pm.out[blockIdx.y][blockIdx.x];
  const uint64_t base = (uint64_t)blockIdx.x * kScanThreads * kScanItems + threadIdx.x * kScanItems;
  uint64_t v[kScanItems], s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = base + i < n ? in[base + i] : 0;
    s += v[i];
  }
  uint64_t total;
  uint64_t run = block_excl_scan(s, sh, total) + off;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = totals[blockIdx.y];
}
// k <= 4 short arrays (per-block totals of a per-block layout) in ONE launch: a block per array
// loops over chunks of 1024 with a carried offset.  out[y][i] = sum(in[y][0..i)), out[y][n] = the
// sum, and totals[y] = the sum when totals is non-null.
__global__ __launch_bounds__(kScanThreads) void k_scan_loop_multi(Multi m, uint64_t n, uint64_t *totals) {
  __shared__ uint64_t sh[4];
  const uint64_t *in = m.in[blockIdx.y];
  uint64_t *out = m.out[blockIdx.y];
  uint64_t carry = 0;
  for (uint64_t c0 = 0; c0 < n; c0 += (uint64_t)kScanThreads * kScanItems) {
    const uint64_t base = c0 + threadIdx.x * kScanItems;
    uint64_t v[kScanItems], s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
      v[i] = base + i < n ? in[base + i] : 0;
      s += v[i];
    }
    uint64_t total;
    uint64_t run = block_excl_scan(s, sh, total) + carry;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
      if (base + i < n) out[base + i] = run;
      run += v[i];
    }
    carry += total;
  }
  if (threadIdx.x == 0) {
    out[n] = carry;
    if (totals) totals[blockIdx.y] = carry;
  }
}
void scan_blocks_multi(const uint64_t *const *in, uint64_t *const *out, int k, uint64_t n, uint64_t *totals,
                       hipStream_t st) {
  Multi m{};
  for (int i = 0; i < k; ++i) {
    m.in[i] = in[i];
    m.out[i] = out[i];
  }
  k_scan_loop_multi<<<dim3(1, k), kScanThreads, 0, st>>>(m, n, totals);
}

__global__ void k_gather_totals(Multi m, uint64_t n, uint64_t *totals) { totals[threadIdx.x] = m.out[threadIdx.x][n]; }

void scan_exclusive_multi(const uint64_t *const *in, uint64_t *const *out, int k, uint64_t n, uint64_t *tmp,
                          uint64_t *totals, hipStream_t st) {
  Multi m{};
  for (int i = 0; i < k; ++i) {
    m.in[i] = in[i];
    m.out[i] = out[i];
  }
  if (n <= (uint64_t)kScanThreads * kScanItems) {
    k_scan_multi<<<dim3(1, k), kScanThreads, 0, st>>>(m, n, totals);
    return;
  }
  const uint64_t per = kScanThreads * kScanItems, nb = (n + per - 1) / per;
  if (nb <= per) {
    // two levels for all k arrays at once: block partials (grid nb x k), one block per array scans
    // its partials (and writes the totals), then every block applies its offset — 3 launches
    // instead of 3k + 1 (config 2: 1M segments, 4 count arrays)
    Multi pm{};
    for (int i = 0; i < k; ++i) {
      pm.in[i] = tmp + i * (nb + 1);
      pm.out[i] = tmp + (k + i) * (nb + 1);
    }
    k_scan_partials_multi<<<dim3((unsigned)nb, k), kScanThreads, 0, st>>>(m, n, tmp, nb + 1);
    k_scan_multi<<<dim3(1, k), kScanThreads, 0, st>>>(pm, nb, totals);
    k_scan_apply_multi<<<dim3((unsigned)nb, k), kScanThreads, 0, st>>>(m, n, pm, totals);
    return;
  }
  for (int i = 0; i < k; ++i) scan_exclusive(in[i], out[i], n, tmp, st);
  k_gather_totals<<<1, k, 0, st>>>(m, n, totals);
}

// An empty dispatch (DeriveTimer): the stream's next event is stamped only once the queue has reached it.
__global__ void k_noop() {}
void launch_noop(hipStream_t st) { k_noop<<<1, 64, 0, st>>>(); }

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_scan() {}
void warm_scan(hipStream_t st) { k_warm_scan<<<1, 64, 0, st>>>(); }

} // namespace rbg
