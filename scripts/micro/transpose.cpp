// Microbenchmark: 8-B record transpose [M members][K keys] -> [K][M] (naive_xor's key-major records), against a
// plain copy of the same bytes.  M = 4096, K = 65536 (2 GiB each way).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
constexpr uint32_t M = 4096, K = 65536;
__global__ void k_copy(const uint4 *__restrict__ a, uint4 *__restrict__ b, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) b[i] = a[i];
}
// baseline: 64 x 64 tiles (the library's)
__global__ __launch_bounds__(256) void k_t64(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst) {
  __shared__ uint64_t tile[64][65];
  const uint32_t k0 = blockIdx.x * 64, m0 = blockIdx.y * 64, t = threadIdx.x, kx = t & 63, ry = t >> 6;
  uint64_t v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = src[(uint64_t)(m0 + ry + 4 * j) * K + k0 + kx];
#pragma unroll
  for (int j = 0; j < 16; ++j) tile[ry + 4 * j][kx] = v[j];
  __syncthreads();
  for (uint32_t r = ry; r < 64; r += 4) dst[(uint64_t)(k0 + r) * M + m0 + kx] = tile[kx][r];
}
// 16-B accesses: 128 keys x 64 members, each lane moves 2 records per access
__global__ __launch_bounds__(256) void k_t128(const uint64_t *__restrict__ src, uint64_t *__restrict__ dst) {
  __shared__ uint64_t tile[64][129];
  const uint32_t k0 = blockIdx.x * 128, m0 = blockIdx.y * 64, t = threadIdx.x, kx = t & 63, ry = t >> 6;
  uint4 v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = reinterpret_cast<const uint4 *>(src + (uint64_t)(m0 + ry + 4 * j) * K + k0)[kx];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    tile[ry + 4 * j][2 * kx] = (uint64_t)v[j].x | ((uint64_t)v[j].y << 32);
    tile[ry + 4 * j][2 * kx + 1] = (uint64_t)v[j].z | ((uint64_t)v[j].w << 32);
  }
  __syncthreads();
  // writes: key row r, members m0 + 2 kx', 16 B per lane: 32 lanes per row, 2 rows per wave-instruction
  const uint32_t lx = t & 31, rr = t >> 5; // 8 rows per pass
  for (uint32_t r = rr; r < 128; r += 8) {
    const uint64_t a = tile[2 * lx][r], b = tile[2 * lx + 1][r];
    reinterpret_cast<uint4 *>(dst + (uint64_t)(k0 + r) * M + m0)[lx] =
        make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
  }
}
int main() {
  uint64_t *a, *b;
  const uint64_t n = (uint64_t)M * K;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, n * 8));
  CK(hipMemset(a, 1, n * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(e0));
      if (v == 0) k_copy<<<256 * 16, 256>>>((const uint4 *)a, (uint4 *)b, n / 2);
      else if (v == 1) k_t64<<<dim3(K / 64, M / 64), 256>>>(a, b);
      else k_t128<<<dim3(K / 128, M / 64), 256>>>(a, b);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) printf("%s %.3f ms %.2f TB/s\n", v == 0 ? "copy" : v == 1 ? "t64" : "t128", ms, 2.0 * n * 8 / ms / 1e9);
    }
  }
  return 0;
}
