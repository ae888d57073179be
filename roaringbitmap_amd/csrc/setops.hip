// setops.hip — small per-set utilities: per-bitmap cardinality, payload gather for downloads.
#include <algorithm>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

// RoaringBitmap.getCardinality (sum of container cardinalities) — one wave per bitmap.
__global__ __launch_bounds__(256) void k_bitmap_cards(SetView s, uint32_t nb, uint64_t *out) {
  const uint64_t b = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const int lane = lane_id();
  uint64_t acc = 0;
  for (uint64_t i = s.begin[b] + lane; i < s.begin[b + 1]; i += 64) acc += s.card[i];
  acc = wave_sum_u64(acc);
  if (lane == 0) out[b] = acc;
}
void launch_bitmap_cards(const SetView &s, uint32_t nbitmaps, uint64_t *out, hipStream_t st) {
  if (!nbitmaps) return;
  k_bitmap_cards<<<(nbitmaps + 3) / 4, 256, 0, st>>>(s, nbitmaps, out);
}

// Copy n payloads (sizes multiple of 16 after rounding) from src offsets to dst offsets.
__global__ __launch_bounds__(256) void k_gather(const uint8_t *src, const uint64_t *soff, const uint64_t *bytes,
                                                uint8_t *dst, const uint64_t *doff, uint64_t n) {
  // grid-stride (a launch may not exceed 2^32 work-items per dimension)
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (uint64_t)gridDim.x * 4)
    copy_payload(src + soff[i], dst + doff[i], bytes[i], lane_id());
}
void launch_gather(const uint8_t *src, const uint64_t *soff, const uint64_t *bytes, uint8_t *dst,
                   const uint64_t *doff, uint64_t n, hipStream_t st) {
  if (!n) return;
  k_gather<<<(unsigned)(n < (4ull << 20) ? (n + 3) / 4 : (1u << 20)), 256, 0, st>>>(src, soff, bytes, dst, doff, n);
}

// Payload layout of generated / uploaded sets: Bitmaps first at 8 KiB strides, then the rest.
__global__ __launch_bounds__(256) void k_layout(const uint64_t *bigflag, const uint64_t *bidx, const uint64_t *soff,
                                                uint64_t small_base, uint64_t *off, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  off[i] = bigflag[i] ? bidx[i] * (uint64_t)kBitmapBytes : small_base + soff[i];
}
void launch_layout(const uint64_t *bigflag, const uint64_t *bidx, const uint64_t *soff, uint64_t small_base,
                   uint64_t *off, uint64_t n, hipStream_t st) {
  if (!n) return;
  k_layout<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(bigflag, bidx, soff, small_base, off, n);
}

// ---- derived metadata of an immutable set (rbgpu_set::mrec / krec / dense_lo)
// mrec[i] = pack_rec(container i): one streaming pass over the four metadata arrays.
__global__ __launch_bounds__(256) void k_pack_records(SetView s, uint64_t n, uint64_t *__restrict__ mrec) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    mrec[i] = pack_rec(s.type[i], s.card[i], s.nruns[i], s.off[i]);
}
void launch_pack_records(const SetView &s, uint64_t n, uint64_t *mrec, hipStream_t st) {
  if (!n) return;
  k_pack_records<<<(unsigned)std::min<uint64_t>((n + 255) / 256, 1u << 16), 256, 0, st>>>(s, n, mrec);
}
// bad[0] |= 1 when a bitmap does not hold exactly the keys [lo, lo + cnt): its container count is cnt
// and, its keys being strictly increasing, its first key lo and its last lo + cnt - 1.
__global__ __launch_bounds__(256) void k_dense_check(SetView s, uint32_t nb, uint32_t lo, uint32_t cnt, uint32_t *bad) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nb) return;
  const uint64_t b0 = s.begin[b], b1 = s.begin[b + 1];
  if (b1 - b0 != cnt || s.key[b0] != lo || s.key[b1 - 1] != lo + cnt - 1) atomicOr(bad, 1u);
}
void launch_dense_check(const SetView &s, uint32_t nb, uint32_t lo, uint32_t cnt, uint32_t *bad, hipStream_t st) {
  if (!nb) return;
  k_dense_check<<<(nb + 255) / 256, 256, 0, st>>>(s, nb, lo, cnt, bad);
}

// RoaringBitmap.runOptimize (RoaringBitmap.java:2764-2775): every container through its runOptimize —
// ArrayContainer / BitmapContainer become a Run when the Run is strictly smaller (ArrayContainer.java:
// 1085-1099, BitmapContainer.java:1227-1246), a RunContainer goes through toEfficientContainer
// (RunContainer.java:2326-2335).  One wave per container: the register bitmap gives c and the maximal
// runs r, the new type follows, the payload is re-emitted.  Every rule picks the smallest encoding, so
// the new payload never exceeds the old one and keeps its offset (the same arena layout); keys,
// cardinalities and offsets are copied by the caller.
__global__ __launch_bounds__(256) void k_run_optimize(SetView s, uint64_t n, uint8_t *__restrict__ type,
                                                      uint16_t *__restrict__ nruns, uint8_t *__restrict__ payload) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4][2048];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + wv; i < n; i += (uint64_t)gridDim.x * 4) {
    const int t = s.type[i];
    const uint32_t card = s.card[i], nr = s.nruns[i];
    uint64_t w[kW];
    load_container(t, s.payload + s.off[i], card, nr, lds[wv], w, lane);
    int c, r;
    metrics(w, lane, true, c, r);
    const int ty = t == kRun ? type_eff(c, r) : type_runopt(c, r);
    emit_container(ty, w, c, r, payload + s.off[i], lds[wv], lane);
    if (lane == 0) {
      type[i] = (uint8_t)ty;
      nruns[i] = (uint16_t)(ty == kRun ? r : 0);
    }
    wave_lds_sync(); // the next container restages the wave's scratch
  }
}
// out[b] = 1 when bitmap b holds a Run container (runOptimize's return value)
__global__ __launch_bounds__(256) void k_any_run(const uint64_t *begin, const uint8_t *type, uint32_t nb, uint8_t *out) {
  const uint64_t b = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= nb) return;
  const int lane = lane_id();
  bool any = false;
  for (uint64_t i = begin[b] + lane; i < begin[b + 1]; i += 64) any |= type[i] == kRun;
  const uint64_t m = __ballot(any);
  if (lane == 0) out[b] = m != 0;
}
void launch_run_optimize(const SetView &s, uint64_t n, uint8_t *type, uint16_t *nruns, uint8_t *payload,
                         uint32_t nb, uint8_t *any_run, hipStream_t st) {
  if (n) k_run_optimize<<<(unsigned)std::min<uint64_t>((n + 3) / 4, 1u << 16), 256, 0, st>>>(s, n, type, nruns, payload);
  if (nb && any_run) k_any_run<<<(nb + 3) / 4, 256, 0, st>>>(s.begin, type, nb, any_run);
}

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_setops() {}
void warm_setops(hipStream_t st) { k_warm_setops<<<1, 64, 0, st>>>(); }

} // namespace rbg
