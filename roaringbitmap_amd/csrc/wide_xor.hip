// wide_xor.hip — FastAggregation.xor (naive_xor, FastAggregation.java:576-582) over Run-heavy keys,
// batch-parallel over the members of a key.
//
// naive_xor is a chain: RoaringBitmap.xor in place (RoaringBitmap.java:3296-3348) folds the key's
// containers in member order, and the container type after every step depends on that step's
// cardinality c_j and maximal run count r_j (RunContainer.xor / ArrayContainer.xor types, SURVEY
// §8a; an empty result removes the key, and the next container is cloned).  The SET is order-free,
// so only the per-step metrics are sequential.  For B = 32 consecutive containers C_0..C_31 of a key
// and the accumulator P (the key's XOR so far, an 8 KiB LDS bitmap) this kernel computes all 32
// (c_j, r_j) at once:
//   * the run boundaries (start, end+1) of the batch — <= 8 runs, <= 16 points per container —
//     are sorted (bitonic, 8 keys per lane); between consecutive points the coverage mask M_i
//     (which containers contain the elementary interval i) is the prefix-xor of the points'
//     container bits;
//   * |P_{j-1} ∩ C_j| = Σ over the intervals i of C_j of |P ∩ i| if popcount(M_i & below_j) is
//     even, else |i| - |P ∩ i| (P ∩ i from a prefix-popcount table of P); c_j = c_{j-1} + |C_j| -
//     2 |P_{j-1} ∩ C_j|;
//   * run boundaries are linear under XOR: T(P ⊕ C) = T(P) △ T(C), so r_j = r_{j-1} + nruns(C_j) -
//     |T(P_{j-1}) ∩ T(C_j)|, and a point x of C_j is in T(P_{j-1}) iff P(x) ≠ P(x-1) xor an odd
//     number of earlier batch containers have the same point x (its rank in its tie group);
//   * each step's type transition is a map on {Array, Bitmap, Run, absent}; the 32 maps are
//     composed by a wave tree reduction, so the key's state after the batch is one lookup;
//   * P is then updated by complementing the intervals with odd coverage.
// Such exact batches run only where a step may cross a type threshold: stretches where no step can
// (see "Fast-forward" below) apply their whole XOR at once and re-measure (c, r) once — on config 4
// about 2 exact batches and 70 stretches per 4096-member key (k_wide_runs_xor 29.6 -> 14.5 ms).
// Keys with another container type, > 8 runs or a full container are routed to the generic kernel
// (route[q] = 1); results are identical either way.
#include <cstdlib>

#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

namespace {

constexpr int kXB = 32;         // containers per batch (2 lanes per container, 4 runs per lane)
constexpr int kXRegion = 1280;  // u32 per wave: pre16 (1024) | then MC (1024) + pos (256)
constexpr uint32_t kNoKey = 0xFFFFFFFFu;

template <int CTRL> __device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
// value of lane (lane ^ M)
template <int M> __device__ __forceinline__ uint32_t xor_lane(uint32_t v, int lane) {
  if constexpr (M == 1) return dpp_mov<0xB1>(v);          // quad_perm [1,0,3,2]
  else if constexpr (M == 2) return dpp_mov<0x4E>(v);     // quad_perm [2,3,0,1]
  else if constexpr (M == 3) return dpp_mov<0x1B>(v);     // quad_perm [3,2,1,0]
  else if constexpr (M == 7) return dpp_mov<0x141>(v);    // row_half_mirror
  else if constexpr (M == 15) return dpp_mov<0x140>(v);   // row_mirror
  else if constexpr (M == 8) return dpp_mov<0x128>(v);    // row_ror:8 (swap the halves of a row of 16)
  else if constexpr (M < 32) {                            // 4, 16, 31: swizzle (xor mode)
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (M << 10));
  } else {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((lane ^ M) << 2, (int)v);
  }
}

// one cross-lane compare-exchange step of the bitonic merge: FLIP pairs element e with element 7-e
// of lane (lane ^ M) (M = 2^j - 1), otherwise element e with element e of lane (lane ^ M).
// median of (a, b, c): with c = 0 it is min(a, b), with c = ~0 it is max(a, b) — one VALU op for
// the lower lane's min / the upper lane's max instead of min + max + select
__device__ __forceinline__ uint32_t med3_u32(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
template <int M, bool FLIP> __device__ __forceinline__ void cross_step(uint32_t (&k)[8], int lane) {
  const bool lower = FLIP ? (lane & ((M + 1) >> 1)) == 0 : (lane & M) == 0;
  const uint32_t sel = lower ? 0u : 0xFFFFFFFFu;
  uint32_t t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = xor_lane<M>(k[FLIP ? 7 - e : e], lane);
#pragma unroll
  for (int e = 0; e < 8; ++e) k[e] = med3_u32(k[e], t[e], sel);
}
__device__ __forceinline__ void inlane_merge(uint32_t (&k)[8]) {
#pragma unroll
  for (int d = 4; d > 0; d >>= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (!(e & d)) {
        const uint32_t a = k[e], b = k[e | d];
        k[e] = min(a, b);
        k[e | d] = max(a, b);
      }
}
// 512 keys, lane l holds positions 8l..8l+7, each lane's 8 already ascending -> globally ascending
__device__ __forceinline__ void sort512(uint32_t (&k)[8], int lane) {
  cross_step<1, true>(k, lane);
  inlane_merge(k);
  cross_step<3, true>(k, lane);
  cross_step<1, false>(k, lane);
  inlane_merge(k);
  cross_step<7, true>(k, lane);
  cross_step<2, false>(k, lane);
  cross_step<1, false>(k, lane);
  inlane_merge(k);
  cross_step<15, true>(k, lane);
  cross_step<4, false>(k, lane);
  cross_step<2, false>(k, lane);
  cross_step<1, false>(k, lane);
  inlane_merge(k);
  cross_step<31, true>(k, lane);
  cross_step<8, false>(k, lane);
  cross_step<4, false>(k, lane);
  cross_step<2, false>(k, lane);
  cross_step<1, false>(k, lane);
  inlane_merge(k);
  cross_step<63, true>(k, lane);
  cross_step<16, false>(k, lane);
  cross_step<8, false>(k, lane);
  cross_step<4, false>(k, lane);
  cross_step<2, false>(k, lane);
  cross_step<1, false>(k, lane);
  inlane_merge(k);
}

__device__ __forceinline__ uint32_t wave_scan_max(uint32_t v) { // inclusive
  v = max(v, dpp<0x111>(v));
  v = max(v, dpp<0x112>(v));
  v = max(v, dpp<0x114>(v));
  v = max(v, dpp<0x118>(v));
  v = max(v, dpp<0x142, 0xa, false>(v));
  v = max(v, dpp<0x143, 0xc, false>(v));
  return v;
}

// type-transition maps on the state {0 Array, 1 Bitmap, 2 Run, 3 absent}: 2 bits per source state
constexpr uint32_t kIdentityMap = 0xE4u;
__device__ __forceinline__ uint32_t compose(uint32_t later, uint32_t earlier) {
  uint32_t out = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const uint32_t mid = (earlier >> (2 * s)) & 3u;
    out |= ((later >> (2 * mid)) & 3u) << (2 * s);
  }
  return out;
}

} // namespace

// Key-major member records.  The SoA metadata is member-major (container m * 65536 + k for dense
// members), so a wave walking one key's members reads type / card / nruns / off as four lines per
// member, ~5 L2 requests per container with the payload: the kernel was L2-request-bound (PMC:
// TCC_BUSY 91 % of the kernel, 1.36G TCC requests per launch, 77 % hits) with its VALU at ~60 %.
// So the kernel reads each (key, member) as one 4-B record (pack_xrec, common.hpp: the payload's 16-B unit and
// the run count; round 6 — 8-B records with the card and type before, whose build read 15 B and wrote 8 B per
// container) in key order.  For a dense set read in member order the records are the set's cached krec
// (built once per set, rbgpu_set); any other member list gets them per call: 64-key x 64-member tiles of the
// set's packed records (mrec) transposed through LDS, so both the reads (along keys) and the writes (along
// members) are coalesced.
__global__ __launch_bounds__(256) void k_records_transpose(const uint64_t *__restrict__ mrec,
                                                           const uint64_t *__restrict__ mbase, uint64_t bias,
                                                           uint32_t M, uint32_t key_lo, uint32_t key_hi,
                                                           uint32_t *__restrict__ rec) {
  __shared__ uint32_t tile[64][65]; // [member][key], padded against bank conflicts on the column reads
  const uint32_t k0 = key_lo + blockIdx.x * 64, m0 = blockIdx.y * 64;
  const uint32_t t = threadIdx.x, kx = t & 63, ry = t >> 6;
  uint64_t rb[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) rb[j] = mbase[min(m0 + ry + 4 * j, M - 1)] - bias;
  const uint32_t k = min(k0 + kx, key_hi - 1);
  uint64_t v[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = mrec[rb[j] + k]; // all 16 loads in flight at once
#pragma unroll
  for (int j = 0; j < 16; ++j) tile[ry + 4 * j][kx] = xrec_of(v[j]);
  __syncthreads();
  for (uint32_t r = ry; r < 64; r += 4) { // writes along members
    const uint32_t kw = k0 + r, i = m0 + kx;
    if (i < M && kw < key_hi) rec[(uint64_t)(kw - key_lo) * M + i] = tile[kx][r];
  }
}
void launch_records_transpose(const uint64_t *mrec, const uint64_t *mbase, uint64_t bias, uint32_t M, uint32_t key_lo,
                              uint32_t key_hi, uint32_t *rec, hipStream_t st) {
  if (!M || key_hi <= key_lo) return;
  k_records_transpose<<<dim3((key_hi - key_lo + 63) / 64, (M + 63) / 64), 256, 0, st>>>(mrec, mbase, bias, M, key_lo,
                                                                                      key_hi, rec);
}

// The same key-major records straight from the set's SoA (no member-major mrec first): a dense set's first
// naive_xor reads the run count and the payload offset once (10 B per container; a container with a run count
// is a Run — rbgpu_set_from_soa stores 0 for the others) and writes the 4-B records transposed.  Same 64 x 64
// tiles: the loads run along keys (a member's containers are consecutive), the stores along members.
// (Measured: 64 x 64 tiles dealt key-tile-major, 128 x 32 and 256 x 16 tiles, and 8 x 8 / 16 x 16 groups of
// tiles dealt together all build config 4's records in 2.0-2.3 ms, profiles/r05/krec.)
__global__ __launch_bounds__(256) void k_records_direct(SetView s, const uint64_t *__restrict__ mbase, uint64_t bias,
                                                        uint32_t M, uint32_t key_lo, uint32_t key_hi,
                                                        uint32_t *__restrict__ rec) {
  __shared__ uint32_t tile[64][65];
  const uint32_t k0 = key_lo + blockIdx.x * 64, m0 = blockIdx.y * 64;
  const uint32_t t = threadIdx.x, kx = t & 63, ry = t >> 6;
  uint64_t rb[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) rb[j] = mbase[min(m0 + ry + 4 * j, M - 1)] - bias;
  const uint32_t k = min(k0 + kx, key_hi - 1);
  uint32_t nr[16];
  uint64_t of[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) { // all 32 loads in flight at once
    const uint64_t i = rb[j] + k;
    nr[j] = s.nruns[i];
    of[j] = s.off[i];
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) tile[ry + 4 * j][kx] = pack_xrec(nr[j] != 0, nr[j], of[j]);
  __syncthreads();
  for (uint32_t r = ry; r < 64; r += 4) { // writes along members
    const uint32_t kw = k0 + r, i = m0 + kx;
    if (i < M && kw < key_hi) rec[(uint64_t)(kw - key_lo) * M + i] = tile[kx][r];
  }
}
// The same with 128-key tiles and two containers per lane (4-B run-count pairs, 16-B offset pairs, 8-B record
// pairs stored): every load row is whole 128-B lines.  Needs even container bases, an even key count and an
// even member count, as a dense set of whole 65536-key members has; other sets take the 64 x 64 tiles above.
__global__ __launch_bounds__(256) void k_records_direct2(SetView s, const uint64_t *__restrict__ mbase, uint64_t bias,
                                                         uint32_t M, uint32_t key_lo, uint32_t key_hi,
                                                         uint32_t *__restrict__ rec) {
  __shared__ uint32_t tile[64][129]; // [member][key]
  const uint32_t k0 = key_lo + blockIdx.x * 128, m0 = blockIdx.y * 64;
  const uint32_t t = threadIdx.x, kx = t & 63, ry = t >> 6;
  uint64_t rb[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) rb[j] = mbase[min(m0 + ry + 4 * j, M - 1)] - bias;
  const uint32_t k = min(k0 + 2 * kx, key_hi - 2);
  uint32_t nr[16];
  uint4 of[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) { // all 32 loads in flight at once
    const uint64_t i = rb[j] + k;
    nr[j] = *reinterpret_cast<const uint32_t *>(s.nruns + i);
    of[j] = *reinterpret_cast<const uint4 *>(s.off + i);
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t n0 = nr[j] & 0xFFFFu, n1 = nr[j] >> 16;
    tile[ry + 4 * j][2 * kx] = pack_xrec(n0 != 0, n0, of[j].x | ((uint64_t)of[j].y << 32));
    tile[ry + 4 * j][2 * kx + 1] = pack_xrec(n1 != 0, n1, of[j].z | ((uint64_t)of[j].w << 32));
  }
  __syncthreads();
  const uint32_t lx = t & 31, rr = t >> 5; // a key row is 32 lanes x 2 members: 8 rows per pass
  const uint32_t i = m0 + 2 * lx;
  for (uint32_t r = rr; r < 128; r += 8) {
    const uint32_t kw = k0 + r;
    if (i < M && kw < key_hi)
      *reinterpret_cast<uint2 *>(rec + (uint64_t)(kw - key_lo) * M + i) = make_uint2(tile[2 * lx][r], tile[2 * lx + 1][r]);
  }
}
// The same with 256-key x 32-member tiles, four containers per lane (8-B run-count quads, two 16-B offset pairs):
// a member's load row is 2 KiB of offsets (a whole HBM page) and 512 B of run counts, and a key's store row one
// 128-B line.  Needs container indices and the key count in fours (quads, build_krec_range).
#ifndef RBG_REC_QUAD
#define RBG_REC_QUAD 0 // study builds: 1 builds dense records by the 256 x 32 tiles
#endif
__global__ __launch_bounds__(256) void k_records_direct4(SetView s, const uint64_t *__restrict__ mbase, uint64_t bias,
                                                         uint32_t M, uint32_t key_lo, uint32_t key_hi,
                                                         uint32_t *__restrict__ rec) {
  __shared__ uint32_t tile[32][257]; // [member][key]
  const uint32_t k0 = key_lo + blockIdx.x * 256, m0 = blockIdx.y * 32;
  const uint32_t t = threadIdx.x, kx = t & 63, ry = t >> 6;
  uint64_t rb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) rb[j] = mbase[min(m0 + ry + 4 * j, M - 1)] - bias;
  const uint32_t k = min(k0 + 4 * kx, key_hi - 4);
  uint2 nr[8];
  uint4 o0[8], o1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { // all 24 loads in flight at once
    const uint64_t i = rb[j] + k;
    nr[j] = *reinterpret_cast<const uint2 *>(s.nruns + i);
    o0[j] = *reinterpret_cast<const uint4 *>(s.off + i);
    o1[j] = *reinterpret_cast<const uint4 *>(s.off + i + 2);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t n[4] = {nr[j].x & 0xFFFFu, nr[j].x >> 16, nr[j].y & 0xFFFFu, nr[j].y >> 16};
    const uint64_t o[4] = {o0[j].x | ((uint64_t)o0[j].y << 32), o0[j].z | ((uint64_t)o0[j].w << 32),
                           o1[j].x | ((uint64_t)o1[j].y << 32), o1[j].z | ((uint64_t)o1[j].w << 32)};
#pragma unroll
    for (int u = 0; u < 4; ++u) tile[ry + 4 * j][4 * kx + u] = pack_xrec(n[u] != 0, n[u], o[u]);
  }
  __syncthreads();
  const uint32_t lx = t & 31, rr = t >> 5; // a key row is 32 members x 4 B: 8 rows per pass
  const uint32_t i = m0 + lx;
  for (uint32_t r = rr; r < 256; r += 8) {
    const uint32_t kw = k0 + r;
    if (i < M && kw < key_hi) rec[(uint64_t)(kw - key_lo) * M + i] = tile[lx][r];
  }
}
void launch_records_direct(const SetView &s, const uint64_t *mbase, uint64_t bias, uint32_t M, uint32_t key_lo,
                           uint32_t key_hi, uint32_t *rec, hipStream_t st, bool pairs, bool quads) {
  if (!M || key_hi <= key_lo) return;
  if (RBG_REC_QUAD && quads && !((key_hi - key_lo) & 3))
    k_records_direct4<<<dim3((key_hi - key_lo + 255) / 256, (M + 31) / 32), 256, 0, st>>>(s, mbase, bias, M, key_lo,
                                                                                         key_hi, rec);
  else if (pairs && !(M & 1) && !((key_hi - key_lo) & 1))
    k_records_direct2<<<dim3((key_hi - key_lo + 127) / 128, (M + 63) / 64), 256, 0, st>>>(s, mbase, bias, M, key_lo,
                                                                                          key_hi, rec);
  else
    k_records_direct<<<dim3((key_hi - key_lo + 63) / 64, (M + 63) / 64), 256, 0, st>>>(s, mbase, bias, M, key_lo,
                                                                                      key_hi, rec);
}

// Members grouped by the counting sort: a gather of the packed records through the container ids (the
// grouped count, seg[65536], can be less than the members' containers when the call is a key-range shard).
__global__ __launch_bounds__(256) void k_records_gather(const uint64_t *__restrict__ mrec,
                                                        const uint32_t *__restrict__ cid,
                                                        const uint64_t *__restrict__ seg, uint32_t *__restrict__ rec) {
  const uint64_t n = seg[65536];
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
    rec[i] = xrec_of(mrec[cid[i]]);
}

namespace {

struct XBatch {
  uint32_t card, nr, typ;
  uint4 r; // runs 4h .. 4h+3 of the lane's container
};
// Lane pair (2j, 2j + 1) holds container j of the batch, lane h of the pair its runs 4h .. 4h+3; the card is
// summed from both halves' run lengths (the 4-B records carry none).  Every lane calls it (DPP).
__device__ __forceinline__ XBatch load_xbatch(const SetView &s, const uint32_t *rec, uint64_t i, uint64_t hi, int h,
                                              int lane) {
  XBatch b;
  b.nr = 0;
  b.typ = kRun;
  b.r = make_uint4(0, 0, 0, 0);
  if (i < hi) {
    const uint32_t r = rec[i];
    b.typ = xrec_ok(r) ? (uint32_t)kRun : (uint32_t)kArray; // kArray: any container the batch cannot take
    b.nr = xrec_nruns(r);
    if (xrec_ok(r) && b.nr > (uint32_t)(4 * h)) b.r = reinterpret_cast<const uint4 *>(s.payload + xrec_off(r))[h];
  }
  const uint32_t w[4] = {b.r.x, b.r.y, b.r.z, b.r.w};
  uint32_t c = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) c += (uint32_t)(4 * h + u) < b.nr ? (w[u] >> 16) + 1u : 0u;
  b.card = c + xor_lane<1>(c, lane);
  return b;
}

__device__ __forceinline__ uint32_t dmask(uint32_t w, uint32_t lo, uint32_t hi) {
  const uint32_t a = max(lo, w * 32), b = min(hi, w * 32 + 31);
  if (a > b) return 0u;
  return (0xFFFFFFFFu >> (31 - (b - a))) << (a - w * 32);
}

} // namespace

// The key's state between steps: container type (0 Array, 1 Bitmap, 2 Run, 3 absent), cardinality and
// maximal run count of the accumulator, and this lane's share of the algorithmic input bytes.
struct XState {
  int state, c, r;
  uint32_t inb;
  int rvalid; // r is only tracked where a rule can read it (see the fast-forward): Run states, exact batches
};

// One exact batch of <= 32 containers starting at `base` (the accumulator P is the LDS bitmap `acc`):
// every step's (c_j, r_j) from the sorted run boundaries, the type maps composed, P updated.  Returns
// false when a container of the batch does not qualify (the key goes to the generic kernel).
__device__ __forceinline__ bool exact_batch(const SetView &s, const uint32_t *rec, uint64_t base, uint64_t hi,
                                            uint32_t *acc, uint32_t *R, int lane, XState &X) {
  uint16_t *R16 = reinterpret_cast<uint16_t *>(R);
  uint16_t *pos = R16 + 2048;                       // [512] sorted position | tie/boundary bit 15
  uint2 *MC = reinterpret_cast<uint2 *>(R);         // [512] (coverage mask, c0 | c1 << 16)
  const int cj = lane >> 1, h = lane & 1;
  const uint32_t below = (1u << cj) - 1u;
  const XBatch cur = load_xbatch(s, rec, base + cj, hi, h, lane);
  const bool valid = base + (uint64_t)cj < hi;
  const bool bad = valid && (cur.typ != kRun || cur.nr > 8u || cur.card >= (uint32_t)kSpan);
  if (__ballot(bad)) return false;
  if (valid && h == 0) X.inb += 4u * cur.nr + 2u + 16u;

  // ---- prefix popcounts of P: row k = dwords [256k, 256k+256), lane l holds 4l..4l+3 of it;
  //      pre16[d] = popcount of row dwords before d (<= 8192), rb (lane k) = popcount before row k
  uint32_t rb = 0, run_tot = 0;
  {
    const uint4 *a4 = reinterpret_cast<const uint4 *>(acc);
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) {
      const uint4 v0 = a4[(2 * k2) * 64 + lane], v1 = a4[(2 * k2 + 1) * 64 + lane];
      const uint32_t p00 = __popc(v0.x), p01 = __popc(v0.y), p02 = __popc(v0.z), p03 = __popc(v0.w);
      const uint32_t p10 = __popc(v1.x), p11 = __popc(v1.y), p12 = __popc(v1.z), p13 = __popc(v1.w);
      const uint32_t s0 = p00 + p01 + p02 + p03, s1 = p10 + p11 + p12 + p13;
      const uint32_t inc = wave_scan_u32(s0 | (s1 << 16), lane);
      const uint32_t ex = inc - (s0 | (s1 << 16));
      const uint32_t e0 = ex & 0xFFFF, e1 = ex >> 16;
      uint2 w0, w1;
      w0.x = e0 | ((e0 + p00) << 16);
      w0.y = (e0 + p00 + p01) | ((e0 + p00 + p01 + p02) << 16);
      w1.x = e1 | ((e1 + p10) << 16);
      w1.y = (e1 + p10 + p11) | ((e1 + p10 + p11 + p12) << 16);
      reinterpret_cast<uint2 *>(R)[(2 * k2) * 64 + lane] = w0;
      reinterpret_cast<uint2 *>(R)[(2 * k2 + 1) * 64 + lane] = w1;
      const uint32_t tot = readlane(inc, 63);
      if (lane == 2 * k2) rb = run_tot;
      run_tot += tot & 0xFFFF;
      if (lane == 2 * k2 + 1) rb = run_tot;
      run_tot += tot >> 16;
    }
  }

  // ---- the batch's run boundaries as sort keys (x << 9 | slot), slot = 8 lane + 2u + (0 start | 1 end+1)
  uint32_t K[8];
  {
    const uint32_t rw[4] = {cur.r.x, cur.r.y, cur.r.z, cur.r.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = valid && (uint32_t)(4 * h + u) < cur.nr;
      const uint32_t st = rw[u] & 0xFFFF, e1 = st + (rw[u] >> 16) + 1;
      K[2 * u] = ok ? (st << 9) | (uint32_t)(8 * lane + 2 * u) : kNoKey;
      K[2 * u + 1] = ok ? (e1 << 9) | (uint32_t)(8 * lane + 2 * u + 1) : kNoKey;
    }
  }
  sort512(K, lane);

  // ---- per sorted position i = 8 lane + e: coverage mask, tie-group rank, P(x), P(x-1), F(x)
  uint32_t P[8], Mv[8], F[8], B[8], Q[8];
  {
    uint32_t m = 0, gl = 0, prevp = dpp<0x138>(K[7] >> 9); // wave_shr:1
    uint32_t hmask = 0;                                     // bit e: position 8 lane + e heads a tie group
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool vld = K[e] != kNoKey;
      P[e] = K[e] >> 9;
      if (vld) m ^= 1u << ((K[e] >> 4) & 31);
      Mv[e] = m;
      const uint32_t pp = e ? P[e - 1] : prevp;
      const bool head = (lane == 0 && e == 0) || P[e] != pp;
      if (head) {
        gl = (uint32_t)(8 * lane + e);
        hmask |= 1u << e;
      }
      B[e] = gl; // last head at or before i, within this lane (0 if none yet)
    }
    const uint32_t mx = wave_xscan_xor(m, lane) ^ m;
    const uint32_t gprev = dpp<0x138>(wave_scan_max(gl));
    // first head after this lane: suffix max of (512 - first head) over the lanes above, via a
    // lane reversal (ds_bpermute) and the forward max-scan
    const uint32_t fh = hmask ? (uint32_t)(8 * lane) + __builtin_ctz(hmask) : 512u;
    const uint32_t rv = (uint32_t)__builtin_amdgcn_ds_bpermute((63 - lane) << 2, (int)(512u - fh));
    const uint32_t sc = (uint32_t)__builtin_amdgcn_ds_bpermute((63 - lane) << 2, (int)wave_scan_max(rv));
    uint32_t nh = 512u - dpp<0x130>(sc); // wave_shl:1 -> lanes above only
#pragma unroll
    for (int e = 7; e >= 0; --e) {
      Mv[e] ^= mx;
      const uint32_t g = max(B[e], gprev);
      B[e] = ((uint32_t)(8 * lane + e) - g) & 1u; // odd number of earlier batch containers share x
      // interval range ends for the A loop: a start point's first positive-length interval is
      // the last of its tie group; an end point's range stops at the first of its tie group
      const bool is_end = K[e] & 1u;
      Q[e] = is_end ? g : nh - 1;
      if (hmask & (1u << e)) nh = (uint32_t)(8 * lane + e);
    }
    uint32_t RB[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) // outside the divergent branch: bpermute sources must be active
      RB[e] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((min(P[e], 65535u) >> 13) << 2), (int)rb);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t x = P[e];
      if (K[e] != kNoKey) {
        const uint32_t xq = min(x, 65535u);
        const uint32_t w = acc[xq >> 5];
        const uint32_t wm1 = acc[(x ? x - 1 : 0) >> 5];
        const uint32_t bx = (w >> (xq & 31)) & 1u;
        const uint32_t bm1 = x ? (wm1 >> ((x - 1) & 31)) & 1u : 0u;
        uint32_t f = RB[e] + R16[xq >> 5] + __popc(w & ((1u << (xq & 31)) - 1u));
        if (x == 65536u) f += bx;
        F[e] = f;
        B[e] ^= (x == 65536u ? 0u : bx) ^ bm1;
      } else {
        F[e] = 0;
      }
    }
  }
  wave_lds_sync(); // pre16 is dead: the region now holds MC and pos
  {
    const uint32_t pn7 = dpp<0x130>(P[0]), fn7 = dpp<0x130>(F[0]); // wave_shl:1
    uint32_t Cv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t pn = e < 7 ? P[e + 1] : pn7, fn = e < 7 ? F[e + 1] : fn7;
      const uint32_t c0 = fn - F[e], c1 = (pn - P[e]) - c0;
      Cv[e] = (c0 & 0xFFFF) | (c1 << 16);
    }
    uint4 *mc4 = reinterpret_cast<uint4 *>(MC + 8 * lane);
#pragma unroll
    for (int e = 0; e < 8; e += 2) mc4[e >> 1] = make_uint4(Mv[e], Cv[e], Mv[e + 1], Cv[e + 1]);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (K[e] != kNoKey) pos[K[e] & 511] = (uint16_t)(Q[e] | (B[e] << 15));
    // ---- P ^= the batch: complement every elementary interval with odd coverage
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t pn = e < 7 ? P[e + 1] : pn7;
      if (K[e] != kNoKey && (__popc(Mv[e]) & 1) && pn > P[e]) { // (tie groups: zero-length intervals)
        const uint32_t a = P[e], b = pn - 1;
        for (uint32_t w = a >> 5; w <= (b >> 5); ++w) atomicXor(&acc[w], dmask(w, a, b));
      }
    }
  }
  wave_lds_sync();

  // ---- |P_{j-1} ∩ C_j| and |T(P_{j-1}) ∩ T(C_j)| for the lane's 4 runs
  uint32_t A = 0, match = 0;
  {
    const uint4 pv = reinterpret_cast<const uint4 *>(pos)[lane];
    const uint32_t pw[4] = {pv.x, pv.y, pv.z, pv.w};
    uint32_t qs[4], qe[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = valid && (uint32_t)(4 * h + u) < cur.nr;
      const uint32_t a = pw[u] & 0xFFFF, b = pw[u] >> 16;
      qs[u] = ok ? (a & 0x7FFF) : 0;
      qe[u] = ok ? (b & 0x7FFF) : 0;
      if (ok) match += (a >> 15) + (b >> 15);
    }
    // one flattened loop over the lane's (up to 4) interval ranges, two entries per trip
    uint32_t cs = qs[0], ce = qe[0], s1 = qs[1], e1 = qe[1], s2 = qs[2], e2 = qe[2], s3 = qs[3], e3 = qe[3];
    while (true) {
      if (cs >= ce) {
        if (s1 >= e1 && s2 >= e2 && s3 >= e3) break;
        cs = s1;
        ce = e1;
        s1 = s2;
        e1 = e2;
        s2 = s3;
        e2 = e3;
        s3 = e3 = 0;
        continue;
      }
      const bool two = cs + 1 < ce;
      const uint2 m0 = MC[cs], m1 = MC[two ? cs + 1 : cs];
      A += (__popc(m0.x & below) & 1) ? (m0.y >> 16) : (m0.y & 0xFFFF);
      if (two) A += (__popc(m1.x & below) & 1) ? (m1.y >> 16) : (m1.y & 0xFFFF);
      cs += two ? 2 : 1;
    }
  }
  wave_lds_sync(); // the next batch rewrites the region
  A += xor_lane<1>(A, lane);
  match += xor_lane<1>(match, lane);
  const bool rep = valid && h == 0;
  const int dc = rep ? (int)cur.card - 2 * (int)A : 0;
  const int dr = rep ? (int)cur.nr - (int)match : 0;
  const int ic = (int)wave_scan_u32((uint32_t)dc, lane), ir = (int)wave_scan_u32((uint32_t)dr, lane);
  // ---- this step's type map (RunContainer.xor / ArrayContainer.xor / BitmapContainer.xor)
  uint32_t f = kIdentityMap;
  if (rep) {
    const int cjv = X.c + ic, rjv = X.r + ir, cprev = cjv - dc;
    const uint32_t te = cjv == 0 ? 3u : (uint32_t)type_eff(cjv, rjv);
    const uint32_t ta = cjv == 0 ? 3u : (uint32_t)type_ab(cjv);
    const uint32_t fa = cprev < kRunArrayThreshold ? te : ta;
    f = fa | (ta << 2) | (te << 4) | (2u << 6); // absent -> clone (Run)
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane + d) & 63) << 2, (int)f);
    f = compose(lane + d < 64 ? y : kIdentityMap, f);
  }
  const uint32_t G = readlane(f, 0);
  X.state = (int)((G >> (2 * X.state)) & 3u);
  X.c += (int)readlane((uint32_t)ic, 63);
  X.r += (int)readlane((uint32_t)ir, 63);
  return true;
}

// Fast-forward.  With Run members the step rules only look at the accumulator's (c, r) through a few
// thresholds: a Bitmap accumulator becomes AB(c_j); an Array one with c_{j-1} >= 32 becomes AB(c_j) too
// (only |A| < 32 switches ArrayContainer.xor(Run) to EFF); a Run one becomes EFF(c_j, r_j); an empty
// result removes the key (the next member is cloned, a Run).  So two kinds of stretches need no
// per-step metrics:
//   AB stretch   the accumulator is a Bitmap, an Array with c >= 32, or a Run whose first step cannot
//                stay a Run (r - nruns > 2047, or 2 (r - nruns) > c + |C|), and every step keeps
//                c_j >= 32: every step is AB(c_j), the last one decides the type;
//   Run stretch  the accumulator is a Run and every step keeps 2 + 4 r_j <= min(8192, 2 c_j + 2): every
//                step stays a Run.
// The bounds: c_j = |P ⊕ X_j| with X_j the stretch's XOR so far, so |c_j - c| <= |X_j|, and
// |X_j| <= Σ over the stretch's member pairs (2m, 2m+1) of |C_2m ⊕ C_2m+1| (+ |C_j| for an unpaired
// last or first member) — pairs of members sharing a core cancel most of it; r_j <= r + Σ nruns.  A
// stretch's XOR is applied at once (XOR commutes) through a toggle image of its run boundaries, and
// (c, r) are re-measured on the result.  Bit-exact by construction; the exact batches run only where a
// threshold may be crossed.
struct XWin { // one container per lane: the fast-forward window
  uint32_t typ, card, nr;
  uint4 r0, r1;
  uint32_t pairx; // even lanes: |C_lane ⊕ C_lane+1| (set by pair_xor)
  uint32_t best;  // the lane's longest run, start | (len - 1) << 16 (set by pair_xor)
};
// A window's loads form a chain (record -> run list), so they are software-pipelined over three windows:
// the records of window w+2 and the runs of w+1 are in flight while window w is processed, and every
// load issued at an advance only uses values loaded a window earlier.  The runs of w+1 go straight to
// LDS (global_load_lds, 2 KiB in the exact batches' region, `kNextRuns`): as VGPR loads, the window
// rotation (W = N) made the compiler load into temporaries and copy them right away, which waited for
// the loads just issued — every window paid the full memory latency (r03 ISA).
constexpr int kNextRuns = 768; // u32 offset in the wave's region of the next window's runs (r0 x 64 | r1 x 64)
#ifndef RBG_XOR_MCOPIES
#define RBG_XOR_MCOPIES 8 // study builds (A/B of the copy count)
#endif
constexpr int kMCopies = RBG_XOR_MCOPIES, kMStride = 33; // touched-word mask copies (lane % copies), strided over distinct banks
constexpr int kPcT = 272;                  // u32 offset of pcT (16-B aligned, after the mask copies)
static_assert(kMCopies * kMStride <= kPcT && kPcT + 256 <= kNextRuns && kNextRuns + 512 <= kXRegion,
              "mask copies, pcT and the next runs inside the region");
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
constexpr int kWaitVm0 = 0x0F70;   // s_waitcnt vmcnt(0)
constexpr int kWaitLgkm0 = 0xC07F; // s_waitcnt lgkmcnt(0)
struct XMeta {
  uint32_t typ, nr;
  uint64_t off;
};
// The loads are unconditional (addresses clamped to valid memory, results selected afterwards): a load
// under a branch makes the waitcnt pass assume the worst at the merge and wait for every load in flight,
// which would expose the whole chain's latency at every window.  A record the fast path cannot take reads as
// kArray (the window routes the key).
__device__ __forceinline__ XMeta xmeta_of(uint32_t r, bool valid) {
  XMeta m;
  m.typ = !valid || xrec_ok(r) ? (uint32_t)kRun : (uint32_t)kArray;
  m.nr = valid ? xrec_nruns(r) : 0u;
  m.off = valid ? xrec_off(r) : 0ull;
  return m;
}
// a container's card from its (<= 8) runs: the runs u < nr of r0 | r1
__device__ __forceinline__ uint32_t runs_card(const uint4 &r0, const uint4 &r1, uint32_t nr) {
  const uint32_t w[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
  uint32_t c = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) c += (uint32_t)u < nr ? (w[u] >> 16) + 1u : 0u;
  return c;
}
__device__ __forceinline__ XWin xwin_from(const SetView &s, const XMeta &m) {
  XWin w;
  w.typ = m.typ;
  w.nr = m.nr;
  const bool runs = m.typ == kRun && m.nr && m.nr <= 8u;
  // a non-Run (or invalid) member reads the arena's first 16 B instead; runs 4..7 exist only if nr > 4
  const uint4 *p = reinterpret_cast<const uint4 *>(s.payload + (runs ? m.off : 0ull));
  // raw loaded values, no select on them: only runs u < nr are ever read, and a lane whose container is
  // not a Run of <= 8 runs routes the key first.  (The card waits for them: only the first window loads here.)
  w.r0 = p[0];
  w.r1 = p[runs && m.nr > 4u ? 1 : 0];
  w.card = runs_card(w.r0, w.r1, w.nr);
  w.pairx = 0;
  w.best = 0;
  return w;
}
// Round 6: the DMA is issued from inline asm.  Through the builtin the compiler knows that a vmcnt event
// writes LDS and, lacking alias scopes, made the window's FIRST LDS access (the first mark, the M clear, the
// first toggle) wait vmcnt(0): the runs of w+1 and the record of w+2, issued at the advance a few dozen
// instructions earlier, were waited for in every window — the prefetch hid nothing (r06 ISA).  Hidden from
// the waitcnt pass, the DMA is waited for only where its slot is read (take_next) or rewritten (exact
// batches), each by an explicit vmcnt(0); the compiler's own vmcnt waits stay correct (loads return in
// order, so an extra untracked load only makes them wait longer).
#ifndef RBG_XOR_DMA_ASM
#define RBG_XOR_DMA_ASM 1
#endif
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// the next window's runs, LDS-DMA into nb (lane-linear: r0 of lane l at nb[4l], r1 at nb[256 + 4l])
__device__ __forceinline__ void stage_next_runs(const SetView &s, const XMeta &m, uint32_t *nb) {
  const bool runs = m.typ == kRun && m.nr && m.nr <= 8u;
  const uint8_t *p = s.payload + (runs ? m.off : 0ull);
  const uint8_t *p1 = p + (runs && m.nr > 4u ? 16 : 0);
#if RBG_XOR_DMA_ASM
  const uint32_t l0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t *)nb);
  // m0 is reserved: the clobber tells the compiler, which sets m0 nowhere else in this kernel (ISA-checked)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
  asm volatile("s_mov_b32 m0, %2\n\t"
               "s_nop 0\n\t"
               "global_load_lds_dwordx4 %0, off\n\t"
               "s_add_u32 m0, m0, 0x400\n\t"
               "s_nop 0\n\t"
               "global_load_lds_dwordx4 %1, off"
               :
               : "v"(p), "v"(p1), "s"(l0)
               : "memory", "m0");
#pragma clang diagnostic pop
#else
  __builtin_amdgcn_global_load_lds((gbl_void_t *)p, (lds_void_t *)nb, 16, 0, 0);
  __builtin_amdgcn_global_load_lds((gbl_void_t *)p1, (lds_void_t *)(nb + 256), 16, 0, 0);
#endif
}
// the window staged by stage_next_runs (every load of the previous window waited for first)
__device__ __forceinline__ XWin take_next(const XMeta &m, const uint32_t *nb, int lane) {
  wait_vm0();
  XWin w;
  w.typ = m.typ;
  w.nr = m.nr;
  w.r0 = reinterpret_cast<const uint4 *>(nb)[lane];
  w.r1 = reinterpret_cast<const uint4 *>(nb)[64 + lane];
  w.card = runs_card(w.r0, w.r1, w.nr);
  w.pairx = 0;
  w.best = 0;
  __builtin_amdgcn_s_waitcnt(kWaitLgkm0); // read before the next DMA overwrites the slot
  return w;
}
// An upper bound of |C_l ⊕ C_l+1| = |C_l| + |C_l+1| - 2 |C_l ∩ C_l+1| for every lane l (meaningful on
// even lanes whose neighbour is in the window): |C_l ∩ C_l+1| is at least the overlap of the two
// containers' longest runs (members that share a core run overlap there); the neighbour's longest run
// comes over by DPP.
// the lane's longest run as its run word, start | (len - 1) << 16 (the last of equal lengths; 0 without runs)
__device__ __forceinline__ uint32_t longest_run(const XWin &w) {
  const uint32_t a[8] = {w.r0.x, w.r0.y, w.r0.z, w.r0.w, w.r1.x, w.r1.y, w.r1.z, w.r1.w};
  uint32_t best = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if ((uint32_t)u < w.nr && (a[u] >> 16) >= (best >> 16)) best = a[u];
  return best;
}
__device__ __forceinline__ void pair_xor(XWin &w) {
  const uint32_t best = longest_run(w);
  w.best = best;
  const uint32_t nbest = dpp<0x130>(best), cb = dpp<0x130>(w.card); // wave_shl:1 — lane l reads lane l+1
  const int sa = (int)(best & 0xFFFF), ea = sa + (int)(best >> 16);
  const int sb = (int)(nbest & 0xFFFF), eb = sb + (int)(nbest >> 16);
  const int inter = w.nr ? max(0, min(ea, eb) - max(sa, sb) + 1) : 0;
  w.pairx = w.card + cb - 2u * (uint32_t)inter;
}
// Core-run de-duplication (round 6; PMC profiles/r06/xor): the members of a key usually share a run (config
// 4: every member holds the key's 1024-value core), so all 64 lanes of a window toggled the same two bits and
// marked the same U' words — same-address LDS atomics, serialised 64 (toggles) and 8 (marks, one copy per
// lane & 7) deep: 120 bank-conflict cycles per window, ~70 % of the toggle pass's conflicts (a duplicated
// toggle pass cost +1.18 ms, +503M conflict cycles).  A wave-uniform candidate run `core` (a lane's longest)
// is handled once: its toggles by parity (k lanes toggling the same bit is the bit toggled k mod 2 times —
// one ballot, one atomic by lane 0), its marks once per union stretch (marks are idempotent and U' is only
// cleared when a stretch starts).  Any run that is not exactly the candidate takes the atomics as before, so
// results do not depend on the choice.
constexpr uint32_t kNoCore = 0xFFFFFFFFu;
// the marks of one run word into the touched-word mask copy Mc (1 bit per 64-bit word of the container)
__device__ __forceinline__ void mark_run(uint32_t *Mc, uint32_t rw) {
  const uint32_t st = rw & 0xFFFF, en = st + (rw >> 16);
  const uint32_t w0 = st >> 6, w1 = en >> 6, d0 = w0 >> 5, d1 = w1 >> 5;
  const uint32_t mlo = 0xFFFFFFFFu << (w0 & 31), mhi = 0xFFFFFFFFu >> (31 - (w1 & 31));
  atomicOr(&Mc[d0], d0 == d1 ? (mlo & mhi) : mlo);
  if (d1 != d0) {
    atomicOr(&Mc[d1], mhi);
    for (uint32_t d = d0 + 1; d < d1; ++d) atomicOr(&Mc[d], 0xFFFFFFFFu); // runs over 2048 values
  }
}
// the boundary toggles of the active lanes' runs into the toggle image, the candidate's by parity (above);
// every lane of the wave calls it (ballots)
__device__ __forceinline__ void toggle_runs_core(const XWin &w, uint32_t *acc, bool act, uint32_t core, int lane) {
  const uint32_t cs = core == kNoCore ? 0x1FFFFu : (core & 0xFFFFu);
  const uint32_t ce = core == kNoCore ? 0x3FFFFu : cs + (core >> 16) + 1;
  const uint32_t rw[8] = {w.r0.x, w.r0.y, w.r0.z, w.r0.w, w.r1.x, w.r1.y, w.r1.z, w.r1.w};
  bool hs = false, he = false;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (act && (uint32_t)u < w.nr) {
      const uint32_t st = rw[u] & 0xFFFF, e1 = st + (rw[u] >> 16) + 1;
      const bool ms = st == cs, me = e1 == ce;
      hs = hs || ms;
      he = he || me;
      if (!ms) atomicXor(&acc[st >> 5], 1u << (st & 31));
      if (!me && e1 < (uint32_t)kSpan) atomicXor(&acc[e1 >> 5], 1u << (e1 & 31));
    }
  }
  const uint64_t bs = __ballot(hs), be = __ballot(he);
  if (lane == 0) {
    if (__popcll(bs) & 1) atomicXor(&acc[cs >> 5], 1u << (cs & 31));
    if ((__popcll(be) & 1) && ce < (uint32_t)kSpan) atomicXor(&acc[ce >> 5], 1u << (ce & 31));
  }
}
#ifndef RBG_XOR_MIN_FAST
#define RBG_XOR_MIN_FAST 8 // study builds (A/B of the heuristic)
#endif
constexpr int kXorMinFast = RBG_XOR_MIN_FAST; // shortest stretch worth a fast-forward (an exact batch costs ~32 stretches' steps)
// Union stretches.  The pair bounds above limit an AB stretch to about one window when the members'
// XOR can reach the accumulator's size (config 4: |C ⊕ C'| ~ 900 per pair, ~29k per window against
// c ~ 32k), so every window paid a toggle -> word conversion and a re-measure (~600 of ~1100 VALU per
// window, ISA count).  A second, bound-free proof covers whole windows at once: every member of a
// stretch lies inside U, the union of its runs, so each intermediate X_j ⊆ U and
//   c_j = |P ⊕ X_j| >= |P \ U| >= |P \ U'|      for any U' ⊇ U,
// with U' = U rounded out to 64-bit words (a 1024-bit touched-word mask in LDS, one or two atomic ORs
// per run).  While |P \ U'| >= 32 every step of an AB-typed accumulator is AB(c_j) (c_j >= 32, never
// empty), so the windows' toggles accumulate in the toggle image with no conversion at all; the stretch
// closes (one conversion, one re-measure of c) when the next window would push |P \ U'| below 32.
#ifndef RBG_XOR_UNION_MINC
#define RBG_XOR_UNION_MINC 1024 // study builds (A/B of the heuristic)
#endif
constexpr int kXorUnionMinC = RBG_XOR_UNION_MINC; // try a union stretch only above this c (a heuristic: results do not depend on it)
#ifndef RBG_STUDY
#define RBG_STUDY 0 // study builds: per-key stretch counts of three keys (printf)
#endif
// Study builds (a per-pass counter split): RBG_XOR_DUP = 1 runs every union window's marks +
// |P \ U'| check twice, 2 its toggles three times, 3 every union flush twice.  Each repeat leaves the result
// unchanged (OR marks are idempotent, three XOR toggles equal one, a flush of a zeroed image adds nothing), so
// the kernel's extra time and counters under a variant are that pass's marginal cost at full occupancy.
#ifndef RBG_XOR_DUP
#define RBG_XOR_DUP 0
#endif
#ifndef RBG_XOR_CORE_MARKS
#define RBG_XOR_CORE_MARKS 0 // study builds: 1 de-duplicates the core run's marks only (toggles as before)
#endif
#ifndef RBG_XOR_CORE
#define RBG_XOR_CORE 0 // study builds: 1 de-duplicates the core run's toggles and marks (slower: DESIGN.md §7 r06)
#endif

__global__ __launch_bounds__(256, 3) void k_wide_runs_xor(SetView s, const uint32_t *__restrict__ rec,
                                                          const uint64_t *__restrict__ seg,
                                                          const uint32_t *__restrict__ klist, uint32_t nk,
                                                          uint8_t *__restrict__ out, WideOut wo,
                                                          uint8_t *__restrict__ route, uint64_t *stats,
                                                          int fastfwd) {
  __shared__ __attribute__((aligned(16))) uint32_t acc_all[4][2048];
  __shared__ __attribute__((aligned(16))) uint32_t reg_all[4][kXRegion];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t q = xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wv;
  if (q >= nk) return;
  // acc: the accumulator P during exact batches, the (zeroed) toggle image of fast-forwards; P itself
  // lives in registers between batches (the 65536-bit register layout of wave.hpp)
  uint32_t *acc = acc_all[wv];
  uint32_t *R = reg_all[wv];
  const uint32_t key = klist[q];
  const uint64_t lo = seg[key], hi = seg[key + 1];
  if (hi <= lo || !xrec_ok(rec[lo])) { // (no member) / first container not a Run of <= 8 runs: the generic kernel
    if (lane == 0) route[q] = 1;
    return;
  }
  lds_zero(acc, lane);
  wave_lds_sync();
  uint64_t Pw[kW];
#pragma unroll
  for (int j = 0; j < kW; ++j) Pw[j] = 0;
  XState X{3, 0, 0, 0u, 1};
  bool fail_route = false;
  uint64_t wbase = lo;
  auto rec_at = [&](uint64_t i) { // unconditional load (clamped address, selected later); hi > lo here
    return rec[i < hi ? i : hi - 1];
  };
  const uint32_t r0 = rec_at(lo + lane), r1 = rec_at(lo + 64 + lane);
  uint32_t *nbuf = R + kNextRuns;
  XWin W = xwin_from(s, xmeta_of(r0, lo + lane < hi));       // window w
  XMeta Nm = xmeta_of(r1, lo + 64 + lane < hi);              // w+1: runs in flight into nbuf
  stage_next_runs(s, Nm, nbuf);
  uint32_t NN = rec_at(lo + 128 + lane);                     // w+2: record in flight
  pair_xor(W);
  uint64_t base = lo;
  // union stretch state: windows whose toggles are pending in acc (P = Pw, X describe the accumulator
  // before them) and their touched-word mask M (in R, which only exact batches use otherwise)
  // M: the touched 64-bit words (1024 bits, 32 dwords) in kMCopies copies, lane l marking copy l & 7 —
  // one copy took every member's core run on one dword, serialising 64 atomics per instruction
  uint32_t *M = R;
  uint8_t *pcT = reinterpret_cast<uint8_t *>(R + kPcT); // [1024] popcount of each word of P
  int upend = 0;
  bool urun = false; // flavour of the pending stretch: Run (every step stays a Run) or AB
  int usum = 0;      // Run flavour: Σ nruns of the pending windows (r_j <= X.r + usum)
  bool wpx = true;   // W.pairx is current
  uint32_t ccore = kNoCore; // the pending union stretch's candidate core run (wave-uniform), already in U'
#if RBG_STUDY
  int tr_u = 0, tr_f = 0, tr_rej = 0, tr_p = 0, tr_pb = 0, tr_e = 0;
#define RBG_TR(x) x
  uint64_t tt[6] = {0, 0, 0, 0, 0, 0}, ts = 0; // s_memtime: mark+check, toggles, flush, stretch, exact, advance
#define RBG_TS() ts = __builtin_amdgcn_s_memtime()
#define RBG_TA(i) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); tt[i] += t_ - ts; ts = t_; }
#else
#define RBG_TR(x)
#define RBG_TS()
#define RBG_TA(i)
#endif
  // the pending windows' XOR into P and (c, r) re-measured: the state is AB(c) (AB flavour) or Run
  auto flush_union = [&]() {
    wave_lds_sync();
    uint64_t t[kW];
    lds_read_words(acc, t, lane);
    wave_lds_sync();
    lds_zero(acc, lane);
    toggles_to_words(t, lane);
#pragma unroll
    for (int j = 0; j < kW; ++j) Pw[j] ^= t[j];
    int cc = X.c, rr = X.r;
    metrics(Pw, lane, urun, cc, rr);
    X.c = cc;
    X.r = rr;
    X.rvalid = urun;
    X.state = urun ? (int)kRun : type_ab(cc);
    upend = 0;
    wave_lds_sync();
  };
  while (base < hi) {
    const uint32_t posw = __builtin_amdgcn_readfirstlane((uint32_t)(base - wbase)); // < 64
    const bool inwin = (uint32_t)lane >= posw && wbase + (uint64_t)lane < hi;
    if (__ballot(inwin && (W.typ != kRun || W.nr > 8u || W.card >= (uint32_t)kSpan))) {
      fail_route = true;
      break;
    }
    const uint32_t wlen = (uint32_t)min<uint64_t>(64, hi - wbase); // containers in the window
    // window's Σ nruns (the Run flavour's r bound); a Run stretch needs 2 + 4 r_j <= min(8192, 2 c_j + 2)
    const int wnr = fastfwd && posw == 0 && (upend ? urun : X.state == kRun)
                        ? (int)wave_sum_u32((uint32_t)lane < wlen ? W.nr : 0u) : 0;
    const bool ab_in = X.state == kBitmap || (X.state == kArray && X.c >= kXorUnionMinC);
    const bool run_in = X.state == kRun && X.rvalid && X.c >= kXorUnionMinC &&
                        X.r + wnr <= 2047 && X.c >= 4 * (X.r + wnr); // |P \ U'| ~ c / 2 after a window
    bool took = false; // the window went into a union stretch
    RBG_TS();
    if (fastfwd && posw == 0 && (upend || ab_in || run_in)) {
      // ---- union stretch: mark the window's words, then |P \ U'| decides (see "Union stretches" above)
      const bool mem = (uint32_t)lane < wlen;
      if (!upend) { // a new stretch: clear U', and the per-word popcounts of P for |P \ U'|
        urun = !ab_in;
        usum = 0;
        for (int i = lane; i < kMCopies * kMStride; i += 64) M[i] = 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          reinterpret_cast<uint16_t *>(pcT)[64 * k + lane] =
              (uint16_t)(__popcll(Pw[2 * k]) | (__popcll(Pw[2 * k + 1]) << 8));
        ccore = readlane(longest_run(W), 0); // lane 0 is a member of every union window (posw == 0)
        wave_lds_sync();
        if (lane == 0 && (RBG_XOR_CORE || RBG_XOR_CORE_MARKS)) mark_run(M, ccore); // once for the stretch (copy 0)
      }
      const uint32_t mcore = RBG_XOR_CORE ? ccore : kNoCore;
      const uint32_t mkcore = RBG_XOR_CORE || RBG_XOR_CORE_MARKS ? ccore : kNoCore;
      int L = 0;
      for (int rep = 0; rep < (RBG_XOR_DUP == 1 ? 2 : 1); ++rep) {
      if (mem) {
        const uint32_t rw[8] = {W.r0.x, W.r0.y, W.r0.z, W.r0.w, W.r1.x, W.r1.y, W.r1.z, W.r1.w};
        uint32_t *Mc = M + kMStride * (lane & (kMCopies - 1));
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if ((uint32_t)u < W.nr && rw[u] != mkcore) mark_run(Mc, rw[u]); // the candidate is in U' already
      }
      wave_lds_sync();
      // |P \ U'|: lane l sums the popcounts of words 16 l .. 16 l + 15 not in U'
      uint32_t ls = 0;
      {
        const uint4 pcv = reinterpret_cast<const uint4 *>(pcT)[lane];
        uint32_t mv = 0;
#pragma unroll
        for (int c = 0; c < kMCopies; ++c) mv |= M[kMStride * c + (lane >> 1)];
        const uint32_t tv = (mv >> (16 * (lane & 1))) & 0xFFFFu;
        const uint32_t p4[4] = {pcv.x, pcv.y, pcv.z, pcv.w};
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
          const uint32_t nib = (tv >> (4 * qd)) & 15u;
          const uint32_t bm = ((nib * 0x00204081u) & 0x01010101u) * 0xFFu; // touched words' bytes
          const uint32_t v = p4[qd] & ~bm;
          ls += (v & 0x00FF00FFu) + ((v >> 8) & 0x00FF00FFu);
        }
        ls = (ls & 0xFFFFu) + (ls >> 16);
      }
      L = (int)wave_sum_u32(ls);
      if (RBG_XOR_DUP == 1) wave_lds_sync();
      }
      RBG_TA(0);
      const int rub = X.r + usum + wnr; // >= every r_j of the stretch (Run flavour)
      if (urun ? (2 + 4 * rub <= min(kBitmapBytes, 2 * L + 2)) : L >= kRunArrayThreshold) {
        usum += wnr;
        for (int rep = 0; rep < (RBG_XOR_DUP == 2 ? 3 : 1); ++rep) toggle_runs_core(W, acc, mem, mcore, lane);
        if (mem) X.inb += 4u * W.nr + 2u + 16u;
        ++upend;
        RBG_TR(++tr_u);
        RBG_TA(1);
        base += wlen;
        took = true; // on to the one shared window advance below
      }
      // this window would let U' cover too much of P: close the stretch before it and take the window
      // again as the first of a fresh stretch (U' then holds its words alone); a window refused as
      // the first of a stretch goes to the per-window rules
      else {
        RBG_TR(++tr_rej);
        if (upend) {
          RBG_TR(++tr_f);
          flush_union();
          if (RBG_XOR_DUP == 3) flush_union();
          RBG_TA(2);
          continue;
        }
      }
    }
    if (!took) { // the per-window rules: a pair-bounded stretch, or an exact batch
      if (!wpx) { // the window's pair bounds, computed only where the per-window rules need them
        pair_xor(W);
        wpx = true;
      }
      // ---- the longest stretch from posw that provably crosses no threshold (see above)
      const int nr_first = (int)readlane(W.nr, (int)posw), card_first = (int)readlane(W.card, (int)posw);
      const uint32_t first_even = posw + (posw & 1u);
      const uint32_t pair_in = dpp<0x138>(W.pairx); // wave_shr:1 — the pair (lane-1, lane) on its odd lane
      const bool odd_end = inwin && (lane & 1) && (uint32_t)lane >= first_even + 1u;
      const int S = (int)wave_scan_u32(odd_end ? pair_in : 0u, lane);
      const bool open_pair = inwin && (uint32_t)lane >= first_even && (((uint32_t)lane - first_even) & 1u) == 0;
      const int bound = ((posw & 1u) ? card_first : 0) + S + (open_pair ? (int)W.card : 0); // >= |X_j|
      const int ab_ok_first = X.state == kBitmap || (X.state == kArray && X.c >= kRunArrayThreshold) ||
                              (X.state == kRun && (X.r - nr_first > 2047 || 2 * (X.r - nr_first) > X.c + card_first));
      bool ok = false;
      int mode = 0; // 1: AB stretch, 2: Run stretch
      if (ab_ok_first) {
        mode = 1;
        ok = inwin && X.c - bound >= kRunArrayThreshold;
      } else if (X.state == kRun) {
        mode = 2;
        const int rub = X.r + (int)wave_scan_u32(inwin ? W.nr : 0u, lane), clb = X.c - bound;
        ok = inwin && clb >= 1 && 2 + 4 * rub <= min(kBitmapBytes, 2 * clb + 2);
      }
      const uint64_t okm = __ballot(ok) >> posw;
      // leading members within the bounds (all 64 when posw == 0 and ~okm == 0: ctz of 0 is undefined)
      const uint32_t B = fastfwd ? min(~okm ? (uint32_t)__builtin_ctzll(~okm) : 64u, wlen - posw) : 0u;
      if (B >= kXorMinFast || (B >= 1 && posw + B == wlen)) {
        const bool act = (uint32_t)lane >= posw && (uint32_t)lane < posw + B;
        toggle_runs_core(W, acc, act, RBG_XOR_CORE ? readlane(W.best, (int)posw) : kNoCore, lane);
        if (act) X.inb += 4u * W.nr + 2u + 16u;
        wave_lds_sync();
        uint64_t t[kW];
        lds_read_words(acc, t, lane);
        wave_lds_sync();
        lds_zero(acc, lane);
        toggles_to_words(t, lane);
#pragma unroll
        for (int j = 0; j < kW; ++j) Pw[j] ^= t[j];
        // an AB stretch leaves a Bitmap / Array accumulator whose next rule reads only c (AB), so r is
        // counted again only when a rule can read it (Run stretch, exact batch, the result)
        int cc = X.c, rr = X.r;
        metrics(Pw, lane, mode == 2, cc, rr);
        X.c = cc;
        X.r = rr;
        X.rvalid = mode == 2;
        X.state = mode == 1 ? type_ab(cc) : kRun;
        base += B;
        RBG_TR(++tr_p; tr_pb += B);
        RBG_TA(3);
      } else {
        if (!X.rvalid) {
          int cc, rr;
          metrics(Pw, lane, true, cc, rr);
          X.r = rr;
          X.rvalid = 1;
        }
        lds_write_words(acc, Pw, lane);
        wait_vm0(); // the next window's runs land before the batch reuses R
        wave_lds_sync();
        if (!exact_batch(s, rec, base, hi, acc, R, lane, X)) {
          fail_route = true;
          break;
        }
        lds_read_words(acc, Pw, lane);
        wave_lds_sync();
        lds_zero(acc, lane);
        stage_next_runs(s, Nm, nbuf); // the batch overwrote them: again
        base += kXB;
        RBG_TR(++tr_e);
        RBG_TA(4);
      }
    }
    wave_lds_sync();
    RBG_TS();
    if (base >= wbase + 64 && base < hi) {
      wbase += 64;
      W = take_next(Nm, nbuf, lane);
      Nm = xmeta_of(NN, wbase + 64 + lane < hi);
      stage_next_runs(s, Nm, nbuf);
      NN = rec_at(wbase + 128 + lane);
      wpx = false;
    }
    RBG_TA(5);
  }
  wait_vm0(); // no DMA into this block's LDS outlives the wave
  if (fail_route) {
    if (lane == 0) route[q] = 1;
    return;
  }
  if (upend) {
    RBG_TR(++tr_f);
    flush_union();
  }
#if RBG_STUDY
  if (lane == 0 && (q == 1000 || q == 30000 || q == 65000))
    printf("xor trace key %u: union windows %d flushes %d refused %d | per-window stretches %d (members %d) | exact %d | c %d state %d"
           " | cycles mark %lu toggles %lu flush %lu stretch %lu exact %lu advance %lu\n",
           q, tr_u, tr_f, tr_rej, tr_p, tr_pb, tr_e, X.c, X.state, tt[0], tt[1], tt[2], tt[3], tt[4], tt[5]);
#endif
  // ---- result
  uint8_t *dst = out + (uint64_t)q * kBitmapBytes;
  const int ty = X.state == 3 ? (int)kEmpty : X.state;
  int c = X.c, r = X.r;
  if (ty != (int)kEmpty) {
    // the chain's metrics must describe the accumulated set; a mismatch (never expected) sends the
    // key to the generic kernel instead of emitting a container sized from wrong metrics
    int cc, rr;
    metrics(Pw, lane, true, cc, rr);
    if (!X.rvalid) r = rr;
    if (cc != c || rr != r) {
      if (lane == 0) route[q] = 1;
      return;
    }
    emit_container(ty, Pw, c, r, dst, acc, lane);
  }
  const uint32_t inb_sum = wave_sum_u32(X.inb);
  if (lane == 0) {
    route[q] = 0;
    wo.type[q] = (uint8_t)ty;
    wo.card[q] = (uint32_t)c;
    wo.nruns[q] = (uint16_t)(ty == kRun ? r : 0);
    const int stripe = q & (kStripes - 1);
    atomicAdd((unsigned long long *)&stats[0 * kStripes + stripe], (unsigned long long)inb_sum);
    if (ty != (int)kEmpty)
      atomicAdd((unsigned long long *)&stats[1 * kStripes + stripe],
                (unsigned long long)(payload_bytes(ty, (uint32_t)c, (uint32_t)r) + (ty == kRun ? 2 : 0) + 16));
  }
}

void launch_wide_runs_xor(const SetView &s, const uint32_t *cid, const uint64_t *seg, const uint32_t *klist,
                          uint32_t nk, uint8_t *out, const WideOut &wo, uint8_t *route, uint64_t *stats,
                          const XorRecords &xr, hipStream_t st) {
  if (!nk) return;
  // RBGPU_XOR_NO_FASTFWD=1: exact batches only (an A/B switch for the parity tests)
  const char *e = getenv("RBGPU_XOR_NO_FASTFWD");
  const int fastfwd = !(e && e[0] == '1');
  if (xr.build == XorRecords::kTranspose) {
    launch_records_transpose(xr.mrec, xr.mbase, 0, xr.M, xr.key_lo, xr.key_hi, xr.rec, st);
  } else if (xr.build == XorRecords::kGather && xr.n) {
    k_records_gather<<<(unsigned)std::min<uint64_t>((xr.n + 255) / 256, 65536), 256, 0, st>>>(xr.mrec, cid, seg,
                                                                                           xr.rec);
  }
#ifndef RBG_XOR_LDS_PAD
#define RBG_XOR_LDS_PAD 0 // study: dynamic LDS a block reserves without using it (8192: 2 waves per SIMD instead of 3)
#endif
  k_wide_runs_xor<<<(nk + 3) / 4, 256, RBG_XOR_LDS_PAD, st>>>(s, xr.rec, seg, klist, nk, out, wo, route, stats, fastfwd);
}

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_wide_xor() {}
void warm_wide_xor(hipStream_t st) { k_warm_wide_xor<<<1, 64, 0, st>>>(); }

} // namespace rbg
