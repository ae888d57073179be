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
// Keys with another container type, > 8 runs or a full container are routed to the generic kernel
// (route[q] = 1); results are identical either way.
#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

namespace {

constexpr int kXB = 32;         // containers per batch (2 lanes per container, 4 runs per lane)
constexpr int kXRegion = 1280;  // u32 per wave: pre16 (1024) | then MC (1024) + pos (256)
constexpr uint32_t kNoKey = 0xFFFFFFFFu;
#ifndef RBG_XOR_APPLY_FLAT
#define RBG_XOR_APPLY_FLAT 0 // 1: one flattened loop over the odd intervals (measured slower: 42.8 vs 35.8 ms)
#endif

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

struct XBatch {
  uint32_t card, nr, typ;
  uint4 r; // runs 4h .. 4h+3 of the lane's container
};
__device__ __forceinline__ XBatch load_xbatch(const SetView &s, const uint32_t *cid, uint64_t i, uint64_t hi,
                                              int h) {
  XBatch b;
  b.card = 0;
  b.nr = 0;
  b.typ = kRun;
  b.r = make_uint4(0, 0, 0, 0);
  if (i < hi) {
    const uint32_t c = cid[i];
    b.typ = s.type[c];
    b.card = s.card[c];
    b.nr = s.nruns[c];
    if (b.typ == kRun && b.nr <= 8 && b.nr > (uint32_t)(4 * h))
      b.r = reinterpret_cast<const uint4 *>(s.payload + s.off[c])[h];
  }
  return b;
}

__device__ __forceinline__ uint32_t dmask(uint32_t w, uint32_t lo, uint32_t hi) {
  const uint32_t a = max(lo, w * 32), b = min(hi, w * 32 + 31);
  if (a > b) return 0u;
  return (0xFFFFFFFFu >> (31 - (b - a))) << (a - w * 32);
}

} // namespace

__global__ __launch_bounds__(256) void k_wide_runs_xor(SetView s, const uint32_t *__restrict__ cid,
                                                       const uint64_t *__restrict__ seg,
                                                       const uint32_t *__restrict__ klist, uint32_t nk,
                                                       uint8_t *__restrict__ out, WideOut wo,
                                                       uint8_t *__restrict__ route, uint64_t *stats) {
  __shared__ __attribute__((aligned(16))) uint32_t acc_all[4][2048];
  __shared__ __attribute__((aligned(16))) uint32_t reg_all[4][kXRegion];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t q = blockIdx.x * 4 + wv;
  if (q >= nk) return;
  uint32_t *acc = acc_all[wv];
  uint32_t *R = reg_all[wv];
  uint16_t *R16 = reinterpret_cast<uint16_t *>(R);
  uint16_t *pos = R16 + 2048;                       // [512] sorted position | tie/boundary bit 15
  uint2 *MC = reinterpret_cast<uint2 *>(R);         // [512] (coverage mask, c0 | c1 << 16)
  const uint32_t key = klist[q];
  const uint64_t lo = seg[key], hi = seg[key + 1];
  if (hi > lo && s.type[cid[lo]] != kRun) { // first container not a Run: route before any batch load
    if (lane == 0) route[q] = 1;
    return;
  }
  lds_zero(acc, lane);
  wave_lds_sync();
  const int cj = lane >> 1, h = lane & 1;
  const uint32_t below = (1u << cj) - 1u;
  int state = 3, c = 0, r = 0;
  uint32_t inb = 0;
  bool fail_route = false;
  XBatch nxt = load_xbatch(s, cid, lo + cj, hi, h);
  for (uint64_t base = lo; base < hi; base += kXB) {
    const XBatch cur = nxt;
    __builtin_amdgcn_sched_barrier(0);
    if (base + kXB < hi) nxt = load_xbatch(s, cid, base + kXB + cj, hi, h);
    const bool valid = base + (uint64_t)cj < hi;
    const bool bad = valid && (cur.typ != kRun || cur.nr > 8u || cur.card >= (uint32_t)kSpan);
    if (__ballot(bad)) {
      fail_route = true;
      break;
    }
    if (valid && h == 0) inb += 4u * cur.nr + 2u + 16u;

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
#if RBG_XOR_APPLY_FLAT
      // one flattened loop over the lane's odd intervals (a queue of up to 8), one dword per trip
      uint32_t live = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t pn = e < 7 ? P[e + 1] : pn7;
        if (K[e] != kNoKey && (__popc(Mv[e]) & 1) && pn > P[e]) live |= 1u << e; // (ties: zero length)
      }
      uint32_t w = 1, wend = 0, ia = 0, ib = 0;
      while (true) {
        if (w > wend) {
          if (!live) break;
          const int e = __builtin_ctz(live);
          live &= live - 1;
          uint32_t a = P[0], pn = P[1];
#pragma unroll
          for (int t = 1; t < 8; ++t)
            if (e == t) {
              a = P[t];
              pn = t < 7 ? P[t + 1] : pn7;
            }
          ia = a;
          ib = pn - 1;
          w = a >> 5;
          wend = ib >> 5;
        }
        atomicXor(&acc[w], dmask(w, ia, ib));
        ++w;
      }
#else
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t pn = e < 7 ? P[e + 1] : pn7;
        if (K[e] != kNoKey && (__popc(Mv[e]) & 1) && pn > P[e]) { // (tie groups: zero-length intervals)
          const uint32_t a = P[e], b = pn - 1;
          for (uint32_t w = a >> 5; w <= (b >> 5); ++w) atomicXor(&acc[w], dmask(w, a, b));
        }
      }
#endif
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
      const int cjv = c + ic, rjv = r + ir, cprev = cjv - dc;
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
    state = (int)((G >> (2 * state)) & 3u);
    c += (int)readlane((uint32_t)ic, 63);
    r += (int)readlane((uint32_t)ir, 63);
  }
  if (fail_route) {
    if (lane == 0) route[q] = 1;
    return;
  }
  // ---- result
  uint8_t *dst = out + (uint64_t)q * kBitmapBytes;
  const int ty = state == 3 ? (int)kEmpty : state;
  if (ty != (int)kEmpty) {
    uint64_t w[kW];
    lds_read_words(acc, w, lane);
    wave_lds_sync();
    // the chain's metrics must describe the accumulated set; a mismatch (never expected) sends the
    // key to the generic kernel instead of emitting a container sized from wrong metrics
    int cc, rr;
    metrics(w, lane, true, cc, rr);
    if (cc != c || rr != r) {
      if (lane == 0) route[q] = 1;
      return;
    }
    emit_container(ty, w, c, r, dst, acc, lane);
  }
  const uint32_t inb_sum = wave_sum_u32(inb);
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
                          hipStream_t st) {
  if (!nk) return;
  k_wide_runs_xor<<<(nk + 3) / 4, 256, 0, st>>>(s, cid, seg, klist, nk, out, wo, route, stats);
}

} // namespace rbg
