// wide_runs.hip — wide aggregation over Run-heavy keys (thousands of small Run
// containers per key) without expanding each container to 65536 bits.
//
// The generic k_wide_reduce expands every container into a register bitmap (~6 µs of latency-bound
// work per 20-byte container).  Here, for a key whose containers are all Runs with <= 8 runs:
//   * 64 containers are prefetched per batch, one per lane (cid, descriptor, both 16-B halves of
//     the run list), double-buffered; container j's runs are broadcast with readlane;
//   * naive_xor (FastAggregation.xor, FastAggregation.java:576-582): the accumulator is an 8 KiB
//     LDS bitmap; XOR with a run = complement of its words, done lane-parallel.  Cardinality after
//     the step = c + |run| - 2 |acc ∩ run| (range popcount of the same words); the number of
//     maximal runs changes only at the run's boundary bits s-1, s, e, e+1 (interior rising and
//     falling edges swap and their difference telescopes to M[e] - M[s]) — so the reference's
//     per-step type automaton (RoaringBitmap.xor in place, :3296-3348; RunContainer.xor /
//     ArrayContainer.xor types) runs exactly with O(words of the runs) work per container;
//   * naive_or (FastAggregation.java:541-548): range OR into the LDS bitmap, LR(c) at the end;
//   * workShyAnd (FastAggregation.java:356-396): the accumulator is a list of <= 64 intervals, one per
//     lane, intersected with each container's runs; LR(c) at the end.
// A key that does not qualify (another container type, > 8 runs, > 64 intervals) is routed to the
// generic kernel (route[q] = 1) — results are identical either way.
#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

constexpr int kMaxRunsFast = 8;

// dword mask of [lo, hi] (inclusive bit positions) restricted to dword w
__device__ __forceinline__ uint32_t dword_mask(uint32_t w, uint32_t lo, uint32_t hi) {
  const uint32_t a = max(lo, w * 32), b = min(hi, w * 32 + 31);
  if (a > b) return 0u;
  return (0xFFFFFFFFu >> (31 - (b - a))) << (a - w * 32);
}
__device__ __forceinline__ uint32_t lds_bit(const uint32_t *s, uint32_t x) { return (s[x >> 5] >> (x & 31)) & 1; }

struct RunBatch {
  uint32_t card, nr, typ;
  uint4 r0, r1;
};
__device__ __forceinline__ RunBatch load_batch(const SetView &s, const KeyCids &cid, uint64_t i, uint64_t hi) {
  RunBatch b;
  b.card = 0;
  b.nr = 0;
  b.typ = kRun;
  b.r0 = make_uint4(0, 0, 0, 0);
  b.r1 = make_uint4(0, 0, 0, 0);
  if (i < hi) {
    const uint32_t c = cid[i];
    b.typ = s.type[c];
    b.card = s.card[c];
    b.nr = s.nruns[c];
    if (b.typ == kRun && b.nr <= kMaxRunsFast) {
      const uint4 *p = reinterpret_cast<const uint4 *>(s.payload + s.off[c]);
      b.r0 = p[0];
      if (b.nr > 4) b.r1 = p[1];
    }
  }
  return b;
}
__device__ __forceinline__ uint32_t run_word(const RunBatch &b, int t) {
  switch (t) {
  case 0: return b.r0.x;
  case 1: return b.r0.y;
  case 2: return b.r0.z;
  case 3: return b.r0.w;
  case 4: return b.r1.x;
  case 5: return b.r1.y;
  case 6: return b.r1.z;
  default: return b.r1.w;
  }
}

template <int SEM>
__global__ __launch_bounds__(256) void k_wide_runs(SetView s, CidMap cm,
                                                   const uint64_t *__restrict__ seg, const uint32_t *__restrict__ klist,
                                                   uint32_t nk, uint8_t *__restrict__ out, WideOut wo,
                                                   uint8_t *__restrict__ route, uint64_t *stats) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_all[4][2048];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t q = xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wv;
  if (q >= nk) return;
  uint32_t *acc = lds_all[wv];
  const uint32_t key = klist[q];
  const uint64_t lo = seg[key], hi = seg[key + 1];
  const KeyCids cid(cm, lo, key);
  if (SEM == RB_FAST_OR && hi - lo < 2) { // a lone container: clone + repairAfterLazy -> generic path
    if (lane == 0) route[q] = 1;
    return;
  }
  if (hi > lo && s.type[cid[lo]] != kRun) { // first container not a Run: route before any batch load
    if (lane == 0) route[q] = 1;
    return;
  }
  lds_zero(acc, lane);
  wave_lds_sync();
  // accumulator state (wave-uniform)
  bool present = false, fail_route = false;
  int t = kRun, c = 0, r = 0;
  uint64_t inb = 0;
  RunBatch nxt = load_batch(s, cid, lo + lane, hi);
  for (uint64_t base = lo; base < hi && !fail_route; base += 64) {
    const RunBatch cur = nxt;
    __builtin_amdgcn_sched_barrier(0);
    if (base + 64 < hi) nxt = load_batch(s, cid, base + 64 + lane, hi);
    // eligibility of the whole batch
    const bool bad = (base + lane < hi) && (cur.typ != kRun || cur.nr > (uint32_t)kMaxRunsFast);
    if (__ballot(bad)) {
      fail_route = true;
      break;
    }
    const int nb = (int)min<uint64_t>(64, hi - base);
    for (int j = 0; j < nb; ++j) {
      const int nr = (int)readlane(cur.nr, j);
      const int cc = (int)readlane(cur.card, j);
      inb += 4ull * nr + 2 + 16;
      // this container's runs, wave-uniform: start / end
      uint32_t rs[kMaxRunsFast], re[kMaxRunsFast];
#pragma unroll
      for (int u = 0; u < kMaxRunsFast; ++u) {
        const uint32_t v = readlane(run_word(cur, u), j);
        rs[u] = v & 0xFFFF;
        re[u] = (v & 0xFFFF) + (v >> 16);
      }
      // ---- range updates over the runs' dwords (OR: set, XOR: complement + metrics)
      uint32_t o[kMaxRunsFast + 1];
      o[0] = 0;
#pragma unroll
      for (int u = 0; u < kMaxRunsFast; ++u) o[u + 1] = o[u] + (u < nr ? (re[u] >> 5) - (rs[u] >> 5) + 1 : 0);
      const uint32_t W = o[nr];
      // XOR: boundary bits before the update (lane u <-> run u)
      int dr = 0;
      if (SEM == RB_FAST_XOR && lane < nr) {
        uint32_t s0 = 0, e0 = 0;
#pragma unroll
        for (int u = 0; u < kMaxRunsFast; ++u)
          if (lane == u) {
            s0 = rs[u];
            e0 = re[u];
          }
        const uint32_t bsm1 = s0 ? lds_bit(acc, s0 - 1) : 0, bs = lds_bit(acc, s0), be = lds_bit(acc, e0);
        const uint32_t bep1 = e0 < 65535 ? lds_bit(acc, e0 + 1) : 0;
        dr = -((int)be - (int)bs);                                         // interior edges
        dr += (int)(!bs && !bsm1) - (int)(bs && !bsm1);                    // pair (s-1, s)
        if (e0 < 65535) dr += (int)(bep1 && be) - (int)(bep1 && !be);     // pair (e, e+1)
      }
      uint32_t inter = 0;
      for (uint32_t g0 = 0; g0 < W; g0 += 64) {
        const uint32_t g = g0 + lane;
        uint32_t m = 0, w = 0;
        if (g < W) {
          int u = 0;
#pragma unroll
          for (int v = 1; v < kMaxRunsFast; ++v) u += (v < nr && g >= o[v]) ? 1 : 0;
          uint32_t su = 0, eu = 0, ou = 0;
#pragma unroll
          for (int v = 0; v < kMaxRunsFast; ++v)
            if (u == v) {
              su = rs[v];
              eu = re[v];
              ou = o[v];
            }
          w = (su >> 5) + (g - ou);
          m = dword_mask(w, su, eu);
          if (SEM == RB_FAST_XOR) inter += (uint32_t)__popc(acc[w] & m);
        }
        if (g < W) {
          if (SEM == RB_FAST_XOR) atomicXor(&acc[w], m);
          else atomicOr(&acc[w], m);
        }
      }
      if (SEM == RB_FAST_XOR) {
        const int isum = (int)wave_sum_u32(inter);
        const int dsum = (int)wave_sum_u32((uint32_t)(dr + 4)) - 4 * 64;
        if (!present) { // key absent: clone (type kept)
          present = true;
          t = kRun;
          c = cc;
          r = nr;
        } else {
          const int ct = t, c0 = c;
          c = c0 + cc - 2 * isum;
          r = r + dsum;
          // RunContainer.xor / ArrayContainer.xor / BitmapContainer.xor types, SURVEY §8a
          if (ct == kRun || (ct == kArray && c0 < kRunArrayThreshold)) t = type_eff(c, r);
          else t = type_ab(c);
          if (c == 0) present = false; // RoaringBitmap.xor in place removes the empty container
        }
      }
      wave_lds_sync();
    }
  }
  if (fail_route) {
    if (lane == 0) route[q] = 1;
    return;
  }
  // ---- result
  uint8_t *dst = out + (uint64_t)q * kBitmapBytes;
  int ty = kEmpty;
  if (SEM == RB_FAST_OR) {
    uint64_t w[kW];
    lds_read_words(acc, w, lane);
    int rr;
    metrics(w, lane, false, c, rr);
    ty = type_lr(c);
    r = ty == kRun ? 1 : 0;
  } else {
    ty = present && c > 0 ? t : kEmpty;
  }
  if (ty != kEmpty) {
    uint64_t w[kW];
    lds_read_words(acc, w, lane);
    wave_lds_sync();
    emit_container(ty, w, c, r, dst, acc, lane);
  }
  if (lane == 0) {
    route[q] = 0;
    wo.type[q] = (uint8_t)ty;
    wo.card[q] = (uint32_t)c;
    wo.nruns[q] = (uint16_t)(ty == kRun ? r : 0);
    const int stripe = q & (kStripes - 1);
    atomicAdd((unsigned long long *)&stats[0 * kStripes + stripe], (unsigned long long)inb);
    if (ty != kEmpty)
      atomicAdd((unsigned long long *)&stats[1 * kStripes + stripe],
                (unsigned long long)(payload_bytes(ty, (uint32_t)c, (uint32_t)r) + (ty == kRun ? 2 : 0) + 16));
  }
}

// ---------------------------------------------------------------- workShyAnd, lane-parallel
// AND is order-free (workShyAnd intersects whole key sets; FastAggregation.java:356-396), so the
// containers of a key need not form one chain.  A wave takes KB consecutive keys of klist; lane
// (kk, g) = (lane % KB, lane / KB) intersects members g, g+G, g+2G, ... (G = 64/KB) of key kk into
// its own interval list, then the G lists of a key are intersected pairwise (log2 G levels).  With
// KB consecutive keys per wave, the containers of one member bitmap for those keys are adjacent in
// the SoA arrays, so each metadata load touches a few cache lines instead of 64.
// Per-lane list: <= kAndCap intervals (start | end << 16) in LDS at L[(b*kAndCap + k)*64 + lane],
// double-buffered (b = 0/1).  Each step's loads form a chain (container id -> packed record -> runs);
// every link of it spans several steps (kAndDc / kAndDr / kAndDp below), so a step waits only on
// loads issued two or more steps earlier.  The loads are unconditional — addresses clamped to a valid
// member, results discarded past the lane's count — because a load under a branch makes the waitcnt
// pass wait for every load in flight at the merge (r03 PMC: vmcnt(0) at every step, one memory
// latency per step).  A key with another container type, > 8 runs or a list overflow is routed to the
// generic kernel (route[q] = 1): results are identical.
constexpr int kAndCap = 16;
#ifndef RBG_AND_RING
#define RBG_AND_RING 2 // steps every link of the load chain spans (at 32 keys: 2 1.55, 3 1.64, 4 1.67 ms)
#endif
constexpr int kAndDc = RBG_AND_RING; // steps between a container id's load and its record's load
constexpr int kAndDr = RBG_AND_RING; // steps between a record's load and its runs' load
constexpr int kAndDp = RBG_AND_RING; // steps between the runs' load and their use
constexpr int kAndU = 2 * RBG_AND_RING; // steps per unrolled loop trip: a multiple of Dp, Dp + Dr and Dc
static_assert(kAndU % kAndDp == 0 && kAndU % (kAndDp + kAndDr) == 0 && kAndU % kAndDc == 0, "ring periods");
struct AndMeta {
  uint32_t typ, nr;
};
struct AndRuns {
  uint4 r0, r1;
};
__device__ __forceinline__ uint32_t and_run(const AndRuns &p, int u) {
  switch (u) {
  case 0: return p.r0.x;
  case 1: return p.r0.y;
  case 2: return p.r0.z;
  case 3: return p.r0.w;
  case 4: return p.r1.x;
  case 5: return p.r1.y;
  case 6: return p.r1.z;
  default: return p.r1.w;
  }
}
__device__ __forceinline__ int and_slot(int b, int k, int lane) { return (b * kAndCap + min(k, kAndCap - 1)) * 64 + lane; }
__device__ __forceinline__ uint32_t iv_s(uint32_t x) { return x & 0xFFFF; }
__device__ __forceinline__ uint32_t iv_e(uint32_t x) { return x >> 16; }

// A member's record at step t: the packed 8-B mrec record (when the set already has one), or (SOA, the
// default since round 6) the set's own run-count / offset arrays read directly: no per-set record pass, so a
// fresh set pays nothing before the call (config 4: kernel 1.64 ms + a 1.14-ms k_pack_records
// on a fresh set -> 1.93 ms with the type load, profiles/r06/and).  Raw loaded values; the fields are taken
// apart only where a step uses them.
template <bool SOA> struct AndRec;
template <> struct AndRec<false> {
  uint64_t r;
  __device__ __forceinline__ void load(const SetView &, const uint64_t *mrec, uint64_t id) { r = mrec[id]; }
  __device__ __forceinline__ uint32_t typ() const { return rec_type(r); }
  __device__ __forceinline__ uint32_t nr() const { return rec_nruns(r); }
  __device__ __forceinline__ uint64_t off() const { return rec_off(r); }
};
// (no type load: a container has a run count > 0 exactly when it is a Run — the SoA stores 0 for the others —
// and any other type routes the key, so "not a Run" is all the step needs)
template <> struct AndRec<true> {
  uint32_t n;
  uint64_t o;
  __device__ __forceinline__ void load(const SetView &s, const uint64_t *, uint64_t id) {
    n = s.nruns[id];
    o = s.off[id];
  }
  __device__ __forceinline__ uint32_t typ() const { return n ? (uint32_t)kRun : (uint32_t)kArray; }
  // the packed record's nruns field saturates at 15: the same test (> kMaxRunsFast routes the key)
  __device__ __forceinline__ uint32_t nr() const { return min(n, 15u); }
  __device__ __forceinline__ uint64_t off() const { return o; }
};

template <int KB, bool DENSE, bool SOA>
__global__ __launch_bounds__(256) void k_wide_runs_and(SetView s, const uint64_t *__restrict__ mrec, CidMap cm,
                                                       const uint64_t *__restrict__ seg, const uint32_t *__restrict__ klist,
                                                       uint32_t nk, uint8_t *__restrict__ out, WideOut wo,
                                                       uint8_t *__restrict__ route, uint64_t *stats) {
  constexpr int G = 64 / KB;
  __shared__ __attribute__((aligned(16))) uint32_t lds_all[4][2 * kAndCap * 64];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t q0 = (xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wv) * KB;
  if (q0 >= nk) return;
  uint32_t *L = lds_all[wv];
  const int kk = lane % KB, g = lane / KB;
  const uint32_t q = q0 + kk;
  uint64_t lo = 0, n = 0;
  uint32_t key = 0;
  if (q < nk) {
    key = klist[q];
    lo = seg[key];
    n = seg[key + 1] - lo;
  }
  const uint32_t cnt = n > (uint64_t)g ? (uint32_t)((n - g + G - 1) / G) : 0u; // this lane's members
  const uint32_t tmax = __builtin_amdgcn_readfirstlane(wave_max_u32(cnt));
  // the AND identity: one interval [0, 65535]
  // A list of at most one interval lives in registers (one = [sa, sb] when na == 1): after the first
  // members a key's intersection is one interval (config 4: the shared core run), and a step against
  // it is a few min / max per run, with none of the LDS round trips of the list walk.
  int cur = 0, na = 1;
  bool one = true;
  uint32_t sa = 0, sb = 65535;
  bool bad = false;
  uint64_t inb = 0;
  if (tmax) {
    // load positions: step t reads member g + G min(t, cnt - 1) of the key; a lane without members
    // borrows the first member of the first lane that has one (loads only, never used)
    const int fl = (int)__builtin_ctzll(__ballot(cnt != 0u));
    const uint32_t bg = cnt ? (uint32_t)g : readlane((uint32_t)g, fl);
    const uint32_t bkey = cnt ? key : readlane(key, fl);
    const uint64_t blo = cnt ? lo : ((uint64_t)readlane((uint32_t)(lo >> 32), fl) << 32 | readlane((uint32_t)lo, fl));
    const uint32_t blast = cnt ? cnt - 1 : 0u;
    // metadata: one packed record per container (the set's mrec) instead of type / nruns / off loads;
    // dense members skip the id load too (the id is the member's base + key)
    // the id load's raw value: the dense member base gets the key added where the id is used (an add
    // right behind the load would make the step wait for it)
    auto ld_cid = [&](uint32_t t) -> uint32_t {
      const uint64_t m = bg + (uint64_t)G * min(t, blast); // position in the key's member list
      if constexpr (DENSE) return reinterpret_cast<const uint32_t *>(cm.mbase)[2 * m]; // the low half (ids are u32)
      else return cm.cid[blo + m];
    };
    const uint32_t cadd = DENSE ? bkey : 0u;
    auto ld_runs = [&](const AndRec<SOA> &r) -> AndRuns { // a non-Run record reads the arena's first 16 B instead
      const bool runs = r.typ() == (uint32_t)kRun && r.nr() <= (uint32_t)kMaxRunsFast;
      const uint4 *pp = reinterpret_cast<const uint4 *>(s.payload + (runs ? r.off() : 0ull));
      AndRuns p;
      p.r0 = pp[0];
      p.r1 = pp[runs && r.nr() > 4u ? 1 : 0];
      return p;
    };
    // Rings indexed modulo their length, the loop unrolled over kAndU steps so every slot index is a
    // constant: rotating the rings through register moves would make each step wait for the loads
    // the moves read.  At the top of step t: P[t % Dp] = runs of t, R[(t + i) % (Dp + Dr)] = record of
    // t + i (i < Dp + Dr), C[t % Dc] = id of t + Dp + Dr.  (The runs a step reads were requested at the
    // end of step t - Dp: Dp - 1 whole steps earlier.)
    AndRuns P[kAndDp];
    AndRec<SOA> R[kAndDp + kAndDr];
    uint32_t C[kAndDc];
#pragma unroll
    // container ids are u32 and a dense member's base is biased by -dense_lo: the sum wraps in 32 bits (a
    // 64-bit sum of the raw id and the key pointed past the arrays of a key-range shard)
    for (int i = 0; i < kAndDp + kAndDr; ++i) R[i].load(s, mrec, (uint32_t)(ld_cid((uint32_t)i) + cadd));
#pragma unroll
    for (int i = 0; i < kAndDc; ++i) C[i] = ld_cid((uint32_t)(kAndDp + kAndDr + i));
#pragma unroll
    for (int i = 0; i < kAndDp; ++i) P[i] = ld_runs(R[i]);
    for (uint32_t t0 = 0; t0 < tmax; t0 += kAndU) {
#pragma unroll
      for (int j = 0; j < kAndU; ++j) {
        const uint32_t t = t0 + (uint32_t)j;
        const AndRec<SOA> &rt = R[j % (kAndDp + kAndDr)];
        const AndMeta mt{rt.typ(), rt.nr()};
        const AndRuns &pt = P[j % kAndDp];
        if (t < cnt && !bad) {
          if (mt.typ != kRun || mt.nr > (uint32_t)kMaxRunsFast) {
            bad = true;
          } else if (one) {
            inb += 4ull * mt.nr + 2 + 16;
            if (na) {
              uint32_t k = 0, ns = 0, ne = 0;
#pragma unroll
              for (int u = 0; u < kMaxRunsFast; ++u) {
                const uint32_t w = and_run(pt, u);
                const uint32_t a = max(sa, w & 0xFFFF), b = min(sb, (w & 0xFFFF) + (w >> 16));
                const bool v = u < (int)mt.nr && a <= b;
                k += v ? 1u : 0u;
                ns = v ? a : ns;
                ne = v ? b : ne;
              }
              if (k <= 1) {
                na = (int)k;
                sa = ns;
                sb = ne;
              } else { // the pieces (runs are sorted and disjoint, so are they) to the LDS list
                const int nx = cur ^ 1;
                int o = 0;
#pragma unroll
                for (int u = 0; u < kMaxRunsFast; ++u) {
                  const uint32_t w = and_run(pt, u);
                  const uint32_t a = max(sa, w & 0xFFFF), b = min(sb, (w & 0xFFFF) + (w >> 16));
                  if (u < (int)mt.nr && a <= b) L[and_slot(nx, o++, lane)] = a | (b << 16);
                }
                na = (int)k;
                cur = nx;
                one = false;
              }
            }
          } else {
            inb += 4ull * mt.nr + 2 + 16;
            const int nx = cur ^ 1;
            int i = 0, k = 0;
            uint32_t x = L[and_slot(cur, 0, lane)];
#pragma unroll
            for (int u = 0; u < kMaxRunsFast; ++u) {
              if (u < (int)mt.nr && i < na) {
                const uint32_t w = and_run(pt, u);
                const uint32_t rs = w & 0xFFFF, re = rs + (w >> 16);
                while (i < na && iv_e(x) < rs) x = L[and_slot(cur, ++i, lane)];
                while (i < na && iv_s(x) <= re) {
                  const uint32_t a = max(iv_s(x), rs), b = min(iv_e(x), re);
                  if (k < kAndCap) L[and_slot(nx, k, lane)] = a | (b << 16);
                  ++k;
                  if (iv_e(x) > re) break;
                  x = L[and_slot(cur, ++i, lane)];
                }
              }
            }
            if (k > kAndCap) bad = true;
            na = k;
            cur = nx;
            if (na <= 1 && !bad) { // back to registers
              const uint32_t x1 = L[and_slot(cur, 0, lane)];
              sa = na ? iv_s(x1) : 0u;
              sb = na ? iv_e(x1) : 0u;
              one = true;
            }
          }
        }
        // the step's loads go out after its compute, into the slots it has just consumed (a slot
        // refilled while its old value is still read would need a second register and a copy at the
        // loop's back edge, which waits for the loads)
        __builtin_amdgcn_sched_barrier(0);
        P[j % kAndDp] = ld_runs(R[(j + kAndDp) % (kAndDp + kAndDr)]); // record loaded kAndDr steps ago
        R[j % (kAndDp + kAndDr)].load(s, mrec, (uint32_t)(C[j % kAndDc] + cadd)); // id loaded kAndDc steps ago
        C[j % kAndDc] = ld_cid(t + (uint32_t)(kAndDp + kAndDr + kAndDc));
      }
      // every lane's list empty (or routed): the remaining containers change nothing
      if (!__ballot(t0 + kAndU < cnt && !bad && na > 0)) break;
    }
  }
  if (one) { // the register list into the LDS list for the tree and the emission
    cur = 0;
    if (na) L[and_slot(0, 0, lane)] = sa | (sb << 16);
  }
  // ---- intersect the G lists of each key pairwise
#pragma unroll
  for (int d = 1; d < G; d *= 2) {
    wave_lds_sync();
    const int pl = lane + KB * d;                 // partner lane (same key, group g + d)
    const int pcur = __shfl(cur, pl & 63), pna = __shfl(na, pl & 63);
    const bool pbad = __shfl((int)bad, pl & 63) != 0;
    if (g % (2 * d) == 0) {
      bad = bad || pbad;
      const int nx = cur ^ 1;
      int i = 0, j = 0, k = 0;
      uint32_t x = L[and_slot(cur, 0, lane)], y = L[(pcur * kAndCap) * 64 + (pl & 63)];
      while (i < na && j < pna) {
        const uint32_t a = max(iv_s(x), iv_s(y)), b = min(iv_e(x), iv_e(y));
        if (a <= b) {
          if (k < kAndCap) L[and_slot(nx, k, lane)] = a | (b << 16);
          ++k;
        }
        if (iv_e(x) < iv_e(y)) x = L[and_slot(cur, ++i, lane)];
        else {
          ++j;
          y = L[(pcur * kAndCap + min(j, kAndCap - 1)) * 64 + (pl & 63)];
        }
      }
      if (k > kAndCap) bad = true;
      na = k;
      cur = nx;
    }
  }
  wave_lds_sync();
  // ---- per key (lane kk of group 0): cardinality, LR type (BitmapContainer.repairAfterLazy :1214-1224)
  uint32_t c = 0;
  if (g == 0 && !bad)
    for (int i = 0; i < na; ++i) {
      const uint32_t x = L[and_slot(cur, i, lane)];
      c += iv_e(x) - iv_s(x) + 1;
    }
  const int ty = c ? type_lr((int)c) : kEmpty;
  const uint64_t inb_sum = wave_sum_u64(inb);
  uint64_t outb = 0;
  if (g == 0 && q < nk) {
    route[q] = bad ? 1 : 0;
    if (!bad) {
      wo.type[q] = (uint8_t)ty;
      wo.card[q] = c;
      wo.nruns[q] = (uint16_t)(ty == kRun ? 1 : 0);
      if (ty != kEmpty) outb = payload_bytes(ty, c, 1) + (ty == kRun ? 2 : 0) + 16;
    }
  }
  const uint64_t outb_sum = wave_sum_u64(outb);
  // ---- emission, one key at a time by the whole wave, straight from the interval list
  for (int key = 0; key < KB && q0 + key < nk; ++key) {
    const int kty = __shfl(ty, key), kn = __shfl(na, key), kcur = __shfl(cur, key);
    const bool kbad = __shfl((int)bad, key) != 0;
    if (kbad || kty == kEmpty) continue;
    uint8_t *dst = out + (uint64_t)(q0 + key) * kBitmapBytes;
    if (kty == kRun) { // the full container: one run (0, 65535)
      if (lane == 0) *reinterpret_cast<uint32_t *>(dst) = 0xFFFF0000u;
    } else if (kty == kArray) {
      uint16_t *o16 = reinterpret_cast<uint16_t *>(dst);
      uint32_t pre = 0;
      for (int i = 0; i < kn; ++i) {
        const uint32_t x = L[(kcur * kAndCap + i) * 64 + key];
        const uint32_t a = iv_s(x), len = iv_e(x) - a + 1;
        for (uint32_t v = lane; v < len; v += 64) o16[pre + v] = (uint16_t)(a + v);
        pre += len;
      }
    } else { // Bitmap: word wi = lane + 64 j, OR of the interval masks
      uint64_t *o64 = reinterpret_cast<uint64_t *>(dst);
      for (int j = 0; j < 16; ++j) {
        const uint32_t wi = (uint32_t)(lane + 64 * j), w0 = wi * 64, w1 = w0 + 63;
        uint64_t m = 0;
        for (int i = 0; i < kn; ++i) {
          const uint32_t x = L[(kcur * kAndCap + i) * 64 + key];
          const uint32_t a = max(iv_s(x), w0), b = min(iv_e(x), w1);
          if (a <= b) m |= (~0ull >> (63 - (b - a))) << (a - w0);
        }
        o64[wi] = m;
      }
    }
  }
  if (lane == 0) {
    const int stripe = (q0 / KB) & (kStripes - 1);
    atomicAdd((unsigned long long *)&stats[0 * kStripes + stripe], (unsigned long long)inb_sum);
    atomicAdd((unsigned long long *)&stats[1 * kStripes + stripe], (unsigned long long)outb_sum);
  }
}

#ifndef RBG_AND_KEYS
#define RBG_AND_KEYS 32 // keys per wave (round 6 A/B, profiles/r06/and: 8 2.14, 16 1.80, 32 1.64, 64 1.94 ms)
#endif
constexpr int kAndKeys = RBG_AND_KEYS; // keys per wave of the lane-parallel workShyAnd

bool launch_wide_runs(int sem, const SetView &s, const uint64_t *mrec, const CidMap &cm, const uint64_t *seg,
                      const uint32_t *klist, uint32_t nk, uint8_t *out, const WideOut &wo, uint8_t *route,
                      uint64_t *stats, const XorRecords &xr, hipStream_t st) {
  const unsigned g = (nk + 3) / 4;
  switch (sem) {
  case RB_FAST_OR: k_wide_runs<RB_FAST_OR><<<g, 256, 0, st>>>(s, cm, seg, klist, nk, out, wo, route, stats); return true;
  case RB_WORKSHY_AND: {
    // no mrec: the SoA-reading kernel (RBG_AND_SOA builds, wide.hip then builds no records)
    if (!mrec && !RBG_AND_SOA) return false;
    const unsigned waves = (nk + kAndKeys - 1) / kAndKeys, gb = (waves + 3) / 4;
    if (cm.cid) {
      if (mrec) k_wide_runs_and<kAndKeys, false, false><<<gb, 256, 0, st>>>(s, mrec, cm, seg, klist, nk, out, wo, route, stats);
      else k_wide_runs_and<kAndKeys, false, true><<<gb, 256, 0, st>>>(s, mrec, cm, seg, klist, nk, out, wo, route, stats);
    } else {
      if (mrec) k_wide_runs_and<kAndKeys, true, false><<<gb, 256, 0, st>>>(s, mrec, cm, seg, klist, nk, out, wo, route, stats);
      else k_wide_runs_and<kAndKeys, true, true><<<gb, 256, 0, st>>>(s, mrec, cm, seg, klist, nk, out, wo, route, stats);
    }
    return true;
  }
  case RB_FAST_XOR: // batch-parallel metrics over key-major records (wide_xor.hip)
    if (!xr.rec) return false;
    launch_wide_runs_xor(s, cm.cid, seg, klist, nk, out, wo, route, stats, xr, st);
    return true;
  default: return false;
  }
}

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_wide_runs() {}
void warm_wide_runs(hipStream_t st) { k_warm_wide_runs<<<1, 64, 0, st>>>(); }

} // namespace rbg
