// wide.hip — wide aggregation over many bitmaps: FastAggregation.or/and/xor, naive_and,
// workShyAnd and ParallelAggregation.or/xor (FastAggregation.java:26-42, 328-396, 541-582,
// 602, 772; ParallelAggregation.java:137-229).
//
// Every high-16-bit key is independent.  Pipeline:
//   k_group_*        stable grouping of the members' containers by key (a tiled counting sort),
//                    so each key's containers stay in member order — the order that naive_and /
//                    naive_xor / the ParallelAggregation chains depend on — and seg[k] per key
//   k_wide_select    keys that produce work (any container; for AND: present in every member)
//   k_wide_reduce    ONE WAVE PER KEY: the key's containers folded in registers (65536-bit
//                    register bitmap, Bitmaps streamed two at a time), reference type decision,
//                    emission into an 8 KiB slot
//   compaction       drop empty results, result CSR
#include <cstdlib>
#include <cstring>

#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {


__device__ __forceinline__ uint64_t alg_bytes_w(int t, uint32_t c, uint32_t r) {
  return t == kBitmap ? 8192ull : t == kArray ? 2ull * c : 4ull * r + 2;
}
__device__ __forceinline__ void stat_add_w(uint64_t *stats, int word, uint64_t v) {
  if ((threadIdx.x & 63) == 0 && v) {
    const int stripe = (blockIdx.x * 4 + (threadIdx.x >> 6)) & (kStripes - 1);
    atomicAdd((unsigned long long *)&stats[word * kStripes + stripe], (unsigned long long)v);
  }
}

// ---------------------------------------------------------------- stable grouping by key
// A counting sort over (member block x key range) tiles.  A member holds at most one container per
// key (its keys are sorted and unique), so the slot of member m's key-k container is (start of key
// k) + (earlier members holding key k): member order within a key is kept, which naive_and /
// naive_xor / the ParallelAggregation chains depend on.
//   k_group_bounds   B[m][j] = first container of member m with key >= key_lo + j*KR (binary search)
//   k_group_count    per tile: Hc[block][k] = members of the block holding key k (LDS counters)
//   k_group_totals / scan / k_group_base: seg[k] = start of key k; H[block][k] = first slot of the
//                    block's key-k containers (a column prefix over the blocks)
//   k_group_scatter  per tile: ranks from per-key member masks, ids staged in LDS, stored per key
// Every container of the members is read twice (its key) and its id written once, both coalesced;
// only keys in [key_lo, key_hi) are grouped (a shard reads nothing outside its range).
constexpr uint32_t kGrpKeys = 256;   // keys per tile (one thread per key slot)
constexpr uint32_t kGrpMembers = 64; // members per block (a 64-bit presence mask per key)
struct GroupArgs {
  SetView s;
  const uint32_t *mem;
  const uint64_t *bnd; // [M][nkr + 1]
  uint32_t M, MB, KR, nkr, key_lo, key_hi;
};
__device__ __forceinline__ uint64_t key_lower_bound(const uint16_t *key, uint64_t lo, uint64_t hi, uint32_t k) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (key[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
__global__ __launch_bounds__(256) void k_group_bounds(GroupArgs a, uint64_t *bnd) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t nb = a.nkr + 1;
  if (t >= (uint64_t)a.M * nb) return;
  const uint32_t m = (uint32_t)(t / nb), j = (uint32_t)(t % nb);
  const uint32_t b = a.mem[m];
  const uint32_t k = j == a.nkr ? a.key_hi : a.key_lo + j * a.KR;
  bnd[t] = key_lower_bound(a.s.key, a.s.begin[b], a.s.begin[b + 1], k);
}
// A tile has <= KR (<= 256) keys, so a member has at most one container per thread there: thread t
// takes the t-th container of every member of the block, all loads in flight at once.
__device__ __forceinline__ void tile_load(const GroupArgs &a, uint32_t mb, uint32_t j, uint32_t k0,
                                          uint32_t (&kk)[kGrpMembers], uint32_t (&ci)[kGrpMembers]) {
  const uint32_t m0 = mb * a.MB;
#pragma unroll
  for (int u = 0; u < (int)kGrpMembers; ++u) {
    kk[u] = ~0u;
    ci[u] = 0;
    const uint32_t m = m0 + u;
    if (u < (int)a.MB && m < a.M) {
      const uint64_t *bm = a.bnd + (uint64_t)m * (a.nkr + 1) + j;
      const uint64_t i = bm[0] + threadIdx.x;
      if (i < bm[1]) {
        kk[u] = (uint32_t)a.s.key[i] - k0;
        ci[u] = (uint32_t)i;
      }
    }
  }
}
__global__ __launch_bounds__(256) void k_group_count(GroupArgs a, uint32_t *Hc) {
  __shared__ uint32_t cnt[kGrpKeys];
  const uint32_t mb = blockIdx.y, j = blockIdx.x;
  const uint32_t k0 = a.key_lo + j * a.KR, nk = min(a.KR, a.key_hi - k0);
  cnt[threadIdx.x] = 0;
  uint32_t kk[kGrpMembers], ci[kGrpMembers];
  tile_load(a, mb, j, k0, kk, ci);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < (int)kGrpMembers; ++u)
    if (kk[u] != ~0u) atomicAdd(&cnt[kk[u]], 1u);
  __syncthreads();
  if (threadIdx.x < nk) Hc[(uint64_t)mb * (a.key_hi - a.key_lo) + (k0 - a.key_lo) + threadIdx.x] = cnt[threadIdx.x];
}
__global__ __launch_bounds__(256) void k_group_totals(const uint32_t *Hc, uint32_t nmb, uint32_t key_lo,
                                                      uint32_t key_hi, uint64_t *tot) {
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  if (k > 65536) return;
  uint64_t s = 0;
  if (k >= key_lo && k < key_hi)
    for (uint32_t b = 0; b < nmb; ++b) s += Hc[(uint64_t)b * (key_hi - key_lo) + (k - key_lo)];
  tot[k] = s;
}
__global__ __launch_bounds__(256) void k_group_base(const uint32_t *Hc, uint64_t *H, uint32_t nmb, uint32_t key_lo,
                                                    uint32_t key_hi, const uint64_t *seg) {
  const uint32_t k = key_lo + blockIdx.x * 256 + threadIdx.x;
  if (k >= key_hi) return;
  uint64_t run = seg[k];
  for (uint32_t b = 0; b < nmb; ++b) {
    const uint64_t x = (uint64_t)b * (key_hi - key_lo) + (k - key_lo);
    H[x] = run;
    run += Hc[x];
  }
}
// Per tile: a 64-bit presence mask per key (bit u = member u of the block holds the key) gives every
// container its rank among the key's containers with one LDS atomic and one barrier; the tile's ids
// are staged in LDS in (key, member) order, then each key's run of <= 64 ids is stored contiguously.
// The staged entry is (member u << 8 | thread t): container id = first container of member u in the
// tile + t, so the stage is 32 KiB of u16 (a u32 stage of the ids halves the blocks per CU).
// Dense members (every member holds every key of [dense_lo, dense_hi): container = begin + key -
// dense_lo) need no sort: key k's containers are mbase[j] + k in member order (CidMap), seg[k] =
// (k - key_lo) * M.  This kernel writes seg and the per-member bases.
__global__ __launch_bounds__(256) void k_group_dense(const uint64_t *__restrict__ begin, const uint32_t *__restrict__ mem,
                                                     uint32_t M, uint32_t dense_lo, uint32_t key_lo, uint32_t key_hi,
                                                     uint64_t *seg, uint64_t *mbase) {
  const uint64_t krange = key_hi - key_lo;
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < M; j += (uint64_t)gridDim.x * 256)
    mbase[j] = begin[mem[j]] - dense_lo;
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k <= 65536; k += (uint64_t)gridDim.x * 256)
    seg[k] = (k < key_lo ? 0 : k >= key_hi ? krange : k - key_lo) * M;
}
__global__ __launch_bounds__(256) void k_group_scatter(GroupArgs a, const uint64_t *H, uint32_t *cid) {
  __shared__ unsigned long long mask[kGrpKeys];
  __shared__ uint64_t gbase[kGrpKeys], mbase[kGrpMembers];
  const uint32_t mb = blockIdx.y, j = blockIdx.x, t = threadIdx.x;
  const uint32_t k0 = a.key_lo + j * a.KR, nk = min(a.KR, a.key_hi - k0);
  mask[t] = 0;
  gbase[t] = t < nk ? H[(uint64_t)mb * (a.key_hi - a.key_lo) + (k0 - a.key_lo) + t] : 0;
  if (t < a.MB && mb * a.MB + t < a.M) mbase[t] = a.bnd[(uint64_t)(mb * a.MB + t) * (a.nkr + 1) + j];
  uint32_t kk[kGrpMembers], ci[kGrpMembers];
  tile_load(a, mb, j, k0, kk, ci);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < (int)kGrpMembers; ++u)
    if (kk[u] != ~0u) atomicOr(&mask[kk[u]], 1ull << u);
  __syncthreads();
  {
  __shared__ uint16_t stage[kGrpMembers * kGrpKeys];
  __shared__ uint32_t lofs[kGrpKeys + 1], wsum[4];
  const uint32_t lane = t & 63, wv = t >> 6;
  // tile-local offsets of the keys: exclusive scan of the mask popcounts
  const uint32_t c = (uint32_t)__popcll(mask[t]);
  const uint32_t incl = wave_scan_u32(c, (int)lane);
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < wv; ++w) before += wsum[w];
  lofs[t] = before + incl - c;
  if (t == 255) lofs[kGrpKeys] = before + incl;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < (int)kGrpMembers; ++u)
    if (kk[u] != ~0u)
      stage[lofs[kk[u]] + (uint32_t)__popcll(mask[kk[u]] & ((1ull << u) - 1))] =
          (uint32_t)(u << 8 | t);
  __syncthreads();
  // one wave per key at a time: the key's ids in member order, one contiguous store
  for (uint32_t k = wv; k < nk; k += 4) {
    const uint32_t o = lofs[k], n = lofs[k + 1] - o;
    if (lane < n) {
      const uint32_t v = stage[o + lane];
      cid[gbase[k] + lane] = (uint32_t)(mbase[v >> 8] + (v & 255));
    }
  }
  }
}

// active[k] = 1 when key k (inside the shard's [lo, hi)) produces work: any container, or (AND
// semantics) one per member
// keys that produce work, in a per-block layout: k_wide_select leaves each 256-key block's count in
// bt, the counts are scanned (scan_blocks_multi: bts, bts[256] = nk) and k_wide_list places the keys
__device__ __forceinline__ bool wide_active(const uint64_t *seg, uint64_t need, uint32_t lo, uint32_t hi, uint32_t k) {
  const uint64_t m = seg[k + 1] - seg[k];
  return (k >= lo && k < hi) && (need ? (m == need) : (m > 0));
}
__global__ __launch_bounds__(256) void k_wide_select(const uint64_t *seg, uint64_t need, uint32_t lo, uint32_t hi,
                                                     uint64_t *bt) {
  __shared__ uint32_t wt[4];
  const uint32_t n = block_flag_count(wide_active(seg, need, lo, hi, blockIdx.x * 256 + threadIdx.x), wt);
  if (threadIdx.x == 0) bt[blockIdx.x] = n;
}
__global__ __launch_bounds__(256) void k_wide_list(const uint64_t *seg, uint64_t need, uint32_t lo, uint32_t hi,
                                                   const uint64_t *bts, uint32_t *klist) {
  __shared__ uint32_t wt[4];
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  const bool f = wide_active(seg, need, lo, hi, k);
  const uint32_t r = block_flag_rank(f, wt);
  if (f) klist[bts[blockIdx.x] + r] = k;
}

// ---------------------------------------------------------------- per-key folding helpers
struct CRef {
  int type;
  uint32_t card, nruns;
  const uint8_t *p;
};
__device__ __forceinline__ CRef cref(const SetView &s, uint32_t c) {
  CRef r;
  r.type = s.type[c];
  r.card = s.card[c];
  r.nruns = s.nruns[c];
  r.p = s.payload + s.off[c];
  return r;
}

template <int OP> __device__ __forceinline__ void fold(uint64_t (&acc)[kW], const uint64_t (&x)[kW]) {
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    if (OP == RB_AND) acc[j] &= x[j];
    else if (OP == RB_OR) acc[j] |= x[j];
    else acc[j] ^= x[j];
  }
}

// Fold every container of [lo, hi) into acc with OP; runs of Bitmaps are streamed two per step
// (16 coalesced 1 KiB loads in flight per wave; four per step measured slower: 6.5-7.1 ms config-3
// steps vs 6.4-6.6).  Returns algorithmic bytes read.
template <int OP>
__device__ __forceinline__ uint64_t fold_all(const SetView &s, const KeyCids &cid, uint64_t lo, uint64_t hi,
                                             uint64_t (&acc)[kW], uint32_t *lds, int lane) {
  uint64_t bytes = 0;
  uint64_t i = lo;
  if (i >= hi) return 0;
  // metadata of the current pair as independent loads (one latency, not a chain)
  CRef r0 = cref(s, cid[i]);
  CRef r1 = i + 1 < hi ? cref(s, cid[i + 1]) : r0;
  while (i < hi) {
    if (r0.type == kBitmap && i + 1 < hi && r1.type == kBitmap) {
      bytes += 2 * (8192 + 16);
      uint64_t x[kW], y[kW];
      load_bitmap(r0.p, x, lane);
      load_bitmap(r1.p, y, lane);
      // the next pair's metadata is in flight while this pair's payloads arrive
      const CRef n0 = i + 2 < hi ? cref(s, cid[i + 2]) : r0;
      const CRef n1 = i + 3 < hi ? cref(s, cid[i + 3]) : r0;
      fold<OP>(acc, x);
      fold<OP>(acc, y);
      i += 2;
      r0 = n0;
      r1 = n1;
      continue;
    }
    bytes += alg_bytes_w(r0.type, r0.card, r0.nruns) + 16;
    uint64_t x[kW];
    load_container(r0.type, r0.p, r0.card, r0.nruns, lds, x, lane);
    fold<OP>(acc, x);
    i += 1;
    r0 = r1;
    if (i + 1 < hi) r1 = cref(s, cid[i + 1]);
  }
  return bytes;
}

__device__ __forceinline__ int type_xor_step(int ta, int tb, uint32_t ca, uint32_t cb, int c, int r) {
  // RunContainer.xor / ArrayContainer.xor / BitmapContainer.xor types
  if ((ta == kRun && tb == kRun) || (ta == kArray && tb == kRun && ca < (uint32_t)kRunArrayThreshold) ||
      (ta == kRun && tb == kArray && cb < (uint32_t)kRunArrayThreshold))
    return type_eff(c, r);
  return type_ab(c);
}

// lazyIOR chain states (Container.lazyIOR, Container.java:717-740)
enum { kStA = 0, kStBValid = 1, kStRun = 2, kStBLazy = 3 };

template <int SEM>
__global__ __launch_bounds__(256) void k_wide_reduce(SetView s, CidMap cm,
                                                     const uint64_t *__restrict__ seg, const uint32_t *__restrict__ klist,
                                                     uint32_t nk, uint8_t *__restrict__ out, WideOut wo,
                                                     const uint8_t *__restrict__ route, uint64_t *stats) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_all[4][2048];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t q = xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wv;
  if (q >= nk) return;
  if (route && route[q] == 0) return; // done by the Run-list fast path (wide_runs.hip)
  uint32_t *lds = lds_all[wv];
  const uint32_t key = klist[q];
  const uint64_t lo = seg[key], hi = seg[key + 1];
  const KeyCids cid(cm, lo, key);
  const uint64_t m = hi - lo;
  uint8_t *dst = out + (uint64_t)q * kBitmapBytes;
  uint64_t acc[kW];
  uint64_t inb = 0;
  int ty = kEmpty, c = 0, r = 0;

  if ((SEM == RB_HORIZONTAL_OR || SEM == RB_HORIZONTAL_XOR) && m == 1) {
    // horizontal_*: a key held by one bitmap is appended as a clone, unrepaired
    // (FastAggregation.java:139-145, 258-264)
    const CRef a = cref(s, cid[lo]);
    inb = alg_bytes_w(a.type, a.card, a.nruns) + 16;
    copy_payload(a.p, dst, payload_bytes(a.type, a.card, a.nruns), lane);
    ty = a.type;
    c = (int)a.card;
    r = (int)a.nruns;
  } else if ((SEM == RB_FAST_OR || SEM == RB_PAR_OR || SEM == RB_BUFFER_NAIVE_OR) && m == 1) {
    // a key seen once: clone, then repairAfterLazy (A, B unchanged; Run -> toEfficientContainer)
    const CRef a = cref(s, cid[lo]);
    inb = alg_bytes_w(a.type, a.card, a.nruns) + 16;
    if (a.type != kRun || 2 + 4 * (int)a.nruns <= min(kBitmapBytes, 2 * (int)a.card + 2)) {
      copy_payload(a.p, dst, payload_bytes(a.type, a.card, a.nruns), lane);
      ty = a.type;
      c = (int)a.card;
      r = (int)a.nruns;
    } else {
      load_container(a.type, a.p, a.card, a.nruns, lds, acc, lane);
      c = (int)a.card;
      r = (int)a.nruns;
      ty = type_ab(c);
      emit_container(ty, acc, c, r, dst, lds, lane);
    }
  } else if (SEM == RB_FAST_OR || (SEM == RB_PAR_OR && m >= 16)) {
    // naive_or: BitmapContainer.lazyIOR over everything, then repairAfterLazy -> LR(c)
#pragma unroll
    for (int j = 0; j < kW; ++j) acc[j] = 0;
    inb = fold_all<RB_OR>(s, cid, lo, hi, acc, lds, lane);
    metrics(acc, lane, false, c, r);
    ty = type_lr(c);
    if (ty == kRun) r = 1;
    emit_container(ty, acc, c, r, dst, lds, lane);
  } else if (SEM == RB_WORKSHY_AND) {
    // workShyAnd: all-ones lazy BitmapContainer.iand over the key's containers, repair -> LR(c)
#pragma unroll
    for (int j = 0; j < kW; ++j) acc[j] = ~0ull;
    inb = fold_all<RB_AND>(s, cid, lo, hi, acc, lds, lane);
    metrics(acc, lane, false, c, r);
    ty = c ? type_lr(c) : kEmpty;
    if (ty == kRun) r = 1;
    if (ty != kEmpty) emit_container(ty, acc, c, r, dst, lds, lane);
  } else if (SEM == RB_NAIVE_AND || SEM == RB_NAIVE_AND_ITER) {
    // clone of the first (smallest) bitmap's container, then in-place and() in member order:
    // R&R -> EFF, otherwise AB; the key disappears once empty (RoaringBitmap.and(x2) :1272-1296)
    const CRef a = cref(s, cid[lo]);
    inb = alg_bytes_w(a.type, a.card, a.nruns) + 16;
    int t = a.type;
    c = (int)a.card;
    r = (int)a.nruns;
    load_container(a.type, a.p, a.card, a.nruns, lds, acc, lane);
    for (uint64_t i = lo + 1; i < hi && c > 0; ++i) {
      const CRef b = cref(s, cid[i]);
      inb += alg_bytes_w(b.type, b.card, b.nruns) + 16;
      uint64_t x[kW];
      load_container(b.type, b.p, b.card, b.nruns, lds, x, lane);
      fold<RB_AND>(acc, x);
      const bool eff = t == kRun && b.type == kRun;
      metrics(acc, lane, eff, c, r);
      t = eff ? type_eff(c, r) : type_ab(c);
    }
    ty = c ? t : kEmpty;
    if (ty != kEmpty) emit_container(ty, acc, c, r, dst, lds, lane);
  } else if (SEM == RB_FAST_XOR || SEM == RB_PAR_XOR || SEM == RB_HORIZONTAL_XOR) {
    // naive_xor: in-place xor() per bitmap — absent key -> clone; empty -> key removed
    //   (RoaringBitmap.xor(x2) :3296-3348).  ParallelAggregation.xor: clone + ixor fold with no
    //   removal (ParallelAggregation.java:189-195); an empty Run accumulator returns the other
    //   operand (RunContainer.lazyxor :1816-1821, xor(Run) :2450-2455).
    bool present = false;
    int t = kArray;
    for (uint64_t i = lo; i < hi; ++i) {
      const CRef b = cref(s, cid[i]);
      inb += alg_bytes_w(b.type, b.card, b.nruns) + 16;
      uint64_t x[kW];
      load_container(b.type, b.p, b.card, b.nruns, lds, x, lane);
      if (!present) {
#pragma unroll
        for (int j = 0; j < kW; ++j) acc[j] = x[j];
        t = b.type;
        c = (int)b.card;
        r = (int)b.nruns;
        present = true;
        continue;
      }
      const int ct = t;
      const uint32_t cc = (uint32_t)c;
      fold<RB_XOR>(acc, x);
      metrics(acc, lane, true, c, r);
      if ((SEM == RB_PAR_XOR || SEM == RB_HORIZONTAL_XOR) && ct == kRun && cc == 0 && b.type != kBitmap) t = b.type;
      else t = type_xor_step(ct, b.type, cc, b.card, c, r);
      if (SEM == RB_FAST_XOR && c == 0) present = false;
    }
    // horizontal_xor appends the key's result even when it is empty (FastAggregation.java:278)
    ty = SEM == RB_HORIZONTAL_XOR ? t : present && c > 0 ? t : kEmpty;
    if (ty != kEmpty) emit_container(ty, acc, c, r, dst, lds, lane);
  } else { // RB_PAR_OR with 2..15 containers and RB_BUFFER_NAIVE_OR with any count (MutableRoaringBitmap.lazyor
           // per bitmap): clone + lazyIOR chain + repairAfterLazy; RB_HORIZONTAL_OR: lazyOR of the first two,
           // then the same lazyIOR chain + repairAfterLazy
    const CRef a = cref(s, cid[lo]);
    inb = alg_bytes_w(a.type, a.card, a.nruns) + 16;
    load_container(a.type, a.p, a.card, a.nruns, lds, acc, lane);
    int st = a.type == kArray ? kStA : a.type == kBitmap ? kStBValid : kStRun;
    c = (int)a.card;
    r = (int)a.nruns;
    uint64_t i0 = lo + 1;
    if (SEM == RB_HORIZONTAL_OR) {
      // Container.lazyOR (Container.java:751-774) of the first two polled containers
      const CRef b = cref(s, cid[lo + 1]);
      inb += alg_bytes_w(b.type, b.card, b.nruns) + 16;
      uint64_t x[kW];
      load_container(b.type, b.p, b.card, b.nruns, lds, x, lane);
      fold<RB_OR>(acc, x);
      metrics(acc, lane, true, c, r);
      if (a.type == kBitmap || b.type == kBitmap) st = kStBLazy;                  // BitmapContainer.lazyor
      else if (a.type == kArray && b.type == kArray)
        st = a.card + b.card > 1024u ? kStBLazy : kStA;                            // ArrayContainer.lazyor :1449
      else if (a.type == kRun && b.type == kRun) {                                 // RunContainer.or -> EFF
        const int e = type_eff(c, r);
        st = c == kSpan ? kStRun : e == kRun ? kStRun : e == kBitmap ? kStBValid : kStA;
      } else st = c == kSpan ? kStRun : (r > kMaxArray ? kStBLazy : kStRun);       // RunContainer.lazyorToRun
      i0 = lo + 2;
    }
    for (uint64_t i = i0; i < hi; ++i) {
      const CRef b = cref(s, cid[i]);
      inb += alg_bytes_w(b.type, b.card, b.nruns) + 16;
      const bool acc_full = st == kStRun && c == kSpan;
      uint64_t x[kW];
      load_container(b.type, b.p, b.card, b.nruns, lds, x, lane);
      if (acc_full) continue; // RunContainer.ilazyor / ior return a full `this`
      const int prev = st;
      const uint32_t cprev = (uint32_t)c;
      fold<RB_OR>(acc, x);
      metrics(acc, lane, true, c, r);
      if (prev == kStBValid || prev == kStBLazy) {
        st = kStBLazy; // BitmapContainer.ilazyor
      } else if (prev == kStA) {
        if (b.type == kArray) st = cprev + b.card > 1024u ? kStBLazy : kStA;     // ArrayContainer.lazyor :1449
        else if (b.type == kBitmap) st = c == kSpan ? kStRun : kStBValid;        // BitmapContainer.or(Array)
        else st = c == kSpan ? kStRun : (r > kMaxArray ? kStBLazy : kStRun);     // RunContainer.lazyorToRun
      } else { // Run accumulator
        if (b.type == kArray) st = r > kMaxArray ? kStBLazy : kStRun;            // ilazyorToRun
        else if (b.type == kBitmap) st = c == kSpan ? kStRun : kStBValid;        // RunContainer.or(Bitmap)
        else {                                                                    // ior(Run) -> toEfficientContainer
          const int e = type_eff(c, r);
          st = e == kRun ? kStRun : e == kBitmap ? kStBValid : kStA;
        }
      }
    }
    if (st == kStA) ty = kArray;
    else if (st == kStBValid) ty = kBitmap;
    else if (st == kStRun) ty = type_eff(c, r);
    else {
      ty = type_lr(c);
      if (ty == kRun) r = 1;
    }
    emit_container(ty, acc, c, r, dst, lds, lane);
  }
  if (lane == 0) {
    wo.type[q] = (uint8_t)ty;
    wo.card[q] = (uint32_t)c;
    wo.nruns[q] = (uint16_t)(ty == kRun ? r : 0);
  }
  stat_add_w(stats, 0, inb);
  if (ty != kEmpty) stat_add_w(stats, 1, alg_bytes_w(ty, (uint32_t)c, (uint32_t)r) + 16);
}

// Keyed compaction in the per-block layout (as the pairwise compaction): k_wide_keep leaves each
// block's kept total, one scan_blocks_multi launch scans the block totals (its total, the result
// container count, goes straight to stats word 8), and k_wide_write ranks its block's results.
__global__ __launch_bounds__(256) void k_wide_keep(const uint8_t *type, uint32_t nk, uint64_t *bk) {
  __shared__ uint32_t wt[4];
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  const uint64_t m = __ballot(q < nk && type[q] != kEmpty);
  if ((threadIdx.x & 63) == 0) wt[threadIdx.x >> 6] = (uint32_t)__popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) bk[blockIdx.x] = (uint64_t)wt[0] + wt[1] + wt[2] + wt[3];
}
// bks: exclusive scans of the block totals (bks[nblocks] = the total); begin: the result's CSR
__global__ __launch_bounds__(256) void k_wide_write(const uint32_t *klist, uint32_t nk, WideOut wo,
                                                    const uint64_t *bks, uint32_t nblocks, OutView ov,
                                                    uint64_t *begin, uint64_t *stats) {
  __shared__ uint32_t wt[4];
  const uint32_t q = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool live = q < nk && wo.type[q] != kEmpty;
  if (blockIdx.x == 0 && threadIdx.x < 2) begin[threadIdx.x] = threadIdx.x ? bks[nblocks] : 0ull;
  // stats word 7: the result's cardinality (RoaringBitmap.getCardinality of the aggregate)
  const uint64_t cs = wave_sum_u64(live ? (uint64_t)wo.card[q] : 0ull);
  if (lane == 0 && cs)
    atomicAdd((unsigned long long *)&stats[7 * kStripes + ((q >> 6) & (kStripes - 1))], (unsigned long long)cs);
  const uint64_t m = __ballot(live);
  if (lane == 0) wt[w] = (uint32_t)__popcll(m);
  __syncthreads();
  if (!live) return;
  uint64_t r = bks[blockIdx.x] + mbcnt64(m);
  for (int i = 0; i < w; ++i) r += wt[i];
  ov.key[r] = (uint16_t)klist[q];
  ov.type[r] = wo.type[q];
  ov.card[r] = wo.card[q];
  ov.nruns[r] = wo.nruns[q];
  ov.off[r] = (uint64_t)q * kBitmapBytes;
}

// ---------------------------------------------------------------- host orchestration
static unsigned nblk(uint64_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

// Result of a keyed reduction (one 8 KiB slot per active key q, type kEmpty = dropped) -> the
// one-bitmap result set: drop empties, write key/type/card/nruns/offset and the CSR, all on the
// device with no read-back: the result container count is stats word 8, which stats_end reads
// (keyed_result_count after it).
int compact_keyed(rbgpu_ctx *ctx, const uint32_t *d_klist, uint32_t nk, const WideOut &wo, rbgpu_set *res) {
  hipStream_t st = ctx->stream;
  if (!nk) {
    HIPCHK(hipMemsetAsync(res->begin, 0, 16, st));
    return RB_OK;
  }
  const uint32_t nb = nblk(nk, 256);
  uint64_t *bk = nullptr, *bks = nullptr;
  if (ctx->pool.alloc((void **)&bk, (nb + 1) * 8ull) || ctx->pool.alloc((void **)&bks, (nb + 1) * 8ull)) {
    ctx->pool.release(bk);
    return fail(RB_ENOMEM, "keyed compaction workspace");
  }
  k_wide_keep<<<nb, 256, 0, st>>>(wo.type, nk, bk);
  const uint64_t *in[1] = {bk};
  uint64_t *outp[1] = {bks};
  scan_blocks_multi(in, outp, 1, nb, ctx->d_stats + 8 * kStripes, st);
  k_wide_write<<<nb, 256, 0, st>>>(d_klist, nk, wo, bks, nb,
                                   OutView{res->key, res->type, res->card, res->nruns, res->off}, res->begin,
                                   ctx->d_stats);
  LAUNCHCHK();
  // pool buffers go back to the pool at once: the pool only hands them out again to later work on
  // this stream, which runs after these kernels
  ctx->pool.release(bk);
  ctx->pool.release(bks);
  return RB_OK;
}
// after stats_end of a call that ran compact_keyed: its result container count, recorded in the stats
uint64_t keyed_result_count(rbgpu_ctx *ctx, rbgpu_set *res) {
  const uint64_t nres = ctx->words[8];
  ctx->last.result_containers = nres;
  res->nc = nres;
  res->h_begin = {0, nres};
  return nres;
}

template <int SEM>
static void launch_reduce(const SetView &s, const CidMap &cm, const uint64_t *seg, const uint32_t *klist,
                          uint32_t nk, uint8_t *out, const WideOut &wo, uint64_t *stats, hipStream_t st,
                          const uint8_t *route = nullptr) {
  k_wide_reduce<SEM><<<nblk(nk, 4), 256, 0, st>>>(s, cm, seg, klist, nk, out, wo, route, stats);
}

// FastAggregation.horizontal_or / horizontal_xor's container order (FastAggregation.java:124-289): a
// ContainerPointer per member in a java.util.PriorityQueue ordered by key, then by cardinality
// descending (RoaringArray.java:708-713); per key the poll order is the fold order.  The tie order
// depends on the whole queue's history, so the host replays the queue over the members' keys and
// cardinalities (6 bytes per container read back) and the device folds each key in that order.
static int horizontal_order(const rbgpu_set *in, const std::vector<uint32_t> &mem, std::vector<uint32_t> &cid,
                            std::vector<uint64_t> &seg) {
  const uint64_t nc = in->nc;
  std::vector<uint16_t> K(nc);
  std::vector<uint32_t> C(nc);
  if (nc) {
    HIPCHK(hipMemcpyAsync(K.data(), in->key, nc * 2, hipMemcpyDeviceToHost, in->ctx->stream));
    HIPCHK(hipMemcpyAsync(C.data(), in->card, nc * 4, hipMemcpyDeviceToHost, in->ctx->stream));
    HIPCHK(hipStreamSynchronize(in->ctx->stream));
  }
  struct P {
    uint32_t m;  // member
    uint64_t k;  // container index in the set
  };
  std::vector<uint64_t> end(mem.size());
  for (size_t i = 0; i < mem.size(); ++i) end[i] = in->h_begin[mem[i] + 1];
  auto cmp = [&](const P &a, const P &b) {
    return K[a.k] != K[b.k] ? (int)K[a.k] - (int)K[b.k] : (int)C[b.k] - (int)C[a.k];
  };
  JavaHeap<P, decltype(cmp)> pq(cmp);
  for (size_t i = 0; i < mem.size(); ++i) {
    const P x{(uint32_t)i, in->h_begin[mem[i]]};
    if (x.k < end[i]) pq.offer(x);
  }
  cid.clear();
  seg.assign(65537, 0);
  int cur = -1;
  auto advance = [&](P x) { // ContainerPointer.advance + re-queue while it points at a container
    ++x.k;
    if (x.k < end[x.m]) pq.offer(x);
    return x.k < end[x.m];
  };
  while (!pq.empty()) {
    const P x1 = pq.poll();
    const int key = K[x1.k];
    for (int k = cur + 1; k <= key; ++k) seg[k] = cid.size();
    cur = key;
    cid.push_back((uint32_t)x1.k);
    if (pq.empty() || K[pq.peek().k] != key) {
      advance(x1);
      continue;
    }
    const P x2 = pq.poll();
    cid.push_back((uint32_t)x2.k);
    while (!pq.empty() && K[pq.peek().k] == key) {
      const P x = pq.poll();
      cid.push_back((uint32_t)x.k);
      if (!advance(x) && pq.empty()) break;
    }
    advance(x1);
    advance(x2);
  }
  for (int k = cur + 1; k <= 65536; ++k) seg[k] = cid.size();
  return RB_OK;
}

int wide_run(rbgpu_ctx *ctx, int sem, const rbgpu_set *in, const std::vector<uint32_t> &members_in,
             uint32_t key_lo, uint32_t key_hi, rbgpu_set **out) {
  hipStream_t st = ctx->stream;
  DevPool &pool = ctx->pool;
  // effective member order: FastAggregation.and(varargs) picks workShyAnd above 10 inputs;
  // naive_and starts from the smallest bitmap (first on ties) and skips it by identity.
  std::vector<uint32_t> members = members_in;
  if (sem == RB_FAST_AND) sem = members.size() > 10 ? RB_WORKSHY_AND : RB_NAIVE_AND;
  if (sem == RB_NAIVE_AND && !members.empty()) {
    uint32_t smallest = members[0];
    for (uint32_t m : members)
      if (in->h_begin[m + 1] - in->h_begin[m] < in->h_begin[smallest + 1] - in->h_begin[smallest]) smallest = m;
    std::vector<uint32_t> ord{smallest};
    for (uint32_t m : members)
      if (m != smallest) ord.push_back(m);
    members.swap(ord);
  }
  const uint32_t M = (uint32_t)members.size();
  std::vector<uint64_t> mstart(M + 1, 0);
  for (uint32_t i = 0; i < M; ++i) mstart[i + 1] = mstart[i] + (in->h_begin[members[i] + 1] - in->h_begin[members[i]]);
  const uint64_t N = mstart[M];
  if (in->nc >= (1ull << 32)) return fail(RB_EINVAL, "wide aggregation supports < 2^32 containers per set");
  const bool and_sem = sem == RB_WORKSHY_AND || sem == RB_NAIVE_AND || sem == RB_NAIVE_AND_ITER;
  const bool horizontal = sem == RB_HORIZONTAL_OR || sem == RB_HORIZONTAL_XOR;
  // Dense members (every bitmap of the set holds every key of [dense_lo, dense_hi)): no grouping, the
  // container ids follow from the member bases (CidMap).  The set's derived metadata is built here, on
  // its first wide use, before the call's accounting starts (rbgpu_set::derive_ms reports its cost).
  static const bool no_dense = getenv("RBGPU_NO_DENSE_GROUPING") != nullptr;
  bool dense = M && !horizontal && !no_dense;
  if (dense) {
    int rc = ensure_dense(in);
    if (rc) return rc;
    dense = in->dense_lo >= 0 && (uint32_t)std::max<int64_t>(key_lo, in->dense_lo) <
                                     (uint32_t)std::min<int64_t>(key_hi, in->dense_hi);
  }
  if (dense) { // keys outside the set's range hold no container: the call's range is the overlap
    key_lo = (uint32_t)std::max<int64_t>(key_lo, in->dense_lo);
    key_hi = (uint32_t)std::min<int64_t>(key_hi, in->dense_hi);
  }
  const bool identity = [&] {
    if (M != in->nb) return false;
    for (uint32_t i = 0; i < M; ++i)
      if (members[i] != i) return false;
    return true;
  }();
  const bool fast_sem = sem == RB_FAST_OR || sem == RB_WORKSHY_AND || sem == RB_FAST_XOR;
  bool fast_ok = fast_sem && !getenv("RBGPU_NO_RUN_FASTPATH"); // parity tests run both paths
  if (fast_ok && (sem == RB_WORKSHY_AND || sem == RB_FAST_XOR)) {
    // workShyAnd / naive_xor fast paths read packed records; naive_xor's key-major ones for a dense set
    // in set order are the set's cached krec
    // (a dense set's krec is built from its SoA when it has no mrec: naive_xor then never needs mrec)
    if (in->payload_bytes >= kRecMaxPayload) fast_ok = false;
    else if (sem == RB_FAST_XOR && dense && identity) fast_ok = !ensure_krec(in);
    else if (!(RBG_AND_SOA && sem == RB_WORKSHY_AND) && ensure_mrec(in)) fast_ok = false;
  }
  (void)hipGetLastError();

  stats_begin(ctx);
  // ---- group by key (stable; keys in [key_lo, key_hi) only): the tiled counting sort above.
  // RBGPU_GROUP_TILE="members,keys" shrinks the tiles so the tests cover many-tile layouts.
  uint32_t MB = kGrpMembers, KR = kGrpKeys;
  if (const char *e = getenv("RBGPU_GROUP_TILE")) {
    unsigned a = 0, b = 0;
    if (sscanf(e, "%u,%u", &a, &b) == 2) {
      MB = std::min<uint32_t>(std::max<uint32_t>(a, 1), kGrpMembers);
      KR = std::min<uint32_t>(std::max<uint32_t>(b, 1), kGrpKeys);
    }
  }
  const uint32_t krange = key_hi > key_lo ? key_hi - key_lo : 0;
  const uint32_t nmb = (M + MB - 1) / MB, nkr = (krange + KR - 1) / KR;
  const bool sorted = !dense && !horizontal; // the counting sort runs
  uint32_t *d_mem = nullptr, *d_cid2 = nullptr, *d_klist = nullptr, *d_Hc = nullptr;
  uint64_t *d_bnd = nullptr, *d_H = nullptr, *d_tot = nullptr, *d_seg = nullptr, *d_active = nullptr,
           *d_apos = nullptr, *d_tmp = nullptr, *d_mbase = nullptr;
  uint32_t *d_rec = nullptr;
  const uint64_t N1 = std::max<uint64_t>(N, 1);
  const uint64_t tmpw = std::max<uint64_t>(scan_tmp_words(65537), 1);
  auto alloc_if = [&](bool need, void **p, uint64_t bytes) { return need ? (bool)pool.alloc(p, bytes) : false; };
  if (pool.alloc((void **)&d_mem, std::max<uint32_t>(M, 1) * 4ull) ||
      alloc_if(sorted, (void **)&d_bnd, std::max<uint64_t>((uint64_t)M * (nkr + 1), 1) * 8) ||
      alloc_if(sorted, (void **)&d_Hc, std::max<uint64_t>((uint64_t)nmb * krange, 1) * 4) ||
      alloc_if(sorted, (void **)&d_H, std::max<uint64_t>((uint64_t)nmb * krange, 1) * 8) ||
      alloc_if(!dense, (void **)&d_cid2, N1 * 4) || alloc_if(dense, (void **)&d_mbase, std::max<uint32_t>(M, 1) * 8ull) ||
      pool.alloc((void **)&d_tot, 65537 * 8ull) || pool.alloc((void **)&d_seg, 65537 * 8ull) ||
      pool.alloc((void **)&d_active, 65537 * 8ull) || pool.alloc((void **)&d_apos, 65537 * 8ull) ||
      pool.alloc((void **)&d_klist, 65536 * 4ull) || pool.alloc((void **)&d_tmp, tmpw * 8))
    return fail(RB_ENOMEM, "wide workspace (%llu containers)", (unsigned long long)N);
  auto release = [&]() {
    for (void *p : {(void *)d_mem, (void *)d_bnd, (void *)d_Hc, (void *)d_H, (void *)d_cid2, (void *)d_tot,
                    (void *)d_seg, (void *)d_active, (void *)d_apos, (void *)d_klist, (void *)d_tmp, (void *)d_rec,
                    (void *)d_mbase})
      if (p) pool.release(p);
  };
  if (M) HIPCHK(hipMemcpyAsync(d_mem, members.data(), M * 4ull, hipMemcpyHostToDevice, st));
  const SetView sv = in->view();
  const GroupArgs ga{sv, d_mem, d_bnd, M, MB, KR, nkr, key_lo, key_hi};
  std::vector<uint32_t> h_cid;
  std::vector<uint64_t> h_seg;
  if (horizontal) {
    // the queue order of FastAggregation.horizontal_* over every member key (ties included), then the
    // per-key containers in that order; keys outside the shard are left to k_wide_select
    int rc = horizontal_order(in, members, h_cid, h_seg);
    if (rc) {
      release();
      return rc;
    }
    if (!h_cid.empty()) HIPCHK(hipMemcpyAsync(d_cid2, h_cid.data(), 4 * h_cid.size(), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_seg, h_seg.data(), 8 * 65537ull, hipMemcpyHostToDevice, st));
  } else if (dense) {
    k_group_dense<<<nblk(std::max<uint64_t>(M, 65537), 256), 256, 0, st>>>(sv.begin, d_mem, M, (uint32_t)in->dense_lo,
                                                                           key_lo, key_hi, d_seg, d_mbase);
  } else {
    if (M && nkr) {
      k_group_bounds<<<nblk((uint64_t)M * (nkr + 1), 256), 256, 0, st>>>(ga, d_bnd);
      k_group_count<<<dim3(nkr, nmb), 256, 0, st>>>(ga, d_Hc);
    }
    k_group_totals<<<nblk(65537, 256), 256, 0, st>>>(d_Hc, M && nkr ? nmb : 0, key_lo, key_hi, d_tot);
    scan_exclusive(d_tot, d_seg, 65536, d_tmp, st);
    if (M && nkr) {
      k_group_base<<<nblk(krange, 256), 256, 0, st>>>(d_Hc, d_H, nmb, key_lo, key_hi, d_seg);
      k_group_scatter<<<dim3(nkr, nmb), 256, 0, st>>>(ga, d_H, d_cid2);
    }
  }
  const CidMap cm{dense ? nullptr : d_cid2, d_mbase};
  {
    const uint64_t need = and_sem ? (uint64_t)M : 0;
    k_wide_select<<<256, 256, 0, st>>>(d_seg, need, key_lo, key_hi, d_active);
    const uint64_t *in1[1] = {d_active};
    uint64_t *out1[1] = {d_apos};
    scan_blocks_multi(in1, out1, 1, 256, nullptr, st);
    k_wide_list<<<256, 256, 0, st>>>(d_seg, need, key_lo, key_hi, d_apos, d_klist);
  }
  uint64_t *pin = ctx->h_pinned;
  HIPCHK(hipMemcpyAsync(pin, d_apos + 256, 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  LAUNCHCHK();
  const uint32_t nk = (and_sem && M == 0) ? 0 : (uint32_t)pin[0];

  // ---- per-key reduction into 8 KiB slots
  rbgpu_set *res = new rbgpu_set;
  int rc = set_alloc(ctx, res, 1, nk, (uint64_t)std::max<uint32_t>(nk, 1) * kBitmapBytes);
  if (rc) {
    delete res;
    release();
    return rc;
  }
  uint8_t *w_type;
  uint32_t *w_card;
  uint16_t *w_nruns;
  const uint64_t nk1 = std::max<uint32_t>(nk, 1);
  if (pool.alloc((void **)&w_type, nk1) || pool.alloc((void **)&w_card, nk1 * 4) ||
      pool.alloc((void **)&w_nruns, nk1 * 2)) {
    rbgpu_set_free(res);
    release();
    return fail(RB_ENOMEM, "wide result workspace");
  }
  WideOut wo{w_type, w_card, w_nruns};
  uint8_t *d_route = nullptr;
  if (pool.alloc((void **)&d_route, nk1)) d_route = nullptr;
  if (!d_route) fast_ok = false;
  // naive_xor's fast path reads key-major member records (wide_xor.hip)
  XorRecords xr{nullptr, N, XorRecords::kGather, in->mrec, d_mbase, M, key_lo, key_hi};
  if (nk && fast_ok && sem == RB_FAST_XOR) {
    if (dense && identity) {
      xr.rec = in->krec + (uint64_t)(key_lo - in->dense_lo) * in->nb;
      xr.build = XorRecords::kCached;
    } else {
      if (pool.alloc((void **)&d_rec, std::max<uint64_t>(N, 1) * 4)) fast_ok = false;
      xr.rec = d_rec;
      xr.build = dense ? XorRecords::kTranspose : XorRecords::kGather;
    }
  }
  HIPCHK(hipEventRecord(ctx->ev[1], st));
  if (nk) {
    // Run-heavy keys first (all Run containers with <= 8 runs): route[q] = 0 when done there
    if (fast_ok && !launch_wide_runs(sem, sv, in->mrec, cm, d_seg, d_klist, nk, res->payload, wo, d_route,
                                     ctx->d_stats, xr, st))
      fast_ok = false;
    const uint8_t *rt = fast_ok ? d_route : nullptr;
    switch (sem) {
    case RB_FAST_OR: launch_reduce<RB_FAST_OR>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st, rt); break;
    case RB_WORKSHY_AND: launch_reduce<RB_WORKSHY_AND>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st, rt); break;
    case RB_NAIVE_AND: launch_reduce<RB_NAIVE_AND>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st); break;
    case RB_NAIVE_AND_ITER: launch_reduce<RB_NAIVE_AND_ITER>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st); break;
    case RB_FAST_XOR: launch_reduce<RB_FAST_XOR>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st, rt); break;
    case RB_PAR_OR: launch_reduce<RB_PAR_OR>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st); break;
    case RB_BUFFER_NAIVE_OR: launch_reduce<RB_BUFFER_NAIVE_OR>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st); break;
    case RB_HORIZONTAL_OR: launch_reduce<RB_HORIZONTAL_OR>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st); break;
    case RB_HORIZONTAL_XOR: launch_reduce<RB_HORIZONTAL_XOR>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st); break;
    default: launch_reduce<RB_PAR_XOR>(sv, cm, d_seg, d_klist, nk, res->payload, wo, ctx->d_stats, st); break;
    }
  }
  HIPCHK(hipEventRecord(ctx->ev[2], st));
  // ---- compaction
  rc = compact_keyed(ctx, d_klist, nk, wo, res);
  if (rc) {
    rbgpu_set_free(res);
    release();
    return rc;
  }
  // the span covers the Run-list fast path (if any) and the generic kernel for the routed keys
  const bool fp = fast_ok;
  const char *name = sem == RB_FAST_OR ? "k_wide_reduce<FAST_OR>"
                     : sem == RB_WORKSHY_AND ? (fp ? "k_wide_runs_and+k_wide_reduce<WORKSHY_AND>" : "k_wide_reduce<WORKSHY_AND>")
                     : sem == RB_FAST_XOR ? (fp ? "k_wide_runs_xor+k_wide_reduce<FAST_XOR>" : "k_wide_reduce<FAST_XOR>")
                     : sem == RB_PAR_OR ? "k_wide_reduce<PAR_OR>"
                     : sem == RB_BUFFER_NAIVE_OR ? "k_wide_reduce<BUFFER_NAIVE_OR>"
                     : sem == RB_PAR_XOR ? "k_wide_reduce<PAR_XOR>"
                     : sem == RB_HORIZONTAL_OR ? "k_wide_reduce<HORIZONTAL_OR>"
                     : sem == RB_HORIZONTAL_XOR ? "k_wide_reduce<HORIZONTAL_XOR>" : "k_wide_reduce<NAIVE_AND>";
  const KernelSpan spans[1] = {{name, 0, 1, nk}};
  // ev[2] -> ev[3]: nothing; stats_end reads ev[1]..ev[2] for kernel 0
  rc = stats_end(ctx, N, 0, spans, 1);
  if (!rc) keyed_result_count(ctx, res);
  pool.release(w_type);
  pool.release(w_card);
  pool.release(w_nruns);
  pool.release(d_route);
  release();
  if (rc) {
    rbgpu_set_free(res);
    return rc;
  }
  *out = res;
  return RB_OK;
}

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_wide() {}
void warm_wide(hipStream_t st) { k_warm_wide<<<1, 64, 0, st>>>(); }

} // namespace rbg
