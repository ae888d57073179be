#include <algorithm>
// pairwise.hip — batched static RoaringBitmap.and/or/xor/andNot on MI355X.
//
// Pipeline (one HIP stream):
//   k_pair_count   thread per pair: merge the two sorted u16 key lists (RoaringBitmap.and/or/
//                  xor/andNot key loops, RoaringBitmap.java:377-473, 860-902, 1071-1118), count
//                  result slots per kernel category + an output-byte bound per slot;
//   scans          exclusive prefix sums -> record index and arena offset of every slot;
//   k_pair_emit    thread per pair: write self-contained task records (payload offsets,
//                  descriptors) in result order;
//   k_pair_tasks   persistent, ONE WAVE PER TASK, software-pipelined: unmatched copies, results
//                  that are a subset of an Array operand (filter against an 8 KiB LDS membership
//                  image), and everything else as 65536-bit register bitmaps (word op, card +
//                  maximal runs, reference type decision, coalesced emission);
//   k_compact_*    drop empty results (isEmpty, RoaringBitmap.java:389-391 etc.) and build the
//                  result CSR.
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

constexpr int kPairThreads = 256;

#ifndef RBG_SMALL_STUDY
#define RBG_SMALL_STUDY 0 // study builds: per-block phase times (s_memrealtime) into g_small_study (rbgpu_internal_small_study)
#endif
#if RBG_SMALL_STUDY
constexpr int kStudyWords = 32; // per block: t0, align, 4 wave ends, 4 key counts, done, compact end, pair, sub, nu, last;
                                // 16 + 4 w: wave w's slowest key (ticks, result | operand types, operand cards, merge phases)
__device__ uint64_t g_small_study[8192 * kStudyWords];
__device__ uint64_t g_merge_ts[8192 * 4][8]; // per wave: merge_run's phase stamps of its last merge
#define RBG_MT(i) if (lane == 0) g_merge_ts[min(blockIdx.x, 8191u) * 4 + (threadIdx.x >> 6)][i] = __builtin_amdgcn_s_memrealtime()
#else
#define RBG_MT(i)
#endif

__device__ __forceinline__ bool keeps_a_only(int op) { return op != RB_AND; }
__device__ __forceinline__ bool keeps_b_only(int op) { return op == RB_OR || op == RB_XOR || is_lazy_op(op); }

// algorithmic payload bytes: Bitmap 8192, Array 2c, Run 4r+2
__device__ __forceinline__ uint64_t alg_bytes(int t, uint32_t c, uint32_t r) {
  return t == kBitmap ? 8192ull : t == kArray ? 2ull * c : 4ull * r + 2;
}

// Upper bound of the result payload of a matched pair: every reference result type fits in
// 2*cmax bytes when cmax <= 4096 (Array 2c; a Run is only chosen when 4r+2 <= 2c+2), and in
// one 8 KiB slot otherwise.
__device__ __forceinline__ void matched_bound(int op, uint32_t ca, uint32_t cb, bool &big, uint64_t &bytes) {
  if (is_lazy_op(op)) { // lazy results (a lazy Bitmap of two small Arrays, a Run of any run count) take 8 KiB
    big = true;
    bytes = 0;
    return;
  }
  uint32_t cmax = op == RB_AND ? min(ca, cb) : op == RB_ANDNOT ? ca : ca + cb;
  big = 2ull * cmax >= (uint64_t)kBitmapBytes;
  bytes = big ? 0 : round16(2ull * cmax);
}
__device__ __forceinline__ void copy_bound_v(int t, uint32_t card, uint32_t nruns, bool &big, uint64_t &bytes) {
  big = t == kBitmap;
  bytes = big ? 0 : round16(payload_bytes(t, card, nruns));
}
__device__ __forceinline__ void copy_bound(const SetView &S, uint64_t i, bool &big, uint64_t &bytes) {
  copy_bound_v(S.type[i], S.card[i], S.nruns[i], big, bytes);
}

// pair_walk writes a TaskRec as five 8-B words: pa, pb, out, t | da << 32, db | ra << 32 | rb << 48
static_assert(sizeof(TaskRec) == 40 && offsetof(TaskRec, out) == 16 && offsetof(TaskRec, t) == 24 &&
                  offsetof(TaskRec, da) == 28 && offsetof(TaskRec, db) == 32 && offsetof(TaskRec, ra) == 36 &&
                  offsetof(TaskRec, rb) == 38,
              "TaskRec layout");

// One container's key and metadata held in registers by the short-segment walk (pair_walk).
constexpr int kWalkRegs = 4; // containers per side a short segment holds
struct WalkMeta {
  uint32_t kt, card, nr; // kt: key | type << 16
  uint64_t off;
  __device__ uint16_t key() const { return (uint16_t)(kt & 0xFFFFu); }
  __device__ int type() const { return (int)(kt >> 16); }
};
template <bool WITH_OFF>
__device__ __forceinline__ WalkMeta walk_meta(const SetView &S, uint64_t i) {
  WalkMeta m;
  m.kt = (uint32_t)S.key[i] | ((uint32_t)S.type[i] << 16);
  m.card = S.card[i];
  m.nr = S.nruns[i];
  m.off = WITH_OFF ? S.off[i] : 0;
  return m;
}
// m[x] for a per-thread x as selects (a dynamically indexed private array would go to scratch)
__device__ __forceinline__ WalkMeta pick_meta(const WalkMeta (&m)[kWalkRegs], uint32_t x) {
  WalkMeta r = m[0];
#pragma unroll
  for (int k = 1; k < kWalkRegs; ++k) {
    const bool s = x == (uint32_t)k;
    r.kt = s ? m[k].kt : r.kt;
    r.card = s ? m[k].card : r.card;
    r.nr = s ? m[k].nr : r.nr;
    r.off = s ? m[k].off : r.off;
  }
  return r;
}

// Array ⊙ Array as a merge (ArrayContainer.and / or / xor / andNot of two Arrays, ArrayContainer.java:
// 184-227, 949-973, 1311-1336, 243-271): both sorted arrays in the wave's 8 KiB LDS scratch and a merge
// path over them instead of two 65536-bit register images.  Lane l walks the merged positions
// [l n / 64, (l + 1) n / 64) of A and B (A first on equal values: a value in both arrays is the pair
// A[i], B[j] next to each other, wherever the lanes' ranges split), once to count the values it keeps
// and once, after a wave scan of the counts, to store them.  With ca + cb <= kMergeMax the result is an
// Array (ArrayContainer.or / xor merge below DEFAULT_MAX_SIZE; and / andNot are subsets of A), the type
// the register path gives these pairs.  Used by the small-batch kernel (k_pair_small).
#ifndef RBG_SMALL_MERGE
#define RBG_SMALL_MERGE 1 // study builds: 0 sends small-batch Array pairs through the register path
#endif
constexpr uint32_t kMergeMax = 4088; // ca + cb: A at 0, B 16-B aligned after it, both in 8 KiB
template <int OP>
__device__ __forceinline__ bool merge_keep(bool from_a, bool matched) {
  if (OP == RB_AND) return from_a && matched;
  if (OP == RB_ANDNOT) return from_a && !matched;
  if (OP == RB_OR) return from_a || !matched;
  return !matched; // XOR
}
// One lane's walk, branch-free (a divergent if / else ran both arms and paid two LDS latencies per
// step): one LDS read per step, the next value of the side just taken.  A and B are one u16 array in LDS
// (B at boff).  Kept values go to out[0..) (STORE), or with STAGE to the lane's own LDS range stage[0..)
// — a single walk, copied out afterwards.  (Holding each side's next value one step ahead gained nothing:
// the compiler waits for the read at the top of the next step either way.)
template <int OP, bool STORE, bool STAGE>
__device__ __forceinline__ uint32_t merge_walk(uint16_t *S, uint32_t ca, uint32_t boff, uint32_t cb, uint32_t i,
                                               uint32_t j, uint32_t steps, uint16_t *out, uint16_t *stage) {
  constexpr uint32_t kEnd = 0x10000u; // past every u16 value
  auto rd = [&](bool valid, uint32_t idx) { // the read unconditional (clamped), the value selected
    const uint32_t x = S[min(idx, 4095u)];
    return valid ? x : kEnd;
  };
  uint32_t av = rd(i < ca, i), bv = rd(j < cb, boff + j);
  uint32_t prev_a = i ? S[i - 1] : kEnd + 1; // the last A value before this position
  uint32_t cnt = 0;
  for (uint32_t d = 0; d < steps; ++d) {
    const bool ta = av <= bv; // A's value (both kEnd is impossible: the walk stays below ca + cb)
    const uint32_t v = ta ? av : bv;
    const bool keep = merge_keep<OP>(ta, ta ? av == bv : prev_a == bv);
    if (STAGE && keep) stage[cnt] = (uint16_t)v;
    else if (STORE && keep) out[cnt] = (uint16_t)v;
    cnt += keep;
    prev_a = ta ? av : prev_a;
    i += ta;
    j += !ta;
    const uint32_t nx = rd(ta ? i < ca : j < cb, ta ? i : boff + j);
    av = ta ? nx : av;
    bv = ta ? bv : nx;
  }
  return cnt;
}
__device__ __forceinline__ uint32_t merge_boff(uint32_t ca) { return (ca + 7u) & ~7u; } // B's first value (u16)
// the two preloaded payloads (register chunks of ca / cb sorted u16 values) as A and B in the scratch
__device__ __forceinline__ void merge_stage(const uint4 (&q)[8], uint32_t ca, const uint4 (&r)[8], uint32_t cb,
                                            uint32_t *s, int lane) {
  uint4 *s4 = reinterpret_cast<uint4 *>(s);
  const uint32_t na4 = (2u * ca + 15u) >> 4, nb4 = (2u * cb + 15u) >> 4, b4 = merge_boff(ca) >> 3;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t c = (uint32_t)lane + 64u * k;
    if (c < na4) s4[c] = q[k];
    if (c < nb4) s4[b4 + c] = r[k];
  }
  wave_lds_sync();
}
// A result made of the small side's values only — AND with one side of <= 64 values, ANDNOT with A of
// <= 64 values and B larger: each small-side value's membership in the other side by a binary search (all
// lanes at once, a value per lane) and one ballot ranking the kept values; no merged walk.  (Closed-form
// placement for OR / XOR / ANDNOT with B small — the large side's values moved by offsets, each lane over
// its slice — measured slower than the staged walk on census, 41 vs 39 µs per OR call, its per-value 2-B
// stores; AND 32.2 → 31.0 µs: profiles/r05/merge/small_side_ab.txt.)
// A merge's result count goes to `pub` before its first payload store (k_pair_small publishes the slot word there, so
// the word is not queued behind the payload stores: NoPub elsewhere).
struct NoPub {
  __device__ void operator()(uint32_t) const {}
};
template <int OP, bool STORE, class Pub = NoPub>
__device__ __forceinline__ uint32_t merge_small_side(const uint16_t *A, uint32_t ca, const uint16_t *B, uint32_t cb,
                                                     uint16_t *out, int lane, const Pub &pub = Pub()) {
  constexpr uint32_t kEnd = 0x10000u;
  const bool s_is_b = OP == RB_AND && cb <= ca; // the small side S (AND: either; ANDNOT: A)
  const uint16_t *L = s_is_b ? A : B, *S = s_is_b ? B : A;
  const uint32_t cl = s_is_b ? ca : cb, cs = s_is_b ? cb : ca;
  const bool live = (uint32_t)lane < cs;
  const uint32_t sv = live ? S[lane] : kEnd;
  uint32_t lo = 0, hi = live ? cl : 0u;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (L[mid] < sv) lo = mid + 1;
    else hi = mid;
  }
  const uint32_t at = cl ? L[min(lo, cl - 1u)] : kEnd;
  const bool m = live && lo < cl && at == sv;
  const bool kept = OP == RB_AND ? m : live && !m;
  const uint64_t bk = __ballot(kept);
  pub((uint32_t)__popcll(bk));
  if (STORE && kept) out[mbcnt64(bk)] = (uint16_t)sv;
  return (uint32_t)__popcll(bk);
}
// OR / XOR of two Arrays, or ANDNOT with B small, when one side S has <= 64 values and the other L many (census:
// the slowest keys of the small-batch kernel are ~2000 | <= 40 values — a 30-step merged walk, its scan and its
// stage copy, profiles/r06/small).  Each S value finds its place in L (one binary search per lane); then, in the
// merged order without deletions M (L's values and the inserted S values), a bit marks each inserted S value (INS)
// and each deleted L value (DEL: XOR / ANDNOT drop L's values equal to an S value; OR drops nothing and inserts
// only the unmatched S values).  One sweep over M, 64 positions a step: an L item is L[j - inserted before it], an
// S item the next inserted value, and each kept item goes to j - deleted before it.  The steps depend on nothing
// but two running counts, so their LDS reads pipeline.  Returns the result count; kLopsidedNo when the bitmaps
// do not fit beside the staged arrays (the caller walks).
constexpr uint32_t kLopsidedNo = 0xFFFFFFFFu;
#ifndef RBG_LOPSIDED
#define RBG_LOPSIDED 1 // lopsided pairs off the walk, counted before the store sweep (0: the walk; profiles/r06/small/early)
#endif
template <int OP, bool STORE, class Pub = NoPub>
__device__ __forceinline__ uint32_t merge_lopsided(uint16_t *A, uint32_t ca, uint32_t boff, uint32_t cb, uint16_t *out,
                                                   int lane, const Pub &pub = Pub()) {
  const bool s_is_b = OP == RB_ANDNOT || cb <= ca; // ANDNOT: the caller sends B small
  const uint16_t *L = s_is_b ? A : A + boff, *S = s_is_b ? A + boff : A;
  const uint32_t cl = s_is_b ? ca : cb, cs = s_is_b ? cb : ca;
  const uint32_t sbase = (boff + cb + 7u) & ~7u;         // u16 index past the staged arrays, 16-B aligned
  const uint32_t nwin = (cl + cs + 63u) >> 6, nw = 2u * nwin; // 64-position windows of M, two u32 words each
  if (sbase + 4u * nw + 64u > 4096u) return kLopsidedNo;
  uint32_t *INS = reinterpret_cast<uint32_t *>(A + sbase), *DEL = INS + nw;
  uint16_t *SL = reinterpret_cast<uint16_t *>(DEL + nw); // the inserted S values in order
  for (uint32_t w = (uint32_t)lane; w < 2u * nw; w += 64u) INS[w] = 0u;
  // S value of this lane: its place in L (lower bound) and whether L holds it
  const bool live = (uint32_t)lane < cs;
  const uint32_t sv = live ? S[lane] : 0x10000u;
  uint32_t lo = 0, hi = live ? cl : 0u;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (L[mid] < sv) lo = mid + 1;
    else hi = mid;
  }
  const bool matched = live && lo < cl && L[min(lo, cl - 1u)] == sv;
  const bool ins = live && !matched && OP != RB_ANDNOT;
  const bool del = matched && OP != RB_OR;
  const uint64_t im = __ballot(ins), dm = __ballot(del);
  const uint32_t ri = mbcnt64(im);
  wave_lds_sync(); // the bitmaps are zero
  // positions in M: an inserted S value at lb + (inserted before it); a matched L value at lb + (inserted before
  // it) — inserted S values below a matched one are exactly the lanes below it
  const uint32_t pm = lo + ri;
  if (ins) {
    atomicOr(&INS[pm >> 5], 1u << (pm & 31));
    SL[ri] = (uint16_t)sv;
  }
  if (del) atomicOr(&DEL[pm >> 5], 1u << (pm & 31));
  wave_lds_sync();
  const uint32_t M = cl + (uint32_t)__popcll(im), kept = M - (uint32_t)__popcll(dm);
  pub(kept); // the count is known before the sweep
  if (STORE && kept) {
    const uint64_t below = (1ull << lane) - 1ull; // lane 0: 0
    uint32_t insb = 0, delb = 0;                   // inserted / deleted items before the window
#pragma unroll 4
    for (uint32_t k = 0; k < nwin; ++k) {
      const uint64_t iw = pack2(INS[2 * k], INS[2 * k + 1]), dw = pack2(DEL[2 * k], DEL[2 * k + 1]);
      const uint32_t j = 64u * k + (uint32_t)lane;
      const bool is_s = (iw >> lane) & 1ull, is_d = (dw >> lane) & 1ull;
      const uint32_t r = insb + (uint32_t)__popcll(iw & below);
      const uint32_t v = is_s ? SL[min(r, 63u)] : L[min(j - r, cl - 1u)];
      if (j < M && !is_d) out[j - delb - (uint32_t)__popcll(dw & below)] = (uint16_t)v;
      insb += (uint32_t)__popcll(iw);
      delb += (uint32_t)__popcll(dw);
    }
  }
  wave_lds_sync(); // the next task restages the scratch
  return kept;
}
template <int OP, bool STORE, class Pub = NoPub>
__device__ __forceinline__ uint32_t merge_run(uint32_t *s, uint32_t ca, uint32_t cb, uint16_t *out, int lane,
                                              const Pub &pub = Pub()) {
  uint16_t *A = reinterpret_cast<uint16_t *>(s);
  const uint32_t boff = merge_boff(ca), n = ca + cb;
  const uint16_t *B = A + boff;
  // a result of the small side's values only: one ballot (merge_small_side)
  if ((OP == RB_AND && min(ca, cb) <= 64u) || (OP == RB_ANDNOT && ca <= 64u && cb > 64u)) {
    const uint32_t tot = merge_small_side<OP, STORE>(A, ca, B, cb, out, lane, pub);
    wave_lds_sync(); // the next task restages the scratch
    return tot;
  }
  // one side of <= 64 values into the other: insertions / deletions (merge_lopsided)
  if (RBG_LOPSIDED && (((OP == RB_OR || OP == RB_XOR) && min(ca, cb) <= 64u) || (OP == RB_ANDNOT && cb <= 64u))) {
    const uint32_t tot = merge_lopsided<OP, STORE>(A, ca, boff, cb, out, lane, pub);
    if (tot != kLopsidedNo) return tot;
  }
  RBG_MT(0);
  const uint32_t d0 = ((uint32_t)lane * n) >> 6, d1 = ((uint32_t)(lane + 1) * n) >> 6;
  // merge path: the number of A values among the first d0 merged values (A first on ties)
  uint32_t lo = d0 > cb ? d0 - cb : 0u, hi = min(d0, ca);
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (A[mid] <= B[d0 - mid - 1]) lo = mid + 1;
    else hi = mid;
  }
  // one walk into a per-lane LDS stage (lane l's at sbase + d0, its merged range) when it fits beside A
  // and B, else a counting walk and a storing walk
  const uint32_t sbase = (boff + cb + 7u) & ~7u;
  const bool staged = STORE && sbase + n <= 4096u; // wave-uniform
  RBG_MT(1);
  uint32_t cnt;
  if (staged) cnt = merge_walk<OP, false, true>(A, ca, boff, cb, lo, d0 - lo, d1 - d0, nullptr, A + sbase + d0);
  else cnt = merge_walk<OP, false, false>(A, ca, boff, cb, lo, d0 - lo, d1 - d0, nullptr, nullptr);
  RBG_MT(2);
  const uint32_t incl = wave_scan_u32(cnt, lane), tot = readlane(incl, 63);
  pub(tot);
  if (STORE && tot) { // out: a 16-B aligned slot
    uint16_t *o = out + (incl - cnt);
    if (staged) { // compacted in LDS over A (every lane is past its walk), then whole 16-B stores
      const uint16_t *st = A + sbase + d0;
      // eight reads, then eight writes: one value at a time, each write waited for the read before it (the
      // compiler cannot tell the stage from the output), ~2 LDS latencies per kept value — 4 us of an OR call's
      // slowest key (census: 2057 | 2 values, profiles/r06/small)
      uint16_t *o16 = A + (incl - cnt);
      for (uint32_t k = 0; k < cnt; k += 8) {
        uint16_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = st[min(k + (uint32_t)u, 4095u - (sbase + d0))];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (k + (uint32_t)u < cnt) o16[k + u] = v[u];
      }
      wave_lds_sync();
      RBG_MT(3);
      const uint4 *a4 = reinterpret_cast<const uint4 *>(A);
      uint4 *o4 = reinterpret_cast<uint4 *>(out);
      for (uint32_t c = (uint32_t)lane; 16u * c < 2u * tot; c += 64u) o4[c] = a4[c];
      RBG_MT(4);
    } else {
      merge_walk<OP, true, false>(A, ca, boff, cb, lo, d0 - lo, d1 - d0, o, nullptr);
    }
  }
  wave_lds_sync(); // the next task restages the scratch
  return tot;
}

// A task is "light" when its result is a subset of one Array operand (AND with an Array, ANDNOT
// with an Array on the left) or when it is an unmatched copy; everything else is "heavy".
// (OR / XOR of two Arrays through merge_run in the light (copy + filter) kernel instead of the heavy
// register path measured slower:
// config 2 OR 12.84 -> 14.09 ms, XOR 10.59 -> 12.85 — the light kernel, already the L2-bound one, became
// the long pole; an LDS-image form of the same tasks 15.8 / 14.2 ms.  profiles/r05/merge.)
__device__ __forceinline__ bool light_task(int op, int ta, int tb) {
  if (ta < 0 || tb < 0) return true;
  if (op == RB_AND) return ta == kArray || tb == kArray;
  if (op == RB_ANDNOT) return ta == kArray;
  return false;
}
// Round 6: an OR with a Bitmap operand of more than 4096 values (canonical, no lazy marks) holds all of that
// operand's values, so its LR type (BitmapContainer.or(Array / Bitmap / Run), BitmapContainer.java:1073-1110;
// RunContainer.or(Bitmap)) is known before the OR: a Bitmap, or the full Run when c = 65536 (and a Bitmap even
// then for BitmapContainer.ior(ArrayContainer), :749-766).  Such a task needs no register image and no
// emission loops: the copy + filter kernel ORs the staged other operand into it row by row (kBits), at that
// kernel's occupancy.  Only the plain OR: the lazy roles keep the register path's lazy types.
#ifndef RBG_OR_BITS
#define RBG_OR_BITS 0 // study builds: 1 sends them to the copy + filter kernel (slower: config 2 OR 13.12 vs 12.36 ms)
#endif
__device__ __forceinline__ bool big_bitmap(int t, uint32_t c) {
  return t == kBitmap && !(c & kCardMarks) && c > (uint32_t)kMaxArray;
}
__device__ __forceinline__ bool bits_task(int op, int ta, uint32_t ca, int tb, uint32_t cb) {
  return RBG_OR_BITS && op == RB_OR && (uint32_t)ta <= 2u && (uint32_t)tb <= 2u &&
         (big_bitmap(ta, ca) || big_bitmap(tb, cb));
}

// Striped accounting (stats word w, stripe = block mod kStripes) of N counters: one atomic per block
// and counter, by a thread of the block after an LDS reduction (every thread of the block must call
// it).  An atomic per wave and counter made ~16k atomics per launch of the 1M-pair kernels on 16 cache lines (k_pair_count
// 69 vs 51 us without them).
template <int N>
__device__ __forceinline__ void stat_add_block(uint64_t *stats, const int (&word)[N], const uint64_t (&v)[N]) {
  static_assert(N <= kPairThreads / 64, "one wave per counter");
  __shared__ uint64_t part[kPairThreads / 64][N];
  const int lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint64_t s = wave_sum_u64(v[k]);
    if (lane == 0) part[w][k] = s;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k)
    if (threadIdx.x == 64 * k) { // one lane of a different wave per counter
      uint64_t s = 0;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += part[i][k];
      if (s) atomicAdd((unsigned long long *)&stats[word[k] * kStripes + (blockIdx.x & (kStripes - 1))],
                       (unsigned long long)s);
    }
}

// Sums over the block (kPairThreads threads) of N per-thread values; every thread gets all N.
template <int N>
__device__ __forceinline__ void block_sums(const uint64_t (&v)[N], uint64_t (&sums)[N]) {
  __shared__ uint64_t part[kPairThreads / 64][N];
  const int lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint64_t s = wave_sum_u64(v[k]);
    if (lane == 0) part[w][k] = s;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; ++k) {
    uint64_t s = 0;
    for (int i = 0; i < kPairThreads / 64; ++i) s += part[i][k];
    sums[k] = s;
  }
  __syncthreads();
}


// ---------------------------------------------------------------- key alignment by merge path
// A pair is cut into segments of <= a.seg_keys merged keys (merge path over the two sorted key lists,
// A first on equal keys), one thread per segment, so a pair of large bitmaps aligns its keys in
// parallel.  A matched key is never split: when a cut falls between A's key and its equal B
// partner, the partner stays with A.  The walk is a chain of dependent loads, so the host picks
// shorter segments when a batch has few keys (pairwise_seg_keys) to keep enough threads walking.

__device__ __forceinline__ void pair_ranges(const PairArgs &a, uint32_t p, uint64_t &i0, uint64_t &na, uint64_t &j0,
                                            uint64_t &nb, bool *ident = nullptr) {
  const uint32_t ai = a.aidx ? a.aidx[p] : p, bi = a.bidx ? a.bidx[p] : p;
  if (ident) *ident = a.inplace && a.same && ai == bi && ai != kEmptyBitmap; // x1.op(x1) in place
  i0 = ai == kEmptyBitmap ? 0 : a.A.begin[ai];
  na = ai == kEmptyBitmap ? 0 : a.A.begin[ai + 1] - i0;
  j0 = bi == kEmptyBitmap ? 0 : a.B.begin[bi];
  nb = bi == kEmptyBitmap ? 0 : a.B.begin[bi + 1] - j0;
}
// position after d merged keys -> (i, j) offsets into A and B
__device__ __forceinline__ void merge_split(const uint16_t *ka, uint64_t na, const uint16_t *kb, uint64_t nb,
                                            uint64_t d, uint64_t &i, uint64_t &j) {
  uint64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (ka[mid] <= kb[d - mid - 1]) lo = mid + 1;
    else hi = mid;
  }
  i = lo;
  j = d - lo;
  if (i > 0 && j < nb && ka[i - 1] == kb[j]) ++j;
}
__global__ __launch_bounds__(kPairThreads) void k_seg_count(PairArgs a, uint64_t *nseg) {
  const uint32_t p = blockIdx.x * kPairThreads + threadIdx.x;
  if (p >= a.npairs) return;
  uint64_t i0, na, j0, nb;
  pair_ranges(a, p, i0, na, j0, nb);
  nseg[p] = (na + nb + a.seg_keys - 1) / a.seg_keys + (na + nb == 0);
}
__global__ __launch_bounds__(kPairThreads) void k_seg_fill(PairArgs a, const uint64_t *seg_begin, uint32_t *seg_pair) {
  const uint32_t p = blockIdx.x * kPairThreads + threadIdx.x;
  if (p >= a.npairs) return;
  for (uint64_t s = seg_begin[p]; s < seg_begin[p + 1]; ++s) seg_pair[s] = p;
}

// largest begin[i+1] - begin[i] (containers of one bitmap), atomicMax into *out (zeroed)
__global__ __launch_bounds__(kPairThreads) void k_max_span(const uint64_t *begin, uint32_t nb, uint64_t *out) {
  uint64_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kPairThreads + threadIdx.x; i < nb; i += (uint64_t)gridDim.x * kPairThreads)
    m = max(m, begin[i + 1] - begin[i]);
  for (int d = 32; d; d >>= 1) m = max(m, (uint64_t)__shfl_xor((unsigned long long)m, d));
  if ((threadIdx.x & 63) == 0 && m) atomicMax((unsigned long long *)out, (unsigned long long)m);
}

// largest run count of the Run containers, atomicMax into *out (zeroed)
__global__ __launch_bounds__(kPairThreads) void k_max_runs(const uint8_t *type, const uint16_t *nruns, uint64_t n,
                                                          uint64_t *out) {
  uint32_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * kPairThreads + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kPairThreads)
    if (type[i] == kRun) m = max(m, (uint32_t)nruns[i]);
  m = wave_max_u32(m);
  if ((threadIdx.x & 63) == 0 && m) atomicMax((unsigned long long *)out, (unsigned long long)m);
}
void launch_max_runs(const uint8_t *type, const uint16_t *nruns, uint64_t n, uint64_t *out, hipStream_t st) {
  if (!n) return;
  const unsigned blocks = (unsigned)std::min<uint64_t>((n + kPairThreads - 1) / kPairThreads, 1024);
  k_max_runs<<<blocks, kPairThreads, 0, st>>>(type, nruns, n, out);
}

// inb[0]: key bytes, inb[1]: light-task input bytes, inb[2]: heavy-task input bytes
// sl / sh (EMIT): when non-null, the records go to this block's LDS stage instead (light record x at
// sl[x - l0], heavy at sh[x - h0]) and the block stores them contiguously afterwards
template <bool EMIT>
__device__ __forceinline__ void pair_walk(const PairArgs &a, uint64_t sg, PairCounts &n, uint64_t (&inb)[3],
                                          const PairBases &base, TaskRec *light, TaskRec *heavy, TaskMeta tm,
                                          TaskRec *sl = nullptr, TaskRec *sh = nullptr, uint64_t l0 = 0,
                                          uint64_t h0 = 0, uint64_t t0 = 0) {
  const uint32_t p = a.seg_pair ? a.seg_pair[sg] : (uint32_t)sg; // no map: segment sg is pair sg, whole
  uint64_t i0, na, j0, nb;
  bool ident;
  pair_ranges(a, p, i0, na, j0, nb, &ident);
  const uint64_t d0 = a.seg_pair ? (sg - a.seg_begin[p]) * a.seg_keys : 0, d1 = d0 + a.seg_keys < na + nb ? d0 + a.seg_keys : na + nb;
  uint64_t si0, sj0, si1, sj1;
  merge_split(a.A.key + i0, na, a.B.key + j0, nb, d0, si0, sj0);
  merge_split(a.A.key + i0, na, a.B.key + j0, nb, d1, si1, sj1);
  uint64_t i = i0 + si0, i1 = i0 + si1, j = j0 + sj0, j1 = j0 + sj1;
  inb[0] += 2 * ((i1 - i) + (j1 - j));
  // one result slot from the two sides' container metadata (ta / tb < 0: no container on that side)
  auto slot_v = [&](int ta, uint32_t ca, uint32_t ra, uint64_t oa, int tb, uint32_t cb, uint32_t rb, uint64_t ob,
                    uint16_t key, bool big, uint64_t bytes) {
    const bool lt = light_task(a.op, ta, tb) || bits_task(a.op, ta, ca, tb, cb);
    if (!EMIT) {
      uint64_t b = 0;
      if (ta >= 0) b += alg_bytes(ta, ca, ra) + 16;
      if (tb >= 0) b += alg_bytes(tb, cb, rb) + 16;
      if (lt) inb[1] += b;
      else inb[2] += b;
    } else {
      const uint64_t t = base.task + n.task;
      const uint64_t out = big ? (base.big + n.big) * (uint64_t)kBitmapBytes : base.small + n.small;
      const uint32_t da = ta >= 0 ? ((uint32_t)ta | (ca << 2)) : kAbsent;
      const uint32_t db = tb >= 0 ? ((uint32_t)tb | (cb << 2)) : kAbsent;
      const uint32_t rr = (ta >= 0 ? ra & 0xFFFFu : 0u) | ((tb >= 0 ? rb & 0xFFFFu : 0u) << 16);
      // the record as its five 8-B words (a TaskRec value copied as an aggregate went through scratch)
      TaskRec *dr;
      if (lt) {
        const uint64_t x = base.light + n.light;
        dr = sl ? sl + (x - l0) : light + x;
      } else {
        const uint64_t x = base.heavy + n.heavy;
        dr = sh ? sh + (x - h0) : heavy + x;
      }
      uint64_t *d = reinterpret_cast<uint64_t *>(dr);
      d[0] = ta >= 0 ? oa : 0;
      d[1] = tb >= 0 ? ob : 0;
      d[2] = out;
      d[3] = (uint64_t)(uint32_t)t | ((uint64_t)da << 32);
      d[4] = (uint64_t)db | ((uint64_t)rr << 32);
      // staged: tm holds the block's LDS arrays, indexed from the block's first task t0
      tm.slot[t - t0] = task_slot(out, key, !lt);
    }
    // branch-free: an `if` between two fields became a select of their addresses, which kept n in scratch
    ++n.task;
    n.light += lt ? 1 : 0;
    n.heavy += lt ? 0 : 1;
    n.big += big ? 1 : 0;
    n.small += big ? 0 : bytes;
  };
  bool big;
  uint64_t bytes;
  const uint64_t sa = i1 - i, sb = j1 - j;
  if (sa <= kWalkRegs && sb <= kWalkRegs && a.a_nc && a.b_nc) {
    // a short segment (config 2: every pair): all its keys and metadata in one round of independent
    // loads, then the merge over registers — the walk below is a chain of dependent loads per key
    WalkMeta ma4[kWalkRegs], mb4[kWalkRegs];
#pragma unroll
    for (int x = 0; x < kWalkRegs; ++x) {
      ma4[x] = walk_meta<EMIT>(a.A, sa ? i + min<uint64_t>(x, sa - 1) : min<uint64_t>(i, a.a_nc - 1));
      mb4[x] = walk_meta<EMIT>(a.B, sb ? j + min<uint64_t>(x, sb - 1) : min<uint64_t>(j, a.b_nc - 1));
    }
    auto take_a = [&](const WalkMeta &m) {
      copy_bound_v(m.type(), m.card, m.nr, big, bytes);
      slot_v(m.type(), m.card, m.nr, m.off, -1, 0u, 0u, 0ull, m.key(), big, bytes);
    };
    auto take_b = [&](const WalkMeta &m) {
      copy_bound_v(m.type(), m.card, m.nr, big, bytes);
      slot_v(-1, 0u, 0u, 0ull, m.type(), m.card, m.nr, m.off, m.key(), big, bytes);
    };
    uint32_t x = 0, y = 0;
    while (x < sa && y < sb) {
      const WalkMeta ma = pick_meta(ma4, x), mb = pick_meta(mb4, y);
      if (ma.key() == mb.key()) {
        if (!ident) {
          matched_bound(a.op, ma.card, mb.card, big, bytes);
          slot_v(ma.type(), ma.card, ma.nr, ma.off, mb.type(), mb.card, mb.nr, mb.off, ma.key(), big, bytes);
        } else if (a.op == RB_AND || a.op == RB_OR) {
          take_a(ma);
        }
        ++x;
        ++y;
      } else if (ma.key() < mb.key()) {
        if (keeps_a_only(a.op)) take_a(ma);
        ++x;
      } else {
        if (keeps_b_only(a.op)) take_b(mb);
        ++y;
      }
    }
    if (keeps_a_only(a.op))
      for (; x < sa; ++x) take_a(pick_meta(ma4, x));
    if (keeps_b_only(a.op))
      for (; y < sb; ++y) take_b(pick_meta(mb4, y));
    return;
  }
  // the general walk: a container's metadata is loaded only when it takes a slot
  auto slot = [&](int64_t ia, int64_t ib, uint16_t key, bool big, uint64_t bytes) {
    slot_v(ia >= 0 ? (int)a.A.type[ia] : -1, ia >= 0 ? a.A.card[ia] : 0u, ia >= 0 ? a.A.nruns[ia] : 0u,
           EMIT && ia >= 0 ? a.A.off[ia] : 0ull, ib >= 0 ? (int)a.B.type[ib] : -1, ib >= 0 ? a.B.card[ib] : 0u,
           ib >= 0 ? a.B.nruns[ib] : 0u, EMIT && ib >= 0 ? a.B.off[ib] : 0ull, key, big, bytes);
  };
  while (i < i1 && j < j1) {
    uint16_t ka = a.A.key[i], kb = a.B.key[j];
    if (ka == kb) {
      if (!ident) {
        matched_bound(a.op, a.A.card[i], a.B.card[j], big, bytes);
        slot((int64_t)i, (int64_t)j, ka, big, bytes);
      } else if (a.op == RB_AND || a.op == RB_OR) { // x.and(x) / x.or(x): x unchanged (its own containers)
        copy_bound(a.A, i, big, bytes);
        slot((int64_t)i, -1, ka, big, bytes);
      } // x.xor(x) / x.andNot(x): cleared
      ++i;
      ++j;
    } else if (ka < kb) {
      if (keeps_a_only(a.op)) {
        copy_bound(a.A, i, big, bytes);
        slot((int64_t)i, -1, ka, big, bytes);
      }
      ++i;
    } else {
      if (keeps_b_only(a.op)) {
        copy_bound(a.B, j, big, bytes);
        slot(-1, (int64_t)j, kb, big, bytes);
      }
      ++j;
    }
  }
  if (keeps_a_only(a.op))
    for (; i < i1; ++i) {
      copy_bound(a.A, i, big, bytes);
      slot((int64_t)i, -1, a.A.key[i], big, bytes);
    }
  if (keeps_b_only(a.op))
    for (; j < j1; ++j) {
      copy_bound(a.B, j, big, bytes);
      slot(-1, (int64_t)j, a.B.key[j], big, bytes);
    }
}

// A segment's four counts in one word: tasks, light tasks and big slots (12 bits each: a segment holds
// <= kMaxSegKeys + 1 tasks) and small-slot bytes (28 bits: < 8 KiB per small slot).
static_assert(kMaxSegKeys < 4095 && (uint64_t)(kMaxSegKeys + 1) * kBitmapBytes < (1ull << 28), "segment counts");
__device__ __forceinline__ uint64_t pack_seg_counts(const PairCounts &n) {
  return n.task | (n.light << 12) | (n.big << 24) | (n.small << 36);
}

// Per-block layout: c holds each segment's counts (pack_seg_counts), bt each block's totals (bt.x[blockIdx]); the
// block totals alone are scanned (scan_blocks_multi), and k_pair_emit ranks its block's segments
// itself — the per-segment scan passes over 4 x 8 MB are gone.
__global__ __launch_bounds__(kPairThreads) void k_pair_count(PairArgs a, uint64_t *c, PairCountArrays bt,
                                                             uint64_t *stats) {
  const uint64_t p = (uint64_t)blockIdx.x * kPairThreads + threadIdx.x; // segment
  uint64_t inb[3] = {0, 0, 0};
  PairCounts n{};
  if (p < a.nseg) {
    PairBases b{};
    pair_walk<false>(a, p, n, inb, b, nullptr, nullptr, TaskMeta{});
    c[p] = pack_seg_counts(n);
  }
  // stats words: 0 total input (with key arrays), 2 filter+copy task input, 3 register-path input,
  // 6 all task input (what k_pair_tasks reads)
  const int words[4] = {0, 2, 3, 6};
  const uint64_t vals[4] = {inb[0] + inb[1] + inb[2], inb[1], inb[2], inb[1] + inb[2]};
  stat_add_block(stats, words, vals);
  const uint64_t cv[4] = {n.task, n.light, n.big, n.small};
  uint64_t sums[4];
  block_sums(cv, sums);
  if (threadIdx.x == 0) {
    bt.task[blockIdx.x] = sums[0];
    bt.light[blockIdx.x] = sums[1];
    bt.big[blockIdx.x] = sums[2];
    bt.small[blockIdx.x] = sums[3];
  }
}

// A block's segments own contiguous ranges of the light and of the heavy record arrays (the scans
// run in segment order), so its records are staged in LDS and stored as contiguous 8-B-per-lane
// runs: a thread's own records are 40-B structs at scattered positions, which the store path
// replays line by line (k_pair_emit measured 189 us per 1M pairs, issue-stall bound).
constexpr uint32_t kEmitStage = 640; // records (25 KiB); a block with more stores directly
// tot (when non-null): the scans' totals on the device (tasks, light, big, small) — the heavy records
// follow the light ones in one array and the small slots follow the big ones, so the launch needs no
// host read-back of the totals (api.hip launches it before the host has them)
// cnt: the segments' counts, bs: the exclusive scans of the block totals (bs.x[blockIdx]); every
// segment's task offset is also stored in task_begin[p] (task_begin[nseg] = the total) for the
// compaction.
#ifndef RBG_EMIT_WAVES
#define RBG_EMIT_WAVES 1 // study builds: waves per SIMD the emit is compiled for (1: no bound; 119 VGPRs = 4 waves)
#endif
__global__ __launch_bounds__(kPairThreads, RBG_EMIT_WAVES) void k_pair_emit(PairArgs a, const uint64_t *cnt, PairCountArrays bs,
                                                            uint64_t small_base, TaskRec *light, TaskRec *heavy,
                                                            TaskMeta tm, uint64_t *task_begin, const uint64_t *tot,
                                                            uint64_t cap, unsigned long long *zero_q) {
  // the task kernels' chunk-queue counters (kQueueWords), zeroed here rather than by a memset launch
  if (zero_q && blockIdx.x == 0)
    for (int i = threadIdx.x; i < kQueueWords; i += kPairThreads) zero_q[i] = 0ull;
  if (tot) {
    heavy = light + tot[1];
    small_base = tot[2] * (uint64_t)kBitmapBytes;
    if (tot[0] > cap) return; // the workspace holds cap tasks: the host fails the call on the totals
  }
  __shared__ __attribute__((aligned(16))) TaskRec stage[kEmitStage];
  __shared__ uint64_t s_slot[kEmitStage];
  __shared__ uint32_t wtot[kPairThreads / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * kPairThreads;
  const uint64_t p = b0 + threadIdx.x; // segment
  const bool live = p < a.nseg;
  // in-block ranks of the segments' counts (a block holds <= 256 x seg_keys tasks and <= 512 MiB of
  // small slots: 32-bit)
  const uint64_t pc = live ? cnt[p] : 0ull;
  const uint32_t ct = (uint32_t)(pc & 0xFFFu), cl = (uint32_t)((pc >> 12) & 0xFFFu);
  const uint32_t cg = (uint32_t)((pc >> 24) & 0xFFFu), cs = (uint32_t)(pc >> 36);
  uint32_t nt32, nl32, ng32, ns32;
  const uint32_t xt = block_xscan(ct, wtot, nt32), xl = block_xscan(cl, wtot, nl32);
  const uint32_t xg = block_xscan(cg, wtot, ng32), xs = block_xscan(cs, wtot, ns32);
  const uint64_t T0 = bs.task[blockIdx.x], L0 = bs.light[blockIdx.x];
  const uint64_t H0 = T0 - L0, nl = nl32, nh = (uint64_t)nt32 - nl32, nt = nt32;
  const bool staged = nt <= kEmitStage; // block-uniform
  if (live) {
    PairCounts n{};
    PairBases b{T0 + xt, L0 + xl, (T0 + xt) - (L0 + xl), bs.big[blockIdx.x] + xg,
                small_base + bs.small[blockIdx.x] + xs};
    task_begin[p] = b.task;
    if (p == a.nseg - 1) task_begin[a.nseg] = b.task + ct;
    uint64_t inb[3] = {0, 0, 0};
    if (staged) {
      TaskMeta sm = tm;
      sm.slot = s_slot;
      pair_walk<true>(a, p, n, inb, b, light, heavy, sm, stage, stage + nl, L0, H0, T0);
    } else {
      pair_walk<true>(a, p, n, inb, b, light, heavy, tm);
    }
  }
  if (!staged) return;
  __syncthreads();
  static_assert(sizeof(TaskRec) == 40, "TaskRec is 5 u64 words");
  const uint64_t *s64 = reinterpret_cast<const uint64_t *>(stage);
  uint64_t *l64 = reinterpret_cast<uint64_t *>(light + L0), *h64 = reinterpret_cast<uint64_t *>(heavy + H0);
  for (uint64_t w = threadIdx.x; w < 5 * nl; w += kPairThreads) l64[w] = s64[w];
  for (uint64_t w = threadIdx.x; w < 5 * nh; w += kPairThreads) h64[w] = s64[5 * nl + w];
  for (uint64_t t = threadIdx.x; t < nt; t += kPairThreads) {
    tm.slot[T0 + t] = s_slot[t];
  }
}

// ---------------------------------------------------------------- the per-task kernels
// Result type of a matched pair (derived from the container implementations):
//   AND:    R&R -> EFF, else AB                      (RunContainer.java:381-456; BitmapContainer.java:162-188)
//   OR:     any Bitmap -> LR, A|A -> AB, else EFF     (BitmapContainer.java:1073-1110; RunContainer.java:1926-1986;
//                                                      ArrayContainer.java:949-973)
//   XOR:    R^R, R^A(|A|<32) -> EFF, else AB         (RunContainer.java:2410-2482; ArrayContainer.java:1311-1336)
//   ANDNOT: R\R, R\A(|A|<32) -> EFF, else AB         (RunContainer.java:574-692; BitmapContainer.java:221-274)
// An AND with an Array operand, or an ANDNOT with an Array on the left, is a subset of that
// Array, so AB == Array: those run as filters.

// A Run payload over 8 KiB (> 2047 runs) is staged straight from global memory; the toggle->
// membership transform runs in LDS so it needs no register bitmap.
__device__ __noinline__ void stage_big_runs(const uint8_t *p, uint32_t nruns, uint32_t *s, int lane) {
  lds_zero(s, lane);
  wave_lds_sync();
  const uint32_t *r32 = reinterpret_cast<const uint32_t *>(p);
  for (uint32_t i = lane; i < nruns; i += 64) toggle_run(s, r32[i]);
  wave_lds_sync();
  toggles_to_words_lds(s, lane);
  wave_lds_sync();
}

struct RecU { // the wave-uniform view of one TaskRec
  uint64_t pa, pb, out;
  uint32_t t, da, db, ra, rb;
};
__device__ __forceinline__ RecU load_rec(const TaskRec *r) {
  RecU u;
  u.pa = r->pa;
  u.pb = r->pb;
  u.out = r->out;
  u.t = r->t;
  u.da = r->da;
  u.db = r->db;
  u.ra = r->ra;
  u.rb = r->rb;
  return u;
}

// One decoded task.  P and Q are the two payloads the task reads (each preloaded as <= 8 x 16 B
// per lane unless it exceeds 8 KiB):
//   kCopy   unmatched container, cloned unchanged (RoaringArray.appendCopy :184-205): P = it;
//   kFilter result is a subset of an Array operand F (AND with an Array, ANDNOT with an Array on
//           the left; ArrayContainer.and/andNot :184-271, BitmapContainer.and(Array) :162-172,
//           RunContainer.and(Array) :305-336): P = F, Q = the other operand X, staged in LDS;
//   kHeavy  everything else: P = A, Q = B as 65536-bit register bitmaps.
#ifndef RBG_HEAVY_NOPF
#define RBG_HEAVY_NOPF 0 // study: register-path tasks without the one-task prefetch, at 128 VGPRs, so three
                         // light waves fit beside each heavy one on a SIMD
#endif
#ifndef RBG_HEAVY_MERGE
#define RBG_HEAVY_MERGE 0 // study builds: 1 merges OR / XOR of two small Arrays here (slower: DESIGN.md §7 r06)
#endif
#ifndef RBG_BAL_EMIT
#define RBG_BAL_EMIT 0 // study builds: 1 emits register-path Array / Run results by per-lane cursor walks (slower)
#endif
constexpr int kLightWaves = 4; // waves per SIMD of the copy + filter kernel (128 VGPRs)
#ifndef RBG_HEAVY_WAVES
#define RBG_HEAVY_WAVES (RBG_HEAVY_NOPF ? 4 : 2)
#endif
constexpr int kHeavyWaves = RBG_HEAVY_WAVES; // waves per SIMD the register-path kernel is allocated for
constexpr bool kHeavyPrefetch = !RBG_HEAVY_NOPF;    // the next task's payloads in flight during this one's emission
#ifndef RBG_STUDY
#define RBG_STUDY 0 // study builds: per-phase s_memtime totals of a few light / heavy waves (printf)
#endif
enum { kCopy = 0, kFilter = 1, kHeavy = 2, kBits = 3 };
struct Task {
  int kind;
  bool bigp, bigq;       // payload exceeds 8 KiB (Run with > 2047 runs): direct path from global
  bool p_is_a;           // P is A's container (kBits: the inplace Bitmap.ior(Array) rule reads it)
  const uint8_t *pp, *pq;
  uint32_t pbytes, qbytes;
  int tp, tq;            // container types of P and Q
  uint32_t cp, cq, rp, rq;
};
// LIGHT: the copy + filter kernel's view, where a matched OR pair is a kBits task (bits_task: the walk sends
// no other matched OR pair there); P is then the large Bitmap (A's when both qualify)
template <int OP, bool LIGHT>
__device__ __forceinline__ Task decode_task(const RecU &r, const uint8_t *pay_a, const uint8_t *pay_b) {
  Task T;
  const uint32_t ta = desc_type(r.da), tb = desc_type(r.db);
  const uint32_t ca = desc_card(r.da), cb = desc_card(r.db);
  const bool bits = LIGHT && RBG_OR_BITS && OP == RB_OR && ta != kAbsent && tb != kAbsent;
  const bool p_is_a = bits ? big_bitmap((int)ta, ca)
                           : ta != kAbsent && !(light_task(OP, (int)ta, (int)tb) && tb == kArray &&
                                                (ta != kArray || (OP != RB_ANDNOT && cb < ca)));
  T.p_is_a = p_is_a;
  if (ta == kAbsent || tb == kAbsent) T.kind = kCopy;
  else if (bits) T.kind = kBits;
  else T.kind = light_task(OP, (int)ta, (int)tb) ? kFilter : kHeavy;
  // kFilter: F is the Array (ANDNOT: always A; AND of two Arrays: the smaller, A on ties)
  T.pp = p_is_a ? pay_a + r.pa : pay_b + r.pb;
  T.pq = p_is_a ? pay_b + r.pb : pay_a + r.pa;
  T.tp = (int)(p_is_a ? ta : tb);
  T.tq = (int)(p_is_a ? tb : ta);
  T.cp = p_is_a ? ca : cb;
  T.cq = p_is_a ? cb : ca;
  T.rp = p_is_a ? r.ra : r.rb;
  T.rq = p_is_a ? r.rb : r.ra;
  T.pbytes = (uint32_t)payload_bytes(T.tp, T.cp, T.rp);
  T.qbytes = T.kind == kCopy ? 0u : (uint32_t)payload_bytes(T.tq, T.cq, T.rq);
  T.bigp = T.pbytes > (uint32_t)kBitmapBytes;
  T.bigq = T.qbytes > (uint32_t)kBitmapBytes;
  return T;
}

// Result type of a matched pair for the register path:
//   AND: R&R -> EFF, else AB; OR: any Bitmap -> LR, A|A -> AB, else EFF;
//   XOR / ANDNOT: R^R, R\R, and R^A / A^R / R\A with |A| < 32 -> EFF, else AB.
template <int OP> __device__ __forceinline__ bool eff_rule(int ta, int tb, uint32_t ca, uint32_t cb) {
  if (OP == RB_AND) return ta == kRun && tb == kRun;
  if (OP == RB_OR) return ta != kBitmap && tb != kBitmap && !(ta == kArray && tb == kArray);
  if (OP == RB_XOR)
    return (ta == kRun && tb == kRun) || (ta == kArray && tb == kRun && ca < (uint32_t)kRunArrayThreshold) ||
           (ta == kRun && tb == kArray && cb < (uint32_t)kRunArrayThreshold);
  return (ta == kRun && tb == kRun) || (ta == kRun && tb == kArray && cb < (uint32_t)kRunArrayThreshold);
}
// FastAggregation.priorityqueue_or's lazy OR of x (P, the in-place target) and y (Q) for their union
// (c, r): the result type of Container.lazyOR (kLazyStatic, RoaringBitmap.lazyor static) or lazyIOR
// (kLazyIor: this.lazyor(x2); kLazyIorBf: lazyorfromlazyinputs, a Bitmap y goes first) — oracle
// c_lazy_or / c_lazy_ior (ArrayContainer.lazyor :1449-1464, RunContainer.lazyorToRun :1769-1813,
// BitmapContainer.lazyor / ilazyor :657-685, 887-918, BitmapContainer.or(Array), RunContainer.or(Bitmap),
// RunContainer.ior(Run)).  cw = the card word to store (kLazyCard: a lazy Bitmap; | kRunAsBitmap: a Run
// of more than 2047 runs kept as bitmap words), bits = the payload is emitted as bitmap words.
__device__ __forceinline__ int lazy_or_type(int mode, int tx, int ty, uint32_t cx, uint32_t cy, int c, int r,
                                            uint32_t &cw, bool &bits) {
  bits = false;
  cw = (uint32_t)c;
  if (mode == kLazyRepair) { // x == y: repairAfterLazy (BitmapContainer :1214-1224 repairs only a lazy
                             // Bitmap — cardinality -1; RunContainer :2073 toEfficientContainer)
    if (tx == kRun) return type_eff(c, r);
    if (tx != kBitmap) return kArray;
    const int t = (cx & kLazyCard) ? type_lr(c) : (int)kBitmap;
    bits = t == kBitmap;
    return t;
  }
  if (mode == kLazyIorBf && ty == kBitmap && tx != kBitmap) { // the Bitmap becomes the target
    const int t = tx;
    tx = ty;
    ty = t;
    const uint32_t u = cx;
    cx = cy;
    cy = u;
  }
  const bool full = c == kSpan, ylazy = ty == kBitmap && (cy & kLazyCard);
  const bool xfull = tx == kRun && (cx & ~kCardMarks) == (uint32_t)kSpan;
  enum { kLazyB, kExactB, kA, kR, kEff } k;
  if (tx == kArray && ty == kArray) {
    k = (cx & ~kCardMarks) + (cy & ~kCardMarks) > 1024u ? kLazyB : kA; // ARRAY_LAZY_LOWERBOUND
  } else if (mode == kLazyStatic) {
    if (tx == kBitmap || ty == kBitmap) k = kLazyB;
    else if (tx == kRun && ty == kRun) k = full ? kR : kEff;                 // run_or_run
    else k = full ? kR : r > kMaxArray ? kLazyB : kR;                        // lazyorToRun
  } else if (tx == kArray) {
    if (ty == kBitmap) k = ylazy ? kLazyB : full ? kR : kExactB;             // y.or(x): full -> Run
    else k = full ? kR : r > kMaxArray ? kLazyB : kR;                        // y.lazyor(x) -> lazyorToRun
  } else if (tx == kRun) {
    if (xfull) k = kR;                                                       // returns a full this
    else if (ty == kArray) k = full ? kR : r > kMaxArray ? kLazyB : kR;      // ilazyorToRun
    else if (ty == kBitmap) k = full ? kR : kExactB;                         // or(Bitmap)
    else k = kEff;                                                           // ior(Run)
  } else {
    k = kLazyB;                                                              // Bitmap.ilazyor
  }
  switch (k) {
  case kLazyB: bits = true; cw = kLazyCard; return kBitmap;
  case kExactB: bits = true; return kBitmap;
  case kA: return kArray;
  case kEff: return type_eff(c, r);
  default:
    if (r > 2047) { // 4r + 2 > 8 KiB: kept as bitmap words (the size stays the reference's 4r + 4)
      bits = true;
      cw = (uint32_t)c | kRunAsBitmap;
    }
    return kRun;
  }
}
template <int OP> __device__ __forceinline__ void word_op(uint64_t &a, uint64_t b) {
  if (OP == RB_AND) a &= b;
  else if (OP == RB_OR) a |= b;
  else if (OP == RB_XOR) a ^= b;
  else a &= ~b;
}

// Run AND Run as an interval intersection (RunContainer.and(RunContainer), RunContainer.java:381-456):
// the two-pointer walk over both run lists advances the list whose current run ends first (A on
// ties), i.e. it visits the states of a merge of the two lists by run END.  Each lane takes an
// equal stretch of that merge (merge-path split by binary search over the runs staged in LDS),
// counts the overlapping pairs and their lengths, and after a wave scan writes its intersections as
// Run pairs.  Intersections of canonical run lists are never adjacent (two consecutive ones lie in
// different runs of A or of B, which leave a gap), so they are the result's maximal runs: c and r
// are exact.  Returns false (nothing written) when EFF(c, r) is not Run — the caller then builds the
// register bitmap.  Needs round4(ra) + rb <= 2048 (both lists in the wave's 8 KiB scratch).
__device__ __forceinline__ uint32_t run_end(uint32_t x) { return (x & 0xFFFF) + (x >> 16); }
template <bool CARD_ONLY>
__device__ __forceinline__ bool and_runs_intervals(const uint4 (&pq)[8], const uint4 (&qq)[8], uint32_t ra,
                                                   uint32_t rb, uint32_t *s, uint8_t *dst, int lane, int &card,
                                                   int &runs) {
  const uint32_t oa = (ra + 3) & ~3u;
  uint4 *s4 = reinterpret_cast<uint4 *>(s);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t c = (uint32_t)(lane + 64 * i);
    if (4 * c < ra) s4[c] = pq[i];
    if (4 * c < rb) s4[oa / 4 + c] = qq[i];
  }
  wave_lds_sync();
  const uint32_t *SA = s, *SB = s + oa;
  const uint32_t total = ra + rb, per = (total + 63) >> 6;
  const uint32_t d0 = min((uint32_t)lane * per, total), d1 = min(d0 + per, total);
  uint32_t lo = d0 > rb ? d0 - rb : 0, hi = min(d0, ra);
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (run_end(SA[mid]) <= run_end(SB[d0 - mid - 1])) lo = mid + 1;
    else hi = mid;
  }
  const uint32_t i0 = lo, j0 = d0 - lo;
  uint32_t cnt = 0, sum = 0;
  {
    uint32_t i = i0, j = j0;
    uint32_t a = i < ra ? SA[i] : 0, b = j < rb ? SB[j] : 0;
    for (uint32_t d = d0; d < d1 && i < ra && j < rb; ++d) {
      const uint32_t ea = run_end(a), eb = run_end(b);
      const uint32_t st = max(a & 0xFFFF, b & 0xFFFF), en = min(ea, eb);
      if (st <= en) {
        ++cnt;
        sum += en - st + 1;
      }
      if (ea <= eb) {
        ++i;
        a = i < ra ? SA[i] : 0;
      } else {
        ++j;
        b = j < rb ? SB[j] : 0;
      }
    }
  }
  card = (int)wave_sum_u32(sum);
  runs = (int)wave_sum_u32(cnt);
  if (CARD_ONLY || card == 0) return true;
  if (type_eff(card, runs) != kRun) {
    wave_lds_sync(); // the register path restages this scratch
    return false;
  }
  uint32_t pos = wave_scan_u32(cnt, lane) - cnt;
  uint32_t *o = reinterpret_cast<uint32_t *>(dst);
  uint32_t i = i0, j = j0;
  uint32_t a = i < ra ? SA[i] : 0, b = j < rb ? SB[j] : 0;
  for (uint32_t d = d0; d < d1 && i < ra && j < rb; ++d) {
    const uint32_t ea = run_end(a), eb = run_end(b);
    const uint32_t st = max(a & 0xFFFF, b & 0xFFFF), en = min(ea, eb);
    if (st <= en) o[pos++] = st | ((en - st) << 16);
    if (ea <= eb) {
      ++i;
      a = i < ra ? SA[i] : 0;
    } else {
      ++j;
      b = j < rb ? SB[j] : 0;
    }
  }
  wave_lds_sync();
  return true;
}
// tasks per claim (one counter: 4 -> 6.0 ms steps from atomic contention, 8 -> 4.64, 16 -> 4.59-4.62,
// 32 -> 4.71-4.78; 8 counters: 8 -> 4.49-4.52)
constexpr uint64_t kQueueChunk = 8;
constexpr uint32_t kQueueStripes = 8; // task sub-ranges with a counter each (a wave moves on when its is empty)
constexpr uint32_t kQueueStride = 16; // counters 128 B apart
// the API reserves 32 counters (4 KiB): 16 for the light tasks' queue, 16 for the heavy tasks'
static_assert(kQueueStripes >= 1 && kQueueStripes <= 16, "two queues of at most 16 counters");
constexpr uint32_t kHeavyQueueOffset = 16 * kQueueStride;
// Next chunk [s, e) of the wave's current sub-range, moving to the following sub-ranges as they run
// dry; s = n when every sub-range is exhausted.  One vector atomic by lane 0 per try, broadcast.
struct Chunk {
  uint64_t s, e;
};
__device__ __forceinline__ Chunk claim_chunk(unsigned long long *queue, uint64_t n, uint32_t &k, uint32_t &tried,
                                             int lane) {
  while (tried < kQueueStripes) {
    const uint64_t lo = n * k / kQueueStripes, hi = n * (k + 1) / kQueueStripes;
    unsigned long long v = 0;
    if (lane == 0)
      v = __hip_atomic_fetch_add(queue + k * kQueueStride, (unsigned long long)kQueueChunk, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t st = lo + pack2(__builtin_amdgcn_readfirstlane((uint32_t)v),
                                   __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)));
    if (st < hi) return Chunk{st, min(st + kQueueChunk, hi)};
    k = (k + 1) % kQueueStripes;
    ++tried;
  }
  return Chunk{n, n};
}

// The task kernel, ONE WAVE PER TASK, persistent waves striding over one record list with a
// one-task software pipeline: the next task's record and both payloads are in flight while the
// current one computes.  Loads sit at fixed points of the loop body (a task with fewer payloads
// re-reads 16 B of its first one) so the prefetch registers carry no phis.
//   ROLE kRoleLight (copies + filters, 4 waves/SIMD): stage X in LDS, load the next Q, filter F
//                   (or store the copy), load the next P;
//   ROLE kRoleHeavy (register path): build the 65536-bit result in registers from P and Q, load
//                   both next payloads, then classify and emit.
enum { kRoleLight = 0, kRoleHeavy = 1 };
template <int OP, bool CARD_ONLY, int ROLE>
__global__ __launch_bounds__(256, ROLE == kRoleHeavy ? kHeavyWaves : kLightWaves) void k_pair_tasks(
    const uint8_t *__restrict__ pay_a, const uint8_t *__restrict__ pay_b, const TaskRec *__restrict__ recs,
    uint64_t n, uint8_t *__restrict__ out, TaskMeta tm, unsigned long long *queue) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4][2048];
  __shared__ __attribute__((aligned(16))) uint16_t stage[ROLE == kRoleLight ? 4 : 1][kStageVals];
  __shared__ uint4 tbuf[ROLE == kRoleLight ? 4 : 1][32]; // per-wave half-row transpose (filter_rows_linear)
  // register path: a second 8 KiB per wave for the balanced Array / Run emission (wave.hpp emit_container_bal)
  __shared__ __attribute__((aligned(16))) uint32_t estage[ROLE == kRoleHeavy && RBG_BAL_EMIT ? 4 : 1]
                                                        [ROLE == kRoleHeavy && RBG_BAL_EMIT ? 2048 : 4];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // static schedule (queue == nullptr): wave w takes tasks w, w + stride, ...; dynamic: chunks of
  // kQueueChunk consecutive tasks from a device counter shared by every launch on it (the
  // concurrent phase's second light launch fills the CUs the heavy kernel leaves), the next chunk
  // claimed one chunk ahead so the atomic's latency is hidden
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  uint64_t g = (uint64_t)blockIdx.x * 4 + wv, cend = 0, nxt = 0, nend = 0;
  uint32_t qk = (uint32_t)(g % kQueueStripes), qtried = 0;
  if (queue) {
    const Chunk c0 = claim_chunk(queue, n, qk, qtried, lane);
    g = c0.s;
    cend = c0.e;
    const Chunk c1 = claim_chunk(queue, n, qk, qtried, lane);
    nxt = c1.s;
    nend = c1.e;
  }
  if (g >= n) return;
  uint32_t *s = lds[wv];
  uint16_t *ob = stage[ROLE == kRoleLight ? wv : 0];
  RecU cur = load_rec(recs + g);
  Task tc = decode_task<OP, ROLE == kRoleLight>(cur, pay_a, pay_b);
  uint4 pq[8], qq[8];
#if RBG_STUDY
  uint64_t lt_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, lt0 = 0, lt1 = 0, lt2 = 0; // decode, stage B/A/R, copy, filter, iteration, tasks
  uint64_t lt_wait = 0; // heavy: cycles waiting for the task's payload loads (an explicit vmcnt(0) at its start)
#define RBG_LT(x) if (ROLE == kRoleLight) { x; }
#define RBG_HT(x) if (ROLE == kRoleHeavy) { x; }
#else
#define RBG_LT(x)
#define RBG_HT(x)
#endif
  load_chunks(pq, tc.pp, tc.bigp ? 16u : tc.pbytes, lane);
  if (ROLE == kRoleHeavy && !kHeavyPrefetch) {
  } else if (tc.kind == kCopy || tc.bigq) load_chunks(qq, tc.pp, 16, lane);
  else load_chunks(qq, tc.pq, tc.qbytes, lane);
  while (true) {
    uint64_t gn = g + stride;
    bool new_chunk = false;
    if (queue) {
      gn = g + 1;
      if (gn >= cend) { // wave-uniform branch: only here is the claimed chunk waited for
        gn = nxt;
        new_chunk = true;
      }
    }
    const bool has_next = gn < n;
    RBG_LT(lt0 = __builtin_amdgcn_s_memtime());
    RBG_HT(lt0 = __builtin_amdgcn_s_memtime());
    const RecU nx = load_rec(recs + (has_next ? gn : g));
    const Task tn = decode_task<OP, ROLE == kRoleLight>(nx, pay_a, pay_b);
    RBG_LT(lt1 = __builtin_amdgcn_s_memtime(); lt_acc[0] += lt1 - lt0);
    RBG_HT(lt1 = __builtin_amdgcn_s_memtime(); lt_acc[0] += lt1 - lt0);
    int ty = kEmpty, c = 0;
    uint32_t nr = 0, cw = 0xFFFFFFFFu; // cw: the card word to store when it is not c (lazy marks)
    uint8_t *dst = out + cur.out;
    bool done = false;
    if (ROLE == kRoleHeavy && OP == RB_AND && tc.tp == kRun && tc.tq == kRun && !tc.bigp &&
        !tc.bigq && ((tc.rp + 3) & ~3u) + tc.rq <= 2048u) {
      int r = 0;
      if (!kHeavyPrefetch) load_chunks(qq, tc.pq, tc.qbytes, lane);
      done = and_runs_intervals<CARD_ONLY>(pq, qq, tc.rp, tc.rq, s, dst, lane, c, r);
      if (done && kHeavyPrefetch) {
        ty = c == 0 ? kEmpty : CARD_ONLY ? kArray : kRun;
        nr = ty == kRun ? (uint32_t)r : 0u;
        __builtin_amdgcn_sched_barrier(0);
        {
          const bool real = has_next && !tn.bigq;
          load_chunks(qq, real ? tn.pq : tn.pp, real ? tn.qbytes : 16u, lane);
        }
        load_chunks(pq, tn.pp, tn.bigp ? 16u : tn.pbytes, lane);
      } else if (done) {
        ty = c == 0 ? kEmpty : CARD_ONLY ? kArray : kRun;
        nr = ty == kRun ? (uint32_t)r : 0u;
      }
    }
    if (ROLE == kRoleHeavy && RBG_HEAVY_MERGE && !done && (OP == RB_OR || OP == RB_XOR) && !tm.lazy &&
        tc.tp == kArray && tc.tq == kArray && tc.cp + tc.cq <= kMergeMax) {
      // ---- Array OR / XOR Array as a merge (merge_run, the small-batch kernel's): the result is an Array
      //      (c <= ca + cb <= 4088), the register path's type, without two 65536-bit images and the per-word
      //      emission loops.  In this kernel, not the copy + filter one (there it made the L2-bound light
      //      kernel the long pole: profiles/r05/merge).
      merge_stage(pq, tc.cp, qq, tc.cq, s, lane);
      __builtin_amdgcn_sched_barrier(0);
      if (kHeavyPrefetch) { // the staged payloads' registers are free: the next task's loads go out now
        {
          const bool real = has_next && !tn.bigq;
          load_chunks(qq, real ? tn.pq : tn.pp, real ? tn.qbytes : 16u, lane);
        }
        load_chunks(pq, tn.pp, tn.bigp ? 16u : tn.pbytes, lane);
      }
      c = (int)merge_run<OP, !CARD_ONLY>(s, tc.cp, tc.cq, reinterpret_cast<uint16_t *>(dst), lane);
      ty = CARD_ONLY ? (c ? kArray : kEmpty) : (c || (OP == RB_XOR && tm.keep_empty)) ? kArray : kEmpty;
      nr = 0;
      done = true;
    }
    if (ROLE == kRoleHeavy && !done) {
      // ---- the result as a register bitmap: P = A, Q = B (never swapped: ANDNOT and the type
      //      rules are ordered)
#if RBG_STUDY
      {
        const uint64_t tw0 = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_waitcnt(0x0F70); // vmcnt(0)
        lt_wait += __builtin_amdgcn_s_memtime() - tw0;
      }
#endif
      uint64_t w[kW];
      if (bitmap_payload(tc.tp, tc.cp)) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          w[2 * k] = pack2(pq[k].x, pq[k].y);
          w[2 * k + 1] = pack2(pq[k].z, pq[k].w);
        }
      } else if (tc.tp == kRun && !tc.bigp) {
        stage_run_toggles(pq, tc.rp, s, lane); // toggles -> registers -> prefix-xor in registers
        lds_read_words(s, w, lane);
        wave_lds_sync();
        toggles_to_words(w, lane);
      } else {
        if (tc.bigp) stage_big_runs(tc.pp, tc.rp, s, lane);
        else stage_from_chunks(tc.tp, pq, tc.cp, tc.rp, s, lane);
        lds_read_words(s, w, lane);
        wave_lds_sync();
      }
      // without prefetch Q is loaded only now, once P's registers are free (P and Q are never live
      // together: the wave fits 128 VGPRs)
      if (!kHeavyPrefetch && !(OP == RB_AND && tc.tp == kRun && tc.tq == kRun && !tc.bigp && !tc.bigq &&
                               ((tc.rp + 3) & ~3u) + tc.rq <= 2048u))
        load_chunks(qq, tc.bigq ? tc.pp : tc.pq, tc.bigq ? 16u : tc.qbytes, lane);
      if (bitmap_payload(tc.tq, tc.cq)) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          word_op<OP>(w[2 * k], pack2(qq[k].x, qq[k].y));
          word_op<OP>(w[2 * k + 1], pack2(qq[k].z, qq[k].w));
        }
      } else if (tc.tq == kRun && !tc.bigq) {
        stage_run_toggles(qq, tc.rq, s, lane);
        uint64_t t[kW];
        lds_read_words(s, t, lane);
        wave_lds_sync();
        toggles_to_words(t, lane);
#pragma unroll
        for (int j = 0; j < kW; ++j) word_op<OP>(w[j], t[j]);
      } else {
        if (tc.bigq) stage_big_runs(tc.pq, tc.rq, s, lane);
        else stage_from_chunks(tc.tq, qq, tc.cq, tc.rq, s, lane);
        const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint4 v = s4[k * 64 + lane];
          word_op<OP>(w[2 * k], pack2(v.x, v.y));
          word_op<OP>(w[2 * k + 1], pack2(v.z, v.w));
        }
        wave_lds_sync();
      }
      // ---- both next payloads in flight during classification and emission (the fence keeps the
      //      scheduler from hoisting these loads above the consumption of the current ones)
      RBG_HT(lt2 = __builtin_amdgcn_s_memtime(); lt_acc[1] += lt2 - lt1);
      __builtin_amdgcn_sched_barrier(0);
      if (kHeavyPrefetch) {
        {
          const bool real = has_next && !tn.bigq;
          load_chunks(qq, real ? tn.pq : tn.pp, real ? tn.qbytes : 16u, lane);
        }
        load_chunks(pq, tn.pp, tn.bigp ? 16u : tn.pbytes, lane);
      }
      const int ta = tc.tp, tb = tc.tq;
      const bool lazy = OP == RB_OR && tm.lazy;
      const bool eff = eff_rule<OP>(ta, tb, tc.cp, tc.cq);
      int r;
      metrics(w, lane, (eff || (lazy && (ta == kRun || tb == kRun))) && !CARD_ONLY, c, r);
      RBG_HT(const uint64_t lt3 = __builtin_amdgcn_s_memtime(); lt_acc[2] += lt3 - lt2; lt2 = lt3);
      bool bits = false;
      if (lazy) {
        ty = lazy_or_type(tm.lazy, ta, tb, tc.cp, tc.cq, c, r, cw, bits);
        if (ty == kRun && c == kSpan) r = 1;
      } else if (OP != RB_OR && c == 0 && !(OP == RB_XOR && tm.keep_empty)) ty = kEmpty;
      else if (eff) ty = type_eff(c, r);
      else if (OP == RB_OR && tm.inplace && ta == kBitmap && tb == kArray) {
        ty = kBitmap; // BitmapContainer.ior(ArrayContainer) returns this, full or not (BitmapContainer.java:749-766)
      } else if (OP == RB_OR && (ta == kBitmap || tb == kBitmap)) {
        ty = type_lr(c);
        if (ty == kRun) r = 1; // LR's Run is the full container: one run
      } else ty = type_ab(c);
      if (CARD_ONLY) ty = c ? kArray : kEmpty;
      else if (ty != kEmpty) {
        if (RBG_BAL_EMIT) emit_container_bal(bits ? (int)kBitmap : ty, w, c, r, dst, s, estage[wv], lane);
        else emit_container(bits ? (int)kBitmap : ty, w, c, r, dst, s, lane);
      }
      nr = ty == kRun ? (uint32_t)r : 0u;
      RBG_HT(lt_acc[3 + (ty == kBitmap ? 0 : ty == kArray ? 1 : 2)] += __builtin_amdgcn_s_memtime() - lt2);
    } else if (ROLE != kRoleHeavy) {
      // ---- phase 1: stage X (filter; kBits: the other operand) or store the clone (copy)
      if (tc.kind == kFilter || tc.kind == kBits) {
        if (tc.bigq) stage_big_runs(tc.pq, tc.rq, s, lane); // only a Run payload exceeds 8 KiB
        else stage_from_chunks(tc.tq, qq, tc.cq, tc.rq, s, lane);
      } else if (!CARD_ONLY) {
        if (tc.bigp) copy_payload(tc.pp, dst, tc.pbytes, lane);
        else store_chunks(pq, dst, tc.pbytes, lane);
      }
      {
        const bool real = has_next && tn.kind != kCopy && !tn.bigq;
        load_chunks(qq, real ? tn.pq : tn.pp, real ? tn.qbytes : 16u, lane);
      }
      RBG_LT(lt2 = __builtin_amdgcn_s_memtime(); lt_acc[tc.kind == kFilter ? 1 + (tc.tq == kBitmap ? 0 : tc.tq == kArray ? 1 : 2) : 4] += lt2 - lt1);
      // ---- phase 2: filter F against the staged X, in value order (adjacent lanes, adjacent values)
      //      through a linear per-wave stage.  (Streaming the next F into pq row by row as the filter
      //      frees it measured 7% slower: loads and the staged stores share vmcnt, so the loads issued
      //      mid-filter serialise the output flushes behind them.)
      if (tc.kind == kFilter) {
        uint16_t *o = CARD_ONLY ? nullptr : reinterpret_cast<uint16_t *>(dst);
        uint4 *tb = tbuf[ROLE == kRoleLight ? wv : 0];
        c = OP == RB_ANDNOT ? filter_rows_linear<true, !CARD_ONLY>(pq, (int)tc.cp, s, ob, tb, o, lane)
                            : filter_rows_linear<false, !CARD_ONLY>(pq, (int)tc.cp, s, ob, tb, o, lane);
        ty = c ? kArray : kEmpty;
      } else if (tc.kind == kBits) {
        // ---- OR into the large Bitmap P (bits_task): the rows ORed and counted first, then stored — as the
        //      Bitmap, or as the full Run (one run [0, 65535], 16-B padded) unless Bitmap.ior(Array) keeps it
        const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
        uint32_t cl = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint4 x = s4[k * 64 + lane];
          pq[k] = make_uint4(pq[k].x | x.x, pq[k].y | x.y, pq[k].z | x.z, pq[k].w | x.w);
          cl += __popc(pq[k].x) + __popc(pq[k].y) + __popc(pq[k].z) + __popc(pq[k].w);
        }
        c = (int)wave_sum_u32(cl);
        const bool keep_bitmap = tm.inplace && tc.p_is_a && tc.tq == kArray;
        ty = c == kSpan && !keep_bitmap ? kRun : kBitmap;
        nr = ty == kRun ? 1u : 0u;
        if (!CARD_ONLY) {
          uint4 *o4 = reinterpret_cast<uint4 *>(dst);
          if (ty == kRun) {
            if (lane == 0) o4[0] = make_uint4(0xFFFF0000u, 0u, 0u, 0u);
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) o4[k * 64 + lane] = pq[k];
          }
        }
        if (CARD_ONLY) { // the card-only kernels mark a non-empty result as an Array (as the register path)
          ty = kArray;
          nr = 0;
        }
      } else {
        ty = tc.tp;
        c = (int)tc.cp;
        nr = tc.rp;
      }
      RBG_LT(lt_acc[5] += __builtin_amdgcn_s_memtime() - lt2);
      load_chunks(pq, tn.pp, tn.bigp ? 16u : tn.pbytes, lane);
    }
    wave_lds_sync(); // the next task restages the same LDS image
    if (lane == 0) {
      tm.type[cur.t] = (uint8_t)ty;
      tm.res[cur.t] = task_res((uint32_t)ty, nr, cw != 0xFFFFFFFFu ? cw : (uint32_t)c);
    }
    RBG_LT(lt_acc[6] += __builtin_amdgcn_s_memtime() - lt0; ++lt_acc[7]);
    RBG_HT(lt_acc[6] += __builtin_amdgcn_s_memtime() - lt0; ++lt_acc[7]);
    if (!has_next) break;
    if (new_chunk) {
      cend = nend;
      const Chunk c1 = claim_chunk(queue, n, qk, qtried, lane);
      nxt = c1.s;
      nend = c1.e;
    }
    g = gn;
    cur = nx;
    tc = tn;
    if (ROLE == kRoleHeavy && !kHeavyPrefetch) // this task's first payload, loaded only now
      load_chunks(pq, tc.pp, tc.bigp ? 16u : tc.pbytes, lane);
  }
#if RBG_STUDY
  if (ROLE == kRoleLight && lane == 0 && wv == 0 && blockIdx.x % 97 == 0)
    printf("light timing blk %u: decode %lu stageB %lu stageA %lu stageR %lu copy %lu filter %lu iter %lu tasks %lu\n",
           blockIdx.x, lt_acc[0], lt_acc[1], lt_acc[2], lt_acc[3], lt_acc[4], lt_acc[5], lt_acc[6], lt_acc[7]);
  if (ROLE == kRoleHeavy && lane == 0 && wv == 0 && blockIdx.x % 61 == 0)
    printf("heavy timing op %d blk %u: decode %lu build %lu (payload wait %lu) metrics %lu emitB %lu emitA %lu emitR %lu iter %lu tasks %lu\n",
           OP, blockIdx.x, lt_acc[0], lt_acc[1], lt_wait, lt_acc[2], lt_acc[3], lt_acc[4], lt_acc[5], lt_acc[6], lt_acc[7]);
#endif
}

// ---------------------------------------------------------------- measurement probes
// Read-only twins of k_pair_tasks for the roofline study (rbgpu_internal_probe): the same
// persistent schedule, records and payload loads, with the compute replaced by an XOR fold, and a
// plain streaming read of one payload arena.  They bound what the memory system delivers for
// this access pattern; nothing in the product calls them.
__device__ __forceinline__ uint32_t fold_chunks(const uint4 (&q)[8]) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x ^= q[i].x ^ q[i].y ^ q[i].z ^ q[i].w;
  return x;
}
template <int OP>
__global__ __launch_bounds__(256, 4) void k_probe_tasks(const uint8_t *__restrict__ pay_a,
                                                     const uint8_t *__restrict__ pay_b,
                                                     const TaskRec *__restrict__ recs, uint64_t n, uint32_t *sink) {
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  uint64_t g = (uint64_t)blockIdx.x * 4 + wv;
  if (g >= n) return;
  RecU cur = load_rec(recs + g);
  Task tc = decode_task<OP, false>(cur, pay_a, pay_b);
  uint4 pq[8], qq[8];
  load_chunks(pq, tc.pp, tc.bigp ? 16u : tc.pbytes, lane);
  if (tc.kind == kCopy || tc.bigq) load_chunks(qq, tc.pp, 16, lane);
  else load_chunks(qq, tc.pq, tc.qbytes, lane);
  uint32_t acc = 0;
  while (true) {
    const uint64_t gn = g + stride;
    const bool has_next = gn < n;
    const RecU nx = load_rec(recs + (has_next ? gn : g));
    const Task tn = decode_task<OP, false>(nx, pay_a, pay_b);
    acc ^= fold_chunks(qq);
    {
      const bool real = has_next && tn.kind != kCopy && !tn.bigq;
      load_chunks(qq, real ? tn.pq : tn.pp, real ? tn.qbytes : 16u, lane);
    }
    acc ^= fold_chunks(pq);
    load_chunks(pq, tn.pp, tn.bigp ? 16u : tn.pbytes, lane);
    if (!has_next) break;
    g = gn;
    tc = tn;
  }
  sink[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}
__global__ __launch_bounds__(256, 4) void k_probe_stream(const uint8_t *__restrict__ p, uint64_t bytes,
                                                      uint32_t *sink) {
  const int lane = lane_id();
  const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
  const uint64_t chunks = bytes / 8192;
  uint32_t acc = 0;
  for (uint64_t c = w; c < chunks; c += nw) {
    uint4 q[8];
    load_chunks(q, p + c * 8192, 8192, lane);
    acc ^= fold_chunks(q);
  }
  sink[(uint64_t)blockIdx.x * 256 + threadIdx.x] = acc;
}
void launch_probe(int op, int mode, const uint8_t *pa, const uint8_t *pb, uint64_t a_bytes, const TaskRec *recs,
                  uint64_t n, uint32_t *sink, unsigned blocks, hipStream_t st) {
  if (mode == 2) {
    k_probe_stream<<<blocks, 256, 0, st>>>(pa, a_bytes, sink);
    return;
  }
  if (!n) return;
  switch (op) {
  case RB_AND: k_probe_tasks<RB_AND><<<blocks, 256, 0, st>>>(pa, pb, recs, n, sink); break;
  case RB_OR: k_probe_tasks<RB_OR><<<blocks, 256, 0, st>>>(pa, pb, recs, n, sink); break;
  case RB_XOR: k_probe_tasks<RB_XOR><<<blocks, 256, 0, st>>>(pa, pb, recs, n, sink); break;
  default: k_probe_tasks<RB_ANDNOT><<<blocks, 256, 0, st>>>(pa, pb, recs, n, sink); break;
  }
}

// ---------------------------------------------------------------- compaction
// compaction runs per segment (units u with tasks [tb[u], tb[u+1])); a pair's results are its
// segments' results in order
// Per-block layout again: k_compact_count leaves each block's kept-result total in bk[blockIdx], the
// block totals are scanned (scan_blocks_multi, whose total is the call's result container count), and
// k_compact_write ranks its block's segments and tasks itself.
__global__ __launch_bounds__(kPairThreads) void k_compact_count(const uint64_t *tb, uint64_t nseg,
                                                                const uint8_t *ttype, uint64_t *bk) {
  const uint64_t p = (uint64_t)blockIdx.x * kPairThreads + threadIdx.x;
  uint64_t n = 0;
  if (p < nseg)
    for (uint64_t t = tb[p]; t < tb[p + 1]; ++t) n += ttype[t] != kEmpty;
  const uint64_t v[1] = {n};
  uint64_t sum[1];
  block_sums(v, sum);
  if (threadIdx.x == 0) bk[blockIdx.x] = sum[0];
}
// bks: exclusive scans of the block totals.  rseg (may be null): each segment's first result index,
// rseg[nseg] = the total (k_pair_rbegin maps them to pairs); rbegin (may be null): the same written
// as the result CSR directly, when every segment is one pair.
__global__ __launch_bounds__(kPairThreads) void k_compact_write(const uint64_t *tb, uint64_t nseg, TaskMeta tm,
                                                                const uint64_t *bks, OutView out,
                                                                const uint32_t *seg_pair, uint64_t *pair_card,
                                                                uint64_t *stats, uint64_t *rseg, uint64_t *rbegin,
                                                                CallTail tail) {
  __shared__ uint32_t wtot[kPairThreads / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * kPairThreads, be = min(b0 + kPairThreads, nseg);
  const uint64_t p = b0 + threadIdx.x;
  const uint64_t R0 = bks[blockIdx.x];
  // the segment's kept results and its rank among the block's (<= 256 x seg_keys: 32-bit)
  uint32_t kept = 0;
  const uint64_t t0 = p < nseg ? tb[p] : 0, t1 = p < nseg ? tb[p + 1] : 0;
  for (uint64_t t = t0; t < t1; ++t) kept += tm.type[t] != kEmpty;
  uint32_t btot;
  const uint64_t rs = R0 + block_xscan(kept, wtot, btot);
  if (p < nseg) {
    if (rseg) rseg[p] = rs;
    if (rbegin) rbegin[p] = rs;
    if (p == nseg - 1) {
      if (rseg) rseg[nseg] = rs + kept;
      if (rbegin) rbegin[nseg] = rs + kept;
    }
  }
  uint64_t outb[2] = {0, 0}, card_sum = 0;
  if (!pair_card && out.key) {
    // A block's segments own the contiguous task range [T0, T1) and result range from R0: one
    // thread per task, ranked by a block scan, so loads and stores are coalesced (a thread walking
    // its own segment's tasks is latency-bound).
    const uint64_t T0 = tb[b0], T1 = tb[be];
    uint64_t R = R0;
    for (uint64_t base = T0; base < T1; base += kPairThreads) {
      const uint64_t t = base + threadIdx.x;
      const uint8_t ty = t < T1 ? tm.type[t] : (uint8_t)kEmpty;
      const bool keep = ty != kEmpty;
      uint32_t tot;
      const uint32_t rank = block_xscan(keep ? 1u : 0u, wtot, tot);
      if (keep) {
        const uint64_t r = R + rank, rm = tm.res[t], sl = tm.slot[t];
        const uint32_t c = (uint32_t)(rm >> 32);
        const uint16_t nr = (uint16_t)(rm >> 8);
        out.key[r] = (uint16_t)(sl >> 40);
        out.type[r] = ty;
        out.card[r] = c;
        out.nruns[r] = nr;
        out.off[r] = sl & (kSlotOffsetLimit - 1);
        outb[(sl >> 56) & 1] += alg_bytes(ty, c, nr) + 16;
        card_sum += c;
      }
      R += tot;
    }
  } else if (p < nseg) {
    uint64_t r = rs, card = 0;
    for (uint64_t t = t0; t < t1; ++t) {
      const uint8_t ty = tm.type[t];
      if (ty == kEmpty) continue;
      const uint64_t rm = tm.res[t];
      const uint32_t c = (uint32_t)(rm >> 32);
      const uint16_t nr = (uint16_t)(rm >> 8);
      card += c;
      if (out.key) {
        const uint64_t sl = tm.slot[t];
        out.key[r] = (uint16_t)(sl >> 40);
        out.type[r] = ty;
        out.card[r] = c;
        out.nruns[r] = nr;
        out.off[r] = sl & (kSlotOffsetLimit - 1);
        outb[(sl >> 56) & 1] += alg_bytes(ty, c, nr) + 16;
      }
      ++r;
    }
    if (pair_card && card) atomicAdd((unsigned long long *)&pair_card[seg_pair ? seg_pair[p] : p], (unsigned long long)card);
    card_sum = card;
  }
  // stats words: 1 total output, 4 light-task output, 5 heavy-task output, 7 result cardinality
  if (stats) {
    const int words[4] = {1, 4, 5, 7};
    const uint64_t vals[4] = {outb[0] + outb[1], outb[0], outb[1], card_sum};
    stat_add_block(stats, words, vals);
  }
  if (!tail.hout) return;
  // ---- the last block to finish hands the call's counters to the host (the hand-off of wave.hpp st_sc1):
  //      every thread's stores and atomics done, then one agent-scope add per block
  __shared__ uint32_t s_last;
  __shared__ uint64_t s_sum[kStatWords];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(tail.ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1ull;
  __syncthreads();
  if (!s_last) return;
  static_assert(kStripes == 64, "a wave sums one counter's stripes");
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  for (int w = wv; w < kStatWords; w += kPairThreads / 64) { // the other blocks' atomics live in L2: sc1 loads
    const uint64_t x = wave_sum_u64(ld_sc1(stats + w * kStripes + lane));
    stats[w * kStripes + lane] = 0ull; // zeroed for the next call (stream order: its kernels start after this one)
    if (lane == 0) s_sum[w] = x;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 0; w < kStatWords; ++w) tail.hout[w] = s_sum[w];
    __hip_atomic_store(tail.ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); // ready for the next call
    __hip_atomic_store(tail.hout + kStatWords, tail.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// result CSR per pair from the per-segment result offsets
// (and the result container count into *count: the stats word the call reads back anyway)
__global__ __launch_bounds__(kPairThreads) void k_pair_rbegin(const uint64_t *seg_begin, uint32_t npairs,
                                                              const uint64_t *rseg, uint64_t *rbegin, uint64_t *count) {
  const uint32_t p = blockIdx.x * kPairThreads + threadIdx.x;
  if (p > npairs) return;
  const uint64_t r = rseg[seg_begin[p]];
  if (rbegin) rbegin[p] = r;
  if (p == npairs && count) *count = r;
}

// ---------------------------------------------------------------- launchers
static unsigned blocks_for(uint64_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

void launch_seg_count(const PairArgs &a, uint64_t *nseg, hipStream_t st) {
  if (!a.npairs) return;
  k_seg_count<<<blocks_for(a.npairs, kPairThreads), kPairThreads, 0, st>>>(a, nseg);
}
void launch_seg_fill(const PairArgs &a, const uint64_t *seg_begin, uint32_t *seg_pair, hipStream_t st) {
  if (!a.npairs) return;
  k_seg_fill<<<blocks_for(a.npairs, kPairThreads), kPairThreads, 0, st>>>(a, seg_begin, seg_pair);
}
void launch_max_span(const uint64_t *begin, uint32_t nb, uint64_t *out, hipStream_t st) {
  const unsigned blocks = std::min<unsigned>(blocks_for(nb, kPairThreads), 1024);
  k_max_span<<<blocks, kPairThreads, 0, st>>>(begin, nb, out);
}
void launch_pair_rbegin(const uint64_t *seg_begin, uint32_t npairs, const uint64_t *rseg, uint64_t *rbegin,
                        uint64_t *count, hipStream_t st) {
  k_pair_rbegin<<<blocks_for((uint64_t)npairs + 1, kPairThreads), kPairThreads, 0, st>>>(seg_begin, npairs, rseg,
                                                                                        rbegin, count);
}
uint64_t pair_blocks(uint64_t nseg) { return blocks_for(nseg, kPairThreads); }
void launch_pair_count(const PairArgs &a, uint64_t *c, const PairCountArrays &bt, uint64_t *stats,
                       hipStream_t st) {
  if (!a.nseg) return;
  k_pair_count<<<blocks_for(a.nseg, kPairThreads), kPairThreads, 0, st>>>(a, c, bt, stats);
}
void launch_pair_emit(const PairArgs &a, const uint64_t *cnt, const PairCountArrays &bs, uint64_t small_base,
                      TaskRec *light, TaskRec *heavy, const TaskMeta &tm, uint64_t *task_begin, const uint64_t *tot,
                      uint64_t cap, unsigned long long *zero_q, hipStream_t st) {
  if (!a.nseg) return;
  k_pair_emit<<<blocks_for(a.nseg, kPairThreads), kPairThreads, 0, st>>>(a, cnt, bs, small_base, light, heavy, tm,
                                                                          task_begin, tot, cap, zero_q);
}
// Persistent grid: every CU filled to the kernel's occupancy, waves stride over the tasks.
template <class K> static unsigned persistent_blocks(K kernel, uint64_t tasks) {
  int dev = 0, cus = 0, occ = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, 256, 0);
  if (cus <= 0) cus = 256;
  if (occ <= 0) occ = 4;
  const uint64_t want = (tasks + 3) / 4, cap = (uint64_t)cus * (uint64_t)occ;
  return (unsigned)(want < cap ? want : cap);
}

static unsigned cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return (unsigned)cus;
}
// per_cu > 0: persistent grid of per_cu blocks per CU (concurrent launches share the CUs)
template <int OP, bool CARD_ONLY, int ROLE>
static void launch_tasks(const uint8_t *pa, const uint8_t *pb, const TaskRec *recs, uint64_t n, uint8_t *out,
                         const TaskMeta &tm, hipStream_t st, unsigned per_cu = 0,
                         unsigned long long *queue = nullptr) {
  if (!n) return;
#ifndef RBG_LDS_PAD
#define RBG_LDS_PAD 0 // study: dynamic LDS a light block reserves without using it (occupancy sensitivity)
#endif
  const size_t dyn = ROLE == kRoleLight ? RBG_LDS_PAD : 0;
  static unsigned occ_cap = 0; // occupancy-derived grid cap, per template instance
  if (!occ_cap) occ_cap = persistent_blocks(k_pair_tasks<OP, CARD_ONLY, ROLE>, ~0ull >> 8);
  const unsigned cap = per_cu ? std::min(occ_cap, per_cu * cu_count()) : occ_cap;
  const uint64_t want = (n + 3) / 4;
  const unsigned blocks = (unsigned)(want < cap ? want : cap);
  k_pair_tasks<OP, CARD_ONLY, ROLE><<<blocks, 256, dyn, st>>>(pa, pb, recs, n, out, tm, queue);
}
template <int OP>
static void launch_op(bool card_only, const uint8_t *pa, const uint8_t *pb, const TaskRec *light, uint64_t nl,
                      const TaskRec *heavy, uint64_t nh, uint8_t *out, const TaskMeta &tm, hipStream_t st,
                      hipEvent_t mid) {
  if (card_only) launch_tasks<OP, true, kRoleLight>(pa, pb, light, nl, out, tm, st);
  else launch_tasks<OP, false, kRoleLight>(pa, pb, light, nl, out, tm, st);
  (void)hipEventRecord(mid, st);
  if (card_only) launch_tasks<OP, true, kRoleHeavy>(pa, pb, heavy, nh, out, tm, st);
  else launch_tasks<OP, false, kRoleHeavy>(pa, pb, heavy, nh, out, tm, st);
}
constexpr unsigned kConcLightPerCu = RBG_HEAVY_NOPF ? 3 : 2; // light blocks per CU beside the heavy kernel (2 x 128 VGPRs per SIMD)
constexpr unsigned kConcHeavyPerCu = 1; // heavy blocks per CU (256 VGPRs per SIMD)
template <int OP>
static void launch_op_concurrent(bool card_only, const uint8_t *pa, const uint8_t *pb, const TaskRec *light,
                                 uint64_t nl, const TaskRec *heavy, uint64_t nh, uint8_t *out, const TaskMeta &tm,
                                 hipStream_t st, hipStream_t side, hipEvent_t light_done, hipEvent_t ev_h0,
                                 hipEvent_t ev_h1, unsigned long long *queue) {
  // Light and heavy tasks each come from a shared queue (both zeroed by the caller before the side
  // stream's wait).  Whichever kernel drains first hands its CUs to the other kind: the side stream
  // runs heavy then light, the library stream light then heavy, and a second launch of a kind
  // takes whatever tasks of that kind are left (AND: the light tasks dominate; OR / XOR: the heavy).
  unsigned long long *hq = queue ? queue + kHeavyQueueOffset : nullptr;
  // heavy first: its blocks need the larger register slot
  (void)hipEventRecord(ev_h0, side);
  if (card_only) launch_tasks<OP, true, kRoleHeavy>(pa, pb, heavy, nh, out, tm, side, kConcHeavyPerCu, hq);
  else launch_tasks<OP, false, kRoleHeavy>(pa, pb, heavy, nh, out, tm, side, kConcHeavyPerCu, hq);
  (void)hipEventRecord(ev_h1, side);
  if (card_only) launch_tasks<OP, true, kRoleLight>(pa, pb, light, nl, out, tm, st, kConcLightPerCu, queue);
  else launch_tasks<OP, false, kRoleLight>(pa, pb, light, nl, out, tm, st, kConcLightPerCu, queue);
  (void)hipEventRecord(light_done, st);
  if (queue) {
    if (card_only) launch_tasks<OP, true, kRoleLight>(pa, pb, light, nl, out, tm, side, kConcLightPerCu, queue);
    else launch_tasks<OP, false, kRoleLight>(pa, pb, light, nl, out, tm, side, kConcLightPerCu, queue);
    if (card_only) launch_tasks<OP, true, kRoleHeavy>(pa, pb, heavy, nh, out, tm, st, kConcHeavyPerCu, hq);
    else launch_tasks<OP, false, kRoleHeavy>(pa, pb, heavy, nh, out, tm, st, kConcHeavyPerCu, hq);
  }
}
void launch_pairwise_concurrent(int op, bool card_only, const uint8_t *pa, const uint8_t *pb, const TaskRec *light,
                                uint64_t nl, const TaskRec *heavy, uint64_t nh, uint8_t *out, const TaskMeta &tm,
                                hipStream_t st, hipStream_t side, hipEvent_t light_done, hipEvent_t ev_h0,
                                hipEvent_t ev_h1, unsigned long long *queue) {
  switch (op) {
  case RB_AND: launch_op_concurrent<RB_AND>(card_only, pa, pb, light, nl, heavy, nh, out, tm, st, side, light_done, ev_h0, ev_h1, queue); break;
  case RB_OR: launch_op_concurrent<RB_OR>(card_only, pa, pb, light, nl, heavy, nh, out, tm, st, side, light_done, ev_h0, ev_h1, queue); break;
  case RB_XOR: launch_op_concurrent<RB_XOR>(card_only, pa, pb, light, nl, heavy, nh, out, tm, st, side, light_done, ev_h0, ev_h1, queue); break;
  default: launch_op_concurrent<RB_ANDNOT>(card_only, pa, pb, light, nl, heavy, nh, out, tm, st, side, light_done, ev_h0, ev_h1, queue); break;
  }
}
void launch_pairwise(int op, bool card_only, const uint8_t *pa, const uint8_t *pb, const TaskRec *light,
                     uint64_t nl, const TaskRec *heavy, uint64_t nh, uint8_t *out, const TaskMeta &tm,
                     hipStream_t st, hipEvent_t mid) {
  switch (op) {
  case RB_AND: launch_op<RB_AND>(card_only, pa, pb, light, nl, heavy, nh, out, tm, st, mid); break;
  case RB_OR: launch_op<RB_OR>(card_only, pa, pb, light, nl, heavy, nh, out, tm, st, mid); break;
  case RB_XOR: launch_op<RB_XOR>(card_only, pa, pb, light, nl, heavy, nh, out, tm, st, mid); break;
  default: launch_op<RB_ANDNOT>(card_only, pa, pb, light, nl, heavy, nh, out, tm, st, mid); break;
  }
}
void launch_compact_count(const uint64_t *task_begin, uint64_t nseg, const uint8_t *ttype, uint64_t *bk,
                          hipStream_t st) {
  if (!nseg) return;
  k_compact_count<<<blocks_for(nseg, kPairThreads), kPairThreads, 0, st>>>(task_begin, nseg, ttype, bk);
}
void launch_compact_write(const uint64_t *task_begin, uint64_t nseg, const TaskMeta &tm, const uint64_t *bks,
                          const OutView &out, const uint32_t *seg_pair, uint64_t *pair_card, uint64_t *stats,
                          uint64_t *rseg, uint64_t *rbegin, hipStream_t st, const CallTail &tail) {
  if (!nseg) return;
  k_compact_write<<<blocks_for(nseg, kPairThreads), kPairThreads, 0, st>>>(task_begin, nseg, tm, bks, out,
                                                                           seg_pair, pair_card, stats, rseg, rbegin,
                                                                           tail);
}

// ---------------------------------------------------------------- small batches: two launches
// A call of a few thousand pairs (config 1: 199 census pairs) is bound by launch and host-sync
// latency, not by bytes: the general pipeline's ~15 launches and two host read-backs cost ~150 us.
// Here ONE kernel does everything per pair (a block per pair: key alignment in LDS, then its 4 waves
// take the merged keys — unmatched copies and every matched pair through the register path, so the
// result types are the register path's, which the general pipeline also uses) into one 8 KiB slot
// per merged key, and one single-block kernel compacts the slots into the result CSR.
__device__ __forceinline__ uint32_t lower_bound_u16(const uint16_t *k, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (k[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Per-slot metadata of k_pair_small, one 8-B word per slot: card word (17-bit value + its two lazy marks,
// bits 0-18), type (bits 19-20; 3 = dropped), key (24-39), run count (40-55).
__device__ __forceinline__ uint64_t small_meta(uint32_t key, int ty, uint32_t cw, uint32_t nr) {
  const uint64_t c = (cw & 0x1FFFFu) | ((cw & kLazyCard) ? 1u << 17 : 0u) | ((cw & kRunAsBitmap) ? 1u << 18 : 0u);
  return c | ((uint64_t)(ty == (int)kEmpty ? 3u : (uint32_t)ty) << 19) | ((uint64_t)key << 24) | ((uint64_t)nr << 40);
}
__device__ __forceinline__ bool meta_empty(uint64_t m) { return ((m >> 19) & 3u) == 3u; }
// A slot's words before its key publishes them (small_meta never sets bits 56-63, the aux word's card is <= 65536):
// the context's slot words (rbgpu_ctx::d_small_slots, [2][kSmallSlots]: slot words, then aux words = the key's input
// bytes | its card << 32) are all kSlotUnset between calls — set so at allocation, and reset by each call's
// compaction after its hand-off.
constexpr uint64_t kSlotUnset = ~0ull;
__device__ __forceinline__ uint32_t meta_cw(uint64_t m) {
  return (uint32_t)(m & 0x1FFFFu) | ((m >> 17) & 1u ? kLazyCard : 0u) | ((m >> 18) & 1u ? kRunAsBitmap : 0u);
}
// Cross-block hand-off: st_sc1 / ld_sc1 (wave.hpp) of the slot words, which the compaction polls for (their
// values replace kSlotUnset); the slot payloads stay plain stores: nothing in the launch reads them.

// The compaction, run by the last block of k_pair_small: drop the empty slots, write the result SoA and
// CSR (slot t's payload stays at t * 8 KiB), add up the blocks' counters and write the call's result words
// to host-visible memory.  xl: the block's LDS scratch (the slot -> result position map when E fits it).
#if RBG_SMALL_STUDY
#define RBG_SS(i) if (threadIdx.x == 0) g_small_study[8191 * kStudyWords + (i)] = __builtin_amdgcn_s_memrealtime()
#else
#define RBG_SS(i)
#endif
constexpr uint32_t kSmallXposLds = 8192;
constexpr uint32_t kXposEmpty = 1u << 31; // xpos flag: the slot holds no result (positions stay < 2^31)
template <class Tab>
__device__ void small_compact(const SmallPairArgs &a, const Tab &tab, uint32_t *xl, uint32_t *wtot) {
  const uint32_t nt = blockDim.x, E = a.E;
  uint32_t *xpos = E <= kSmallXposLds ? xl : a.xpos;
  const OutView &out = a.out;
  RBG_SS(0);
  // the result CSR's first slot table entry and the first tile of slot words: independent loads first
  const uint32_t slot_own = a.rbegin && threadIdx.x <= a.np ? tab.slot_at(threadIdx.x) : 0u;
  // the call's counters, summed from the slot words: input bytes (with the key arrays), key-array bytes, output
  // bytes, result cardinality
  uint64_t pin = 0, pkey = 0, pout = 0, pcs = 0;
  for (uint32_t q = threadIdx.x; q < a.np; q += nt) {
    const uint32_t ab = tab.counts(q);
    pkey += 2ull * ((ab & 0xFFFFu) + (ab >> 16));
  }
  bool bad = false; // a slot word that never came (bounded polls: the host then finds no hand-over)
  constexpr int kPer = 16; // slot words per thread and tile
  uint32_t base = 0;       // results of the tiles before
  // Tiles of kPer x 256 slots, thread x taking slots x, x + 256, ...: the loads and the result SoA stores run in
  // slot order (coalesced), and a slot's result position is its row's base + the wave totals before it in the
  // row + its rank in its wave's ballot — one barrier per tile.  (A thread owning 16 consecutive slots needed a
  // block scan and stored its results 16 apart from its neighbours': every store touched 64 lines.)
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  uint32_t(*rowtot)[4] = reinterpret_cast<uint32_t(*)[4]>(wtot); // [kPer][4 waves] (wtot holds 64 words)
  static_assert(kPer * 4 <= 64, "row totals within wtot");
  for (uint32_t t0 = 0; t0 < E; t0 += kPer * nt) {
    uint64_t m[kPer], x[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t t = t0 + (uint32_t)k * nt + threadIdx.x;
      m[k] = t < E ? ld_sc1(a.smeta + t) : (3ull << 19);
      x[k] = t < E ? ld_sc1(a.smeta + kSmallSlots + t) : 0ull;
    }
    // a block still on its keys has not published: poll, every missing word of the tile in each round trip
    // (2^16 rounds, ~0.1 s, then the call fails instead of hanging)
    for (uint32_t it = 0; it < (1u << 16); ++it) {
      bool miss = false;
#pragma unroll
      for (int k = 0; k < kPer; ++k) miss = miss || m[k] == kSlotUnset || x[k] == kSlotUnset;
      if (!miss) break;
      __builtin_amdgcn_s_sleep(2);
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const uint32_t t = t0 + (uint32_t)k * nt + threadIdx.x;
        if (m[k] == kSlotUnset) m[k] = ld_sc1(a.smeta + t);
        if (x[k] == kSlotUnset) x[k] = ld_sc1(a.smeta + kSmallSlots + t);
      }
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      if (m[k] == kSlotUnset || x[k] == kSlotUnset) {
        bad = true;
        m[k] = 3ull << 19;
        x[k] = 0ull;
      }
      pin += (uint32_t)x[k];
      if (!meta_empty(m[k])) {
        const uint32_t cc = (uint32_t)(x[k] >> 32);
        pcs += cc;
        if (out.key) pout += alg_bytes((int)((m[k] >> 19) & 3u), cc, (uint32_t)(m[k] >> 40) & 0xFFFFu) + 16;
      }
    }
    uint32_t pre[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint64_t b = __ballot(!meta_empty(m[k]));
      pre[k] = mbcnt64(b);
      if (lane == 0) rowtot[k][wv] = (uint32_t)__popcll(b);
    }
    __syncthreads();
    uint32_t rb = base;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t w0 = rowtot[k][0], w1 = rowtot[k][1], w2 = rowtot[k][2], w3 = rowtot[k][3];
      const uint32_t before = (wv > 0 ? w0 : 0u) + (wv > 1 ? w1 : 0u) + (wv > 2 ? w2 : 0u);
      const uint32_t r = rb + before + pre[k], t = t0 + (uint32_t)k * nt + threadIdx.x;
      rb += w0 + w1 + w2 + w3;
      if (t >= E) continue;
      const bool e = meta_empty(m[k]);
      xpos[t] = r | (e ? kXposEmpty : 0u);
      if (e || !out.key) continue;
      out.key[r] = (uint16_t)(m[k] >> 24);
      out.type[r] = (uint8_t)((m[k] >> 19) & 3u);
      out.card[r] = meta_cw(m[k]);
      out.nruns[r] = (uint16_t)(m[k] >> 40);
      out.off[r] = (uint64_t)t * kBitmapBytes;
    }
    base = rb;
    __syncthreads(); // the row totals are read; the next tile rewrites them
  }
  RBG_SS(1);
  if (a.rbegin)
    for (uint32_t p = threadIdx.x; p <= a.np; p += nt) {
      const uint32_t t = p == threadIdx.x ? slot_own : tab.slot_at(p);
      a.rbegin[p] = t < E ? xpos[t] & ~kXposEmpty : base;
    }
  RBG_SS(2);
  if (a.pcard) // per-pair result cardinality (RoaringBitmap.andCardinality etc.)
    for (uint32_t p = threadIdx.x; p < a.np; p += nt) {
      uint64_t c = 0;
      for (uint32_t t = tab.slot_at(p), te = tab.slot_at(p + 1); t < te; ++t) {
        const uint64_t m = ld_sc1(a.smeta + t);
        if (!meta_empty(m)) c += m & 0x1FFFFu;
      }
      a.pcard[p] = c;
    }
  // the result words to host memory by one thread, then the call's sequence number with a system-scope
  // release: the host may return as soon as it reads that number (pairwise_small), before the kernel's
  // end is signalled
  uint64_t *vs = reinterpret_cast<uint64_t *>(wtot);
  RBG_SS(3);
  __syncthreads(); // wtot's last readers (the scans) are done
  {
    const uint64_t s0 = wave_sum_u64(pin + pkey), s1 = wave_sum_u64(pkey), s2 = wave_sum_u64(pout), s3 = wave_sum_u64(pcs);
    if (lane == 0) {
      vs[4 * wv] = s0;
      vs[4 * wv + 1] = s1;
      vs[4 * wv + 2] = s2;
      vs[4 * wv + 3] = s3;
    }
  }
  const bool fail = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    __hip_atomic_store(a.ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); // ready for the next call
    if (!fail) {
      for (int k = 0; k < 4; ++k) {
        uint64_t t = 0;
        for (uint32_t w = 0; w < (nt >> 6); ++w) t += vs[4 * w + k];
        a.hout[1 + k] = t;
      }
      a.hout[0] = base;
      // the words are host memory (fine-grained: no device cache holds them), so their stores done is all the host
      // needs before the number; a system-scope release would also write this XCD's L2 back, where the other
      // blocks' payload stores may still be landing (+1.7 us on census; the payloads reach a consumer through the
      // stream, wait_call_seq)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.hout + 5, a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    RBG_SS(4);
  }
  // the slot words back to kSlotUnset for the next call, after the hand-off (the next kernel on the stream starts
  // after this one ends; after a failed call the host resets them, seq_end)
  if (!fail)
    for (uint32_t t = threadIdx.x; t < E; t += nt) {
      a.smeta[t] = kSlotUnset;
      a.smeta[kSmallSlots + t] = kSlotUnset;
    }
}

// Dynamic LDS of k_pair_small: per wave an 8 KiB scratch, then the merged-key list, the keys, the match
// prefix and the work order, each sized by the batch's largest na + nb (kmax).
constexpr int kSmallLdsMax = 96 * 1024; // >= small_lds_bytes(4, kSmallPairKeys) (~64 KiB), beside the static LDS
// (All LDS of the kernel is in the dynamic region, whose base stays 16-B aligned — the 8 KiB scratch
// takes 16-B accesses.)
__host__ __device__ constexpr uint32_t small_lds_bytes(uint32_t waves, uint32_t kmax) {
  return waves * 8192u + 256u + 4u * kmax + 2u * kmax + 2u * (kmax + 1) + 2u * kmax + 16u;
}
#ifndef RBG_SMALL_ONE_STAGE
#define RBG_SMALL_ONE_STAGE 1 // study builds: 0 inlines the staging code once per operand
#endif
constexpr int kSmallWaves = 2; // waves per SIMD of the small-batch kernel (the register path takes ~235 VGPRs; 3 and 4 spill)
template <int OP, bool CARD_ONLY, class Tab>
__global__ __launch_bounds__(256, kSmallWaves) void k_pair_small(SmallPairArgs a, uint32_t kmax, Tab tab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
  __shared__ uint32_t s_last;
#if RBG_SMALL_STUDY
  __shared__ uint64_t s_t[8];
  __shared__ uint32_t s_keys[4];
  __shared__ uint64_t s_slow[4][3];
  if (threadIdx.x == 0) s_t[0] = __builtin_amdgcn_s_memrealtime();
#endif
  const uint32_t nw = blockDim.x >> 6;
  uint32_t *wtot = reinterpret_cast<uint32_t *>(dyn_lds + nw * 8192u); // [64] block-scan wave totals / row totals
  uint32_t *ent = wtot + 64; // merged key: A index | B index << 16
  uint16_t *K = reinterpret_cast<uint16_t *>(ent + kmax);             // A's keys, then B's
  uint16_t *mpref = K + kmax;                                          // matched keys among A[0, i)
  uint16_t *ord = mpref + kmax + 1;                                    // merged positions in work order
  const int lane = lane_id(), wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // the block's pair and rank within it: the last pair whose first block is <= blockIdx.x (the host's
  // per-pair block prefix; small_pair_nsub blocks per pair)
  uint32_t p = 0;
  {
    // 64 probes per round, one per lane (a binary search was ~8 dependent loads of the table, the first step of
    // every block's critical path: profiles/r06/small): the probes increase with the lane, so the lanes whose
    // probe passes are a prefix
    uint32_t lo = 0, hi = a.np; // blk_at(lo) <= blockIdx.x < blk_at(hi)
    while (hi - lo > 1) {
      const uint32_t span = hi - lo;
      const uint32_t q = lo + (uint32_t)(((uint64_t)span * (uint32_t)(lane + 1)) / 65u); // in [lo, hi)
      const bool le = q > lo && tab.blk_at(q) <= blockIdx.x;
      const uint64_t m = __ballot(le), gt = __ballot(q > lo && !le);
      const uint32_t nlo = m ? (uint32_t)readlane(q, 63 - __builtin_clzll(m)) : lo;
      const uint32_t nhi = gt ? (uint32_t)readlane(q, __builtin_ctzll(gt)) : hi;
      lo = nlo;
      hi = nhi;
    }
    p = lo;
  }
  const uint32_t sub = blockIdx.x - tab.blk_at(p), nsub = tab.blk_at(p + 1) - tab.blk_at(p), nt = blockDim.x;
  const bool ident = tab.same(p); // x1.op(x1) in place
  const uint64_t i0 = tab.a0(p), j0 = tab.b0(p);
  const uint32_t na = tab.counts(p) & 0xFFFFu, nb = tab.counts(p) >> 16;
#ifndef RBG_SMALL_TICKET
#define RBG_SMALL_TICKET 0 // study builds: 1 elects the compaction block by a start ticket instead of the last block id
#endif
#if RBG_SMALL_TICKET
  // the block's start ticket (the compaction's election, below), its round trip beside the key loads'
  uint64_t tk = 0;
  if (threadIdx.x == 0) tk = __hip_atomic_fetch_add(a.ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
  for (uint32_t t = threadIdx.x; t < na; t += nt) K[t] = a.A.key[i0 + t];
  for (uint32_t t = threadIdx.x; t < nb; t += nt) K[na + t] = a.B.key[j0 + t];
#if RBG_SMALL_TICKET
  if (threadIdx.x == 0) s_last = tk == a.nblocks - 1ull;
#else
  if (threadIdx.x == 0) s_last = blockIdx.x == gridDim.x - 1;
#endif
  __syncthreads();
  const uint16_t *KA = K, *KB = K + na;
  // ---- merged key order (RoaringBitmap.and/or/xor/andNot key loops, RoaringBitmap.java:377-473,
  //      860-902, 1071-1118): A[i] lands at i + #B below it - #matches below it
  const uint32_t per = (na + nt - 1) / nt, lo = min(threadIdx.x * per, na), hi = min(lo + per, na);
  uint32_t cnt = 0;
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t lb = lower_bound_u16(KB, nb, KA[i]);
    cnt += lb < nb && KB[lb] == KA[i];
  }
  uint32_t matches;
  uint32_t base = block_xscan(cnt, wtot, matches);
  for (uint32_t i = lo; i < hi; ++i) {
    const uint32_t lb = lower_bound_u16(KB, nb, KA[i]);
    const bool m = lb < nb && KB[lb] == KA[i];
    mpref[i] = (uint16_t)base;
    ent[i + lb - base] = i | ((m ? lb : 0xFFFFu) << 16);
    base += m;
  }
  if (threadIdx.x == 0) mpref[na] = (uint16_t)matches;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < nb; j += nt) {
    const uint32_t la = lower_bound_u16(KA, na, KB[j]);
    if (la < na && KA[la] == KB[j]) continue;
    ent[j + la - mpref[la]] = 0xFFFFu | (j << 16);
  }
  __syncthreads();
  const uint32_t nu = na + nb - matches;
  // ---- work order: the matched keys first (each takes the register path, the costly kind), then the rest,
  //      dealt to the pair's waves back and forth (below), so a matched key rarely waits behind another
  //      (census: a pair of 55 matched keys among 66 had two waves with two of them)
  {
    const uint32_t per2 = (nu + nt - 1) / nt, e0 = min(threadIdx.x * per2, nu), e1 = min(e0 + per2, nu);
    uint32_t mc = 0;
    for (uint32_t e = e0; e < e1; ++e) mc += (ent[e] & 0xFFFFu) != 0xFFFFu && (ent[e] >> 16) != 0xFFFFu;
    uint32_t mtot;
    uint32_t mb = block_xscan(mc, wtot, mtot), ub = e0 - mb;
    for (uint32_t e = e0; e < e1; ++e) {
      if ((ent[e] & 0xFFFFu) != 0xFFFFu && (ent[e] >> 16) != 0xFFFFu) ord[mb++] = (uint16_t)e;
      else ord[mtot + ub++] = (uint16_t)e;
    }
    __syncthreads();
  }
  // ---- one wave per merged key
#if RBG_SMALL_STUDY
  if (threadIdx.x == 0) s_t[1] = __builtin_amdgcn_s_memrealtime();
  uint32_t st_keys = 0;
  uint64_t sl_dur = 0, sl_d1 = 0, sl_d2 = 0;
#endif
  uint32_t *s = reinterpret_cast<uint32_t *>(dyn_lds) + wv * 2048;
  const uint32_t slot0 = tab.slot_at(p), slot1 = tab.slot_at(p + 1);
  // slots past the merged keys hold nothing
  if (sub == 0)
    for (uint32_t t = slot0 + nu + threadIdx.x; t < slot1; t += nt) {
      st_sc1(a.smeta + t, 3ull << 19);
      st_sc1(a.smeta + kSmallSlots + t, 0ull);
    }
  const uint32_t gw = nw * sub + wv, W = nw * nsub; // this wave among the pair's
  for (uint32_t k = 0; k * W < nu; ++k) {
    const uint32_t pos = (k & 1) ? (k + 1) * W - 1 - gw : k * W + gw;
    if (pos >= nu) continue;
    const uint32_t e = ord[pos];
#if RBG_SMALL_STUDY
    ++st_keys;
    const uint64_t st_k0 = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t en = ent[e], ia = en & 0xFFFF, ib = en >> 16;
    const bool has_a = ia != 0xFFFFu, has_b = ib != 0xFFFFu;
    const uint32_t kkey = has_a ? KA[ia] : KB[ib];
    const uint64_t slot = (uint64_t)slot0 + e;
    uint8_t *dst = a.arena + slot * kBitmapBytes;
    int ty = kEmpty, c = 0, nr = 0;
    uint32_t cw = 0xFFFFFFFFu; // the card word to store when it is not c (priorityqueue_or's lazy marks)
    // the key's slot word and its aux word (input bytes | card << 32), by lane 0, BEFORE the key's payload
    // stores: issued after them, the words (and the compaction polling for them) would wait for those stores
    auto publish = [&](int ty_, uint32_t c_, uint32_t nr_, uint32_t cw_, uint32_t inb_) {
      if (lane == 0) {
        st_sc1(a.smeta + slot, small_meta(kkey, ty_, cw_ != 0xFFFFFFFFu ? cw_ : c_, nr_));
        st_sc1(a.smeta + kSmallSlots + slot, (uint64_t)inb_ | ((uint64_t)c_ << 32));
      }
    };
    if (RBG_SMALL_MERGE && has_a && has_b && !ident && a.A.type[i0 + ia] == kArray &&
        a.B.type[j0 + ib] == kArray && !(OP == RB_OR && a.lazy) && a.A.card[i0 + ia] + a.B.card[j0 + ib] <= kMergeMax) {
      // two Arrays: the merge (merge_run), an Array result
      const uint64_t xa = i0 + ia, xb = j0 + ib;
      const uint32_t ca = a.A.card[xa], cb = a.B.card[xb];
      const uint32_t kin = (uint32_t)(alg_bytes(kArray, ca, 0) + alg_bytes(kArray, cb, 0) + 32);
      RBG_MT(5);
      {
        uint4 q[8], r[8];
        load_chunks(q, a.A.payload + a.A.off[xa], 2u * ca, lane);
        load_chunks(r, a.B.payload + a.B.off[xb], 2u * cb, lane);
        merge_stage(q, ca, r, cb, s, lane);
      }
      auto mty = [&](uint32_t n) { return n || (OP == RB_XOR && a.keep_empty && !CARD_ONLY) ? (int)kArray : (int)kEmpty; };
      c = (int)merge_run<OP, !CARD_ONLY>(s, ca, cb, reinterpret_cast<uint16_t *>(dst), lane,
                                         [&](uint32_t n) { publish(mty(n), n, 0u, 0xFFFFFFFFu, kin); });
      RBG_MT(6);
      ty = mty((uint32_t)c);
    } else if (has_a && has_b && !ident) {
      const uint64_t xa = i0 + ia, xb = j0 + ib;
      const int ta = a.A.type[xa], tb = a.B.type[xb];
      const uint32_t ca = a.A.card[xa], cb = a.B.card[xb], ra = a.A.nruns[xa], rb = a.B.nruns[xb];
      const uint8_t *pa = a.A.payload + a.A.off[xa], *pb = a.B.payload + a.B.off[xb];
      const uint32_t ba = (uint32_t)payload_bytes(ta, ca, ra), bb = (uint32_t)payload_bytes(tb, cb, rb);
      const uint32_t kin = (uint32_t)(alg_bytes(ta, ca, ra) + alg_bytes(tb, cb, rb) + 32);
      uint64_t w[kW];
#if RBG_SMALL_ONE_STAGE
      // both operands through ONE copy of the staging code (a loop of two): this kernel's code (82 KB, of which
      // each staging copy ~17 KB) outgrew the instruction cache, and its misses sat on the slowest keys' path
      // (SQC_ICACHE_MISSES, profiles/r06/small)
#pragma unroll 1
      for (int side = 0; side < 2; ++side) {
        const int t = side ? tb : ta;
        const uint32_t c_ = side ? cb : ca, r_ = side ? rb : ra, b_ = side ? bb : ba;
        const uint8_t *p_ = side ? pb : pa;
        uint4 q[8];
        if (bitmap_payload(t, c_)) {
          load_chunks(q, p_, kBitmapBytes, lane);
        } else {
          if (b_ > (uint32_t)kBitmapBytes) stage_big_runs(p_, r_, s, lane);
          else {
            load_chunks(q, p_, b_, lane);
            stage_from_chunks(t, q, c_, r_, s, lane);
          }
          const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
#pragma unroll
          for (int k = 0; k < 8; ++k) q[k] = s4[k * 64 + lane];
          wave_lds_sync();
        }
        if (side == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            w[2 * k] = pack2(q[k].x, q[k].y);
            w[2 * k + 1] = pack2(q[k].z, q[k].w);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            word_op<OP>(w[2 * k], pack2(q[k].x, q[k].y));
            word_op<OP>(w[2 * k + 1], pack2(q[k].z, q[k].w));
          }
        }
      }
#else
      uint4 q[8];
      if (bitmap_payload(ta, ca)) {
        load_bitmap(pa, w, lane);
      } else {
        if (ba > (uint32_t)kBitmapBytes) stage_big_runs(pa, ra, s, lane);
        else {
          load_chunks(q, pa, ba, lane);
          stage_from_chunks(ta, q, ca, ra, s, lane);
        }
        lds_read_words(s, w, lane);
        wave_lds_sync();
      }
      if (bitmap_payload(tb, cb)) {
        load_chunks(q, pb, kBitmapBytes, lane);
      } else {
        if (bb > (uint32_t)kBitmapBytes) stage_big_runs(pb, rb, s, lane);
        else {
          load_chunks(q, pb, bb, lane);
          stage_from_chunks(tb, q, cb, rb, s, lane);
        }
        const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = s4[k * 64 + lane];
        wave_lds_sync();
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        word_op<OP>(w[2 * k], pack2(q[k].x, q[k].y));
        word_op<OP>(w[2 * k + 1], pack2(q[k].z, q[k].w));
      }
#endif
      const bool lazy = OP == RB_OR && a.lazy;
      const bool eff = eff_rule<OP>(ta, tb, ca, cb);
      int r;
      metrics(w, lane, (eff || (lazy && (ta == kRun || tb == kRun))) && !CARD_ONLY, c, r);
      bool bits = false;
      if (lazy) {
        ty = lazy_or_type(a.lazy, ta, tb, ca, cb, c, r, cw, bits);
        if (ty == kRun && c == kSpan) r = 1;
      } else if (OP != RB_OR && c == 0 && !(OP == RB_XOR && a.keep_empty)) ty = kEmpty;
      else if (eff) ty = type_eff(c, r);
      else if (OP == RB_OR && a.inplace && ta == kBitmap && tb == kArray) {
        ty = kBitmap; // BitmapContainer.ior(ArrayContainer) returns this, full or not (BitmapContainer.java:749-766)
      } else if (OP == RB_OR && (ta == kBitmap || tb == kBitmap)) {
        ty = type_lr(c);
        if (ty == kRun) r = 1; // LR's Run is the full container: one run
      } else ty = type_ab(c);
      if (CARD_ONLY) ty = c ? kArray : kEmpty;
      nr = ty == kRun ? r : 0;
      publish(ty, (uint32_t)c, (uint32_t)nr, cw, kin);
      if (!CARD_ONLY && ty != kEmpty) emit_container(bits ? (int)kBitmap : ty, w, c, r, dst, s, lane);
    } else if (ident ? (OP == RB_AND || OP == RB_OR) : has_a ? keeps_a_only(OP) : keeps_b_only(OP)) {
      // x.and(x) / x.or(x) in place leave x's own containers
      // unmatched key: RoaringArray.appendCopy (RoaringArray.java:184-205)
      const SetView &S = has_a ? a.A : a.B;
      const uint64_t x = has_a ? i0 + ia : j0 + ib;
      const int sty = S.type[x];
      c = (int)S.card[x];
      nr = S.nruns[x];
      ty = CARD_ONLY ? (int)kArray : sty;
      publish(ty, (uint32_t)c, (uint32_t)nr, cw, (uint32_t)(alg_bytes(sty, (uint32_t)c, (uint32_t)nr) + 16));
      if (!CARD_ONLY) copy_payload(S.payload + S.off[x], dst, payload_bytes(sty, (uint32_t)c, (uint32_t)nr), lane);
    } else {
      publish(kEmpty, 0u, 0u, 0xFFFFFFFFu, 0u); // a key the op drops
    }
#if RBG_SMALL_STUDY
    {
      const uint64_t d = __builtin_amdgcn_s_memrealtime() - st_k0;
      if (d > sl_dur) {
        const uint32_t ta = has_a ? a.A.type[i0 + ia] : 3u, tb = has_b ? a.B.type[j0 + ib] : 3u;
        const uint32_t ca = has_a ? a.A.card[i0 + ia] : 0u, cb = has_b ? a.B.card[j0 + ib] : 0u;
        const uint32_t ra = has_a ? a.A.nruns[i0 + ia] : 0u, rb = has_b ? a.B.nruns[j0 + ib] : 0u;
        sl_dur = d;
        if (lane == 0) { // merge phases relative to the key's start (0 when the key took no merge)
          const uint64_t *mt = g_merge_ts[min(blockIdx.x, 8191u) * 4 + wv];
          const uint64_t tend = __builtin_amdgcn_s_memrealtime();
          g_small_study[min(blockIdx.x, 8191u) * kStudyWords + 19 + 4 * wv] =
              mt[5] >= st_k0 ? ((mt[5] - st_k0) | (mt[1] - mt[5]) << 10 | (mt[2] - mt[1]) << 20 | (mt[3] - mt[2]) << 30 |
                                (mt[4] - mt[3]) << 40 | (mt[6] - mt[4]) << 50)
                             : 0ull;
          g_small_study[min(blockIdx.x, 8191u) * kStudyWords + 31 - wv] = mt[6] >= st_k0 ? tend - mt[6] : 0ull;
        }
        sl_d1 = ta | (tb << 2) | ((uint64_t)(ty & 0xFF) << 8) | ((uint64_t)(nr & 0xFFFF) << 16) | ((uint64_t)(uint32_t)c << 32);
        sl_d2 = (uint64_t)ca | ((uint64_t)cb << 20) | ((uint64_t)(ra & 0xFFF) << 40) | ((uint64_t)(rb & 0xFFF) << 52);
      }
    }
#endif
  }
#if RBG_SMALL_STUDY
  if (lane == 0) {
    s_keys[wv] = st_keys;
    s_t[2 + wv] = __builtin_amdgcn_s_memrealtime();
    s_slow[wv][0] = sl_dur;
    s_slow[wv][1] = sl_d1;
    s_slow[wv][2] = sl_d2;
  }
#endif
  // ---- the last block compacts (s_last; RBG_SMALL_TICKET: the last to start): it is the only block that waits,
  //      and the blocks it waits for wait on nothing, so they finish whatever the dispatch order (its polls are
  //      bounded besides); the others just end, their payload stores in flight (nothing in the launch reads a
  //      payload; the stream contract covers the rest, wait_call_seq)
#if RBG_SMALL_STUDY
  __syncthreads();
  uint64_t *gs = g_small_study + (uint64_t)min(blockIdx.x, 8191u) * kStudyWords;
  if (threadIdx.x == 0) {
    gs[0] = s_t[0];
    gs[1] = s_t[1];
    for (int w = 0; w < 4; ++w) gs[2 + w] = s_t[2 + w];
    for (int w = 0; w < 4; ++w) gs[6 + w] = s_keys[w];
    gs[10] = __builtin_amdgcn_s_memrealtime();
    gs[11] = 0;
    gs[12] = p;
    gs[13] = sub | ((uint64_t)nsub << 32);
    gs[14] = nu;
    gs[15] = s_last;
    for (int w = 0; w < 4; ++w) {
      gs[16 + 4 * w] = s_slow[w][0];
      gs[17 + 4 * w] = s_slow[w][1];
      gs[18 + 4 * w] = s_slow[w][2];
    }
  }
#else
  if (!s_last) return;
  __syncthreads(); // the block's waves are past their scratch use
#endif
  if (!s_last) return;
  small_compact(a, tab, reinterpret_cast<uint32_t *>(dyn_lds), wtot);
#if RBG_SMALL_STUDY
  __syncthreads();
  if (threadIdx.x == 0) gs[11] = __builtin_amdgcn_s_memrealtime();
#endif
}
#if RBG_SMALL_STUDY
} // namespace rbg
extern "C" int rbgpu_internal_small_study(uint64_t *host, uint64_t words) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(rbg::g_small_study), words * 8) == hipSuccess ? 0 : -1;
}
namespace rbg {
#endif

template <int OP, bool CARD_ONLY, class Tab>
static void launch_small_tab(const SmallPairArgs &a, const Tab &tab, unsigned waves, unsigned nblocks, uint32_t kmax,
                             hipStream_t st) {
  static bool attr = false; // allow more than the default 64 KiB of dynamic LDS
  if (!attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pair_small<OP, CARD_ONLY, Tab>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, kSmallLdsMax) != hipSuccess)
      (void)hipGetLastError(); // (the launch reports a real failure)
    attr = true;
  }
  // the compaction's LDS map of E <= kSmallXposLds slots fits the waves' scratch (4 x 8 KiB)
  static_assert(kSmallXposLds * 4 <= 4 * 8192, "slot map inside the scratch");
  static_assert(small_lds_bytes(4, kSmallPairKeys) <= kSmallLdsMax, "LDS of the largest small batch");
  k_pair_small<OP, CARD_ONLY, Tab><<<nblocks, 64 * waves, small_lds_bytes(waves, kmax), st>>>(a, kmax, tab);
}
template <int OP>
static void launch_small_op(bool card_only, const SmallPairArgs &a, const SmallTabInline *inl, const SmallTabDev &dev,
                            unsigned waves, unsigned nblocks, uint32_t kmax, hipStream_t st) {
  if (inl) {
    if (card_only) launch_small_tab<OP, true>(a, *inl, waves, nblocks, kmax, st);
    else launch_small_tab<OP, false>(a, *inl, waves, nblocks, kmax, st);
  } else {
    if (card_only) launch_small_tab<OP, true>(a, dev, waves, nblocks, kmax, st);
    else launch_small_tab<OP, false>(a, dev, waves, nblocks, kmax, st);
  }
}
unsigned small_resident_blocks() { return 2 * cu_count(); }
// The call is latency-bound (a wave's merged keys run one after the other): 4 waves per block and
// enough blocks per pair that each wave takes ~1 merged key — sized per pair (small_pair_nsub), so a
// batch of small pairs with one large pair launches no idle blocks for the small ones (census: a
// uniform 10 blocks per pair left ~60 % of the waves without a key after the alignment) — but no more
// than run at once: a second round of blocks starts only as the first ends (census, 812 blocks: the
// last started 11 us in), so the host doubles the keys per wave until the blocks fit.
void launch_pair_small(int op, bool card_only, const SmallPairArgs &a, const SmallTabInline *inl,
                       const SmallTabDev &dev, uint32_t max_keys, uint32_t nblocks, hipStream_t st) {
  if (!a.np) return;
  const uint32_t kmax = std::max(1u, max_keys);
  const unsigned waves = 4;
  switch (op) {
  case RB_AND: launch_small_op<RB_AND>(card_only, a, inl, dev, waves, nblocks, kmax, st); break;
  case RB_OR: launch_small_op<RB_OR>(card_only, a, inl, dev, waves, nblocks, kmax, st); break;
  case RB_XOR: launch_small_op<RB_XOR>(card_only, a, inl, dev, waves, nblocks, kmax, st); break;
  default: launch_small_op<RB_ANDNOT>(card_only, a, inl, dev, waves, nblocks, kmax, st); break;
  }
}

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_pairwise() {}
void warm_pairwise(hipStream_t st) { k_warm_pairwise<<<1, 64, 0, st>>>(); }

} // namespace rbg
