// pairwise.hip — batched static RoaringBitmap.and/or/xor/andNot on MI355X.
//
// Pipeline (one HIP stream):
//   k_pair_count   thread per pair: merge the two sorted u16 key lists (RoaringBitmap.and/or/
//                  xor/andNot key loops, RoaringBitmap.java:377-473, 860-902, 1071-1118) and
//                  count result slots + an output-byte bound per slot;
//   scans          exclusive prefix sums -> task index and arena offset of every slot;
//   k_pair_emit    thread per pair: write the task list in result (key) order;
//   k_pairwise     ONE WAVE PER TASK: both containers -> 65536-bit register bitmaps, word op,
//                  card + maximal runs, reference type decision, coalesced emission;
//   k_compact_*    drop empty results (isEmpty, RoaringBitmap.java:389-391 etc.) and build
//                  the result CSR.
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

constexpr int kPairThreads = 256;

__device__ __forceinline__ bool keeps_a_only(int op) { return op != RB_AND; }
__device__ __forceinline__ bool keeps_b_only(int op) { return op == RB_OR || op == RB_XOR; }

// algorithmic payload bytes: Bitmap 8192, Array 2c, Run 4r+2
__device__ __forceinline__ uint64_t alg_bytes(int t, uint32_t c, uint32_t r) {
  return t == kBitmap ? 8192ull : t == kArray ? 2ull * c : 4ull * r + 2;
}

// Upper bound of the result payload of a matched pair: every reference result type fits in
// 2*cmax bytes when cmax <= 4096 (Array 2c; a Run is only chosen when 4r+2 <= 2c+2), and in
// one 8 KiB slot otherwise.
__device__ __forceinline__ void matched_bound(int op, uint32_t ca, uint32_t cb, bool &big, uint64_t &bytes) {
  uint32_t cmax = op == RB_AND ? min(ca, cb) : op == RB_ANDNOT ? ca : ca + cb;
  big = 2ull * cmax >= (uint64_t)kBitmapBytes;
  bytes = big ? 0 : round16(2ull * cmax);
}
__device__ __forceinline__ void copy_bound(const SetView &S, uint64_t i, bool &big, uint64_t &bytes) {
  int t = S.type[i];
  big = t == kBitmap;
  bytes = big ? 0 : round16(payload_bytes(t, S.card[i], S.nruns[i]));
}

template <bool EMIT>
__device__ __forceinline__ void pair_walk(const PairArgs &a, uint32_t p, uint64_t &nt, uint64_t &nb, uint64_t &sm,
                                          uint64_t &inb, Task *tasks, uint16_t *tkey, uint64_t big_base_idx,
                                          uint64_t small_off) {
  const uint32_t ai = a.aidx ? a.aidx[p] : p, bi = a.bidx ? a.bidx[p] : p;
  uint64_t i = a.A.begin[ai], i1 = a.A.begin[ai + 1], j = a.B.begin[bi], j1 = a.B.begin[bi + 1];
  inb += 2 * ((i1 - i) + (j1 - j));
  auto slot = [&](int64_t ia, int64_t ib, uint16_t key, bool big, uint64_t bytes) {
    if (EMIT) {
      Task t;
      t.ia = (int32_t)ia;
      t.ib = (int32_t)ib;
      t.out = big ? (big_base_idx + nb) * (uint64_t)kBitmapBytes : small_off + sm;
      tasks[nt] = t;
      tkey[nt] = key;
    }
    ++nt;
    if (big) ++nb;
    else sm += bytes;
  };
  bool big;
  uint64_t bytes;
  while (i < i1 && j < j1) {
    uint16_t ka = a.A.key[i], kb = a.B.key[j];
    if (ka == kb) {
      matched_bound(a.op, a.A.card[i], a.B.card[j], big, bytes);
      if (!EMIT)
        inb += alg_bytes(a.A.type[i], a.A.card[i], a.A.nruns[i]) + alg_bytes(a.B.type[j], a.B.card[j], a.B.nruns[j]) + 32;
      slot((int64_t)i, (int64_t)j, ka, big, bytes);
      ++i;
      ++j;
    } else if (ka < kb) {
      if (keeps_a_only(a.op)) {
        copy_bound(a.A, i, big, bytes);
        if (!EMIT) inb += alg_bytes(a.A.type[i], a.A.card[i], a.A.nruns[i]) + 16;
        slot((int64_t)i, -1, ka, big, bytes);
      }
      ++i;
    } else {
      if (keeps_b_only(a.op)) {
        copy_bound(a.B, j, big, bytes);
        if (!EMIT) inb += alg_bytes(a.B.type[j], a.B.card[j], a.B.nruns[j]) + 16;
        slot(-1, (int64_t)j, kb, big, bytes);
      }
      ++j;
    }
  }
  if (keeps_a_only(a.op))
    for (; i < i1; ++i) {
      copy_bound(a.A, i, big, bytes);
      if (!EMIT) inb += alg_bytes(a.A.type[i], a.A.card[i], a.A.nruns[i]) + 16;
      slot((int64_t)i, -1, a.A.key[i], big, bytes);
    }
  if (keeps_b_only(a.op))
    for (; j < j1; ++j) {
      copy_bound(a.B, j, big, bytes);
      if (!EMIT) inb += alg_bytes(a.B.type[j], a.B.card[j], a.B.nruns[j]) + 16;
      slot(-1, (int64_t)j, a.B.key[j], big, bytes);
    }
}

__global__ __launch_bounds__(kPairThreads) void k_pair_count(PairArgs a, uint64_t *ntask, uint64_t *nbig,
                                                             uint64_t *small, uint64_t *stats) {
  const uint32_t p = blockIdx.x * kPairThreads + threadIdx.x;
  uint64_t nt = 0, nb = 0, sm = 0, inb = 0;
  if (p < a.npairs) {
    pair_walk<false>(a, p, nt, nb, sm, inb, nullptr, nullptr, 0, 0);
    ntask[p] = nt;
    nbig[p] = nb;
    small[p] = sm;
  }
  uint64_t w = wave_sum_u64(inb);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd((unsigned long long *)&stats[0], (unsigned long long)w);
}

__global__ __launch_bounds__(kPairThreads) void k_pair_emit(PairArgs a, const uint64_t *task_begin,
                                                            const uint64_t *big_begin, const uint64_t *small_begin,
                                                            uint64_t small_base, Task *tasks, uint16_t *tkey) {
  const uint32_t p = blockIdx.x * kPairThreads + threadIdx.x;
  if (p >= a.npairs) return;
  uint64_t nt = 0, nb = 0, sm = 0, inb = 0;
  pair_walk<true>(a, p, nt, nb, sm, inb, tasks + task_begin[p], tkey + task_begin[p], big_begin[p],
                  small_base + small_begin[p]);
}

// ---------------------------------------------------------------- the per-task kernel
// Result type of a matched pair (derived from the container implementations):
//   AND:    R&R -> EFF, else AB                      (RunContainer.java:381-456; BitmapContainer.java:162-188)
//   OR:     any Bitmap -> LR, A|A -> AB, else EFF     (BitmapContainer.java:1073-1110; RunContainer.java:1926-1986;
//                                                      ArrayContainer.java:949-973)
//   XOR:    R^R, R^A(|A|<32) -> EFF, else AB         (RunContainer.java:2410-2482; ArrayContainer.java:1311-1336)
//   ANDNOT: R\R, R\A(|A|<32) -> EFF, else AB         (RunContainer.java:574-692; BitmapContainer.java:221-274)
template <int OP, bool CARD_ONLY>
__global__ __launch_bounds__(256) void k_pairwise(SetView A, SetView B, const Task *__restrict__ tasks,
                                                  uint64_t ntasks, uint8_t *__restrict__ out, TaskMeta tm) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[4][2048];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t t = (uint64_t)blockIdx.x * 4 + wv;
  if (t >= ntasks) return;
  uint32_t *s = lds[wv];
  const int32_t ia = __builtin_amdgcn_readfirstlane(tasks[t].ia);
  const int32_t ib = __builtin_amdgcn_readfirstlane(tasks[t].ib);
  const uint64_t o = tasks[t].out;
  if (ia < 0 || ib < 0) { // unmatched container: cloned unchanged (RoaringArray.appendCopy :184-205)
    const SetView &S = ia >= 0 ? A : B;
    const int64_t i = ia >= 0 ? ia : ib;
    const int ty = S.type[i];
    const uint32_t c = S.card[i], nr = S.nruns[i];
    if (!CARD_ONLY) copy_payload(S.payload + S.off[i], out + o, payload_bytes(ty, c, nr), lane);
    if (lane == 0) {
      tm.type[t] = (uint8_t)ty;
      tm.card[t] = c;
      tm.nruns[t] = (uint16_t)nr;
    }
    return;
  }
  const int ta = A.type[ia], tb = B.type[ib];
  const uint32_t ca = A.card[ia], cb = B.card[ib];
  uint64_t wa[kW], wb[kW];
  load_container(ta, A.payload + A.off[ia], ca, A.nruns[ia], s, wa, lane);
  load_container(tb, B.payload + B.off[ib], cb, B.nruns[ib], s, wb, lane);
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    if (OP == RB_AND) wa[j] &= wb[j];
    else if (OP == RB_OR) wa[j] |= wb[j];
    else if (OP == RB_XOR) wa[j] ^= wb[j];
    else wa[j] &= ~wb[j];
  }
  bool eff;
  if (OP == RB_AND) eff = ta == kRun && tb == kRun;
  else if (OP == RB_OR) eff = ta != kBitmap && tb != kBitmap && !(ta == kArray && tb == kArray);
  else if (OP == RB_XOR)
    eff = (ta == kRun && tb == kRun) || (ta == kArray && tb == kRun && ca < (uint32_t)kRunArrayThreshold) ||
          (ta == kRun && tb == kArray && cb < (uint32_t)kRunArrayThreshold);
  else eff = (ta == kRun && tb == kRun) || (ta == kRun && tb == kArray && cb < (uint32_t)kRunArrayThreshold);
  int c, r;
  metrics(wa, lane, eff && !CARD_ONLY, c, r);
  int ty;
  if (OP != RB_OR && c == 0) ty = kEmpty;
  else if (eff) ty = type_eff(c, r);
  else if (OP == RB_OR && (ta == kBitmap || tb == kBitmap)) {
    ty = type_lr(c);
    if (ty == kRun) r = 1; // LR's Run is the full container: one run
  } else ty = type_ab(c);
  if (CARD_ONLY) {
    if (lane == 0) {
      tm.type[t] = c ? (uint8_t)kArray : kEmpty;
      tm.card[t] = (uint32_t)c;
      tm.nruns[t] = 0;
    }
    return;
  }
  if (ty != kEmpty) emit_container(ty, wa, c, r, out + o, s, lane);
  if (lane == 0) {
    tm.type[t] = (uint8_t)ty;
    tm.card[t] = (uint32_t)c;
    tm.nruns[t] = (uint16_t)(ty == kRun ? r : 0);
  }
}

// ---------------------------------------------------------------- compaction
__global__ __launch_bounds__(kPairThreads) void k_compact_count(const uint64_t *tb, uint32_t npairs,
                                                                const uint8_t *ttype, uint64_t *cnt) {
  const uint32_t p = blockIdx.x * kPairThreads + threadIdx.x;
  if (p >= npairs) return;
  uint64_t n = 0;
  for (uint64_t t = tb[p]; t < tb[p + 1]; ++t) n += ttype[t] != kEmpty;
  cnt[p] = n;
}
__global__ __launch_bounds__(kPairThreads) void k_compact_write(const uint64_t *tb, uint32_t npairs, TaskMeta tm,
                                                                const Task *tasks, const uint64_t *rbegin, OutView out,
                                                                uint64_t *pair_card, uint64_t *stats) {
  const uint32_t p = blockIdx.x * kPairThreads + threadIdx.x;
  uint64_t outb = 0;
  if (p < npairs) {
    uint64_t r = rbegin ? rbegin[p] : 0, card = 0;
    for (uint64_t t = tb[p]; t < tb[p + 1]; ++t) {
      const uint8_t ty = tm.type[t];
      if (ty == kEmpty) continue;
      card += tm.card[t];
      if (out.key) {
        out.key[r] = tm.key[t];
        out.type[r] = ty;
        out.card[r] = tm.card[t];
        out.nruns[r] = tm.nruns[t];
        out.off[r] = tasks[t].out;
        outb += alg_bytes(ty, tm.card[t], tm.nruns[t]) + 16;
      }
      ++r;
    }
    if (pair_card) pair_card[p] = card;
  }
  uint64_t w = wave_sum_u64(outb);
  if (stats && (threadIdx.x & 63) == 0 && w) atomicAdd((unsigned long long *)&stats[1], (unsigned long long)w);
}

// ---------------------------------------------------------------- launchers
static unsigned blocks_for(uint64_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

void launch_pair_count(const PairArgs &a, uint64_t *ntask, uint64_t *nbig, uint64_t *small, uint64_t *stats,
                       hipStream_t st) {
  if (!a.npairs) return;
  k_pair_count<<<blocks_for(a.npairs, kPairThreads), kPairThreads, 0, st>>>(a, ntask, nbig, small, stats);
}
void launch_pair_emit(const PairArgs &a, const uint64_t *task_begin, const uint64_t *big_begin,
                      const uint64_t *small_begin, uint64_t small_base, Task *tasks, uint16_t *task_key,
                      hipStream_t st) {
  if (!a.npairs) return;
  k_pair_emit<<<blocks_for(a.npairs, kPairThreads), kPairThreads, 0, st>>>(a, task_begin, big_begin, small_begin,
                                                                           small_base, tasks, task_key);
}
template <int OP>
static void launch_op(bool card_only, const SetView &A, const SetView &B, const Task *tasks, uint64_t ntasks,
                      uint8_t *out, const TaskMeta &tm, hipStream_t st) {
  const unsigned g = blocks_for(ntasks, 4);
  if (card_only) k_pairwise<OP, true><<<g, 256, 0, st>>>(A, B, tasks, ntasks, out, tm);
  else k_pairwise<OP, false><<<g, 256, 0, st>>>(A, B, tasks, ntasks, out, tm);
}
void launch_pairwise(int op, bool card_only, const SetView &A, const SetView &B, const Task *tasks, uint64_t ntasks,
                     uint8_t *out, const TaskMeta &tm, hipStream_t st) {
  if (!ntasks) return;
  switch (op) {
  case RB_AND: launch_op<RB_AND>(card_only, A, B, tasks, ntasks, out, tm, st); break;
  case RB_OR: launch_op<RB_OR>(card_only, A, B, tasks, ntasks, out, tm, st); break;
  case RB_XOR: launch_op<RB_XOR>(card_only, A, B, tasks, ntasks, out, tm, st); break;
  default: launch_op<RB_ANDNOT>(card_only, A, B, tasks, ntasks, out, tm, st); break;
  }
}
void launch_compact_count(const uint64_t *task_begin, uint32_t npairs, const uint8_t *ttype, uint64_t *cnt,
                          hipStream_t st) {
  if (!npairs) return;
  k_compact_count<<<blocks_for(npairs, kPairThreads), kPairThreads, 0, st>>>(task_begin, npairs, ttype, cnt);
}
void launch_compact_write(const uint64_t *task_begin, uint32_t npairs, const TaskMeta &tm, const Task *tasks,
                          const uint64_t *rbegin, const OutView &out, uint64_t *pair_card, uint64_t *stats,
                          hipStream_t st) {
  if (!npairs) return;
  k_compact_write<<<blocks_for(npairs, kPairThreads), kPairThreads, 0, st>>>(task_begin, npairs, tm, tasks, rbegin,
                                                                             out, pair_card, stats);
}

} // namespace rbg
