// bsi.hip — bit-sliced index compare (bsi module: Roaring64BitmapSliceIndex.compare /
// RoaringBitmapSliceIndex.compare, the O'Neil chains of oNeilCompare) as ONE fused pass per high key.
//
// The reference evaluates a query as ~2 static RoaringBitmap ops per slice over whole bitmaps
// (RoaringBitmapSliceIndex.java:432-472), materialising EQ / GT / LT after every slice.  Every high
// key is independent, so here ONE WAVE PER KEY walks the slices once: EQ lives in registers as a
// 65536-bit register bitmap, the GT or LT accumulator in an 8 KiB LDS image, the current slice is
// staged in a second LDS image while the next slice's payload is already in flight (registers).
// Each intermediate carries the container type the reference's static op would have produced
// (pairwise contract, SURVEY §8a: AND R&R->EFF else AB, ANDNOT R\R, R\A(|A|<32)->EFF else AB, OR any
// Bitmap->LR, A|A->AB, else EFF; absent keys: and -> absent, andNot(x, absent) -> clone x,
// or(x, absent) -> clone x; empty results dropped), so the result is byte-identical.
#include <algorithm>
#include <cstring>

#include "internal.hpp"
#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

struct Meta {
  int present, type, card, runs;
};

// table[row * 65536 + key] = container index of bitmap (first + row) at key, else -1
__global__ __launch_bounds__(256) void k_bsi_index(SetView s, uint32_t first, int32_t *table) {
  const uint32_t row = blockIdx.y;
  const uint64_t lo = s.begin[first + row], hi = s.begin[first + row + 1];
  for (uint64_t c = lo + (uint64_t)blockIdx.x * 256 + threadIdx.x; c < hi; c += (uint64_t)gridDim.x * 256)
    table[(uint64_t)row * 65536 + s.key[c]] = (int32_t)c;
}
// keys of F (ebM or foundSet) inside the shard's [key_lo, key_hi), in a per-block layout: k_bsi_active
// leaves each 256-key block's count in bt, the counts are scanned (bts, bts[256] = nk) and k_bsi_list
// places the keys
__global__ __launch_bounds__(256) void k_bsi_active(const int32_t *frow, uint32_t key_lo, uint32_t key_hi,
                                                    uint64_t *bt) {
  __shared__ uint32_t wt[4];
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  const uint32_t n = block_flag_count(frow[k] >= 0 && k >= key_lo && k < key_hi, wt);
  if (threadIdx.x == 0) bt[blockIdx.x] = n;
}
__global__ __launch_bounds__(256) void k_bsi_list(const int32_t *frow, uint32_t key_lo, uint32_t key_hi,
                                                  const uint64_t *bts, uint32_t *klist) {
  __shared__ uint32_t wt[4];
  const uint32_t k = blockIdx.x * 256 + threadIdx.x;
  const bool f = frow[k] >= 0 && k >= key_lo && k < key_hi;
  const uint32_t r = block_flag_rank(f, wt);
  if (f) klist[bts[blockIdx.x] + r] = k;
}

// ---- per-key value algebra with the reference's type rules --------------------------------
__device__ __forceinline__ uint64_t lds_word(const uint32_t *s, int j, int lane) {
  const uint2 v = reinterpret_cast<const uint2 *>(s)[(j >> 1) * 128 + 2 * lane + (j & 1)];
  return pack2(v.x, v.y);
}
__device__ __forceinline__ void lds_put_word(uint32_t *s, int j, int lane, uint64_t w) {
  reinterpret_cast<uint2 *>(s)[(j >> 1) * 128 + 2 * lane + (j & 1)] = make_uint2((uint32_t)w, (uint32_t)(w >> 32));
}
// metadata of a fresh result in w under rule `eff` (EFF) / `or_bitmap` (LR) / otherwise AB
__device__ __forceinline__ Meta classify(const uint64_t (&w)[kW], int lane, bool eff, bool lr, bool never_empty) {
  Meta m;
  int c, r;
  metrics(w, lane, eff, c, r);
  m.card = c;
  m.runs = 0;
  m.present = c > 0 || never_empty;
  if (!m.present) return m;
  if (eff) {
    m.type = type_eff(c, r);
    m.runs = m.type == kRun ? r : 0;
  } else if (lr) {
    m.type = type_lr(c);
    m.runs = m.type == kRun ? 1 : 0;
  } else {
    m.type = type_ab(c);
  }
  return m;
}
__device__ __forceinline__ bool eff_and(const Meta &a, const Meta &b) { return a.type == kRun && b.type == kRun; }
__device__ __forceinline__ bool eff_andnot(const Meta &a, const Meta &b) {
  return a.type == kRun && (b.type == kRun || (b.type == kArray && b.card < kRunArrayThreshold));
}
__device__ __forceinline__ bool lr_or(const Meta &a, const Meta &b) { return a.type == kBitmap || b.type == kBitmap; }
__device__ __forceinline__ bool eff_or(const Meta &a, const Meta &b) {
  return !lr_or(a, b) && !(a.type == kArray && b.type == kArray);
}

// Any container (global payload) -> LDS image s.
__device__ __forceinline__ Meta stage_global(const SetView &v, int32_t c, uint32_t *s, int lane) {
  Meta m{0, 0, 0, 0};
  if (c < 0) return m;
  m.present = 1;
  m.type = v.type[c];
  m.card = (int)v.card[c];
  m.runs = v.nruns[c];
  stage_container(m.type, v.payload + v.off[c], (uint32_t)m.card, (uint32_t)m.runs, s, lane);
  return m;
}

enum { kBsiEQ = 0, kBsiNEQ = 1, kBsiLE = 2, kBsiLT = 3, kBsiGE = 4, kBsiGT = 5 };

template <int FINAL>
__global__ __launch_bounds__(256, 2) void k_bsi_chain(SetView bsi, SetView fnd, int has_found,
                                                      const int32_t *__restrict__ table, uint32_t nbits, uint64_t pred,
                                                      const uint32_t *__restrict__ klist, uint32_t nk,
                                                      uint8_t *__restrict__ out, WideOut wo, uint64_t *stats) {
  constexpr int TRACK = (FINAL == kBsiGE || FINAL == kBsiGT) ? 1 : (FINAL == kBsiLE || FINAL == kBsiLT) ? 2 : 0;
  __shared__ __attribute__((aligned(16))) uint32_t lds[4][2][2048];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t q = xcd_swizzle(blockIdx.x, gridDim.x) * 4 + wv;
  if (q >= nk) return;
  uint32_t *sS = lds[wv][0], *sX = lds[wv][1];
  const uint32_t key = klist[q];
  uint64_t inb = 0;

  // EQ = ebM's container (RoaringBitmapSliceIndex.java:438: EQ = this.ebM, no copy)
  uint64_t e[kW];
  Meta eq = stage_global(bsi, table[(uint64_t)nbits * 65536 + key], sS, lane);
  if (eq.present) {
    lds_read_words(sS, e, lane);
    inb += payload_bytes(eq.type, eq.card, eq.runs) + 16;
  } else {
#pragma unroll
    for (int j = 0; j < kW; ++j) e[j] = 0;
  }
  wave_lds_sync();
  Meta x{0, 0, 0, 0};

  // slice descriptors, lane i <-> slice i (nbits <= 64)
  const int32_t sc = lane < (int)nbits ? table[(uint64_t)lane * 65536 + key] : -1;
  int st = 0;
  uint32_t scard = 0, sruns = 0;
  uint64_t soff = 0;
  if (sc >= 0) {
    st = bsi.type[sc];
    scard = bsi.card[sc];
    sruns = bsi.nruns[sc];
    soff = bsi.off[sc];
  }
  auto sbytes = [&](int i) -> uint32_t {
    const int t = (int)readlane((uint32_t)st, i);
    return (uint32_t)payload_bytes(t, readlane(scard, i), readlane(sruns, i));
  };
  auto sptr = [&](int i) -> const uint8_t * {
    return bsi.payload + pack2(readlane((uint32_t)soff, i), readlane((uint32_t)(soff >> 32), i));
  };
  uint4 pq[8];
  if (nbits) {
    const int i0 = (int)nbits - 1;
    const bool ok = (int)readlane((uint32_t)sc, i0) >= 0 && sbytes(i0) <= (uint32_t)kBitmapBytes;
    load_chunks(pq, ok ? sptr(i0) : bsi.payload, ok ? sbytes(i0) : 16u, lane);
  }
  for (int i = (int)nbits - 1; i >= 0; --i) {
    const bool spresent = (int)readlane((uint32_t)sc, i) >= 0;
    Meta sm{0, 0, 0, 0};
    if (spresent) {
      sm.present = 1;
      sm.type = (int)readlane((uint32_t)st, i);
      sm.card = (int)readlane(scard, i);
      sm.runs = (int)readlane(sruns, i);
      inb += payload_bytes(sm.type, sm.card, sm.runs) + 16;
      if (payload_bytes(sm.type, sm.card, sm.runs) > (uint64_t)kBitmapBytes) {
        // > 2047 runs: straight from global
        lds_zero(sS, lane);
        wave_lds_sync();
        const uint32_t *r32 = reinterpret_cast<const uint32_t *>(sptr(i));
        for (int k = lane; k < sm.runs; k += 64) toggle_run(sS, r32[k]);
        wave_lds_sync();
        toggles_to_words_lds(sS, lane);
        wave_lds_sync();
      } else {
        stage_from_chunks(sm.type, pq, (uint32_t)sm.card, (uint32_t)sm.runs, sS, lane);
      }
    }
    // ---- next slice in flight during this step's algebra
    __builtin_amdgcn_sched_barrier(0);
    if (i > 0) {
      const bool ok = (int)readlane((uint32_t)sc, i - 1) >= 0 && sbytes(i - 1) <= (uint32_t)kBitmapBytes;
      load_chunks(pq, ok ? sptr(i - 1) : bsi.payload, ok ? sbytes(i - 1) : 16u, lane);
    }
    if (!eq.present) continue; // and/andNot of an absent EQ stay absent; GT/LT unchanged
    const int bit = (int)((pred >> i) & 1);
    const bool feeds = (TRACK == 2 && bit) || (TRACK == 1 && !bit);
    // t = bit ? andNot(EQ, S) : and(EQ, S);  EQ = bit ? and(EQ, S) : andNot(EQ, S)
    uint64_t t[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) {
      const uint64_t sw = spresent ? lds_word(sS, j, lane) : 0ull;
      t[j] = bit ? (e[j] & ~sw) : (e[j] & sw);
      e[j] = bit ? (e[j] & sw) : (e[j] & ~sw);
    }
    wave_lds_sync();
    Meta tm{0, 0, 0, 0};
    if (!spresent) {
      if (bit) {
        tm = eq;          // andNot(EQ, absent) = clone of EQ
        eq.present = 0;   // and(EQ, absent) = absent
      } // else: t absent, EQ = clone of EQ (unchanged)
    } else {
      const Meta e0 = eq;
      if (feeds) tm = classify(t, lane, bit ? eff_andnot(e0, sm) : eff_and(e0, sm), false, false);
      eq = classify(e, lane, bit ? eff_and(e0, sm) : eff_andnot(e0, sm), false, false);
    }
    if (feeds && tm.present) {
      if (!x.present) {
        lds_write_words(sX, t, lane); // or(absent, t) = clone of t
        x = tm;
      } else {
        const Meta x0 = x;
#pragma unroll
        for (int j = 0; j < kW; ++j) t[j] |= lds_word(sX, j, lane);
        x = classify(t, lane, eff_or(x0, tm), lr_or(x0, tm), true);
        lds_write_words(sX, t, lane);
      }
      wave_lds_sync();
    }
  }

  // ---- the final ops with the found set F (foundSet, or ebM when null)
  const int32_t fc = has_found ? table[(uint64_t)(nbits + 1) * 65536 + key] : table[(uint64_t)nbits * 65536 + key];
  const Meta fm = stage_global(has_found ? fnd : bsi, fc, sS, lane); // present: keys come from F
  if (has_found) inb += payload_bytes(fm.type, fm.card, fm.runs) + 16;
  // EQ = and(fixedFoundSet, EQ)
  if (eq.present) {
    const Meta e0 = eq;
#pragma unroll
    for (int j = 0; j < kW; ++j) e[j] &= lds_word(sS, j, lane);
    eq = classify(e, lane, eff_and(fm, e0), false, false);
  }
  Meta rm{0, 0, 0, 0};
  uint64_t t[kW]; // the result (EQ copies e in)
  if (FINAL == kBsiEQ) {
    rm = eq;
#pragma unroll
    for (int j = 0; j < kW; ++j) t[j] = e[j];
  } else if (FINAL == kBsiNEQ) { // andNot(fixedFoundSet, EQ)
    if (!eq.present) {
#pragma unroll
      for (int j = 0; j < kW; ++j) t[j] = lds_word(sS, j, lane);
      rm = fm;
    } else {
#pragma unroll
      for (int j = 0; j < kW; ++j) t[j] = lds_word(sS, j, lane) & ~e[j];
      rm = classify(t, lane, eff_andnot(fm, eq), false, false);
    }
  } else {
    // Y = GT / LT, or or(LT|GT, EQ) for LE / GE
    Meta ym = x;
#pragma unroll
    for (int j = 0; j < kW; ++j) t[j] = x.present ? lds_word(sX, j, lane) : 0ull;
    if (FINAL == kBsiLE || FINAL == kBsiGE) {
      if (!x.present) {
#pragma unroll
        for (int j = 0; j < kW; ++j) t[j] = e[j];
        ym = eq;
      } else if (eq.present) {
#pragma unroll
        for (int j = 0; j < kW; ++j) t[j] |= e[j];
        ym = classify(t, lane, eff_or(x, eq), lr_or(x, eq), true);
      }
    }
    // and(Y, fixedFoundSet)
    if (ym.present) {
#pragma unroll
      for (int j = 0; j < kW; ++j) t[j] &= lds_word(sS, j, lane);
      rm = classify(t, lane, eff_and(ym, fm), false, false);
    }
  }
  wave_lds_sync();
  const int ty = rm.present ? rm.type : kEmpty;
  if (rm.present) emit_container(ty, t, rm.card, rm.runs, out + (uint64_t)q * kBitmapBytes, sS, lane);
  if (lane == 0) {
    wo.type[q] = (uint8_t)ty;
    wo.card[q] = (uint32_t)(rm.present ? rm.card : 0);
    wo.nruns[q] = (uint16_t)(ty == kRun ? rm.runs : 0);
    if (inb) atomicAdd((unsigned long long *)&stats[0 * kStripes + (q & (kStripes - 1))], (unsigned long long)inb);
    if (rm.present)
      atomicAdd((unsigned long long *)&stats[1 * kStripes + (q & (kStripes - 1))],
                (unsigned long long)(payload_bytes(ty, rm.card, rm.runs) + (ty == kRun ? 2 : 0) + 16));
  }
}

// ---- RANGE fused: both O'Neil chains (GE(start) and LE(end)) walk the slices in ONE pass, so every
// slice container is staged once for the two comparators; the keyed static AND of the two results
// (RoaringBitmapSliceIndex.java:492-497; AND rule R&R -> EFF else AB, empty / one-sided dropped)
// closes the kernel.  Each chain keeps its own EQ (registers) and GT / LT accumulator (LDS image)
// with the same per-step type rules as k_bsi_chain.
// One chain step (k_bsi_chain's loop body after the slice is staged): TRACK 1 = GT (GE), 2 = LT (LE).
__device__ __forceinline__ void bsi_step(uint64_t (&e)[kW], Meta &eq, Meta &x, uint32_t *sX, int bit, int track,
                                         bool spresent, const Meta &sm, const uint32_t *sS, int lane) {
  if (!eq.present) return; // and/andNot of an absent EQ stay absent; GT/LT unchanged
  const bool feeds = (track == 2 && bit) || (track == 1 && !bit);
  uint64_t t[kW];
#pragma unroll
  for (int j = 0; j < kW; ++j) {
    const uint64_t sw = spresent ? lds_word(sS, j, lane) : 0ull;
    t[j] = bit ? (e[j] & ~sw) : (e[j] & sw);
    e[j] = bit ? (e[j] & sw) : (e[j] & ~sw);
  }
  wave_lds_sync();
  Meta tm{0, 0, 0, 0};
  if (!spresent) {
    if (bit) {
      tm = eq;        // andNot(EQ, absent) = clone of EQ
      eq.present = 0; // and(EQ, absent) = absent
    }
  } else {
    const Meta e0 = eq;
    if (feeds) tm = classify(t, lane, bit ? eff_andnot(e0, sm) : eff_and(e0, sm), false, false);
    eq = classify(e, lane, bit ? eff_and(e0, sm) : eff_andnot(e0, sm), false, false);
  }
  if (feeds && tm.present) {
    if (!x.present) {
      lds_write_words(sX, t, lane); // or(absent, t) = clone of t
      x = tm;
    } else {
      const Meta x0 = x;
#pragma unroll
      for (int j = 0; j < kW; ++j) t[j] |= lds_word(sX, j, lane);
      x = classify(t, lane, eff_or(x0, tm), lr_or(x0, tm), true);
      lds_write_words(sX, t, lane);
    }
    wave_lds_sync();
  }
}
// GE / LE result of one chain: Y = or(GT|LT, EQ), then and(Y, fixedFoundSet) (F staged in sS)
__device__ __forceinline__ Meta bsi_final_ge_le(uint64_t (&t)[kW], const uint64_t (&e)[kW], const Meta &eq,
                                                const Meta &x, const uint32_t *sX, const Meta &fm,
                                                const uint32_t *sS, int lane) {
  Meta ym = x;
#pragma unroll
  for (int j = 0; j < kW; ++j) t[j] = x.present ? lds_word(sX, j, lane) : 0ull;
  if (!x.present) {
#pragma unroll
    for (int j = 0; j < kW; ++j) t[j] = e[j];
    ym = eq;
  } else if (eq.present) {
#pragma unroll
    for (int j = 0; j < kW; ++j) t[j] |= e[j];
    ym = classify(t, lane, eff_or(x, eq), lr_or(x, eq), true);
  }
  Meta rm{0, 0, 0, 0};
  if (ym.present) {
#pragma unroll
    for (int j = 0; j < kW; ++j) t[j] &= lds_word(sS, j, lane);
    rm = classify(t, lane, eff_and(ym, fm), false, false);
  }
  return rm;
}
// RANGE's one launch: per key both chains and the final AND (bsi_range_key), then the call's tail in the
// last block to finish (the hand-off of wave.hpp's st_sc1 / ld_sc1): the keyed results compacted into the
// result SoA and CSR, the counters and the result count written to host-visible words, the call's sequence
// number last (the host returns on it: wait_call_seq).
struct BsiTail {
  uint64_t *kmeta;  // [nk] per key: card (bits 0-16), type (19-20; 3 = none), key (24-39), run count (40-55)
  uint64_t *ctr;    // [0] finished blocks, [8] / [16] / [24] input bytes / output bytes / cardinality
  OutView ov;
  uint64_t *rbegin; // [2]
  uint64_t *hout;   // host-visible: [0] result containers, [1..3] the counters, [5] = seq
  uint64_t seq;
  uint32_t nblocks;
};
__device__ __forceinline__ uint64_t bsi_meta(uint32_t key, int ty, uint32_t card, uint32_t nr) {
  return (card & 0x1FFFFu) | ((uint64_t)(ty == (int)kEmpty ? 3u : (uint32_t)ty) << 19) | ((uint64_t)key << 24) |
         ((uint64_t)nr << 40);
}
__global__ __launch_bounds__(128, 2) void k_bsi_range(SetView bsi, SetView fnd, int has_found,
                                                      const int32_t *__restrict__ table, uint32_t nbits,
                                                      uint64_t start, uint64_t end, const uint32_t *__restrict__ klist,
                                                      uint32_t nk, uint8_t *__restrict__ out, BsiTail tl) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[2][3][2048];
  __shared__ uint64_t red[2][3];
  __shared__ uint32_t s_last, wt[4];
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t q = xcd_swizzle(blockIdx.x, gridDim.x) * 2 + wv;
  uint64_t inb = 0, outb = 0, csum = 0;
  if (q < nk) { // wave-uniform
  uint32_t *sS = lds[wv][0], *sG = lds[wv][1], *sL = lds[wv][2];
  const uint32_t key = klist[q];
  uint64_t eg[kW], el[kW];
  Meta eqg = stage_global(bsi, table[(uint64_t)nbits * 65536 + key], sS, lane);
  if (eqg.present) {
    lds_read_words(sS, eg, lane);
    inb += payload_bytes(eqg.type, eqg.card, eqg.runs) + 16; // ebM, read once for both comparators
  } else {
#pragma unroll
    for (int j = 0; j < kW; ++j) eg[j] = 0;
  }
#pragma unroll
  for (int j = 0; j < kW; ++j) el[j] = eg[j];
  Meta eql = eqg;
  wave_lds_sync();
  Meta xg{0, 0, 0, 0}, xl{0, 0, 0, 0};
  const int32_t sc = lane < (int)nbits ? table[(uint64_t)lane * 65536 + key] : -1;
  int st = 0;
  uint32_t scard = 0, sruns = 0;
  uint64_t soff = 0;
  if (sc >= 0) {
    st = bsi.type[sc];
    scard = bsi.card[sc];
    sruns = bsi.nruns[sc];
    soff = bsi.off[sc];
  }
  auto sbytes = [&](int i) -> uint32_t {
    const int t = (int)readlane((uint32_t)st, i);
    return (uint32_t)payload_bytes(t, readlane(scard, i), readlane(sruns, i));
  };
  auto sptr = [&](int i) -> const uint8_t * {
    return bsi.payload + pack2(readlane((uint32_t)soff, i), readlane((uint32_t)(soff >> 32), i));
  };
  uint4 pq[8];
  if (nbits) {
    const int i0 = (int)nbits - 1;
    const bool ok = (int)readlane((uint32_t)sc, i0) >= 0 && sbytes(i0) <= (uint32_t)kBitmapBytes;
    load_chunks(pq, ok ? sptr(i0) : bsi.payload, ok ? sbytes(i0) : 16u, lane);
  }
  for (int i = (int)nbits - 1; i >= 0; --i) {
    const bool spresent = (int)readlane((uint32_t)sc, i) >= 0;
    Meta sm{0, 0, 0, 0};
    if (spresent) {
      sm.present = 1;
      sm.type = (int)readlane((uint32_t)st, i);
      sm.card = (int)readlane(scard, i);
      sm.runs = (int)readlane(sruns, i);
      inb += payload_bytes(sm.type, sm.card, sm.runs) + 16; // one read serves both comparators
      if (payload_bytes(sm.type, sm.card, sm.runs) > (uint64_t)kBitmapBytes) {
        lds_zero(sS, lane);
        wave_lds_sync();
        const uint32_t *r32 = reinterpret_cast<const uint32_t *>(sptr(i));
        for (int k = lane; k < sm.runs; k += 64) toggle_run(sS, r32[k]);
        wave_lds_sync();
        toggles_to_words_lds(sS, lane);
        wave_lds_sync();
      } else {
        stage_from_chunks(sm.type, pq, (uint32_t)sm.card, (uint32_t)sm.runs, sS, lane);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (i > 0) {
      const bool ok = (int)readlane((uint32_t)sc, i - 1) >= 0 && sbytes(i - 1) <= (uint32_t)kBitmapBytes;
      load_chunks(pq, ok ? sptr(i - 1) : bsi.payload, ok ? sbytes(i - 1) : 16u, lane);
    }
    bsi_step(eg, eqg, xg, sG, (int)((start >> i) & 1), 1, spresent, sm, sS, lane);
    bsi_step(el, eql, xl, sL, (int)((end >> i) & 1), 2, spresent, sm, sS, lane);
  }
  // ---- the final ops with the found set F (foundSet, or ebM when null), per chain
  const int32_t fc = has_found ? table[(uint64_t)(nbits + 1) * 65536 + key] : table[(uint64_t)nbits * 65536 + key];
  const Meta fm = stage_global(has_found ? fnd : bsi, fc, sS, lane);
  if (has_found) inb += payload_bytes(fm.type, fm.card, fm.runs) + 16;
  // EQ = and(fixedFoundSet, EQ), both chains
  if (eqg.present) {
    const Meta e0 = eqg;
#pragma unroll
    for (int j = 0; j < kW; ++j) eg[j] &= lds_word(sS, j, lane);
    eqg = classify(eg, lane, eff_and(fm, e0), false, false);
  }
  if (eql.present) {
    const Meta e0 = eql;
#pragma unroll
    for (int j = 0; j < kW; ++j) el[j] &= lds_word(sS, j, lane);
    eql = classify(el, lane, eff_and(fm, e0), false, false);
  }
  uint64_t t[kW];
  const Meta rg = bsi_final_ge_le(t, eg, eqg, xg, sG, fm, sS, lane);
  wave_lds_sync();
  lds_write_words(sG, t, lane); // GE result parked in its (now free) accumulator image
  wave_lds_sync();
  const Meta rl = bsi_final_ge_le(t, el, eql, xl, sL, fm, sS, lane);
  Meta rm{0, 0, 0, 0};
  if (rg.present && rl.present) {
#pragma unroll
    for (int j = 0; j < kW; ++j) t[j] &= lds_word(sG, j, lane);
    rm = classify(t, lane, eff_and(rg, rl), false, false);
  }
  wave_lds_sync();
  const int ty = rm.present ? rm.type : kEmpty;
  if (rm.present) emit_container(ty, t, rm.card, rm.runs, out + (uint64_t)q * kBitmapBytes, sS, lane);
  if (lane == 0)
    st_sc1(tl.kmeta + q, bsi_meta(key, ty, rm.present ? (uint32_t)rm.card : 0u, ty == kRun ? (uint32_t)rm.runs : 0u));
  if (rm.present) {
    outb = payload_bytes(ty, rm.card, rm.runs) + (ty == kRun ? 2 : 0) + 16;
    csum = (uint64_t)rm.card;
  }
  } // q < nk
  // ---- the block's counters (one agent atomic per counter), then the finished-block add
  if (lane == 0) {
    red[wv][0] = inb;
    red[wv][1] = outb;
    red[wv][2] = csum;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const uint64_t x = red[0][threadIdx.x] + red[1][threadIdx.x];
    if (x) __hip_atomic_fetch_add(tl.ctr + 8 + 8 * threadIdx.x, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(tl.ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tl.nblocks - 1ull;
  __syncthreads();
  if (!s_last) return;
  // ---- the last block: the keyed results compacted in key order (dropped keys leave no container)
  const uint64_t v = threadIdx.x < 3 ? ld_sc1(tl.ctr + 8 + 8 * threadIdx.x) : 0;
  constexpr int kPer = 16;
  uint32_t base = 0;
  for (uint32_t t0 = 0; t0 < nk; t0 += kPer * blockDim.x) {
    const uint32_t lo = t0 + kPer * threadIdx.x;
    uint64_t m[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) m[k] = lo + k < nk ? ld_sc1(tl.kmeta + lo + k) : (3ull << 19);
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) cnt += ((m[k] >> 19) & 3u) != 3u;
    uint32_t tot;
    uint32_t r = base + block_xscan(cnt, wt, tot);
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      if (((m[k] >> 19) & 3u) == 3u) continue;
      tl.ov.key[r] = (uint16_t)(m[k] >> 24);
      tl.ov.type[r] = (uint8_t)((m[k] >> 19) & 3u);
      tl.ov.card[r] = (uint32_t)(m[k] & 0x1FFFFu);
      tl.ov.nruns[r] = (uint16_t)(m[k] >> 40);
      tl.ov.off[r] = (uint64_t)(lo + k) * kBitmapBytes;
      ++r;
    }
    base += tot;
  }
  if (threadIdx.x < 3) {
    red[0][threadIdx.x] = v;
    __hip_atomic_store(tl.ctr + 8 + 8 * threadIdx.x, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_store(tl.ctr, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); // ready for the next call
    tl.rbegin[0] = 0;
    tl.rbegin[1] = base;
    for (int k = 0; k < 3; ++k) tl.hout[1 + k] = red[0][k];
    tl.hout[0] = base;
    __hip_atomic_store(tl.hout + 5, tl.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------- host side
static unsigned nblk(uint64_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

// Keyed slots of one reduction: an 8 KiB payload slot per active key plus its type / card / runs.
struct KeyedSlots {
  uint8_t *payload = nullptr;
  WideOut wo{nullptr, nullptr, nullptr};
  int alloc(rbgpu_ctx *ctx, uint32_t nk, bool with_payload) {
    const uint64_t nk1 = std::max<uint32_t>(nk, 1);
    if ((with_payload && ctx->pool.alloc((void **)&payload, nk1 * kBitmapBytes)) ||
        ctx->pool.alloc((void **)&wo.type, nk1) || ctx->pool.alloc((void **)&wo.card, nk1 * 4) ||
        ctx->pool.alloc((void **)&wo.nruns, nk1 * 2))
      return fail(RB_ENOMEM, "bsi slots for %u keys", nk);
    return RB_OK;
  }
  void release(rbgpu_ctx *ctx, bool with_payload) {
    if (with_payload) ctx->pool.release(payload);
    for (void *p : {(void *)wo.type, (void *)wo.card, (void *)wo.nruns}) ctx->pool.release(p);
  }
};

// One O'Neil chain (oNeilCompare with `final_op`) over the keys of F into keyed slots.
static void bsi_chain(rbgpu_ctx *ctx, const rbgpu_set *bsi, uint32_t nbits, int final_op, uint64_t pred,
                      const rbgpu_set *found, const int32_t *d_table, const uint32_t *d_klist, uint32_t nk,
                      uint8_t *o, const WideOut &wo) {
  if (!nk) return;
  hipStream_t st = ctx->stream;
  const SetView bv = bsi->view();
  const SetView fv = found ? found->view() : bv;
  const int hf = found != nullptr;
  const unsigned g = nblk(nk, 4);
  switch (final_op) {
  case kBsiEQ: k_bsi_chain<kBsiEQ><<<g, 256, 0, st>>>(bv, fv, hf, d_table, nbits, pred, d_klist, nk, o, wo, ctx->d_stats); break;
  case kBsiNEQ: k_bsi_chain<kBsiNEQ><<<g, 256, 0, st>>>(bv, fv, hf, d_table, nbits, pred, d_klist, nk, o, wo, ctx->d_stats); break;
  case kBsiLE: k_bsi_chain<kBsiLE><<<g, 256, 0, st>>>(bv, fv, hf, d_table, nbits, pred, d_klist, nk, o, wo, ctx->d_stats); break;
  case kBsiLT: k_bsi_chain<kBsiLT><<<g, 256, 0, st>>>(bv, fv, hf, d_table, nbits, pred, d_klist, nk, o, wo, ctx->d_stats); break;
  case kBsiGE: k_bsi_chain<kBsiGE><<<g, 256, 0, st>>>(bv, fv, hf, d_table, nbits, pred, d_klist, nk, o, wo, ctx->d_stats); break;
  default: k_bsi_chain<kBsiGT><<<g, 256, 0, st>>>(bv, fv, hf, d_table, nbits, pred, d_klist, nk, o, wo, ctx->d_stats); break;
  }
}

// compareUsingMinMax (RoaringBitmapSliceIndex.java:505-577), values unsigned: 1 = all, 0 = empty,
// -1 = evaluate
static int min_max_shortcut(int op, uint64_t a, uint64_t b, uint64_t mn, uint64_t mx) {
  switch (op) {
  case kBsiLT: return a > mx ? 1 : a <= mn ? 0 : -1;
  case kBsiLE: return a >= mx ? 1 : a < mn ? 0 : -1;
  case kBsiGT: return a < mn ? 1 : a >= mx ? 0 : -1;
  case kBsiGE: return a <= mn ? 1 : a > mx ? 0 : -1;
  case kBsiEQ: return (mn == mx && mn == a) ? 1 : (a < mn || a > mx) ? 0 : -1;
  case kBsiNEQ: return mn == mx ? (mn == a ? 0 : 1) : -1;
  default: return (a <= mn && b >= mx) ? 1 : (a > mx || b < mn) ? 0 : -1; // RANGE
  }
}

// The set's key -> container tables (rows 0..nbits: its slices and ebM; row nbits + 1: a call's foundSet)
// and ebM's key list, built on the set's first compare and kept with it (sets are immutable): the device
// time and bytes are the set's setup part 3 (rbgpu_set_setup_parts).
static int ensure_bsi_tables(rbgpu_ctx *ctx, const rbgpu_set *cs, uint32_t nbits) {
  rbgpu_set *s = const_cast<rbgpu_set *>(cs);
  if (s->bsi_table) return RB_OK;
  int rc = ensure_h_begin(s);
  if (rc) return rc;
  hipStream_t st = ctx->stream;
  int32_t *t = nullptr;
  uint32_t *kl = nullptr;
  uint64_t *bt = nullptr, *bts = nullptr;
  if (ctx->pool.alloc((void **)&t, (nbits + 2ull) * 65536 * 4) || ctx->pool.alloc((void **)&kl, 65536 * 4ull) ||
      ctx->pool.alloc((void **)&bt, 65537 * 8ull) || ctx->pool.alloc((void **)&bts, 65537 * 8ull)) {
    for (void *p : {(void *)t, (void *)kl, (void *)bt, (void *)bts}) ctx->pool.release(p);
    return fail(RB_ENOMEM, "bsi tables");
  }
  {
    DeriveTimer tm(s, 3);
    if (hipMemsetAsync(t, 0xFF, (nbits + 1ull) * 65536 * 4, st) != hipSuccess) {
      for (void *p : {(void *)t, (void *)kl, (void *)bt, (void *)bts}) ctx->pool.release(p);
      return fail(RB_EDEVICE, "bsi table memset failed");
    }
    k_bsi_index<<<dim3(64, nbits + 1), 256, 0, st>>>(s->view(), 0, t);
    const int32_t *frow = t + (uint64_t)nbits * 65536;
    k_bsi_active<<<256, 256, 0, st>>>(frow, 0, 65536, bt);
    const uint64_t *in1[1] = {bt};
    uint64_t *out1[1] = {bts};
    scan_blocks_multi(in1, out1, 1, 256, nullptr, st);
    k_bsi_list<<<256, 256, 0, st>>>(frow, 0, 65536, bts, kl);
  }
  ctx->pool.release(bt); // stream-ordered: the pool hands them only to later work on this stream
  ctx->pool.release(bts);
  if (hipGetLastError() != hipSuccess) {
    ctx->pool.release(t);
    ctx->pool.release(kl);
    return fail(RB_EDEVICE, "bsi table kernels failed");
  }
  s->bsi_nk = (uint32_t)(s->h_begin[nbits + 1] - s->h_begin[nbits]);
  if (s->bsi_nk) { // ebM's first and last key: a key-range shard that holds them all takes the cached list
    uint32_t *h = reinterpret_cast<uint32_t *>(ctx->h_pinned);
    if (hipMemcpyAsync(h, kl, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(h + 1, kl + s->bsi_nk - 1, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess) {
      ctx->pool.release(t);
      ctx->pool.release(kl);
      return fail(RB_EDEVICE, "bsi key list read-back failed");
    }
    s->bsi_kmin = h[0];
    s->bsi_kmax = h[1];
  }
  s->bsi_table = t;
  s->bsi_klist = kl;
  // keys read, table entries written (4 B per container), ebM's key list written
  const uint64_t b = 6ull * (s->h_begin[nbits + 1] - s->h_begin[0]) + 4ull * s->bsi_nk;
  s->derive_bytes += b;
  s->part_bytes[3] += b;
  return RB_OK;
}

// RANGE over nk >= 1 keys of F: k_bsi_range writes the result set (CSR, SoA, payload slots) and the call's
// counters itself; the host returns on the call's sequence number (wait_call_seq).
static int bsi_range_one_launch(rbgpu_ctx *ctx, const rbgpu_set *bsi, const rbgpu_set *found, const int32_t *d_table,
                                uint32_t nbits, uint64_t start, uint64_t end, const uint32_t *d_klist, uint32_t nk,
                                rbgpu_set *res) {
  hipStream_t st = ctx->stream;
  int rc = ensure_call_words(ctx);
  if (!rc) rc = seq_begin(ctx);
  if (rc) return rc;
  uint64_t *kmeta = nullptr;
  if (ctx->pool.alloc((void **)&kmeta, 8ull * nk)) return fail(RB_ENOMEM, "bsi key results");
  const uint32_t nblocks = nblk(nk, 2);
  BsiTail tl{kmeta, ctx->d_small_ctr, OutView{res->key, res->type, res->card, res->nruns, res->off}, res->begin,
             reinterpret_cast<uint64_t *>(ctx->d_small), ++ctx->small_seq, nblocks};
  HIPCHK(hipEventRecord(ctx->ev[1], st));
  k_bsi_range<<<nblocks, 128, 0, st>>>(bsi->view(), found ? found->view() : bsi->view(), found != nullptr, d_table,
                                       nbits, start, end, d_klist, nk, res->payload, tl);
  HIPCHK(hipEventRecord(ctx->ev[2], st));
  HIPCHK(hipEventRecord(ctx->ev[5], st));
  ctx->pool.release(kmeta); // stream-ordered: handed out again only to later work on this stream
  bool seen = false;
  rc = seq_end(ctx, tl.seq, true, "bsi range", &seen);
  if (rc) return rc;
  const uint64_t *hout = reinterpret_cast<const uint64_t *>(ctx->h_small);
  uint64_t *w = ctx->words;
  for (int i = 0; i < kStatWords; ++i) w[i] = 0;
  w[0] = hout[1]; // input bytes
  w[1] = hout[2]; // output bytes
  w[7] = hout[3]; // result cardinality
  w[8] = hout[0]; // result containers
  const uint64_t nres = hout[0];
  const KernelSpan spans[1] = {{"k_bsi_range", 0, 1, 2ull * nk}};
  rc = stats_fill(ctx, nk, nres, spans, 1, !seen);
  ctx->stats_pending = seen;
  ctx->stats_pending_k = seen;
  if (rc) return rc;
  ctx->last.result_containers = nres;
  res->nc = nres;
  res->h_begin = {0, nres};
  res->end_seq = seen ? tl.seq : 0;
  return RB_OK;
}

int bsi_compare(rbgpu_ctx *ctx, const rbgpu_set *bsi, int op, uint64_t start, uint64_t end, uint64_t vmin,
                uint64_t vmax, const rbgpu_set *found, uint32_t key_lo, uint32_t key_hi, rbgpu_set **out) {
  const uint32_t nbits = bsi->nb - 1;
  hipStream_t st = ctx->stream;
  stats_begin(ctx);
  const int sc = min_max_shortcut(op, start, end, vmin, vmax);
  if (sc >= 0 && (key_lo > 0 || key_hi < 65536)) {
    // a key-range shard of the shortcut's answer: the whole-range answer, restricted
    rbgpu_set *whole = nullptr;
    int rc = bsi_compare(ctx, bsi, op, start, end, vmin, vmax, found, 0, 65536, &whole);
    if (rc) return rc;
    rc = set_key_subset(whole, key_lo, key_hi, out);
    rbgpu_set_free(whole);
    return rc;
  }
  if (sc >= 0) {
    // all = foundSet == null ? ebM.clone() : and(ebM, foundSet); empty = new bitmap.  rb_stats describes this
    // call's answer (no compare kernel ran: no kernel times), not the previous call's
    auto shortcut_stats = [&](rbgpu_set *r, uint64_t card) {
      for (int i = 0; i < kStatWords; ++i) ctx->words[i] = 0;
      ctx->words[7] = card;
      return stats_fill(ctx, 0, r->nc, nullptr, 0, false);
    };
    if (sc == 0) {
      rbgpu_set *e = new rbgpu_set;
      const int rc = set_alloc(ctx, e, 1, 0, 16);
      if (rc) {
        delete e;
        return rc;
      }
      const uint64_t hb[2] = {0, 0};
      HIPCHK(hipMemcpyAsync(e->begin, hb, 16, hipMemcpyHostToDevice, st));
      HIPCHK(hipStreamSynchronize(st));
      LAUNCHCHK();
      e->h_begin = {0, 0};
      *out = e;
      return shortcut_stats(e, 0);
    }
    if (!found) {
      int rc = rbgpu_set_extract(bsi, nbits, 1, out);
      uint64_t card = 0;
      if (!rc) rc = rbgpu_set_cardinalities(*out, &card);
      if (!rc) rc = shortcut_stats(*out, card);
      if (rc && *out) {
        rbgpu_set_free(*out);
        *out = nullptr;
      }
      return rc;
    }
    const uint32_t ai = nbits, bi = 0;
    return rbgpu_pairwise(ctx, RB_AND, bsi, found, &ai, &bi, 1, out); // its own stats: the AND's answer
  }
  // key -> container tables: rows 0..nbits-1 slices, nbits ebM (the set's, cached), nbits+1 foundSet
  int rc = ensure_bsi_tables(ctx, bsi, nbits);
  if (rc) return rc;
  int32_t *d_table = bsi->bsi_table;
  if (found) {
    int32_t *frow = d_table + (uint64_t)(nbits + 1) * 65536;
    HIPCHK(hipMemsetAsync(frow, 0xFF, 65536 * 4, st));
    k_bsi_index<<<dim3(64, 1), 256, 0, st>>>(found->view(), 0, frow);
  }
  // F's keys: ebM's over the whole key range are the set's cached list; a foundSet's or a shard's are
  // listed per call, and their count comes from F's host CSR over the whole range, else by a read-back
  uint32_t nk = 0;
  const uint32_t *d_klist = nullptr;
  uint64_t *d_active = nullptr, *d_pos = nullptr;
  uint32_t *d_kl = nullptr;
  auto release = [&]() {
    for (void *p : {(void *)d_active, (void *)d_pos, (void *)d_kl}) ctx->pool.release(p);
  };
  const bool full = key_lo == 0 && key_hi >= 65536;
  if (!found && (full || !bsi->bsi_nk || (key_lo <= bsi->bsi_kmin && bsi->bsi_kmax < key_hi))) {
    // every key of ebM lies in the range (the whole range, or a shard holding the index's own keys)
    d_klist = bsi->bsi_klist;
    nk = bsi->bsi_nk;
  } else {
    if (ctx->pool.alloc((void **)&d_active, 65537 * 8ull) || ctx->pool.alloc((void **)&d_pos, 65537 * 8ull) ||
        ctx->pool.alloc((void **)&d_kl, 65536 * 4ull)) {
      release();
      return fail(RB_ENOMEM, "bsi key list");
    }
    const int32_t *frow = d_table + (uint64_t)(found ? nbits + 1 : nbits) * 65536;
    k_bsi_active<<<256, 256, 0, st>>>(frow, key_lo, key_hi, d_active);
    const uint64_t *in1[1] = {d_active};
    uint64_t *out1[1] = {d_pos};
    scan_blocks_multi(in1, out1, 1, 256, nullptr, st);
    k_bsi_list<<<256, 256, 0, st>>>(frow, key_lo, key_hi, d_pos, d_kl);
    d_klist = d_kl;
    const rbgpu_set *fs = found ? found : bsi;
    const uint32_t fb = found ? 0u : nbits;
    if (full && !ensure_h_begin(fs)) {
      nk = (uint32_t)(fs->h_begin[fb + 1] - fs->h_begin[fb]);
      LAUNCHCHK();
    } else {
      HIPCHK(hipMemcpyAsync(ctx->h_pinned, d_pos + 256, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      LAUNCHCHK();
      nk = (uint32_t)ctx->h_pinned[0];
    }
  }
  // result set: one 8 KiB slot per key of F, compacted at the end
  rbgpu_set *res = new rbgpu_set;
  rc = set_alloc(ctx, res, 1, nk, (uint64_t)std::max<uint32_t>(nk, 1) * kBitmapBytes);
  if (rc) {
    delete res;
    release();
    return rc;
  }
  if (op == 6 && nk) { // RANGE: one launch (k_bsi_range's tail compacts and hands the results to the host)
    rc = bsi_range_one_launch(ctx, bsi, found, d_table, nbits, start, end, d_klist, nk, res);
    release();
    if (rc) {
      rbgpu_set_free(res);
      return rc;
    }
    *out = res;
    return RB_OK;
  }
  KeyedSlots fin;
  rc = fin.alloc(ctx, nk, false);
  if (!rc) {
    HIPCHK(hipEventRecord(ctx->ev[1], st));
    if (op != 6) {
      bsi_chain(ctx, bsi, nbits, op, start, found, d_table, d_klist, nk, res->payload, fin.wo);
    }
    HIPCHK(hipEventRecord(ctx->ev[2], st));
    rc = compact_keyed(ctx, d_klist, nk, fin.wo, res);
    const KernelSpan spans[1] = {{op == 6 ? "k_bsi_range" : "k_bsi_chain", 0, 1, op == 6 ? 2ull * nk : nk}};
    if (!rc) rc = stats_end(ctx, nk, 0, spans, 1);
    if (!rc) keyed_result_count(ctx, res);
  }
  fin.release(ctx, false);
  release();
  if (rc) {
    rbgpu_set_free(res);
    return rc;
  }
  *out = res;
  return RB_OK;
}

// this file's code object, loaded at context creation (warm_code_objects, api.hip)
__global__ void k_warm_bsi() {}
void warm_bsi(hipStream_t st) { k_warm_bsi<<<1, 64, 0, st>>>(); }

} // namespace rbg
