// wave.hpp — wave64 building blocks for container algebra on gfx950.
//
// A 65536-bit container lives in the registers of ONE wave: lane L holds 16 u64 words
// w[j], j = 2k + h (k = 0..7, h = 0..1), which is container word 128*k + 2*L + h.  With
// this interleaving every 16-byte-per-lane access to a Bitmap payload (global or LDS) is one
// fully coalesced 1 KiB wave instruction: uint4 index k*64 + L holds words 2*(k*64+L), +1.
//
// Array and Run operands are expanded into that register form through an 8 KiB per-wave LDS
// scratch (Array: ds_or of value bits; Run: ds_xor of start / end+1 toggles, then an
// in-register prefix-xor with a wave parity scan).  Results are classified exactly like the
// reference (card c, maximal run count r -> Array / Bitmap / Run) and emitted in
// RoaringFormatSpec payload form through the same scratch so global stores stay coalesced.
#pragma once
#include "common.hpp"

namespace rbg {

constexpr int kW = 16; // words per lane

__device__ __forceinline__ void wave_lds_sync() {
  // LDS ops of one wave execute in order; this keeps the compiler from reordering across it.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// XCD-aware block order (cdna_hip_programming.md §5 T1): blocks b, b+8, b+16, ... share an XCD's L2,
// so they get consecutive logical indices — neighbouring keys of a wide aggregation then read the
// same metadata lines (type / card / run-count / offset arrays are member-major: key k and k+1 of a
// member are adjacent) from one L2 instead of eight.  A bijection on [0, nwg) for any nwg; a pure
// speed choice (placement is not guaranteed).
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t orig, uint32_t nwg) {
  const uint32_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// ---- wave collectives on DPP (VALU lane crossbar: no LDS round trip, no bpermute chain).
// dpp_ctrl: row_shr:n = 0x110+n, wave_shl:1 = 0x130, wave_shr:1 = 0x138, row_bcast:15 = 0x142,
// row_bcast:31 = 0x143.  Lanes without a source (or in rows masked off) read 0.
template <int CTRL, int ROW_MASK = 0xf, bool BOUND_ZERO = true>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xf, BOUND_ZERO);
}
__device__ __forceinline__ uint32_t readlane(uint32_t x, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}
// inclusive prefix sum over the 64 lanes: Hillis-Steele within each row of 16, then the row
// totals broadcast forward (row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3)
__device__ __forceinline__ uint32_t wave_scan_u32(uint32_t v, int /*lane*/) {
  v += dpp<0x111>(v);
  v += dpp<0x112>(v);
  v += dpp<0x114>(v);
  v += dpp<0x118>(v);
  v += dpp<0x142, 0xa, false>(v);
  v += dpp<0x143, 0xc, false>(v);
  return v;
}
__device__ __forceinline__ uint32_t wave_xscan_xor(uint32_t v, int /*lane*/) { // inclusive xor-scan
  v ^= dpp<0x111>(v);
  v ^= dpp<0x112>(v);
  v ^= dpp<0x114>(v);
  v ^= dpp<0x118>(v);
  v ^= dpp<0x142, 0xa, false>(v);
  v ^= dpp<0x143, 0xc, false>(v);
  return v;
}
// inclusive prefix sum of packed 16-bit fields (no field may reach 65536 over the wave): the two
// 32-bit halves scan independently
__device__ __forceinline__ uint64_t wave_scan_u64(uint64_t v, int lane) {
  return (uint64_t)wave_scan_u32((uint32_t)v, lane) | ((uint64_t)wave_scan_u32((uint32_t)(v >> 32), lane) << 32);
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) { return readlane(wave_scan_u32(v, 0), 63); }
// 64-bit sum (accounting counters): shuffles, off the hot loops
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, o);
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

__device__ __forceinline__ uint64_t pack2(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }

// ---------------------------------------------------------------- loading operands
__device__ __forceinline__ void load_bitmap(const uint8_t *p, uint64_t (&w)[kW], int lane) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  uint4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = q[k * 64 + lane];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w[2 * k] = pack2(v[k].x, v[k].y);
    w[2 * k + 1] = pack2(v[k].z, v[k].w);
  }
}
__device__ __forceinline__ void lds_zero(uint32_t *s, int lane) {
  uint4 *s4 = reinterpret_cast<uint4 *>(s);
#pragma unroll
  for (int k = 0; k < 8; ++k) s4[k * 64 + lane] = make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ void lds_read_words(const uint32_t *s, uint64_t (&w)[kW], int lane) {
  const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint4 v = s4[k * 64 + lane];
    w[2 * k] = pack2(v.x, v.y);
    w[2 * k + 1] = pack2(v.z, v.w);
  }
}

__device__ __forceinline__ void lds_write_words(uint32_t *s, const uint64_t (&w)[kW], int lane) {
  uint4 *s4 = reinterpret_cast<uint4 *>(s);
#pragma unroll
  for (int k = 0; k < 8; ++k)
    s4[k * 64 + lane] = make_uint4((uint32_t)w[2 * k], (uint32_t)(w[2 * k] >> 32), (uint32_t)w[2 * k + 1],
                                   (uint32_t)(w[2 * k + 1] >> 32));
}

// OR one lane's chunk of sorted values (n <= 8) into the LDS bitmap: a segmented OR over runs of
// equal word index in registers, then one ds_or per value, carrying the group's mask at the group's
// last value and 0 elsewhere (an OR of 0 changes nothing).  No value-dependent branch: the earlier
// form branched per value on "new word?", which cost ~16 SALU exec-mask instructions per value.
// Values past n OR 0 into the word of the last live value.
template <bool XOR = false> // XOR: ds_xor instead of ds_or (a second operand into the same image)
__device__ __forceinline__ void or_chunk_values(const uint32_t (&x)[8], int n, uint32_t *s) {
  uint32_t acc = 0, prev = x[0] >> 5;
  const uint32_t lastw = x[n - 1 < 7 ? n - 1 : 7] >> 5;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool live = i < n;
    const uint32_t wi = live ? x[i] >> 5 : lastw;
    acc = (wi == prev ? acc : 0u) | (live ? 1u << (x[i] & 31) : 0u);
    prev = wi;
    // past n the last group's mask is re-emitted: harmless for ds_or, not for ds_xor
    const bool last = (!XOR || live) && (i == 7 || i + 1 >= n || (x[i + 1] >> 5) != wi);
    if (XOR) atomicXor(&s[wi], last ? acc : 0u);
    else atomicOr(&s[wi], last ? acc : 0u);
  }
}

// OR the values of a sorted u16 array (payload 16-B aligned) into the LDS bitmap `s`.  Each lane
// takes 8 consecutive values per 16-B load (coalesced), folds them per 32-bit word and issues
// one ds_or per word.
__device__ __forceinline__ void lds_or_array(const uint16_t *vals, int card, uint32_t *s, int lane) {
  const uint4 *v4 = reinterpret_cast<const uint4 *>(vals);
  const int nchunks = (card + 7) >> 3;
  for (int c = lane; c < nchunks; c += 64) {
    uint4 q = v4[c];
    uint32_t x[8] = {q.x & 0xFFFF, q.x >> 16, q.y & 0xFFFF, q.y >> 16,
                     q.z & 0xFFFF, q.z >> 16, q.w & 0xFFFF, q.w >> 16};
    or_chunk_values(x, min(8, card - 8 * c), s);
  }
}

// Sorted u16 array -> register bitmap (through the LDS scratch).
__device__ __forceinline__ void expand_array(const uint16_t *vals, int card, uint32_t *s,
                                             uint64_t (&w)[kW], int lane) {
  lds_zero(s, lane);
  wave_lds_sync();
  lds_or_array(vals, card, s, lane);
  wave_lds_sync();
  lds_read_words(s, w, lane);
  wave_lds_sync();
}

__device__ __forceinline__ uint64_t prefix_xor64(uint64_t x) {
  x ^= x << 1;
  x ^= x << 2;
  x ^= x << 4;
  x ^= x << 8;
  x ^= x << 16;
  x ^= x << 32;
  return x;
}

// Toggle image (bit `start` and bit `end+1` of every run set in t) -> membership words:
// in-register prefix-xor per word plus a wave parity scan for the carry into each word.
__device__ __forceinline__ void toggles_to_words(uint64_t (&t)[kW], int lane) { // in place
  uint32_t q = 0, p0 = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t a = __popcll(t[2 * k]) & 1, b = __popcll(t[2 * k + 1]) & 1;
    q |= (a ^ b) << k;
    p0 |= a << k;
  }
  const uint32_t incl = wave_xscan_xor(q, lane);
  const uint32_t excl = incl ^ q;
  const uint32_t tot = readlane(incl, 63);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t rowc = __popc(tot & ((1u << k) - 1)) & 1;
    uint32_t c0 = rowc ^ ((excl >> k) & 1);
    uint32_t c1 = c0 ^ ((p0 >> k) & 1);
    t[2 * k] = prefix_xor64(t[2 * k]) ^ (c0 ? ~0ull : 0ull);
    t[2 * k + 1] = prefix_xor64(t[2 * k + 1]) ^ (c1 ? ~0ull : 0ull);
  }
}

// The same transform in place on the LDS image, one 16-B row per step (two passes over LDS
// instead of 32 live VGPRs: used where the caller already holds prefetched payloads).
__device__ __forceinline__ void toggles_to_words_lds(uint32_t *s, int lane) {
  uint4 *s4 = reinterpret_cast<uint4 *>(s);
  uint32_t q = 0, p0 = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 v = s4[k * 64 + lane];
    const uint32_t a = (__popc(v.x) + __popc(v.y)) & 1, b = (__popc(v.z) + __popc(v.w)) & 1;
    q |= (a ^ b) << k;
    p0 |= a << k;
  }
  const uint32_t incl = wave_xscan_xor(q, lane);
  const uint32_t excl = incl ^ q;
  const uint32_t tot = readlane(incl, 63);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint4 v = s4[k * 64 + lane];
    const uint32_t rowc = __popc(tot & ((1u << k) - 1)) & 1;
    const uint32_t c0 = rowc ^ ((excl >> k) & 1);
    const uint32_t c1 = c0 ^ ((p0 >> k) & 1);
    const uint64_t w0 = prefix_xor64(pack2(v.x, v.y)) ^ (c0 ? ~0ull : 0ull);
    const uint64_t w1 = prefix_xor64(pack2(v.z, v.w)) ^ (c1 ? ~0ull : 0ull);
    s4[k * 64 + lane] = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ void toggle_run(uint32_t *s, uint32_t q) {
  const uint32_t st = q & 0xFFFF, e1 = st + (q >> 16) + 1;
  atomicXor(&s[st >> 5], 1u << (st & 31));
  if (e1 < (uint32_t)kSpan) atomicXor(&s[e1 >> 5], 1u << (e1 & 31));
}

// Run list ((start, len-1) u16 pairs) -> register bitmap: toggle bit `start` and bit
// `start+len` (end+1) of every run into LDS, then membership = prefix-xor of the toggles.
__device__ __forceinline__ void expand_runs(const uint16_t *runs, int nruns, uint32_t *s,
                                            uint64_t (&w)[kW], int lane) {
  lds_zero(s, lane);
  wave_lds_sync();
  const uint32_t *r32 = reinterpret_cast<const uint32_t *>(runs);
  for (int i = lane; i < nruns; i += 64) toggle_run(s, r32[i]);
  wave_lds_sync();
  lds_read_words(s, w, lane);
  wave_lds_sync();
  toggles_to_words(w, lane);
}

// Any container -> register bitmap.
__device__ __forceinline__ void load_container(int type, const uint8_t *p, uint32_t card, uint32_t nruns,
                                               uint32_t *s, uint64_t (&w)[kW], int lane) {
  if (type == kBitmap) load_bitmap(p, w, lane);
  else if (type == kArray) expand_array(reinterpret_cast<const uint16_t *>(p), (int)card, s, w, lane);
  else expand_runs(reinterpret_cast<const uint16_t *>(p), (int)nruns, s, w, lane);
}

// Any container -> membership bitmap in the wave's LDS scratch (bit v of the 65536-bit image).
__device__ __forceinline__ void stage_container(int type, const uint8_t *p, uint32_t card, uint32_t nruns,
                                                uint32_t *s, int lane) {
  if (type == kBitmap) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = q[k * 64 + lane];
    uint4 *s4 = reinterpret_cast<uint4 *>(s);
#pragma unroll
    for (int k = 0; k < 8; ++k) s4[k * 64 + lane] = v[k];
  } else if (type == kArray) {
    lds_zero(s, lane);
    wave_lds_sync();
    lds_or_array(reinterpret_cast<const uint16_t *>(p), (int)card, s, lane);
  } else {
    uint64_t w[kW];
    expand_runs(reinterpret_cast<const uint16_t *>(p), (int)nruns, s, w, lane);
    lds_write_words(s, w, lane);
  }
  wave_lds_sync();
}

// Filter a sorted u16 array F against the LDS membership image `s`: keep the values whose bit
// equals !NEGATE.  F is preloaded as up to 8 uint4 chunks per lane (chunk c = lane + 64*i holds
// values 8c..8c+7; nfc chunks, nf values).  Kept values are written in order to `out` (unless
// null); returns their count (wave-uniform).  This is the whole of A&x, x&A and A\x: the result
// is a subset of an Array, hence an Array (ArrayContainer.and/andNot, BitmapContainer.and(Array),
// RunContainer.and(Array): ArrayContainer.java:184-271, BitmapContainer.java:162-172,
// RunContainer.java:305-336).
template <bool NEGATE>
__device__ __forceinline__ int filter_chunks(const uint4 (&fq)[8], int nfc, int nf, const uint32_t *s, uint16_t *out,
                                             int lane) {
  const int iters = (nfc + 63) >> 6; // wave-uniform, <= 8
  uint32_t total = 0;
  // One chunk row per step, kept values written in the same step: a scan per row keeps only
  // one row's values live (the scheduling fence stops the compiler from hoisting all 64 LDS
  // probes of the unrolled loop, which would double the kernel's VGPR footprint).
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < iters) {
      const int c = lane + 64 * i;
      const int n = c < nfc ? min(8, nf - 8 * c) : 0;
      const uint32_t x[8] = {fq[i].x & 0xFFFF, fq[i].x >> 16, fq[i].y & 0xFFFF, fq[i].y >> 16,
                             fq[i].z & 0xFFFF, fq[i].z >> 16, fq[i].w & 0xFFFF, fq[i].w >> 16};
      uint32_t keep = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t m = (s[x[k] >> 5] >> (x[k] & 31)) & 1;
        if (k < n && (m ^ (NEGATE ? 1u : 0u))) keep |= 1u << k;
      }
      const uint32_t cnt = (uint32_t)__popc(keep);
      const uint32_t incl = wave_scan_u32(cnt, lane);
      if (out) {
        uint32_t pos = total + incl - cnt;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if ((keep >> k) & 1) out[pos++] = (uint16_t)x[k];
      }
      total += readlane(incl, 63);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return (int)total;
}

// ---------------------------------------------------------------- register-preloaded payloads
// A payload of at most 8 KiB as 8 uint4 per lane: chunk c = lane + 64*i (16 bytes) in q[i].
// Buffer loads: a 32-bit per-lane offset against a wave-uniform descriptor, and lanes past the
// (16-B padded) payload get zeros from the range check without touching memory.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t chunk_rsrc(const uint8_t *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), (short)0, (int)((bytes + 15) & ~15u), 0x00020000);
}
__device__ __forceinline__ uint4 load_chunk_row(__amdgpu_buffer_rsrc_t rs, int i, int lane) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + 64 * i) * 16, 0, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void load_chunks(uint4 (&q)[8], const uint8_t *p, uint32_t bytes, int lane) {
  const __amdgpu_buffer_rsrc_t rs = chunk_rsrc(p, bytes);
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = load_chunk_row(rs, i, lane);
}
// load_chunks issuing only the 1 KiB rows the payload reaches (wave-uniform guards): a fully
// out-of-range row costs no memory request but still a full 64-lane return through the texture
// data path.  Rows past the payload keep stale registers — every consumer bounds its rows by the
// payload's count (Array values, runs, F's values, copy bytes).
__device__ __forceinline__ void load_chunks_used(uint4 (&q)[8], const uint8_t *p, uint32_t bytes, int lane) {
  const __amdgpu_buffer_rsrc_t rs = chunk_rsrc(p, bytes);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if ((uint32_t)(1024 * i) < bytes) q[i] = load_chunk_row(rs, i, lane);
}

// Exclusive prefix (over lanes) and wave total of a per-lane count in [0, 16), by bit-sliced ballots
// and mbcnt: no cross-lane data movement through LDS, no dependency chain of shuffles.
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ void ballot_scan4(uint32_t cnt, uint32_t &excl, uint32_t &total) {
  excl = 0;
  total = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const uint64_t m = __ballot((cnt >> b) & 1);
    excl += mbcnt64(m) << b;
    total += (uint32_t)__popcll(m) << b;
  }
}

// The same filter with coalesced output.  Kept values are ranked into a per-wave LDS ring `ob` of
// kStageRing u16 (16-B aligned); after each row every complete 16-B block of ranked values is
// written with one 16-B-per-lane store.  At most 7 + 512 values are pending, so a ring of 576
// never overwrites a pending value, and a block never straddles the wrap (576 % 8 == 0).  One
// wave's LDS operations execute in order, so the ranked writes, the block reads and the next
// row's writes need no drains between them.  The final partial block is written whole: result
// slots are round16(2 * bound) bytes, so bytes past the last value stay in the slot's padding.
// Rejected values go to a per-lane dummy slot instead of being branched around.
constexpr int kStageRing = 576; // >= 7 + 512 pending values, a multiple of 8
constexpr int kStageVals = kStageRing + 64;   // + one dummy slot per lane
// `reload(i)` is called once per row i as soon as fq[i] is free — right after the row's values are
// in registers, or at the start for rows this payload does not have — so the caller can stream the
// next task's payload into fq row by row instead of after the whole filter.
template <bool NEGATE, class Reload>
__device__ __forceinline__ int filter_chunks_staged(uint4 (&fq)[8], int nfc, int nf, const uint32_t *s,
                                                    uint16_t *ob, uint16_t *out, int lane, const Reload &reload) {
  const int iters = (nfc + 63) >> 6; // wave-uniform, <= 8
  uint32_t flushed = 0, tot = 0;     // values written out / ranked so far (wave-uniform)
  uint4 *out4 = reinterpret_cast<uint4 *>(out);
  const uint4 *ob4 = reinterpret_cast<const uint4 *>(ob);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i >= iters) reload(i);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < iters) {
      const int c = lane + 64 * i;
      const int n = c < nfc ? min(8, nf - 8 * c) : 0;
      const uint32_t x[8] = {fq[i].x & 0xFFFF, fq[i].x >> 16, fq[i].y & 0xFFFF, fq[i].y >> 16,
                             fq[i].z & 0xFFFF, fq[i].z >> 16, fq[i].w & 0xFFFF, fq[i].w >> 16};
      reload(i);
      // all 8 probes in flight before the first wait: one LDS round trip per row, not eight
      uint32_t m[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) m[k] = s[x[k] >> 5];
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0); // DS reads first
      __builtin_amdgcn_sched_group_barrier(0x002, 64, 0); // then the VALU work
      uint32_t keep = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) keep |= (((m[k] >> (x[k] & 31)) & 1) ^ (NEGATE ? 1u : 0u)) << k;
      keep &= (1u << n) - 1; // n <= 8: lanes past the payload keep nothing
      uint32_t excl, rowtot;
      ballot_scan4((uint32_t)__popc(keep), excl, rowtot);
      if (out) {
        uint32_t base = tot % kStageRing + excl; // < 640 + 512
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          uint32_t pos = base + (uint32_t)__popc(keep & ((1u << k) - 1));
          pos = pos >= (uint32_t)kStageRing ? pos - kStageRing : pos;
          ob[((keep >> k) & 1) ? pos : (uint32_t)(kStageRing + lane)] = (uint16_t)x[k];
        }
        const uint32_t full = (tot + rowtot) & ~7u; // values in complete blocks
        const uint32_t nb = (full - flushed) >> 3, b0 = flushed >> 3;
        if ((uint32_t)lane < nb) {
          uint32_t rb = b0 + lane; // ring block
          rb %= (uint32_t)(kStageRing / 8);
          out4[b0 + lane] = ob4[rb];
        }
        flushed = full;
      }
      tot += rowtot;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (out && tot > flushed && lane == 0) out4[flushed >> 3] = ob4[(flushed >> 3) % (kStageRing / 8)];
  return (int)tot;
}

// The staged filter with the row transposed before probing: a row's 512 values arrive as chunks of
// 8 consecutive values per lane, so in chunk order the 64 lanes of one probe instruction read
// words ~8 values apart — for a sparse F that is a fixed stride of many words and a 16-way LDS bank
// conflict (SQ_LDS_BANK_CONFLICT ≈ 13 extra cycles per probe, profiles/r01/v7).  Written once to a
// per-wave 1 KiB buffer `tb` and read back as value 64k + lane, adjacent lanes probe adjacent
// values (nearby or shared words).  Kept values are then ranked per k by one ballot, which also
// keeps them in sorted order for the same ring / 16-B block flush as filter_chunks_staged.
template <bool NEGATE>
__device__ __forceinline__ int filter_rows_transposed(const uint4 (&fq)[8], int nf, const uint32_t *s, uint16_t *ob,
                                                      uint4 *tb, uint16_t *out, int lane) {
  const int iters = (nf + 511) >> 9; // wave-uniform, <= 8
  uint32_t flushed = 0, tot = 0;
  uint4 *out4 = reinterpret_cast<uint4 *>(out);
  const uint4 *ob4 = reinterpret_cast<const uint4 *>(ob);
  const uint16_t *t16 = reinterpret_cast<const uint16_t *>(tb);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < iters) {
      // two halves of 256 values (lanes 0-31's chunks, then lanes 32-63's) through a 512-B buffer
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if ((lane >> 5) == hf) tb[lane & 31] = fq[i];
        wave_lds_sync(); // other lanes' stores: without the fence the compiler may reuse the last reads
        const int nh = min(256, nf - 512 * i - 256 * hf); // values of this half (may be <= 0)
        uint32_t y[4], m[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = t16[64 * k + lane];
#pragma unroll
        for (int k = 0; k < 4; ++k) m[k] = s[y[k] >> 5];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool keep = ((((m[k] >> (y[k] & 31)) & 1) ^ (NEGATE ? 1u : 0u)) != 0) && (64 * k + lane < nh);
          const uint64_t b = __ballot(keep);
          if (out) {
            const uint32_t pos = (tot + mbcnt64(b)) % (uint32_t)kStageRing;
            ob[keep ? pos : (uint32_t)(kStageRing + lane)] = (uint16_t)y[k];
          }
          tot += (uint32_t)__popcll(b);
        }
      }
      if (out) {
        wave_lds_sync(); // the blocks hold other lanes' ranked values
        const uint32_t full = tot & ~7u; // values in complete blocks
        const uint32_t nb = (full - flushed) >> 3, b0 = flushed >> 3;
        if ((uint32_t)lane < nb) out4[b0 + lane] = ob4[(b0 + lane) % (uint32_t)(kStageRing / 8)];
        flushed = full;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (out && tot > flushed && lane == 0) out4[flushed >> 3] = ob4[(flushed >> 3) % (kStageRing / 8)];
  return (int)tot;
}

// filter_rows_transposed with a LINEAR stage instead of a ring: after each row's flush the partial
// block (< 8 kept values) moves to the front, so a kept value's slot is (pending + mbcnt) with no
// wrap — mbcnt adds the pending count itself — and rejected lanes are masked off instead of writing a
// dummy slot.  ~8 VALU per 64 probed values instead of ~15 (ISA count).  Pending values stay < 8 + 512.
// `next()` runs once the last row of F is in the transpose buffer — F's registers are free from
// there, so the caller's prefetch of the next task's F overlaps the last row's probes and flush.
#ifndef RBG_SKIP_EMPTY_HALF
#define RBG_SKIP_EMPTY_HALF 1 // filter_rows_linear: a last row with <= 256 values skips its empty second half
#endif
template <bool NEGATE, bool STORE, class Next>
__device__ __forceinline__ int filter_rows_linear(const uint4 (&fq)[8], int nf, const uint32_t *s, uint16_t *ob,
                                                  uint4 *tb, uint16_t *out, int lane, const Next &next) {
  static_assert(7 + 512 <= kStageRing, "every slot (pending < 8, + < 512 of a row) lies below the dummies");
  const int iters = (nf + 511) >> 9; // wave-uniform, <= 8
  uint32_t tot = 0, flushed = 0;     // kept / written out so far (wave-uniform; flushed % 8 == 0)
  uint4 *out4 = reinterpret_cast<uint4 *>(out);
  uint4 *ob4 = reinterpret_cast<uint4 *>(ob);
  const uint16_t *t16 = reinterpret_cast<const uint16_t *>(tb);
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  lds_u32 *ls = (lds_u32 *)s;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < iters) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if (RBG_SKIP_EMPTY_HALF && hf == 1 && nf - 512 * i <= 256) { // the row's values all lie in its first half
          if (i == iters - 1) next();
          continue;
        }
        if ((lane >> 5) == hf) tb[lane & 31] = fq[i];
        wave_lds_sync();
        if (hf == 1 && i == iters - 1) next();
        const int nh = min(256, nf - 512 * i - 256 * hf); // values of this half (may be <= 0)
        uint32_t y[4], m[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) y[k] = t16[64 * k + lane];
#pragma unroll
        for (int k = 0; k < 4; ++k) { // word y >> 5 of the image: v_bfe + v_lshl_add (the compiler's
          uint32_t wi;                 // own lowering of the same index takes four VALU)
          asm("v_bfe_u32 %0, %1, 5, 11" : "=v"(wi) : "v"(y[k]));
          m[k] = ls[wi];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          // membership bit (v_bfe reads the offset's low 5 bits), its ballot as an integer compare (no
          // bool round trip), lanes past the half masked off in scalar registers
          const uint32_t bit = __builtin_amdgcn_ubfe(m[k], y[k], 1u);
          uint64_t b = __builtin_amdgcn_uicmp(bit, 0u, NEGATE ? 32 : 33); // ICMP_EQ / ICMP_NE
          const int lim = nh - 64 * k;
          if (lim < 64) b &= lim > 0 ? (1ull << lim) - 1ull : 0ull;
          if (STORE) {
            // kept lanes take the next slots of the linear stage, the others a per-lane dummy (a lane past
            // the half may land on the slot after the last kept value: never read as a value)
            const uint32_t pos =
                __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, tot - flushed));
            uint32_t slot;
            asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(slot) : "v"((uint32_t)(kStageRing + lane)), "v"(pos), "s"(b));
            ob[slot] = (uint16_t)y[k];
          }
          tot += (uint32_t)__popcll(b);
        }
      }
      if (STORE) {
        wave_lds_sync(); // the blocks hold other lanes' values
        const uint32_t pend = tot - flushed, nb = pend >> 3;
        if ((uint32_t)lane < nb) out4[(flushed >> 3) + lane] = ob4[lane];
        if (lane == 0 && nb && (pend & 7u)) ob4[0] = ob4[nb]; // the partial block to the front
        wave_lds_sync();
        flushed += nb << 3;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (STORE && tot > flushed && lane == 0) out4[flushed >> 3] = ob4[0];
  return (int)tot;
}

// ---- F in word order: register word j (component j & 3 of q[j >> 2]) holds payload u32 word
// 64 j + lane, i.e. values 2(64 j + lane) and +1, so adjacent lanes hold adjacent values without the
// LDS transpose of filter_rows_linear.  Only the words of the payload are loaded (wave-uniform guards).
__device__ __forceinline__ uint32_t &qword(uint4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
__device__ __forceinline__ uint32_t qword(const uint4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
__device__ __forceinline__ void load_words(uint4 (&q)[8], const uint8_t *p, uint32_t bytes, int lane) {
  const __amdgpu_buffer_rsrc_t rs = chunk_rsrc(p, bytes);
#pragma unroll
  for (int j = 0; j < 32; ++j)
    if ((uint32_t)(256 * j) < bytes) qword(q[j >> 2], j & 3) = __builtin_amdgcn_raw_buffer_load_b32(rs, (64 * j + lane) * 4, 0, 0);
}

// filter_rows_linear over F in word order: per register word the lane's two values are probed (two
// probe instructions cover 128 consecutive values), ranked with two ballots (the low value first),
// and written to the same linear stage and 16-B block flush.
template <bool NEGATE, bool STORE>
__device__ __forceinline__ int filter_words_linear(const uint4 (&fq)[8], int nf, const uint32_t *s, uint16_t *ob,
                                                   uint16_t *out, int lane) {
  static_assert(7 + 512 <= kStageRing, "every slot (pending < 8, + < 512 of a row) lies below the dummies");
  const int iters = (nf + 511) >> 9; // wave-uniform, <= 8
  uint32_t tot = 0, flushed = 0;
  uint4 *out4 = reinterpret_cast<uint4 *>(out);
  uint4 *ob4 = reinterpret_cast<uint4 *>(ob);
  typedef __attribute__((address_space(3))) const uint32_t lds_u32;
  lds_u32 *ls = (lds_u32 *)s;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (i < iters) {
      uint32_t m[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) { // all 8 probes of the row in flight
        const uint32_t x = qword(fq[i], k);
        uint32_t wl, wh;
        asm("v_bfe_u32 %0, %1, 5, 11" : "=v"(wl) : "v"(x));
        asm("v_bfe_u32 %0, %1, 21, 11" : "=v"(wh) : "v"(x));
        m[2 * k] = ls[wl];
        m[2 * k + 1] = ls[wh];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t x = qword(fq[i], k);
        const uint32_t bl = __builtin_amdgcn_ubfe(m[2 * k], x, 1u), bh = __builtin_amdgcn_ubfe(m[2 * k + 1], x >> 16, 1u);
        uint64_t b0 = __builtin_amdgcn_uicmp(bl, 0u, NEGATE ? 32 : 33);
        uint64_t b1 = __builtin_amdgcn_uicmp(bh, 0u, NEGATE ? 32 : 33);
        const int lim = nf - 128 * (4 * i + k); // values left from this word's first
        if (lim < 128) { // lane l holds values 2l, 2l+1 of the 128
          const int l0 = (lim + 1) >> 1, l1 = lim >> 1;
          b0 &= l0 > 0 ? (l0 >= 64 ? ~0ull : (1ull << l0) - 1ull) : 0ull;
          b1 &= l1 > 0 ? (1ull << l1) - 1ull : 0ull;
        }
        if (STORE) {
          const uint32_t p0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, tot - flushed));
          const uint32_t p1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b1, p0));
          uint32_t s0, s1; // the high value after the low one when both are kept
          asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(s0) : "v"((uint32_t)(kStageRing + lane)), "v"(p1), "s"(b0));
          const uint32_t ph = p1 + (uint32_t)((b0 >> lane) & 1);
          asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(s1) : "v"((uint32_t)(kStageRing + lane)), "v"(ph), "s"(b1));
          ob[s0] = (uint16_t)x;
          ob[s1] = (uint16_t)(x >> 16);
        }
        tot += (uint32_t)__popcll(b0) + (uint32_t)__popcll(b1);
      }
      if (STORE) {
        wave_lds_sync(); // the blocks hold other lanes' values
        const uint32_t pend = tot - flushed, nb = pend >> 3;
        if ((uint32_t)lane < nb) out4[(flushed >> 3) + lane] = ob4[lane];
        if (lane == 0 && nb && (pend & 7u)) ob4[0] = ob4[nb]; // the partial block to the front
        wave_lds_sync();
        flushed += nb << 3;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if (STORE && tot > flushed && lane == 0) out4[flushed >> 3] = ob4[0];
  return (int)tot;
}

__device__ __forceinline__ void store_chunks(const uint4 (&q)[8], uint8_t *p, uint32_t bytes, int lane) {
  uint4 *p4 = reinterpret_cast<uint4 *>(p);
  const int n = (int)((bytes + 15) >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + 64 * i;
    if (c < n) p4[c] = q[i];
  }
}

// The toggle image of a register-preloaded Run payload (<= 2047 runs) in the wave's LDS scratch: bit
// start and bit end+1 of every run (see stage_from_chunks); the caller reads it into registers and
// finishes with toggles_to_words — one LDS pass instead of toggles_to_words_lds's three.
__device__ __forceinline__ void stage_run_toggles(const uint4 (&q)[8], uint32_t nruns, uint32_t *s, int lane) {
  lds_zero(s, lane);
  wave_lds_sync();
  const int nchunks = (int)((nruns + 3) >> 2);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunks) {
      const uint32_t r[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
      uint32_t x[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x[2 * k] = r[k] & 0xFFFF;
        x[2 * k + 1] = (r[k] & 0xFFFF) + (r[k] >> 16) + 1;
      }
      const int nr = min(4, (int)nruns - 4 * c);
      int n = 2 * nr;
      const uint32_t last = nr == 4 ? x[7] : nr == 3 ? x[5] : nr == 2 ? x[3] : x[1];
      if (last >= (uint32_t)kSpan) --n; // only the container's last run can end at 65535
      or_chunk_values(x, n, s);
    }
  }
  wave_lds_sync();
}

// Two operands into ONE LDS image for the register path's OR / XOR (the caller zeroes it first):
// an Array's values (ds_or, or ds_xor for the second operand of an XOR: an Array's own values are
// distinct bits, so the image becomes P | Q or P ^ Q), or a Run's toggles (the second Run's by
// ds_xor: toggle images are linear under xor, so the prefix-xor of the sum is P ^ Q).
template <bool XOR>
__device__ __forceinline__ void scatter_array_chunks(const uint4 (&q)[8], uint32_t card, uint32_t *s, int lane) {
  const int nchunks = (int)((card + 7) >> 3);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunks) {
      const uint32_t x[8] = {q[i].x & 0xFFFF, q[i].x >> 16, q[i].y & 0xFFFF, q[i].y >> 16,
                             q[i].z & 0xFFFF, q[i].z >> 16, q[i].w & 0xFFFF, q[i].w >> 16};
      or_chunk_values<XOR>(x, min(8, (int)card - 8 * c), s);
    }
  }
}
template <bool XOR>
__device__ __forceinline__ void scatter_run_toggles(const uint4 (&q)[8], uint32_t nruns, uint32_t *s, int lane) {
  const int nchunks = (int)((nruns + 3) >> 2);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = lane + 64 * i;
    if (c < nchunks) {
      const uint32_t r[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
      uint32_t x[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x[2 * k] = r[k] & 0xFFFF;
        x[2 * k + 1] = (r[k] & 0xFFFF) + (r[k] >> 16) + 1;
      }
      const int nr = min(4, (int)nruns - 4 * c);
      int n = 2 * nr;
      const uint32_t last = nr == 4 ? x[7] : nr == 3 ? x[5] : nr == 2 ? x[3] : x[1];
      if (last >= (uint32_t)kSpan) --n; // only the container's last run can end at 65535
      or_chunk_values<XOR>(x, n, s);
    }
  }
}

// Membership image in LDS from a register-preloaded payload (Array <= 4096 values, Run <= 2047
// runs, Bitmap 8 KiB — i.e. every canonical container whose payload fits 8 KiB).
__device__ __forceinline__ void stage_from_chunks(int type, const uint4 (&q)[8], uint32_t card, uint32_t nruns,
                                                  uint32_t *s, int lane) {
  uint4 *s4 = reinterpret_cast<uint4 *>(s);
  if (type == kBitmap) {
#pragma unroll
    for (int i = 0; i < 8; ++i) s4[i * 64 + lane] = q[i];
  } else {
    lds_zero(s, lane);
    wave_lds_sync();
    if (type == kArray) {
      const int nchunks = (int)((card + 7) >> 3);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = lane + 64 * i;
        if (c < nchunks) {
          const uint32_t x[8] = {q[i].x & 0xFFFF, q[i].x >> 16, q[i].y & 0xFFFF, q[i].y >> 16,
                                 q[i].z & 0xFFFF, q[i].z >> 16, q[i].w & 0xFFFF, q[i].w >> 16};
          or_chunk_values(x, min(8, (int)card - 8 * c), s);
        }
      }
    } else {
      // A lane's chunk of 4 canonical runs gives 8 strictly increasing toggle positions (start,
      // end+1; runs are sorted and non-adjacent), so they group by word exactly like sorted Array
      // values: only the first and last word of a chunk can be shared with a neighbour chunk, and
      // within a word the toggles are distinct bits (OR == XOR).  An end+1 of 65536 is dropped.
      const int nchunks = (int)((nruns + 3) >> 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = lane + 64 * i;
        if (c < nchunks) {
          const uint32_t r[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
          uint32_t x[8];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            x[2 * k] = r[k] & 0xFFFF;
            x[2 * k + 1] = (r[k] & 0xFFFF) + (r[k] >> 16) + 1;
          }
          const int nr = min(4, (int)nruns - 4 * c);
          int n = 2 * nr;
          const uint32_t last = nr == 4 ? x[7] : nr == 3 ? x[5] : nr == 2 ? x[3] : x[1];
          if (last >= (uint32_t)kSpan) --n; // only the container's last run can end at 65535
          or_chunk_values(x, n, s);
        }
      }
      wave_lds_sync();
      toggles_to_words_lds(s, lane);
    }
  }
  wave_lds_sync();
}

// ---------------------------------------------------------------- metrics
// "top bit of the previous word" for every word of this lane, as per-row masks.
struct Neigh {
  uint32_t prev_top_h0; // bit k: top bit of the word before (k, lane, 0)
  uint32_t next_bot_h1; // bit k: bottom bit of the word after (k, lane, 1)
};
__device__ __forceinline__ Neigh neighbours(const uint64_t (&w)[kW], int lane) {
  uint32_t top1 = 0, bot0 = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    top1 |= (uint32_t)(w[2 * k + 1] >> 63) << k;
    bot0 |= (uint32_t)(w[2 * k] & 1) << k;
  }
  const uint32_t up = dpp<0x138>(top1);  // wave_shr:1 — lane L reads lane L-1
  const uint32_t last = readlane(top1, 63);
  const uint32_t dn = dpp<0x130>(bot0);  // wave_shl:1 — lane L reads lane L+1
  const uint32_t first = readlane(bot0, 0);
  Neigh n;
  n.prev_top_h0 = lane ? up : ((last << 1) & 0xFE);
  n.next_bot_h1 = lane < 63 ? dn : ((first >> 1) & 0x7F);
  return n;
}
__device__ __forceinline__ uint64_t run_starts(const uint64_t (&w)[kW], const Neigh &n, int j) {
  const int k = j >> 1;
  uint64_t prev = (j & 1) ? (w[j - 1] >> 63) : (uint64_t)((n.prev_top_h0 >> k) & 1);
  return w[j] & ~((w[j] << 1) | prev);
}
__device__ __forceinline__ uint64_t run_ends(const uint64_t (&w)[kW], const Neigh &n, int j) {
  const int k = j >> 1;
  uint64_t next = (j & 1) ? (uint64_t)((n.next_bot_h1 >> k) & 1) : (w[j + 1] & 1);
  return w[j] & ~((w[j] >> 1) | (next << 63));
}
__device__ __forceinline__ uint32_t lane_card(const uint64_t (&w)[kW]) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kW; ++j) c += __popcll(w[j]);
  return c;
}
// cardinality (and maximal-run count if want_runs) of the register bitmap, wave-uniform.
__device__ __forceinline__ void metrics(const uint64_t (&w)[kW], int lane, bool want_runs, int &card,
                                        int &runs) {
  uint32_t c = lane_card(w);
  uint32_t r = 0;
  if (want_runs) {
    Neigh n = neighbours(w, lane);
#pragma unroll
    for (int j = 0; j < kW; ++j) r += __popcll(run_starts(w, n, j));
  }
  card = (int)wave_sum_u32(c);
  runs = want_runs ? (int)wave_sum_u32(r) : 0;
}

// ---------------------------------------------------------------- type rules
// AB(c): BitmapContainer.and/xor/andNot, RunContainer.toBitmapOrArrayContainer (:2300-2323)
__device__ __forceinline__ int type_ab(int c) { return c <= kMaxArray ? kArray : kBitmap; }
// EFF(c,r): RunContainer.toEfficientContainer (:2326-2335), ties go to Run
__device__ __forceinline__ int type_eff(int c, int r) {
  return 2 + 4 * r <= min(kBitmapBytes, 2 * c + 2) ? kRun : type_ab(c);
}
// LR(c): BitmapContainer.repairAfterLazy (:1214-1224)
__device__ __forceinline__ int type_lr(int c) {
  return c <= kMaxArray ? kArray : (c == kSpan ? kRun : kBitmap);
}
// runOptimize on a freshly built container (ArrayContainer.java:1085-1099,
// BitmapContainer.java:1227-1246): natural AB type, then Run iff strictly smaller.
__device__ __forceinline__ int type_runopt(int c, int r) {
  if (c <= kMaxArray) return 2 * c > 2 + 4 * r ? kRun : kArray;
  return kBitmapBytes > 2 + 4 * r ? kRun : kBitmap;
}

// ---------------------------------------------------------------- emission
// Writes the container payload for `type` at `out` (16-B aligned slot); returns payload bytes.
// `s` is the wave's 8 KiB LDS scratch (free on entry).
#ifndef RBG_EMIT_ARRAY_PAIRS
#define RBG_EMIT_ARRAY_PAIRS 0 // 1: two values per trip of the Array emission loop (measured neutral)
#endif
__device__ __forceinline__ uint32_t emit_container(int type, const uint64_t (&w)[kW], int card, int runs,
                                                   uint8_t *out, uint32_t *s, int lane) {
  if (type == kBitmap) {
    uint4 *o = reinterpret_cast<uint4 *>(out);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      o[k * 64 + lane] = make_uint4((uint32_t)w[2 * k], (uint32_t)(w[2 * k] >> 32),
                                    (uint32_t)w[2 * k + 1], (uint32_t)(w[2 * k + 1] >> 32));
    return kBitmapBytes;
  }
  uint16_t *s16 = reinterpret_cast<uint16_t *>(s);
  if (type == kArray) {
    // rank of the first value of every word: packed per-row (16-bit fields) wave scan
    uint32_t n[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) n[k] = __popcll(w[2 * k]) + __popcll(w[2 * k + 1]);
    const uint64_t P0 = (uint64_t)n[0] | ((uint64_t)n[1] << 16) | ((uint64_t)n[2] << 32) | ((uint64_t)n[3] << 48);
    const uint64_t P1 = (uint64_t)n[4] | ((uint64_t)n[5] << 16) | ((uint64_t)n[6] << 32) | ((uint64_t)n[7] << 48);
    const uint64_t S0 = wave_scan_u64(P0, lane), S1 = wave_scan_u64(P1, lane);
    const uint64_t E0 = S0 - P0, E1 = S1 - P1;
    const uint64_t T0 = pack2(readlane((uint32_t)S0, 63), readlane((uint32_t)(S0 >> 32), 63));
    const uint64_t T1 = pack2(readlane((uint32_t)S1, 63), readlane((uint32_t)(S1 >> 32), 63));
    uint32_t rowoff = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint64_t E = k < 4 ? E0 : E1, T = k < 4 ? T0 : T1;
      const int sh = 16 * (k & 3);
      uint32_t pos = rowoff + (uint32_t)((E >> sh) & 0xFFFF);
      rowoff += (uint32_t)((T >> sh) & 0xFFFF);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint64_t x = w[2 * k + h];
        const uint32_t base = (uint32_t)(128 * k + 2 * lane + h) << 6;
#if RBG_EMIT_ARRAY_PAIRS
        // two values per trip: a divergent while runs for the lane with the most values of the word
        while (x) {
          s16[pos] = (uint16_t)(base + __builtin_ctzll(x));
          x &= x - 1;
          if (x) {
            s16[pos + 1] = (uint16_t)(base + __builtin_ctzll(x));
            x &= x - 1;
            ++pos;
          }
          ++pos;
        }
#else
        while (x) {
          s16[pos++] = (uint16_t)(base + __builtin_ctzll(x));
          x &= x - 1;
        }
#endif
      }
    }
    wave_lds_sync();
    const uint32_t bytes = 2u * (uint32_t)card;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
    uint4 *o = reinterpret_cast<uint4 *>(out);
    for (uint32_t i = lane; i * 16 < bytes; i += 64) o[i] = s4[i];
    wave_lds_sync();
    return bytes;
  }
  // Run: S[rank] = start, E[rank] = end; the i-th end closes the i-th run.  Run starts are
  // recomputed where they are used (3 ops per word) rather than held in 32 more VGPRs.
  Neigh nb = neighbours(w, lane);
  uint32_t ns[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) ns[k] = __popcll(run_starts(w, nb, 2 * k)) + __popcll(run_starts(w, nb, 2 * k + 1));
  const uint64_t P0 = (uint64_t)ns[0] | ((uint64_t)ns[1] << 16) | ((uint64_t)ns[2] << 32) | ((uint64_t)ns[3] << 48);
  const uint64_t P1 = (uint64_t)ns[4] | ((uint64_t)ns[5] << 16) | ((uint64_t)ns[6] << 32) | ((uint64_t)ns[7] << 48);
  const uint64_t S0 = wave_scan_u64(P0, lane), S1 = wave_scan_u64(P1, lane);
  const uint64_t E0 = S0 - P0, E1 = S1 - P1;
  const uint64_t T0 = pack2(readlane((uint32_t)S0, 63), readlane((uint32_t)(S0 >> 32), 63));
  const uint64_t T1 = pack2(readlane((uint32_t)S1, 63), readlane((uint32_t)(S1 >> 32), 63));
  uint16_t *S = s16, *E = s16 + 2048;
  uint32_t rowoff = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t Ex = k < 4 ? E0 : E1, T = k < 4 ? T0 : T1;
    const int sh = 16 * (k & 3);
    uint32_t sp = rowoff + (uint32_t)((Ex >> sh) & 0xFFFF);
    rowoff += (uint32_t)((T >> sh) & 0xFFFF);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * k + h;
      // a run is open into this word iff the bit before it AND its bit 0 are set (a run that ends on
      // the previous word's last bit was already counted there)
      const uint32_t open = (uint32_t)(h ? (w[j - 1] >> 63) : ((nb.prev_top_h0 >> k) & 1)) & (uint32_t)(w[j] & 1);
      uint32_t ep = sp - open;
      const uint32_t base = (uint32_t)(128 * k + 2 * lane + h) << 6;
      // starts and ends of the word in ONE loop: a divergent while runs for the slowest lane, so two
      // loops cost (max starts) + (max ends) trips, one costs about max(starts, ends)
      uint64_t x = run_starts(w, nb, j), y = run_ends(w, nb, j);
      while (x | y) {
        if (x) {
          S[sp++] = (uint16_t)(base + __builtin_ctzll(x));
          x &= x - 1;
        }
        if (y) {
          E[ep++] = (uint16_t)(base + __builtin_ctzll(y));
          y &= y - 1;
        }
      }
    }
  }
  wave_lds_sync();
  uint32_t *o = reinterpret_cast<uint32_t *>(out);
  for (int i = lane; i < runs; i += 64) {
    uint32_t a = S[i], b = E[i];
    o[i] = a | ((b - a) << 16);
  }
  wave_lds_sync();
  return 4u * (uint32_t)runs;
}

// Copy a payload (multiple of 16 bytes after rounding; slots are 16-B padded).
__device__ __forceinline__ void copy_payload(const uint8_t *src, uint8_t *dst, uint64_t bytes, int lane) {
  const uint4 *a = reinterpret_cast<const uint4 *>(src);
  uint4 *b = reinterpret_cast<uint4 *>(dst);
  const uint64_t n = (bytes + 15) >> 4;
  for (uint64_t i = lane; i < n; i += 64) b[i] = a[i];
}

} // namespace rbg
