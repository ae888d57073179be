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

// exclusive block-wide prefix of v (blockDim.x a multiple of 64, <= 1024); *total = the sum
__device__ __forceinline__ uint32_t block_xscan(uint32_t v, uint32_t *wtot, uint32_t &total) {
  const int lane = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t inc = wave_scan_u32(v, lane);
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
  for (int i = 0; i < nw; ++i) {
    const uint32_t t = wtot[i];
    if (i < w) before += t;
    total += t;
  }
  __syncthreads();
  return before + inc - v;
}
// Cross-block hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, first table row): every block's
// words and counters are stored sc1, each storing wave waits for them (s_waitcnt vmcnt(0)), then one
// agent-scope add per block; the block whose add comes last reads them with sc1 loads.  This leans on the
// gfx94x / gfx95x meaning of sc1 (relaxed agent-scope atomics go to the device-coherent L2) and on vmcnt
// covering stores and no-return atomics — not on the HIP memory model's release / acquire pairs:
// other targets are refused at compile time rather than given a hand-off that could read stale words.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "the one-launch hand-off (st_sc1 / ld_sc1 + s_waitcnt vmcnt) is written for gfx942 / gfx950"
#endif
__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
  return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
// lanes below this one with their bit set in m
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// Flags of a 256-thread block: the block's number of set flags (every thread) and a thread's exclusive
// rank among them — stream compaction of a per-block layout (block totals scanned separately).
__device__ __forceinline__ uint32_t block_flag_count(bool f, uint32_t *wt) {
  const uint64_t m = __ballot(f);
  if ((threadIdx.x & 63) == 0) wt[threadIdx.x >> 6] = (uint32_t)__popcll(m);
  __syncthreads();
  return wt[0] + wt[1] + wt[2] + wt[3];
}
__device__ __forceinline__ uint32_t block_flag_rank(bool f, uint32_t *wt) {
  const uint64_t m = __ballot(f);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) wt[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t r = mbcnt64(m);
  for (int i = 0; i < w; ++i) r += wt[i];
  return r;
}
// The Array filter (A&x, x&A, A\x: the result is a subset of an Array, hence an Array —
// ArrayContainer.and/andNot, BitmapContainer.and(Array), RunContainer.and(Array):
// ArrayContainer.java:184-271, BitmapContainer.java:162-172, RunContainer.java:305-336).  F, a sorted
// u16 array, is preloaded as up to 8 uint4 chunks per lane (chunk c = lane + 64*i holds values
// 8c..8c+7); its values whose bit in the LDS membership image `s` equals !NEGATE are kept, in order.
// Each row of 512 values is transposed through a per-wave buffer `tb` first: in chunk order the 64
// lanes of one probe read words ~8 values apart, a 16-way LDS bank conflict for a sparse F
// (SQ_LDS_BANK_CONFLICT ≈ 13 extra cycles per probe, profiles/r01/v7); read back as value 64k + lane,
// adjacent lanes probe adjacent values.  Kept values are ranked per probe by one ballot into a per-wave
// linear LDS stage `ob` and written as whole 16-B blocks, one 16-B-per-lane store per row; the final
// partial block is written whole (result slots are round16(2 * bound) bytes, so bytes past the last
// value stay in the slot's padding).  Rejected lanes write a per-lane dummy slot.
constexpr int kStageRing = 576;             // >= 7 + 512 pending values, a multiple of 8
constexpr int kStageVals = kStageRing + 64; // + one dummy slot per lane
// The stage is LINEAR: after each row's flush the partial block (< 8 kept values) moves to the front,
// so a kept value's slot is (pending + mbcnt) with no wrap — mbcnt adds the pending count itself.
// ~8 VALU per 64 probed values (a ring with modulo took ~15, ISA count).  Pending values stay < 8 + 512.
// A last row with <= 256 values skips its empty second half.
template <bool NEGATE, bool STORE>
__device__ __forceinline__ int filter_rows_linear(const uint4 (&fq)[8], int nf, const uint32_t *s, uint16_t *ob,
                                                  uint4 *tb, uint16_t *out, int lane) {
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
        if (hf == 1 && nf - 512 * i <= 256) continue; // the row's values all lie in its first half
        if ((lane >> 5) == hf) tb[lane & 31] = fq[i];
        wave_lds_sync();
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
        while (x) {
          s16[pos++] = (uint16_t)(base + __builtin_ctzll(x));
          x &= x - 1;
        }
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
  // four runs per lane per trip: 8-B reads of S and E, one 16-B store (the slot is 16-B padded and
  // holds round16(4 runs) bytes: a Run result has 4r <= 2c <= its slot bound; the pad is zeroed)
  const uint2 *S2 = reinterpret_cast<const uint2 *>(S), *E2 = reinterpret_cast<const uint2 *>(E);
  uint4 *o4 = reinterpret_cast<uint4 *>(out);
  for (int i = lane; 4 * i < runs; i += 64) {
    const uint2 a = S2[i], b = E2[i];
    const uint32_t s0 = a.x & 0xFFFF, s1 = a.x >> 16, s2 = a.y & 0xFFFF, s3 = a.y >> 16;
    const uint32_t e0 = b.x & 0xFFFF, e1 = b.x >> 16, e2 = b.y & 0xFFFF, e3 = b.y >> 16;
    const int n = runs - 4 * i;
    o4[i] = make_uint4(s0 | ((e0 - s0) << 16), n > 1 ? s1 | ((e1 - s1) << 16) : 0u,
                       n > 2 ? s2 | ((e2 - s2) << 16) : 0u, n > 3 ? s3 | ((e3 - s3) << 16) : 0u);
  }
  wave_lds_sync();
  return 4u * (uint32_t)runs;
}

// ---------------------------------------------------------------- balanced emission (round 6)
// emit_container's Array / Run loops run per word: a word's trip count is the largest bit count any lane has in
// that word, so a container pays Σ over its 16 word slots of the wave's maximum (OR's Run results: ~37 % of a
// register-path wave).  Here each lane owns 16 CONSECUTIVE words (1024 bit positions), counts
// its values / run starts, one wave scan ranks them, and ONE loop per lane walks its own bits with a cursor
// over the LDS image: the trip count is the largest per-lane total, ~2-3x fewer trips.  The image is stored
// transposed (word 16 q + j at u64 index 64 j + q, q = the walking lane) so lanes reading their j-th words hit
// distinct banks; the results go to a second 8 KiB LDS stage `o2` and leave as 16-B blocks.
__device__ __forceinline__ uint32_t tword(uint32_t g) { return ((g & 15u) << 6) | (g >> 4); }
__device__ __forceinline__ void lds_write_words_t(uint32_t *s, const uint64_t (&w)[kW], int lane) {
  uint64_t *s64 = reinterpret_cast<uint64_t *>(s);
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int h = 0; h < 2; ++h) s64[tword((uint32_t)(128 * k + 2 * lane + h))] = w[2 * k + h];
}
// the 16-B blocks of `bytes` bytes of the stage to out (slots are 16-B padded; the pad is written as zeros)
__device__ __forceinline__ uint32_t pad_word(uint32_t v, int valid) { // valid bytes of the word, from the low end
  return valid >= 4 ? v : valid <= 0 ? 0u : v & ((1u << (8 * valid)) - 1u);
}
__device__ __forceinline__ void stage_out(const uint32_t *o2, uint32_t bytes, uint8_t *out, int lane) {
  const uint4 *s4 = reinterpret_cast<const uint4 *>(o2);
  uint4 *o = reinterpret_cast<uint4 *>(out);
  for (uint32_t i = lane; i * 16 < bytes; i += 64) {
    uint4 v = s4[i];
    const int rem = (int)(bytes - i * 16);
    if (rem < 16) v = make_uint4(pad_word(v.x, rem), pad_word(v.y, rem - 4), pad_word(v.z, rem - 8), pad_word(v.w, rem - 12));
    o[i] = v;
  }
}
__device__ __forceinline__ uint32_t emit_array_bal(const uint64_t (&w)[kW], int card, uint8_t *out, uint32_t *s,
                                                   uint32_t *o2, int lane) {
  lds_write_words_t(s, w, lane);
  wave_lds_sync();
  const uint64_t *s64 = reinterpret_cast<const uint64_t *>(s);
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) cnt += (uint32_t)__popcll(s64[64 * j + lane]);
  uint32_t pos = wave_scan_u32(cnt, lane) - cnt;
  uint16_t *v16 = reinterpret_cast<uint16_t *>(o2);
  uint32_t j = 0;
  uint64_t cur = s64[lane], nxt = s64[64 + lane];
  const uint32_t base = (uint32_t)lane << 10;
  for (uint32_t t = 0; t < cnt; ++t) {
    while (cur == 0) { // the next non-empty word (its successor already in flight)
      ++j;
      cur = nxt;
      nxt = j < 15 ? s64[64 * (j + 1) + lane] : 0ull;
    }
    v16[pos++] = (uint16_t)(base + (j << 6) + (uint32_t)__builtin_ctzll(cur));
    cur &= cur - 1;
  }
  wave_lds_sync();
  const uint32_t bytes = 2u * (uint32_t)card;
  stage_out(o2, bytes, out, lane);
  wave_lds_sync();
  return bytes;
}
// Run: a lane takes the runs that START in its words; each run's end is the first run end at or after its start
// (it may lie in a later lane's words: the end cursor walks on through the image)
__device__ __forceinline__ uint32_t emit_run_bal(const uint64_t (&w)[kW], int runs, uint8_t *out, uint32_t *s,
                                                 uint32_t *o2, int lane) {
  lds_write_words_t(s, w, lane);
  wave_lds_sync();
  const uint64_t *s64 = reinterpret_cast<const uint64_t *>(s);
  const uint32_t g0 = 16u * (uint32_t)lane;
  // the top bit of the word before the lane's first (run starts: a set bit whose predecessor is clear)
  const uint64_t top0 = lane ? s64[tword(g0 - 1)] >> 63 : 0ull;
  uint32_t cnt = 0;
  {
    uint64_t p = top0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t v = s64[64 * j + lane];
      cnt += (uint32_t)__popcll(v & ~((v << 1) | p));
      p = v >> 63;
    }
  }
  const uint32_t pos = wave_scan_u32(cnt, lane) - cnt;
  uint32_t js = 0;
  uint64_t vs = s64[lane], xs = vs & ~((vs << 1) | top0);
  uint32_t ge = 0;            // end cursor: word index, its word, the next word's bit 0, the word's unread ends
  uint64_t ve = 0, vn = 0, xe = 0;
  bool einit = false;
  for (uint32_t t = 0; t < cnt; ++t) {
    while (xs == 0) {
      const uint64_t p = vs >> 63;
      ++js;
      vs = s64[64 * js + lane];
      xs = vs & ~((vs << 1) | p);
    }
    const uint32_t sb = (uint32_t)__builtin_ctzll(xs);
    xs &= xs - 1;
    const uint32_t st = ((g0 + js) << 6) + sb;
    if (!einit) { // the end cursor starts at the first start
      einit = true;
      ge = g0 + js;
      ve = vs;
      vn = ge < 1023 ? s64[tword(ge + 1)] : 0ull;
      xe = (ve & ~((ve >> 1) | ((vn & 1ull) << 63))) & (~0ull << sb);
    }
    while (xe == 0) {
      ++ge;
      ve = vn;
      vn = ge < 1023 ? s64[tword(ge + 1)] : 0ull;
      xe = ve & ~((ve >> 1) | ((vn & 1ull) << 63));
    }
    const uint32_t en = (ge << 6) + (uint32_t)__builtin_ctzll(xe);
    xe &= xe - 1;
    o2[pos + t] = st | ((en - st) << 16);
  }
  wave_lds_sync();
  const uint32_t bytes = 4u * (uint32_t)runs;
  stage_out(o2, bytes, out, lane);
  wave_lds_sync();
  return bytes;
}
// emit_container with the balanced Array / Run emission; o2: a second 8 KiB LDS stage of the wave
__device__ __forceinline__ uint32_t emit_container_bal(int type, const uint64_t (&w)[kW], int card, int runs,
                                                       uint8_t *out, uint32_t *s, uint32_t *o2, int lane) {
  if (type == kArray) return emit_array_bal(w, card, out, s, o2, lane);
  if (type == kRun) return emit_run_bal(w, runs, out, s, o2, lane);
  return emit_container(type, w, card, runs, out, s, lane);
}

// Copy a payload (multiple of 16 bytes after rounding; slots are 16-B padded), 8 KiB per round with every
// load of the round in flight before its stores (a load -> store loop waits one memory latency per 1 KiB:
// the compiler cannot move a load above the previous iteration's store)
__device__ __forceinline__ void copy_payload(const uint8_t *src, uint8_t *dst, uint64_t bytes, int lane) {
  for (uint64_t o = 0; o < bytes; o += kBitmapBytes) {
    const uint32_t nb = (uint32_t)min<uint64_t>(bytes - o, (uint64_t)kBitmapBytes);
    uint4 q[8];
    load_chunks(q, src + o, nb, lane);
    store_chunks(q, dst + o, nb, lane);
  }
}

} // namespace rbg
