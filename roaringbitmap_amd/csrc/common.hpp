// common.hpp — shared host/device definitions of librbgpu (MI355X / gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rbgpu.h"

namespace rbg {

constexpr int kArray = RB_ARRAY, kBitmap = RB_BITMAP, kRun = RB_RUN;
constexpr uint8_t kEmpty = 0xFF;      // result slot whose container was dropped (isEmpty)
constexpr int kMaxArray = 4096;       // ArrayContainer.DEFAULT_MAX_SIZE (ArrayContainer.java:27)
constexpr int kSpan = 65536;          // values per container
constexpr int kBitmapBytes = 8192;    // BitmapContainer payload
constexpr int kRunArrayThreshold = 32; // RunContainer.andNot/xor array threshold (RunContainer.java:576,2412)

// Read-only device view of one rbgpu_set.
struct SetView {
  const uint64_t *begin;  // [n_bitmaps+1]
  const uint16_t *key;    // [n_cont]
  const uint8_t *type;    // [n_cont]
  const uint32_t *card;   // [n_cont]
  const uint16_t *nruns;  // [n_cont]
  const uint64_t *off;    // [n_cont]
  const uint8_t *payload;
};

// Writable device view of a result set's container arrays.
struct OutView {
  uint16_t *key;
  uint8_t *type;
  uint32_t *card;
  uint16_t *nruns;
  uint64_t *off;
};

// One container-level work item of a pairwise call, self-contained so the compute kernels reach
// the payloads after a single (scalar) record load.  Records are stored per kernel category.
struct TaskRec {
  uint64_t pa, pb; // payload byte offsets in A / B (unused side: 0)
  uint64_t out;    // byte offset of the output slot in the result arena
  uint32_t t;      // merged (result-order) task index
  uint32_t da, db; // descriptor: type | card << 2; type 3 = no container on that side
  uint16_t ra, rb; // run counts
};
constexpr uint32_t kAbsent = 3;
constexpr uint32_t kEmptyBitmap = 0xFFFFFFFFu; // RB_EMPTY_BITMAP: a pair index naming an empty bitmap
__host__ __device__ inline uint32_t desc_type(uint32_t d) { return d & 3; }
__host__ __device__ inline uint32_t desc_card(uint32_t d) { return d >> 2; }

// Striped accounting counters (stats word w, stripe s): d_stats[w * kStripes + s].
// Word 8 is a per-call result word (the small-batch path's result container count), read back
// with the counters so the call needs one device-to-host copy.
constexpr int kStatWords = 9, kStripes = 64;

// FastAggregation.priorityqueue_or's intermediate bitmaps (api.hip pq_or) carry two marks in the card
// word of their containers, never seen outside that call: a lazy Bitmap (the reference's cardinality
// -1 after a lazy OR) and a Run kept as 8 KiB of bitmap words (a lazily merged Run of 2048..4096 runs,
// RunContainer.lazyorToRun, whose run list would not fit an 8 KiB slot).
constexpr uint32_t kLazyCard = 1u << 28;
constexpr uint32_t kRunAsBitmap = 1u << 29;
constexpr uint32_t kCardMarks = kLazyCard | kRunAsBitmap;
// internal pairwise ops of priorityqueue_or (Container.lazyOR / lazyIOR roles, run as the OR kernels;
// kLazyRepair: a bitmap with itself, each container through its repairAfterLazy)
enum { kLazyStatic = 16, kLazyIor = 17, kLazyIorBf = 18, kLazyRepair = 19 };
__host__ __device__ inline bool is_lazy_op(int op) { return op >= kLazyStatic && op <= kLazyRepair; }
__host__ __device__ inline bool bitmap_payload(int type, uint32_t card) {
  return type == kBitmap || (type == kRun && (card & kRunAsBitmap));
}
__host__ __device__ inline uint64_t payload_bytes(int type, uint32_t card, uint32_t nruns) {
  return bitmap_payload(type, card) ? (uint64_t)kBitmapBytes : type == kArray ? 2ull * card : 4ull * nruns;
}
__host__ __device__ inline uint64_t round16(uint64_t x) { return (x + 15) & ~15ull; }

// Packed 8-B container record (rbgpu_set::mrec / krec): payload byte offset (40 bits), card (17),
// min(nruns, 15) (4), type (2).  A run count of 15 means ">= 15" (the Run-list fast paths take <= 8).
__host__ __device__ inline uint64_t pack_rec(uint32_t typ, uint32_t card, uint32_t nr, uint64_t off) {
  return off | ((uint64_t)card << 40) | ((uint64_t)(nr < 15u ? nr : 15u) << 57) | ((uint64_t)(typ & 3u) << 61);
}
__host__ __device__ inline uint32_t rec_type(uint64_t r) { return (uint32_t)(r >> 61) & 3u; }
__host__ __device__ inline uint32_t rec_card(uint64_t r) { return (uint32_t)(r >> 40) & 0x1FFFFu; }
__host__ __device__ inline uint32_t rec_nruns(uint64_t r) { return (uint32_t)(r >> 57) & 15u; }
__host__ __device__ inline uint64_t rec_off(uint64_t r) { return r & ((1ull << 40) - 1); }
constexpr uint64_t kRecMaxPayload = 1ull << 40;
// naive_xor's 4-B member record (round 6; rbgpu_set::krec and the per-call records): a Run of 1..8 runs as
// its 16-B payload unit (29 bits) and nruns - 1 (3 bits); any other container — another type, more runs,
// an offset past 8 GiB or not 16-B aligned — is kXBad (its key goes to the generic kernel).  The card is
// not stored: the kernel sums it from the runs it loads anyway.
constexpr uint32_t kXBad = 0xFFFFFFFFu;
__host__ __device__ inline uint32_t pack_xrec(bool run, uint32_t nr, uint64_t off) {
  const uint64_t u = off >> 4;
  return run && nr >= 1u && nr <= 8u && !(off & 15u) && u < (1ull << 29) - 1u ? (uint32_t)(u << 3) | (nr - 1u) : kXBad;
}
__host__ __device__ inline bool xrec_ok(uint32_t r) { return r != kXBad; }
__host__ __device__ inline uint32_t xrec_nruns(uint32_t r) { return r != kXBad ? (r & 7u) + 1u : 0u; }
__host__ __device__ inline uint64_t xrec_off(uint32_t r) { return r != kXBad ? (uint64_t)(r >> 3) << 4 : 0ull; }
// the same from a packed 8-B record
__host__ __device__ inline uint32_t xrec_of(uint64_t m) { return pack_xrec(rec_type(m) == (uint32_t)kRun, rec_nruns(m), rec_off(m)); }

} // namespace rbg
