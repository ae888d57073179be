/*
 * rbref — CPU restatement of the reference RoaringBitmap set-algebra hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity oracle for the MI355X engine
 * (roaringbitmap_amd / librbgpu).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker or as the timed CPU baseline —
 * never as the thing measured or shipped.  The product path never links it.
 *
 * Reference: ponder-lab/RoaringBitmap 1.3.1-SNAPSHOT (Java).  Every function in rbref.cpp
 * cites the reference file:line it restates (paths relative to
 * RoaringBitmap/src/main/java/org/roaringbitmap/).
 *
 * Pinning: the real-data golden cardinalities of
 * jmh/src/test/java/org/roaringbitmap/realdata/RealDataBenchmark*Test.java, the byte-level
 * fixtures testdata/bitmapwithruns.bin / bitmapwithoutruns.bin (round trip + runOptimize KAT),
 * the crashproneinput*.bin rejections (TestAdversarialInputs.java:18-62), and the container
 * type pins of TestRunContainer / TestBitmapContainer.  The Java reference itself cannot run
 * here (no JDK), so it is not built under oracle/_ref.
 */
#ifndef RBREF_H
#define RBREF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rbref_bitmap rbref_bitmap;

/* op codes, identical to rbgpu.h */
enum { RBREF_AND = 0, RBREF_OR = 1, RBREF_XOR = 2, RBREF_ANDNOT = 3 };

/* wide semantics, identical to rbgpu.h rb_wide_sem */
enum {
  RBREF_FAST_OR = 0,      /* FastAggregation.or == naive_or            FastAggregation.java:602 */
  RBREF_FAST_AND = 1,     /* FastAggregation.and(varargs)              FastAggregation.java:37  */
  RBREF_WORKSHY_AND = 2,  /* FastAggregation.workShyAnd                FastAggregation.java:356 */
  RBREF_NAIVE_AND = 3,    /* FastAggregation.naive_and(varargs)        FastAggregation.java:328 */
  RBREF_FAST_XOR = 4,     /* FastAggregation.xor == naive_xor          FastAggregation.java:772 */
  RBREF_PAR_OR = 5,       /* ParallelAggregation.or                    ParallelAggregation.java:161 */
  RBREF_PAR_XOR = 6,      /* ParallelAggregation.xor                   ParallelAggregation.java:182 */
  RBREF_NAIVE_AND_ITER = 7, /* FastAggregation.and(Iterator)           FastAggregation.java:26,304 */
  RBREF_HORIZONTAL_OR = 8,  /* FastAggregation.horizontal_or           FastAggregation.java:124-231 */
  RBREF_HORIZONTAL_XOR = 9, /* FastAggregation.horizontal_xor          FastAggregation.java:243-289 */
  RBREF_PQ_OR = 10,         /* FastAggregation.priorityqueue_or        FastAggregation.java:615-721 */
  RBREF_PQ_XOR = 11,        /* FastAggregation.priorityqueue_xor       FastAggregation.java:732-752 */
  /* buffer/BufferFastAggregation entry points whose results differ from FastAggregation's */
  RBREF_BUFFER_NAIVE_OR = 12,   /* naive_or / or(MutableRoaringBitmap...)  buffer/BufferFastAggregation.java:711-717 */
  RBREF_BUFFER_PQ_OR = 13,      /* priorityqueue_or(ImmutableRoaringBitmap...)                       :810-866 */
  RBREF_BUFFER_PQ_OR_ITER = 14, /* priorityqueue_or(Iterator)                                        :869-930 */
  RBREF_BUFFER_PQ_XOR = 15      /* priorityqueue_xor (< 2 bitmaps: IllegalArgumentException -> NULL) :933-958 */
};

/* container type tags (RoaringFormatSpec order used by the device SoA) */
enum { RBREF_ARRAY = 0, RBREF_BITMAP = 1, RBREF_RUN = 2 };

/* status codes (same values as rbgpu.h) */
enum { RBREF_OK = 0, RBREF_EFORMAT = -1, RBREF_EINVAL = -2 };

rbref_bitmap *rbref_new(void);
void rbref_free(rbref_bitmap *b);
rbref_bitmap *rbref_clone(const rbref_bitmap *b);

/* RoaringBitmap.bitmapOf(int...) — RoaringBitmap.java:566, add path ArrayContainer.add */
rbref_bitmap *rbref_bitmap_of(const uint32_t *vals, size_t n);
/* RoaringBitmap.runOptimize — RoaringBitmap.java:2764; returns 1 if any Run container */
int rbref_run_optimize(rbref_bitmap *b);

uint64_t rbref_cardinality(const rbref_bitmap *b);
uint32_t rbref_container_count(const rbref_bitmap *b);
int rbref_container_info(const rbref_bitmap *b, uint32_t i, uint16_t *key, uint8_t *type,
                         uint32_t *card, uint32_t *nruns);
/* all values, ascending; returns count (writes at most cap) */
uint64_t rbref_to_array(const rbref_bitmap *b, uint32_t *out, uint64_t cap);

/* RoaringArray.deserialize / serialize — RoaringArray.java:276-348, 851-953 */
int rbref_deserialize(const uint8_t *buf, size_t len, rbref_bitmap **out);
uint64_t rbref_serialized_size(const rbref_bitmap *b);
int rbref_serialize(const rbref_bitmap *b, uint8_t *dst, uint64_t cap);

/* Build from one bitmap's host SoA slice (keys/types/cards/nruns + payload pointers). */
int rbref_from_soa(uint32_t n, const uint16_t *keys, const uint8_t *types, const uint32_t *cards,
                   const uint16_t *nruns, const uint8_t *payload, const uint64_t *offsets,
                   rbref_bitmap **out);

/* static RoaringBitmap.and/or/xor/andNot — RoaringBitmap.java:377,860,1071,444 */
rbref_bitmap *rbref_op(int op, const rbref_bitmap *a, const rbref_bitmap *b);
/* RoaringBitmap.andCardinality/orCardinality/xorCardinality/andNotCardinality */
int64_t rbref_op_cardinality(int op, const rbref_bitmap *a, const rbref_bitmap *b);
/* Roaring64Bitmap.xor's per-key rule (longlong/Roaring64Bitmap.java:392-460): matched keys xor'd, the
 * result kept even when empty; unmatched keys cloned */
rbref_bitmap *rbref_xor_keep_empty(const rbref_bitmap *a, const rbref_bitmap *b);
/* in-place RoaringBitmap.and/or/xor/andNot(x2) — RoaringBitmap.java:1272,2481,3296,1346 */
int rbref_op_inplace(int op, rbref_bitmap *a, const rbref_bitmap *b);

/* wide aggregation over bitmaps[0..n) (pointer identity matters for naive_and); NULL when the
 * reference throws (BUFFER_PQ_XOR below 2 bitmaps) */
rbref_bitmap *rbref_wide(int sem, const rbref_bitmap *const *bitmaps, size_t n);
/* The same aggregation computed key-parallel on `threads` host threads (every semantics is per-key
 * independent; ParallelAggregation.or/xor are the reference's own key-parallel entry points,
 * ParallelAggregation.java:161-195).  Identical result; the CPU baseline on all host cores. */
rbref_bitmap *rbref_wide_mt(int sem, const rbref_bitmap *const *bitmaps, size_t n, int threads);
/* FastAggregation.andCardinality / orCardinality — FastAggregation.java:71-101 */
int64_t rbref_wide_cardinality(int op, const rbref_bitmap *const *bitmaps, size_t n);

/* CPU-baseline helper: runs op over npairs pairs with `threads` threads (pairs split by
 * contiguous ranges).  Returns total result cardinality and total serialized payload bytes
 * of the results. */
int rbref_pairwise_batch(int op, const rbref_bitmap *const *a, const rbref_bitmap *const *b,
                         size_t npairs, int threads, uint64_t *total_card, uint64_t *total_containers);

/* BitSliceIndex compare (bsi/.../RoaringBitmapSliceIndex.java:475-577; the static ops of
 * Roaring64BitmapSliceIndex.compare are the same Container and/or/andNot): compareUsingMinMax, then
 * oNeilCompare (:432-472), RANGE as GE(start) AND LE(end).  slices[0..nslices) low bit first, ebm the
 * existence bitmap, found NULL or the foundSet; op is BitmapSliceIndex.Operation's ordinal (EQ, NEQ, LE, LT,
 * GE, GT, RANGE).  Values unsigned.  The C++ twin of oracle/rbref.py bsi_compare. */
enum { RBREF_BSI_EQ = 0, RBREF_BSI_NEQ, RBREF_BSI_LE, RBREF_BSI_LT, RBREF_BSI_GE, RBREF_BSI_GT, RBREF_BSI_RANGE };
rbref_bitmap *rbref_bsi_compare(const rbref_bitmap *const *slices, size_t nslices, const rbref_bitmap *ebm, int op,
                                uint64_t start, uint64_t end, const rbref_bitmap *found, uint64_t vmin, uint64_t vmax);
/* CPU-baseline helper: the compare over nkeys independent indexes (per high key: nslices slices then ebM,
 * per_key[k * (nslices + 1) + i]), keys split over `threads` host threads in contiguous ranges, the way a
 * key-parallel BSI (BitSliceIndexBase.java:99-166's parallel split) divides the work.  Returns the total
 * result cardinality. */
uint64_t rbref_bsi_compare_keys(const rbref_bitmap *const *per_key, size_t nkeys, size_t nslices, int op,
                                uint64_t start, uint64_t end, uint64_t vmin, uint64_t vmax, int threads);

#ifdef __cplusplus
}
#endif
#endif
