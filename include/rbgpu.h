/*
 * rbgpu.h — C ABI of the MI355X-native RoaringBitmap set-algebra engine (librbgpu.so).
 *
 * This is the drop-in boundary: plain pointers and sizes, no torch / HIP types.  A Java
 * host binds it through Panama FFM; the Python mirror
 * roaringbitmap_amd/ binds it through ctypes.  Each entry point names the reference
 * interface it replaces (paths relative to /root/reference/RoaringBitmap/src/main/java/
 * org/roaringbitmap/).
 *
 * Data model.  An rbgpu_set is a device-resident batch of bitmaps in SoA form (per container:
 * u16 key, u8 type 0=Array 1=Bitmap 2=Run, u32 cardinality, u16 run count, u64 payload
 * offset; per bitmap: a CSR begin index).  Container payloads are byte-identical to
 * RoaringFormatSpec container payloads (Array: sorted u16; Bitmap: 1024 LE u64; Run:
 * (start, length-1) u16 pairs — the u16 run count lives in the metadata), so serializing a
 * result is a copy.  Result sets have the same layout and can be fed back as inputs.
 *
 * Semantics.  Every result is bit-exact to the reference entry point it names: same values,
 * same container types, hence identical serialized bytes.  Inputs are borrowed read-only;
 * results are owned by the caller until rbgpu_set_free (the reference clones unmatched
 * containers — RoaringArray.java:184-205 — and so do we).
 *
 * Errors.  Every int-returning call returns RB_OK (0) or a negative status; the message is
 * available from rbgpu_last_error() (thread-local).  The reference's InvalidRoaringFormat /
 * IOException (RoaringArray.java:279-288, RoaringBitmap.java:1762-1811) maps to RB_EFORMAT;
 * IllegalArgumentException (RoaringArray.java:112-115, FastAggregation.java:53-55) maps to
 * RB_EINVAL.  Inputs must be canonical (sorted unique keys, Array card <= 4096, Bitmap card
 * equal to its popcount, Run lists sorted / non-overlapping / non-adjacent); the reference
 * does not check this on deserialize (RoaringArray.java:328-337) — we do and return RB_EINVAL.
 *
 * Threading.  One rbgpu_ctx per host thread (it owns a HIP stream and workspaces).  Calls are
 * synchronous, like the Java API (RoaringBitmap.java:367-369 thread-safety contract).
 */
#ifndef RBGPU_H
#define RBGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rbgpu_ctx rbgpu_ctx;
typedef struct rbgpu_set rbgpu_set;

enum rb_status {
  RB_OK = 0,
  RB_EFORMAT = -1, /* bad cookie / size > 65536 / truncated (InvalidRoaringFormat -> IOException) */
  RB_EINVAL = -2,  /* non-canonical input, bad index, bad argument (IllegalArgumentException) */
  RB_ENOMEM = -3,  /* device or host allocation failed */
  RB_EDEVICE = -4  /* HIP failure, or no MI355X visible */
};

enum rb_op { RB_AND = 0, RB_OR = 1, RB_XOR = 2, RB_ANDNOT = 3 };

enum rb_type { RB_ARRAY = 0, RB_BITMAP = 1, RB_RUN = 2 };

/* Wide-aggregation semantics: which reference entry point the result reproduces. */
enum rb_wide_sem {
  RB_FAST_OR = 0,      /* FastAggregation.or(RoaringBitmap...) == naive_or   FastAggregation.java:541-548,602 */
  RB_FAST_AND = 1,     /* FastAggregation.and(RoaringBitmap...)              FastAggregation.java:37-42      */
  RB_WORKSHY_AND = 2,  /* FastAggregation.workShyAnd                         FastAggregation.java:356-396    */
  RB_NAIVE_AND = 3,    /* FastAggregation.naive_and(RoaringBitmap...)        FastAggregation.java:328-346    */
  RB_FAST_XOR = 4,     /* FastAggregation.xor == naive_xor                   FastAggregation.java:576-582,772 */
  RB_PAR_OR = 5,       /* ParallelAggregation.or                             ParallelAggregation.java:161-175 */
  RB_PAR_XOR = 6,      /* ParallelAggregation.xor                            ParallelAggregation.java:182-195 */
  RB_NAIVE_AND_ITER = 7, /* FastAggregation.and(Iterator) == naive_and(Iterator) FastAggregation.java:26,304 */
  /* Global-order semantics: which containers meet, and in which order, follows a priority queue over
   * all the members (java.util.PriorityQueue ties included), so the order is computed on the host from
   * the members' keys and cardinalities and the per-key work runs on the device. */
  RB_HORIZONTAL_OR = 8,  /* FastAggregation.horizontal_or(List / varargs)     FastAggregation.java:124-231 */
  RB_HORIZONTAL_XOR = 9, /* FastAggregation.horizontal_xor                    FastAggregation.java:243-289 */
  RB_PQ_OR = 10,         /* FastAggregation.priorityqueue_or: the two smallest bitmaps (getLongSizeInBytes)
                            lazily OR'd on the device (lazyor / in-place lazyor / lazyorfromlazyinputs by
                            which operands are temporaries), re-queued, the survivor repaired
                            FastAggregation.java:675-721 (whole result only: no key range) */
  RB_PQ_XOR = 11,        /* FastAggregation.priorityqueue_xor: the two smallest bitmaps (getLongSizeInBytes)
                            replaced by their RoaringBitmap.xor, on the device, until one is left
                            FastAggregation.java:732-752 (whole result only: no key range) */
  /* buffer/ front end: BufferFastAggregation over ImmutableRoaringBitmap / MutableRoaringBitmap runs the
   * same container algebra; these are its entry points whose results differ from FastAggregation's
   * (paths under buffer/).  The others map onto the values above:
   *   and(ImmutableRoaringBitmap...), and(long[], Immutable...)     RB_FAST_AND   BufferFastAggregation.java:29-58
   *   and(Iterator), and(long[], Iterator), and(MutableRoaringBitmap...), workShyAnd,
   *   workAndMemoryShyAnd                                             RB_WORKSHY_AND          :67-108, 423-675
   *   naive_and(ImmutableRoaringBitmap...)                            RB_NAIVE_AND            :348-370
   *   naive_and(Iterator), naive_and(MutableRoaringBitmap...)         RB_NAIVE_AND_ITER       :384-418
   *   naive_or / or(Immutable... / Iterator), horizontal_or(Iterator) RB_FAST_OR             :675-692, 776-790, 246-249
   *   naive_xor / xor (every overload)                                RB_FAST_XOR             :728-768, 962-990
   *   horizontal_or / horizontal_xor(Immutable... / Mutable...)       RB_HORIZONTAL_OR / _XOR :188-244, 259-337
   * and BufferParallelAggregation (buffer/BufferParallelAggregation.java), whose per-key folds are
   * ParallelAggregation's (clone + lazyIOR below 16 containers, a lazy Bitmap from 16, clone + ixor
   * with no removal for xor, :194-230):
   *   BufferParallelAggregation.or(ImmutableRoaringBitmap...)         RB_PAR_OR               :166-180
   *   BufferParallelAggregation.xor(ImmutableRoaringBitmap...)        RB_PAR_XOR              :187-192
   */
  RB_BUFFER_NAIVE_OR = 12,   /* naive_or / or(MutableRoaringBitmap...): answer.lazyor(b) per bitmap, then
                                repairAfterLazy — per key the lazyIOR chain from a clone of the first
                                container, for any count (ParallelAggregation.or switches at 16)  :711-717, 797-799 */
  RB_BUFFER_PQ_OR = 13,      /* priorityqueue_or(ImmutableRoaringBitmap...): the lazy merges of RB_PQ_OR ordered
                                by serializedSizeInBytes; one bitmap comes back as a copy (no repair)  :810-866 */
  RB_BUFFER_PQ_OR_ITER = 14, /* priorityqueue_or(Iterator): ordered by ImmutableRoaringBitmap.getLongSizeInBytes
                                (a lazy Bitmap counts 2 bytes: getCardinality() is -1); one bitmap: a copy  :869-930 */
  RB_BUFFER_PQ_XOR = 15      /* priorityqueue_xor: RB_PQ_XOR ordered by ImmutableRoaringBitmap.getLongSizeInBytes;
                                fewer than 2 bitmaps -> RB_EINVAL (IllegalArgumentException)  :933-958 */
};

/* Host-side SoA description of a batch of bitmaps (used for upload and download). */
typedef struct rb_soa {
  uint32_t n_bitmaps;
  uint64_t n_containers;
  uint64_t payload_bytes;
  uint64_t *begin;   /* [n_bitmaps + 1] CSR: containers of bitmap i are [begin[i], begin[i+1]) */
  uint16_t *key;     /* [n_containers] high 16 bits, strictly increasing within a bitmap */
  uint8_t *type;     /* [n_containers] rb_type */
  uint32_t *card;    /* [n_containers] cardinality, 1..65536 */
  uint16_t *nruns;   /* [n_containers] run count (Run containers), else 0 */
  uint64_t *offset;  /* [n_containers] byte offset of the payload in `payload` */
  uint8_t *payload;  /* [payload_bytes] */
} rb_soa;

/* Per-call accounting of the last operation on a context (for the roofline report). */
typedef struct rb_stats {
  uint64_t tasks;            /* container-level work items launched */
  uint64_t input_bytes;      /* algorithmic input bytes (payload + 16 B metadata per container read, + 2 B per key) */
  uint64_t output_bytes;     /* algorithmic output bytes (payload + 16 B metadata per result container) */
  uint64_t result_containers;
  double main_kernel_ms;     /* duration of the dominant kernel (HIP events on the ctx stream) */
  uint64_t main_kernel_bytes; /* algorithmic bytes (in + out) of the work that kernel did */
  double total_ms;           /* whole call, device time between first and last launch */
  char main_kernel[64];      /* name of the dominant kernel */
  uint32_t n_kernels;        /* per-kernel breakdown of the compute phase */
  char kernel_name[4][48];
  double kernel_ms[4];
  uint64_t kernel_bytes[4];
  uint64_t kernel_items[4];
  uint64_t result_cardinality; /* Σ cardinality of every result bitmap of the call */
  double call_us;              /* host wall time of the call, entry to return (pairwise calls) */
} rb_stats;

/* ---- context ---------------------------------------------------------------------- */
int rbgpu_device_count(void);
/* A context: one stream pair, an allocation cache and the library's kernels loaded on the device (every
 * source file's code object is loaded here, ~1 ms each, so no later call pays a first-launch load).
 * Open one per device and keep it for the process. */
int rbgpu_open(int device, rbgpu_ctx **out);
void rbgpu_close(rbgpu_ctx *ctx);
const char *rbgpu_last_error(void);
int rbgpu_synchronize(rbgpu_ctx *ctx);
int rbgpu_get_stats(rbgpu_ctx *ctx, rb_stats *out);

/* ---- sets (RoaringBitmap / RoaringArray storage) ----------------------------------- */
/* RoaringBitmap.deserialize(ByteBuffer) for n bitmaps — RoaringArray.java:547-629 */
int rbgpu_set_from_serialized(rbgpu_ctx *ctx, const uint8_t *const *bufs, const uint64_t *lens,
                              uint32_t n, rbgpu_set **out);
/* The same for serialized bytes already in device memory (e.g. read from storage straight into HBM):
 * bitmap i is d_bytes[offsets[i], offsets[i+1]) with offsets[n+1] on the host; d_bytes must be
 * readable up to offsets[n] rounded up to 4.  Parsed and validated on the GPU (codec.hip) with the
 * same results and error codes as rbgpu_set_from_serialized. */
int rbgpu_set_from_serialized_device(rbgpu_ctx *ctx, const uint8_t *d_bytes, const uint64_t *offsets,
                                     uint32_t n, rbgpu_set **out);
/* Upload a host SoA batch (validated like deserialize). */
int rbgpu_set_from_soa(rbgpu_ctx *ctx, const rb_soa *soa, rbgpu_set **out);
void rbgpu_set_free(rbgpu_set *set);
uint32_t rbgpu_set_bitmap_count(const rbgpu_set *set);
uint64_t rbgpu_set_container_count(const rbgpu_set *set);
/* Bytes of the set's payload arena in HBM (every container payload padded to 16 B; a result set's arena also
 * holds its slots' padding).  What a kernel reading every payload once must fetch at least — the bench's
 * provable-minimum traffic for the config-4 lines (no Java counterpart: RoaringBitmap.getSizeInBytes counts
 * the serialized sizes, rbgpu_set_summaries). */
uint64_t rbgpu_set_payload_capacity(const rbgpu_set *set);
/* RoaringBitmap.getCardinality per bitmap (computed on device). */
int rbgpu_set_cardinalities(const rbgpu_set *set, uint64_t *out /* [n_bitmaps] */);
/* RoaringBitmap.serializedSizeInBytes per bitmap — RoaringArray.java:947-953 */
int rbgpu_set_serialized_sizes(const rbgpu_set *set, uint64_t *out /* [n_bitmaps] */);
/* RoaringBitmap.serialize(ByteBuffer) of bitmaps [first, first+count) back to back into dst;
 * offsets[count+1] receives each bitmap's start — RoaringArray.java:851-940 */
int rbgpu_set_serialize(const rbgpu_set *set, uint32_t first, uint32_t count, uint8_t *dst,
                        uint64_t cap, uint64_t *offsets);
/* rbgpu_set_serialize into device memory d_dst (cap bytes); offsets[count+1] on the host. */
int rbgpu_set_serialize_device(const rbgpu_set *set, uint32_t first, uint32_t count, uint8_t *d_dst,
                               uint64_t cap, uint64_t *offsets);
/* Per-bitmap summary: what a RoaringFormatSpec header over a sharded result needs
 * (RoaringBitmap.getCardinality, RoaringArray.size / hasRunContainer / serializedSizeInBytes,
 * RoaringArray.java:851-953). */
typedef struct rb_bitmap_summary {
  uint64_t cardinality;
  uint64_t n_containers;
  uint64_t n_run_containers;
  uint64_t payload_bytes; /* serialized container payloads (Run: 2 + 4 * nruns), no header */
  uint64_t size_in_bytes; /* RoaringBitmap.getLongSizeInBytes (RoaringBitmap.java:2212-2219) */
} rb_bitmap_summary;
int rbgpu_set_summaries(const rbgpu_set *set, uint32_t first, uint32_t count, rb_bitmap_summary *out);
/* Container mix of the whole set, what insights/BitmapAnalyser reports (insights/BitmapAnalyser.java:
 * 1-50): out[0..2] = Array / Bitmap / Run container counts, out[3..5] = their serialized payload bytes. */
int rbgpu_set_type_stats(const rbgpu_set *set, uint64_t *out /* [6] */);
/* Algorithmic bytes (payload + 16 B metadata) per high key over every container of the set:
 * out[65536].  Feeds the byte-balanced key-range partition of a sharded wide aggregation. */
int rbgpu_set_key_bytes(const rbgpu_set *set, uint64_t *out);
/* Containers of each member (members NULL = bitmaps 0..n-1) with high key in [key_lo, key_hi) ->
 * out[n].  Summed over the ranks of a key-range partition it is each bitmap's
 * highLowContainer.size(), the order FastAggregation.naive_and(varargs) starts from
 * (FastAggregation.java:328-346): rbgpu_wide_sharded and ShardedWide use it so every shard starts
 * from the globally smallest member. */
int rbgpu_set_range_counts(const rbgpu_set *set, const uint32_t *members, uint32_t n, uint32_t key_lo,
                           uint32_t key_hi, uint64_t *out);
/* Download bitmaps [first, first+count) as host SoA.  Call once with soa->key == NULL to get
 * n_containers / payload_bytes, allocate, call again to fill. */
int rbgpu_set_download(const rbgpu_set *set, uint32_t first, uint32_t count, rb_soa *soa);

/* ---- pairwise set algebra (static RoaringBitmap ops) ------------------------------- */
/* An a_idx / b_idx entry equal to RB_EMPTY_BITMAP stands for an empty bitmap (no containers): op with
 * it clones the other side's containers (or, xor, andNot with an empty right side) or gives nothing. */
#define RB_EMPTY_BITMAP 0xFFFFFFFFu
/* result[i] = op(a[a_idx[i]], b[b_idx[i]]); a_idx / b_idx may be NULL (identity).
 * RoaringBitmap.and/or/xor/andNot — RoaringBitmap.java:377-401, 860-902, 1071-1118, 444-473 */
int rbgpu_pairwise(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b,
                   const uint32_t *a_idx, const uint32_t *b_idx, uint32_t npairs, rbgpu_set **out);
/* In-place x1.op(x2): result[i] = a[a_idx[i]] after a[a_idx[i]].and/or/xor/andNot(b[b_idx[i]]) —
 * RoaringBitmap.and(x2) :1270-1296, or(x2) :2481-2523, xor(x2) :3296-3348, andNot(x2) :1346-1382.
 * The container algebra is the static one (Container.iand / iandNot / ixor return the static ops' types)
 * except x1.or(x2)'s BitmapContainer.ior(ArrayContainer), which keeps a Bitmap even when it fills up
 * (BitmapContainer.java:749-766; the static or() gives a full Run).  A pair whose operands are the
 * same bitmap object (a == b and a_idx[i] == b_idx[i]) follows the `x2 == this` branches: and / or
 * leave x1 as it is, xor / andNot clear it.  Inputs stay unchanged (results are new sets). */
/* Asynchronous rbgpu_pairwise (SURVEY §8b threading row: "an _async variant takes a stream").  The
 * call returns once its task kernels and compaction are enqueued; `stream` (a hipStream_t, NULL: the
 * context's own) is ordered around the call: the caller's earlier work on it runs first, its later work
 * runs after the result is complete.  *out is usable at once by later library calls on this context (they
 * are stream-ordered behind it; a call that needs the result's metadata on the host waits for it), and by
 * the host after rbgpu_set_wait.  The host thread can so prepare and enqueue the next batch while this one
 * runs on the device.  Batches of <= 4096 pairs (the small-batch path) and more than 256 pending results
 * per context complete before the return.  rb_stats is not updated by an asynchronous call. */
int rbgpu_pairwise_async(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b,
                         const uint32_t *a_idx, const uint32_t *b_idx, uint32_t npairs, void *stream,
                         rbgpu_set **out);
/* Wait until an asynchronous result is complete, and until the kernel of a call that returned on its last
 * block's sequence word (small batches, BSI RANGE: the host had the result before the kernel's end was
 * signalled) has ended (a no-op for any other set). */
int rbgpu_set_wait(const rbgpu_set *set);
/* Device addresses of a set's SoA in HBM (the layout of rb_soa), for a caller's own device work on results
 * where they are — the hand-off of a Java caller's MemorySegment over device memory.  Valid while the set
 * lives; the call never blocks.  Device work may read them once it is ordered after the call that produced
 * the set: on the `stream` given to rbgpu_pairwise_async (its later work runs after the result is complete,
 * small batches included), or after rbgpu_set_wait.  n_containers of a pending asynchronous result is
 * RB_UNKNOWN_COUNT until it is settled; the device's begin[n_bitmaps] holds it once the call is complete. */
#define RB_UNKNOWN_COUNT 0xFFFFFFFFFFFFFFFFull
typedef struct rb_device_view {
  uint32_t n_bitmaps;
  uint64_t n_containers;
  uint64_t payload_bytes; /* capacity of the payload arena */
  const uint64_t *begin;
  const uint16_t *key;
  const uint8_t *type;
  const uint32_t *card;
  const uint16_t *nruns;
  const uint64_t *offset;
  const uint8_t *payload;
} rb_device_view;
int rbgpu_set_device_view(const rbgpu_set *set, rb_device_view *out);
int rbgpu_pairwise_inplace(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b,
                           const uint32_t *a_idx, const uint32_t *b_idx, uint32_t npairs, rbgpu_set **out);
/* RoaringBitmap.andCardinality/orCardinality/xorCardinality/andNotCardinality
 * — RoaringBitmap.java:413-434, 916-920, 931-933, 944-985 */
int rbgpu_pairwise_cardinality(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b,
                               const uint32_t *a_idx, const uint32_t *b_idx, uint32_t npairs,
                               uint64_t *out /* [npairs] */);

/* ---- wide aggregation over members[0..n) of `in` (NULL = all bitmaps, in order) ------
 * A repeated member index is the same bitmap object (naive_and skips its smallest member by identity,
 * FastAggregation.java:337-341).  The long[] aggregation-buffer overloads (FastAggregation.and(long[],
 * RoaringBitmap...) :51-63, workAndMemoryShyAnd :477-514) take no buffer here: the caller checks the
 * reference's "buffer should have at least 1024 elements" IllegalArgumentException (more than 10
 * bitmaps for and(long[], ...), always for workAndMemoryShyAnd) and zero-fills it; the results are
 * RB_FAST_AND / RB_WORKSHY_AND.  priorityqueue_or(Iterator) (:615-664) is RB_PQ_OR. */
int rbgpu_wide(rbgpu_ctx *ctx, int sem, const rbgpu_set *in, const uint32_t *members, uint32_t n,
               rbgpu_set **out);
/* The same aggregation restricted to high keys in [key_lo, key_hi): one key-range shard of it.
 * Every key is independent and keeps its member order, so the shards of a partition of
 * [0, 65536), concatenated in key order, are exactly rbgpu_wide's result.  For
 * RB_NAIVE_AND the smallest member is chosen within the shard's containers; a sharded caller
 * passes the globally ordered member list with RB_NAIVE_AND_ITER instead (rbgpu_wide_sharded and
 * ShardedWide.aggregate do, from the all-reduced rbgpu_set_range_counts). */
int rbgpu_wide_keys(rbgpu_ctx *ctx, int sem, const rbgpu_set *in, const uint32_t *members, uint32_t n,
                    uint32_t key_lo, uint32_t key_hi, rbgpu_set **out);
/* FastAggregation.andCardinality / orCardinality — FastAggregation.java:71-101 */
int rbgpu_wide_cardinality(rbgpu_ctx *ctx, int op, const rbgpu_set *in, const uint32_t *members,
                           uint32_t n, uint64_t *out);

/* ---- bit-sliced index (bsi module) ------------------------------------------------------ */
/* BitmapSliceIndex.Operation ordinals (bsi/.../BitmapSliceIndex.java:9-25) */
enum rb_bsi_op { RB_BSI_EQ = 0, RB_BSI_NEQ = 1, RB_BSI_LE = 2, RB_BSI_LT = 3, RB_BSI_GE = 4, RB_BSI_GT = 5,
                 RB_BSI_RANGE = 6 };
/* Roaring64BitmapSliceIndex.compare(operation, startOrValue, end, foundSet) /
 * RoaringBitmapSliceIndex.compare (bsi/.../longlong/Roaring64BitmapSliceIndex.java:460-503,
 * bsi/.../RoaringBitmapSliceIndex.java:475-503): `bsi` holds the bitCount slices bA[0..n) followed
 * by the existence bitmap ebM (n + 1 bitmaps); min_value / max_value are the BSI's fields (they
 * drive compareUsingMinMax); `found` is a one-bitmap set or NULL (= ebM).  Values and predicates are
 * unsigned 64-bit (the reference's signed longs agree for values < 2^63).  The result is a
 * one-bitmap set, byte-identical to the reference's Roaring(64)Bitmap containers. */
int rbgpu_bsi_compare(rbgpu_ctx *ctx, const rbgpu_set *bsi, int op, uint64_t start_or_value, uint64_t end,
                      uint64_t min_value, uint64_t max_value, const rbgpu_set *found, rbgpu_set **out);
/* The high keys [key_lo, key_hi) of rbgpu_bsi_compare's answer: a rank that owns that key range of
 * the index (rbgpu_generate_bsi_keys, or any bsi set whose other keys it ignores) computes exactly
 * those containers of the result.  The compare is key-local (each 2^16-row chunk is independent),
 * so the disjoint shards of a partition concatenate, in key order, to the whole answer
 * (key-range sharding, no data-path collective). */
int rbgpu_bsi_compare_keys(rbgpu_ctx *ctx, const rbgpu_set *bsi, int op, uint64_t start_or_value, uint64_t end,
                           uint64_t min_value, uint64_t max_value, const rbgpu_set *found, uint32_t key_lo,
                           uint32_t key_hi, rbgpu_set **out);
/* RoaringBitmap.runOptimize (RoaringBitmap.java:2764-2775) of every bitmap of `in` into a new set:
 * each Array / Bitmap container becomes a Run when that is strictly smaller, each Run goes through
 * toEfficientContainer (ArrayContainer.java:1085-1099, BitmapContainer.java:1227-1246,
 * RunContainer.java:2326-2335).  any_run[n_bitmaps] (may be NULL) receives runOptimize's return value
 * per bitmap (1 when the bitmap holds a Run container afterwards). */
int rbgpu_set_run_optimize(const rbgpu_set *in, rbgpu_set **out, uint8_t *any_run);
/* RoaringBitmap.clone of bitmaps [first, first+count) into a new set (device copy). */
int rbgpu_set_extract(const rbgpu_set *set, uint32_t first, uint32_t count, rbgpu_set **out);
/* The per-set metadata the wide kernels derive on a set's first use and keep with it (sets are
 * immutable: a cached index, never a cached result): the dense-layout check, packed 8-B container
 * records and, for naive_xor, their key-major transpose.  *ms = device time spent building them so far,
 * *bytes = their algorithmic bytes (metadata read + records written).  A caller that uploads a fresh
 * set per aggregation pays this once per set on top of the call. */
int rbgpu_set_setup_stats(const rbgpu_set *set, double *ms, uint64_t *bytes);
/* The same split by derived item: ms[0] / bytes[0] the dense-layout check, [1] the packed member-major
 * records (workShyAnd's fast path), [2] the key-major records (naive_xor's; built from [1] when the set
 * has it, else straight from the set's metadata), [3] a BitSliceIndex set's key -> container tables and
 * ebM key list (rbgpu_bsi_compare).  What a fresh set costs a path: the items it uses. */
int rbgpu_set_setup_parts(const rbgpu_set *set, double ms[4], uint64_t bytes[4]);

/* ---- synthetic inputs for the benchmark (device-side generator, SplitMix64) ---------- */
enum rb_workload {
  RB_WL_FILTER_POSTING = 0, /* a = filters (4 keys, A/B/R .4/.3/.3),
                               b = posting lists (keys w.p. .5, A/B/R .7/.1/.2), n pairs */
  RB_WL_WIDE_DENSE = 1,     /* config 3: n bitmaps over 65536 keys, key w.p. 1/16, all Bitmap */
  RB_WL_WIDE_MIXED = 2,     /* config 3b: as 1 with 70% B / 20% A / 10% R */
  RB_WL_WIDE_RUNS = 3       /* config 4: n bitmaps x 65536 keys of run-heavy containers */
};
/* Only the containers with high keys in [key_lo, key_hi) of a wide workload (1..3): the shard a
 * rank owns.  Container contents are keyed by (bitmap, key), so the shards of a partition are
 * exactly the full dataset's containers. */
int rbgpu_generate_keys(rbgpu_ctx *ctx, int workload, uint32_t n, uint64_t seed, uint32_t key_lo, uint32_t key_hi,
                        rbgpu_set **a);
/* a runOptimize'd BSI over rows [0, nrows) with nslices random value bits per
 * row (every slice container Bernoulli(1/2)), i.e. nslices + 1 bitmaps (slices, then ebM). */
int rbgpu_generate_bsi(rbgpu_ctx *ctx, uint32_t nslices, uint64_t nrows, uint64_t seed, rbgpu_set **out);
/* The containers of rbgpu_generate_bsi's index with high keys in [key_lo, key_hi) (a rank's shard). */
int rbgpu_generate_bsi_keys(rbgpu_ctx *ctx, uint32_t nslices, uint64_t nrows, uint64_t seed, uint32_t key_lo,
                            uint32_t key_hi, rbgpu_set **out);
/* Generates a (and b for RB_WL_FILTER_POSTING; *b may be NULL otherwise).  n = pairs or
 * bitmaps.  Every container goes through runOptimize semantics, as
 * RoaringBitmapWriter(runCompress=true) does (ContainerAppender.java:130-137). */
int rbgpu_generate(rbgpu_ctx *ctx, int workload, uint32_t n, uint64_t seed, rbgpu_set **a,
                   rbgpu_set **b);

/* ---- 64-bit bitmaps (longlong/): Roaring64NavigableMap and Roaring64Bitmap ----------------------
 * A 64-bit bitmap is a list of buckets (high 32 bits, 32-bit RoaringBitmap of the low halves) in
 * ascending unsigned order: Roaring64NavigableMap's highToBitmap (default unsigned comparator) and
 * Roaring64Bitmap's 48-bit ART keys grouped by their high 32 bits.  Bytes cross the boundary in the
 * RoaringFormatSpec 64-bit extension ("portable": u64 bucket count, then per bucket u32 high and the
 * 32-bit RoaringBitmap), Roaring64NavigableMap.serializePortable / deserializePortable
 * (longlong/Roaring64NavigableMap.java:1254-1261).  The bucket algebra is the 32-bit engine's: one
 * batched pairwise call per batch of 64-bit pairs. */
typedef struct rbgpu_set64 rbgpu_set64;
enum rb64_flavor {
  RB64_BITMAP = 0,   /* Roaring64Bitmap: static and/or/xor/andNot(x1, x2) (longlong/Roaring64Bitmap.java:345-390,
                        421-460, 497-517, 630-650) and in place x1.op(x2) (:319-343, 392-419, 468-495, 599-628):
                        per 48-bit key the container op (in place: iand / ior / ixor / iandNot), an empty and /
                        andNot result removed, an empty xor result KEPT (the reference stores it unchecked) */
  RB64_NAVIGABLE = 1 /* Roaring64NavigableMap in place x1.and/or/xor/andNot(x2) (longlong/Roaring64NavigableMap.java:
                        773-977): per bucket the 32-bit RoaringBitmap's in-place op; a bucket left empty stays */
};
/* n 64-bit bitmaps from portable bytes (RB_EFORMAT: truncated / bad bucket; RB_EINVAL: bucket highs
 * not strictly increasing — the reference's TreeMap would reorder them). */
int rbgpu_set64_from_portable(rbgpu_ctx *ctx, const uint8_t *const *bufs, const uint64_t *lens, uint32_t n,
                              rbgpu_set64 **out);
/* n 64-bit bitmaps from a 32-bit set of their buckets: bitmap i is buckets [begin[i], begin[i+1]) of
 * `buckets` with highs[begin[i]..] (begin[n] == bitmaps of `buckets`); the buckets are copied. */
int rbgpu_set64_from_buckets(const rbgpu_set *buckets, const uint32_t *highs, const uint64_t *begin, uint32_t n,
                             rbgpu_set64 **out);
void rbgpu_set64_free(rbgpu_set64 *set);
uint32_t rbgpu_set64_bitmap_count(const rbgpu_set64 *set);
/* bucket highs of bitmap i (up to cap of them into highs, may be NULL); *count = its bucket count */
int rbgpu_set64_buckets(const rbgpu_set64 *set, uint32_t i, uint32_t *highs, uint64_t cap, uint64_t *count);
/* The buckets of 64-bit bitmap i as a new 32-bit set, bitmap k = its k-th bucket (highs from
 * rbgpu_set64_buckets), containers bytes-identical — empty ones a Roaring64Bitmap keeps included: the
 * view toArray / select iterate (longlong/Roaring64Bitmap.java:106, 946; Roaring64NavigableMap.java:351,
 * 1409). */
int rbgpu_set64_bucket_set(const rbgpu_set64 *set, uint32_t i, rbgpu_set **out);
/* A copy of 64-bit bitmaps [first, first+count), buckets and all (Roaring64Bitmap.clone,
 * longlong/Roaring64Bitmap.java:1159; Roaring64NavigableMap's copy is per bucket, :744-803). */
int rbgpu_set64_extract(const rbgpu_set64 *set, uint32_t first, uint32_t count, rbgpu_set64 **out);
/* getLongCardinality per bitmap */
int rbgpu_set64_cardinalities(const rbgpu_set64 *set, uint64_t *out);
/* portable serialized size per bitmap, and the bytes of bitmaps [first, first+count) back to back */
int rbgpu_set64_portable_sizes(const rbgpu_set64 *set, uint64_t *out);
int rbgpu_set64_serialize_portable(const rbgpu_set64 *set, uint32_t first, uint32_t count, uint8_t *dst,
                                   uint64_t cap, uint64_t *offsets);
/* Roaring64NavigableMap's default ("legacy", SERIALIZATION_MODE_LEGACY) format, serializeLegacy /
 * deserializeLegacy (longlong/Roaring64NavigableMap.java:1229-1240, 1295-1325): a signedLongs byte, a
 * big-endian int bucket count, then per bucket a big-endian int high and the RoaringBitmap bytes, in
 * the map's order (signed ints when signedLongs).  The flag travels with the bitmap; in-place results
 * keep x1's.  Parity unpinned: the reference holds no legacy fixture. */
int rbgpu_set64_from_legacy(rbgpu_ctx *ctx, const uint8_t *const *bufs, const uint64_t *lens, uint32_t n,
                            rbgpu_set64 **out);
int rbgpu_set64_legacy_sizes(const rbgpu_set64 *set, uint64_t *out);
int rbgpu_set64_serialize_legacy(const rbgpu_set64 *set, uint32_t first, uint32_t count, uint8_t *dst,
                                 uint64_t cap, uint64_t *offsets);
/* Roaring64Bitmap.serialize / deserialize (longlong/Roaring64Bitmap.java:880-908 -> HighLowContainer
 * .serialize / deserialize, longlong/HighLowContainer.java:230-254): an empty tag, the ART over the 6-byte
 * high keys (art/Art.java:309-391, art/Node.java:326-400, Node4/16/48/256 and LeafNode bodies) and the
 * Containers arrays (art/Containers.java:210-303), little-endian.  Ingest reads any tree and null-slot
 * layout (a card-0 container — a kept-empty xor result — holds no value and is dropped); emit writes the
 * canonical stream of the containers inserted in ascending key order (path-compressed tree, smallest node
 * type per child count, container i at index i of one ArrayList-grown array).  Parity unpinned: the
 * reference holds no fixture of this format. */
int rbgpu_set64_from_art(rbgpu_ctx *ctx, const uint8_t *const *bufs, const uint64_t *lens, uint32_t n,
                         rbgpu_set64 **out);
int rbgpu_set64_art_sizes(const rbgpu_set64 *set, uint64_t *out);
int rbgpu_set64_serialize_art(const rbgpu_set64 *set, uint32_t first, uint32_t count, uint8_t *dst,
                              uint64_t cap, uint64_t *offsets);
/* new Roaring64NavigableMap(signedLongs) for bitmap i: the order its two serializations write the buckets */
int rbgpu_set64_set_signed_longs(rbgpu_set64 *set, uint32_t i, int signed_longs);
int rbgpu_set64_get_signed_longs(const rbgpu_set64 *set, uint32_t i, int *signed_longs);
/* out[i] = the cardinality of the static op's result, without materialising it:
 * Roaring64Bitmap.andCardinality(x1, x2) (longlong/Roaring64Bitmap.java:562-592) for RB_AND, and the
 * same bucket merge for or / xor / andNot (getLongCardinality of Roaring64Bitmap.or/xor/andNot). */
int rbgpu_pairwise64_cardinality(rbgpu_ctx *ctx, int op, const rbgpu_set64 *a, const rbgpu_set64 *b,
                                 const uint32_t *a_idx, const uint32_t *b_idx, uint32_t npairs, uint64_t *out);
/* result[i] = op(a[a_idx[i]], b[b_idx[i]]) with flavor's rules; inplace != 0: the state of a[a_idx[i]]
 * after a[a_idx[i]].op(b[b_idx[i]]) (same set and index on both sides: the `x2 == this` branches).
 * RB64_NAVIGABLE needs inplace (the class has no static and/or/xor/andNot). */
int rbgpu_pairwise64(rbgpu_ctx *ctx, int flavor, int op, int inplace, const rbgpu_set64 *a, const rbgpu_set64 *b,
                     const uint32_t *a_idx, const uint32_t *b_idx, uint32_t npairs, rbgpu_set64 **out);

/* ---- multi-GPU: one process (or host thread) per GPU, RCCL over xGMI ------------------------
 * The reference scales one JVM over a ForkJoin pool (ParallelAggregation.java:161-195, keys
 * grouped and reduced in parallel).  Here each GPU owns a high-key range of the data (the key
 * partition is exact: every key's result depends only on that key's containers) and the exchange
 * happens inside the library on the communicator: an all-gather of the shard summaries and, on
 * request, the gather of the shards' serialized bytes to one rank, assembled there on the device
 * into the RoaringFormatSpec bytes of the whole result (RoaringArray.serialize, RoaringArray.java:
 * 851-940).  RCCL is opened at rbgpu_comm_init (dlopen of librccl.so.1: the library itself has no
 * link-time dependency on it). */
typedef struct rbgpu_comm rbgpu_comm;
enum { RB_COMM_ID_BYTES = 128 };
/* A communicator id (ncclGetUniqueId): made on one rank and handed to the others by the caller
 * over any channel (the JVM's own transport, torch.distributed, an environment variable). */
int rbgpu_comm_unique_id(uint8_t id[RB_COMM_ID_BYTES]);
/* Joins the communicator of `nranks` ranks as `rank` on ctx's GPU (collective: every rank calls it). */
int rbgpu_comm_init(rbgpu_ctx *ctx, const uint8_t id[RB_COMM_ID_BYTES], int nranks, int rank, rbgpu_comm **out);
void rbgpu_comm_destroy(rbgpu_comm *comm);

/* A caller-provided host transport (the JVM's own channel, MPI, a torch.distributed group): the same
 * exchange as the RCCL communicator — summaries, failure agreement, naive_and's global order, the shard
 * gather and the header assembly — with the shard bytes moving through host memory.  Every callback is
 * collective in the usual sense (all ranks call it in the same order) except send / recv, which pair
 * rank -> root.  Return 0 on success.  The callbacks must outlive the communicator. */
typedef struct rb_host_transport {
  void *user;
  int nranks, rank;
  /* recv[r * bytes .. (r + 1) * bytes) = rank r's `bytes` bytes at send */
  int (*all_gather)(void *user, const void *send, void *recv, uint64_t bytes);
  /* element-wise sum of n u64 over the ranks, in place */
  int (*all_reduce_sum_u64)(void *user, uint64_t *values, uint32_t n);
  int (*send)(void *user, const void *buf, uint64_t bytes, int peer);
  int (*recv)(void *user, void *buf, uint64_t bytes, int peer);
} rb_host_transport;
/* A communicator over a host transport.  ctx may be NULL: then only the byte-level entry points below
 * (rbgpu_shard_summarize_serialized, rbgpu_shard_gather_host, rbgpu_comm_naive_and_order,
 * rbgpu_comm_allreduce_sum) apply; with a ctx every sharded entry point works, over host memory. */
int rbgpu_comm_init_host(rbgpu_ctx *ctx, const rb_host_transport *t, rbgpu_comm **out);

/* The whole result of a key-range-sharded aggregation, as every rank sees it after the exchange. */
typedef struct rb_shard_summary {
  uint64_t cardinality;       /* RoaringBitmap.getCardinality of the whole result */
  uint64_t n_containers;
  uint64_t n_run_containers;
  uint64_t payload_bytes;     /* container payload bytes of the whole result (Run counts included) */
  uint64_t serialized_size;   /* RoaringBitmap.serializedSizeInBytes of the whole result */
  uint64_t payload_offset;    /* where this rank's first container payload starts in those bytes */
  uint64_t container_offset;  /* this rank's first container index in the whole result */
  uint64_t local_serialized;  /* serializedSizeInBytes of this rank's shard alone */
} rb_shard_summary;
/* The exchange for a one-bitmap shard `local` (keys of every rank disjoint and increasing with rank):
 * an all-gather of (cardinality, containers, Run containers, payload bytes, shard bytes) over the
 * communicator.  Collective. */
int rbgpu_shard_summarize(rbgpu_comm *comm, const rbgpu_set *local, rb_shard_summary *out);
/* rbgpu_wide_keys over [key_lo, key_hi) on this rank's GPU + rbgpu_shard_summarize.  Collective.
 * RB_NAIVE_AND (and RB_FAST_AND over <= 10 members, which is naive_and) first all-reduces the
 * members' rbgpu_set_range_counts so every shard folds from the globally smallest bitmap, as the
 * unsharded call does.  RB_PQ_OR / RB_PQ_XOR are refused (their merge order follows whole-bitmap
 * sizes of intermediate results). */
int rbgpu_wide_sharded(rbgpu_comm *comm, int sem, const rbgpu_set *in, const uint32_t *members, uint32_t n,
                       uint32_t key_lo, uint32_t key_hi, rbgpu_set **local, rb_shard_summary *summary);
/* rbgpu_bsi_compare_keys over [key_lo, key_hi) + rbgpu_shard_summarize.  Collective. */
int rbgpu_bsi_compare_sharded(rbgpu_comm *comm, const rbgpu_set *bsi, int op, uint64_t start_or_value, uint64_t end,
                              uint64_t min_value, uint64_t max_value, const rbgpu_set *found, uint32_t key_lo,
                              uint32_t key_hi, rbgpu_set **local, rb_shard_summary *summary);
/* The serialized bytes of the whole result on rank `root`, written to device memory d_dst (cap >=
 * summary->serialized_size; ignored on the other ranks): every rank serializes its shard on its
 * GPU, the shards travel to `root` as one grouped RCCL send/recv, and one kernel there writes the
 * global header (cookie, Run-container bitmap, key / cardinality-1 pairs, offsets) around the
 * concatenated payloads.  Collective. */
int rbgpu_shard_gather_serialized(rbgpu_comm *comm, const rbgpu_set *local, const rb_shard_summary *summary,
                                  int root, uint8_t *d_dst, uint64_t cap);
/* rbgpu_shard_summarize for a shard given as its standalone serialized bytes (host memory).  Collective. */
int rbgpu_shard_summarize_serialized(rbgpu_comm *comm, const uint8_t *shard, uint64_t len, rb_shard_summary *out);
/* rbgpu_shard_gather_serialized for a shard given as host bytes (len == summary->local_serialized);
 * the root receives the whole result's bytes in host memory dst.  Collective. */
int rbgpu_shard_gather_host(rbgpu_comm *comm, const uint8_t *shard, uint64_t len, const rb_shard_summary *summary,
                            int root, uint8_t *dst, uint64_t cap);
/* naive_and's fold order over a key-range partition (FastAggregation.java:328-346): the members'
 * per-rank container counts (rbgpu_set_range_counts) are summed over the ranks; order[0] = the member
 * with the fewest containers (first on ties), then the others in order, that member's other occurrences
 * skipped by identity (*n_order <= n; RB_NAIVE_AND_ITER folds it).
 * local_failed != 0: this rank could not count; every rank then fails together.  Collective. */
int rbgpu_comm_naive_and_order(rbgpu_comm *comm, const uint32_t *members, const uint64_t *local_counts, uint32_t n,
                               int local_failed, uint32_t *order, uint32_t *n_order);
/* Sum of `n` u64 values over the ranks, in place (the pairwise batch's cardinality exchange:
 * each rank runs its own pairs, the sum of the results' cardinalities is a global fact).  Collective. */
int rbgpu_comm_allreduce_sum(rbgpu_comm *comm, uint64_t *values, uint32_t n);
/* The header assembly of rbgpu_shard_gather_serialized on host buffers (the same code the device
 * kernel runs): parts[r] = the standalone serialized bytes of rank r's shard (keys increasing with
 * r); writes the whole result's bytes to dst (cap bytes) and their length to *written. */
int rbgpu_shard_assemble_host(const uint8_t *const *parts, const uint64_t *part_lens, uint32_t nparts,
                              uint8_t *dst, uint64_t cap, uint64_t *written);

#ifdef __cplusplus
}
#endif
#endif
