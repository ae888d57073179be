// kernels.hpp — launch wrappers of the librbgpu device kernels (all on one HIP stream).
#pragma once
#include "common.hpp"

// workShyAnd's run fast path reads the set's SoA metadata directly instead of packed per-set records (mrec):
// no setup pass on a fresh set (wide_runs.hip AndRec)
#ifndef RBG_AND_SOA
#define RBG_AND_SOA 1 // study builds: 0 packs the set's records (mrec) on its first workShyAnd and reads those
#endif
namespace rbg {

// ---- scan.hip
uint64_t scan_tmp_words(uint64_t n);
uint64_t scan_multi_tmp_words(uint64_t n, int k);
void scan_exclusive(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *tmp, hipStream_t st);
// k scans of n words each (k <= 4); totals[i] = out[i][n].  One launch when n fits one block.
void scan_exclusive_multi(const uint64_t *const *in, uint64_t *const *out, int k, uint64_t n, uint64_t *tmp,
                          uint64_t *totals, hipStream_t st);
// the same for short arrays (per-block totals, n up to ~1M) in one launch; totals may be null
void launch_noop(hipStream_t st);
// one empty launch per source file: HIP loads a file's code object at the first launch of any of its kernels
void warm_bsi(hipStream_t st);
void warm_codec(hipStream_t st);
void warm_generate(hipStream_t st);
void warm_pairwise(hipStream_t st);
void warm_scan(hipStream_t st);
void warm_setops(hipStream_t st);
void warm_wide(hipStream_t st);
void warm_wide_runs(hipStream_t st);
void warm_wide_xor(hipStream_t st);
void scan_blocks_multi(const uint64_t *const *in, uint64_t *const *out, int k, uint64_t n, uint64_t *totals,
                       hipStream_t st);

// ---- pairwise.hip
constexpr uint32_t kMaxSegKeys = 2048; // merged keys per merge-path segment, at most
struct PairArgs {
  int op;
  SetView A, B;
  const uint32_t *aidx; // may be null (identity)
  const uint32_t *bidx; // may be null (identity)
  uint32_t npairs;
  const uint64_t *seg_begin; // [npairs + 1] first merge-path segment of each pair
  const uint32_t *seg_pair;  // [nseg] pair of each segment; null: one segment per pair (segment p = pair p)
  uint64_t nseg;
  uint32_t seg_keys; // merged keys per segment (a power of two in [8, 256]; <= kMaxSegKeys)
  // in-place x1.op(x2) (RoaringBitmap.and/or/xor/andNot(x2)): `same` = A and B are one set, so a pair
  // with equal indices is one bitmap with itself — x.and(x) / x.or(x) leave x as it is, x.xor(x) /
  // x.andNot(x) clear it (RoaringBitmap.java:1271, 1347-1350, 2482, 3297-3300)
  int inplace, same;
  uint64_t a_nc, b_nc; // containers in A / B (a short segment's clamped loads need one to exist)
};
// per task result metadata (workspace, indexed like tasks)
struct TaskMeta {
  uint8_t *type;   // result type (kEmpty when dropped), written by the task kernels
  uint64_t *res;   // the result's type | nruns << 8 | card word << 32 (task_res), task kernels
  uint64_t *slot;  // output slot offset | key << 40 | heavy << 56 (task_slot), k_pair_emit
  int lazy;        // 0, or the priorityqueue_or role (kLazyStatic / kLazyIor / kLazyIorBf) of an OR call
  int inplace;     // x1.or(x2) in place: BitmapContainer.ior(ArrayContainer) keeps a Bitmap even when full
  int keep_empty;  // XOR results are kept when empty (Roaring64Bitmap.xor: Roaring64Bitmap.java:392-460)
};
__host__ __device__ inline uint64_t task_res(uint32_t type, uint32_t nruns, uint32_t card) {
  return (uint64_t)(type & 0xFFu) | ((uint64_t)(nruns & 0xFFFFu) << 8) | ((uint64_t)card << 32);
}
__host__ __device__ inline uint64_t task_slot(uint64_t out, uint32_t key, bool heavy) {
  return out | ((uint64_t)(key & 0xFFFFu) << 40) | ((uint64_t)heavy << 56);
}
constexpr uint64_t kSlotOffsetLimit = 1ull << 40; // result arena offsets a task_slot holds
struct PairCounts {
  uint64_t task, light, heavy, big, small;
};
struct PairBases {
  uint64_t task, light, heavy, big, small;
};
// per pair arrays (counts, or their exclusive scans), each [npairs + 1]; heavy = task - light
struct PairCountArrays {
  uint64_t *task, *light, *big, *small;
};
// stats words (striped, see common.hpp): 0/1 total input/output bytes, 2/3 filter+copy / register-path
// input, 4/5 filter+copy / register-path output
// merge-path segments of every pair (<= 256 merged keys each): counts, then the segment -> pair map
void launch_seg_count(const PairArgs &a, uint64_t *nseg, hipStream_t st);
void launch_seg_fill(const PairArgs &a, const uint64_t *seg_begin, uint32_t *seg_pair, hipStream_t st);
void launch_max_span(const uint64_t *begin, uint32_t nb, uint64_t *out, hipStream_t st);
void launch_max_runs(const uint8_t *type, const uint16_t *nruns, uint64_t n, uint64_t *out, hipStream_t st);
// result CSR per pair (rbegin may be null) and the result container count into *count (may be null)
void launch_pair_rbegin(const uint64_t *seg_begin, uint32_t npairs, const uint64_t *rseg, uint64_t *rbegin,
                        uint64_t *count, hipStream_t st);
// per segment from here on
// per-block layout (segments in blocks of pair_blocks' size): c = each segment's counts (one packed
// word), bt = each
// block's totals; the emit reads the counts and the exclusive scans of the block totals (bs)
uint64_t pair_blocks(uint64_t nseg);
void launch_pair_count(const PairArgs &a, uint64_t *c, const PairCountArrays &bt, uint64_t *stats,
                       hipStream_t st);
// tot non-null: heavy and small_base come from the device totals (heavy = light + tot[1]) and the
// workspace holds cap tasks (nothing is written when tot[0] exceeds it)
// task_begin[p] = segment p's first task ([nseg] = the total), for the compaction; zero_q (may be
// null): the task kernels' queue counters, zeroed before any record is written
void launch_pair_emit(const PairArgs &a, const uint64_t *cnt, const PairCountArrays &bs, uint64_t small_base,
                      TaskRec *light, TaskRec *heavy, const TaskMeta &tm, uint64_t *task_begin, const uint64_t *tot,
                      uint64_t cap, unsigned long long *zero_q, hipStream_t st);
// the task kernels' chunk-queue counters (words; zeroed by the emit when zero_q is given)
constexpr int kQueueWords = 512;
// light records: copies + subset-of-an-Array filters; heavy records: the register path.  `mid` is
// recorded between the two persistent launches.
void launch_pairwise(int op, bool card_only, const uint8_t *pa, const uint8_t *pb, const TaskRec *light,
                     uint64_t nl, const TaskRec *heavy, uint64_t nh, uint8_t *out, const TaskMeta &tm,
                     hipStream_t st, hipEvent_t mid);
// the same two kernels launched concurrently: heavy on `side` (1 block per CU, between ev_h0 / ev_h1),
// light on `st` (2 blocks per CU, `light_done` recorded after it)
void launch_pairwise_concurrent(int op, bool card_only, const uint8_t *pa, const uint8_t *pb, const TaskRec *light,
                                uint64_t nl, const TaskRec *heavy, uint64_t nh, uint8_t *out, const TaskMeta &tm,
                                hipStream_t st, hipStream_t side, hipEvent_t light_done, hipEvent_t ev_h0,
                                hipEvent_t ev_h1, unsigned long long *queue);
// measurement probes (rbgpu_internal_probe): mode 1 = task-order payload reads, 2 = streaming read
void launch_probe(int op, int mode, const uint8_t *pa, const uint8_t *pb, uint64_t a_bytes, const TaskRec *recs,
                  uint64_t n, uint32_t *sink, unsigned blocks, hipStream_t st);
// bk[block] = the block's kept results; the write takes their exclusive scans (bks) and writes each
// segment's first result index to rseg and / or rbegin (either may be null)
void launch_compact_count(const uint64_t *task_begin, uint64_t nseg, const uint8_t *ttype, uint64_t *bk,
                          hipStream_t st);
// The compaction's one-launch tail (round 6, VERDICT r05 #2a): the last block to finish sums the call's
// striped counters, zeroes them for the next call and writes the sums and then `seq` (system-scope release)
// to host-visible words, so the host returns on them instead of a counters copy, a memset and a stream wait.
struct CallTail {
  uint64_t *ctr;   // finished-block count (reset by the last block)
  uint64_t *hout;  // host-visible words: [0, kStatWords) the summed counters, [kStatWords] = seq; null: no tail
  uint64_t seq;
};
constexpr int kTailWord = 16; // the general pipeline's words in the context's host-visible block (after the small path's)
void launch_compact_write(const uint64_t *task_begin, uint64_t nseg, const TaskMeta &tm, const uint64_t *bks,
                          const OutView &out, const uint32_t *seg_pair, uint64_t *pair_card, uint64_t *stats,
                          uint64_t *rseg, uint64_t *rbegin, hipStream_t st, const CallTail &tail = CallTail{});

// small batches (<= kSmallPairs pairs, <= kSmallPairKeys keys per pair, <= kSmallSlots merged keys in
// all): ONE kernel per call computes every pair into one 8 KiB slot per merged key, and its last block to
// finish compacts the slots into the result CSR (pairwise.hip, k_pair_small)
constexpr uint32_t kSmallPairs = 4096, kSmallPairKeys = 4096, kSmallSlots = 32768;
// The call's tables, per pair: first container of its A and B bitmaps (i0, j0) and their container counts
// (na | nb << 16; the host has the CSR), first slot (prefix of na + nb, np + 1 entries), first block
// (np + 1), and the x1.op(x1) in-place flag.  Up to kSmallInline pairs they travel in the kernel arguments
// (no copy, no host-memory reads); larger batches copy them to device memory first.
constexpr uint32_t kSmallInline = 200;
struct SmallTabInline {
  uint32_t ident[(kSmallInline + 31) / 32];
  uint32_t i0[kSmallInline], j0[kSmallInline], nab[kSmallInline], slot[kSmallInline + 1];
  uint16_t blk[kSmallInline + 1];
  __device__ uint32_t a0(uint32_t p) const { return i0[p]; }
  __device__ uint32_t b0(uint32_t p) const { return j0[p]; }
  __device__ uint32_t counts(uint32_t p) const { return nab[p]; }
  __device__ bool same(uint32_t p) const { return (ident[p >> 5] >> (p & 31)) & 1u; }
  __device__ uint32_t slot_at(uint32_t p) const { return slot[p]; }
  __device__ uint32_t blk_at(uint32_t p) const { return blk[p]; }
};
struct SmallTabDev {
  const uint32_t *ident, *i0, *j0, *nab, *slot, *blk;
  __device__ uint32_t a0(uint32_t p) const { return i0[p]; }
  __device__ uint32_t b0(uint32_t p) const { return j0[p]; }
  __device__ uint32_t counts(uint32_t p) const { return nab[p]; }
  __device__ bool same(uint32_t p) const { return (ident[p >> 5] >> (p & 31)) & 1u; }
  __device__ uint32_t slot_at(uint32_t p) const { return slot[p]; }
  __device__ uint32_t blk_at(uint32_t p) const { return blk[p]; }
};
struct SmallPairArgs {
  SetView A, B;
  uint32_t np;
  uint8_t *arena;              // slot t's payload at t * 8 KiB (null for cardinality only)
  uint64_t *smeta;             // [2][kSmallSlots] per slot: key, type, card word, run count (small_meta), then
                               // input bytes | card << 32 — sc1 stores the compaction polls for (kSlotUnset
                               // between calls: the context's buffer, reset by the compaction)
  uint64_t *pcard;             // [np] result cardinality per pair, or null
  uint64_t *ctr;               // [0] started blocks (agent atomic; zero between calls: the last block resets it)
  int lazy;                    // 0, or the priorityqueue_or role of an OR call (TaskMeta::lazy)
  int inplace;                 // in-place x1.op(x2) (PairArgs::inplace)
  int keep_empty;              // TaskMeta::keep_empty
  // the compaction's: E slots, nblocks blocks, slot -> result position scratch (used above
  // kSmallXposLds slots), result SoA (key null: cardinality only), result CSR or null, host-visible
  // words: [0] result containers, [1..4] the summed counters
  uint32_t E, nblocks;
  uint32_t *xpos;
  uint64_t *rbegin, *hout; // hout: host-visible result words [0..4], and [5] = seq once they are written
  uint64_t seq;
  OutView out;
};
// blocks of one pair of nk = na + nb keys: up to kpw merged keys per wave, 4 waves per block, at most `cap`
// (a floor of one wave per key of the larger side — a matched key takes the costly register path — measured
// slower on census: 769 blocks, two rounds)
__host__ __device__ inline uint32_t small_pair_nsub(uint64_t nk, uint32_t cap, uint32_t kpw) {
  const uint64_t b = (nk + 4ull * kpw - 1) / (4ull * kpw);
  return (uint32_t)(b < 1 ? 1 : b > cap ? cap : b);
}
static_assert(sizeof(SmallTabInline) + sizeof(SmallPairArgs) + 16 <= 4096, "kernel arguments within 4 KiB");
// blocks of 256 threads resident at once (2 per CU: the register path takes up to 256 VGPRs)
unsigned small_resident_blocks();
void launch_pair_small(int op, bool card_only, const SmallPairArgs &a, const SmallTabInline *inl,
                       const SmallTabDev &dev, uint32_t max_keys, uint32_t nblocks, hipStream_t st);

// ---- wide.hip: per-key reduction outputs (one 8 KiB slot per active key q)
struct WideOut {
  uint8_t *type;   // per active key, kEmpty if dropped
  uint32_t *card;
  uint16_t *nruns;
};

// ---- wide_runs.hip: Run-list fast path for naive_or / workShyAnd / naive_xor keys whose containers
// are all Runs with <= 8 runs; route[q] = 0 where done, 1 where the generic kernel must run
// The container ids of the grouped keys.  Grouped by the counting sort: cid[i] for position i of key k's
// segment [seg[k], seg[k+1]).  Dense members (every member holds every key of [dense_lo, dense_hi) —
// the config-4 shape): no grouping at all, seg[k] = (k - key_lo) * M and the container of member j at
// key k is mbase[j] + k, with mbase[j] = begin[mem[j]] - dense_lo (mod 2^64).
struct CidMap {
  const uint32_t *cid;   // null: dense
  const uint64_t *mbase; // [M] (dense)
};
// one key's view of a CidMap: operator[] takes the grouped position i of a container of that key
struct KeyCids {
  const uint32_t *cid;
  const uint64_t *mbase;
  uint64_t lo;  // seg[key]
  uint32_t key;
  __device__ __forceinline__ KeyCids(const CidMap &m, uint64_t lo_, uint32_t key_)
      : cid(m.cid), mbase(m.mbase), lo(lo_), key(key_) {}
  __device__ __forceinline__ uint32_t operator[](uint64_t i) const {
    return cid ? cid[i] : (uint32_t)(mbase[i - lo] + key);
  }
};
// naive_xor's key-major member records (wide_xor.hip): `rec` holds one 4-B record (pack_xrec) per
// grouped container, in grouped order.  kCached: `rec` is the set's krec (dense set, members in set
// order: nothing to build); kTranspose: dense members in another order, transposed per call from the
// set's mrec through mbase; kGather: grouped by the counting sort, gathered through the ids.
struct XorRecords {
  enum Build { kCached = 0, kTranspose = 1, kGather = 2 };
  uint32_t *rec;
  uint64_t n;
  Build build;
  const uint64_t *mrec, *mbase;
  uint32_t M, key_lo, key_hi;
};
// member m's container at key k is mbase[m] - bias + k (a dense set: mbase = the set's begin, bias = key_lo)
// pairs: every mbase[m] - bias + key_lo is even (two containers per lane, 128-key tiles)
void launch_records_direct(const SetView &s, const uint64_t *mbase, uint64_t bias, uint32_t M, uint32_t key_lo,
                           uint32_t key_hi, uint32_t *rec, hipStream_t st, bool pairs = false, bool quads = false);
void launch_records_transpose(const uint64_t *mrec, const uint64_t *mbase, uint64_t bias, uint32_t M, uint32_t key_lo,
                              uint32_t key_hi, uint32_t *rec, hipStream_t st);
void launch_wide_runs_xor(const SetView &s, const uint32_t *cid, const uint64_t *seg, const uint32_t *klist,
                          uint32_t nk, uint8_t *out, const WideOut &wo, uint8_t *route, uint64_t *stats,
                          const XorRecords &xr, hipStream_t st);
// mrec: the set's packed records (workShyAnd's one-load metadata)
bool launch_wide_runs(int sem, const SetView &s, const uint64_t *mrec, const CidMap &cm, const uint64_t *seg,
                      const uint32_t *klist, uint32_t nk, uint8_t *out, const WideOut &wo, uint8_t *route,
                      uint64_t *stats, const XorRecords &xr, hipStream_t st);

// ---- setops.hip
void launch_bitmap_cards(const SetView &s, uint32_t nbitmaps, uint64_t *out, hipStream_t st);
void launch_gather(const uint8_t *src, const uint64_t *soff, const uint64_t *bytes, uint8_t *dst,
                   const uint64_t *doff, uint64_t n, hipStream_t st);
void launch_layout(const uint64_t *bigflag, const uint64_t *bidx, const uint64_t *soff, uint64_t small_base,
                   uint64_t *off, uint64_t n, hipStream_t st);
void launch_pack_records(const SetView &s, uint64_t n, uint64_t *mrec, hipStream_t st);
void launch_dense_check(const SetView &s, uint32_t nb, uint32_t lo, uint32_t cnt, uint32_t *bad, hipStream_t st);
// RoaringBitmap.runOptimize of every container of s into type / nruns / payload (same offsets); any_run[nb]
// (may be null): per bitmap, whether it holds a Run container afterwards
void launch_run_optimize(const SetView &s, uint64_t n, uint8_t *type, uint16_t *nruns, uint8_t *payload,
                         uint32_t nb, uint8_t *any_run, hipStream_t st);

// ---- generate.hip
struct GenSpec {
  // per container: key, target type (0 A, 1 B, 2 R) and parameter
  //   A: target cardinality; B: density numerator /256; R: target run count
  const uint16_t *key;
  const uint8_t *target;
  const uint32_t *param;
  const uint64_t *uid;   // content stream id: position (config 2) or (bitmap << 16 | key) (wide)
  uint64_t seed;
};
// pass 1: card / runs / final type / payload bytes per container
void launch_gen_measure(const GenSpec &g, uint64_t n, uint8_t *type, uint32_t *card, uint16_t *nruns,
                        uint64_t *big, uint64_t *small, hipStream_t st);
// pass 2: materialize at offsets
void launch_gen_emit(const GenSpec &g, uint64_t n, const uint8_t *type, const uint64_t *off, uint8_t *payload,
                     hipStream_t st);

} // namespace rbg
