// internal.hpp — host-side object model shared by the librbgpu translation units.
#pragma once
#include <algorithm>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace rbg {

int fail(int code, const char *fmt, ...);

#define HIPCHK(x)                                                                                      \
  do {                                                                                                 \
    hipError_t e_ = (x);                                                                               \
    if (e_ != hipSuccess) return ::rbg::fail(RB_EDEVICE, "%s failed: %s", #x, hipGetErrorString(e_));  \
  } while (0)

// A failed kernel launch (bad grid, out of resources) is only visible through hipGetLastError: every
// API call checks it once its launches are queued (before it reports success).
#define LAUNCHCHK()                                                                                    \
  do {                                                                                                 \
    hipError_t e_ = hipGetLastError();                                                                 \
    if (e_ != hipSuccess) return ::rbg::fail(RB_EDEVICE, "kernel launch failed: %s", hipGetErrorString(e_)); \
  } while (0)

// Device allocation cache: a freed block is reused for requests in [size/2, size].
struct DevPool {
  std::multimap<size_t, void *> free_;
  std::unordered_map<void *, size_t> size_;
  ~DevPool() { clear(); }
  void clear() {
    for (auto &kv : free_) {
      size_.erase(kv.second);
      (void)hipFree(kv.second);
    }
    free_.clear();
  }
  hipError_t alloc(void **p, size_t n) {
    n = std::max<size_t>((n + 255) & ~size_t(255), 256);
    auto it = free_.lower_bound(n);
    if (it != free_.end() && it->first <= 2 * n) {
      *p = it->second;
      free_.erase(it);
      return hipSuccess;
    }
    hipError_t e = hipMalloc(p, n);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      clear();
      e = hipMalloc(p, n);
      if (e != hipSuccess) return e;
    }
    size_[*p] = n;
    return hipSuccess;
  }
  void release(void *p) {
    if (!p) return;
    auto it = size_.find(p);
    if (it != size_.end()) free_.emplace(it->second, p);
  }
};

// Grow-only scratch region with bump allocation (reset by reserve()).
struct Workspace {
  uint8_t *base = nullptr;
  size_t cap = 0, used = 0;
  void destroy() {
    if (base) (void)hipFree(base);
    base = nullptr;
    cap = used = 0;
  }
  hipError_t reserve(size_t n, hipStream_t st) {
    used = 0;
    if (n <= cap) return hipSuccess;
    if (base) {
      (void)hipStreamSynchronize(st);
      (void)hipFree(base);
      base = nullptr;
    }
    cap = std::max(n, cap * 2);
    return hipMalloc((void **)&base, cap);
  }
  template <class T> T *take(size_t count) {
    size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
    T *p = reinterpret_cast<T *>(base + used);
    used += bytes;
    return p;
  }
};
inline size_t aligned256(size_t b) { return (b + 255) & ~size_t(255); }

// java.util.PriorityQueue's binary heap (OpenJDK: offer = append + siftUp, poll = the last element
// sifted down from the root), so elements that compare equal come out in the reference's order.
// cmp(a, b) < 0 / 0 / > 0 like compareTo.  Used by the global-order aggregations
// (FastAggregation.horizontal_* and priorityqueue_*), whose order the host computes.
template <class T, class Cmp> struct JavaHeap {
  std::vector<T> q;
  Cmp cmp;
  explicit JavaHeap(Cmp c) : cmp(c) {}
  bool empty() const { return q.empty(); }
  size_t size() const { return q.size(); }
  const T &peek() const { return q[0]; }
  void offer(const T &x) {
    size_t k = q.size();
    q.push_back(x);
    while (k > 0) {
      const size_t parent = (k - 1) >> 1;
      if (cmp(x, q[parent]) >= 0) break;
      q[k] = q[parent];
      k = parent;
    }
    q[k] = x;
  }
  T poll() {
    T result = q[0];
    T x = q.back();
    q.pop_back();
    const size_t n = q.size();
    if (n > 0) {
      size_t k = 0;
      while (k < (n >> 1)) {
        size_t child = 2 * k + 1;
        if (child + 1 < n && cmp(q[child], q[child + 1]) > 0) ++child;
        if (cmp(x, q[child]) <= 0) break;
        q[k] = q[child];
        k = child;
      }
      q[k] = x;
    }
    return result;
  }
};

// A compute-phase kernel span of a call's accounting (stats_end / stats_fill): kernels k = 0..n-1 ran between
// events ev[1+k] and ev[2+k] unless the span names its own (e0, e1); its algorithmic bytes are the counters
// in_word + out_word (+ in2 + out2: a concurrent pair), -1 = none.
struct KernelSpan {
  const char *name;
  int in_word, out_word;
  uint64_t items;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int in2 = -1, out2 = -1;
};
} // namespace rbg

struct rbgpu_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr; // second stream: the heavy task kernel runs beside the light one
  hipEvent_t ev[6] = {};   // [0] call start, [1..n] around the compute kernels, [5] call end
  hipEvent_t ev_side[3] = {}; // around the kernel on `side`; [2] after the side stream's last launch
  hipEvent_t ev_ext = {};     // ordering against a caller's stream (the asynchronous entry points)
  hipEvent_t ev_tot = {};     // pairwise: after the read-back of the scan totals (the early emit runs past it)
  rbg::DevPool pool;
  rbg::Workspace ws_pairs, ws_tasks, ws_segs; // per pair / per task / per merge-path segment
  uint64_t *d_stats = nullptr;  // [kStatWords * kStripes] striped algorithmic byte counters
  uint64_t *h_pinned = nullptr; // [16]
  uint64_t *h_stats = nullptr;  // [kStatWords * kStripes]
  uint8_t *h_stage = nullptr;   // pinned staging for small host->device arguments (pair indices)
  size_t h_stage_cap = 0;
  // host memory the GPU reads and writes directly (pinned, mapped, coherent): the small-batch
  // pairwise call's arguments and result words, so that call needs no copy engine
  uint8_t *h_small = nullptr, *d_small = nullptr; // one-launch result words (host-visible, 256 B: [0, 8) small batches
                                                  // and BSI RANGE, [kTailWord, +10) the general pipeline's tail)
  uint64_t *d_small_ctr = nullptr;                  // one-launch kernels' block tickets and counters (BSI, call tail)
  uint64_t *d_small_slots = nullptr;                // small-batch slot words, [2][kSmallSlots] (k_pair_small's kSlotUnset)
  uint64_t small_seq = 0;   // small-batch calls launched (the kernel's last block writes it to h_small[5])
  // A one-launch call returns on its sequence word, before its kernel's end is signalled (and before the
  // kernel-end release writes other XCDs' payload stores back from their L2s).  ev[5] is recorded behind
  // the latest such kernel (or behind a later call's work on the same stream), whose sequence number is
  // seq_recorded; seq_settled is the highest sequence number known complete.  Later work on `stream` is
  // ordered behind the kernel anyway; a use anywhere else (a caller's stream, rbgpu_set_wait) waits for ev[5]
  // (seq_settle).
  uint64_t seq_recorded = 0, seq_settled = 0;
  // a general-pipeline call that returned on its compaction's tail (CallTail): its kernel spans, timed when the
  // stats are asked for (rbgpu_get_stats; 0 = none pending)
  rbg::KernelSpan pend_spans[4];
  int pend_n = 0;
  uint64_t pend_tasks = 0;
  bool stats_pending = false; // ctx->last's times wait for their events (a small batch returned on h_small[5])
  bool stats_pending_k = false; // ... and the kernel's own pair (RBGPU_SMALL_KERNEL_TIMES)
  rbg::SmallTabInline small_inline{};               // small-batch tables passed in the kernel arguments
  std::vector<uint32_t> small_tab;                  // ... or copied to device memory (larger batches)
  rb_stats last{};
  uint64_t words[rbg::kStatWords] = {}; // the last call's counters, summed over stripes
  int refs = 1;                 // the handle + one per live set; destroyed at zero
  bool closed = false;
  bool stats_clean = false; // d_stats zeroed after the last read-back (stats_begin / stats_end)
  // pinned words the asynchronous calls' result counts land in (kAsyncSlots, a free list)
  uint64_t *h_async = nullptr; // [kAsyncSlots]
  std::vector<int> async_free;
};

struct rbgpu_set {
  rbgpu_ctx *ctx = nullptr;
  uint32_t nb = 0;
  uint64_t nc = 0, payload_bytes = 0;
  uint64_t *begin = nullptr;
  uint16_t *key = nullptr;
  uint8_t *type = nullptr;
  uint32_t *card = nullptr;
  uint16_t *nruns = nullptr;
  uint64_t *off = nullptr;
  uint8_t *payload = nullptr;
  std::vector<uint64_t> h_begin; // host copy of the CSR, downloaded on demand
  int64_t max_keys = -1;          // most containers in one bitmap (cached on first pairwise use)
  int64_t max_runs = -1;          // most runs in one Run container (cached on first small-batch use)
  // Derived metadata, built on first use and kept with the set (sets are immutable, like the
  // reference's immutable bitmaps: a cached index, never a cached result):
  //   dense_lo / dense_hi  every bitmap holds exactly the high keys [dense_lo, dense_hi) (-1: no; -2: unknown)
  //   mrec                 one packed 8-B record per container in set order (pack_rec: payload offset,
  //                        card, min(nruns, 15), type) — one load instead of four metadata arrays
  //   krec                 dense sets only: naive_xor's 4-B records (pack_xrec) key-major, krec[(k - dense_lo) * nb + b]
  int64_t dense_lo = -2, dense_hi = -2;
  uint64_t *mrec = nullptr;
  uint32_t *krec = nullptr;
  // rbgpu_pairwise_async: the call's work is still running; `nc` arrives in the context's pinned slot
  // `pend_slot` when `pending` completes (settle() waits for it and fills nc)
  hipEvent_t pending = nullptr;
  int pend_slot = -1;
  bool failed = false;            // its asynchronous call failed: every later use reports RB_EDEVICE
  // the last asynchronous call that reads this set as an input completes at `read_done` (its kernels may
  // still read the buffers after the call returned): freeing the set waits for it
  hipEvent_t read_done = nullptr;
  // written by the one-launch call with this sequence number (0: none): complete for the host's purposes
  // (nc known), but its kernel may not have ended (rbgpu_ctx::seq_recorded)
  uint64_t end_seq = 0;
  double derive_ms = 0.0;         // device time spent building mrec / krec (reported, not hidden)
  uint64_t derive_bytes = 0;      // their algorithmic bytes (metadata read + records written)
  // per derived item: 0 dense check, 1 mrec, 2 krec, 3 BSI key tables (rbgpu_set_setup_parts)
  double part_ms[4] = {0, 0, 0, 0};
  uint64_t part_bytes[4] = {0, 0, 0, 0};
  // BitSliceIndex compare (bsi.hip): key -> container tables of the set's bitmaps (one row each, then one
  // scratch row for a call's foundSet) and the keys of its last bitmap (ebM), built on first use
  int32_t *bsi_table = nullptr;
  uint32_t *bsi_klist = nullptr;
  uint32_t bsi_nk = 0, bsi_kmin = 0, bsi_kmax = 0; // ebM's key count and first / last key
  rbg::SetView view() const { return rbg::SetView{begin, key, type, card, nruns, off, payload}; }
};

namespace rbg {
int set_alloc(rbgpu_ctx *ctx, rbgpu_set *s, uint32_t nb, uint64_t nc, uint64_t payload);
// the pairwise pipeline with its flags (api.hip): x1.op(x2) in place (PairArgs::inplace), XOR results
// kept when empty (TaskMeta::keep_empty); a_idx / b_idx may hold kEmptyBitmap
int pairwise_call(rbgpu_ctx *ctx, int op, const rbgpu_set *a, const rbgpu_set *b, const uint32_t *a_idx,
                  const uint32_t *b_idx, uint32_t npairs, rbgpu_set **out, bool inplace, bool keep_empty);
void ctx_unref(rbgpu_ctx *ctx);
void set_release(rbgpu_set *s);
int ensure_h_begin(const rbgpu_set *s);
int ensure_call_words(rbgpu_ctx *ctx);
bool wait_call_seq(rbgpu_ctx *ctx, uint64_t seq, int word = 5);
// The one-launch hand-off around a kernel whose last block writes the result words and then `seq`:
// seq_begin surfaces a fault of an earlier one-launch kernel that ended after its call returned
// (non-blocking); seq_end (ctx->ev[5] recorded behind the kernel) waits for the sequence word (else for the
// stream) and fails with RB_EDEVICE when the words are not this call's — then the block counters and slot words
// are reset, since no block of the call handed over.  seq_settle waits for the kernel
// end of call `seq` (a no-op once known complete).
int seq_begin(rbgpu_ctx *ctx);
int seq_end(rbgpu_ctx *ctx, uint64_t seq, bool poll, const char *what, bool *seen, int word = 5);
int seq_settle(rbgpu_ctx *ctx, uint64_t seq);
// Derived metadata (rbgpu_set): built once per set on the set's stream, timed with events so the cost
// is reported (rbgpu_set_derive_ms), then cached — the set is immutable.  The start event follows an empty
// dispatch: an event recorded on an idle stream is stamped when the host records it, so it would also time
// the host's launch calls (scripts/micro/idle_event.cpp).
struct DeriveTimer {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  rbgpu_set *s;
  int part;
  DeriveTimer(rbgpu_set *s_, int part_) : s(s_), part(part_) {
    if (hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess) {
      launch_noop(s->ctx->stream);
      (void)hipEventRecord(e0, s->ctx->stream);
    }
  }
  ~DeriveTimer() {
    float ms = 0.f;
    if (e0 && e1 && hipEventRecord(e1, s->ctx->stream) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
        hipEventElapsedTime(&ms, e0, e1) == hipSuccess) {
      s->derive_ms += ms;
      s->part_ms[part] += ms;
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }
};
// A set returned by rbgpu_pairwise_async is usable by the host once its work is done: every entry point
// that reads a set first settles it (waits, fills nc).  A no-op for every other set.
int settle(const rbgpu_set *s);
// rbgpu_set_from_soa; allow_empty keeps empty Array / Run containers (a Roaring64Bitmap's kept-empty ones)
int set_from_soa(rbgpu_ctx *ctx, const rb_soa *soa, rbgpu_set **out, bool allow_empty);
constexpr int kAsyncSlots = 256; // asynchronous results pending at once per context (more: complete synchronously)
#define SETTLE(...)                                                                                    \
  do {                                                                                                 \
    for (const rbgpu_set *settle_s_ : {__VA_ARGS__})                                                   \
      if (const int settle_rc_ = ::rbg::settle(settle_s_)) return settle_rc_;                           \
  } while (0)
int ensure_max_keys(const rbgpu_set *s);
int ensure_max_runs(const rbgpu_set *s);
// derived metadata of an immutable set (see rbgpu_set): computed once, then cached
int ensure_dense(const rbgpu_set *s);
int ensure_mrec(const rbgpu_set *s);
int ensure_krec(const rbgpu_set *s); // needs a dense set (dense_lo >= 0)
uint64_t build_krec_range(const rbgpu_set *s, uint32_t *k, uint32_t a, uint32_t b, hipStream_t st);
// call accounting: zero the byte counters + record the start event / read everything back
// zero = false: the caller's counters come zeroed some other way (the small-batch path's H2D copy)
void stats_begin(rbgpu_ctx *ctx, bool zero = true);
// Compute-phase kernels k = 0..n-1 ran between events ev[1+k] and ev[2+k]; their algorithmic
// bytes are d_stats[in_word[k]] + d_stats[out_word[k]] (-1: none).
// A span may name its own events (e0, e1) and two more byte words (in2, out2: a concurrent pair).
// d_src: the counters (default ctx->d_stats)
int stats_end(rbgpu_ctx *ctx, uint64_t tasks, uint64_t result_containers, const KernelSpan *k, int n,
              const uint64_t *d_src = nullptr);
// stats_end's second half: ctx->words already hold the call's counters and the stream is idle
int stats_fill(rbgpu_ctx *ctx, uint64_t tasks, uint64_t result_containers, const KernelSpan *k, int n,
               bool timed = true);
// wide.hip
// keys outside [key_lo, key_hi) produce no result containers (key-range shard of the aggregation)
int wide_run(rbgpu_ctx *ctx, int sem, const rbgpu_set *in, const std::vector<uint32_t> &members, uint32_t key_lo,
             uint32_t key_hi, rbgpu_set **out);
int compact_keyed(rbgpu_ctx *ctx, const uint32_t *d_klist, uint32_t nk, const WideOut &wo, rbgpu_set *res);
uint64_t keyed_result_count(rbgpu_ctx *ctx, rbgpu_set *res);
// bsi.hip: op = BitmapSliceIndex.Operation ordinal (EQ, NEQ, LE, LT, GE, GT, RANGE); only the high keys in
// [key_lo, key_hi) are computed (a key-range shard of the answer)
int bsi_compare(rbgpu_ctx *ctx, const rbgpu_set *bsi, int op, uint64_t start, uint64_t end, uint64_t vmin,
                uint64_t vmax, const rbgpu_set *found, uint32_t key_lo, uint32_t key_hi, rbgpu_set **out);
// api.hip: the containers of bitmap 0 of `s` with keys in [key_lo, key_hi), as a new one-bitmap set
int set_key_subset(const rbgpu_set *s, uint32_t key_lo, uint32_t key_hi, rbgpu_set **out);
int set_gather(const rbgpu_set *s, const uint32_t *idx, uint32_t n, rbgpu_set **out);
// codec.hip: RoaringFormatSpec on the device.  d_in is readable up to in_lim; d_in_off[n + 1] (device).
int deserialize_device(rbgpu_ctx *ctx, const uint8_t *d_in, uint64_t in_lim, const uint64_t *d_in_off, uint32_t n,
                       rbgpu_set **out);
// host_dst: dst is host memory (staged through the device); offsets[count + 1] on the host
int serialize_device(const rbgpu_set *s, uint32_t first, uint32_t count, uint8_t *dst, uint64_t cap,
                     uint64_t *offsets, bool host_dst);
void set_mix(const int *m);
int generate_bsi(rbgpu_ctx *ctx, uint32_t nslices, uint64_t nrows, uint64_t seed, uint32_t key_lo, uint32_t key_hi,
                 rbgpu_set **out);
// generate.hip
int generate_sets(rbgpu_ctx *ctx, int workload, uint32_t n, uint64_t seed, uint32_t key_lo, uint32_t key_hi,
                  rbgpu_set **a, rbgpu_set **b);
} // namespace rbg
