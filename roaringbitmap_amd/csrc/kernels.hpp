// kernels.hpp — launch wrappers of the librbgpu device kernels (all on one HIP stream).
#pragma once
#include "common.hpp"

namespace rbg {

// ---- scan.hip
uint64_t scan_tmp_words(uint64_t n);
void scan_exclusive(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *tmp, hipStream_t st);

// ---- pairwise.hip
struct PairArgs {
  int op;
  SetView A, B;
  const uint32_t *aidx; // may be null (identity)
  const uint32_t *bidx; // may be null (identity)
  uint32_t npairs;
};
// per task result metadata (workspace, indexed like tasks)
struct TaskMeta {
  uint16_t *key;
  uint8_t *type;   // kEmpty when dropped
  uint32_t *card;
  uint16_t *nruns;
};
// stats[0] += algorithmic input bytes, stats[1] += output bytes (see rb_stats)
void launch_pair_count(const PairArgs &a, uint64_t *ntask, uint64_t *nbig, uint64_t *small, uint64_t *stats,
                       hipStream_t st);
void launch_pair_emit(const PairArgs &a, const uint64_t *task_begin, const uint64_t *big_begin,
                      const uint64_t *small_begin, uint64_t small_base, Task *tasks, uint16_t *task_key,
                      hipStream_t st);
void launch_pairwise(int op, bool card_only, const SetView &A, const SetView &B, const Task *tasks,
                     uint64_t ntasks, uint8_t *out_payload, const TaskMeta &tm, hipStream_t st);
void launch_compact_count(const uint64_t *task_begin, uint32_t npairs, const uint8_t *ttype,
                          uint64_t *cnt, hipStream_t st);
void launch_compact_write(const uint64_t *task_begin, uint32_t npairs, const TaskMeta &tm, const Task *tasks,
                          const uint64_t *rbegin, const OutView &out, uint64_t *pair_card, uint64_t *stats,
                          hipStream_t st);

// ---- setops.hip
void launch_bitmap_cards(const SetView &s, uint32_t nbitmaps, uint64_t *out, hipStream_t st);
void launch_gather(const uint8_t *src, const uint64_t *soff, const uint64_t *bytes, uint8_t *dst,
                   const uint64_t *doff, uint64_t n, hipStream_t st);
void launch_layout(const uint64_t *bigflag, const uint64_t *bidx, const uint64_t *soff, uint64_t small_base,
                   uint64_t *off, uint64_t n, hipStream_t st);

// ---- generate.hip
struct GenSpec {
  // per container: key, target type (0 A, 1 B, 2 R) and parameter
  //   A: target cardinality; B: density numerator /256; R: target run count
  const uint16_t *key;
  const uint8_t *target;
  const uint32_t *param;
  uint64_t seed;
};
// pass 1: card / runs / final type / payload bytes per container
void launch_gen_measure(const GenSpec &g, uint64_t n, uint8_t *type, uint32_t *card, uint16_t *nruns,
                        uint64_t *big, uint64_t *small, hipStream_t st);
// pass 2: materialize at offsets
void launch_gen_emit(const GenSpec &g, uint64_t n, const uint8_t *type, const uint64_t *off, uint8_t *payload,
                     hipStream_t st);

} // namespace rbg
