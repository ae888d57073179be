// wide.hip — wide FastAggregation / ParallelAggregation over many bitmaps (filled in below).
#include "internal.hpp"
#include "kernels.hpp"

namespace rbg {
int wide_run(rbgpu_ctx *ctx, int sem, const rbgpu_set *in, const std::vector<uint32_t> &members, rbgpu_set **out) {
  (void)ctx; (void)sem; (void)in; (void)members; (void)out;
  return fail(RB_EINVAL, "wide aggregation not implemented yet");
}
} // namespace rbg
