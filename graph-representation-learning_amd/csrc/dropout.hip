// Feature dropout keyed on (seed, call, global row, column).
//
// Replaces nn.Dropout(0.5) on node-feature rows (gnn/models/networks/
// drop_robust_gcn.py:64,77,81,86,100).  The reference draws the mask from
// torch's generator over the tensor it is given, so a node-range shard of
// the graph could not reproduce the one-GPU mask of its rows, and ranks
// seeded alike would draw the same pattern over different rows.  Here the
// mask of element (r, c) is a counter hash of the global element id
// (row0 + r) * cols + c under the DropEdge key (seed, call): the same bits
// for a row wherever it is computed, and any row block's mask is computable
// on its own.  The backward is the same map applied to the gradient.
//
// HBM-bound elementwise pass: rows * cols * 8 bytes (one read, one write).
#include "grl_internal.h"

namespace grl {
namespace {

// out[r][c] = keep(row0 + r, c) ? x[r][c] * scale : 0; cols % 4 == 0 with
// 16-B aligned rows take the float4 form (one hash per element either way)
template <bool VEC>
__global__ __launch_bounds__(256) void feature_dropout_kernel(const float* __restrict__ x, int64_t ldx,
                                                              float* __restrict__ out, int64_t ldo, int64_t rows,
                                                              int cols, int64_t row0, DropDev d) {
  d = resolve_key(d);
  const int64_t per_row = VEC ? cols / 4 : cols;
  const int64_t n = rows * per_row;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / per_row;
    const int64_t j = i - r * per_row;
    const uint64_t id = (uint64_t)(row0 + r) * (uint64_t)cols;
    if (VEC) {
      float4 v = *reinterpret_cast<const float4*>(x + r * ldx + 4 * j);
      const uint64_t e = id + 4 * (uint64_t)j;
      v.x = dropedge_weight(d, v.x, e);
      v.y = dropedge_weight(d, v.y, e + 1);
      v.z = dropedge_weight(d, v.z, e + 2);
      v.w = dropedge_weight(d, v.w, e + 3);
      *reinterpret_cast<float4*>(out + r * ldo + 4 * j) = v;
    } else {
      out[r * ldo + j] = dropedge_weight(d, x[r * ldx + j], id + (uint64_t)j);
    }
  }
}

}  // namespace
}  // namespace grl

using namespace grl;

extern "C" int grl_feature_dropout(const float* x, int64_t ldx, float* out, int64_t ldo, int64_t rows, int32_t cols,
                                   int64_t row0, const GrlDropEdge* de, grl_stream_t stream) {
  TraceRange trace_("grl_feature_dropout");
  GRL_CHECK_ARG(rows >= 0 && cols >= 0 && row0 >= 0, "grl_feature_dropout: negative size");
  GRL_CHECK_ARG(ldx >= cols && ldo >= cols, "grl_feature_dropout: row strides below cols");
  if (rows == 0 || cols == 0) return GRL_OK;
  GRL_CHECK_ARG(x && out, "grl_feature_dropout: NULL pointer");
  const DropDev d = to_dev(de);
  const bool vec = cols % 4 == 0 && ldx % 4 == 0 && ldo % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 &&
                   reinterpret_cast<uintptr_t>(out) % 16 == 0;
  const int64_t n = rows * (vec ? cols / 4 : cols);
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(n, 256), 8 * 1024);
  hipStream_t st = as_stream(stream);
  if (vec)
    hipLaunchKernelGGL(feature_dropout_kernel<true>, dim3(grid), dim3(256), 0, st, x, ldx, out, ldo, rows, (int)cols,
                       row0, d);
  else
    hipLaunchKernelGGL(feature_dropout_kernel<false>, dim3(grid), dim3(256), 0, st, x, ldx, out, ldo, rows, (int)cols,
                       row0, d);
  GRL_LAUNCH_CHECK();
  return GRL_OK;
}
