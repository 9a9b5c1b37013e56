// Coordinate volumes of the volumetric model for gfx950.
//
// Replaces the per-frame Python loop of mvn/models/triangulation.py:280-341: a cuboid of
// side `cuboid_side` around each frame's base point, sampled on a V^3 grid
// (meshgrid 'ij'), rotated about the base point (volumetric.py:87-114; identity in eval,
// a random angle in training) and optionally re-axed for CMU data (permute + flip).
// One thread per output voxel; the host (mvn_rocm/volumetric.py) forms the float64
// cuboid position / centre / step / rotation exactly as the reference's numpy does and
// rounds them to f32 as torch does when they meet the f32 grid.  Per voxel, the f32 op
// order of the reference on CPU (verified bit-exact against its goldens):
//   c_k = pos_k + step_k * idx_k          (triangulation.py:313-315: mul, then add)
//   d_k = c_k - centre_k                  (:333)
//   r_r = fma(R[r][2], d_2, fma(R[r][1], d_1, R[r][0] * d_0))   (rot.mm, MKL K=3 order)
//   out_r = r_r + centre_r                (:335)
// with the CMU transfer (:338-341) as an index map: out[i][j][k] = v[i][k][V-1-j]
// (cuboid_coord, common.hpp — shared with the in-kernel coordinates of the *_cuboid ops).
#include "common.hpp"

namespace mvn {
namespace {

__global__ __launch_bounds__(256) void coord_volumes(const float* __restrict__ pos, const float* __restrict__ centre,
                                                     const float* __restrict__ step, const float* __restrict__ rot,
                                                     float* __restrict__ out, int V, int transfer) {
  const int b = blockIdx.y;
  const int nvox = V * V * V;
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= nvox) return;
  const int i = o / (V * V), j = (o / V) % V, k = o % V;
  float c[3];
  cuboid_coord(pos + b * 3, centre + b * 3, step + b * 3, rot + b * 9, V, i, j, k, transfer, c);
  float* op = out + (size_t(b) * nvox + o) * 3;
  op[0] = c[0]; op[1] = c[1]; op[2] = c[2];
}

}  // namespace
}  // namespace mvn

extern "C" int mvn_coord_volumes(const float* position, const float* centre, const float* step, const float* rot,
                                 float* out, int B, int V, int transfer_cmu, void* stream) {
  using namespace mvn;
  if (!position || !centre || !step || !rot || !out) return MVN_ERR_ARG;
  if (transfer_cmu != 0 && transfer_cmu != 1) return MVN_ERR_ARG;
  if (B <= 0 || V <= 0 || B > 65535 || (long long)V * V * V > (1LL << 30)) return MVN_ERR_SHAPE;
  const int nvox = V * V * V;
  coord_volumes<<<dim3((nvox + 255) / 256, B), 256, 0, static_cast<hipStream_t>(stream)>>>(
      position, centre, step, rot, out, V, transfer_cmu);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}
