// Nearest-voxel search of the volumetric cross-entropy loss for gfx950 (SURVEY.md §8f
// rank 4).
//
// Replaces the distance volume + torch.argmin of mvn/models/loss.py:63-67
// (VolumetricCELoss): for every (frame, joint) the index of the voxel whose coordinate is
// closest to the ground-truth keypoint.  Same rule as the reference: the f32 squared
// distance summed in sequence over x, y, z (verified), its square root (IEEE, correctly
// rounded: torch.sqrt on the GPU; numpy), and the FIRST index among equal roots — two
// distinct squared distances whose roots round to one f32 value tie, as in torch.argmin.
// One 256-thread block per (frame, joint); the coordinate volume is read once per joint
// (L2-resident across the joints of a frame).  Output: int32 flat voxel index.
#include <climits>

#include "common.hpp"

namespace mvn {
namespace {

constexpr int kBlock = 256;

// torch.argmin's order: NaN below every number (a NaN distance wins; the first NaN among
// several), then the smallest value, ties to the first index
__device__ __forceinline__ void better(float& d, int& i, float d2, int i2) {
  const bool n = d != d, n2 = d2 != d2;
  const bool take = n2 ? (!n || i2 < i) : (!n && (d2 < d || (d2 == d && i2 < i)));
  if (take) { d = d2; i = i2; }
}

__global__ __launch_bounds__(kBlock) void nearest_voxel(const float* __restrict__ coords, const float* __restrict__ kps,
                                                       int* __restrict__ out, int J, int nvox) {
  __shared__ float sd[kBlock / kWave];
  __shared__ int si[kBlock / kWave];
  const int bj = blockIdx.x, b = bj / J;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const float kx = kps[bj * 3], ky = kps[bj * 3 + 1], kz = kps[bj * 3 + 2];
  const float* c = coords + size_t(b) * nvox * 3;
  float best = INFINITY;
  int bi = INT_MAX;
  for (int i = t; i < nvox; i += kBlock) {
    const float dx = c[size_t(i) * 3] - kx, dy = c[size_t(i) * 3 + 1] - ky, dz = c[size_t(i) * 3 + 2] - kz;
    const float d2 = (dx * dx + dy * dy) + dz * dz;  // loss.py:63, summed x, y, z in order
    better(best, bi, sqrtf(d2), i);   // sqrtf: correctly rounded (v_sqrt + fma correction)
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) better(best, bi, __shfl_xor(best, o, kWave), __shfl_xor(bi, o, kWave));
  if (lane == 0) { sd[wid] = best; si[wid] = bi; }
  __syncthreads();
  if (t == 0) {
    for (int w = 1; w < kBlock / kWave; ++w) better(best, bi, sd[w], si[w]);
    out[bj] = (bi == INT_MAX) ? 0 : bi;             // (every voxel is a candidate: bi < nvox)
  }
}

}  // namespace
}  // namespace mvn

extern "C" int mvn_nearest_voxel(const float* coords, const float* keypoints, int* out_index, int B, int J,
                                 int Vx, int Vy, int Vz, void* stream) {
  using namespace mvn;
  if (!coords || !keypoints || !out_index) return MVN_ERR_ARG;
  if (B <= 0 || J <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0) return MVN_ERR_SHAPE;
  const long long nvox = (long long)Vx * Vy * Vz;
  if (nvox > (1LL << 30) || (long long)B * J > (1LL << 31) - 1) return MVN_ERR_SHAPE;
  nearest_voxel<<<B * J, kBlock, 0, static_cast<hipStream_t>(stream)>>>(coords, keypoints, out_index, J, int(nvox));
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}
