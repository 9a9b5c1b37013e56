// 2D soft-argmax of per-view heatmaps for gfx950 — the algebraic path's producer of the
// DLT's 2D points.
//
// Replaces mvn/utils/op.py:11-47 (integrate_tensor_2d), with the caller's
// `heatmaps * heatmap_multiplier` (triangulation.py:164) fused:
//   softmax (op.py:25) or relu (op.py:27) over the flattened H*W map of every (b, j);
//   x = sum_w w * sum_h p[h, w], y = sum_h h * sum_w p[h, w] (op.py:31-38); with relu the
//   sums are divided by the mass (op.py:40-42), with softmax the map is already
//   normalised, so both modes are x = sum(p * w) / sum(p) — the exp / relu weights are
//   never normalised in registers, only the returned map is.
//
// One 256-thread block per map (a 96x96 map is 37 KB: three passes over it run from L2):
// pass 1 the max, pass 2 (sum e, sum e*w, sum e*h), pass 3 the normalised map (skipped when
// the caller does not want it).  Reductions: DPP within a wave, LDS across the 4 waves.
#include <math.h>

#include "common.hpp"

namespace mvn {
namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;

template <int CTRL, int RMASK> __device__ __forceinline__ float dpp(float v, float ident) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ident), __float_as_int(v), CTRL, RMASK, 0xf, false));
}
// Wave reductions valid in lane 63 (row_shr steps, then row_bcast:15 / row_bcast:31).
__device__ __forceinline__ float wave_max63(float v) {
  const float I = -INFINITY;
  v = fmaxf(v, dpp<0x111, 0xf>(v, I)); v = fmaxf(v, dpp<0x112, 0xf>(v, I));
  v = fmaxf(v, dpp<0x114, 0xf>(v, I)); v = fmaxf(v, dpp<0x118, 0xf>(v, I));
  v = fmaxf(v, dpp<0x142, 0xa>(v, I)); v = fmaxf(v, dpp<0x143, 0xc>(v, I));
  return v;
}
__device__ __forceinline__ float wave_sum63(float v) {
  v += dpp<0x111, 0xf>(v, 0.f); v += dpp<0x112, 0xf>(v, 0.f);
  v += dpp<0x114, 0xf>(v, 0.f); v += dpp<0x118, 0xf>(v, 0.f);
  v += dpp<0x142, 0xa>(v, 0.f); v += dpp<0x143, 0xc>(v, 0.f);
  return v;
}

template <typename T, typename TO, bool SOFTMAX>
__global__ __launch_bounds__(kBlock) void softargmax2d(const T* __restrict__ hm, float mult, float* __restrict__ xy,
                                                      TO* __restrict__ out, int H, int W) {
  __shared__ float red[3][kWaves];
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const size_t map = blockIdx.x;
  const int n = H * W;
  const T* p = hm + map * size_t(n);

  // pass 1: max of mult * x (softmax only)
  float M = 0.f;
  if constexpr (SOFTMAX) {
    float lm = -INFINITY;
    for (int i = t; i < n; i += kBlock) lm = fmaxf(lm, to_f32(p[i]) * mult);
    lm = wave_max63(lm);
    if (lane == kWave - 1) red[0][wid] = lm;
    __syncthreads();
    M = red[0][0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) M = fmaxf(M, red[0][w]);
    __syncthreads();
  }

  // pass 2: mass and first moments
  float s = 0.f, sx = 0.f, sy = 0.f;
  for (int i = t; i < n; i += kBlock) {
    const float v = to_f32(p[i]) * mult;
    const float e = SOFTMAX ? __expf(v - M) : fmaxf(v, 0.f);
    const int h = i / W, w = i - h * W;
    s += e;
    sx = __builtin_fmaf(e, float(w), sx);
    sy = __builtin_fmaf(e, float(h), sy);
  }
  s = wave_sum63(s); sx = wave_sum63(sx); sy = wave_sum63(sy);
  if (lane == kWave - 1) { red[0][wid] = s; red[1][wid] = sx; red[2][wid] = sy; }
  __syncthreads();
  s = red[0][0]; sx = red[1][0]; sy = red[2][0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) { s += red[0][w]; sx += red[1][w]; sy += red[2][w]; }
  if (t == 0) {
    xy[map * 2] = sx / s;                     // op.py:34, 40: x, normalised by the mass
    xy[map * 2 + 1] = sy / s;
  }

  // pass 3: the returned map — softmax normalised, relu as is (op.py:25-27)
  if (out != nullptr) {
    const float inv = 1.f / s;
    TO* o = out + map * size_t(n);
    for (int i = t; i < n; i += kBlock) {
      const float v = to_f32(p[i]) * mult;
      store_elem(o + i, SOFTMAX ? __expf(v - M) * inv : fmaxf(v, 0.f));
    }
  }
}

// Register-resident form (r17) for maps of at most kBlock * 4 * RUNS pixels with W % 4 == 0 and
// 16-byte aligned maps (every BASELINE config: 96^2): each thread loads its runs of 4
// consecutive pixels ONCE (vector loads), reduces the max, then (sum e, sum e*w, sum e*h), and
// writes the normalised map from registers — one pass over memory instead of three, and the
// (h, w) of a run from one division instead of one per pixel.  Config 1's 4 x 17 maps of 96^2:
// 16.6 -> 4.9 us (256 x 17 maps: 105 -> 64 us), profiles/r17_ab_softargmax2d.txt.
constexpr int kRuns = 12;                      // up to 12,288 pixels per map
template <typename T, typename TO, bool SOFTMAX>
__global__ __launch_bounds__(kBlock) void softargmax2d_reg(const T* __restrict__ hm, float mult, float* __restrict__ xy,
                                                          TO* __restrict__ out, int H, int W) {
  __shared__ float red[3][kWaves];
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const size_t map = blockIdx.x;
  const int n = H * W;
  const T* p = hm + map * size_t(n);
  float v[kRuns][4];
#pragma unroll
  for (int r = 0; r < kRuns; ++r) {
    const int i = (r * kBlock + t) * 4;
    if (i < n) {
      if constexpr (sizeof(T) == 4) {
        const float4 q = *reinterpret_cast<const float4*>(p + i);
        v[r][0] = q.x; v[r][1] = q.y; v[r][2] = q.z; v[r][3] = q.w;
      } else {
        const uint2 q = *reinterpret_cast<const uint2*>(p + i);
        v[r][0] = __uint_as_float(q.x << 16); v[r][1] = __uint_as_float(q.x & 0xffff0000u);
        v[r][2] = __uint_as_float(q.y << 16); v[r][3] = __uint_as_float(q.y & 0xffff0000u);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) v[r][k] = v[r][k] * mult;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[r][k] = SOFTMAX ? -INFINITY : 0.f;
    }
  }
  float M = 0.f;
  if constexpr (SOFTMAX) {
    float lm = -INFINITY;
#pragma unroll
    for (int r = 0; r < kRuns; ++r)
#pragma unroll
      for (int k = 0; k < 4; ++k) lm = fmaxf(lm, v[r][k]);
    lm = wave_max63(lm);
    if (lane == kWave - 1) red[0][wid] = lm;
    __syncthreads();
    M = red[0][0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) M = fmaxf(M, red[0][w]);
    __syncthreads();
  }
  float s = 0.f, sx = 0.f, sy = 0.f;
#pragma unroll
  for (int r = 0; r < kRuns; ++r) {
    const int i = (r * kBlock + t) * 4;
    if (i >= n) continue;
    const int h = i / W, w0 = i - h * W;      // a run of 4 stays in one row (W % 4 == 0)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float e = SOFTMAX ? __expf(v[r][k] - M) : fmaxf(v[r][k], 0.f);
      v[r][k] = e;
      s += e;
      sx = __builtin_fmaf(e, float(w0 + k), sx);
      sy = __builtin_fmaf(e, float(h), sy);
    }
  }
  s = wave_sum63(s); sx = wave_sum63(sx); sy = wave_sum63(sy);
  if (lane == kWave - 1) { red[0][wid] = s; red[1][wid] = sx; red[2][wid] = sy; }
  __syncthreads();
  s = red[0][0]; sx = red[1][0]; sy = red[2][0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) { s += red[0][w]; sx += red[1][w]; sy += red[2][w]; }
  if (t == 0) {
    xy[map * 2] = sx / s;
    xy[map * 2 + 1] = sy / s;
  }
  if (out != nullptr) {
    const float inv = SOFTMAX ? 1.f / s : 1.f;
    TO* o = out + map * size_t(n);
#pragma unroll
    for (int r = 0; r < kRuns; ++r) {
      const int i = (r * kBlock + t) * 4;
      if (i >= n) continue;
      float y[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = SOFTMAX ? v[r][k] * inv : v[r][k];
      if constexpr (sizeof(TO) == 4)
        *reinterpret_cast<float4*>(o + i) = make_float4(y[0], y[1], y[2], y[3]);
      else
        *reinterpret_cast<uint2*>(o + i) = make_uint2(pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]));
    }
  }
}

template <typename T, typename TO>
int launch(const void* hm, float mult, int softmax, float* xy, void* out, int maps, int H, int W, hipStream_t s) {
  const bool reg = (long long)H * W <= (long long)kBlock * 4 * kRuns && W % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(hm) % 16 == 0 && (out == nullptr || reinterpret_cast<uintptr_t>(out) % 16 == 0);
  if (reg) {
    if (softmax)
      softargmax2d_reg<T, TO, true><<<maps, kBlock, 0, s>>>(static_cast<const T*>(hm), mult, xy, static_cast<TO*>(out), H, W);
    else
      softargmax2d_reg<T, TO, false><<<maps, kBlock, 0, s>>>(static_cast<const T*>(hm), mult, xy, static_cast<TO*>(out), H, W);
    return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
  }
  if (softmax)
    softargmax2d<T, TO, true><<<maps, kBlock, 0, s>>>(static_cast<const T*>(hm), mult, xy, static_cast<TO*>(out), H, W);
  else
    softargmax2d<T, TO, false><<<maps, kBlock, 0, s>>>(static_cast<const T*>(hm), mult, xy, static_cast<TO*>(out), H, W);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

}  // namespace
}  // namespace mvn

extern "C" int mvn_softargmax2d(const void* heatmaps, int dtype, float multiplier, int softmax, float* out_xy,
                                void* out_maps, int out_dtype, int B, int J, int H, int W, void* stream) {
  using namespace mvn;
  if (!heatmaps || !out_xy) return MVN_ERR_ARG;
  if (softmax != 0 && softmax != 1) return MVN_ERR_ARG;
  if (B <= 0 || J <= 0 || H <= 0 || W <= 0) return MVN_ERR_SHAPE;
  if ((long long)B * J > (1LL << 31) - 1 || (long long)H * W > (1LL << 30)) return MVN_ERR_SHAPE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int maps = B * J;
  if (dtype == MVN_DTYPE_F32 && out_dtype == MVN_DTYPE_F32)
    return launch<float, float>(heatmaps, multiplier, softmax, out_xy, out_maps, maps, H, W, s);
  if (dtype == MVN_DTYPE_BF16 && out_dtype == MVN_DTYPE_BF16)
    return launch<uint16_t, uint16_t>(heatmaps, multiplier, softmax, out_xy, out_maps, maps, H, W, s);
  if (dtype == MVN_DTYPE_BF16 && out_dtype == MVN_DTYPE_F32)
    return launch<uint16_t, float>(heatmaps, multiplier, softmax, out_xy, out_maps, maps, H, W, s);
  return MVN_ERR_DTYPE;
}
