// 3D soft-argmax over voxel world coordinates for gfx950.
//
// Replaces mvn/utils/op.py:84-96 (integrate_tensor_3d_with_coordinates):
//   softmax (op.py:89) or relu (op.py:91, no mass normalisation) over the flattened
//   V^3 volume of every (b, j), then coords = einsum("bnxyz,bxyzc->bnc") (op.py:94).
// The caller's `volumes * volume_multiplier` (triangulation.py:353) is fused.
//
// Two stream-ordered launches, both HBM-streaming:
//   pass 1  softargmax_partials : one wave per (2048-voxel chunk, joint, frame) streams
//           the chunk once and reduces (max, sum e, sum e*x, sum e*y, sum e*z) with wave
//           shuffles into one 5-float partial; no barriers, no LDS.
//   pass 2  softargmax_finalize : one block per (chunk, joint, frame).  Each wave folds
//           the frame/joint's partials (online-softmax rescale), chunk 0 writes the
//           coordinates, and every block writes its chunk of the normalised volume.
#include "common.hpp"

namespace mvn {
namespace {

constexpr int kSaBlock = 256;
constexpr int kSaVpt = 16;                      // voxels per thread
constexpr int kSaChunk = kSaBlock * kSaVpt;     // 4096 voxels per block
constexpr int kPartial = 5;                     // m, s, sx, sy, sz
constexpr int kPartChunk = 2048;                // voxels per pass-1 wave

template <typename T> struct Vec;
template <> struct Vec<float> { static constexpr int n = 4; };
template <> struct Vec<uint16_t> { static constexpr int n = 8; };

// Load `n` consecutive elements starting at i (vector load when fully in range).
template <typename T, int n>
__device__ __forceinline__ void load_run(const T* __restrict__ p, int i, int nvox, bool vec_ok, float (&v)[n], float fill) {
  if (vec_ok && i + n <= nvox) {
    if constexpr (sizeof(T) == 4) {
      const float4 q = *reinterpret_cast<const float4*>(p + i);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
      const uint4 q = *reinterpret_cast<const uint4*>(p + i);
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v[2 * k] = __uint_as_float(w[k] << 16);
        v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < n; ++k) v[k] = (i + k < nvox) ? to_f32(p[i + k]) : fill;
  }
}

template <typename T, int n>
__device__ __forceinline__ void store_run(T* __restrict__ p, int i, int nvox, bool vec_ok, const float (&v)[n]) {
  if (vec_ok && i + n <= nvox) {
    if constexpr (sizeof(T) == 4) {
      *reinterpret_cast<float4*>(p + i) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      uint32_t w[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) w[k] = uint32_t(f32_to_bf16(v[2 * k])) | (uint32_t(f32_to_bf16(v[2 * k + 1])) << 16);
      *reinterpret_cast<uint4*>(p + i) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < n; ++k) if (i + k < nvox) store_elem(p + i + k, v[k]);
  }
}

// Fold partial b into a (online softmax merge); relu mode is a plain sum.
template <bool SOFTMAX>
__device__ __forceinline__ void merge(float& m, float& s, float& sx, float& sy, float& sz,
                                      float m2, float s2, float sx2, float sy2, float sz2) {
  if constexpr (SOFTMAX) {
    const float M = fmaxf(m, m2);
    const float ka = (m == -INFINITY) ? 0.f : __expf(m - M);
    const float kb = (m2 == -INFINITY) ? 0.f : __expf(m2 - M);
    s = s * ka + s2 * kb;
    sx = sx * ka + sx2 * kb;
    sy = sy * ka + sy2 * kb;
    sz = sz * ka + sz2 * kb;
    m = M;
  } else {
    s += s2; sx += sx2; sy += sy2; sz += sz2;
  }
}

template <bool SOFTMAX>
__device__ __forceinline__ void wave_merge(float& m, float& s, float& sx, float& sy, float& sz) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, kWave), s2 = __shfl_xor(s, o, kWave);
    const float x2 = __shfl_xor(sx, o, kWave), y2 = __shfl_xor(sy, o, kWave), z2 = __shfl_xor(sz, o, kWave);
    merge<SOFTMAX>(m, s, sx, sy, sz, m2, s2, x2, y2, z2);
  }
}

// Pass 1: one WAVE per (frame, joint, 2048-voxel chunk) — no barriers, no LDS.  Each lane
// streams 32 voxels as vector runs, keeps an online (max, sum e, sum e*xyz) and the wave
// merges the lanes once.  Coordinates are re-read per joint from L2 (they are 12 B per
// voxel against 2-4 B of volume; L2 absorbs the re-reads, HBM sees them once).
template <typename T, bool SOFTMAX>
__global__ __launch_bounds__(kSaBlock) void softargmax_partials(
    const T* __restrict__ vol, long long bstride, long long jstride, const float* __restrict__ coords,
    float mult, float* __restrict__ part, int J, int nvox, int nchunk, bool vec_ok) {
  constexpr int VEC = Vec<T>::n;
  constexpr int RUNS = kPartChunk / (kWave * VEC);
  const int chunk = blockIdx.x, b = blockIdx.z;
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int j = blockIdx.y * (kSaBlock / kWave) + wid;
  if (j >= J) return;                                  // whole wave; this kernel has no barriers
  const T* vj = vol + b * bstride + j * jstride;
  const float* cb = coords + size_t(b) * nvox * 3;

  float m = SOFTMAX ? -INFINITY : 0.f, s = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
#pragma unroll
  for (int r = 0; r < RUNS; ++r) {
    const int i = chunk * kPartChunk + r * kWave * VEC + lane * VEC;
    float x[VEC];
    load_run<T, VEC>(vj, i, nvox, vec_ok, x, SOFTMAX ? -INFINITY : 0.f);
    float c[3 * VEC];
    if (vec_ok && i + VEC <= nvox) {
      const float4* cp = reinterpret_cast<const float4*>(cb + size_t(i) * 3);
#pragma unroll
      for (int q = 0; q < 3 * VEC / 4; ++q) {
        const float4 f = cp[q];
        c[4 * q] = f.x; c[4 * q + 1] = f.y; c[4 * q + 2] = f.z; c[4 * q + 3] = f.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 3 * VEC; ++q) c[q] = (i + q / 3 < nvox) ? cb[size_t(i) * 3 + q] : 0.f;
    }
    if constexpr (SOFTMAX) {
      float mr = -INFINITY;
#pragma unroll
      for (int k = 0; k < VEC; ++k) { x[k] = x[k] * mult; mr = fmaxf(mr, x[k]); }
      const float mn = fmaxf(m, mr);
      if (mn != -INFINITY) {
        const float kk = (m == -INFINITY) ? 0.f : __expf(m - mn);
        s *= kk; sx *= kk; sy *= kk; sz *= kk;
        m = mn;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const float e = __expf(x[k] - mn);
          s += e;
          sx = __builtin_fmaf(e, c[3 * k], sx);
          sy = __builtin_fmaf(e, c[3 * k + 1], sy);
          sz = __builtin_fmaf(e, c[3 * k + 2], sz);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        const float e = fmaxf(x[k] * mult, 0.f);
        s += e;
        sx = __builtin_fmaf(e, c[3 * k], sx);
        sy = __builtin_fmaf(e, c[3 * k + 1], sy);
        sz = __builtin_fmaf(e, c[3 * k + 2], sz);
      }
    }
  }
  wave_merge<SOFTMAX>(m, s, sx, sy, sz);
  if (lane == 0) {
    float* o = part + ((size_t(b) * J + j) * nchunk + chunk) * kPartial;
    o[0] = m; o[1] = s; o[2] = sx; o[3] = sy; o[4] = sz;
  }
}

template <typename T, typename TO, bool SOFTMAX>
__global__ __launch_bounds__(kSaBlock) void softargmax_finalize(
    const T* __restrict__ vol, long long bstride, long long jstride, float mult,
    const float* __restrict__ part, float* __restrict__ xyz, TO* __restrict__ out, int J, int nvox,
    int nchunk, int npart, bool vec_ok) {
  constexpr int VEC = Vec<T>::n;
  constexpr int RUNS = kSaVpt / VEC;
  const int chunk = blockIdx.x, j = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & (kWave - 1);

  // every wave folds the (b, j) partials redundantly: no LDS, no barrier
  const float* pj = part + (size_t(b) * J + j) * npart * kPartial;
  float m = SOFTMAX ? -INFINITY : 0.f, s = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
  for (int k = lane; k < npart; k += kWave) {
    const float* q = pj + size_t(k) * kPartial;
    merge<SOFTMAX>(m, s, sx, sy, sz, q[0], q[1], q[2], q[3], q[4]);
  }
  wave_merge<SOFTMAX>(m, s, sx, sy, sz);

  if (chunk == 0 && tid == 0) {
    float* o = xyz + (size_t(b) * J + j) * 3;
    if constexpr (SOFTMAX) {
      o[0] = sx / s; o[1] = sy / s; o[2] = sz / s;
    } else {
      o[0] = sx; o[1] = sy; o[2] = sz;
    }
  }
  if (out == nullptr) return;

  const float inv = 1.f / s;
  const T* vj = vol + b * bstride + j * jstride;
  TO* oj = out + (size_t(b) * J + j) * nvox;
#pragma unroll
  for (int r = 0; r < RUNS; ++r) {
    const int i = chunk * kSaChunk + r * kSaBlock * VEC + tid * VEC;
    float t[VEC];
    load_run<T, VEC>(vj, i, nvox, vec_ok, t, 0.f);
    float y[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const float v = t[k] * mult;
      y[k] = SOFTMAX ? __expf(v - m) * inv : fmaxf(v, 0.f);
    }
    if constexpr (sizeof(TO) == sizeof(T)) {
      store_run<TO, VEC>(oj, i, nvox, vec_ok, y);
    } else {  // bf16 in -> f32 out: two float4 runs
      float lo[4] = {y[0], y[1], y[2], y[3]};
      store_run<TO, 4>(oj, i, nvox, vec_ok, lo);
      if constexpr (VEC == 8) {
        float hi[4] = {y[4], y[5], y[6], y[7]};
        store_run<TO, 4>(oj, i + 4, nvox, vec_ok, hi);
      }
    }
  }
}

template <typename T, typename TO, bool SOFTMAX>
int launch(const void* vol, long long bs, long long js, const float* coords, float mult, float* xyz,
           void* out, float* part, int B, int J, int nvox, hipStream_t st) {
  const int nchunk = (nvox + kSaChunk - 1) / kSaChunk;       // pass-2 blocks per (b, j)
  const int npart = (nvox + kPartChunk - 1) / kPartChunk;     // pass-1 partials per (b, j)
  const bool vec_ok = (reinterpret_cast<uintptr_t>(vol) % 16 == 0) && (bs * sizeof(T)) % 16 == 0 &&
                      (js * sizeof(T)) % 16 == 0 && (nvox % 8 == 0) &&
                      (out == nullptr || reinterpret_cast<uintptr_t>(out) % 16 == 0);
  softargmax_partials<T, SOFTMAX><<<dim3(npart, (J + kSaBlock / kWave - 1) / (kSaBlock / kWave), B), kSaBlock, 0, st>>>(
      static_cast<const T*>(vol), bs, js, coords, mult, part, J, nvox, npart, vec_ok);
  if (!launch_ok()) return MVN_ERR_LAUNCH;
  softargmax_finalize<T, TO, SOFTMAX><<<dim3(out ? nchunk : 1, J, B), kSaBlock, 0, st>>>(
      static_cast<const T*>(vol), bs, js, mult, part, xyz, static_cast<TO*>(out), J, nvox, nchunk, npart, vec_ok);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

template <typename T, typename TO>
int launch_mode(int softmax, const void* vol, long long bs, long long js, const float* coords, float mult,
                float* xyz, void* out, float* part, int B, int J, int nvox, hipStream_t st) {
  return softmax ? launch<T, TO, true>(vol, bs, js, coords, mult, xyz, out, part, B, J, nvox, st)
                 : launch<T, TO, false>(vol, bs, js, coords, mult, xyz, out, part, B, J, nvox, st);
}

}  // namespace
}  // namespace mvn

extern "C" size_t mvn_softargmax3d_workspace_bytes(int B, int J, int Vx, int Vy, int Vz) {
  if (B <= 0 || J <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0) return 0;
  const long long nvox = (long long)Vx * Vy * Vz;
  const long long npart = (nvox + mvn::kPartChunk - 1) / mvn::kPartChunk;
  return size_t(B) * J * npart * mvn::kPartial * sizeof(float);
}

extern "C" int mvn_softargmax3d(const void* vol, int vol_dtype, int64_t vol_bstride, int64_t vol_jstride,
                                const float* coords, float multiplier, int softmax, float* out_xyz,
                                void* out_vol, int out_dtype, void* workspace, size_t workspace_bytes,
                                int B, int J, int Vx, int Vy, int Vz, void* stream) {
  using namespace mvn;
  if (!vol || !coords || !out_xyz) return MVN_ERR_ARG;
  if (softmax != 0 && softmax != 1) return MVN_ERR_ARG;
  if (B <= 0 || J <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0 || B > 65535 || J > 65535) return MVN_ERR_SHAPE;
  const long long nvox = (long long)Vx * Vy * Vz;
  if (nvox > (1LL << 30)) return MVN_ERR_SHAPE;
  if (vol_bstride < 0 || vol_jstride < 0) return MVN_ERR_SHAPE;
  const size_t need = mvn_softargmax3d_workspace_bytes(B, J, Vx, Vy, Vz);
  if (!workspace || workspace_bytes < need) return MVN_ERR_WORKSPACE;
  float* part = static_cast<float*>(workspace);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int n = int(nvox);
  if (vol_dtype == MVN_DTYPE_F32 && out_dtype == MVN_DTYPE_F32)
    return launch_mode<float, float>(softmax, vol, vol_bstride, vol_jstride, coords, multiplier, out_xyz, out_vol, part, B, J, n, st);
  if (vol_dtype == MVN_DTYPE_BF16 && out_dtype == MVN_DTYPE_BF16)
    return launch_mode<uint16_t, uint16_t>(softmax, vol, vol_bstride, vol_jstride, coords, multiplier, out_xyz, out_vol, part, B, J, n, st);
  if (vol_dtype == MVN_DTYPE_BF16 && out_dtype == MVN_DTYPE_F32)
    return launch_mode<uint16_t, float>(softmax, vol, vol_bstride, vol_jstride, coords, multiplier, out_xyz, out_vol, part, B, J, n, st);
  return MVN_ERR_DTYPE;
}
