// 3D soft-argmax over voxel world coordinates for gfx950.
//
// Replaces mvn/utils/op.py:84-96 (integrate_tensor_3d_with_coordinates):
//   softmax (op.py:89) or relu (op.py:91, no mass normalisation) over the flattened
//   V^3 volume of every (b, j), then coords = einsum("bnxyz,bxyzc->bnc") (op.py:94).
// The caller's `volumes * volume_multiplier` (triangulation.py:353) is fused.
//
// Three stream-ordered launches (the middle one tiny):
//   pass 1  softargmax_partials : one wave per (512-voxel chunk, frame) holds the chunk's
//           coordinates and loops over the joints, reducing (max, sum e, sum e*x, sum e*y,
//           sum e*z) per joint with DPP into one 5-float partial; no barriers, no LDS.
//   pass 2  softargmax_combine  : one wave per (frame, joint) folds the partials (online
//           rescale), writes the coordinates and (max, 1/sum).
//   pass 3  softargmax_finalize : one block per (4096-voxel chunk, joint, frame) streams
//           the normalised volume (skipped when the caller does not want it).
#include <algorithm>
#include <atomic>

#include "common.hpp"

// The finalize is the volume's last reader and its output is written once: both streams
// non-temporal, so that they do not evict what the next launches read from the MALL (the
// unprojection's feature maps and coordinates: bench step 292 -> 261 us at config 2).

namespace mvn {
namespace {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));

constexpr int kSaBlock = 256;
constexpr int kSaVpt = 16;                      // voxels per thread
constexpr int kSaChunk = kSaBlock * kSaVpt;     // 4096 voxels per block
constexpr int kPartial = 5;                     // m, s, sx, sy, sz
constexpr bool kFinalNtLoads = true, kFinalNtStores = true;   // the finalize's streams (comment above)
// voxels per pass-1 wave (all joints), per volume dtype; the workspace is sized for the
// smaller.  1024 (16 voxels per lane in flight per joint, half the DPP reductions per voxel)
// vs 512: config 2 soft-argmax 81.2 -> 76.2 us, config 3 186.1 -> 182.4 us (A/B, r09).
template <typename T> constexpr int kPartChunkT = 1024;
constexpr int kPartChunkMin = 1024;

template <typename T> struct Vec;
template <> struct Vec<float> { static constexpr int n = 4; };
template <> struct Vec<uint16_t> { static constexpr int n = 8; };

// Load `n` consecutive elements starting at i (vector load when fully in range).
template <typename T, int n, bool NT = false>
__device__ __forceinline__ void load_run(const T* __restrict__ p, int i, int nvox, bool vec_ok, float (&v)[n], float fill) {
  if (vec_ok && i + n <= nvox) {
    if constexpr (sizeof(T) == 4) {
      const f4v q = NT ? __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p + i))
                       : *reinterpret_cast<const f4v*>(p + i);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
      const u4v q = NT ? __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p + i))
                       : *reinterpret_cast<const u4v*>(p + i);
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

template <typename T, int n, bool NT = false>
__device__ __forceinline__ void store_run(T* __restrict__ p, int i, int nvox, bool vec_ok, const float (&v)[n]) {
  if (vec_ok && i + n <= nvox) {
    if constexpr (sizeof(T) == 4) {
      const f4v q = {v[0], v[1], v[2], v[3]};
      if (NT) __builtin_nontemporal_store(q, reinterpret_cast<f4v*>(p + i));
      else *reinterpret_cast<f4v*>(p + i) = q;
    } else {
      u4v q;
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = pack_bf16x2(v[2 * k], v[2 * k + 1]);
      if (NT) __builtin_nontemporal_store(q, reinterpret_cast<u4v*>(p + i));
      else *reinterpret_cast<u4v*>(p + i) = q;
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

// Wave reductions: row_shr DPP steps, then row_bcast:15 / row_bcast:31; the result is
// valid in lane 63 (6 DPP-fused VALU ops each).
template <int CTRL, int RMASK> __device__ __forceinline__ float dpp_f(float v, float ident) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(ident), __float_as_int(v), CTRL, RMASK, 0xf, false));
}
__device__ __forceinline__ float wave_max63(float v) {
  constexpr float I = -INFINITY;
  v = fmaxf(v, dpp_f<0x111, 0xf>(v, I)); v = fmaxf(v, dpp_f<0x112, 0xf>(v, I));
  v = fmaxf(v, dpp_f<0x114, 0xf>(v, I)); v = fmaxf(v, dpp_f<0x118, 0xf>(v, I));
  v = fmaxf(v, dpp_f<0x142, 0xa>(v, I)); v = fmaxf(v, dpp_f<0x143, 0xc>(v, I));
  return v;
}
__device__ __forceinline__ float wave_sum63(float v) {
  v += dpp_f<0x111, 0xf>(v, 0.f); v += dpp_f<0x112, 0xf>(v, 0.f);
  v += dpp_f<0x114, 0xf>(v, 0.f); v += dpp_f<0x118, 0xf>(v, 0.f);
  v += dpp_f<0x142, 0xa>(v, 0.f); v += dpp_f<0x143, 0xc>(v, 0.f);
  return v;
}

// Pass 1: one WAVE per (frame, 512-voxel chunk), looping over ALL joints — no barriers,
// no LDS.  The chunk's coordinates are loaded into registers once (12 B per voxel; one
// wave per joint would re-read them J times), then per joint every lane loads its 16
// voxels as vector runs (the next joint's loads are in flight during this joint's math),
// the wave max is reduced first so that all lanes exponentiate against the same max
// (plain additive sums, no per-lane rescaling), and (sum e, sum e*x, sum e*y, sum e*z)
// are DPP-reduced into one 5-float partial per (frame, joint, chunk).
template <typename T, bool SOFTMAX>
__global__ __launch_bounds__(kSaBlock) void softargmax_partials(
    const T* __restrict__ vol, long long bstride, long long jstride, const float* __restrict__ coords,
    const float* __restrict__ cub, int V, int transfer, float mult, float* __restrict__ part, int J, int nvox,
    int nchunk, bool vec_ok) {
  constexpr int VEC = Vec<T>::n;
  constexpr int kPartChunk = kPartChunkT<T>;
  constexpr int RUNS = kPartChunk / (kWave * VEC);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  const int chunk = blockIdx.x * (kSaBlock / kWave) + wid, b = blockIdx.y;
  // joints [ja, jb) of this wave: gridDim.z splits the joints when the frames alone give too
  // few waves to fill the chip (config 2: 8 frames x 256 chunks = 2 waves per SIMD)
  const int jn = (J + int(gridDim.z) - 1) / int(gridDim.z), ja = int(blockIdx.z) * jn, jb = min(J, ja + jn);
  if (ja >= jb) return;
  if (chunk >= nchunk) return;                         // whole wave; this kernel has no barriers
  const T* vb = vol + b * bstride;
  const float* cb = cub ? nullptr : coords + size_t(b) * nvox * 3;
  const float fill = SOFTMAX ? -INFINITY : 0.f;

  float c[RUNS][3 * VEC];
  if (cub) {
    // coordinates formed in-kernel from the frame's cuboid (bit-identical to mvn_coord_volumes)
    const float* cf = cub + size_t(b) * MVN_CUBOID_FLOATS;
#pragma unroll
    for (int r = 0; r < RUNS; ++r) {
      const int i = chunk * kPartChunk + r * kWave * VEC + lane * VEC;
      int gi = i / (V * V), gj = (i / V) % V, gk = i % V;
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        float o[3];
        cuboid_coord(cf, V, gi, gj, gk, transfer, o);
        const bool in = i + u < nvox;
        c[r][3 * u] = in ? o[0] : 0.f; c[r][3 * u + 1] = in ? o[1] : 0.f; c[r][3 * u + 2] = in ? o[2] : 0.f;
        if (++gk == V) { gk = 0; if (++gj == V) { gj = 0; ++gi; } }
      }
    }
  } else {
#pragma unroll
  for (int r = 0; r < RUNS; ++r) {
    const int i = chunk * kPartChunk + r * kWave * VEC + lane * VEC;
    if (vec_ok && i + VEC <= nvox) {
      const float4* cp = reinterpret_cast<const float4*>(cb + size_t(i) * 3);
#pragma unroll
      for (int u = 0; u < 3 * VEC / 4; ++u) {
        const float4 f = cp[u];
        c[r][4 * u] = f.x; c[r][4 * u + 1] = f.y; c[r][4 * u + 2] = f.z; c[r][4 * u + 3] = f.w;
      }
    } else {
#pragma unroll
      for (int u = 0; u < 3 * VEC; ++u) c[r][u] = (i + u / 3 < nvox) ? cb[size_t(i) * 3 + u] : 0.f;
    }
  }
  }
  auto load = [&](int j, float (&x)[RUNS][VEC]) {
#pragma unroll
    for (int r = 0; r < RUNS; ++r)
      load_run<T, VEC>(vb + j * jstride, chunk * kPartChunk + r * kWave * VEC + lane * VEC, nvox, vec_ok, x[r], fill);
  };
  // One joint's 5-float partial from its (multiplier-scaled) values, wave-uniform in q.
  auto reduce_values = [&](float (&x)[RUNS][VEC], float (&q)[kPartial]) __attribute__((always_inline)) {
    float m = 0.f, s = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
    if constexpr (SOFTMAX) {
      constexpr float kLog2e = 1.4426950408889634f;
      float lm = -INFINITY;
#pragma unroll
      for (int r = 0; r < RUNS; ++r)
#pragma unroll
        for (int k = 0; k < VEC; ++k) { x[r][k] = x[r][k] * mult; lm = fmaxf(lm, x[r][k]); }
      m = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wave_max63(lm)), kWave - 1));
      if (m != -INFINITY) {                            // wave-uniform
        const float ml = m * kLog2e;
#pragma unroll
        for (int r = 0; r < RUNS; ++r)
#pragma unroll
          for (int k = 0; k < VEC; ++k) {
            const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(x[r][k], kLog2e, -ml));
            s += e;
            sx = __builtin_fmaf(e, c[r][3 * k], sx);
            sy = __builtin_fmaf(e, c[r][3 * k + 1], sy);
            sz = __builtin_fmaf(e, c[r][3 * k + 2], sz);
          }
      }
    } else {
#pragma unroll
      for (int r = 0; r < RUNS; ++r)
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          const float e = fmaxf(x[r][k] * mult, 0.f);
          s += e;
          sx = __builtin_fmaf(e, c[r][3 * k], sx);
          sy = __builtin_fmaf(e, c[r][3 * k + 1], sy);
          sz = __builtin_fmaf(e, c[r][3 * k + 2], sz);
        }
    }
    s = wave_sum63(s); sx = wave_sum63(sx); sy = wave_sum63(sy); sz = wave_sum63(sz);
    auto l63 = [](float v) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), kWave - 1)); };
    q[0] = m; q[1] = l63(s); q[2] = l63(sx); q[3] = l63(sy); q[4] = l63(sz);
  };
  auto reduce_joint = [&](int j, float (&x)[RUNS][VEC]) __attribute__((always_inline)) {
    float q[kPartial];
    reduce_values(x, q);
    if (lane == kWave - 1) {
      float* o = part + ((size_t(b) * J + j) * nchunk + chunk) * kPartial;
#pragma unroll
      for (int k = 0; k < kPartial; ++k) o[k] = q[k];
    }
  };

  const int i0 = chunk * kPartChunk + lane * VEC;
  const size_t frame_bytes = (size_t(J - 1) * size_t(jstride) + size_t(nvox)) * sizeof(T);
  if (vec_ok && chunk * kPartChunk + kPartChunk <= nvox && jb - ja <= kWave && frame_bytes < (size_t(1) << 31) &&
      jstride * sizeof(T) < (1u << 31)) {
    // Full chunk, aligned, frame addressable by a buffer descriptor: the raw 16-byte loads
    // of PF joints in flight (a ring of register sets refilled PF joints ahead), issued
    // UNCONDITIONALLY (past the last joint the offset is out of range: no memory access),
    // and no stores inside the joint loop — each joint's partial is parked in lane j % 64 of
    // five registers and the lanes store together after the loop.  gfx950's vmcnt counts
    // loads and stores in issue order: a conditional load or a divergent store in the loop
    // made the compiler's waits conservative (vmcnt(0) at every ring turn, draining the
    // prefetch ring).  J <= 64 (one lane per joint); more joints take the path below.
    constexpr int PF = sizeof(T) == 2 ? 8 : 4;
    const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(vb), 0, int(frame_bytes), 0x00020000);
    uint4 raw[PF][RUNS];
    // past the last joint the out-of-range marker rides in the per-lane offset (voffset, which
    // the range check always covers: frame_bytes < 2^31), soffset 0 — the load returns zeros
    // without a memory access
    auto issue = [&](int j, uint4 (&q)[RUNS]) __attribute__((always_inline)) {
      const bool live = j < jb;
      const uint32_t jo = live ? uint32_t(j) * uint32_t(jstride) * uint32_t(sizeof(T)) : 0u;
#pragma unroll
      for (int r = 0; r < RUNS; ++r)
        q[r] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                             vrs, live ? uint32_t((i0 + r * kWave * VEC) * sizeof(T)) : 0x80000000u, jo, 0));
    };
    float acc[kPartial] = {0.f, 0.f, 0.f, 0.f, 0.f};
    auto flush = [&](int jbase, int n) __attribute__((always_inline)) {
      if (lane < n) {
        float* o = part + ((size_t(b) * J + jbase + lane) * nchunk + chunk) * kPartial;
#pragma unroll
        for (int k = 0; k < kPartial; ++k) o[k] = acc[k];
      }
    };
    // ring slots filled in joint order (the scheduler otherwise reverses them, and the wait
    // analysis then merges "slot 0 issued last" into the loop: vmcnt at every ring turn)
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      issue(ja + p, raw[p]);
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int j0 = ja; j0 < jb; j0 += PF) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const int j = j0 + p;
        if (j >= jb) goto joints_done;     // an exit edge, not a merge into the loop latch
        float x[RUNS][VEC];
#pragma unroll
        for (int r = 0; r < RUNS; ++r) {
          const uint32_t w[4] = {raw[p][r].x, raw[p][r].y, raw[p][r].z, raw[p][r].w};
          if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) x[r][k] = __uint_as_float(w[k]);
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              x[r][2 * k] = __uint_as_float(w[k] << 16);
              x[r][2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
            }
          }
        }
        issue(j + PF, raw[p]);
        float q[kPartial];
        reduce_values(x, q);
        const bool mine = lane == j - ja;
#pragma unroll
        for (int k = 0; k < kPartial; ++k) acc[k] = mine ? q[k] : acc[k];
      }
    }
  joints_done:
    flush(ja, jb - ja);
    return;
  }
  if (vec_ok && chunk * kPartChunk + kPartChunk <= nvox) {
    // Full chunk, aligned: the raw 16-byte loads of PF joints in flight (a ring of register
    // sets refilled PF joints ahead), widened only when their joint is reduced.  One joint
    // ahead left the loads' latency exposed (the volume was just written by the
    // unprojection and streams from HBM): 2.5 TB/s at config 3 in r06.
    constexpr int PF = sizeof(T) == 2 ? 8 : 4;
    uint4 raw[PF][RUNS];
    auto issue = [&](int j, uint4 (&q)[RUNS]) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < RUNS; ++r)
        q[r] = *reinterpret_cast<const uint4*>(vb + j * jstride + i0 + r * kWave * VEC);
    };
#pragma unroll
    for (int p = 0; p < PF; ++p)
      if (ja + p < jb) issue(ja + p, raw[p]);
    for (int j0 = ja; j0 < jb; j0 += PF) {
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const int j = j0 + p;
        if (j >= jb) break;
        float x[RUNS][VEC];
#pragma unroll
        for (int r = 0; r < RUNS; ++r) {
          const uint32_t w[4] = {raw[p][r].x, raw[p][r].y, raw[p][r].z, raw[p][r].w};
          if constexpr (sizeof(T) == 4) {
#pragma unroll
            for (int k = 0; k < 4; ++k) x[r][k] = __uint_as_float(w[k]);
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              x[r][2 * k] = __uint_as_float(w[k] << 16);
              x[r][2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
            }
          }
        }
        if (j + PF < jb) issue(j + PF, raw[p]);
        reduce_joint(j, x);
      }
    }
    return;
  }

  float x[RUNS][VEC];
  load(ja, x);
  for (int j = ja; j < jb; ++j) {
    float xn[RUNS][VEC];
    if (j + 1 < jb) load(j + 1, xn);
    reduce_joint(j, x);
    if (j + 1 < jb) {
#pragma unroll
      for (int r = 0; r < RUNS; ++r)
#pragma unroll
        for (int k = 0; k < VEC; ++k) x[r][k] = xn[r][k];
    }
  }
}

// Pass 2: one wave per (b, j) folds the pass-1 partials, writes the coordinates and the
// (max, 1 / sum) the normalisation pass needs.
template <bool SOFTMAX>
__global__ __launch_bounds__(kSaBlock) void softargmax_combine(const float* __restrict__ part,
                                                              float* __restrict__ xyz, float* __restrict__ stat,
                                                              int BJ, int npart) {
  const int bj = blockIdx.x * (kSaBlock / kWave) + threadIdx.x / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  if (bj >= BJ) return;
  const float* pj = part + size_t(bj) * npart * kPartial;
  float m = SOFTMAX ? -INFINITY : 0.f, s = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
  for (int k = lane; k < npart; k += kWave) {
    const float* q = pj + size_t(k) * kPartial;
    merge<SOFTMAX>(m, s, sx, sy, sz, q[0], q[1], q[2], q[3], q[4]);
  }
  wave_merge<SOFTMAX>(m, s, sx, sy, sz);
  if (lane == 0) {
    float* o = xyz + size_t(bj) * 3;
    if constexpr (SOFTMAX) {
      o[0] = sx / s; o[1] = sy / s; o[2] = sz / s;      // op.py:94 on the normalised volume
    } else {
      o[0] = sx; o[1] = sy; o[2] = sz;                  // relu: no mass normalisation (op.py:91)
    }
    stat[size_t(bj) * 2] = m;
    stat[size_t(bj) * 2 + 1] = 1.f / s;
  }
}

// Pass 3: stream the normalised volume, exp(mult * x - max) / sum (or relu(mult * x)).
template <typename T, typename TO, bool SOFTMAX>
__global__ __launch_bounds__(kSaBlock) void softargmax_finalize(
    const T* __restrict__ vol, long long bstride, long long jstride, float mult,
    const float* __restrict__ stat, TO* __restrict__ out, int J, int nvox, bool vec_ok) {
  constexpr int VEC = Vec<T>::n;
  constexpr int RUNS = kSaVpt / VEC;
  const int chunk = blockIdx.x, j = blockIdx.y, b = blockIdx.z;
  const int tid = threadIdx.x;
  const float m = stat[(size_t(b) * J + j) * 2], inv = stat[(size_t(b) * J + j) * 2 + 1];
  const T* vj = vol + b * bstride + j * jstride;
  TO* oj = out + (size_t(b) * J + j) * nvox;
  float t[RUNS][VEC];
#pragma unroll
  for (int r = 0; r < RUNS; ++r)
    load_run<T, VEC, kFinalNtLoads>(vj, chunk * kSaChunk + r * kSaBlock * VEC + tid * VEC, nvox, vec_ok, t[r], 0.f);
#pragma unroll
  for (int r = 0; r < RUNS; ++r) {
    const int i = chunk * kSaChunk + r * kSaBlock * VEC + tid * VEC;
    float y[VEC];
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const float v = t[r][k] * mult;
      y[k] = SOFTMAX ? __expf(v - m) * inv : fmaxf(v, 0.f);
    }
    if constexpr (sizeof(TO) == sizeof(T)) {
      store_run<TO, VEC, kFinalNtStores>(oj, i, nvox, vec_ok, y);
    } else {  // bf16 in -> f32 out: two float4 runs
      float lo[4] = {y[0], y[1], y[2], y[3]};
      store_run<TO, 4, kFinalNtStores>(oj, i, nvox, vec_ok, lo);
      if constexpr (VEC == 8) {
        float hi[4] = {y[4], y[5], y[6], y[7]};
        store_run<TO, 4, kFinalNtStores>(oj, i + 4, nvox, vec_ok, hi);
      }
    }
  }
}

template <typename T, typename TO, bool SOFTMAX>
int launch3(const void* vol, long long bs, long long js, const float* coords, const float* cub, int V, int transfer,
            float mult, float* xyz, void* out, float* part, int B, int J, int nvox, hipStream_t st);

// Test hook (mvn_debug_set_softargmax): 1 = force the three-launch path.
std::atomic<int> g_sa_force3{0};
inline bool single_pass_enabled() { return g_sa_force3.load(std::memory_order_relaxed) != 1; }
inline int single_dbg() { return g_sa_force3.load(std::memory_order_relaxed); }

// ---- single pass (round 3): the volume is read once --------------------------------------
// The three launches above read the volume twice (pass 1, then the finalize); the second read
// misses the MALL at config 3 (285 MB of bf16 volume).  softargmax_single keeps a block's
// values ON CHIP between its reduction and its normalised write: a block owns a unit =
// (frame, 1024-voxel chunk) for every joint (4 voxels x J joints per thread, in registers),
// publishes the unit's 5-float partial per joint, and the frame's LAST arriving block folds
// all of the frame's partials (the combine of pass 2, same order) into (max, 1/sum) and the
// coordinates; the frame's other blocks wait for that, then normalise their registers.
// HBM traffic: volume read once, normalised volume written once, coordinates read once —
// the algorithmic bytes of op.py:84-96.
//
// Inter-block protocol (cdna_hip_programming.md §6 Guideline 16: agent-scope release /
// acquire, no assumption on dispatch order or placement):
//   * units are handed out by an ORDERED ticket counter, so a block waits only on a frame
//     all of whose units have been taken by running blocks: with R resident blocks and
//     units per frame <= R / 2 (each block holds at most a current and a next ticket) the
//     lowest unfinished frame always completes — no deadlock whatever the residency;
//   * partials: plain stores, every storing wave s_waitcnt vmcnt(0), release fence (agent),
//     then the frame's arrival counter (atomic add, agent scope);
//   * the last arriver: acquire fence, folds the partials, stores stat / xyz, release fence,
//     flag store (atomic, agent scope); the others poll the flag relaxed (s_sleep), then one
//     acquire fence;
//   * control words (ticket, arrivals, flags) at the start of the workspace, zeroed by a
//     hipMemsetAsync before every launch (Guideline 16: "re-initialise every call").
constexpr int kSpChunk = 1024;                  // voxels per unit: the workspace's partial count
constexpr int kSpVpt = kSpChunk / kSaBlock;     // 4 voxels per thread
static_assert(kSpChunk == kPartChunkMin, "single-pass units are the workspace's partial chunks");
template <typename T> struct Raw4;              // 4 voxels of one joint as loaded
typedef unsigned u2v __attribute__((ext_vector_type(2)));
template <> struct Raw4<float> { using type = u4v; };
template <> struct Raw4<uint16_t> { using type = u2v; };
__device__ __forceinline__ void widen4(const u4v& q, float (&x)[4]) {
  x[0] = __uint_as_float(q.x); x[1] = __uint_as_float(q.y); x[2] = __uint_as_float(q.z); x[3] = __uint_as_float(q.w);
}
__device__ __forceinline__ void widen4(const u2v& q, float (&x)[4]) {
  x[0] = __uint_as_float(q.x << 16); x[1] = __uint_as_float(q.x & 0xffff0000u);
  x[2] = __uint_as_float(q.y << 16); x[3] = __uint_as_float(q.y & 0xffff0000u);
}
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) float gf32;
constexpr int kSpSpinLimit = 1 << 22;           // bounded poll (~1 s): a broken protocol cannot hang the GPU

// Control words (hierarchical, so that no word takes more than kSpGroup + 1 arrivals or
// pollers: same-address agent-scope atomics serialise at the memory side):
//   [0] ticket; then per frame b: top[b] (arrivals of finished groups), sub[b][g] (arrivals in
//   group g = chunk / kSpGroup), flag[b][g] (set by the frame's last arriver, polled by group g)
constexpr int kSpGroup = 16;
__host__ __device__ constexpr int sp_groups(int nchunk) { return (nchunk + kSpGroup - 1) / kSpGroup; }
__host__ __device__ constexpr size_t sp_ctrl_bytes(int B, int nchunk) {
  return (size_t(4 + B * (1 + 2 * sp_groups(nchunk))) * 4 + 15) / 16 * 16;
}

template <typename T, typename TO, bool SOFTMAX, int JM>
__global__ __launch_bounds__(kSaBlock) void softargmax_single(
    const T* __restrict__ vol, long long bstride, long long jstride, const float* __restrict__ coords,
    const float* __restrict__ cub, int V, int transfer, float mult, float* __restrict__ xyz, TO* __restrict__ out,
    float* part, float* stat, unsigned* ctrl, int B, int J, int nvox, int nchunk, int dbg) {
  using Raw = typename Raw4<T>::type;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  constexpr int kWaves = kSaBlock / kWave;
  const unsigned total = unsigned(B) * unsigned(nchunk);
  gu32* ticket = (gu32*)(ctrl);
  const int ng = sp_groups(nchunk);
  gu32* top = (gu32*)(ctrl + 4);
  gu32* sub = top + B;
  gu32* flag = sub + size_t(B) * ng;

  __shared__ float s_part[kWaves][JM][kPartial];
  __shared__ float s_stat[JM][2];
  __shared__ float s_comb[JM][kSaBlock / 16][kPartial];   // combine: J * (256 / J) <= 256 sub-results
  __shared__ unsigned s_unit, s_last;

  if (t == 0) s_unit = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  unsigned unit = s_unit;
  while (unit < total) {
    const int b = int(unit / unsigned(nchunk)), chunk = int(unit % unsigned(nchunk));
    const int i = chunk * kSpChunk + t * kSpVpt;
    const bool in = i < nvox;                      // nvox % 8 == 0: a thread's 4 voxels are all in or all out
    const T* vb = vol + b * bstride + i;
    Raw raw[JM];
#pragma unroll
    for (int j = 0; j < JM; ++j)
      if (j < J && in) raw[j] = __builtin_nontemporal_load(reinterpret_cast<const Raw*>(vb + j * jstride));
    float c[3 * kSpVpt];
    if (cub) {
      const float* cf = cub + size_t(b) * MVN_CUBOID_FLOATS;
      int gi = i / (V * V), gj = (i / V) % V, gk = i % V;
#pragma unroll
      for (int u = 0; u < kSpVpt; ++u) {
        float o[3];
        cuboid_coord(cf, V, gi, gj, gk, transfer, o);
        c[3 * u] = in ? o[0] : 0.f; c[3 * u + 1] = in ? o[1] : 0.f; c[3 * u + 2] = in ? o[2] : 0.f;
        if (++gk == V) { gk = 0; if (++gj == V) { gj = 0; ++gi; } }
      }
    } else {
      const float4* cp = reinterpret_cast<const float4*>(coords + (size_t(b) * nvox + (in ? i : 0)) * 3);
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const float4 f = in ? cp[u] : make_float4(0.f, 0.f, 0.f, 0.f);
        c[4 * u] = f.x; c[4 * u + 1] = f.y; c[4 * u + 2] = f.z; c[4 * u + 3] = f.w;
      }
    }
    // the next unit's ticket, fetched now so that its round trip hides behind this unit
    unsigned next = 0;
    if (t == 0) next = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // ---- per-wave partial of every joint (pass 1's formula over the wave's 256 voxels) ----
    const float fill = SOFTMAX ? -INFINITY : 0.f;
#pragma unroll
    for (int j = 0; j < JM; ++j) {
      if (j >= J) continue;         // (not break: the loop must unroll, raw[] stays in registers)
      float x[4];
      if (in) {
        widen4(raw[j], x);
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = x[k] * mult;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = fill;
      }
      float m = 0.f, s = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
      if constexpr (SOFTMAX) {
        constexpr float kLog2e = 1.4426950408889634f;
        const float lm = fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3]));
        m = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(wave_max63(lm)), kWave - 1));
        if (m != -INFINITY) {
          const float ml = m * kLog2e;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(x[k], kLog2e, -ml));
            s += e;
            sx = __builtin_fmaf(e, c[3 * k], sx);
            sy = __builtin_fmaf(e, c[3 * k + 1], sy);
            sz = __builtin_fmaf(e, c[3 * k + 2], sz);
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float e = fmaxf(x[k], 0.f);
          s += e;
          sx = __builtin_fmaf(e, c[3 * k], sx);
          sy = __builtin_fmaf(e, c[3 * k + 1], sy);
          sz = __builtin_fmaf(e, c[3 * k + 2], sz);
        }
      }
      s = wave_sum63(s); sx = wave_sum63(sx); sy = wave_sum63(sy); sz = wave_sum63(sz);
      if (lane == kWave - 1) {
        s_part[wid][j][0] = m; s_part[wid][j][1] = s; s_part[wid][j][2] = sx; s_part[wid][j][3] = sy;
        s_part[wid][j][4] = sz;
      }
    }
    __syncthreads();
    // ---- the unit's partial per joint (waves folded in order), published -------------------
    // Payload stores are write-through (sc1: relaxed agent-scope atomic stores) and drained
    // before the arrival add, so no release fence (Guideline 16 R1; a release fence = an L2
    // write-back, which under this kernel's output stream cost more than the whole pass).
    if (wid == 0) {
      if (lane < J) {
        float m = s_part[0][lane][0], s = s_part[0][lane][1], sx = s_part[0][lane][2], sy = s_part[0][lane][3],
              sz = s_part[0][lane][4];
#pragma unroll
        for (int w = 1; w < kWaves; ++w)
          merge<SOFTMAX>(m, s, sx, sy, sz, s_part[w][lane][0], s_part[w][lane][1], s_part[w][lane][2],
                         s_part[w][lane][3], s_part[w][lane][4]);
        gf32* o = (gf32*)(part) + ((size_t(b) * J + lane) * nchunk + chunk) * kPartial;
        __hip_atomic_store(o, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o + 1, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o + 2, sx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o + 3, sy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o + 4, sz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        // arrival: in the chunk's group; the group's last arriver then counts in the frame's top word
        const int g = chunk / kSpGroup, gsize = min(kSpGroup, nchunk - g * kSpGroup);
        unsigned last = 0u;
        if (dbg != 2 &&
            __hip_atomic_fetch_add(sub + size_t(b) * ng + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                unsigned(gsize - 1))
          last = __hip_atomic_fetch_add(top + b, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == unsigned(ng - 1);
        s_last = last;
        s_unit = next;
      }
    }
    __syncthreads();
    if (s_last) {
      // ---- last arriver of the frame: fold the frame's partials --------------------------
      // P = kSaBlock / J threads per joint, thread (j, sub) folds chunks sub, sub + P, ... (all
      // loads of a batch in flight), then lane j of wave 0 folds the P sub-results in order:
      // one load round trip instead of one per chunk.
      if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      const int P = min(kSaBlock / J, kSaBlock / 16), j = t / P, sub = t - j * P;
      if (j < J) {
        const float* pj = part + (size_t(b) * J + j) * nchunk * kPartial;
        float m = SOFTMAX ? -INFINITY : 0.f, s = 0.f, sx = 0.f, sy = 0.f, sz = 0.f;
        constexpr int kBatch = 4;
        for (int k0 = sub; k0 < nchunk; k0 += kBatch * P) {
          float q[kBatch][kPartial];
#pragma unroll
          for (int u = 0; u < kBatch; ++u) {
            const int k = k0 + u * P;
#pragma unroll
            for (int f = 0; f < kPartial; ++f)
              q[u][f] = k < nchunk ? pj[size_t(k) * kPartial + f] : (f == 0 && SOFTMAX ? -INFINITY : 0.f);
          }
#pragma unroll
          for (int u = 0; u < kBatch; ++u) merge<SOFTMAX>(m, s, sx, sy, sz, q[u][0], q[u][1], q[u][2], q[u][3], q[u][4]);
        }
        s_comb[j][sub][0] = m; s_comb[j][sub][1] = s; s_comb[j][sub][2] = sx; s_comb[j][sub][3] = sy;
        s_comb[j][sub][4] = sz;
      }
      __syncthreads();
      if (wid == 0) {
        if (lane < J) {
          float m = s_comb[lane][0][0], s = s_comb[lane][0][1], sx = s_comb[lane][0][2], sy = s_comb[lane][0][3],
                sz = s_comb[lane][0][4];
          for (int u = 1; u < P; ++u)
            merge<SOFTMAX>(m, s, sx, sy, sz, s_comb[lane][u][0], s_comb[lane][u][1], s_comb[lane][u][2],
                           s_comb[lane][u][3], s_comb[lane][u][4]);
          float* o = xyz + (size_t(b) * J + lane) * 3;
          if constexpr (SOFTMAX) {
            o[0] = sx / s; o[1] = sy / s; o[2] = sz / s;      // op.py:94 on the normalised volume
          } else {
            o[0] = sx; o[1] = sy; o[2] = sz;                  // relu: no mass normalisation (op.py:91)
          }
          const float inv = 1.f / s;
          gf32* sp = (gf32*)(stat) + (size_t(b) * J + lane) * 2;
          __hip_atomic_store(sp, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(sp + 1, inv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_stat[lane][0] = m;
          s_stat[lane][1] = inv;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the storing wave drains, then flags
        for (int g = lane; g < ng; g += kWave)
          __hip_atomic_store(flag + size_t(b) * ng + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      // ---- the others: poll the frame's flag (one lane, relaxed, s_sleep), then read the
      // stat with sc1 loads (atomic, agent scope: not served by this CU's L1) ------------
      if (wid == 0) {
        if (lane == 0 && dbg < 2) {
          for (int spins = 0; spins < kSpSpinLimit; ++spins) {
            if (__hip_atomic_load(flag + size_t(b) * ng + chunk / kSpGroup, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT) != 0u)
              break;
            __builtin_amdgcn_s_sleep(2);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < J) {
          gf32* sp = (gf32*)(stat) + (size_t(b) * J + lane) * 2;
          s_stat[lane][0] = __hip_atomic_load(sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_stat[lane][1] = __hip_atomic_load(sp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __syncthreads();
    // ---- normalised volume from the registers (the finalize's formula) -------------------
    if (out != nullptr && in) {
      TO* ob = out + size_t(b) * J * nvox + i;
#pragma unroll
      for (int j = 0; j < JM; ++j) {
        if (j >= J) continue;
        float x[4], y[4];
        widen4(raw[j], x);
        const float m = s_stat[j][0], inv = s_stat[j][1];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float v = x[k] * mult;
          y[k] = SOFTMAX ? __expf(v - m) * inv : fmaxf(v, 0.f);
        }
        TO* oj = ob + size_t(j) * nvox;
        if constexpr (sizeof(TO) == 4) {
          __builtin_nontemporal_store(f4v{y[0], y[1], y[2], y[3]}, reinterpret_cast<f4v*>(oj));
        } else {
          __builtin_nontemporal_store(u2v{pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3])},
                                      reinterpret_cast<u2v*>(oj));
        }
      }
    }
    unit = s_unit;
    __syncthreads();      // s_unit / s_stat / s_part are rewritten by the next unit
  }
}

// Resident blocks of a single-pass instantiation on one CU (one below the occupancy API's
// answer: it can be one high, MI355X_MICROARCH.md 'Correctness boundaries').
template <typename T, typename TO, bool SOFTMAX, int JM>
int single_blocks_per_cu() {
  static const int n = [] {
    int k = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&k, softargmax_single<T, TO, SOFTMAX, JM>, kSaBlock, 0) !=
        hipSuccess)
      return 0;
    return k > 1 ? k - 1 : k;
  }();
  return n;
}

// 1 = the single pass does not apply (the caller runs the three launches), else MVN_OK / error.
template <typename T, typename TO, bool SOFTMAX, int JM>
int launch_single(const void* vol, long long bs, long long js, const float* coords, const float* cub, int V,
                  int transfer, float mult, float* xyz, void* out, void* ws, int B, int J, int nvox, hipStream_t st) {
  const int nchunk = (nvox + kSpChunk - 1) / kSpChunk;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 1;
  const long long resident = (long long)single_blocks_per_cu<T, TO, SOFTMAX, JM>() * cus;
  if (resident < 2LL * nchunk) return 1;            // the no-deadlock condition above, with margin
  unsigned* ctrl = static_cast<unsigned*>(ws);
  float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + sp_ctrl_bytes(B, nchunk));
  float* stat = part + size_t(B) * J * nchunk * kPartial;
  if (hipMemsetAsync(ctrl, 0, sp_ctrl_bytes(B, nchunk), st) != hipSuccess) return MVN_ERR_LAUNCH;
  const long long units = (long long)B * nchunk;
  const int grid = int(units < resident ? units : resident);
  softargmax_single<T, TO, SOFTMAX, JM><<<grid, kSaBlock, 0, st>>>(
      static_cast<const T*>(vol), bs, js, coords, cub, V, transfer, mult, xyz, static_cast<TO*>(out), part, stat,
      ctrl, B, J, nvox, nchunk, single_dbg());
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

template <typename T, typename TO, bool SOFTMAX>
int launch(const void* vol, long long bs, long long js, const float* coords, const float* cub, int V, int transfer,
           float mult, float* xyz, void* out, void* ws, int B, int J, int nvox, hipStream_t st) {
  const bool aligned = (reinterpret_cast<uintptr_t>(vol) % 16 == 0) && (bs * sizeof(T)) % 16 == 0 &&
                       (js * sizeof(T)) % 16 == 0 && (nvox % 8 == 0) &&
                       (out == nullptr || reinterpret_cast<uintptr_t>(out) % 16 == 0) &&
                       (cub != nullptr || reinterpret_cast<uintptr_t>(coords) % 16 == 0);
  if (aligned && single_pass_enabled() && (long long)B * ((nvox + kSpChunk - 1) / kSpChunk) < (1LL << 31)) {
    int r = 1;
    if (J <= 17)
      r = launch_single<T, TO, SOFTMAX, 17>(vol, bs, js, coords, cub, V, transfer, mult, xyz, out, ws, B, J, nvox, st);
    else if (J <= 24)
      r = launch_single<T, TO, SOFTMAX, 24>(vol, bs, js, coords, cub, V, transfer, mult, xyz, out, ws, B, J, nvox, st);
    if (r != 1) return r;
  }
  float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + sp_ctrl_bytes(B, (nvox + kSpChunk - 1) / kSpChunk));
  return launch3<T, TO, SOFTMAX>(vol, bs, js, coords, cub, V, transfer, mult, xyz, out, part, B, J, nvox, st);
}

template <typename T, typename TO, bool SOFTMAX>
int launch3(const void* vol, long long bs, long long js, const float* coords, const float* cub, int V, int transfer,
            float mult, float* xyz, void* out, float* part, int B, int J, int nvox, hipStream_t st) {
  const int nchunk = (nvox + kSaChunk - 1) / kSaChunk;       // pass-2 blocks per (b, j)
  const int npart = (nvox + kPartChunkT<T> - 1) / kPartChunkT<T>;   // pass-1 partials per (b, j)
  const bool vec_ok = (reinterpret_cast<uintptr_t>(vol) % 16 == 0) && (bs * sizeof(T)) % 16 == 0 &&
                      (js * sizeof(T)) % 16 == 0 && (nvox % 8 == 0) &&
                      (out == nullptr || reinterpret_cast<uintptr_t>(out) % 16 == 0);
  // pass 1 takes every joint in one wave per chunk (gridDim.z = 1; splitting the joints over
  // gridDim.z at small batches was measured and gave nothing, r14)
  const int nsplit = 1;
  softargmax_partials<T, SOFTMAX><<<dim3((npart + kSaBlock / kWave - 1) / (kSaBlock / kWave), B, nsplit), kSaBlock, 0, st>>>(
      static_cast<const T*>(vol), bs, js, coords, cub, V, transfer, mult, part, J, nvox, npart, vec_ok);
  if (!launch_ok()) return MVN_ERR_LAUNCH;
  float* stat = part + size_t(B) * J * npart * kPartial;
  softargmax_combine<SOFTMAX><<<(B * J + kSaBlock / kWave - 1) / (kSaBlock / kWave), kSaBlock, 0, st>>>(
      part, xyz, stat, B * J, npart);
  if (!launch_ok()) return MVN_ERR_LAUNCH;
  if (out == nullptr) return MVN_OK;
  softargmax_finalize<T, TO, SOFTMAX><<<dim3(nchunk, J, B), kSaBlock, 0, st>>>(
      static_cast<const T*>(vol), bs, js, mult, stat, static_cast<TO*>(out), J, nvox, vec_ok);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

template <typename T, typename TO>
int launch_mode(int softmax, const void* vol, long long bs, long long js, const float* coords, const float* cub,
                int V, int transfer, float mult, float* xyz, void* out, void* ws, int B, int J, int nvox,
                hipStream_t st) {
  return softmax ? launch<T, TO, true>(vol, bs, js, coords, cub, V, transfer, mult, xyz, out, ws, B, J, nvox, st)
                 : launch<T, TO, false>(vol, bs, js, coords, cub, V, transfer, mult, xyz, out, ws, B, J, nvox, st);
}

int softargmax_entry(const void* vol, int vol_dtype, int64_t vol_bstride, int64_t vol_jstride, const float* coords,
                     const float* cub, int transfer, float multiplier, int softmax, float* out_xyz, void* out_vol,
                     int out_dtype, void* workspace, size_t workspace_bytes, int B, int J, int Vx, int Vy, int Vz,
                     void* stream);

}  // namespace
}  // namespace mvn

extern "C" size_t mvn_softargmax3d_workspace_bytes(int B, int J, int Vx, int Vy, int Vz) {
  if (B <= 0 || J <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0) return 0;
  const long long nvox = (long long)Vx * Vy * Vz;
  const long long npart = (nvox + mvn::kPartChunkMin - 1) / mvn::kPartChunkMin;
  // single-pass control words + partials + (max, 1/sum)
  return mvn::sp_ctrl_bytes(B, int(npart)) + size_t(B) * J * (npart * mvn::kPartial + 2) * sizeof(float);
}

namespace mvn {
namespace {
int softargmax_entry(const void* vol, int vol_dtype, int64_t vol_bstride, int64_t vol_jstride, const float* coords,
                     const float* cub, int transfer, float multiplier, int softmax, float* out_xyz, void* out_vol,
                     int out_dtype, void* workspace, size_t workspace_bytes, int B, int J, int Vx, int Vy, int Vz,
                     void* stream) {
  if (!vol || !(coords || cub) || !out_xyz) return MVN_ERR_ARG;
  if (softmax != 0 && softmax != 1) return MVN_ERR_ARG;
  if (transfer != 0 && transfer != 1) return MVN_ERR_ARG;
  if (B <= 0 || J <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0 || B > 65535 || J > 65535) return MVN_ERR_SHAPE;
  const long long nvox = (long long)Vx * Vy * Vz;
  if (nvox > (1LL << 30)) return MVN_ERR_SHAPE;
  if (vol_bstride < 0 || vol_jstride < 0) return MVN_ERR_SHAPE;
  const size_t need = mvn_softargmax3d_workspace_bytes(B, J, Vx, Vy, Vz);
  if (!workspace || workspace_bytes < need) return MVN_ERR_WORKSPACE;
  void* part = workspace;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int n = int(nvox);
  if (vol_dtype == MVN_DTYPE_F32 && out_dtype == MVN_DTYPE_F32)
    return launch_mode<float, float>(softmax, vol, vol_bstride, vol_jstride, coords, cub, Vx, transfer, multiplier, out_xyz, out_vol, part, B, J, n, st);
  if (vol_dtype == MVN_DTYPE_BF16 && out_dtype == MVN_DTYPE_BF16)
    return launch_mode<uint16_t, uint16_t>(softmax, vol, vol_bstride, vol_jstride, coords, cub, Vx, transfer, multiplier, out_xyz, out_vol, part, B, J, n, st);
  if (vol_dtype == MVN_DTYPE_BF16 && out_dtype == MVN_DTYPE_F32)
    return launch_mode<uint16_t, float>(softmax, vol, vol_bstride, vol_jstride, coords, cub, Vx, transfer, multiplier, out_xyz, out_vol, part, B, J, n, st);
  return MVN_ERR_DTYPE;
}
}  // namespace
}  // namespace mvn

extern "C" int mvn_softargmax3d(const void* vol, int vol_dtype, int64_t vol_bstride, int64_t vol_jstride,
                                const float* coords, float multiplier, int softmax, float* out_xyz,
                                void* out_vol, int out_dtype, void* workspace, size_t workspace_bytes,
                                int B, int J, int Vx, int Vy, int Vz, void* stream) {
  if (!coords) return MVN_ERR_ARG;
  return mvn::softargmax_entry(vol, vol_dtype, vol_bstride, vol_jstride, coords, nullptr, 0, multiplier, softmax,
                               out_xyz, out_vol, out_dtype, workspace, workspace_bytes, B, J, Vx, Vy, Vz, stream);
}

extern "C" int mvn_debug_set_softargmax(int three_pass) {
  if (three_pass < 0 || three_pass > 3) return MVN_ERR_ARG;
  mvn::g_sa_force3.store(three_pass, std::memory_order_relaxed);
  return MVN_OK;
}

extern "C" int mvn_softargmax3d_cuboid(const void* vol, int vol_dtype, int64_t vol_bstride, int64_t vol_jstride,
                                       const float* cuboids, int transfer_cmu, float multiplier, int softmax,
                                       float* out_xyz, void* out_vol, int out_dtype, void* workspace,
                                       size_t workspace_bytes, int B, int J, int V, void* stream) {
  if (!cuboids) return MVN_ERR_ARG;
  return mvn::softargmax_entry(vol, vol_dtype, vol_bstride, vol_jstride, nullptr, cuboids, transfer_cmu, multiplier,
                               softmax, out_xyz, out_vol, out_dtype, workspace, workspace_bytes, B, J, V, V, V,
                               stream);
}
