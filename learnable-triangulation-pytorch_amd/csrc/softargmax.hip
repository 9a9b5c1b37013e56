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
// (the max written as DPP-fused v_max_f32 with dst == src1: a lane without a source is
// disabled and keeps its value; through fmaxf every DPP result was canonicalised first)
__device__ __forceinline__ float wave_max63(float v) {
  asm("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
      "s_nop 1"
      : "+v"(v));
  return v;
}
__device__ __forceinline__ float wave_sum63(float v) {
  v += dpp_f<0x111, 0xf>(v, 0.f); v += dpp_f<0x112, 0xf>(v, 0.f);
  v += dpp_f<0x114, 0xf>(v, 0.f); v += dpp_f<0x118, 0xf>(v, 0.f);
  v += dpp_f<0x142, 0xa>(v, 0.f); v += dpp_f<0x143, 0xc>(v, 0.f);
  return v;
}

// Max of a lane's values as a tree of three-operand maxima: 8 v_max3_f32 for 16 values.
// (fmaxf on the raw loaded values would first canonicalise each input — one more v_max per
// value in IEEE mode — so the instruction is written out.)  NaN: v_max3_f32 / the DPP v_max
// return the other operand for a quiet NaN, so the max of a chunk with some NaN voxels is
// the max of the rest, and the max of an all-NaN chunk (or a signalling NaN) is NaN.  Either
// way the NaN voxel's exponential is NaN, so the joint's sums, coordinates and normalised
// volume are NaN — torch's softmax over a volume holding a NaN (op.py:89) is NaN everywhere
// (tests/test_gpu_parity.py::test_softargmax_nan_volume_follows_torch).
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// level by level: groups of three, a leftover pair or single carried up
template <int N>
__device__ __forceinline__ float max_level(const float* v) {
  if constexpr (N == 1) {
    return v[0];
  } else {
    constexpr int M = (N + 2) / 3;
    float w[M];
#pragma unroll
    for (int i = 0; i < N / 3; ++i) w[i] = vmax3(v[3 * i], v[3 * i + 1], v[3 * i + 2]);
    if constexpr (N % 3 == 2) w[M - 1] = vmax3(v[N - 2], v[N - 1], v[N - 1]);
    if constexpr (N % 3 == 1) w[M - 1] = v[N - 1];
    return max_level<M>(w);
  }
}
template <int R, int V>
__device__ __forceinline__ float max_tree(const float (&x)[R][V]) {
  return max_level<R * V>(&x[0][0]);
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
  // frames in DESCENDING order: the unprojection just wrote (and read the coordinates of) the
  // last frames, which the 256 MiB MALL still holds; pass 1 then leaves the first frames there
  // for the finalize, which walks them in ascending order (config 3 soft-argmax 182.9 -> 169.6 us
  // inside the bench step, bit-identical; profiles/r17_ab_sa_rev.txt)
  const int chunk = blockIdx.x * (kSaBlock / kWave) + wid, b = int(gridDim.y) - 1 - int(blockIdx.y);
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
      // x * 1 == x: the reference's models use volume_multiplier 1.0 (a scalar branch)
      if (mult != 1.f) {
#pragma unroll
        for (int r = 0; r < RUNS; ++r)
#pragma unroll
          for (int k = 0; k < VEC; ++k) x[r][k] = x[r][k] * mult;
      }
      const float lm = max_tree(x);
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
      MVN_DASSERT(j < J && chunk < nchunk);
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
        MVN_DASSERT(jbase + lane < J && chunk < nchunk);
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
  // the lane's partials k = lane, lane + 64, ... merged in that order; CK of them loaded at once
  // (one wave per (b, j): a latency-bound kernel, the loads of a dependent loop went out one
  // partial at a time — 4.8 us per launch at config 2)
  constexpr int CK = 4;
  int k = lane;
  for (; k + (CK - 1) * kWave < npart; k += CK * kWave) {
    float q[CK][kPartial];
#pragma unroll
    for (int i = 0; i < CK; ++i)
#pragma unroll
      for (int c = 0; c < kPartial; ++c) q[i][c] = pj[size_t(k + i * kWave) * kPartial + c];
#pragma unroll
    for (int i = 0; i < CK; ++i) merge<SOFTMAX>(m, s, sx, sy, sz, q[i][0], q[i][1], q[i][2], q[i][3], q[i][4]);
  }
  for (; k < npart; k += kWave) {
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
int launch(const void* vol, long long bs, long long js, const float* coords, const float* cub, int V, int transfer,
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
                int V, int transfer, float mult, float* xyz, void* out, float* part, int B, int J, int nvox,
                hipStream_t st) {
  return softmax ? launch<T, TO, true>(vol, bs, js, coords, cub, V, transfer, mult, xyz, out, part, B, J, nvox, st)
                 : launch<T, TO, false>(vol, bs, js, coords, cub, V, transfer, mult, xyz, out, part, B, J, nvox, st);
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
  return size_t(B) * J * (npart * mvn::kPartial + 2) * sizeof(float);   // partials + (max, 1/sum)
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
  float* part = static_cast<float*>(workspace);
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

extern "C" int mvn_softargmax3d_cuboid(const void* vol, int vol_dtype, int64_t vol_bstride, int64_t vol_jstride,
                                       const float* cuboids, int transfer_cmu, float multiplier, int softmax,
                                       float* out_xyz, void* out_vol, int out_dtype, void* workspace,
                                       size_t workspace_bytes, int B, int J, int V, void* stream) {
  if (!cuboids) return MVN_ERR_ARG;
  return mvn::softargmax_entry(vol, vol_dtype, vol_bstride, vol_jstride, nullptr, cuboids, transfer_cmu, multiplier,
                               softmax, out_xyz, out_vol, out_dtype, workspace, workspace_bytes, B, J, V, V, V,
                               stream);
}
