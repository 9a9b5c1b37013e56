// Shared device code of the unprojection kernels (unproject.hip, unproject_tiled.hip).
#pragma once

#include <climits>

#include "common.hpp"

namespace mvn {
namespace unproj {

// ---- the one f32 form of the cross-view softmax (op.py:153-159) ----------------------
// Every unprojection path — the staged LDS paths, the global-gather fallback, the simple
// kernels and the backward — evaluates it the same way, so a tensor never mixes two
// roundings (which path a tile takes depends on LDS budget and camera distance):
//   m = max_v s_v;  e_v = exp2(fma(s_v, log2 e, -(m * log2 e)));  den = ((e_0 + e_1) + ...);
//   value = fma chain of s_v * e_v, times rcp(den).   (<= 1e-5 of the reference's softmax)
constexpr float kLog2e = 1.4426950408889634f;
__device__ __forceinline__ float softmax_exp(float s, float ml) {   // ml = m * kLog2e
  return __builtin_amdgcn_exp2f(__builtin_fmaf(s, kLog2e, -ml));
}

// 'max' aggregation in torch.max(dim)'s order (ATen greater_or_nan): NaN above every number
// (the first NaN wins), otherwise the larger value, ties to the first view.
__device__ __forceinline__ bool max_takes(float s, float r) { return s > r || (s != s && r == r); }

// Bilinear taps of one voxel in one view: 4 clamped plane offsets + 4 weights + the mask
// of corners inside the image.  Out-of-bounds corners read the value 0 (grid_sample's
// padding_mode='zeros': the corner VALUE is zero, so its product is +0 whatever the sign
// of the clamped pixel) and, like every corner of an invalid (behind-camera) voxel, carry
// weight 0 (0 * 0: no NaN from the weights of far-off or non-finite coordinates).
struct Taps {
  int o0, o1, o2, o3;
  float w0, w1, w2, w3;
  unsigned in;        // bit k: corner k (nw, ne, sw, se) inside the image, voxel valid
};

// Continuous grid_sample pixel coordinate of one voxel in one view, plus the depth mask.
struct Proj {
  float ix, iy;      // x indexes W, y indexes H
  bool invalid;      // depth <= 0 (op.py:121)
};

__device__ __forceinline__ Proj project(const float* __restrict__ Pv, float x, float y, float z, int H, int W,
                                        int align_corners) {
  // op.py:117-119 -> multiview.py:96   [x y z 1] @ P^T
  const float uh = __builtin_fmaf(1.f, Pv[3], __builtin_fmaf(z, Pv[2], __builtin_fmaf(y, Pv[1], x * Pv[0])));
  const float vh = __builtin_fmaf(1.f, Pv[7], __builtin_fmaf(z, Pv[6], __builtin_fmaf(y, Pv[5], x * Pv[4])));
  float wh = __builtin_fmaf(1.f, Pv[11], __builtin_fmaf(z, Pv[10], __builtin_fmaf(y, Pv[9], x * Pv[8])));
  Proj p;
  p.invalid = wh <= 0.f;                   // op.py:121, taken before the guard
  if (wh == 0.f) wh = 1.f;                 // op.py:123
  const float u = uh / wh;                 // multiview.py:75 (IEEE division)
  const float v = vh / wh;
  // op.py:128-129 — x is divided by heatmap_shape[0] (H) and y by [1] (W): reference quirk kept.
  const float gx = 2.f * (u / float(H) - 0.5f);
  const float gy = 2.f * (v / float(W) - 0.5f);
  // grid_sample unnormalisation
  if (align_corners) {
    p.ix = (gx + 1.f) * (float(W - 1) * 0.5f);
    p.iy = (gy + 1.f) * (float(H - 1) * 0.5f);
  } else {
    // ATen: (g + 1) * (size / 2) - 0.5, contracted to one fma
    p.ix = __builtin_fmaf(gx + 1.f, float(W) * 0.5f, -0.5f);
    p.iy = __builtin_fmaf(gy + 1.f, float(H) * 0.5f, -0.5f);
  }
  return p;
}

// ---- projection with a cheaper exact division (the tiled kernel's prologue) --------
// f32 '/' is compiled to v_div_scale x2, v_rcp, 5 fma/mul, v_div_fmas, v_div_fixup.  When
// no range scaling is needed (v_div_scale leaves both operands alone and VCC clear),
// v_div_fmas is a plain fma and v_div_fixup returns its input for finite normal results,
// so the remaining refinement chain below is bit-identical to '/'.  div_core_safe()
// bounds the operands so that this holds (|d| in [2^-30, 2^30], |n| <= 2^60: exponent
// difference < 96, no denormal reciprocal; a tiny |n| can only yield a tiny quotient,
// which the following `2 * (q / size - 0.5)` absorbs identically in both forms).
struct Recip {
  float d, r;   // denominator and its once-refined reciprocal (the compiler's fma0/fma1)
};
__device__ __forceinline__ Recip recip_refined(float d) {
  const float r0 = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r0, 1.f);
  return Recip{d, __builtin_fmaf(e, r0, r0)};
}
__device__ __forceinline__ float div_core(float n, Recip q) {
  const float q0 = n * q.r;
  const float t0 = __builtin_fmaf(-q.d, q0, n);
  const float q1 = __builtin_fmaf(t0, q.r, q0);
  const float t1 = __builtin_fmaf(-q.d, q1, n);
  return __builtin_fmaf(t1, q.r, q1);
}

struct Homog {
  float uh, vh, wh;   // [x y z 1] @ P^T (op.py:117-119 -> multiview.py:96)
};
__device__ __forceinline__ Homog homog(const float* __restrict__ Pv, float x, float y, float z) {
  Homog h;
  h.uh = __builtin_fmaf(1.f, Pv[3], __builtin_fmaf(z, Pv[2], __builtin_fmaf(y, Pv[1], x * Pv[0])));
  h.vh = __builtin_fmaf(1.f, Pv[7], __builtin_fmaf(z, Pv[6], __builtin_fmaf(y, Pv[5], x * Pv[4])));
  h.wh = __builtin_fmaf(1.f, Pv[11], __builtin_fmaf(z, Pv[10], __builtin_fmaf(y, Pv[9], x * Pv[8])));
  return h;
}
__device__ __forceinline__ bool div_core_safe(const Homog& h) {
  const float aw = fabsf(h.wh == 0.f ? 1.f : h.wh);
  return aw >= 0x1p-30f && aw <= 0x1p30f && fabsf(h.uh) <= 0x1p60f && fabsf(h.vh) <= 0x1p60f;
}
// project() from a homogeneous point; FAST: div_core (caller checked div_core_safe on the
// whole wave), else IEEE '/'.  Same op order as project().
template <bool FAST>
__device__ __forceinline__ Proj project_h(const Homog& hp, int H, int W, int align_corners, Recip rH, Recip rW) {
  Proj p;
  p.invalid = hp.wh <= 0.f;                // op.py:121
  const float wh = hp.wh == 0.f ? 1.f : hp.wh;
  float gx, gy;
  if constexpr (FAST) {
    const Recip rw = recip_refined(wh);
    gx = 2.f * (div_core(div_core(hp.uh, rw), rH) - 0.5f);
    gy = 2.f * (div_core(div_core(hp.vh, rw), rW) - 0.5f);
  } else {
    gx = 2.f * ((hp.uh / wh) / float(H) - 0.5f);
    gy = 2.f * ((hp.vh / wh) / float(W) - 0.5f);
  }
  if (align_corners) {
    p.ix = (gx + 1.f) * (float(W - 1) * 0.5f);
    p.iy = (gy + 1.f) * (float(H - 1) * 0.5f);
  } else {
    p.ix = __builtin_fmaf(gx + 1.f, float(W) * 0.5f, -0.5f);
    p.iy = __builtin_fmaf(gy + 1.f, float(H) * 0.5f, -0.5f);
  }
  return p;
}

__device__ __forceinline__ Taps view_taps(const float* __restrict__ Pv, float x, float y, float z,
                                          int H, int W, int align_corners) {
  const Proj p = project(Pv, x, y, z, H, W, align_corners);
  const float ix = p.ix, iy = p.iy;
  const bool invalid = p.invalid;
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const float tx = ix - fx0, sx = 1.f - tx;
  const float ty = iy - fy0, sy = 1.f - ty;
  // corner validity in float (robust to huge / non-finite coordinates)
  const bool x0in = (fx0 >= 0.f) & (fx0 < float(W));
  const bool x1in = (fx0 >= -1.f) & (fx0 < float(W - 1));
  const bool y0in = (fy0 >= 0.f) & (fy0 < float(H));
  const bool y1in = (fy0 >= -1.f) & (fy0 < float(H - 1));
  const bool ok = !invalid;
  const int x0 = x0in ? int(fx0) : 0, x1 = x1in ? int(fx0) + 1 : 0;
  const int y0 = y0in ? int(fy0) : 0, y1 = y1in ? int(fy0) + 1 : 0;
  Taps t;
  const bool i0 = ok & y0in & x0in, i1 = ok & y0in & x1in, i2 = ok & y1in & x0in, i3 = ok & y1in & x1in;
  t.o0 = y0 * W + x0;  t.w0 = i0 ? sy * sx : 0.f;   // nw
  t.o1 = y0 * W + x1;  t.w1 = i1 ? sy * tx : 0.f;   // ne
  t.o2 = y1 * W + x0;  t.w2 = i2 ? ty * sx : 0.f;   // sw
  t.o3 = y1 * W + x1;  t.w3 = i3 ? ty * tx : 0.f;   // se
  t.in = (i0 ? 1u : 0u) | (i1 ? 2u : 0u) | (i2 ? 4u : 0u) | (i3 ? 8u : 0u);
  return t;
}

template <typename TIn>
__device__ __forceinline__ float sample(const TIn* __restrict__ plane, const Taps& t) {
  const float a = (t.in & 1u) ? to_f32(plane[t.o0]) : 0.f;
  const float b = (t.in & 2u) ? to_f32(plane[t.o1]) : 0.f;
  const float c = (t.in & 4u) ? to_f32(plane[t.o2]) : 0.f;
  const float d = (t.in & 8u) ? to_f32(plane[t.o3]) : 0.f;
  return __builtin_fmaf(d, t.w3, __builtin_fmaf(c, t.w2, __builtin_fmaf(b, t.w1, a * t.w0)));
}

// View aggregation of one (voxel, channel) from its N per-view samples (op.py:147-161).
// sum / max / conf reduce sequentially over v = 0..N-1 in the reference's f32 op order.
template <int AGG, int NV>
__device__ __forceinline__ float aggregate(const float (&s)[NV], int N, const float* __restrict__ cf, int cstride) {
  float r;
  if constexpr (AGG == MVN_AGG_SUM) {              // op.py:150
    r = s[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) if (v < N) r = r + s[v];
  } else if constexpr (AGG == MVN_AGG_MAX) {       // op.py:152
    r = s[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) if (v < N) r = max_takes(s[v], r) ? s[v] : r;
  } else if constexpr (AGG == MVN_AGG_CONF) {      // op.py:148: product rounded, then summed
    r = s[0] * cf[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) if (v < N) r = r + s[v] * cf[size_t(v) * cstride];
  } else {                                         // op.py:153-159: softmax over the views
    float m = s[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) if (v < N) m = fmaxf(m, s[v]);
    const float ml = m * kLog2e;
    float den = 0.f, num = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (v < N) {
        const float e = softmax_exp(s[v], ml);
        den += e;
        num = __builtin_fmaf(s[v], e, num);
      }
    r = num * __builtin_amdgcn_rcpf(den);
  }
  return r;
}

constexpr uint32_t kOob = 0x80000000u;            // buffer byte offset past any frame

// 16-byte buffer store followed by two wait states.  A VMEM store of more than 8 bytes reads
// its data VGPRs after issue; a VALU write to them in the next cycles (cdna_asm_programming.md
// §4.1 rows 8/9) makes the store write the NEW value.  hipcc left that pair unpadded in the
// bf16 channels-last unprojection (a register copy right after the store: channels 14-15
// nondeterministic, r14; tools/check_store_hazard.py scans the assembly for it), so every
// 16-byte store goes through here.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <int AUX = 0>
__device__ __forceinline__ void store_b128_padded(u32x4_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, AUX);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1");
  __builtin_amdgcn_sched_barrier(0);
}

// Wave-wide integer min / max, returned wave-uniform.  row_shr DPP steps (identity
// shifted in) leave each row's reduction in its lane 15; four readlanes combine the rows.
__device__ __forceinline__ int wave_min_u(int v) {
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x111, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x112, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x114, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x118, 0xf, 0xf, false));
  return min(min(__builtin_amdgcn_readlane(v, 15), __builtin_amdgcn_readlane(v, 31)),
             min(__builtin_amdgcn_readlane(v, 47), __builtin_amdgcn_readlane(v, 63)));
}
__device__ __forceinline__ int wave_max_u(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x111, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x112, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x114, 0xf, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x118, 0xf, 0xf, false));
  return max(max(__builtin_amdgcn_readlane(v, 15), __builtin_amdgcn_readlane(v, 31)),
             max(__builtin_amdgcn_readlane(v, 47), __builtin_amdgcn_readlane(v, 63)));
}

// Buffer descriptor from block-uniform inputs, provably in SGPRs (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(a >> 32));
  void* p = reinterpret_cast<void*>((uint64_t(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, int(__builtin_amdgcn_readfirstlane(bytes)), 0x00020000);
}

// One voxel, all channels, taps gathered from global memory (oversize-footprint fallback).
// Rolled loops and geometry recomputed per (channel, view): slow but register-lean, so
// the staged path's register allocation is unaffected.  Same arithmetic and op order.
template <int AGG, typename TIn, typename TOut>
__device__ __forceinline__ void gather_voxel(const TIn* __restrict__ fb, const float* __restrict__ Pb,
                                             const float* __restrict__ cfb, TOut* __restrict__ ov, int nvox,
                                             int N, int C, int H, int W, float x, float y, float z,
                                             int align_corners) {
  const size_t HW = size_t(H) * W;
#pragma unroll 1
  for (int c = 0; c < C; ++c) {
    float r = 0.f, m = 0.f, den = 0.f;
#pragma unroll 1
    for (int pass = 0; pass < (AGG == MVN_AGG_SOFTMAX ? 2 : 1); ++pass) {
#pragma unroll 1
      for (int v = 0; v < N; ++v) {
        const float sv = sample(fb + (size_t(v) * C + c) * HW, view_taps(Pb + v * 12, x, y, z, H, W, align_corners));
        if constexpr (AGG == MVN_AGG_SUM) {
          r = v == 0 ? sv : r + sv;
        } else if constexpr (AGG == MVN_AGG_MAX) {
          r = (v == 0 || max_takes(sv, r)) ? sv : r;
        } else if constexpr (AGG == MVN_AGG_CONF) {
          const float p = sv * cfb[size_t(v) * C + c];
          r = v == 0 ? p : r + p;
        } else if (pass == 0) {
          m = v == 0 ? sv : fmaxf(m, sv);
        } else {
          const float e = softmax_exp(sv, m * kLog2e);
          den += e;
          r = __builtin_fmaf(sv, e, r);
        }
      }
    }
    if constexpr (AGG == MVN_AGG_SOFTMAX) r = r * __builtin_amdgcn_rcpf(den);
    store_elem(ov + size_t(c) * nvox, r);
  }
}

// Launchers (defined in unproject_tiled.hip); return MVN_OK or an error code.
template <int AGG, typename TIn, typename TOut>
// cub != nullptr: voxel coordinates formed in-kernel from the per-frame cuboids (coords unused;
// Vx = Vy = Vz), see cuboid_coord in common.hpp.
int launch_tiled(const void* feat, const float* P, const float* coords, const float* cub, int transfer,
                 const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                 int align_corners, int out_cl, int fast, hipStream_t s);

// ---- helpers of the chunk-staged kernel (unproject_x4.hip) ------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// Element k of a pair in both lanes.  Kept as a shuffle of the pair, the backend folds it
// into the packed instruction's op_sel / op_sel_hi: the bilinear weights live as (w0, w1),
// (w2, w3) pairs, 2 VGPRs per view-pair of weights instead of a {w, w} copy per weight.
template <int K> __device__ __forceinline__ f2 splat(f2 p) { return __builtin_shufflevector(p, p, K, K); }

template <typename TIn> struct ChunkT;               // 4 pixels of one channel plane
template <> struct ChunkT<float> { using type = uint4; };
template <> struct ChunkT<uint16_t> { using type = uint2; };

template <typename TIn>
__device__ __forceinline__ typename ChunkT<TIn>::type load_chunk(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s);
template <>
__device__ __forceinline__ uint4 load_chunk<float>(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
  const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, v, s, 0);
  return make_uint4(q[0], q[1], q[2], q[3]);
}
template <>
__device__ __forceinline__ uint2 load_chunk<uint16_t>(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
  const auto q = __builtin_amdgcn_raw_buffer_load_b64(r, v, s, 0);
  return make_uint2(q[0], q[1]);
}
// f32 bits of pixel p (0..3) of a chunk
__device__ __forceinline__ uint32_t chunk_px(const uint4& q, int p) {
  return p == 0 ? q.x : p == 1 ? q.y : p == 2 ? q.z : q.w;
}
__device__ __forceinline__ uint32_t chunk_px(const uint2& q, int p) {
  const uint32_t d = p < 2 ? q.x : q.y;
  return (p & 1) ? (d & 0xffff0000u) : (d << 16);      // bf16 -> f32 bits, exact
}

__device__ __forceinline__ f2 lo2(const uint4& q) { return f2{__uint_as_float(q.x), __uint_as_float(q.y)}; }
__device__ __forceinline__ f2 hi2(const uint4& q) { return f2{__uint_as_float(q.z), __uint_as_float(q.w)}; }
// View aggregation of a channel pair (op.py:147-161), lane-wise the op order of
// aggregate<> (sum / max / conf, reference order; softmax, the unified formula).
template <int AGG, int NV>
__device__ __forceinline__ f2 aggregate_pair(const f2 (&s)[NV], const f2 (&cf)[NV]) {
  if constexpr (AGG == MVN_AGG_SUM) {
    f2 r = s[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) r = r + s[v];
    return r;
  } else if constexpr (AGG == MVN_AGG_MAX) {
    f2 r = s[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) {
      r.x = max_takes(s[v].x, r.x) ? s[v].x : r.x;
      r.y = max_takes(s[v].y, r.y) ? s[v].y : r.y;
    }
    return r;
  } else if constexpr (AGG == MVN_AGG_CONF) {
    f2 r = s[0] * cf[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) r = r + s[v] * cf[v];
    return r;
  } else {
    constexpr float kLog2e = 1.4426950408889634f;
    f2 m = s[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) {
      m.x = fmaxf(m.x, s[v].x);
      m.y = fmaxf(m.y, s[v].y);
    }
    const f2 nml = -(m * f2{kLog2e, kLog2e});
    f2 e[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const f2 a = pk_fma(s[v], f2{kLog2e, kLog2e}, nml);
      e[v] = f2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
    }
    // den = ((0 + e0) + e1 + ...), num = fma(s, e, num) from 0: e0 + 0 == e0 and
    // fma(s0, e0, 0) == s0 * e0 exactly, so the first terms start the chains
    f2 den = e[0], num = s[0] * e[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) {
      den = den + e[v];
      num = pk_fma(s[v], e[v], num);
    }
    return num * f2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  }
}

// v_dot2_f32_bf16 with a zero accumulator in its VOP3P form: the builtin selects the VOP2
// v_dot2c (accumulator = destination), which costs a v_mov of 0 per first row (16 per group
// of the fast bf16 kernel).  Non-volatile: the scheduler places it like any VALU op.
__device__ __forceinline__ float dot2_bf16_from0(uint32_t a, uint32_t w) {
  float r;
  asm("v_dot2_f32_bf16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(w));
  return r;
}
// three-operand max / min (v_max3_f32 / v_min3_f32: quiet NaNs dropped, as fmaxf / fminf)
__device__ __forceinline__ float vmax3f(float a, float b, float c) { return __builtin_fmaxf(a, __builtin_fmaxf(b, c)); }
__device__ __forceinline__ float vmin3f(float a, float b, float c) { return __builtin_fminf(a, __builtin_fminf(b, c)); }

// View softmax of a channel pair from log2-scaled samples t_v = s_v * log2(e) (the fast
// unprojection, MVN_PRECISION_FAST): value = ln2 * sum_v t_v 2^t_v / sum_v 2^t_v, which is
// sum_v s_v softmax_v(s).  MAXSUB = false skips the max pass (exact in real arithmetic; the
// caller guards the denominator's range), true is the max-first form the guard falls back to.
// den receives the denominators (of the form used).
template <int NV, bool MAXSUB>
__device__ __forceinline__ f2 softmax_pair_log2(const f2 (&t)[NV], f2& den) {
  constexpr float kLn2 = 0.6931471805599453f;
  f2 nm = f2{0.f, 0.f};
  if constexpr (MAXSUB) {
    f2 m = t[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) {
      m.x = fmaxf(m.x, t[v].x);
      m.y = fmaxf(m.y, t[v].y);
    }
    nm = -m;
  }
  f2 e[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const f2 a = MAXSUB ? t[v] + nm : t[v];
    e[v] = f2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
  }
  den = e[0];
  f2 num = t[0] * e[0];
#pragma unroll
  for (int v = 1; v < NV; ++v) {
    den = den + e[v];
    num = pk_fma(t[v], e[v], num);
  }
  return (num * f2{kLn2, kLn2}) * f2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
}

// Cache policy of the four-view kernel's NCDHW output stores (2 = nt).  f32 planes stream
// out non-temporally so that they do not evict the feature maps the next tiles re-read
// (whole step at config 2: 261.5 -> 257.8 us); 2-byte bf16 stores must not (577 -> 1,664 us).
constexpr int kStorePolicyF32 = 2;     // nt
constexpr int kStorePolicyBf16 = 0;    // default
// POL_F32: the f32 store's cache policy (the non-temporal default suits 64-byte z-runs;
// 32-byte runs, whose lines several blocks complete, merge better through L2 with 0)
template <typename T, int POL_F32 = kStorePolicyF32>
__device__ __forceinline__ void store_plane(float x, __amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
  if constexpr (sizeof(T) == 4)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, v, s, POL_F32);
  else
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, static_cast<__bf16>(x)), r, v, s, kStorePolicyBf16);
}

// Per-view region of the LDS image (block-uniform, SGPRs).
struct Region {
  int x0, y0, bw, bh, pitch, sbase, xa, cw, cbase, pass, cend;
  float inv_cw;
};

// rg[u] for a runtime u, field by field through selects (an indexed copy of the struct
// array would go through scratch memory).
// (each operand goes through readfirstlane — a no-op on these uniform values — so that the
// select is not folded into an indexed load from a stack copy of the array.)
__device__ __forceinline__ int rfl(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ float rfl(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }
template <int NV>
__device__ __forceinline__ Region pick_region(const Region (&rg)[NV], int u) {
  Region r;
  if constexpr (NV == 4) {
#define MVN_PICK(f) r.f = u == 0 ? rfl(rg[0].f) : u == 1 ? rfl(rg[1].f) : u == 2 ? rfl(rg[2].f) : rfl(rg[3].f)
    MVN_PICK(x0); MVN_PICK(y0); MVN_PICK(bw); MVN_PICK(bh); MVN_PICK(pitch); MVN_PICK(sbase); MVN_PICK(xa);
    MVN_PICK(cw); MVN_PICK(cbase); MVN_PICK(pass); MVN_PICK(cend); MVN_PICK(inv_cw);
#undef MVN_PICK
  } else {
#define MVN_PICK(f)                                                   \
  r.f = rfl(rg[0].f);                                                 \
  _Pragma("unroll") for (int k = 1; k < NV; ++k) r.f = u == k ? rfl(rg[k].f) : r.f
    MVN_PICK(x0); MVN_PICK(y0); MVN_PICK(bw); MVN_PICK(bh); MVN_PICK(pitch); MVN_PICK(sbase); MVN_PICK(xa);
    MVN_PICK(cw); MVN_PICK(cbase); MVN_PICK(pass); MVN_PICK(cend); MVN_PICK(inv_cw);
#undef MVN_PICK
  }
  return r;
}

// The chunk-staged kernel for 4 and 8 views (unproject_x4.hip): MVN_OK, an error code, or 1
// when it does not apply to the call (then launch_tiled runs the generic kernel).
template <int AGG, typename TIn, typename TOut>
int launch_x4(const void* feat, const float* P, const float* coords, const float* cub, int transfer,
              const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
              int align_corners, int out_cl, int fast, hipStream_t s);

}  // namespace unproj
}  // namespace mvn
