// Shared device code of the unprojection kernels (unproject.hip, unproject_tiled.hip).
#pragma once

#include "common.hpp"

namespace mvn {
namespace unproj {

// Bilinear taps of one voxel in one view: 4 clamped plane offsets + 4 weights.
// Out-of-bounds corners and invalid (behind-camera) voxels get weight 0, which is
// bit-identical to the reference's zero-valued corner / zeroed sample for finite
// feature values (fma(v, 0, acc) == acc).
struct Taps {
  int o0, o1, o2, o3;
  float w0, w1, w2, w3;
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
  t.o0 = y0 * W + x0;  t.w0 = (ok & y0in & x0in) ? sy * sx : 0.f;   // nw
  t.o1 = y0 * W + x1;  t.w1 = (ok & y0in & x1in) ? sy * tx : 0.f;   // ne
  t.o2 = y1 * W + x0;  t.w2 = (ok & y1in & x0in) ? ty * sx : 0.f;   // sw
  t.o3 = y1 * W + x1;  t.w3 = (ok & y1in & x1in) ? ty * tx : 0.f;   // se
  return t;
}

template <typename TIn>
__device__ __forceinline__ float sample(const TIn* __restrict__ plane, const Taps& t) {
  const float a = to_f32(plane[t.o0]);
  const float b = to_f32(plane[t.o1]);
  const float c = to_f32(plane[t.o2]);
  const float d = to_f32(plane[t.o3]);
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
    for (int v = 1; v < NV; ++v) if (v < N) r = s[v] > r ? s[v] : r;
  } else if constexpr (AGG == MVN_AGG_CONF) {      // op.py:148: product rounded, then summed
    r = s[0] * cf[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) if (v < N) r = r + s[v] * cf[size_t(v) * cstride];
  } else {                                         // op.py:153-159: softmax over the views
    float m = s[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) if (v < N) m = fmaxf(m, s[v]);
    float den = 0.f, num = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (v < N) {
        const float e = __expf(s[v] - m);
        den += e;
        num = __builtin_fmaf(s[v], e, num);
      }
    r = num / den;
  }
  return r;
}

// Launchers (defined in unproject_tiled.hip); return MVN_OK or an error code.
template <int AGG, typename TIn, typename TOut>
// cub != nullptr: voxel coordinates formed in-kernel from the per-frame cuboids (coords unused;
// Vx = Vy = Vz), see cuboid_coord in common.hpp.
int launch_tiled(const void* feat, const float* P, const float* coords, const float* cub, int transfer,
                 const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                 int align_corners, int out_cl, hipStream_t s);

}  // namespace unproj
}  // namespace mvn
