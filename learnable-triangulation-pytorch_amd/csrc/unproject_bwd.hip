// Backward of the unprojection (mvn/utils/op.py:99-163) w.r.t. the feature maps (and the
// view confidences for 'conf*' aggregation), for gfx950.
//
// dL/dfeat[b,v,c,y,x] = sum over voxels i and taps t of  g[b,c,i] * dagg/ds_v(c,i) * w_t(i,v)
// with, per aggregation (s_v = sample of view v, out = aggregated value):
//   sum       1
//   conf*     conf[b,v,c]                 (and dL/dconf[b,v,c] = sum_i g * s_v)
//   max       1 for the first maximal view, else 0
//   softmax   p_v (1 + s_v - out),  p = softmax_v(s)
// Invalid (behind-camera) voxels and out-of-image taps carry no gradient, as in ATen's
// grid_sampler backward followed by the masked assignment.  Gradients w.r.t. the
// projection matrices and coordinate volumes are not produced (the reference's callers
// build both from numpy constants: triangulation.py:272-341).
//
// Structure mirrors the forward kernel: a block owns a 4x8x8 voxel tile, stages the
// forward features of its footprint when the aggregation needs samples, accumulates the
// tile's tap contributions into an LDS copy of the footprint with ds_add_f32, and flushes
// it with one global float atomic per touched (pixel, channel) — ~10x fewer global atomics
// than scattering every tap.  Float atomics make the result order-nondeterministic in the
// last bits (documented in DESIGN.md).
//
// Fixed-point mode (DET; mvn_unproject_backward_deterministic — the Python layer's default):
// every finite contribution — the same f32 product as above — is scaled by a power of two 2^e
// and rounded to a 64-bit integer; the LDS and the global accumulation are integer adds
// (ds_add_u64 / global_atomic_add_x2), which are associative, so the sums do not depend on
// the order the waves and blocks arrive in and two runs are bit-identical.  e is chosen per
// (frame, channel) plane — every element of grad_feat[b, :, c] and grad_conf[b, :, c] shares
// it — on the device (fix_scale_planes: no host sync) from that plane's finite maxima, so
// that no sum of the plane can leave +-2^62.  Range: the unit u is 2^-62 of the plane's bound
// nvox * max|g| * factor; each contribution is rounded to a whole unit, so an element fed by n
// contributions is the f32 rounding of an integer sum within n/2 units of its exact sum —
// absolute error <= n/2 * u + half an f32 ulp, i.e. relative <= n * 2^-25 + 2^-24 once the
// element is above 2^24 units = 2^-38 of the bound (2^-20 of max|g| * factor at 64^3); a frame
// or channel whose gradients are 1e8 x smaller than another's has its own scale.
// Non-finite contributions (a NaN or infinite grad_out / feature / confidence reaching a tap)
// are not summed: they set per-element flags (NaN, +inf, -inf) with atomicOr, and the element
// comes out as the reference's sequential float sum would: NaN if a NaN or both infinities
// reached it, else the infinity.  Elements no non-finite contribution reaches stay finite —
// ATen's grid_sampler backward confines a NaN to the taps it touches.
#include <algorithm>

#include "unproject_common.hpp"

namespace mvn {
namespace unproj {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int kSlots = 1024;                 // 16-byte slots per LDS buffer (two buffers)
constexpr int kZero = kSlots - 2;            // zero slots for voxel-views that sample nothing
constexpr int G = 4;                         // channels per slot (f32 accumulation)
constexpr int TX = 4, TY = 8, TZ = 8;        // one voxel per thread

template <typename T> __device__ __forceinline__ float ldf(const T* p, size_t i) { return to_f32(p[i]); }

// Fixed-point mode (DET): a finite f32 contribution x becomes round(x * 2^e) in a 64-bit integer
// (e of the element's (frame, channel) plane, so that no sum can leave +-2^62; clamp: guard only).
__device__ __forceinline__ unsigned long long to_fix(float x, float scale) {
  const float y = fminf(fmaxf(x * scale, -0x1p62f), 0x1p62f);
  return static_cast<unsigned long long>(__float2ll_rn(y));
}
// non-finite contribution flags (per element, atomicOr): the reference's float sum of them
constexpr unsigned kFlagNaN = 1u, kFlagPinf = 2u, kFlagNinf = 4u;
__device__ __forceinline__ unsigned nonfinite_flag(float x) {
  return x != x ? kFlagNaN : (x > 0.f ? kFlagPinf : kFlagNinf);
}
// the workspace: a 256-byte header, the per-(frame, channel) scales 2^e as f32 and 2^-e as f64,
// then a 64-bit word and a 32-bit flag word per feature element and confidence
constexpr size_t kFixHeaderBytes = 256;
// the fixed-point outputs of a call (DET)
struct FixArgs {
  unsigned long long* qfeat;   // per feature element
  unsigned long long* qconf;   // per confidence (conf* with grad_conf)
  unsigned* ffeat;             // non-finite flags per feature element
  unsigned* fconf;             // non-finite flags per confidence
  const float* scale;          // 2^e per (frame, channel)
};
// one contribution into global memory: float atomics (default) or the fixed point + flags (DET)
template <bool DET>
__device__ __forceinline__ void global_add(float* f, unsigned long long* q, unsigned* fl, size_t i, float x,
                                           float scale) {
  if constexpr (DET) {
    if (__builtin_isfinite(x)) atomicAdd(q + i, to_fix(x, scale));
    else atomicOr(fl + i, nonfinite_flag(x));
  } else {
    atomicAdd(f + i, x);
  }
}
// a fixed-point sum q (scaled by 2^e) -> the f32 rounding of its value: the top 53 bits of |q|
// with the rest folded into the last bit (round to odd), exact in f64, then one f64 -> f32
// rounding (53 >= 24 + 2: correct, f32 subnormals included; a plain double(q) would round twice)
__device__ __forceinline__ float fix_to_float(unsigned long long q, int e) {
  const bool neg = static_cast<long long>(q) < 0;
  const unsigned long long m = neg ? ~q + 1ull : q;
  if (m == 0ull) return 0.f;                           // +0, as a float sum of x and -x
  const int lz = __clzll(static_cast<long long>(m));
  const unsigned long long top = m << lz;
  const unsigned long long t53 = (top >> 11) | ((top & 0x7ffull) != 0ull ? 1ull : 0ull);
  const float f = static_cast<float>(ldexp(static_cast<double>(t53), 63 - lz - 52 - e));
  return neg ? -f : f;
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long x, int o) {
  const int lo = __shfl_xor(int(unsigned(x)), o, kWave), hi = __shfl_xor(int(unsigned(x >> 32)), o, kWave);
  return (static_cast<unsigned long long>(unsigned(hi)) << 32) | unsigned(lo);
}

template <int AGG, typename TIn, typename TG, int NV, bool DET>
__global__ __launch_bounds__(kThreads) void unproject_bwd_tiled(
    const TIn* __restrict__ feat, const float* __restrict__ P, const float* __restrict__ coords,
    const float* __restrict__ conf, const TG* __restrict__ gout, float* __restrict__ gfeat,
    float* __restrict__ gconf, FixArgs fa, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz, int align_corners) {
  constexpr bool kNeedSamples = AGG == MVN_AGG_SOFTMAX || AGG == MVN_AGG_MAX || AGG == MVN_AGG_CONF;
  __shared__ float4 fstage[kSlots];          // forward features (channels-last)
  __shared__ float4 gacc[DET ? 1 : kSlots];  // gradient accumulator (channels-last)
  __shared__ unsigned long long gq[DET ? kSlots * G : 1];   // the same in fixed point (DET)
  __shared__ int red[kWaves][NV][4];
  __shared__ int region[NV][5];              // xs, ys, bw, pitch, base
  __shared__ float gconf_acc[NV][G];
  __shared__ unsigned long long gconf_q[DET ? NV : 1][G];
  __shared__ int info[2];                    // total slots (or -1: direct global path)

  const int nTx = (Vx + TX - 1) / TX, nTy = (Vy + TY - 1) / TY, nTz = (Vz + TZ - 1) / TZ;
  int L = xcd_remap(blockIdx.x, B * nTx * nTy * nTz);
  const int tz = L % nTz; L /= nTz;
  const int ty = L % nTy; L /= nTy;
  const int tx = L % nTx;
  const int b = L / nTx;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int X = tx * TX + t / (TZ * TY), Y = ty * TY + (t / TZ) % TY, Z = tz * TZ + t % TZ;
  const bool act = (X < Vx) & (Y < Vy) & (Z < Vz);
  const int nvox = Vx * Vy * Vz, HW = H * W;
  const int vox = act ? (X * Vy + Y) * Vz + Z : 0;
  const float* cp = coords + (size_t(b) * nvox + vox) * 3;
  const float cx = cp[0], cy = cp[1], cz = cp[2];
  const float* Pb = P + size_t(b) * N * 12;
  const TIn* fb = feat + size_t(b) * N * C * HW;
  const size_t fbo = size_t(b) * N * C * HW;   // this frame's first element of grad_feat

  if (t < 2) { fstage[kZero + t] = make_float4(0.f, 0.f, 0.f, 0.f); }

  int fx[NV], fy[NV];
  float w[NV][4];
  bool has[NV];
  int bb[NV][4];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    bb[v][0] = INT_MAX; bb[v][1] = INT_MIN; bb[v][2] = INT_MAX; bb[v][3] = INT_MIN;
    has[v] = false; fx[v] = fy[v] = 0; w[v][0] = w[v][1] = w[v][2] = w[v][3] = 0.f;
    if (v < N) {
      const Proj p = project(Pb + v * 12, cx, cy, cz, H, W, align_corners);
      const float fx0 = floorf(p.ix), fy0 = floorf(p.iy);
      const bool h = act & !p.invalid & (fx0 >= -1.f) & (fx0 < float(W)) & (fy0 >= -1.f) & (fy0 < float(H));
      if (h) {
        const float a = p.ix - fx0, c = p.iy - fy0;
        w[v][0] = (1.f - c) * (1.f - a); w[v][1] = (1.f - c) * a; w[v][2] = c * (1.f - a); w[v][3] = c * a;
        fx[v] = int(fx0); fy[v] = int(fy0);
        bb[v][0] = fx[v]; bb[v][1] = fx[v]; bb[v][2] = fy[v]; bb[v][3] = fy[v];
      }
      has[v] = h;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      bb[v][0] = min(bb[v][0], __shfl_xor(bb[v][0], o, kWave));
      bb[v][1] = max(bb[v][1], __shfl_xor(bb[v][1], o, kWave));
      bb[v][2] = min(bb[v][2], __shfl_xor(bb[v][2], o, kWave));
      bb[v][3] = max(bb[v][3], __shfl_xor(bb[v][3], o, kWave));
    }
    if (lane == 0) { red[wid][v][0] = bb[v][0]; red[wid][v][1] = bb[v][1]; red[wid][v][2] = bb[v][2]; red[wid][v][3] = bb[v][3]; }
  }
  __syncthreads();
  if (t == 0) {
    int next = 0;
    for (int v = 0; v < NV && v < N; ++v) {
      int x0 = INT_MAX, x1 = INT_MIN, y0 = INT_MAX, y1 = INT_MIN;
      for (int q = 0; q < kWaves; ++q) {
        x0 = min(x0, red[q][v][0]); x1 = max(x1, red[q][v][1]);
        y0 = min(y0, red[q][v][2]); y1 = max(y1, red[q][v][3]);
      }
      int bw = 0, bh = 0;
      if (x0 <= x1) { bw = x1 - x0 + 2; bh = y1 - y0 + 2; }
      const int pitch = bw | 1;
      region[v][0] = x0; region[v][1] = y0; region[v][2] = bw; region[v][3] = pitch; region[v][4] = next;
      next += pitch * bh;
    }
    info[0] = next <= kZero ? next : -1;
  }
  __syncthreads();
  const int total = __builtin_amdgcn_readfirstlane(info[0]);

  const TG* gb = gout + size_t(b) * C * nvox + vox;
  if (total < 0) {
    // footprint larger than the LDS budget: scatter every tap with a global atomic.  Threads
    // past the volume's edge (partial tiles) have no voxel: they scatter nothing (their taps
    // sit at voxel 0's coordinates, where 0 * an infinite coefficient would add a NaN)
    if (!act) return;
    for (int c = 0; c < C; ++c) {
      float s[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) s[v] = 0.f;
      Taps tp[NV];
#pragma unroll
      for (int v = 0; v < NV; ++v)
        if (v < N) {
          tp[v] = view_taps(Pb + v * 12, cx, cy, cz, H, W, align_corners);
          if constexpr (kNeedSamples) s[v] = sample(fb + (size_t(v) * C + c) * HW, tp[v]);
        }
      const float g = act ? ldf(gb, size_t(c) * nvox) : 0.f;
      float coef[NV];
      float out = 0.f, den = 0.f, m = s[0];
      int arg = 0;
      if constexpr (AGG == MVN_AGG_SOFTMAX) {
#pragma unroll
        for (int v = 1; v < NV; ++v) if (v < N) m = fmaxf(m, s[v]);
#pragma unroll
        for (int v = 0; v < NV; ++v) if (v < N) { const float e = softmax_exp(s[v], m * kLog2e); den += e; out = __builtin_fmaf(s[v], e, out); }
        out *= __builtin_amdgcn_rcpf(den);
      }
      if constexpr (AGG == MVN_AGG_MAX) {
#pragma unroll
        for (int v = 1; v < NV; ++v) if (v < N && max_takes(s[v], s[arg])) arg = v;
      }
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if (v >= N) { coef[v] = 0.f; continue; }
        if constexpr (AGG == MVN_AGG_SUM) coef[v] = g;
        else if constexpr (AGG == MVN_AGG_CONF) coef[v] = g * conf[(size_t(b) * N + v) * C + c];
        else if constexpr (AGG == MVN_AGG_MAX) coef[v] = v == arg ? g : 0.f;
        else coef[v] = g * (softmax_exp(s[v], m * kLog2e) * __builtin_amdgcn_rcpf(den)) * (1.f + s[v] - out);
        const float fsc = DET ? fa.scale[size_t(b) * C + c] : 0.f;
        if (coef[v] != 0.f) {
          // every in-image tap of the voxel-view receives coef * w (ATen grid_sampler backward:
          // a zero weight still carries a NaN or infinite coefficient as NaN)
          const size_t pl = fbo + (size_t(v) * C + c) * HW;
          const int o[4] = {tp[v].o0, tp[v].o1, tp[v].o2, tp[v].o3};
          const float wt[4] = {tp[v].w0, tp[v].w1, tp[v].w2, tp[v].w3};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float x = coef[v] * wt[q];
            if (((tp[v].in >> q) & 1u) && x != 0.f) global_add<DET>(gfeat, fa.qfeat, fa.ffeat, pl + o[q], x, fsc);
          }
        }
        // (an invalid voxel-view's sample is the masked 0: g * 0, NaN only for a NaN / inf g)
        if constexpr (AGG == MVN_AGG_CONF)
          if (gconf && v < N && g * s[v] != 0.f)
            global_add<DET>(gconf, fa.qconf, fa.fconf, (size_t(b) * N + v) * C + c, g * s[v], fsc);
      }
    }
    return;
  }

  int rx[NV], ry[NV], rbw[NV], rpitch[NV], rbase[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    rx[v] = __builtin_amdgcn_readfirstlane(region[v][0]);
    ry[v] = __builtin_amdgcn_readfirstlane(region[v][1]);
    rbw[v] = __builtin_amdgcn_readfirstlane(region[v][2]);
    rpitch[v] = __builtin_amdgcn_readfirstlane(region[v][3]);
    rbase[v] = __builtin_amdgcn_readfirstlane(region[v][4]);
  }
  int slot[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) slot[v] = has[v] ? rbase[v] + (fy[v] - ry[v]) * rpitch[v] + (fx[v] - rx[v]) : kZero;

  for (int c0 = 0; c0 < C; c0 += G) {
    // ---- zero the accumulator, stage forward features ---------------------------------
    for (int idx = t; idx < total; idx += kThreads) {
      if constexpr (DET) {
#pragma unroll
        for (int k = 0; k < G; ++k) gq[idx * G + k] = 0ull;
      } else {
        gacc[idx] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if constexpr (kNeedSamples) {
        int v = 0;
#pragma unroll
        for (int u = 1; u < NV; ++u) if (u < N && idx >= rbase[u]) v = u;
        int px = 0, py = 0, bwv = 0, pv = 1, xs = 0, ys = 0, base = 0;
#pragma unroll
        for (int u = 0; u < NV; ++u) if (u == v) { pv = rpitch[u]; bwv = rbw[u]; xs = rx[u]; ys = ry[u]; base = rbase[u]; }
        py = (idx - base) / pv;
        px = idx - base - py * pv;
        const int gx = xs + px, gy = ys + py;
        const bool in = (px < bwv) & (gx >= 0) & (gx < W) & (gy >= 0) & (gy < H);
        float q[G];
#pragma unroll
        for (int k = 0; k < G; ++k) q[k] = (in && c0 + k < C) ? ldf(fb, (size_t(v) * C + c0 + k) * HW + size_t(gy) * W + gx) : 0.f;
        MVN_DASSERT(idx >= 0 && idx < kZero);
        fstage[idx] = make_float4(q[0], q[1], q[2], q[3]);
      }
    }
    if (t < NV * G) {
      if constexpr (DET) gconf_q[t / G][t % G] = 0ull;
      else gconf_acc[t / G][t % G] = 0.f;
    }
    __syncthreads();

    // ---- per voxel: samples, upstream gradient, d agg / d s_v, LDS scatter ------------
    float g[G], fsc[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      g[k] = (act && c0 + k < C) ? ldf(gb, size_t(c0 + k) * nvox) : 0.f;
      fsc[k] = (DET && c0 + k < C) ? fa.scale[size_t(b) * C + c0 + k] : 0.f;   // 2^e of the plane
    }
    float s[NV][G];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
#pragma unroll
      for (int k = 0; k < G; ++k) s[v][k] = 0.f;
      if constexpr (kNeedSamples) {
        if (v < N) {
          const int o = slot[v], o2 = has[v] ? slot[v] + rpitch[v] : kZero;
          MVN_DASSERT(o >= 0 && o + 1 < kSlots && o2 >= 0 && o2 + 1 < kSlots);
          const float4 a = fstage[o], bq = fstage[o + 1], c = fstage[o2], d = fstage[o2 + 1];
          const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {bq.x, bq.y, bq.z, bq.w};
          const float cv[4] = {c.x, c.y, c.z, c.w}, dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
          for (int k = 0; k < G; ++k)
            s[v][k] = __builtin_fmaf(dv[k], w[v][3], __builtin_fmaf(cv[k], w[v][2], __builtin_fmaf(bv[k], w[v][1], av[k] * w[v][0])));
        }
      }
    }
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int c = c0 + k;
      float coef[NV];
      if constexpr (AGG == MVN_AGG_SOFTMAX) {
        float m = s[0][k];
#pragma unroll
        for (int v = 1; v < NV; ++v) if (v < N) m = fmaxf(m, s[v][k]);
        float den = 0.f, out = 0.f, e[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) { e[v] = v < N ? softmax_exp(s[v][k], m * kLog2e) : 0.f; den += e[v]; out = __builtin_fmaf(s[v][k], e[v], out); }
        const float inv = __builtin_amdgcn_rcpf(den);
        out *= inv;
#pragma unroll
        for (int v = 0; v < NV; ++v) coef[v] = g[k] * e[v] * inv * (1.f + s[v][k] - out);
      } else if constexpr (AGG == MVN_AGG_MAX) {
        int arg = 0;
#pragma unroll
        for (int v = 1; v < NV; ++v) if (v < N && max_takes(s[v][k], s[arg][k])) arg = v;
#pragma unroll
        for (int v = 0; v < NV; ++v) coef[v] = v == arg ? g[k] : 0.f;
      } else if constexpr (AGG == MVN_AGG_CONF) {
#pragma unroll
        for (int v = 0; v < NV; ++v) coef[v] = (v < N && c < C) ? g[k] * conf[(size_t(b) * N + v) * C + c] : 0.f;
      } else {
#pragma unroll
        for (int v = 0; v < NV; ++v) coef[v] = g[k];
      }
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if (v >= N || !has[v] || coef[v] == 0.f) continue;
        if constexpr (DET) {
          // the weights are finite and at most 1, so coef * w is non-finite exactly when coef
          // is: that rare case (a NaN or infinite input) flags the in-image taps directly
          if (__builtin_isfinite(coef[v])) {
            unsigned long long* q0 = &gq[slot[v] * G + k];
            unsigned long long* q1 = &gq[(slot[v] + rpitch[v]) * G + k];
            atomicAdd(q0, to_fix(coef[v] * w[v][0], fsc[k]));
            atomicAdd(q0 + G, to_fix(coef[v] * w[v][1], fsc[k]));
            atomicAdd(q1, to_fix(coef[v] * w[v][2], fsc[k]));
            atomicAdd(q1 + G, to_fix(coef[v] * w[v][3], fsc[k]));
          } else {
#pragma unroll 1
            for (int q = 0; q < 4; ++q) {
              const int gx = fx[v] + (q & 1), gy = fy[v] + (q >> 1);
              if (gx >= 0 && gx < W && gy >= 0 && gy < H && c < C)
                atomicOr(fa.ffeat + fbo + (size_t(v) * C + c) * HW + size_t(gy) * W + gx,
                         nonfinite_flag(coef[v] * w[v][q]));
            }
          }
        } else {
          float* base0 = reinterpret_cast<float*>(&gacc[slot[v]]) + k;
          float* base1 = reinterpret_cast<float*>(&gacc[slot[v] + rpitch[v]]) + k;
          atomicAdd(base0, coef[v] * w[v][0]);
          atomicAdd(base0 + 4, coef[v] * w[v][1]);
          atomicAdd(base1, coef[v] * w[v][2]);
          atomicAdd(base1 + 4, coef[v] * w[v][3]);
        }
      }
      if constexpr (AGG == MVN_AGG_CONF) {
        if (gconf) {
#pragma unroll
          for (int v = 0; v < NV; ++v) {
            if (v >= N) continue;
            // (an invalid voxel-view's sample is the masked 0, op.py:137: g * 0 carries only a
            // NaN / infinite g; g is 0 past the tile and C)
            float part = g[k] * s[v][k];
            if constexpr (DET) {
              // exact: each lane's term in fixed point, summed by integer butterflies
              unsigned long long q = 0ull;
              if (__builtin_isfinite(part)) q = to_fix(part, fsc[k]);
              else atomicOr(fa.fconf + (size_t(b) * N + v) * C + c, nonfinite_flag(part));
#pragma unroll
              for (int o = 32; o > 0; o >>= 1) q += shfl_xor_u64(q, o);
              if (lane == 0 && q != 0ull) atomicAdd(&gconf_q[v][k], q);
            } else {
#pragma unroll
              for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, kWave);
              if (lane == 0 && part != 0.f) atomicAdd(&gconf_acc[v][k], part);
            }
          }
        }
      }
    }
    __syncthreads();

    // ---- flush the footprint: one global atomic per touched (pixel, channel) ---------
    for (int idx = t; idx < total; idx += kThreads) {
      int v = 0;
#pragma unroll
      for (int u = 1; u < NV; ++u) if (u < N && idx >= rbase[u]) v = u;
      int bwv = 0, pv = 1, xs = 0, ys = 0, base = 0;
#pragma unroll
      for (int u = 0; u < NV; ++u) if (u == v) { pv = rpitch[u]; bwv = rbw[u]; xs = rx[u]; ys = ry[u]; base = rbase[u]; }
      const int py = (idx - base) / pv, px = idx - base - py * pv;
      const int gx = xs + px, gy = ys + py;
      if ((px < bwv) & (gx >= 0) & (gx < W) & (gy >= 0) & (gy < H)) {
        const size_t pix = fbo + size_t(gy) * W + gx;
        if constexpr (DET) {
#pragma unroll
          for (int k = 0; k < G; ++k) {
            const unsigned long long q = gq[idx * G + k];
            if (c0 + k < C && q != 0ull) atomicAdd(fa.qfeat + pix + (size_t(v) * C + c0 + k) * HW, q);
          }
        } else {
          const float4 a = gacc[idx];
          const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
          for (int k = 0; k < G; ++k)
            if (c0 + k < C && av[k] != 0.f) atomicAdd(gfeat + pix + (size_t(v) * C + c0 + k) * HW, av[k]);
        }
      }
    }
    if constexpr (AGG == MVN_AGG_CONF) {
      if (gconf && t < NV * G) {
        const int v = t / G, k = t % G;
        const size_t o = (size_t(b) * N + v) * C + c0 + k;
        if constexpr (DET) {
          if (v < N && c0 + k < C && gconf_q[v][k] != 0ull) atomicAdd(fa.qconf + o, gconf_q[v][k]);
        } else {
          if (v < N && c0 + k < C && gconf_acc[v][k] != 0.f) atomicAdd(gconf + o, gconf_acc[v][k]);
        }
      }
    }
    __syncthreads();
  }
}

// max |x| over the finite values among n elements at x[i * stride .. + len) (several strided
// runs: the views of a (frame, channel) plane), as f32 bits (|x| >= 0 orders like its bits), one
// 256-thread block
template <typename T>
__device__ __forceinline__ unsigned block_absmax(const T* __restrict__ x, int runs, size_t stride, size_t len,
                                                 unsigned* red) {
  unsigned m = 0;
  for (int r = 0; r < runs; ++r)
    for (size_t i = threadIdx.x; i < len; i += blockDim.x) {
      const unsigned bits = __float_as_uint(fabsf(to_f32(x[r * stride + i])));
      m = max(m, bits < 0x7f800000u ? bits : 0u);        // non-finite values are flagged, not summed
    }
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) m = max(m, unsigned(__shfl_xor(int(m), o, kWave)));
  __syncthreads();
  if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = m;
  __syncthreads();
  unsigned b = 0;
#pragma unroll
  for (int w = 0; w < 256 / kWave; ++w) b = max(b, red[w]);
  return b;
}
// the fixed-point scale 2^e of each (frame, channel) plane, one block per plane.  Bound on any
// sum of the plane (finite contributions only; a voxel-view's bilinear weights sum to <= 1, so
// each voxel adds at most |coefficient| to an element): nvox * max|g| * factor, factor = 1
// (sum, max), max(1, max|conf|) for the feature and max|feat| for the confidence gradient
// (conf*), 1 + 2 max|feat| (softmax: |d agg / d s_v| <= 1 + 2 max|s|).  e puts it below 2^62.
template <typename TIn, typename TG>
__global__ __launch_bounds__(256) void fix_scale_planes(const TIn* __restrict__ feat, const TG* __restrict__ gout,
                                                        const float* __restrict__ conf, float* __restrict__ scale,
                                                        int* __restrict__ expo, int N, int C, int HW, int nvox,
                                                        int agg) {
  __shared__ unsigned red[256 / kWave];
  const int b = blockIdx.x / C, c = blockIdx.x % C;
  const double g = __uint_as_float(block_absmax(gout + (size_t(b) * C + c) * nvox, 1, 0, size_t(nvox), red));
  double factor = 1.0;
  if (agg == MVN_AGG_SOFTMAX || agg == MVN_AGG_CONF) {
    const double f = __uint_as_float(
        block_absmax(feat + (size_t(b) * N * C + c) * HW, N, size_t(C) * HW, size_t(HW), red));
    if (agg == MVN_AGG_SOFTMAX) {
      factor = 1.0 + 2.0 * f;
    } else {
      unsigned cm = 0;
      for (int v = 0; v < N; ++v) {
        const unsigned bits = __float_as_uint(fabsf(conf[(size_t(b) * N + v) * C + c]));
        cm = max(cm, bits < 0x7f800000u ? bits : 0u);
      }
      factor = fmax(fmax(1.0, double(__uint_as_float(cm))), f);
    }
  }
  if (threadIdx.x != 0) return;
  const double bound = double(nvox) * g * factor;
  int e = 62;
  if (bound > 0.0) e = int(floor(62.0 - log2(bound))) - 1;
  e = min(max(e, -120), 120);
  scale[blockIdx.x] = ldexpf(1.f, e);
  expo[blockIdx.x] = e;
}
// fixed-point sums + non-finite flags (DET) -> f32 gradients; element i belongs to the plane
// (i / per_b) * C + (i / per_c) % C (per_c elements per channel run, per_b per frame)
__global__ void fix_to_f32(const unsigned long long* __restrict__ q, const unsigned* __restrict__ flags,
                           float* __restrict__ out, size_t n, const int* __restrict__ expo, int C, size_t per_c,
                           size_t per_b) {
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
    const size_t plane = (i / per_b) * C + (i / per_c) % C;
    const unsigned f = flags[i];
    float r = fix_to_float(q[i], expo[plane]);
    if (f) r = ((f & kFlagNaN) || (f & (kFlagPinf | kFlagNinf)) == (kFlagPinf | kFlagNinf))
                   ? __builtin_nanf("")
                   : (f & kFlagPinf ? __builtin_inff() : -__builtin_inff());
    out[i] = r;
  }
}

template <int AGG, typename TIn, typename TG, bool DET>
int launch_bwd(const void* feat, const float* P, const float* coords, const float* conf, const void* gout, float* gfeat,
               float* gconf, FixArgs fa, int B, int N,
               int C, int H, int W, int Vx, int Vy, int Vz, int ac, hipStream_t s) {
  const long long nb = (long long)B * ((Vx + TX - 1) / TX) * ((Vy + TY - 1) / TY) * ((Vz + TZ - 1) / TZ);
  if (nb > INT_MAX) return MVN_ERR_SHAPE;
  if (N <= 4)
    unproject_bwd_tiled<AGG, TIn, TG, 4, DET><<<int(nb), kThreads, 0, s>>>(static_cast<const TIn*>(feat), P, coords,
        conf, static_cast<const TG*>(gout), gfeat, gconf, fa, B, N, C, H, W, Vx, Vy, Vz, ac);
  else if (N <= 8)
    unproject_bwd_tiled<AGG, TIn, TG, 8, DET><<<int(nb), kThreads, 0, s>>>(static_cast<const TIn*>(feat), P, coords,
        conf, static_cast<const TG*>(gout), gfeat, gconf, fa, B, N, C, H, W, Vx, Vy, Vz, ac);
  else
    return MVN_ERR_SHAPE;
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

template <typename TIn, typename TG, bool DET>
int dispatch_bwd(int agg, const void* feat, const float* P, const float* coords, const float* conf, const void* gout,
                 float* gfeat, float* gconf, FixArgs fa,
                 int B, int N, int C, int H, int W, int Vx, int Vy, int Vz, int ac, hipStream_t s) {
  switch (agg) {
    case MVN_AGG_SUM:
      return launch_bwd<MVN_AGG_SUM, TIn, TG, DET>(feat, P, coords, conf, gout, gfeat, gconf, fa, B, N, C, H,
                                                   W, Vx, Vy, Vz, ac, s);
    case MVN_AGG_MAX:
      return launch_bwd<MVN_AGG_MAX, TIn, TG, DET>(feat, P, coords, conf, gout, gfeat, gconf, fa, B, N, C, H,
                                                   W, Vx, Vy, Vz, ac, s);
    case MVN_AGG_SOFTMAX:
      return launch_bwd<MVN_AGG_SOFTMAX, TIn, TG, DET>(feat, P, coords, conf, gout, gfeat, gconf, fa, B, N,
                                                       C, H, W, Vx, Vy, Vz, ac, s);
    case MVN_AGG_CONF:
      return launch_bwd<MVN_AGG_CONF, TIn, TG, DET>(feat, P, coords, conf, gout, gfeat, gconf, fa, B, N, C,
                                                    H, W, Vx, Vy, Vz, ac, s);
  }
  return MVN_ERR_ARG;
}

template <bool DET>
int backward_entry(const void* feat, int feat_dtype, const float* proj, const float* coords, const float* conf,
                   const void* grad_out, int grad_out_dtype, float* grad_feat, float* grad_conf,
                   FixArgs fa, int B, int N, int C, int H,
                   int W, int Vx, int Vy, int Vz, int agg, int align_corners, hipStream_t s) {
  const bool f16 = feat_dtype == MVN_DTYPE_BF16, g16 = grad_out_dtype == MVN_DTYPE_BF16;
  if ((feat_dtype != MVN_DTYPE_F32 && !f16) || (grad_out_dtype != MVN_DTYPE_F32 && !g16)) return MVN_ERR_DTYPE;
  if (!f16 && !g16)
    return dispatch_bwd<float, float, DET>(agg, feat, proj, coords, conf, grad_out, grad_feat, grad_conf, fa,
                                           B, N, C, H, W, Vx, Vy, Vz, align_corners, s);
  if (f16 && g16)
    return dispatch_bwd<uint16_t, uint16_t, DET>(agg, feat, proj, coords, conf, grad_out, grad_feat, grad_conf, fa, B, N, C, H, W, Vx, Vy, Vz, align_corners, s);
  if (f16)
    return dispatch_bwd<uint16_t, float, DET>(agg, feat, proj, coords, conf, grad_out, grad_feat, grad_conf, fa, B, N, C, H, W, Vx, Vy, Vz, align_corners, s);
  return dispatch_bwd<float, uint16_t, DET>(agg, feat, proj, coords, conf, grad_out, grad_feat, grad_conf, fa,
                                            B, N, C, H, W, Vx, Vy, Vz, align_corners, s);
}

int check_bwd_args(const void* feat, const float* proj, const float* coords, const float* conf, const void* grad_out,
                   const float* grad_feat, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz, int agg,
                   int align_corners) {
  if (!feat || !proj || !coords || !grad_out || !grad_feat) return MVN_ERR_ARG;
  if (agg < MVN_AGG_SUM || agg > MVN_AGG_CONF) return MVN_ERR_ARG;
  if (agg == MVN_AGG_CONF && !conf) return MVN_ERR_ARG;
  if (align_corners != 0 && align_corners != 1) return MVN_ERR_ARG;
  if (B <= 0 || N <= 0 || C <= 0 || H <= 0 || W <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0) return MVN_ERR_SHAPE;
  if ((long long)Vx * Vy * Vz > (1LL << 30) || (long long)H * W > (1LL << 30) || N > 8) return MVN_ERR_SHAPE;
  return MVN_OK;
}

}  // namespace
}  // namespace unproj
}  // namespace mvn

extern "C" int mvn_unproject_backward(const void* feat, int feat_dtype, const float* proj, const float* coords,
                                      const float* conf, const void* grad_out, int grad_out_dtype, float* grad_feat,
                                      float* grad_conf, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                                      int agg, int align_corners, void* stream) {
  using namespace mvn;
  using namespace mvn::unproj;
  const int e = check_bwd_args(feat, proj, coords, conf, grad_out, grad_feat, B, N, C, H, W, Vx, Vy, Vz, agg,
                               align_corners);
  if (e != MVN_OK) return e;
  return backward_entry<false>(feat, feat_dtype, proj, coords, conf, grad_out, grad_out_dtype, grad_feat, grad_conf,
                               FixArgs{}, B, N, C, H, W, Vx, Vy, Vz, agg, align_corners,
                               static_cast<hipStream_t>(stream));
}

extern "C" size_t mvn_unproject_backward_workspace_bytes(int B, int N, int C, int H, int W) {
  if (B <= 0 || N <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  // header, 2^e (f32) and e (int) per (frame, channel), then a 64-bit word and a 32-bit flag per
  // feature element and confidence
  const size_t planes = size_t(B) * C;
  return mvn::unproj::kFixHeaderBytes + ((planes * 8 + 255) / 256) * 256 +
         (size_t(B) * N * C * size_t(H) * W + size_t(B) * N * C) * (sizeof(unsigned long long) + sizeof(unsigned));
}

extern "C" int mvn_unproject_backward_deterministic(const void* feat, int feat_dtype, const float* proj,
                                                    const float* coords, const float* conf, const void* grad_out,
                                                    int grad_out_dtype, float* grad_feat, float* grad_conf,
                                                    void* workspace, size_t workspace_bytes, int B, int N, int C,
                                                    int H, int W, int Vx, int Vy, int Vz, int agg, int align_corners,
                                                    void* stream) {
  using namespace mvn;
  using namespace mvn::unproj;
  const int e = check_bwd_args(feat, proj, coords, conf, grad_out, grad_feat, B, N, C, H, W, Vx, Vy, Vz, agg,
                               align_corners);
  if (e != MVN_OK) return e;
  const size_t nfeat = size_t(B) * N * C * size_t(H) * W, nconf = size_t(B) * N * C;
  if (!workspace || workspace_bytes < mvn_unproject_backward_workspace_bytes(B, N, C, H, W)) return MVN_ERR_WORKSPACE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const size_t planes = size_t(B) * C;
  char* ws = static_cast<char*>(workspace);
  auto* scale = reinterpret_cast<float*>(ws + kFixHeaderBytes);
  auto* expo = reinterpret_cast<int*>(scale + planes);
  auto* qfeat = reinterpret_cast<unsigned long long*>(ws + kFixHeaderBytes + ((planes * 8 + 255) / 256) * 256);
  auto* qconf = qfeat + nfeat;
  auto* ffeat = reinterpret_cast<unsigned*>(qconf + nconf);
  auto* fconf = ffeat + nfeat;
  if (hipMemsetAsync(qfeat, 0, (nfeat + nconf) * (sizeof(unsigned long long) + sizeof(unsigned)), s) != hipSuccess)
    return MVN_ERR_LAUNCH;
  // the fixed-point scale of each (frame, channel) plane from its finite maxima (device-side)
  if (planes > INT_MAX) return MVN_ERR_SHAPE;
  const int nvox = Vx * Vy * Vz, HW = H * W;
  const bool f16 = feat_dtype == MVN_DTYPE_BF16, g16 = grad_out_dtype == MVN_DTYPE_BF16;
  if ((feat_dtype != MVN_DTYPE_F32 && !f16) || (grad_out_dtype != MVN_DTYPE_F32 && !g16)) return MVN_ERR_DTYPE;
  const int nb = int(planes);
  if (f16 && g16)
    fix_scale_planes<<<nb, 256, 0, s>>>(static_cast<const uint16_t*>(feat), static_cast<const uint16_t*>(grad_out), conf,
                                        scale, expo, N, C, HW, nvox, agg);
  else if (f16)
    fix_scale_planes<<<nb, 256, 0, s>>>(static_cast<const uint16_t*>(feat), static_cast<const float*>(grad_out), conf,
                                        scale, expo, N, C, HW, nvox, agg);
  else if (g16)
    fix_scale_planes<<<nb, 256, 0, s>>>(static_cast<const float*>(feat), static_cast<const uint16_t*>(grad_out), conf,
                                        scale, expo, N, C, HW, nvox, agg);
  else
    fix_scale_planes<<<nb, 256, 0, s>>>(static_cast<const float*>(feat), static_cast<const float*>(grad_out), conf,
                                        scale, expo, N, C, HW, nvox, agg);
  const int r = backward_entry<true>(feat, feat_dtype, proj, coords, conf, grad_out, grad_out_dtype, grad_feat,
                                     grad_conf, FixArgs{qfeat, qconf, ffeat, fconf, scale}, B, N, C, H, W, Vx,
                                     Vy, Vz, agg, align_corners, s);
  if (r != MVN_OK) return r;
  auto cvt_blocks = [](size_t n) { return int(std::min<size_t>((n + 255) / 256, 65536)); };
  fix_to_f32<<<cvt_blocks(nfeat), 256, 0, s>>>(qfeat, ffeat, grad_feat, nfeat, expo, C, size_t(HW), size_t(N) * C * HW);
  if (grad_conf) fix_to_f32<<<cvt_blocks(nconf), 256, 0, s>>>(qconf, fconf, grad_conf, nconf, expo, C, 1, size_t(N) * C);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}
