// Microbenchmark (design aid, not product code): the MEASURED arithmetic floor of the
// 4-view unprojection.  Each thread runs the per-voxel instruction
// stream the reference's f32 semantics require and nothing else:
//   * the voxel's coordinates (one 12-byte load, as the real kernel),
//   * the 4-view projection with the exact IEEE divisions (op.py:117-130, the production
//     project_h path of unproject_common.hpp: homog FMA chain, w<=0 mask, w==0 guard,
//     two exact divisions per coordinate, grid unnormalisation, floor, bilinear weights),
//   * per channel group of 4 channels (8 groups for C = 32): 4 views x 4 taps of 4 channels
//     as packed f32 FMAs in the reference's order (op.py:134), then the view aggregation of
//     op.py:147-161 (softmax: max, exp2, sum, fma chain, reciprocal; or sum),
// with the tap VALUES taken from registers (no LDS, no staging loads, no footprints, no
// barriers) and the outputs folded into one packed accumulator per thread (16 v_pk_add per
// voxel, the only non-semantic VALU) stored once.  asm volatile("" : "+v") fences make the
// tap registers opaque per view and group, so nothing is hoisted or shared across groups.
//
// Round 6 adds the fast arithmetic (MVN_PRECISION_FAST), modes 4-6: the
// reciprocal projection, bf16 pixel-pair tap slots (2 per view and 4 channels) sampled by
// v_dot2_f32_bf16 with bf16 weights, and the max-free view softmax (or sum).
//
// Build (CPU container):  tools/micro/build_floor.sh   ->  tools/bin/unproject_floor.so
// Run   (GPU box):        python tools/micro/unproject_floor.py
#include <hip/hip_runtime.h>

#include "unproject_common.hpp"

using namespace mvn;
using namespace mvn::unproj;

namespace {

// MODE: 0 projection + taps + softmax, 1 projection + taps + sum, 2 projection only,
//       3 taps + softmax (weights from the coordinates, no projection);
//       fast arithmetic: 4 projection + dot2 taps + softmax, 5 ... + sum, 6 projection only
template <int MODE>
__global__ __launch_bounds__(256) void floor_kernel(const float* __restrict__ P, const float* __restrict__ coords,
                                                    const uint4* __restrict__ seed, float* __restrict__ out,
                                                    int nvox, int H, int W, int C) {
  constexpr int NV = 4;
  const int gid = int(blockIdx.x) * 256 + int(threadIdx.x);
  const int b = gid / nvox;
  const float* Pb = P + size_t(b) * NV * 12;
  const float* cp = coords + size_t(gid) * 3;
  const float cx = cp[0], cy = cp[1], cz = cp[2];

  f2 wp[NV][2];
  uint32_t wq[NV][2];
  int fx[NV], fy[NV];
  constexpr bool FASTM = MODE >= 4;
  if constexpr (FASTM) {
    const float fW = float(W), fH = float(H);
    const float ax = fW * __builtin_amdgcn_rcpf(fH), ay = fH * __builtin_amdgcn_rcpf(fW);
    const float ks = MODE == 4 ? kLog2e : 1.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const Homog hp = homog(Pb + v * 12, cx, cy, cz);
      const float r = __builtin_amdgcn_rcpf(hp.wh == 0.f ? 1.f : hp.wh);
      const float ix = __builtin_fmaf(hp.uh, ax * r, -0.5f), iy = __builtin_fmaf(hp.vh, ay * r, -0.5f);
      const float fx0 = floorf(ix), fy0 = floorf(iy);
      const bool h = !(hp.wh <= 0.f) & (fx0 >= -1.f) & (fx0 < fW) & (fy0 >= -1.f) & (fy0 < fH);
      const float tx_ = ix - fx0, sx_ = 1.f - tx_, ty_ = (iy - fy0) * ks, sy_ = ks - ty_;
      wp[v][0] = f2{h ? sy_ * sx_ : 0.f, h ? sy_ * tx_ : 0.f};
      wp[v][1] = f2{h ? ty_ * sx_ : 0.f, h ? ty_ * tx_ : 0.f};
      wq[v][0] = pack_bf16x2(wp[v][0].x, wp[v][0].y);
      wq[v][1] = pack_bf16x2(wp[v][1].x, wp[v][1].y);
      fx[v] = h ? int(fx0) : 0;
      fy[v] = h ? int(fy0) : 0;
    }
  } else if constexpr (MODE != 3) {
    bool lane_fast = true;
#pragma unroll
    for (int v = 0; v < NV; ++v) lane_fast &= div_core_safe(homog(Pb + v * 12, cx, cy, cz));
    const bool wave_fast = __builtin_amdgcn_ballot_w64(!lane_fast) == 0;
    const Recip rH = recip_refined(float(H)), rW = recip_refined(float(W));
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const Homog hp = homog(Pb + v * 12, cx, cy, cz);
      const Proj p = wave_fast ? project_h<true>(hp, H, W, 0, rH, rW) : project_h<false>(hp, H, W, 0, rH, rW);
      const float fx0 = floorf(p.ix), fy0 = floorf(p.iy);
      const bool h = !p.invalid & (fx0 >= -1.f) & (fx0 < float(W)) & (fy0 >= -1.f) & (fy0 < float(H));
      const float tx_ = p.ix - fx0, sx_ = 1.f - tx_, ty_ = p.iy - fy0, sy_ = 1.f - ty_;
      wp[v][0] = f2{h ? sy_ * sx_ : 0.f, h ? sy_ * tx_ : 0.f};
      wp[v][1] = f2{h ? ty_ * sx_ : 0.f, h ? ty_ * tx_ : 0.f};
      fx[v] = h ? int(fx0) : 0;
      fy[v] = h ? int(fy0) : 0;
    }
  } else {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const float a = cx * Pb[v * 12] + 0.25f, c = cy * Pb[v * 12 + 1] + 0.5f;
      wp[v][0] = f2{a, c};
      wp[v][1] = f2{c * a, a - c};
      fx[v] = fy[v] = 0;
    }
  }

  f2 acc = f2{0.f, 0.f};
  if constexpr (MODE == 6) {
#pragma unroll
    for (int v = 0; v < NV; ++v)
      acc += f2{__uint_as_float(wq[v][0]), __uint_as_float(wq[v][1])} + f2{float(fx[v]), float(fy[v])};
  } else if constexpr (FASTM) {
    // 2 pixel-pair slots (rows y0, y1) of 4 channels per view, opaque per view and group
    uint4 s0 = seed[threadIdx.x & 63], s2 = seed[128 + (threadIdx.x & 63)];
    float dmx = 0.f, dmn = INFINITY;
#pragma unroll 1
    for (int c0 = 0; c0 < C; c0 += 4) {
      f2 sv[2][NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        asm volatile("" : "+v"(s0.x), "+v"(s0.y), "+v"(s0.z), "+v"(s0.w), "+v"(s2.x), "+v"(s2.y), "+v"(s2.z),
                     "+v"(s2.w));
        const bf16x2_t w1 = __builtin_bit_cast(bf16x2_t, wq[v][1]);
        const uint32_t an[4] = {s0.x, s0.y, s0.z, s0.w}, as[4] = {s2.x, s2.y, s2.z, s2.w};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          float o[2];
#pragma unroll
          for (int h = 0; h < 2; ++h)
            o[h] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, as[2 * q + h]), w1,
                                                   dot2_bf16_from0(an[2 * q + h], wq[v][0]), false);
          sv[q][v] = f2{o[0], o[1]};
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        if constexpr (MODE == 5) {
          acc += sv[q][0] + sv[q][1] + sv[q][2] + sv[q][3];
        } else {
          f2 den;
          acc += softmax_pair_log2<NV, false>(sv[q], den);
          dmx = vmax3f(dmx, den.x, den.y);
          dmn = vmin3f(dmn, den.x, den.y);
        }
      }
    }
    acc.x += dmx + dmn;
  } else if constexpr (MODE == 2) {
#pragma unroll
    for (int v = 0; v < NV; ++v) acc += wp[v][0] + wp[v][1] + f2{float(fx[v]), float(fy[v])};
  } else {
    // 4 tap slots of 4 channels, the same registers for every view and group but opaque to
    // the compiler at each use (the real kernel reads them from LDS)
    uint4 s0 = seed[threadIdx.x & 63], s1 = seed[64 + (threadIdx.x & 63)];
    uint4 s2 = seed[128 + (threadIdx.x & 63)], s3 = seed[192 + (threadIdx.x & 63)];
#pragma unroll 1
    for (int c0 = 0; c0 < C; c0 += 4) {
      f2 sv[2][NV];
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        asm volatile("" : "+v"(s0.x), "+v"(s0.y), "+v"(s0.z), "+v"(s0.w), "+v"(s1.x), "+v"(s1.y), "+v"(s1.z),
                     "+v"(s1.w), "+v"(s2.x), "+v"(s2.y), "+v"(s2.z), "+v"(s2.w), "+v"(s3.x), "+v"(s3.y),
                     "+v"(s3.z), "+v"(s3.w));
        const f2 w0 = splat<0>(wp[v][0]), w1 = splat<1>(wp[v][0]), w2 = splat<0>(wp[v][1]), w3 = splat<1>(wp[v][1]);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const f2 a = q ? hi2(s0) : lo2(s0), bq = q ? hi2(s1) : lo2(s1);
          const f2 cq = q ? hi2(s2) : lo2(s2), d = q ? hi2(s3) : lo2(s3);
          sv[q][v] = pk_fma(d, w3, pk_fma(cq, w2, pk_fma(bq, w1, a * w0)));
        }
      }
      f2 cf[NV];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f2 o = MODE == 1 ? aggregate_pair<MVN_AGG_SUM>(sv[q], cf) : aggregate_pair<MVN_AGG_SOFTMAX>(sv[q], cf);
        acc += o;
      }
    }
  }
  if (gid < 0x7fffffff) out[gid] = acc.x + acc.y;
}

}  // namespace

extern "C" int floor_run(int mode, const float* P, const float* coords, const void* seed, float* out, int B,
                         int nvox, int H, int W, int C, hipStream_t s) {
  const int n = B * nvox;
  if (n % 256) return -1;
  const dim3 g(n / 256), blk(256);
  const uint4* sd = static_cast<const uint4*>(seed);
  switch (mode) {
    case 0: floor_kernel<0><<<g, blk, 0, s>>>(P, coords, sd, out, nvox, H, W, C); break;
    case 1: floor_kernel<1><<<g, blk, 0, s>>>(P, coords, sd, out, nvox, H, W, C); break;
    case 2: floor_kernel<2><<<g, blk, 0, s>>>(P, coords, sd, out, nvox, H, W, C); break;
    case 3: floor_kernel<3><<<g, blk, 0, s>>>(P, coords, sd, out, nvox, H, W, C); break;
    case 4: floor_kernel<4><<<g, blk, 0, s>>>(P, coords, sd, out, nvox, H, W, C); break;
    case 5: floor_kernel<5><<<g, blk, 0, s>>>(P, coords, sd, out, nvox, H, W, C); break;
    case 6: floor_kernel<6><<<g, blk, 0, s>>>(P, coords, sd, out, nvox, H, W, C); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
