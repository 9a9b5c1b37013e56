// Tiled, LDS-staged unprojection for gfx950 — the production kernel behind mvn_unproject.
//
// Same contract and numerics as the reference op (mvn/utils/op.py:99-163) and the simple
// kernels in unproject.hip; what changes is where the bilinear taps come from.
//
// Why: a lane per voxel gathering its 4 taps per (view, channel) straight from the NCHW
// maps touches a different cache line per lane (neighbouring z-voxels project ~1.6 px
// apart, i.e. onto different image rows), so the gathers run at L1/L2 request rate, not
// bandwidth.  Here a block owns a compact voxel tile (TX x TY x TZ).  For every view it
//   1. projects its voxels once (geometry kept in registers),
//   2. reduces the bounding box of their bilinear footprints (+1 px each way),
//   3. stages that footprint for G channels into LDS channels-last — 16 bytes per pixel
//      (4 f32 / 8 bf16 channels) — reading the NCHW rows coalesced and writing ZERO for
//      pixels outside the image, which is exactly ATen's padding_mode='zeros',
//   4. samples: 4 x ds_read_b128 per voxel-view give the 4 taps of G channels.
// Views are aggregated in registers (max-first softmax: one exp per sample) and each
// channel plane of the tile is written with z-consecutive lanes.  Blocks are remapped
// XCD-contiguously so a frame's maps stay in one XCD's L2 and z-neighbouring tiles
// (which share output lines) run back to back on the same L2.
//
// Footprints that do not fit the LDS budget together are staged in several passes; only a
// single footprint larger than the whole budget sends its block to direct global gathers.
#include <stdlib.h>

#include "unproject_common.hpp"

namespace mvn {
namespace unproj {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / kWave;
constexpr int kSlots = 2048;          // 16-byte LDS pixel slots (32 KiB); slot 0 is a zero pad

template <int NV> struct TileShape;                 // tile dims and voxels per thread
template <> struct TileShape<4> { static constexpr int TX = 8, TY = 8, TZ = 8, VPT = 2; };
template <> struct TileShape<8> { static constexpr int TX = 4, TY = 8, TZ = 8, VPT = 1; };

// 16-byte slot <-> G floats
__device__ __forceinline__ void unpack(const uint4& q, float (&v)[4]) {
  v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
}
__device__ __forceinline__ void unpack(const uint4& q, float (&v)[8]) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

template <typename TIn> __device__ __forceinline__ uint32_t raw_bits(TIn v);
template <> __device__ __forceinline__ uint32_t raw_bits<float>(float v) { return __float_as_uint(v); }
template <> __device__ __forceinline__ uint32_t raw_bits<uint16_t>(uint16_t v) { return v; }

// One voxel, all channels, taps gathered from global memory (LDS-overflow fallback).
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
          r = (v == 0 || sv > r) ? sv : r;
        } else if constexpr (AGG == MVN_AGG_CONF) {
          const float p = sv * cfb[size_t(v) * C + c];
          r = v == 0 ? p : r + p;
        } else if (pass == 0) {
          m = v == 0 ? sv : fmaxf(m, sv);
        } else {
          const float e = __expf(sv - m);
          den += e;
          r = __builtin_fmaf(sv, e, r);
        }
      }
    }
    if constexpr (AGG == MVN_AGG_SOFTMAX) r = r / den;
    store_elem(ov + size_t(c) * nvox, r);
  }
}

template <int AGG, typename TIn, typename TOut, int NV>
__global__ __launch_bounds__(kThreads) void unproject_tiled(
    const TIn* __restrict__ feat, const float* __restrict__ P, const float* __restrict__ coords,
    const float* __restrict__ conf, TOut* __restrict__ out, int B, int N, int C, int H, int W, int Vx,
    int Vy, int Vz, int align_corners, int budget) {
  using S = TileShape<NV>;
  constexpr int TX = S::TX, TY = S::TY, TZ = S::TZ, VPT = S::VPT;
  static_assert(TX * TY * TZ == kThreads * VPT, "tile must give every thread VPT voxels");
  constexpr int G = 16 / int(sizeof(TIn));            // channels per 16-byte slot

  __shared__ uint4 stage[kSlots];
  __shared__ int red[kWaves][NV][4];
  __shared__ int region[NV][4];                       // xs, ys, bw, first slot (-1: global fallback)
  __shared__ int region_end[NV];
  __shared__ int region_pass[NV];
  __shared__ float region_inv_bw[NV];
  __shared__ int block_info[1];                       // number of LDS passes, -1 = global fallback

  // ---- which tile (XCD-contiguous order, z-tiles fastest) -------------------------
  const int nTx = (Vx + TX - 1) / TX, nTy = (Vy + TY - 1) / TY, nTz = (Vz + TZ - 1) / TZ;
  const int nblk = B * nTx * nTy * nTz;
  int L = xcd_remap(blockIdx.x, nblk);
  const int tz = L % nTz; L /= nTz;
  const int ty = L % nTy; L /= nTy;
  const int tx = L % nTx;
  const int b = L / nTx;

  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int lz = t % TZ, ly = (t / TZ) % TY, lx = t / (TZ * TY);
  const int nvox = Vx * Vy * Vz;
  const size_t HW = size_t(H) * W;
  const float* Pb = P + size_t(b) * N * 12;

  if (t == 0) stage[0] = make_uint4(0, 0, 0, 0);

  // ---- voxels of this thread ------------------------------------------------------
  int vox[VPT];
  bool act[VPT];
  float cx[VPT], cy[VPT], cz[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int X = tx * TX + lx + k * (TX / VPT), Y = ty * TY + ly, Z = tz * TZ + lz;
    act[k] = (X < Vx) & (Y < Vy) & (Z < Vz);
    vox[k] = act[k] ? (X * Vy + Y) * Vz + Z : 0;
    const float* cp = coords + (size_t(b) * nvox + vox[k]) * 3;
    cx[k] = cp[0]; cy[k] = cp[1]; cz[k] = cp[2];
  }

  // ---- per-view geometry: footprint base pixel, weights, "samples the image" flag --
  int fx[NV][VPT], fy[NV][VPT];
  float w[NV][VPT][4];
  bool has[NV][VPT];
  int bb[NV][4];                                      // thread-local xmin, xmax, ymin, ymax
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    bb[v][0] = INT_MAX; bb[v][1] = INT_MIN; bb[v][2] = INT_MAX; bb[v][3] = INT_MIN;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      has[v][k] = false;
      fx[v][k] = fy[v][k] = 0;
      w[v][k][0] = w[v][k][1] = w[v][k][2] = w[v][k][3] = 0.f;
      if (v < N) {
        const Proj p = project(Pb + v * 12, cx[k], cy[k], cz[k], H, W, align_corners);
        const float fx0 = floorf(p.ix), fy0 = floorf(p.iy);
        // at least one of the 4 taps lies inside the image, and the voxel is in front
        const bool h = act[k] & !p.invalid & (fx0 >= -1.f) & (fx0 < float(W)) & (fy0 >= -1.f) & (fy0 < float(H));
        if (h) {
          const float tx_ = p.ix - fx0, sx_ = 1.f - tx_, ty_ = p.iy - fy0, sy_ = 1.f - ty_;
          w[v][k][0] = sy_ * sx_; w[v][k][1] = sy_ * tx_; w[v][k][2] = ty_ * sx_; w[v][k][3] = ty_ * tx_;
          fx[v][k] = int(fx0); fy[v][k] = int(fy0);
          bb[v][0] = min(bb[v][0], fx[v][k]); bb[v][1] = max(bb[v][1], fx[v][k]);
          bb[v][2] = min(bb[v][2], fy[v][k]); bb[v][3] = max(bb[v][3], fy[v][k]);
        }
        has[v][k] = h;
      }
    }
  }

  // ---- block bounding boxes -> LDS regions ------------------------------------------
#pragma unroll
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      bb[v][0] = min(bb[v][0], __shfl_xor(bb[v][0], o, kWave));
      bb[v][1] = max(bb[v][1], __shfl_xor(bb[v][1], o, kWave));
      bb[v][2] = min(bb[v][2], __shfl_xor(bb[v][2], o, kWave));
      bb[v][3] = max(bb[v][3], __shfl_xor(bb[v][3], o, kWave));
    }
    if (lane == 0) {
      red[wid][v][0] = bb[v][0]; red[wid][v][1] = bb[v][1]; red[wid][v][2] = bb[v][2]; red[wid][v][3] = bb[v][3];
    }
  }
  __syncthreads();
  if (t == 0) {
    // Pack the views' footprints into LDS passes (first fit in view order).  Normally all
    // N views fit one pass; a close camera needs more passes, never a slow path.  Only a
    // single footprint larger than the whole budget sends the block to global gathers.
    int next = 1, pass = 0;                           // slot 0 stays a zero pad
    bool too_big = false;
    for (int v = 0; v < NV; ++v) {
      if (v >= N) break;
      int x0 = INT_MAX, x1 = INT_MIN, y0 = INT_MAX, y1 = INT_MIN;
      for (int q = 0; q < kWaves; ++q) {
        x0 = min(x0, red[q][v][0]); x1 = max(x1, red[q][v][1]);
        y0 = min(y0, red[q][v][2]); y1 = max(y1, red[q][v][3]);
      }
      int bw = 0, bh = 0;
      if (x0 <= x1) { bw = x1 - x0 + 2; bh = y1 - y0 + 2; }   // +1 px for the east / south taps
      const long long area = (long long)bw * bh;
      if (area > budget - 1) too_big = true;
      if (next + area > budget) { ++pass; next = 1; }
      region[v][0] = x0; region[v][1] = y0; region[v][2] = bw; region[v][3] = next;
      region_end[v] = next + int(area);
      region_pass[v] = pass;
      region_inv_bw[v] = bw > 0 ? 1.f / float(bw) : 0.f;
      next += int(area);
    }
    block_info[0] = too_big ? -1 : pass + 1;
  }
  __syncthreads();

  int rx[NV], ry[NV], rbw[NV], rbase[NV], rend[NV], rpass[NV];
  float rinv[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {       // block-uniform: keep in SGPRs
    rx[v] = __builtin_amdgcn_readfirstlane(region[v][0]);
    ry[v] = __builtin_amdgcn_readfirstlane(region[v][1]);
    rbw[v] = __builtin_amdgcn_readfirstlane(region[v][2]);
    rbase[v] = __builtin_amdgcn_readfirstlane(region[v][3]);
    rend[v] = __builtin_amdgcn_readfirstlane(region_end[v]);
    rpass[v] = __builtin_amdgcn_readfirstlane(region_pass[v]);
    rinv[v] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(region_inv_bw[v])));
  }
  const int npass = __builtin_amdgcn_readfirstlane(block_info[0]);

  const TIn* fb = feat + size_t(b) * N * C * HW;
  const float* cfb = conf ? conf + size_t(b) * N * C : nullptr;

  if (npass < 0) {
    // Pathological geometry (one view's footprint exceeds the whole LDS budget): the block
    // gathers straight from global memory instead; same arithmetic and op order.
#pragma unroll
    for (int k = 0; k < VPT; ++k)
      if (act[k])
        gather_voxel<AGG, TIn, TOut>(fb, Pb, cfb, out + size_t(b) * C * nvox + vox[k], nvox, N, C, H, W,
                                     cx[k], cy[k], cz[k], align_corners);
    return;
  }

  // slot of each voxel-view's north-west tap
  int slot[NV][VPT];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int k = 0; k < VPT; ++k)
      slot[v][k] = rbase[v] + (fy[v][k] - ry[v]) * rbw[v] + (fx[v][k] - rx[v]);

  for (int c0 = 0; c0 < C; c0 += G) {
    float sv[VPT][G][NV];
    for (int pass = 0; pass < npass; ++pass) {
      // ---- stage this pass's footprints for channels [c0, c0 + G) -----------------
      int total = 1;
#pragma unroll
      for (int v = 0; v < NV; ++v) if (v < N && rpass[v] == pass) total = max(total, rend[v]);
      for (int idx = 1 + t; idx < total; idx += kThreads) {
        int v = 0;
#pragma unroll
        for (int u = 0; u < NV; ++u)
          if (u < N && rpass[u] == pass && idx >= rbase[u]) v = u;
        const int li = idx - rbase[v];
        const int py = int((float(li) + 0.5f) * rinv[v]);
        const int px = li - py * rbw[v];
        const int gx = rx[v] + px, gy = ry[v] + py;
        const bool in = (gx >= 0) & (gx < W) & (gy >= 0) & (gy < H);
        const TIn* src = fb + (size_t(v) * C + c0) * HW + (in ? size_t(gy) * W + gx : 0);
        uint32_t bits[G];
#pragma unroll
        for (int k = 0; k < G; ++k) bits[k] = (in && c0 + k < C) ? raw_bits<TIn>(src[size_t(k) * HW]) : 0u;
        uint4 q;
        if constexpr (G == 4) {
          q = make_uint4(bits[0], bits[1], bits[2], bits[3]);
        } else {
          q = make_uint4(bits[0] | (bits[1] << 16), bits[2] | (bits[3] << 16), bits[4] | (bits[5] << 16),
                         bits[6] | (bits[7] << 16));
        }
        stage[idx] = q;
      }
      __syncthreads();

      // ---- sample this pass's views -----------------------------------------------
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if (v >= N || rpass[v] != pass) continue;
#pragma unroll
        for (int k = 0; k < VPT; ++k) {
          float a[G], bq[G], cq[G], d[G];
          if (has[v][k]) {
            const int o = slot[v][k];
            unpack(stage[o], a);
            unpack(stage[o + 1], bq);
            unpack(stage[o + rbw[v]], cq);
            unpack(stage[o + rbw[v] + 1], d);
          } else {
#pragma unroll
            for (int ch = 0; ch < G; ++ch) a[ch] = bq[ch] = cq[ch] = d[ch] = 0.f;
          }
#pragma unroll
          for (int ch = 0; ch < G; ++ch)
            sv[k][ch][v] = __builtin_fmaf(d[ch], w[v][k][3], __builtin_fmaf(cq[ch], w[v][k][2],
                           __builtin_fmaf(bq[ch], w[v][k][1], a[ch] * w[v][k][0])));
        }
      }
      __syncthreads();                                // stage[] is rewritten next
    }

    // ---- aggregate over views, store ------------------------------------------------
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
#pragma unroll
      for (int ch = 0; ch < G; ++ch) {
        const int c = c0 + ch;
        if (c < C) {
          const float r = aggregate<AGG, NV>(sv[k][ch], N, cfb ? cfb + c : nullptr, C);
          if (act[k]) store_elem(out + (size_t(b) * C + c) * nvox + vox[k], r);
        }
      }
    }
  }
}

}  // namespace

template <int AGG, typename TIn, typename TOut>
int launch_tiled(const void* feat, const float* P, const float* coords, const float* conf, void* out, int B,
                 int N, int C, int H, int W, int Vx, int Vy, int Vz, int align_corners, hipStream_t s) {
  // LDS slot budget per pass; MVN_UNPROJECT_LDS_SLOTS lowers it (tests force the multi-pass
  // and global-gather paths with it).
  int budget = kSlots;
  if (const char* e = getenv("MVN_UNPROJECT_LDS_SLOTS")) budget = max(2, min(kSlots, atoi(e)));
  auto blocks = [&](auto shape) {
    using S = decltype(shape);
    return (long long)B * ((Vx + S::TX - 1) / S::TX) * ((Vy + S::TY - 1) / S::TY) * ((Vz + S::TZ - 1) / S::TZ);
  };
  if (N <= 4) {
    const long long nb = blocks(TileShape<4>{});
    if (nb > INT_MAX) return MVN_ERR_SHAPE;
    unproject_tiled<AGG, TIn, TOut, 4><<<int(nb), kThreads, 0, s>>>(
        static_cast<const TIn*>(feat), P, coords, conf, static_cast<TOut*>(out), B, N, C, H, W, Vx, Vy, Vz,
        align_corners, budget);
  } else {
    const long long nb = blocks(TileShape<8>{});
    if (nb > INT_MAX) return MVN_ERR_SHAPE;
    unproject_tiled<AGG, TIn, TOut, 8><<<int(nb), kThreads, 0, s>>>(
        static_cast<const TIn*>(feat), P, coords, conf, static_cast<TOut*>(out), B, N, C, H, W, Vx, Vy, Vz,
        align_corners, budget);
  }
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

#define MVN_INSTANTIATE(AGG)                                                                                   \
  template int launch_tiled<AGG, float, float>(const void*, const float*, const float*, const float*, void*,    \
                                               int, int, int, int, int, int, int, int, int, hipStream_t);       \
  template int launch_tiled<AGG, uint16_t, uint16_t>(const void*, const float*, const float*, const float*,     \
                                                     void*, int, int, int, int, int, int, int, int, int,        \
                                                     hipStream_t);                                              \
  template int launch_tiled<AGG, uint16_t, float>(const void*, const float*, const float*, const float*, void*, \
                                                  int, int, int, int, int, int, int, int, int, hipStream_t);
MVN_INSTANTIATE(MVN_AGG_SUM)
MVN_INSTANTIATE(MVN_AGG_MAX)
MVN_INSTANTIATE(MVN_AGG_SOFTMAX)
MVN_INSTANTIATE(MVN_AGG_CONF)
#undef MVN_INSTANTIATE

}  // namespace unproj
}  // namespace mvn
