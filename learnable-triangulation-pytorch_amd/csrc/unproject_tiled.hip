// Tiled, LDS-staged unprojection for gfx950 — the production kernel behind mvn_unproject.
//
// Same contract and numerics as the reference op (mvn/utils/op.py:99-163) and the simple
// kernels in unproject.hip; what changes is where the bilinear taps come from.
//
// Why: a lane per voxel gathering its 4 taps per (view, channel) straight from the NCHW
// maps touches a different cache line per lane (neighbouring z-voxels project ~1.6 px
// apart, i.e. onto different image rows), so gathers run at L1/L2 request rate, not
// bandwidth.  Here a block owns a compact voxel tile (4x8x16 for up to 4 views, z
// fastest so that a wave's stores are 64-byte runs).  Once per block it
//   1. projects its voxels in every view (geometry kept in registers),
//   2. reduces per view the bounding box of the bilinear footprints (+1 px each way; DPP
//      wave reductions) and lays the N boxes out in LDS channels-last, 16 bytes per pixel
//      (4 f32 channels; bf16 maps are widened when staged), with an odd row pitch so that
//      z-neighbouring lanes spread over banks,
//   3. turns every LDS pixel slot this thread stages into one byte offset into the
//      frame's NCHW maps (or an out-of-range offset for pixels outside the image).
// Then per group of G channels staging is only buffer loads — whose hardware range check
// returns 0 for out-of-range offsets, which is exactly ATen's padding_mode='zeros' — and
// one ds_write_b128 per pixel, and sampling is 4 ds_read_b128 per voxel-view.  The next
// group's loads are in flight while the current group is sampled (two LDS buffers, one
// barrier per group).  Views are aggregated in registers and each channel plane is
// stored through a buffer descriptor (z-consecutive lanes).  Block order: see the
// comment at the tile index (balanced over frames per XCD).
//
// Footprints that do not fit one LDS buffer together are staged in several passes
// (slower, unpipelined); a single footprint larger than a whole buffer (a camera inside
// the cuboid) sends its block to direct global gathers.
#include <climits>
#include <utility>

#include "unproject_common.hpp"

namespace mvn {
namespace unproj {
namespace {

// 4 views: skip, per wave, staged slots past the tile's footprint (A/B r04: 194.2 -> 191.1 us
// at config 2, bit-identical); 8 views stage every slot a thread owns (1,031 vs 1,061 us).


// Tile of voxels per block (z fastest: a wave's output stores are 16-voxel = 64-byte runs
// of a channel plane) and 16-byte LDS pixel slots per staging buffer (two per block; the
// last 2 slots of each hold zeros: the taps of voxel-views that sample nothing point there).
//   4 views: 4x8x16 tile, 512 threads, 2048 slots = 2 x 32 KiB (footprints of such tiles
//            take ~2.2 slots / voxel)
//   8 views: 4x8x16 tile, 512 threads, 4096 8-byte slots (2 channels) per buffer
template <int NV> struct TileShape;
// WAVES: waves per SIMD the register allocation must allow (4: two 512-thread blocks per CU).
template <> struct TileShape<4> { static constexpr int TX = 4, TY = 8, TZ = 16, THREADS = 512, SLOTS = 2048, G = 4, WAVES = 4; };
// 8 views: 8-byte slots (2 channels) so that the two 4,096-slot buffers take 64 KiB and two
// blocks share a CU (one block's prologue / barriers overlap the other's staging and
// sampling): config 4 1,278 -> 1,027 us at 16 frames, bit-identical (A/B).
// The 4-view kernel keeps 16-byte slots (2-channel slots at 6 waves/SIMD: no gain).
template <> struct TileShape<8> {
  static constexpr int TX = 4, TY = 8, TZ = 16, THREADS = 512, SLOTS = 4096, G = 2, WAVES = 4;
};

template <typename T> __device__ __forceinline__ uint32_t buf_load(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s);
template <> __device__ __forceinline__ uint32_t buf_load<float>(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, v, s, 0);
}
template <> __device__ __forceinline__ uint32_t buf_load<uint16_t>(__amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
  return __builtin_amdgcn_raw_buffer_load_b16(r, v, s, 0);
}

template <typename T> __device__ __forceinline__ void buf_store(float x, __amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s);
// f32 planes non-temporal (A/B: 8 views, step 1,195 -> 1,179 us at 16 frames); XCD slabs from
// 16 frames on
constexpr int kTiledStorePolicyF32 = 2, kTiledXcdMinFrames = 16;
template <> __device__ __forceinline__ void buf_store<float>(float x, __amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, v, s, kTiledStorePolicyF32);
}
template <> __device__ __forceinline__ void buf_store<uint16_t>(float x, __amdgpu_buffer_rsrc_t r, uint32_t v, uint32_t s) {
  __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, static_cast<__bf16>(x)), r, v, s, 0);
}

// LDS slots hold G f32 channels whatever the input dtype (G = 4: 16-byte slots; G = 2:
// 8-byte slots, half the LDS per block, so that two 8-view blocks share a CU): bf16 maps
// are widened once when staged (each staged pixel is read ~7 times by the taps), not per tap.
template <int G> struct SlotT;
template <> struct SlotT<4> { using type = uint4; };
template <> struct SlotT<2> { using type = uint2; };
__device__ __forceinline__ void unpack(const uint4& q, float (&v)[4]) {
  v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
}
__device__ __forceinline__ void unpack(const uint2& q, float (&v)[2]) {
  v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y);
}
template <typename TIn> __device__ __forceinline__ uint4 pack(const uint32_t (&b)[4]) {
  if constexpr (sizeof(TIn) == 4) return make_uint4(b[0], b[1], b[2], b[3]);
  else return make_uint4(b[0] << 16, b[1] << 16, b[2] << 16, b[3] << 16);   // bf16 -> f32 bits
}
template <typename TIn> __device__ __forceinline__ uint2 pack(const uint32_t (&b)[2]) {
  if constexpr (sizeof(TIn) == 4) return make_uint2(b[0], b[1]);
  else return make_uint2(b[0] << 16, b[1] << 16);
}

// View aggregation, fast form for the staged path.  sum / max / conf are the reference's
// sequential f32 op order (bit-exact); softmax is max-first with exp2 and one reciprocal.
template <int AGG, int NV>
__device__ __forceinline__ float aggregate_fast(const float (&s)[NV], int N, const float* __restrict__ cf, int cstride) {
  if constexpr (AGG != MVN_AGG_SOFTMAX) {
    return aggregate<AGG, NV>(s, N, cf, cstride);
  } else {
    constexpr float kLog2e = 1.4426950408889634f;
    float m = s[0];
#pragma unroll
    for (int v = 1; v < NV; ++v) if (v < N) m = fmaxf(m, s[v]);
    const float ml = m * kLog2e;
    float den = 0.f, num = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (v < N) {
        const float e = __builtin_amdgcn_exp2f(__builtin_fmaf(s[v], kLog2e, -ml));
        den += e;
        num = __builtin_fmaf(s[v], e, num);
      }
    return num * __builtin_amdgcn_rcpf(den);
  }
}

// The LDS region (view) a staged slot index falls in, for one pass.  A select chain over
// the views: indexing the per-view arrays with a per-lane view number would force them
// into scratch memory.
struct SlotRegion {
  int v, x, y, bw, pitch, base;
  float inv;
};
template <int NV>
__device__ __forceinline__ SlotRegion find_region(int idx, int pass, int N, const int (&rx)[NV], const int (&ry)[NV],
                                                  const int (&rbw)[NV], const int (&rpitch)[NV],
                                                  const int (&rbase)[NV], const int (&rpass)[NV],
                                                  const float (&rinv)[NV]) {
  SlotRegion q{0, rx[0], ry[0], rbw[0], rpitch[0], rbase[0], rinv[0]};
#pragma unroll
  for (int u = 0; u < NV; ++u)
    if (u < N && rpass[u] == pass && idx >= rbase[u]) q = SlotRegion{u, rx[u], ry[u], rbw[u], rpitch[u], rbase[u], rinv[u]};
  return q;
}

// NV = views held in registers (4 or 8); EXACT: the launch has exactly NV views, so every
// per-view guard is a compile-time constant (no selects in the sampling / aggregation).
template <int AGG, typename TIn, typename TOut, int NV, bool EXACT>
__global__ __launch_bounds__(TileShape<NV>::THREADS)
__attribute__((amdgpu_waves_per_eu(TileShape<NV>::WAVES))) void unproject_tiled(
    const TIn* __restrict__ feat, const float* __restrict__ P, const float* __restrict__ coords,
    const float* __restrict__ cub, int transfer, const float* __restrict__ conf, TOut* __restrict__ out, int B,
    int n_views, int C, int H, int W, int Vx, int Vy, int Vz, int align_corners, int budget, int out_cl) {
  const int N = EXACT ? NV : n_views;
  using S = TileShape<NV>;
  constexpr int TX = S::TX, TY = S::TY, TZ = S::TZ, kThreads = S::THREADS, kBuf = S::SLOTS;
  static_assert(TX * TY * TZ == kThreads, "one voxel per thread");
  constexpr int kWaves = kThreads / kWave;
  constexpr int G = S::G;                             // f32 channels per LDS slot
  using Slot = typename SlotT<G>::type;
  constexpr uint32_t kSlotB = sizeof(Slot);
  constexpr int kZeroSlot = kBuf - 2;
  constexpr int MS = kBuf / kThreads;                 // staged slots per thread (max)

  __shared__ Slot stage[2 * kBuf];
  __shared__ int red[kWaves][NV][4];
  __shared__ int region[NV][6];                       // xs, ys, bw, pitch, first slot, end slot
  __shared__ int region_pass[NV];
  __shared__ float region_inv_pitch[NV];
  __shared__ int block_info[2];                       // passes (-1: global fallback), slots of pass 0

  // ---- which tile (z-tiles fastest) -------------------------------------------------
  const int nTx = (Vx + TX - 1) / TX, nTy = (Vy + TY - 1) / TY, nTz = (Vz + TZ - 1) / TZ;
  // Block order.  Hardware deals blocks round-robin over the 8 XCDs.  Few frames (< 16):
  // plain order, so every XCD gets an equal mix of every frame — an XCD-contiguous order
  // would give each XCD whole frames and the most expensive frame would set the time
  // (measured: 10-15 % slower at 8 frames).  Many frames: every XCD gets the same x-slab
  // of every frame (balanced over frames, neighbouring tiles share the XCD's L2).
  int L = int(blockIdx.x);
  {
    const int nf = nTx * nTy * nTz;
    if (B >= kTiledXcdMinFrames && nf % 8 == 0) {
      const int xcd = int(blockIdx.x) % 8, k = int(blockIdx.x) / 8, slab = nf / 8;
      L = (k / slab) * nf + xcd * slab + k % slab;
    }
  }
  const int tz = L % nTz; L /= nTz;
  const int ty = L % nTy; L /= nTy;
  const int tx = L % nTx;
  const int b = L / nTx;

  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int nvox = Vx * Vy * Vz;
  const int HW = H * W;
  const float* Pb = P + size_t(b) * N * 12;
  const TIn* fb = feat + size_t(b) * N * C * HW;
  const float* cfb = conf ? conf + size_t(b) * N * C : nullptr;

  if (t < 4) stage[(t >> 1) * kBuf + kZeroSlot + (t & 1)] = Slot{};

  // ---- this thread's voxel -----------------------------------------------------------
  const int X = tx * TX + t / (TZ * TY), Y = ty * TY + (t / TZ) % TY, Z = tz * TZ + t % TZ;
  const bool act = (X < Vx) & (Y < Vy) & (Z < Vz);
  const int vox = act ? (X * Vy + Y) * Vz + Z : 0;
  float cx, cy, cz;
  if (cub) {                          // block-uniform: formed in-kernel, bit-identical to the volume
    float o[3];
    cuboid_coord(cub + b * MVN_CUBOID_FLOATS, Vx, X, Y, Z, transfer, o);
    cx = o[0]; cy = o[1]; cz = o[2];
  } else {
    const float* cp = coords + (size_t(b) * nvox + vox) * 3;
    cx = cp[0]; cy = cp[1]; cz = cp[2];
  }

  // ---- per-view geometry: footprint base pixel, weights, "samples the image" flag --
  int fx[NV], fy[NV];
  float w[NV][4];
  bool has[NV];
  bool lane_fast = true;
#pragma unroll
  for (int v = 0; v < NV; ++v)
    if (v < N) lane_fast &= div_core_safe(homog(Pb + v * 12, cx, cy, cz));
  // wave-uniform choice of the division form (bit-identical results either way)
  const bool wave_fast = __builtin_amdgcn_ballot_w64(!lane_fast) == 0;
  const Recip rH = recip_refined(float(H)), rW = recip_refined(float(W));
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    has[v] = false;
    fx[v] = fy[v] = 0;
    w[v][0] = w[v][1] = w[v][2] = w[v][3] = 0.f;
    if (v < N) {
      const Homog hp = homog(Pb + v * 12, cx, cy, cz);
      const Proj p = (EXACT && wave_fast) ? project_h<true>(hp, H, W, align_corners, rH, rW)
                                          : project_h<false>(hp, H, W, align_corners, rH, rW);
      const float fx0 = floorf(p.ix), fy0 = floorf(p.iy);
      // at least one of the 4 taps lies inside the image, and the voxel is in front
      const bool h = act & !p.invalid & (fx0 >= -1.f) & (fx0 < float(W)) & (fy0 >= -1.f) & (fy0 < float(H));
      if (h) {
        const float tx_ = p.ix - fx0, sx_ = 1.f - tx_, ty_ = p.iy - fy0, sy_ = 1.f - ty_;
        w[v][0] = sy_ * sx_; w[v][1] = sy_ * tx_; w[v][2] = ty_ * sx_; w[v][3] = ty_ * tx_;
        fx[v] = int(fx0); fy[v] = int(fy0);
      }
      has[v] = h;
    }
  }

  // ---- block bounding boxes -> LDS regions ------------------------------------------
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    if (v >= N) break;
    const int x0 = wave_min_u(has[v] ? fx[v] : INT_MAX), x1 = wave_max_u(has[v] ? fx[v] : INT_MIN);
    const int y0 = wave_min_u(has[v] ? fy[v] : INT_MAX), y1 = wave_max_u(has[v] ? fy[v] : INT_MIN);
    if (lane == 0) { red[wid][v][0] = x0; red[wid][v][1] = x1; red[wid][v][2] = y0; red[wid][v][3] = y1; }
  }
  __syncthreads();
  if (t == 0) {
    int next = 0, pass = 0, slots0 = 0;
    bool too_big = false;
    budget = min(budget, kZeroSlot);
    for (int v = 0; v < NV; ++v) {
      if (v >= N) break;
      int x0 = INT_MAX, x1 = INT_MIN, y0 = INT_MAX, y1 = INT_MIN;
      for (int q = 0; q < kWaves; ++q) {
        x0 = min(x0, red[q][v][0]); x1 = max(x1, red[q][v][1]);
        y0 = min(y0, red[q][v][2]); y1 = max(y1, red[q][v][3]);
      }
      int bw = 0, bh = 0;
      if (x0 <= x1) { bw = x1 - x0 + 2; bh = y1 - y0 + 2; }   // +1 px for the east / south taps
      const int pitch = bw | 1;                                 // odd: spreads rows over banks
      const long long area = (long long)pitch * bh;
      if (area > budget) too_big = true;
      if (next + area > budget) { ++pass; next = 0; }
      region[v][0] = x0; region[v][1] = y0; region[v][2] = bw; region[v][3] = pitch;
      region[v][4] = next; region[v][5] = next + int(area);
      region_pass[v] = pass;
      region_inv_pitch[v] = 1.f / float(pitch);
      next += int(area);
      if (pass == 0) slots0 = next;
    }
    block_info[0] = too_big ? -1 : pass + 1;
    block_info[1] = slots0;
  }
  __syncthreads();

  int rx[NV], ry[NV], rbw[NV], rpitch[NV], rbase[NV], rend[NV], rpass[NV];
  float rinv[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {       // block-uniform: keep in SGPRs
    rx[v] = __builtin_amdgcn_readfirstlane(region[v][0]);
    ry[v] = __builtin_amdgcn_readfirstlane(region[v][1]);
    rbw[v] = __builtin_amdgcn_readfirstlane(region[v][2]);
    rpitch[v] = __builtin_amdgcn_readfirstlane(region[v][3]);
    rbase[v] = __builtin_amdgcn_readfirstlane(region[v][4]);
    rend[v] = __builtin_amdgcn_readfirstlane(region[v][5]);
    rpass[v] = __builtin_amdgcn_readfirstlane(region_pass[v]);
    rinv[v] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(region_inv_pitch[v])));
  }
  const int npass = __builtin_amdgcn_readfirstlane(block_info[0]);

  if (npass < 0) {
    // A single footprint exceeds the LDS buffer: gather straight from global memory.
    if (act)
      gather_voxel<AGG, TIn, TOut>(fb, Pb, cfb, out + size_t(b) * C * nvox + (out_cl ? size_t(vox) * C : vox),
                                   out_cl ? 1 : nvox, N, C, H, W, cx, cy, cz,
                                   align_corners);
    return;
  }

  const __amdgpu_buffer_rsrc_t frs = make_rsrc(fb, uint32_t(size_t(N) * C * HW * sizeof(TIn)));
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(out + size_t(b) * C * nvox, uint32_t(size_t(C) * nvox * sizeof(TOut)));
  const uint32_t ooff = act ? uint32_t(vox) * uint32_t(sizeof(TOut)) : kOob;

  // LDS byte offsets of each view's north-west and south-west taps (buffer 0)
  uint32_t anw[NV], asw[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int slot = rbase[v] + (fy[v] - ry[v]) * rpitch[v] + (fx[v] - rx[v]);
    anw[v] = uint32_t(has[v] ? slot : kZeroSlot) * kSlotB;
    asw[v] = uint32_t(has[v] ? slot + rpitch[v] : kZeroSlot) * kSlotB;
  }

  // sample the views staged in an LDS buffer (ONE_PASS: all of them; else those of `pass`)
  auto sample_views = [&](const char* buf, auto one_pass, int pass, float (&sv)[G][NV]) __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (v >= N) continue;
      if (!decltype(one_pass)::value && rpass[v] != pass) continue;
      // branch-free: voxel-views that sample nothing read the zero slots with zero weights
      float a[G], bq[G], cq[G], d[G];
      unpack(*reinterpret_cast<const Slot*>(buf + anw[v]), a);
      unpack(*reinterpret_cast<const Slot*>(buf + anw[v] + kSlotB), bq);
      unpack(*reinterpret_cast<const Slot*>(buf + asw[v]), cq);
      unpack(*reinterpret_cast<const Slot*>(buf + asw[v] + kSlotB), d);
#pragma unroll
      for (int ch = 0; ch < G; ++ch)
        sv[ch][v] = __builtin_fmaf(d[ch], w[v][3], __builtin_fmaf(cq[ch], w[v][2],
                    __builtin_fmaf(bq[ch], w[v][1], a[ch] * w[v][0])));
      if (v & 1) __builtin_amdgcn_sched_barrier(0);   // at most two views' taps in flight
    }
  };
  // out_cl (channels-last (B, Vx, Vy, Vz, C) output, C % 4 == 0; the V2V front block's input
  // layout): one 16-byte (f32) / 8-byte (bf16) store of the group's 4 channels per voxel.
  const uint32_t ooff_cl = act ? uint32_t(vox) * uint32_t(C) * uint32_t(sizeof(TOut)) : kOob;
  auto aggregate_store = [&](int c0, const float (&sv)[G][NV]) __attribute__((always_inline)) {
    if (out_cl) {
      float r[G];
#pragma unroll
      for (int ch = 0; ch < G; ++ch) r[ch] = aggregate_fast<AGG, NV>(sv[ch], N, cfb ? cfb + c0 + ch : nullptr, C);
      const uint32_t soff = uint32_t(c0) * uint32_t(sizeof(TOut));
      if constexpr (G == 2) {
        if constexpr (sizeof(TOut) == 4)
          __builtin_amdgcn_raw_buffer_store_b64(
              __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int,
                                 make_uint2(__float_as_uint(r[0]), __float_as_uint(r[1]))),
              ors, ooff_cl, soff, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b32(pack_bf16x2(r[0], r[1]), ors, ooff_cl, soff, 0);
      } else if constexpr (sizeof(TOut) == 4) {
        store_b128_padded(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int,
                               make_uint4(__float_as_uint(r[0]), __float_as_uint(r[1]), __float_as_uint(r[2]),
                                          __float_as_uint(r[3]))),
            ors, ooff_cl, soff);
      } else {
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int,
                               make_uint2(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]))),
            ors, ooff_cl, soff, 0);
      }
      return;
    }
#pragma unroll
    for (int ch = 0; ch < G; ++ch) {
      const int c = c0 + ch;
      if (c >= C) break;
      const uint32_t soff = uint32_t(c) * uint32_t(nvox) * uint32_t(sizeof(TOut));
      buf_store<TOut>(aggregate_fast<AGG, NV>(sv[ch], N, cfb ? cfb + c : nullptr, C), ors, ooff, soff);
    }
  };

  if (npass == 1) {
    // ---- fast path: one pass, staging descriptors in registers, two LDS buffers -----
    // Slot t + kThreads * i is staged by this thread.  The guard is per WAVE (scalar
    // branch): lanes past `total` load from the out-of-range offset and write zeros
    // into unused slots (never the zero slots' neighbours in use: total <= kZeroSlot).
    const int total = __builtin_amdgcn_readfirstlane(block_info[1]);
    const int wfirst = __builtin_amdgcn_readfirstlane(wid * kWave);
    uint32_t goff[MS];
#pragma unroll
    for (int i = 0; i < MS; ++i) {
      const int idx = t + kThreads * i;
      const SlotRegion q = find_region<NV>(idx, 0, N, rx, ry, rbw, rpitch, rbase, rpass, rinv);
      const int li = idx - q.base;
      const int py = int((float(li) + 0.5f) * q.inv);
      const int px = li - py * q.pitch;
      const int gx = q.x + px, gy = q.y + py;
      const bool in = (idx < total) & (px < q.bw) & (gx >= 0) & (gx < W) & (gy >= 0) & (gy < H);
      goff[i] = in ? uint32_t((q.v * C * HW + gy * W + gx) * int(sizeof(TIn))) : kOob;
    }
    uint32_t pre[MS][G];
    constexpr bool UNCOND = NV == 8;
    auto issue = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MS; ++i)
        if (UNCOND || wfirst + kThreads * i < total) {
#pragma unroll
          for (int k = 0; k < G; ++k) pre[i][k] = buf_load<TIn>(frs, goff[i], uint32_t((c0 + k) * HW * int(sizeof(TIn))));
        }
    };
    auto commit = [&](Slot* buf) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MS; ++i)
        if (UNCOND || wfirst + kThreads * i < total) buf[t + kThreads * i] = pack<TIn>(pre[i]);
    };
    auto consume = [&](const Slot* buf, int c0) __attribute__((always_inline)) {
      float sv[G][NV];
      sample_views(reinterpret_cast<const char*>(buf), std::true_type{}, 0, sv);
      aggregate_store(c0, sv);
      __builtin_amdgcn_sched_barrier(0);     // bounds the LDS reads in flight (registers)
    };

    issue(0);
    commit(stage);
    __syncthreads();
    for (int c0 = 0; c0 < C; c0 += 2 * G) {
      const bool more1 = c0 + G < C, more2 = c0 + 2 * G < C;
      if (more1) issue(c0 + G);
      consume(stage, c0);
      if (!more1) break;
      commit(stage + kBuf);
      __syncthreads();
      if (more2) issue(c0 + 2 * G);
      consume(stage + kBuf, c0 + G);
      if (!more2) break;
      commit(stage);
      __syncthreads();
    }
    return;
  }

  // ---- several passes per channel group (close cameras): stage, sample, repeat -------
  for (int c0 = 0; c0 < C; c0 += G) {
    float sv[G][NV];
    for (int pass = 0; pass < npass; ++pass) {
      int total = 0;
#pragma unroll
      for (int v = 0; v < NV; ++v) if (v < N && rpass[v] == pass) total = max(total, rend[v]);
      for (int idx = t; idx < total; idx += kThreads) {
        const SlotRegion q = find_region<NV>(idx, pass, N, rx, ry, rbw, rpitch, rbase, rpass, rinv);
        const int li = idx - q.base;
        const int py = int((float(li) + 0.5f) * q.inv);
        const int px = li - py * q.pitch;
        const int gx = q.x + px, gy = q.y + py;
        const bool in = (px < q.bw) & (gx >= 0) & (gx < W) & (gy >= 0) & (gy < H);
        const uint32_t go = in ? uint32_t((q.v * C * HW + gy * W + gx) * int(sizeof(TIn))) : kOob;
        uint32_t bits[G];
#pragma unroll
        for (int k = 0; k < G; ++k) bits[k] = buf_load<TIn>(frs, go, uint32_t((c0 + k) * HW * int(sizeof(TIn))));
        MVN_DASSERT(idx >= 0 && idx < kZeroSlot);
        stage[idx] = pack<TIn>(bits);
      }
      __syncthreads();
      sample_views(reinterpret_cast<const char*>(stage), std::false_type{}, pass, sv);
      __syncthreads();
    }
    aggregate_store(c0, sv);
  }
}

}  // namespace

template <int AGG, typename TIn, typename TOut>
int launch_tiled(const void* feat, const float* P, const float* coords, const float* cub, int transfer,
                 const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                 int align_corners, int out_cl, int fast, hipStream_t s) {
  if (out_cl && C % 4 != 0) return MVN_ERR_SHAPE;
  if (!unproject_force_generic()) {
    // (fast = MVN_PRECISION_FAST is a property of the chunk-staged kernel; where it does not
    // apply the exact kernel below runs, which is inside the fast mode's tolerance)
    const int r = launch_x4<AGG, TIn, TOut>(feat, P, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy, Vz,
                                            align_corners, out_cl, fast, s);
    if (r != 1) return r;
  }
  // 32-bit buffer offsets: a frame's maps and volume must stay below 2 GiB
  if ((long long)N * C * H * W * sizeof(TIn) >= (1LL << 31) ||
      (long long)C * Vx * Vy * Vz * sizeof(TOut) >= (1LL << 31))
    return MVN_ERR_SHAPE;
  // LDS slot budget per pass (clamped in-kernel to the buffer); tests lower it through
  // mvn_debug_set_unproject to force the multi-pass and global-gather paths.
  const int knob = unproject_lds_slot_budget();
  const int budget = knob > 0 ? knob : 1 << 30;
  auto go = [&](auto nv, auto exact) {
    constexpr int NV = decltype(nv)::value;
    using S = TileShape<NV>;
    const long long nb = (long long)B * ((Vx + S::TX - 1) / S::TX) * ((Vy + S::TY - 1) / S::TY) *
                         ((Vz + S::TZ - 1) / S::TZ);
    if (nb > INT_MAX) return false;
    unproject_tiled<AGG, TIn, TOut, NV, decltype(exact)::value><<<int(nb), S::THREADS, 0, s>>>(
        static_cast<const TIn*>(feat), P, coords, cub, transfer, conf, static_cast<TOut*>(out), B, N, C, H, W,
        Vx, Vy, Vz, align_corners, budget, out_cl);
    return true;
  };
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  using T_ = std::true_type;
  using F_ = std::false_type;
  const bool ok = N == 4 ? go(I4{}, T_{}) : N < 4 ? go(I4{}, F_{}) : N == 8 ? go(I8{}, T_{}) : go(I8{}, F_{});
  if (!ok) return MVN_ERR_SHAPE;
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

#define MVN_INSTANTIATE(AGG)                                                                                   \
  template int launch_tiled<AGG, float, float>(const void*, const float*, const float*, const float*, int, const float*, void*,    \
                                               int, int, int, int, int, int, int, int, int, int, int, hipStream_t);  \
  template int launch_tiled<AGG, uint16_t, uint16_t>(const void*, const float*, const float*, const float*, int, const float*,     \
                                                     void*, int, int, int, int, int, int, int, int, int, int,   \
                                                     int, hipStream_t);                                              \
  template int launch_tiled<AGG, uint16_t, float>(const void*, const float*, const float*, const float*, int, const float*, void*, \
                                                  int, int, int, int, int, int, int, int, int, int, int, hipStream_t);
MVN_INSTANTIATE(MVN_AGG_SUM)
MVN_INSTANTIATE(MVN_AGG_MAX)
MVN_INSTANTIATE(MVN_AGG_SOFTMAX)
MVN_INSTANTIATE(MVN_AGG_CONF)
#undef MVN_INSTANTIATE

}  // namespace unproj
}  // namespace mvn
