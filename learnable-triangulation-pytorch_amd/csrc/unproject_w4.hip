// Four-view unprojection for gfx950, wave-autonomous: every wave owns a 4 x 4 x 4 voxel
// tile, stages that tile's footprint in its own LDS region and never waits for another
// wave — no workgroup barrier anywhere.
//
// Contract and numerics: mvn/utils/op.py:99-163 exactly as unproject_x4 / unproject_tiled
// (sum / max / conf bit-exact with the reference, softmax in the staged-path op order:
// the three kernels agree bit for bit).
//
// Why: in the block-cooperative kernels (unproject_tiled, unproject_x4) a block of 8
// waves stages a 512-voxel tile's footprint together, one barrier per channel group.
// Per-block phase stamps (tools/x4_stamps.py) put ~40 % of a block's
// lifetime in its prologue (footprint reduction across waves + barriers + first loads)
// and ~35 % of its channel loop in barrier and staging waits — at 4 waves per SIMD
// (registers, LDS) nothing else runs meanwhile.  A 4x4x4 wave tile has a larger footprint
// per voxel (3.4 vs 2.2 pixels at the bench configs: more staging), but its box is a
// wave-level DPP reduction straight into scalar registers, and while one wave waits for
// its loads the other three on the SIMD are independent.
//
// Per wave: lane -> voxel (x, y, z) = (lane / 16, lane / 4 % 4, lane % 4) in the tile;
// LDS region of kWSlots 16-byte slots = up to kWTrash image slots (4 f32 channels per
// pixel, views back to back, odd row pitch), 64 per-lane trash slots (masked-off pixels
// of a staged chunk), 2 zero slots (taps of voxel-views that sample nothing).  Staging in
// chunks of 4 x-consecutive pixels (one 16-/8-byte buffer load per chunk and channel, the
// hardware range check returns 0 = padding 'zeros'); the next channel group's loads are
// in flight while the current group is sampled from the single LDS region (a wave's LDS
// operations execute in order).  A block is 4 waves stacked in z (a 4 x 4 x 16 column).
#include "unproject_common.hpp"

namespace mvn {
namespace unproj {
namespace {

constexpr int kWThreads = 256;                       // 4 waves: a 4 x 4 x 16 voxel column
constexpr int kWSlots = 512;                         // per wave: 8 KiB of LDS
constexpr int kWZero = kWSlots - 2, kWTrash = kWSlots - 2 - kWave;
constexpr int kWMC = 2;                              // chunks per lane in one pass

#ifndef MVN_W4_WAVES
#define MVN_W4_WAVES 4                               // waves per SIMD the registers must allow
#endif

template <int AGG, typename TIn, typename TOut>
__global__ __launch_bounds__(kWThreads) __attribute__((amdgpu_waves_per_eu(MVN_W4_WAVES))) void unproject_w4(
    const TIn* __restrict__ feat, const float* __restrict__ P, const float* __restrict__ coords,
    const float* __restrict__ cub, int transfer, const float* __restrict__ conf, TOut* __restrict__ out, int B,
    int C, int H, int W, int Vx, int Vy, int Vz, int align_corners, int budget, int out_cl) {
  constexpr int NV = 4, G = 4, MC = kWMC;
  constexpr uint32_t kSlotB = 16, E = sizeof(TIn);
  __shared__ uint4 lds[(kWThreads / kWave) * kWSlots];

  const int lane = int(threadIdx.x) & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / kWave);
  uint4* stage = lds + wid * kWSlots;

  // ---- which 4 x 4 x 16 column (z fastest), XCD-balanced as the other kernels --------
  const int nTx = (Vx + 3) / 4, nTy = (Vy + 3) / 4, nTz = (Vz + 15) / 16;
  int L = int(blockIdx.x);
  {
    const int nf = nTx * nTy * nTz;
    if (B >= 16 && nf % 8 == 0) {
      const int xcd = int(blockIdx.x) % 8, k = int(blockIdx.x) / 8, slab = nf / 8;
      L = (k / slab) * nf + xcd * slab + k % slab;
    }
  }
  const int tz = L % nTz; L /= nTz;
  const int ty = L % nTy; L /= nTy;
  const int tx = L % nTx;
  const int b = L / nTx;
  const int nvox = Vx * Vy * Vz;
  const int HW = H * W;
  const float* Pb = P + size_t(b) * NV * 12;
  const TIn* fb = feat + size_t(b) * NV * C * HW;
  const float* cfb = conf ? conf + size_t(b) * NV * C : nullptr;

  if (lane < 2) stage[kWZero + lane] = uint4{0u, 0u, 0u, 0u};

  // ---- this lane's voxel and its per-view geometry -----------------------------------
  const int X = tx * 4 + lane / 16, Y = ty * 4 + (lane / 4) % 4, Z = tz * 16 + wid * 4 + lane % 4;
  const bool act = (X < Vx) & (Y < Vy) & (Z < Vz);
  const int vox = act ? (X * Vy + Y) * Vz + Z : 0;
  float cx, cy, cz;
  if (cub) {
    float o[3];
    cuboid_coord(cub + b * MVN_CUBOID_FLOATS, Vx, X, Y, Z, transfer, o);
    cx = o[0]; cy = o[1]; cz = o[2];
  } else {
    const float* cp = coords + (size_t(b) * nvox + vox) * 3;
    cx = cp[0]; cy = cp[1]; cz = cp[2];
  }
  int fx[NV], fy[NV];
  float w[NV][4];
  bool has[NV];
  {
    bool lane_fast = true;
#pragma unroll
    for (int v = 0; v < NV; ++v) lane_fast &= div_core_safe(homog(Pb + v * 12, cx, cy, cz));
    const bool wave_fast = __builtin_amdgcn_ballot_w64(!lane_fast) == 0;
    const Recip rH = recip_refined(float(H)), rW = recip_refined(float(W));
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const Homog hp = homog(Pb + v * 12, cx, cy, cz);
      const Proj p = wave_fast ? project_h<true>(hp, H, W, align_corners, rH, rW)
                               : project_h<false>(hp, H, W, align_corners, rH, rW);
      const float fx0 = floorf(p.ix), fy0 = floorf(p.iy);
      const bool h = act & !p.invalid & (fx0 >= -1.f) & (fx0 < float(W)) & (fy0 >= -1.f) & (fy0 < float(H));
      const float tx_ = p.ix - fx0, sx_ = 1.f - tx_, ty_ = p.iy - fy0, sy_ = 1.f - ty_;
      w[v][0] = h ? sy_ * sx_ : 0.f; w[v][1] = h ? sy_ * tx_ : 0.f;
      w[v][2] = h ? ty_ * sx_ : 0.f; w[v][3] = h ? ty_ * tx_ : 0.f;
      fx[v] = h ? int(fx0) : 0; fy[v] = h ? int(fy0) : 0;
      has[v] = h;
    }
  }

  // ---- this wave's footprint boxes (DPP) -> regions of its LDS image (scalar) --------
  Region rg[NV];
  int npass, total;
  {
    int snext = 0, cnext = 0, pass = 0, chunks0 = 0;
    bool too_big = false;
    const int lim = min(budget, kWTrash);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int x0 = wave_min_u(has[v] ? fx[v] : INT_MAX);
      const int x1 = wave_max_u(has[v] ? fx[v] : INT_MIN);
      int y0 = wave_min_u(has[v] ? fy[v] : INT_MAX);
      const int y1 = wave_max_u(has[v] ? fy[v] : INT_MIN);
      int bw = 0, bh = 0;
      if (x0 <= x1) { bw = x1 - x0 + 2; bh = y1 - y0 + 2; }    // +1 px: east / south taps
      else { x0 = 0; y0 = 0; }
      const int pitch = bw | 1;                                  // odd: spreads rows over banks
      const int xa = x0 & ~3;                                    // chunk origin, x % 4 == 0
      const int cw = bw ? (x0 + bw - xa + 3) >> 2 : 0;           // chunks per row
      const int area = pitch * bh, nch = cw * bh;
      if (area > lim || nch > MC * kWave) too_big = true;
      if (snext + area > lim || cnext + nch > MC * kWave) { ++pass; snext = 0; cnext = 0; }
      rg[v].x0 = x0; rg[v].y0 = y0; rg[v].bw = bw; rg[v].bh = bh; rg[v].pitch = pitch; rg[v].sbase = snext;
      rg[v].xa = xa; rg[v].cw = cw; rg[v].cbase = cnext; rg[v].pass = pass; rg[v].cend = cnext + nch;
      rg[v].inv_cw = cw ? __builtin_amdgcn_rcpf(float(cw)) : 0.f;
      snext += area;
      cnext += nch;
      if (pass == 0) chunks0 = cnext;
    }
    npass = too_big ? -1 : pass + 1;
    total = chunks0;
  }

  if (npass < 0) {
    // one view's footprint exceeds the wave's LDS region: global gathers for this tile
    if (act)
      gather_voxel<AGG, TIn, TOut>(fb, Pb, cfb, out + size_t(b) * C * nvox + (out_cl ? size_t(vox) * C : vox),
                                   out_cl ? 1 : nvox, NV, C, H, W, cx, cy, cz, align_corners);
    return;
  }

  const __amdgpu_buffer_rsrc_t frs = make_rsrc(fb, uint32_t(size_t(NV) * C * HW * E));
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(out + size_t(b) * C * nvox, uint32_t(size_t(C) * nvox * sizeof(TOut)));
  const uint32_t ooff = act ? uint32_t(vox) * uint32_t(sizeof(TOut)) : kOob;
  const uint32_t ooff_cl = act ? uint32_t(vox) * uint32_t(C) * uint32_t(sizeof(TOut)) : kOob;

  // LDS byte offsets (within the wave's region) of each view's north-west / south-west taps
  uint32_t anw[NV], asw[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int slot = rg[v].sbase + (fy[v] - rg[v].y0) * rg[v].pitch + (fx[v] - rg[v].x0);
    anw[v] = uint32_t(has[v] ? slot : kWZero) * kSlotB;
    asw[v] = uint32_t(has[v] ? slot + rg[v].pitch : kWZero) * kSlotB;
  }

  // chunk li of view `sel` -> global byte offset (kOob outside the image), first slot, and
  // the mask of its 4 pixels inside the view's box
  auto chunk_fields = [&](const Region& r, int sel, int li, uint32_t& goff, int& s0, uint32_t& mask, bool live)
      __attribute__((always_inline)) {
    const int py = int((float(li) + 0.5f) * r.inv_cw);
    const int gx = r.xa + 4 * (li - py * r.cw), gy = r.y0 + py;
    const bool in = live & (gx >= 0) & (gx < W) & (gy >= 0) & (gy < H);
    goff = in ? uint32_t((sel * C * HW + gy * W + gx) * int(E)) : kOob;
    s0 = r.sbase + py * r.pitch + (gx - r.x0);
    mask = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int dx = gx + p - r.x0;
      mask |= (live & (dx >= 0) & (dx < r.bw)) ? (1u << p) : 0u;
    }
  };
  using Chunk = typename ChunkT<TIn>::type;
  auto load_group = [&](Chunk (&pre)[G], uint32_t goff, int c0) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < G; ++k) pre[k] = load_chunk<TIn>(frs, goff, uint32_t((c0 + k) * HW) * E);
  };
  auto write_group = [&](const Chunk (&pre)[G], int s0, uint32_t mask) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
      stage[(mask & (1u << p)) ? s0 + p : kWTrash + lane] =
          make_uint4(chunk_px(pre[0], p), chunk_px(pre[1], p), chunk_px(pre[2], p), chunk_px(pre[3], p));
  };
  auto sample_views = [&](bool all, int pass, f2 (&sv)[2][NV]) __attribute__((always_inline)) {
    const char* buf = reinterpret_cast<const char*>(stage);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (!all && rg[v].pass != pass) continue;
      const uint4 a = *reinterpret_cast<const uint4*>(buf + anw[v]);
      const uint4 bq = *reinterpret_cast<const uint4*>(buf + anw[v] + kSlotB);
      const uint4 cq = *reinterpret_cast<const uint4*>(buf + asw[v]);
      const uint4 d = *reinterpret_cast<const uint4*>(buf + asw[v] + kSlotB);
      const f2 w0{w[v][0], w[v][0]}, w1{w[v][1], w[v][1]}, w2{w[v][2], w[v][2]}, w3{w[v][3], w[v][3]};
      sv[0][v] = pk_fma(lo2(d), w3, pk_fma(lo2(cq), w2, pk_fma(lo2(bq), w1, lo2(a) * w0)));
      sv[1][v] = pk_fma(hi2(d), w3, pk_fma(hi2(cq), w2, pk_fma(hi2(bq), w1, hi2(a) * w0)));
      if (v & 1) __builtin_amdgcn_sched_barrier(0);   // at most two views' taps in flight
    }
  };
  auto aggregate_store = [&](int c0, const f2 (&sv)[2][NV]) __attribute__((always_inline)) {
    float r[G];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      f2 cf[NV];
      if constexpr (AGG == MVN_AGG_CONF) {
#pragma unroll
        for (int v = 0; v < NV; ++v) cf[v] = f2{cfb[v * C + c0 + 2 * q], cfb[v * C + c0 + 2 * q + 1]};
      }
      const f2 o = aggregate_pair<AGG>(sv[q], cf);
      r[2 * q] = o.x;
      r[2 * q + 1] = o.y;
    }
    if (out_cl) {
      const uint32_t soff = uint32_t(c0) * uint32_t(sizeof(TOut));
      if constexpr (sizeof(TOut) == 4)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int,
                               make_uint4(__float_as_uint(r[0]), __float_as_uint(r[1]), __float_as_uint(r[2]),
                                          __float_as_uint(r[3]))),
            ors, ooff_cl, soff, 0);
      else
        __builtin_amdgcn_raw_buffer_store_b64(
            __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int,
                               make_uint2(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]))),
            ors, ooff_cl, soff, 0);
      return;
    }
#pragma unroll
    for (int ch = 0; ch < G; ++ch)
      store_plane<TOut>(r[ch], ors, ooff, uint32_t(c0 + ch) * uint32_t(nvox) * uint32_t(sizeof(TOut)));
  };

  if (npass == 1) {
    // ---- one pass: MC chunks per lane, next group's loads in flight --------------------
    uint32_t goff[MC], mask[MC];
    int s0[MC];
#pragma unroll
    for (int i = 0; i < MC; ++i) {
      const int k = lane + kWave * i;
      int sel = 0;
#pragma unroll
      for (int u = 1; u < NV; ++u)
        if (rg[u].cw > 0 && k >= rg[u].cbase) sel = u;
      const Region r = pick_region(rg, sel);
      chunk_fields(r, sel, k - r.cbase, goff[i], s0[i], mask[i], k < total);
    }
    Chunk pre[MC][G];
    auto issue = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MC; ++i)
        if (kWave * i < total) load_group(pre[i], goff[i], c0);
    };
    auto commit = [&]() __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MC; ++i)
        if (kWave * i < total) write_group(pre[i], s0[i], mask[i]);
    };
    issue(0);
    commit();
    for (int c0 = 0; c0 < C; c0 += G) {
      if (c0 + G < C) issue(c0 + G);
      f2 sv[2][NV];
      sample_views(true, 0, sv);
      aggregate_store(c0, sv);
      __builtin_amdgcn_sched_barrier(0);
      if (c0 + G < C) commit();      // in-order LDS: lands after this group's tap reads
    }
    return;
  }

  // ---- several passes of whole views per channel group --------------------------------
  for (int c0 = 0; c0 < C; c0 += G) {
    f2 sv[2][NV];
    for (int pass = 0; pass < npass; ++pass) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if (rg[v].pass != pass) continue;
        const int nch = rg[v].cend - rg[v].cbase;
        for (int li = lane; li < nch; li += kWave) {
          uint32_t goff, mask;
          int s0;
          chunk_fields(rg[v], v, li, goff, s0, mask, true);
          Chunk pre[G];
          load_group(pre, goff, c0);
          write_group(pre, s0, mask);
        }
      }
      sample_views(false, pass, sv);
    }
    aggregate_store(c0, sv);
  }
}

}  // namespace

// Returns MVN_OK, an error code, or 1 when this kernel does not apply.
template <int AGG, typename TIn, typename TOut>
int launch_w4(const void* feat, const float* P, const float* coords, const float* cub, int transfer,
              const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
              int align_corners, int out_cl, hipStream_t s) {
  if (N != 4 || W % 4 != 0 || C % 4 != 0) return 1;
  if ((long long)N * C * H * W * sizeof(TIn) >= (1LL << 31) ||
      (long long)C * Vx * Vy * Vz * sizeof(TOut) >= (1LL << 31))
    return MVN_ERR_SHAPE;
  const int knob = unproject_lds_slot_budget();
  const int budget = knob > 0 ? knob : 1 << 30;
  const long long nb = (long long)B * ((Vx + 3) / 4) * ((Vy + 3) / 4) * ((Vz + 15) / 16);
  if (nb > INT_MAX) return MVN_ERR_SHAPE;
  unproject_w4<AGG, TIn, TOut><<<int(nb), kWThreads, 0, s>>>(
      static_cast<const TIn*>(feat), P, coords, cub, transfer, conf, static_cast<TOut*>(out), B, C, H, W, Vx, Vy,
      Vz, align_corners, budget, out_cl);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

#define MVN_INSTANTIATE(AGG)                                                                                   \
  template int launch_w4<AGG, float, float>(const void*, const float*, const float*, const float*, int,        \
                                            const float*, void*, int, int, int, int, int, int, int, int, int,  \
                                            int, hipStream_t);                                                 \
  template int launch_w4<AGG, uint16_t, uint16_t>(const void*, const float*, const float*, const float*, int,  \
                                                  const float*, void*, int, int, int, int, int, int, int, int, \
                                                  int, int, hipStream_t);                                      \
  template int launch_w4<AGG, uint16_t, float>(const void*, const float*, const float*, const float*, int,     \
                                               const float*, void*, int, int, int, int, int, int, int, int,    \
                                               int, int, hipStream_t);
MVN_INSTANTIATE(MVN_AGG_SUM)
MVN_INSTANTIATE(MVN_AGG_MAX)
MVN_INSTANTIATE(MVN_AGG_SOFTMAX)
MVN_INSTANTIATE(MVN_AGG_CONF)
#undef MVN_INSTANTIATE

}  // namespace unproj
}  // namespace mvn
