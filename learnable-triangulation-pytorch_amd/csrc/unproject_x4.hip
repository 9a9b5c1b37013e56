// Chunk-staged unprojection for gfx950 — the production kernel behind mvn_unproject for the
// configurations of BASELINE.json: 4 views (W % 4 == 0, C % 4 == 0; 16-byte LDS slots of 4
// channels) and 8 views (config 4: W % 4 == 0, C % 2 == 0, NCDHW; 8-byte slots of 2).
//
// Contract and numerics: mvn/utils/op.py:99-163 exactly as unproject_tiled.hip (sum / max /
// conf bit-exact with the reference; softmax max-first with exp2 and one reciprocal, same
// op order as unproject_tiled's staged path, so the two kernels agree bit for bit).
//
// What differs from unproject_tiled (the generic N <= 8 kernel) is how the per-block LDS
// image of the views' footprints is filled and consumed:
//   * staging in CHUNKS of 4 x-consecutive pixels: one 16-byte (f32) / 8-byte (bf16) buffer
//     load per chunk and channel instead of one 4- / 2-byte load per pixel and channel —
//     a quarter of the vector-memory instructions (the texture path, not HBM, was the
//     busiest unit: TD 82 % at config 3, profiles/r07a_*).  Chunks start at x % 4 == 0, so
//     with W % 4 == 0 a chunk lies wholly inside or wholly outside the image (the hardware
//     range check of an out-of-range offset returns zeros = padding_mode 'zeros'); pixels
//     of a chunk outside the block's footprint are simply not written to LDS.  The 4 x 4
//     (pixel x channel) block a lane loads is transposed for free into 4 slots of
//     (4 channels) 16 bytes, one ds_write_b128 each;
//   * bilinear sampling and view aggregation on channel PAIRS with packed f32 arithmetic
//     (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32: per lane exactly the scalar fma / mul /
//     add of the reference order, two channels per instruction).
// Everything else — voxel tile per block (TX x 8 x 16, z fastest), per-view footprint
// bounding boxes with odd row pitch, two LDS buffers with the next channel group's loads
// in flight, XCD-balanced block order, buffer-descriptor stores — follows unproject_tiled.
// Footprints that exceed one LDS buffer are staged in several passes of whole views;
// a single view larger than a buffer sends its block to the global-gather fallback.
#include <type_traits>

#include "unproject_common.hpp"

namespace mvn {
namespace unproj {
namespace {

// Voxel tile per block and LDS image size.  Tiles short in z project more compactly:
// footprint slots per voxel at the bench configs 2.2 (4x8x16), 1.7 (8x8x8), 2.2 (4x8x8);
// the largest footprints 2,156 / 1,428 / 965 slots (tools: /tmp-free model in DESIGN.md).
// NV views, G channels per LDS slot (16-byte slots of 4 f32 channels, or 8-byte slots of 2),
// MC chunk slots per thread, WAVES waves per SIMD the register allocation must allow.
template <int K> struct X4Shape;
// STORE_F32: cache policy of f32 output stores (non-temporal for 64-byte z-runs).
template <> struct X4Shape<0> {   // 4 views, f32 maps
  static constexpr int NV = 4, G = 4, TX = 4, TY = 8, TZ = 16, THREADS = 512, SLOTS = 2048, MC = 2, WAVES = 4;
  static constexpr int STORE_F32 = kStorePolicyF32;
};
// 4 views, bf16 maps (widened exactly to f32 slots when staged): an 8x8x8 tile of 512 threads,
// 1.7 instead of 2.2 staged pixels per voxel at 4 waves per SIMD (2 blocks of 66 KB per CU; its
// 115 VGPRs keep 6 waves out of reach): cfg3 softmax 535 -> 512 us against the 4x8x8 tile of 256
// threads (r21, profiles/r21_ab_exact_bf16_tile.txt)
template <> struct X4Shape<2> {
  static constexpr int NV = 4, G = 4, TX = 8, TY = 8, TZ = 8, THREADS = 512, SLOTS = 2048, MC = 1, WAVES = 4;
  static constexpr int STORE_F32 = kStorePolicyF32;
};
// 8 views (BASELINE config 4, CMU-style): the footprint of 8 views doubles, so slots of 2
// channels (8 bytes) keep two 2,048-slot buffers in 32 KiB (footprints of a 4x8x8 tile at
// config 4: 1,170 slots mean, 1,897 max — tools/footprints.py); 8 views' per-voxel weights and
// tap offsets (48 VGPRs) need the 168-register budget of 3 waves per SIMD (3 blocks per CU).
// f32 output: the tile's 32-byte z-runs leave through L2 with the default policy (4 blocks
// complete each 128-byte line; non-temporal stores wrote 1.47x the output, 686 -> 647 us, r16).
template <> struct X4Shape<3> {
  static constexpr int NV = 8, G = 2, TX = 4, TY = 8, TZ = 8, THREADS = 256, SLOTS = 2048, MC = 3, WAVES = 3;
  static constexpr int STORE_F32 = 0;
};
// 4 views, bf16 maps, fast arithmetic (pixel-pair slots): an 8x8x8 tile of 512 threads —
// 1.92 instead of 2.65 staged pixels per voxel (tools/footprints.py: the footprint of a
// cube grows slower than its volume), one chunk slot per thread (the largest footprint at
// the bench geometry is 421 chunks), two 1,536-slot buffers: 49 KB of LDS and 78 VGPRs, so 3
// blocks per CU, 6 waves per SIMD (cfg3 503 -> 437 us against 4 waves, r21).  The f32 and
// exact kernels need 113-117 VGPRs on this tile and spill in the tap loop (2.4-3.2x slower,
// profiles/r21_ab_tile_occupancy_negatives.txt)
template <> struct X4Shape<4> {
  static constexpr int NV = 4, G = 4, TX = 8, TY = 8, TZ = 8, THREADS = 512, SLOTS = 1536, MC = 1, WAVES = 6;
  static constexpr int STORE_F32 = kStorePolicyF32;
};
#ifndef MVN_FAST_BF16_SHAPE
#define MVN_FAST_BF16_SHAPE 4
#endif

// LDS slot: one pixel's G channels as f32
template <int G> struct SlotT;
template <> struct SlotT<4> { using type = uint4; };
template <> struct SlotT<2> { using type = uint2; };
// channel pair q of a slot
__device__ __forceinline__ f2 slot_pair(const uint4& s, int q) { return q ? hi2(s) : lo2(s); }
__device__ __forceinline__ f2 slot_pair(const uint2& s, int) { return f2{__uint_as_float(s.x), __uint_as_float(s.y)}; }

// Per-view LDS regions (block-uniform, scalar registers), packed 3 words per view —
// (x0 + 1, y0 + 1), (bw, bh), sbase | cbase << 13 | pass << 24 — the derived fields
// recomputed on use (unpacked, the 48 SGPRs of 4 views spilled to VGPR lanes: ~60
// v_writelane / v_readlane in the prologue, round 2).
__device__ __forceinline__ Region make_region(int x0, int y0, int bw, int bh, int sbase, int cbase, int pass) {
  Region r;
  r.x0 = x0; r.y0 = y0; r.bw = bw; r.bh = bh; r.sbase = sbase; r.cbase = cbase; r.pass = pass;
  r.pitch = bw | 1;                                          // odd: spreads rows over banks
  r.xa = x0 & ~3;                                            // chunk origin, x % 4 == 0
  r.cw = bw ? (x0 + bw - r.xa + 3) >> 2 : 0;                 // chunks per row
  // chunks are numbered over groups of 4 rows, rows fastest (see chunk_fields): rows padded
  // to a multiple of 4
  r.cend = cbase + r.cw * bh;
  r.inv_cw = r.cw ? __builtin_amdgcn_rcpf(float(r.cw)) : 0.f;
  return r;
}
template <int NV> struct RegionSet {
  uint32_t a[NV], b[NV], c[NV];
  __device__ __forceinline__ void set(int v, const Region& r) {
    a[v] = uint32_t(r.x0 + 1) | (uint32_t(r.y0 + 1) << 16);
    b[v] = uint32_t(r.bw) | (uint32_t(r.bh) << 16);
    c[v] = uint32_t(r.sbase) | (uint32_t(r.cbase) << 13) | (uint32_t(r.pass) << 24);
  }
  __device__ __forceinline__ static Region unpack(uint32_t a, uint32_t b, uint32_t c) {
    return make_region(int(a & 0xffffu) - 1, int(a >> 16) - 1, int(b & 0xffffu), int(b >> 16), int(c & 0x1fffu),
                       int((c >> 13) & 0x7ffu), int(c >> 24));
  }
  __device__ __forceinline__ Region get(int v) const { return unpack(a[v], b[v], c[v]); }
  // u per lane: plain selects (9 v_cndmask).  Not through readfirstlane as pick_region does:
  // a convergent op cannot be speculated, so each select became a branch tree with exec
  // masking (~4,200 cycles of block prologue at config 2, profiles/r13_x4_stamps.txt).
  __device__ __forceinline__ Region pick(int u) const {
    uint32_t pa = a[0], pb = b[0], pc = c[0];
#pragma unroll
    for (int k = 1; k < NV; ++k) {
      pa = u == k ? a[k] : pa;
      pb = u == k ? b[k] : pb;
      pc = u == k ? c[k] : pc;
    }
    return unpack(pa, pb, pc);
  }
};

// CL: channels-last output (config 5) — a compile-time layout, so that the NCDHW kernels'
// output stores are straight-line code: the compiler's vmcnt for a staging commit then counts
// exactly the stores issued after the loads it waits for.
// FAST (MVN_PRECISION_FAST): the same function within the north_star
// tolerance instead of the reference's rounding — reciprocal projection, the view softmax
// without its max pass (log2-scaled samples, a range guard that falls back to the max-first
// formula), and for bf16 maps pixel-pair slots sampled by v_dot2_f32_bf16 with bf16 weights.
template <int AGG, typename TIn, typename TOut, int K, int CL, int FAST>
__global__ __launch_bounds__(X4Shape<K>::THREADS) __attribute__((amdgpu_waves_per_eu(X4Shape<K>::WAVES))) void unproject_x4(
    const TIn* __restrict__ feat, const float* __restrict__ P, const float* __restrict__ coords,
    const float* __restrict__ cub, int transfer, const float* __restrict__ conf, TOut* __restrict__ out, int B,
    int C, int H, int W, int Vx, int Vy, int Vz, int align_corners, int budget) {
  using S = X4Shape<K>;
  constexpr bool out_cl = CL != 0;
  constexpr int NV = S::NV, G = S::G, NP = G / 2;      // NP channel pairs per group
  constexpr int TX = S::TX, TY = S::TY, TZ = S::TZ;
  constexpr int kThreads = S::THREADS, kBuf = S::SLOTS, MC = S::MC, kWaves = kThreads / kWave;
  static_assert(TX * TY * TZ == kThreads, "one voxel per thread");
  // validated tiles: TX 4 or 8, TY 8, TZ 8 or 16 (an 8x4x16 variant was not bit-identical, r21)
  static_assert(TY == 8 && (TX == 4 || TX == 8), "tile shape outside the validated set");
  // PAIR: bf16 pixel-pair slots — dword k of the slot at pixel (x, y) holds channel k's
  // (x, x+1) bf16 pair, so a voxel-view reads 2 slots (rows y0, y1) per 4 channels instead of
  // 4, and each row is one v_dot2_f32_bf16 against the (west, east) bf16 weight pair.  A
  // slot needs pixel x+4 of its chunk's right neighbour: chunks are dealt to a wave's lanes
  // 63 at a time, lane 63 loading the next wave's first chunk only to hand it to lane 62
  // (DPP wave_shl:1) and writing nothing.
  constexpr bool PAIR = FAST != 0 && sizeof(TIn) == 2 && G == 4;
  constexpr bool SMXF = FAST != 0 && AGG == MVN_AGG_SOFTMAX;   // samples carry a log2(e) factor
  constexpr int kLanesW = PAIR ? kWave - 1 : kWave;               // chunks a wave owns per slot i
  constexpr int kCap = MC * kWaves * kLanesW;                       // chunk capacity of one pass
  // per buffer: image slots [0, kTrash), 64 per-lane trash slots (the masked-off pixels of
  // a chunk are written there: no exec-mask branch per write), 2 zero slots
  constexpr int kZeroSlot = kBuf - 2, kTrash = kBuf - 2 - kWave;
  // LDS slot = one pixel's G channels as f32 (16 / 8 bytes; bf16 maps are widened exactly
  // when staged: bf16 slots halve the LDS bytes but the per-tap widening costs more VALU, r13)
  using Slot = typename SlotT<G>::type;
  constexpr uint32_t kSlotB = sizeof(Slot);
  constexpr uint32_t E = sizeof(TIn);

  __shared__ Slot stageA[kBuf];
  __shared__ Slot stageB[kBuf];
  __shared__ int red[kWaves][NV][4];

  // ---- which tile (z-tiles fastest; block order as unproject_tiled) ------------------
  const int nTx = (Vx + TX - 1) / TX, nTy = (Vy + TY - 1) / TY, nTz = (Vz + TZ - 1) / TZ;
  int L = int(blockIdx.x);
  {
    const int nf = nTx * nTy * nTz;
    if (nf % 8 == 0) {
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
  const float* Pb = P + size_t(b) * NV * 12;
  const TIn* fb = feat + size_t(b) * NV * C * HW;
  const float* cfb = conf ? conf + size_t(b) * NV * C : nullptr;

  if (t < 4) (t < 2 ? stageA : stageB)[kZeroSlot + (t & 1)] = Slot{};

  const int X0 = tx * TX, Y0 = ty * TY, Z0 = tz * TZ;

  // ---- this thread's voxel ------------------------------------------------------------
  // A wave takes 64 / TZ consecutive y-rows of one x-plane.  A ds_read_b128 is serviced in
  // four groups of 16 lanes ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32);
  // lanes are assigned to voxels so that each group is a compact 2 (y) x 8 (z) patch, whose
  // taps land on fewer, closer pixels: fewer LDS bank conflicts (tools/lds_conflicts.py
  // model: 9.3 -> 7.6 cycles per read at 4x8x16, 9.1 -> 7.9 at 4x8x8) than z-fastest lanes.
  // vt = the voxel's index in the tile (x, y, z row-major).
  int vt;
  {
    const int m = lane & 31;
    const bool g1 = (m >= 4 && m < 12) || (m >= 16 && m < 20) || m >= 28;
    const int i = g1 ? (m < 12 ? m - 4 : m < 20 ? m - 8 : m - 16) : (m < 4 ? m : m < 16 ? m - 8 : m - 12);
    const int g = 2 * (lane >> 5) + (g1 ? 1 : 0);
    constexpr int ZH = TZ / 8;                                  // 8-voxel z halves per row
    const int yw = 2 * (g / ZH) + (i >> 3), z = 8 * (g % ZH) + (i & 7);
    vt = (t & ~(kWave - 1)) + yw * TZ + z;
  }
  static_assert(TZ % 8 == 0 && kWave % TZ == 0 && (kWave / TZ) * (TZ / 8) == 8,
                "patch lanes: a wave is 2 x 8-voxel rows per lane group");
  const int X = X0 + vt / (TZ * TY), Y = Y0 + (vt / TZ) % TY, Z = Z0 + vt % TZ;
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
  f2 wp[NV][2];                        // bilinear weights (nw, ne), (sw, se) per view
  uint32_t wq[NV][2];                  // PAIR: the same as bf16 pairs (nw | ne << 16), (sw | se << 16)
  bool has[NV];
  // per-voxel geometry: footprint base pixel, bilinear weights, "samples the image" flag
  auto project_voxel = [&]() __attribute__((always_inline)) {
    if constexpr (FAST != 0) {
      // ix = u / H * W - 0.5 (align_corners=False) or u / H * (W - 1) (True), u = uh / wh:
      // op.py:121-130 + grid_sample's unnormalisation folded into one reciprocal of the depth
      // and one fma per axis.  The validity mask is the reference's (same wh, same compare).
      const float fW = float(W), fH = float(H);
      const float ax = (align_corners ? fW - 1.f : fW) * __builtin_amdgcn_rcpf(fH);
      const float ay = (align_corners ? fH - 1.f : fH) * __builtin_amdgcn_rcpf(fW);
      const float bo = align_corners ? 0.f : -0.5f;
      // softmax: the weights carry log2(e), so each sample is s * log2(e) (aggregate below)
      const float ks = SMXF ? kLog2e : 1.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const Homog hp = homog(Pb + v * 12, cx, cy, cz);
        const float r = __builtin_amdgcn_rcpf(hp.wh == 0.f ? 1.f : hp.wh);
        const float ix = __builtin_fmaf(hp.uh, ax * r, bo), iy = __builtin_fmaf(hp.vh, ay * r, bo);
        const float fx0 = floorf(ix), fy0 = floorf(iy);
        const bool h = act & !(hp.wh <= 0.f) & (fx0 >= -1.f) & (fx0 < fW) & (fy0 >= -1.f) & (fy0 < fH);
        const float tx_ = ix - fx0, sx_ = 1.f - tx_, ty_ = (iy - fy0) * ks, sy_ = ks - ty_;
        wp[v][0] = f2{h ? sy_ * sx_ : 0.f, h ? sy_ * tx_ : 0.f};
        wp[v][1] = f2{h ? ty_ * sx_ : 0.f, h ? ty_ * tx_ : 0.f};
        if constexpr (PAIR) {
          wq[v][0] = pack_bf16x2(wp[v][0].x, wp[v][0].y);
          wq[v][1] = pack_bf16x2(wp[v][1].x, wp[v][1].y);
        }
        fx[v] = h ? int(fx0) : 0; fy[v] = h ? int(fy0) : 0;
        has[v] = h;
      }
      return;
    }
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
      wp[v][0] = f2{h ? sy_ * sx_ : 0.f, h ? sy_ * tx_ : 0.f};
      wp[v][1] = f2{h ? ty_ * sx_ : 0.f, h ? ty_ * tx_ : 0.f};
      fx[v] = h ? int(fx0) : 0; fy[v] = h ? int(fy0) : 0;
      has[v] = h;
    }
  };

  project_voxel();

  // ---- per-view boxes (ints, clipped to the pixels a tap can start at) ----------------
  int box[NV][4];
  {
    // exact: every voxel's base pixel.  Per 4 views, the 16 per-wave reductions (min x0, max x1,
    // min y0, max y1; maxima as minima of negated values) run as one transposing butterfly:
    // lanes 32 apart swap halves of their 16 values (v_permlane32_swap), then rows 16 apart
    // (v_permlane16_swap), then lanes 8 and "4" apart (DPP row_ror:8, row_half_mirror) each
    // keep one of two, and the quads reduce — 35 instructions instead of 16 DPP reductions
    // with their readlanes.  Lane l ends with value (l >> 2) & 15 of the whole wave.
#pragma unroll
    for (int h = 0; h < NV / 4; ++h) {      // one butterfly per 4 views
      int q16[16];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int v = 4 * h + u;
        q16[4 * u + 0] = has[v] ? fx[v] : INT_MAX;
        q16[4 * u + 1] = has[v] ? -fx[v] : INT_MAX;
        q16[4 * u + 2] = has[v] ? fy[v] : INT_MAX;
        q16[4 * u + 3] = has[v] ? -fy[v] : INT_MAX;
      }
      int q8[8], q4[4], q2[2];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const auto r = __builtin_amdgcn_permlane32_swap(unsigned(q16[i]), unsigned(q16[8 + i]), false, false);
        q8[i] = min(int(r[0]), int(r[1]));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const auto r = __builtin_amdgcn_permlane16_swap(unsigned(q8[i]), unsigned(q8[4 + i]), false, false);
        q4[i] = min(int(r[0]), int(r[1]));
      }
      const bool b3 = lane & 8, b2 = lane & 4;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int send = b3 ? q4[m] : q4[m + 2], keep = b3 ? q4[m + 2] : q4[m];
        q2[m] = min(keep, __builtin_amdgcn_update_dpp(INT_MAX, send, 0x128, 0xf, 0xf, false));   // row_ror:8
      }
      int q1;
      {
        const int send = b2 ? q2[0] : q2[1], keep = b2 ? q2[1] : q2[0];
        q1 = min(keep, __builtin_amdgcn_update_dpp(INT_MAX, send, 0x141, 0xf, 0xf, false));     // row_half_mirror
      }
      q1 = min(q1, __builtin_amdgcn_update_dpp(INT_MAX, q1, 0xb1, 0xf, 0xf, false));              // quad_perm 1,0,3,2
      q1 = min(q1, __builtin_amdgcn_update_dpp(INT_MAX, q1, 0x4e, 0xf, 0xf, false));              // quad_perm 2,3,0,1
      if ((lane & 3) == 0) (&red[wid][4 * h][0])[(lane >> 2) & 15] = q1;
    }
    __syncthreads();
    int part = INT_MAX;
    {
      const int idx = lane & (4 * NV - 1);      // lane 4v+k reduces component k of view v
#pragma unroll
      for (int q = 0; q < kWaves; ++q) part = min(part, (&red[q][0][0])[idx]);
    }
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int m = __builtin_amdgcn_readlane(part, 4 * v + k);
        box[v][k] = (k & 1) ? -m : m;
      }
  }

  // ---- LDS regions (slots and chunks), in scalar registers ----------------------------
  RegionSet<NV> rs;
  int npass, total;
  {
    int snext = 0, cnext = 0, pass = 0, chunks0 = 0;
    bool too_big = false;
    const int lim = min(budget, kTrash);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int x0 = box[v][0], y0 = box[v][2];
      const int x1 = box[v][1], y1 = box[v][3];
      int bw = 0, bh = 0;
      if (x0 <= x1 && y0 <= y1) { bw = x1 - x0 + 2; bh = y1 - y0 + 2; }   // +1 px: east / south taps
      else { x0 = 0; y0 = 0; }
      const Region r0 = make_region(x0, y0, bw, bh, 0, 0, 0);
      const int area = r0.pitch * bh, nch = r0.cend;
      if (area > lim || nch > kCap) too_big = true;
      if (snext + area > lim || cnext + nch > kCap) { ++pass; snext = 0; cnext = 0; }
      rs.set(v, make_region(x0, y0, bw, bh, snext, cnext, pass));
      snext += area;
      cnext += nch;
      if (pass == 0) chunks0 = cnext;
    }
    npass = too_big ? -1 : pass + 1;
    total = chunks0;
    MVN_DASSERT(too_big || (total <= kCap && snext <= lim));
  }

  if (npass < 0) {
    // A single view's footprint exceeds the LDS buffer: gather straight from global memory.
    if (act)
      gather_voxel<AGG, TIn, TOut>(fb, Pb, cfb, out + size_t(b) * C * nvox + (out_cl ? size_t(vox) * C : vox),
                                   out_cl ? 1 : nvox, NV, C, H, W, cx, cy, cz, align_corners);
    return;
  }

  const __amdgpu_buffer_rsrc_t frs = make_rsrc(fb, uint32_t(size_t(NV) * C * HW * E));
  const __amdgpu_buffer_rsrc_t ors = make_rsrc(out + size_t(b) * C * nvox, uint32_t(size_t(C) * nvox * sizeof(TOut)));
  const uint32_t ooff = act ? uint32_t(vox) * uint32_t(sizeof(TOut)) : kOob;

  const uint32_t ooff_cl = act ? uint32_t(vox) * uint32_t(C) * uint32_t(sizeof(TOut)) : kOob;

  // LDS byte offsets of each view's north-west and south-west taps (the exact boxes contain
  // every voxel's base pixel by construction; voxels that sample nothing read the zero slots)
  uint32_t anw[NV], asw[NV];
  auto tap_slots = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const Region rv = rs.get(v);
      const int dx = fx[v] - rv.x0, dy = fy[v] - rv.y0;
      const bool use = has[v];
      const int slot = rv.sbase + dy * rv.pitch + dx;
      anw[v] = uint32_t(use ? slot : kZeroSlot) * kSlotB;
      asw[v] = uint32_t(use ? slot + rv.pitch : kZeroSlot) * kSlotB;
      // the four taps (and the east neighbour of the zero slot) lie inside one buffer
      MVN_DASSERT(!use || (dx >= 0 && dy >= 0 && dx + 1 < rv.bw && dy + 1 < rv.bh &&
                           slot + rv.pitch + 1 < kTrash));
    }
  };
  // Chunk (k of a pass) -> global byte offset (kOob outside the image), first LDS slot and
  // the mask of its 4 pixels that lie in the view's box (empty past the pass's chunks).
  const bool writer = !PAIR || lane != kWave - 1;      // PAIR: lane 63 only feeds lane 62
  auto chunk_fields = [&](const Region& r, int sel, int li, uint32_t& goff, int& s0, uint32_t& mask, bool live)
      __attribute__((always_inline)) {
    // li = row * cw + chunk column (rows fastest-varying outer)
    const int py = int((float(li) + 0.5f) * r.inv_cw);
    const int gx = r.xa + 4 * (li - py * r.cw), gy = r.y0 + py;
    const bool in = live & (gx >= 0) & (gx < W) & (gy >= 0) & (gy < H);
    goff = in ? uint32_t((sel * C * HW + gy * W + gx) * int(E)) : kOob;
    s0 = r.sbase + py * r.pitch + (gx - r.x0);
    mask = 0;
    // PAIR: the slot of pixel dx holds (dx, dx+1): the box's last column is never a base
    const int xend = PAIR ? r.bw - 1 : r.bw;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int dx = gx + p - r.x0;
      mask |= (live & writer & (dx >= 0) & (dx < xend)) ? (1u << p) : 0u;
    }
  };
  using Chunk = typename ChunkT<TIn>::type;
  auto load_group = [&](Chunk (&pre)[G], uint32_t goff, int c0) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < G; ++k) pre[k] = load_chunk<TIn>(frs, goff, uint32_t((c0 + k) * HW) * E);
  };
  // masked-off pixels: bf16 maps and 2-channel slots write them to the lane's trash slot
  // (no exec-mask branch per write), f32 maps on 4-channel slots branch (A/B at the bench
  // configs: each is the faster for its case; 8 views 694 -> 677 us, r16)
  auto write_group = [&](Slot* buf, const Chunk (&pre)[G], int s0, uint32_t mask) __attribute__((always_inline)) {
    if constexpr (PAIR) {
      // chunk dwords: lo = (px0, px1), hi = (px2, px3) of one channel; pixels 4, 5 are the
      // right neighbour lane's lo.  Slot p, dword k: channel k's (px p, px p+1).
      uint32_t nb[G];
#pragma unroll
      for (int k = 0; k < G; ++k) nb[k] = uint32_t(__builtin_amdgcn_mov_dpp(int(pre[k].x), 0x130, 0xf, 0xf, true));
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint32_t d[G];
#pragma unroll
        for (int k = 0; k < G; ++k)
          d[k] = p == 0 ? pre[k].x : p == 1 ? __builtin_amdgcn_alignbit(pre[k].y, pre[k].x, 16)
               : p == 2 ? pre[k].y : __builtin_amdgcn_alignbit(nb[k], pre[k].y, 16);
        MVN_DASSERT(!(mask & (1u << p)) || (s0 + p >= 0 && s0 + p < kTrash));
        buf[(mask & (1u << p)) ? s0 + p : kTrash + lane] = make_uint4(d[0], d[1], d[2], d[3]);
      }
      return;
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      Slot q;
      if constexpr (G == 4)
        q = make_uint4(chunk_px(pre[0], p), chunk_px(pre[1], p), chunk_px(pre[2], p), chunk_px(pre[3], p));
      else
        q = make_uint2(chunk_px(pre[0], p), chunk_px(pre[1], p));
      MVN_DASSERT(!(mask & (1u << p)) || (s0 + p >= 0 && s0 + p < kTrash));   // a box slot, not trash / zero
      if constexpr (sizeof(TIn) == 2 || G == 2)
        buf[(mask & (1u << p)) ? s0 + p : kTrash + lane] = q;
      else if (mask & (1u << p))
        buf[s0 + p] = q;
    }
  };

  // one tap's slot.  8-byte slots are read as single ds_read_b64 (2 LDS cycles, 64 banks):
  // left to itself the compiler pairs the two taps of a row into ds_read2_b64, which the
  // LDS services as two 16-lane-group accesses at half the rate (8 cycles, 32 banks) —
  // config 4: 774 -> 694 us (r16).  A volatile LDS load is not merged; its order relative
  // to the other taps is the program order anyway.
  auto tap = [&](const char* p) __attribute__((always_inline)) -> Slot {
    if constexpr (sizeof(Slot) == 8) {
      typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
      typedef const volatile __attribute__((address_space(3))) u32x2* lds_ptr;
      const u32x2 q = *(lds_ptr)(p);
      return make_uint2(q.x, q.y);
    } else {
      return *reinterpret_cast<const Slot*>(p);
    }
  };
  // sample the views staged in an LDS buffer (all, or those of `pass`) into channel pairs
  auto sample_views = [&](const char* buf, bool all, int pass, f2 (&sv)[NP][NV]) __attribute__((always_inline)) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      if (!all && rs.get(v).pass != pass) continue;
      if constexpr (PAIR) {
        // two slots per view (rows y0, y1), one v_dot2_f32_bf16 per row and channel
        const Slot a = tap(buf + anw[v]);
        const Slot cq = tap(buf + asw[v]);
        const bf16x2_t w1 = __builtin_bit_cast(bf16x2_t, wq[v][1]);
        const uint32_t an[4] = {a.x, a.y, a.z, a.w}, as[4] = {cq.x, cq.y, cq.z, cq.w};
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          float o[2];
#pragma unroll
          for (int h = 0; h < 2; ++h)
            o[h] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, as[2 * q + h]), w1,
                                                   dot2_bf16_from0(an[2 * q + h], wq[v][0]), false);
          sv[q][v] = f2{o[0], o[1]};
        }
        if (v & 1) __builtin_amdgcn_sched_barrier(0);
        continue;
      }
      const Slot a = tap(buf + anw[v]);
      const Slot bq = tap(buf + anw[v] + kSlotB);
      const Slot cq = tap(buf + asw[v]);
      const Slot d = tap(buf + asw[v] + kSlotB);
      const f2 w0 = splat<0>(wp[v][0]), w1 = splat<1>(wp[v][0]), w2 = splat<0>(wp[v][1]), w3 = splat<1>(wp[v][1]);
#pragma unroll
      for (int q = 0; q < NP; ++q)
        sv[q][v] = pk_fma(slot_pair(d, q), w3,
                          pk_fma(slot_pair(cq, q), w2, pk_fma(slot_pair(bq, q), w1, slot_pair(a, q) * w0)));
      if (v & 1) __builtin_amdgcn_sched_barrier(0);   // at most two views' taps in flight
    }
  };
  // SMXF: range of the max-free softmax's denominators over every channel of this voxel.
  // Outside [2^-100, 2^120] (|s| beyond ~70: overflow, or underflow in every view) the wave
  // recomputes its voxels with the exact gather path after the channel loop (rare; NaNs do
  // not trip it — a NaN sample gives a NaN value in either form, as in the reference).
  constexpr bool kDeferredGuard = NV == 4 && (sizeof(TIn) == 2 || CL == 0);   // (f32 channels-last: spills)
  float dmx = 0.f, dmn = INFINITY;
  auto range_fallback = [&]() __attribute__((always_inline)) {
    if constexpr (SMXF && kDeferredGuard) {
      if (__builtin_amdgcn_ballot_w64(!(dmx <= 0x1p120f) || !(dmn >= 0x1p-100f))) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the fast values' stores land first
        // the voxel's coordinates formed again from its index (opaque to the compiler, so that
        // the prologue's coordinates are not kept live across the channel loop for this path)
        int v2 = vox;
        asm volatile("" : "+v"(v2));
        float c2[3];
        if (cub) {
          cuboid_coord(cub + b * MVN_CUBOID_FLOATS, Vx, v2 / (Vy * Vz), (v2 / Vz) % Vy, v2 % Vz, transfer, c2);
        } else {
          const float* cp = coords + (size_t(b) * nvox + v2) * 3;
          c2[0] = cp[0]; c2[1] = cp[1]; c2[2] = cp[2];
        }
        if (act)
          gather_voxel<AGG, TIn, TOut>(fb, Pb, cfb, out + size_t(b) * C * nvox + (out_cl ? size_t(v2) * C : v2),
                                       out_cl ? 1 : nvox, NV, C, H, W, c2[0], c2[1], c2[2], align_corners);
      }
    }
  };
  constexpr int NG = 4;                    // bf16 channels-last: groups per run of 16-byte stores
  uint2 cl_buf[NG - 1];
#pragma unroll
  for (int k = 0; k < NG - 1; ++k) cl_buf[k] = make_uint2(0u, 0u);
  auto aggregate = [&](int c0, const f2 (&sv)[NP][NV], float (&r)[G]) __attribute__((always_inline)) {
    if constexpr (SMXF) {
      // max-free softmax of the log2-scaled samples; the denominators' range is tracked over
      // all groups and checked once per voxel at the end (range_fallback).  8 views: at the
      // register limit of 3 waves per SIMD the loop-carried range spills, so the group checks
      // its own range and redoes itself max-first.
      float gmx = 0.f, gmn = INFINITY;
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        f2 den;
        const f2 o = softmax_pair_log2<NV, false>(sv[q], den);
        if constexpr (kDeferredGuard) {
          dmx = vmax3f(dmx, den.x, den.y);
          dmn = vmin3f(dmn, den.x, den.y);
        } else {
          gmx = vmax3f(gmx, den.x, den.y);
          gmn = vmin3f(gmn, den.x, den.y);
        }
        r[2 * q] = o.x;
        r[2 * q + 1] = o.y;
      }
      if constexpr (!kDeferredGuard) {
        if (__builtin_amdgcn_ballot_w64(!(gmx <= 0x1p120f) || !(gmn >= 0x1p-100f))) {
#pragma unroll
          for (int q = 0; q < NP; ++q) {
            f2 den;
            const f2 o = softmax_pair_log2<NV, true>(sv[q], den);
            r[2 * q] = o.x;
            r[2 * q + 1] = o.y;
          }
        }
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      f2 cf[NV];
      if constexpr (AGG == MVN_AGG_CONF) {
#pragma unroll
        for (int v = 0; v < NV; ++v) cf[v] = f2{cfb[v * C + c0 + 2 * q], cfb[v * C + c0 + 2 * q + 1]};
      }
      const f2 o = aggregate_pair<AGG>(sv[q], cf);
      r[2 * q] = o.x;
      r[2 * q + 1] = o.y;
    }
  };
  // The group's G output values of this voxel: NCDHW planes, or the voxel's channels-last
  // record (config 5).  bf16 NCDHW planes are direct 2-byte stores (r14: once the stores were
  // deferred past the next commit they beat 16-byte rows gathered through LDS, 542 -> 530 us).
  auto store_out = [&](int c0, const float (&r)[G]) __attribute__((always_inline)) {
    if constexpr (G == 4 && CL != 0) {      // (launch_x4 sends channels-last 8-view calls to the tiled kernel)
      // c0 is block-uniform; readfirstlane keeps it scalar (soffset operands must be SGPRs)
      const uint32_t soff = __builtin_amdgcn_readfirstlane(uint32_t(c0) * uint32_t(sizeof(TOut)));
      if constexpr (sizeof(TOut) == 2) {
        // bf16 channels-last: NG groups' 8-byte pieces of the voxel's record are held in
        // registers and go out as 16-byte stores of consecutive channels
        const uint2 cur = make_uint2(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]));
        const int gi = (c0 / G) % NG;
        if (gi == NG - 1) {
#pragma unroll
          for (int k = 0; k + 1 < NG; k += 2) {
            const uint2 hi = k + 1 == NG - 1 ? cur : cl_buf[k + 1];
            store_b128_padded(
                __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int,
                                   make_uint4(cl_buf[k].x, cl_buf[k].y, hi.x, hi.y)),
                ors, ooff_cl, soff - uint32_t((NG - 1 - k) * G * sizeof(TOut)));
          }
        } else if (c0 + G >= C) {            // C / G not a multiple of NG: the tail group by itself
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int, cur),
                                                ors, ooff_cl, soff, 0);
#pragma unroll
          for (int k = 0; k < NG - 1; ++k)
            if (k < gi)
              __builtin_amdgcn_raw_buffer_store_b64(
                  __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int, cl_buf[k]), ors, ooff_cl,
                  soff - uint32_t((gi - k) * G * sizeof(TOut)), 0);
        } else {
#pragma unroll
          for (int k = 0; k < NG - 1; ++k)
            if (k == gi) cl_buf[k] = cur;
        }
        return;
      }
      store_b128_padded(
          __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int,
                             make_uint4(__float_as_uint(r[0]), __float_as_uint(r[1]), __float_as_uint(r[2]),
                                        __float_as_uint(r[3]))),
          ors, ooff_cl, soff);
      return;
    }
#pragma unroll
    for (int ch = 0; ch < G; ++ch)
      store_plane<TOut, S::STORE_F32>(r[ch], ors, ooff, uint32_t(c0 + ch) * uint32_t(nvox) * uint32_t(sizeof(TOut)));
  };
  auto consume = [&](const Slot* buf, int c0, float (&r)[G]) __attribute__((always_inline)) {
    f2 sv[NP][NV];
    sample_views(reinterpret_cast<const char*>(buf), true, 0, sv);
    aggregate(c0, sv, r);
    __builtin_amdgcn_sched_barrier(0);
  };

  // fast: the tap offsets before the staging starts, so that the per-view base pixels die here
  // (live into the multi-pass branch they spilled at 6 waves per SIMD)
  if constexpr (FAST != 0) tap_slots();
  if (npass == 1) {
    // ---- one pass: up to MC chunks per thread (chunk t + kThreads * i over the views'
    // concatenated chunk ranges), two LDS buffers, the next group's loads in flight --------
    uint32_t goff[MC], mask[MC];
    int s0[MC];
#pragma unroll
    for (int i = 0; i < MC; ++i) {
      const int k = i * kWaves * kLanesW + wid * kLanesW + lane;     // = t + kThreads * i unless PAIR
      int sel = 0;
#pragma unroll
      for (int u = 1; u < NV; ++u)
        if (rs.get(u).cw > 0 && k >= rs.get(u).cbase) sel = u;
      const Region r = rs.pick(sel);
      chunk_fields(r, sel, k - r.cbase, goff[i], s0[i], mask[i], k < total);
    }
    const int wfirst = __builtin_amdgcn_readfirstlane(wid * kLanesW);
    Chunk pre[MC][G];
    auto issue = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MC; ++i)
        if (wfirst + kWaves * kLanesW * i < total) load_group(pre[i], goff[i], c0);
    };
    auto commit = [&](Slot* buf) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < MC; ++i)
        if (wfirst + kWaves * kLanesW * i < total) write_group(buf, pre[i], s0[i], mask[i]);
    };
    issue(0);
    if constexpr (FAST == 0) tap_slots();
    commit(stageA);
    __syncthreads();
    // A group's outputs are stored after the NEXT group's commit: on gfx950 vmcnt counts
    // stores as well as loads, in issue order, so stores issued at the end of a consume made
    // the commit's wait for the next group's loads also wait for their write acknowledgement.
    float r[G];
    for (int c0 = 0; c0 < C; c0 += 2 * G) {
      const bool more1 = c0 + G < C, more2 = c0 + 2 * G < C;
      if (more1) issue(c0 + G);
      consume(stageA, c0, r);
      if (!more1) { store_out(c0, r); break; }
      commit(stageB);
      __builtin_amdgcn_sched_barrier(0);
      store_out(c0, r);
      __syncthreads();
      if (more2) issue(c0 + 2 * G);
      consume(stageB, c0 + G, r);
      if (!more2) { store_out(c0 + G, r); break; }
      commit(stageA);
      __builtin_amdgcn_sched_barrier(0);
      store_out(c0 + G, r);
      __syncthreads();
    }
    range_fallback();
    return;
  }

  // ---- several passes of whole views per channel group (close cameras) ---------------
  if constexpr (FAST == 0) tap_slots();
  for (int c0 = 0; c0 < C; c0 += G) {
    f2 sv[NP][NV];
    for (int pass = 0; pass < npass; ++pass) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {          // every thread stages chunks of each view of the pass
        const Region rv = rs.get(v);
        if (rv.pass != pass) continue;
        const int nch = rv.cend - rv.cbase;
        for (int li = wid * kLanesW + lane; li < nch; li += kWaves * kLanesW) {
          uint32_t goff, mask;
          int s0;
          chunk_fields(rv, v, li, goff, s0, mask, true);
          Chunk pre[G];
          load_group(pre, goff, c0);
          write_group(stageA, pre, s0, mask);
        }
      }
      __syncthreads();
      sample_views(reinterpret_cast<const char*>(stageA), false, pass, sv);
      __syncthreads();
    }
    float r[G];
    aggregate(c0, sv, r);
    store_out(c0, r);
  }
  range_fallback();
}

}  // namespace

// Returns MVN_OK, an error code, or 1 when this kernel does not apply (the caller then
// runs unproject_tiled).
template <int AGG, typename TIn, typename TOut>
int launch_x4(const void* feat, const float* P, const float* coords, const float* cub, int transfer,
              const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
              int align_corners, int out_cl, int fast, hipStream_t s) {
  if (H > 32000 || W > 32000 || W % 4 != 0) return 1;
  // 4 views: tile per input dtype (A/B at the bench configs), f32 4x8x16,
  // bf16 4x8x8; 8 views: 2-channel slots, NCDHW output only
  const bool four = N == 4 && C % 4 == 0, eight = N == 8 && C % 2 == 0 && !out_cl;
  if (!four && !eight) return 1;
  if ((long long)N * C * H * W * sizeof(TIn) >= (1LL << 31) ||
      (long long)C * Vx * Vy * Vz * sizeof(TOut) >= (1LL << 31))
    return MVN_ERR_SHAPE;
  const int knob = unproject_lds_slot_budget();
  const int budget = knob > 0 ? knob : 1 << 30;
  auto go = [&](auto shape, auto cl) {
    constexpr int K = decltype(shape)::value, CL = decltype(cl)::value;
    using S = X4Shape<K>;
    const long long nb = (long long)B * ((Vx + S::TX - 1) / S::TX) * ((Vy + S::TY - 1) / S::TY) *
                         ((Vz + S::TZ - 1) / S::TZ);
    if (nb > INT_MAX) return MVN_ERR_SHAPE;
    if constexpr (K == 2 && CL == 0 && MVN_FAST_BF16_SHAPE == 4) {
      if (fast) {       // bf16 maps, NCDHW, fast arithmetic: the 8x8x8 tile (X4Shape<4>)
        using S4 = X4Shape<4>;
        const long long nb4 = (long long)B * ((Vx + S4::TX - 1) / S4::TX) * ((Vy + S4::TY - 1) / S4::TY) *
                              ((Vz + S4::TZ - 1) / S4::TZ);
        if (nb4 > INT_MAX) return MVN_ERR_SHAPE;
        unproject_x4<AGG, TIn, TOut, 4, 0, 1><<<int(nb4), S4::THREADS, 0, s>>>(
            static_cast<const TIn*>(feat), P, coords, cub, transfer, conf, static_cast<TOut*>(out), B, C, H, W, Vx,
            Vy, Vz, align_corners, budget);
        return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
      }
    }
    if (fast)
      unproject_x4<AGG, TIn, TOut, K, CL, 1><<<int(nb), S::THREADS, 0, s>>>(
          static_cast<const TIn*>(feat), P, coords, cub, transfer, conf, static_cast<TOut*>(out), B, C, H, W, Vx, Vy,
          Vz, align_corners, budget);
    else
      unproject_x4<AGG, TIn, TOut, K, CL, 0><<<int(nb), S::THREADS, 0, s>>>(
          static_cast<const TIn*>(feat), P, coords, cub, transfer, conf, static_cast<TOut*>(out), B, C, H, W, Vx, Vy,
          Vz, align_corners, budget);
    return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
  };
  using NC = std::integral_constant<int, 0>;
  using CLv = std::integral_constant<int, 1>;
  if (eight) return go(std::integral_constant<int, 3>{}, NC{});
  using K4 = std::integral_constant<int, sizeof(TIn) == 2 ? 2 : 0>;
  return out_cl ? go(K4{}, CLv{}) : go(K4{}, NC{});
}

// Diagnostics (mvn_debug_unproject_occupancy): resident blocks per CU of the softmax kernels.
int x4_blocks_per_cu(int bf16) {
  int n = 0;
  const hipError_t e =
      bf16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, unproject_x4<MVN_AGG_SOFTMAX, uint16_t, uint16_t, 2, 0, 0>,
                                                          X4Shape<2>::THREADS, 0)
           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, unproject_x4<MVN_AGG_SOFTMAX, float, float, 0, 0, 0>,
                                                          X4Shape<0>::THREADS, 0);
  return e == hipSuccess ? n : MVN_ERR_LAUNCH;
}

#define MVN_INSTANTIATE(AGG)                                                                                   \
  template int launch_x4<AGG, float, float>(const void*, const float*, const float*, const float*, int,        \
                                            const float*, void*, int, int, int, int, int, int, int, int, int,  \
                                            int, int, hipStream_t);                                            \
  template int launch_x4<AGG, uint16_t, uint16_t>(const void*, const float*, const float*, const float*, int,  \
                                                  const float*, void*, int, int, int, int, int, int, int, int, \
                                                  int, int, int, hipStream_t);                                      \
  template int launch_x4<AGG, uint16_t, float>(const void*, const float*, const float*, const float*, int,     \
                                               const float*, void*, int, int, int, int, int, int, int, int,    \
                                               int, int, int, hipStream_t);
MVN_INSTANTIATE(MVN_AGG_SUM)
MVN_INSTANTIATE(MVN_AGG_MAX)
MVN_INSTANTIATE(MVN_AGG_SOFTMAX)
MVN_INSTANTIATE(MVN_AGG_CONF)
#undef MVN_INSTANTIATE

}  // namespace unproj
}  // namespace mvn
