// Four-view unprojection for gfx950 — the production kernel behind mvn_unproject for the
// configurations of BASELINE.json (4 views, W % 4 == 0, C % 4 == 0).
//
// Contract and numerics: mvn/utils/op.py:99-163 exactly as unproject_tiled.hip (sum / max /
// conf bit-exact with the reference; softmax max-first with exp2 and one reciprocal, same
// op order as unproject_tiled's staged path, so the two kernels agree bit for bit).
//
// Work decomposition.  A voxel TILE (f32 maps 4 x 8 x 16, bf16 maps 4 x 8 x 8; one voxel per
// thread, z fastest) is unprojected by staging, per group of G = 4 channels, the views'
// footprint boxes of the tile into an LDS image, then bilinear-sampling that image:
//   * staging in CHUNKS of 4 x-consecutive pixels: one 16-byte (f32) / 8-byte (bf16) buffer
//     load per chunk and channel.  Chunks start at x % 4 == 0, so with W % 4 == 0 a chunk
//     lies wholly inside or wholly outside the image (the hardware range check of an
//     out-of-range offset returns zeros = padding_mode 'zeros'); the 4 x 4 (pixel x channel)
//     block a lane loads is transposed in registers into 4 slots of (4 channels) 16 bytes,
//     one ds_write_b128 each;
//   * two LDS buffers: group g+1's loads are in flight while group g is sampled;
//   * bilinear sampling and view aggregation on channel PAIRS with packed f32 arithmetic
//     (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32: per lane exactly the scalar fma / mul /
//     add of the reference order, two channels per instruction).
//
// Persistent blocks, pipelined across tiles (round 3).  A block walks tiles blockIdx.x,
// blockIdx.x + gridDim.x, ...  A tile's PROLOGUE — coordinates, the projection into all
// views (two IEEE divisions per view), the exact per-view footprint boxes (a wave butterfly
// and a block combine), the chunk descriptors and the first group's staging loads — used
// to run before the tile's channel loop with the LDS idle: 42 % of a block's life at
// config 2 (profiles/r12_x4_stamps.txt).  Here the NEXT tile's prologue runs inside the
// current tile's channel loop, where the LDS array (the loop's bound) is busy and VALU
// issue has room:
//   group 0           the next tile's coordinate loads are issued;
//   group proj_g (2)  after the commit of group 3 (the staging registers are free there),
//                     the next tile is projected: each thread parks its voxel's continuous
//                     grid_sample coordinates (ix, iy per view, -inf for voxels that sample
//                     nothing) in a thread-private LDS slot, and the per-wave box partials go
//                     to `red` (the butterfly of round 2);
//   last group        its loads were committed, so the staging registers are free again:
//                     the next tile's regions and chunk descriptors are formed and its group
//                     0 is issued, in flight while the last group is sampled;
//   tile switch       the parked coordinates become the bilinear weights / base pixels (the
//                     same f32 ops as before: floor, subtract, multiply — bit-identical), and
//                     group 0 is committed into the buffer the last group did not use.
// Only the first tile of a block runs its prologue exposed.  Tiles whose footprints need
// several LDS passes (close cameras) or exceed a buffer (global gather) are processed
// unpipelined by a separate, non-inlined function (its registers do not count against the
// pipelined loop's); the tile after them runs its prologue exposed.
#include <algorithm>

#include "unproject_common.hpp"

namespace mvn {
namespace unproj {
namespace {

constexpr int NV = 4, G = 4;                 // views, channels per LDS slot / group
constexpr uint32_t kSlotB = 16;              // bytes per LDS slot (4 f32 channels)
#ifndef X4_SLOTS_F32
#define X4_SLOTS_F32 2000
#endif
#ifndef X4_SLOTS_BF16
#define X4_SLOTS_BF16 1000
#endif
#ifndef X4_STAGGER
#define X4_STAGGER 0
#endif
#ifndef X4_PROJ_SPREAD
#define X4_PROJ_SPREAD 0
#endif
#ifndef X4_PROJ_SPLIT
#define X4_PROJ_SPLIT 0
#endif
#ifndef X4_GRID_MODE
#define X4_GRID_MODE 0
#endif
#ifndef X4_INLOOP
#define X4_INLOOP 1
#endif
#ifndef X4_TAPS_INFLIGHT
#define X4_TAPS_INFLIGHT 2
#endif

// Voxel tile per block and LDS image size (slots).  Footprint slots per voxel at the bench
// configs: 2.2 (4x8x16), 2.2 (4x8x8).  LDS per block: 2 buffers + the park (2 x 16 bytes per
// thread) + red: f32 80,896 B (2 blocks per CU), bf16 40,448 B (4 blocks per CU) of 160 KiB.
template <int K> struct X4Shape;
// SLOW: capacity of the per-block list of tiles deferred to the unpipelined path (the
// launcher keeps the tiles per block below it).
template <> struct X4Shape<0> {
  static constexpr int TX = 4, TY = 8, TZ = 16, THREADS = 512, SLOTS = X4_SLOTS_F32, MC = 2, SLOW = 256;
};
template <> struct X4Shape<1> {
  static constexpr int TX = 4, TY = 8, TZ = 8, THREADS = 256, SLOTS = X4_SLOTS_BF16, MC = 2, SLOW = 64;
};

struct X4Args {
  const void* feat;
  const float* P;
  const float* coords;
  const float* cub;
  const float* conf;
  void* out;
  int transfer, B, C, H, W, Vx, Vy, Vz, align_corners, budget, ntiles;
};

// Per-view LDS regions (block-uniform, scalar registers), packed 3 words per view —
// (x0 + 1, y0 + 1), (bw, bh), sbase | cbase << 13 | pass << 24 — the derived fields
// recomputed on use (12 SGPRs per view unpacked spilled to VGPR lanes in round 2).
__device__ __forceinline__ Region make_region(int x0, int y0, int bw, int bh, int sbase, int cbase, int pass) {
  Region r;
  r.x0 = x0; r.y0 = y0; r.bw = bw; r.bh = bh; r.sbase = sbase; r.cbase = cbase; r.pass = pass;
  r.pitch = bw | 1;                                          // odd: spreads rows over banks
  r.xa = x0 & ~3;                                            // chunk origin, x % 4 == 0
  r.cw = bw ? (x0 + bw - r.xa + 3) >> 2 : 0;                 // chunks per row
  r.cend = cbase + r.cw * bh;
  r.inv_cw = r.cw ? __builtin_amdgcn_rcpf(float(r.cw)) : 0.f;
  return r;
}
struct RegionSet {
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
  // u per lane: plain selects (9 v_cndmask) — through readfirstlane each select became a
  // branch tree with exec masking (profiles/r13_x4_stamps.txt)
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

// Per-voxel sampling geometry: bilinear weights (nw, ne), (sw, se), base pixel and "samples
// the image" per view, from the parked continuous coordinates (ix, iy) — the same f32 ops as
// the projection they replace (floor, subtract, multiply).
struct Geometry {
  int fx[NV], fy[NV];
  f2 wp[NV][2];
  bool has[NV];
};
__device__ __forceinline__ void load_geometry(const float4* __restrict__ park, int t, int nthreads, int H, int W,
                                              Geometry& g) {
  const float4 a = park[t], c = park[nthreads + t];
  const float px[NV] = {a.x, a.z, c.x, c.z}, py[NV] = {a.y, a.w, c.y, c.w};
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const float fx0 = floorf(px[v]), fy0 = floorf(py[v]);
    const bool h = (fx0 >= -1.f) & (fx0 < float(W)) & (fy0 >= -1.f) & (fy0 < float(H));
    const float tx_ = px[v] - fx0, sx_ = 1.f - tx_, ty_ = py[v] - fy0, sy_ = 1.f - ty_;
    g.wp[v][0] = f2{h ? sy_ * sx_ : 0.f, h ? sy_ * tx_ : 0.f};
    g.wp[v][1] = f2{h ? ty_ * sx_ : 0.f, h ? ty_ * tx_ : 0.f};
    g.fx[v] = h ? int(fx0) : 0;
    g.fy[v] = h ? int(fy0) : 0;
    g.has[v] = h;
  }
}
// LDS byte offsets of each view's north-west and south-west taps (the exact boxes contain
// every voxel's base pixel by construction; voxels that sample nothing read the zero slots)
__device__ __forceinline__ void tap_slots(const RegionSet& rs, const Geometry& g, int zero_slot, uint32_t (&anw)[NV],
                                          uint32_t (&asw)[NV]) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const Region rv = rs.get(v);
    const int slot = rv.sbase + (g.fy[v] - rv.y0) * rv.pitch + (g.fx[v] - rv.x0);
    anw[v] = uint32_t(g.has[v] ? slot : zero_slot) * kSlotB;
    asw[v] = uint32_t(g.has[v] ? slot + rv.pitch : zero_slot) * kSlotB;
  }
}
// Chunk (li of a view's range) -> global byte offset in the frame's maps (kOob outside the
// image), first LDS slot, and the mask of its 4 pixels inside the view's box (empty when
// !live).
__device__ __forceinline__ void chunk_fields(const Region& r, int sel, int li, int C, int H, int W, uint32_t E,
                                             uint32_t& goff, int& s0, uint32_t& mask, bool live) {
  const int HW = H * W;
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
}
// Bilinear samples of the views staged in an LDS buffer (all, or those of `pass`), as
// channel pairs (op.py:133-134 with the grid_sample recipe of unproject_common.hpp).
__device__ __forceinline__ void sample_views(const uint4* buf, const RegionSet& rs, bool all, int pass,
                                             const uint32_t (&anw)[NV], const uint32_t (&asw)[NV], const Geometry& g,
                                             f2 (&sv)[2][NV]) {
  const char* bb = reinterpret_cast<const char*>(buf);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    if (!all && rs.get(v).pass != pass) continue;
    const uint4 a = *reinterpret_cast<const uint4*>(bb + anw[v]);
    const uint4 bq = *reinterpret_cast<const uint4*>(bb + anw[v] + kSlotB);
    const uint4 cq = *reinterpret_cast<const uint4*>(bb + asw[v]);
    const uint4 d = *reinterpret_cast<const uint4*>(bb + asw[v] + kSlotB);
    const f2 w0 = splat<0>(g.wp[v][0]), w1 = splat<1>(g.wp[v][0]), w2 = splat<0>(g.wp[v][1]),
             w3 = splat<1>(g.wp[v][1]);
    sv[0][v] = pk_fma(lo2(d), w3, pk_fma(lo2(cq), w2, pk_fma(lo2(bq), w1, lo2(a) * w0)));
    sv[1][v] = pk_fma(hi2(d), w3, pk_fma(hi2(cq), w2, pk_fma(hi2(bq), w1, hi2(a) * w0)));
    if (X4_TAPS_INFLIGHT == 1 || (v & 1)) __builtin_amdgcn_sched_barrier(0);   // taps of at most X4_TAPS_INFLIGHT views in flight
  }
}
template <int AGG>
__device__ __forceinline__ void aggregate(int c0, int C, const float* __restrict__ cfb, const f2 (&sv)[2][NV],
                                          float (&r)[G]) {
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
}

// Output of one group (G channels of this voxel): NCDHW planes, or channels-last records
// (config 5; bf16 records leave as 16-byte stores of NG_CL groups held in registers).
constexpr int NG_CL = 4;
template <typename TOut, bool OUT_CL>
struct GroupStore {
  __amdgpu_buffer_rsrc_t ors;
  uint32_t off;                      // NCDHW: the voxel's byte offset; channels-last: its record's
  uint2 held[OUT_CL && sizeof(TOut) == 2 ? NG_CL - 1 : 1];
  __device__ __forceinline__ void put(int c0, int C, int nvox, const float (&r)[G]) {
    if constexpr (!OUT_CL) {
#pragma unroll
      for (int ch = 0; ch < G; ++ch)
        store_plane<TOut>(r[ch], ors, off, uint32_t(c0 + ch) * uint32_t(nvox) * uint32_t(sizeof(TOut)));
    } else {
      // c0 is block-uniform; readfirstlane keeps it scalar (soffset operands must be SGPRs)
      const uint32_t soff = __builtin_amdgcn_readfirstlane(uint32_t(c0) * uint32_t(sizeof(TOut)));
      if constexpr (sizeof(TOut) == 2) {
        const uint2 cur = make_uint2(pack_bf16x2(r[0], r[1]), pack_bf16x2(r[2], r[3]));
        const int gi = (c0 / G) % NG_CL;
        if (gi == NG_CL - 1) {
#pragma unroll
          for (int k = 0; k + 1 < NG_CL; k += 2) {
            const uint2 hi = k + 1 == NG_CL - 1 ? cur : held[k + 1];
            store_b128_padded(__builtin_bit_cast(u32x4_t, make_uint4(held[k].x, held[k].y, hi.x, hi.y)), ors, off,
                              soff - uint32_t((NG_CL - 1 - k) * G * sizeof(TOut)));
          }
        } else if (c0 + G >= C) {            // C / G not a multiple of NG_CL: the tail groups by themselves
          typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, cur), ors, off, soff, 0);
#pragma unroll
          for (int k = 0; k < NG_CL - 1; ++k)
            if (k < gi)
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, held[k]), ors, off,
                                                    soff - uint32_t((gi - k) * G * sizeof(TOut)), 0);
        } else {
#pragma unroll
          for (int k = 0; k < NG_CL - 1; ++k)
            if (k == gi) held[k] = cur;
        }
      } else {
        store_b128_padded(__builtin_bit_cast(u32x4_t, make_uint4(__float_as_uint(r[0]), __float_as_uint(r[1]),
                                                                 __float_as_uint(r[2]), __float_as_uint(r[3]))),
                          ors, off, soff);
      }
    }
  }
};

// ---- tiles that do not take the pipelined loop ---------------------------------------------
// A view's footprint larger than an LDS buffer: every voxel gathers its taps from global
// memory; footprints larger than the buffer together: several passes of whole views per
// channel group.  Run after the pipelined loop (the block's slow tiles are listed in LDS), so
// that nothing of the loop is live around it: its registers do not add to the loop's.
template <int AGG, typename TIn, typename TOut, int K, bool OUT_CL>
__device__ __forceinline__ void x4_unpipelined_tile(const X4Args& a, int b, int vox, bool act, float cx,
                                                              float cy, float cz, RegionSet rs, int npass,
                                                              uint4* stage, const float4* park) {
  using S = X4Shape<K>;
  constexpr int kThreads = S::THREADS, kBuf = S::SLOTS;
  const int t = threadIdx.x;
  const int C = a.C, H = a.H, W = a.W, HW = H * W, nvox = a.Vx * a.Vy * a.Vz;
  constexpr uint32_t E = sizeof(TIn);
  const TIn* fb = static_cast<const TIn*>(a.feat) + size_t(b) * NV * C * HW;
  const float* cfb = a.conf ? a.conf + size_t(b) * NV * C : nullptr;
  TOut* ob = static_cast<TOut*>(a.out) + size_t(b) * C * nvox;
  if (npass < 0) {
    if (act)
      gather_voxel<AGG, TIn, TOut>(fb, a.P + size_t(b) * NV * 12, cfb, ob + (OUT_CL ? size_t(vox) * C : vox),
                                   OUT_CL ? 1 : nvox, NV, C, H, W, cx, cy, cz, a.align_corners);
  } else {
    Geometry g;
    load_geometry(park, t, kThreads, H, W, g);
    uint32_t anw[NV], asw[NV];
    tap_slots(rs, g, kBuf - 2, anw, asw);
    const __amdgpu_buffer_rsrc_t frs = make_rsrc(fb, uint32_t(size_t(NV) * C * HW * E));
    GroupStore<TOut, OUT_CL> st;
    st.ors = make_rsrc(ob, uint32_t(size_t(C) * nvox * sizeof(TOut)));
    st.off = act ? uint32_t(vox) * uint32_t(OUT_CL ? C : 1) * uint32_t(sizeof(TOut)) : kOob;
    for (int c0 = 0; c0 < C; c0 += G) {
      f2 sv[2][NV];
      for (int pass = 0; pass < npass; ++pass) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {          // every thread stages chunks of each view of the pass
          const Region rv = rs.get(v);
          if (rv.pass != pass) continue;
          const int nch = rv.cend - rv.cbase;
          for (int li = t; li < nch; li += kThreads) {
            uint32_t go, mk;
            int so;
            chunk_fields(rv, v, li, C, H, W, E, go, so, mk, true);
            typename ChunkT<TIn>::type q[G];
#pragma unroll
            for (int k = 0; k < G; ++k) q[k] = load_chunk<TIn>(frs, go, uint32_t((c0 + k) * HW) * E);
#pragma unroll
            for (int p = 0; p < 4; ++p)
              if (mk & (1u << p))
                stage[so + p] = make_uint4(chunk_px(q[0], p), chunk_px(q[1], p), chunk_px(q[2], p), chunk_px(q[3], p));
          }
        }
        __syncthreads();
        sample_views(stage, rs, false, pass, anw, asw, g, sv);
        __syncthreads();
      }
      float r[G];
      aggregate<AGG>(c0, C, cfb, sv, r);
      st.put(c0, C, nvox, r);
    }
  }
  __syncthreads();             // LDS (stage / red) free for the next tile's exposed prologue
}

template <int AGG, typename TIn, typename TOut, int K, bool OUT_CL>
__global__ __launch_bounds__(X4Shape<K>::THREADS) __attribute__((amdgpu_waves_per_eu(4))) void unproject_x4(
    const X4Args a) {
  using S = X4Shape<K>;
  constexpr int TX = S::TX, TY = S::TY, TZ = S::TZ;
  constexpr int kThreads = S::THREADS, kBuf = S::SLOTS, MC = S::MC, kWaves = kThreads / kWave;
  static_assert(TX * TY * TZ == kThreads, "one voxel per thread");
  // per buffer: image slots [0, kTrash), 64 per-lane trash slots (the masked-off pixels of
  // a bf16 chunk are written there: no exec-mask branch per write), 2 zero slots
  constexpr int kZeroSlot = kBuf - 2, kTrash = kBuf - 2 - kWave;
  constexpr uint32_t E = sizeof(TIn);

  __shared__ uint4 stage[2 * kBuf];
  __shared__ float4 park[2 * kThreads];     // thread-private: (ix, iy) of views 0, 1 | 2, 3
  __shared__ int red[kWaves][16];           // per-wave box partials: 4 views x (min x, -max x, min y, -max y)
  __shared__ int slow[S::SLOW];             // this block's tiles left for the unpipelined path

  const TIn* __restrict__ feat = static_cast<const TIn*>(a.feat);
  const int C = a.C, H = a.H, W = a.W, Vx = a.Vx, Vy = a.Vy, Vz = a.Vz;
  const int nTx = (Vx + TX - 1) / TX, nTy = (Vy + TY - 1) / TY, nTz = (Vz + TZ - 1) / TZ;
  const int nf = nTx * nTy * nTz;
  const int nvox = Vx * Vy * Vz;
  const int HW = H * W;
  const int t = threadIdx.x, lane = t & (kWave - 1), wid = t / kWave;
  const int wfirst = __builtin_amdgcn_readfirstlane(wid * kWave);

  // ---- this thread's voxel inside a tile ---------------------------------------------
  // A wave takes 64 / TZ consecutive y-rows of one x-plane.  A ds_read_b128 is serviced in
  // four groups of 16 lanes ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same + 32);
  // lanes are assigned to voxels so that each group is a compact 2 (y) x 8 (z) patch, whose
  // taps land on fewer, closer pixels: fewer LDS bank conflicts (tools/lds_conflicts.py).
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
  const int dX = vt / (TZ * TY), dY = (vt / TZ) % TY, dZ = vt % TZ;

  if (t < 4) stage[(t >> 1) * kBuf + kZeroSlot + (t & 1)] = make_uint4(0u, 0u, 0u, 0u);

  // tile -> frame, and this thread's voxel (z-tiles fastest).  XCD slabs: block b runs on
  // XCD b % 8 and walks tiles b + k * gridDim.x (gridDim.x % 8 == 0), so tile % 8 is its
  // XCD; each XCD takes the same contiguous slab of every frame (its maps stay in that
  // XCD's L2).
  auto locate = [&](int tile, int& b, int& X, int& Y, int& Z) __attribute__((always_inline)) {
    int L = tile;
    if (nf % 8 == 0) {
      const int xcd = tile % 8, k = tile / 8, slab = nf / 8;
      L = (k / slab) * nf + xcd * slab + k % slab;
    }
    const int tz = L % nTz; L /= nTz;
    const int ty = L % nTy; L /= nTy;
    const int tx = L % nTx;
    b = L / nTx;
    X = tx * TX + dX; Y = ty * TY + dY; Z = tz * TZ + dZ;
  };
  auto coords_of = [&](int b, int X, int Y, int Z, float& cx, float& cy, float& cz) __attribute__((always_inline)) {
    const bool act = (X < Vx) & (Y < Vy) & (Z < Vz);
    if (a.cub) {
      float o[3];
      cuboid_coord(a.cub + b * MVN_CUBOID_FLOATS, Vx, X, Y, Z, a.transfer, o);
      cx = o[0]; cy = o[1]; cz = o[2];
    } else {
      const int vox = act ? (X * Vy + Y) * Vz + Z : 0;
      const float* cp = a.coords + (size_t(b) * nvox + vox) * 3;
      cx = cp[0]; cy = cp[1]; cz = cp[2];
    }
  };

  // Project the voxel into every view (op.py:117-130, exact recipe of unproject_common.hpp),
  // park (ix, iy) per view (-inf: invalid voxel / inactive lane), and write the wave's box
  // partials.  The 16 per-wave reductions (4 views x min x0, max x1, min y0, max y1; maxima
  // as minima of negated values) run as one transposing butterfly: lanes 32 apart swap halves
  // of their 16 values (v_permlane32_swap), then rows 16 apart (v_permlane16_swap), then
  // lanes 8 and "4" apart (DPP row_ror:8, row_half_mirror) each keep one of two, and the
  // quads reduce — lane l ends with value (l >> 2) & 15 of the whole wave.
  // One view: project (per-view wave decision between the exact fast division and IEEE '/',
  // bit-identical either way) and park (ix, iy) — -inf for an invalid voxel / inactive lane.
  auto project_view = [&](int b, bool act, float cx, float cy, float cz, int u) __attribute__((always_inline)) {
    const float* Pv = a.P + (size_t(b) * NV + u) * 12;
    const Homog hp = homog(Pv, cx, cy, cz);
    const bool wave_fast = __builtin_amdgcn_ballot_w64(!div_core_safe(hp)) == 0;
    const Recip rH = recip_refined(float(H)), rW = recip_refined(float(W));
    const Proj p = wave_fast ? project_h<true>(hp, H, W, a.align_corners, rH, rW)
                             : project_h<false>(hp, H, W, a.align_corners, rH, rW);
    reinterpret_cast<float2*>(park)[(u >> 1) * 2 * kThreads + 2 * t + (u & 1)] =
        make_float2((act & !p.invalid) ? p.ix : -INFINITY, p.iy);
  };
  // The wave's box partials from the parked coordinates of all views.
  auto box_partials = [&]() __attribute__((always_inline)) {
    const float4 pa = park[t], pc = park[kThreads + t];
    const float px[NV] = {pa.x, pa.z, pc.x, pc.z}, py[NV] = {pa.y, pa.w, pc.y, pc.w};
    int q16[16];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const float fx0 = floorf(px[u]), fy0 = floorf(py[u]);
      const bool h = (fx0 >= -1.f) & (fx0 < float(W)) & (fy0 >= -1.f) & (fy0 < float(H));
      q16[4 * u + 0] = h ? int(fx0) : INT_MAX;
      q16[4 * u + 1] = h ? -int(fx0) : INT_MAX;
      q16[4 * u + 2] = h ? int(fy0) : INT_MAX;
      q16[4 * u + 3] = h ? -int(fy0) : INT_MAX;
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
    if ((lane & 3) == 0) red[wid][(lane >> 2) & 15] = q1;
  };
  // Project the voxel into every view (op.py:117-130, exact recipe of unproject_common.hpp),
  // park the coordinates and write the wave's box partials.  The 16 per-wave reductions (4
  // views x min x0, max x1, min y0, max y1; maxima as minima of negated values) run as one
  // transposing butterfly: lanes 32 apart swap halves of their 16 values (v_permlane32_swap),
  // then rows 16 apart (v_permlane16_swap), then lanes 8 and "4" apart (DPP row_ror:8,
  // row_half_mirror) each keep one of two, and the quads reduce — lane l ends with value
  // (l >> 2) & 15 of the whole wave.
  auto project_tile = [&](int b, bool act, float cx, float cy, float cz) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NV; ++u) project_view(b, act, cx, cy, cz, u);
    box_partials();
  };

  // After a barrier behind project_tile: the block's exact per-view boxes (lane 4v+k
  // reduces component k of view v over the waves), laid out back to back in an LDS buffer
  // (+1 px east / south for the second taps); views that do not fit start another pass.
  // npass: 1, >1 (several passes of whole views), or -1 (a single view exceeds a buffer).
  auto regions = [&](RegionSet& rs, int& npass, int& total) __attribute__((always_inline)) {
    int part = INT_MAX;
    {
      const int idx = lane & 15;
#pragma unroll
      for (int q = 0; q < kWaves; ++q) part = min(part, red[q][idx]);
    }
    int snext = 0, cnext = 0, pass = 0, chunks0 = 0;
    bool too_big = false;
    const int lim = min(a.budget, kTrash);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int x0 = __builtin_amdgcn_readlane(part, 4 * v + 0), y0 = __builtin_amdgcn_readlane(part, 4 * v + 2);
      const int x1 = -__builtin_amdgcn_readlane(part, 4 * v + 1), y1 = -__builtin_amdgcn_readlane(part, 4 * v + 3);
      int bw = 0, bh = 0;
      if (x0 <= x1 && y0 <= y1) { bw = x1 - x0 + 2; bh = y1 - y0 + 2; }
      else { x0 = 0; y0 = 0; }
      const Region r0 = make_region(x0, y0, bw, bh, 0, 0, 0);
      const int area = r0.pitch * bh, nch = r0.cend;
      if (area > lim || nch > MC * kThreads) too_big = true;
      if (snext + area > lim || cnext + nch > MC * kThreads) { ++pass; snext = 0; cnext = 0; }
      rs.set(v, make_region(x0, y0, bw, bh, snext, cnext, pass));
      snext += area;
      cnext += nch;
      if (pass == 0) chunks0 = cnext;
    }
    npass = too_big ? -1 : pass + 1;
    total = chunks0;
  };

  // Chunk slot i of this thread: (k = t + kThreads * i) over the views' concatenated chunk
  // ranges — global offset, and LDS slot | pixel mask << 16 packed in one register.
  uint32_t goff[MC], slm[MC];
  auto descriptors = [&](const RegionSet& rs, int total) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < MC; ++i) {
      const int k = t + kThreads * i;
      int sel = 0;
#pragma unroll
      for (int u = 1; u < NV; ++u)
        if (rs.get(u).cw > 0 && k >= rs.get(u).cbase) sel = u;
      const Region r = rs.pick(sel);
      int s0;
      uint32_t mask;
      chunk_fields(r, sel, k - r.cbase, C, H, W, E, goff[i], s0, mask, k < total);
      slm[i] = (uint32_t(s0) & 0xffffu) | (mask << 16);
    }
  };
  // ONE chunk slot of registers (16 VGPRs f32, 8 bf16).  Chunk slot 0 of the next group is in
  // flight while a group is sampled; the tiles whose footprint has more chunks than threads
  // (8 % at config 2, 4 % at config 3 — tools/footprints.py) load and commit their further
  // slots right after, serialised.  Every element is (re)defined by issue — loaded, or zeroed
  // when the wave stages nothing in that slot — so it is dead between a commit and the next
  // issue (a conditional definition kept the registers live through the whole loop).
  using Chunk = typename ChunkT<TIn>::type;
  Chunk pre[G];
  __amdgpu_buffer_rsrc_t frs;
  int total = 0;
  auto issue = [&](int c0, int i) __attribute__((always_inline)) {
    if (wfirst + kThreads * i < total) {
#pragma unroll
      for (int k = 0; k < G; ++k) pre[k] = load_chunk<TIn>(frs, goff[i], uint32_t((c0 + k) * HW) * E);
    } else {
#pragma unroll
      for (int k = 0; k < G; ++k) pre[k] = Chunk{};
    }
  };
  // masked-off pixels: bf16 maps write them to the lane's trash slot (no exec-mask branch
  // per write), f32 maps branch (A/B at the bench configs: each is the faster for its dtype)
  auto commit = [&](uint4* buf, int i) __attribute__((always_inline)) {
    if (wfirst + kThreads * i < total) {
      const int s0 = int(slm[i] << 16) >> 16;       // signed: a row's first chunk may start left of the box
      const uint32_t mask = slm[i] >> 16;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint4 q = make_uint4(chunk_px(pre[0], p), chunk_px(pre[1], p), chunk_px(pre[2], p), chunk_px(pre[3], p));
        if constexpr (sizeof(TIn) == 2)
          buf[(mask & (1u << p)) ? s0 + p : kTrash + lane] = q;
        else if (mask & (1u << p))
          buf[s0 + p] = q;
      }
    }
  };
  // the further chunk slots of a group (big footprints only), loaded and committed in turn
  auto stage_rest = [&](uint4* buf, int c0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 1; i < MC; ++i)
      if (kThreads * i < total) {          // block-uniform
        issue(c0, i);
        commit(buf, i);
      }
  };

  // ---- the tile loop ---------------------------------------------------------------------
  const int ng = (C + G - 1) / G;                     // channel groups per tile
#if X4_PROJ_SPLIT
  // co-resident blocks (b and b + gridDim / 2 share a CU under in-order dispatch) project their
  // next tiles in different groups, so the projections do not coincide
  const int proj_want = (blockIdx.x >= gridDim.x / 2) ? X4_PROJ_SPLIT : 2;
#else
  const int proj_want = 2;
#endif
  // spread: views projected in groups proj_g .. proj_g+3, box partials in proj_g+4 (<= ng-2)
  const bool spread = X4_PROJ_SPREAD && ng >= NV + 3;
  const int proj_g = spread ? 1 : ng >= 2 ? min(proj_want, ng - 2) : -1;
  int tile = blockIdx.x;
  int ab = 0;                // LDS buffer of the current tile's group 0
  bool prepared = false;     // park + red of `tile` written (inside the previous tile's loop)
  bool prefetched = false;   // group 0 of `tile` issued into pre (single-pass tiles)
  RegionSet rs;
  int npass = 0;
  Geometry geo;
  uint32_t anw[NV], asw[NV];
  GroupStore<TOut, OUT_CL> st;
  int nslow = 0;
#if X4_STAGGER
  // desynchronise co-resident blocks (b and b + gridDim / 2): the second half starts later
  if (blockIdx.x >= gridDim.x / 2)
    for (int i = 0; i < X4_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
#endif
  while (tile < a.ntiles) {
    int b, X, Y, Z;
    locate(tile, b, X, Y, Z);
    const bool act = (X < Vx) & (Y < Vy) & (Z < Vz);
    const int vox = act ? (X * Vy + Y) * Vz + Z : 0;
    if (!prepared) {
      float cx, cy, cz;
      coords_of(b, X, Y, Z, cx, cy, cz);
      project_tile(b, act, cx, cy, cz);
      __syncthreads();
      regions(rs, npass, total);
    }
    const int next = tile + int(gridDim.x);
    const bool has_next = next < a.ntiles;
    if (npass != 1) {          // deferred to the unpipelined path after the loop
      if (t == 0) slow[nslow] = tile;
      ++nslow;
      __syncthreads();         // red is rewritten by the next tile's exposed prologue
      prepared = prefetched = false;
      ab = 0;
      tile = next;
      continue;
    }
    const float* cfb = a.conf ? a.conf + size_t(b) * NV * C : nullptr;
    st.ors = make_rsrc(static_cast<TOut*>(a.out) + size_t(b) * C * nvox, uint32_t(size_t(C) * nvox * sizeof(TOut)));
    st.off = act ? uint32_t(vox) * uint32_t(OUT_CL ? C : 1) * uint32_t(sizeof(TOut)) : kOob;
    load_geometry(park, t, kThreads, H, W, geo);

    // ---- one pass: up to MC chunks per thread (chunk t + kThreads * i over the views'
    // concatenated chunk ranges), two LDS buffers, the next group's loads in flight ------
    if (!prefetched) {
      frs = make_rsrc(feat + size_t(b) * NV * C * HW, uint32_t(size_t(NV) * C * HW * E));
      descriptors(rs, total);
      issue(0, 0);
    }
    tap_slots(rs, geo, kZeroSlot, anw, asw);
    commit(stage + ab * kBuf, 0);
    stage_rest(stage + ab * kBuf, 0);
    __syncthreads();

    bool projected = false;
    prefetched = false;
    float r[G];
    // A group's outputs are stored after the NEXT group's commit: on gfx950 vmcnt counts
    // stores as well as loads, in issue order, so stores issued at the end of a group made
    // the commit's wait for the next group's loads also wait for their write acknowledgement.
    for (int g = 0; g < ng; ++g) {
      const uint4* buf = stage + ((ab + g) & 1) * kBuf;
      if (g + 1 < ng) {
        issue((g + 1) * G, 0);
      } else if (projected) {
        // last group: its loads were committed, the staging registers are free — the next
        // tile's regions, chunk descriptors and group-0 loads
        regions(rs, npass, total);
        if (npass == 1) {
          int nb, nX, nY, nZ;
          locate(next, nb, nX, nY, nZ);
          frs = make_rsrc(feat + size_t(nb) * NV * C * HW, uint32_t(size_t(NV) * C * HW * E));
          descriptors(rs, total);
          issue(0, 0);
          prefetched = true;
        }
      }
      f2 sv[2][NV];
      sample_views(buf, rs, true, 0, anw, asw, geo, sv);
      aggregate<AGG>(g * G, C, cfb, sv, r);
      __builtin_amdgcn_sched_barrier(0);
      if (g + 1 < ng) {
        uint4* nbuf = stage + ((ab + g + 1) & 1) * kBuf;
        commit(nbuf, 0);
        __builtin_amdgcn_sched_barrier(0);
        st.put(g * G, C, nvox, r);
        stage_rest(nbuf, (g + 1) * G);
        if (has_next) {
          // the next tile's projection, in the slot between this group's commit and the
          // barrier (its coordinates are loaded here: the other waves and blocks cover it)
          if (spread) {
            const int u = g - proj_g;          // one view per group, then the box partials
            if (u >= 0 && u < NV) {
              int nb, nX, nY, nZ;
              locate(next, nb, nX, nY, nZ);
              float ncx, ncy, ncz;
              coords_of(nb, nX, nY, nZ, ncx, ncy, ncz);
              project_view(nb, (nX < Vx) & (nY < Vy) & (nZ < Vz), ncx, ncy, ncz, u);
            } else if (u == NV) {
              box_partials();
              projected = true;
            }
          } else if (g == proj_g) {
            int nb, nX, nY, nZ;
            locate(next, nb, nX, nY, nZ);
            float ncx, ncy, ncz;
            coords_of(nb, nX, nY, nZ, ncx, ncy, ncz);
            project_tile(nb, (nX < Vx) & (nY < Vy) & (nZ < Vz), ncx, ncy, ncz);
            projected = true;
          }
        }
        __syncthreads();
      } else {
        st.put(g * G, C, nvox, r);
      }
    }
    if (!has_next) break;
    if (!projected) {          // a single channel group: no slot inside the loop
      int nb, nX, nY, nZ;
      locate(next, nb, nX, nY, nZ);
      float ncx, ncy, ncz;
      coords_of(nb, nX, nY, nZ, ncx, ncy, ncz);
      project_tile(nb, (nX < Vx) & (nY < Vy) & (nZ < Vz), ncx, ncy, ncz);
      __syncthreads();
      regions(rs, npass, total);
    }
    prepared = true;
    ab = (ab + ng) & 1;        // the buffer the last group did not use
    tile = next;
  }

  // ---- the block's tiles that need several LDS passes or a global gather ----------------
  __syncthreads();
  for (int i = 0; i < nslow; ++i) {
    const int tl = slow[i];
    int b, X, Y, Z;
    locate(tl, b, X, Y, Z);
    const bool act = (X < Vx) & (Y < Vy) & (Z < Vz);
    float cx, cy, cz;
    coords_of(b, X, Y, Z, cx, cy, cz);
    project_tile(b, act, cx, cy, cz);
    __syncthreads();
    regions(rs, npass, total);
    x4_unpipelined_tile<AGG, TIn, TOut, K, OUT_CL>(a, b, act ? (X * Vy + Y) * Vz + Z : 0, act, cx, cy, cz, rs, npass,
                                                   stage, park);
  }
}

}  // namespace

// Blocks of a kernel resident per CU (its LDS and registers), queried once per kernel.
template <auto KERN>
int resident_blocks_per_cu(int threads) {
  static const int n = [threads] {
    int k = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&k, KERN, threads, 0) != hipSuccess || k <= 0) k = 1;
    return k;
  }();
  return n;
}

// Returns MVN_OK, an error code, or 1 when this kernel does not apply (the caller then
// runs unproject_tiled).
template <int AGG, typename TIn, typename TOut>
int launch_x4(const void* feat, const float* P, const float* coords, const float* cub, int transfer,
              const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
              int align_corners, int out_cl, hipStream_t s) {
  if (N != 4 || W % 4 != 0 || C % 4 != 0 || H > 32000 || W > 32000) return 1;
  if ((long long)N * C * H * W * sizeof(TIn) >= (1LL << 31) ||
      (long long)C * Vx * Vy * Vz * sizeof(TOut) >= (1LL << 31))
    return MVN_ERR_SHAPE;
  const int knob = unproject_lds_slot_budget();
  // tile per input dtype: f32 4x8x16 (512 threads), bf16 4x8x8 (256)
  constexpr int K = sizeof(TIn) == 2 ? 1 : 0;
  using S = X4Shape<K>;
  const long long nt = (long long)B * ((Vx + S::TX - 1) / S::TX) * ((Vy + S::TY - 1) / S::TY) *
                       ((Vz + S::TZ - 1) / S::TZ);
  if (nt > INT_MAX) return MVN_ERR_SHAPE;
  X4Args a{feat, P, coords, cub, conf, out, transfer, B, C, H, W, Vx, Vy, Vz, align_corners,
           knob > 0 ? knob : 1 << 30, int(nt)};
  // persistent grid: as many blocks as are resident at once (a multiple of 8: one XCD each
  // by round-robin placement), each walking every gridDim-th tile
  auto go = [&](auto kern, int per_cu) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    long long grid = (long long)per_cu * cus;
    grid = grid >= 8 ? grid / 8 * 8 : grid;
#if X4_GRID_MODE == 1
    grid = nt;
#elif X4_GRID_MODE == 2
    grid = (sizeof(TIn) == 2 ? 4 : 2) * 256;
#endif
    // frames per launch: at most S::SLOW tiles per block (the block's deferred-tile list)
    const long long per_frame = nt / B;
    const long long fpl = std::max(1LL, grid * S::SLOW / per_frame);
    for (long long f0 = 0; f0 < B; f0 += fpl) {
      const int nb = int(std::min<long long>(fpl, B - f0));
      X4Args c = a;
      c.feat = static_cast<const char*>(a.feat) + size_t(f0) * 4 * C * H * W * sizeof(TIn);
      c.P = a.P + f0 * 4 * 12;
      c.coords = a.coords ? a.coords + size_t(f0) * Vx * Vy * Vz * 3 : nullptr;
      c.cub = a.cub ? a.cub + f0 * MVN_CUBOID_FLOATS : nullptr;
      c.conf = a.conf ? a.conf + f0 * 4 * C : nullptr;
      c.out = static_cast<char*>(a.out) + size_t(f0) * C * Vx * Vy * Vz * sizeof(TOut);
      c.B = nb;
      c.ntiles = int(per_frame * nb);
      kern<<<int(std::min<long long>(grid, c.ntiles)), S::THREADS, 0, s>>>(c);
    }
  };
  if (out_cl) go(unproject_x4<AGG, TIn, TOut, K, true>, resident_blocks_per_cu<unproject_x4<AGG, TIn, TOut, K, true>>(S::THREADS));
  else go(unproject_x4<AGG, TIn, TOut, K, false>, resident_blocks_per_cu<unproject_x4<AGG, TIn, TOut, K, false>>(S::THREADS));
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

// Diagnostics: resident blocks per CU of the softmax NCDHW kernels (f32 maps, bf16 maps) as
// the launcher sizes the persistent grid with them.
int x4_blocks_per_cu(int bf16) {
  return bf16 ? resident_blocks_per_cu<unproject_x4<MVN_AGG_SOFTMAX, uint16_t, uint16_t, 1, false>>(X4Shape<1>::THREADS)
              : resident_blocks_per_cu<unproject_x4<MVN_AGG_SOFTMAX, float, float, 0, false>>(X4Shape<0>::THREADS);
}

#define MVN_INSTANTIATE(AGG)                                                                                   \
  template int launch_x4<AGG, float, float>(const void*, const float*, const float*, const float*, int,        \
                                            const float*, void*, int, int, int, int, int, int, int, int, int,  \
                                            int, hipStream_t);                                                 \
  template int launch_x4<AGG, uint16_t, uint16_t>(const void*, const float*, const float*, const float*, int,  \
                                                  const float*, void*, int, int, int, int, int, int, int, int, \
                                                  int, int, hipStream_t);                                      \
  template int launch_x4<AGG, uint16_t, float>(const void*, const float*, const float*, const float*, int,     \
                                               const float*, void*, int, int, int, int, int, int, int, int,    \
                                               int, int, hipStream_t);
MVN_INSTANTIATE(MVN_AGG_SUM)
MVN_INSTANTIATE(MVN_AGG_MAX)
MVN_INSTANTIATE(MVN_AGG_SOFTMAX)
MVN_INSTANTIATE(MVN_AGG_CONF)
#undef MVN_INSTANTIATE

}  // namespace unproj
}  // namespace mvn
