// V2V front block on bf16 MFMA for gfx950 (BASELINE config 5).
//
// Replaces V2VModel.front_layers[0] = Basic3DBlock(32, 16, 7) of mvn/models/v2v.py:7-17
// (Conv3d 32 -> 16, kernel 7, stride 1, padding 3, then BatchNorm3d and ReLU) in eval
// mode: BN folded by the host into a per-channel scale and shift (conv bias included).
// Input: the unprojected volume channels-last (B, V, V, V, 32) bf16 — the unprojection
// writes that layout directly (mvn_unproject_ex, MVN_LAYOUT_NDHWC), so the two launches
// form the fused unproject + view-softmax + front-block pipeline of config 5.
//
// Implicit GEMM, one MFMA per (16 output voxels, tap): A = 16 z-consecutive voxels x 32
// input channels (the tap-shifted input, read from an LDS halo), B = the tap's 32 x 16
// weights (prepacked [tap][lane][8], straight from L2 into registers), C = 16 voxels x 16
// output channels in f32.  A block walks a column of 4 x 4 x 16 output tiles along x: the
// 10 x 10 x 22-voxel input halo (140,800 B of LDS, zero-padded at the volume border like
// Conv3d's padding=3) is a ring of x-slices, 4 new slices per tile.  4 waves, one per SIMD,
// each computing the whole 4 x 4 x 16 tile (16 accumulators, so every B fragment feeds 16
// MFMAs) over a quarter of the 49 (dx, dz) tap passes (12 each, and the 49th split by
// output x-row); the partial sums meet in the tile's dead halo slots.
// Arithmetic: 2 * 32 * 16 * 343 * V^3 flop per frame (92.1 GFLOP at V = 64): MFMA-bound.
#include <climits>
#include <type_traits>

#include "common.hpp"

namespace mvn {
namespace {

constexpr int CI = 32, CO = 16, KS = 7, PAD = 3, NTAP = KS * KS * KS;
constexpr int TX = 4, TY = 4, TZ = 16;
constexpr int HX = TX + KS - 1, HY = TY + KS - 1, HZ = TZ + KS - 1;   // 10, 10, 22
constexpr int HVOX = HX * HY * HZ;                                     // 2200 voxels, 64 B each
constexpr int kWaves = 4, kThreads = kWaves * kWave;
constexpr int kPass = KS * KS;                                         // (dx, dz) tap passes
constexpr int kStage = (TX * HY * HZ * 4 + kThreads - 1) / kThreads;   // halo chunks per thread per tile: 14
// __builtin_amdgcn_sched_group_barrier instruction classes
constexpr int kSgMfma = 0x008, kSgVmemRead = 0x020, kSgDsRead = 0x100;
constexpr uint32_t kOob = 0x80000000u;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(uint32_t(a >> 32));
  void* p = reinterpret_cast<void*>((uint64_t(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, int(__builtin_amdgcn_readfirstlane(bytes)), 0x00020000);
}

// LDS swizzle of a halo voxel's four 16-byte channel chunks: chunk c of a voxel at halo z
// index hz sits at position c ^ swz(hz).  The A-operand read of one MFMA has lanes
// r = 0..15 (16 z-consecutive voxels) x chunk kb = 0..3; unswizzled, the 64-byte voxel
// pitch maps voxels 4 apart to the same bank quad (2-way conflicts in every lane group of
// ds_read_b128); with this swizzle every group hits 16 distinct quads for any z offset
// (exhaustive check over the four gfx950 lane groups).
__device__ __forceinline__ int swz(int hz) { return ((hz >> 2) & 1) << 1; }

template <typename TO>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void v2v_front(
    const uint16_t* __restrict__ in, const uint4* __restrict__ wpk, const float* __restrict__ scale,
    const float* __restrict__ shift, TO* __restrict__ out, int V) {
  __shared__ uint4 halo[HVOX * 4];          // ring of HX x-slices: [slot][hy][hz][8-channel chunk]
  const int t = threadIdx.x, lane = t & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(t / kWave);
  const int nTz = V / TZ, nTy = V / TY, nTx = V / TX;
  // A block walks one column of tiles along x (nTx tiles): consecutive tiles' halos share
  // HX - TX = 6 of their 10 x-slices, so per tile only TX = 4 new slices are loaded into a
  // ring (slot = (gx + PAD) mod HX).  Blocks: (frame, ty, tz), XCD-contiguous.
  int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tz = L % nTz; L /= nTz;
  const int ty = L % nTy; L /= nTy;
  const int b = L;
  const int y0 = ty * TY, z0 = tz * TZ;
  const size_t nvox = size_t(V) * V * V;
  const __amdgpu_buffer_rsrc_t irs = make_rsrc(in + size_t(b) * nvox * CI, uint32_t(nvox * CI * 2));
  constexpr int kSliceChunks = HY * HZ * 4;                  // 880 chunks of 16 B per x-slice
  constexpr int kSlotBytes = kSliceChunks * 16;              // 14,080 B

  // halo chunk q of the slices gx0, gx0 + 1, ...: its global byte offset (kOob: zero,
  // outside the volume or past the last chunk) and its LDS index in the ring
  static_assert((kWaves - 1) * TY * kWave * 16 <= kSlotBytes, "partial-sum blocks must fit a halo slot");
  auto chunk_src = [&](int gx0, int q, int total) -> uint32_t {
    const int sl = q / kSliceChunks, rem = q - sl * kSliceChunks;
    const int v = rem >> 2, c = rem & 3;
    const int hz = v % HZ, hy = v / HZ;
    const int gx = gx0 + sl, gy = y0 + hy - PAD, gz = z0 + hz - PAD;
    const bool ok = (q < total) & (unsigned(gx) < unsigned(V)) & (unsigned(gy) < unsigned(V)) &
                    (unsigned(gz) < unsigned(V));
    return ok ? uint32_t(((size_t(gx) * V + gy) * V + gz) * CI * 2 + c * 16) : kOob;
  };
  auto chunk_dst = [&](int gx0, int q) -> int {
    const int sl = q / kSliceChunks, rem = q - sl * kSliceChunks;
    const int v = rem >> 2, c = rem & 3;
    const int hz = v % HZ;
    return ((gx0 + sl + PAD) % HX) * kSliceChunks + v * 4 + (c ^ swz(hz));
  };
  auto ld_chunk = [&](uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(irs, off, 0, 0));
  };
  {  // the first tile's 10 slices
    constexpr int kBatch = 7, total = HX * kSliceChunks;
    for (int i0 = 0; i0 * kThreads < total; i0 += kBatch) {
      uint4 vals[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u) vals[u] = ld_chunk(chunk_src(-PAD, t + (i0 + u) * kThreads, total));
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        const int q = t + (i0 + u) * kThreads;
        MVN_DASSERT(q >= total || (chunk_dst(-PAD, q) >= 0 && chunk_dst(-PAD, q) < HVOX * 4));
        if (q < total) halo[chunk_dst(-PAD, q)] = vals[u];
      }
    }
  }

  // Per-tile staging of chunk q = t + u * kThreads (u < kStage) of the 4 new slices: the
  // in-slice part is tile-invariant, so it is decoded once into a packed descriptor:
  // bit 0 valid (q in range), bits 1-2 slice, bits 3-12 LDS index within the slot,
  // bit 13 y/z inside the volume, bits 14-31 (gy * V + gz) * 4 + c (V <= 256).
  uint32_t sdesc[kStage];
#pragma unroll
  for (int u = 0; u < kStage; ++u) {
    const int q = t + u * kThreads;
    const int sl = q / kSliceChunks, rem = q - sl * kSliceChunks;
    const int v = rem >> 2, c = rem & 3;
    const int hz = v % HZ, hy = v / HZ;
    const int gy = y0 + hy - PAD, gz = z0 + hz - PAD;
    const bool yz = (unsigned(gy) < unsigned(V)) & (unsigned(gz) < unsigned(V));
    sdesc[u] = (q < TX * kSliceChunks ? 1u : 0u) | (uint32_t(sl & 3) << 1) | (uint32_t(v * 4 + (c ^ swz(hz))) << 3) |
               (yz ? (1u << 13) | (uint32_t((gy * V + gz) * 4 + c) << 14) : 0u);
  }
  auto stage_src = [&](int u, int gx0) -> uint32_t {
    const uint32_t d = sdesc[u];
    const int gx = gx0 + int((d >> 1) & 3u);
    const bool ok = ((d & ((1u << 13) | 1u)) == ((1u << 13) | 1u)) & (unsigned(gx) < unsigned(V));
    return ok ? uint32_t(gx) * uint32_t(V * V * CI * 2) + (d >> 14) * 16u : kOob;
  };

  const int r = lane & 15, kb = lane >> 4;
  // packed weights [tap][64 lanes][16 B]: lane offset in a VGPR, tap offset in an SGPR
  const __amdgpu_buffer_rsrc_t wrs = make_rsrc(wpk, uint32_t(NTAP * kWave * 16));
  const int lane16 = lane * 16;
  const int co = lane & 15, zr = (lane >> 4) * 4;
  const float s = scale[co], sh = shift[co];
  const char* hbase = reinterpret_cast<const char*>(halo);
  constexpr int kCommon = (kPass - 1) / kWaves;              // 12 whole passes per wave; pass 48 split by x-row
  const int p0 = w * kCommon;

  // B fragments: the 7 taps (dx, 0..6, dz) of a pass
  uint4 Bf[KS];
  auto ld_b = [&](int wq, int dy) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane16, wq + dy * KS * kWave * 16, 0));
  };
  auto b_off = [&](int q) {
    const int dx = q / KS, dz = q - dx * KS;
    return __builtin_amdgcn_readfirstlane((dx * KS * KS + dz) * kWave * 16);   // tap (dx, 0, dz), bytes
  };

  for (int tx = 0; tx < nTx; ++tx) {
    __syncthreads();                          // the tile's slices are in LDS
    const int x0 = tx * TX;
    const bool more = tx + 1 < nTx;
    const int gxn = x0 + TX + HX - TX - PAD;  // next tile's new slices: gx = x0+7 .. x0+10
    f32x4_t acc[TX][TY];
#pragma unroll
    for (int x = 0; x < TX; ++x)
#pragma unroll
      for (int m = 0; m < TY; ++m) acc[x][m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // Pass (dx, dz): for each output x-row x the 10 halo y-rows at halo x = x + dx, z offset
    // dz (40 ds_read_b128) and the 7 taps (dx, 0..6, dz) (7 buffer loads); output (x, m)
    // takes tap dy from halo row hy = dy + m: 112 MFMAs per pass, each A fragment used for
    // up to 4 of them, each B fragment for 16 (B from L2 is 1/16 of a load per MFMA).  Step
    // hy of a pass runs the MFMAs of halo row hy, after which A[.][hy] and B[hy - 3] are
    // dead: the next pass's fragments are loaded into them right there, one pass ahead of
    // use, with one register set.  The passes are unrolled into straight-line code: at a
    // loop back-edge the compiler drains every load (more LDS reads are in flight than
    // lgkmcnt counts) and shuffles accumulators.
    uint4 A[TX][HY];
    // local x-row x of this wave <-> output x-row (w + x) & 3: every wave's own row is its
    // local row 0, so the last pass and the final sum need no per-wave code copies (a switch
    // on w made the compiler shuffle the 64 accumulators between register assignments)
    auto a_addr = [&](int q, int x) {
      const int dx = q / KS, dz = q - dx * KS;
      int slot = (x0 + dx) % HX + ((w + x) & 3);            // halo x = dx + row  <->  gx = x0 - PAD + dx + row
      if (slot >= HX) slot -= HX;
      return hbase + uint32_t(slot * HY * HZ * 64 + ((r + dz) * 4 + (kb ^ swz(r + dz))) * 16);
    };
    auto ld_a = [&](const char* hb, int hy) { return *reinterpret_cast<const uint4*>(hb + hy * HZ * 64); };
    // run the pass held in A / Bf (all x-rows, or x-row XONLY into slot 0) and load pass qn
    // (all x-rows, or only x-row w into slot 0 when NEXT_ONE)
    // run the pass held in A / Bf (all x-rows, or x-row XONLY in slot 0) and load pass qn
    // (all x-rows, or only x-row w into slot 0 when NEXT_ONE; nothing when qn < 0)
    auto pass = [&](int qn, auto next_one, auto xonly) {
      constexpr bool NEXT_ONE = decltype(next_one)::value;
      constexpr int XONLY = decltype(xonly)::value;
      const int wq = b_off(qn < 0 ? 0 : qn);
      const char* hb[TX];
#pragma unroll
      for (int x = 0; x < TX; ++x) hb[x] = a_addr(qn < 0 ? 0 : qn, NEXT_ONE ? 0 : x);
#pragma unroll
      for (int hy = 0; hy < HY; ++hy) {
        __builtin_amdgcn_sched_barrier(0);
        const int m_lo = hy - (KS - 1) > 0 ? hy - (KS - 1) : 0, m_hi = hy < TY - 1 ? hy : TY - 1;
        const int nm = m_hi - m_lo + 1;                       // MFMAs per x-row in this step
        const bool la = qn >= 0, lb = qn >= 0 && hy >= TY - 1;
#pragma unroll
        for (int x = 0; x < TX; ++x) {
          if (XONLY >= 0 && x > 0) break;
#pragma unroll
          for (int m = m_lo; m <= m_hi; ++m) {
            const int xa = XONLY >= 0 ? XONLY : x;
            acc[xa][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, A[x][hy]),
                                                                 __builtin_bit_cast(bf16x8_t, Bf[hy - m]), acc[xa][m], 0, 0, 0);
          }
          if (la && (!NEXT_ONE || x == 0)) A[x][hy] = ld_a(hb[x], hy);
        }
        if (lb) Bf[hy - (TY - 1)] = ld_b(wq, hy - (TY - 1));
        // issue order: each x-row's MFMAs, then its A reload (one LDS read per MFMA group)
#pragma unroll
        for (int x = 0; x < TX; ++x) {
          if (XONLY >= 0 && x > 0) break;
#pragma unroll
          for (int i = 0; i < nm; ++i) __builtin_amdgcn_sched_group_barrier(kSgMfma, 1, 0);
          if (la && (!NEXT_ONE || x == 0)) __builtin_amdgcn_sched_group_barrier(kSgDsRead, 1, 0);
        }
        if (lb) __builtin_amdgcn_sched_group_barrier(kSgVmemRead, 1, 0);
      }
    };
    using F = std::false_type;
    using T = std::true_type;
    using ALLX = std::integral_constant<int, -1>;
    {  // first pass of this wave
      const int wq = b_off(p0);
#pragma unroll
      for (int i = 0; i < KS; ++i) Bf[i] = ld_b(wq, i);
#pragma unroll
      for (int x = 0; x < TX; ++x) {
        const char* hb = a_addr(p0, x);
#pragma unroll
        for (int i = 0; i < HY; ++i) A[x][i] = ld_a(hb, i);
      }
    }
    // the next tile's 4 new slices: loaded into registers during the passes (2 per pass),
    // written to LDS once every wave is done with the slots they replace
    uint4 sv[kStage];
#pragma unroll
    for (int i = 0; i < kCommon; ++i) {
      if (i + 1 < kCommon) pass(p0 + i + 1, F{}, ALLX{});
      else pass(kPass - 1, T{}, ALLX{});                   // then pass 48, own x-row only
      if (2 * i < kStage) {
#pragma unroll
        for (int u = 2 * i; u < 2 * i + 2 && u < kStage; ++u) sv[u] = ld_chunk(more ? stage_src(u, gxn) : kOob);
      }
    }
    pass(-1, T{}, std::integral_constant<int, 0>{});   // pass 48, own x-row (local row 0)
    __builtin_amdgcn_sched_barrier(0);

    // ---- partial sums: wave k owns output x-row k.  The 4 slots of slices x0-3 .. x0 are
    // dead now (they take the next tile's slices): each wave writes its partials of the 3
    // x-rows it does not own there — 4 KiB blocks [m][lane] f32x4, block (owner, source j)
    // at slot owner, offset j * 4 KiB (3 blocks fit a 13.75 KiB slot) — then sums its own.
    const int s0 = x0 % HX;
    auto red_addr = [&](int owner, int j, int m) {
      int slot = s0 + owner;
      if (slot >= HX) slot -= HX;
      return reinterpret_cast<f32x4_t*>(const_cast<char*>(hbase) + slot * kSlotBytes + j * (TY * kWave * 16) +
                                        (m * kWave + lane) * 16);
    };
    __syncthreads();                          // every wave is done with the halo
#pragma unroll
    for (int x = 1; x < TX; ++x) {
      const int k = (w + x) & 3, j = w < k ? w : w - 1;
#pragma unroll
      for (int m = 0; m < TY; ++m) *red_addr(k, j, m) = acc[x][m];
    }
    __syncthreads();
    f32x4_t sum[TY];
#pragma unroll
    for (int m = 0; m < TY; ++m) {
      sum[m] = acc[0][m];
#pragma unroll
      for (int j = 0; j < kWaves - 1; ++j) sum[m] += *red_addr(w, j, m);
    }
    __syncthreads();                          // the dead slots are read: the next slices go in
    if (more) {
#pragma unroll
      for (int u = 0; u < kStage; ++u) {
        const uint32_t d = sdesc[u];
        if (d & 1u) {
          int slot = ((gxn + PAD) % HX) + int((d >> 1) & 3u);
          if (slot >= HX) slot -= HX;
          MVN_DASSERT(slot * kSliceChunks + int((d >> 3) & 1023u) < HVOX * 4);
          halo[slot * kSliceChunks + int((d >> 3) & 1023u)] = sv[u];
        }
      }
    }

    // ---- epilogue: folded BN + ReLU, 4 consecutive z of one output channel per lane ----
#pragma unroll
    for (int m = 0; m < TY; ++m) {
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = fmaxf(__builtin_fmaf(sum[m][i], s, sh), 0.f);
      TO* o = out + (((size_t(b) * CO + co) * V + (x0 + w)) * V + (y0 + m)) * V + z0 + zr;
      if constexpr (sizeof(TO) == 4) {
        *reinterpret_cast<float4*>(o) = make_float4(y[0], y[1], y[2], y[3]);
      } else {
        *reinterpret_cast<uint2*>(o) = make_uint2(pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3]));
      }
    }
  }
}

}  // namespace
}  // namespace mvn

extern "C" size_t mvn_v2v_front_packed_weight_bytes(void) { return size_t(mvn::NTAP) * 64 * 16; }

extern "C" int mvn_v2v_front(const void* vol_cl, const void* weight_packed, const float* scale, const float* shift,
                             void* out, int out_dtype, int B, int V, void* stream) {
  using namespace mvn;
  if (!vol_cl || !weight_packed || !scale || !shift || !out) return MVN_ERR_ARG;
  if (B <= 0 || V <= 0 || V > 256 || V % TZ != 0 || V % TX != 0 || V % TY != 0) return MVN_ERR_SHAPE;
  if ((long long)V * V * V * CI * 2 >= (1LL << 31)) return MVN_ERR_SHAPE;
  const long long nblk = (long long)B * (V / TY) * (V / TZ);       // one block per tile column along x
  if (nblk > INT_MAX) return MVN_ERR_SHAPE;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const auto* in = static_cast<const uint16_t*>(vol_cl);
  const auto* w = static_cast<const uint4*>(weight_packed);
  if (out_dtype == MVN_DTYPE_F32)
    v2v_front<float><<<int(nblk), kThreads, 0, s>>>(in, w, scale, shift, static_cast<float*>(out), V);
  else if (out_dtype == MVN_DTYPE_BF16)
    v2v_front<uint16_t><<<int(nblk), kThreads, 0, s>>>(in, w, scale, shift, static_cast<uint16_t*>(out), V);
  else
    return MVN_ERR_DTYPE;
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}
