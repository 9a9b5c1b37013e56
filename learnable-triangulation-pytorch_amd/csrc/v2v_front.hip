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
// weights (prepacked [tap][cout][cin], straight from L2 into registers, one 7-tap row ahead),
// C = 16 voxels x 16 output channels in f32.  A block walks a column of 4 x 4 x 16 output
// tiles along x: the 10 x 10 x 22-voxel input halo (140,800 B of LDS, zero-padded at the
// volume border like Conv3d's padding=3) is a ring of x-slices, 4 new slices per tile; each
// of the 4 waves takes one x-row of the tile (4 M-blocks = 4 accumulators) and walks the
// 343 taps.  Per tap and wave: 1 global 16-B
// weight load and 4 x (ds_read_b128 + v_mfma_f32_16x16x32_bf16).
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
constexpr int kThreads = 256;
constexpr uint32_t kOob = 0x80000000u;

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

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
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void v2v_front(const uint16_t* __restrict__ in, const uint4* __restrict__ wpk,
                                                     const float* __restrict__ scale, const float* __restrict__ shift,
                                                     TO* __restrict__ out, int V) {
  __shared__ uint4 halo[HVOX * 4];          // ring of HX x-slices: [slot][hy][hz][8-channel chunk]
  const int t = threadIdx.x, lane = t & (kWave - 1), w = t / kWave;
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

  // load x-slices gx0 .. gx0 + n - 1 (zero outside the volume) into their ring slots;
  // batches of 14 loads per thread in flight before the LDS writes
  auto load_slices = [&](int gx0, int n) {
    const int total = n * kSliceChunks;
    constexpr int kBatch = 14;
    for (int i0 = 0; i0 * kThreads < total; i0 += kBatch) {
      uint4 vals[kBatch];
      int dst[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; ++u) {
        const int q = t + (i0 + u) * kThreads;
        dst[u] = -1;
        if (q < total) {
          const int sl = q / kSliceChunks, rem = q - sl * kSliceChunks;
          const int v = rem >> 2, c = rem & 3;
          const int hz = v % HZ, hy = v / HZ;
          const int gx = gx0 + sl, gy = y0 + hy - PAD, gz = z0 + hz - PAD;
          const bool ok = (unsigned(gx) < unsigned(V)) & (unsigned(gy) < unsigned(V)) & (unsigned(gz) < unsigned(V));
          const uint32_t off = ok ? uint32_t(((size_t(gx) * V + gy) * V + gz) * CI * 2 + c * 16) : kOob;
          vals[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(irs, off, 0, 0));
          const int slot = (gx + PAD) % HX;
          dst[u] = slot * kSliceChunks + v * 4 + (c ^ swz(hz));
        }
      }
#pragma unroll
      for (int u = 0; u < kBatch; ++u)
        if (dst[u] >= 0) halo[dst[u]] = vals[u];
    }
  };

  const int r = lane & 15, kb = lane >> 4;
  const uint4* wl = wpk + lane;              // [tap][64 lanes]: lane's 16 B of the tap's B fragment
  uint32_t zoff[KS];                         // byte offset of (hz = r + dz, chunk kb) within a halo row
#pragma unroll
  for (int dz = 0; dz < KS; ++dz) zoff[dz] = uint32_t(((r + dz) * 4 + (kb ^ swz(r + dz))) * 16);
  const int co = lane & 15, zr = (lane >> 4) * 4;
  const float s = scale[co], sh = shift[co];

  load_slices(-PAD, HX);
  for (int tx = 0; tx < nTx; ++tx) {
    __syncthreads();                          // the tile's slices are in LDS
    const int x0 = tx * TX;
    f32x4_t acc[TY];
#pragma unroll
    for (int m = 0; m < TY; ++m) acc[m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // Register reuse of the A operand: tap (dx, dy, dz) of output row m reads halo y-row
    // hy = dy + m, so for a fixed dx the 4 accumulators share 10 halo rows.  The rows live in
    // a 5-slot register ring (slot hy % 5; 10 rows per dx keep the mapping across dx) and
    // each is read from LDS once per dx: 70 ds_read_b128 per dx instead of 196, which takes
    // the LDS array (4 cycles per read per wave, 4 waves per CU) off the critical path of
    // the 16-cycle MFMA.  Step dy runs taps (dx, dy, *) on rows dy..dy+3 (one accumulation
    // chain per row, full rate on 16x16x32); a row is loaded 28 MFMAs before it is first
    // used — at the start of step dy - 4, or, across a dx boundary, as soon as the last step
    // of the previous dx frees its slot.  B (7 fragments per tap row, from L2) is a 2-slot
    // ring one step ahead; its parity flips every dx (7 steps), hence the P template.
    uint4 A[5][KS], Bw[2][KS];
    const char* hbase = reinterpret_cast<const char*>(halo);
    auto lds_row = [&](int dx, int hy, uint4 (&dst)[KS]) {
      const int slot = (x0 + w + dx) % HX;                  // halo x = w + dx  <->  gx = x0 - PAD + w + dx
      const char* hb = hbase + uint32_t((slot * HY + hy) * HZ * 64);
#pragma unroll
      for (int dz = 0; dz < KS; ++dz) dst[dz] = *reinterpret_cast<const uint4*>(hb + zoff[dz]);
    };
    auto ld_b = [&](int dx, int dy, uint4 (&dst)[KS]) {
#pragma unroll
      for (int dz = 0; dz < KS; ++dz) dst[dz] = wl[((dx * KS + dy) * KS + dz) * kWave];
    };
    auto dx_body = [&](int dx, auto parity) {
      constexpr int P = decltype(parity)::value;
      const bool more = dx + 1 < KS;
#pragma unroll
      for (int dy = 0; dy < KS; ++dy) {
        __builtin_amdgcn_sched_barrier(0);
        if (dy + 1 < KS) {
          lds_row(dx, dy + 4, A[(dy + 4) % 5]);
          ld_b(dx, dy + 1, Bw[(dy + 1 + P) & 1]);
        } else if (more) {
          lds_row(dx + 1, 0, A[0]);
          ld_b(dx + 1, 0, Bw[(KS + P) & 1]);
        }
#pragma unroll
        for (int m = 0; m < TY; ++m) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int dz = 0; dz < KS; ++dz)
            acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, A[(dy + m) % 5][dz]),
                                                             __builtin_bit_cast(bf16x8_t, Bw[(dy + P) & 1][dz]),
                                                             acc[m], 0, 0, 0);
          if (dy + 1 == KS && more && m + 1 < TY) {         // rows 1..3 of dx + 1 into the freed slots
            __builtin_amdgcn_sched_barrier(0);
            lds_row(dx + 1, m + 1, A[m + 1]);
          }
        }
      }
    };
#pragma unroll
    for (int hy = 0; hy < TY; ++hy) lds_row(0, hy, A[hy]);
    ld_b(0, 0, Bw[0]);
    for (int dx = 0; dx < KS; dx += 2) {
      dx_body(dx, std::integral_constant<int, 0>{});
      if (dx + 1 < KS) dx_body(dx + 1, std::integral_constant<int, 1>{});
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();                          // every wave is done with slices x0-3 .. x0
    if (tx + 1 < nTx) load_slices(x0 + TX + HX - TX - PAD, TX);   // gx = x0+7 .. x0+10

    // ---- epilogue: folded BN + ReLU, 4 consecutive z of one output channel per lane ----
#pragma unroll
    for (int m = 0; m < TY; ++m) {
      float y[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) y[i] = fmaxf(__builtin_fmaf(acc[m][i], s, sh), 0.f);
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
  if (B <= 0 || V <= 0 || V % TZ != 0 || V % TX != 0 || V % TY != 0) return MVN_ERR_SHAPE;
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
