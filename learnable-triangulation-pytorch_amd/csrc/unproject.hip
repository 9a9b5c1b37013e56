// Fused volumetric unprojection for gfx950.
//
// Replaces mvn/utils/op.py:99-163 (unproject_heatmaps).  The reference runs a
// Python loop over batch x view (op.py:107,113) issuing ~10 ATen launches per
// (b, v): a K=4 sgemm projection (multiview.py:80-101), depth mask / divide
// (op.py:121-124), [-1,1] normalisation (op.py:127-130), F.grid_sample bilinear
// with zero padding (op.py:134), masking (op.py:138) and a view aggregation
// (op.py:147-161).  Here one kernel does all of it: each lane owns one voxel,
// computes the N view projections once, then walks the channels writing each
// channel plane of the output coalesced (64 consecutive voxels per wave).
//
// Numerics (parity mode, compiled with -ffp-contract=off):
//   projection  r = fma(1, P3, fma(z, P2, fma(y, P1, x*P0)))   (MKL K=4 sgemm order)
//   sampling    fma(v_se,se, fma(v_sw,sw, fma(v_ne,ne, v_nw*nw)))  (ATen CPU grid sampler, §8a a1.5)
// so 'sum' / 'max' / 'conf' are bit-exact with the torch CPU reference and
// 'softmax' differs only by exp() rounding (<= 1e-6 rel).
#include <stdlib.h>

#include <atomic>

#include "unproject_common.hpp"

namespace mvn {
namespace {

using namespace unproj;

constexpr int kUnprojBlock = 256;
constexpr int kMaxRegViews = 8;   // views whose geometry is held in registers

// ---- register-resident geometry, N <= 8 ----------------------------------
template <int AGG, typename TIn, typename TOut>
__global__ __launch_bounds__(kUnprojBlock) void unproject_regviews(
    const TIn* __restrict__ feat, const float* __restrict__ P, const float* __restrict__ coords,
    const float* __restrict__ conf, TOut* __restrict__ out, int N, int C, int H, int W, int nvox,
    int align_corners) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * kUnprojBlock + threadIdx.x;
  if (i >= nvox) return;
  const float* cp = coords + (size_t(b) * nvox + i) * 3;
  const float x = cp[0], y = cp[1], z = cp[2];

  Taps t[kMaxRegViews];
#pragma unroll
  for (int v = 0; v < kMaxRegViews; ++v)
    if (v < N) t[v] = view_taps(P + (size_t(b) * N + v) * 12, x, y, z, H, W, align_corners);

  const size_t HW = size_t(H) * W;
  const TIn* fb = feat + size_t(b) * N * C * HW;
  TOut* ob = out + size_t(b) * C * nvox + i;
  for (int c = 0; c < C; ++c) {
    float s[kMaxRegViews];
#pragma unroll
    for (int v = 0; v < kMaxRegViews; ++v)
      if (v < N) s[v] = sample(fb + (size_t(v) * C + c) * HW, t[v]);

    float r;
    if constexpr (AGG == MVN_AGG_SUM) {            // op.py:150, sequential over views
      r = s[0];
#pragma unroll
      for (int v = 1; v < kMaxRegViews; ++v) if (v < N) r = r + s[v];
    } else if constexpr (AGG == MVN_AGG_MAX) {     // op.py:152
      r = s[0];
#pragma unroll
      for (int v = 1; v < kMaxRegViews; ++v) if (v < N) r = max_takes(s[v], r) ? s[v] : r;
    } else if constexpr (AGG == MVN_AGG_CONF) {    // op.py:148: product rounded, then summed
      const float* cf = conf + size_t(b) * N * C + c;
      r = s[0] * cf[0];
#pragma unroll
      for (int v = 1; v < kMaxRegViews; ++v) if (v < N) r = r + s[v] * cf[size_t(v) * C];
    } else {                                       // op.py:153-159, softmax over views
      float m = s[0];
#pragma unroll
      for (int v = 1; v < kMaxRegViews; ++v) if (v < N) m = fmaxf(m, s[v]);
      const float ml = m * kLog2e;
      float den = 0.f, num = 0.f;
#pragma unroll
      for (int v = 0; v < kMaxRegViews; ++v)
        if (v < N) {
          const float e = softmax_exp(s[v], ml);
          den += e;
          num = __builtin_fmaf(s[v], e, num);
        }
      r = num * __builtin_amdgcn_rcpf(den);
    }
    store_elem(ob + size_t(c) * nvox, r);
  }
}

// ---- generic N (> 8): geometry recomputed per channel -------------------
template <int AGG, typename TIn, typename TOut>
__global__ __launch_bounds__(kUnprojBlock) void unproject_anyviews(
    const TIn* __restrict__ feat, const float* __restrict__ P, const float* __restrict__ coords,
    const float* __restrict__ conf, TOut* __restrict__ out, int N, int C, int H, int W, int nvox,
    int align_corners) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * kUnprojBlock + threadIdx.x;
  if (i >= nvox) return;
  const float* cp = coords + (size_t(b) * nvox + i) * 3;
  const float x = cp[0], y = cp[1], z = cp[2];
  const size_t HW = size_t(H) * W;
  const TIn* fb = feat + size_t(b) * N * C * HW;
  const float* Pb = P + size_t(b) * N * 12;
  TOut* ob = out + size_t(b) * C * nvox + i;
  for (int c = 0; c < C; ++c) {
    float r = 0.f, m = -INFINITY, den = 0.f, num = 0.f;
    for (int v = 0; v < N; ++v) {
      const Taps t = view_taps(Pb + v * 12, x, y, z, H, W, align_corners);
      const float s = sample(fb + (size_t(v) * C + c) * HW, t);
      if constexpr (AGG == MVN_AGG_SUM) {
        r = v == 0 ? s : r + s;
      } else if constexpr (AGG == MVN_AGG_MAX) {
        r = (v == 0 || max_takes(s, r)) ? s : r;
      } else if constexpr (AGG == MVN_AGG_CONF) {
        const float p = s * conf[(size_t(b) * N + v) * C + c];
        r = v == 0 ? p : r + p;
      } else {  // online softmax over views
        if (s > m) {
          const float k = __expf(m - s);
          den *= k;
          num *= k;
          m = s;
        }
        const float e = __expf(s - m);
        den += e;
        num = __builtin_fmaf(s, e, num);
      }
    }
    if constexpr (AGG == MVN_AGG_SOFTMAX) r = num / den;
    store_elem(ob + size_t(c) * nvox, r);
  }
}

// Kernel choice: the tiled LDS-staged kernel (unproject_tiled.hip) for N <= 8 views, the
// register-geometry kernel above when a test forces it (mvn_debug_set_unproject), and the
// any-N kernel for more than 8 views.
inline bool use_simple_kernel() { return unproject_force_simple(); }

template <int AGG, typename TIn, typename TOut>
int launch_agg(const void* feat, const float* P, const float* coords, const float* cub, int transfer,
               const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
               int align_corners, int out_cl, int fast, hipStream_t s) {
  const int nvox = Vx * Vy * Vz;
  if (N <= kMaxRegViews && !use_simple_kernel())
    return launch_tiled<AGG, TIn, TOut>(feat, P, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy, Vz,
                                        align_corners, out_cl, fast, s);
  if (cub) return MVN_ERR_SHAPE;     // in-kernel coordinates: the tiled kernel only (N <= 8)
  if (out_cl) return MVN_ERR_ARG;    // channels-last output: the tiled kernel only (N <= 8)
  dim3 grid((nvox + kUnprojBlock - 1) / kUnprojBlock, B);
  if (N <= kMaxRegViews)
    unproject_regviews<AGG, TIn, TOut><<<grid, kUnprojBlock, 0, s>>>(
        static_cast<const TIn*>(feat), P, coords, conf, static_cast<TOut*>(out), N, C, H, W, nvox,
        align_corners);
  else
    unproject_anyviews<AGG, TIn, TOut><<<grid, kUnprojBlock, 0, s>>>(
        static_cast<const TIn*>(feat), P, coords, conf, static_cast<TOut*>(out), N, C, H, W, nvox,
        align_corners);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

template <typename TIn, typename TOut>
int launch_types(int agg, const void* feat, const float* P, const float* coords, const float* cub, int transfer,
                 const float* conf, void* out, int B, int N, int C, int H, int W, int Vx, int Vy, int Vz,
                 int align_corners, int out_cl, int fast, hipStream_t s) {
  switch (agg) {
    case MVN_AGG_SUM:
      return launch_agg<MVN_AGG_SUM, TIn, TOut>(feat, P, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy, Vz, align_corners, out_cl, fast, s);
    case MVN_AGG_MAX:
      return launch_agg<MVN_AGG_MAX, TIn, TOut>(feat, P, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy, Vz, align_corners, out_cl, fast, s);
    case MVN_AGG_SOFTMAX:
      return launch_agg<MVN_AGG_SOFTMAX, TIn, TOut>(feat, P, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy, Vz, align_corners, out_cl, fast, s);
    case MVN_AGG_CONF:
      return launch_agg<MVN_AGG_CONF, TIn, TOut>(feat, P, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy, Vz, align_corners, out_cl, fast, s);
  }
  return MVN_ERR_ARG;
}

}  // namespace
}  // namespace mvn

namespace mvn {
namespace {
int unproject_entry(const void* feat, int feat_dtype, const float* proj, const float* coords, const float* cub,
                    int transfer, const float* conf, void* out, int out_dtype, int out_layout, int B, int N, int C,
                    int H, int W, int Vx, int Vy, int Vz, int agg, int align_corners, int precision,
                    void* stream) {
  if (!feat || !proj || !(coords || cub) || !out) return MVN_ERR_ARG;
  if (precision != MVN_PRECISION_EXACT && precision != MVN_PRECISION_FAST) return MVN_ERR_ARG;
  const int fast = precision == MVN_PRECISION_FAST;
  if (agg < MVN_AGG_SUM || agg > MVN_AGG_CONF) return MVN_ERR_ARG;
  if (agg == MVN_AGG_CONF && !conf) return MVN_ERR_ARG;
  if (align_corners != 0 && align_corners != 1) return MVN_ERR_ARG;
  if (transfer != 0 && transfer != 1) return MVN_ERR_ARG;
  if (out_layout != MVN_LAYOUT_NCDHW && out_layout != MVN_LAYOUT_NDHWC) return MVN_ERR_ARG;
  if (B <= 0 || N <= 0 || C <= 0 || H <= 0 || W <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0) return MVN_ERR_SHAPE;
  const long long nvox = (long long)Vx * Vy * Vz;
  if (nvox > (1LL << 30) || (long long)H * W > (1LL << 30) || B > 65535) return MVN_ERR_SHAPE;
  const int cl = out_layout == MVN_LAYOUT_NDHWC;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (feat_dtype == MVN_DTYPE_F32 && out_dtype == MVN_DTYPE_F32)
    return launch_types<float, float>(agg, feat, proj, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy, Vz,
                                      align_corners, cl, fast, s);
  if (feat_dtype == MVN_DTYPE_BF16 && out_dtype == MVN_DTYPE_BF16)
    return launch_types<uint16_t, uint16_t>(agg, feat, proj, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy,
                                            Vz, align_corners, cl, fast, s);
  if (feat_dtype == MVN_DTYPE_BF16 && out_dtype == MVN_DTYPE_F32)
    return launch_types<uint16_t, float>(agg, feat, proj, coords, cub, transfer, conf, out, B, N, C, H, W, Vx, Vy, Vz,
                                         align_corners, cl, fast, s);
  return MVN_ERR_DTYPE;
}
}  // namespace
}  // namespace mvn

namespace mvn {
namespace {
std::atomic<int> g_lds_slots{0}, g_force_simple{0};
}  // namespace
int unproject_lds_slot_budget() { return g_lds_slots.load(std::memory_order_relaxed); }
bool unproject_force_simple() { return g_force_simple.load(std::memory_order_relaxed) == 1; }
bool unproject_force_generic() { return g_force_simple.load(std::memory_order_relaxed) == 2; }
}  // namespace mvn

namespace mvn {
namespace unproj {
int x4_blocks_per_cu(int bf16);
}  // namespace unproj
}  // namespace mvn

extern "C" int mvn_debug_unproject_occupancy(int bf16_maps) {
  return mvn::unproj::x4_blocks_per_cu(bf16_maps ? 1 : 0);
}

namespace mvn {
std::vector<DassertReader>& dassert_registry() {
  static std::vector<DassertReader> r;
  return r;
}
}  // namespace mvn

namespace mvn {
namespace {
// one deliberately failing check per lane >= n (the mechanism's self-test)
__global__ void dassert_selftest(int n) { MVN_DASSERT(int(threadIdx.x) < n); }
}  // namespace
}  // namespace mvn

extern "C" int mvn_debug_dassert_selftest(int n, void* stream) {
  if (n < 0 || n > 64) return MVN_ERR_ARG;
  mvn::dassert_selftest<<<1, 64, 0, static_cast<hipStream_t>(stream)>>>(n);
  return mvn::launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

extern "C" int mvn_debug_device_asserts(int* enabled, unsigned* count, unsigned* first_line) {
  if (!enabled || !count || !first_line) return MVN_ERR_ARG;
#ifdef MVN_DEVICE_ASSERTS
  *enabled = 1;
#else
  *enabled = 0;
#endif
  *count = 0;
  *first_line = 0;
  for (auto rd : mvn::dassert_registry()) {
    unsigned c = 0, l = 0;
    if (rd(&c, &l) != 0) return MVN_ERR_LAUNCH;
    if (c && !*count) *first_line = l;
    *count += c;
  }
  return MVN_OK;
}

extern "C" int mvn_debug_set_unproject(int lds_slots, int kernel) {
  if (lds_slots < 0 || kernel < 0 || kernel > 2) return MVN_ERR_ARG;
  mvn::g_lds_slots.store(lds_slots, std::memory_order_relaxed);
  mvn::g_force_simple.store(kernel, std::memory_order_relaxed);
  return MVN_OK;
}

extern "C" int mvn_unproject_ex(const void* feat, int feat_dtype, const float* proj, const float* coords,
                                const float* conf, void* out, int out_dtype, int out_layout, int B, int N, int C,
                                int H, int W, int Vx, int Vy, int Vz, int agg, int align_corners, void* stream) {
  if (!coords) return MVN_ERR_ARG;
  return mvn::unproject_entry(feat, feat_dtype, proj, coords, nullptr, 0, conf, out, out_dtype, out_layout, B, N, C,
                              H, W, Vx, Vy, Vz, agg, align_corners, MVN_PRECISION_EXACT, stream);
}

extern "C" int mvn_unproject_cuboid(const void* feat, int feat_dtype, const float* proj, const float* cuboids,
                                    int transfer_cmu, const float* conf, void* out, int out_dtype, int out_layout,
                                    int B, int N, int C, int H, int W, int V, int agg, int align_corners,
                                    void* stream) {
  if (!cuboids) return MVN_ERR_ARG;
  if (N > mvn::kMaxRegViews) return MVN_ERR_SHAPE;
  return mvn::unproject_entry(feat, feat_dtype, proj, nullptr, cuboids, transfer_cmu, conf, out, out_dtype,
                              out_layout, B, N, C, H, W, V, V, V, agg, align_corners, MVN_PRECISION_EXACT, stream);
}

extern "C" int mvn_unproject_precision(const void* feat, int feat_dtype, const float* proj, const float* coords,
                                       const float* cuboids, int transfer_cmu, const float* conf, void* out,
                                       int out_dtype, int out_layout, int B, int N, int C, int H, int W, int Vx,
                                       int Vy, int Vz, int agg, int align_corners, int precision, void* stream) {
  if ((coords == nullptr) == (cuboids == nullptr)) return MVN_ERR_ARG;     // exactly one coordinate source
  if (cuboids && (N > mvn::kMaxRegViews || Vx != Vy || Vx != Vz)) return MVN_ERR_SHAPE;
  return mvn::unproject_entry(feat, feat_dtype, proj, coords, cuboids, cuboids ? transfer_cmu : 0, conf, out,
                              out_dtype, out_layout, B, N, C, H, W, Vx, Vy, Vz, agg, align_corners, precision, stream);
}

extern "C" int mvn_unproject(const void* feat, int feat_dtype, const float* proj, const float* coords,
                             const float* conf, void* out, int out_dtype, int B, int N, int C, int H,
                             int W, int Vx, int Vy, int Vz, int agg, int align_corners, void* stream) {
  return mvn_unproject_ex(feat, feat_dtype, proj, coords, conf, out, out_dtype, MVN_LAYOUT_NCDHW, B, N, C, H, W,
                          Vx, Vy, Vz, agg, align_corners, stream);
}
