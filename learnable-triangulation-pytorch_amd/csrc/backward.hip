// Backward kernels for the autograd surface of the hot path (gfx950).
//
//   mvn_softargmax3d_backward  d/d(volumes) of op.py:84-96 (softmax or relu, multiplier fused)
//   mvn_dlt_backward           d/d(points, confidences) of multiview.py:132-174
//
// The reference gets these from ATen autograd (softmax / einsum / torch.svd backward); here
// they are closed forms evaluated in one or two streaming passes.
#include "common.hpp"

namespace mvn {
namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 2048;        // voxels per pass-1 wave
constexpr int kBwdPartial = 3;      // m, S = sum e, T = sum e * d

// ---------------------------------------------------------------- soft-argmax backward
//
// p = softmax(mult * x) (or relu(mult * x)), xyz = sum_i p_i c_i.  With upstream gradients
// gx (B,J,3) and gv (B,J,V):   d_i = gv_i + gx . c_i
//   softmax:  dL/dx_i = mult * p_i * (d_i - sum_k p_k d_k)
//   relu:     dL/dx_i = mult * [mult * x_i > 0] * d_i
// Pass 1 (softmax only) reduces, per (b, j, chunk), the local max m, S = sum e^(mx-m) and
// T = sum e^(mx-m) d with one wave per chunk; pass 2 folds them (r = T / S, M, S) and
// writes dL/dx elementwise.

template <typename T> __device__ __forceinline__ float ld(const T* p, long long i) { return to_f32(p[i]); }

__device__ __forceinline__ void merge3(float& m, float& s, float& t, float m2, float s2, float t2) {
  const float M = fmaxf(m, m2);
  const float ka = (m == -INFINITY) ? 0.f : __expf(m - M);
  const float kb = (m2 == -INFINITY) ? 0.f : __expf(m2 - M);
  s = s * ka + s2 * kb;
  t = t * ka + t2 * kb;
  m = M;
}

template <typename TV, typename TG>
__global__ __launch_bounds__(kThreads) void sa_bwd_partials(const TV* __restrict__ vol, long long bs, long long js,
                                                            const float* __restrict__ coords, float mult,
                                                            const float* __restrict__ gxyz, const TG* __restrict__ gvol,
                                                            float* __restrict__ part, int J, int nvox, int npart) {
  const int chunk = blockIdx.x, b = blockIdx.z;
  const int lane = threadIdx.x & (kWave - 1);
  const int j = blockIdx.y * (kThreads / kWave) + threadIdx.x / kWave;
  if (j >= J) return;                                   // no barriers in this kernel
  const TV* vj = vol + b * bs + j * js;
  const TG* gj = gvol ? gvol + (size_t(b) * J + j) * nvox : nullptr;
  const float* cb = coords + size_t(b) * nvox * 3;
  float g0 = 0.f, g1 = 0.f, g2 = 0.f;
  if (gxyz) { const float* g = gxyz + (size_t(b) * J + j) * 3; g0 = g[0]; g1 = g[1]; g2 = g[2]; }
  float m = -INFINITY, s = 0.f, t = 0.f;
  for (int i = chunk * kChunk + lane; i < min(nvox, (chunk + 1) * kChunk); i += kWave) {
    const float x = ld(vj, i) * mult;
    const float d = (gj ? ld(gj, i) : 0.f) + g0 * cb[size_t(i) * 3] + g1 * cb[size_t(i) * 3 + 1] + g2 * cb[size_t(i) * 3 + 2];
    if (x > m) {
      const float k = (m == -INFINITY) ? 0.f : __expf(m - x);
      s *= k; t *= k; m = x;
    }
    const float e = __expf(x - m);
    s += e;
    t = __builtin_fmaf(e, d, t);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, kWave), s2 = __shfl_xor(s, o, kWave), t2 = __shfl_xor(t, o, kWave);
    merge3(m, s, t, m2, s2, t2);
  }
  if (lane == 0) {
    float* o = part + ((size_t(b) * J + j) * npart + chunk) * kBwdPartial;
    o[0] = m; o[1] = s; o[2] = t;
  }
}

template <typename TV, typename TG, typename TO, bool SOFTMAX>
__global__ __launch_bounds__(kThreads) void sa_bwd_apply(const TV* __restrict__ vol, long long bs, long long js,
                                                         const float* __restrict__ coords, float mult,
                                                         const float* __restrict__ gxyz, const TG* __restrict__ gvol,
                                                         const float* __restrict__ part, TO* __restrict__ gin,
                                                         int J, int nvox, int npart) {
  const int j = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & (kWave - 1);
  float M = 0.f, S = 1.f, r = 0.f;
  if constexpr (SOFTMAX) {
    const float* pj = part + (size_t(b) * J + j) * npart * kBwdPartial;
    float m = -INFINITY, s = 0.f, t = 0.f;
    for (int k = lane; k < npart; k += kWave) merge3(m, s, t, pj[k * 3], pj[k * 3 + 1], pj[k * 3 + 2]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(m, o, kWave), s2 = __shfl_xor(s, o, kWave), t2 = __shfl_xor(t, o, kWave);
      merge3(m, s, t, m2, s2, t2);
    }
    M = m; S = s; r = t / s;
  }
  const TV* vj = vol + b * bs + j * js;
  const TG* gj = gvol ? gvol + (size_t(b) * J + j) * nvox : nullptr;
  const float* cb = coords + size_t(b) * nvox * 3;
  float g0 = 0.f, g1 = 0.f, g2 = 0.f;
  if (gxyz) { const float* g = gxyz + (size_t(b) * J + j) * 3; g0 = g[0]; g1 = g[1]; g2 = g[2]; }
  const float invS = 1.f / S;
  TO* oj = gin + (size_t(b) * J + j) * nvox;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < nvox; i += gridDim.x * kThreads) {
    const float x = ld(vj, i) * mult;
    const float d = (gj ? ld(gj, i) : 0.f) + g0 * cb[size_t(i) * 3] + g1 * cb[size_t(i) * 3 + 1] + g2 * cb[size_t(i) * 3 + 2];
    float g;
    if constexpr (SOFTMAX) {
      const float p = __expf(x - M) * invS;
      g = mult * p * (d - r);
    } else {
      g = x > 0.f ? mult * d : 0.f;
    }
    store_elem(oj + i, g);
  }
}

// ---------------------------------------------------------------- DLT backward
//
// M = A^T A (A the 2N x 4 design matrix of multiview.py:150-152), v4 its eigenvector of the
// smallest eigenvalue (= last right singular vector), X = v4, p = X[:3] / X[3].
//   gX = (gp / X3, -(gp . X[:3]) / X3^2)
//   dL/dM = G = sum_{k != 4} ((gX . v_k) / (l4 - l_k)) v_k v4^T        (eigenvector perturbation)
//   dL/dA = A (G + G^T)
//   a_{v,r} = c_v (pt_{v,r} P_v2 - P_vr)  ->  dL/dpt_{v,r} = c_v (dL/da_{v,r} . P_v2)
//                                             dL/dc_v = sum_r dL/da_{v,r} . (pt_{v,r} P_v2 - P_vr)
// The eigen-decomposition is recomputed exactly as in the forward (Givens QR + Jacobi, f64).

__device__ __forceinline__ void givens_fold_b(double (&R)[4][4], double (&a)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (a[k] == 0.0) continue;
    const double r = hypot(R[k][k], a[k]);
    const double c = R[k][k] / r, s = a[k] / r;
    R[k][k] = r;
    a[k] = 0.0;
#pragma unroll
    for (int l = k + 1; l < 4; ++l) {
      const double rk = R[k][l], al = a[l];
      R[k][l] = c * rk + s * al;
      a[l] = -s * rk + c * al;
    }
  }
}

__device__ __forceinline__ void jacobi_b(double (&U)[4][4], double (&V)[4][4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) V[i][k] = i == k ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 40; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        double alpha = 0.0, beta = 0.0, gamma = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          alpha += U[i][p] * U[i][p];
          beta += U[i][q] * U[i][q];
          gamma += U[i][p] * U[i][q];
        }
        if (gamma == 0.0 || fabs(gamma) <= 1e-15 * sqrt(alpha * beta)) continue;
        rotated = true;
        const double zeta = (beta - alpha) / (2.0 * gamma);
        const double t = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const double up = U[i][p], uq = U[i][q];
          U[i][p] = c * up - s * uq;
          U[i][q] = s * up + c * uq;
          const double vp = V[i][p], vq = V[i][q];
          V[i][p] = c * vp - s * vq;
          V[i][q] = s * vp + c * vq;
        }
      }
    if (!rotated) break;
  }
}

__device__ __forceinline__ void design_row(const float* Pv, float pt, float cf, int r, double (&a)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float e = Pv[8 + k] * pt;     // multiview.py:150
    e = e - Pv[r * 4 + k];        // :151
    e = e * cf;                   // :152
    a[k] = double(e);
  }
}

__global__ __launch_bounds__(64) void dlt_bwd_kernel(const float* __restrict__ P, const float* __restrict__ pts,
                                                     const float* __restrict__ conf, const float* __restrict__ gout,
                                                     float* __restrict__ gpts, float* __restrict__ gconf, int B, int N,
                                                     int J) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= B * J) return;
  const int b = t / J, j = t - b * J;

  double R[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) R[i][k] = 0.0;
  for (int v = 0; v < N; ++v) {
    const float* Pv = P + (size_t(b) * N + v) * 12;
    const size_t pj = (size_t(b) * N + v) * J + j;
    const float cf = conf ? conf[pj] : 1.f;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      double a[4];
      design_row(Pv, pts[pj * 2 + r], cf, r, a);
      givens_fold_b(R, a);
    }
  }
  double V[4][4];
  jacobi_b(R, V);
  double lam[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) lam[k] = R[0][k] * R[0][k] + R[1][k] * R[1][k] + R[2][k] * R[2][k] + R[3][k] * R[3][k];
  int kmin = 0;
#pragma unroll
  for (int k = 1; k < 4; ++k) if (lam[k] < lam[kmin]) kmin = k;
  double X[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    X[i] = V[i][0];
#pragma unroll
    for (int k = 1; k < 4; ++k) if (kmin == k) X[i] = V[i][k];
  }
  const float* go = gout + size_t(t) * 3;
  const double gp0 = go[0], gp1 = go[1], gp2 = go[2];
  const double gX[4] = {gp0 / X[3], gp1 / X[3], gp2 / X[3], -(gp0 * X[0] + gp1 * X[1] + gp2 * X[2]) / (X[3] * X[3])};
  // G = sum_{k != kmin} c_k v_k X^T
  double G[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int l = 0; l < 4; ++l) G[i][l] = 0.0;
  double lmin = lam[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) if (kmin == k) lmin = lam[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k == kmin) continue;
    const double dot = gX[0] * V[0][k] + gX[1] * V[1][k] + gX[2] * V[2][k] + gX[3] * V[3][k];
    const double ck = dot / (lmin - lam[k]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int l = 0; l < 4; ++l) G[i][l] += ck * V[i][k] * X[l];
  }
  double S[4][4];                                     // G + G^T
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int l = 0; l < 4; ++l) S[i][l] = G[i][l] + G[l][i];

  for (int v = 0; v < N; ++v) {
    const float* Pv = P + (size_t(b) * N + v) * 12;
    const size_t pj = (size_t(b) * N + v) * J + j;
    const float cf = conf ? conf[pj] : 1.f;
    double gc = 0.0;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const float pt = pts[pj * 2 + r];
      double a[4];
      design_row(Pv, pt, cf, r, a);
      double ga[4];                                   // dL/da = a (G + G^T)
#pragma unroll
      for (int l = 0; l < 4; ++l) ga[l] = a[0] * S[0][l] + a[1] * S[1][l] + a[2] * S[2][l] + a[3] * S[3][l];
      double gpt = 0.0;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        gpt += ga[l] * double(Pv[8 + l]);
        gc += ga[l] * (double(pt) * double(Pv[8 + l]) - double(Pv[r * 4 + l]));
      }
      gpts[pj * 2 + r] = float(double(cf) * gpt);
    }
    if (gconf) gconf[pj] = float(gc);
  }
}

template <typename TV, typename TG, typename TO>
int sa_bwd_launch(const void* vol, long long bs, long long js, const float* coords, float mult, int softmax,
                  const float* gxyz, const void* gvol, void* gin, float* part, int B, int J, int nvox, hipStream_t st) {
  const int npart = (nvox + kChunk - 1) / kChunk;
  if (softmax) {
    sa_bwd_partials<TV, TG><<<dim3(npart, (J + 3) / 4, B), kThreads, 0, st>>>(
        static_cast<const TV*>(vol), bs, js, coords, mult, gxyz, static_cast<const TG*>(gvol), part, J, nvox, npart);
    if (!launch_ok()) return MVN_ERR_LAUNCH;
  }
  const int gx = min((nvox + kThreads - 1) / kThreads, 64);
  if (softmax)
    sa_bwd_apply<TV, TG, TO, true><<<dim3(gx, J, B), kThreads, 0, st>>>(
        static_cast<const TV*>(vol), bs, js, coords, mult, gxyz, static_cast<const TG*>(gvol), part,
        static_cast<TO*>(gin), J, nvox, npart);
  else
    sa_bwd_apply<TV, TG, TO, false><<<dim3(gx, J, B), kThreads, 0, st>>>(
        static_cast<const TV*>(vol), bs, js, coords, mult, gxyz, static_cast<const TG*>(gvol), part,
        static_cast<TO*>(gin), J, nvox, npart);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

}  // namespace
}  // namespace mvn

extern "C" size_t mvn_softargmax3d_backward_workspace_bytes(int B, int J, int Vx, int Vy, int Vz) {
  if (B <= 0 || J <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0) return 0;
  const long long nvox = (long long)Vx * Vy * Vz;
  return size_t(B) * J * ((nvox + mvn::kChunk - 1) / mvn::kChunk) * mvn::kBwdPartial * sizeof(float);
}

extern "C" int mvn_softargmax3d_backward(const void* vol, int vol_dtype, int64_t vol_bstride, int64_t vol_jstride,
                                         const float* coords, float multiplier, int softmax, const float* grad_xyz,
                                         const void* grad_vol, int grad_vol_dtype, void* grad_in, int grad_in_dtype,
                                         void* workspace, size_t workspace_bytes, int B, int J, int Vx, int Vy,
                                         int Vz, void* stream) {
  using namespace mvn;
  if (!vol || !coords || !grad_in) return MVN_ERR_ARG;
  if (softmax != 0 && softmax != 1) return MVN_ERR_ARG;
  if (B <= 0 || J <= 0 || Vx <= 0 || Vy <= 0 || Vz <= 0 || B > 65535 || J > 65535) return MVN_ERR_SHAPE;
  const long long nvox = (long long)Vx * Vy * Vz;
  if (nvox > (1LL << 30) || vol_bstride < 0 || vol_jstride < 0) return MVN_ERR_SHAPE;
  if (softmax && (!workspace || workspace_bytes < mvn_softargmax3d_backward_workspace_bytes(B, J, Vx, Vy, Vz)))
    return MVN_ERR_WORKSPACE;
  if (grad_in_dtype != vol_dtype) return MVN_ERR_DTYPE;
  if (grad_vol && grad_vol_dtype != MVN_DTYPE_F32 && grad_vol_dtype != MVN_DTYPE_BF16) return MVN_ERR_DTYPE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(workspace);
  const int n = int(nvox);
  const bool gv16 = grad_vol && grad_vol_dtype == MVN_DTYPE_BF16;
  if (vol_dtype == MVN_DTYPE_F32)
    return gv16 ? sa_bwd_launch<float, uint16_t, float>(vol, vol_bstride, vol_jstride, coords, multiplier, softmax,
                                                        grad_xyz, grad_vol, grad_in, part, B, J, n, st)
                : sa_bwd_launch<float, float, float>(vol, vol_bstride, vol_jstride, coords, multiplier, softmax,
                                                     grad_xyz, grad_vol, grad_in, part, B, J, n, st);
  if (vol_dtype == MVN_DTYPE_BF16)
    return gv16 ? sa_bwd_launch<uint16_t, uint16_t, uint16_t>(vol, vol_bstride, vol_jstride, coords, multiplier,
                                                              softmax, grad_xyz, grad_vol, grad_in, part, B, J, n, st)
                : sa_bwd_launch<uint16_t, float, uint16_t>(vol, vol_bstride, vol_jstride, coords, multiplier,
                                                           softmax, grad_xyz, grad_vol, grad_in, part, B, J, n, st);
  return MVN_ERR_DTYPE;
}

extern "C" int mvn_dlt_backward(const float* proj, const float* pts, const float* conf, const float* grad_out,
                                float* grad_pts, float* grad_conf, int B, int N, int J, void* stream) {
  using namespace mvn;
  if (!proj || !pts || !grad_out || !grad_pts) return MVN_ERR_ARG;
  if (grad_conf && !conf) return MVN_ERR_ARG;
  if (B <= 0 || N <= 0 || J <= 0 || (long long)B * J > (1LL << 30)) return MVN_ERR_SHAPE;
  const int n = B * J;
  dlt_bwd_kernel<<<(n + 63) / 64, 64, 0, static_cast<hipStream_t>(stream)>>>(proj, pts, conf, grad_out, grad_pts,
                                                                              grad_conf, B, N, J);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}
