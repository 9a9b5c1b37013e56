// Batched confidence-weighted algebraic (DLT) triangulation for gfx950.
//
// Replaces mvn/utils/multiview.py:162-174 (triangulate_batch_of_points) and its
// per-point solver multiview.py:132-159.  The reference loops over B x J in Python
// and calls torch.svd on each 2N x 4 matrix (B*J LAPACK / rocSOLVER calls).
//
// Here one lane owns one (b, j):
//   1. rows of A are formed in f32 exactly as multiview.py:150-152 forms them
//      (A = P[2]*pt; A -= P[:2]; A *= conf — three separately rounded ops),
//   2. each row is folded into a 4x4 upper-triangular R by Givens rotations (f64,
//      Newton-refined hardware reciprocal square roots: round 3, config 1 latency),
//      so R^T R = A^T A without ever squaring the condition number and for any N,
//   3. the right singular vector of the smallest singular value is the homogeneous point
//      (multiview.py:154-156): inverse iteration on R^T R (2-3 steps), or, when that does
//      not converge (near-equal smallest singular values), a one-sided Jacobi SVD of R (f64),
//   4. X[:3] / X[3] (multiview.py:157; sign of the null vector cancels).
#include "common.hpp"

namespace mvn {
namespace {

constexpr int kDltBlock = 64;

// f64 reciprocal and reciprocal square root: the hardware estimates (v_rcp_f64 / v_rsq_f64,
// about half the mantissa) refined by two Newton steps (fma): within an ulp or two of the IEEE
// result, in ~5 dependent operations instead of the ~10-20 of IEEE '/', sqrt and hypot.  The
// solve is one lane's serial f64 chain, so its latency is the kernel's time (config 1).
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
  return __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
}
__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double h = 0.5 * y, g = x * y;
    y = __builtin_fma(y, __builtin_fma(-g, h, 0.5), y);   // y (1.5 - x y^2 / 2)
  }
  return y;
}

// Fold row a into the upper-triangular R: one Givens rotation per non-zero entry
// (r = |(R_kk, a_k)|, c = R_kk / r, s = a_k / r from one reciprocal square root).
__device__ __forceinline__ void givens_fold(double (&R)[4][4], double (&a)[4]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (a[k] == 0.0) continue;
    const double n2 = __builtin_fma(R[k][k], R[k][k], a[k] * a[k]);
    const double ri = rsqrt_nr(n2);
    const double c = R[k][k] * ri, s = a[k] * ri;
    R[k][k] = n2 * ri;
    a[k] = 0.0;
#pragma unroll
    for (int l = k + 1; l < 4; ++l) {
      const double rk = R[k][l], al = a[l];
      R[k][l] = c * rk + s * al;
      a[l] = -s * rk + c * al;
    }
  }
}

// One-sided Jacobi on the columns of U (= R on entry); V accumulates the rotations.
// Convergence test |gamma| <= 1e-15 sqrt(alpha beta) as gamma^2 <= 1e-30 alpha beta (no sqrt).
__device__ __forceinline__ void jacobi_svd(double (&U)[4][4], double (&V)[4][4]) {
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
        if (gamma == 0.0 || gamma * gamma <= 1e-30 * (alpha * beta)) continue;
        rotated = true;
        const double zeta = (beta - alpha) * rcp_nr(2.0 * gamma);
        const double z2 = __builtin_fma(zeta, zeta, 1.0);
        const double root = z2 * rsqrt_nr(z2);                       // sqrt(1 + zeta^2)
        // |zeta| > 1e150: zeta^2 overflows (inf * rsqrt(inf) = NaN); there t = 1 / (2 zeta) to
        // working precision, which is what the IEEE form tends to
        const double t = fabs(zeta) > 1e150 ? 0.5 * rcp_nr(zeta)
                                            : (zeta >= 0.0 ? 1.0 : -1.0) * rcp_nr(fabs(zeta) + root);
        const double c = rsqrt_nr(__builtin_fma(t, t, 1.0)), s = c * t;
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

// Null vector by inverse iteration on R^T R = A^T A (its eigenvector of the smallest eigenvalue,
// the right singular vector multiview.py:154-156 takes): two triangular solves per step, each
// vector rescaled by its largest entry and the result normalised.  The null component grows by
// (sigma_2 / sigma_min)^2 per step: at the bench and test geometries 4-6 steps reach a step
// change below 1e-10 (results within 2e-13 of the f64 LAPACK restatement, numpy model); still
// moving after 12 steps (near-equal smallest singular values) returns false and the caller
// runs the Jacobi SVD instead.  A zero
// pivot (an exact null vector) is replaced by 1e-30 of the largest one.
__device__ __forceinline__ bool inverse_iteration(const double (&R)[4][4], double (&x)[4]) {
  double dmax = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) dmax = fmax(dmax, fabs(R[k][k]));
  if (!(dmax > 0.0)) return false;
  double rinv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double d = R[k][k];
    rinv[k] = rcp_nr(fabs(d) > 1e-30 * dmax ? d : (d < 0.0 ? -1e-30 : 1e-30) * dmax);
  }
  auto rescale = [](double (&v)[4]) {
    const double m = fmax(fmax(fabs(v[0]), fabs(v[1])), fmax(fabs(v[2]), fabs(v[3])));
    const double r = rcp_nr(m);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] *= r;
  };
#pragma unroll
  for (int i = 0; i < 4; ++i) x[i] = 0.5;
  for (int it = 0; it < 12; ++it) {
    double z[4], y[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {                 // R^T z = x (forward substitution)
      double acc = x[k];
#pragma unroll
      for (int i = 0; i < k; ++i) acc = __builtin_fma(-R[i][k], z[i], acc);
      z[k] = acc * rinv[k];
    }
    rescale(z);
#pragma unroll
    for (int k = 3; k >= 0; --k) {                // R y = z (back substitution)
      double acc = z[k];
#pragma unroll
      for (int l = k + 1; l < 4; ++l) acc = __builtin_fma(-R[k][l], y[l], acc);
      y[k] = acc * rinv[k];
    }
    rescale(y);
    const double n = rsqrt_nr(y[0] * y[0] + y[1] * y[1] + y[2] * y[2] + y[3] * y[3]);
    const double sg = (y[0] * x[0] + y[1] * x[1] + y[2] * x[2] + y[3] * x[3]) < 0.0 ? -n : n;
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y[i] *= sg;
      d += (y[i] - x[i]) * (y[i] - x[i]);
      x[i] = y[i];
    }
    if (!(d == d)) return false;                  // NaN (non-finite input): the Jacobi path decides
    if (it > 0 && d < 1e-20) return true;
  }
  return false;
}

__global__ __launch_bounds__(kDltBlock) void dlt_kernel(const float* __restrict__ P, const float* __restrict__ pts,
                                                        const float* __restrict__ conf, float* __restrict__ out,
                                                        int B, int N, int J) {
  const int t = blockIdx.x * kDltBlock + threadIdx.x;
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
    const float pt[2] = {pts[pj * 2 + 0], pts[pj * 2 + 1]};
    const float cf = conf ? conf[pj] : 1.f;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      double a[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float e = Pv[8 + k] * pt[r];   // multiview.py:150
        e = e - Pv[r * 4 + k];         // multiview.py:151
        e = e * cf;                    // multiview.py:152
        a[k] = double(e);
      }
      givens_fold(R, a);
    }
  }

  // An exactly zero column k of A (all-zero confidences, a coordinate no camera sees) leaves
  // R's column k exactly zero (the rotations mix rows, never columns), and e_k is an exact null
  // vector; LAPACK's SVD returns it as V[:, 3], the last of the tied smallest singular values
  // when there are several (A = 0: V = I, so e_4 and the point (0, 0, 0)).  The reference's
  // X[:3] / X[3] then gives (0, 0, 0) for k = 3 and (nan, nan, +-inf) otherwise
  // (multiview.py:154-157); iterating on the singular R would return ratios of tiny numbers.
  int zcol = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    bool z = true;
#pragma unroll
    for (int i = 0; i <= k; ++i) z &= R[i][k] == 0.0;
    if (z) zcol = k;
  }
  double X[4];
  if (zcol >= 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) X[i] = i == zcol ? 1.0 : 0.0;
  } else if (!inverse_iteration(R, X)) {
    double V[4][4];
    jacobi_svd(R, V);
    int kmin = 0;
    double smin = 0.0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double n2 = R[0][k] * R[0][k] + R[1][k] * R[1][k] + R[2][k] * R[2][k] + R[3][k] * R[3][k];
      if (k == 0 || n2 <= smin) { smin = n2; kmin = k; }     // ties: the last, as LAPACK's order
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      X[i] = V[i][0];
#pragma unroll
      for (int k = 1; k < 4; ++k) if (kmin == k) X[i] = V[i][k];
    }
  }
  float* o = out + size_t(t) * 3;
  o[0] = float(X[0] / X[3]);
  o[1] = float(X[1] / X[3]);
  o[2] = float(X[2] / X[3]);
}

}  // namespace
}  // namespace mvn

extern "C" int mvn_dlt(const float* proj, const float* pts, const float* conf, float* out, int B, int N, int J,
                       void* stream) {
  using namespace mvn;
  if (!proj || !pts || !out) return MVN_ERR_ARG;
  if (B <= 0 || N <= 0 || J <= 0) return MVN_ERR_SHAPE;
  if ((long long)B * J > (1LL << 30)) return MVN_ERR_SHAPE;
  const int n = B * J;
  dlt_kernel<<<(n + kDltBlock - 1) / kDltBlock, kDltBlock, 0, static_cast<hipStream_t>(stream)>>>(proj, pts, conf, out, B, N, J);
  return launch_ok() ? MVN_OK : MVN_ERR_LAUNCH;
}

extern "C" int mvn_version(void) { return (0 << 16) | (1 << 8) | 0; }

extern "C" const char* mvn_strerror(int code) {
  switch (code) {
    case MVN_OK: return "ok";
    case MVN_ERR_ARG: return "invalid argument (null pointer, enum or flag)";
    case MVN_ERR_SHAPE: return "invalid shape (non-positive or too large extent)";
    case MVN_ERR_DTYPE: return "unsupported dtype combination";
    case MVN_ERR_LAUNCH: return "HIP kernel launch failed";
    case MVN_ERR_WORKSPACE: return "workspace missing or too small";
  }
  return "unknown error";
}
