// Shared device helpers for libmvn_hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "mvn_hip.h"

namespace mvn {

constexpr int kWave = 64;

// ---- element access ------------------------------------------------------
// bf16 is carried as raw uint16_t bits; widening is exact (bits << 16).
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(uint16_t v) { return __uint_as_float(uint32_t(v) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN stays NaN): gfx950's v_cvt_pk_bf16_f32.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}
// Two values -> one dword (lo in bits 0-15): a single v_cvt_pk_bf16_f32.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

template <typename T> __device__ __forceinline__ void store_elem(T* p, float v);
template <> __device__ __forceinline__ void store_elem<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void store_elem<uint16_t>(uint16_t* p, float v) { *p = f32_to_bf16(v); }

// ---- wave reductions (64 lanes) -----------------------------------------
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// ---- cuboid coordinates (triangulation.py:280-341) ----------------------------------
// World coordinate of grid voxel (i, j, k) of a V^3 cuboid, from the frame's geometry
// p = position (base - side/2), cc = centre (base point), st = step, R = rotation (3x3,
// row-major), all f32 as the host rounds them (mvn_rocm/volumetric.py).  The reference's
// f32 op order on CPU (bit-exact against its goldens):
//   d_k = (p_k + st_k * g_k) - cc_k          (:313-315 mul then add; :333)
//   o_r = fma(R[r][2], d_2, fma(R[r][1], d_1, R[r][0] * d_0)) + cc_r   (rot.mm, MKL K=3; :335)
// CMU transfer (:338-341) as an index map: out[i][j][k] = grid[i][k][V-1-j].
// Every kernel that needs voxel coordinates either reads them from a coordinate volume
// built by this function (mvn_coord_volumes) or calls it in-kernel (the *_cuboid entry
// points), so both give the same bits.
__device__ __forceinline__ void cuboid_coord(const float* __restrict__ p, const float* __restrict__ cc,
                                             const float* __restrict__ st, const float* __restrict__ R, int V,
                                             int i, int j, int k, int transfer, float (&o)[3]) {
  int gx = i, gy = j, gz = k;
  if (transfer) { gy = k; gz = V - 1 - j; }
  const float d0 = (p[0] + st[0] * float(gx)) - cc[0];
  const float d1 = (p[1] + st[1] * float(gy)) - cc[1];
  const float d2 = (p[2] + st[2] * float(gz)) - cc[2];
#pragma unroll
  for (int r = 0; r < 3; ++r)
    o[r] = __builtin_fmaf(R[3 * r + 2], d2, __builtin_fmaf(R[3 * r + 1], d1, R[3 * r] * d0)) + cc[r];
}
// Packed per-frame cuboid descriptor of the *_cuboid entry points: MVN_CUBOID_FLOATS f32 =
// position[3], centre[3], step[3], rot[9].
__device__ __forceinline__ void cuboid_coord(const float* __restrict__ cub, int V, int i, int j, int k, int transfer,
                                             float (&o)[3]) {
  cuboid_coord(cub, cub + 3, cub + 6, cub + 9, V, i, j, k, transfer, o);
}

inline bool launch_ok() { return hipGetLastError() == hipSuccess; }

// ---- device-side assertions (debug build: make debug -> libmvn_hip_debug.so) ----------------
// SURVEY.md §5 'race detection / sanitizers'.  MVN_DASSERT(cond) checks an index or layout
// invariant inside a kernel.  A failure does not trap (a GPU fault takes the whole device down):
// it counts into a per-translation-unit device word and keeps the first failing line; the host
// reads and clears every unit's words through mvn_debug_device_asserts() (tests/conftest.py
// checks it after every GPU test when the debug library is loaded).  Release builds compile the
// checks away.
using DassertReader = int (*)(unsigned* count, unsigned* line);
std::vector<DassertReader>& dassert_registry();      // defined in unproject.hip
#ifdef MVN_DEVICE_ASSERTS
namespace {
__device__ unsigned g_dassert[2];                    // failures, first failing line (this unit)
int dassert_read_clear(unsigned* count, unsigned* line) {
  unsigned v[2] = {0u, 0u};
  if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_dassert), sizeof(v)) != hipSuccess) return -1;
  const unsigned zero[2] = {0u, 0u};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_dassert), zero, sizeof(zero)) != hipSuccess) return -1;
  *count = v[0];
  *line = v[1];
  return 0;
}
const bool g_dassert_registered = (dassert_registry().push_back(&dassert_read_clear), true);
}  // namespace
#define MVN_DASSERT(cond)                                                         \
  do {                                                                            \
    if (!(cond)) {                                                                \
      if (__hip_atomic_fetch_add(&::mvn::g_dassert[0], 1u, __ATOMIC_RELAXED,      \
                                 __HIP_MEMORY_SCOPE_AGENT) == 0u)                 \
        __hip_atomic_store(&::mvn::g_dassert[1], unsigned(__LINE__), __ATOMIC_RELAXED, \
                           __HIP_MEMORY_SCOPE_AGENT);                             \
    }                                                                             \
  } while (0)
#else
#define MVN_DASSERT(cond) \
  do {                    \
  } while (0)
#endif

// Test-only knobs of the unprojection dispatch (mvn_debug_set_unproject, unproject.hip):
// process-wide atomics set by tests to force the multi-pass / global-gather / simple
// kernel paths; nothing is read from the environment on the launch path.
int unproject_lds_slot_budget();   // 0 = the kernel's own budget
bool unproject_force_simple();
bool unproject_force_generic();    // skip the four-view kernel (unproject_x4.hip)

// XCD-aware block order (cdna_hip_programming.md §5.5 T1, bijective form): hardware deals
// blocks round-robin over the 8 XCDs, so block b runs on XCD b % 8.  Remapping gives each
// XCD one contiguous range of logical work items, which keeps a frame's feature maps in
// one XCD's L2 and lets neighbouring tiles' partial output lines merge there.  Speed only:
// any placement computes the same result.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  constexpr int kXcd = 8;
  const int q = nblk / kXcd, r = nblk % kXcd;
  const int xcd = bid % kXcd, k = bid / kXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

}  // namespace mvn
