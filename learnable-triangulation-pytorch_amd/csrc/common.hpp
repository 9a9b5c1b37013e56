// Shared device helpers for libmvn_hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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

inline bool launch_ok() { return hipGetLastError() == hipSuccess; }

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
