// Microbenchmark (design aid, not product code): issue cost per wave64 instruction on gfx950
// for the VALU / LDS instructions the unprojection mixes, at 1..8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/valu_rates.hip -o tools/bin/valu_rates && tools/bin/valu_rates
// Each thread runs ITER iterations of 8 independent chains of one instruction (inline asm,
// so the instruction is exactly the one named); per-wave cycles from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int ITER = 512;

#define CHAIN8(INS)                                                                     \
  asm volatile(INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)                   \
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), \
                 "+v"(a[6]), "+v"(a[7])                                                  \
               : "v"(b), "v"(c));

#define I_FMA(k) "v_fma_f32 %" #k ", %" #k ", %8, %9\n"
#define I_MUL(k) "v_mul_f32 %" #k ", %" #k ", %8\n"
#define I_EXP(k) "v_exp_f32 %" #k ", %" #k "\n"
#define I_RCP(k) "v_rcp_f32 %" #k ", %" #k "\n"
#define I_MAX3(k) "v_max3_f32 %" #k ", %" #k ", %8, %9\n"
#define I_MIX(k) "v_fma_mix_f32 %" #k ", %8, %" #k ", %9 op_sel:[1,0,0] op_sel_hi:[1,0,0]\n"
#define I_CVT(k) "v_cvt_f32_bf16_sdwa %" #k ", %8 src0_sel:WORD_1\n"
#define I_AND(k) "v_and_b32 %" #k ", %" #k ", %8\n"
#define I_PERM(k) "v_perm_b32 %" #k ", %" #k ", %8, %9\n"
#define I_DOT2(k) "v_dot2_f32_bf16 %" #k ", %8, %9, %" #k "\n"

template <int OP>
__global__ __launch_bounds__(256) void valu(float* out, unsigned long long* cyc, float b, float c) {
  float a[8];
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 1e-3f + k;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
    if constexpr (OP == 0) { CHAIN8(I_FMA) }
    if constexpr (OP == 1) { CHAIN8(I_MUL) }
    if constexpr (OP == 2) { CHAIN8(I_EXP) }
    if constexpr (OP == 3) { CHAIN8(I_RCP) }
    if constexpr (OP == 4) { CHAIN8(I_MAX3) }
    if constexpr (OP == 5) { CHAIN8(I_MIX) }
    if constexpr (OP == 6) { CHAIN8(I_CVT) }
    if constexpr (OP == 7) { CHAIN8(I_AND) }
    if constexpr (OP == 8) { CHAIN8(I_PERM) }
    if constexpr (OP == 9) { CHAIN8(I_DOT2) }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int k = 0; k < 8; ++k) s += a[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

// packed f32: 8 chains of 64-bit pairs
template <int OP>
__global__ __launch_bounds__(256) void valu_pk(float* out, unsigned long long* cyc, float b, float c) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a[8];
  const f2 bb = {b, c}, cc = {c, b};
  for (int k = 0; k < 8; ++k) a[k] = f2{threadIdx.x * 1e-3f + k, k * 0.5f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
#define P(k) (OP == 0 ? "v_pk_fma_f32 %" #k ", %" #k ", %8, %9\n" : OP == 1 ? "v_pk_mul_f32 %" #k ", %" #k ", %8\n" : "v_pk_add_f32 %" #k ", %" #k ", %8\n")
    if constexpr (OP == 0)
      asm volatile("v_pk_fma_f32 %0, %0, %8, %9\nv_pk_fma_f32 %1, %1, %8, %9\nv_pk_fma_f32 %2, %2, %8, %9\nv_pk_fma_f32 %3, %3, %8, %9\n"
                   "v_pk_fma_f32 %4, %4, %8, %9\nv_pk_fma_f32 %5, %5, %8, %9\nv_pk_fma_f32 %6, %6, %8, %9\nv_pk_fma_f32 %7, %7, %8, %9\n"
                   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
                   : "v"(bb), "v"(cc));
    else
      asm volatile("v_pk_mul_f32 %0, %0, %8\nv_pk_mul_f32 %1, %1, %8\nv_pk_mul_f32 %2, %2, %8\nv_pk_mul_f32 %3, %3, %8\n"
                   "v_pk_mul_f32 %4, %4, %8\nv_pk_mul_f32 %5, %5, %8\nv_pk_mul_f32 %6, %6, %8\nv_pk_mul_f32 %7, %7, %8\n"
                   : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
                   : "v"(bb), "v"(cc));
#undef P
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int k = 0; k < 8; ++k) s += a[k].x + a[k].y;
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

// LDS: ds_read_b128 / b64 with a lane -> address pattern: 0 = conflict-free (lane-linear),
// 1 = broadcast (one address per 16-lane group), 2 = 2-way per 16-lane group
template <int OP, int PAT>
__global__ __launch_bounds__(256) void lds(float* out, unsigned long long* cyc) {
  __shared__ uint4 buf[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) buf[i] = make_uint4(i, i + 1, i + 2, i + 3);
  __syncthreads();
  const int l = threadIdx.x & 63;
  unsigned addr = PAT == 0 ? l * 16 : PAT == 1 ? (l / 16) * 16 : (l % 8) * 16 + (l / 8) * 256;
  addr += (threadIdx.x / 64) * 4096;
  uint4 acc = make_uint4(0, 0, 0, 0);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
    uint4 r0, r1, r2, r3;
    if constexpr (OP == 0) {
      asm volatile("ds_read_b128 %0, %4\nds_read_b128 %1, %4 offset:1024\nds_read_b128 %2, %4 offset:2048\nds_read_b128 %3, %4 offset:3072\ns_waitcnt lgkmcnt(0)"
                   : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3) : "v"(addr));
      acc.x ^= r0.x ^ r1.y ^ r2.z ^ r3.w;
    } else {
      uint2 q0, q1, q2, q3;
      asm volatile("ds_read_b64 %0, %4\nds_read_b64 %1, %4 offset:1024\nds_read_b64 %2, %4 offset:2048\nds_read_b64 %3, %4 offset:3072\ns_waitcnt lgkmcnt(0)"
                   : "=v"(q0), "=v"(q1), "=v"(q2), "=v"(q3) : "v"(addr));
      acc.x ^= q0.x ^ q1.y ^ q2.x ^ q3.y;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = float(acc.x);
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <typename K>
double run(K kern, int wps, bool pk, int ninstr, float* out, unsigned long long* cyc, hipEvent_t e0, hipEvent_t e1, float* ms) {
  const int blocks = 256 * wps;   // 4 waves per block, one wave per SIMD: wps blocks per CU
  kern<<<blocks, 256>>>(out, cyc, 1.0001f, 0.5f);
  hipEventRecord(e0);
  kern<<<blocks, 256>>>(out, cyc, 1.0001f, 0.5f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(ms, e0, e1);
  std::vector<unsigned long long> h(blocks * 4);
  hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
  double s = 0;
  for (auto v : h) s += double(v);
  s /= h.size();
  // s_memtime ticks at a constant 100 MHz on gfx9?  report both: wall-derived cycles per instr per SIMD
  return s;
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 8 * 256 * 4);
  hipMalloc(&cyc, 256 * 8 * 4 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v_fma_f32", "v_mul_f32", "v_exp_f32", "v_rcp_f32", "v_max3_f32", "v_fma_mix_f32", "v_cvt_f32_bf16_sdwa", "v_and_b32", "v_perm_b32", "v_dot2_f32_bf16"};
  void* ks[] = {(void*)valu<0>, (void*)valu<1>, (void*)valu<2>, (void*)valu<3>, (void*)valu<4>, (void*)valu<5>, (void*)valu<6>, (void*)valu<7>, (void*)valu<8>, (void*)valu<9>};
  const double ninstr = 8.0 * ITER;
  // warm the clocks
  for (int r = 0; r < 20; ++r) valu<0><<<2048, 256>>>(out, cyc, 1.0001f, 0.5f);
  hipDeviceSynchronize();
  printf("instruction             waves/SIMD  ns/instr/SIMD  memtime/instr/wave\n");
  for (int wps : {1, 2, 4, 8}) {
    for (int k = 0; k < 10; ++k) {
      float ms;
      typedef void (*F)(float*, unsigned long long*, float, float);
      double mt = run((F)ks[k], wps, false, 0, out, cyc, e0, e1, &ms);
      // wall: ms covers wps waves per SIMD each issuing ninstr
      printf("%-22s %4d  %8.3f  %8.3f\n", names[k], wps, ms * 1e6 / (wps * ninstr), mt / ninstr);
    }
    for (int k = 0; k < 2; ++k) {
      float ms;
      typedef void (*F)(float*, unsigned long long*, float, float);
      F f = k == 0 ? (F)valu_pk<0> : (F)valu_pk<1>;
      double mt = run(f, wps, true, 0, out, cyc, e0, e1, &ms);
      printf("%-22s %4d  %8.3f  %8.3f\n", k == 0 ? "v_pk_fma_f32" : "v_pk_mul_f32", wps, ms * 1e6 / (wps * ninstr), mt / ninstr);
    }
    for (int k = 0; k < 6; ++k) {
      typedef void (*G)(float*, unsigned long long*);
      G g = k == 0 ? (G)lds<0, 0> : k == 1 ? (G)lds<0, 1> : k == 2 ? (G)lds<0, 2> : k == 3 ? (G)lds<1, 0> : k == 4 ? (G)lds<1, 1> : (G)lds<1, 2>;
      const int blocks = 256 * wps;
      g<<<blocks, 256>>>(out, cyc);
      hipEventRecord(e0);
      g<<<blocks, 256>>>(out, cyc);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const char* ln[] = {"ds_read_b128 linear", "ds_read_b128 bcast16", "ds_read_b128 2way", "ds_read_b64 linear", "ds_read_b64 bcast16", "ds_read_b64 2way"};
      // per CU: 4*wps waves each 4*ITER reads
      printf("%-22s %4d  ns/instr/CU %8.3f\n", ln[k], wps, ms * 1e6 / (4.0 * wps * 4 * ITER));
    }
  }
  return 0;
}
