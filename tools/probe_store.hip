// Microbenchmark: HBM write efficiency of the unprojection's output store patterns.
// Output (B=8, C=32, 64^3) f32 = 268 MB, written by 256-thread blocks as
//   run8 : each wave writes 8 runs of 8 consecutive floats (32 B) per channel  (4x8x8 tiles)
//   run16: 4 runs of 16 floats (64 B)                                          (TZ = 16)
//   run32: 2 runs of 32 floats (128 B)                                         (TZ = 32)
//   run64: 1 run of 64 floats (256 B)                                          (lane = z)
// plus a float4 copy of the same size as the achievable-bandwidth reference.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_store.hip -o /tmp/probe_store
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int V = 64, C = 32, B = 8;

template <int TZ>
__global__ __launch_bounds__(256) void store_runs(float* out, float val) {
  // tile: (256 / TZ / 8) x 8 x TZ voxels; lanes z-fastest, then y, then x
  constexpr int TY = (256 / TZ) < 8 ? (256 / TZ) : 8, TX = 256 / (TZ * TY);
  const int nTz = V / TZ, nTy = V / TY, nTx = V / TX;
  int L = blockIdx.x;
  const int tz = L % nTz; L /= nTz;
  const int ty = L % nTy; L /= nTy;
  const int tx = L % nTx;
  const int b = L / nTx;
  const int t = threadIdx.x;
  const int z = tz * TZ + t % TZ, y = ty * TY + (t / TZ) % TY, x = tx * TX + t / (TZ * TY);
  float* o = out + size_t(b) * C * V * V * V + (size_t(x) * V + y) * V + z;
  for (int c = 0; c < C; ++c) o[size_t(c) * V * V * V] = val + c;
}

__global__ void copy4(const float4* __restrict__ in, float4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    out[i] = in[i];
}

template <typename F>
float time_ms(F f, int iters = 20) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main() {
  const size_t n = size_t(B) * C * V * V * V;
  const double bytes = double(n) * 4;
  float *out, *in;
  hipMalloc(&out, n * 4);
  hipMalloc(&in, n * 4);
  hipMemset(in, 0, n * 4);
  const int nblk = B * V * V * V / 256;
  auto report = [&](const char* name, float ms, double b) {
    printf("%-8s %8.1f us  %7.0f GB/s\n", name, ms * 1e3, b / (ms * 1e-3) / 1e9);
  };
  for (int round = 0; round < 2; ++round) {
    report("run8", time_ms([&] { store_runs<8><<<nblk, 256>>>(out, 1.f); }), bytes);
    report("run16", time_ms([&] { store_runs<16><<<nblk, 256>>>(out, 1.f); }), bytes);
    report("run32", time_ms([&] { store_runs<32><<<nblk, 256>>>(out, 1.f); }), bytes);
    report("run64", time_ms([&] { store_runs<64><<<nblk, 256>>>(out, 1.f); }), bytes);
    report("copy4", time_ms([&] { copy4<<<4096, 256>>>((const float4*)in, (float4*)out, n / 4); }), 2 * bytes);
  }
  hipFree(out);
  hipFree(in);
  return 0;
}
