// MFMA issue-rate probe (diagnostic, not product code): back-to-back independent
// v_mfma_f32_16x16x16_f16 / v_mfma_f32_16x16x32_f16 chains, one kernel per opcode, every CU
// busy; prints the cycles per MFMA per SIMD implied by the measured time at the clock read
// from s_memtime.  Build: hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_rate.hip -o tools/probe/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 4096;

template <int K>
__global__ __launch_bounds__(256) void probe(float* out, unsigned long long* cyc) {
  f4 acc[4] = {};
  const float s = (float)threadIdx.x;
  h8 a8 = {(_Float16)s, 1, 2, 3, 4, 5, 6, 7}, b8 = {1, 1, 1, 1, 1, 1, 1, 1};
  h4 a4 = {(_Float16)s, 1, 2, 3}, b4 = {1, 1, 1, 1};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (K == 32)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, acc[j], 0, 0, 0);
      else
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, acc[j], 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
}

int main() {
  float* out;
  unsigned long long* cyc;
  const int blocks = 256;  // one 4-wave block per CU: one wave per SIMD
  hipMalloc(&out, blocks * 256 * sizeof(float));
  hipMalloc(&cyc, sizeof(unsigned long long));
  for (int k : {16, 32}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (k == 32)
        hipLaunchKernelGGL(probe<32>, dim3(blocks), dim3(256), 0, 0, out, cyc);
      else
        hipLaunchKernelGGL(probe<16>, dim3(blocks), dim3(256), 0, 0, out, cyc);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c = 0;
      hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost);
      const double mfma = (double)kIters * 4;  // per wave (one wave per SIMD)
      printf("16x16x%d: %.3f ms, s_memtime %llu ticks, %.2f ticks per MFMA per SIMD, %.1f TFLOP/s\n", k, ms, c,
             c / mfma, 2.0 * 16 * 16 * k * mfma * blocks * 4 / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
