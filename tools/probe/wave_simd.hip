// Which SIMD does each wave of a 512-thread workgroup run on?  (HW_ID: wave_id [3:0],
// simd_id [5:4], cu_id [11:8], sh_id [12], se_id [15:13] on gfx9-family parts.)
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void probe(unsigned* out) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + threadIdx.x / 64] = hw;
}

int main() {
  unsigned* d;
  const int nb = 64;
  hipMalloc(&d, nb * 8 * sizeof(unsigned));
  hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 0, 0, d);
  unsigned h[nb * 8];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int b = 0; b < 4; ++b) {
    printf("block %d:", b);
    for (int w = 0; w < 8; ++w) {
      const unsigned v = h[b * 8 + w];
      printf("  w%d simd %u slot %u cu %u", w, (v >> 4) & 3, v & 15, (v >> 8) & 15);
    }
    printf("\n");
  }
  int same = 0, tot = 0;
  for (int b = 0; b < nb; ++b)
    for (int w = 0; w < 4; ++w) {
      tot++;
      same += ((h[b * 8 + w] >> 4) & 3) == ((h[b * 8 + w + 4] >> 4) & 3);
    }
  printf("waves w and w+4 share a SIMD in %d / %d pairs\n", same, tot);
  return 0;
}
