// scratch check: raw buffer store / load with a large num_records and out-of-range lanes
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int i2 __attribute__((ext_vector_type(2)));
__global__ void k(int* out, const int* in, int n) {
  const int i = threadIdx.x;
  __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)(out + 2), 0, 0x7FFFFFF0, 0x00020000);
  __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)in, 0, 0x7FFFFFF0, 0x00020000);
  const bool ok = i < n;
  i2 v = __builtin_amdgcn_raw_buffer_load_b64(ri, ok ? i * 8 : 0x7FFFFFF8, 0, 0);
  v += i2{1000, 2000};
  __builtin_amdgcn_raw_buffer_store_b64(v, ro, ok ? i * 8 : 0x7FFFFFF8, 0, 0);
}
int main() {
  int *o, *in;
  hipMalloc(&o, 4096); hipMalloc(&in, 4096);
  std::vector<int> h(1024);
  for (int i = 0; i < 1024; ++i) h[i] = i;
  hipMemcpy(in, h.data(), 4096, hipMemcpyHostToDevice);
  hipMemset(o, 0xff, 4096);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, in, 40);
  hipMemcpy(h.data(), o, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 64; ++i) {
    int e0 = i < 40 ? 2 * i + 1000 : -1, e1 = i < 40 ? 2 * i + 1 + 2000 : -1;
    if (h[2 + 2 * i] != e0 || h[3 + 2 * i] != e1) { if (bad < 5) printf("lane %d got %d %d want %d %d\n", i, h[2+2*i], h[3+2*i], e0, e1); ++bad; }
  }
  printf("bufstore: %d bad, h[0..1]=%d %d\n", bad, h[0], h[1]);
  return 0;
}
