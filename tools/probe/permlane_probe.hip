#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  unsigned l = threadIdx.x;
  unsigned a = 1000 + l, b = 2000 + l;
  auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
  out[l * 4 + 0] = r32[0]; out[l * 4 + 1] = r32[1];
  out[l * 4 + 2] = r16[0]; out[l * 4 + 3] = r16[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 64 * 16);
  k<<<1, 64>>>(d);
  unsigned h[256]; hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l += 1) printf("lane %2d: p32 {%u,%u} p16 {%u,%u}\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
  return 0;
}
