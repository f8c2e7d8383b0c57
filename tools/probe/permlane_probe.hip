// Which lane's value does each output of v_permlane16_swap / v_permlane32_swap carry (gfx950)?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
  const unsigned x = threadIdx.x, y = 100 + threadIdx.x;
  auto r16 = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  auto r32 = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  out[threadIdx.x * 4 + 0] = r16[0]; out[threadIdx.x * 4 + 1] = r16[1];
  out[threadIdx.x * 4 + 2] = r32[0]; out[threadIdx.x * 4 + 3] = r32[1];
}
int main() {
  int* d; hipMalloc(&d, 64 * 16); k<<<1, 64>>>(d); int h[256]; hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l++) printf("lane %2d: p16 (%3d, %3d)  p32 (%3d, %3d)\n", l, h[l*4], h[l*4+1], h[l*4+2], h[l*4+3]);
  return 0;
}
