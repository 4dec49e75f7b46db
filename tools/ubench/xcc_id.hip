// tools/ubench/xcc_id.hip -- which XCD (HW_REG_XCC_ID) each workgroup of a 2048-block grid runs on,
// and how often that equals blockIdx % 8 (the round-robin dispatch assumption).
#include <stdio.h>
#include <hip/hip_runtime.h>
__global__ void k(unsigned *o) {
  unsigned v = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
  if (threadIdx.x == 0) o[blockIdx.x] = v;
}
int main() {
  unsigned *d; (void)hipMalloc(&d, 4096 * 4);
  hipLaunchKernelGGL(k, dim3(2048), dim3(256), 0, 0, d);
  unsigned h[2048]; (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int cnt[16] = {0}; int match = 0;
  for (int i = 0; i < 2048; ++i) { cnt[h[i] & 15]++; match += (h[i] & 7) == (unsigned)(i % 8); }
  for (int i = 0; i < 16; ++i) printf("%d ", cnt[i]);
  printf("\nblockIdx%%8 == xcc: %d of 2048\n", match);
  return 0;
}
