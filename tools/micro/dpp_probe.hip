// Which lane a DPP wave shift reads from on this GPU (calibration only).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(int* o) {
  int l = threadIdx.x;
  o[l] = __builtin_amdgcn_update_dpp(-1, l, 0x130, 0xf, 0xf, false);
  o[64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x138, 0xf, 0xf, false);
  o[128 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x134, 0xf, 0xf, false);
  o[192 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x13C, 0xf, 0xf, false);
}
int main() {
  int* d; int h[256];
  (void)hipMalloc(&d, 1024);
  k<<<1, 64>>>(d);
  (void)hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
  const char* nm[4] = {"wave_shl1 0x130", "wave_shr1 0x138", "wave_rol1 0x134", "wave_ror1 0x13C"};
  for (int r = 0; r < 4; ++r) {
    printf("%s:", nm[r]);
    for (int l = 0; l < 64; ++l) printf(" %d", h[64 * r + l]);
    printf("\n");
  }
}
