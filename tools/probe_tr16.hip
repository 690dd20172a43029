// Probe: exact lane mapping of ds_read_b64_tr_b16 on gfx950.
// LDS holds M[r][c] = r*256 + c (u16), 8 rows x 64 cols. Lane l (g=l>>4, t=l&15, q=t>>2, p=t&3)
// supplies &M[q + 4*(g>>1)][16*(g&1) + 4p]; prints the 4 values each lane receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
__global__ void k(unsigned short* out) {
  __shared__ unsigned short M[8 * 64];
  for (int i = threadIdx.x; i < 8 * 64; i += 64) M[i] = (unsigned short)((i / 64) * 256 + (i % 64));
  __syncthreads();
  int l = threadIdx.x, g = l >> 4, t = l & 15, q = t >> 2, p = t & 3;
  const unsigned short* a = &M[(q + 4 * (g >> 1)) * 64 + 16 * (g & 1) + 4 * p];
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = (unsigned short)v[e];
}
int main() {
  unsigned short* d; hipMalloc(&d, 64 * 4 * 2);
  k<<<1, 64>>>(d);
  unsigned short h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int e = 0; e < 4; ++e) printf(" (r%d,c%2d)", h[l * 4 + e] >> 8, h[l * 4 + e] & 255);
    printf("\n");
  }
  return 0;
}
