// Probe: is v_sin_f32 / v_cos_f32 of (128 + ph / 65536) revolutions bit-identical to the same
// instruction on ph / 65536 for every 16-bit phase ph? (lets a kernel build the argument with one
// v_perm_b32: the float with bits 0x4300_0000 | ph is exactly 128 + ph * 2^-16)
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_sin tools/probe_sin.hip && ./tools/probe_sin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(unsigned* mism) {
  const unsigned ph = blockIdx.x * blockDim.x + threadIdx.x;
  if (ph >= 65536) return;
  const float r0 = (float)ph * (1.0f / 65536.0f);
  const float r1 = __builtin_bit_cast(float, 0x43000000u | ph);
  const float s0 = __builtin_amdgcn_sinf(r0), s1 = __builtin_amdgcn_sinf(r1);
  const float c0 = __builtin_amdgcn_cosf(r0), c1 = __builtin_amdgcn_cosf(r1);
  if (__builtin_bit_cast(unsigned, s0) != __builtin_bit_cast(unsigned, s1)) atomicAdd(&mism[0], 1u);
  if (__builtin_bit_cast(unsigned, c0) != __builtin_bit_cast(unsigned, c1)) atomicAdd(&mism[1], 1u);
  // max abs difference in units of 2^-24
  const float ds = fabsf(s0 - s1) * 16777216.0f, dc = fabsf(c0 - c1) * 16777216.0f;
  atomicMax(&mism[2], (unsigned)ds);
  atomicMax(&mism[3], (unsigned)dc);
}

int main() {
  unsigned* d;
  unsigned h[4] = {0, 0, 0, 0};
  if (hipMalloc(&d, 16) != hipSuccess) return 1;
  hipMemcpy(d, h, 16, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(256), dim3(256), 0, 0, d);
  hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("sin mismatches %u, cos mismatches %u, max |diff| sin %u, cos %u (x 2^-24)\n", h[0], h[1], h[2], h[3]);
  hipFree(d);
  return 0;
}
