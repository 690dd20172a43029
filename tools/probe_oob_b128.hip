// Partly out-of-range multi-dword buffer loads on gfx950: does a 16-byte raw buffer load (to VGPRs,
// and as LDS-DMA) whose last dwords lie past the resource's num_records return the in-range dwords,
// or zeros for the whole access? Lane t loads 16 bytes at byte offset 4 t (so every alignment and
// every straddle position occurs) through a resource of `valid` bytes.
//   hipcc --offload-arch=gfx950 -O3 -o build/probe_oob_b128 tools/probe_oob_b128.hip && build/probe_oob_b128
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void probe_vgpr(const float* src, unsigned* out, int valid_bytes) {
  const int t = threadIdx.x;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, valid_bytes, 0x00020000);
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, t * 4, 0, 0);
  for (int e = 0; e < 4; ++e) out[4 * t + e] = v[e];
}

__global__ void probe_lds(const float* src, unsigned* out, int valid_bytes) {
  __shared__ __attribute__((aligned(16))) unsigned buf[256];
  const int t = threadIdx.x;
  for (int i = t; i < 256; i += 64) buf[i] = 0xdeadbeefu;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, valid_bytes, 0x00020000);
  // 16-byte pieces at 16-byte-aligned LDS slots, global offset shifted by 4 bytes (piece t covers
  // global dwords t*4+1 .. t*4+4)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)buf, 16, t * 16 + 4, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = t; i < 256; i += 64) out[i] = buf[i];
}

int main() {
  float h[512];
  for (int i = 0; i < 512; ++i) h[i] = 1000.f + i;
  float* s;
  unsigned* o;
  hipMalloc(&s, sizeof(h));
  hipMalloc(&o, 4096);
  hipMemcpy(s, h, sizeof(h), hipMemcpyHostToDevice);
  for (int valid : {40, 44, 48, 52, 56, 60, 64, 72}) {
    unsigned r[256];
    hipLaunchKernelGGL(probe_vgpr, dim3(1), dim3(64), 0, 0, s, o, valid);
    hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    printf("VGPR b128, valid %3d B:", valid);
    // lanes whose access straddles the end: 4t < valid < 4t + 16
    for (int t = 0; t < 64; ++t) {
      const int b0 = 4 * t;
      if (!(b0 < valid && valid < b0 + 16)) continue;
      printf("  lane %d [", t);
      for (int e = 0; e < 4; ++e) {
        const float f = __builtin_bit_cast(float, r[4 * t + e]);
        const bool inr = b0 + 4 * e < valid;
        printf("%s%s", e ? " " : "", f == 1000.f + t + e ? (inr ? "ok" : "DATA!") : (f == 0.f ? (inr ? "ZERO!" : "0") : "?"));
      }
      printf("]");
    }
    printf("\n");
    hipLaunchKernelGGL(probe_lds, dim3(1), dim3(64), 0, 0, s, o, valid);
    hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    printf("LDS-DMA  , valid %3d B:", valid);
    for (int t = 0; t < 64; ++t) {
      const int b0 = 16 * t + 4;
      if (!(b0 < valid && valid < b0 + 16)) continue;
      printf("  piece %d [", t);
      for (int e = 0; e < 4; ++e) {
        const float f = __builtin_bit_cast(float, r[4 * t + e]);
        const bool inr = b0 + 4 * e < valid;
        printf("%s%s", e ? " " : "", f == 1000.f + 4 * t + 1 + e ? (inr ? "ok" : "DATA!") : (f == 0.f ? (inr ? "ZERO!" : "0") : (r[4 * t + e] == 0xdeadbeefu ? "untouched" : "?")));
      }
      printf("]");
    }
    printf("\n");
  }
  return 0;
}
