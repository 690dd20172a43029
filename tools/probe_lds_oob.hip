// Does an out-of-range buffer_load ... lds (LDS-DMA through a raw buffer resource) write zeros
// into LDS, or leave LDS as it was? Prefill LDS with a pattern, DMA 1 KB per wave through a
// resource that covers only the first `valid` bytes, read LDS back.
//   hipcc --offload-arch=gfx950 -O3 -o build/probe_lds_oob tools/probe_lds_oob.hip && build/probe_lds_oob
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(3))) void lds_void;

__global__ void probe(const float* src, float* out, int valid_bytes) {
  __shared__ __attribute__((aligned(16))) float buf[256];
  const int t = threadIdx.x;
  for (int i = t; i < 256; i += 64) buf[i] = -1.0f;  // pattern
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(src), (short)0, valid_bytes, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)buf, 16, t * 16, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = t; i < 256; i += 64) out[i] = buf[i];
}

int main() {
  float h[256];
  for (int i = 0; i < 256; ++i) h[i] = 1000.f + i;
  float *s, *o;
  hipMalloc(&s, 1024);
  hipMalloc(&o, 1024);
  hipMemcpy(s, h, 1024, hipMemcpyHostToDevice);
  for (int valid : {1024, 512, 8, 0}) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, s, o, valid);
    float r[256];
    hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    int same = 0, zero = 0, pat = 0;
    for (int i = 0; i < 256; ++i) {
      if (r[i] == h[i]) ++same;
      else if (r[i] == 0.f) ++zero;
      else if (r[i] == -1.f) ++pat;
    }
    printf("valid %4d bytes: %d floats loaded, %d zero, %d untouched (prefill), first OOB value %g\n", valid, same, zero,
           pat, valid / 4 < 256 ? r[valid / 4 + (valid % 16 ? 4 - (valid / 4) % 4 : 0)] : 0.f);
  }
  return 0;
}
