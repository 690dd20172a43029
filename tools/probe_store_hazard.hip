// When does a buffer store read its data VGPRs? (VERDICT r3 "store hazard".)
// Each wave issues a buffer_store_dwordx4 of a known per-lane pattern from v[200:203], then `gap`
// independent VALU instructions (writing other registers), then overwrites v[200:203] — all in one
// inline-asm block, so the compiler's hazard recognizer and wait-count pass see nothing to fix.
// Afterwards the host counts stored dwords that hold the overwrite instead of the pattern.
// Traffic beside the stores (mode):
//   0 none
//   1 the same wave issues `k` LDS-DMA loads (buffer_load_dword ... lds) right before the store
//   2 the other half of the workgroup (waves 4-7) streams LDS-DMA loads the whole time
//   3 the same wave issues `k` ordinary buffer_load_dwordx4 (to VGPRs) right before the store
//   4 as 1, plus s_waitcnt expcnt(0) right after the store
//   5 as 1, plus s_waitcnt vmcnt(0) right after the store
//   6 as 2, plus s_waitcnt expcnt(0) right after the store
//   hipcc --offload-arch=gfx950 -O3 -o build/probe_store_hazard tools/probe_store_hazard.hip
//   build/probe_store_hazard
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define STR2(x) #x
#define STR(x) STR2(x)

constexpr int ITERS = 64;
constexpr int WAVES = 8;

template <int GAP, int MODE, int K, int NOPK = 0>
__global__ __launch_bounds__(512) void probe(uint32_t* out, const uint32_t* src, int src_words) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[WAVES][K > 0 ? K * 64 : 64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const bool storer = (MODE == 2 || MODE == 6) ? wave < 4 : true;
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(src), (short)0,
                                                                      src_words * 4, 0x00020000);
  const uint32_t ldsbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)&lds[wave][0];
  if (!storer) {
    // streaming LDS-DMA partner: K-deep bursts of dword loads from scattered lines, 4 * ITERS times
    for (int it = 0; it < 4 * ITERS; ++it) {
      uint32_t soff = (((blockIdx.x * 977u + it * 131u + wave * 17u) * 4096u) % (uint32_t)(src_words * 4 - 1024)) & ~255u;
      soff += lane * 4;
      asm volatile(
          "s_mov_b32 m0, %1\n"
          ".rept 8\n"
          "buffer_load_dword %0, %2, 0 offen lds\n"
          ".endr\n"
          "s_waitcnt vmcnt(0)\n" ::"v"(soff),
          "s"(ldsbase), "s"(rs)
          : "memory", "m0");
    }
    return;
  }
  const int slot0 = (blockIdx.x * (storer && (MODE == 2 || MODE == 6) ? 4 : WAVES) + wave) * ITERS;
  for (int it = 0; it < ITERS; ++it) {
    const uint32_t tag = (uint32_t)(slot0 + it) * 64u + lane;
    const uint32_t voff = ((uint32_t)(slot0 + it) * 64u + lane) * 16u;
    uint32_t soff = (((blockIdx.x * 577u + it * 97u + wave * 13u) * 4096u) % (uint32_t)(src_words * 4 - 1024)) & ~255u;
    soff += lane * 4;
    asm volatile(
        "v_mov_b32 v200, %0\n"
        "v_or_b32 v201, 0x10000000, %0\n"
        "v_or_b32 v202, 0x20000000, %0\n"
        "v_or_b32 v203, 0x30000000, %0\n"
        "s_mov_b32 m0, %3\n"
#if 1
        // traffic before the store
        ".if %6 == 1 || %6 == 4 || %6 == 5\n"
        ".rept %7\n"
        "buffer_load_dword %2, %4, 0 offen lds\n"
        ".endr\n"
        ".endif\n"
        ".if %6 == 3\n"
        ".rept %7\n"
        "buffer_load_dwordx4 v[210:213], %2, %4, 0 offen\n"
        ".endr\n"
        ".endif\n"
#endif
        "buffer_store_dwordx4 v[200:203], %1, %5, 0 offen\n"
        ".if %6 == 4 || %6 == 6\n"
        "s_waitcnt expcnt(0)\n"
        ".endif\n"
        ".if %6 == 5\n"
        "s_waitcnt vmcnt(0)\n"
        ".endif\n"
        ".if %9\n"
        ".rept %8\n"
        "s_nop %9 - 1\n"
        ".endr\n"
        ".else\n"
        ".rept %8\n"
        "v_add_u32 v220, 1, v220\n"
        ".endr\n"
        ".endif\n"
        "v_mov_b32 v200, 0xdead0000\n"
        "v_mov_b32 v201, 0xdead0001\n"
        "v_mov_b32 v202, 0xdead0002\n"
        "v_mov_b32 v203, 0xdead0003\n"
        "s_waitcnt vmcnt(0)\n" ::"v"(tag),
        "v"(voff), "v"(soff), "s"(ldsbase), "s"(rs), "s"(ro), "n"(MODE), "n"(K), "n"(GAP), "n"(NOPK)
        : "memory", "m0", "v200", "v201", "v202", "v203", "v210", "v211", "v212", "v213", "v220");
  }
}

// Deep store queue: 8 buffer_store_dwordx4 back to back (v[200:231]), optionally behind K LDS-DMA
// loads, then GAP filler instructions (VALU adds, or s_nop when NOP), then every data register is
// overwritten. The stores' data may be read out of the VGPRs late when the queue ahead is deep.
template <int GAP, int K, int NOP>
__global__ __launch_bounds__(512) void probe8(uint32_t* out, const uint32_t* src, int src_words) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[WAVES][K > 0 ? K * 64 : 64];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(src), (short)0,
                                                                      src_words * 4, 0x00020000);
  const uint32_t ldsbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t*)&lds[wave][0];
  const int slot0 = (blockIdx.x * WAVES + wave) * (ITERS / 8);
  for (int it = 0; it < ITERS / 8; ++it) {
    const uint32_t tag = ((uint32_t)(slot0 + it) * 64u + lane) * 8u;  // store j of this lane: tag + j
    const uint32_t voff = tag * 16u;                                     // + 16 * 64 * ... per store j below
    uint32_t soff = (((blockIdx.x * 577u + it * 97u + wave * 13u) * 4096u) % (uint32_t)(src_words * 4 - 1024)) & ~255u;
    soff += lane * 4;
    asm volatile(
        ".irp j, 0,1,2,3,4,5,6,7\n"
        "v_add_u32 v[200+4*\\j], \\j, %0\n"
        "v_or_b32 v[201+4*\\j], 0x10000000, v[200+4*\\j]\n"
        "v_or_b32 v[202+4*\\j], 0x20000000, v[200+4*\\j]\n"
        "v_or_b32 v[203+4*\\j], 0x30000000, v[200+4*\\j]\n"
        ".endr\n"
        "s_mov_b32 m0, %3\n"
        ".rept %6\n"
        "buffer_load_dword %2, %4, 0 offen lds\n"
        ".endr\n"
        ".irp j, 0,1,2,3,4,5,6,7\n"
        "buffer_store_dwordx4 v[200+4*\\j:203+4*\\j], %1, %5, 0 offen offset:16*\\j\n"
        ".endr\n"
        ".if %8\n"
        ".rept %7\n"
        "s_nop 0\n"
        ".endr\n"
        ".else\n"
        ".rept %7\n"
        "v_add_u32 v240, 1, v240\n"
        ".endr\n"
        ".endif\n"
        ".irp r, 200,201,202,203,204,205,206,207,208,209,210,211,212,213,214,215,216,217,218,219,220,221,222,223,224,225,226,227,228,229,230,231\n"
        "v_mov_b32 v\\r, 0xdead0000\n"
        ".endr\n"
        "s_waitcnt vmcnt(0)\n" ::"v"(tag),
        "v"(voff), "v"(soff), "s"(ldsbase), "s"(rs), "s"(ro), "n"(K), "n"(GAP), "n"(NOP)
        : "memory", "m0", "v200", "v201", "v202", "v203", "v204", "v205", "v206", "v207", "v208", "v209", "v210",
          "v211", "v212", "v213", "v214", "v215", "v216", "v217", "v218", "v219", "v220", "v221", "v222", "v223",
          "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v240");
  }
}

template <int GAP, int K, int NOP>
void run8(uint32_t* out, const uint32_t* src, int src_words, int blocks, const char* name) {
  const size_t stores = (size_t)blocks * WAVES * (ITERS / 8) * 64 * 8;
  hipMemset(out, 0, stores * 16);
  long bad = 0, trials = 0;
  int lanes[64] = {0};
  std::vector<uint32_t> h(stores * 4);
  for (int rep = 0; rep < 20; ++rep) {
    hipLaunchKernelGGL((probe8<GAP, K, NOP>), dim3(blocks), dim3(512), 0, 0, out, src, src_words);
    hipMemcpy(h.data(), out, stores * 16, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < stores; ++i) {
      const uint32_t t = (uint32_t)i;  // store index = tag + j (row-major: lane-major tags x 8 stores)
      for (int q = 0; q < 4; ++q) {
        const uint32_t want = q == 0 ? t : (t | ((uint32_t)q << 28));
        if (h[4 * i + q] != want) {
          ++bad;
          ++lanes[(i / 8) & 63];
        }
      }
    }
    trials += (long)stores;
  }
  printf("%-44s gap %3d (%s): %10ld corrupted dwords of %ld stores x 4", name, GAP, NOP ? "s_nop" : "VALU", bad, trials);
  if (bad) {
    printf("  lanes:");
    for (int l = 0; l < 64; ++l)
      if (lanes[l]) printf(" %d", l);
  }
  printf("\n");
}

template <int GAP, int MODE, int K, int NOPK = 0>
void run(uint32_t* out, const uint32_t* src, int src_words, int blocks, const char* name) {
  const int storers = (MODE == 2 || MODE == 6) ? 4 : WAVES;
  const size_t words = (size_t)blocks * storers * ITERS * 64 * 4;
  hipMemset(out, 0, words * 4);
  int bad = 0, bad_first = 0, trials = 0;
  std::vector<uint32_t> h(words);
  int lanes[64] = {0};
  for (int rep = 0; rep < 20; ++rep) {
    hipLaunchKernelGGL((probe<GAP, MODE, K, NOPK>), dim3(blocks), dim3(512), 0, 0, out, src, src_words);
    hipMemcpy(h.data(), out, words * 4, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < words / 4; ++i) {
      const uint32_t tag = (uint32_t)i;
      for (int j = 0; j < 4; ++j) {
        const uint32_t want = j == 0 ? tag : (tag | ((uint32_t)j << 28));
        if (h[4 * i + j] != want) {
          ++bad;
          if (j == 0) ++bad_first;
          ++lanes[i & 63];
        }
      }
    }
    trials += (int)(words / 4);
  }
  printf("%-44s gap %3d %-9s: %9d corrupted dwords (%d first-dword) of %d stores x 4", name, GAP,
         NOPK ? (NOPK == 1 ? "s_nop 0" : "s_nop 1") : "VALU", bad, bad_first, trials);
  if (bad) {
    printf("  lanes:");
    for (int l = 0; l < 64; ++l)
      if (lanes[l]) printf(" %d", l);
  }
  printf("\n");
}

int main() {
  const int src_words = 64 << 20;  // 256 MB of scattered sources (HBM misses)
  const int blocks = 1024;
  uint32_t *src, *out;
  hipMalloc(&src, (size_t)src_words * 4);
  hipMalloc(&out, (size_t)blocks * WAVES * ITERS * 64 * 16);
  hipMemset(src, 0x5a, (size_t)src_words * 4);
  run<0, 0, 0>(out, src, src_words, blocks, "no other traffic");
  run<1, 0, 0>(out, src, src_words, blocks, "no other traffic");
  run<2, 0, 0>(out, src, src_words, blocks, "no other traffic");
  run<1, 0, 0, 1>(out, src, src_words, blocks, "no other traffic");
  run<2, 0, 0, 1>(out, src, src_words, blocks, "no other traffic");
  run<3, 0, 0, 1>(out, src, src_words, blocks, "no other traffic");
  run<1, 0, 0, 2>(out, src, src_words, blocks, "no other traffic");
  run<2, 0, 0, 2>(out, src, src_words, blocks, "no other traffic");
  run<1, 1, 8, 2>(out, src, src_words, blocks, "8 LDS-DMA loads before the store");
  run<2, 1, 8, 2>(out, src, src_words, blocks, "8 LDS-DMA loads before the store");
  run<1, 2, 8, 2>(out, src, src_words, blocks, "partner waves stream LDS-DMA");
  run<2, 2, 8, 1>(out, src, src_words, blocks, "partner waves stream LDS-DMA");
  run<4, 2, 8, 1>(out, src, src_words, blocks, "partner waves stream LDS-DMA");
  run<2, 1, 8>(out, src, src_words, blocks, "8 LDS-DMA loads before the store");
  run8<0, 0, 0>(out, src, src_words, blocks, "8 stores in flight");
  run8<2, 0, 0>(out, src, src_words, blocks, "8 stores in flight");
  run8<4, 0, 0>(out, src, src_words, blocks, "8 stores in flight");
  run8<2, 8, 0>(out, src, src_words, blocks, "8 LDS-DMA + 8 stores in flight");
  run8<4, 8, 0>(out, src, src_words, blocks, "8 LDS-DMA + 8 stores in flight");
  run8<16, 8, 0>(out, src, src_words, blocks, "8 LDS-DMA + 8 stores in flight");
  run8<4, 8, 1>(out, src, src_words, blocks, "8 LDS-DMA + 8 stores in flight");
  run8<16, 8, 1>(out, src, src_words, blocks, "8 LDS-DMA + 8 stores in flight");
  run8<64, 8, 1>(out, src, src_words, blocks, "8 LDS-DMA + 8 stores in flight");
  hipError_t e = hipDeviceSynchronize();
  printf("status %s\n", hipGetErrorString(e));
  return 0;
}
