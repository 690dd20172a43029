// Standalone timing harness for the register-resident forward (siren_fwdreg.hip) at the metric
// shape (262,144 rows, 2-256-256-256-256-1, w0 = 30): builds in seconds, so kernel variants
// (-D flags) can be compared on one box without rebuilding the library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I siren_mri_amd/csrc [-DSIREN_FREG_DBG=n] \
//       -o build/fwd_bench tools/fwd_bench.hip && build/fwd_bench [iters]
// Prints the average kernel time (HIP events) and checksums of y and the phase codes (equal
// checksums across variants = the same bits).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <algorithm>
#include <vector>

#include "siren_valu.hip"
#include "siren_gemm.hip"
#include "siren_fused.hip"
#ifdef FWD_RG2  // an experimental copy with a row-group template argument (4 waves x 64 rows)
#include FWD_RG2
#define FWD_KERNEL fused_fwd_reg_kernel<2, 1, 2>
#define FWD_THREADS 256
#else
#include "siren_fwdreg.hip"
#ifndef FWD_FORM  // 1: the magic epilogue form, 0: the fract form
#define FWD_FORM 1
#endif
#define FWD_KERNEL fused_fwd_reg_kernel<2, 1, FWD_FORM>
#define FWD_THREADS 512
#endif

using namespace siren;

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

static uint32_t lcg = 12345u;
static float urand(float a) {  // uniform in [-a, a]
  lcg = lcg * 1664525u + 1013904223u;
  return a * (2.f * ((lcg >> 8) * (1.f / 16777216.f)) - 1.f);
}

// order-dependent hash of a buffer's 32-bit words, one value per workgroup (determinism checks)
__global__ void hash_kernel(const uint32_t* p, int64_t n, uint32_t* out) {
  uint32_t h = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    h ^= (p[i] + 0x9e3779b9u * (uint32_t)(i & 0xffff)) * (uint32_t)(2 * i + 1);
  for (int o = 32; o > 0; o >>= 1) h ^= __shfl_xor(h, o);
  __shared__ uint32_t sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0] ^ sh[1] ^ sh[2] ^ sh[3];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 50;
  const int64_t side = 512, rows = side * side;
  const int F = 256, C = 2, O = 1, nh = 3;
  const float w0 = 30.f;
  std::vector<float> hx(rows * C), hW0(F * C), hb0(F), hW(nh * F * F), hb(nh * F), hWL(F), hbL(1);
  for (int64_t i = 0; i < side; ++i)
    for (int64_t j = 0; j < side; ++j) {
      hx[(i * side + j) * 2 + 0] = 2.f * i / (side - 1) - 1.f;
      hx[(i * side + j) * 2 + 1] = 2.f * j / (side - 1) - 1.f;
    }
  for (auto& v : hW0) v = urand(0.5f);
  for (auto& v : hb0) v = urand(0.7f);
  for (auto& v : hW) v = urand(0.0051f);
  for (auto& v : hb) v = urand(0.0625f);
  for (auto& v : hWL) v = urand(0.0051f);
  hbL[0] = 0.01f;

  float *x, *W0, *b0, *W, *b, *WL, *bL, *y;
  _Float16 *wreg, *wlreg;
  char* P;
  CK(hipMalloc(&x, hx.size() * 4));
  CK(hipMalloc(&W0, hW0.size() * 4));
  CK(hipMalloc(&b0, hb0.size() * 4));
  CK(hipMalloc(&W, hW.size() * 4));
  CK(hipMalloc(&b, hb.size() * 4));
  CK(hipMalloc(&WL, hWL.size() * 4));
  CK(hipMalloc(&bL, 4));
  CK(hipMalloc(&y, rows * O * 4));
  CK(hipMalloc(&wreg, (size_t)nh * F * F * 2));
  CK(hipMalloc(&wlreg, FREG_WL_BYTES));
  float* wbound;
  CK(hipMalloc(&wbound, nh * F * 4));
  const int64_t pstride = rows * F * 2;
  CK(hipMalloc(&P, nh * pstride));
  CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W0, hW0.data(), hW0.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b0, hb0.data(), hb0.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(WL, hWL.data(), hWL.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bL, hbL.data(), 4, hipMemcpyHostToDevice));
  CK(hipMemset(P, 0, nh * pstride));

  RegPrepArgs p;
  memset(&p, 0, sizeof(p));
  for (int l = 0; l < nh; ++l) p.W[l] = W + (int64_t)l * F * F;
  p.WL = WL;
  p.out = wreg;
  p.outL = wlreg;
  p.wbound = wbound;
  p.nb = 1;
  p.nh = nh;
  p.O = O;
  p.k1 = w0 * kInv2Pi;
  hipLaunchKernelGGL(prep_reg_kernel, dim3(256), dim3(256), 0, 0, p);
  CK(hipGetLastError());

  FwdRegArgs a;
  memset(&a, 0, sizeof(a));
  a.x = x;
  a.W0 = W0;
  a.b0 = b0;
  a.Wreg = wreg;
  a.WLreg = wlreg;
  for (int l = 0; l < nh; ++l) a.bias[l] = b + l * F;
  a.bL = bL;
  a.wbound = FWD_FORM ? wbound : nullptr;  // (the fract form exits when the magic form applies)
  a.P0 = nullptr;
  a.Pb = P;
  a.pstride = pstride;
  a.y = y;
  a.rows_per_batch = rows;
  a.batched = 0;
  a.O = O;
  a.nh = nh;
  a.sine_out = 0;
  a.w0 = w0;
#ifdef SIREN_FREG_CLOCK
  long long* clk;
  CK(hipMalloc(&clk, 256 * 4 * sizeof(long long)));
  a.clk = clk;
#endif
  const int64_t tiles = (rows + FREG_WG_ROWS - 1) / FREG_WG_ROWS;
  dim3 grid((unsigned)std::min<int64_t>(tiles, 256)), block(FWD_THREADS);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((FWD_KERNEL), grid, block, 0, 0, a);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((FWD_KERNEL), grid, block, 0, 0, a);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<float> hy(rows);
  std::vector<uint16_t> hp(nh * rows * F);
  CK(hipMemcpy(hy.data(), y, rows * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hp.data(), P, nh * pstride, hipMemcpyDeviceToHost));
  if (argc > 2) {  // determinism: K more launches, each output's hash against the first's
    const int K = atoi(argv[2]);
    uint32_t* dh;
    CK(hipMalloc(&dh, 2 * 1024 * 4));
    std::vector<uint32_t> h0(2048), h1(2048);
    int bad = 0;
    for (int k = 0; k <= K; ++k) {
      if (k) hipLaunchKernelGGL((FWD_KERNEL), grid, block, 0, 0, a);
      hipLaunchKernelGGL(hash_kernel, dim3(1024), dim3(256), 0, 0, (const uint32_t*)y, (int64_t)rows * O, dh);
      hipLaunchKernelGGL(hash_kernel, dim3(1024), dim3(256), 0, 0, (const uint32_t*)P, (int64_t)nh * pstride / 4, dh + 1024);
      CK(hipMemcpy((k ? h1 : h0).data(), dh, 2048 * 4, hipMemcpyDeviceToHost));
      if (!k) {
        CK(hipMemcpy(hy.data(), y, rows * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hp.data(), P, nh * pstride, hipMemcpyDeviceToHost));
      }
      if (k && h1 != h0) {
        int by = 0, bp = 0;
        for (int i = 0; i < 1024; ++i) { by += h1[i] != h0[i]; bp += h1[i + 1024] != h0[i + 1024]; }
        if (bad < 5) printf("  launch %d differs: y hash blocks %d, code hash blocks %d\n", k, by, bp);
        if (bad < 3) {  // where: rows of y, and per phase layer the rows / features / blocks of the codes
          std::vector<float> yb(rows);
          std::vector<uint16_t> pb(nh * rows * F);
          CK(hipMemcpy(yb.data(), y, rows * 4, hipMemcpyDeviceToHost));
          CK(hipMemcpy(pb.data(), P, nh * pstride, hipMemcpyDeviceToHost));
          int64_t n = 0, r0 = -1, r1 = -1;
          for (int64_t i = 0; i < rows; ++i)
            if (memcmp(&yb[i], &hy[i], 4)) { ++n; if (r0 < 0) r0 = i; r1 = i; }
          printf("    y: %lld rows differ, rows %lld..%lld (tile %lld, round %lld, waves %lld..%lld)\n", (long long)n,
                 (long long)r0, (long long)r1, (long long)(r0 / 256), (long long)(r0 / 256 / grid.x),
                 (long long)(r0 % 256 / 32), (long long)(r1 % 256 / 32));
          for (int l = 0; l < nh; ++l) {
            int64_t m = 0, q0 = -1, q1 = -1;
            unsigned fmask = 0;
            for (int64_t i = 0; i < rows * F; ++i)
              if (pb[l * rows * F + i] != hp[l * rows * F + i]) {
                ++m; if (q0 < 0) q0 = i / F; q1 = i / F; fmask |= 1u << ((i % F) / 32);
              }
            if (m) printf("    P%d: %lld codes differ, rows %lld..%lld, blocks mask %02x\n", l + 1, (long long)m,
                          (long long)q0, (long long)q1, fmask);
          }
        }
        ++bad;
      }
    }
    printf("determinism: %d of %d launches differ from the first\n", bad, K);
  }
  {  // run-to-run: one more launch, bitwise comparison of y and the codes
    std::vector<float> hy2(rows);
    std::vector<uint16_t> hp2(nh * rows * F);
    hipLaunchKernelGGL((FWD_KERNEL), grid, block, 0, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hy2.data(), y, rows * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hp2.data(), P, nh * pstride, hipMemcpyDeviceToHost));
    int64_t ny = 0, np = 0, fy = -1, fp = -1;
    for (int64_t i = 0; i < rows; ++i)
      if (memcmp(&hy[i], &hy2[i], 4)) { ++ny; if (fy < 0) fy = i; }
    for (int64_t i = 0; i < (int64_t)hp.size(); ++i)
      if (hp[i] != hp2[i]) { ++np; if (fp < 0) fp = i; }
    std::vector<float> hb(nh * F);
    CK(hipMemcpy(hb.data(), wbound, nh * F * 4, hipMemcpyDeviceToHost));
    float bmax = 0.f;
    for (float v : hb) bmax = std::max(bmax, v);
    printf("rerun: y differs in %lld rows (first %lld), codes in %lld (first %lld); wbound max %.3f\n",
           (long long)ny, (long long)fy, (long long)np, (long long)fp, bmax);
  }
  double sy = 0.0;
  for (float v : hy) sy += v;
  uint64_t sp = 1469598103934665603ull;
  for (uint16_t v : hp) sp = (sp ^ v) * 1099511628211ull;
  const double us = ms * 1e3 / iters;
#ifdef SIREN_FREG_CLOCK
  {  // last launch: per-workgroup shader cycles and in-kernel clock (memtime / realtime x 100 MHz)
    std::vector<long long> hc(256 * 4);
    CK(hipMemcpy(hc.data(), clk, hc.size() * sizeof(long long), hipMemcpyDeviceToHost));
    std::vector<double> cyc, ghz;
    for (unsigned b = 0; b < grid.x; ++b) {
      const double dc = (double)(hc[4 * b + 1] - hc[4 * b]), dr = (double)(hc[4 * b + 3] - hc[4 * b + 2]);
      cyc.push_back(dc);
      ghz.push_back(dr > 0 ? dc / dr * 0.1 : 0.0);
    }
    std::sort(cyc.begin(), cyc.end());
    std::sort(ghz.begin(), ghz.end());
    printf("clock: median %.3f GHz (min %.3f, max %.3f); workgroup cycles median %.0f (max %.0f)\n",
           ghz[ghz.size() / 2], ghz.front(), ghz.back(), cyc[cyc.size() / 2], cyc.back());
  }
#endif
  {  // accuracy on the first 1024 rows against a double-precision forward of the fp32 weights:
     // y, and each stored phase code against round(fract(p / 2 pi) 2^16) (circular code steps)
    const int nchk = 1024;
    double ymax = 0.0, yref2 = 0.0, yerr2 = 0.0;
    long long cmax[8] = {0};
    double csum[8] = {0};
    std::vector<double> h(F), z(F);
    for (int r = 0; r < nchk; ++r) {
      for (int f = 0; f < F; ++f) {
        double s = hb0[f];
        for (int c = 0; c < C; ++c) s += (double)hW0[f * C + c] * hx[r * C + c];
        h[f] = std::sin(w0 * s);
      }
      for (int l = 0; l < nh; ++l) {
        for (int f = 0; f < F; ++f) {
          double s = hb[l * F + f];
          for (int k = 0; k < F; ++k) s += (double)hW[(int64_t)l * F * F + f * F + k] * h[k];
          z[f] = w0 * s;
        }
        for (int f = 0; f < F; ++f) {
          const double rev = z[f] / (2.0 * M_PI);
          const long long cref = (long long)std::llround((rev - std::floor(rev)) * 65536.0) & 0xffff;
          const long long cg = hp[(int64_t)l * rows * F + (int64_t)r * F + f];
          long long d = std::llabs(cg - cref);
          d = std::min(d, 65536 - d);
          cmax[l] = std::max(cmax[l], d);
          csum[l] += (double)d;
          h[f] = std::sin(z[f]);
        }
      }
      double yo = hbL[0];
      for (int k = 0; k < F; ++k) yo += (double)hWL[k] * h[k];
      ymax = std::max(ymax, std::fabs(yo - hy[r]));
      yref2 += yo * yo;
      yerr2 += (yo - hy[r]) * (yo - hy[r]);
    }
    printf("check (%d rows): y max-abs %.3e norm-rel %.3e; code steps", nchk, ymax, std::sqrt(yerr2 / yref2));
    for (int l = 0; l < nh; ++l) printf("  P%d max %lld mean %.2f", l + 1, cmax[l], csum[l] / ((double)nchk * F));
    printf("\n");
  }
  printf("forward %.2f us  (%.1f TF/s of %.1f GFLOP)  y-sum %.9e  P-hash %016llx\n", us,
         2.0 * rows * (C * F + nh * F * F + F * O) / (us * 1e-6) / 1e12, 2.0 * rows * (C * F + nh * F * F + F * O) / 1e9,
         sy, (unsigned long long)sp);
  return 0;
}
