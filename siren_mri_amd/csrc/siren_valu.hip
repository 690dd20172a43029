// siren_valu.hip — HBM-streaming kernels around the MFMA layers of the SIREN stack (gfx950).
//
// The first layer (in_features = 2 coords or 2m Fourier features) and the output layer
// (out_features 1..8) are far too narrow for MFMA: they are rank-C / rank-O products streamed at
// HBM speed. Mapping used throughout: a 32-lane half-wave owns one coordinate row and each lane
// 8 consecutive features (one 16-byte access of a 2-byte phase/grad row), so every row is read
// or written as 512 contiguous bytes; reductions over features are 5 half-wave shuffles.
//
//   first_fwd   P0 = enc(w0 (x W0^T + b0))                                  modules.py:25-26,38
//   last_fwd    y  = sin(P) W_L^T + b_L   (optionally sin(w0 .))             modules.py:25-26,78
//   last_bwd    dZ = (g W_L) cos(P) w0 ; partial dW_L = g^T sin(P), db_L = sum g
//   first_bwd   partial dW0 = dZ^T x, db0 = sum dZ ; dx = dZ W0
//   reduce      split-K slab reduction (float4 streams, 8 split lanes per column)
//   prep_weight fp32 W -> op_t W and W^T (once per call)
#include "siren_common.h"

namespace siren {

struct FirstFwdArgs {
  const float* x;      // [rows, C]
  const float* W;      // [nb_w][F, C]
  const float* b;      // [nb_w][F]
  void* P;             // [rows, F] phase_t
  int64_t rows_per_batch;
  int64_t w_bstride, b_bstride;
  int C, F;
  float w0;
};

struct LastFwdArgs {
  const void* P;       // [rows, F] phase_t
  const float* W;      // [nb_w][O, F]
  const float* b;      // [nb_w][O]
  float* y;            // [rows, O]
  int64_t rows_per_batch;
  int64_t w_bstride, b_bstride;
  int F, O;
  int sine_out;        // 1: y = sin(w0 * z) (outermost_linear == False)
  float w0;
  // LOSS (last_fwd_kernel<.., true>): the image loss of siren_mlp_forward_loss in the output
  // epilogue, the register forward's arithmetic (siren_fwdreg.hip FwdRegArgs l* fields)
  const float* ltgt;   // [B*N, O]
  const float* lk0;    // [B, O, N] or null
  const float* lmask;  // [B, O, N]
  const float* lhf;    // [N] or null
  float* ldc;          // [B*N, O] or null
  float* ldy;          // [B*N, O]
  float* lloss;        // [1]
  float* lpart;        // [grid] per-workgroup sums
  unsigned* lcounter;  // zero between launches
  float lnoise, lweight;
};

struct LastBwdArgs {
  const void* P;       // [rows, F] phase_t
  const float* W;      // [nb_w][O, F]
  const float* b;      // [nb_w][O]
  const float* dy;     // [rows, O]
  const float* dy_scale;  // [1] device scalar multiplying dy (a fused loss's upstream gradient), or null
  void* dZ;            // [rows, F] grad_t
  float* part;         // split s, batch b slab at part + s*split_stride + b*(O*F + O)
  int64_t rows_per_batch;
  int64_t rows_per_split;
  int64_t split_stride;
  int64_t w_bstride, b_bstride;
  int F, O;
  int sine_out;
  float w0;
};

struct FirstBwdArgs {
  const void* dZ;      // [rows, F] grad_t
  const float* x;      // [rows, C]
  const float* W;      // [nb_w][F, C]
  float* dx;           // [rows, C] or null
  float* part;         // split s, batch b slab at part + s*split_stride + b*(F*C + F)
  int64_t rows_per_batch;
  int64_t rows_per_split;
  int64_t split_stride;
  int64_t w_bstride;
  int F, C;
  const float* ffB;    // first_bwd_wide_mfma: Fourier-feature input (x = ffin raw coordinates per row), or null
  int ffin;
};

// 8-element row chunk loads/stores (16 B for 2-byte types, 32 B for fp32).
DEV void load8(const uint16_t* p, uint16_t (&v)[8]) {
  const u16x8 t = *(const u16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = t[e];
}
DEV void load8(const float* p, float (&v)[8]) {
  const f32x4 a = ((const f32x4*)p)[0], b = ((const f32x4*)p)[1];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = a[e];
    v[e + 4] = b[e];
  }
}
DEV void load8f(const bf16* p, float (&v)[8]) {
  const bf16x8 t = *(const bf16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)t[e];
}
DEV void load8f(const float* p, float (&v)[8]) { load8(p, v); }

DEV void store8(uint16_t* p, const uint16_t (&v)[8]) {
  u16x8 t;
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = v[e];
  *(u16x8*)p = t;
}
DEV void store8(float* p, const float (&v)[8]) {
  f32x4 a, b;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] = v[e];
    b[e] = v[e + 4];
  }
  ((f32x4*)p)[0] = a;
  ((f32x4*)p)[1] = b;
}
DEV void store8f(bf16* p, const float (&v)[8]) {
  bf16x8 t;
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = (bf16)v[e];
  *(bf16x8*)p = t;
}
DEV void store8f(float* p, const float (&v)[8]) { store8(p, v); }

// Sum over the 32 lanes of a half-wave (every lane gets the total).
DEV float half_sum(float v) {
#pragma unroll
  for (int off = 16; off >= 1; off >>= 1) v += __shfl_xor(v, off, 32);
  return v;
}

// ------------------------------------------------------------------------------------------
// first_fwd: W0 is staged transposed in LDS ([C][F], then b0) so every thread reads its 8
// features' weights with two 16-byte LDS reads per input channel; no dependent global loads.
template <int PREC, int MAXC>
__global__ __launch_bounds__(256) void first_fwd_kernel(FirstFwdArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  __shared__ __attribute__((aligned(16))) float Ws[(MAXC + 1) * 512];
  const int64_t batch = blockIdx.y;
  const int F = a.F, C = a.C;
  const float* W = a.W + batch * a.w_bstride;
  const float* bias = a.b + batch * a.b_bstride;
  for (int i = threadIdx.x; i < F * C; i += 256) {
    const int f = i / C, c = i - f * C;
    Ws[c * F + f] = W[i];
  }
  for (int f = threadIdx.x; f < F; f += 256) Ws[MAXC * F + f] = bias[f];
  __syncthreads();
  const uint32_t F8 = (uint32_t)(F >> 3);
  const uint32_t total = (uint32_t)a.rows_per_batch * F8;
  for (uint32_t idx = blockIdx.x * 256u + threadIdx.x; idx < total; idx += gridDim.x * 256u) {
    const uint32_t r = idx / F8;
    const int f = (int)(idx - r * F8) * 8;
    const int64_t row = batch * a.rows_per_batch + r;
    float xv[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) xv[c] = (c < C) ? a.x[row * C + c] : 0.f;
    float z[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      if (c < C) {
        const f32x4 w0v = *(const f32x4*)(Ws + c * F + f);
        const f32x4 w1v = *(const f32x4*)(Ws + c * F + f + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          z[e] = fmaf(xv[c], w0v[e], z[e]);
          z[e + 4] = fmaf(xv[c], w1v[e], z[e + 4]);
        }
      }
    }
    const f32x4 b0v = *(const f32x4*)(Ws + MAXC * F + f);
    const f32x4 b1v = *(const f32x4*)(Ws + MAXC * F + f + 4);
    phase_t out[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      out[e] = PT::encz(z[e], b0v[e], a.w0);
      out[e + 4] = PT::encz(z[e + 4], b1v[e], a.w0);
    }
    store8((phase_t*)a.P + row * F + f, out);
  }
}

// ------------------------------------------------------------------------------------------
// LOSS: also the fused image loss (siren_mlp_forward_loss on the per-layer path: fp32 mode and the
// bf16 shapes outside the register forward): per output element p = DC(y) (with k0), d = hf (p - t),
// the lane's sum of d^2, DC(y) and dL/dy = 2 w hf d dDC/dy — fused_fwd_reg_kernel's LOSS epilogue
// arithmetic — then the workgroup sums through the write-through ticket hand-off of siren_loss.hip
// (deterministic: fixed per-lane row order, wave / workgroup trees, workgroup sums in index order).
template <int PREC, int IT, int MAXO, bool LOSS = false>
__global__ __launch_bounds__(256) void last_fwd_kernel(LastFwdArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  const int l32 = threadIdx.x & 31;
  float lsum = 0.f;
  const int64_t batch = blockIdx.y;
  const float* W = a.W + batch * a.w_bstride;
  const float* bias = a.b + batch * a.b_bstride;
  float w[IT][MAXO][8];
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int o = 0; o < MAXO; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int f = 256 * it + 8 * l32 + e;
        w[it][o][e] = (o < a.O && f < a.F) ? W[o * a.F + f] : 0.f;
      }
  for (int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); r < a.rows_per_batch;
       r += (int64_t)gridDim.x * 8) {
    const int64_t row = batch * a.rows_per_batch + r;
    const phase_t* pr = (const phase_t*)a.P + row * a.F;
    float acc[MAXO];
#pragma unroll
    for (int o = 0; o < MAXO; ++o) acc[o] = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int f = 256 * it + 8 * l32;
      if (f < a.F) {
        phase_t pv[8];
        load8(pr + f, pv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float h = PT::sinp(pv[e]);
#pragma unroll
          for (int o = 0; o < MAXO; ++o) acc[o] = fmaf(h, w[it][o][e], acc[o]);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < MAXO; ++o) {
      if (o < a.O) {
        float z = half_sum(acc[o]) + bias[o];
        if (a.sine_out) z = PT::sinr(a.w0 * z);
        if (l32 == o) {
          a.y[row * a.O + o] = z;
          if constexpr (LOSS) {
            const int64_t q = row * a.O + o;  // [B*N, O] element
            float p = z, coef = 1.f;
            if (a.lk0) {
              const int64_t pl = (batch * a.O + o) * a.rows_per_batch + r;  // NCHW plane element
              const float m = a.lmask[pl];
              p = dc_value(z, a.lk0[pl], m, a.lnoise);
              coef = dc_coef(m, a.lnoise);
              a.ldc[q] = p;
            }
            const float h = a.lhf ? a.lhf[r] : 1.f;
            const float dd = __fmul_rn(h, __fsub_rn(p, a.ltgt[q]));
            lsum = fmaf(dd, dd, lsum);
            float v = h * (dd * (2.f * a.lweight));
            if (a.lk0) v *= coef;
            a.ldy[q] = v;
          }
        }
      }
    }
  }
  if constexpr (LOSS) {
    __shared__ float lred[4];
    __shared__ unsigned lticket;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float ws_ = wave_sum(lsum);
    if (lane == 0) lred[wave] = ws_;
    __syncthreads();
    const unsigned nwg = gridDim.x * gridDim.y, wg = blockIdx.y * gridDim.x + blockIdx.x;
    if (tid == 0) {
      const float sacc = (lred[0] + lred[1]) + (lred[2] + lred[3]);
      __hip_atomic_store(a.lpart + wg, sacc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lticket = __hip_atomic_fetch_add(a.lcounter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (lticket == nwg - 1) {
      float sacc = 0.f;
      for (unsigned b = tid; b < nwg; b += 256) sacc += __hip_atomic_load(a.lpart + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sacc = wave_sum(sacc);
      __syncthreads();
      if (lane == 0) lred[wave] = sacc;
      __syncthreads();
      if (tid == 0) {
        a.lloss[0] = ((lred[0] + lred[1]) + (lred[2] + lred[3])) * a.lweight;
        __hip_atomic_store(a.lcounter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
template <int PREC, int IT, int MAXO>
__global__ __launch_bounds__(256) void last_bwd_kernel(LastBwdArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  __shared__ float red[8][MAXO * 256 + MAXO];
  const int l32 = threadIdx.x & 31;
  const int grp = threadIdx.x >> 5;  // 8 row groups (half-waves) per block
  const int split = blockIdx.x;
  const int64_t batch = blockIdx.y;
  const float* W = a.W + batch * a.w_bstride;
  const float* bias = a.b + batch * a.b_bstride;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.rows_per_batch) r_end = a.rows_per_batch;
  float w[IT][MAXO][8];
  float dw[IT][MAXO][8];
  const float dys = a.dy_scale ? *a.dy_scale : 1.f;
  float db[MAXO];
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int o = 0; o < MAXO; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int f = 256 * it + 8 * l32 + e;
        w[it][o][e] = (o < a.O && f < a.F) ? W[o * a.F + f] : 0.f;
        dw[it][o][e] = 0.f;
      }
#pragma unroll
  for (int o = 0; o < MAXO; ++o) db[o] = 0.f;

  // RU rows per half-wave in flight: their loads are issued together (memory-level parallelism),
  // then processed in row order (the same per-thread summation order as one row at a time).
  constexpr int RU = (IT == 1 && MAXO <= 2) ? 4 : (IT == 2 && MAXO <= 2) ? 2 : 1;
  for (int64_t r0 = r_begin + grp; r0 < r_end; r0 += 8 * RU) {
  float gq[RU][MAXO];
  phase_t pq[RU][IT][8];
#pragma unroll
  for (int k = 0; k < RU; ++k) {
    const int64_t r = r0 + 8 * k;
    const int64_t row = batch * a.rows_per_batch + (r < r_end ? r : r0);
    const phase_t* pr = (const phase_t*)a.P + row * a.F;
#pragma unroll
    for (int o = 0; o < MAXO; ++o) gq[k][o] = (o < a.O) ? a.dy[row * a.O + o] * dys : 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int f = 256 * it + 8 * l32;
      if (f < a.F) load8(pr + f, pq[k][it]);
    }
  }
#pragma unroll
  for (int k = 0; k < RU; ++k) {
    const int64_t r = r0 + 8 * k;
    if (r >= r_end) break;
    const int64_t row = batch * a.rows_per_batch + r;
    float g[MAXO];
#pragma unroll
    for (int o = 0; o < MAXO; ++o) g[o] = gq[k][o];
    phase_t (&pv)[IT][8] = pq[k];
    if (a.sine_out) {
      float acc[MAXO];
#pragma unroll
      for (int o = 0; o < MAXO; ++o) acc[o] = 0.f;
#pragma unroll
      for (int it = 0; it < IT; ++it)
        if (256 * it + 8 * l32 < a.F)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float h = PT::sinp(pv[it][e]);
#pragma unroll
            for (int o = 0; o < MAXO; ++o) acc[o] = fmaf(h, w[it][o][e], acc[o]);
          }
#pragma unroll
      for (int o = 0; o < MAXO; ++o)
        if (o < a.O) g[o] = (g[o] * PT::cosr(a.w0 * (half_sum(acc[o]) + bias[o]))) * a.w0;
    }
#pragma unroll
    for (int o = 0; o < MAXO; ++o) db[o] += g[o];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int f = 256 * it + 8 * l32;
      if (f < a.F) {
        float dz[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float s = PT::sinp(pv[it][e]), c = PT::cosp(pv[it][e]);
          // (sum_o g_o (W_L[o][f] w0)) cos(P): the arithmetic of every output-layer fusion
          // (siren_gemm.hip, W_L prescaled by w0 once)
          float dh = g[0] * (w[it][0][e] * a.w0);
#pragma unroll
          for (int o = 1; o < MAXO; ++o) dh = fmaf(g[o], w[it][o][e] * a.w0, dh);
#pragma unroll
          for (int o = 0; o < MAXO; ++o) dw[it][o][e] = fmaf(g[o], s, dw[it][o][e]);
          dz[e] = dh * c;
        }
        store8f((grad_t*)a.dZ + row * a.F + f, dz);
      }
    }
  }
  }
  // Reduce the 8 row groups through LDS, 256 features at a time; one slab write per block.
  float* part = a.part + (int64_t)split * a.split_stride + batch * (int64_t)(a.O * a.F + a.O);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
#pragma unroll
    for (int o = 0; o < MAXO; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[grp][o * 256 + 8 * l32 + e] = dw[it][o][e];
    if (it == 0 && l32 == 0) {
#pragma unroll
      for (int o = 0; o < MAXO; ++o) red[grp][MAXO * 256 + o] = db[o];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < a.O * 256; idx += 256) {
      const int o = idx >> 8, f = 256 * it + (idx & 255);
      if (f < a.F) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += red[k][idx];
        part[o * a.F + f] = s;
      }
    }
    if (it == 0 && (int)threadIdx.x < a.O) {
      const int k0 = MAXO * 256 + threadIdx.x;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += red[k][k0];
      part[a.O * a.F + threadIdx.x] = s;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// first_bwd: LPR lanes per row, FPL features per lane (C <= 4: 32 x 8; else 64 x 4).
template <int PREC, int IT, int MAXC>
__global__ __launch_bounds__(256) void first_bwd_kernel(FirstBwdArgs a) {
  using PT = Prec<PREC>;
  using grad_t = typename PT::grad_t;
  constexpr int FPL = (MAXC <= 4) ? 8 : 4;
  constexpr int LPR = 256 / FPL;
  constexpr int GROUPS = 256 / LPR;
  __shared__ float red[GROUPS][256 * (MAXC + 1)];
  const int li = threadIdx.x % LPR;
  const int grp = threadIdx.x / LPR;
  const int split = blockIdx.x;
  const int64_t batch = blockIdx.y;
  const float* W = a.W + batch * a.w_bstride;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.rows_per_batch) r_end = a.rows_per_batch;
  float wv[IT][FPL][MAXC];
  float dw[IT][FPL][MAXC];
  float db[IT][FPL];
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int e = 0; e < FPL; ++e) {
      const int f = 256 * it + FPL * li + e;
      db[it][e] = 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        wv[it][e][c] = (f < a.F && c < a.C) ? W[f * a.C + c] : 0.f;
        dw[it][e][c] = 0.f;
      }
    }
  constexpr int RU = 1;  // (4 rows in flight measured slower here than in last_bwd_kernel)
  for (int64_t r0 = r_begin + grp; r0 < r_end; r0 += GROUPS * RU) {
  float xq[RU][MAXC];
  float dzq[RU][IT][8];
#pragma unroll
  for (int k = 0; k < RU; ++k) {
    const int64_t r = r0 + GROUPS * k;
    const int64_t row = batch * a.rows_per_batch + (r < r_end ? r : r0);
#pragma unroll
    for (int c = 0; c < MAXC; ++c) xq[k][c] = (c < a.C) ? a.x[row * a.C + c] : 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int f = 256 * it + FPL * li;
      if (f < a.F) {
        if constexpr (FPL == 8) {
          load8f((const grad_t*)a.dZ + row * a.F + f, dzq[k][it]);
        } else {
          const grad_t* src = (const grad_t*)a.dZ + row * a.F + f;
#pragma unroll
          for (int e = 0; e < 4; ++e) dzq[k][it][e] = to_f32(src[e]);
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < RU; ++k) {
    const int64_t r = r0 + GROUPS * k;
    if (r >= r_end) break;
    const int64_t row = batch * a.rows_per_batch + r;
    float xv[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) xv[c] = xq[k][c];
    float dxp[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) dxp[c] = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int f = 256 * it + FPL * li;
      if (f < a.F) {
        float (&dz)[8] = dzq[k][it];
#pragma unroll
        for (int e = 0; e < FPL; ++e) {
          db[it][e] += dz[e];
#pragma unroll
          for (int c = 0; c < MAXC; ++c) {
            dw[it][e][c] = fmaf(dz[e], xv[c], dw[it][e][c]);
            dxp[c] = fmaf(dz[e], wv[it][e][c], dxp[c]);
          }
        }
      }
    }
    if (a.dx) {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        if (c < a.C) {
          float s = dxp[c];
#pragma unroll
          for (int off = LPR / 2; off >= 1; off >>= 1) s += __shfl_xor(s, off, LPR);
          if (li == 0) a.dx[row * a.C + c] = s;
        }
      }
    }
  }
  }
  float* part = a.part + (int64_t)split * a.split_stride + batch * (int64_t)(a.F * a.C + a.F);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
#pragma unroll
    for (int e = 0; e < FPL; ++e) {
      const int fl = FPL * li + e;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) red[grp][fl * (MAXC + 1) + c] = dw[it][e][c];
      red[grp][fl * (MAXC + 1) + MAXC] = db[it][e];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < 256 * (MAXC + 1); idx += 256) {
      const int fl = idx / (MAXC + 1), c = idx % (MAXC + 1);
      const int f = 256 * it + fl;
      if (f >= a.F || (c >= a.C && c != MAXC)) continue;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < GROUPS; ++k) s += red[k][idx];
      if (c < a.C) part[f * a.C + c] = s;
      else part[a.F * a.C + f] = s;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// first_bwd_wide: dW_0 = dZ_0^T x and db_0 = sum dZ_0 for the wide first layer (5..16 inputs:
// configs 4/5's Fourier features) when no input gradient is asked for. One thread per hidden
// feature f (F <= 256), accumulating its C + 1 sums in registers over the split's rows: a row is one
// coalesced 2-byte dZ read per lane plus the row's x (<= 64 B, the same address in every lane),
// eight rows in flight. first_bwd_kernel's lanes-per-row mapping kept 64 lanes on one row and one
// row in flight, ~1.4 ms per C4 step. Each (split, f) sum runs in a fixed row order (deterministic).
constexpr int FBW_ROWS = 8;
template <int PREC, int CC>  // CC: the input count when known at compile time (16), else 0
__global__ __launch_bounds__(256) void first_bwd_wide_kernel(FirstBwdArgs a) {
  using grad_t = typename Prec<PREC>::grad_t;
  constexpr int MAXC = 16;
  const int f = threadIdx.x;
  const int split = blockIdx.x;
  const int64_t batch = blockIdx.y;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  const int64_t r_end = r_begin + a.rows_per_split < a.rows_per_batch ? r_begin + a.rows_per_split : a.rows_per_batch;
  const int C = CC ? CC : a.C;
  const bool live = f < a.F;
  float dw[MAXC], db = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) dw[c] = 0.f;
  const grad_t* dz = (const grad_t*)a.dZ + batch * a.rows_per_batch * a.F + (live ? f : 0);
  const float* xb = a.x + batch * a.rows_per_batch * C;
  for (int64_t r0 = r_begin; r0 < r_end; r0 += FBW_ROWS) {
    float z[FBW_ROWS], xv[FBW_ROWS][MAXC];
#pragma unroll
    for (int k = 0; k < FBW_ROWS; ++k) {
      const int64_t r = r0 + k < r_end ? r0 + k : r_end - 1;
      z[k] = r0 + k < r_end ? to_f32(dz[r * a.F]) : 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) xv[k][c] = c < C ? xb[r * C + c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < FBW_ROWS; ++k) {
      db += z[k];
#pragma unroll
      for (int c = 0; c < MAXC; ++c) dw[c] = fmaf(z[k], xv[k][c], dw[c]);
    }
  }
  if (!live) return;
  float* part = a.part + (int64_t)split * a.split_stride + batch * (int64_t)(a.F * C + a.F);
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
    if (c < C) part[f * C + c] = dw[c];
  part[a.F * C + f] = db;
}

// ------------------------------------------------------------------------------------------
// first_bwd_wide_mfma (bf16 mode, F = 256, 5..16 inputs): dW_0 = dZ_0^T x and db_0 = sum dZ_0 on
// the bf16 MFMA, rows as the K dimension. Per 32-row chunk the dZ_0 rows (32 x 256 bf16, rows of 576
// bytes) and x as bf16 hi | lo columns (32 x 32, rows of 64 bytes) are staged in LDS and read with
// transposing ds_read_b64_tr_b16 (tn_dw_kernel's lane roles); wave w owns features 64 w .. 64 w + 63:
// D[f][c'] = dZ^T [x_hi | x_lo] (dW = D[:, c] + D[:, 16 + c], ~2^-16 of x) and db from a second
// MFMA against a ones column. The next chunk's global loads are in flight during this chunk's
// MFMAs. One partial slab per workgroup, first_bwd_wide_kernel's layout and split.
// (first_bwd_wide_kernel, one thread per feature: 0.34 ms of the C4 step.)
constexpr int FBM_DZROW = 576;   // bytes per staged dZ row (512 + 64: 4-row transposing reads conflict-free)
constexpr int FBM_XROW = 64;     // bytes per staged x row (32 bf16)
__global__ __launch_bounds__(256) void first_bwd_wide_mfma_kernel(FirstBwdArgs a) {
  __shared__ __attribute__((aligned(16))) char sdz[32 * FBM_DZROW];
  __shared__ __attribute__((aligned(16))) char sx[32 * FBM_XROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x;
  const int64_t batch = blockIdx.y;
  const int64_t rows = a.rows_per_batch;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  const int64_t r_end = r_begin + a.rows_per_split < rows ? r_begin + a.rows_per_split : rows;
  const int C = a.C;
  const bf16* dz = (const bf16*)a.dZ + batch * rows * 256;
  const float* xb = a.x + batch * rows * C;
  const float* xraw = a.x + batch * rows * (a.ffB ? a.ffin : 0);
  __shared__ float sB[32];  // Fourier-feature input: B [ffin][C / 2]
  if (a.ffB && tid < 32) sB[tid] = tid < a.ffin * (C / 2) ? a.ffB[tid] : 0.f;
  __syncthreads();
  f32x16 acc[2], acd[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = acd[i][e] = 0.f;
  // ones column for db: B[k][0] = 1
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (lane & 31) == 0 ? (bf16)1.f : (bf16)0.f;

  // loads of chunk r0: dZ pieces q = tid + 256 j (row q / 32, 16-byte piece q % 32), x: thread t < 128
  // holds row t / 4, channels 4 (t % 4) .. + 4 (zeros past C and past the range)
  u32x4_t zv[4];
  f32x4 xv;
  auto load = [&](int64_t r0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = tid + 256 * j, r = q >> 5, pc = q & 31;
      const int64_t row = r0 + r < r_end ? r0 + r : r_end - 1;
      const u32x4_t v = *(const u32x4_t*)(dz + row * 256 + 8 * pc);
      const u32x4_t zero = {0u, 0u, 0u, 0u};
      zv[j] = r0 + r < r_end ? v : zero;
    }
    if (tid < 128) {
      const int r = tid >> 2, c0 = 4 * (tid & 3);
      const int64_t row = r0 + r;
      if (a.ffB) {
        // features c0 .. c0 + 3 of the row from its raw coordinates (the forward's ff_feature)
        float xr[4] = {0.f, 0.f, 0.f, 0.f};
        if (row < r_end)
          for (int c = 0; c < a.ffin; ++c) xr[c] = xraw[row * a.ffin + c];
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[e] = row < r_end ? ff_feature(xr, sB, a.ffin, C / 2, c0 + e) : 0.f;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[e] = (row < r_end && c0 + e < C) ? xb[row * C + c0 + e] : 0.f;
      }
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = tid + 256 * j, r = q >> 5, pc = q & 31;
      *(u32x4_t*)(sdz + r * FBM_DZROW + 16 * pc) = zv[j];
    }
    if (tid < 128) {
      const int r = tid >> 2, c0 = 4 * (tid & 3);
      bf16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (bf16)xv[e];
        lo[e] = (bf16)(xv[e] - (float)hi[e]);
      }
      *(bf16x4*)(sx + r * FBM_XROW + 2 * c0) = hi;
      *(bf16x4*)(sx + r * FBM_XROW + 2 * (16 + c0)) = lo;
    }
  };
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  if (r_begin < r_end) load(r_begin);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 32) {
    __syncthreads();  // the previous chunk's reads are done
    stage();
    __syncthreads();
    if (r0 + 32 < r_end) load(r0 + 32);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int nb = 16 * ks + 8 * (g >> 1) + tq;
      const int cx = 16 * (g & 1) + 4 * tp;
      const bf16x8 bx = lds_read_tr16_pair(sx + nb * FBM_XROW + 2 * cx, sx + (nb + 4) * FBM_XROW + 2 * cx);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int cf = 64 * wave + 32 * i + 16 * (g & 1) + 4 * tp;
        const bf16x8 af = lds_read_tr16_pair(sdz + nb * FBM_DZROW + 2 * cf, sdz + (nb + 4) * FBM_DZROW + 2 * cf);
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bx, acc[i], 0, 0, 0);
        acd[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, ones, acd[i], 0, 0, 0);
      }
    }
  }
  float* part = a.part + (int64_t)split * a.split_stride + batch * (int64_t)(256 * C + 256);
  const int cn = lane & 31;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int f = 64 * wave + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      const float lo = __shfl_xor(acc[i][e], 16, 32);
      if (cn < C) part[f * C + cn] = acc[i][e] + lo;
      if (cn == 0) part[256 * C + f] = acd[i][e];
    }
}

// ------------------------------------------------------------------------------------------
// first_dx_wide (bf16 mode, F = 256, 5..16 inputs): the wide first layer's input gradient
// dx = dZ_0 W_0 ([rows, 256] x [256, C]) on the bf16 MFMA, beside first_bwd_wide_kernel (which has
// no input gradient). Per wave, 32-row tiles: the A operand is the tile's dZ_0 rows straight from
// HBM (16-byte loads), the B operand W_0 split into bf16 hi (columns 0..15) and lo (16..31) parts
// held in registers, so acc[:, c] + acc[:, 16 + c] is dZ_0 W_0 to ~2^-16 of W_0 (the precision of
// the bottom pair's dx, dx_ring_body_v2bot). The hi and lo halves meet in lanes n and n + 16.
// (first_bwd_kernel's 64 lanes per row took ~1.4 ms of the C4 step for this product.)
__global__ __launch_bounds__(256) void first_dx_wide_kernel(FirstBwdArgs a) {
  constexpr int F = 256, NKS = F / 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = lane & 31, kh = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int C = a.C;
  // B fragments: lane (n, kh) holds B[16 ks + 8 kh + e][n], B = [W_0 hi | W_0 lo] (K = features)
  const float* W = a.W + batch * a.w_bstride;
  bf16x8 wb[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int f = 16 * ks + 8 * kh + e, c = n & 15;
      const float w = c < C ? W[f * C + c] : 0.f;
      const bf16 hi = (bf16)w;
      wb[ks][e] = n < 16 ? hi : (bf16)(w - (float)hi);
    }
  const int64_t rows = a.rows_per_batch;
  const bf16* dz = (const bf16*)a.dZ + batch * rows * F;
  float* dx = a.dx + batch * rows * C;
  const int64_t ntile = (rows + 31) / 32;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < ntile; t += (int64_t)gridDim.x * 4) {
    const int64_t r0 = t * 32;
    const int64_t ra = r0 + n < rows ? r0 + n : rows - 1;
    const bf16* src = dz + ra * F + 8 * kh;
    bf16x8 av[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) av[ks] = *(const bf16x8*)(src + 16 * ks);
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[ks], wb[ks], acc, 0, 0, 0);
    // acc[e] = C[i][n], i = (e & 3) + 8 (e >> 2) + 4 kh; column n < 16: hi part, n + 16: lo part
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float lo = __shfl_xor(acc[e], 16, 32);
      const int64_t r = r0 + (e & 3) + 8 * (e >> 2) + 4 * kh;
      if (n < C && r < rows) dx[r * C + n] = acc[e] + lo;
    }
  }
}

// ------------------------------------------------------------------------------------------
// reduce: out[e] = sum_s part[s * split_stride + e] for e < total (= nb * slab). Element e of
// batch slab b goes to out0[b*n_first + r] (r < n_first) or out1[b*(slab-n_first) + r-n_first].
// Block = 32 float4 columns x 8 split lanes; split_stride % 4 == 0.
__global__ __launch_bounds__(256) void reduce_kernel(const float* part, int nsplit, int64_t split_stride,
                                                     int total, int slab, int n_first, float* out0,
                                                     float* out1) {
  __shared__ f32x4 red[8][32];
  const int c4 = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int base = (blockIdx.x * 32 + c4) * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (base < total) {
    int s = sl;
    for (; s + 24 < nsplit; s += 32) {
      const f32x4 v0 = *(const f32x4*)(part + (int64_t)s * split_stride + base);
      const f32x4 v1 = *(const f32x4*)(part + (int64_t)(s + 8) * split_stride + base);
      const f32x4 v2 = *(const f32x4*)(part + (int64_t)(s + 16) * split_stride + base);
      const f32x4 v3 = *(const f32x4*)(part + (int64_t)(s + 24) * split_stride + base);
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; s < nsplit; s += 8) acc += *(const f32x4*)(part + (int64_t)s * split_stride + base);
  }
  red[sl][c4] = acc;
  __syncthreads();
  if (sl == 0 && base < total) {
    f32x4 t = red[0][c4];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += red[k][c4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = base + e;
      if (idx >= total) break;
      const int b = idx / slab, r = idx - b * slab;
      if (r < n_first) out0[(int64_t)b * n_first + r] = t[e];
      else out1[(int64_t)b * (slab - n_first) + (r - n_first)] = t[e];
    }
  }
}

// Several reductions in one launch (the slabs of one backward kernel: a layer's dW/db and the
// folded first or output layer's): block b belongs to the segment whose block range holds it.
// Each segment's arithmetic is reduce_kernel's (same summation order).
constexpr int REDUCE_MAXSEG = 3;
struct ReduceSeg {
  const float* part;
  float* out0;
  float* out1;
  int64_t split_stride;
  int nsplit, total, slab, n_first, blocks;
};
struct ReduceMultiArgs {
  ReduceSeg seg[REDUCE_MAXSEG];
  int nseg;
};
// One 128-float block of a segmented slab reduction (256 threads t = threadIdx.x - t0; red: this
// group's 8 x 32 f32x4 of LDS). Shared by reduce_multi_kernel and the tail of the next paired
// backward launch (pair_ring_bf16_kernel), so both sum in the same order.
DEV int reduce_total_blocks(const ReduceMultiArgs& a) {
  int n = 0;
  for (int i = 0; i < a.nseg; ++i) n += a.seg[i].blocks;
  return n;
}
DEV void reduce_block(const ReduceMultiArgs& a, int blk, int t, f32x4 (*red)[32]) {
  int si = 0;
  while (si + 1 < a.nseg && blk >= a.seg[si].blocks) blk -= a.seg[si++].blocks;
  const ReduceSeg& g = a.seg[si];
  const int c4 = t & 31, sl = t >> 5;
  const int base = (blk * 32 + c4) * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (base < g.total) {
    int s = sl;
    for (; s + 24 < g.nsplit; s += 32) {
      const f32x4 v0 = *(const f32x4*)(g.part + (int64_t)s * g.split_stride + base);
      const f32x4 v1 = *(const f32x4*)(g.part + (int64_t)(s + 8) * g.split_stride + base);
      const f32x4 v2 = *(const f32x4*)(g.part + (int64_t)(s + 16) * g.split_stride + base);
      const f32x4 v3 = *(const f32x4*)(g.part + (int64_t)(s + 24) * g.split_stride + base);
      acc += (v0 + v1) + (v2 + v3);
    }
    for (; s < g.nsplit; s += 8) acc += *(const f32x4*)(g.part + (int64_t)s * g.split_stride + base);
  }
  red[sl][c4] = acc;
  __syncthreads();
  if (sl == 0 && base < g.total) {
    f32x4 v = red[0][c4];
#pragma unroll
    for (int k = 1; k < 8; ++k) v += red[k][c4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = base + e;
      if (idx >= g.total) break;
      const int b = idx / g.slab, r = idx - b * g.slab;
      if (r < g.n_first) g.out0[(int64_t)b * g.n_first + r] = v[e];
      else g.out1[(int64_t)b * (g.slab - g.n_first) + (r - g.n_first)] = v[e];
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void reduce_multi_kernel(ReduceMultiArgs a) {
  __shared__ f32x4 red[8][32];
  reduce_block(a, blockIdx.x, threadIdx.x, red);
}

// ------------------------------------------------------------------------------------------
// Weight preparation for every MFMA layer in one launch (blockIdx.y = layer):
// W [nb][O][I] fp32 -> Wop [nb][O][I] op_t (bf16 only) and WtOp [nb][I][O] op_t.
struct PrepArgs {
  const float* W[16];
  void* Wop[16];  // [nb][O, Kp] op_t, zero-padded along K (Kp >= I), or null
  void* Wt[16];   // [nb][I, O] op_t
  int O[16], I[16], Kp[16];
  int64_t nb;
};

// Every MFMA layer's operand copies in one launch (blockIdx.y = layer).
template <int PREC>
__global__ __launch_bounds__(256) void prep_weights_kernel(PrepArgs a) {
  using op_t = typename Prec<PREC>::op_t;
  const int l = blockIdx.y;
  const int O = a.O[l], I = a.I[l], Kp = a.Kp[l];
  const float* W = a.W[l];
  op_t* Wop = (op_t*)a.Wop[l];
  op_t* Wt = (op_t*)a.Wt[l];
  const int64_t per = (int64_t)O * I;
  const int64_t perp = (int64_t)O * Kp;
  const int64_t total = a.nb * perp;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t b = idx / perp;
    const int rem = (int)(idx - b * perp);
    const int o = rem / Kp, i = rem - o * Kp;
    if (i >= I) {
      if (Wop) Wop[idx] = from_f32<op_t>(0.f);
      continue;
    }
    const op_t v = from_f32<op_t>(W[b * per + (int64_t)o * I + i]);
    if (Wop) Wop[idx] = v;
    Wt[b * per + (int64_t)i * O + o] = v;
  }
}

// sin / cos of fp32 radian arguments through the fp32 mode's functions (impl 0: Prec<F32>::sinp /
// cosp, i.e. the Cody-Waite + minimax sin_f32 / cos_f32) or OCML's sinf / cosf (impl 1): the
// accuracy probe behind siren_sincos_f32.
__global__ __launch_bounds__(256) void sincos_probe_kernel(const float* x, float* s, float* c, int64_t n, int impl) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = x[i];
    if (impl == 0) {
      s[i] = Prec<kPrecF32>::sinp(v);
      c[i] = Prec<kPrecF32>::cosp(v);
    } else {
      s[i] = sinf(v);
      c[i] = cosf(v);
    }
  }
}

}  // namespace siren
