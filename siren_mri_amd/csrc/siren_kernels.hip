// siren_kernels.hip — gfx950 (MI355X / CDNA4) kernels for the SIREN SineLayer stack.
//
// Reference semantics (jonbmartin/siren_mri):
//   BatchLinear.forward  modules.py:16-27   z = x @ W^T ; z += b   (W shared [out,in] or batched [B,out,in])
//   Sine.forward         modules.py:35-38   h = sin(w0 * z)
//   FCBlock              modules.py:45-97   [Linear+Sine] x (1+num_hidden_layers) + outermost Linear
//   autograd backward    training.py:91     dz = (dh * cos(w0 z)) * w0 ; dW = dz^T x ; db = sum dz ; dx = dz W
//
// Kernels (one launch each, all asynchronous on the caller's stream):
//   first_fwd   x[rows,C] -> P0[rows,F]           VALU (C is 2 for coords, 2m for Fourier features)
//   nt_gemm     MODE_FWD: P_l = enc(w0*(sin(P_{l-1}) W_l^T + b_l))      MFMA, bias+w0+phase epilogue
//               MODE_DX : dZ_{l-1} = (dZ_l W_l) * cos(P_{l-1}) * w0      MFMA, cos-weighted epilogue
//   tn_dw       dW_l partials = dZ_l^T sin(P_{l-1}), db_l partials        MFMA, split-K over rows
//   last_fwd    y = sin(P) W_L^T + b_L (out_features <= 8)               VALU + wave reduction
//   last_bwd    dZ = cos(P) w0 (dy W_L) ; dW_L, db_L partials              VALU
//   first_bwd   dW_0, db_0 partials ; dx = dZ_0 W_0                        VALU
//   reduce      sum of split-K partial slabs                               HBM streaming
#include "siren_common.h"

namespace siren {

// ------------------------------------------------------------------------------------------
// Argument blocks
// ------------------------------------------------------------------------------------------
struct NTArgs {
  const void* A;       // [rows, K] phase_t (FWD) or grad_t (DX)
  const void* Bt;      // [nb_w][N, K] op_t   (FWD: W_l ; DX: W_l^T)
  const float* bias;   // [nb_w][N] (FWD only)
  const void* Paux;    // [rows, N] phase_t (DX: P_{l-1})
  void* C;             // [rows, N] phase_t (FWD) or grad_t (DX)
  int64_t rows_per_batch;
  int64_t bt_bstride;    // elements between weight sets (0 = shared)
  int64_t bias_bstride;  // elements between bias sets (0 = shared)
  int K;
  int N;
  float w0;
};

struct TNArgs {
  const void* D;       // [rows, M] grad_t  (dZ_l)
  const void* P;       // [rows, N] phase_t (P_{l-1})
  float* part;         // [nsplit][batch][M*N + M]  (dW then db)
  int64_t rows_per_batch;
  int64_t rows_per_split;
  int M;
  int N;
  int batch;
};

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
};

struct LastBwdArgs {
  const void* P;       // [rows, F] phase_t
  const float* W;      // [nb_w][O, F]
  const float* b;      // [nb_w][O]
  const float* dy;     // [rows, O]
  void* dZ;            // [rows, F] grad_t
  float* part;         // [nsplit][batch][O*F + O]
  int64_t rows_per_batch;
  int64_t rows_per_split;
  int64_t w_bstride, b_bstride;
  int F, O, batch;
  int sine_out;
  float w0;
};

struct FirstBwdArgs {
  const void* dZ;      // [rows, F] grad_t
  const float* x;      // [rows, C]
  const float* W;      // [nb_w][F, C]
  float* dx;           // [rows, C] or null
  float* part;         // [nsplit][batch][F*C + F]
  int64_t rows_per_batch;
  int64_t rows_per_split;
  int64_t w_bstride;
  int F, C, batch;
};

// ------------------------------------------------------------------------------------------
// first_fwd: P0 = enc(w0 * (x W0^T + b0)). One thread per (row, 4 consecutive features).
// ------------------------------------------------------------------------------------------
template <int PREC>
__global__ __launch_bounds__(256) void first_fwd_kernel(FirstFwdArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  const int64_t batch = blockIdx.y;
  const int f4n = a.F >> 2;
  const float* W = a.W + batch * a.w_bstride;
  const float* b = a.b + batch * a.b_bstride;
  const int64_t total = a.rows_per_batch * f4n;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int64_t r = idx / f4n;
    const int f = (int)(idx - r * f4n) * 4;
    const int64_t row = batch * a.rows_per_batch + r;
    const float* xr = a.x + row * a.C;
    float z[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = 0.f;
    for (int c = 0; c < a.C; ++c) {
      const float xv = xr[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) z[e] = fmaf(xv, W[(f + e) * a.C + c], z[e]);
    }
    phase_t* out = (phase_t*)a.P + row * a.F + f;
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = PT::enc(a.w0 * (z[e] + b[f + e]));
  }
}

// ------------------------------------------------------------------------------------------
// nt_gemm: C[row][n] = sum_k A'[row][k] * Bt[n][k] with a fused prologue/epilogue.
// Tile 128 rows x 256 columns, 4 waves (2 x 2), each wave 64 x 128 = 2 x 4 MFMA 32x32 blocks.
// K is staged through LDS in chunks of 32 with a one-chunk register prefetch.
// ------------------------------------------------------------------------------------------
constexpr int MODE_FWD = 0;
constexpr int MODE_DX = 1;
constexpr int NT_BM = 128;
constexpr int NT_BN = 256;
constexpr int NT_KC = 32;

template <int PREC> struct NTLds;
template <> struct NTLds<kPrecBF16> {
  static constexpr int ROW = 40;  // bf16 elements per LDS row: 32 + 8 pad (80 B, conflict-free b128)
  static constexpr int BYTES = (NT_BM + NT_BN) * ROW * 2;
};
template <> struct NTLds<kPrecF32> {
  static constexpr int ROW = 33;  // f32 per LDS row: 32 + 1 pad (conflict-free b32 column reads)
  static constexpr int BYTES = (NT_BM + NT_BN) * ROW * 4;
};

template <int PREC, int MODE>
__global__ __launch_bounds__(256) void nt_gemm_kernel(NTArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  using op_t = typename PT::op_t;
  constexpr int ROW = NTLds<PREC>::ROW;
  __shared__ __attribute__((aligned(16))) char smem[NTLds<PREC>::BYTES];
  op_t* As = (op_t*)smem;
  op_t* Bs = As + NT_BM * ROW;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t batch = blockIdx.z;
  const int64_t m0 = (int64_t)blockIdx.x * NT_BM;  // row within batch
  const int n0 = blockIdx.y * NT_BN;
  const int64_t rowbase = batch * a.rows_per_batch;
  const op_t* Bt = (const op_t*)a.Bt + batch * a.bt_bstride;
  const int K = a.K;
  const int nk = K / NT_KC;

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  if constexpr (PREC == kPrecBF16) {
    // A chunk: 128 rows x 4 units of 8 elements -> 2 units per thread.
    // B chunk: 256 rows x 4 units -> 4 units per thread.
    using a_in_t = typename std::conditional<MODE == MODE_FWD, u16x8, bf16x8>::type;
    a_in_t areg[2];
    bf16x8 breg[4];
    auto load = [&](int kc) {
      const int k0 = kc * NT_KC;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int u = tid + 256 * i;
        const int r = u >> 2, kq = u & 3;
        const int64_t row = m0 + r;
        if (row < a.rows_per_batch) {
          const char* src = (const char*)a.A + ((rowbase + row) * K + k0 + kq * 8) * 2;
          areg[i] = *(const a_in_t*)src;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) areg[i][e] = 0;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = tid + 256 * i;
        const int r = u >> 2, kq = u & 3;
        const int n = n0 + r;
        if (n < a.N) {
          breg[i] = *(const bf16x8*)(Bt + (int64_t)n * K + k0 + kq * 8);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) breg[i][e] = (bf16)0.f;
        }
      }
    };
    auto store = [&]() {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int u = tid + 256 * i;
        const int r = u >> 2, kq = u & 3;
        bf16x8 v;
        if constexpr (MODE == MODE_FWD) {
          const bool valid = (m0 + r) < a.rows_per_batch;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (bf16)(valid ? PT::sinp(areg[i][e]) : 0.f);
        } else {
          v = areg[i];
        }
        *(bf16x8*)(As + r * ROW + kq * 8) = v;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = tid + 256 * i;
        const int r = u >> 2, kq = u & 3;
        *(bf16x8*)(Bs + r * ROW + kq * 8) = breg[i];
      }
    };
    const int r32 = lane & 31, h = lane >> 5;
    load(0);
    for (int kc = 0; kc < nk; ++kc) {
      __syncthreads();
      store();
      __syncthreads();
      if (kc + 1 < nk) load(kc + 1);
#pragma unroll
      for (int ks = 0; ks < NT_KC / 16; ++ks) {
        bf16x8 af[2], bfr[4];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
          af[bm] = *(const bf16x8*)(As + (64 * wm + 32 * bm + r32) * ROW + ks * 16 + h * 8);
#pragma unroll
        for (int bn = 0; bn < 4; ++bn)
          bfr[bn] = *(const bf16x8*)(Bs + (128 * wn + 32 * bn + r32) * ROW + ks * 16 + h * 8);
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int bn = 0; bn < 4; ++bn)
            acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
      }
    }
  } else {
    // fp32: A chunk 128 x 32 floats = 4 float4 per thread; B chunk 256 x 32 = 8 float4 per thread.
    f32x4 areg[4];
    f32x4 breg[8];
    auto load = [&](int kc) {
      const int k0 = kc * NT_KC;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = tid + 256 * i;
        const int r = u >> 3, kq = u & 7;
        const int64_t row = m0 + r;
        if (row < a.rows_per_batch) {
          areg[i] = *(const f32x4*)((const float*)a.A + (rowbase + row) * K + k0 + kq * 4);
        } else {
          areg[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int u = tid + 256 * i;
        const int r = u >> 3, kq = u & 7;
        const int n = n0 + r;
        if (n < a.N) {
          breg[i] = *(const f32x4*)(Bt + (int64_t)n * K + k0 + kq * 4);
        } else {
          breg[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    };
    auto store = [&]() {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int u = tid + 256 * i;
        const int r = u >> 3, kq = u & 7;
        const bool valid = (m0 + r) < a.rows_per_batch;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = areg[i][e];
          if constexpr (MODE == MODE_FWD) v = valid ? PT::sinp(v) : 0.f;
          As[r * ROW + kq * 4 + e] = v;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int u = tid + 256 * i;
        const int r = u >> 3, kq = u & 7;
#pragma unroll
        for (int e = 0; e < 4; ++e) Bs[r * ROW + kq * 4 + e] = breg[i][e];
      }
    };
    const int r32 = lane & 31, kk = lane >> 5;
    load(0);
    for (int kc = 0; kc < nk; ++kc) {
      __syncthreads();
      store();
      __syncthreads();
      if (kc + 1 < nk) load(kc + 1);
#pragma unroll 4
      for (int ks = 0; ks < NT_KC / 2; ++ks) {
        float af[2], bfr[4];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm) af[bm] = As[(64 * wm + 32 * bm + r32) * ROW + 2 * ks + kk];
#pragma unroll
        for (int bn = 0; bn < 4; ++bn) bfr[bn] = Bs[(128 * wn + 32 * bn + r32) * ROW + 2 * ks + kk];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int bn = 0; bn < 4; ++bn)
            acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
      }
    }
  }

  // Epilogue. C/D map of the 32x32 MFMAs: col = lane&31, row = (e&3) + 8*(e>>2) + 4*(lane>>5).
  const float* bias = (MODE == MODE_FWD) ? a.bias + batch * a.bias_bstride : nullptr;
#pragma unroll
  for (int bn = 0; bn < 4; ++bn) {
    const int col = n0 + 128 * wn + 32 * bn + (lane & 31);
    if (col >= a.N) continue;
    const float bcol = (MODE == MODE_FWD) ? bias[col] : 0.f;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t r = m0 + 64 * wm + 32 * bm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (r >= a.rows_per_batch) continue;
        const int64_t off = (rowbase + r) * a.N + col;
        if constexpr (MODE == MODE_FWD) {
          ((phase_t*)a.C)[off] = PT::enc(a.w0 * (acc[bm][bn][e] + bcol));
        } else {
          const float c = PT::cosp(((const phase_t*)a.Paux)[off]);
          ((grad_t*)a.C)[off] = from_f32<grad_t>((acc[bm][bn][e] * c) * a.w0);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// tn_dw: dW[i][j] partial = sum_{rows in split} D[row][i] * sin(P[row][j]); db[i] partial.
// Tile 128 x 128 (4 waves 2x2, each 64x64 = 2x2 MFMA blocks). Rows are the reduction (K) axis;
// each workgroup reduces its split of rows and writes one fp32 slab (no atomics).
// bf16: both operands are k-strided in the row-major tiles, so fragments are built with the
// gfx950 transposing LDS read ds_read_b64_tr_b16.
// ------------------------------------------------------------------------------------------
constexpr int TN_BM = 128;
constexpr int TN_BN = 128;

template <int PREC> struct TNLds;
template <> struct TNLds<kPrecBF16> {
  static constexpr int KC = 64;
  static constexpr int ROW = 160;  // bf16 per LDS row: 128 + 32 pad (320 B: conflict-free tr reads)
  static constexpr int BYTES = 2 * KC * ROW * 2;
};
template <> struct TNLds<kPrecF32> {
  static constexpr int KC = 32;
  static constexpr int ROW = 128;
  static constexpr int BYTES = 2 * KC * ROW * 4;
};

template <int PREC>
__global__ __launch_bounds__(256) void tn_dw_kernel(TNArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  using op_t = typename PT::op_t;
  constexpr int KC = TNLds<PREC>::KC;
  constexpr int ROW = TNLds<PREC>::ROW;
  __shared__ __attribute__((aligned(16))) char smem[TNLds<PREC>::BYTES];
  op_t* Ds = (op_t*)smem;
  op_t* Hs = Ds + KC * ROW;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (a.N + TN_BN - 1) / TN_BN;
  const int ti = blockIdx.x / tiles_n, tj = blockIdx.x % tiles_n;
  const int i0 = ti * TN_BM, j0 = tj * TN_BN;
  const int split = blockIdx.y;
  const int64_t batch = blockIdx.z;
  const int64_t rowbase = batch * a.rows_per_batch;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.rows_per_batch) r_end = a.rows_per_batch;
  const bool do_db = (tj == 0);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  constexpr int VEC = (PREC == kPrecBF16) ? 8 : 4;            // elements per 16-byte unit
  constexpr int UPR = 128 / VEC;                               // units per tile row
  constexpr int UPT = KC * UPR / 256;                          // units per thread (4 for both)
  float dbacc[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) dbacc[e] = 0.f;

  using d_in_t = typename std::conditional<PREC == kPrecBF16, bf16x8, f32x4>::type;
  using p_in_t = typename std::conditional<PREC == kPrecBF16, u16x8, f32x4>::type;
  d_in_t dreg[UPT];
  p_in_t preg[UPT];
  const int cu = tid % UPR;  // this thread's column unit (fixed across chunks)

  auto load = [&](int64_t rc) {
#pragma unroll
    for (int q = 0; q < UPT; ++q) {
      const int r = (tid + 256 * q) / UPR;
      const int64_t row = rc + r;
      const int ci = i0 + cu * VEC, cj = j0 + cu * VEC;
      if (row < r_end && ci < a.M) {
        dreg[q] = *(const d_in_t*)((const grad_t*)a.D + (rowbase + row) * a.M + ci);
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) dreg[q][e] = 0;
      }
      if (row < r_end && cj < a.N) {
        preg[q] = *(const p_in_t*)((const phase_t*)a.P + (rowbase + row) * a.N + cj);
      } else {
#pragma unroll
        for (int e = 0; e < VEC; ++e) preg[q][e] = 0;
      }
    }
  };
  auto store = [&](int64_t rc) {
#pragma unroll
    for (int q = 0; q < UPT; ++q) {
      const int r = (tid + 256 * q) / UPR;
      const bool valid = (rc + r) < r_end;
      d_in_t dv = dreg[q];
      *(d_in_t*)(Ds + r * ROW + cu * VEC) = dv;
#pragma unroll
      for (int e = 0; e < VEC; ++e) dbacc[e] += to_f32(dv[e]);
      d_in_t hv;
#pragma unroll
      for (int e = 0; e < VEC; ++e) hv[e] = from_f32<op_t>(valid ? PT::sinp(preg[q][e]) : 0.f);
      *(d_in_t*)(Hs + r * ROW + cu * VEC) = hv;
    }
  };

  if (r_begin < r_end) {
    load(r_begin);
    for (int64_t rc = r_begin; rc < r_end; rc += KC) {
      __syncthreads();
      store(rc);
      __syncthreads();
      if (rc + KC < r_end) load(rc + KC);
      if constexpr (PREC == kPrecBF16) {
        const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
#pragma unroll
        for (int ks = 0; ks < KC / 16; ++ks) {
          const int nb = 16 * ks + 8 * (g >> 1) + q;
          bf16x8 af[2], bfr[2];
#pragma unroll
          for (int bm = 0; bm < 2; ++bm) {
            const int c = 64 * wm + 32 * bm + 16 * (g & 1) + 4 * p;
            af[bm] = lds_read_tr16_pair(Ds + nb * ROW + c, Ds + (nb + 4) * ROW + c);
          }
#pragma unroll
          for (int bn = 0; bn < 2; ++bn) {
            const int c = 64 * wn + 32 * bn + 16 * (g & 1) + 4 * p;
            bfr[bn] = lds_read_tr16_pair(Hs + nb * ROW + c, Hs + (nb + 4) * ROW + c);
          }
#pragma unroll
          for (int bm = 0; bm < 2; ++bm)
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
              acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
        }
      } else {
        const int r32 = lane & 31, kk = lane >> 5;
#pragma unroll 4
        for (int ks = 0; ks < KC / 2; ++ks) {
          float af[2], bfr[2];
#pragma unroll
          for (int bm = 0; bm < 2; ++bm) af[bm] = Ds[(2 * ks + kk) * ROW + 64 * wm + 32 * bm + r32];
#pragma unroll
          for (int bn = 0; bn < 2; ++bn) bfr[bn] = Hs[(2 * ks + kk) * ROW + 64 * wn + 32 * bn + r32];
#pragma unroll
          for (int bm = 0; bm < 2; ++bm)
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
              acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
        }
      }
    }
  }

  // Partial slab write.
  float* part = a.part + ((int64_t)split * a.batch + batch) * ((int64_t)a.M * a.N + a.M);
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int col = j0 + 64 * wn + 32 * bn + (lane & 31);
    if (col >= a.N) continue;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = i0 + 64 * wm + 32 * bm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (row < a.M) part[(int64_t)row * a.N + col] = acc[bm][bn][e];
      }
  }
  if (do_db) {
    // Reduce the per-thread column sums over the threads sharing a column unit.
    __syncthreads();
    float* red = (float*)smem;  // [256 / UPR][128]
    const int slot = tid / UPR;
#pragma unroll
    for (int e = 0; e < VEC; ++e) red[slot * 128 + cu * VEC + e] = dbacc[e];
    __syncthreads();
    if (tid < 128) {
      float s = 0.f;
      for (int k = 0; k < 256 / UPR; ++k) s += red[k * 128 + tid];
      const int row = i0 + tid;
      if (row < a.M) part[(int64_t)a.M * a.N + row] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------
// last_fwd: y[row][o] = sum_f sin(P[row][f]) W[o][f] + b[o]   (optionally sin(w0*.)).
// One wave per row; each lane covers 4 consecutive features per 256-feature step.
// IT = ceil(F / 256), MAXO >= out_features (compile-time bounds keep the arrays in registers).
// ------------------------------------------------------------------------------------------
template <int PREC, int IT, int MAXO>
__global__ __launch_bounds__(256) void last_fwd_kernel(LastFwdArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  const int lane = threadIdx.x & 63;
  const int64_t batch = blockIdx.y;
  const float* W = a.W + batch * a.w_bstride;
  const float* b = a.b + batch * a.b_bstride;
  const int64_t wave_id = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t r = wave_id; r < a.rows_per_batch; r += nwaves) {
    const int64_t row = batch * a.rows_per_batch + r;
    const phase_t* pr = (const phase_t*)a.P + row * a.F;
    float acc[MAXO];
#pragma unroll
    for (int o = 0; o < MAXO; ++o) acc[o] = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int f = lane * 4 + 256 * it;
      if (f < a.F) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float hv = PT::sinp(pr[f + e]);
#pragma unroll
          for (int o = 0; o < MAXO; ++o)
            if (o < a.O) acc[o] = fmaf(hv, W[o * a.F + f + e], acc[o]);
        }
      }
    }
#pragma unroll
    for (int o = 0; o < MAXO; ++o) {
      if (o < a.O) {
        float z = wave_sum(acc[o]) + b[o];
        if (a.sine_out) z = sinf(a.w0 * z);
        if (lane == o) a.y[row * a.O + o] = z;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// last_bwd: g[row][o] = dy (or dy*cos(w0 z)*w0 when the last layer is a sine layer);
//           dZ[row][f] = (sum_o g[o] W[o][f]) * cos(P[row][f]) * w0;
//           partial dW[o][f] = sum_rows g[o] sin(P[row][f]); partial db[o] = sum_rows g[o].
// Grid (nsplit, batch); 4 waves stride over the split's rows; one slab write per workgroup.
// ------------------------------------------------------------------------------------------
template <int PREC, int IT, int MAXO>
__global__ __launch_bounds__(256) void last_bwd_kernel(LastBwdArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  __shared__ float red[4][MAXO * 256 + MAXO];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int split = blockIdx.x;
  const int64_t batch = blockIdx.y;
  const float* W = a.W + batch * a.w_bstride;
  const float* b = a.b + batch * a.b_bstride;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.rows_per_batch) r_end = a.rows_per_batch;
  float dw[IT][MAXO][4];
  float db[MAXO];
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int o = 0; o < MAXO; ++o)
#pragma unroll
      for (int e = 0; e < 4; ++e) dw[it][o][e] = 0.f;
#pragma unroll
  for (int o = 0; o < MAXO; ++o) db[o] = 0.f;

  for (int64_t r = r_begin + wave; r < r_end; r += 4) {
    const int64_t row = batch * a.rows_per_batch + r;
    const phase_t* pr = (const phase_t*)a.P + row * a.F;
    float g[MAXO];
#pragma unroll
    for (int o = 0; o < MAXO; ++o) g[o] = (o < a.O) ? a.dy[row * a.O + o] : 0.f;
    if (a.sine_out) {
      // Recompute z of the (sine) output layer to get cos(w0 z).
      float acc[MAXO];
#pragma unroll
      for (int o = 0; o < MAXO; ++o) acc[o] = 0.f;
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int f = lane * 4 + 256 * it;
        if (f < a.F) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float hv = PT::sinp(pr[f + e]);
#pragma unroll
            for (int o = 0; o < MAXO; ++o)
              if (o < a.O) acc[o] = fmaf(hv, W[o * a.F + f + e], acc[o]);
          }
        }
      }
#pragma unroll
      for (int o = 0; o < MAXO; ++o)
        if (o < a.O) g[o] = (g[o] * cosf(a.w0 * (wave_sum(acc[o]) + b[o]))) * a.w0;
    }
#pragma unroll
    for (int o = 0; o < MAXO; ++o) db[o] += g[o];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int f = lane * 4 + 256 * it;
      if (f < a.F) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const phase_t pv = pr[f + e];
          const float s = PT::sinp(pv), c = PT::cosp(pv);
          float dh = 0.f;
#pragma unroll
          for (int o = 0; o < MAXO; ++o) {
            if (o < a.O) {
              dh = fmaf(g[o], W[o * a.F + f + e], dh);
              dw[it][o][e] = fmaf(g[o], s, dw[it][o][e]);
            }
          }
          ((grad_t*)a.dZ)[row * a.F + f + e] = from_f32<grad_t>((dh * c) * a.w0);
        }
      }
    }
  }
  // Workgroup reduction of the 4 waves' partials, then one slab write (256 features at a time).
  float* part = a.part + ((int64_t)split * a.batch + batch) * (int64_t)(a.O * a.F + a.O);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
#pragma unroll
    for (int o = 0; o < MAXO; ++o)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wave][o * 256 + lane * 4 + e] = dw[it][o][e];
    if (it == 0 && lane == 0) {
#pragma unroll
      for (int o = 0; o < MAXO; ++o) red[wave][MAXO * 256 + o] = db[o];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < a.O * 256; idx += 256) {
      const int o = idx / 256, fl = idx % 256;
      const int f = 256 * it + fl;
      if (f < a.F) part[o * a.F + f] = red[0][idx] + red[1][idx] + red[2][idx] + red[3][idx];
    }
    if (it == 0 && (int)threadIdx.x < a.O) {
      const int k = MAXO * 256 + threadIdx.x;
      part[a.O * a.F + threadIdx.x] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// first_bwd: partial dW0[f][c] = sum_rows dZ[row][f] x[row][c]; partial db0[f] = sum dZ;
//            dx[row][c] = sum_f dZ[row][f] W0[f][c] (when dx != null).
// ------------------------------------------------------------------------------------------
template <int PREC, int IT, int MAXC>
__global__ __launch_bounds__(256) void first_bwd_kernel(FirstBwdArgs a) {
  using PT = Prec<PREC>;
  using grad_t = typename PT::grad_t;
  __shared__ float red[4][256 * (MAXC + 1)];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int split = blockIdx.x;
  const int64_t batch = blockIdx.y;
  const float* W = a.W + batch * a.w_bstride;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > a.rows_per_batch) r_end = a.rows_per_batch;
  float dw[IT][4][MAXC];
  float db[IT][4];
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      db[it][e] = 0.f;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) dw[it][e][c] = 0.f;
    }
  for (int64_t r = r_begin + wave; r < r_end; r += 4) {
    const int64_t row = batch * a.rows_per_batch + r;
    float xv[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) xv[c] = (c < a.C) ? a.x[row * a.C + c] : 0.f;
    float dxp[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) dxp[c] = 0.f;
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int f = lane * 4 + 256 * it;
      if (f < a.F) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float dz = to_f32(((const grad_t*)a.dZ)[row * a.F + f + e]);
          db[it][e] += dz;
#pragma unroll
          for (int c = 0; c < MAXC; ++c) {
            dw[it][e][c] = fmaf(dz, xv[c], dw[it][e][c]);
            if (c < a.C) dxp[c] = fmaf(dz, W[(f + e) * a.C + c], dxp[c]);
          }
        }
      }
    }
    if (a.dx) {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) {
        if (c < a.C) {
          const float s = wave_sum(dxp[c]);
          if (lane == 0) a.dx[row * a.C + c] = s;
        }
      }
    }
  }
  float* part = a.part + ((int64_t)split * a.batch + batch) * (int64_t)(a.F * a.C + a.F);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int fl = lane * 4 + e;
#pragma unroll
      for (int c = 0; c < MAXC; ++c) red[wave][fl * (MAXC + 1) + c] = dw[it][e][c];
      red[wave][fl * (MAXC + 1) + MAXC] = db[it][e];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < 256 * (MAXC + 1); idx += 256) {
      const int fl = idx / (MAXC + 1), c = idx % (MAXC + 1);
      const int f = 256 * it + fl;
      if (f >= a.F) continue;
      const float s = red[0][idx] + red[1][idx] + red[2][idx] + red[3][idx];
      if (c < a.C) part[f * a.C + c] = s;
      else if (c == MAXC) part[a.F * a.C + f] = s;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------
// reduce: out[b][e] = sum_s part[s][b][e]   (out may be split into two destinations: the first
// n_first elements of each batch slab go to out0[b*n_first + e], the rest to out1).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void reduce_kernel(const float* part, int nsplit, int64_t batch,
                                                     int64_t slab, int64_t n_first, float* out0,
                                                     float* out1) {
  const int64_t total = batch * slab;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    float s = 0.f;
    for (int k = 0; k < nsplit; ++k) s += part[(int64_t)k * total + idx];
    const int64_t b = idx / slab, e = idx - b * slab;
    if (e < n_first) out0[b * n_first + e] = s;
    else out1[b * (slab - n_first) + (e - n_first)] = s;
  }
}

// ------------------------------------------------------------------------------------------
// Weight preparation: W [nb][O][I] fp32 -> Wop [nb][O][I] op_t and WtOp [nb][I][O] op_t.
// ------------------------------------------------------------------------------------------
template <int PREC>
__global__ __launch_bounds__(256) void prep_weight_kernel(const float* W, void* Wop, void* WtOp,
                                                          int64_t nb, int O, int I) {
  using op_t = typename Prec<PREC>::op_t;
  const int64_t total = nb * (int64_t)O * I;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * 256) {
    const int64_t b = idx / ((int64_t)O * I);
    const int64_t rem = idx - b * (int64_t)O * I;
    const int o = (int)(rem / I), i = (int)(rem - (int64_t)o * I);
    const op_t v = from_f32<op_t>(W[idx]);
    if (Wop) ((op_t*)Wop)[idx] = v;
    ((op_t*)WtOp)[b * (int64_t)O * I + (int64_t)i * O + o] = v;
  }
}

}  // namespace siren
