// fp64 SIREN layer stack (SIREN_PREC_F64): the reference's double_precision=True training
// (training.py:56-58, with the model cast to float64) — forward and first-order backward of the
// [BatchLinear -> Sine] x L stack (modules.py:16-27, 35-38, 92-97) in IEEE double throughout.
//
// One LDS-tiled GEMM kernel in three operand layouts, its epilogue fused per use:
//   forward   Z = H W^T + b;  saved Z, next H = sin(w0 Z)  (or y = Z, the linear output layer)
//   dH        dH = dZ W, then dZ_prev = dH w0 cos(w0 Z_prev)  (or dx = dZ_0 W_0)
//   dW / db   [dW | db] = dZ^T [sin(w0 Z_prev) | 1]  over a row range: split-K partial slabs,
//             added in split order by f64_reduce_kernel (deterministic)
// MI355X's fp64 matrix rate equals its fp64 vector rate (78.6 TFLOP/s, MI355X_MICROARCH.md), so
// the tile runs on the VALU: 64 x 64 outputs per 256-thread workgroup, 4 x 4 per thread, K in
// 16-deep LDS stages. The fp64 path is the reference-arithmetic mode, not a speed path.
namespace siren {

struct F64Args {
  const double* A;     // TA 0: [M][lda] (row m, column k); TA 1: [K][lda] (row k, column m)
  const double* B;     // TB 0: [N][ldb] (row n, column k); TB 1: [K][ldb] (row k, column n)
  const double* bias;  // forward: [N]
  const double* Zp;    // dH: Z of the layer below ([M][N]); dW: B is Z_prev, transformed by sin(w0 .)
  double* C;           // output [M][ldc] (dW: partial slab [M][N + 1])
  double* Zs;          // forward: saved Z [M][N] (or null)
  int64_t M, N, K;
  int64_t lda, ldb, ldc;
  int64_t a_bs, b_bs, c_bs, zs_bs, bias_bs;  // per-weight-set strides (blockIdx.z)
  int64_t k_per_split;                       // dW: rows per split (blockIdx.z = split * nb + set)
  int nb;                                    // weight sets
  double w0;
};

enum { F64_FWD_SINE = 0, F64_FWD_LIN = 1, F64_DH = 2, F64_DX = 3, F64_DW = 4 };

template <int TA, int TB, int EPI>
__global__ __launch_bounds__(256) void f64_gemm_kernel(F64Args a) {
  constexpr int BM = 64, BN = 64, BK = 16;
  __shared__ double As[BK][BM + 1];
  __shared__ double Bs[BK][BN + 1];
  const int tid = threadIdx.x;
  const int tm = tid & 15, tn = tid >> 4;  // 4 x 4 outputs: rows tm + 16 i, columns tn + 16 j
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  int64_t set = blockIdx.z, k0 = 0, k1 = a.K;
  if constexpr (EPI == F64_DW) {
    set = blockIdx.z % a.nb;
    const int64_t split = blockIdx.z / a.nb;
    k0 = split * a.k_per_split;
    k1 = k0 + a.k_per_split < a.K ? k0 + a.k_per_split : a.K;
  }
  const double* A = a.A + set * a.a_bs;
  const double* B = a.B + set * a.b_bs;
  // dW: B's column N is the all-ones column (db)
  const int64_t NB = EPI == F64_DW ? a.N + 1 : a.N;

  double acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;

  for (int64_t kb = k0; kb < k1; kb += BK) {
    // 64 x 16 elements per operand, 4 per thread
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      int mm, kk;
      if (TA == 0) { kk = e & 15; mm = e >> 4; }   // k fastest: row-major A rows
      else { mm = e & 63; kk = e >> 6; }           // m fastest: A^T rows
      const int64_t m = m0 + mm, k = kb + kk;
      double v = 0.0;
      if (m < a.M && k < k1) v = TA == 0 ? A[m * a.lda + k] : A[k * a.lda + m];
      As[kk][mm] = v;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      int nn, kk;
      if (TB == 0) { kk = e & 15; nn = e >> 4; }
      else { nn = e & 63; kk = e >> 6; }
      const int64_t n = n0 + nn, k = kb + kk;
      double v = 0.0;
      if (k < k1 && n < NB) {
        if (EPI == F64_DW && n == a.N) v = 1.0;
        else {
          v = TB == 0 ? B[n * a.ldb + k] : B[k * a.ldb + n];
          if (EPI == F64_DW && a.Zp) v = sin(a.w0 * v);
        }
      }
      Bs[kk][nn] = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; ++kk) {
      double av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = As[kk][tm + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tn + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fma(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + tm + 16 * i;
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t n = n0 + tn + 16 * j;
      if (n >= NB) continue;
      double v = acc[i][j];
      if constexpr (EPI == F64_FWD_SINE || EPI == F64_FWD_LIN) {
        v += a.bias[set * a.bias_bs + n];
        if constexpr (EPI == F64_FWD_SINE) {
          if (a.Zs) a.Zs[set * a.zs_bs + m * a.N + n] = v;
          v = sin(a.w0 * v);
        }
        a.C[set * a.c_bs + m * a.ldc + n] = v;
      } else if constexpr (EPI == F64_DH) {
        const double z = a.Zp[set * a.zs_bs + m * a.N + n];
        a.C[set * a.c_bs + m * a.ldc + n] = v * (a.w0 * cos(a.w0 * z));
      } else if constexpr (EPI == F64_DX) {
        a.C[set * a.c_bs + m * a.ldc + n] = v;
      } else {
        a.C[(int64_t)blockIdx.z * a.c_bs + m * a.ldc + n] = v;
      }
    }
  }
}

// dZ of a sine output layer: dZ = dy w0 cos(w0 Z)
__global__ __launch_bounds__(256) void f64_top_kernel(const double* dy, const double* Z, double* dZ, int64_t n,
                                                      double w0) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dZ[i] = dy[i] * (w0 * cos(w0 * Z[i]));
}

// dW[set][M][N], db[set][M] = sum over splits s (in order) of part[s][set][M][N + 1]
__global__ __launch_bounds__(256) void f64_reduce_kernel(const double* part, double* dW, double* db, int64_t M,
                                                         int64_t N, int nb, int nsplit) {
  const int64_t slab = M * (N + 1);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= slab * nb) return;
  const int64_t set = i / slab, r = i % slab;
  double s = 0.0;
  for (int sp = 0; sp < nsplit; ++sp) s += part[((int64_t)sp * nb + set) * slab + r];
  const int64_t m = r / (N + 1), n = r % (N + 1);
  if (n < N) dW[set * M * N + m * N + n] = s;
  else db[set * M + m] = s;
}

}  // namespace siren
