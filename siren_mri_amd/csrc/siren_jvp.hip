// siren_jvp.hip — analytic spatial derivatives of a SIREN (diff_operators.gradient / laplace)
// and the adjoint of the gradient (the double backward of gradients_mse), for gfx950.
//
// Reference: diff_operators.py:27-43 computes them with autograd (create_graph=True), i.e. a
// recorded reverse pass plus a double-backward for loss_functions.gradients_mse (:330-335).
// Here they are forward-mode "tangent streams" carried next to the primal through every layer:
//
//   h = sin(p), p = w0 a, a_l = W_l h_{l-1} + b_l
//   u_l^k = W_l t_{l-1}^k        t_l^k = w0 cos(p_l) u_l^k      (u_0^k = W_0[:, k])
//   V_l   = W_l S_{l-1}          S_l   = w0 cos(p_l) V_l - w0^2 sin(p_l) sum_k (u_l^k)^2   (V_0 = 0)
//   gradient_k = sum_o (W_L t_{L-1}^k)_o          laplace = sum_o (W_L S_{L-1})_o
//
// Rows of every GEMM are STREAM-STACKED: for weight set b the operand is [S][N][K] (stream 0 the
// primal, 1..C the tangents, C+1 the Laplacian stream), so one MFMA GEMM per layer advances all
// streams with the same W_l; the prologue builds each stream's operand from the stored primal
// phase P and the stored pre-activation tangents U, the epilogue stores P (stream 0) or U.
//
// Backward of a loss on the gradient / the Laplacian (adjoints, stream-stacked
// D = [a_bar; u_bar^1..C (; V_bar)] with Q = sum_k (u^k)^2, c = cos(p), s = sin(p)):
//   u_bar^k = w0 c t_bar^k - 2 w0^2 s S_bar u^k          V_bar = w0 c S_bar
//   a_bar   = w0 (c h_bar - w0 s sum_k t_bar^k u^k - w0 S_bar (s V + w0 c Q))
//   W_bar_l = D^T [h_{l-1}; t_{l-1}^k; S_{l-1}] ; b_bar_l = sum a_bar ;
//   [h_bar; t_bar^k; S_bar]_{l-1} = D W_l
//   first layer: W_bar_0 = a_bar^T x + [sum_n u_bar^k as column k] ; x_bar = a_bar W_0 (V_0 = 0)
// (order 1 has no S stream: S_bar = 0; the Laplacian loss has no gradient stream at the top)
#include "siren_common.h"

namespace siren {

constexpr int JMODE_FWD = 0;  // stream-stacked forward (phase/tangent prologue, P/U epilogue)
constexpr int JMODE_BWD = 1;  // adjoint: A = D (grad_t), raw fp32 output

struct JNTArgs {
  const void* P;      // [B][N][K] phase_t (JFWD)
  const float* U;     // [B][S-1][N][K] fp32 (JFWD)
  const void* D;      // [B][S][N][K] grad_t (JBWD)
  const void* W;      // [nb_w][Nout][K] op_t
  const float* bias;  // [nb_w][Nout]
  void* Pout;         // [B][N][Nout] phase_t (JFWD)
  float* Uout;        // JFWD: [B][S-1][N][Nout]; JBWD: raw [B][S][N][Nout]
  int64_t N;          // rows per stream
  int64_t srow0;      // first stacked row processed (N: the primal stream is given, not computed)
  int S, C, lap;
  int64_t w_bstride, b_bstride;
  int K, Nout;
  float w0;
};

constexpr int JNT_BM = 128;
constexpr int JNT_BN = 256;
constexpr int JNT_KC = 32;

template <int PREC> struct JNTLds;
template <> struct JNTLds<kPrecBF16> {
  static constexpr int ROW = 40;
  static constexpr int BYTES = (JNT_BM + JNT_BN) * ROW * 2;
};
template <> struct JNTLds<kPrecF32> {
  static constexpr int ROW = 33;
  static constexpr int BYTES = (JNT_BM + JNT_BN) * ROW * 4;
};

// Operand element of stacked row (s, n), column k, from the stored layer-(l-1) quantities.
template <int PREC>
DEV void jvp_operand4(const JNTArgs& a, int64_t b, int s, int64_t n, int k, float (&out)[4]) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  const phase_t* P = (const phase_t*)a.P + (b * a.N + n) * a.K + k;
  const int64_t plane = a.N * (int64_t)a.K;  // one stream of U
  const float* Ub = a.U + b * (int64_t)(a.S - 1) * plane + n * a.K + k;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const phase_t p = P[e];
    if (s == 0) {
      out[e] = PT::sinp(p);
    } else if (s <= a.C) {
      out[e] = a.w0 * PT::cosp(p) * Ub[(int64_t)(s - 1) * plane + e];
    } else {
      float ss = 0.f;
      for (int j = 0; j < a.C; ++j) {
        const float u = Ub[(int64_t)j * plane + e];
        ss = fmaf(u, u, ss);
      }
      out[e] = a.w0 * PT::cosp(p) * Ub[(int64_t)a.C * plane + e] - a.w0 * a.w0 * PT::sinp(p) * ss;
    }
  }
}

// LAP: the operand has a Laplacian stream (order 2); the gradient / Jacobian forms omit its code.
template <int PREC, int MODE, bool LAP = false>
__global__ __launch_bounds__(256) void jvp_nt_kernel(JNTArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  using op_t = typename PT::op_t;
  constexpr int ROW = JNTLds<PREC>::ROW;
  constexpr bool BF = PREC == kPrecBF16;
  __shared__ __attribute__((aligned(16))) char smem[JNTLds<PREC>::BYTES];
  op_t* As = (op_t*)smem;
  op_t* Bs = As + JNT_BM * ROW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t b = blockIdx.z;
  const int64_t rows = (int64_t)a.S * a.N;  // stacked rows of this weight set
  const int64_t m0 = a.srow0 + (int64_t)blockIdx.x * JNT_BM;
  const int n0 = blockIdx.y * JNT_BN;
  const int K = a.K;
  const op_t* W = (const op_t*)a.W + b * a.w_bstride;

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // A chunk: 128 rows x 32 k = 1024 units of 4 -> 4 per thread. B chunk: 256 x 32 -> 8 units/thread.
  // The chunk's raw operands (phases, tangents / adjoints, weights) are fetched into registers
  // before the previous chunk's MFMAs and turned into operands (sin / cos / products) only when
  // staged, after those MFMAs: the loads' latency overlaps the MFMAs instead of stalling the wave
  // in front of them. A unit's stacked row (stream s, row n) is the same in every chunk.
  float areg[4][4];
  float breg[8][4];
  phase_t praw[4][4];
  float uraw[4][4];
  int sq[4];
  int64_t nq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t row = m0 + ((tid + 256 * q) >> 3);
    sq[q] = row < rows ? (int)(row / a.N) : -1;
    nq[q] = row < rows ? row - (int64_t)sq[q] * a.N : 0;
  }
  const int64_t plane = a.N * (int64_t)K;
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 256 * q;
      const int k = k0 + (u & 7) * 4;
      const int s = sq[q];
      const int64_t n = nq[q];
      if (s >= 0) {
        if constexpr (MODE == JMODE_FWD) {
          // four consecutive columns: one 16-byte (fp32) or 8-byte (16-bit phase) load each
          const phase_t* P = (const phase_t*)a.P + (b * a.N + n) * K + k;
          if constexpr (BF) {
            const u16x4 pv = *(const u16x4*)P;
#pragma unroll
            for (int e = 0; e < 4; ++e) praw[q][e] = pv[e];
          } else {
            const f32x4 pv = *(const f32x4*)P;
#pragma unroll
            for (int e = 0; e < 4; ++e) praw[q][e] = pv[e];
          }
          if (s >= 1 && s <= a.C) {
            const f32x4 uv = *(const f32x4*)(a.U + b * (int64_t)(a.S - 1) * plane + (int64_t)(s - 1) * plane + n * K + k);
#pragma unroll
            for (int e = 0; e < 4; ++e) uraw[q][e] = uv[e];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) uraw[q][e] = 0.f;
          }
        } else {
          const grad_t* D = (const grad_t*)a.D + (b * rows + m0 + (u >> 3)) * K + k;
          if constexpr (BF) {
            const bf16x4 dv = *(const bf16x4*)D;
#pragma unroll
            for (int e = 0; e < 4; ++e) areg[q][e] = (float)dv[e];
          } else {
            const f32x4 dv = *(const f32x4*)D;
#pragma unroll
            for (int e = 0; e < 4; ++e) areg[q][e] = dv[e];
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) areg[q][e] = 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int u = tid + 256 * q;
      const int c = u >> 3, k = k0 + (u & 7) * 4;
      const int col = n0 + c;
      if (col < a.Nout) {
        if constexpr (BF) {
          const bf16x4 wv = *(const bf16x4*)(W + (int64_t)col * K + k);
#pragma unroll
          for (int e = 0; e < 4; ++e) breg[q][e] = (float)wv[e];
        } else {
          const f32x4 wv = *(const f32x4*)((const float*)W + (int64_t)col * K + k);
#pragma unroll
          for (int e = 0; e < 4; ++e) breg[q][e] = wv[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) breg[q][e] = 0.f;
      }
    }
  };
  auto store = [&](int k0) {
    if constexpr (MODE == JMODE_FWD) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int s = sq[q];
        if (s < 0) continue;
        if (s == 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) areg[q][e] = PT::sinp(praw[q][e]);
        } else if (!LAP || s <= a.C) {
#pragma unroll
          for (int e = 0; e < 4; ++e) areg[q][e] = a.w0 * PT::cosp(praw[q][e]) * uraw[q][e];
        } else {
          if constexpr (LAP)  // the Laplacian stream (C + 1 tangent planes): from memory
            jvp_operand4<PREC>(a, b, s, nq[q], k0 + ((tid + 256 * q) & 7) * 4, areg[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 256 * q;
      const int r = u >> 3, kq = (u & 7) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) As[r * ROW + kq + e] = from_f32<op_t>(areg[q][e]);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int u = tid + 256 * q;
      const int c = u >> 3, kq = (u & 7) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[c * ROW + kq + e] = from_f32<op_t>(breg[q][e]);
    }
  };

  const int r32 = lane & 31, h = lane >> 5;
  const int nk = K / JNT_KC;
  load(0);
  for (int kc = 0; kc < nk; ++kc) {
    __syncthreads();
    store(kc * JNT_KC);
    __syncthreads();
    if (kc + 1 < nk) load((kc + 1) * JNT_KC);
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < JNT_KC / 16; ++ks) {
        bf16x8 af[2], bfr[4];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int e = 0; e < 8; ++e) af[bm][e] = As[(64 * wm + 32 * bm + r32) * ROW + ks * 16 + h * 8 + e];
#pragma unroll
        for (int bn = 0; bn < 4; ++bn)
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[bn][e] = Bs[(128 * wn + 32 * bn + r32) * ROW + ks * 16 + h * 8 + e];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int bn = 0; bn < 4; ++bn)
            acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
      }
    } else {
#pragma unroll 4
      for (int ks = 0; ks < JNT_KC / 2; ++ks) {
        float af[2], bfr[4];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm) af[bm] = As[(64 * wm + 32 * bm + r32) * ROW + 2 * ks + h];
#pragma unroll
        for (int bn = 0; bn < 4; ++bn) bfr[bn] = Bs[(128 * wn + 32 * bn + r32) * ROW + 2 * ks + h];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int bn = 0; bn < 4; ++bn)
            acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
      }
    }
  }

  const float* bias = a.bias ? a.bias + b * a.b_bstride : nullptr;
  // stacked row -> (stream, row) from one division for the block's first row (the epilogue's 128
  // rows per thread each paid a 64-bit division: a third of the kernel's instructions)
  const int64_t s_m0 = m0 / a.N, n_m0 = m0 - s_m0 * a.N;
  // this lane's 4 output columns (one per bn) and their biases
  const int colb = n0 + 128 * wn + (lane & 31);
  float bcol[4];
#pragma unroll
  for (int bn = 0; bn < 4; ++bn)
    bcol[bn] = (MODE == JMODE_FWD && s_m0 == 0 && colb + 32 * bn < a.Nout) ? bias[colb + 32 * bn] : 0.f;
  // row-major: each of the lane's 32 rows is resolved to (stream, row) and a base pointer once,
  // then its 4 columns are stored
#pragma unroll
  for (int bm = 0; bm < 2; ++bm)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int off = 64 * wm + 32 * bm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      const int64_t row = m0 + off;
      if (row >= rows) continue;
      if constexpr (MODE == JMODE_FWD) {
        int s = (int)s_m0;
        int64_t n = n_m0 + off;
        while (n >= a.N) {
          n -= a.N;
          ++s;
        }
        if (s == 0) {
          phase_t* dst = (phase_t*)a.Pout + (b * a.N + n) * a.Nout + colb;
#pragma unroll
          for (int bn = 0; bn < 4; ++bn) {
            // (a block that starts in stream s > 0 never holds stream-0 rows: bcol only when s_m0 == 0)
            if (colb + 32 * bn < a.Nout) dst[32 * bn] = PT::encz(acc[bm][bn][e], bcol[bn], a.w0);
          }
        } else {
          float* dst = a.Uout + ((b * (a.S - 1) + (s - 1)) * a.N + n) * a.Nout + colb;
#pragma unroll
          for (int bn = 0; bn < 4; ++bn)
            if (colb + 32 * bn < a.Nout) dst[32 * bn] = acc[bm][bn][e];
        }
      } else {
        float* dst = a.Uout + (b * rows + row) * a.Nout + colb;
#pragma unroll
        for (int bn = 0; bn < 4; ++bn)
          if (colb + 32 * bn < a.Nout) dst[32 * bn] = acc[bm][bn][e];
      }
    }
}

// ------------------------------------------------------------------------------------------
// Weight gradient over stream-stacked rows: dW[i][j] = sum_r D[r][i] X[r][j] (split-K over the
// S' * N stacked rows), X = [sin(P); w0 cos(P) U^k]; db[i] = sum over stream-0 rows of D.
struct JTNArgs {
  const void* D;      // [B][S'][N][M] grad_t
  const void* P;      // [B][N][Kin] phase_t (layer l-1)
  const float* U;     // [B][Su][N][Kin] fp32 tangents of layer l-1 (Su = stored U streams)
  float* part;        // split s, batch b slab at part + s*split_stride + b*(M*Kin + M)
  int64_t N;
  int64_t rows_per_split;
  int64_t split_stride;
  int S, Su, C;       // S' adjoint streams (1 + C, + 1 with the Laplacian stream)
  int M, Kin;
  float w0;
};

template <int PREC, bool LAP = false>
__global__ __launch_bounds__(256) void jvp_tn_kernel(JTNArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  using op_t = typename PT::op_t;
  constexpr int KC = 32;
  constexpr int ROWF = 128 + 1;  // fp32 staging row (padded)
  __shared__ float Ds[KC][ROWF];
  __shared__ float Xs[KC][ROWF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (a.Kin + 127) / 128;
  const int i0 = (blockIdx.x / tiles_n) * 128, j0 = (blockIdx.x % tiles_n) * 128;
  const int split = blockIdx.y;
  const int64_t b = blockIdx.z;
  const int64_t rows = (int64_t)a.S * a.N;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  const int64_t r_end = min(r_begin + a.rows_per_split, rows);
  const int64_t plane = a.N * (int64_t)a.Kin;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  float dbacc[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) dbacc[e] = 0.f;

  // Thread units: column c = tid & 127 of rows (tid >> 7) + 2 q, q < 16, of each 32-row chunk. The
  // chunk's raw values (D, the phase, the tangent) are fetched into registers before the previous
  // chunk's MFMAs and turned into X only when staged after them; a row's (stream, row) pair comes
  // from one division per chunk (rows of a chunk are consecutive).
  const int cu = tid & 127, ru = tid >> 7;
  float draw[16], uraw[16];
  phase_t praw[16];
  // (stream, row) of the chunk's row r from the chunk's first row (s0, n0): one scalar division
  // per chunk, outside the unrolled per-row loops
  auto row_sn = [&](int64_t s0, int64_t n0, int r, int& s, int64_t& n) {
    s = (int)s0;
    n = n0 + r;
    while (n >= a.N) {
      n -= a.N;
      ++s;
    }
  };
  auto fetch = [&](int64_t rc) {
    const int64_t s0 = rc / a.N, n0 = rc - s0 * a.N;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = ru + 2 * q;
      const int64_t row = rc + r;
      draw[q] = 0.f;
      uraw[q] = 0.f;
      praw[q] = phase_t(0);
      if (row < r_end) {
        int s;
        int64_t n;
        row_sn(s0, n0, r, s, n);
        if (i0 + cu < a.M) draw[q] = to_f32(((const grad_t*)a.D)[(b * rows + row) * a.M + i0 + cu]);
        if (j0 + cu < a.Kin) {
          praw[q] = ((const phase_t*)a.P)[(b * a.N + n) * a.Kin + j0 + cu];
          if (s >= 1 && s <= a.C) uraw[q] = a.U[b * a.Su * plane + (int64_t)(s - 1) * plane + n * a.Kin + j0 + cu];
        }
      }
    }
  };
  fetch(r_begin);
  for (int64_t rc = r_begin; rc < r_end; rc += KC) {
    __syncthreads();
    const int64_t s0 = rc / a.N, n0 = rc - s0 * a.N;
    // stage 32 rows x 128 columns of D and X (16 elements per thread each)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = ru + 2 * q;
      const int64_t row = rc + r;
      float dv = 0.f, xv = 0.f;
      if (row < r_end) {
        int s;
        int64_t n;
        row_sn(s0, n0, r, s, n);
        dv = draw[q];
        if (j0 + cu < a.Kin) {
          const phase_t p = praw[q];
          if (s == 0) {
            xv = PT::sinp(p);
          } else if (!LAP || s <= a.C) {
            xv = a.w0 * PT::cosp(p) * uraw[q];
          } else if constexpr (LAP) {  // Laplacian stream: S = w0 c V - w0^2 s Q (C + 1 planes from memory)
            const float* Ue = a.U + b * a.Su * plane + n * a.Kin + j0 + cu;
            float qq = 0.f;
            for (int j = 0; j < a.C; ++j) qq = fmaf(Ue[j * plane], Ue[j * plane], qq);
            xv = a.w0 * PT::cosp(p) * Ue[a.C * plane] - a.w0 * a.w0 * PT::sinp(p) * qq;
          }
        }
        if (s == 0) dbacc[q] += dv;
      }
      Ds[r][cu] = to_f32(from_f32<op_t>(dv));
      Xs[r][cu] = to_f32(from_f32<op_t>(xv));
    }
    __syncthreads();
    if (rc + KC < r_end) fetch(rc + KC);
    const int r32 = lane & 31, h = lane >> 5;
    if constexpr (PREC == kPrecBF16) {
#pragma unroll
      for (int ks = 0; ks < KC / 16; ++ks) {
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int e = 0; e < 8; ++e) af[bm][e] = (bf16)Ds[16 * ks + 8 * h + e][64 * wm + 32 * bm + r32];
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[bn][e] = (bf16)Xs[16 * ks + 8 * h + e][64 * wn + 32 * bn + r32];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
      }
    } else {
#pragma unroll 4
      for (int ks = 0; ks < KC / 2; ++ks) {
        float af[2], bfr[2];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm) af[bm] = Ds[2 * ks + h][64 * wm + 32 * bm + r32];
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) bfr[bn] = Xs[2 * ks + h][64 * wn + 32 * bn + r32];
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
      }
    }
  }
  float* part = a.part + (int64_t)split * a.split_stride + b * ((int64_t)a.M * a.Kin + a.M);
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int col = j0 + 64 * wn + 32 * bn + (lane & 31);
    if (col >= a.Kin) continue;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = i0 + 64 * wm + 32 * bm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        if (row < a.M) part[(int64_t)row * a.Kin + col] = acc[bm][bn][e];
      }
  }
  if (j0 == 0) {
    // every thread staged the same column (tid & 127) in all 16 of its units
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) s += dbacc[e];
    Ds[tid >> 7][tid & 127] = s;
    __syncthreads();
    if (tid < 128 && i0 + tid < a.M) part[(int64_t)a.M * a.Kin + i0 + tid] = Ds[0][tid] + Ds[1][tid];
  }
}

// ------------------------------------------------------------------------------------------
// jvp_tn_kernel for fp32 (exact-fp32 MFMA), restructured: a workgroup owns ALL M = 256 rows of
// dW and 128 of its columns, so each X element (a sin / cos of a stored phase times a tangent) is
// formed once per launch instead of once per 128-row tile of dW; 8 waves (wave (wm, wn): dW rows
// 64 wm .. + 63, columns 64 wn .. + 63 of the tile); LDS double-buffered, one barrier per 32-row
// chunk, and chunk k + 1's staging (global loads issued before chunk k's MFMAs, the X arithmetic
// and the LDS stores spread between them) overlapping chunk k's MFMAs. Same products and the same
// K order within a split as jvp_tn_kernel<kPrecF32>; half as many splits (a workgroup covers twice
// the dW tile), so the split-K sums round differently (fp32 rounding level).
constexpr int JTN2_KC = 32;
constexpr int JTN2_BN = 128;
constexpr int JTN2_DROW = 256 + 4;  // fp32 words per staged D row (16-byte aligned rows)
constexpr int JTN2_XROW = 128 + 4;

template <bool LAP>
__global__ __launch_bounds__(512) void jvp_tn2_kernel(JTNArgs a) {
  using PT = Prec<kPrecF32>;
  constexpr int KC = JTN2_KC;
  __shared__ __attribute__((aligned(16))) float Ds[2][KC * JTN2_DROW];
  __shared__ __attribute__((aligned(16))) float Xs[2][KC * JTN2_XROW];
  __shared__ float dbs[8][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int j0 = blockIdx.x * JTN2_BN;
  const int split = blockIdx.y;
  const int64_t b = blockIdx.z;
  const int64_t rows = (int64_t)a.S * a.N;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  const int64_t r_end = min(r_begin + a.rows_per_split, rows);
  const int64_t plane = a.N * (int64_t)a.Kin;
  const float* Dg = (const float*)a.D + b * rows * a.M;
  const float* Pg = (const float*)a.P + b * plane;
  const float* Ug = a.U + b * a.Su * plane;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  f32x4 dbacc = {0.f, 0.f, 0.f, 0.f};  // db of columns 4 (tid & 63) .. + 3 over this thread's stream-0 rows

  // staging units: D q < 4: row (tid >> 6) + 8 q, columns 4 (tid & 63) .. + 3 (M = 256);
  //                X q < 2: row (tid >> 5) + 16 q, columns j0 + 4 (tid & 31) .. + 3
  f32x4 dr[4], pr[2], ur[2];
  int xs_[2];
  int64_t xn_[2];
  const int dcol = 4 * (tid & 63), xcol = 4 * (tid & 31);
  auto fetch = [&](int64_t rc) {
    const int64_t s0 = rc / a.N, nn0 = rc - s0 * a.N;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t row = rc + (tid >> 6) + 8 * q;
      dr[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (row < r_end && dcol < a.M) dr[q] = *(const f32x4*)(Dg + row * a.M + dcol);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int r = (tid >> 5) + 16 * q;
      const int64_t row = rc + r;
      pr[q] = ur[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      xs_[q] = -1;
      if (row < r_end && j0 + xcol < a.Kin) {
        int s = (int)s0;
        int64_t n = nn0 + r;
        while (n >= a.N) {
          n -= a.N;
          ++s;
        }
        xs_[q] = s;
        xn_[q] = n;
        pr[q] = *(const f32x4*)(Pg + n * a.Kin + j0 + xcol);
        // (a Laplacian-stream row reads its C + 1 planes when it is staged)
        if (s >= 1 && s <= a.C) ur[q] = *(const f32x4*)(Ug + (int64_t)(s - 1) * plane + n * a.Kin + j0 + xcol);
      }
    }
  };
  auto stage_d = [&](int buf, int q, int64_t rc) {
    const int r = (tid >> 6) + 8 * q;
    *(f32x4*)(&Ds[buf][r * JTN2_DROW + dcol]) = dr[q];
    const int64_t row = rc + r;
    if (row < r_end && row < a.N) dbacc += dr[q];  // stream-0 rows are the first N stacked rows
  };
  auto stage_x = [&](int buf, int q) {
    const int r = (tid >> 5) + 16 * q;
    const int s = xs_[q];
    f32x4 xv = {0.f, 0.f, 0.f, 0.f};
    if (s == 0) {
#pragma unroll
      for (int e = 0; e < 4; ++e) xv[e] = PT::sinp(pr[q][e]);
    } else if (s >= 1 && (!LAP || s <= a.C)) {
#pragma unroll
      for (int e = 0; e < 4; ++e) xv[e] = a.w0 * PT::cosp(pr[q][e]) * ur[q][e];
    } else if constexpr (LAP) {
      if (s == a.C + 1) {
        const int64_t n = xn_[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float* Ue = Ug + n * a.Kin + j0 + xcol + e;
          float qq = 0.f;
          for (int j = 0; j < a.C; ++j) qq = fmaf(Ue[j * plane], Ue[j * plane], qq);
          const float p = pr[q][e];
          xv[e] = a.w0 * PT::cosp(p) * Ue[a.C * plane] - a.w0 * a.w0 * PT::sinp(p) * qq;
        }
      }
    }
    *(f32x4*)(&Xs[buf][r * JTN2_XROW + xcol]) = xv;
  };

  const int r32 = lane & 31, h = lane >> 5;
  int buf = 0;
  fetch(r_begin);
#pragma unroll
  for (int q = 0; q < 4; ++q) stage_d(0, q, r_begin);
#pragma unroll
  for (int q = 0; q < 2; ++q) stage_x(0, q);
  __syncthreads();
  for (int64_t rc = r_begin; rc < r_end; rc += KC) {
    const bool more = rc + KC < r_end;
    if (more) fetch(rc + KC);
    const float* D_ = Ds[buf];
    const float* X_ = Xs[buf];
    static_for<0, KC / 2>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      float af[2], bfr[2];
#pragma unroll
      for (int bm = 0; bm < 2; ++bm) af[bm] = D_[(2 * ks + h) * JTN2_DROW + 64 * wm + 32 * bm + r32];
#pragma unroll
      for (int bn = 0; bn < 2; ++bn) bfr[bn] = X_[(2 * ks + h) * JTN2_XROW + 64 * wn + 32 * bn + r32];
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
          acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[bm], bfr[bn], acc[bm][bn], 0, 0, 0);
      // the next chunk's staging, spread over the K steps (the other buffer: its last reads were
      // the previous chunk's MFMAs, before the barrier that ended it)
      if (more) {
        if constexpr (ks == 3 || ks == 5 || ks == 7 || ks == 9) stage_d(buf ^ 1, (ks - 3) / 2, rc + KC);
        if constexpr (ks == 11 || ks == 13) stage_x(buf ^ 1, (ks - 11) / 2);
      }
    });
    __syncthreads();
    buf ^= 1;
  }

  float* part = a.part + (int64_t)split * a.split_stride + b * ((int64_t)a.M * a.Kin + a.M);
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int col = j0 + 64 * wn + 32 * bn + r32;
    if (col >= a.Kin) continue;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 64 * wm + 32 * bm + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (row < a.M) part[(int64_t)row * a.Kin + col] = acc[bm][bn][e];
      }
  }
  if (j0 == 0) {
    // db: the 8 waves' column sums (wave w summed rows w + 8 q), added in wave order
    *(f32x4*)(&dbs[wave][dcol]) = dbacc;
    __syncthreads();
    if (tid < a.M) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) s += dbs[w][tid];
      part[(int64_t)a.M * a.Kin + tid] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------
// First layer: P0 = enc(w0 (x W0^T + b0)), U0[k] = W0[:, k] broadcast over rows, V0 = 0.
struct JFirstArgs {
  const float* x;     // [B][N][C]
  const float* W;     // [nb_w][F][C]
  const float* bias;  // [nb_w][F]
  void* P;            // [B][N][F], or null (the primal's phases are given)
  float* U;           // [B][Su][N][F]
  int64_t N;
  int C, F, Su;
  int64_t w_bstride, b_bstride;
  float w0;
};

template <int PREC>
__global__ __launch_bounds__(256) void jvp_first_kernel(JFirstArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  const int64_t b = blockIdx.y;
  const float* W = a.W + b * a.w_bstride;
  const float* bias = a.bias + b * a.b_bstride;
  const int64_t total = a.N * a.F;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t n = idx / a.F;
    const int f = (int)(idx - n * a.F);
    const float* xr = a.x + (b * a.N + n) * a.C;
    float z = 0.f;
    for (int c = 0; c < a.C; ++c) z = fmaf(xr[c], W[f * a.C + c], z);
    if (a.P) ((phase_t*)a.P)[(b * a.N + n) * a.F + f] = PT::encz(z, bias[f], a.w0);
    for (int s = 0; s < a.Su; ++s)
      a.U[((b * a.Su + s) * a.N + n) * a.F + f] = (s < a.C) ? W[f * a.C + s] : 0.f;
  }
}

// Output layer: grad[n][k] = sum_o sum_f W[o][f] t^k[f]; lap[n] = sum_o sum_f W[o][f] S[f].
// jac = 1 (the per-channel Jacobian, SIREN_JVP_JACOBIAN): grad[n][o][k] = sum_f W[o][f] t^k[f].
// One half-wave per row.
struct JLastArgs {
  const void* P;      // [B][N][F]
  const float* U;     // [B][Su][N][F]
  const float* W;     // [nb_w][O][F]
  float* grad;        // [B][N][C], or [B][N][O][C] when jac
  float* lap;         // [B][N] or null
  int64_t N;
  int C, F, O, Su, jac;
  int64_t w_bstride;
  float w0;
};

template <int PREC>
__global__ __launch_bounds__(256) void jvp_last_kernel(JLastArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  const int l32 = threadIdx.x & 31;
  const int64_t b = blockIdx.y;
  const float* W = a.W + b * a.w_bstride;
  const int64_t plane = a.N * (int64_t)a.F;
  if (a.jac) {
    // per output channel (O <= 8 passes over the row's tangents; not a hot path)
    for (int64_t n = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); n < a.N; n += (int64_t)gridDim.x * 8) {
      for (int o = 0; o < a.O; ++o) {
        float g[4] = {0.f, 0.f, 0.f, 0.f};
        for (int f = l32; f < a.F; f += 32) {
          const float wc = a.w0 * W[o * a.F + f] * PT::cosp(((const phase_t*)a.P)[(b * a.N + n) * a.F + f]);
          const float* Ub = a.U + b * (int64_t)a.Su * plane + n * a.F + f;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k < a.C) g[k] = fmaf(wc, Ub[(int64_t)k * plane], g[k]);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < a.C) {
            float v = g[k];
#pragma unroll
            for (int off = 16; off >= 1; off >>= 1) v += __shfl_xor(v, off, 32);
            if (l32 == 0) a.grad[((b * a.N + n) * a.O + o) * a.C + k] = v;
          }
        }
      }
    }
    return;
  }
  for (int64_t n = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); n < a.N; n += (int64_t)gridDim.x * 8) {
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    float lp = 0.f;
    for (int f = l32; f < a.F; f += 32) {
      float ws = 0.f;
      for (int o = 0; o < a.O; ++o) ws += W[o * a.F + f];
      const phase_t p = ((const phase_t*)a.P)[(b * a.N + n) * a.F + f];
      const float c = PT::cosp(p), s = PT::sinp(p);
      const float* Ub = a.U + b * (int64_t)a.Su * plane + n * a.F + f;
      float ss = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k < a.C) {
          const float u = Ub[(int64_t)k * plane];
          g[k] = fmaf(ws, a.w0 * c * u, g[k]);
          ss = fmaf(u, u, ss);
        }
      }
      if (a.lap) lp = fmaf(ws, a.w0 * c * Ub[(int64_t)a.C * plane] - a.w0 * a.w0 * s * ss, lp);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < a.C) {
        float v = g[k];
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) v += __shfl_xor(v, off, 32);
        if (l32 == 0) a.grad[(b * a.N + n) * a.C + k] = v;
      }
    }
    if (a.lap) {
#pragma unroll
      for (int off = 16; off >= 1; off >>= 1) lp += __shfl_xor(lp, off, 32);
      if (l32 == 0) a.lap[b * a.N + n] = lp;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Adjoint combine for a sine layer: from [h_bar; t_bar^k; S_bar] to D = [a_bar; u_bar^k; V_bar].
// top = 1: the output layer's adjoint, t_bar^k[f] = gbar[n][k] ws[f], S_bar[f] = lbar[n] ws[f]
//          (ws = sum_o W_L[o][f]), h_bar = 0, and also the output-layer weight-gradient
//          partials dW_L[o][f] = sum_n (sum_k gbar t^k[f] + lbar S[f]).
// top = 1 and jac = 1 (per-channel Jacobian adjoint): gbar is [B][N][O][C],
//          t_bar^k[f] = sum_o gbar[n][o][k] W_L[o][f], dW_L[o][f] = sum_n sum_k gbar[n][o][k] t^k[f].
// top = 0: raw = [h_bar; t_bar^1..C (; S_bar)] (fp32, [B][S'][N][F]) from the adjoint GEMM.
struct JCombArgs {
  const void* P;      // [B][N][F] phase_t of this layer
  const float* U;     // [B][Su][N][F] tangents of this layer
  const float* raw;   // top=0
  const float* gbar;  // top=1: [B][N][C] ([B][N][O][C] when jac) or null (Laplacian loss)
  const float* lbar;  // top=1: [B][N] (lap = 1)
  const float* WL;    // top=1: [nb_w][O][F]
  void* D;            // [B][S'][N][F] grad_t
  float* part;        // top=1: dW_L partial slabs (split s, batch b at s*split_stride + b*(O*F + O))
  int64_t N;
  int64_t rows_per_split;
  int64_t split_stride;
  int C, F, O, Su, S, top, lap, jac;
  int64_t w_bstride;
  float w0;
};

// The output layer's adjoint for the per-channel Jacobian (top = 1, jac = 1); same outputs as the
// top branch of jvp_combine_kernel (no Laplacian stream).
template <int PREC>
__global__ __launch_bounds__(256) void jvp_combine_jac_kernel(JCombArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  const int64_t b = blockIdx.y;
  const int S = a.S;
  const int64_t plane = a.N * (int64_t)a.F;
  const float* WL = a.WL + b * a.w_bstride;
  const float w0 = a.w0;
  grad_t* D = (grad_t*)a.D;
  const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_split;
  const int64_t r_end = min(r_begin + a.rows_per_split, a.N);
  for (int f = threadIdx.x; f < a.F; f += 256) {
    float wl[FUSED_MAXO], dwl[FUSED_MAXO];
#pragma unroll
    for (int o = 0; o < FUSED_MAXO; ++o) {
      wl[o] = o < a.O ? WL[o * a.F + f] : 0.f;
      dwl[o] = 0.f;
    }
    for (int64_t n = r_begin; n < r_end; ++n) {
      const phase_t p = ((const phase_t*)a.P)[(b * a.N + n) * a.F + f];
      const float c = PT::cosp(p), s = PT::sinp(p);
      const float* Ub = a.U + b * (int64_t)a.Su * plane + n * a.F + f;
      const float* gb = a.gbar + (b * a.N + n) * (int64_t)a.O * a.C;
      float cross = 0.f;
      for (int k = 0; k < a.C; ++k) {
        const float u = Ub[(int64_t)k * plane];
        float tbar = 0.f;
#pragma unroll
        for (int o = 0; o < FUSED_MAXO; ++o) {
          if (o < a.O) {
            const float gk = gb[o * a.C + k];
            tbar = fmaf(gk, wl[o], tbar);
            dwl[o] = fmaf(gk, w0 * c * u, dwl[o]);
          }
        }
        cross = fmaf(tbar, u, cross);
        D[((b * S + 1 + k) * a.N + n) * a.F + f] = from_f32<grad_t>(w0 * c * tbar);
      }
      D[(b * S * a.N + n) * a.F + f] = from_f32<grad_t>(w0 * (-w0 * s * cross));
    }
    float* part = a.part + (int64_t)blockIdx.x * a.split_stride + b * (int64_t)(a.O * a.F + a.O);
#pragma unroll
    for (int o = 0; o < FUSED_MAXO; ++o)
      if (o < a.O) part[o * a.F + f] = dwl[o];
    if (f < a.O) part[a.O * a.F + f] = 0.f;
  }
}

template <int PREC>
__global__ __launch_bounds__(256) void jvp_combine_kernel(JCombArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  const int64_t b = blockIdx.y;
  const int S = a.S;
  const int64_t plane = a.N * (int64_t)a.F;
  const float* WL = a.top ? a.WL + b * a.w_bstride : nullptr;
  const float w0 = a.w0, w02 = a.w0 * a.w0;
  grad_t* D = (grad_t*)a.D;
  // thread owns feature column f = threadIdx.x (+256 k) for rows of its split
  const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_split;
  const int64_t r_end = min(r_begin + a.rows_per_split, a.N);
  for (int f = threadIdx.x; f < a.F; f += 256) {
    float ws = 0.f;
    if (a.top)
      for (int o = 0; o < a.O; ++o) ws += WL[o * a.F + f];
    float dwl = 0.f;
    // four rows at a time: every load of the four first (in flight together), then the arithmetic
    // and the stores — the stores would otherwise order each row's loads behind the previous row's
    constexpr int RR = 4, MC = 4;  // rows per group; tangent streams (jvp_check: in_features <= 4)
    for (int64_t n0 = r_begin; n0 < r_end; n0 += RR) {
      phase_t pv[RR];
      float uv[RR][MC + 1], rv[RR][MC + 2], gv[RR][MC], lv[RR];
#pragma unroll
      for (int j = 0; j < RR; ++j) {
        const int64_t n = n0 + j < r_end ? n0 + j : r_end - 1;
        pv[j] = ((const phase_t*)a.P)[(b * a.N + n) * a.F + f];
        const float* Ub = a.U + b * (int64_t)a.Su * plane + n * a.F + f;
#pragma unroll
        for (int k = 0; k < MC + 1; ++k) uv[j][k] = k < a.Su ? Ub[(int64_t)k * plane] : 0.f;
        if (a.top) {
#pragma unroll
          for (int k = 0; k < MC; ++k) gv[j][k] = (a.gbar && k < a.C) ? a.gbar[(b * a.N + n) * a.C + k] : 0.f;
          lv[j] = a.lap ? a.lbar[b * a.N + n] : 0.f;
        } else {
          const float* rw = a.raw + (b * S * a.N + n) * a.F + f;  // stream j: rw[j * plane]
#pragma unroll
          for (int k = 0; k < MC + 2; ++k) rv[j][k] = k < S ? rw[(int64_t)k * plane] : 0.f;
        }
      }
#pragma unroll
      for (int j = 0; j < RR; ++j) {
        const int64_t n = n0 + j;
        if (n >= r_end) break;
        const float c = PT::cosp(pv[j]), s = PT::sinp(pv[j]);
        const float hbar = a.top ? 0.f : rv[j][0];
        float sbar = 0.f;
        if (a.lap) sbar = a.top ? lv[j] * ws : rv[j][1 + a.C];
        float cross = 0.f, q = 0.f;
#pragma unroll
        for (int k = 0; k < MC; ++k) {
          if (k >= a.C) break;
          const float u = uv[j][k];
          float tbar = 0.f;
          if (a.top) {
            if (a.gbar) {
              const float gk = gv[j][k];
              tbar = gk * ws;
              dwl = fmaf(gk, w0 * c * u, dwl);
            }
          } else {
            tbar = rv[j][1 + k];
          }
          cross = fmaf(tbar, u, cross);
          q = fmaf(u, u, q);
          D[((b * S + 1 + k) * a.N + n) * a.F + f] = from_f32<grad_t>(w0 * c * tbar - 2.f * w02 * s * sbar * u);
        }
        float abar = c * hbar - w0 * s * cross;
        if (a.lap) {
          const float v = uv[j][a.C];
          abar -= w0 * sbar * (s * v + w0 * c * q);
          D[((b * S + 1 + a.C) * a.N + n) * a.F + f] = from_f32<grad_t>(w0 * c * sbar);
          if (a.top) dwl = fmaf(lv[j], w0 * c * v - w02 * s * q, dwl);
        }
        D[(b * S * a.N + n) * a.F + f] = from_f32<grad_t>(w0 * abar);
      }
    }
    if (a.top) {
      float* part = a.part + (int64_t)blockIdx.x * a.split_stride + b * (int64_t)(a.O * a.F + a.O);
      for (int o = 0; o < a.O; ++o) part[o * a.F + f] = dwl;
      if (f < a.O) part[a.O * a.F + f] = 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------------
// The adjoint GEMM of a hidden layer WITH the combine in its epilogue (replaces jvp_nt_kernel
// <JMODE_BWD> + jvp_combine_kernel<top = 0>): raw[s] = D[s] W_l for all S adjoint streams of the
// same 64 rows in one workgroup, so a lane holds h_bar, t_bar^1..C (and S_bar) of the same
// (row, feature) in its accumulators and forms the layer below's adjoints [a_bar; u_bar^k; V_bar]
// in registers (the formulas of jvp_combine_kernel on the same fp32 accumulator values; the
// compiler's FMA contraction may differ by an ulp). The fp32 raw tensor never goes to HBM: per layer
// 2 x S x 4 B per (row, feature) less traffic and one launch less.
//
// Tile: 64 rows x S streams (A) x 256 output features (B, all of them: each D row is read once),
// 8 waves: wave (wm, wn) owns rows 32 wm .. 32 wm + 31 of EVERY stream and features 64 wn .. + 63.
// K chunks of 32, operands staged through LDS (fp32 rows padded to 33 words / bf16 to 40), the next
// chunk's raw values in registers during this chunk's MFMAs.
struct JAdjArgs {
  const void* D;      // [B][S][N][K] grad_t: adjoints of layer l (K = its width)
  const void* W;      // [nb_w][Nout][K] op_t: W_l^T (prepared for the adjoint)
  const void* P;      // [B][N][Nout] phase_t of layer l - 1
  const float* U;     // [B][Su][N][Nout] tangents of layer l - 1
  void* Dout;         // [B][S][N][Nout] grad_t: adjoints of layer l - 1
  int64_t N;
  int Su;
  int64_t w_bstride;
  int K, Nout;
  float w0;
};

constexpr int JADJ_ROWS = 64;
constexpr int JADJ_BN = 256;

template <int PREC, int S, bool LAP>
__global__ __launch_bounds__(512) void jvp_adj_kernel(JAdjArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using grad_t = typename PT::grad_t;
  using op_t = typename PT::op_t;
  constexpr bool BF = PREC == kPrecBF16;
  constexpr int C = LAP ? S - 2 : S - 1;
  static_assert(C >= 1, "at least one tangent stream");
  constexpr int ROW = JNTLds<PREC>::ROW;
  constexpr int AROWS = S * JADJ_ROWS;
  __shared__ __attribute__((aligned(16))) op_t As[AROWS * ROW];
  __shared__ __attribute__((aligned(16))) op_t Bs[JADJ_BN * ROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int64_t b = blockIdx.y;
  const int64_t N = a.N;
  const int64_t n0 = (int64_t)blockIdx.x * JADJ_ROWS;
  const int K = a.K;
  const op_t* W = (const op_t*)a.W + b * a.w_bstride;
  const grad_t* Dg = (const grad_t*)a.D + b * (int64_t)S * N * K;

  f32x16 acc[S][2];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[s][j][e] = 0.f;

  // A chunk: S x 64 rows x 32 k in units of 4 -> S * 512 / 512 = S units per thread (unit u: row
  // u >> 3 = stream (u >> 9) and row (u >> 3) & 63, k 4 (u & 7)); B chunk: 256 x 32 -> 4 units.
  constexpr int AU = S;
  float areg[AU][4];
  float breg[4][4];
  auto load = [&](int k0) {
#pragma unroll
    for (int q = 0; q < AU; ++q) {
      const int u = tid + 512 * q;
      const int s = u >> 9, r = (u >> 3) & 63, k = k0 + (u & 7) * 4;
      const int64_t n = n0 + r;
      if (n < N) {
        const grad_t* src = Dg + ((int64_t)s * N + n) * K + k;
        if constexpr (BF) {
          const bf16x4 v = *(const bf16x4*)src;
#pragma unroll
          for (int e = 0; e < 4; ++e) areg[q][e] = (float)v[e];
        } else {
          const f32x4 v = *(const f32x4*)src;
#pragma unroll
          for (int e = 0; e < 4; ++e) areg[q][e] = v[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) areg[q][e] = 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int c = u >> 3, k = k0 + (u & 7) * 4;
      if (c < a.Nout) {
        if constexpr (BF) {
          const bf16x4 v = *(const bf16x4*)(W + (int64_t)c * K + k);
#pragma unroll
          for (int e = 0; e < 4; ++e) breg[q][e] = (float)v[e];
        } else {
          const f32x4 v = *(const f32x4*)((const float*)W + (int64_t)c * K + k);
#pragma unroll
          for (int e = 0; e < 4; ++e) breg[q][e] = v[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) breg[q][e] = 0.f;
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int q = 0; q < AU; ++q) {
      const int u = tid + 512 * q;
      const int r = u >> 3, kq = (u & 7) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) As[r * ROW + kq + e] = from_f32<op_t>(areg[q][e]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int c = u >> 3, kq = (u & 7) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[c * ROW + kq + e] = from_f32<op_t>(breg[q][e]);
    }
  };

  const int r32 = lane & 31, h = lane >> 5;
  const int nk = K / JNT_KC;
  load(0);
  for (int kc = 0; kc < nk; ++kc) {
    __syncthreads();
    store();
    __syncthreads();
    if (kc + 1 < nk) load((kc + 1) * JNT_KC);
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < JNT_KC / 16; ++ks) {
        bf16x8 af[S], bfr[2];
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int e = 0; e < 8; ++e) af[s][e] = As[(s * JADJ_ROWS + 32 * wm + r32) * ROW + ks * 16 + h * 8 + e];
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[bn][e] = Bs[(64 * wn + 32 * bn + r32) * ROW + ks * 16 + h * 8 + e];
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            acc[s][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bfr[bn], acc[s][bn], 0, 0, 0);
      }
    } else {
#pragma unroll 4
      for (int ks = 0; ks < JNT_KC / 2; ++ks) {
        float af[S], bfr[2];
#pragma unroll
        for (int s = 0; s < S; ++s) af[s] = As[(s * JADJ_ROWS + 32 * wm + r32) * ROW + 2 * ks + h];
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) bfr[bn] = Bs[(64 * wn + 32 * bn + r32) * ROW + 2 * ks + h];
#pragma unroll
        for (int s = 0; s < S; ++s)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            acc[s][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bfr[bn], acc[s][bn], 0, 0, 0);
      }
    }
  }

  // ---- the combine (jvp_combine_kernel, top = 0) on the accumulators ----
  // Per 32-column block: the block's 16 phases and C (+1) tangents of every row this lane holds are
  // loaded first (all in flight together: one memory latency per block, not one per element — the
  // stores in between would otherwise order every load behind the previous element's stores),
  // then combined and stored.
  const int F = a.Nout;
  const int64_t plane = N * (int64_t)F;
  const float w0 = a.w0, w02 = a.w0 * a.w0;
  grad_t* Do = (grad_t*)a.Dout + b * (int64_t)S * plane;
  const phase_t* Pb = (const phase_t*)a.P + b * plane;
  const float* Ub = a.U + b * (int64_t)a.Su * plane;
  constexpr int NU = LAP ? C + 1 : C;
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int f = 64 * wn + 32 * bn + r32;
    if (f >= F) continue;
    phase_t pv[16];
    float uv[NU][16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t n = n0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
      const int64_t idx = (n < N ? n : N - 1) * F + f;
      pv[e] = Pb[idx];
#pragma unroll
      for (int k = 0; k < NU; ++k) uv[k][e] = Ub[(int64_t)k * plane + idx];
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t n = n0 + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
      if (n >= N) continue;
      const int64_t idx = n * F + f;
      const float c = PT::cosp(pv[e]), sn = PT::sinp(pv[e]);
      const float hbar = acc[0][bn][e];
      const float sbar = LAP ? acc[1 + C][bn][e] : 0.f;
      float cross = 0.f, q = 0.f;
#pragma unroll
      for (int k = 0; k < C; ++k) {
        const float u = uv[k][e];
        const float tbar = acc[1 + k][bn][e];
        cross = fmaf(tbar, u, cross);
        q = fmaf(u, u, q);
        Do[(int64_t)(1 + k) * plane + idx] = from_f32<grad_t>(w0 * c * tbar - 2.f * w02 * sn * sbar * u);
      }
      float abar = c * hbar - w0 * sn * cross;
      if constexpr (LAP) {
        const float v = uv[C][e];
        abar -= w0 * sbar * (sn * v + w0 * c * q);
        Do[(int64_t)(1 + C) * plane + idx] = from_f32<grad_t>(w0 * c * sbar);
      }
      Do[idx] = from_f32<grad_t>(w0 * abar);
    }
  }
}

// ------------------------------------------------------------------------------------------
// The tangent streams of a hidden layer, STACKED BY ROW (replaces jvp_nt_kernel<JMODE_FWD> when the
// primal stream is given and there is no Laplacian stream): U_l^k = (w0 cos(P_{l-1}) U_{l-1}^k) W_l^T
// for all C tangent streams of the same 64 rows in one workgroup, so each operand element's
// phase is loaded and its cosine formed ONCE for the C streams (jvp_nt_kernel's stacked rows hold
// the streams of a row in different tiles: C loads and C cosines per element) — the layout of
// jvp_adj_kernel: 8 waves, wave (wm, wn) owns rows 32 wm .. + 31 of EVERY stream and features
// 64 wn .. + 63; K chunks of 32 staged through LDS (fp32 rows padded to 33 words / bf16 to 40),
// the next chunk's raw phases, tangents and weights in registers during this chunk's MFMAs.
// Same products as jvp_nt_kernel (w0 * cos(p) * u, rounded to the operand type) and the same K
// order, so the tangents are bit-identical to the stacked-row kernel's.
struct JTanArgs {
  const void* P;   // [B][N][K] phase_t of layer l - 1 (RB_DX: the phases of layer l - 1 are the
                   // epilogue's [B][N][Nout])
  const float* U;  // JT_TAN: [B][Su][N][K] tangents of layer l - 1 (streams 0..C-1 used);
                   // JT_DX: [B][N][K] the incoming gradient dZ_l
  const void* W;   // [nb_w][Nout][K] op_t: W_l (JT_DX: W_l^T)
  const float* bias;  // JT_FWD: [nb_w][Nout] b_l
  float* Uout;     // JT_TAN: [B][Su][N][Nout] tangents of layer l; JT_FWD: phases P_l [B][N][Nout];
                   // JT_DX: dZ_{l-1} [B][N][Nout]
  int64_t N;
  int Su;
  int64_t w_bstride, b_bstride;
  int K, Nout;
  float w0;
};

// Modes of jvp_tan_kernel. JT_TAN: C tangent streams of the same 64 rows (above). The same tile
// serves the fp32 stack's plain hidden layers with the C "streams" taken as C consecutive 64-row
// blocks of one plane (nt_f32_kernel's products, K order and epilogues):
//   JT_FWD: P_l = w0 (sin(P_{l-1}) W_l^T + b_l)                     (modules.py:25-26,38)
//   JT_DX : dZ_{l-1} = (dZ_l W_l) cos(P_{l-1}) w0                    (the Sine's backward)
constexpr int JT_TAN = 0, JT_FWD = 1, JT_DX = 2;

template <int PREC, int C, int MODE = JT_TAN>
__global__ __launch_bounds__(512) void jvp_tan_kernel(JTanArgs a) {
  using PT = Prec<PREC>;
  using phase_t = typename PT::phase_t;
  using op_t = typename PT::op_t;
  constexpr bool BF = PREC == kPrecBF16;
  constexpr bool STREAMS = MODE == JT_TAN;  // C planes of the same rows, or C row blocks of one plane
  constexpr int ROW = JNTLds<PREC>::ROW;
  __shared__ __attribute__((aligned(16))) op_t As[C * JADJ_ROWS * ROW];
  __shared__ __attribute__((aligned(16))) op_t Bs[JADJ_BN * ROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int64_t b = blockIdx.y;
  const int64_t N = a.N;
  const int64_t n0 = (int64_t)blockIdx.x * JADJ_ROWS * (STREAMS ? 1 : C);
  const int K = a.K;
  const int64_t plane = N * (int64_t)K;
  const op_t* W = (const op_t*)a.W + b * a.w_bstride;
  const phase_t* Pg = (const phase_t*)a.P + b * plane;
  const float* Ug = a.U + b * (int64_t)(MODE == JT_TAN ? a.Su : 1) * plane;

  f32x16 acc[C][2];
#pragma unroll
  for (int s = 0; s < C; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[s][j][e] = 0.f;

  // A chunk: 64 rows x 32 k in units of 4 -> one unit per thread (row tid >> 3, k 4 (tid & 7)) in
  // each of the C streams / row blocks; B chunk: 256 x 32 -> 4 units per thread.
  const int ar = tid >> 3, akq = (tid & 7) * 4;
  auto arow = [&](int s) -> int64_t { return n0 + (STREAMS ? 0 : JADJ_ROWS * s) + ar; };
  phase_t praw[STREAMS ? 1 : C][4];
  float uraw[C][4];
  float breg[4][4];
  auto load = [&](int k0) {
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int64_t an = arow(s);
      const bool ok = an < N;
      const int64_t idx = an * K + k0 + akq;
      if constexpr (MODE == JT_DX) {
        const f32x4 v = ok ? *(const f32x4*)(Ug + idx) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) uraw[s][e] = v[e];
      } else {
        if (MODE == JT_FWD || s == 0) {
          if constexpr (BF) {
            const u16x4 pv = ok ? *(const u16x4*)(Pg + idx) : u16x4{0, 0, 0, 0};
#pragma unroll
            for (int e = 0; e < 4; ++e) praw[STREAMS ? 0 : s][e] = pv[e];
          } else {
            const f32x4 pv = ok ? *(const f32x4*)(Pg + idx) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e) praw[STREAMS ? 0 : s][e] = pv[e];
          }
        }
        if constexpr (MODE == JT_TAN) {
          const f32x4 uv = ok ? *(const f32x4*)(Ug + (int64_t)s * plane + idx) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int e = 0; e < 4; ++e) uraw[s][e] = uv[e];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int c = u >> 3, k = k0 + (u & 7) * 4;
      if (c < a.Nout) {
        if constexpr (BF) {
          const bf16x4 v = *(const bf16x4*)(W + (int64_t)c * K + k);
#pragma unroll
          for (int e = 0; e < 4; ++e) breg[q][e] = (float)v[e];
        } else {
          const f32x4 v = *(const f32x4*)((const float*)W + (int64_t)c * K + k);
#pragma unroll
          for (int e = 0; e < 4; ++e) breg[q][e] = v[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) breg[q][e] = 0.f;
      }
    }
  };
  auto store = [&]() {
    if constexpr (MODE == JT_TAN) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float wc = a.w0 * PT::cosp(praw[0][e]);  // one cosine for the C streams
#pragma unroll
        for (int s = 0; s < C; ++s) As[(s * JADJ_ROWS + ar) * ROW + akq + e] = from_f32<op_t>(wc * uraw[s][e]);
      }
    } else {
#pragma unroll
      for (int s = 0; s < C; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          As[(s * JADJ_ROWS + ar) * ROW + akq + e] =
              from_f32<op_t>(MODE == JT_FWD ? PT::sinp(praw[STREAMS ? 0 : s][e]) : uraw[s][e]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int c = u >> 3, kq = (u & 7) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[c * ROW + kq + e] = from_f32<op_t>(breg[q][e]);
    }
  };

  const int r32 = lane & 31, h = lane >> 5;
  const int nk = K / JNT_KC;
  load(0);
  for (int kc = 0; kc < nk; ++kc) {
    __syncthreads();
    store();
    __syncthreads();
    if (kc + 1 < nk) load((kc + 1) * JNT_KC);
    if constexpr (BF) {
#pragma unroll
      for (int ks = 0; ks < JNT_KC / 16; ++ks) {
        bf16x8 af[C], bfr[2];
#pragma unroll
        for (int s = 0; s < C; ++s)
#pragma unroll
          for (int e = 0; e < 8; ++e) af[s][e] = As[(s * JADJ_ROWS + 32 * wm + r32) * ROW + ks * 16 + h * 8 + e];
#pragma unroll
        for (int bn = 0; bn < 2; ++bn)
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[bn][e] = Bs[(64 * wn + 32 * bn + r32) * ROW + ks * 16 + h * 8 + e];
#pragma unroll
        for (int s = 0; s < C; ++s)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            acc[s][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bfr[bn], acc[s][bn], 0, 0, 0);
      }
    } else {
#pragma unroll 4
      for (int ks = 0; ks < JNT_KC / 2; ++ks) {
        float af[C], bfr[2];
#pragma unroll
        for (int s = 0; s < C; ++s) af[s] = As[(s * JADJ_ROWS + 32 * wm + r32) * ROW + 2 * ks + h];
#pragma unroll
        for (int bn = 0; bn < 2; ++bn) bfr[bn] = Bs[(64 * wn + 32 * bn + r32) * ROW + 2 * ks + h];
#pragma unroll
        for (int s = 0; s < C; ++s)
#pragma unroll
          for (int bn = 0; bn < 2; ++bn)
            acc[s][bn] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[s], bfr[bn], acc[s][bn], 0, 0, 0);
      }
    }
  }

  // Epilogue. A lane's 16 elements of a tile are 16 rows of one column, the 32 lanes of a
  // half-wave 32 consecutive columns (128-byte rows). JT_TAN: U_l^k = acc (pre-activation tangents:
  // no bias); JT_FWD: P_l = w0 (acc + b); JT_DX: dZ_{l-1} = (acc cos(P_{l-1})) w0, the block's 16
  // phases loaded before the first is used.
  const int64_t oplane = N * (int64_t)a.Nout;
  float* Uo = a.Uout + b * (int64_t)(MODE == JT_TAN ? a.Su : 1) * oplane;
  const phase_t* Po = (const phase_t*)a.P + b * oplane;  // JT_DX: P_{l-1} [N][Nout]
#pragma unroll
  for (int bn = 0; bn < 2; ++bn) {
    const int f = 64 * wn + 32 * bn + r32;
    if (f >= a.Nout) continue;
    float bcol = 0.f;
    if constexpr (MODE == JT_FWD) bcol = a.bias[b * a.b_bstride + f];
#pragma unroll
    for (int s = 0; s < C; ++s) {
      phase_t pv[16];
      if constexpr (MODE == JT_DX) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t n = arow(s) - ar + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
          pv[e] = Po[(n < N ? n : N - 1) * a.Nout + f];
        }
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t n = arow(s) - ar + 32 * wm + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (n >= N) continue;
        float v = acc[s][bn][e];
        if constexpr (MODE == JT_FWD) v = PT::encz(v, bcol, a.w0);
        if constexpr (MODE == JT_DX) v = (v * PT::cosp(pv[e])) * a.w0;
        Uo[(STREAMS ? (int64_t)s * oplane : 0) + n * a.Nout + f] = v;
      }
    }
  }
}

// First layer adjoint: dW0[f][c] = sum_n a_bar[n][f] x[n][c] + sum_n u_bar^c[n][f] (c < C),
// db0[f] = sum_n a_bar[n][f], dx[n][c] = sum_f a_bar[n][f] W0[f][c]. Thread per feature column;
// dx via a separate pass (jvp_first_dx_kernel).
struct JFirstBwdArgs {
  const void* D;      // [B][S'][N][F] grad_t
  const float* x;     // [B][N][C]
  const float* W;     // [nb_w][F][C]
  float* dx;          // [B][N][C] or null
  float* part;        // slabs of F*C + F
  int64_t N;
  int64_t rows_per_split;
  int64_t split_stride;
  int C, F, S;        // S = adjoint streams (stride of D)
  int64_t w_bstride;
};

template <int PREC>
__global__ __launch_bounds__(256) void jvp_first_bwd_kernel(JFirstBwdArgs a) {
  using PT = Prec<PREC>;
  using grad_t = typename PT::grad_t;
  const int64_t b = blockIdx.y;
  const int S = a.S;
  const int64_t r_begin = (int64_t)blockIdx.x * a.rows_per_split;
  const int64_t r_end = min(r_begin + a.rows_per_split, a.N);
  float* part = a.part + (int64_t)blockIdx.x * a.split_stride + b * (int64_t)(a.F * a.C + a.F);
  for (int f = threadIdx.x; f < a.F; f += 256) {
    float dw[4] = {0.f, 0.f, 0.f, 0.f}, db = 0.f;
    for (int64_t n = r_begin; n < r_end; ++n) {
      const float abar = to_f32(((const grad_t*)a.D)[(b * S * a.N + n) * a.F + f]);
      db += abar;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < a.C) {
          const float ubar = to_f32(((const grad_t*)a.D)[((b * S + 1 + c) * a.N + n) * a.F + f]);
          dw[c] += fmaf(abar, a.x[(b * a.N + n) * a.C + c], ubar);
        }
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (c < a.C) part[f * a.C + c] = dw[c];
    part[a.F * a.C + f] = db;
  }
}

template <int PREC>
__global__ __launch_bounds__(256) void jvp_first_dx_kernel(JFirstBwdArgs a) {
  using PT = Prec<PREC>;
  using grad_t = typename PT::grad_t;
  const int64_t b = blockIdx.y;
  const int S = a.S;
  const float* W = a.W + b * a.w_bstride;
  const int l32 = threadIdx.x & 31;
  for (int64_t n = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); n < a.N; n += (int64_t)gridDim.x * 8) {
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int f = l32; f < a.F; f += 32) {
      const float abar = to_f32(((const grad_t*)a.D)[(b * S * a.N + n) * a.F + f]);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < a.C) s[c] = fmaf(abar, W[f * a.C + c], s[c]);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c < a.C) {
        float v = s[c];
#pragma unroll
        for (int off = 16; off >= 1; off >>= 1) v += __shfl_xor(v, off, 32);
        if (l32 == 0) a.dx[(b * a.N + n) * a.C + c] = v;
      }
    }
  }
}

}  // namespace siren
