// siren_gemm.hip — MFMA layers of the SIREN stack on gfx950 (CDNA4).
//
//   nt_gemm   MODE_FWD: P_l = enc(w0 * (sin(P_{l-1}) W_l^T + b_l))          (modules.py:25-26,38)
//             MODE_DX : dZ_{l-1} = (dZ_l W_l) * cos(P_{l-1}) * w0            (autograd Mm/Sin/Mul bwd)
//             MODE_FIRST: P_0 = enc(w0 * (x W_0^T + b_0)) for wide inputs (in_features > 16, e.g. the
//                         Fourier-feature coordinates of the hypernetwork SIREN, meta_modules.py:205-213)
//             MODE_DXLIN: dx = dZ_0 W_0 (fp32, no activation) for wide inputs
//   tn_dw     partial dW_l = dZ_l^T sin(P_{l-1}) (or dZ_0^T x), db_l = sum dZ_l   (split-K over rows)
//
// nt_gemm structure (one launch per layer, persistent workgroups):
//   * 8 waves; wave w owns output columns [32w, 32w+32) and keeps that slice of W (its MFMA B
//     operand, K/16 bf16x8 fragments or K/2 fp32 values) in registers for the whole launch.
//   * row tiles of BM coordinates stream through a double-buffered LDS A tile; the prologue
//     transform (sin of the 16-bit phase, or the stored gradient) happens in the register-staged
//     write, the next tile's global loads are in flight under the current tile's MFMAs.
//   * epilogue through LDS: each lane writes its accumulator elements (bias, w0 and the phase
//     encoding, or the cos(P) weighting read from the staged P tile) into a BM x 256 tile, and
//     the workgroup then stores it with coalesced 16-byte writes.
#include "siren_common.h"

namespace siren {

constexpr int MODE_FWD = 0;
constexpr int MODE_DX = 1;
constexpr int MODE_FIRST = 2;
constexpr int MODE_DXLIN = 3;

struct NTArgs {
  const void* A;       // [rows, lda] phase_t (FWD), grad_t (DX, DXLIN) or f32 (FIRST)
  const void* W;       // [nb_w][N, K] op_t   (FWD: W_l ; DX: W_l^T ; FIRST: W_0 zero-padded to K)
  const float* bias;   // [nb_w][N] (FWD only)
  const void* Paux;    // [rows, N] phase_t (DX: P_{l-1})
  void* C;             // [rows, N] phase_t (FWD, FIRST), grad_t (DX) or f32 (DXLIN)
  int64_t rows_per_batch;
  int64_t w_bstride;     // elements between weight sets (0 = shared)
  int64_t bias_bstride;  // elements between bias sets (0 = shared)
  int K;
  int N;
  int lda;             // FIRST: row stride of x (= in_features <= K); otherwise K
  int a_vec;           // FIRST: x rows are 16-byte aligned (lda % 4 == 0, aligned base)
  float w0;
};

// Largest power-of-two divisor of the 16-byte chunks per row, capped at 16, minus one: the XOR
// swizzle c ^ (r & smask) then stays inside the row for every K that is a multiple of 16.
DEV int swizzle_mask(int chunks) { return min(16, chunks & -chunks) - 1; }

struct TNArgs {
  const void* D;       // [rows, M] grad_t  (dZ_l)
  const void* P;       // [rows, N] phase_t (P_{l-1}), or f32 x for the wide first layer
  float* part;         // split s, batch b slab at part + s*split_stride + b*(M*N + M)  (dW then db)
  int64_t rows_per_batch;
  int64_t rows_per_split;
  int64_t split_stride;
  int M;
  int N;
  int p_vec;           // RAW: x rows are 16-byte aligned (N % 4 == 0, aligned base)
};

// ------------------------------------------------------------------------------------------
// bf16 nt_gemm. LDS images (all linear, so LDS-DMA can fill them):
//   A[buf]: BM rows x K bf16, row r chunk c (16 B) stored at chunk c ^ (r & smask): the 32 lanes of
//           an MFMA A-fragment read (32 rows, same chunk) then hit 16 distinct bank slots.
//   C[buf]: BM rows x ncols 2-byte elements (the staged P tile for DX, overwritten in place by the
//           output tile, then stored with coalesced 16-byte writes).
// ------------------------------------------------------------------------------------------
DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
DEV void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

typedef __attribute__((address_space(3))) void lds_void;

template <int MODE, int KMAX>
__global__ __launch_bounds__(512) void nt_bf16_kernel(NTArgs a) {
  using PT = Prec<kPrecBF16>;
  constexpr int BM = 64 * 256 / KMAX;
  constexpr int A_BYTES = BM * KMAX * 2;
  constexpr int C_BYTES = BM * 256 * 2;
  constexpr int NKS = KMAX / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * A_BYTES + 2 * C_BYTES];
  char* const Abase = smem;
  char* const Cbase = smem + 2 * A_BYTES;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int n0 = blockIdx.z * 256;
  const int K = a.K, N = a.N;
  const int ncols = min(256, N - n0);
  const int64_t rows = a.rows_per_batch;
  const int64_t rowbase = batch * rows;
  const int64_t ntiles = (rows + BM - 1) / BM;
  const int col_l = 32 * wave + r32;
  const bool col_ok = col_l < ncols;
  const bool wave_on = 32 * wave < ncols;
  const int a_cpr = K >> 3;                 // 16-byte chunks per A row
  const int smask = swizzle_mask(a_cpr);
  const int c_cpr = ncols >> 3;             // 16-byte chunks per C row
  const int nks = K >> 4;

  // W slice: B operand of wave w = rows [n0+32w, +32) of W (or W^T), all K.
  const bf16* Wb = (const bf16*)a.W + batch * a.w_bstride + (int64_t)(n0 + col_l) * K;
  bf16x8 wf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (ks < nks && col_ok) wf[ks] = *(const bf16x8*)(Wb + 16 * ks + 8 * h);
    else
#pragma unroll
      for (int e = 0; e < 8; ++e) wf[ks][e] = (bf16)0.f;
  }
  constexpr bool FWDLIKE = MODE == MODE_FWD || MODE == MODE_FIRST;
  float bcol = 0.f;
  if constexpr (FWDLIKE) bcol = col_ok ? a.bias[batch * a.bias_bstride + n0 + col_l] : 0.f;

  auto a_off = [&](int r, int c) -> int { return r * K * 2 + ((c ^ (r & smask)) << 4); };

  // ---- staging ----
  u16x8 areg[4];  // FWD: next tile's phases (register staged: the sin transform happens on write)
  f32x4 xreg[4][2];  // FIRST: next tile's raw inputs
  auto fwd_load = [&](int64_t t) {
    const int64_t m0 = t * BM;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int r = u / a_cpr, c = u - r * a_cpr;
      const bool in = r < BM && m0 + r < rows;
      if constexpr (MODE == MODE_FIRST) {
        const float* src = (const float*)a.A + (rowbase + m0 + r) * a.lda + c * 8;
        if (in && a.a_vec && c * 8 + 8 <= a.lda) {
          xreg[q][0] = *(const f32x4*)src;
          xreg[q][1] = *(const f32x4*)(src + 4);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) xreg[q][e >> 2][e & 3] = (in && c * 8 + e < a.lda) ? src[e] : 0.f;
        }
      } else {
        if (in)
          areg[q] = *(const u16x8*)((const uint16_t*)a.A + (rowbase + m0 + r) * K + c * 8);
        else
          areg[q] = u16x8{};
      }
    }
  };
  auto fwd_store = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int r = u / a_cpr, c = u - r * a_cpr;
      if (r < BM) {
        bf16x8 v;
        if constexpr (MODE == MODE_FIRST) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (bf16)xreg[q][e >> 2][e & 3];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = (bf16)PT::sinp(areg[q][e]);
        }
        *(bf16x8*)(Abase + buf * A_BYTES + a_off(r, c)) = v;
      }
    }
  };
  // DX: LDS-DMA of the dZ tile (A image, swizzle applied on the source address) and the P tile.
  auto dx_dma = [&](int64_t t, int buf) {
    const int64_t m0 = t * BM;
    const int n_a = BM * a_cpr / 64, n_p = BM * c_cpr / 64;
    for (int i = wave; i < n_a; i += 8) {
      const int u = i * 64 + lane;
      const int r = u / a_cpr, p = u - r * a_cpr;
      const int c = p ^ (r & smask);
      const int64_t row = min(m0 + r, rows - 1);
      __builtin_amdgcn_global_load_lds((const void*)((const bf16*)a.A + (rowbase + row) * K + c * 8),
                                       (lds_void*)(Abase + buf * A_BYTES + i * 1024), 16, 0, 0);
    }
    if constexpr (MODE == MODE_DX)
    for (int i = wave; i < n_p; i += 8) {
      const int u = i * 64 + lane;
      const int r = u / c_cpr, c = u - r * c_cpr;
      const int64_t row = min(m0 + r, rows - 1);
      __builtin_amdgcn_global_load_lds((const void*)((const uint16_t*)a.Paux + (rowbase + row) * N + n0 + c * 8),
                                       (lds_void*)(Cbase + buf * C_BYTES + i * 1024), 16, 0, 0);
    }
  };

  int64_t t = blockIdx.x;
  if (t >= ntiles) return;
  if constexpr (FWDLIKE) {
    fwd_load(t);
    fwd_store(0);
  } else {
    dx_dma(t, 0);
    vm_drain();
  }
  lds_barrier();
  int cur = 0;
  for (; t < ntiles; t += gridDim.x) {
    const int64_t tn = t + gridDim.x;
    const bool has_next = tn < ntiles;
    if (has_next) {
      if constexpr (FWDLIKE) fwd_load(tn);
      else dx_dma(tn, cur ^ 1);
    }
    f32x16 acc[BM / 32];
#pragma unroll
    for (int bm = 0; bm < BM / 32; ++bm)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[bm][e] = 0.f;
    // MFMA operands come from every lane: the compute guard must be wave-uniform (a wave with a
    // partial column slice computes with zero W rows and masks its stores below).
    if (wave_on) {
      const char* As = Abase + cur * A_BYTES;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        if (ks < nks) {
#pragma unroll
          for (int bm = 0; bm < BM / 32; ++bm) {
            const bf16x8 af = *(const bf16x8*)(As + a_off(32 * bm + r32, 2 * ks + h));
            acc[bm] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, wf[ks], acc[bm], 0, 0, 0);
          }
        }
      }
      // epilogue 1: accumulators -> LDS C tile (in place over the staged P tile for DX)
      uint16_t* Cs = (uint16_t*)(Cbase + cur * C_BYTES);
#pragma unroll
      for (int bm = 0; bm < BM / 32 && col_ok; ++bm)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int rl = 32 * bm + (e & 3) + 8 * (e >> 2) + 4 * h;
          uint16_t* dst = Cs + rl * ncols + col_l;
          if constexpr (FWDLIKE) {
            *dst = PT::encz(acc[bm][e], bcol, a.w0);
          } else if constexpr (MODE == MODE_DXLIN) {
            const int64_t row = t * BM + rl;
            if (row < rows) ((float*)a.C)[(rowbase + row) * N + n0 + col_l] = acc[bm][e];
          } else {
            const float c = PT::cosp(*dst);
            *dst = __builtin_bit_cast(uint16_t, (bf16)((acc[bm][e] * c) * a.w0));
          }
        }
    }
    if constexpr (MODE == MODE_DX || MODE == MODE_DXLIN) vm_drain();  // next tile's DMA has landed
    lds_barrier();
    // epilogue 2: coalesced 16-byte stores of the finished tile
    if constexpr (MODE != MODE_DXLIN) {
      const int64_t m0 = t * BM;
      const int nch = BM * c_cpr;
      for (int u = tid; u < nch; u += 512) {
        const int r = u / c_cpr, c = u - r * c_cpr;
        if (m0 + r < rows)
          *(u16x8*)((uint16_t*)a.C + (rowbase + m0 + r) * N + n0 + c * 8) =
              *(const u16x8*)(Cbase + cur * C_BYTES + (r * ncols + c * 8) * 2);
      }
    }
    if constexpr (FWDLIKE) {
      if (has_next) fwd_store(cur ^ 1);
    }
    lds_barrier();
    cur ^= 1;
  }
}

// ------------------------------------------------------------------------------------------
// fp32 nt_gemm (exact-fp32 MFMA 32x32x2). Register-staged A (and P for DX) tiles, 32 rows per
// tile, padded LDS rows (K+1 floats) for conflict-free column reads; same epilogue scheme.
// ------------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(512) void nt_f32_kernel(NTArgs a) {
  using PT = Prec<kPrecF32>;
  constexpr int KMAX = 256;
  constexpr int BM = 32;
  constexpr int AROW = KMAX + 1;
  constexpr int A_BYTES = BM * AROW * 4;
  constexpr int C_BYTES = BM * 256 * 4;
  constexpr int NKS = KMAX / 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * A_BYTES + 2 * C_BYTES];
  float* const As0 = (float*)smem;
  char* const Cs0 = smem + 2 * A_BYTES;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int n0 = blockIdx.z * 256;
  const int K = a.K, N = a.N;
  const int ncols = min(256, N - n0);
  const int64_t rows = a.rows_per_batch;
  const int64_t rowbase = batch * rows;
  const int64_t ntiles = (rows + BM - 1) / BM;
  const int col_l = 32 * wave + r32;
  const bool col_ok = col_l < ncols;
  const bool wave_on = 32 * wave < ncols;
  const int nks = K >> 1;
  const int a_cpr = K >> 2, c_cpr = ncols >> 2;

  const float* Wb = (const float*)a.W + batch * a.w_bstride + (int64_t)(n0 + col_l) * K;
  float wf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) wf[ks] = (ks < nks && col_ok) ? Wb[2 * ks + h] : 0.f;
  constexpr bool FWDLIKE = MODE == MODE_FWD || MODE == MODE_FIRST;
  float bcol = 0.f;
  if constexpr (FWDLIKE) bcol = col_ok ? a.bias[batch * a.bias_bstride + n0 + col_l] : 0.f;

  f32x4 areg[4], preg[4];
  auto load_tile = [&](int64_t t) {
    const int64_t m0 = t * BM;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int r = u / a_cpr, c = u - r * a_cpr;
      const bool in = r < BM && m0 + r < rows;
      if constexpr (MODE == MODE_FIRST) {
        const float* src = (const float*)a.A + (rowbase + m0 + r) * a.lda + c * 4;
        if (in && a.a_vec && c * 4 + 4 <= a.lda) {
          areg[q] = *(const f32x4*)src;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) areg[q][e] = (in && c * 4 + e < a.lda) ? src[e] : 0.f;
        }
      } else {
        areg[q] = in ? *(const f32x4*)((const float*)a.A + (rowbase + m0 + r) * K + c * 4)
                     : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      if constexpr (MODE == MODE_DX) {
        const int rp = u / c_cpr, cp = u - rp * c_cpr;
        preg[q] = (rp < BM && m0 + rp < rows)
                      ? *(const f32x4*)((const float*)a.Paux + (rowbase + m0 + rp) * N + n0 + cp * 4)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto store_tile = [&](int buf) {
    float* As = As0 + buf * (A_BYTES / 4);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int r = u / a_cpr, c = u - r * a_cpr;
      if (r < BM) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          As[r * AROW + c * 4 + e] = (MODE == MODE_FWD) ? PT::sinp(areg[q][e]) : areg[q][e];
      }
      if constexpr (MODE == MODE_DX) {
        const int rp = u / c_cpr, cp = u - rp * c_cpr;
        if (rp < BM) *(f32x4*)(Cs0 + buf * C_BYTES + (rp * ncols + cp * 4) * 4) = preg[q];
      }
    }
  };

  int64_t t = blockIdx.x;
  if (t >= ntiles) return;
  load_tile(t);
  store_tile(0);
  __syncthreads();
  int cur = 0;
  for (; t < ntiles; t += gridDim.x) {
    const int64_t tn = t + gridDim.x;
    if (tn < ntiles) load_tile(tn);
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    if (wave_on) {
      const float* As = As0 + cur * (A_BYTES / 4);
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        if (ks < nks) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[r32 * AROW + 2 * ks + h], wf[ks], acc, 0, 0, 0);
      float* Cs = (float*)(Cs0 + cur * C_BYTES);
#pragma unroll
      for (int e = 0; e < 16 && col_ok; ++e) {
        const int rl = (e & 3) + 8 * (e >> 2) + 4 * h;
        float* dst = Cs + rl * ncols + col_l;
        if constexpr (FWDLIKE) {
          *dst = PT::encz(acc[e], bcol, a.w0);
        } else if constexpr (MODE == MODE_DXLIN) {
          const int64_t row = t * BM + rl;
          if (row < rows) ((float*)a.C)[(rowbase + row) * N + n0 + col_l] = acc[e];
        } else {
          *dst = (acc[e] * PT::cosp(*dst)) * a.w0;
        }
      }
    }
    __syncthreads();
    if constexpr (MODE != MODE_DXLIN) {
      const int64_t m0 = t * BM;
      const int nch = BM * c_cpr;
      for (int u = tid; u < nch; u += 512) {
        const int r = u / c_cpr, c = u - r * c_cpr;
        if (m0 + r < rows)
          *(f32x4*)((float*)a.C + (rowbase + m0 + r) * N + n0 + c * 4) =
              *(const f32x4*)(Cs0 + cur * C_BYTES + (r * ncols + c * 4) * 4);
      }
    }
    if (tn < ntiles) store_tile(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
}

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

template <int PREC, bool RAW>
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
  float xr[UPT][VEC];  // RAW: fp32 inputs of the wide first layer
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
      if constexpr (RAW) {
        const float* src = (const float*)a.P + (rowbase + row) * a.N + cj;
        const bool in = row < r_end && cj < a.N;
        if (in && a.p_vec && cj + VEC <= a.N) {
#pragma unroll
          for (int v = 0; v < VEC / 4; ++v) {
            const f32x4 t4 = *(const f32x4*)(src + 4 * v);
#pragma unroll
            for (int e = 0; e < 4; ++e) xr[q][4 * v + e] = t4[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < VEC; ++e) xr[q][e] = (in && cj + e < a.N) ? src[e] : 0.f;
        }
      } else if (row < r_end && cj < a.N) {
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
      for (int e = 0; e < VEC; ++e) {
        float v = 0.f;
        if constexpr (RAW) v = xr[q][e];
        else v = PT::sinp(preg[q][e]);
        hv[e] = from_f32<op_t>(valid ? v : 0.f);
      }
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
  float* part = a.part + (int64_t)split * a.split_stride + batch * ((int64_t)a.M * a.N + a.M);
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


}  // namespace siren
