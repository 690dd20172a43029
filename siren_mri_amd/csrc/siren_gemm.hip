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

// Output-layer fusion into the top hidden layer's backward (outermost_linear, O <= 2): the
// kernels form dZ_top = (dy W_L) cos(P_top) w0 on the fly instead of reading it from HBM, exactly
// as last_bwd_kernel computes it (modules.py:25-26 backward; the output layer is linear).
constexpr int TOP_MAXO = 2;
struct TopArgs {
  const void* Ptop;    // [rows, F_top] phase of the last sine layer
  const float* dy;     // [rows, O]
  const float* dy_scale;  // [1] device scalar multiplying dy (the upstream gradient of a fused loss), or null
  const float* WL;     // [nb_w][O, F_top]
  int64_t wl_bstride;
  float* partL;        // tn_dw only: dW_L / db_L partial slabs [split][nb][O*F_top + O]
  int64_t partL_stride;
  int O;
};
// First-layer fusion into the bottom hidden layer's input-gradient kernel (C <= 4, no dx): the
// epilogue accumulates dW_0 = dZ_0^T x and db_0 = sum dZ_0 (first_bwd_kernel's sums) instead of
// storing dZ_0.
constexpr int BOT_MAXC = 4;
struct BotArgs {
  const float* x;      // [rows, C]
  const float* W0;     // [nb_w][F0, C] fp32 (dx_ring: dx = dZ_0 W_0)
  int64_t w0_bstride;
  const float* b0;     // [nb_w][F0] (P_0 recompute)
  int64_t b0_bstride;
  float* part;         // [grid.x][nb][F0*C + F0] partial slabs (slab index = workgroup)
  int64_t split_stride;
  int C;
};

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
  TopArgs top;         // DX with TOP
  BotArgs bot;         // DX with BOT
  long long* prof;     // debug: [grid.x][8 waves][RING_NPROF] segment cycle counters (null: off)
  int stagger;         // dx_ring_body_v2: waves 4-7 run each epilogue one tile late (option dx_stagger)
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
  float w0;            // TOP, dw_ring RECC
  const float* rec_W0; // dw_ring RECC: W_0 [nb_w][F0, C], b_0 [nb_w][F0] (P = x)
  int64_t rec_w0_bstride;
  const float* rec_b0;
  int64_t rec_b0_bstride;
  TopArgs top;         // TOP: D = dZ_top formed from P_top, dy and W_L; also dW_L / db_L partials
  int pair_roles;      // pair_ring (debug timing only): bit 0 runs the dx role, bit 1 the dw role
  long long* prof;     // debug: [grid.x][8 waves][RING_NPROF] segment cycle counters (null: off)
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


template <int MODE, int KMAX, bool TOP = false, bool BOT = false>
__global__ __launch_bounds__(512) void nt_bf16_kernel(NTArgs a) {
  using PT = Prec<kPrecBF16>;
  constexpr int BM = 64 * 256 / KMAX;
  constexpr int A_BYTES = BM * KMAX * 2;
  constexpr int C_BYTES = BM * 256 * 2;
  constexpr int X_BYTES = BOT ? BM * BOT_MAXC * 4 : 0;  // staged x tile (BOT)
  constexpr int G_BYTES = TOP ? BM * TOP_MAXO * 4 : 0;  // staged dy tile (TOP)
  constexpr int WL_BYTES = TOP ? TOP_MAXO * KMAX * 4 : 0;  // W_L (TOP)
  constexpr int NKS = KMAX / 16;
  static_assert(!(TOP || BOT) || MODE == MODE_DX, "fusions apply to the input-gradient GEMM");
  __shared__ __attribute__((aligned(16)))
  char smem[2 * A_BYTES + 2 * C_BYTES + 2 * X_BYTES + 2 * G_BYTES + WL_BYTES];
  char* const Abase = smem;
  char* const Cbase = smem + 2 * A_BYTES;
  char* const Xbase = smem + 2 * A_BYTES + 2 * C_BYTES;
  char* const Gbase = Xbase + 2 * X_BYTES;
  float* const WLs = (float*)(Gbase + 2 * G_BYTES);

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
  // TOP: the dZ_top tile is formed from the register-staged P_top phases, the dy tile (LDS-DMA)
  // and W_L (LDS), exactly as last_bwd_kernel forms it, and written into the A image.
  const float dys = (TOP && a.top.dy_scale) ? *a.top.dy_scale : 1.f;
  if constexpr (TOP) {
    for (int i = tid; i < TOP_MAXO * K; i += 512) {
      const int o = i / K, f = i - o * K;
      WLs[i] = o < a.top.O ? a.top.WL[batch * a.top.wl_bstride + (int64_t)o * K + f] * a.w0 : 0.f;
    }
  }
  // In place over the A image, whose chunks the DMA filled with P_top phases (same swizzle).
  auto top_store = [&](int buf) {
    const float* gt = (const float*)(Gbase + buf * G_BYTES);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int u = tid + 512 * q;
      const int r = u / a_cpr, c = u - r * a_cpr;
      if (r < BM) {
        char* p = Abase + buf * A_BYTES + a_off(r, c);
        const u16x8 ph = *(const u16x8*)p;
        float g[TOP_MAXO];
#pragma unroll
        for (int o = 0; o < TOP_MAXO; ++o) g[o] = o < a.top.O ? gt[r * a.top.O + o] * dys : 0.f;
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float dh = g[0] * WLs[8 * c + e];
#pragma unroll
          for (int o = 1; o < TOP_MAXO; ++o) dh = fmaf(g[o], WLs[o * K + 8 * c + e], dh);
          v[e] = (bf16)(dh * PT::cosp(ph[e]));
        }
        *(bf16x8*)p = v;
      }
    }
  };
  // BOT: per-lane sums of dZ_0 x (its column, C inputs) and dZ_0, over every row it sees.
  float bot_dw[BOT ? BOT_MAXC : 1], bot_db = 0.f;
#pragma unroll
  for (int ci = 0; ci < (BOT ? BOT_MAXC : 1); ++ci) bot_dw[ci] = 0.f;

  // DX: LDS-DMA of the dZ tile (A image, swizzle applied on the source address) and the P tile.
  auto dx_dma = [&](int64_t t, int buf) {
    const int64_t m0 = t * BM;
    const int n_a = BM * a_cpr / 64, n_p = BM * c_cpr / 64;
    if constexpr (BOT) {
      // x tile rows [m0, m0 + BM) are contiguous: BM*C floats in 16-byte pieces
      const int nx = BM * a.bot.C / 4;
      if (wave == 7 && lane < nx) {
        const int64_t el = min((int64_t)(m0 * a.bot.C) + 4 * lane, rows * a.bot.C - 4);
        __builtin_amdgcn_global_load_lds((const void*)(a.bot.x + rowbase * a.bot.C + el),
                                         (lds_void*)(Xbase + buf * X_BYTES), 16, 0, 0);
      }
    }
    if constexpr (TOP) {
      // dy rows [m0, m0 + BM): BM*O floats in 16-byte pieces (rows past the end are masked later)
      const int ng = BM * a.top.O / 4;
      if (wave == 6 && lane < ng) {
        const int64_t el = min((int64_t)(m0 * a.top.O) + 4 * lane, rows * a.top.O - 4);
        __builtin_amdgcn_global_load_lds((const void*)(a.top.dy + rowbase * a.top.O + el),
                                         (lds_void*)(Gbase + buf * G_BYTES), 16, 0, 0);
      }
    }
    const void* asrc = TOP ? a.top.Ptop : a.A;  // TOP: P_top phases, converted in place later
    for (int i = wave; i < n_a; i += 8) {
      const int u = i * 64 + lane;
      const int r = u / a_cpr, p = u - r * a_cpr;
      const int c = p ^ (r & smask);
      const int64_t row = min(m0 + r, rows - 1);
      __builtin_amdgcn_global_load_lds((const void*)((const bf16*)asrc + (rowbase + row) * K + c * 8),
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
    if constexpr (TOP) {
      lds_barrier();  // W_L and the dy tile visible
      top_store(0);
    }
  }
  lds_barrier();
  int cur = 0;
  for (; t < ntiles; t += gridDim.x) {
    const int64_t tn = t + gridDim.x;
    const bool has_next = tn < ntiles;
    if (has_next) {
      if constexpr (FWDLIKE) fwd_load(tn);
      else {
        dx_dma(tn, cur ^ 1);
      }
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
          } else if constexpr (BOT) {
            // the bf16-rounded dZ_0 (what first_bwd would read back), summed against x
            const float c = PT::cosp(*dst);
            const float dz = (float)(bf16)((acc[bm][e] * c) * a.w0);
            if (t * BM + rl < rows) {
              const float* xr = (const float*)(Xbase + cur * X_BYTES) + rl * a.bot.C;
              bot_db += dz;
#pragma unroll
              for (int ci = 0; ci < BOT_MAXC; ++ci)
                if (ci < a.bot.C) bot_dw[ci] = fmaf(dz, xr[ci], bot_dw[ci]);
            }
          } else {
            const float c = PT::cosp(*dst);
            *dst = __builtin_bit_cast(uint16_t, (bf16)((acc[bm][e] * c) * a.w0));
          }
        }
    }
    if constexpr (MODE == MODE_DX || MODE == MODE_DXLIN) vm_drain();  // next tile's DMA has landed
    lds_barrier();
    // epilogue 2: coalesced 16-byte stores of the finished tile
    if constexpr (MODE != MODE_DXLIN && !BOT) {
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
    if constexpr (TOP) {
      if (has_next) top_store(cur ^ 1);
    }
    lds_barrier();
    cur ^= 1;
  }
  if constexpr (BOT) {
    // lanes l and l + 32 hold the same column: combine, then one slab row per column
    bot_db += __shfl_xor(bot_db, 32, 64);
#pragma unroll
    for (int ci = 0; ci < BOT_MAXC; ++ci) bot_dw[ci] += __shfl_xor(bot_dw[ci], 32, 64);
    if (h == 0 && col_ok) {
      const int F0 = N, f = n0 + col_l;
      float* part = a.bot.part + (int64_t)blockIdx.x * a.bot.split_stride + batch * (int64_t)(F0 * a.bot.C + F0);
      for (int ci = 0; ci < a.bot.C; ++ci) part[f * a.bot.C + ci] = bot_dw[ci];
      part[F0 * a.bot.C + f] = bot_db;
    }
  }
}

// ------------------------------------------------------------------------------------------
// fp32 nt_gemm (exact-fp32 MFMA 32x32x2). Register-staged A (and P for DX) tiles, 32 rows per
// tile, padded LDS rows (K+1 floats) for conflict-free column reads; same epilogue scheme.
// ------------------------------------------------------------------------------------------
// KMAX 512 (hidden width 257..512, fp32 mode): the K range is two chunks of 256; the wave's W
// columns of one chunk are in registers at a time (reloaded from L2 per chunk and tile: 1 KB per
// lane per tile against 256 fp32 MFMAs of 64 cycles), and the A tile is single-buffered (its
// 32 x 513 floats twice would not fit beside the C staging).
template <int MODE, int KMAX = 256>
__global__ __launch_bounds__(512) void nt_f32_kernel(NTArgs a) {
  using PT = Prec<kPrecF32>;
  static_assert(KMAX == 256 || KMAX == 512, "fp32 GEMM K bound");
  constexpr int BM = 32;
  constexpr int AROW = KMAX + 1;
  constexpr int A_BYTES = BM * AROW * 4;
  constexpr int NABUF = KMAX == 256 ? 2 : 1;
  constexpr int C_BYTES = BM * 256 * 4;
  constexpr int NKC = 128;                 // K steps (of 2) per register chunk
  constexpr int NCH = KMAX / 256;          // chunks
  constexpr int AQ = KMAX / 64;            // A-tile float4 units per thread (32 rows x KMAX / 4 / 512)
  __shared__ __attribute__((aligned(16))) char smem[NABUF * A_BYTES + 2 * C_BYTES];
  float* const As0 = (float*)smem;
  char* const Cs0 = smem + NABUF * A_BYTES;

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
  float wf[NKC];
  auto load_w = [&](int c) {
#pragma unroll
    for (int ks = 0; ks < NKC; ++ks) {
      const int kk = NKC * c + ks;
      wf[ks] = (kk < nks && col_ok) ? Wb[2 * kk + h] : 0.f;
    }
  };
  load_w(0);
  constexpr bool FWDLIKE = MODE == MODE_FWD || MODE == MODE_FIRST;
  float bcol = 0.f;
  if constexpr (FWDLIKE) bcol = col_ok ? a.bias[batch * a.bias_bstride + n0 + col_l] : 0.f;

  f32x4 areg[AQ], preg[4];
  auto load_tile = [&](int64_t t) {
    const int64_t m0 = t * BM;
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
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
    }
    if constexpr (MODE == MODE_DX) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = tid + 512 * q;
        const int rp = u / c_cpr, cp = u - rp * c_cpr;
        preg[q] = (rp < BM && m0 + rp < rows)
                      ? *(const f32x4*)((const float*)a.Paux + (rowbase + m0 + rp) * N + n0 + cp * 4)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto store_tile = [&](int buf) {
    float* As = As0 + (NABUF == 2 ? buf : 0) * (A_BYTES / 4);
#pragma unroll
    for (int q = 0; q < AQ; ++q) {
      const int u = tid + 512 * q;
      const int r = u / a_cpr, c = u - r * a_cpr;
      if (r < BM) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          As[r * AROW + c * 4 + e] = (MODE == MODE_FWD) ? PT::sinp(areg[q][e]) : areg[q][e];
      }
    }
    if constexpr (MODE == MODE_DX) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = tid + 512 * q;
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
      const float* As = As0 + (NABUF == 2 ? cur : 0) * (A_BYTES / 4);
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        if (NCH > 1 && (c > 0 || t != blockIdx.x)) load_w(c);  // (chunk 0 of the first tile: loaded above)
#pragma unroll
        for (int ks = 0; ks < NKC; ++ks)
          if (NKC * c + ks < nks)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[r32 * AROW + 2 * (NKC * c + ks) + h], wf[ks], acc, 0, 0, 0);
      }
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

template <int PREC, bool RAW, bool TOP = false>
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
  // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so consecutive slots of one
  // XCD take all output tiles of one (split, batch) row range — its dZ / P rows are then read from
  // HBM once and re-read from that XCD's L2.
  int tile, split;
  int64_t batch;
  {
    const int64_t gx = gridDim.x, groups = (int64_t)gridDim.y * gridDim.z;
    const int64_t lin = blockIdx.x + gx * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z);
    int64_t grp;
    if (groups % 8 == 0) {
      const int64_t slot = lin >> 3;
      tile = (int)(slot % gx);
      grp = (slot / gx) * 8 + (lin & 7);
    } else {
      tile = blockIdx.x;
      grp = blockIdx.y + (int64_t)gridDim.y * blockIdx.z;
    }
    split = (int)(grp % gridDim.y);
    batch = grp / gridDim.y;
  }
  const int ti = tile / tiles_n, tj = tile % tiles_n;
  const int i0 = ti * TN_BM, j0 = tj * TN_BN;
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
  static_assert(!TOP || PREC == kPrecBF16, "output-layer fusion is a bf16-mode path");
  // TOP: phases of P_top for the D columns, dy rows, this thread's W_L columns, dW_L/db_L sums
  u16x8 tph[TOP ? UPT : 1];
  float tg[TOP ? UPT : 1][TOP_MAXO];
  float twl[TOP_MAXO][TOP ? VEC : 1];
  const float dys = (TOP && a.top.dy_scale) ? *a.top.dy_scale : 1.f;
  float tdw[TOP_MAXO][TOP ? VEC : 1];
  float tdb[TOP_MAXO];
  if constexpr (TOP) {
#pragma unroll
    for (int o = 0; o < TOP_MAXO; ++o) {
      tdb[o] = 0.f;
#pragma unroll
      for (int e = 0; e < VEC; ++e) {
        const int ci = i0 + cu * VEC + e;
        twl[o][e] = (o < a.top.O && ci < a.M) ? a.top.WL[batch * a.top.wl_bstride + (int64_t)o * a.M + ci] * a.w0 : 0.f;
        tdw[o][e] = 0.f;
      }
    }
  }

  auto load = [&](int64_t rc) {
#pragma unroll
    for (int q = 0; q < UPT; ++q) {
      const int r = (tid + 256 * q) / UPR;
      const int64_t row = rc + r;
      const int ci = i0 + cu * VEC, cj = j0 + cu * VEC;
      if constexpr (TOP) {
        const bool in = row < r_end && ci < a.M;
        const int64_t rr = rowbase + (in ? row : 0);
        tph[q] = in ? *(const u16x8*)((const uint16_t*)a.top.Ptop + rr * a.M + ci) : u16x8{};
#pragma unroll
        for (int o = 0; o < TOP_MAXO; ++o) tg[q][o] = (in && o < a.top.O) ? a.top.dy[rr * a.top.O + o] * dys : 0.f;
      } else if (row < r_end && ci < a.M) {
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
      if constexpr (TOP) {
        // dZ_top exactly as last_bwd_kernel forms it; dW_L / db_L sums on the side (tj == 0)
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          float dh = tg[q][0] * twl[0][e];
#pragma unroll
          for (int o = 1; o < TOP_MAXO; ++o) dh = fmaf(tg[q][o], twl[o][e], dh);
          dv[e] = from_f32<op_t>(dh * PT::cosp(tph[q][e]));
        }
        if (do_db) {
#pragma unroll
          for (int e = 0; e < VEC; ++e) {
            const float sv = PT::sinp(tph[q][e]);
#pragma unroll
            for (int o = 0; o < TOP_MAXO; ++o) tdw[o][e] = fmaf(tg[q][o], sv, tdw[o][e]);
          }
#pragma unroll
          for (int o = 0; o < TOP_MAXO; ++o) tdb[o] += tg[q][o];
        }
      }
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
  if constexpr (TOP) {
    if (do_db) {
      // dW_L[o][i0 + cu*VEC + e] summed over the 256/UPR threads sharing the column unit
      __syncthreads();
      float* red = (float*)smem;  // [256 / UPR][TOP_MAXO * 128 + TOP_MAXO]
      constexpr int RS = TOP_MAXO * 128 + TOP_MAXO;
      const int slot = tid / UPR;
#pragma unroll
      for (int o = 0; o < TOP_MAXO; ++o)
#pragma unroll
        for (int e = 0; e < VEC; ++e) red[slot * RS + o * 128 + cu * VEC + e] = tdw[o][e];
      if (cu == 0) {
#pragma unroll
        for (int o = 0; o < TOP_MAXO; ++o) red[slot * RS + TOP_MAXO * 128 + o] = tdb[o];
      }
      __syncthreads();
      float* pl = a.top.partL + (int64_t)split * a.top.partL_stride + batch * (int64_t)(a.top.O * a.M + a.top.O);
      for (int idx = tid; idx < a.top.O * 128; idx += 256) {
        const int o = idx >> 7, col = i0 + (idx & 127);
        if (col < a.M) {
          float sum = 0.f;
          for (int k = 0; k < 256 / UPR; ++k) sum += red[k * RS + idx];
          pl[o * a.M + col] = sum;
        }
      }
      if (ti == 0 && tid < a.top.O) {
        float sum = 0.f;
        for (int k = 0; k < 256 / UPR; ++k) sum += red[k * RS + TOP_MAXO * 128 + tid];
        pl[a.top.O * a.M + tid] = sum;
      }
    }
  }
}


}  // namespace siren

namespace siren {

// ------------------------------------------------------------------------------------------
// dx_ring: the 256 x 256 input-gradient layer (MODE_DX of nt_bf16_kernel) with a deeper load
// pipeline. 32-row tiles flow through a 4-stage LDS ring (dZ tile in the swizzled A image, P tile
// in the C image; 32 KB per stage), so three tiles' DMA (96 KB per CU) are in flight while one
// is computed. Waits are counted (s_waitcnt vmcnt(N) for exactly the stage being consumed), never
// vmcnt(0) in steady state, so the stores of earlier tiles keep draining under the compute.
// ------------------------------------------------------------------------------------------
constexpr int RING_S = 4;
constexpr int RING_BM = 32;
constexpr int RING_NPROF = 6;

// debug segment timer of the ring kernels (s_memtime; perturbs timing by ~10 %)
#ifdef SIREN_RING_PROF
struct RingProf {
  long long* out;
  long long acc[RING_NPROF];
  long long mark;
  DEV RingProf(long long* p) : out(p), mark(0) {
    for (int i = 0; i < RING_NPROF; ++i) acc[i] = 0;
    if (out) mark = clock64();
  }
  DEV void tick(int k) {
    if (out) {
      const long long now = clock64();
      acc[k] += now - mark;
      mark = now;
    }
  }
  DEV void flush(int64_t slot) {
    if (out && (threadIdx.x & 63) == 0)
      for (int i = 0; i < RING_NPROF; ++i) out[(slot * 8 + (threadIdx.x >> 6)) * RING_NPROF + i] = acc[i];
  }
};
#else
// product builds: no counters (a runtime null check would split every tile's schedule at the ticks)
struct RingProf {
  DEV RingProf(long long*) {}
  DEV void tick(int) {}
  DEV void flush(int64_t) {}
};
#endif

template <int VMCNT>
DEV void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMCNT) : "memory"); }

// The dx_ring MFMA chain over K = 256: acc = sum_ks W^T[ks] . B(ks), the B fragments read from
// the staged 32-row tile (row r, 16-byte chunk c at chunk c ^ (r & 15)). The lane's fragment of
// K step ks sits at byte off0 ^ (32 ks) of the image (off0 = r * 512 + 16 (h ^ (r & 15))), so
// each read is one XOR and one add. The reads are inline asm, PF in flight, each MFMA tied to
// its own read by a counted wait: the compiler neither serialises them (one read, wait, MFMA)
// under register pressure nor drains the ring's LDS-DMA in front of them (vmcnt(0)).
DEV void ring_read_b128(bf16x8& d, uint32_t va) { asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(va)); }
template <int N>
DEV void ring_lgkm(bf16x8& v) { asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N)); }
template <int PF = 4>
DEV f32x16 ring_chain(const bf16x8 (&wf)[16], uint32_t sbase, uint32_t off0) {
  bf16x8 b[PF];
  static_for<0, PF>([&](auto k_c) {
    constexpr int k = decltype(k_c)::value;
    ring_read_b128(b[k], sbase + (off0 ^ (32 * k)));
  });
  f32x16 acc;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc[e] = 0.f;
  static_for<0, 16>([&](auto ks_c) {
    constexpr int ks = decltype(ks_c)::value;
    constexpr int after = (15 - ks) < (PF - 1) ? (15 - ks) : (PF - 1);  // reads issued after ks's
    ring_lgkm<after>(b[ks % PF]);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], b[ks % PF], acc, 0, 0, 0);
    if constexpr (ks + PF < 16) ring_read_b128(b[ks % PF], sbase + (off0 ^ (32 * (ks + PF))));
  });
  return acc;
}

// BOTC > 0: the bottom hidden layer with the first layer folded in (C = BOTC inputs): dZ_0 stays
// in LDS; a VALU pass over it accumulates dW_0 / db_0 (first_bwd_kernel's sums, per-workgroup
// partial slabs in a.bot.part) and, with DXOUT, writes dx = dZ_0 W_0 (a.C, [rows, C] f32).
// The x tile rides in the ring with the other operands (one 16-byte DMA lane per input channel
// per wave), so the counted vector-memory waits stay exact.
// REC (with BOTC > 0): P_0 was not kept by the forward; the epilogue recomputes each phase from
// the staged x tile, W_0 and b_0 with the forward's arithmetic (first layer of fused_fwd_bf16 /
// first_fwd: fmaf chain over the inputs, then PT::encz), so cos(P_0) is bit-identical.
// TOPO > 0 (top hidden layer, outermost_linear, O = TOPO outputs): the A operand dZ_top is not
// read; the ring carries P_top (in the A image) and the dy tile, and a pass forms
// dZ_top = (dy W_L) cos(P_top) w0 in place exactly as last_bwd_kernel does.
// (BOTC == 0: plus the staggered half's private store staging, 4 waves x 32 rows x 80 B)
constexpr int DX_STAGE_ROW = 80;
template <int BOTC, int TOPO>
constexpr int dx_ring_lds_bytes() {
  return RING_S * (RING_BM * 256 * 2 * 2 + (BOTC > 0 ? RING_BM * BOTC * 4 : 0) + (TOPO > 0 ? RING_BM * TOPO * 4 : 0)) +
         (BOTC == 0 ? 4 * RING_BM * DX_STAGE_ROW : 0);
}

// The tiles of one workgroup: t = t0 + i * G for i < niter; `slab` indexes the BOTC first-layer
// partial slab it writes.
template <int BOTC, bool DXOUT, bool REC = false, int TOPO = 0>
DEV void dx_ring_body_v1(const NTArgs& a, char* smem, const int64_t t0, const int64_t G, const int64_t niter,
                         const int64_t slab) {
  using PT = Prec<kPrecBF16>;
  constexpr int K = 256, N = 256, BM = RING_BM, S = RING_S;
  constexpr int X_BYTES = BOTC > 0 ? BM * BOTC * 4 : 0;
  constexpr int G_BYTES = TOPO > 0 ? BM * TOPO * 4 : 0;
  constexpr int A_BYTES = BM * K * 2, C_BYTES = BM * N * 2, STAGE = A_BYTES + C_BYTES + X_BYTES + G_BYTES;
  static_assert(S * STAGE == dx_ring_lds_bytes<BOTC, TOPO>(), "dx_ring LDS size");
  constexpr int NKS = K / 16;
  constexpr int A_CPR = K / 8, C_CPR = N / 8;   // 16-byte chunks per row
  constexpr int SMASK = 15;
  constexpr int NA = BM * A_CPR / 64 / 8;       // DMA instructions per wave per stage (A) = 2
  constexpr int NP = REC ? 0 : BM * C_CPR / 64 / 8;  // (P) = 2, none when P_0 is recomputed
  static_assert(!REC || BOTC > 0, "P_0 recompute needs the staged x tile");
  constexpr int NQ = BM * C_CPR / 512;          // chunks per thread in the store / BOT pass = 2
  constexpr bool BOT = BOTC > 0;
  constexpr int NST = BOT ? (DXOUT ? NQ : 0) : NQ;  // vector stores per thread per tile
  // VMEM ops issued after stage i's DMA when iteration i waits for it: the stores of the S-1
  // previous tiles and the DMAs of the S-2 stages issued in between.
  constexpr int NX = (BOT ? 1 : 0) + (TOPO > 0 ? 1 : 0);  // x / dy DMA instructions per wave per stage
  constexpr int STEADY = (S - 1) * NST + (S - 2) * (NA + NP + NX);
  static_assert(TOPO <= TOP_MAXO && !(TOPO > 0 && BOTC > 0), "output-layer fusion: top layer only");
  static_assert(!DXOUT || BOT, "dx output belongs to the first-layer fusion");

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int64_t rows = a.rows_per_batch;
  const int64_t rowbase = batch * rows;
  const int col = 32 * wave + r32;

  const bf16* Wb = (const bf16*)a.W + batch * a.w_bstride + (int64_t)col * K;
  bf16x8 wf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) wf[ks] = *(const bf16x8*)(Wb + 16 * ks + 8 * h);

  // BOT pass mapping: thread owns features 8 cth .. +8 of rows rth + 16 q
  constexpr int CB = BOT ? BOTC : 1;
  const int cth = tid & 31, rth = tid >> 5;
  float w0r[8][CB], bdw[8][CB], bdb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bdb[e] = 0.f;
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      bdw[e][c] = 0.f;
      w0r[e][c] = 0.f;
    }
  }
  if constexpr (BOT) {
    const float* W0 = a.bot.W0 + batch * a.bot.w0_bstride;
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int c = 0; c < CB; ++c) w0r[e][c] = W0[(8 * cth + e) * BOTC + c];
  }
  // REC: this lane's epilogue column of W_0 and b_0
  float wcol[CB], bcol0 = 0.f;
#pragma unroll
  for (int c = 0; c < CB; ++c) wcol[c] = 0.f;
  if constexpr (REC) {
    const float* W0 = a.bot.W0 + batch * a.bot.w0_bstride;
#pragma unroll
    for (int c = 0; c < CB; ++c) wcol[c] = W0[col * BOTC + c];
    bcol0 = a.bot.b0[batch * a.bot.b0_bstride + col];
  }

  // TOP: this thread's W_L columns for the in-place dZ_top pass (chunk tid % 32 is fixed)
  float twl[TOPO > 0 ? TOPO : 1][8];
  const float dys = (TOPO > 0 && a.top.dy_scale) ? *a.top.dy_scale : 1.f;
  if constexpr (TOPO > 0) {
#pragma unroll
    for (int o = 0; o < TOPO; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) twl[o][e] = a.top.WL[batch * a.top.wl_bstride + (int64_t)o * K + 8 * (tid & 31) + e] * a.w0;
  }

  auto a_off = [&](int r, int c) -> int { return r * K * 2 + ((c ^ (r & SMASK)) << 4); };
  auto dma = [&](int64_t t, int st) {
    char* base = smem + st * STAGE;
    const int64_t m0 = t * BM;
    const void* asrc = TOPO > 0 ? a.top.Ptop : a.A;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
      const int i = wave + 8 * k;
      const int u = i * 64 + lane;
      const int r = u / A_CPR, p = u - r * A_CPR;
      const int c = p ^ (r & SMASK);
      const int64_t row = min(m0 + r, rows - 1);
      __builtin_amdgcn_global_load_lds((const void*)((const bf16*)asrc + (rowbase + row) * K + c * 8),
                                       (lds_void*)(base + i * 1024), 16, 0, 0);
    }
    if constexpr (TOPO > 0) {
      // dy rows [m0, m0 + BM): BM*O floats; wave w moves bytes [16 O w, 16 O (w + 1)) (O lanes)
      if (lane < TOPO) {
        const int64_t el = min((m0 + rowbase) * TOPO + 4 * (TOPO * wave + lane), (rowbase + rows) * TOPO - 4);
        __builtin_amdgcn_global_load_lds((const void*)(a.top.dy + el),
                                         (lds_void*)(base + A_BYTES + C_BYTES + X_BYTES + 16 * TOPO * wave), 16, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int i = wave + 8 * k;
      const int u = i * 64 + lane;
      const int r = u / C_CPR, c = u - r * C_CPR;
      const int64_t row = min(m0 + r, rows - 1);
      __builtin_amdgcn_global_load_lds((const void*)((const uint16_t*)a.Paux + (rowbase + row) * N + c * 8),
                                       (lds_void*)(base + A_BYTES + i * 1024), 16, 0, 0);
    }
    if constexpr (BOT) {
      // x rows [m0, m0 + BM): BM*C floats; wave w moves bytes [16 C w, 16 C (w + 1)) (C lanes)
      if (lane < BOTC) {
        const int64_t el = min((m0 + rowbase) * BOTC + 4 * (BOTC * wave + lane), (rowbase + rows) * BOTC - 4);
        __builtin_amdgcn_global_load_lds((const void*)(a.bot.x + el),
                                         (lds_void*)(base + A_BYTES + C_BYTES + 16 * BOTC * wave), 16, 0, 0);
      }
    }
  };

  for (int s = 0; s < S - 1; ++s)
    if (s < niter) dma(t0 + s * G, s);

  RingProf prof(a.prof);
  for (int64_t i = 0; i < niter; ++i) {
    const int st = (int)(i % S);
    const int64_t t = t0 + i * G;
    // wait for this stage's DMA (this wave's part), then for every wave's part and for every
    // wave to be done with the stage the next DMA overwrites (consumed in iteration i - 1)
    if (i + S - 2 < niter && i >= S - 1) vm_wait<STEADY>();
    else vm_drain();
    prof.tick(0);
    lds_barrier();
    prof.tick(1);
    if (i + S - 1 < niter) dma(t0 + (i + S - 1) * G, (int)((i + S - 1) % S));
    prof.tick(2);
    char* base = smem + st * STAGE;
    if constexpr (TOPO > 0) {
      // dZ_top = (dy W_L) cos(P_top) w0 over the staged phases, in place (last_bwd's arithmetic)
      const float* gt = (const float*)(base + A_BYTES + C_BYTES + X_BYTES);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int u = tid + 512 * q;
        const int r = u / A_CPR, c = u - r * A_CPR;
        char* p = base + a_off(r, c);
        const u16x8 ph = *(const u16x8*)p;
        float g[TOP_MAXO];
#pragma unroll
        for (int o = 0; o < TOP_MAXO; ++o) g[o] = o < TOPO ? gt[r * TOPO + o] * dys : 0.f;
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float dh = g[0] * twl[0][e];
#pragma unroll
          for (int o = 1; o < TOPO; ++o) dh = fmaf(g[o], twl[o][e], dh);
          v[e] = (bf16)(dh * PT::cosp(ph[e]));
        }
        *(bf16x8*)p = v;
      }
      lds_barrier();
    }
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 af = *(const bf16x8*)(base + a_off(r32, 2 * ks + h));
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, wf[ks], acc, 0, 0, 0);
    }
    // epilogue 1: dZ_{l-1} = acc * cos(P) * w0, in place over the staged P tile
    uint16_t* Cs = (uint16_t*)(base + A_BYTES);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int rl = (e & 3) + 8 * (e >> 2) + 4 * h;
      uint16_t* dst = Cs + rl * N + col;
      uint16_t ph;
      if constexpr (REC) {
        const float* xr = (const float*)(base + A_BYTES + C_BYTES) + rl * BOTC;
        float z = 0.f;
#pragma unroll
        for (int c = 0; c < CB; ++c) z = fmaf(xr[c], wcol[c], z);
        ph = PT::encz(z, bcol0, a.w0);
      } else {
        ph = *dst;
      }
      const float c = PT::cosp(ph);
      *dst = __builtin_bit_cast(uint16_t, (bf16)((acc[e] * c) * a.w0));
    }
    prof.tick(3);
    lds_barrier();
    prof.tick(4);
    const int64_t m0 = t * BM;
    if constexpr (!BOT) {
      // epilogue 2: coalesced 16-byte stores
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int u = tid + 512 * q;
        const int r = u / C_CPR, c = u - r * C_CPR;
        const u16x8 v = *(const u16x8*)(base + A_BYTES + (r * N + c * 8) * 2);
        if (m0 + r < rows) *(u16x8*)((uint16_t*)a.C + (rowbase + m0 + r) * N + c * 8) = v;
      }
    } else {
      // first layer: dW_0 += dZ_0^T x, db_0 += sum dZ_0, dx = dZ_0 W_0 (32-lane row reduction)
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int r = rth + 16 * q;
        const bf16x8 dv = *(const bf16x8*)(base + A_BYTES + (r * N + 8 * cth) * 2);
        const float* xs = (const float*)(base + A_BYTES + C_BYTES) + r * BOTC;
        float xv[CB];
#pragma unroll
        for (int c = 0; c < CB; ++c) xv[c] = xs[c];
        const bool valid = m0 + r < rows;
        float dxp[CB];
#pragma unroll
        for (int c = 0; c < CB; ++c) dxp[c] = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dz = valid ? (float)dv[e] : 0.f;
          bdb[e] += dz;
#pragma unroll
          for (int c = 0; c < CB; ++c) {
            bdw[e][c] = fmaf(dz, xv[c], bdw[e][c]);
            dxp[c] = fmaf(dz, w0r[e][c], dxp[c]);
          }
        }
        if constexpr (DXOUT) {
#pragma unroll
          for (int c = 0; c < CB; ++c)
#pragma unroll
            for (int off = 16; off >= 1; off >>= 1) dxp[c] += __shfl_xor(dxp[c], off, 32);
          typedef float fvec __attribute__((ext_vector_type(BOTC == 3 ? 4 : BOTC)));
          if (cth == 0 && valid) {
            float* dst = (float*)a.C + (rowbase + m0 + r) * BOTC;
            if constexpr (BOTC == 3) {
              dst[0] = dxp[0];
              dst[1] = dxp[1];
              dst[2] = dxp[2];
            } else {
              fvec v;
#pragma unroll
              for (int c = 0; c < CB; ++c) v[c] = dxp[c];
              *(fvec*)dst = v;
            }
          }
        }
      }
    }
    prof.tick(5);
  }
  prof.flush(blockIdx.x);
  if constexpr (BOT) {
    // per-workgroup slab: dW_0 [F0][C] then db_0 [F0], summed over the 16 row slots
    __syncthreads();
    float* red = (float*)smem;  // [16][256 * (C + 1)]
    constexpr int RS = 256 * (CB + 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int f = 8 * cth + e;
#pragma unroll
      for (int c = 0; c < CB; ++c) red[rth * RS + f * BOTC + c] = bdw[e][c];
      red[rth * RS + 256 * BOTC + f] = bdb[e];
    }
    __syncthreads();
    float* part = a.bot.part + slab * a.bot.split_stride + batch * (int64_t)RS;
    for (int idx = tid; idx < RS; idx += 512) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) sum += red[k * RS + idx];
      part[idx] = sum;
    }
  }
}

// dx_ring body for the layers without the first-layer fusion (middle and top). The MFMA runs
// transposed, dZ_{l-1}^T = W_l^T . dZ_l^T, so each lane holds one row's 4 consecutive output
// features per accumulator group: the cos(P) epilogue reads the phases and writes the result as
// 8-byte LDS accesses in place over the staged P tile, and the wave stores its own 32 columns of
// the tile from there (wave-local: no barrier between the MFMAs and the stores). Loads are LDS-DMA
// through buffer resources bounded by the tile's valid rows (rows past the end arrive as zeros),
// stores are buffer stores bounded the same way. One barrier per tile (two with TOPO).
template <int TOPO>
DEV void dx_ring_body_v2(const NTArgs& a, char* smem, const int64_t t0, const int64_t G, const int64_t niter,
                         const int64_t slab) {
  using PT = Prec<kPrecBF16>;
  constexpr int K = 256, N = 256, BM = RING_BM, S = RING_S;
  constexpr int G_BYTES = TOPO > 0 ? BM * TOPO * 4 : 0;
  constexpr int A_BYTES = BM * K * 2, C_BYTES = BM * N * 2, STAGE = A_BYTES + C_BYTES + G_BYTES;
  static_assert(S * STAGE + 4 * BM * DX_STAGE_ROW == dx_ring_lds_bytes<0, TOPO>(), "dx_ring LDS size");
  constexpr int NKS = K / 16;
  // the ring's DMA is issued by waves 0..NIO-1 only (4 dZ + 4 P pieces each): waves 4-7 lose the
  // VALU/MFMA arbitration to their SIMD partners, and the issue cost lands where the barrier
  // wait is (measured: the partners wait for them at every barrier)
  constexpr int NIO = 4;
  constexpr int NPC = 16 / NIO;                        // 1 KB pieces per image per I/O wave
  constexpr int NDMA = 2 * NPC + (TOPO > 0 ? 1 : 0);  // VMEM loads per I/O wave per stage
  constexpr int NST = 2;                               // buffer stores per wave per tile
  // VMEM ops issued after DMA(i) when iteration i waits for it: stores of tiles i-3..i-1 and the
  // DMAs of tiles i+1, i+2
  constexpr int STEADY = 3 * NST + 2 * NDMA;
  static_assert(TOPO <= TOP_MAXO, "output-layer fusion: O <= 2");

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int64_t rows = a.rows_per_batch;
  const int64_t rowbase = batch * rows;

  // W_l^T slice of this wave's 32 output features: the MFMA A operand, in registers
  const bf16* Wb = (const bf16*)a.W + batch * a.w_bstride + (int64_t)(32 * wave + r32) * K;
  bf16x8 wf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) wf[ks] = *(const bf16x8*)(Wb + 16 * ks + 8 * h);

  // TOPO: this thread's W_L columns for the in-place dZ_top pass (chunk tid % 32 is fixed)
  float twl[TOPO > 0 ? TOPO : 1][8];
  const float dys = (TOPO > 0 && a.top.dy_scale) ? *a.top.dy_scale : 1.f;
  if constexpr (TOPO > 0) {
#pragma unroll
    for (int o = 0; o < TOPO; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) twl[o][e] = a.top.WL[batch * a.top.wl_bstride + (int64_t)o * K + 8 * (tid & 31) + e] * a.w0;
  }

  // both images: row r (512 B), 16-byte chunk c stored at chunk c ^ (r & 15)
  const uint32_t boff0 = r32 * 512 + 16 * (h ^ (r32 & 15));  // B fragment of K step 0 (ring_chain)
  auto img_off = [](int r, int c) -> int { return r * 512 + ((c ^ (r & 15)) << 4); };
  uint32_t dvoff[NPC];  // DMA piece j: rows 2 i, 2 i + 1 (i = wave + NIO j)
#pragma unroll
  for (int j = 0; j < NPC; ++j) {
    const int i = wave + NIO * j;
    const int r = 2 * i + (lane >> 5), p = lane & 31;
    dvoff[j] = r * 512 + 16 * (p ^ (r & 15));
  }
  // epilogue: group g = this lane's row r32, features 32 w + 8 g + 4 h .. +4 (chunk 4 w + g, half h)
  int eoff[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) eoff[g] = A_BYTES + img_off(r32, 4 * wave + g) + 8 * h;
  // store pass: lane's 16-byte pieces q = lane + 64 j -> row q / 4, chunk 4 w + q % 4
  int soff[2], goff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int qd = lane + 64 * j, r = qd >> 2, c = 4 * wave + (qd & 3);
    soff[j] = A_BYTES + img_off(r, c);
    goff[j] = r * 512 + 16 * c;
  }

  // late half (waves 4-7): private staging of the wave's 32 x 32 output tile, rows of 80 B
  char* stg = smem + S * STAGE + (wave & 3) * BM * DX_STAGE_ROW;
  auto nval = [&](int64_t t) -> int64_t {
    const int64_t n = rows - t * BM;
    return n < BM ? n : BM;
  };
  // DMA of tile t into slot st, in parts (0: dZ / P_top pieces + dy, 1: P pieces) so the main
  // loop can spread the issue of the next stage's pieces between its MFMAs
  auto dma_part = [&](int64_t t, int st, int part) {
    char* base = smem + st * STAGE;
    const int64_t m0 = rowbase + t * BM, nv = nval(t);
    if (part == 0) {
      const __amdgpu_buffer_rsrc_t rA = make_rsrc((const bf16*)(TOPO > 0 ? a.top.Ptop : a.A) + m0 * K, nv * K * 2);
#pragma unroll
      for (int j = 0; j < NPC; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(base + (wave + NIO * j) * 1024), 16, dvoff[j], 0, 0,
                                                 0);
      if constexpr (TOPO > 0) {
        // dy rows of the tile: BM * O floats; I/O wave w moves bytes [16 GL w, 16 GL (w + 1))
        constexpr int GL = 8 * TOPO / NIO;
        const __amdgpu_buffer_rsrc_t rG = make_rsrc(a.top.dy + m0 * TOPO, nv * TOPO * 4);
        if (lane < GL)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rG, (lds_void*)(base + A_BYTES + C_BYTES + 16 * GL * wave), 16,
                                                   16 * (GL * wave + lane), 0, 0, 0);
      }
    } else {
      const __amdgpu_buffer_rsrc_t rP = make_rsrc((const uint16_t*)a.Paux + m0 * N, nv * N * 2);
#pragma unroll
      for (int j = 0; j < NPC; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rP, (lds_void*)(base + A_BYTES + (wave + NIO * j) * 1024), 16,
                                                 dvoff[j], 0, 0, 0);
    }
  };
  auto dma = [&](int64_t t, int st) {
    dma_part(t, st, 0);
    dma_part(t, st, 1);
  };

  // epilogue of tile t held in slot st with accumulator acc: dZ_{l-1} = acc cos(P) w0 (4 features
  // per group, in place over the staged P tile), then the wave's 32 columns to dZ_{l-1} rows
  auto epilogue = [&](int64_t t, int st, const f32x16& acc) {
    char* base = smem + st * STAGE;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      char* pp = base + eoff[g];
      const u16x4 ph = *(const u16x4*)pp;
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (bf16)((acc[4 * g + e] * PT::cosp(ph[e])) * a.w0);
      *(bf16x4*)pp = v;
    }
    const __amdgpu_buffer_rsrc_t rC = make_rsrc((const bf16*)a.C + (rowbase + t * BM) * N, nval(t) * N * 2);
#pragma unroll
    for (int j = 0; j < NST; ++j) {
      const u32x4_t v = *(const u32x4_t*)(base + soff[j]);
      store_b128_gemm(v, rC, goff[j]);
    }
  };

  // TOPO: dZ_top = (dy W_L) cos(P_top) w0 over the staged phases of slot st, in place
  // (last_bwd's arithmetic); run for tile i + 1 right after tile i's MFMAs, so no barrier
  // separates it from the MFMAs that read it (the next iteration's barrier publishes it)
  auto top_pass = [&](int st) {
    if constexpr (TOPO > 0) {
      char* base = smem + st * STAGE;
      const float* gt = (const float*)(base + A_BYTES + C_BYTES);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int u = tid + 512 * q;
        const int r = u >> 5, c = u & 31;
        char* pp = base + img_off(r, c);
        const u16x8 ph = *(const u16x8*)pp;
        float gg[TOP_MAXO];
#pragma unroll
        for (int o = 0; o < TOP_MAXO; ++o) gg[o] = o < TOPO ? gt[r * TOPO + o] * dys : 0.f;
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float dh = gg[0] * twl[0][e];
#pragma unroll
          for (int o = 1; o < TOPO; ++o) dh = fmaf(gg[o], twl[o][e], dh);
          v[e] = (bf16)(dh * PT::cosp(ph[e]));
        }
        *(bf16x8*)pp = v;
      }
    }
  };
  // TOPO: iteration i waits for DMA(i + 1) (its pass runs in iteration i); issued in iteration
  // i + 2 - S, then followed by the stores of S - 2 iterations and S - 3 DMAs
  constexpr int STEADY_T = (S - 2) * NST + (S - 3) * NDMA;

  // late half: the epilogue of tile t from registers (its accumulator and the 16 phases read
  // before the stage was recycled), staged privately, then the same two 16-byte stores per lane
  auto late_epilogue = [&](int64_t t, const f32x16& acc, const u16x4 (&ph)[4]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (bf16)((acc[4 * g + e] * PT::cosp(ph[g][e])) * a.w0);
      *(bf16x4*)(stg + r32 * DX_STAGE_ROW + 16 * g + 8 * h) = v;
    }
    const __amdgpu_buffer_rsrc_t rC = make_rsrc((const bf16*)a.C + (rowbase + t * BM) * N, nval(t) * N * 2);
#pragma unroll
    for (int j = 0; j < NST; ++j) {
      const int qd = lane + 64 * j;
      const u32x4_t v = *(const u32x4_t*)(stg + (qd >> 2) * DX_STAGE_ROW + 16 * (qd & 3));
      store_b128_gemm(v, rC, goff[j]);
    }
  };

  // Stagger (as dx_ring_body_v2bot): waves 4-7 run each tile's epilogue one tile late, from
  // registers, so on every SIMD one wave's MFMA chain runs beside its partner's epilogue.
  const bool io = wave < NIO;
  if (io)
    for (int s = 0; s < S - 1; ++s)
      if (s < niter) dma(t0 + s * G, s);
  if constexpr (TOPO > 0) {
    if (io) vm_drain();
    lds_barrier();
    if (niter > 0) top_pass(0);
  }

  auto loop = [&](auto late_tag) {
    constexpr bool LATE = decltype(late_tag)::value;
    f32x16 accp;
    u16x4 php[4];
    RingProf prof(a.prof);
    for (int64_t i = 0; i < niter; ++i) {
      const int st = (int)(i % S);
      const int64_t t = t0 + i * G;
      // this stage's DMA (this wave's part) landed; then every wave's part, and every wave is done
      // with the stage the next DMA overwrites (tile i - 1: MFMA reads and its store pass)
      if (io) {
        if constexpr (TOPO > 0) {
          if (i + 1 < niter) {
            if (i >= S - 2 && i + S - 2 < niter) vm_wait<STEADY_T>();
            else vm_drain();
          }
        } else {
          if (i >= S - 1 && i + S - 2 < niter) vm_wait<STEADY>();
          else vm_drain();
        }
      }
      prof.tick(0);
      lds_barrier();
      prof.tick(1);
      // (issuing these pieces between the MFMAs instead measured slower)
      if (io && i + S - 1 < niter) dma(t0 + (i + S - 1) * G, (int)((i + S - 1) % S));
      if constexpr (LATE) {
        if (i > 0) late_epilogue(t - G, accp, php);
      }
      prof.tick(2);
      char* base = smem + st * STAGE;
      // dZ_{l-1}^T (32 features x 32 rows) = W^T slice . dZ_l^T: B fragments = dZ rows from LDS
      const f32x16 acc = ring_chain(wf, lds_addr(base), boff0);
      prof.tick(3);
      if constexpr (TOPO > 0) {
        if (i + 1 < niter) top_pass((int)((i + 1) % S));
      }
      if constexpr (LATE) {
        accp = acc;
#pragma unroll
        for (int g = 0; g < 4; ++g) php[g] = *(const u16x4*)(base + eoff[g]);
      } else {
        epilogue(t, st, acc);
      }
      prof.tick(5);
    }
    if constexpr (LATE) {
      if (niter > 0) late_epilogue(t0 + (niter - 1) * G, accp, php);
    }
    prof.flush(blockIdx.x);
  };
  if (a.stagger && wave >= 4) loop(std::true_type{});
  else loop(std::false_type{});
  (void)slab;
}

// dx_ring body of the bottom hidden layer with the first layer folded in and P_0 rebuilt from x
// (C = BOTC <= 4 inputs). Transposed MFMA as dx_ring_body_v2 (lane (row r32, half h) holds the
// wave's features 32 w + 8 g + 4 h + e in accumulator element 4 g + e). Per tile the epilogue
//   z_0 (revolutions) = one or two f32 MFMAs (32x32x2) with operands W_0 w0/2pi, x and b_0 w0/2pi:
//                       the register-resident forward's layer-0 instructions on the same values,
//                       so the phase is bit-identical to the one its sin() used
//   dZ_0 = bf16((acc cos(fract(z_0))) w0)                       (modules.py:38 chain rule)
//   dx partial = W_0^T dZ_0^T over the wave's 32 features: two bf16 MFMAs whose A operand holds
//                W_0 split into bf16 hi + lo rows (hi rows 0..C-1, lo rows 4..4+C-1), so the
//                product is exact to ~2^-16 of W_0; the dZ_0 fragments are the accumulator
//                elements in order (K step s = elements 8 s .. 8 s + 7)
//   db_0, dW_0 = dZ_0^T x: per-lane VALU sums (reduced over the lanes once, at the end).
// The ring carries dZ_1 and x only (no P image).
// Stagger (MI355X_MICROARCH.md, two waves per SIMD, item 9): waves 4-7 run each tile's epilogue
// one tile late, at the head of the next iteration, keeping the accumulator and the x values in
// registers across the barrier; so on every SIMD one wave's MFMA chain runs beside its partner's
// VALU epilogue instead of both waves contending for the matrix pipe and then for VALU issue.
// Per-lane sums keep their tile order (bit-identical to the unstaggered order). The dx partials
// of tile j (waves 0-3 in iteration j, waves 4-7 in j + 1) sit in Yp[j % 3] and are summed over
// the 8 waves x 2 halves by the dx store pass of iteration j + 2.
template <int BOTC, bool DXOUT>
DEV void dx_ring_body_v2bot(const NTArgs& a, char* smem, const int64_t t0, const int64_t G, const int64_t niter,
                            const int64_t slab) {
  constexpr int K = 256, F0 = 256, BM = RING_BM, S = RING_S, C = BOTC;
  constexpr int NKK = (C + 1) / 2;                // K = 2 steps of the z_0 MFMA
  constexpr int A_BYTES = BM * K * 2, X_BYTES = BM * C * 4, STAGE = A_BYTES + X_BYTES;
  constexpr int YP_BYTES = 3 * 16 * BM * C * 4;  // dx partials [3][wave][half][row][C]
  static_assert(C <= 4, "dx MFMA rows: hi 0..3, lo 4..7");
  static_assert(S * STAGE + YP_BYTES <= dx_ring_lds_bytes<BOTC, 0>(), "dx_ring LDS size");
  constexpr int NKS = K / 16;
  // C <= 2: staggered halves (waves 4-7 run each epilogue one tile late; C = 3, 4: the late
  // copies of acc and x would spill). With the stagger the ring's I/O (DMA issue, vm waits and
  // dx stores) is all done by waves 0-3, which otherwise wait at the barrier for the late half.
  constexpr bool STAG = C <= 2;
  constexpr int NIO = STAG ? 4 : 8;        // waves that issue the DMA and the dx stores
  constexpr int NPC = 16 / NIO;            // dZ_1 pieces (1 KB) per I/O wave per tile
  constexpr int XL = 8 * C / NIO;          // lanes (16 B) of the x piece per I/O wave
  constexpr int SR = BM / NIO;             // dx rows stored per I/O wave
  constexpr int NDMA = NPC + 1;            // dZ_1 pieces + the x piece
  constexpr int NST = DXOUT ? 1 : 0;       // dx stores per I/O wave per tile
  constexpr int STEADY = (S - 1) * NST + (S - 2) * NDMA;
  float* Yp = (float*)(smem + S * STAGE);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int64_t rows = a.rows_per_batch;
  const int64_t rowbase = batch * rows;
  const float k1 = a.w0 * kInv2Pi;
  const int fw = 32 * wave;

  const bf16* Wb = (const bf16*)a.W + batch * a.w_bstride + (int64_t)(fw + r32) * K;
  bf16x8 wf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) wf[ks] = *(const bf16x8*)(Wb + 16 * ks + 8 * h);
  const float* W0 = a.bot.W0 + batch * a.bot.w0_bstride;
  const float* b0 = a.bot.b0 + batch * a.bot.b0_bstride;
  // z_0 MFMA: A lane (i, k) = W_0[fw + i][2 kk + k] w0/2pi, C = b_0 w0/2pi of the lane's features
  float w0a[NKK];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) w0a[kk] = 2 * kk + h < C ? W0[(fw + r32) * C + 2 * kk + h] * k1 : 0.f;
  f32x16 zb;
#pragma unroll
  for (int v = 0; v < 16; ++v) zb[v] = b0[fw + 8 * (v >> 2) + 4 * h + (v & 3)] * k1;
  // dx MFMA: A lane (i, kh) for K step s holds W_0 (hi for i < C, lo for 4 <= i < 4 + C) at the
  // features f(s, 8 kh + m) = fw + 8 (2 s + m / 4) + 4 kh + m % 4 of the B fragment's K order
  bf16x8 dxa[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int f = fw + 8 * (2 * s + (m >> 2)) + 4 * h + (m & 3);
      const int c = r32 & 3;
      bf16 v = (bf16)0.f;
      if (r32 < 8 && c < C) {
        const float w = W0[f * C + c];
        const bf16 hi = (bf16)w;
        v = r32 < 4 ? hi : (bf16)(w - (float)hi);
      }
      dxa[s][m] = v;
    }
  float dwacc[16][C], dbacc[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    dbacc[u] = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) dwacc[u][c] = 0.f;
  }

  const uint32_t boff0 = r32 * 512 + 16 * (h ^ (r32 & 15));  // B fragment of K step 0 (ring_chain)
  auto img_off = [](int r, int c) -> int { return r * 512 + ((c ^ (r & 15)) << 4); };
  uint32_t dvoff[NPC];  // DMA piece q = wave + NIO j: rows 2 q, 2 q + 1
#pragma unroll
  for (int j = 0; j < NPC; ++j) {
    const int q = wave + NIO * j;
    const int r = 2 * q + (lane >> 5), p = lane & 31;
    dvoff[j] = r * 512 + 16 * (p ^ (r & 15));
  }
  auto nval = [&](int64_t t) -> int64_t {
    const int64_t n = rows - t * BM;
    return n < BM ? n : BM;
  };
  auto dma = [&](int64_t t, int st) {
    char* base = smem + st * STAGE;
    const int64_t m0 = rowbase + t * BM, nv = nval(t);
    const __amdgpu_buffer_rsrc_t rA = make_rsrc((const bf16*)a.A + m0 * K, nv * K * 2);
    const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.bot.x + m0 * C, nv * C * 4);
#pragma unroll
    for (int j = 0; j < NPC; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void*)(base + (wave + NIO * j) * 1024), 16, dvoff[j], 0, 0,
                                               0);
    // x rows of the tile: BM * C floats; I/O wave w moves bytes [16 XL w, 16 XL (w + 1)) (XL lanes)
    if (lane < XL)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)(base + A_BYTES + 16 * XL * wave), 16,
                                               16 * (XL * wave + lane), 0, 0, 0);
  };
  // dx of tile t from the partials in Yp[buf]: I/O wave w stores rows SR w .. SR (w + 1) - 1
  auto dx_store = [&](int64_t t, int buf) {
    if constexpr (DXOUT) {
      const int idx = SR * C * wave + lane;  // (row, c) element of the tile, row-major
      float v = 0.f;
      if (lane < SR * C) {
#pragma unroll
        for (int w = 0; w < 16; ++w) v += Yp[(buf * 16 + w) * BM * C + idx];
      }
      const __amdgpu_buffer_rsrc_t rD = make_rsrc(a.C ? (float*)a.C + (rowbase + t * BM) * C : nullptr,
                                                  a.C ? nval(t) * C * 4 : 0);
      if (lane < SR * C) store_b32_gemm(__builtin_bit_cast(uint32_t, v), rD, idx * 4);
    }
  };

  // epilogue of tile j from its accumulator and x values (see the header)
  auto epilogue = [&](const f32x16& acc, const float (&xb)[NKK], const float (&xv)[C], int64_t j) {
    f32x16 z = zb;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) z = __builtin_amdgcn_mfma_f32_32x32x2f32(w0a[kk], xb[kk], z, 0, 0, 0);
    bf16x8 dzb[2];
#pragma unroll
    for (int v = 0; v < 16; ++v)
      dzb[v >> 3][v & 7] = (bf16)((acc[v] * __builtin_amdgcn_cosf(__builtin_amdgcn_fractf(z[v]))) * a.w0);
    if constexpr (DXOUT) {
      f32x16 dd;
#pragma unroll
      for (int e = 0; e < 16; ++e) dd[e] = 0.f;
      dd = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dxa[0], dzb[0], dd, 0, 0, 0);
      dd = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dxa[1], dzb[1], dd, 0, 0, 0);
      float* yp = Yp + (((int)(j % 3) * 8 + wave) * 2 + h) * BM * C + r32 * C;
#pragma unroll
      for (int c = 0; c < C; ++c) yp[c] = dd[c];
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const float dz = (float)dzb[v >> 3][v & 7];
      dbacc[v] += dz;
#pragma unroll
      for (int c = 0; c < C; ++c) dwacc[v][c] = fmaf(dz, xv[c], dwacc[v][c]);
    }
  };

  if (wave < NIO)
    for (int s = 0; s < S - 1; ++s)
      if (s < niter) dma(t0 + s * G, s);

  auto loop = [&](auto late_tag) {
    constexpr bool LATE = decltype(late_tag)::value;
    f32x16 accp;
    float xbp[NKK], xvp[C];
    RingProf prof(a.prof);
    for (int64_t i = 0; i < niter; ++i) {
      const int st = (int)(i % S);
      // counted wait: from iteration S + 1 on, S - 1 dx stores and S - 2 DMAs follow DMA(i)
      if constexpr (!LATE) {
        if (i >= S + 1 && i + S - 2 < niter) vm_wait<STEADY>();
        else vm_drain();
      }
      prof.tick(0);
      lds_barrier();  // DMA(i) of every I/O wave landed; also publishes tile i - 2's dx partials
      prof.tick(1);
      if constexpr (!LATE) {
        if (i + S - 1 < niter) dma(t0 + (i + S - 1) * G, (int)((i + S - 1) % S));
        if (i > 1) dx_store(t0 + (i - 2) * G, (int)((i - 2) % 3));
      }
      prof.tick(2);
      if constexpr (LATE) {
        if (i > 0) epilogue(accp, xbp, xvp, i - 1);
      }
      prof.tick(3);
      char* base = smem + st * STAGE;
      const float* xr = (const float*)(base + A_BYTES) + r32 * C;
      float xb[NKK], xv[C];
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) xb[kk] = 2 * kk + h < C ? xr[2 * kk + h] : 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) xv[c] = xr[c];
      const f32x16 acc = ring_chain(wf, lds_addr(base), boff0);
      prof.tick(4);
      if constexpr (LATE) {
        accp = acc;
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) xbp[kk] = xb[kk];
#pragma unroll
        for (int c = 0; c < C; ++c) xvp[c] = xv[c];
      } else {
        epilogue(acc, xb, xv, i);
      }
      prof.tick(5);
    }
    prof.flush(blockIdx.x);
    if constexpr (LATE) {
      if (niter > 0) epilogue(accp, xbp, xvp, niter - 1);
    }
  };
  if constexpr (STAG) {
    if (wave >= 4) loop(std::true_type{});
    else loop(std::false_type{});
  } else {
    loop(std::false_type{});
  }
  if (niter > 0) {
    lds_barrier();
    if (wave < NIO) {
      if (niter > 1) dx_store(t0 + (niter - 2) * G, (int)((niter - 2) % 3));
      dx_store(t0 + (niter - 1) * G, (int)((niter - 1) % 3));
    }
  }
  // per-workgroup slab: dW_0 [F0][C] then db_0 [F0]: sums over the 32 lanes of each half-wave
#pragma unroll
  for (int u = 0; u < 16; ++u) {
#pragma unroll
    for (int off = 16; off >= 1; off >>= 1) {
      dbacc[u] += __shfl_xor(dbacc[u], off, 32);
#pragma unroll
      for (int c = 0; c < C; ++c) dwacc[u][c] += __shfl_xor(dwacc[u][c], off, 32);
    }
  }
  if (r32 == 0) {
    float* part = a.bot.part + slab * a.bot.split_stride + batch * (int64_t)(F0 * (C + 1));
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int f = fw + 8 * g + 4 * h + e, u = 4 * g + e;
#pragma unroll
        for (int c = 0; c < C; ++c) part[f * C + c] = dwacc[u][c];
        part[F0 * C + f] = dbacc[u];
      }
  }
}

template <int BOTC, bool DXOUT, bool REC = false, int TOPO = 0>
DEV void dx_ring_body(const NTArgs& a, char* smem, const int64_t t0, const int64_t G, const int64_t niter,
                      const int64_t slab) {
  if constexpr (BOTC == 0) dx_ring_body_v2<TOPO>(a, smem, t0, G, niter, slab);
  else if constexpr (REC) dx_ring_body_v2bot<BOTC, DXOUT>(a, smem, t0, G, niter, slab);
  else dx_ring_body_v1<BOTC, DXOUT, REC, TOPO>(a, smem, t0, G, niter, slab);
}

template <int BOTC, bool DXOUT, bool REC = false, int TOPO = 0>
__global__ __launch_bounds__(512) void dx_ring_bf16_kernel(NTArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[dx_ring_lds_bytes<BOTC, TOPO>()];
  const int64_t ntiles = (a.rows_per_batch + RING_BM - 1) / RING_BM;
  const int64_t t0 = blockIdx.x, G = gridDim.x;
  const int64_t niter = t0 < ntiles ? (ntiles - t0 + G - 1) / G : 0;
  dx_ring_body<BOTC, DXOUT, REC, TOPO>(a, smem, t0, G, niter, blockIdx.x);
}

}  // namespace siren

namespace siren {

// ------------------------------------------------------------------------------------------
// dw_ring: the 256 x 256 weight-gradient layer, dW_l = dZ_l^T sin(P_{l-1}), db_l = sum dZ_l,
// one 256 x 256 fp32 partial per workgroup over a contiguous row range (split-K; 128 accumulator
// registers per lane: wave w owns dW rows [64 (w & 3), +64) x cols [128 (w >> 2), +128)).
// 32-row chunks of dZ and P stream through a 4-stage LDS ring by DMA (16-byte chunks XOR-
// swizzled by 4 (row & 3), which keeps the transposing ds_read_b64_tr_b16 fragment reads
// conflict-free); each stage's phases are turned into bf16 sin(P) in place, then 16 MFMAs per
// wave per stage. Counted waits keep three stages (96 KB per CU) in flight.
// ------------------------------------------------------------------------------------------
// RECC > 0: layer 1 with P_0 not kept by the forward: the x tile (RECC inputs) rides in the ring
// instead of P_0, and the convert pass rebuilds H_0 = sin(fract(z_0)) from x and the prescaled
// W_0 w0/2pi, b_0 w0/2pi (the register-resident forward's layer-0 arithmetic, exact fp32 phase).
// TOPO > 0: the top hidden layer with the output layer folded in (outermost_linear, O = TOPO): the
// ring carries P_top (in the dZ image) and the dy tile; the convert pass forms dZ_top in place
// (last_bwd_kernel's arithmetic) and sums the output layer's dW_L = dy^T sin(P_top), db_L = sum dy
// into per-workgroup slabs (a.top.partL).
template <int RECC, int TOPO>
constexpr int dw_ring_lds_bytes() {
  return RING_S * (32 * 256 * 2 * 2 + (RECC > 0 ? 32 * RECC * 4 : 0) + (TOPO > 0 ? 32 * TOPO * 4 : 0));
}

// Rows [r_begin, r_end) of weight set blockIdx.y into partial slab `split`.
//
// Loads are LDS-DMA through raw buffer resources that span exactly this row range, so rows past
// r_end arrive as zeros (dZ = 0: no contribution to dW, db or the output-layer sums) and no lane
// ever tests a row bound. Per chunk and lane, VALU work is the convert pass alone: every LDS
// address is a per-lane base fixed at entry plus the stage base plus an immediate offset.
template <int RECC = 0, int TOPO = 0>
DEV void dw_ring_body(const TNArgs& a, char* smem, const int64_t r_begin, const int64_t r_end, const int64_t split) {
  using PT = Prec<kPrecBF16>;
  constexpr int M = 256, N = 256, KC = 32, S = RING_S;
  constexpr int X_BYTES = RECC > 0 ? KC * RECC * 4 : 0;
  constexpr int G_BYTES = TOPO > 0 ? KC * TOPO * 4 : 0;
  constexpr int D_BYTES = KC * M * 2, P_BYTES = KC * N * 2, STAGE = D_BYTES + P_BYTES + X_BYTES + G_BYTES;
  static_assert(S * STAGE == dw_ring_lds_bytes<RECC, TOPO>(), "dw_ring LDS size");
  // the ring's DMA is issued by waves 0..NIO-1 only (see dx_ring_body_v2)
  constexpr int NIO = 4;
  constexpr int NPC = 16 / NIO;                      // 1 KB pieces per image per I/O wave
  constexpr int ND = NPC + (TOPO > 0 ? 1 : 0);       // DMA per I/O wave per stage: dZ (or P_top) (+ dy)
  constexpr int NP = RECC > 0 ? 1 : NPC;             // P_{l-1} (or x)
  constexpr int NDMA = ND + NP;
  static_assert(!(RECC > 0 && TOPO > 0), "one hidden layer: the plain output-layer path");

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;
  const int64_t batch = blockIdx.y;
  const int64_t row0 = batch * a.rows_per_batch + r_begin;
  const int64_t nrows = r_end > r_begin ? r_end - r_begin : 0;
  const int64_t nchunk = (nrows + KC - 1) / KC;

  const __amdgpu_buffer_rsrc_t rD =
      make_rsrc((const bf16*)(TOPO > 0 ? a.top.Ptop : a.D) + row0 * M, nrows * M * 2);
  const __amdgpu_buffer_rsrc_t rP =
      RECC > 0 ? make_rsrc((const float*)a.P + row0 * (RECC > 0 ? RECC : 1), nrows * (RECC > 0 ? RECC : 1) * 4)
               : make_rsrc((const uint16_t*)a.P + row0 * N, nrows * N * 2);
  const __amdgpu_buffer_rsrc_t rG =
      TOPO > 0 ? make_rsrc(a.top.dy + row0 * (TOPO > 0 ? TOPO : 1), nrows * (TOPO > 0 ? TOPO : 1) * 4) : rD;

  // 16-byte chunk c of row r sits at chunk c ^ 4 (r & 3): the four rows of a transposing read
  // (4 consecutive chunks each) then fall on four disjoint bank groups
  auto swz = [](int r, int c) -> int { return c ^ (4 * (r & 3)); };
  // DMA piece j of a 32-row image: rows 2 i, 2 i + 1 (i = wave + 8 j), lane -> (row, chunk)
  uint32_t dvoff[NPC];
#pragma unroll
  for (int j = 0; j < NPC; ++j) {
    const int i = wave + NIO * j;
    const int r = 2 * i + (lane >> 5), p = lane & 31;
    dvoff[j] = r * 512 + 16 * swz(r, p);
  }
  auto dma = [&](int64_t k, int st) {
    char* base = smem + st * STAGE;
    const uint32_t cb = (uint32_t)(k * KC * 512);  // the chunk's first byte in a 512-byte-row tensor
#pragma unroll
    for (int j = 0; j < NPC; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rD, (lds_void*)(base + (wave + NIO * j) * 1024), 16, dvoff[j] + cb, 0,
                                               0, 0);
    if constexpr (TOPO > 0) {
      // dy rows of the chunk: KC * O floats; I/O wave w moves bytes [16 GL w, 16 GL (w + 1))
      constexpr int GL = 8 * TOPO / NIO;
      if (lane < GL)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rG, (lds_void*)(base + D_BYTES + P_BYTES + X_BYTES + 16 * GL * wave),
                                                 16, (uint32_t)(k * KC * TOPO * 4) + 16 * (GL * wave + lane), 0, 0, 0);
    }
    if constexpr (RECC > 0) {
      constexpr int XL = 8 * RECC / NIO;
      if (lane < XL)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rP, (lds_void*)(base + D_BYTES + P_BYTES + 16 * XL * wave), 16,
                                                 (uint32_t)(k * KC * RECC * 4) + 16 * (XL * wave + lane), 0, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < NPC; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rP, (lds_void*)(base + D_BYTES + (wave + NIO * j) * 1024), 16,
                                                 dvoff[j] + cb, 0, 0, 0);
    }
  };

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
  // db: the convert pass thread owns columns 8 * (tid & 31) .. +8 of rows tid/32 + 16 q
  const int cth = tid & 31, rth = tid >> 5;
  float dbacc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) dbacc[e] = 0.f;
  // RECC: W_0 rows and b_0 of this thread's 8 features
  constexpr int CR = RECC > 0 ? RECC : 1;
  float w0r[8][CR], b0r[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    b0r[e] = 0.f;
#pragma unroll
    for (int c = 0; c < CR; ++c) w0r[e][c] = 0.f;
  }
  // TOPO: W_L columns of this thread's chunk, dW_L / db_L sums
  constexpr int TO = TOPO > 0 ? TOPO : 1;
  float twl[TO][8], tdw[TO][8], tdb[TO];
  const float dys = (TOPO > 0 && a.top.dy_scale) ? *a.top.dy_scale : 1.f;
#pragma unroll
  for (int o = 0; o < TO; ++o) {
    tdb[o] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      tdw[o][e] = 0.f;
      twl[o][e] = TOPO > 0 ? a.top.WL[batch * a.top.wl_bstride + (int64_t)o * M + 8 * cth + e] * a.w0 : 0.f;
    }
  }
  if constexpr (RECC > 0) {
    const float* W0 = a.rec_W0 + batch * a.rec_w0_bstride;
    const float* b0 = a.rec_b0 + batch * a.rec_b0_bstride;
    const float k1 = a.w0 * kInv2Pi;  // operands in revolutions, as the forward's layer 0
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      b0r[e] = b0[8 * cth + e] * k1;
#pragma unroll
      for (int c = 0; c < CR; ++c) w0r[e][c] = W0[(8 * cth + e) * RECC + c] * k1;
    }
  }

  // convert pass, piece qq of the chunk in slot st: P -> bf16 sin(P) in place; db from the same
  // rows; TOPO: dZ_top in place and the output-layer sums (rows past the range are all zeros)
  const int coff = rth * 512 + swz(rth, cth) * 16;  // piece 1: + 16 rows = + 8192
  auto convert = [&](int st, int qq) {
    char* Db = smem + st * STAGE;
    char* Pb = Db + D_BYTES;
    const int r = rth + 16 * qq;
    const int off = coff + 8192 * qq;
    bf16x8 hv;
    if constexpr (RECC > 0) {
      // H_0 = sin(fract(z_0)), z_0 in revolutions from the prescaled operands (fma chain over the
      // inputs from the bias, the order of the forward's f32 MFMA)
      const float* xr = (const float*)(Pb + P_BYTES) + r * RECC;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float z = b0r[e];
#pragma unroll
        for (int c = 0; c < CR; ++c) z = fmaf(xr[c], w0r[e][c], z);
        hv[e] = (bf16)__builtin_amdgcn_sinf(__builtin_amdgcn_fractf(z));
      }
    } else {
      const u16x8 ph = *(const u16x8*)(Pb + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) hv[e] = (bf16)PT::sinp(ph[e]);
    }
    *(bf16x8*)(Pb + off) = hv;
    if constexpr (TOPO > 0) {
      const float* gt = (const float*)(Pb + P_BYTES + X_BYTES) + r * TOPO;
      const u16x8 pt = *(const u16x8*)(Db + off);
      float gg[TOP_MAXO];
#pragma unroll
      for (int o = 0; o < TOP_MAXO; ++o) gg[o] = o < TOPO ? gt[o] * dys : 0.f;
      bf16x8 dz;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float dh = gg[0] * twl[0][e];
#pragma unroll
        for (int o = 1; o < TO; ++o) dh = fmaf(gg[o], twl[o][e], dh);
        dz[e] = (bf16)(dh * PT::cosp(pt[e]));
        const float sv = PT::sinp(pt[e]);
#pragma unroll
        for (int o = 0; o < TO; ++o) tdw[o][e] = fmaf(gg[o], sv, tdw[o][e]);
      }
      *(bf16x8*)(Db + off) = dz;
      if (cth == 0) {
#pragma unroll
        for (int o = 0; o < TO; ++o) tdb[o] += gg[o];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) dbacc[e] += (float)dz[e];
    } else {
      const bf16x8 dv = *(const bf16x8*)(Db + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) dbacc[e] += (float)dv[e];
    }
  };

  // per-lane bases of the transposing fragment reads (bytes within a stage): K step 1 = + 16 rows
  // (+ 8192), the upper 4 rows of a read pair = + 2048
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p = t & 3;
  uint32_t abase[2], bbase[4];
  {
    const int nb = 8 * (g >> 1) + q;
#pragma unroll
    for (int bm = 0; bm < 2; ++bm) {
      const int c = 64 * wm + 32 * bm + 16 * (g & 1) + 4 * p;
      abase[bm] = nb * 512 + swz(nb, c >> 3) * 16 + (c & 7) * 2;
    }
#pragma unroll
    for (int bn = 0; bn < 4; ++bn) {
      const int c = 128 * wn + 32 * bn + 16 * (g & 1) + 4 * p;
      bbase[bn] = D_BYTES + nb * 512 + swz(nb, c >> 3) * 16 + (c & 7) * 2;
    }
  }
  const uint32_t smem_lds = lds_addr(smem);

  const bool io = wave < NIO;
  if (io)
    for (int s = 0; s < S - 1; ++s)
      if (s < nchunk) dma(s, s);

  // The convert pass of chunk k + 1 runs beside the MFMAs of chunk k (different slots); one
  // barrier per chunk. Slots in use at iteration k: k (MFMA), k + 1 (convert); DMAs k + 2, k + 3
  // in flight (issued two iterations ahead).
  if (nchunk > 0) {
    if (!io) {
    } else if (nchunk >= 3) vm_wait<2 * NDMA>();
    else if (nchunk == 2) vm_wait<NDMA>();
    else vm_drain();
    lds_barrier();
    convert(0, 0);
    convert(0, 1);
  }
  RingProf prof(a.prof);
  for (int64_t k = 0; k < nchunk; ++k) {
    const int st = (int)(k % S);
    const bool next = k + 1 < nchunk;
    // DMA(k + 1) landed (issued after it: DMA(k + 2), if any)
    if (next && io) {
      if (k + 2 < nchunk) vm_wait<NDMA>();
      else vm_drain();
    }
    prof.tick(0);
    lds_barrier();  // convert(k) visible, DMA(k + 1) visible, MFMA(k - 1) done with slot k - 1
    prof.tick(1);
    if (io && k + S - 1 < nchunk) dma(k + S - 1, (int)((k + S - 1) % S));
    prof.tick(2);
    const int stn = (int)((k + 1) % S);
    const uint32_t sb = smem_lds + st * STAGE;
    const uint32_t va0 = sb + abase[0], va1 = sb + abase[1];
    const uint32_t vb0 = sb + bbase[0], vb1 = sb + bbase[1], vb2 = sb + bbase[2], vb3 = sb + bbase[3];
    // both K steps' fragment reads up front (24 transposing reads), counted waits per step
    TrFrag fa[2][2], fb[2][4];
#define SIREN_TR(F, V, OFF)          \
  tr16_read<(OFF)>((F).lo, V);       \
  tr16_read<(OFF) + 2048>((F).hi, V);
    SIREN_TR(fa[0][0], va0, 0) SIREN_TR(fa[0][1], va1, 0)
    SIREN_TR(fb[0][0], vb0, 0) SIREN_TR(fb[0][1], vb1, 0) SIREN_TR(fb[0][2], vb2, 0) SIREN_TR(fb[0][3], vb3, 0)
    SIREN_TR(fa[1][0], va0, 8192) SIREN_TR(fa[1][1], va1, 8192)
    SIREN_TR(fb[1][0], vb0, 8192) SIREN_TR(fb[1][1], vb1, 8192) SIREN_TR(fb[1][2], vb2, 8192) SIREN_TR(fb[1][3], vb3, 8192)
#undef SIREN_TR
    static_assert(KC / 16 == 2, "two K steps per chunk");
    asm volatile("s_waitcnt lgkmcnt(12)"
                 : "+v"(fa[0][0].lo), "+v"(fa[0][0].hi), "+v"(fa[0][1].lo), "+v"(fa[0][1].hi), "+v"(fb[0][0].lo),
                   "+v"(fb[0][0].hi), "+v"(fb[0][1].lo), "+v"(fb[0][1].hi), "+v"(fb[0][2].lo), "+v"(fb[0][2].hi),
                   "+v"(fb[0][3].lo), "+v"(fb[0][3].hi));
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int bn = 0; bn < 4; ++bn)
        acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr16_value(fa[0][bm]), tr16_value(fb[0][bn]),
                                                              acc[bm][bn], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (next) convert(stn, 0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(fa[1][0].lo), "+v"(fa[1][0].hi), "+v"(fa[1][1].lo), "+v"(fa[1][1].hi), "+v"(fb[1][0].lo),
                   "+v"(fb[1][0].hi), "+v"(fb[1][1].lo), "+v"(fb[1][1].hi), "+v"(fb[1][2].lo), "+v"(fb[1][2].hi),
                   "+v"(fb[1][3].lo), "+v"(fb[1][3].hi));
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int bn = 0; bn < 4; ++bn)
        acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr16_value(fa[1][bm]), tr16_value(fb[1][bn]),
                                                              acc[bm][bn], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (next) convert(stn, 1);
    prof.tick(3);
  }
  prof.flush(blockIdx.x);

  // partial slab: dW (row-major M x N) then db (M)
  float* part = a.part + (int64_t)split * a.split_stride + batch * ((int64_t)M * N + M);
#pragma unroll
  for (int bm = 0; bm < 2; ++bm)
#pragma unroll
    for (int bn = 0; bn < 4; ++bn) {
      const int col = 128 * wn + 32 * bn + (lane & 31);
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 64 * wm + 32 * bm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        part[(int64_t)row * N + col] = acc[bm][bn][e];
      }
    }
  __syncthreads();
  float* red = (float*)smem;  // [16 row slots][256]
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rth * 256 + 8 * cth + e] = dbacc[e];
  __syncthreads();
  if (tid < 256) {
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) sum += red[k * 256 + tid];
    part[(int64_t)M * N + tid] = sum;
  }
  if constexpr (TOPO > 0) {
    // dW_L [O][M] and db_L [O] over the 16 row slots
    __syncthreads();
    constexpr int RS = TOPO * 256 + TOPO;
#pragma unroll
    for (int o = 0; o < TOPO; ++o)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[rth * RS + o * 256 + 8 * cth + e] = tdw[o][e];
    if (cth == 0) {
#pragma unroll
      for (int o = 0; o < TOPO; ++o) red[rth * RS + TOPO * 256 + o] = tdb[o];
    }
    __syncthreads();
    float* pl = a.top.partL + (int64_t)split * a.top.partL_stride + batch * (int64_t)RS;
    for (int idx = tid; idx < RS; idx += 512) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) sum += red[k * RS + idx];
      pl[idx] = sum;
    }
  }
}

template <int RECC = 0, int TOPO = 0>
__global__ __launch_bounds__(512) void dw_ring_bf16_kernel(TNArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[dw_ring_lds_bytes<RECC, TOPO>()];
  const int64_t split = blockIdx.x;
  const int64_t r_begin = split * a.rows_per_split;
  const int64_t r_end = r_begin + a.rows_per_split < a.rows_per_batch ? r_begin + a.rows_per_split : a.rows_per_batch;
  dw_ring_body<RECC, TOPO>(a, smem, r_begin, r_end, split);
}

// ------------------------------------------------------------------------------------------
// pair_ring: one 256 x 256 layer's two gradients in ONE launch, on two co-scheduled roles.
// Workgroups b and b + 8 land on the same XCD under round-robin dispatch (speed only, never
// correctness); pair p = the two workgroups (b & 7) + 16 k and (b & 7) + 16 k + 8. Both walk the
// same contiguous range of 32-row tiles in the same order — the first as dx_ring (input
// gradient), the second as dw_ring (weight gradient, one partial slab per pair) — so the tile one
// of them streams from HBM is, most of the time, still in the XCD's L2 when the other asks for
// it: dZ_l and P_{l-1} leave HBM about once instead of twice, and there are half as many slabs.
// gridDim.x = 2 * npair, a multiple of 16.
// ------------------------------------------------------------------------------------------
template <int BOTC, bool DXOUT, bool REC, int TOPO, int RECC>
__global__ __launch_bounds__(512) void pair_ring_bf16_kernel(NTArgs ax, TNArgs aw, ReduceMultiArgs prev) {
  constexpr int LX = dx_ring_lds_bytes<BOTC, TOPO>(), LW = dw_ring_lds_bytes<RECC, TOPO>();
  __shared__ __attribute__((aligned(16))) char smem[LX > LW ? LX : LW];
  const int b = blockIdx.x;
  const int64_t G = gridDim.x;
  const int64_t rows = ax.rows_per_batch;
  const int64_t ntiles = (rows + RING_BM - 1) / RING_BM;
  // pair (b & 7) + 16 k, (b & 7) + 16 k + 8: two workgroups on one XCD under round-robin dispatch
  // (speed only), the first as the input-gradient role, the second as the weight-gradient role, both
  // walking the same tile range; npair = weight-gradient workgroups = slabs
  const int64_t idx = (b & 7) | ((b >> 4) << 3);
  const int64_t nrole = G >> 1, nw = nrole;
  const bool dxrole = ((b >> 3) & 1) == 0;
  const int64_t tb = ntiles * idx / nrole, te = ntiles * (idx + 1) / nrole;
  if (dxrole) {
    if (!(aw.pair_roles & 1)) return;
    // slab: the first-layer slab (BOTC)
    dx_ring_body<BOTC, DXOUT, REC, TOPO>(ax, smem, tb, 1, te - tb, idx);
  } else {
    const int64_t r_end = te * RING_BM < rows ? te * RING_BM : rows;
    if (aw.pair_roles & 2) dw_ring_body<RECC, TOPO>(aw, smem, tb * RING_BM, r_end, idx);
    // tail: the previous pair launch's slab reduction (this role finishes ahead of the
    // input-gradient role), 128-float blocks dealt over the weight-gradient workgroups, two
    // 256-thread groups each; reduce_multi_kernel's block body and summation order
    if (prev.nseg > 0) {
      __syncthreads();
      f32x4(*red)[32] = (f32x4(*)[32])(smem + (threadIdx.x >> 8) * (8 * 32 * 16));
      const int nblk = reduce_total_blocks(prev);
      const int wg = (int)(idx + nw * blockIdx.y), per = (int)(2 * nw * gridDim.y);
      for (int k = 0; k * per < nblk; ++k) reduce_block(prev, k * per + 2 * wg + (threadIdx.x >> 8), threadIdx.x & 255, red);
    }
  }
}

}  // namespace siren

namespace siren {

// ------------------------------------------------------------------------------------------
// bwd_ring: one 256 x 256 hidden layer's whole backward in one pass over its inputs —
//   dZ_{l-1} = (dZ_l W_l) cos(P_{l-1}) w0          (input gradient, as dx_ring_bf16_kernel)
//   dW_l += dZ_l^T sin(P_{l-1}), db_l += sum dZ_l   (weight gradient, as dw_ring_bf16_kernel)
// so dZ_l and P_{l-1} are read from HBM once instead of twice.
//
// One wave per SIMD (4 waves, up to 512 registers): wave w holds the 64 input-gradient columns
// [64 w, +64) (W_l^T slice, 128 VGPRs) and a 128 x 128 block of the dW partial (256 accumulator
// registers, AGPRs). 32-row tiles of dZ_l and P_{l-1} (32 KB) stream through a 4-stage DMA ring;
// per tile: input-gradient MFMAs -> epilogue (dZ_{l-1} to an output tile, sin(P) in place) ->
// barrier -> weight-gradient MFMAs on transposing fragment reads -> coalesced dZ_{l-1} stores.
// Each workgroup owns a contiguous row range (a.rows_per_split) and writes one dW/db slab.
// ------------------------------------------------------------------------------------------
struct BwdArgs {
  const bf16* dZ;        // [rows, 256] grad_t (dZ_l)
  const uint16_t* P;     // [rows, 256] phase (P_{l-1})
  const bf16* Wt;        // [nb_w][256 (out cols), 256 (K)] op_t = W_l^T rows
  bf16* dZo;             // [rows, 256] grad_t (dZ_{l-1})
  float* part;           // [split][nb][256*256 + 256] dW / db partials
  int64_t rows_per_batch;
  int64_t rows_per_split;
  int64_t split_stride;
  int64_t w_bstride;
  float w0;
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void bwd_ring_bf16_kernel(BwdArgs a) {
  using PT = Prec<kPrecBF16>;
  constexpr int F = 256, BM = 32, S = RING_S, NT = 256;
  // rows padded to 544 B: every LDS address is a per-lane base plus a compile-time offset, and
  // the 4-row transposing reads hit 4 disjoint bank groups. Each DMA instruction moves one row
  // (the 32 low lanes; the high half is masked off).
  constexpr int RS = F * 2 + 32;
  constexpr int T_BYTES = BM * RS;                     // one padded 32 x 256 2-byte tile
  constexpr int STAGE = 2 * T_BYTES;                   // dZ_l tile, P tile
  constexpr int O_BYTES = BM * F * 2;                  // output tile (linear rows)
  constexpr int NKS = F / 16;
  constexpr int NDMA = BM / 4;                         // DMA instructions per wave per tile and operand (8)
  constexpr int NST = O_BYTES / 16 / NT;               // 16-byte stores per thread per tile (4)
  constexpr int STEADY = (S - 1) * NST + (S - 2) * 2 * NDMA;
  static_assert(STEADY == 44, "counted wait below");
  __shared__ __attribute__((aligned(16))) char smem[S * STAGE + O_BYTES];
  char* const Obuf = smem + S * STAGE;                 // dZ_{l-1} output tile

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int split = blockIdx.x;
  const int64_t batch = blockIdx.y;
  const int64_t rows = a.rows_per_batch;
  const int64_t rowbase = batch * rows;
  const int64_t r_begin = (int64_t)split * a.rows_per_split;
  int64_t r_end = r_begin + a.rows_per_split;
  if (r_end > rows) r_end = rows;
  const int64_t ntile = r_end > r_begin ? (r_end - r_begin + BM - 1) / BM : 0;

  auto off = [&](int r, int c) -> int { return r * RS + (c << 4); };

  // input-gradient B operand: W_l^T rows of this wave's 64 columns
  bf16x8 wf[2][NKS];
  {
    const bf16* Wb = a.Wt + batch * a.w_bstride;
#pragma unroll
    for (int fb = 0; fb < 2; ++fb)
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks)
        wf[fb][ks] = *(const bf16x8*)(Wb + (int64_t)(64 * wave + 32 * fb + r32) * F + 16 * ks + 8 * h);
  }

  auto dma = [&](int64_t k, int st) {
    char* base = smem + st * STAGE;
    const int64_t r0 = r_begin + k * BM;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint16_t* src = t == 0 ? (const uint16_t*)a.dZ : a.P;
#pragma unroll
      for (int j = 0; j < NDMA; ++j) {
        const int r = wave + 4 * j;                  // one row per instruction
        const int64_t row = min(r0 + r, r_end - 1);
        if (lane < 32)
          __builtin_amdgcn_global_load_lds((const void*)(src + (rowbase + row) * F + 8 * lane),
                                           (lds_void*)(base + t * T_BYTES + r * RS), 16, 0, 0);
      }
    }
  };

  f32x16 dw[4][4];  // wave (wm, wn): dW rows [128 wm + 32 i, +32), cols [128 wn + 32 j, +32)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) dw[i][j][e] = 0.f;
  const int wm = wave & 1, wn = wave >> 1;
  float dbacc[8];  // db: thread's chunk column cth, summed over its rows 4 rth .. 4 rth + 3
  const int cth = tid & 31, rth = tid >> 5;  // 8 row groups of 4 rows
#pragma unroll
  for (int e = 0; e < 8; ++e) dbacc[e] = 0.f;

  for (int s = 0; s < S - 1; ++s)
    if (s < ntile) dma(s, s);

  const int g = lane >> 4, t16 = lane & 15, q4 = t16 >> 2, p4 = t16 & 3;
  for (int64_t k = 0; k < ntile; ++k) {
    const int st = (int)(k % S);
    if (k + S - 2 < ntile && k >= S - 1) vm_wait<STEADY>();
    else vm_drain();
    lds_barrier();
    if (k + S - 1 < ntile) dma(k + S - 1, (int)((k + S - 1) % S));
    char* Ab = smem + st * STAGE;
    char* Pb = Ab + T_BYTES;
    const int64_t r0 = r_begin + k * BM;
    const int nval = (int)(r_end - r0 < BM ? r_end - r0 : BM);

    // db over the valid rows of the dZ_l tile (chunk task: rows 4 rth + q, chunk cth)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 4 * rth + q;
      if (r < nval) {
        const bf16x8 dv = *(const bf16x8*)(Ab + off(r, cth));
#pragma unroll
        for (int e = 0; e < 8; ++e) dbacc[e] += (float)dv[e];
      }
    }
    // input gradient, one 32-column block at a time (16 accumulator registers live):
    // acc = dZ_l tile (32 rows) . W_l^T cols [64 w + 32 fb, +32); epilogue: dZ_{l-1} = acc cos(P) w0
    // -> output tile, P -> bf16 sin(P) in place (0 past the end)
#pragma unroll
    for (int fb = 0; fb < 2; ++fb) {
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 af = *(const bf16x8*)(Ab + off(r32, 2 * ks + h));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, wf[fb][ks], acc, 0, 0, 0);
      }
      const int col = 64 * wave + 32 * fb + r32;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rl = (e & 3) + 8 * (e >> 2) + 4 * h;
        uint16_t* pp = (uint16_t*)(Pb + off(rl, col >> 3)) + (col & 7);
        const uint16_t ph = *pp;
        const float c = PT::cosp(ph);
        ((uint16_t*)Obuf)[rl * F + col] = __builtin_bit_cast(uint16_t, (bf16)((acc[e] * c) * a.w0));
        *pp = __builtin_bit_cast(uint16_t, (bf16)(rl < nval ? PT::sinp(ph) : 0.f));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lds_barrier();
    // weight gradient: dW[m][n] += sum_r dZ_l[r][m] sin(P)[r][n] (transposing fragment reads)
#pragma unroll
    for (int ks = 0; ks < BM / 16; ++ks) {
      const int nb = 16 * ks + 8 * (g >> 1) + q4;
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 128 * wm + 32 * i + 16 * (g & 1) + 4 * p4;
        af[i] = lds_read_tr16_pair(Ab + off(nb, c >> 3) + (c & 7) * 2, Ab + off(nb + 4, c >> 3) + (c & 7) * 2);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = 128 * wn + 32 * j + 16 * (g & 1) + 4 * p4;
        bfr[j] = lds_read_tr16_pair(Pb + off(nb, c >> 3) + (c & 7) * 2, Pb + off(nb + 4, c >> 3) + (c & 7) * 2);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          dw[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], dw[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);  // one K step's fragments live at a time
    }
    // coalesced dZ_{l-1} stores (rows past the range skipped)
#pragma unroll
    for (int q = 0; q < NST; ++q) {
      const int u = tid + NT * q;
      const int r = u >> 5, c = u & 31;
      const u16x8 v = *(const u16x8*)(Obuf + (r * F + 8 * c) * 2);
      if (r < nval) *(u16x8*)((uint16_t*)a.dZo + (rowbase + r0 + r) * F + 8 * c) = v;
    }
  }

  // partial slab: dW (row-major 256 x 256) then db (256)
  float* part = a.part + (int64_t)split * a.split_stride + batch * ((int64_t)F * F + F);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = 128 * wn + 32 * j + r32;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 128 * wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
        part[(int64_t)row * F + col] = dw[i][j][e];
      }
    }
  __syncthreads();
  float* red = (float*)smem;  // [8 row groups][256]
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rth * 256 + 8 * cth + e] = dbacc[e];
  __syncthreads();
  {
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) sum += red[k * 256 + tid];
    part[(int64_t)F * F + tid] = sum;
  }
}

}  // namespace siren
