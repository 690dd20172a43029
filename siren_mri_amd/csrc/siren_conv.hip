// siren_conv.hip — the weight gradient of the conv encoder's residual-block convolutions
// (Conv2dResBlock, modules.py:433-450: 128 -> 128 channels, 5x5, stride 1, padding 2) in bf16
// channels-last, on the bf16 MFMA:
//
//   dW[co][kh][kw][ci] = sum_{n,h,w} dY[n][h][w][co] X[n][h + kh - 2][w + kw - 2][ci]   (0 outside)
//
// i.e. 25 GEMMs (one per tap) of M = co, N = ci, K = N H W pixels. MIOpen's best solver for this
// shape (igemm_wrw, bf16 NHWC) ran 0.6 ms per convolution in the C4 step (0.27 of the bf16 peak).
//
// Work split: workgroup (split, kh, co half) owns the 5 taps of one filter row for 64 output
// channels — 40 accumulator blocks of 32 x 32, five per wave: wave w holds co block w & 1 and ci
// block w >> 1 for all five kw (80 accumulator registers) — over a contiguous range of output
// image rows (split-K), and writes one fp32 partial; conv_wrw_reduce_kernel adds the partials in
// split order (deterministic) straight into the fp32, channels-last [co][kh][kw][ci] gradient.
// Per 64-pixel chunk of an output row, the dY chunk (64 px x 64 co) and the X halo (68 px x 128 ci
// of input row h + kh - 2, zeros outside the image) are staged in LDS (three stages; the global
// loads of the chunk after next are in flight during this chunk's MFMAs); the MFMA operands come from
// transposing reads (ds_read_b64_tr_b16: pixels are the K dimension), the five taps reading the X
// halo at row offsets kw. LDS rows are padded to 192 / 320 bytes (4-row transposing reads on
// distinct bank groups).
#include <type_traits>

#include "siren_common.h"

namespace siren {

constexpr int CW_C = 128;                    // channels (in and out)
constexpr int CW_K = 5;                      // filter size
constexpr int CW_PX = 64;                    // output pixels per chunk
constexpr int CW_XROWS = CW_PX + CW_K - 1;   // 68 halo rows
constexpr int CW_DROW = 96;                  // bf16 per staged dY row (64 co + 32 pad: 192 B)
constexpr int CW_XROW = 160;                 // bf16 per staged X row (128 ci + 32 pad: 320 B)
constexpr int CW_NB = 3;                     // LDS stages
constexpr int CW_XPIECES = CW_XROWS * 16;    // 16-byte pieces of the X halo (1088)
constexpr int CW_NXL = (CW_XPIECES + 511) / 512;  // per thread (3)
constexpr int CW_SLAB = CW_K * CW_K * CW_C * CW_C;  // floats of one partial

struct ConvWArgs {
  const bf16* x;    // [N][H][W][128]
  const bf16* dy;   // [N][H][W][128]
  float* part;      // [nsplit][5 kh][5 kw][128 co][128 ci]
  float* dw;        // [128 co][5 kh][5 kw][128 ci] (reduce)
  int N, H, W;
  int64_t rows_per_split;  // output image rows (of N * H) per split
  int nsplit;
};

// Pipeline: chunk t + 2's global loads go to register set t % 2 while chunk t's MFMAs run; at the
// top of iteration t + 1 that set is written to LDS stage (t + 2) % 3 (last read in iteration
// t - 1, before the barrier that closed it); one barrier per chunk.
// DMA (option wrw_dma): the same LDS image filled by LDS-DMA (buffer_load ... lds, 1 KB per
// wave-instruction) straight into stage (t + 2) % 3 at the top of iteration t, no register sets and
// no staging writes. A chunk is 12 dY instructions (64 rows x 12 slots: 8 channel pieces + 4 pad)
// and 22 X instructions (68 halo rows x 20 slots: 16 + 4 pad; the X stage padded to 22 KB); a lane's
// source offsets are fixed per workgroup: the chunk moves the buffer bases (scalar), and halo pixels
// left or right of the image, pad slots and X rows outside the image (a zero-size buffer) are out of
// range, so they arrive as zeros.
// PX = 128 (option wrw_dma 2, DMA only, W a multiple of 128): 128-pixel chunks in two LDS stages
// (135 KB), the chunk after next's DMA one chunk ahead; twice the MFMAs per barrier, DMA issue and
// fragment-read ramp-up of a 64-pixel chunk.
template <bool DMA, int PX = CW_PX>
__global__ __launch_bounds__(512) void conv_wrw_k5_kernel(ConvWArgs a) {
  static_assert(PX == CW_PX || (DMA && PX == 2 * CW_PX), "64-pixel chunks, or 128 with the DMA fill");
  constexpr int NB = PX == CW_PX ? CW_NB : 2;                // LDS stages
  constexpr int XROWS = PX + CW_K - 1;                       // halo rows
  constexpr int DMA_D = PX * 12 / 64;                        // dY instructions per chunk (12 / 24)
  constexpr int DMA_X = (XROWS * 20 + 63) / 64;              // X instructions per chunk (22 / 42)
  constexpr int DMA_N = DMA_D + DMA_X;
  constexpr int DMA_PER_WAVE = (DMA_N + 7) / 8;
  constexpr int XSTAGE_DMA = DMA_X * 1024;
  __shared__ __attribute__((aligned(16))) bf16 sD[NB][PX * CW_DROW];
  __shared__ __attribute__((aligned(16))) bf16 sX[NB][DMA ? XSTAGE_DMA / 2 : CW_XROWS * CW_XROW];
  const int split = blockIdx.x, kh = blockIdx.y, ch = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cb = wave & 1, ib = wave >> 1;
  const int nrows = a.N * a.H;
  const int r0 = split * (int)a.rows_per_split;
  const int r1 = r0 + (int)a.rows_per_split < nrows ? r0 + (int)a.rows_per_split : nrows;
  const int nch = a.W / PX;
  const int T = r1 > r0 ? (r1 - r0) * nch : 0;

  f32x16 acc[CW_K];
#pragma unroll
  for (int k = 0; k < CW_K; ++k)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[k][e] = 0.f;

  // loader: one dY piece per thread (row tid / 8, piece tid % 8 of the 64-channel half), X halo
  // pieces p = tid + 512 i (row p / 16, piece p % 16; zeros outside the image)
  // (two register sets, selected at compile time: the loop below is unrolled by two, since a
  // run-time set index became indexed register moves)
  // chunks are loaded in order, so the loader keeps a cursor (image n, row h, first pixel px0)
  // advanced one chunk per load: no per-chunk 64-bit division on the scalar unit (the divisions of
  // the chunk index made SALU instructions outnumber VALU ones 1.7 : 1 in the PMC counters)
  int cn = r0 / a.H, ch_row = r0 - (r0 / a.H) * a.H, cpx = 0;
  u32x4_t dv[2], xv[2][CW_NXL];
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  auto load = [&](auto set_c) {
    constexpr int set = decltype(set_c)::value;
    const int n = cn, h = ch_row, px0 = cpx;
    cpx += CW_PX;
    if (cpx == a.W) {
      cpx = 0;
      if (++ch_row == a.H) {
        ch_row = 0;
        ++cn;
      }
    }
    const int xr = h + kh - CW_K / 2;
    const bool rowok = xr >= 0 && xr < a.H;
    dv[set] = *(const u32x4_t*)(a.dy + (((int64_t)n * a.H + h) * a.W + px0 + (tid >> 3)) * CW_C + 64 * ch +
                                8 * (tid & 7));
    const bf16* xrow = a.x + ((int64_t)n * a.H + (rowok ? xr : 0)) * a.W * CW_C;
#pragma unroll
    for (int i = 0; i < CW_NXL; ++i) {
      const int p = tid + 512 * i;
      const int w = px0 - CW_K / 2 + (p >> 4);
      const bool ok = p < CW_XPIECES && rowok && w >= 0 && w < a.W;
      xv[set][i] = ok ? *(const u32x4_t*)(xrow + (int64_t)w * CW_C + 8 * (p & 15)) : zero;
    }
  };
  auto stage = [&](auto set_c, int buf) {
    constexpr int set = decltype(set_c)::value;
    *(u32x4_t*)(&sD[buf][(tid >> 3) * CW_DROW + 8 * (tid & 7)]) = dv[set];
#pragma unroll
    for (int i = 0; i < CW_NXL; ++i) {
      const int p = tid + 512 * i;
      if (p < CW_XPIECES) *(u32x4_t*)(&sX[buf][(p >> 4) * CW_XROW + 8 * (p & 15)]) = xv[set][i];
    }
  };

  // transposing-read lane roles (tn_dw_kernel's): rows nb, nb + 4 of a 16-row K step, 4 columns.
  // The reads are inline asm with counted lgkmcnt waits: hipcc puts an s_waitcnt vmcnt(0) in
  // front of the ds_read_tr builtin, which would drain the next chunks' global loads every step.
  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int ca = 32 * cb + 16 * (g & 1) + 4 * tp;   // co column within the half
  const int cx = 32 * ib + 16 * (g & 1) + 4 * tp;   // ci column
  const int r8 = 8 * (g >> 1) + tq;                  // row of K step 0
  const uint32_t dbase = lds_addr(&sD[0][0]) + (uint32_t)((r8 * CW_DROW + ca) * 2);
  const uint32_t xbase = lds_addr(&sX[0][0]) + (uint32_t)((r8 * CW_XROW + cx) * 2);
  constexpr uint32_t DSTAGE = PX * CW_DROW * 2, XSTAGE = DMA ? XSTAGE_DMA : CW_XROWS * CW_XROW * 2;
  constexpr int DROWB = CW_DROW * 2, XROWB = CW_XROW * 2;

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  // DMA: lane source offsets of this wave's instructions g = wave + 8 i (dY: row * 256 + piece;
  // X: (halo row - 2) * 256 + piece, plus 256 px0 per chunk; out of range for the pad slots)
  int voff[DMA_PER_WAVE];
  if constexpr (DMA) {
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; ++i) {
      const int g = wave + 8 * i;
      if (g < DMA_D) {
        const int slot = 64 * g + lane, row = slot / 12, pc = slot - 12 * (slot / 12);
        voff[i] = pc < 8 ? row * CW_C * 2 + 16 * pc : 0x7fffffff;
      } else {
        const int slot = 64 * (g - DMA_D) + lane, row = slot / 20, pc = slot - 20 * (slot / 20);
        voff[i] = (pc < 16 && row < XROWS) ? (row - CW_K / 2) * CW_C * 2 + 16 * pc : 0x40000000;
      }
    }
  }
  // DMA of the chunk at the cursor into stage buf, then the cursor advances one chunk
  auto dma = [&](int buf) {
    const int n = cn, h = ch_row, px0 = cpx;
    cpx += PX;
    if (cpx == a.W) {
      cpx = 0;
      if (++ch_row == a.H) {
        ch_row = 0;
        ++cn;
      }
    }
    const int xr = h + kh - CW_K / 2;
    const bool rowok = xr >= 0 && xr < a.H;
    const __amdgpu_buffer_rsrc_t rD =
        make_rsrc(a.dy + (((int64_t)n * a.H + h) * a.W + px0) * CW_C + 64 * ch, (PX * CW_C - 64) * 2);
    const __amdgpu_buffer_rsrc_t rX =
        make_rsrc(a.x + ((int64_t)n * a.H + (rowok ? xr : 0)) * a.W * CW_C, rowok ? (int64_t)a.W * CW_C * 2 : 0);
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; ++i) {
      const int g = wave + 8 * i;  // wave-uniform
      if (g < DMA_D)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rD, (lds_void*)((char*)&sD[buf][0] + 1024 * g), 16, (uint32_t)voff[i],
                                                 0, 0, 0);
      else if (g < DMA_N)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)((char*)&sX[buf][0] + 1024 * (g - DMA_D)), 16,
                                                 (uint32_t)(voff[i] + px0 * CW_C * 2), 0, 0, 0);
    }
  };
  if constexpr (NB == 2) {
    if (T > 0) dma(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else if constexpr (DMA) {
    if (T > 0) dma(0);
    if (T > 1) {
      dma(1);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // chunk 0 (the younger chunk 1 is 4 or 5)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else {
    if (T > 0) {
      load(S0{});
      stage(S0{}, 0);
    }
    if (T > 1) load(S1{});
    __syncthreads();
  }
  int bcur = 0;  // t % CW_NB
  // iteration t: chunk t + 1 (register set (t + 1) & 1) to LDS, chunk t + 2's loads into set t & 1,
  // chunk t's MFMAs (DMA: chunk t + 2 into stage (t + 2) % 3, chunk t's MFMAs, wait for chunk t + 1)
  auto iter = [&](int t, auto par_c) {
    constexpr int par = decltype(par_c)::value;  // t & 1
    using SN = std::integral_constant<int, par ^ 1>;
    using SC = std::integral_constant<int, par>;
    const int buf = NB == 2 ? par : bcur;
    bcur = bcur == NB - 1 ? 0 : bcur + 1;
    if constexpr (NB == 2) {
      if (t + 1 < T) dma(par ^ 1);  // stage (t + 1) & 1: last read by chunk t - 1
    } else if constexpr (DMA) {
      if (t + 2 < T) dma(bcur == NB - 1 ? 0 : bcur + 1);
    } else {
      if (t + 1 < T) stage(SN{}, bcur);
      if (t + 2 < T) load(SC{});
    }
    const uint32_t db = dbase + buf * DSTAGE, xb = xbase + buf * XSTAGE;
    // K step ks's 12 fragment reads are issued before step ks - 1's MFMAs (a wait for the older 12
    // then covers step ks - 1 exactly: lgkmcnt(12))
    TrFrag fa[2], fb[2][CW_K];
#define SIREN_CW_RD(KS)                                                                  \
  {                                                                                      \
    constexpr int ks_ = (KS), b_ = (KS) & 1;                                             \
    tr16_read<16 * ks_ * DROWB>(fa[b_].lo, db);                                          \
    tr16_read<16 * ks_ * DROWB + 4 * DROWB>(fa[b_].hi, db);                              \
    static_for<0, CW_K>([&](auto kw_c) {                                                 \
      constexpr int kw = decltype(kw_c)::value;                                          \
      tr16_read<(16 * ks_ + kw) * XROWB>(fb[b_][kw].lo, xb);                             \
      tr16_read<(16 * ks_ + kw + 4) * XROWB>(fb[b_][kw].hi, xb);                         \
    });                                                                                  \
  }
    SIREN_CW_RD(0)
    static_for<0, PX / 16>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value, b = ks & 1;
      if constexpr (ks + 1 < PX / 16) {
        SIREN_CW_RD(ks + 1)
        asm volatile("s_waitcnt lgkmcnt(12)"
                     : "+v"(fa[b].lo), "+v"(fa[b].hi), "+v"(fb[b][0].lo), "+v"(fb[b][0].hi), "+v"(fb[b][1].lo),
                       "+v"(fb[b][1].hi), "+v"(fb[b][2].lo), "+v"(fb[b][2].hi), "+v"(fb[b][3].lo), "+v"(fb[b][3].hi),
                       "+v"(fb[b][4].lo), "+v"(fb[b][4].hi));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(fa[b].lo), "+v"(fa[b].hi), "+v"(fb[b][0].lo), "+v"(fb[b][0].hi), "+v"(fb[b][1].lo),
                       "+v"(fb[b][1].hi), "+v"(fb[b][2].lo), "+v"(fb[b][2].hi), "+v"(fb[b][3].lo), "+v"(fb[b][3].hi),
                       "+v"(fb[b][4].lo), "+v"(fb[b][4].hi));
      }
      static_for<0, CW_K>([&](auto kw_c) {
        constexpr int kw = decltype(kw_c)::value;
        acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr16_value(fa[b]), tr16_value(fb[b][kw]), acc[kw], 0, 0, 0);
      });
    });
#undef SIREN_CW_RD
    if constexpr (DMA) {
      // this wave's part of chunk t + 1 landed (chunk t + 2's 4 or 5 are younger); a barrier without
      // __syncthreads' fence, which would drain chunk t + 2's DMA too (vmcnt(0)); two stages: chunk
      // t + 1 is the youngest
      if (NB == 3 && t + 2 < T) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };
  for (int t = 0; t < T; t += 2) {
    iter(t, S0{});
    if (t + 1 < T) iter(t + 1, S1{});
  }

  // partial: [split][kh][kw][co][ci]
  float* P = a.part + ((int64_t)split * CW_K + kh) * CW_K * CW_C * CW_C;
#pragma unroll
  for (int kw = 0; kw < CW_K; ++kw) {
    const int ci = 32 * ib + (lane & 31);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int co = 64 * ch + 32 * cb + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      P[((int64_t)kw * CW_C + co) * CW_C + ci] = acc[kw][e];
    }
  }
}

// dw[co][kh][kw][ci] = sum_s part[s][kh][kw][co][ci], splits in order
__global__ __launch_bounds__(256) void conv_wrw_reduce_kernel(ConvWArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over [kh][kw][co][ci]
  if (i >= CW_SLAB) return;
  const int ci = (int)(i % CW_C);
  const int co = (int)((i / CW_C) % CW_C);
  const int tap = (int)(i / ((int64_t)CW_C * CW_C));  // kh * 5 + kw
  float s = 0.f;
  for (int sp = 0; sp < a.nsplit; ++sp) s += a.part[(int64_t)sp * CW_SLAB + i];
  a.dw[((int64_t)co * CW_K * CW_K + tap) * CW_C + ci] = s;
}

}  // namespace siren

namespace siren {

// ------------------------------------------------------------------------------------------
// conv_fwd_k5: y = conv(x, W) for the same 128 -> 128, 5x5, stride-1, padding-2 shape, bf16 NHWC
// in and out, fp32 accumulation (the residual blocks' forward convolutions, and their input
// gradients as forward convolutions of the flipped, transposed filter W'[ci][kh][kw][co] =
// W[co][4 - kh][4 - kw][ci] — the same layout, so one kernel serves both).
//
//   y[n][h][w][co] = sum_{kh, kw, ci} x[n][h + kh - 2][w + kw - 2][ci] W[co][kh][kw][ci]  (0 outside)
//
// Workgroup tile: two output image rows (256 pixels when W = 128) x all 128 output channels, as
// D[co][px] = W . X^T on the bf16 MFMA (A = filter rows, B = pixel channel vectors: both operands
// are 16-byte LDS reads of 8 consecutive input channels). Wave w holds co half w & 1 and pixel
// quarter w >> 1: four 32 x 32 accumulator blocks. K loop: 20 stages (filter row kh x 32-channel
// chunk cc); a stage holds the two input rows h0 + kh - 2, h0 + kh - 1 (132 px with the zero halo)
// and the 5 x 128 filter rows of that chunk in LDS (rows padded to 80 bytes), and runs 5 taps x 2
// K steps of MFMAs; the next stage's global loads are in flight meanwhile (two register sets,
// compile-time selected, two LDS stages). Epilogue: bf16(acc) (optionally + bias, ReLU: the bias
// add and the ReLU of the conv + bias + ReLU chain, same rounding) through LDS to coalesced
// 16-byte stores.
// ------------------------------------------------------------------------------------------
constexpr int CF_W = 128;                    // image width (pixels per row), fixed
constexpr int CF_HALO = CF_W + CW_K - 1;     // 132
constexpr int CF_CC = 32;                    // input channels per stage
constexpr int CF_ROWB = 80;                  // bytes per LDS row (32 bf16 + 16 pad)
// LDS pixel rows per image row: the 132 halo pixels padded to 136 (17 blocks of 8; the 4 pad rows
// are staged as zeros and never read) so that the staging writes can pair rows j and j + 4
constexpr int CF_HALOP = 136;
constexpr int CF_XB = 2 * CF_HALOP * CF_ROWB;        // x part of a stage (21,760 B)
constexpr int CF_WB = CW_K * CW_C * CF_ROWB;          // filter part (51,200 B)
constexpr int CF_STAGE = CF_XB + CF_WB;               // 72,960 B
constexpr int CF_XP = 2 * CF_HALOP * 4;               // 16-byte x pieces per stage (1088)
constexpr int CF_WP = CW_K * CW_C * 4;                // filter pieces (2560)
constexpr int CF_NL = (CF_XP + CF_WP + 511) / 512;    // loads per thread per stage (8)

struct ConvFArgs {
  const bf16* x;     // [N][H][128][128]
  const bf16* w;     // [128 out][5][5][128 in]
  const bf16* bias;  // [128] or null
  bf16* y;           // [N][H][128][128]
  int N, H;
  int relu;          // with bias: y = relu(bf16(bf16(acc) + bias))
  // gradient epilogues (EPI > 0, the input-gradient convolutions of the conv encoder's backward):
  const bf16* g2;    // second gradient summand, or null
  const bf16* m;     // mask source (> 0 keeps the element)
  const bf16* pa;    // EPI_RES: the block's second convolution output a (bias-free)
  const bf16* cb;    // EPI_RES: that convolution's bias
  bf16* y2;          // EPI_RES: second output plane (ga)
  float* part;       // [blocks][128] per-workgroup channel sums of the gradient the bias takes
};

// Epilogues of conv_fwd_k5_kernel. The input gradient of a ReLU'd convolution, g = bf16(acc), is
// consumed at once by an elementwise pass in the encoder's backward (siren_encoder.hip); these
// forms run that pass on the tile while it is in LDS, so g never goes to HBM and the pass's launch
// and plane traffic are gone (enc_relu_bwd_kernel / enc_res_bwd_kernel arithmetic, element for
// element; the channel sums are per-workgroup partials reduced in a fixed order by
// conv_chan_reduce_kernel, deterministic):
//   EPI_RELU: y = bf16((g [+ g2]) [m > 0]);                 part = sums of y
//   EPI_RES : s = g + g2; y = bf16(s [m > 0]) (the skip gradient);
//             y2 = y [bf16(pa + cb) > 0] (the block's pre-activation gradient); part = sums of y2
//   EPI_RESFWD (the forward of Conv2dResBlock's tail, enc_res_fwd_kernel's arithmetic): y = a =
//             bf16(acc) (kept for the backward), y2 = relu(bf16(relu(bf16(a + cb)) + g2)), g2 the
//             block input
constexpr int EPI_PLAIN = 0, EPI_RELU = 1, EPI_RES = 2, EPI_RESFWD = 3;

// LDS row of staging piece w (blocks of 32 pieces = 8 rows x 4 16-byte pieces): lanes 8 m .. 8 m + 7
// of a ds_write_b128 lane group take rows m and m + 4 of the block, 80 dwords apart (see the staging
// comment in conv_fwd_k5_kernel)
DEV int cf_row(int w) {
  const int t = (w >> 2) & 7;
  return 8 * (w >> 5) + (t >> 1) + 4 * (t & 1);
}

// DMA (option conv_dma, default on: C4 17.24 -> 17.01 ms/step in a three-round one-box A/B,
// profiles/r6_ab_conv_dma.txt; bit-identical, tests/test_gpu_encoder.py): the stage image is filled by LDS-DMA (buffer_load ... lds: 1 KB per wave-instruction, no
// VGPR staging, no LDS write transfer from the register file) one stage ahead, instead of global
// loads two stages ahead into registers and ds_write_b128 staging. The image is the same
// (pad slots and pixels outside the image arrive as zeros through out-of-range buffer offsets);
// each stage is padded to a multiple of 1 KB (CF_STAGE_DMA) so the last instruction's tail stays
// inside it.
// In that image the x part is padded to whole 1 KB instructions (no instruction spans both parts:
// an LDS-DMA instruction writes every lane's 16 bytes).
constexpr int CF_DMA_XN = (CF_XB + 1023) / 1024;                  // x-part instructions (22)
constexpr int CF_XB_DMA = CF_DMA_XN * 1024;                       // 22,528 B
constexpr int CF_DMA_N = CF_DMA_XN + (CF_WB + 1023) / 1024;       // per stage (72)
constexpr int CF_STAGE_DMA = CF_DMA_N * 1024;                     // 73,728 B
constexpr int CF_DMA_PER_WAVE = (CF_DMA_N + 7) / 8;               // 9
// DMA 2 (option conv_dma 2): the same stage image, with each lane's source offsets computed once
// per workgroup instead of once per stage. A stage (kh, cc) moves every offset by a wave-uniform
// amount (x: kh image rows + cc channel pieces; filter: kh filter rows + cc), and an x piece's row
// test is one compare of (h0 + r - 2 + kh) against H; the per-stage address arithmetic of form 1
// (a division by 5, the halo row split, four range tests: ~150 VALU per wave and stage, issued
// while no wave runs MFMAs) becomes one add and a compare-select per instruction. Default: C4
// 17.02 -> 16.67 ms/step over six interleaved one-box pairs (profiles/r6_ab_conv_dma2.txt), bit-identical.
template <int EPI, int DMA = 0>
__global__ __launch_bounds__(512) void conv_fwd_k5_kernel(ConvFArgs a) {
  constexpr int STG = DMA ? CF_STAGE_DMA : CF_STAGE;
  __shared__ __attribute__((aligned(16))) char smem_cf[2 * STG];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave & 1, wp = wave >> 1;
  const int hp = a.H / 2;  // row pairs per image (H even)
  const int n = blockIdx.x / hp, h0 = 2 * (blockIdx.x % hp);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // stage s = (kh = s / 4, cc = s % 4). Pieces in blocks of 32 (8 LDS rows x 4 16-byte channel
  // pieces); within a block, lanes 8 m .. 8 m + 7 take rows m and m + 4 (cf_row), whose 80-byte rows
  // lie 80 dwords apart: the two 64-byte pieces fill the 32 banks of a ds_write_b128 lane group
  // exactly once (rows m and m + 1 shared 4 banks: every staging write paid a 2-way conflict).
  // Piece q < CF_XP: x row r = q / (4 CF_HALOP) of the pair, halo pixel j (zeros past the 132
  // real ones), channel piece pc; else filter piece q' = q - CF_XP: tap kw = q' / 512, out
  // channel co, piece pc.
  u32x4_t lv[2][CF_NL];
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  auto load = [&](int s, auto set_c) {
    constexpr int set = decltype(set_c)::value;
    const int kh = s >> 2, cc = s & 3;
#pragma unroll
    for (int i = 0; i < CF_NL; ++i) {
      const int q = tid + 512 * i;
      u32x4_t v = zero;
      if (q < CF_XP) {
        const int r = q / (4 * CF_HALOP), j = cf_row(q - r * 4 * CF_HALOP), pc = q & 3;
        const int xr = h0 + r + kh - CW_K / 2, w = j - CW_K / 2;
        if (xr >= 0 && xr < a.H && w >= 0 && w < CF_W)
          v = *(const u32x4_t*)(a.x + (((int64_t)n * a.H + xr) * CF_W + w) * CW_C + CF_CC * cc + 8 * pc);
      } else if (q < CF_XP + CF_WP) {
        const int q2 = q - CF_XP, kw = q2 >> 9, co = cf_row(q2 & 511), pc = q2 & 3;
        v = *(const u32x4_t*)(a.w + ((int64_t)(co * CW_K + kh) * CW_K + kw) * CW_C + CF_CC * cc + 8 * pc);
      }
      lv[set][i] = v;
    }
  };
  auto stage = [&](auto set_c, int buf) {
    constexpr int set = decltype(set_c)::value;
    char* base = smem_cf + buf * CF_STAGE;
#pragma unroll
    for (int i = 0; i < CF_NL; ++i) {
      const int q = tid + 512 * i;
      if (q < CF_XP) {
        const int r = q / (4 * CF_HALOP), j = cf_row(q - r * 4 * CF_HALOP), pc = q & 3;
        *(u32x4_t*)(base + (r * CF_HALOP + j) * CF_ROWB + 16 * pc) = lv[set][i];
      } else if (q < CF_XP + CF_WP) {
        const int q2 = q - CF_XP, kw = q2 >> 9, co = cf_row(q2 & 511), pc = q2 & 3;
        *(u32x4_t*)(base + CF_XB + (kw * CW_C + co) * CF_ROWB + 16 * pc) = lv[set][i];
      }
    }
  };

  // operand reads: A (filter) lane -> out channel 64 wc + 32 i + (lane & 31), channels 8 (lane >> 5)
  // (+16 for the second K step); B (pixels) lane -> pixel 64 wp + 32 j + (lane & 31) of the pair
  // (row (pixel >> 7), column pixel & 127), the tap's halo column + kw
  const int l32 = lane & 31, kh2 = lane >> 5;
  uint32_t aoff[2], boff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) aoff[i] = (DMA ? CF_XB_DMA : CF_XB) + (64 * wc + 32 * i + l32) * CF_ROWB + 16 * kh2;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int px = 64 * wp + 32 * j + l32;
    boff[j] = ((px >> 7) * CF_HALOP + (px & 127)) * CF_ROWB + 16 * kh2;
  }
  const uint32_t sbase = lds_addr(smem_cf);

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  constexpr int NS = CW_K * 4;
  // DMA: wave w issues instructions g = w + 8 i (slots 64 g .. 64 g + 63 of the stage image)
  const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.x + (int64_t)n * a.H * CF_W * CW_C, (int64_t)a.H * CF_W * CW_C * 2);
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.w, (int64_t)CW_C * CW_K * CW_K * CW_C * 2);
  // DMA 2: per instruction i, the lane's stage-(0, 0) offset and (x part) its row test value
  int pbase[CF_DMA_PER_WAVE], prow[CF_DMA_PER_WAVE];
  if constexpr (DMA == 2) {
#pragma unroll
    for (int i = 0; i < CF_DMA_PER_WAVE; ++i) {
      const int g = wave + 8 * i;
      if (g < CF_DMA_XN) {
        const int slot = 64 * g + lane;
        const int row = slot / 5, pc = slot - row * 5;
        const int r = row >= CF_HALOP ? 1 : 0, j = row - r * CF_HALOP;
        const int w = j - CW_K / 2;
        const bool ok = row < 2 * CF_HALOP && pc < 4 && w >= 0 && w < CF_W;
        prow[i] = ok ? h0 + r - CW_K / 2 : -(1 << 20);  // x row = prow + kh; never in range when !ok
        pbase[i] = ((h0 + r - CW_K / 2) * CF_W + w) * CW_C * 2 + 16 * pc;
      } else {
        const int slot = 64 * (g - CF_DMA_XN) + lane;
        const int row = slot / 5, pc = slot - row * 5;
        const int kw = row >> 7, co = row & 127;
        prow[i] = 0;
        pbase[i] = (g < CF_DMA_N && pc < 4 && kw < CW_K) ? (co * CW_K * CW_K * CW_C + kw * CW_C + 8 * pc) * 2
                                                          : 0x7fff0000;  // + a stage's 5,312 B: still out of range
      }
    }
  }
  auto dma = [&](int s, int buf) {
    const int kh = s >> 2, cc = s & 3;
    char* base = smem_cf + buf * STG;
    if constexpr (DMA == 2) {
      const int xadd = kh * CF_W * CW_C * 2 + CF_CC * cc * 2, wadd = kh * CW_K * CW_C * 2 + CF_CC * cc * 2;
#pragma unroll
      for (int i = 0; i < CF_DMA_PER_WAVE; ++i) {
        const int g = wave + 8 * i;  // wave-uniform
        if (g < CF_DMA_XN) {
          const uint32_t off = (uint32_t)(prow[i] + kh) < (uint32_t)a.H ? (uint32_t)(pbase[i] + xadd) : 0x7fffffffu;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)(base + 1024 * g), 16, off, 0, 0, 0);
        } else if (g < CF_DMA_N) {
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(base + 1024 * g), 16, (uint32_t)(pbase[i] + wadd),
                                                   0, 0, 0);
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < CF_DMA_PER_WAVE; ++i) {
      const int g = wave + 8 * i;  // (wave-uniform: the branches below are too)
      if (g < CF_DMA_XN) {
        // x part: slots 64 g + lane of rows (r, j) x 5 (4 channel pieces + the pad slot)
        const int slot = 64 * g + lane;
        const int row = slot / 5, pc = slot - row * 5;
        const int r = row >= CF_HALOP ? 1 : 0, j = row - r * CF_HALOP;
        const int xr = h0 + r + kh - CW_K / 2, w = j - CW_K / 2;
        uint32_t off = 0x7fffffffu;  // out of range: zeros
        if (row < 2 * CF_HALOP && pc < 4 && xr >= 0 && xr < a.H && w >= 0 && w < CF_W)
          off = (uint32_t)(((xr * CF_W + w) * CW_C + CF_CC * cc + 8 * pc) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)(base + 1024 * g), 16, off, 0, 0, 0);
      } else if (g < CF_DMA_N) {
        // filter part: rows (kw, co) x 5
        const int slot = 64 * (g - CF_DMA_XN) + lane;
        const int row = slot / 5, pc = slot - row * 5;
        const int kw = row >> 7, co = row & 127;
        uint32_t off = 0x7fffffffu;
        if (pc < 4 && kw < CW_K) off = (uint32_t)((((co * CW_K + kh) * CW_K + kw) * CW_C + CF_CC * cc + 8 * pc) * 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(base + 1024 * g), 16, off, 0, 0, 0);
      }
    }
  };
  if constexpr (DMA) {
    dma(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    load(0, S0{});
    stage(S0{}, 0);
    load(1, S1{});
  }
  __syncthreads();
  auto iter = [&](int s, auto par_c) {
    constexpr int par = decltype(par_c)::value;
    using SN = std::integral_constant<int, par ^ 1>;
    using SC = std::integral_constant<int, par>;
    if constexpr (DMA) {
      if (s + 1 < NS) dma(s + 1, (s + 1) & 1);
    } else {
      if (s + 1 < NS) stage(SN{}, (s + 1) & 1);
      if (s + 2 < NS) load(s + 2, SC{});
    }
    const uint32_t sb = sbase + (s & 1) * STG;
    // 10 K steps (kw, ks); the fragments of step i + 1 are read while step i's MFMAs run
    bf16x8 af[2][2], bfr[2][2];
#define SIREN_CF_RD(I)                                                                                            \
  {                                                                                                               \
    constexpr int kw_ = (I) >> 1, ks_ = (I) & 1, b_ = (I) & 1;                                                    \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(af[b_][0]) : "v"(sb + aoff[0]), "n"(kw_ * CW_C * CF_ROWB + 32 * ks_)); \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(af[b_][1]) : "v"(sb + aoff[1]), "n"(kw_ * CW_C * CF_ROWB + 32 * ks_)); \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bfr[b_][0]) : "v"(sb + boff[0]), "n"(kw_ * CF_ROWB + 32 * ks_));      \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bfr[b_][1]) : "v"(sb + boff[1]), "n"(kw_ * CF_ROWB + 32 * ks_));      \
  }
    SIREN_CF_RD(0)
    static_for<0, 2 * CW_K>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value, b = i & 1;
      if constexpr (i + 1 < 2 * CW_K) {
        SIREN_CF_RD(i + 1)
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(af[b][0]), "+v"(af[b][1]), "+v"(bfr[b][0]), "+v"(bfr[b][1]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[b][0]), "+v"(af[b][1]), "+v"(bfr[b][0]), "+v"(bfr[b][1]));
      }
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[b][ii], bfr[b][j], acc[ii][j], 0, 0, 0);
    });
#undef SIREN_CF_RD
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage s + 1
    __syncthreads();
  };
  for (int s = 0; s < NS; s += 2) {
    iter(s, S0{});
    iter(s + 1, S1{});
  }

  // epilogue: D[co][px] -> LDS tile [256 px][128 co] bf16 (rows of 256 + 16 bytes), then 16-byte
  // stores of whole pixel rows
  constexpr int OROW = CW_C * 2 + 16;
  char* ot = smem_cf;
  float bia[2][16];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int co = 64 * wc + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * kh2;
      bia[i][e] = a.bias ? (float)a.bias[co] : 0.f;
    }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int px = 64 * wp + 32 * j + l32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float z = (float)(bf16)acc[i][j][4 * g + e];
          if (a.bias) {
            z = (float)(bf16)(z + bia[i][4 * g + e]);
            if (a.relu) z = fmaxf(z, 0.f);
          }
          v[e] = (bf16)z;
        }
        const int co = 64 * wc + 32 * i + 8 * g + 4 * kh2;
        *(bf16x4*)(ot + px * OROW + co * 2) = v;
      }
    }
  __syncthreads();
  // the pair's 64 KB as 16-byte buffer stores, each followed by its 2 wait states (siren_common.h
  // store_b128_ws2)
  const int64_t pair0 = ((int64_t)n * a.H + h0) * CF_W * CW_C;  // the pair's first element
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.y + pair0, 2 * CF_W * CW_C * 2);
  if constexpr (EPI == EPI_PLAIN) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = tid + 512 * k;        // 16-byte piece: pixel q / 16, channels 8 (q % 16)
      const int px = q >> 4, pc = q & 15;
      store_b128_ws2(*(const u32x4_t*)(ot + px * OROW + 16 * pc), ry, (uint32_t)(q * 16), 0);
    }
  } else if constexpr (EPI == EPI_RESFWD) {
    const int pc = tid & 15;
    bf16x8 xv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) xv[k] = *(const bf16x8*)(a.g2 + pair0 + (int64_t)(tid + 512 * k) * 8);
    float cbv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) cbv[e] = (float)a.cb[8 * pc + e];
    const __amdgpu_buffer_rsrc_t ry2 = make_rsrc(a.y2 + pair0, 2 * CF_W * CW_C * 2);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = tid + 512 * k;
      const int px = q >> 4;
      const bf16x8 av = *(const bf16x8*)(ot + px * OROW + 16 * pc);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = (float)(bf16)((float)av[e] + cbv[e]);
        const float s = (float)(bf16)(fmaxf(v, 0.f) + (float)xv[k][e]);
        o[e] = (bf16)fmaxf(s, 0.f);
      }
      store_b128_ws2(__builtin_bit_cast(u32x4_t, av), ry, (uint32_t)(q * 16), 0);
      store_b128_ws2(__builtin_bit_cast(u32x4_t, o), ry2, (uint32_t)(q * 16), 0);
    }
  } else {
    // a thread's 8 pieces share its 8 channels (pc = tid % 16); every operand piece of the 8 is
    // loaded before the first is used (one memory latency for the epilogue)
    const int pc = tid & 15;
    bf16x8 mv[8], gv[8], av[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int64_t off = pair0 + (int64_t)(tid + 512 * k) * 8;
      mv[k] = *(const bf16x8*)(a.m + off);
      if (a.g2) gv[k] = *(const bf16x8*)(a.g2 + off);
      if constexpr (EPI == EPI_RES) av[k] = *(const bf16x8*)(a.pa + off);
    }
    float cbv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) cbv[e] = EPI == EPI_RES ? (float)a.cb[8 * pc + e] : 0.f;
    const __amdgpu_buffer_rsrc_t ry2 =
        make_rsrc(EPI == EPI_RES ? a.y2 + pair0 : a.y + pair0, 2 * CF_W * CW_C * 2);
    float sum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) sum[e] = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = tid + 512 * k;
      const int px = q >> 4;
      const bf16x8 gt = *(const bf16x8*)(ot + px * OROW + 16 * pc);
      bf16x8 o, o2;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float g = (float)gt[e];
        if (a.g2) g += (float)gv[k][e];
        o[e] = (bf16)((float)mv[k][e] > 0.f ? g : 0.f);
        if constexpr (EPI == EPI_RES) {
          const float pre = (float)(bf16)((float)av[k][e] + cbv[e]);  // bf16(a + cb), enc_res_bwd's
          o2[e] = pre > 0.f ? o[e] : (bf16)0.f;
          sum[e] += (float)o2[e];
        } else {
          sum[e] += (float)o[e];
        }
      }
      store_b128_ws2(__builtin_bit_cast(u32x4_t, o), ry, (uint32_t)(q * 16), 0);
      if constexpr (EPI == EPI_RES) store_b128_ws2(__builtin_bit_cast(u32x4_t, o2), ry2, (uint32_t)(q * 16), 0);
    }
    // the workgroup's channel sums: [32 pixel slots][128 channels] in LDS (the tile's reads are done
    // after the barrier), then rows added in slot order
    __syncthreads();
    float* red = (float*)smem_cf;
#pragma unroll
    for (int e = 0; e < 8; ++e) red[(tid >> 4) * CW_C + 8 * pc + e] = sum[e];
    __syncthreads();
    if (tid < CW_C) {
      float t = 0.f;
#pragma unroll 8
      for (int r = 0; r < 32; ++r) t += red[r * CW_C + tid];
      a.part[(int64_t)blockIdx.x * CW_C + tid] = t;
    }
  }
}

// db[c] = sum over the workgroups' partial rows part[b][c], b in order: one workgroup per channel,
// thread t adds rows t, t + 256, ... (all loads in flight), then a fixed-order tree in LDS.
__global__ __launch_bounds__(256) void conv_chan_reduce_kernel(const float* part, int nblk, float* db) {
  __shared__ float red[256];
  const int c = blockIdx.x, t = threadIdx.x;
  float s = 0.f;
  for (int b = t; b < nblk; b += 256) s += part[(int64_t)b * CW_C + c];
  red[t] = s;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) db[c] = red[0];
}

}  // namespace siren

namespace siren {

// ------------------------------------------------------------------------------------------
// The same two kernels for the encoder's other convolution shapes: an odd
// filter size KS (3, 5, 7), CI input channels (a multiple of 32), output channels in tiles of COT
// (forward) or 32 CB (weight gradient), images 128 pixels wide (forward) / a multiple of 64
// (weight gradient). ConvImgEncoder's cnn[0] (64 -> 128, 7x7 in configs 4/5: modules.py:351) and
// its input gradient (128 -> 64, the flipped filter), their 3x3 forms (kernel_size=3, the default),
// and the 128 -> 128 5x5 residual convolutions (which keep conv_fwd_k5_kernel / conv_wrw_k5_kernel).
// Same tiling, pipelines and arithmetic as those: per stage one filter row kh and a 32-channel
// chunk; the K order per output element is (kh, chunk, kw, channel), as there.
// ------------------------------------------------------------------------------------------
struct ConvGArgs {
  const bf16* x;     // [N][H][W][CI]
  const bf16* w;     // forward: [CO][KS][KS][CI]
  const bf16* bias;  // [CO] or null
  bf16* y;           // forward: [N][H][W][CO]
  const bf16* dy;    // weight gradient: [N][H][W][CO]
  float* part;       // weight gradient: [nsplit][KS][KS][CO][CI]
  float* dw;         // weight gradient: [CO][KS][KS][CI]
  int N, H, W, CO;
  int relu;
  int64_t rows_per_split;
  int nsplit;
};

// wait for all but the N youngest LDS reads, then tie every fragment to that wait (the compiler
// takes an asm output as defined at the asm: an MFMA operand tied after the wait reads landed data)
// (the counter holds 15 at most: a larger N waits for 15, i.e. for more of the reads — still correct)
template <int N>
DEV void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N < 15 ? N : 15) : "memory");
}
DEV void tie(TrFrag& f) { asm volatile("" : "+v"(f.lo), "+v"(f.hi)); }
DEV void tie(bf16x8& v) { asm volatile("" : "+v"(v)); }

// DMA (option conv_dma 2, as conv_fwd_k5_kernel's form 2): the stage image filled by LDS-DMA
// one stage ahead, each lane's source offsets computed once per workgroup; the x part padded to
// whole 1 KB instructions (the filter part is KS x COT rows of 80 bytes: a multiple of 1 KB).
template <int KS, int CI, int COT, bool DMA = false>
__global__ __launch_bounds__(512) void conv_fwd_gen_kernel(ConvGArgs a) {
  constexpr int HALO = CF_W + KS - 1;
  constexpr int HALOP = (HALO + 7) / 8 * 8;  // LDS rows per image row, padded (conv_fwd_k5_kernel's cf_row)
  constexpr int XB0 = 2 * HALOP * CF_ROWB;
  constexpr int XB = DMA ? (XB0 + 1023) / 1024 * 1024 : XB0;
  constexpr int WB = KS * COT * CF_ROWB;
  static_assert(!DMA || WB % 1024 == 0, "filter part in whole DMA instructions");
  constexpr int STAGE = XB + WB;
  constexpr int DXN = XB / 1024, DN = DXN + WB / 1024, DPW = (DN + 7) / 8;  // DMA instructions
  constexpr int XP = 2 * HALOP * 4, WP = KS * COT * 4;
  constexpr int NL = (XP + WP + 511) / 512;
  constexpr int NCC = CI / CF_CC;
  constexpr int NS = KS * NCC;
  constexpr int NI = COT / 64;  // 32-channel blocks per wave
  static_assert(CI % CF_CC == 0 && (COT == 64 || COT == 128) && KS % 2 == 1, "conv shape");
  static_assert(2 * STAGE <= 160 * 1024, "two LDS stages");
  __shared__ __attribute__((aligned(16))) char smem_g[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave & 1, wp = wave >> 1;
  const int hp = a.H / 2;
  const int n = blockIdx.x / hp, h0 = 2 * (blockIdx.x % hp);
  const int co0 = blockIdx.y * COT;
  // the epilogue's kernel arguments, loaded here: a scalar load left in flight inside the K loop
  // would void its counted LDS waits (lgkmcnt counts both, scalar loads out of order;
  // tools/check_lds_hazard.py)
  int CO = a.CO, relu = a.relu;
  uint64_t ybits = (uint64_t)a.y, bbits = (uint64_t)a.bias;
  asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(CO), "+s"(relu), "+s"(ybits), "+s"(bbits));
  bf16* const yout = (bf16*)ybits;
  const bf16* const bias = (const bf16*)bbits;

  f32x16 acc[NI][2];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  u32x4_t lv[2][NL];
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  auto load = [&](int s, auto set_c) {
    constexpr int set = decltype(set_c)::value;
    const int kh = s / NCC, cc = s % NCC;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int q = tid + 512 * i;
      u32x4_t v = zero;
      if (q < XP) {
        const int r = q / (4 * HALOP), j = cf_row(q - r * 4 * HALOP), pc = q & 3;
        const int xr = h0 + r + kh - KS / 2, w = j - KS / 2;
        if (xr >= 0 && xr < a.H && w >= 0 && w < CF_W && j < HALO)
          v = *(const u32x4_t*)(a.x + (((int64_t)n * a.H + xr) * CF_W + w) * CI + CF_CC * cc + 8 * pc);
      } else if (q < XP + WP) {
        const int q2 = q - XP, kw = q2 / (4 * COT), co = cf_row(q2 % (4 * COT)), pc = q2 & 3;
        v = *(const u32x4_t*)(a.w + ((int64_t)((co0 + co) * KS + kh) * KS + kw) * CI + CF_CC * cc + 8 * pc);
      }
      lv[set][i] = v;
    }
  };
  auto stage = [&](auto set_c, int buf) {
    constexpr int set = decltype(set_c)::value;
    char* base = smem_g + buf * STAGE;
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int q = tid + 512 * i;
      if (q < XP) {
        const int r = q / (4 * HALOP), j = cf_row(q - r * 4 * HALOP), pc = q & 3;
        *(u32x4_t*)(base + (r * HALOP + j) * CF_ROWB + 16 * pc) = lv[set][i];
      } else if (q < XP + WP) {
        const int q2 = q - XP, kw = q2 / (4 * COT), co = cf_row(q2 % (4 * COT)), pc = q2 & 3;
        *(u32x4_t*)(base + XB + (kw * COT + co) * CF_ROWB + 16 * pc) = lv[set][i];
      }
    }
  };

  // A (filter) lane -> out channel (COT / 2) wc + 32 i + (lane & 31); B (pixels) lane -> pixel
  // 64 wp + 32 j + (lane & 31) of the row pair, the tap's halo column + kw
  const int l32 = lane & 31, kh2 = lane >> 5;
  uint32_t aoff[NI], boff[2];
#pragma unroll
  for (int i = 0; i < NI; ++i) aoff[i] = XB + ((COT / 2) * wc + 32 * i + l32) * CF_ROWB + 16 * kh2;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int px = 64 * wp + 32 * j + l32;
    boff[j] = ((px >> 7) * HALOP + (px & 127)) * CF_ROWB + 16 * kh2;
  }
  const uint32_t sbase = lds_addr(smem_g);

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  // DMA: instruction g = wave + 8 i fills slots 64 g .. 64 g + 63 of the stage (rows of 5 slots: 4
  // channel pieces + the pad); per lane the stage-(0, 0) source offset and (x part) the row test
  int pbase[DPW], prow[DPW];
  const __amdgpu_buffer_rsrc_t rX = make_rsrc(a.x + (int64_t)n * a.H * CF_W * CI, (int64_t)a.H * CF_W * CI * 2);
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(a.w, (int64_t)CO * KS * KS * CI * 2);
  if constexpr (DMA) {
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int g = wave + 8 * i;
      if (g < DXN) {
        const int slot = 64 * g + lane, row = slot / 5, pc = slot - 5 * (slot / 5);
        const int r = row >= HALOP ? 1 : 0, j = row - r * HALOP, w = j - KS / 2;
        const bool ok = row < 2 * HALOP && pc < 4 && j < HALO && w >= 0 && w < CF_W;
        prow[i] = ok ? h0 + r - KS / 2 : -(1 << 20);
        pbase[i] = ((h0 + r - KS / 2) * CF_W + w) * CI * 2 + 16 * pc;
      } else {
        const int slot = 64 * (g - DXN) + lane, row = slot / 5, pc = slot - 5 * (slot / 5);
        const int kw = row / COT, co = row - COT * (row / COT);
        prow[i] = 0;
        pbase[i] = (g < DN && pc < 4 && kw < KS) ? ((co0 + co) * KS * KS * CI + kw * CI + 8 * pc) * 2 : 0x7fff0000;
      }
    }
  }
  auto dma = [&](int s, int buf) {
    const int kh = s / NCC, cc = s % NCC;
    char* base = smem_g + buf * STAGE;
    const int xadd = kh * CF_W * CI * 2 + CF_CC * cc * 2, wadd = kh * KS * CI * 2 + CF_CC * cc * 2;
#pragma unroll
    for (int i = 0; i < DPW; ++i) {
      const int g = wave + 8 * i;  // wave-uniform
      if (g < DXN) {
        const uint32_t off = (uint32_t)(prow[i] + kh) < (uint32_t)a.H ? (uint32_t)(pbase[i] + xadd) : 0x7fffffffu;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)(base + 1024 * g), 16, off, 0, 0, 0);
      } else if (g < DN) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(base + 1024 * g), 16, (uint32_t)(pbase[i] + wadd), 0,
                                                 0, 0);
      }
    }
  };
  if constexpr (DMA) {
    dma(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    load(0, S0{});
    stage(S0{}, 0);
    if (NS > 1) load(1, S1{});
  }
  __syncthreads();
  auto iter = [&](int s, auto par_c) {
    constexpr int par = decltype(par_c)::value;
    using SN = std::integral_constant<int, par ^ 1>;
    using SC = std::integral_constant<int, par>;
    if constexpr (DMA) {
      if (s + 1 < NS) dma(s + 1, (s + 1) & 1);
    } else {
      if (s + 1 < NS) stage(SN{}, (s + 1) & 1);
      if (s + 2 < NS) load(s + 2, SC{});
    }
    const uint32_t sb = sbase + (s & 1) * STAGE;
    // 2 KS K steps (kw, ks); step i + 1's fragments are read while step i's MFMAs run
    bf16x8 af[2][NI], bfr[2][2];
#define SIREN_CG_RD(I)                                                                                               \
  {                                                                                                                  \
    constexpr int kw_ = (I) >> 1, ks_ = (I) & 1, b_ = (I) & 1;                                                       \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(af[b_][0]) : "v"(sb + aoff[0]), "n"(kw_ * COT * CF_ROWB + 32 * ks_)); \
    if constexpr (NI > 1)                                                                                            \
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(af[b_][NI - 1]) : "v"(sb + aoff[NI - 1]), "n"(kw_ * COT * CF_ROWB + 32 * ks_)); \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bfr[b_][0]) : "v"(sb + boff[0]), "n"(kw_ * CF_ROWB + 32 * ks_));    \
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(bfr[b_][1]) : "v"(sb + boff[1]), "n"(kw_ * CF_ROWB + 32 * ks_));    \
  }
    static_assert(NI == 1 || NI == 2, "one or two 32-channel blocks per wave");
    SIREN_CG_RD(0)
    static_for<0, 2 * KS>([&](auto i_c) {
      constexpr int i = decltype(i_c)::value, b = i & 1;
      if constexpr (i + 1 < 2 * KS) {
        SIREN_CG_RD(i + 1)
        lgkm_wait<NI + 2>();
      } else {
        lgkm_wait<0>();
      }
#pragma unroll
      for (int ii = 0; ii < NI; ++ii) tie(af[b][ii]);
      tie(bfr[b][0]);
      tie(bfr[b][1]);
#pragma unroll
      for (int ii = 0; ii < NI; ++ii)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ii][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[b][ii], bfr[b][j], acc[ii][j], 0, 0, 0);
    });
#undef SIREN_CG_RD
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage s + 1
    __syncthreads();
  };
  for (int s = 0; s < NS; s += 2) {
    iter(s, S0{});
    if (s + 1 < NS) iter(s + 1, S1{});
  }

  // epilogue: D[co][px] -> LDS tile [256 px][COT] bf16, then 16-byte stores of whole pixel rows
  constexpr int OROW = COT * 2 + 16;
  static_assert(256 * OROW <= 2 * STAGE, "output tile");
  char* ot = smem_g;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int px = 64 * wp + 32 * j + l32;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = (COT / 2) * wc + 32 * i + 8 * g + 4 * kh2 + e;
          float z = (float)(bf16)acc[i][j][4 * g + e];
          if (bias) {
            z = (float)(bf16)(z + (float)bias[co0 + co]);
            if (relu) z = fmaxf(z, 0.f);
          }
          v[e] = (bf16)z;
        }
        const int co = (COT / 2) * wc + 32 * i + 8 * g + 4 * kh2;
        *(bf16x4*)(ot + px * OROW + co * 2) = v;
      }
    }
  __syncthreads();
  // the pair's 256 px x COT channels as 16-byte buffer stores (each with its 2 wait states)
  const __amdgpu_buffer_rsrc_t ry = make_rsrc(yout + ((int64_t)n * a.H + h0) * CF_W * CO, 2 * CF_W * CO * 2);
  constexpr int PPR = COT / 8;  // 16-byte pieces per pixel
#pragma unroll
  for (int k = 0; k < 256 * PPR / 512; ++k) {
    const int q = tid + 512 * k;
    const int px = q / PPR, pc = q % PPR;
    store_b128_ws2(*(const u32x4_t*)(ot + px * OROW + 16 * pc), ry, (uint32_t)((px * CO + co0 + 8 * pc) * 2), 0);
  }
}

// DMA (option wrw_dma 3, W a multiple of 128): conv_wrw_k5_kernel's 128-pixel LDS-DMA form for
// these shapes — two stages, the next chunk's DMA one chunk ahead, lane offsets fixed per
// workgroup (rows of COW / 8 + 4 and CI / 8 + 4 16-byte slots, the pads and pixels outside the
// image out of range); the same K steps in the same pixel order as the 64-pixel form.
template <int KS, int CI, int CB, bool DMA = false>
__global__ __launch_bounds__(512) void conv_wrw_gen_kernel(ConvGArgs a) {
  constexpr int IB = CI / 32;
  static_assert(CB * IB == 8, "8 waves: CB co blocks x IB ci blocks");
  constexpr int PX = DMA ? 2 * CW_PX : CW_PX;  // pixels per chunk
  constexpr int NB = DMA ? 2 : CW_NB;          // LDS stages
  constexpr int COW = 32 * CB;                 // output channels per workgroup
  constexpr int XR = PX + KS - 1;              // halo rows
  constexpr int DROW = COW + 32, XROW = CI + 32;  // bf16 per staged row (+64-byte pad)
  constexpr int DP = CW_PX * COW / 8, XPC = (CW_PX + KS - 1) * CI / 8;  // 16-byte pieces (64-pixel form)
  constexpr int NDL = (DP + 511) / 512, NXL = (XPC + 511) / 512;
  constexpr int DSL = COW / 8 + 4, XSL = CI / 8 + 4;  // 16-byte slots per staged row
  constexpr int DMA_D = PX * DSL / 64, DMA_X = (XR * XSL + 63) / 64, DMA_N = DMA_D + DMA_X;
  constexpr int DMA_PER_WAVE = (DMA_N + 7) / 8;
  __shared__ __attribute__((aligned(16))) bf16 sD[NB][PX * DROW];
  __shared__ __attribute__((aligned(16))) bf16 sX[NB][DMA ? DMA_X * 512 : XR * XROW];
  const int split = blockIdx.x, kh = blockIdx.y, ch = blockIdx.z;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cb = wave % CB, ib = wave / CB;
  const int nrows = a.N * a.H;
  const int r0 = split * (int)a.rows_per_split;
  const int r1 = r0 + (int)a.rows_per_split < nrows ? r0 + (int)a.rows_per_split : nrows;
  const int nch = a.W / PX;
  const int T = r1 > r0 ? (r1 - r0) * nch : 0;
  const int CO = a.CO;

  f32x16 acc[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[k][e] = 0.f;

  // loader cursor over the chunks, loaded in order (conv_wrw_k5_kernel: no per-chunk division)
  int cn = r0 / a.H, crow = r0 - (r0 / a.H) * a.H, cpx = 0;
  u32x4_t dv[2][NDL], xv[2][NXL];
  const u32x4_t zero = {0u, 0u, 0u, 0u};
  auto load = [&](auto set_c) {
    constexpr int set = decltype(set_c)::value;
    const int n = cn, h = crow, px0 = cpx;
    cpx += CW_PX;
    if (cpx == a.W) {
      cpx = 0;
      if (++crow == a.H) {
        crow = 0;
        ++cn;
      }
    }
    const int xr = h + kh - KS / 2;
    const bool rowok = xr >= 0 && xr < a.H;
#pragma unroll
    for (int i = 0; i < NDL; ++i) {
      const int q = tid + 512 * i;
      const int px = q / (COW / 8), pc = q % (COW / 8);
      dv[set][i] = q < DP ? *(const u32x4_t*)(a.dy + (((int64_t)n * a.H + h) * a.W + px0 + px) * CO + COW * ch + 8 * pc)
                          : zero;
    }
    const bf16* xrow = a.x + ((int64_t)n * a.H + (rowok ? xr : 0)) * a.W * CI;
#pragma unroll
    for (int i = 0; i < NXL; ++i) {
      const int p = tid + 512 * i;
      const int w = px0 - KS / 2 + p / (CI / 8);
      const bool ok = p < XPC && rowok && w >= 0 && w < a.W;
      xv[set][i] = ok ? *(const u32x4_t*)(xrow + (int64_t)w * CI + 8 * (p % (CI / 8))) : zero;
    }
  };
  auto stage = [&](auto set_c, int buf) {
    constexpr int set = decltype(set_c)::value;
#pragma unroll
    for (int i = 0; i < NDL; ++i) {
      const int q = tid + 512 * i;
      if (q < DP) *(u32x4_t*)(&sD[buf][(q / (COW / 8)) * DROW + 8 * (q % (COW / 8))]) = dv[set][i];
    }
#pragma unroll
    for (int i = 0; i < NXL; ++i) {
      const int p = tid + 512 * i;
      if (p < XPC) *(u32x4_t*)(&sX[buf][(p / (CI / 8)) * XROW + 8 * (p % (CI / 8))]) = xv[set][i];
    }
  };

  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int ca = 32 * cb + 16 * (g & 1) + 4 * tp;
  const int cx = 32 * ib + 16 * (g & 1) + 4 * tp;
  const int r8 = 8 * (g >> 1) + tq;
  const uint32_t dbase = lds_addr(&sD[0][0]) + (uint32_t)((r8 * DROW + ca) * 2);
  const uint32_t xbase = lds_addr(&sX[0][0]) + (uint32_t)((r8 * XROW + cx) * 2);
  constexpr uint32_t DSTAGE = PX * DROW * 2, XSTAGE = DMA ? DMA_X * 1024 : XR * XROW * 2;
  constexpr int DROWB = DROW * 2, XROWB = XROW * 2;
  constexpr int NRD = 2 + 2 * KS;  // fragment reads per K step

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  int voff[DMA_PER_WAVE];
  if constexpr (DMA) {
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; ++i) {
      const int gi = wave + 8 * i;
      if (gi < DMA_D) {
        const int slot = 64 * gi + lane, row = slot / DSL, pc = slot - DSL * (slot / DSL);
        voff[i] = pc < COW / 8 ? row * CO * 2 + 16 * pc : 0x7fffffff;
      } else {
        const int slot = 64 * (gi - DMA_D) + lane, row = slot / XSL, pc = slot - XSL * (slot / XSL);
        voff[i] = (pc < CI / 8 && row < XR) ? (row - KS / 2) * CI * 2 + 16 * pc : 0x40000000;
      }
    }
  }
  auto dma = [&](int buf) {
    const int n = cn, h = crow, px0 = cpx;
    cpx += PX;
    if (cpx == a.W) {
      cpx = 0;
      if (++crow == a.H) {
        crow = 0;
        ++cn;
      }
    }
    const int xr = h + kh - KS / 2;
    const bool rowok = xr >= 0 && xr < a.H;
    const __amdgpu_buffer_rsrc_t rD = make_rsrc(a.dy + (((int64_t)n * a.H + h) * a.W + px0) * CO + COW * ch,
                                                ((int64_t)(PX - 1) * CO + COW) * 2);
    const __amdgpu_buffer_rsrc_t rX =
        make_rsrc(a.x + ((int64_t)n * a.H + (rowok ? xr : 0)) * a.W * CI, rowok ? (int64_t)a.W * CI * 2 : 0);
#pragma unroll
    for (int i = 0; i < DMA_PER_WAVE; ++i) {
      const int gi = wave + 8 * i;  // wave-uniform
      if (gi < DMA_D)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rD, (lds_void*)((char*)&sD[buf][0] + 1024 * gi), 16,
                                                 (uint32_t)voff[i], 0, 0, 0);
      else if (gi < DMA_N)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_void*)((char*)&sX[buf][0] + 1024 * (gi - DMA_D)), 16,
                                                 (uint32_t)(voff[i] + px0 * CI * 2), 0, 0, 0);
    }
  };
  if constexpr (DMA) {
    if (T > 0) dma(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else {
    if (T > 0) {
      load(S0{});
      stage(S0{}, 0);
    }
    if (T > 1) load(S1{});
  }
  int bcur = 0;  // t % CW_NB
  __syncthreads();
  auto iter = [&](int t, auto par_c) {
    constexpr int par = decltype(par_c)::value;
    using SN = std::integral_constant<int, par ^ 1>;
    using SC = std::integral_constant<int, par>;
    const int buf = DMA ? par : bcur;
    bcur = bcur == CW_NB - 1 ? 0 : bcur + 1;
    if constexpr (DMA) {
      if (t + 1 < T) dma(par ^ 1);  // stage (t + 1) & 1: last read by chunk t - 1
    } else {
      if (t + 1 < T) stage(SN{}, bcur);
      if (t + 2 < T) load(SC{});
    }
    const uint32_t db = dbase + buf * DSTAGE, xb = xbase + buf * XSTAGE;
    TrFrag fa[2], fb[2][KS];
#define SIREN_CWG_RD(KS_)                                                         \
  {                                                                               \
    constexpr int ks_ = (KS_), b_ = (KS_) & 1;                                    \
    tr16_read<16 * ks_ * DROWB>(fa[b_].lo, db);                                   \
    tr16_read<16 * ks_ * DROWB + 4 * DROWB>(fa[b_].hi, db);                       \
    static_for<0, KS>([&](auto kw_c) {                                            \
      constexpr int kw = decltype(kw_c)::value;                                   \
      tr16_read<(16 * ks_ + kw) * XROWB>(fb[b_][kw].lo, xb);                      \
      tr16_read<(16 * ks_ + kw + 4) * XROWB>(fb[b_][kw].hi, xb);                  \
    });                                                                           \
  }
    SIREN_CWG_RD(0)
    static_for<0, PX / 16>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value, b = ks & 1;
      if constexpr (ks + 1 < PX / 16) {
        SIREN_CWG_RD(ks + 1)
        lgkm_wait<NRD>();
      } else {
        lgkm_wait<0>();
      }
      tie(fa[b]);
      static_for<0, KS>([&](auto kw_c) { tie(fb[b][decltype(kw_c)::value]); });
      static_for<0, KS>([&](auto kw_c) {
        constexpr int kw = decltype(kw_c)::value;
        acc[kw] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr16_value(fa[b]), tr16_value(fb[b][kw]), acc[kw], 0, 0, 0);
      });
    });
#undef SIREN_CWG_RD
    if constexpr (DMA) {
      // this wave's part of chunk t + 1 landed; a barrier without __syncthreads' fence
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      __syncthreads();
    }
  };
  for (int t = 0; t < T; t += 2) {
    iter(t, S0{});
    if (t + 1 < T) iter(t + 1, S1{});
  }

  // partial: [split][kh][kw][co][ci]
  float* P = a.part + ((int64_t)split * KS + kh) * KS * (int64_t)CO * CI;
#pragma unroll
  for (int kw = 0; kw < KS; ++kw) {
    const int ci = 32 * ib + (lane & 31);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int co = COW * ch + 32 * cb + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      P[((int64_t)kw * CO + co) * CI + ci] = acc[kw][e];
    }
  }
}

// dw[co][kh][kw][ci] = sum_s part[s][kh][kw][co][ci], splits in order
template <int KS, int CI>
__global__ __launch_bounds__(256) void conv_wrw_gen_reduce_kernel(ConvGArgs a) {
  const int64_t slab = (int64_t)KS * KS * a.CO * CI;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // over [kh][kw][co][ci]
  if (i >= slab) return;
  const int ci = (int)(i % CI);
  const int co = (int)((i / CI) % a.CO);
  const int tap = (int)(i / ((int64_t)CI * a.CO));
  float s = 0.f;
  for (int sp = 0; sp < a.nsplit; ++sp) s += a.part[(int64_t)sp * slab + i];
  a.dw[((int64_t)co * KS * KS + tap) * CI + ci] = s;
}

}  // namespace siren

namespace siren {

// ------------------------------------------------------------------------------------------
// conv_theta: ConvImgEncoder's first convolution (modules.py:359) over the 2-channel k-space image
// (real, imaginary): CI = 2, a KS x KS filter (3, 5, 7), CO a multiple of 32 up to 128. The
// reduction per output is only 2 KS^2 <= 98 long, so the GEMM is laid out per filter row: one
// 32x32x16 MFMA per (kh, 32 outputs, 32 channels) whose 16 K slots are the row's (kw, ci) pairs —
// 2 KS consecutive bf16 of the NHWC input row, zero-weighted past 2 KS. The output (64 channels,
// 67 MB per C4 step) is the traffic that bounds the forward; the weight gradient reads dy once.
// ------------------------------------------------------------------------------------------
struct ConvTArgs {
  const bf16* x;      // [N][H][W][2]
  const bf16* w;      // forward: [CO][KS][KS][2]
  const bf16* bias;   // [CO] or null
  bf16* y;            // forward: [N][H][W][CO]
  const bf16* dy;     // weight gradient: [N][H][W][CO]
  float* part;        // weight gradient: [nsplit][CO][32 NNT] (column kh * 16 + 2 kw + ci)
  float* dw;          // weight gradient: [CO][KS][KS][2]
  int N, H, W, CO;
  int relu;
  int rows_per_block;      // forward: image rows per workgroup
  int64_t chunks_per_split;  // weight gradient: 32-pixel chunks per split
  int nsplit;
};

constexpr int CT_W = 128;   // forward: image width (4 waves x 32 pixels)
constexpr int CT_RPB = 4;   // forward: image rows per workgroup

template <int KS, int NCT>
__global__ __launch_bounds__(256) void conv_t_fwd_kernel(ConvTArgs a) {
  constexpr int PAD = KS / 2, CO = 32 * NCT, OROW = CO * 2 + 16;
  static_assert(KS % 2 == 1 && KS <= 7 && NCT >= 1 && NCT <= 4, "conv_theta shape");
  __shared__ __attribute__((aligned(16))) char ot[CT_W * OROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hf = lane >> 5;
  const int px = 32 * wave + l32;
  const int H = a.H;
  const int64_t nrows = (int64_t)a.N * H;
  const int64_t r0 = (int64_t)blockIdx.x * a.rows_per_block;
  const int64_t r1 = r0 + a.rows_per_block < nrows ? r0 + a.rows_per_block : nrows;

  // A operands (filter rows): lane -> out channel 32 ct + l32, K slots 8 hf .. 8 hf + 7 = (kw, ci)
  bf16x8 af[KS][NCT];
#pragma unroll
  for (int kh = 0; kh < KS; ++kh)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kw = 4 * hf + (j >> 1), ci = j & 1;
        af[kh][ct][j] = kw < KS ? a.w[(((32 * ct + l32) * KS + kh) * KS + kw) * 2 + ci] : (bf16)0.f;
      }
  const uint32_t* xw = (const uint32_t*)a.x;  // one 32-bit word = one pixel's two channels

  for (int64_t r = r0; r < r1; ++r) {
    const int n = (int)(r / H), h = (int)(r % H);
    // B operands: lane -> pixel px, K slots (kw = 4 hf + q, ci): 4 words per filter row
    u32x4_t xv[KS];
#pragma unroll
    for (int kh = 0; kh < KS; ++kh) {
      const int xr = h + kh - PAD;
      const bool rok = xr >= 0 && xr < H;
      const int64_t rb = ((int64_t)n * H + (rok ? xr : 0)) * a.W;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int kw = 4 * hf + q, p = px + kw - PAD;
        xv[kh][q] = (rok && kw < KS && p >= 0 && p < a.W) ? xw[rb + p] : 0u;
      }
    }
    f32x16 acc[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[ct][e] = 0.f;
#pragma unroll
    for (int kh = 0; kh < KS; ++kh) {
      const bf16x8 bv = __builtin_bit_cast(bf16x8, xv[kh]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kh][ct], bv, acc[ct], 0, 0, 0);
    }
    // D[co][px] -> LDS tile [128 px][CO] (bias, ReLU: the conv + bias-add + ReLU chain's roundings)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = 32 * ct + 8 * g + 4 * hf + e;
          float z = (float)(bf16)acc[ct][4 * g + e];
          if (a.bias) {
            z = (float)(bf16)(z + (float)a.bias[co]);
            if (a.relu) z = fmaxf(z, 0.f);
          }
          v[e] = (bf16)z;
        }
        *(bf16x4*)(ot + px * OROW + (32 * ct + 8 * g + 4 * hf) * 2) = v;
      }
    __syncthreads();
    // the row's CT_W x CO outputs as 16-byte buffer stores, each with its 2 wait states
    // (siren_common.h store_b128_ws2)
    constexpr int PPR = CO / 8;  // 16-byte pieces per pixel
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.y + r * (int64_t)CT_W * CO, CT_W * CO * 2);
#pragma unroll
    for (int k = 0; k < CT_W * PPR / 256; ++k) {
      const int q = tid + 256 * k;
      const int p = q / PPR, pc = q % PPR;
      store_b128_ws2(*(const u32x4_t*)(ot + p * OROW + 16 * pc), ry, (uint32_t)(q * 16), 0);
    }
    __syncthreads();
  }
}

// Weight gradient: D[co][kh 16 + 2 kw + ci] = sum over pixels of dy[px][co] x[px + (kh, kw)][ci].
// Per 64-pixel chunk of an image row: an LDS dy tile [64 px][CO], the chunk's KS input rows
// (64 + KS - 1 pixels each, staged as they come from HBM), and from those an im2col tile
// [64 px][32 NNT] (the KS rows' (kw, ci) pairs, zero past each row's 2 KS slots); both tiles are
// read by transposing fragment reads (pixels = K). Each chunk's dy and input words are loaded
// into registers two chunks ahead of its expansion and multiply (~48 KB in flight per CU at 3
// workgroups). 4 waves, the (CO / 32) x NNT output tiles dealt round-robin; one partial slab per split, reduced in split order by
// conv_t_wrw_reduce_kernel.
constexpr int CT_PX = 64;  // weight gradient: pixels per chunk
template <int KS, int NCT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NCT == 4 ? 2 : 3))) void conv_t_wrw_kernel(ConvTArgs a) {
  constexpr int PAD = KS / 2, CO = 32 * NCT;
  constexpr int NNT = (KS * 16 + 31) / 32, NCOL = 32 * NNT;
  constexpr int NTILE = NCT * NNT, TPW = (NTILE + 3) / 4;
  constexpr int DROW = CO + 16, XROW = NCOL + 16;  // bf16 per LDS row (+32-byte pad)
  constexpr int XW = CT_PX + KS - 1;              // input pixels per staged row
  constexpr int NDY = CT_PX * CO / 8 / 256;       // 16-byte dy pieces per thread
  constexpr int NXV = (KS * XW + 255) / 256;      // input words per thread
  static_assert(CT_PX * CO / 8 % 256 == 0, "dy pieces");
  __shared__ __attribute__((aligned(16))) bf16 sD[CT_PX * DROW];
  __shared__ __attribute__((aligned(16))) bf16 sX[CT_PX * XROW];
  __shared__ uint32_t sR[KS * XW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int split = blockIdx.x;
  const int nch = a.W / CT_PX;
  const int64_t nchunk = (int64_t)a.N * a.H * nch;
  const int64_t c0 = (int64_t)split * a.chunks_per_split;
  const int64_t c1 = c0 + a.chunks_per_split < nchunk ? c0 + a.chunks_per_split : nchunk;

  // the im2col tile's zero columns (past 2 KS in each row's 16, and rows kh >= KS) are never
  // rewritten: clear the whole tile once
  for (int i = tid; i < CT_PX * XROW / 2; i += 256) ((uint32_t*)sX)[i] = 0u;

  f32x16 acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

  const int g = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const int r8 = 8 * (g >> 1) + tq, cc = 16 * (g & 1) + 4 * tp;
  const uint32_t dl = lds_addr(sD) + (uint32_t)((r8 * DROW + cc) * 2);
  const uint32_t xl = lds_addr(sX) + (uint32_t)((r8 * XROW + cc) * 2);
  const uint32_t* xw = (const uint32_t*)a.x;

  // two chunks' loads in flight ahead of the one being multiplied (register sets 0 / 1)
  u32x4_t dyv[2][NDY];
  uint32_t xv[2][NXV];
  auto load = [&](int64_t c, auto set_c) {
    constexpr int set = decltype(set_c)::value;
    const int64_t r = c / nch;
    const int px0 = (int)(c % nch) * CT_PX;
    const int n = (int)(r / a.H), h = (int)(r % a.H);
#pragma unroll
    for (int i = 0; i < NDY; ++i) {
      const int q = tid + 256 * i;
      const int p = q / (CO / 8), pc = q % (CO / 8);
      dyv[set][i] = *(const u32x4_t*)(a.dy + (r * a.W + px0 + p) * CO + 8 * pc);
    }
#pragma unroll
    for (int i = 0; i < NXV; ++i) {
      const int q = tid + 256 * i;
      const int kh = q / XW, j = q % XW;
      const int xr = h + kh - PAD, xp = px0 + j - PAD;
      xv[set][i] = (q < KS * XW && xr >= 0 && xr < a.H && xp >= 0 && xp < a.W) ? xw[((int64_t)n * a.H + xr) * a.W + xp]
                                                                                 : 0u;
    }
  };
  auto body = [&](int64_t c, auto set_c) {
    constexpr int set = decltype(set_c)::value;
    __syncthreads();  // the previous chunk's fragment reads and expansion are done
#pragma unroll
    for (int i = 0; i < NDY; ++i) {
      const int q = tid + 256 * i;
      *(u32x4_t*)(sD + (q / (CO / 8)) * DROW + 8 * (q % (CO / 8))) = dyv[set][i];
    }
#pragma unroll
    for (int i = 0; i < NXV; ++i) {
      const int q = tid + 256 * i;
      if (q < KS * XW) sR[q] = xv[set][i];
    }
    if (c + 2 < c1) load(c + 2, set_c);
    __syncthreads();
    // im2col: pixel p, filter row kh, tap kw -> one 32-bit word (both channels)
    for (int q = tid; q < CT_PX * KS * KS; q += 256) {
      const int p = q % CT_PX, t = q / CT_PX, kw = t % KS, kh = t / KS;
      *(uint32_t*)(sX + p * XROW + kh * 16 + 2 * kw) = sR[kh * XW + p + kw];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < CT_PX / 16; ++ks) {
      TrFrag fa[TPW], fb[TPW];
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int t = wave + 4 * i;
        const int ct = t < NTILE ? t / NNT : 0, nt = t < NTILE ? t % NNT : 0;
        const uint32_t da = dl + (uint32_t)((16 * ks * DROW + 32 * ct) * 2);
        const uint32_t xa = xl + (uint32_t)((16 * ks * XROW + 32 * nt) * 2);
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(fa[i].lo) : "v"(da));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(fa[i].hi) : "v"(da), "n"(4 * DROW * 2));
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(fb[i].lo) : "v"(xa));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(fb[i].hi) : "v"(xa), "n"(4 * XROW * 2));
      }
      lgkm_wait<0>();
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        tie(fa[i]);
        tie(fb[i]);
        if (wave + 4 * i < NTILE)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr16_value(fa[i]), tr16_value(fb[i]), acc[i], 0, 0, 0);
      }
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  if (c0 < c1) load(c0, S0{});
  if (c0 + 1 < c1) load(c0 + 1, S1{});
  for (int64_t c = c0; c < c1; c += 2) {
    body(c, S0{});
    if (c + 1 < c1) body(c + 1, S1{});
  }

  float* P = a.part + (int64_t)split * CO * NCOL;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wave + 4 * i;
    if (t >= NTILE) continue;
    const int ct = t / NNT, nt = t % NNT;
    const int col = 32 * nt + (lane & 31);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int co = 32 * ct + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      P[(int64_t)co * NCOL + col] = acc[i][e];
    }
  }
}

// dw[co][kh][kw][ci] = sum over splits of part[s][co][kh 16 + 2 kw + ci]: 16 outputs per
// workgroup, 16 split groups (s = g mod 16) summed in order, then the groups in order
template <int KS>
__global__ __launch_bounds__(256) void conv_t_wrw_reduce_kernel(ConvTArgs a) {
  constexpr int NCOL = 32 * ((KS * 16 + 31) / 32);
  __shared__ float red[16][17];
  const int o = threadIdx.x & 15, gs = threadIdx.x >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + o;  // over [co][kh][kw][ci]
  const int64_t total = (int64_t)a.CO * KS * KS * 2;
  float s = 0.f;
  int64_t src = 0;
  if (i < total) {
    const int ci = (int)(i & 1), kw = (int)((i >> 1) % KS), kh = (int)((i / (2 * KS)) % KS), co = (int)(i / (2 * KS * KS));
    src = (int64_t)co * NCOL + kh * 16 + 2 * kw + ci;
    const int64_t slab = (int64_t)a.CO * NCOL;
    for (int sp = gs; sp < a.nsplit; sp += 16) s += a.part[sp * slab + src];
  }
  red[gs][o] = s;
  __syncthreads();
  if (gs == 0 && i < total) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][o];
    a.dw[i] = t;
  }
}

}  // namespace siren

