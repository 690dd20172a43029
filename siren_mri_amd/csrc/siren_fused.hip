// siren_fused.hip — the whole SIREN forward in one persistent kernel (bf16 mode, gfx950).
//
// Per 128-row tile of coordinates the workgroup runs every layer on chip; HBM sees only x, the
// 16-bit phase tensors P_l the backward needs (skipped when no backward follows) and y:
//
//   layer 0   (VALU)  P_0 = enc(w0 (x W_0^T + b_0))                      modules.py:25-26,38
//   hidden l  (MFMA)  P_l = enc(w0 (sin(P_{l-1}) W_l^T + b_l))             modules.py:25-26,38
//   output    (VALU)  y   = sin(P_{L-2}) W_L^T + b_L  (optionally sin(w0 .))   modules.py:78
//
// Same arithmetic as the per-layer kernels (first_fwd / nt_bf16 / last_fwd), so the phases and y
// agree with the unfused path up to the MFMA's internal summation order.
//
// Structure (512 threads = 8 waves, one workgroup per CU):
//   * H (LDS, BM x F x 2 B, XOR-swizzled 16-byte chunks) holds the current layer's input. The
//     MFMA runs transposed, P^T = W . H^T: wave w owns output features [32w, 32w+32) for all BM
//     rows, its W_l operand is one coalesced 1 KB fragment per 16-wide K step, streamed from L2
//     (weights are prepared in fragment order) into registers one layer ahead; H supplies the B
//     fragments (ds_read_b128, conflict-free under the swizzle).
//   * epilogue: each lane holds 4 consecutive features of a row per accumulator group, so the
//     phases go to LDS as 8-byte writes, in place over H (all waves are past their reads).
//   * convert pass: each thread takes 16-byte phase chunks, stores them to P_l (coalesced rows),
//     and writes sin(P_l) as bf16 back to the same LDS chunk (the next layer's operand), or — for
//     the last sine layer — forms the output dot products (32-lane shuffle reduction per row).
#include <type_traits>

#include "siren_common.h"

namespace siren {

constexpr int FUSED_BM = 128;

struct FusedFwdArgs {
  const float* x;                 // [rows, C]
  const float* W0;                // [nb_w][F, C]
  const float* b0;                // [nb_w][F]
  const bf16* Wfrag;              // [nb_w][nh][F/32][F/16][64 lanes][8] bf16 (fragment order)
  const float* bias[FUSED_MAXH];  // hidden layer biases [nb_w][F]
  const float* WL;                // [nb_w][O, F]
  const float* bL;                // [nb_w][O]
  void* P[FUSED_MAXH + 1];        // phase outputs of sine layers 0..nh (null: not kept)
  float* y;                       // [rows, O]
  long long* prof;                // debug: per-workgroup phase cycle counters (null: off)
  int64_t rows_per_batch;
  int batched;                    // 1: weight set = blockIdx.y
  int C, F, O, nh;
  int sine_out;
  float w0;
  int dbg;                        // debug timing only: bit 0 skips the K-loop fillers, bit 1 the VALU segment
};

constexpr int FUSED_NPROF = 4;    // layer-0 pass, MFMA K loop, epilogue, convert pass

DEV void fused_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int F, int C>
__global__ __launch_bounds__(512) void fused_fwd_bf16_kernel(FusedFwdArgs a) {
  using PT = Prec<kPrecBF16>;
  constexpr int BM = FUSED_BM;
  constexpr int CPR = F / 8;                // 16-byte chunks per row
  constexpr int LG_CPR = __builtin_ctz(CPR);
  constexpr int SMASK = (CPR < 16 ? CPR : 16) - 1;
  constexpr int NQ = BM * CPR / 512;        // chunks per thread in the VALU passes
  constexpr int RSTEP = 512 / CPR;          // rows between a thread's chunks
  constexpr int NKS = F / 16;               // MFMA K steps
  constexpr int NBM = BM / 32;
  constexpr int NWAVE_F = F / 32;           // waves with MFMA work

  __shared__ __attribute__((aligned(16))) char H[BM * F * 2];
  __shared__ __attribute__((aligned(16))) float Sw0[C * F + F];      // W0^T [C][F], k * b0
  __shared__ __attribute__((aligned(16))) float Sb[FUSED_MAXH * F];  // k * hidden biases
  __shared__ __attribute__((aligned(16))) float Swl[FUSED_MAXO * F + FUSED_MAXO];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j32 = lane & 31, h = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int64_t wb = a.batched ? batch : 0;
  const int O = a.O;
  const int nh = a.nh;
  const float w0 = a.w0;
  const float kph = PT::enck(w0);  // phase units per unit of (z + b)
  const int64_t rows = a.rows_per_batch;
  const int64_t ntiles = (rows + BM - 1) / BM;

  // ---- stage the small per-weight-set operands ----
  for (int i = tid; i < F * C; i += 512) {
    const int f = i / C, c = i - f * C;
    Sw0[c * F + f] = a.W0[wb * F * C + i];
  }
  for (int f = tid; f < F; f += 512) Sw0[C * F + f] = a.b0[wb * F + f] * kph;
  for (int l = 0; l < nh; ++l)
    for (int f = tid; f < F; f += 512) Sb[l * F + f] = a.bias[l][wb * F + f] * kph;
  for (int i = tid; i < O * F; i += 512) Swl[i] = a.WL[wb * O * F + i];
  if (tid < O) Swl[FUSED_MAXO * F + tid] = a.bL[wb * O + tid];

  auto h_off = [&](int r, int c) -> int { return r * (F * 2) + ((c ^ (r & SMASK)) << 4); };

  // ---- per-thread fixed chunk (feature group) of the VALU passes ----
  const int cth = tid & (CPR - 1);
  const int rth = tid >> LG_CPR;

  // ---- W fragments of the first hidden layer ----
  const bool mfma_wave = wave < NWAVE_F;
  const bf16x8* wf_base = (const bf16x8*)(a.Wfrag + wb * (int64_t)nh * F * F) + wave * (NKS * 64) + lane;
  auto wfrag = [&](int l, int ks) -> bf16x8 { return wf_base[(l * NWAVE_F * NKS + ks) * 64]; };
  bf16x8 wreg[NKS];
  if (nh > 0 && mfma_wave) {
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) wreg[ks] = wfrag(0, ks);
  }

  // ---- x prefetch (the thread's NQ rows; rows past the end read the last row) ----
  float xreg[NQ][C];
  auto load_x = [&](int64_t t) {
    const float* xb = a.x + (batch * rows) * C;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      int64_t row = t * BM + rth + RSTEP * q;
      row = row < rows ? row : rows - 1;
#pragma unroll
      for (int ci = 0; ci < C; ++ci) xreg[q][ci] = xb[row * C + ci];
    }
  };

  long long tprof[FUSED_NPROF] = {0, 0, 0, 0};
  long long tmark = 0;
  auto pmark = [&](int k) {
    if (a.prof) {
      const long long now = clock64();
      tprof[k] += now - tmark;
      tmark = now;
    }
  };

  int64_t t = blockIdx.x;
  if (t < ntiles) load_x(t);
  fused_barrier();  // staged operands visible
  if (a.prof) tmark = clock64();

  for (; t < ntiles; t += gridDim.x) {
    const int64_t m0 = t * BM;
    const int64_t tile_el = (batch * rows + m0) * F;  // element offset of the tile's first row
    const int nvalid = (int)(rows - m0 < BM ? rows - m0 : BM);
    // ================= layer 0 (VALU): phases -> P_0 and into H =================
    {
      const f32x4 b0a = *(const f32x4*)(Sw0 + C * F + 8 * cth);
      const f32x4 b0b = *(const f32x4*)(Sw0 + C * F + 8 * cth + 4);
      uint16_t* P0 = a.P[0] ? (uint16_t*)a.P[0] + tile_el : nullptr;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int r = rth + RSTEP * q;
        float z[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) z[e] = 0.f;
#pragma unroll
        for (int ci = 0; ci < C; ++ci) {
          const f32x4 wa = *(const f32x4*)(Sw0 + ci * F + 8 * cth);
          const f32x4 wc = *(const f32x4*)(Sw0 + ci * F + 8 * cth + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            z[e] = fmaf(xreg[q][ci], wa[e], z[e]);
            z[e + 4] = fmaf(xreg[q][ci], wc[e], z[e + 4]);
          }
        }
        u16x8 ph;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ph[e] = PT::enc_scaled(z[e], b0a[e], kph);
          ph[e + 4] = PT::enc_scaled(z[e + 4], b0b[e], kph);
        }
        if (P0 && r < nvalid) *(u16x8*)(P0 + r * F + 8 * cth) = ph;
        *(u16x8*)(H + h_off(r, cth)) = ph;
      }
    }
    // next tile's inputs (latency hidden behind the hidden layers)
    if (t + gridDim.x < ntiles) load_x(t + gridDim.x);
    fused_barrier();
    pmark(0);

    for (int l = 0; l <= nh; ++l) {
      if (l > 0) {
        // ================= hidden layer l-1 (MFMA) =================
        const int lh = l - 1;
        f32x16 acc[NBM];
#pragma unroll
        for (int bm = 0; bm < NBM; ++bm)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[bm][e] = 0.f;
        const int lnext = (lh + 1 < nh) ? lh + 1 : 0;
        if (mfma_wave) {
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks) {
#pragma unroll
            for (int bm = 0; bm < NBM; ++bm) {
              const bf16x8 hf = *(const bf16x8*)(H + h_off(32 * bm + j32, 2 * ks + h));
              acc[bm] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wreg[ks], hf, acc[bm], 0, 0, 0);
            }
            // refill the slot with the next layer's fragment (next tile's first after the last)
            wreg[ks] = wfrag(lnext, ks);
          }
        }
        fused_barrier();  // every wave is past its H reads
        pmark(1);
        // epilogue: P^T accumulators -> phases, in place over H (8-byte writes of 4 features)
        if (mfma_wave) {
          const float* bl = Sb + lh * F;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int f = 32 * wave + 8 * g + 4 * h;
            const f32x4 bv = *(const f32x4*)(bl + f);
#pragma unroll
            for (int bm = 0; bm < NBM; ++bm) {
              u16x4 ph;
#pragma unroll
              for (int e = 0; e < 4; ++e) ph[e] = PT::enc_scaled(acc[bm][4 * g + e], bv[e], kph);
              *(u16x4*)(H + h_off(32 * bm + j32, f >> 3) + 8 * h) = ph;
            }
          }
        }
        fused_barrier();
        pmark(2);
      }
      // ====== convert pass: H holds phases of sine layer l: store P_l (l > 0; P_0 is already
      // out), then sin -> bf16 in place (next layer's operand) or the output layer ======
      {
        uint16_t* Pl = (l > 0 && a.P[l]) ? (uint16_t*)a.P[l] + tile_el : nullptr;
        const bool last = (l == nh);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int r = rth + RSTEP * q;
          char* hp = H + h_off(r, cth);
          const u16x8 ph = *(const u16x8*)hp;
          if (Pl && r < nvalid) *(u16x8*)(Pl + r * F + 8 * cth) = ph;
          if (!last) {  // (for the last layer the phases stay in H for the output layer below)
            bf16x8 hv;
#pragma unroll
            for (int e = 0; e < 8; ++e) hv[e] = (bf16)PT::sinp(ph[e]);
            *(bf16x8*)hp = hv;
          }
        }
        if (last) {
          // y[row][o] = sum_f sin(P[row][f]) W_L[o][f] + b_L[o]. Row mapping: 4 threads per row,
          // each an fmaf chain over F/4 features; the quad is reduced with two DPP adds.
          constexpr int FQ = F / 4;
          const int r = tid >> 2, qq = tid & 3;
          float acc[FUSED_MAXO];
#pragma unroll
          for (int o = 0; o < FUSED_MAXO; ++o) acc[o] = 0.f;
#pragma unroll
          for (int ch = 0; ch < FQ / 8; ++ch) {
            const int c = qq * (FQ / 8) + ch;
            const u16x8 ph = *(const u16x8*)(H + h_off(r, c));
            float hv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) hv[e] = PT::sinp(ph[e]);
#pragma unroll
            for (int o = 0; o < FUSED_MAXO; ++o) {
              if (o < O) {
                const f32x4 wa = *(const f32x4*)(Swl + o * F + 8 * c);
                const f32x4 wc = *(const f32x4*)(Swl + o * F + 8 * c + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[o] = fmaf(hv[e], wa[e], acc[o]);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[o] = fmaf(hv[e + 4], wc[e], acc[o]);
              }
            }
          }
          float* yb = a.y + (batch * rows + m0 + r) * O;
#pragma unroll
          for (int o = 0; o < FUSED_MAXO; ++o) {
            if (o < O) {
              float v = acc[o];
              v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
              v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
              float z = v + Swl[FUSED_MAXO * F + o];
              if (a.sine_out) z = PT::sinr(w0 * z);
              if ((o & 3) == qq && r < nvalid) yb[o] = z;
            }
          }
        }
      }
      fused_barrier();
      pmark(3);
    }
  }
  if (a.prof && tid == 0) {
    long long* pb = a.prof + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * FUSED_NPROF;
#pragma unroll
    for (int k = 0; k < FUSED_NPROF; ++k) pb[k] = tprof[k];
  }
}

// Prepared-weight layout of the fused kernel: for weight set b, hidden layer l, feature block fb
// (32 outputs) and K step ks, the 64 lanes' 16-byte MFMA A-fragments are contiguous:
//   Wfrag[b][l][fb][ks][lane][j] = W_l[b][32 fb + (lane & 31)][16 ks + 8 (lane >> 5) + j]
struct FragPrepArgs {
  const float* W[FUSED_MAXH];  // hidden layer weights [nb_w][F, F] fp32
  bf16* Wt[FUSED_MAXH];        // optional: the backward's transposed bf16 copy [nb_w][F (in), F (out)]
  bf16* out;
  int64_t nb;
  int f16;  // fragments in fp16 (the pipe kernel's operands) instead of bf16
  int F, nh;
};

__global__ __launch_bounds__(256) void prep_frag_kernel(FragPrepArgs a) {
  const int F = a.F;
  const int64_t per_layer = (int64_t)F * F;
  const int64_t total = a.nb * a.nh * per_layer / 8;  // 16-byte fragments slices
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    // idx enumerates (b, l, fb, ks, lane) in row-major order
    int64_t rem = idx;
    const int lane = (int)(rem & 63);
    rem >>= 6;
    const int nks = F / 16, nfb = F / 32;
    const int ks = (int)(rem % nks);
    rem /= nks;
    const int fb = (int)(rem % nfb);
    rem /= nfb;
    const int l = (int)(rem % a.nh);
    const int64_t b = rem / a.nh;
    const float* src = a.W[l] + b * per_layer + (int64_t)(32 * fb + (lane & 31)) * F + 16 * ks + 8 * (lane >> 5);
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)src[j];
    if (a.f16) {
      h16x8 hv;
#pragma unroll
      for (int j = 0; j < 8; ++j) hv[j] = (_Float16)src[j];
      *(h16x8*)(a.out + idx * 8) = hv;
    } else {
      *(bf16x8*)(a.out + idx * 8) = v;
    }
    if (a.Wt[l]) {  // W^T[i][o] for the 8 inputs i of this slice, o = 32 fb + (lane & 31)
      bf16* dst = a.Wt[l] + b * per_layer + (int64_t)(16 * ks + 8 * (lane >> 5)) * F + 32 * fb + (lane & 31);
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[(int64_t)j * F] = v[j];
    }
  }
}

}  // namespace siren

namespace siren {

// ------------------------------------------------------------------------------------------
// fused_fwd_pipe: the same forward (hidden width 256, 1..14 hidden layers) with the MFMA work of
// one half-tile overlapped with the VALU work of the other. A 128-row tile is two 64-row halves
// A and B with their own LDS operand buffers; every segment pairs the K loop of one half with the
// epilogue/convert (EC) of the other, and segments are separated by one barrier:
//
//   K(1,A) + EC(nh,B of previous tile) + L0(B) | K(1,B) + EC(1,A) | K(2,A) + EC(1,B) | ...
//   ... | K(nh,B) + EC(nh,A) + L0(A of next tile) | (next tile) K(1,A') + EC(nh,B) + L0(B') ...
//
// (only the first tile's L0(A) runs without MFMA work beside it).
// EC is wave-local: a wave converts only the 32 features it computed (phases to LDS, read back as
// 16-byte chunks, stored to P_l, turned into bf16 sin in place), so K and EC of different halves
// need no barrier between them and the compiler can interleave MFMA and VALU issue. Stores go
// through buffer resources sized to the valid rows (ragged tiles drop out-of-range stores in
// hardware, no branches). The output layer accumulates per-wave partial dot products in LDS
// (ds_add_f32) and a small pass writes y after the next barrier. x comes in one tile ahead and
// is parked in LDS so no vector-memory wait ever covers the stores.
// ------------------------------------------------------------------------------------------

DEV __amdgpu_buffer_rsrc_t fused_rsrc(const void* base, int64_t bytes) { return make_rsrc(base, bytes); }

// SIREN_PIPE_NW waves (8: two per SIMD, 256 registers each; 4: one per SIMD, 512): wave w owns
// FB = 8 / NW blocks of 32 features, holds their W_l fragments and the accumulators of both
// halves, and issues a slice of the other half's VALU work after each K step's MFMAs.
#ifndef SIREN_PIPE_NW
#define SIREN_PIPE_NW 8
#endif
// OC: the output width when known at compile time (1: the image-fitting nets; 0: a.O at run time)
template <int C, int OC>
__global__ __launch_bounds__(64 * SIREN_PIPE_NW)
void fused_fwd_pipe_kernel(FusedFwdArgs a) {
  using PT = Prec<kPrecBF16>;
#ifdef SIREN_FWD_DEBUG
  const int dbg = a.dbg;  // timing experiments only: a runtime flag puts branches in the K loop
#else
  constexpr int dbg = 0;
#endif
  constexpr int F = 256, BM = 128, HB = 64, NKS = F / 16, SMASK = 15;
  constexpr int NW = SIREN_PIPE_NW, NT = 64 * NW, FB = 8 / NW;  // waves, threads, 32-feature blocks per wave
  // H rows padded to 528 bytes (no swizzle): every LDS address below is one per-lane base plus a
  // compile-time offset, and the MFMA B-fragment reads stay conflict-free (row stride = 4 banks)
  constexpr int RS = F * 2 + 16;
  constexpr int H_BYTES = HB * RS;
  constexpr int CPW = F / 8 / NW;          // 16-byte chunks per row owned by a wave (8)
  constexpr int NTASK = HB * CPW / 64;     // wave-local chunk tasks per lane (8)

  __shared__ __attribute__((aligned(16))) char Hs[2][H_BYTES];
  __shared__ __attribute__((aligned(16))) float Sw0[C * F + F];           // W0^T [C][F], k * b0
  __shared__ __attribute__((aligned(16))) float Sb[FUSED_MAXH * F];       // k * hidden biases
  __shared__ __attribute__((aligned(16))) float Swl[FUSED_MAXO * F + FUSED_MAXO];
  __shared__ __attribute__((aligned(16))) float Xs[2][BM * C];            // x tiles
  // output partial sums, one slot per wave (summed in wave order: deterministic)
  __shared__ __attribute__((aligned(16))) float Yp[2][NW][HB * FUSED_MAXO];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int j32 = lane & 31, hh = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int64_t wb = a.batched ? batch : 0;
  const int O = OC > 0 ? OC : a.O, nh = a.nh;
  const float w0 = a.w0;
  const float kph = PT::enck(w0);
  const int64_t rows = a.rows_per_batch;
  const int64_t ntiles = (rows + BM - 1) / BM;
  const int64_t G = gridDim.x;

  for (int i = tid; i < F * C; i += NT) {
    const int f = i / C, c = i - f * C;
    Sw0[c * F + f] = a.W0[wb * F * C + i];
  }
  for (int f = tid; f < F; f += NT) Sw0[C * F + f] = a.b0[wb * F + f] * kph;
  for (int l = 0; l < nh; ++l)
    for (int f = tid; f < F; f += NT) Sb[l * F + f] = a.bias[l][wb * F + f] * kph;
  for (int i = tid; i < O * F; i += NT) Swl[i] = a.WL[wb * O * F + i];
  if (tid < O) Swl[FUSED_MAXO * F + tid] = a.bL[wb * O + tid];
  for (int i = tid; i < 2 * NW * HB * FUSED_MAXO; i += NT) (&Yp[0][0][0])[i] = 0.f;

  // (an XOR-swizzled 512-byte-row layout without the chunk-task bank conflicts measured slower:
  // per-step address math and 19 spilled registers)
  auto h_off = [&](int r, int c) -> int { return r * RS + (c << 4); };

  // W fragments (fragment order, see prep_frag_kernel); wave w takes blocks FB w .. FB w + FB - 1.
  // Buffer loads: the per-lane offset is one VGPR, the layer / block / K-step offset a scalar.
  const __amdgpu_buffer_rsrc_t wrs =
      fused_rsrc(a.Wfrag + wb * (int64_t)nh * F * F, (int64_t)nh * F * F * 2);
  auto wfrag = [&](int l, int fb, int ks) -> h16x8 {
    const int soff = __builtin_amdgcn_readfirstlane((((l * 8 + FB * wave + fb) * NKS + ks) * 64) * 16);
    return __builtin_bit_cast(h16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, lane * 16, soff, 0));
  };
  h16x8 wreg[FB][NKS];
#pragma unroll
  for (int fb = 0; fb < FB; ++fb)
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) wreg[fb][ks] = wfrag(0, fb, ks);

  // x tile: BM*C floats, NX per thread (rows past the end: last row)
  constexpr int NX = (BM * C + NT - 1) / NT;
  float xr[NX];
  auto x_issue = [&](int64_t t) {
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      // an in-range index for every lane (lanes past the tile's BM * C values are never parked):
      // no select on the loaded value, so nothing waits for the load before x_park
      const int i = (tid + NT * k) < BM * C ? tid + NT * k : 0;
      int64_t r = t * BM + i / C;
      r = r < rows ? r : rows - 1;
      xr[k] = a.x[(batch * rows + r) * C + (i % C)];
    }
  };
  auto x_park = [&](int xb) {
#pragma unroll
    for (int k = 0; k < NX; ++k) {
      const int i = tid + NT * k;
      if (i < BM * C) Xs[xb][i] = xr[k];
    }
  };
  auto nvalid = [&](int64_t r0) -> int {
    const int64_t n = rows - r0;
    return (int)(n < 0 ? 0 : (n < HB ? n : HB));
  };

  // wave-local chunk tasks of a half: task i = lane + 64 k -> row i / CPW, chunk CPW w + i % CPW
  // L0 task k of half h: phases of layer 0 for this wave's features -> (P_0) -> bf16 sin into H[h]
  auto L0_task = [&](int64_t t, int h, int xb, int k) {
    const int64_t r0 = t * BM + HB * h;
    const int nval = nvalid(r0);
    const __amdgpu_buffer_rsrc_t rs =
        fused_rsrc(a.P[0] ? (const uint16_t*)a.P[0] + (batch * rows + r0) * F : nullptr,
                   a.P[0] ? (int64_t)nval * F * 2 : 0);
    const float* xs = Xs[xb] + HB * h * C;
    int tl = tid;
    asm volatile("" : "+v"(tl));  // per-lane offsets recomputed per task, not held (VGPR pressure)
    const int i = (tl & 63) + 64 * k;
    const int r = i / CPW, cc = CPW * (tl >> 6) + (i % CPW);
    const f32x4 ba = *(const f32x4*)(Sw0 + C * F + 8 * cc);
    const f32x4 bb = *(const f32x4*)(Sw0 + C * F + 8 * cc + 4);
    float z[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = 0.f;
#pragma unroll
    for (int ci = 0; ci < C; ++ci) {
      const float xv = xs[r * C + ci];
      const f32x4 wa = *(const f32x4*)(Sw0 + ci * F + 8 * cc);
      const f32x4 wc = *(const f32x4*)(Sw0 + ci * F + 8 * cc + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        z[e] = fmaf(xv, wa[e], z[e]);
        z[e + 4] = fmaf(xv, wc[e], z[e + 4]);
      }
    }
    u16x8 ph;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ph[e] = PT::enc_scaled(z[e], ba[e], kph);
      ph[e + 4] = PT::enc_scaled(z[e + 4], bb[e], kph);
    }
    store_b128_sync(__builtin_bit_cast(u32x4_t, ph), rs, (r * F + 8 * cc) * 2);
    h16x8 hv;
#pragma unroll
    for (int e = 0; e < 8; ++e) hv[e] = (_Float16)PT::sinp(ph[e]);
    *(h16x8*)(Hs[h] + h_off(r, cc)) = hv;
  };

  // EC of half h, hidden layer lh, in 16 slices: slices 0..7 write two accumulator groups each
  // (phases, 8-byte LDS writes of 4 features), slices 8..15 take one 16-byte chunk task each
  // (store to P_{lh+1}, then bf16 sin in place, or the output-layer partial sums if last)
  auto EC_slice = [&](int64_t t, int h, const f32x16 (&acc)[FB][2], int lh, auto last_tag, int sl) {
    constexpr bool last = decltype(last_tag)::value;
    constexpr int ESL = FB * 4;  // epilogue slices (2 of the FB * 8 accumulator groups each)
    if (sl < ESL) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int gi = 2 * sl + u;
        const int fb = gi >> 3, g = (gi >> 1) & 3, bm = gi & 1;
        int tl = tid;
        asm volatile("" : "+v"(tl));
        const int f = 32 * FB * (tl >> 6) + 32 * fb + 8 * g + 4 * ((tl >> 5) & 1);
        const f32x4 bv = *(const f32x4*)(Sb + lh * F + f);
        u16x4 ph;
#pragma unroll
        for (int e = 0; e < 4; ++e) ph[e] = PT::enc_scaled(acc[fb][bm][4 * g + e], bv[e], kph);
        *(u16x4*)(Hs[h] + h_off(32 * bm + j32, f >> 3) + 8 * hh) = ph;
      }
      return;
    }
    if (sl == ESL) asm volatile("" ::: "memory");  // this wave's phase writes precede its chunk reads
    const int k = sl - ESL;
    if (k >= NTASK) return;
    const int64_t r0 = t * BM + HB * h;
    const int nval = nvalid(r0);
    void* Pl = a.P[lh + 1];
    const __amdgpu_buffer_rsrc_t rs =
        fused_rsrc(Pl ? (const uint16_t*)Pl + (batch * rows + r0) * F : nullptr, Pl ? (int64_t)nval * F * 2 : 0);
    int tl = tid;
    asm volatile("" : "+v"(tl));  // per-lane offsets recomputed per task, not held (VGPR pressure)
    const int i = (tl & 63) + 64 * k;
    const int r = i / CPW, cc = CPW * (tl >> 6) + (i % CPW);
    char* hp = Hs[h] + h_off(r, cc);
    const u16x8 ph = *(const u16x8*)hp;
    store_b128_sync(__builtin_bit_cast(u32x4_t, ph), rs, (r * F + 8 * cc) * 2);
    if constexpr (!last) {
      h16x8 hv;
#pragma unroll
      for (int e = 0; e < 8; ++e) hv[e] = (_Float16)PT::sinp(ph[e]);
      *(h16x8*)hp = hv;
    } else {
      float hv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) hv[e] = PT::sinp(ph[e]);
      for (int o = 0; o < O; ++o) {
        const f32x4 wa = *(const f32x4*)(Swl + o * F + 8 * cc);
        const f32x4 wc = *(const f32x4*)(Swl + o * F + 8 * cc + 4);
        float sacc = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc = fmaf(hv[e], wa[e], sacc);
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc = fmaf(hv[e + 4], wc[e], sacc);
        // the CPW lanes of a row: DPP butterfly (quad swaps, then row_ror 4 when CPW = 8; the
        // row's first lane, the only writer, ends with the full sum)
        sacc += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, sacc), 0xB1, 0xF, 0xF, true));
        sacc += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, sacc), 0x4E, 0xF, 0xF, true));
        if constexpr (CPW == 8)
          sacc += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, sacc), 0x124, 0xF, 0xF, true));
        if ((i % CPW) == 0) Yp[h][wave][r * FUSED_MAXO + o] += sacc;
      }
    }
  };

  // K(h): acc[fb][bm] (features 64 w + 32 fb, rows 32 bm + j32 of half h) = W_l . H[h]^T, with a
  // VALU filler(ks) issued after each K step's MFMAs (EC or L0 of the other half); with refill,
  // each W slot is reloaded with layer `lref` right after its last use
  auto K = [&](int h, f32x16 (&acc)[FB][2], auto refill, int lref, auto&& filler) {
#pragma unroll
    for (int fb = 0; fb < FB; ++fb)
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[fb][bm][e] = 0.f;
    // H fragments one K step ahead: the reads of step ks + 1 are in flight under step ks's MFMAs
    auto hread = [&](h16x8 (&hf)[2], int ks) {
#pragma unroll
      for (int bm = 0; bm < 2; ++bm)
        hf[bm] = *(const h16x8*)(Hs[h] + h_off(32 * bm + j32, 2 * ((dbg & 8) ? 0 : ks) + hh));
    };
    h16x8 hbuf[2][2];
    hread(hbuf[0], 0);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks + 1 < NKS) hread(hbuf[(ks + 1) & 1], ks + 1);
      h16x8 (&hf)[2] = hbuf[ks & 1];
#pragma unroll
      for (int fb = 0; fb < FB; ++fb)
#pragma unroll
        for (int bm = 0; bm < 2; ++bm)
          acc[fb][bm] = __builtin_amdgcn_mfma_f32_32x32x16_f16(wreg[fb][ks], hf[bm], acc[fb][bm], 0, 0, 0);
      if constexpr (decltype(refill)::value) {
        if (!(dbg & 4))
#pragma unroll
        for (int fb = 0; fb < FB; ++fb) wreg[fb][ks] = wfrag(lref, fb, ks);
      }
      if (!(dbg & 1)) filler(ks);
    }
  };
  auto EC = [&](int64_t t, int h, const f32x16 (&acc)[FB][2], int lh, auto last_tag) {
#pragma unroll
    for (int sl = 0; sl < FB * 4 + NTASK; ++sl) EC_slice(t, h, acc, lh, last_tag, sl);
  };
  auto L0 = [&](int64_t t, int h, int xb) {
#pragma unroll
    for (int k = 0; k < NTASK; ++k) L0_task(t, h, xb, k);
  };

  // Y(h): y rows of half h of tile t from the partial sums; partials reset for reuse
  auto Ypass = [&](int64_t t, int h) {
    for (int idx = tid; idx < HB * O; idx += NT) {
      const int r = idx / O, o = idx - r * O;
      const int64_t row = t * BM + HB * h + r;
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        acc += Yp[h][w][r * FUSED_MAXO + o];
        Yp[h][w][r * FUSED_MAXO + o] = 0.f;
      }
      float z = acc + Swl[FUSED_MAXO * F + o];
      if (a.sine_out) z = PT::sinr(w0 * z);
      if (row < rows) a.y[(batch * rows + row) * O + o] = z;
    }
  };

  using T_ = std::true_type;
  using F_ = std::false_type;
  int64_t t = blockIdx.x;
  if (t >= ntiles) return;
  int xb = 0;  // x tile buffer of the current tile (alternates per iteration)
  x_issue(t);
  x_park(xb);
  fused_barrier();
  L0(t, 0, xb);  // prologue: layer 0 of half A of the first tile (later tiles: in the last segment)
  fused_barrier();

  // Every segment pairs a K loop with VALU filler. The first one also takes the output EC of the
  // previous tile's half B and the last one layer 0 of the next tile's half A (EC and L0 of one
  // half are wave-local, in program order, so they share the half's LDS buffer in one segment).
  // The first tile's "previous tile" is a dummy past the end: its stores and y rows drop out, so
  // no run-time condition splits the K loop's schedule.
  constexpr int ECS = FB * 4 + NTASK;  // EC slices
  static_assert(ECS + NTASK <= NKS, "EC + L0 tasks must fit one K loop");
  f32x16 accA[FB][2], accB[FB][2];
#pragma unroll
  for (int fb = 0; fb < FB; ++fb)
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int e = 0; e < 16; ++e) accB[fb][bm][e] = 0.f;
  int64_t tp = ntiles;
  for (; t < ntiles; t += G) {
    const bool more = t + G < ntiles;
    if (more) x_issue(t + G);
    Ypass(tp, 0);  // y rows of the previous tile's half A (its EC ended the previous iteration)
    // seg 1: K(1, A) + EC(nh, B) of the previous tile + L0(B); park x(t + G)
    K(0, accA, F_{}, 0, [&](int ks) {
      if (ks < ECS) EC_slice(tp, 1, accB, nh - 1, T_{}, ks);
      else if (ks - ECS < NTASK) L0_task(t, 1, xb, ks - ECS);
    });
    if (more) x_park(xb ^ 1);
    fused_barrier();
    Ypass(tp, 1);
    for (int l = 0; l < nh; ++l) {
      const int lnext = (l + 1 < nh) ? l + 1 : 0;
      if (l + 1 < nh) {
        // K(l, B) + EC(l, A); W slots refilled with the next layer
        K(1, accB, T_{}, lnext, [&](int ks) { EC_slice(t, 0, accA, l, F_{}, ks); });
        fused_barrier();
        // K(l + 1, A) + EC(l, B)
        K(0, accA, F_{}, 0, [&](int ks) { EC_slice(t, 1, accB, l, F_{}, ks); });
        fused_barrier();
      } else {
        // last layer: K(nh, B) + EC(nh, A) with the output layer + L0(A) of the next tile (past
        // the end on the last iteration: its stores drop out); slots refilled for the next tile
        K(1, accB, T_{}, lnext, [&](int ks) {
          if (ks < ECS) EC_slice(t, 0, accA, l, T_{}, ks);
          else if (ks - ECS < NTASK) L0_task(t + G, 0, xb ^ 1, ks - ECS);
        });
        fused_barrier();
      }
    }
    tp = t;
    xb ^= 1;
  }
  // drain: EC(nh, B) of the last tile and its y rows
  EC(tp, 1, accB, nh - 1, T_{});
  Ypass(tp, 0);
  fused_barrier();
  Ypass(tp, 1);
}

}  // namespace siren
