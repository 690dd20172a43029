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
#include "siren_common.h"

namespace siren {

constexpr int FUSED_BM = 128;
constexpr int FUSED_MAXC = 4;
constexpr int FUSED_MAXO = 8;
constexpr int FUSED_MAXH = 14;

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
  bf16* out;
  int64_t nb;
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
    *(bf16x8*)(a.out + idx * 8) = v;
  }
}

}  // namespace siren
