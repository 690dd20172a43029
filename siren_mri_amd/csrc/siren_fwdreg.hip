// siren_fwdreg.hip — the whole SIREN forward with the activations kept in registers
// (bf16 mode, hidden width 256, gfx950).
//
//   layer 0   P_0 = w0 (x W_0^T + b_0)                    modules.py:25-26,38 (f32 MFMA, exact fp32)
//   hidden l  P_l = w0 (sin(P_{l-1}) W_l^T + b_l)           modules.py:25-26,38 (f16 MFMA, fp32 acc)
//   output    y   = sin(P_{L-2}) W_L^T + b_L  (sin(w0 .))   modules.py:78      (f16 MFMA, fp32 acc)
//
// Design: every wave owns 32 coordinate rows and computes ALL 256 features of every layer for
// them, so a layer's output never leaves the wave. The MFMA runs transposed, P^T = W . H^T
// (A = weight fragment, B = activation fragment), and the weights are prepared so that the
// accumulator a lane holds IS the next layer's B fragment:
//   * output-feature order (freg_phi): lane (j, h) of a 32x32 accumulator holds features
//     32 fb + 8 h + 0..7 and 32 fb + 16 + 8 h + 0..7 of row j;
//   * input-feature order (freg_in0): K step s, lane half h supplies features
//     32 (s >> 1) + 16 (s & 1) + 8 h + 0..7 — exactly one converted half of one accumulator.
// So the epilogue is register-to-register: no LDS exchange, no barrier between layers. The
// weights (pre-multiplied by w0 / 2 pi, so an accumulator is a phase in revolutions; the bias is
// the accumulator's initial value) are streamed block by block (32 output features x 256 inputs =
// 16 KB of f16 fragments) through an 8-slot LDS ring that every wave of the workgroup reads; one
// barrier per block keeps the ring in step, and each slot is refilled by LDS-DMA seven blocks
// before it is read again.
//
// Epilogue per element: fr = fract(acc) (v_fract_f32), h = sin(fr) (v_sin_f32 takes revolutions),
// f16 pack (v_cvt_pk_f16_f32), phase code for the backward = unorm16(fr) (v_cvt_pknorm_u16_f32,
// two per instruction). The code is round(fr * 65535); the backward decodes it as code / 65536
// revolutions (siren_common.h Prec<kPrecBF16>::rev128), a difference of at most one code step
// (9.6e-5 rad), well inside the bf16 backward's own rounding.
//
// The epilogue of block fb runs beside the MFMAs of block fb + 1 (the last block's beside the
// next layer's first: its two fragments are the last two K steps there), so VALU and MFMA issue
// overlap inside every wave, and two waves per SIMD fill each other's gaps.
#include <type_traits>

#include "siren_common.h"

namespace siren {

constexpr int FREG_WROWS = 32;      // rows per wave tile
constexpr int FREG_WG_ROWS = 256;   // rows per workgroup round (8 waves)
constexpr int FREG_SLOT = 16384;    // bytes of one block: 16 K steps x 64 lanes x 16 B
constexpr int FREG_WL_BYTES = 4096; // output-layer fragments, rows 0..7 only: [16 ks][2 h][8 rows][16 B]
// Wide first layer (5..16 inputs, C template 16: the Fourier-feature inputs of configs 4/5): layer 0
// is one f16 MFMA K step split into hi + lo halves (W hi x x hi + W hi x x lo + W lo x x hi, each
// product exact to ~2^-22), its fragments staged in LDS; the LDS that the x tiles and the bias
// table of the narrow form use pays for them, so at most FREG_WIDE_MAXH hidden layers.
constexpr int FREG_WIDE_MAXH = 6;
constexpr int FREG_W0F_BYTES = 16384;  // [8 fb][hi, lo][64 lanes][16 B]
// Blocks per ring synchronisation (one barrier every FREG_SYNC blocks, 1 or 2).
#ifndef SIREN_FREG_SYNC
#define SIREN_FREG_SYNC 2
#endif
constexpr int FREG_SYNC = SIREN_FREG_SYNC;
// 1: one vmcnt(0) per block for both phase-code stores (the first store's data held until then)
// SIREN_FREG_DEFER 1 (magic form, off): each code store waits vmcnt(1) — for the store before it —
// instead of its own completion, the older data held in a variable until then. Off: the compiler
// copied that data to other registers and reused the store's own at once (check_store_hazard.py:
// 32 stores), so a held value does not pin the registers a store reads.
#ifndef SIREN_FREG_DEFER
#define SIREN_FREG_DEFER 0
#endif
#ifndef SIREN_FREG_STORE_PAIR
#define SIREN_FREG_STORE_PAIR 1
#endif
// cache-policy bits of the phase-code stores (timing experiments: 2 = nt)
#ifndef SIREN_FREG_STORE_AUX
#define SIREN_FREG_STORE_AUX 0
#endif
static_assert(FREG_SYNC == 1 || FREG_SYNC == 2, "ring sync interval");
// 1: hidden-layer accumulators start at bias + FREG_MAGIC revolutions (see epi_part)
#ifndef SIREN_FREG_MAGIC
#define SIREN_FREG_MAGIC 1
#endif
#ifndef SIREN_FREG_FORCE  // timing only: 1 fract form, 2 magic form, regardless of the weights
#define SIREN_FREG_FORCE 0
#endif
constexpr float FREG_MAGIC = 192.0f;  // 1.5 x 2^7: [128, 256) has an fp32 ulp of exactly 2^-16
// The magic form holds while |fract(b) + z - b| < 63 revolutions for every feature: the hidden
// layers' inputs are sines, so k1 sum_k |W_fk| < FREG_MAGIC_BOUND (prep_reg_kernel's wbound) is enough.
constexpr float FREG_MAGIC_BOUND = 62.0f;
// Vector-memory operations a wave has issued after the ring refill it must see land (every block
// issues two phase stores — a null tensor's are still issued and dropped by their resource — and
// every refill of a slot two DMAs):
//   FREG_SYNC 1: the slot read by block k + 1 was refilled at the barrier of block k - 6: at least
//                1 + 2 x 5 (refills) + 2 x 6 (stores) = 23 are younger;
//   FREG_SYNC 2: the slot read by block k + 2 (its first three fragments are prefetched by block
//                k + 1, before the next barrier) was refilled (first of two slots) at the barrier of
//                block k - 4: after this wave's LAST DMA into it, at least 2 (the second slot) +
//                4 (refills at k - 2) + 2 x 4 (stores) = 14 are younger. (vmcnt(n) returns once at
//                most n are outstanding, in issue order; vmcnt(15) would leave the wave's second
//                piece of the slot — fragment 1 for wave 0 — unchecked.)
#ifdef SIREN_FREG_VMN  // timing experiments only: a looser wait (reads may see unlanded slots)
#define SIREN_FREG_STR2(x) #x
#define SIREN_FREG_STR(x) SIREN_FREG_STR2(x)
#define SIREN_FREG_VMWAIT "s_waitcnt vmcnt(" SIREN_FREG_STR(SIREN_FREG_VMN) ")"
#elif SIREN_FREG_SYNC == 1
#define SIREN_FREG_VMWAIT "s_waitcnt vmcnt(22)"
#else
#define SIREN_FREG_VMWAIT "s_waitcnt vmcnt(14)"
#endif

struct FwdRegArgs {
  const float* x;             // [rows, C] per weight set
  const float* W0;            // [nb_w][F, C]
  const float* b0;            // [nb_w][F]
  const _Float16* Wreg;       // [nb_w][nh][8 fb][16 ks][64 lanes][8] prepared hidden fragments
  const _Float16* WLreg;      // [nb_w][16 ks][2 h][8 rows][8] prepared output fragments
  const float* bias[FUSED_MAXH];
  const float* bL;            // [nb_w][O]
  const float* wbound;        // [nb_w][nh][F] k1 sum_k |W_l[f][k]| (prep_reg_kernel); null: fract form
  void* P0;                   // phase codes of sine layer 0 (null: not kept)
  char* Pb;                   // phase codes of sine layer 1 (null: none kept); layer l at Pb + (l - 1) pstride
  int64_t pstride;
  float* y;                   // [rows, O]
  int64_t rows_per_batch;
  int batched;
  int O, nh, sine_out;
  int cin;                    // inputs of layer 0 (= C, or 5..16 for the wide form C = 16)
  float w0;
  // wide form: Fourier-feature input (siren_mlp_desc.ff_B): x holds ffin raw coordinates per row and
  // layer 0's cin = 2m inputs are computed from them and ffB [ffin][m] (ff_feature)
  const float* ffB;
  int ffin;
  // LOSS instantiations: image_mse's (masked k-space) SSE of the output,
  // with the data consistency of DataConsistencyInKspace applied first, in the output layer's
  // epilogue. Layouts as siren_kspace.hip: rows [B*N, O]; k0 / mask NCHW planes [B, O, N].
  const float* ltgt;          // [B*N, O] target
  const float* lk0;           // [B, O, N] k-space samples, or null (no data consistency)
  const float* lmask;         // [B, O, N] sampling mask
  const float* lhf;           // [N] high-frequency mask, or null
  float* ldc;                 // [B*N, O] DC(y) (model_out of the DC module), or null
  float* ldy;                 // [B*N, O] dL/dy for a unit upstream gradient
  float* lloss;               // [1] the loss
  float* lpart;               // [grid] per-workgroup partial sums
  unsigned* lcounter;         // zero between launches (the last workgroup resets it)
  float lnoise, lweight;
#ifdef SIREN_FREG_CLOCK
  long long* clk;             // diagnostic builds only: [grid][4] s_memtime / s_memrealtime stamps
#endif
};

// Every prefetched fragment read has landed (lgkmcnt(0)). The compiler takes an inline-asm read's
// output as defined at the asm, so register allocation may copy it (v_mov at a control-flow edge:
// a loop back-edge, a branch) before its counted wait — a copy of bytes not yet landed, seen in
// round 3 as one wave's block differing in a few runs out of 100. So no fragment read is in flight
// at a control-flow edge: a drain at the end of every layer and before the round loop
// (tools/check_lds_hazard.py checks every path of the code object).
DEV void freg_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

DEV void freg_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Feature offset (within a 32-feature block) of MFMA output row i = 8 g + 4 h + e, which lane half
// h holds as accumulator element v = 4 g + e: features 8 h + v for v < 8 and 16 + 8 h + (v - 8)
// for v >= 8, so the two lane halves of a row hold adjacent 16-byte phase chunks (one 32-byte
// piece of the row per store instruction) and K step 2 fb + q of the next layer takes features
// 32 fb + 16 q + 0..15 (lane half h: 32 fb + 16 q + 8 h + 0..7).
DEV constexpr int freg_phi(int i) {
  const int h = (i >> 2) & 1, v = 4 * (i >> 3) + (i & 3);
  return v + 8 * h + (v >= 8 ? 8 : 0);
}
DEV constexpr int freg_in0(int ks, int h) { return 32 * (ks >> 1) + 16 * (ks & 1) + 8 * h; }

// The 8 two-element parts of a pending epilogue are spread over K steps 0..13 (part p at step
// 13 p / 7): one part per one or two MFMAs, and both converted halves are ready before K steps
// 14 and 15, which read them when the pending block is the previous layer's last.
// SIREN_FREG_SPAN: the last part's K step (parts at SPAN p / 7); SIREN_FREG_WAITAT >= 0: the block's
// store-completion wait at that K step instead of right after its second store (the two stores'
// data held until then), so the store's latency overlaps the MFMAs in between.
#ifndef SIREN_FREG_SPAN
#define SIREN_FREG_SPAN 9
#endif
// 1 (default): the phase-code and y stores are asm stores followed by s_nop 1 (siren_common.h
// store_b128_ws2: the measured 2 wait states), no store-completion waits; 0: the round-3 form
// (builtin stores, data held until an s_waitcnt vmcnt(0) at K step SIREN_FREG_WAITAT)
#ifndef SIREN_FREG_STORE_WS2
#define SIREN_FREG_STORE_WS2 1
#endif
#ifndef SIREN_FREG_WAITAT
#if SIREN_FREG_STORE_WS2
#define SIREN_FREG_WAITAT -1
#else
#define SIREN_FREG_WAITAT 15
#endif
#endif
static_assert(SIREN_FREG_SPAN >= 7 && SIREN_FREG_SPAN <= 13, "epilogue span");
static_assert(SIREN_FREG_WAITAT < 0 || (SIREN_FREG_WAITAT > SIREN_FREG_SPAN && SIREN_FREG_WAITAT < 16), "wait step");
DEV constexpr int freg_part_at(int ks) {
  for (int p = 0; p < 8; ++p)
    if (SIREN_FREG_SPAN * p / 7 == ks) return p;
  return -1;
}


// Fragment reads from the ring as inline asm: the compiler's wait-count pass cannot tell them
// apart from the LDS-DMA refills in flight and would drain the DMA (vmcnt(0)) before them. The
// caller owns the wait: freg_lgkm<N>(v) (N = fragment reads issued after v's) ties v to it.
template <int OFF>
DEV void freg_read(h16x8& d, uint32_t va) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(va), "n"(OFF));
}
template <int N>
DEV void freg_lgkm(h16x8& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

// Prepared weights of the register-resident forward (see the header comment):
//   hidden: Wreg[b][l][fb][ks][lane][m] = f16(W_l[b][32 fb + phi(lane & 31)][in0(ks, lane >> 5) + m] w0/2pi)
//   output: WLreg[b][ks][h][i][m] = f16(W_L[b][i][in0(ks, h) + m]) (0 for i >= O)
// and, optionally, the backward's bf16 W_l^T copies.
struct RegPrepArgs {
  const float* W[FUSED_MAXH];
  bf16* Wt[FUSED_MAXH];
  const float* WL;
  _Float16* out;
  _Float16* outL;
  float* wbound;  // [nb][nh][F] k1 sum_k |W_l[f][k]| (the forward's magic-form check), or null
  int64_t nb;
  int nh, O;
  float k1;
};

// FORM (SIREN_FREG_MAGIC): 1 = the magic epilogue (epi_part), 0 = the fract epilogue. Both forms are
// launched back to back; each reads the weight bounds and the one whose form does not apply exits
// at once (one kernel holding both forms needs more than 256 VGPRs). Without the bounds (null
// wbound) FORM 0 does the work.
// LOSS: the output layer's epilogue also computes the fused image loss (FwdRegArgs l* fields): per
// output element p = DC(y) (if k0), d = hf (p - t), the loss sum d^2 (per-lane, per-workgroup,
// then the last workgroup adds the workgroup sums in index order: deterministic), DC(y) and
// dL/dy = 2 w hf d dDC/dy (the backward's output-layer kernels scale it by the loss's upstream
// gradient, TopArgs::dy_scale). The arithmetic is ksse_fwd_kernel's / ksse_bwd_kernel's.
#ifdef SIREN_FWDREG_DECL_ONLY  // the kernels are compiled in siren_fwdreg_inst.hip
template <int C, int OC, int FORM, bool LOSS = false>
__global__ __launch_bounds__(512) void fused_fwd_reg_kernel(FwdRegArgs a);
__global__ __launch_bounds__(256) void prep_reg_kernel(RegPrepArgs a);
#else
template <int C, int OC, int FORM, bool LOSS = false>
__global__ __launch_bounds__(512) void fused_fwd_reg_kernel(FwdRegArgs a) {
  constexpr int F = 256, NKS = 16, NB = 8;
  constexpr bool WIDE = C > 4;
  constexpr int NKK = WIDE ? 1 : (C + 1) / 2;  // K pairs of the f32 layer-0 MFMA (narrow form)
  constexpr int MAXH_ = WIDE ? FREG_WIDE_MAXH : FUSED_MAXH;
  static_assert((C >= 1 && C <= 4) || C == 16 || C == 17,
                "1..4 inputs, or the wide form (C = 16: 5..16 inputs; C = 17: the same from the Fourier-feature input)");
  constexpr bool FFI = C == 17;  // wide form, layer 0's inputs formed from raw coordinates (ff_feature)
  // the ring's 8 slots as separate objects: the compiler's wait-count pass then knows that a read
  // of slot fb cannot alias the LDS-DMA just issued into slot fb - 1 (one array would put an
  // s_waitcnt vmcnt(0) in front of every fragment read after a refill)
  __shared__ __attribute__((aligned(16))) char ring0[FREG_SLOT], ring1[FREG_SLOT], ring2[FREG_SLOT], ring3[FREG_SLOT],
      ring4[FREG_SLOT], ring5[FREG_SLOT], ring6[FREG_SLOT], ring7[FREG_SLOT];
  auto slot = [&](int fb) -> char* {
    switch (fb) {
      case 0: return ring0;
      case 1: return ring1;
      case 2: return ring2;
      case 3: return ring3;
      case 4: return ring4;
      case 5: return ring5;
      case 6: return ring6;
      default: return ring7;
    }
  };
  __shared__ __attribute__((aligned(16))) char wlf[FREG_WL_BYTES + 16];   // + a zero fragment
  __shared__ __attribute__((aligned(16))) float sbias[(MAXH_ + 1) * F];  // layer 0, hidden 0..nh-1
  __shared__ __attribute__((aligned(16))) float xs[2][WIDE ? 4 : FREG_WG_ROWS * 4];
  __shared__ __attribute__((aligned(16))) char w0f[WIDE ? FREG_W0F_BYTES : 16];  // wide layer-0 fragments
  __shared__ __attribute__((aligned(16))) float sbl[8];
  __shared__ __attribute__((aligned(16))) float w0s[WIDE ? 4 : NB * NKK * 64];  // narrow layer-0 A operands
  __shared__ float sffB[FFI ? 32 : 1];  // C = 17: the Fourier-feature input's B [ffin][m]

#ifdef SIREN_FREG_DBG
  // timing builds only (compile-time, so the schedule of the rest is unchanged): 1: no hidden-
  // layer epilogue, 2: no barriers / ring refills, 4: no phase stores, 8: no layer-0 epilogue,
  // 16: no hidden-layer MFMAs, 256: half of the phase stores, 512: phase codes computed, not stored
  constexpr int dbg = SIREN_FREG_DBG;
#else
  constexpr int dbg = 0;
#endif
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar) index
  const int j = lane & 31, hh = lane >> 5;
  const int64_t batch = blockIdx.y;
  const int64_t wb = a.batched ? batch : 0;
  const int nh = a.nh;
  const int O = OC > 0 ? OC : a.O;
  const float w0 = a.w0;
  const float k1 = w0 * kInv2Pi;
  const int64_t rows = a.rows_per_batch;
  const int64_t ntiles = (rows + FREG_WG_ROWS - 1) / FREG_WG_ROWS;
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x;
  if (t0 >= ntiles) return;
#ifdef SIREN_FREG_CLOCK  // diagnostic builds only (MI355X_MICROARCH.md 'DVFS give-back' item 6)
  const long long clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
#endif

  using T_ = std::true_type;
  using F_ = std::false_type;
  const _Float16* wsrc = a.Wreg + wb * (int64_t)nh * F * F;

  // ---- the epilogue form (epi_part): magic unless a hidden row's weights could leave its range ----
  int unsafe = 1;
  if (SIREN_FREG_MAGIC && a.wbound) {
    unsafe = 0;
    for (int i = tid; i < nh * F; i += 512) unsafe |= !(a.wbound[wb * nh * F + i] < FREG_MAGIC_BOUND);
  }
  unsafe = __syncthreads_or(unsafe);
#if SIREN_FREG_FORCE == 0
  if (unsafe != (FORM == 0)) return;  // the other form's launch does the work
#endif

  // ---- stage the small per-weight-set operands ----
  for (int i = tid; i < F; i += 512) sbias[i] = a.b0[wb * F + i] * k1;
  for (int l = 0; l < nh; ++l)
    for (int i = tid; i < F; i += 512) {
      const float bk = a.bias[l][wb * F + i] * k1;
      // magic form: the bias reduced mod 1 revolution (sin and the phase code are periodic in it)
      sbias[(l + 1) * F + i] = unsafe ? bk : __builtin_amdgcn_fractf(bk) + FREG_MAGIC;
    }
  if (tid < 8) sbl[tid] = tid < O ? a.bL[wb * O + tid] : 0.f;
  constexpr bool ffin_on = FFI;
  if (FFI && tid < 32) sffB[tid] = tid < a.ffin * (a.cin / 2) ? a.ffB[tid] : 0.f;
  if (tid < FREG_WL_BYTES / 16)
    *(u32x4_t*)(wlf + 16 * tid) = *(const u32x4_t*)((const char*)(a.WLreg + wb * (FREG_WL_BYTES / 2)) + 16 * tid);
  if (tid == FREG_WL_BYTES / 16) *(u32x4_t*)(wlf + FREG_WL_BYTES) = u32x4_t{0u, 0u, 0u, 0u};

  // layer-0 weights as f32 MFMA A operands (lane (i, k): W_0[32 fb + phi(i)][2 kk + k] w0/2pi)
  const int cin = WIDE ? a.cin : C;
  // (staged in LDS, [fb][kk][lane], and read per layer-0 MFMA: as registers they were 8-16 VGPRs
  // held across the whole kernel, which spilled the C = 3, 4 forms)
  if constexpr (!WIDE) {
    for (int i = tid; i < NB * NKK * 64; i += 512) {
      const int fb = i / (NKK * 64), kk = (i >> 6) % NKK, ln = i & 63;
      const int col = 2 * kk + (ln >> 5);
      w0s[i] = col < C ? a.W0[(wb * F + 32 * fb + freg_phi(ln & 31)) * C + col] * k1 : 0.f;
    }
  } else {
    // wide: thread (fb, lane (i, kh)) stages the f16 hi and lo A fragments of block fb,
    // W_0[32 fb + phi(i)][8 kh + m] w0/2pi (zero past the inputs)
    const int fbs = tid >> 6, i = lane & 31, kh = lane >> 5;
    const float* wr = a.W0 + (wb * F + 32 * fbs + freg_phi(i)) * (int64_t)cin;
    h16x8 hi, lo;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int col = 8 * kh + m;
      const float v = col < cin ? wr[col] * k1 : 0.f;
      hi[m] = (_Float16)v;
      lo[m] = (_Float16)(v - (float)hi[m]);
    }
    *(h16x8*)(w0f + ((2 * fbs) * 64 + lane) * 16) = hi;
    *(h16x8*)(w0f + ((2 * fbs + 1) * 64 + lane) * 16) = lo;
  }

  // ---- LDS-DMA: ring blocks and x tiles ----
  // block (layer, fb) of hidden layer `layer` into ring slot fb (the slot of every layer's block fb)
  // (a buffer resource over the weight set's blocks: one per-lane offset VGPR, the block offset in
  // SOFFSET — a per-lane 64-bit source address was a register pair the wide form spilled)
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(wsrc, (int64_t)nh * NB * FREG_SLOT);
  const uint32_t wvoff = wave * 2048 + lane * 16;
  auto dma_block = [&](int layer, int fb) {
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)((layer * NB + fb) * FREG_SLOT));
    char* dst = slot(fb) + wave * 2048;
    // (the instruction's immediate offset would move the LDS destination too: SOFFSET carries it)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)dst, 16, wvoff, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lds_void*)(dst + 1024), 16, wvoff, soff + 1024, 0, 0);
  };
  // wide: the lane's 8 inputs 8 hh .. 8 hh + 7 of its row of tile t, straight from global memory
  // into registers (rows past the end and inputs past cin read as 0); issued a layer ahead
  float xw[WIDE ? (FFI ? 4 : 8) : 1];  // (C = 17: the row's raw coordinates)
  auto load_xw = [&](int64_t t) {
    if constexpr (!WIDE) return;
    const int64_t r0 = t * FREG_WG_ROWS;
    const int64_t nv = rows - r0 < 0 ? 0 : (rows - r0 < FREG_WG_ROWS ? rows - r0 : FREG_WG_ROWS);
    if constexpr (ffin_on) {
      // the row's raw coordinates (the features are formed at layer 0 from these)
      // Exactly fin dword loads: a 16-byte load of the tile's last row (fin = 2) would reach 8
      // bytes past the resource, and a partly out-of-range multi-dword buffer load returns zeros
      // for all of it — that row's coordinates became (0, 0) (round 4's fused-input loss error).
      const int fin = a.ffin;
      const __amdgpu_buffer_rsrc_t rr = make_rsrc(a.x + (batch * rows + r0) * fin, nv * fin * 4);
      const uint32_t xo = (uint32_t)((wave * FREG_WROWS + j) * fin) * 4;
#pragma unroll
      for (int m = 0; m < 4; ++m)
        xw[m] = m < fin ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rr, xo, 4 * m, 0)) : 0.f;
      return;
    }
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x + (batch * rows + r0) * cin, nv * cin * 4);
    // from the lane's first input: two 16-byte loads when a row is exactly 16 inputs (64-byte rows,
    // no load crosses the resource's end), else eight dword loads — a 16-byte load that ends past
    // the resource reads as zeros entirely, which would drop the tile's last row's valid inputs.
    // Inputs past cin belong to the next row and are zeroed, rows past the end read as 0.
    const uint32_t xv = (uint32_t)((wave * FREG_WROWS + j) * cin + 8 * hh) * 4;
    if (cin == 16) {
      const u32x4_t v0 = __builtin_amdgcn_raw_buffer_load_b128(rx, xv, 0, 0);
      const u32x4_t v1 = __builtin_amdgcn_raw_buffer_load_b128(rx, xv, 16, 0);
#pragma unroll
      for (int m = 0; m < 8; ++m) xw[m] = __builtin_bit_cast(float, m < 4 ? v0[m] : v1[m - 4]);
    } else {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(rx, xv, 4 * m, 0);
        xw[m] = 8 * hh + m < cin ? __builtin_bit_cast(float, v) : 0.f;
      }
    }
  };
  // x rows of workgroup tile t (C KB; rows past the end arrive as zeros): waves 0..C-1, 1 KB each
  auto dma_x = [&](int64_t t, int xb) {
    if constexpr (WIDE) return;
    if (wave < C) {
      const int64_t r0 = t * FREG_WG_ROWS;
      const int64_t nv = rows - r0 < 0 ? 0 : (rows - r0 < FREG_WG_ROWS ? rows - r0 : FREG_WG_ROWS);
      const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.x + (batch * rows + r0) * C, nv * C * 4);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_void*)((char*)xs[xb] + wave * 1024), 16,
                                               wave * 1024 + lane * 16, 0, 0, 0);
    }
  };
#pragma unroll
  for (int fb = 0; fb < NB; ++fb) dma_block(0, fb);
  if constexpr (WIDE) load_xw(t0);
  else dma_x(t0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  freg_barrier();

  // ---- helpers ----
  auto bias_acc = [&](int layer, int fb) __attribute__((always_inline)) -> f32x16 {  // layer 0 = first layer, 1 + l = hidden l
    const float* bp = sbias + layer * F + 32 * fb + 8 * hh;
    f32x16 r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 v = *(const f32x4*)(bp + 4 * (q & 1) + 16 * (q >> 1));
#pragma unroll
      for (int e = 0; e < 4; ++e) r[4 * q + e] = v[e];
    }
    return r;
  };
  const int frag_lane = lane * 16;
  auto slot_va = [&](int fb) -> uint32_t { return lds_addr(slot(fb)) + frag_lane; };
  // output fragments: rows >= 8 read the zero fragment (offset by -ks * 256 so every K step's
  // immediate offset lands on it)
  const uint32_t wl_va = lds_addr(wlf) + (j < 8 ? hh * 128 + j * 16 : FREG_WL_BYTES);
#ifndef SIREN_FREG_PFD
#define SIREN_FREG_PFD 3
#endif
  constexpr int PFD = SIREN_FREG_PFD;  // fragment prefetch distance (K steps, <= 3: four buffers)

  // phase-code stores: sine layer pl, block pfb, of the wave's 32 rows of tile t (buffer resource
  // sized to the valid rows: stores past the end are dropped; null layer: everything dropped)
  int64_t tcur = t0;
  int64_t p_rowoff = 0;  // byte offset of the current tile's first row in a phase tensor
  int p_bytes = 0;       // valid bytes of the current tile in a phase tensor
  auto p_rsrc = [&](int pl) -> __amdgpu_buffer_rsrc_t {
    const char* base = pl == 0 ? (const char*)a.P0 : (a.Pb ? a.Pb + (int64_t)(pl - 1) * a.pstride : nullptr);
    const uint64_t addr = base ? (uint64_t)(base + p_rowoff) : 0;
    // every operand is wave-uniform; say so, or the compiler wraps each store in a waterfall loop
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)addr);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(addr >> 32));
    const int nb = __builtin_amdgcn_readfirstlane(base ? p_bytes : 0);
    return make_rsrc((const void*)(((uint64_t)hi << 32) | lo), nb);
  };
  const int p_voff = (wave * FREG_WROWS + j) * (F * 2) + hh * 16;
  // The block's two 16-byte code stores. A store's data VGPRs must not be rewritten before the
  // store has completed (siren_common.h, the store hazard): store_b128_sync waits vmcnt(0) after
  // it. (Holding the first store's data until the second store's wait — one wait per block —
  // needs 4 more VGPRs than this kernel has: 11-23 spilled.)
  u32x4_t prevst = {0u, 0u, 0u, 0u};  // SIREN_FREG_DEFER: the data of the last code store
  auto p_store = [&](int pl, int pfb, int half, const u32x4_t& c, const u32x4_t& held) __attribute__((always_inline)) {
    if constexpr ((dbg & 4) != 0) return;
    if constexpr ((dbg & 512) != 0) {  // timing only: the codes computed, not stored
      asm volatile("" ::"v"(c));
      return;
    }
    if constexpr ((dbg & 256) != 0) {  // timing only: half of the code stores (half 0 of every block)
      if (half == 1) {
        asm volatile("" ::"v"(c));
        return;
      }
    }
    if constexpr ((dbg & 1024) != 0) {
      // timing only: every store instruction writes whole 128-byte lines — store k = 2 (pfb & 1) +
      // half of a block pair covers rows 8 k .. 8 k + 7 of the wave, the pair's 128 bytes each
      const int k = 2 * (pfb & 1) + half;
      const uint32_t vo = (uint32_t)((wave * FREG_WROWS + 8 * k + (lane >> 3)) * (F * 2) + (lane & 7) * 16);
      store_b128_ws2(c, p_rsrc(pl), vo, (pfb >> 1) * 128);
      return;
    }
    if constexpr ((dbg & 32) != 0) {  // timing only: the same bytes as one contiguous 1 KB per store
      __builtin_amdgcn_raw_buffer_store_b128(c, p_rsrc(pl), wave * 16384 + lane * 16, (pfb * 2 + half) * 1024, 0);
      return;
    }
    // the block offset as the store's constant SOFFSET (one address VGPR for every store: folding
    // it into the VGPR offset costs a register per store and spilled)
#if SIREN_FREG_STORE_WS2
    store_b128_ws2(c, p_rsrc(pl), p_voff, pfb * 64 + half * 32);
    return;
#endif
    __builtin_amdgcn_raw_buffer_store_b128(c, p_rsrc(pl), p_voff, pfb * 64 + half * 32, 0);
#if SIREN_FREG_STORE_PAIR
    if constexpr (FORM == 1 && SIREN_FREG_DEFER && !WIDE) {  // (the wide form: 24 VGPRs short)
      // deferred: vmcnt(1) = every vector-memory operation but this store has completed, so the
      // previous store (its data held in prevst until this wait) has read its registers
      asm volatile("s_waitcnt vmcnt(1)" ::"v"(prevst));
      prevst = c;
    } else {
      // one wait per block: the half-0 store's data stays reserved (an input of the half-1 wait)
      if (half == 1 && SIREN_FREG_WAITAT < 0 && !SIREN_FREG_STORE_WS2) store_complete2(c, held);
    }
#else
    store_complete(c);
#endif
  };

  // Epilogue of one accumulator, in 8 parts of 2 elements (part p: elements 2p, 2p + 1, packed
  // at once into one f16 pair and one phase-code pair); after part 3 the first K fragment (and
  // 16-byte phase chunk) is complete, after part 7 the second.
  struct Epi {
    uint32_t hp[4];
    uint32_t cp[4];
    u32x4_t held;  // SIREN_FREG_STORE_PAIR: the half-0 store's data until the half-1 store's wait
    u32x4_t last;  // SIREN_FREG_WAITAT: the half-1 store's data until the block's wait
  };
  // Hidden layers (magic_tag true, SIREN_FREG_MAGIC): the accumulator started at bias + 192, so it
  // holds 192 + z with z the phase in revolutions; while |z| < 64 the sum lies in [128, 256), whose
  // fp32 ulp is exactly 2^-16 revolution, so its low 16 mantissa bits ARE the phase code
  // round(fract(z) 2^16) mod 2^16 (one v_perm_b32 packs two), and v_sin_f32 (revolutions, domain
  // +-256, exact reduction) takes the accumulator as it is: no v_fract_f32, no v_cvt_pknorm_u16 —
  // 24 instead of 32 issue cycles per element pair. The runtime checks |z| < 64 for every row of
  // every hidden layer from the weights (prep_reg_kernel; the inputs are sines, |h| <= 1) and
  // takes the fract form when it does not hold.
  auto epi_part = [&](Epi& ep, const f32x16& acc, int p, h16x8& t0h, h16x8& t1h, int pl, int pfb,
                      auto codes_tag, auto magic_tag) __attribute__((always_inline)) {
    constexpr bool codes = decltype(codes_tag)::value;  // false: the phases are not kept
    constexpr bool magic = decltype(magic_tag)::value;
    typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
    h16x2 hv;
    float f0, f1;
    if constexpr (magic && (dbg & 64) == 0) {
#ifdef SIREN_FREG_SINNOP  // diagnostic: extra wait states before the first reads of a finished MFMA chain
      if (p < 2) asm volatile("s_nop 7\n s_nop 7" ::: "memory");
#endif
      hv[0] = (_Float16)__builtin_amdgcn_sinf(acc[2 * p]);
      hv[1] = (_Float16)__builtin_amdgcn_sinf(acc[2 * p + 1]);
      uint32_t hpk = __builtin_bit_cast(uint32_t, hv);
      asm volatile("" : "+v"(hpk));
      ep.hp[p & 3] = hpk;
      if constexpr (codes) {
        // (elements copied to scalars first: hipcc 7.2's __builtin_bit_cast of an ext_vector element
        // reads element 0 whatever the index)
        const float a0 = acc[2 * p], a1 = acc[2 * p + 1];
        ep.cp[p & 3] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, a1), __builtin_bit_cast(uint32_t, a0),
                                             0x05040100u);  // low halves: a1 << 16 | a0
      }
    } else {
    if constexpr ((dbg & 64) != 0) {  // timing only: convert without fract / sin
      f0 = acc[2 * p];
      f1 = acc[2 * p + 1];
      hv[0] = (_Float16)f0;
      hv[1] = (_Float16)f1;
    } else {
      f0 = __builtin_amdgcn_fractf(acc[2 * p]);
      f1 = __builtin_amdgcn_fractf(acc[2 * p + 1]);
      hv[0] = (_Float16)__builtin_amdgcn_sinf(f0);
      hv[1] = (_Float16)__builtin_amdgcn_sinf(f1);
    }
    uint32_t hpk = __builtin_bit_cast(uint32_t, hv);
    // computed here, not sunk to the next layer's MFMA that reads it: the unpacked fp32 values
    // would otherwise stay live across the layer (twice the registers of the packed pair)
    asm volatile("" : "+v"(hpk));
    ep.hp[p & 3] = hpk;
    if constexpr (codes) ep.cp[p & 3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pknorm_u16(f0, f1));
    }
    if ((p & 3) == 3) {
      const u32x4_t hq = {ep.hp[0], ep.hp[1], ep.hp[2], ep.hp[3]};
      const u32x4_t c = codes ? u32x4_t{ep.cp[0], ep.cp[1], ep.cp[2], ep.cp[3]} : u32x4_t{0u, 0u, 0u, 0u};
      if (p == 3) t0h = __builtin_bit_cast(h16x8, hq);
      else t1h = __builtin_bit_cast(h16x8, hq);
      if constexpr (codes) {
        p_store(pl, pfb, p == 3 ? 0 : 1, c, ep.held);
        if (p == 3) ep.held = c;
        else ep.last = c;
      }
    }
  };

  auto out_init = [&]() -> f32x16 {  // output accumulator rows 0..7 = b_L (lanes' elements 0..3)
    f32x16 r;
#pragma unroll
    for (int e = 0; e < 16; ++e) r[e] = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = sbl[4 * hh + e];
    return r;
  };

  h16x8 Ha[NKS], Hb[NKS];
  h16x8 wq[4];    // rolling fragment prefetch (two steps ahead)
  f32x16 accP;    // the block whose epilogue is pending
  f32x16 accNx;   // the next block's initial accumulator (its bias), loaded into accP's registers
                  // once that block's epilogue is done
  int pend_pl = 0;
  int64_t kblk = 0;  // blocks consumed so far (ring position)
  const bool refill = nh > 1;

  // Ring synchronisation before block (l, fb), every FREG_SYNC blocks. FREG_SYNC 1: the slot of
  // the block after it has landed (this wave's part: vmcnt; every wave's: the barrier) and the
  // slot of the block before it is free: refill it with (l + 1 mod nh, fb - 1), or (l, 7) at
  // fb = 0. FREG_SYNC 2 (even fb): slots fb + 1 and fb + 2 have landed; slots fb - 2 and fb - 1
  // are free: refill them with layer l + 1 mod nh (at fb = 0: slots 6 and 7 with layer l).
  auto block_sync = [&](int l, int fb) __attribute__((always_inline)) {
    if constexpr ((dbg & 2) != 0) return;
    if (FREG_SYNC == 2 && (fb & 1)) {
      ++kblk;
      return;
    }
    asm volatile(SIREN_FREG_VMWAIT ::: "memory");
    freg_barrier();
    if (refill && kblk >= FREG_SYNC) {
      const int ln = l + 1 == nh ? 0 : l + 1;
      if (FREG_SYNC == 1) {
        if (fb > 0) dma_block(ln, fb - 1);
        else dma_block(l, NB - 1);
      } else {
        if (fb > 0) {
          dma_block(ln, fb - 2);
          dma_block(ln, fb - 1);
        } else {
          dma_block(l, NB - 2);
          dma_block(l, NB - 1);
        }
      }
    }
    ++kblk;
  };

  // one hidden layer l: Hin -> Hout (runtime l; register arrays bound at the call site;
  // last_tag: whether the output layer follows — its fragments are prefetched at the end)
  auto hidden_layer = [&](int l, h16x8 (&Hin)[NKS], h16x8 (&Hout)[NKS], auto last_tag, auto mtag) __attribute__((always_inline)) {
    constexpr bool last = decltype(last_tag)::value;
    // block fb (ptag: the form of the pending epilogue — at fb = 0 of hidden layer 0 it is layer 0's
    // last block, always in the fract form)
    auto blk = [&](auto fb_c, auto ptag) __attribute__((always_inline)) {
      constexpr int fb = decltype(fb_c)::value;
      block_sync(l, fb);
      if (fb == 0 && l == 0) dma_x(tcur + G, (int)(((tcur - t0) / G + 1) & 1));  // next round's x
      f32x16 accN = accNx;
      const uint32_t va_cur = slot_va(fb);
      const uint32_t va_nxt = (fb + 1 < NB) ? slot_va(fb + 1) : (last ? wl_va : slot_va(0));
      Epi ep;
      static_for<0, NKS>([&](auto ks_c) {
        constexpr int ks = decltype(ks_c)::value;
        constexpr int k3 = ks + PFD;
        if constexpr (k3 < NKS) freg_read<k3 * 1024>(wq[k3 & 3], va_cur);
        else if constexpr (fb + 1 < NB || !last) freg_read<(k3 - NKS) * 1024>(wq[k3 & 3], va_nxt);
        else freg_read<(k3 - NKS) * 256>(wq[k3 & 3], va_nxt);
        freg_lgkm<PFD>(wq[ks & 3]);
        if constexpr (!(dbg & 16)) accN = __builtin_amdgcn_mfma_f32_32x32x16_f16(wq[ks & 3], Hin[ks], accN, 0, 0, 0);
        constexpr int part = freg_part_at(ks);
        if constexpr (part >= 0 && !(dbg & 1)) {
          if constexpr (fb == 0) epi_part(ep, accP, part, Hin[14], Hin[15], pend_pl, 7, T_{}, ptag);
          else epi_part(ep, accP, part, Hout[2 * fb - 2], Hout[2 * fb - 1], l + 1, fb - 1, T_{}, ptag);
        }
        if constexpr (ks == SIREN_FREG_WAITAT && !(dbg & 1)) store_complete2(ep.last, ep.held);
        if constexpr (ks == NKS - 2) {  // the pending epilogue is done: the next block's bias
          if constexpr (fb + 1 < NB) accNx = bias_acc(l + 1, fb + 1);
          else if constexpr (!last) accNx = bias_acc(l + 2, 0);
          else accNx = out_init();
        }
      });
      accP = accN;
      pend_pl = l + 1;
    };
    static_for<0, NB>([&](auto fb_c) {
      if constexpr (decltype(fb_c)::value == 0 && decltype(mtag)::value) {
        // (a runtime branch: no fragment read may be in flight across it — freg_drain before, at
        // the end of the previous layer, and after, at the end of block 0)
        if (l == 0) blk(fb_c, F_{});
        else blk(fb_c, mtag);
        freg_drain();
      } else {
        blk(fb_c, mtag);
      }
    });
    freg_drain();  // the next layer's first fragments (prefetched) land before any control flow
  };

  float lsum = 0.f;  // LOSS: this lane's sum of d^2 over its rounds
  // output layer: y = H W_L^T + b_L (MFMA rows = outputs), beside the last hidden block's epilogue
  auto output_layer = [&](h16x8 (&Hin)[NKS], auto mtag) __attribute__((always_inline)) {
    if constexpr (WIDE) load_xw(tcur + G);  // the next round's inputs
    f32x16 accO = accNx;
    Epi ep;
    const uint32_t va_nxt = slot_va(0);  // the next round's first block
    static_for<0, NKS>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      constexpr int k3 = ks + PFD;
      if constexpr (k3 < NKS) freg_read<k3 * 256>(wq[k3 & 3], wl_va);
      else freg_read<(k3 - NKS) * 1024>(wq[k3 & 3], va_nxt);
      freg_lgkm<PFD>(wq[ks & 3]);
      accO = __builtin_amdgcn_mfma_f32_32x32x16_f16(wq[ks & 3], Hin[ks], accO, 0, 0, 0);
      constexpr int part = freg_part_at(ks);
      if constexpr (part >= 0) epi_part(ep, accP, part, Hin[14], Hin[15], pend_pl, 7, T_{}, mtag);
      if constexpr (ks == SIREN_FREG_WAITAT) store_complete2(ep.last, ep.held);
    });
    // y[row][o], o = 4 h + e (rows 0..7 of the output accumulator are lanes' elements 0..3)
    const int64_t r0 = tcur * FREG_WG_ROWS;
    const int64_t nv = rows - r0 < FREG_WG_ROWS ? rows - r0 : FREG_WG_ROWS;
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(a.y + (batch * rows + r0) * O, nv * O * 4);
    const int yrow = wave * FREG_WROWS + j;
    // one address VGPR for the lane's outputs 4 hh .. 4 hh + 3, the output index as the constant
    // SOFFSET (per-output address registers were spilled across the kernel)
    const uint32_t yv = (uint32_t)(yrow * O + 4 * hh) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (4 * hh + e < O) {
        float z = accO[e];
        if (a.sine_out) z = Prec<kPrecBF16>::sinr(w0 * z);
        const uint32_t zb = __builtin_bit_cast(uint32_t, z);
#if SIREN_FREG_STORE_WS2
        store_b32_ws2(zb, ry, yv, 4 * e);
#else
        __builtin_amdgcn_raw_buffer_store_b32(zb, ry, yv, 4 * e, 0);
        store_complete(zb);
#endif
        if constexpr (LOSS) {
          if (yrow < nv) {
            const int o = 4 * hh + e;
            const int64_t n = r0 + yrow;                    // the row within its weight set
            const int64_t q = (batch * rows + n) * O + o;   // [B*N, O] element
            float p = z;
            float coef = 1.f;
            if (a.lk0) {
              const int64_t pl = (batch * O + o) * rows + n;  // NCHW plane element
              const float m = a.lmask[pl];
              p = dc_value(z, a.lk0[pl], m, a.lnoise);
              coef = dc_coef(m, a.lnoise);
              a.ldc[q] = p;
            }
            const float h = a.lhf ? a.lhf[n] : 1.f;
            const float t = a.ltgt[q];
            const float dd = __fmul_rn(h, __fsub_rn(p, t));
            lsum = fmaf(dd, dd, lsum);
            float v = h * (dd * (2.f * a.lweight));
            if (a.lk0) v *= coef;
            a.ldy[q] = v;
          }
        }
      }
    }
    freg_drain();  // the next round's first fragments
  };

  // first fragments of the stream (later rounds: prefetched by the output layer)
  {
    const uint32_t va0 = slot_va(0);
    freg_read<0>(wq[0], va0);
    freg_read<1024>(wq[1], va0);
    freg_read<2048>(wq[2], va0);
    freg_drain();
  }

  auto run = [&](auto mtag) __attribute__((always_inline)) {
  for (int64_t t = t0; t < ntiles; t += G) {
    tcur = t;
    {
      const int64_t r0 = t * FREG_WG_ROWS;
      p_rowoff = (batch * rows + r0) * (F * 2);
      p_bytes = (int)((rows - r0 < FREG_WG_ROWS ? rows - r0 : FREG_WG_ROWS) * F * 2);
    }
    const int xb = (int)(((t - t0) / G) & 1);
    // This round's x tile was issued (LDS-DMA, waves 0..C-1) at the previous round's hidden
    // layer 0 block 0. With two or more hidden layers at least 28 vector-memory operations are
    // younger at the next layer's first ring sync, whose vmcnt(14) + barrier cover it. With one
    // hidden layer the ring is never refilled and only the phase stores follow it, so wait for
    // it here explicitly.
    if (!WIDE && nh == 1 && t != t0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      freg_barrier();
    }
    // ---- layer 0 (f32 MFMA, K = C): blocks 0..6 converted here, block 7 beside hidden block 0 ----
    auto layer0 = [&](auto codes_tag) __attribute__((always_inline)) {
      const float* xt = xs[xb] + (wave * FREG_WROWS + j) * C;
      float xr[NKK];
      h16x8 xh, xl;  // wide: the f16 hi / lo B fragments of the inputs
      if constexpr (!WIDE) {
#pragma unroll
        for (int kk = 0; kk < NKK; ++kk) xr[kk] = (2 * kk + hh) < C ? xt[2 * kk + hh] : 0.f;
      } else {
        if constexpr (ffin_on) {
          // Fourier features 8 hh .. 8 hh + 7 of the lane's row from its raw coordinates, one at a
          // time, each split into its f16 hi / lo parts at once (eight fp32 features in flight spilled)
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            const float f = ff_feature(xw, sffB, a.ffin, cin / 2, 8 * hh + m);
            xh[m] = (_Float16)f;
            xl[m] = (_Float16)(f - (float)xh[m]);
            asm volatile("" : "+v"(xh), "+v"(xl));
          }
        } else {
#pragma unroll
          for (int m = 0; m < 8; ++m) {
            xh[m] = (_Float16)xw[m];
            xl[m] = (_Float16)(xw[m] - (float)xh[m]);
          }
        }
      }
      // block fb + 1's MFMAs are issued before block fb's epilogue (its result latency and the
      // bias reads overlap the conversion)
      auto l0_mfma = [&](int fb) __attribute__((always_inline)) {
        f32x16 acc = bias_acc(0, fb);
        if constexpr (!WIDE) {
#pragma unroll
          for (int kk = 0; kk < NKK; ++kk)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w0s[(fb * NKK + kk) * 64 + lane], xr[kk], acc, 0, 0, 0);
        } else {
          const h16x8 ah = *(const h16x8*)(w0f + ((2 * fb) * 64 + lane) * 16);
          const h16x8 al = *(const h16x8*)(w0f + ((2 * fb + 1) * 64 + lane) * 16);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xh, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, xl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, xh, acc, 0, 0, 0);
        }
        return acc;
      };
      f32x16 acc = l0_mfma(0);
#pragma unroll
      for (int fb = 0; fb < NB; ++fb) {
        if (fb + 1 < NB) {
          const f32x16 accn = l0_mfma(fb + 1);
          Epi ep;
          if constexpr (!(dbg & 8))
#pragma unroll
            for (int p = 0; p < 8; ++p) epi_part(ep, acc, p, Ha[2 * fb], Ha[2 * fb + 1], 0, fb, codes_tag, F_{});
          if constexpr (SIREN_FREG_WAITAT >= 0 && decltype(codes_tag)::value) store_complete2(ep.last, ep.held);
          acc = accn;
        } else {
          accP = acc;
          pend_pl = 0;
        }
      }
      accNx = bias_acc(1, 0);  // hidden layer 0, block 0
    };
    if constexpr ((dbg & 128) != 0) {  // timing only: no layer 0
      accNx = bias_acc(1, 0);
    } else if (a.P0) {
      layer0(T_{});
    } else {
      layer0(F_{});
    }
    int l = 0;
    for (; l + 2 < nh; l += 2) {
      hidden_layer(l, Ha, Hb, F_{}, mtag);
      hidden_layer(l + 1, Hb, Ha, F_{}, mtag);
    }
    if (nh - l == 2) {
      hidden_layer(l, Ha, Hb, F_{}, mtag);
      hidden_layer(l + 1, Hb, Ha, T_{}, mtag);
      output_layer(Ha, mtag);
    } else {
      hidden_layer(l, Ha, Hb, T_{}, mtag);
      output_layer(Hb, mtag);
    }
  }
  };
#if SIREN_FREG_FORCE == 1
  run(F_{});
#elif SIREN_FREG_FORCE == 2
  run(T_{});
#else
  if constexpr (FORM == 1) run(T_{});
  else run(F_{});
#endif
  // no LDS-DMA may land after the workgroup has released its LDS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (LOSS) {
    // workgroup sum (waves in order), then the last workgroup to finish adds the workgroup sums in
    // index order (the hand-off of siren_loss.hip / siren_kspace.hip)
    __shared__ float lred[8];
    __shared__ unsigned lticket;
    const float ws_ = wave_sum(lsum);
    if (lane == 0) lred[wave] = ws_;
    __syncthreads();
    const unsigned nwg = gridDim.x * gridDim.y, wg = blockIdx.y * gridDim.x + blockIdx.x;
    if (tid == 0) {
      float sacc = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sacc += lred[w];
      __hip_atomic_store(a.lpart + wg, sacc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lticket = __hip_atomic_fetch_add(a.lcounter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (lticket == nwg - 1) {
      float sacc = 0.f;
      for (unsigned b = tid; b < nwg; b += 512) sacc += __hip_atomic_load(a.lpart + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sacc = wave_sum(sacc);
      __syncthreads();
      if (lane == 0) lred[wave] = sacc;
      __syncthreads();
      if (tid == 0) {
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) tot += lred[w];
        a.lloss[0] = tot * a.lweight;
        __hip_atomic_store(a.lcounter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
#ifdef SIREN_FREG_CLOCK
  if (tid == 0) {
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    long long* c = a.clk + 4 * (blockIdx.x + (int64_t)gridDim.x * blockIdx.y);
    c[0] = clk_t0;
    c[1] = t1;
    c[2] = clk_r0;
    c[3] = r1;
  }
#endif
}

__global__ __launch_bounds__(256) void prep_reg_kernel(RegPrepArgs a) {
  constexpr int F = 256;
  const int64_t nhid = a.nb * a.nh * (F * F / 8);
  const int64_t nout = a.nb * (FREG_WL_BYTES / 16);
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < nhid + nout; idx += (int64_t)gridDim.x * 256) {
    if (idx < nhid) {
      const int lane = (int)(idx & 63), ks = (int)((idx >> 6) & 15), fb = (int)((idx >> 10) & 7);
      const int64_t lb = idx >> 13;
      const int l = (int)(lb % a.nh);
      const int64_t b = lb / a.nh;
      const int orow = 32 * fb + freg_phi(lane & 31);
      const int in0 = freg_in0(ks, lane >> 5);
      const float* src = a.W[l] + b * F * F + (int64_t)orow * F + in0;
      h16x8 v;
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = (_Float16)(src[m] * a.k1);
      *(h16x8*)(a.out + idx * 8) = v;
      if (a.Wt[l]) {
        bf16* dst = a.Wt[l] + b * F * F + (int64_t)in0 * F + orow;
#pragma unroll
        for (int m = 0; m < 8; ++m) dst[(int64_t)m * F] = (bf16)src[m];
      }
    } else {
      const int64_t o = idx - nhid;
      const int i = (int)(o & 7), h = (int)((o >> 3) & 1), ks = (int)((o >> 4) & 15);
      const int64_t b = o >> 8;
      const int in0 = freg_in0(ks, h);
      h16x8 v;
#pragma unroll
      for (int m = 0; m < 8; ++m) v[m] = i < a.O ? (_Float16)a.WL[(b * a.O + i) * F + in0 + m] : (_Float16)0.f;
      *(h16x8*)(a.outL + o * 8) = v;
    }
  }
  if (a.wbound) {  // one wave per hidden-layer row: k1 sum_k |W_l[b][f][k]|
    const int64_t nrow = a.nb * a.nh * F;
    const int lane = threadIdx.x & 63;
    for (int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6; r < nrow; r += ((int64_t)gridDim.x * 256) >> 6) {
      const int64_t f = r % F, lb = r / F;
      const int l = (int)(lb % a.nh);
      const int64_t b = lb / a.nh;
      const f32x4 v = *(const f32x4*)(a.W[l] + (b * F + f) * F + 4 * lane);
      float s = fabsf(v[0]) + fabsf(v[1]) + fabsf(v[2]) + fabsf(v[3]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
      if (lane == 0) a.wbound[r] = s * a.k1;
    }
  }
}

#endif  // SIREN_FWDREG_DECL_ONLY

}  // namespace siren
