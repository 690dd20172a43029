// siren_runtime.hip — host-side orchestration of the SIREN layer stack behind the C ABI
// declared in include/siren_mri_amd.h. One call launches every kernel of a forward or a
// backward pass on the caller's stream; nothing here allocates, frees or synchronises.
#include <string>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <cstdarg>

#include "../../include/siren_mri_amd.h"
#include "siren_valu.hip"
#include "siren_gemm.hip"
#include "siren_jvp.hip"
#include "siren_fused.hip"
#define SIREN_FWDREG_DECL_ONLY  // its kernels: siren_fwdreg_inst.hip (a translation unit of its own)
#include "siren_fwdreg.hip"
#include "siren_adam.hip"
#include "siren_loss.hip"
#include "siren_kspace.hip"
#include "siren_encoder.hip"
#include "siren_conv.hip"
#include "siren_f64.hip"
#include "siren_hyper.hip"

using namespace siren;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

inline int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }
inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

constexpr int kTargetBlocks = 1024;  // ~4 workgroups per CU on 256 CUs

// Effective batching: shared weights collapse every row into one weight set.
struct Geo {
  int L;
  int64_t nb;     // weight sets
  int64_t rows;   // rows per weight set
  int64_t total;  // all rows
  int prec;
  int64_t phase_sz, grad_sz, op_sz;
};

Geo geo_of(const siren_mlp_desc* d) {
  Geo g;
  g.L = d->num_layers;
  if (d->weights_batched) {
    g.nb = d->batch;
    g.rows = d->rows_per_batch;
  } else {
    g.nb = 1;
    g.rows = d->batch * d->rows_per_batch;
  }
  g.total = d->batch * d->rows_per_batch;
  g.prec = d->prec;
  g.phase_sz = d->prec == SIREN_PREC_BF16 ? 2 : 4;
  g.grad_sz = g.phase_sz;
  g.op_sz = g.phase_sz;
  return g;
}

// Wide inputs (in_features > 16: Fourier-feature coordinates) run layer 0 on the MFMA GEMM path;
// its prepared weights are zero-padded along K to a whole number of MFMA K-steps (16 bf16 / 4 f32).
constexpr int kValuMaxIn = 16;
inline bool wide_input(const siren_mlp_desc* d) { return d->dims[0] > kValuMaxIn; }
inline int first_kp(const siren_mlp_desc* d) {
  return (int)align_up(d->dims[0], d->prec == SIREN_PREC_BF16 ? 16 : 4);
}
inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Shapes the single-kernel forward (siren_fused.hip) covers: bf16, 1..4 inputs, 1..8 outputs,
// every hidden width 256, up to FUSED_MAXH hidden MFMA layers.
bool g_fused_forward = true;
bool g_fused_backward = true;
bool g_fuse_top = false;   // output-layer fusion into the tiled kernels: slower than last_bwd, off
bool g_ring_top = true;    // output layer folded into the top 256x256 layer's ring kernels
bool g_bwd_ring = false;   // middle 256x256 layers in one ring kernel: measured slower (179 vs 145 us)
bool g_fwd_pipe = true;    // fused forward: half-tile MFMA/VALU pipelined kernel
bool g_fwd_reg = true;     // fused forward: activations resident in registers (siren_fwdreg.hip)
// its hidden layers in the magic epilogue form where the weights allow it: off by default — the
// forward ~3-5 % faster, but the bf16 PSNR at step 500 lands 0.085 dB under the reference (54.891
// vs 54.967 dB fract form; both forms track to 0.01 dB up to step 480, then the spiky regime)
bool g_freg_magic = false;
bool g_dx_ring = true;     // 256x256 input-gradient layers on the 4-stage ring kernel
bool g_dw_ring = true;     // 256x256 weight-gradient layers on the 4-stage ring kernel
bool g_pair_ring = true;   // both gradients of a ring layer in one launch (pair_ring_bf16_kernel)
int g_pair_roles = 3;      // debug timing: which pair_ring roles run (results are wrong unless 3)
bool g_dx_stagger = false;  // middle/top input-gradient ring: staggered wave halves (measured slower: +5-9 us/step)
bool g_tail_reduce = true;  // a pair launch reduces the previous pair launch's slabs (no reduce launch)
bool g_jvp_adj = true;
bool g_jvp_tan = true;      // tangent streams of a hidden layer stacked by row (jvp_tan_kernel)
bool g_f32_rows = true;     // fp32 hidden layers' forward / input gradient on the row-stacked tile
int g_wrw_dma = 2;          // the 5x5 weight-gradient convolution's chunks filled by LDS-DMA (conv_wrw_k5_kernel DMA;
                            // 2: 128-pixel chunks where W allows, C4 -0.33..-0.52 ms/step: profiles/r6_ab_wrw_128px.txt;
                            // C4 -0.05 ms/step, 5 of 6 one-box pairs: profiles/r6_ab_wrw_dma.txt)
int g_conv_dma = 2;         // the 5x5 encoder convolutions' stages: 0 register staging, 1 LDS-DMA, 2 LDS-DMA with
                            // per-workgroup source offsets (conv_fwd_k5_kernel DMA; 2 is C4 -2 %,
                            // profiles/r6_ab_conv_dma2.txt)
bool g_jvp_tn2 = true;      // fp32 analytic-derivative weight gradients on jvp_tn2_kernel      // analytic-derivative backward: adjoint GEMM + combine in one launch (jvp_adj_kernel)
// pair_ring role split, input-gradient workgroups per 32 of the grid, per pair kind (middle, top,
// bottom); 16 = the paired mapping (npair + npair, same tiles on one XCD)
long long* g_ring_prof = nullptr;   // debug: pair_ring segment cycle counters, one block per launch
int g_ring_prof_n = 0;
long long* g_fused_prof = nullptr;
int g_fwd_dbg = 0;  // debug timing: fused_fwd_pipe_kernel skip bits (results wrong unless 0)  // debug: per-workgroup phase cycle counters of the fused forward
// Wide first layer (5..16 inputs: Fourier features): the register-resident forward only, with at
// most FREG_WIDE_MAXH hidden layers; P_0 is kept (the layer-1 backward reads it).
bool fused_wide(const siren_mlp_desc* d) { return d->dims[0] > FUSED_MAXC && d->dims[0] <= 16; }
bool fused_shape(const siren_mlp_desc* d) {
  if (d->prec != SIREN_PREC_BF16) return false;
  if (d->dims[d->num_layers] > FUSED_MAXO) return false;
  if (fused_wide(d)) {
    if (!g_fwd_reg || d->num_layers - 2 < 1 || d->num_layers - 2 > FREG_WIDE_MAXH) return false;
  } else if (d->dims[0] > FUSED_MAXC) {
    return false;
  }
  const int F = d->dims[1];
  if (F != 256) return false;
  for (int l = 1; l < d->num_layers; ++l)
    if (d->dims[l] != F) return false;
  return d->num_layers - 2 <= FUSED_MAXH;
}

// bf16 stacks of the fused/ring shapes do not keep P_0: the layer-1 ring kernels recompute it from
// x (C <= 4 inputs) — 2 B per row-feature less written by the forward and read twice by the
// backward. Decided from the descriptor alone, so forward and backward always agree.
// Every row count qualifies: x moves by LDS-DMA through buffer resources whose bounds are checked
// per dword (a 16-byte piece straddling the end loads its valid dwords and zeros,
// tools/probe_lds_oob.hip) and whose base may sit 8 bytes past a 16-byte boundary (a weight set's x
// rows when rows_per_batch x C is not a multiple of 4; the forward reads x the same way). Keeping
// P_0 instead (the round-2 rule for such shapes) made the register-resident forward's layer-0
// phase-code stores differ from run to run in a few words (tools/det_saved.py), so the stored-P_0
// path is no longer taken by fused shapes.
bool g_keep_p0 = false;  // debug: fused shapes keep P_0 (the stored-P_0 path) instead of rebuilding it
bool p0_recompute(const siren_mlp_desc* d) {
  if (g_keep_p0 || !fused_shape(d) || fused_wide(d) || d->num_layers < 3) return false;
  const int64_t C = d->dims[0], total = d->batch * d->rows_per_batch;
  return total * C >= 1;
}

int max_hidden(const siren_mlp_desc* d) {
  int m = 0;
  for (int l = 1; l < d->num_layers; ++l) m = std::max(m, d->dims[l]);
  return m;
}

// Split-K geometry of the weight-gradient reductions.
struct Split {
  int64_t nsplit, rows_per_split;
};
Split split_rows(int64_t rows, int64_t blocks_per_split, int64_t nb, int64_t granule) {
  int64_t want = std::max<int64_t>(1, kTargetBlocks / std::max<int64_t>(1, blocks_per_split * nb));
  int64_t rps = align_up(cdiv(rows, want), granule);
  rps = std::max<int64_t>(rps, granule);
  Split s;
  s.rows_per_split = rps;
  s.nsplit = std::max<int64_t>(1, cdiv(rows, rps));
  return s;
}

Split tn_split(const Geo& g, int M, int N) {
  const int64_t tiles = cdiv(M, TN_BM) * cdiv(N, TN_BN);
  return split_rows(g.rows, tiles, g.nb, 64);
}
Split valu_split(const Geo& g) { return split_rows(g.rows, 1, g.nb, 64); }
// dw_ring_bf16_kernel: one workgroup per CU, each a contiguous row range of one weight set
Split dw_ring_split(const Geo& g) {
  const int64_t want = std::max<int64_t>(1, 256 / g.nb);
  Split s;
  s.rows_per_split = std::max<int64_t>(32, align_up(cdiv(g.rows, want), 32));
  s.nsplit = std::max<int64_t>(1, cdiv(g.rows, s.rows_per_split));
  return s;
}

// Distance between consecutive split slabs (all weight sets of one split), padded to float4.
int64_t split_stride(const Geo& g, int64_t slab) { return align_up(g.nb * slab, 4); }

// pair_ring_bf16_kernel: npair input-gradient / weight-gradient workgroup pairs per weight set
// (a multiple of 8, so the grid is a multiple of 16 and every pair shares an XCD); with nb <= 16
// weight sets all 2 * npair * nb workgroups are resident together (one per CU). Past that (configs
// 4/5: 32 slices, 512 workgroups) the two workgroups of a pair are still dispatched next to each
// other (speed only; correctness never depends on residency).
constexpr int64_t kMaxPairs = 128;
bool pair_ok(const Geo& g) { return g.nb <= 64; }
int64_t pair_count(const Geo& g) {
  const int64_t ntiles = cdiv(g.rows, 32);
  const int64_t np = std::max<int64_t>(8, (kMaxPairs / g.nb) / 8 * 8);
  return std::min<int64_t>(np, align_up(ntiles, 8));
}

Split jtn2_split(const Geo& g, int64_t stacked_rows, int N);
bool jvp_tn2_ok(int M, int N);

struct Layout {
  // saved
  int64_t saved_off[SIREN_MAX_LAYERS];
  int64_t saved_bytes;
  // workspace
  int64_t w_op_off[SIREN_MAX_LAYERS];
  int64_t wt_op_off[SIREN_MAX_LAYERS];
  int64_t pp_off[2];     // phase ping-pong (forward without saved buffer)
  int64_t dz_off[2];     // dZ ping-pong
  int64_t part_off;
  int64_t partL_off;      // output-layer partial slabs of the fused top backward layer
  int64_t partB_off;      // first-layer partial slabs of the paired bottom layer (P_0 recompute)
  int64_t part2_off;      // second slab buffer of consecutive pair launches (-1: none)
  int64_t xcopy_off;      // 16-byte aligned copy of x (P_0 recompute with a misaligned x)
  bool p0_rec;
  int64_t ws_bytes;
  int64_t weights_bytes;  // prepared MFMA weights (front of `saved`, or of the workspace)
  int64_t frag_off;       // fused-forward fragment-order hidden weights (-1: shape not eligible)
};

Layout layout_of(const siren_mlp_desc* d) {
  const Geo g = geo_of(d);
  Layout lo;
  memset(&lo, 0, sizeof(lo));
  // saved = [prepared MFMA weights][one phase tensor per sine layer 0..L-2]
  int64_t off = 0;
  for (int l = 0; l < SIREN_MAX_LAYERS; ++l) lo.w_op_off[l] = lo.wt_op_off[l] = -1;
  if (wide_input(d)) {
    lo.w_op_off[0] = off;
    off = align_up(off + g.nb * (int64_t)d->dims[1] * first_kp(d) * g.op_sz, 256);
    lo.wt_op_off[0] = off;
    off = align_up(off + g.nb * (int64_t)d->dims[1] * d->dims[0] * g.op_sz, 256);
  }
  for (int l = 1; l + 1 < g.L; ++l) {
    const int64_t n = g.nb * (int64_t)d->dims[l + 1] * d->dims[l];
    if (g.prec == SIREN_PREC_BF16) {
      lo.w_op_off[l] = off;
      off = align_up(off + n * g.op_sz, 256);
    } else {
      lo.w_op_off[l] = -1;
    }
    lo.wt_op_off[l] = off;
    off = align_up(off + n * g.op_sz, 256);
  }
  lo.frag_off = -1;
  if (fused_shape(d) && g.L > 2) {
    // hidden-layer fragments, then (register-resident forward) the output-layer fragments
    lo.frag_off = off;
    // + the rows' weight bounds of the forward's magic-form check ([nb][L - 2][F] f32)
    off = align_up(off + g.nb * ((int64_t)(g.L - 2) * d->dims[1] * d->dims[1] + FREG_WL_BYTES / 2) * 2 +
                       g.nb * (int64_t)(g.L - 2) * d->dims[1] * 4, 256);
  }
  lo.weights_bytes = off;
  lo.p0_rec = p0_recompute(d);
  for (int l = 0; l + 1 < g.L; ++l) {
    if (l == 0 && lo.p0_rec) {
      lo.saved_off[0] = -1;
      continue;
    }
    lo.saved_off[l] = off;
    off = align_up(off + g.total * d->dims[l + 1] * g.phase_sz, 256);
  }
  lo.saved_bytes = off;

  // workspace = [prepared weights when no saved buffer][phase ping-pong][dZ ping-pong][partials]
  off = align_up(lo.weights_bytes, 256);
  const int64_t act = g.total * (int64_t)max_hidden(d);
  for (int k = 0; k < 2; ++k) {
    lo.pp_off[k] = off;
    off = align_up(off + act * g.phase_sz, 256);
  }
  for (int k = 0; k < 2; ++k) {
    lo.dz_off[k] = off;
    off = align_up(off + act * g.grad_sz, 256);
  }
  int64_t part = 0;
  for (int l = 1; l + 1 < g.L; ++l) {
    const int M = d->dims[l + 1], N = d->dims[l];
    const Split s = tn_split(g, M, N);
    part = std::max(part, s.nsplit * split_stride(g, (int64_t)M * N + M));
    part = std::max(part, dw_ring_split(g).nsplit * split_stride(g, (int64_t)M * N + M));
    part = std::max(part, pair_count(g) * split_stride(g, (int64_t)M * N + M));
    part = std::max(part, jtn2_split(g, g.rows, N).nsplit * split_stride(g, (int64_t)M * N + M));
  }
  {
    const Split s = valu_split(g);
    const int F = d->dims[g.L - 1], O = d->dims[g.L];
    part = std::max(part, s.nsplit * split_stride(g, (int64_t)O * F + O));
    const int F0 = d->dims[1], C = d->dims[0];
    const Split s0 = wide_input(d) ? tn_split(g, F0, C) : s;
    part = std::max(part, s0.nsplit * split_stride(g, (int64_t)F0 * C + F0));
    // fused bottom layer: one first-layer slab per input-gradient workgroup (<= 256)
    part = std::max(part, (int64_t)256 * split_stride(g, (int64_t)F0 * C + F0));
  }
  lo.part_off = off;
  off = align_up(off + part * 4, 256);
  lo.partL_off = off;
  if (g.L >= 3) {
    const int F = d->dims[g.L - 1], O = d->dims[g.L];
    const int64_t ns = std::max(std::max(tn_split(g, F, d->dims[g.L - 2]).nsplit, dw_ring_split(g).nsplit),
                                pair_count(g));
    off = align_up(off + ns * split_stride(g, (int64_t)O * F + O) * 4, 256);
  }
  lo.partB_off = off;
  // (the bottom pair's input-gradient role: one first-layer slab per pair)
  if (lo.p0_rec) off = align_up(off + kMaxPairs * split_stride(g, (int64_t)d->dims[1] * d->dims[0] + d->dims[1]) * 4, 256);
  lo.xcopy_off = off;
  if (lo.p0_rec) off = align_up(off + g.total * d->dims[0] * 4, 256);
  // paired 256x256 layers alternate between part and part2: a pair launch reduces the previous
  // one's slabs in its weight-gradient role's tail (pair_ring_bf16_kernel)
  lo.part2_off = -1;
  if (fused_shape(d) && g.L >= 4) {
    lo.part2_off = off;
    off = align_up(off + pair_count(g) * split_stride(g, (int64_t)256 * 256 + 256) * 4, 256);
  }
  lo.ws_bytes = off;
  return lo;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(SIREN_ELAUNCH, "%s: %s", what, hipGetErrorString(e));
  return SIREN_OK;
}

// Optional per-kernel-class timing (bench / profiling only): while enabled, every launch of the
// selected class is bracketed by a hipEventRecord pair on its own stream.
struct Timing {
  int cls = 0;
  int cap = 0;
  int used = 0;
  hipEvent_t* ev = nullptr;
};
Timing g_timing;

inline void tmark_begin(int cls, hipStream_t st) {
  if (g_timing.cls == cls && g_timing.used < g_timing.cap)
    (void)hipEventRecord(g_timing.ev[2 * g_timing.used], st);
}
inline void tmark_end(int cls, hipStream_t st) {
  if (g_timing.cls == cls && g_timing.used < g_timing.cap) {
    (void)hipEventRecord(g_timing.ev[2 * g_timing.used + 1], st);
    ++g_timing.used;
  }
}

inline unsigned grid1d(int64_t work, int64_t cap = 4096) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(work, 256), cap));
}

int launch_reduce(const float* part, int64_t nsplit, int64_t sstride, int64_t nb, int64_t slab,
                  int64_t n_first, float* out0, float* out1, hipStream_t st) {
  const int64_t total = nb * slab;
  hipLaunchKernelGGL(reduce_kernel, dim3((unsigned)cdiv(total, 128)), dim3(256), 0, st, part,
                     (int)nsplit, sstride, (int)total, (int)slab, (int)n_first, out0, out1);
  return check_launch("reduce");
}

// Up to REDUCE_MAXSEG reductions (same arguments as launch_reduce) in one launch.
struct ReduceList {
  ReduceMultiArgs a;
  int64_t blocks = 0;
  ReduceList() { memset(&a, 0, sizeof(a)); }
  void add(const float* part, int64_t nsplit, int64_t sstride, int64_t nb, int64_t slab, int64_t n_first, float* out0,
           float* out1) {
    ReduceSeg& g = a.seg[a.nseg++];
    g.part = part;
    g.nsplit = (int)nsplit;
    g.split_stride = sstride;
    g.total = (int)(nb * slab);
    g.slab = (int)slab;
    g.n_first = (int)n_first;
    g.out0 = out0;
    g.out1 = out1;
    g.blocks = (int)cdiv(nb * slab, 128);
    blocks += g.blocks;
  }
  int launch(hipStream_t st) {
    if (a.nseg == 0) return SIREN_OK;
    hipLaunchKernelGGL(reduce_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
    return check_launch("reduce_multi");
  }
};

// Convert every MFMA layer's weights (bf16 copy + transpose) into `dst` in one launch.
template <int PREC>
int prep_weights(const siren_mlp_desc* d, const Geo& g, const Layout& lo, char* dst, hipStream_t st) {
  PrepArgs pa;
  memset(&pa, 0, sizeof(pa));
  int64_t maxn = 0;
  int k = 0;
  for (int l = wide_input(d) ? 0 : 1; l + 1 < g.L; ++l, ++k) {
    pa.W[k] = d->weight[l];
    pa.Wop[k] = lo.w_op_off[l] >= 0 ? dst + lo.w_op_off[l] : nullptr;
    pa.Wt[k] = dst + lo.wt_op_off[l];
    pa.O[k] = d->dims[l + 1];
    pa.I[k] = d->dims[l];
    pa.Kp[k] = l == 0 ? first_kp(d) : d->dims[l];
    maxn = std::max(maxn, (int64_t)pa.O[k] * pa.Kp[k]);
  }
  if (k == 0) return SIREN_OK;
  pa.nb = g.nb;
  hipLaunchKernelGGL(prep_weights_kernel<PREC>, dim3(grid1d(g.nb * maxn, 512), (unsigned)k),
                     dim3(256), 0, st, pa);
  return check_launch("prep_weights");
}

template <int PREC, int IT, int MAXO>
void launch_last_fwd(const LastFwdArgs& a, int64_t nb, hipStream_t st) {
  if (a.lloss) {  // fused image loss: at most SSE_MAX_BLOCKS workgroups (the hand-off's slots)
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(a.rows_per_batch, 8),
                                                                        std::max<int64_t>(1, SSE_MAX_BLOCKS / nb)));
    hipLaunchKernelGGL((last_fwd_kernel<PREC, IT, MAXO, true>), dim3(gx, (unsigned)nb), dim3(256), 0, st, a);
    return;
  }
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(a.rows_per_batch, 8),
                                                                      std::max<int64_t>(1, 4096 / nb)));
  hipLaunchKernelGGL((last_fwd_kernel<PREC, IT, MAXO>), dim3(gx, (unsigned)nb), dim3(256), 0, st, a);
}

template <int PREC>
int dispatch_last_fwd(const LastFwdArgs& a, int64_t nb, hipStream_t st) {
  const int it = (int)cdiv(a.F, 256);
  if (a.O <= 2) {
    if (it == 1) launch_last_fwd<PREC, 1, 2>(a, nb, st);
    else if (it == 2) launch_last_fwd<PREC, 2, 2>(a, nb, st);
    else launch_last_fwd<PREC, 4, 2>(a, nb, st);
  } else {
    if (it == 1) launch_last_fwd<PREC, 1, 8>(a, nb, st);
    else if (it == 2) launch_last_fwd<PREC, 2, 8>(a, nb, st);
    else launch_last_fwd<PREC, 4, 8>(a, nb, st);
  }
  return check_launch("last_fwd");
}

template <int PREC>
int dispatch_last_bwd(const LastBwdArgs& a, int64_t nsplit, int64_t nb, hipStream_t st) {
  const int it = (int)cdiv(a.F, 256);
  dim3 grid((unsigned)nsplit, (unsigned)nb);
  if (a.O <= 2) {
    if (it == 1) hipLaunchKernelGGL((last_bwd_kernel<PREC, 1, 2>), grid, dim3(256), 0, st, a);
    else if (it == 2) hipLaunchKernelGGL((last_bwd_kernel<PREC, 2, 2>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((last_bwd_kernel<PREC, 4, 2>), grid, dim3(256), 0, st, a);
  } else {
    if (it == 1) hipLaunchKernelGGL((last_bwd_kernel<PREC, 1, 8>), grid, dim3(256), 0, st, a);
    else if (it == 2) hipLaunchKernelGGL((last_bwd_kernel<PREC, 2, 8>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((last_bwd_kernel<PREC, 4, 8>), grid, dim3(256), 0, st, a);
  }
  return check_launch("last_bwd");
}

template <int PREC>
int dispatch_first_bwd(const FirstBwdArgs& a, int64_t nsplit, int64_t nb, hipStream_t st) {
  const int it = (int)cdiv(a.F, 256);
  dim3 grid((unsigned)nsplit, (unsigned)nb);
  if (a.ffB) {  // Fourier-feature input: the MFMA weight-gradient kernel forms the features itself
    if (!(PREC == kPrecBF16 && a.F == 256 && a.C > 4 && a.rows_per_split % 32 == 0 && !a.dx))
      return fail(SIREN_EINVAL, "fourier input: first-layer backward needs the bf16 wide MFMA path and no dx");
    hipLaunchKernelGGL(first_bwd_wide_mfma_kernel, grid, dim3(256), 0, st, a);
    return check_launch("first_bwd_wide_mfma (fourier input)");
  }
  if (a.C <= 4) {
    if (it == 1) hipLaunchKernelGGL((first_bwd_kernel<PREC, 1, 4>), grid, dim3(256), 0, st, a);
    else if (it == 2) hipLaunchKernelGGL((first_bwd_kernel<PREC, 2, 4>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((first_bwd_kernel<PREC, 4, 4>), grid, dim3(256), 0, st, a);
  } else if (a.F <= 256 && (!a.dx || (PREC == kPrecBF16 && a.F == 256))) {
    // weight gradient without dx; the input gradient (bf16 mode) as its own MFMA launch
    FirstBwdArgs aw = a;
    aw.dx = nullptr;
    if (PREC == kPrecBF16 && a.F == 256 && a.rows_per_split % 32 == 0)
      hipLaunchKernelGGL(first_bwd_wide_mfma_kernel, grid, dim3(256), 0, st, aw);
    else if (a.C == 16) hipLaunchKernelGGL((first_bwd_wide_kernel<PREC, 16>), grid, dim3(256), 0, st, aw);
    else hipLaunchKernelGGL((first_bwd_wide_kernel<PREC, 0>), grid, dim3(256), 0, st, aw);
    if (a.dx) {
      int rc = check_launch("first_bwd_wide");
      if (rc) return rc;
      const int64_t ntile = cdiv(a.rows_per_batch, 32);
      hipLaunchKernelGGL(first_dx_wide_kernel, dim3((unsigned)cdiv(ntile, 4), (unsigned)nb), dim3(256), 0, st, a);
    }
  } else {
    if (it == 1) hipLaunchKernelGGL((first_bwd_kernel<PREC, 1, 16>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((first_bwd_kernel<PREC, 2, 16>), grid, dim3(256), 0, st, a);
  }
  return check_launch("first_bwd");
}

// One hidden-layer GEMM launch (MODE_FWD or MODE_DX). Persistent grid: one 512-thread workgroup
// per CU (~131 KB LDS each), spread over weight sets and 256-column tiles.
dim3 nt_grid(const NTArgs& a, int64_t nb, int prec) {
  const int ntn = (int)cdiv(a.N, 256);
  const int kmax = a.K <= 256 ? 256 : 512;  // siren_mlp_check bounds K by 512 (bf16) / 256 (f32)
  const int bm = prec == kPrecBF16 ? 64 * 256 / kmax : 32;
  const int64_t tiles = cdiv(a.rows_per_batch, bm);
  const int64_t per = std::max<int64_t>(1, 256 / std::max<int64_t>(1, nb * ntn));
  return dim3((unsigned)std::min<int64_t>(tiles, per), (unsigned)nb, (unsigned)ntn);
}

dim3 ring_grid(const NTArgs& a, int64_t nb) {
  const int64_t tiles = cdiv(a.rows_per_batch, RING_BM);
  const int64_t per = std::max<int64_t>(1, 256 / nb);
  return dim3((unsigned)std::min<int64_t>(tiles, per), (unsigned)nb, 1);
}

// Bottom 256x256 input-gradient layer with the first layer folded in (dx_ring_bf16_kernel BOTC).
int launch_dx_ring_bot(const NTArgs& a, int64_t nb, int C, bool dxout, bool rec, int kclass, hipStream_t st) {
  const dim3 grid = ring_grid(a, nb);
  tmark_begin(kclass, st);
#define SIREN_RING_BOT(CC)                                                                              \
  if (rec) {                                                                                             \
    if (dxout) hipLaunchKernelGGL((dx_ring_bf16_kernel<CC, true, true>), grid, dim3(512), 0, st, a);     \
    else hipLaunchKernelGGL((dx_ring_bf16_kernel<CC, false, true>), grid, dim3(512), 0, st, a);          \
  } else {                                                                                               \
    if (dxout) hipLaunchKernelGGL((dx_ring_bf16_kernel<CC, true>), grid, dim3(512), 0, st, a);           \
    else hipLaunchKernelGGL((dx_ring_bf16_kernel<CC, false>), grid, dim3(512), 0, st, a);                \
  }
  switch (C) {
    case 1: SIREN_RING_BOT(1) break;
    case 2: SIREN_RING_BOT(2) break;
    case 3: SIREN_RING_BOT(3) break;
    default: SIREN_RING_BOT(4) break;
  }
#undef SIREN_RING_BOT
  tmark_end(kclass, st);
  return check_launch("dx_ring first-layer");
}

template <int PREC, int MODE, bool TOP = false, bool BOT = false>
int launch_nt(const NTArgs& a, int64_t nb, int kclass, hipStream_t st) {
  const int kmax = a.K <= 256 ? 256 : 512;
  if constexpr (PREC == kPrecF32 && (MODE == MODE_FWD || MODE == MODE_DX) && !TOP && !BOT) {
    // fp32 hidden layers on the row-stacked tile (jvp_tan_kernel JT_FWD / JT_DX: 128 rows x all
    // 256 output features per workgroup, 8 waves; nt_f32_kernel's products, K order and epilogues)
    if (g_f32_rows && a.K % JNT_KC == 0 && a.K <= 512 && a.N <= JADJ_BN && a.lda == a.K &&
        (MODE == MODE_FWD || a.Paux)) {
      JTanArgs t;
      memset(&t, 0, sizeof(t));
      t.P = MODE == MODE_FWD ? a.A : a.Paux;
      t.U = MODE == MODE_DX ? (const float*)a.A : nullptr;
      t.W = a.W;
      t.bias = a.bias;
      t.Uout = (float*)a.C;
      t.N = a.rows_per_batch;
      t.Su = 1;
      t.w_bstride = a.w_bstride;
      t.b_bstride = a.bias_bstride;
      t.K = a.K;
      t.Nout = a.N;
      t.w0 = a.w0;
      const dim3 grid((unsigned)cdiv(a.rows_per_batch, 2 * JADJ_ROWS), (unsigned)nb);
      tmark_begin(kclass, st);
      if constexpr (MODE == MODE_FWD) hipLaunchKernelGGL((jvp_tan_kernel<kPrecF32, 2, JT_FWD>), grid, dim3(512), 0, st, t);
      else hipLaunchKernelGGL((jvp_tan_kernel<kPrecF32, 2, JT_DX>), grid, dim3(512), 0, st, t);
      tmark_end(kclass, st);
      return check_launch(MODE == MODE_FWD ? "f32 rows fwd" : "f32 rows dx");
    }
  }
  if constexpr (PREC == kPrecBF16 && MODE == MODE_DX && !TOP && !BOT) {
    if (g_dx_ring && a.K == 256 && a.N == 256) {
      tmark_begin(SIREN_KCLASS_DX_RING, st);
      hipLaunchKernelGGL((dx_ring_bf16_kernel<0, false>), ring_grid(a, nb), dim3(512), 0, st, a);
      tmark_end(SIREN_KCLASS_DX_RING, st);
      return check_launch("dx_ring");
    }
  }
  const dim3 grid = nt_grid(a, nb, PREC);
  tmark_begin(kclass, st);
  if constexpr (PREC == kPrecBF16) {
    if (kmax == 256) hipLaunchKernelGGL((nt_bf16_kernel<MODE, 256, TOP, BOT>), grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((nt_bf16_kernel<MODE, 512, TOP, BOT>), grid, dim3(512), 0, st, a);
  } else {
    static_assert(PREC == kPrecBF16 || !(TOP || BOT), "backward fusions are bf16-mode paths");
    if (kmax == 256) hipLaunchKernelGGL((nt_f32_kernel<MODE>), grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((nt_f32_kernel<MODE, 512>), grid, dim3(512), 0, st, a);
  }
  tmark_end(kclass, st);
  static const char* const names[] = {"nt_gemm fwd", "nt_gemm dx", "nt_gemm first", "nt_gemm dx-input"};
  return check_launch(names[MODE]);
}

// Register-resident forward (siren_fwdreg.hip): one weight-prep launch, one forward launch.
int fused_forward_reg(const siren_mlp_desc* d, const Geo& g, const Layout& lo, const float* x, float* y,
                      char* saved, char* wbuf, hipStream_t st, const siren_loss_desc* L = nullptr) {
  const int F = d->dims[1], nh = g.L - 2;
  _Float16* wreg = (_Float16*)(wbuf + lo.frag_off);
  _Float16* wlreg = wreg + g.nb * (int64_t)nh * F * F;
  float* wbound = (float*)(wlreg + g.nb * (FREG_WL_BYTES / 2));
  {
    RegPrepArgs p;
    memset(&p, 0, sizeof(p));
    for (int l = 1; l + 1 < g.L; ++l) {
      p.W[l - 1] = d->weight[l];
      p.Wt[l - 1] = saved ? (bf16*)(saved + lo.wt_op_off[l]) : nullptr;  // the backward's W^T
    }
    p.WL = d->weight[g.L - 1];
    p.out = wreg;
    p.outL = wlreg;
    p.wbound = g_freg_magic ? wbound : nullptr;  // (the magic form's check only)
    p.nb = g.nb;
    p.nh = nh;
    p.O = d->dims[g.L];
    p.k1 = d->w0 * kInv2Pi;
    const int64_t work = g.nb * ((int64_t)nh * F * F / 8 + FREG_WL_BYTES / 16 + (int64_t)nh * F * 64);
    hipLaunchKernelGGL(prep_reg_kernel, dim3(grid1d(work, 1024)), dim3(256), 0, st, p);
    int rc = check_launch("prep_reg");
    if (rc) return rc;
  }
  FwdRegArgs a;
  memset(&a, 0, sizeof(a));
  a.x = x;
  a.W0 = d->weight[0];
  a.b0 = d->bias[0];
  a.Wreg = wreg;
  a.WLreg = wlreg;
  for (int l = 1; l + 1 < g.L; ++l) a.bias[l - 1] = d->bias[l];
  a.bL = d->bias[g.L - 1];
  a.wbound = wbound;
  a.P0 = (saved && lo.saved_off[0] >= 0) ? saved + lo.saved_off[0] : nullptr;
  a.Pb = saved ? saved + lo.saved_off[1] : nullptr;
  a.pstride = (saved && nh >= 2) ? lo.saved_off[2] - lo.saved_off[1] : 0;
  a.y = y;
  a.rows_per_batch = g.rows;
  a.batched = d->weights_batched ? 1 : 0;
  a.O = d->dims[g.L];
  a.nh = nh;
  a.sine_out = d->outermost_linear ? 0 : 1;
  a.cin = d->dims[0];
  a.w0 = d->w0;
  a.ffB = d->ff_B;
  a.ffin = d->ff_B ? d->ff_in : 0;
  if (L) {
    a.ltgt = L->target;
    a.lk0 = L->k0;
    a.lmask = L->mask;
    a.lhf = L->hf;
    a.ldc = L->y_dc;
    a.ldy = L->dy;
    a.lloss = L->loss;
    a.lpart = (float*)L->loss_workspace;
    a.lcounter = (unsigned*)((char*)L->loss_workspace + SSE_MAX_BLOCKS * 4);
    a.lnoise = L->noise;
    a.lweight = L->weight;
  }
  const int64_t tiles = cdiv(g.rows, FREG_WG_ROWS);
  const int64_t per = std::max<int64_t>(1, 256 / g.nb);
  dim3 grid((unsigned)std::min<int64_t>(tiles, per), (unsigned)g.nb);
  using KernelFn = void (*)(FwdRegArgs);
#define SIREN_FREG_FORMS(CC, OC) {fused_fwd_reg_kernel<CC, OC, 0>, fused_fwd_reg_kernel<CC, OC, 1>}
  static const KernelFn table[2][FUSED_MAXC][2] = {
      {SIREN_FREG_FORMS(1, 0), SIREN_FREG_FORMS(2, 0), SIREN_FREG_FORMS(3, 0), SIREN_FREG_FORMS(4, 0)},
      {SIREN_FREG_FORMS(1, 1), SIREN_FREG_FORMS(2, 1), SIREN_FREG_FORMS(3, 1), SIREN_FREG_FORMS(4, 1)}};
  static const KernelFn wide[2][2][2] = {{SIREN_FREG_FORMS(16, 0), SIREN_FREG_FORMS(16, 1)},
                                         {SIREN_FREG_FORMS(17, 0), SIREN_FREG_FORMS(17, 1)}};
#undef SIREN_FREG_FORMS
  const int ffi = d->ff_B ? 1 : 0;  // C = 17: the Fourier-feature input (siren_mlp_check: wide shapes only)
  const KernelFn* k = fused_wide(d) ? wide[ffi][a.O == 1 ? 1 : 0] : table[a.O == 1 ? 1 : 0][d->dims[0] - 1];
  if (L) {  // the fused-loss forms (siren_mlp_loss_check admitted this shape)
    static const KernelFn lnarrow[FUSED_MAXC] = {fused_fwd_reg_kernel<1, 1, 0, true>, fused_fwd_reg_kernel<2, 1, 0, true>,
                                                 fused_fwd_reg_kernel<3, 1, 0, true>, fused_fwd_reg_kernel<4, 1, 0, true>};
    static const KernelFn lwide[2][2] = {{fused_fwd_reg_kernel<16, 0, 0, true>, fused_fwd_reg_kernel<16, 1, 0, true>},
                                         {fused_fwd_reg_kernel<17, 0, 0, true>, fused_fwd_reg_kernel<17, 1, 0, true>}};
    const KernelFn kl = fused_wide(d) ? lwide[ffi][a.O == 1 ? 1 : 0] : lnarrow[d->dims[0] - 1];
    a.wbound = nullptr;  // the fract form alone (no magic-form exit test on an unwritten bound)
    tmark_begin(SIREN_KCLASS_FWD_FUSED, st);
    hipLaunchKernelGGL(kl, grid, dim3(512), 0, st, a);
    tmark_end(SIREN_KCLASS_FWD_FUSED, st);
    return check_launch("fused_fwd_reg (loss)");
  }
  tmark_begin(SIREN_KCLASS_FWD_FUSED, st);
  // magic form (option freg_magic): both forms are launched, the one whose form does not apply to
  // these weights exits at its start (siren_fwdreg.hip); otherwise the fract form alone
  if (g_freg_magic) hipLaunchKernelGGL(k[1], grid, dim3(512), 0, st, a);
  else a.wbound = nullptr;
  hipLaunchKernelGGL(k[0], grid, dim3(512), 0, st, a);
  tmark_end(SIREN_KCLASS_FWD_FUSED, st);
  return check_launch("fused_fwd_reg");
}

int fused_forward(const siren_mlp_desc* d, const Geo& g, const Layout& lo, const float* x, float* y,
                  char* saved, char* wbuf, hipStream_t st) {
  const int F = d->dims[1], nh = g.L - 2;
  if (g_fwd_reg && nh > 0) return fused_forward_reg(d, g, lo, x, y, saved, wbuf, st);
  if (nh > 0) {
    FragPrepArgs fp;
    memset(&fp, 0, sizeof(fp));
    for (int l = 1; l + 1 < g.L; ++l) {
      fp.W[l - 1] = d->weight[l];
      // the backward's W^T copies, written by the same launch (prep_weights is skipped)
      fp.Wt[l - 1] = saved ? (bf16*)(saved + lo.wt_op_off[l]) : nullptr;
    }
    fp.out = (bf16*)(wbuf + lo.frag_off);
    fp.nb = g.nb;
    fp.F = F;
    fp.nh = nh;
    fp.f16 = g_fwd_pipe ? 1 : 0;  // the pipe kernel multiplies in fp16 (sin values need no bf16 range)
    hipLaunchKernelGGL(prep_frag_kernel, dim3(grid1d(g.nb * nh * (int64_t)F * F / 8, 1024)), dim3(256), 0,
                       st, fp);
    int rc = check_launch("prep_frag");
    if (rc) return rc;
  }
  FusedFwdArgs a;
  memset(&a, 0, sizeof(a));
  a.x = x;
  a.W0 = d->weight[0];
  a.b0 = d->bias[0];
  a.Wfrag = nh > 0 ? (const bf16*)(wbuf + lo.frag_off) : nullptr;
  for (int l = 1; l + 1 < g.L; ++l) a.bias[l - 1] = d->bias[l];
  a.WL = d->weight[g.L - 1];
  a.bL = d->bias[g.L - 1];
  for (int l = 0; l + 1 < g.L; ++l) a.P[l] = (saved && lo.saved_off[l] >= 0) ? saved + lo.saved_off[l] : nullptr;
  a.y = y;
  a.prof = g_fused_prof;
  a.dbg = g_fwd_dbg;
  a.rows_per_batch = g.rows;
  a.batched = d->weights_batched ? 1 : 0;
  a.C = d->dims[0];
  a.F = F;
  a.O = d->dims[g.L];
  a.nh = nh;
  a.sine_out = d->outermost_linear ? 0 : 1;
  a.w0 = d->w0;
  const int64_t tiles = cdiv(g.rows, FUSED_BM);
  const int64_t per = std::max<int64_t>(1, 256 / g.nb);
  dim3 grid((unsigned)std::min<int64_t>(tiles, per), (unsigned)g.nb);
  tmark_begin(SIREN_KCLASS_FWD_FUSED, st);
  using KernelFn = void (*)(FusedFwdArgs);
  static const KernelFn table[FUSED_MAXC] = {fused_fwd_bf16_kernel<256, 1>, fused_fwd_bf16_kernel<256, 2>,
                                             fused_fwd_bf16_kernel<256, 3>, fused_fwd_bf16_kernel<256, 4>};
  static const KernelFn pipe[2][FUSED_MAXC] = {
      {fused_fwd_pipe_kernel<1, 0>, fused_fwd_pipe_kernel<2, 0>, fused_fwd_pipe_kernel<3, 0>, fused_fwd_pipe_kernel<4, 0>},
      {fused_fwd_pipe_kernel<1, 1>, fused_fwd_pipe_kernel<2, 1>, fused_fwd_pipe_kernel<3, 1>, fused_fwd_pipe_kernel<4, 1>}};
  const bool use_pipe = g_fwd_pipe && nh > 0;
  hipLaunchKernelGGL((use_pipe ? pipe[a.O == 1 ? 1 : 0] : table)[a.C - 1], grid,
                     dim3(use_pipe ? 64 * SIREN_PIPE_NW : 512), 0, st, a);
  tmark_end(SIREN_KCLASS_FWD_FUSED, st);
  return check_launch("fused_fwd");
}

// L: the fused image loss in the output layer's epilogue (siren_mlp_forward_loss on the per-layer
// path; the register forward has its own, fused_forward_reg)
template <int PREC>
int forward_impl(const siren_mlp_desc* d, const float* x, float* y, char* saved, char* ws,
                 hipStream_t st, const siren_loss_desc* L = nullptr) {
  const Geo g = geo_of(d);
  const Layout lo = layout_of(d);
  char* wbuf = saved ? saved : ws;  // prepared weights live in `saved` so backward reuses them
  const bool fused = PREC == kPrecBF16 && g_fused_forward && fused_shape(d);
  if (fused && !L) return fused_forward(d, g, lo, x, y, saved, wbuf, st);  // prepares its own weights
  int rc = prep_weights<PREC>(d, g, lo, wbuf, st);
  if (rc) return rc;
  auto phase_buf = [&](int l) -> char* {
    if (saved && lo.saved_off[l] >= 0) return saved + lo.saved_off[l];
    return ws + lo.pp_off[l & 1];  // (P_0 of a recompute stack: only layer 1 reads it)
  };
  // Layer 0: MFMA GEMM for wide inputs, VALU otherwise.
  if (wide_input(d)) {
    NTArgs a;
    a.A = x;
    a.W = wbuf + lo.w_op_off[0];
    a.bias = d->bias[0];
    a.Paux = nullptr;
    a.C = phase_buf(0);
    a.rows_per_batch = g.rows;
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[1] * first_kp(d) : 0;
    a.bias_bstride = d->weights_batched ? d->dims[1] : 0;
    a.K = first_kp(d);
    a.N = d->dims[1];
    a.lda = d->dims[0];
    a.a_vec = (d->dims[0] % 4 == 0) && aligned16(x);
    a.w0 = d->w0;
    if ((rc = launch_nt<PREC, MODE_FIRST>(a, g.nb, 0, st))) return rc;
  } else {
    FirstFwdArgs a;
    a.x = x;
    a.W = d->weight[0];
    a.b = d->bias[0];
    a.P = phase_buf(0);
    a.rows_per_batch = g.rows;
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[1] * d->dims[0] : 0;
    a.b_bstride = d->weights_batched ? d->dims[1] : 0;
    a.C = d->dims[0];
    a.F = d->dims[1];
    a.w0 = d->w0;
    const unsigned gx = grid1d(g.rows * (a.F / 8), std::max<int64_t>(1, 4096 / g.nb));
    if (a.C <= 4)
      hipLaunchKernelGGL((first_fwd_kernel<PREC, 4>), dim3(gx, (unsigned)g.nb), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((first_fwd_kernel<PREC, 16>), dim3(gx, (unsigned)g.nb), dim3(256), 0, st, a);
    if ((rc = check_launch("first_fwd"))) return rc;
  }
  // Hidden MFMA layers.
  for (int l = 1; l + 1 < g.L; ++l) {
    NTArgs a;
    a.A = phase_buf(l - 1);
    a.W = PREC == kPrecBF16 ? (const void*)(wbuf + lo.w_op_off[l]) : (const void*)d->weight[l];
    a.bias = d->bias[l];
    a.Paux = nullptr;
    a.C = phase_buf(l);
    a.rows_per_batch = g.rows;
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[l + 1] * d->dims[l] : 0;
    a.bias_bstride = d->weights_batched ? d->dims[l + 1] : 0;
    a.K = d->dims[l];
    a.N = d->dims[l + 1];
    a.lda = a.K;
    a.a_vec = 0;
    a.w0 = d->w0;
    if ((rc = launch_nt<PREC, MODE_FWD>(a, g.nb, SIREN_KCLASS_FWD_GEMM, st))) return rc;
  }
  // Output layer (VALU).
  {
    const int l = g.L - 1;
    LastFwdArgs a;
    a.P = phase_buf(l - 1);
    a.W = d->weight[l];
    a.b = d->bias[l];
    a.y = y;
    a.rows_per_batch = g.rows;
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[l + 1] * d->dims[l] : 0;
    a.b_bstride = d->weights_batched ? d->dims[l + 1] : 0;
    a.F = d->dims[l];
    a.O = d->dims[l + 1];
    a.sine_out = d->outermost_linear ? 0 : 1;
    a.w0 = d->w0;
    a.ltgt = a.lk0 = a.lmask = a.lhf = nullptr;
    a.ldc = a.ldy = a.lloss = a.lpart = nullptr;
    a.lcounter = nullptr;
    a.lnoise = a.lweight = 0.f;
    if (L) {
      a.ltgt = L->target;
      a.lk0 = L->k0;
      a.lmask = L->mask;
      a.lhf = L->hf;
      a.ldc = L->y_dc;
      a.ldy = L->dy;
      a.lloss = L->loss;
      a.lpart = (float*)L->loss_workspace;
      a.lcounter = (unsigned*)((char*)L->loss_workspace + SSE_MAX_BLOCKS * 4);
      a.lnoise = L->noise;
      a.lweight = L->weight;
    }
    if ((rc = dispatch_last_fwd<PREC>(a, g.nb, st))) return rc;
  }
  return SIREN_OK;
}

// One pair_ring_bf16_kernel launch for hidden layer l (kind: see backward_impl) and the
// reductions of its partial slabs.
template <int PREC>
int launch_pair(const siren_mlp_desc* d, const Geo& g, const Layout& lo, int kind, int l, const float* x,
                const TopArgs& ta, char* ws, const char* saved, float* part, float* const* dW, float* const* db,
                float* dx, int cur, ReduceList& pend, hipStream_t st) {
  const int M = d->dims[l + 1], N = d->dims[l], C = d->dims[0], F0 = d->dims[1], O = d->dims[g.L];
  const int64_t npair = pair_count(g);
  TNArgs w;
  memset(&w, 0, sizeof(w));
  w.D = ws + lo.dz_off[cur];
  w.P = kind == 3 ? (const void*)x : (const void*)(saved + lo.saved_off[l - 1]);
  w.part = part;
  w.rows_per_batch = g.rows;
  w.rows_per_split = 0;  // ranges come from the pair index
  w.split_stride = split_stride(g, (int64_t)M * N + M);
  w.M = M;
  w.N = N;
  w.w0 = d->w0;
  w.top = ta;
  w.pair_roles = g_pair_roles;
  w.prof = g_ring_prof ? g_ring_prof + (int64_t)(g_ring_prof_n++) * 256 * 8 * RING_NPROF : nullptr;
  NTArgs a;
  memset(&a, 0, sizeof(a));
  a.A = ws + lo.dz_off[cur];
  a.W = saved + lo.wt_op_off[l];
  a.Paux = kind == 3 ? nullptr : (const void*)(saved + lo.saved_off[l - 1]);
  a.C = ws + lo.dz_off[cur ^ 1];
  a.rows_per_batch = g.rows;
  a.w_bstride = d->weights_batched ? (int64_t)M * N : 0;
  a.K = M;
  a.N = N;
  a.lda = M;
  a.w0 = d->w0;
  a.top = ta;
  a.prof = w.prof;
  a.stagger = g_dx_stagger ? 1 : 0;
  const int64_t bot_stride = split_stride(g, (int64_t)F0 * C + F0);
  if (kind == 3) {
    w.rec_W0 = d->weight[0];
    w.rec_w0_bstride = d->weights_batched ? (int64_t)F0 * C : 0;
    w.rec_b0 = d->bias[0];
    w.rec_b0_bstride = d->weights_batched ? F0 : 0;
    a.C = dx;
    a.bot.x = x;
    a.bot.W0 = d->weight[0];
    a.bot.w0_bstride = w.rec_w0_bstride;
    a.bot.b0 = d->bias[0];
    a.bot.b0_bstride = w.rec_b0_bstride;
    a.bot.part = (float*)(ws + lo.partB_off);
    a.bot.split_stride = bot_stride;
    a.bot.C = C;
  }
  const int64_t nx = npair, nw = npair;  // input-gradient / weight-gradient workgroups (slabs)
  const dim3 grid((unsigned)(2 * npair), (unsigned)g.nb);
  const int kcls = kind == 1 ? SIREN_KCLASS_PAIR_RING : kind == 2 ? SIREN_KCLASS_PAIR_RING_TOP : SIREN_KCLASS_PAIR_RING_BOT;
  tmark_begin(kcls, st);
  const ReduceMultiArgs prev = pend.a;  // the previous pair launch's slabs, reduced in this one's tail
  if (kind == 1) {
    hipLaunchKernelGGL((pair_ring_bf16_kernel<0, false, false, 0, 0>), grid, dim3(512), 0, st, a, w, prev);
  } else if (kind == 2) {
    if (O == 1) hipLaunchKernelGGL((pair_ring_bf16_kernel<0, false, false, 1, 0>), grid, dim3(512), 0, st, a, w, prev);
    else hipLaunchKernelGGL((pair_ring_bf16_kernel<0, false, false, 2, 0>), grid, dim3(512), 0, st, a, w, prev);
  } else {
#define SIREN_PAIR_BOT(CC)                                                                                         \
  if (dx) hipLaunchKernelGGL((pair_ring_bf16_kernel<CC, true, true, 0, CC>), grid, dim3(512), 0, st, a, w, prev);   \
  else hipLaunchKernelGGL((pair_ring_bf16_kernel<CC, false, true, 0, CC>), grid, dim3(512), 0, st, a, w, prev);
    switch (C) {
      case 1: SIREN_PAIR_BOT(1) break;
      case 2: SIREN_PAIR_BOT(2) break;
      case 3: SIREN_PAIR_BOT(3) break;
      default: SIREN_PAIR_BOT(4) break;
    }
#undef SIREN_PAIR_BOT
  }
  tmark_end(kcls, st);
  int rc = check_launch("pair_ring");
  if (rc) return rc;
  // this launch's slabs: reduced by the next pair launch, or by a reduce_multi launch (flush)
  ReduceList red;
  red.add(part, nw, w.split_stride, g.nb, (int64_t)M * N + M, (int64_t)M * N, dW[l], db[l]);
  if (kind == 2) red.add(ta.partL, nw, ta.partL_stride, g.nb, (int64_t)O * M + O, (int64_t)O * M, dW[g.L - 1], db[g.L - 1]);
  if (kind == 3) red.add(a.bot.part, nx, bot_stride, g.nb, (int64_t)F0 * C + F0, (int64_t)F0 * C, dW[0], db[0]);
  pend = red;
  return SIREN_OK;
}

template <int PREC>
int backward_impl(const siren_mlp_desc* d, const float* x, const float* dy, const char* saved,
                  char* ws, float* const* dW, float* const* db, float* dx, hipStream_t st,
                  const float* dy_scale = nullptr) {
  const Geo g = geo_of(d);
  const Layout lo = layout_of(d);
  int rc = SIREN_OK;
  float* part = (float*)(ws + lo.part_off);
  auto P = [&](int l) -> const void* { return saved + lo.saved_off[l]; };
  const int O = d->dims[g.L], C = d->dims[0], F0 = d->dims[1];
  // slab reduction of the last pair launch, not yet issued (see launch_pair)
  ReduceList pend;
  int npair_launches = 0;
  auto flush = [&]() -> int {
    const int r = pend.launch(st);
    pend = ReduceList();
    return r;
  };
  // bf16-mode fusions (siren_gemm.hip TopArgs / BotArgs): the output layer's backward folds into
  // the top hidden layer's kernels, the first layer's weight gradient into the bottom one's.
  const bool fuse = PREC == kPrecBF16 && g_fused_backward && g.L >= 3;
  // P_0 not kept (p0_recompute): layer 1 runs on the ring kernels that rebuild it from x, whatever
  // the options say; they DMA x in 16-byte pieces, so a misaligned x is copied first.
  const bool rec = lo.p0_rec;
  if (rec && !aligned16(x)) {
    if (hipMemcpyAsync(ws + lo.xcopy_off, x, g.total * C * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess)
      return fail(SIREN_ELAUNCH, "x copy: %s", hipGetErrorString(hipGetLastError()));
    x = (const float*)(ws + lo.xcopy_off);
  }
  const bool top_ok = fuse && d->outermost_linear && O <= TOP_MAXO && (g.rows * O) % 4 == 0 && g.rows * O >= 4 &&
                      aligned16(dy) && !(rec && g.L == 3);
  // output layer folded into the top layer's ring kernels (256x256 top layer below another layer)
  const bool ring_top = top_ok && g_ring_top && g.L >= 4 && d->dims[g.L - 1] == 256 && d->dims[g.L - 2] == 256;
  const bool top = ring_top || (top_ok && g_fuse_top && d->dims[g.L - 1] <= 256);
  // first-layer fusion: the ring kernel (256x256 bottom layer) also produces dx; the older
  // kernel only without dx
  const bool ring_bot = rec || (fuse && g_dx_ring && !wide_input(d) && C <= BOT_MAXC && F0 == 256 &&
                                d->dims[2] == 256 && !(top && g.L == 3) && (g.rows * C) % 4 == 0 &&
                                g.rows * C >= 4 && aligned16(x));
  const bool bot = ring_bot || (fuse && !dx && !wide_input(d) && C <= BOT_MAXC && F0 <= 256 &&
                                (g.rows * C) % 4 == 0 && g.rows * C >= 4 && aligned16(x) &&
                                !(top && g.L == 3));  // one hidden layer: the output-layer fusion only
  int cur = 0;  // dz ping-pong index holding dZ of the current layer
  // Output layer: dZ_{L-2}, dW_{L-1}, db_{L-1}.
  if (!top) {
    const int l = g.L - 1;
    const Split s = valu_split(g);
    LastBwdArgs a;
    a.P = P(l - 1);
    a.W = d->weight[l];
    a.b = d->bias[l];
    a.dy = dy;
    a.dy_scale = dy_scale;
    a.dZ = ws + lo.dz_off[cur];
    a.part = part;
    a.rows_per_batch = g.rows;
    a.rows_per_split = s.rows_per_split;
    a.F = d->dims[l];
    a.O = d->dims[l + 1];
    a.split_stride = split_stride(g, (int64_t)a.O * a.F + a.O);
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[l + 1] * d->dims[l] : 0;
    a.b_bstride = d->weights_batched ? d->dims[l + 1] : 0;
    a.sine_out = d->outermost_linear ? 0 : 1;
    a.w0 = d->w0;
    if ((rc = dispatch_last_bwd<PREC>(a, s.nsplit, g.nb, st))) return rc;
    if ((rc = launch_reduce(part, s.nsplit, a.split_stride, g.nb, (int64_t)a.O * a.F + a.O,
                            (int64_t)a.O * a.F, dW[l], db[l], st)))
      return rc;
  }
  TopArgs ta;
  memset(&ta, 0, sizeof(ta));
  if (top) {
    const int FL = d->dims[g.L - 1];
    ta.Ptop = P(g.L - 2);
    ta.dy = dy;
    ta.dy_scale = dy_scale;
    ta.WL = d->weight[g.L - 1];
    ta.wl_bstride = d->weights_batched ? (int64_t)O * FL : 0;
    ta.partL = (float*)(ws + lo.partL_off);
    ta.partL_stride = split_stride(g, (int64_t)O * FL + O);
    ta.O = O;
  }
  // Hidden MFMA layers, top to bottom.
  for (int l = g.L - 2; l >= 1; --l) {
    const int M = d->dims[l + 1], N = d->dims[l];
    const bool is_top = top && l == g.L - 2;
    const bool is_bot = bot && l == 1;
    const bool rec1 = rec && l == 1;
    const bool ring_t = ring_top && l == g.L - 2;
    if (PREC == kPrecBF16 && g_bwd_ring && !is_top && !is_bot && !rec1 && M == 256 && N == 256) {
      // both gradients of a middle layer in one pass (bwd_ring_bf16_kernel)
      const Split s = dw_ring_split(g);
      BwdArgs b;
      memset(&b, 0, sizeof(b));
      b.dZ = (const bf16*)(ws + lo.dz_off[cur]);
      b.P = (const uint16_t*)P(l - 1);
      b.Wt = (const bf16*)(saved + lo.wt_op_off[l]);
      b.dZo = (bf16*)(ws + lo.dz_off[cur ^ 1]);
      b.part = part;
      b.rows_per_batch = g.rows;
      b.rows_per_split = s.rows_per_split;
      b.split_stride = split_stride(g, (int64_t)M * N + M);
      b.w_bstride = d->weights_batched ? (int64_t)M * N : 0;
      b.w0 = d->w0;
      if ((rc = flush())) return rc;
      tmark_begin(SIREN_KCLASS_BWD_FUSED, st);
      hipLaunchKernelGGL(bwd_ring_bf16_kernel, dim3((unsigned)s.nsplit, (unsigned)g.nb), dim3(256), 0, st, b);
      tmark_end(SIREN_KCLASS_BWD_FUSED, st);
      if ((rc = check_launch("bwd_ring"))) return rc;
      if ((rc = launch_reduce(part, s.nsplit, b.split_stride, g.nb, (int64_t)M * N + M, (int64_t)M * N, dW[l],
                              db[l], st)))
        return rc;
      cur ^= 1;
      continue;
    }
    if (PREC == kPrecBF16 && g_pair_ring && pair_ok(g) && M == 256 && N == 256) {
      // both gradients in one launch on co-scheduled workgroup pairs (pair_ring_bf16_kernel):
      // 1 = middle layer, 2 = top layer with the output layer folded in, 3 = bottom layer with the
      // first layer folded in and P_0 rebuilt from x
      const int kind = (rec1 && !is_top)                                   ? 3
                       : (ring_t && !is_bot)                               ? 2
                       : (!is_top && !is_bot && !rec1 && g_dw_ring && g_dx_ring) ? 1
                                                                           : 0;
      if (kind) {
        // consecutive pair launches alternate slab buffers (the pending reduction reads the other
        // one); without a second buffer the pending reduction goes first
        float* pp = part;
        if (!g_tail_reduce && (rc = flush())) return rc;
        if (lo.part2_off >= 0) {
          if (npair_launches++ & 1) pp = (float*)(ws + lo.part2_off);
        } else if ((rc = flush())) {
          return rc;
        }
        if ((rc = launch_pair<PREC>(d, g, lo, kind, l, x, ta, ws, saved, pp, dW, db, dx, cur, pend, st))) return rc;
        if (kind == 3) return flush();  // first layer done
        cur ^= 1;
        continue;
      }
    }
    if ((rc = flush())) return rc;  // the per-layer kernels below reuse `part`
    const bool ring = rec1 || ring_t || (PREC == kPrecBF16 && g_dw_ring && !is_top && M == 256 && N == 256);
    {
      const Split s = ring ? dw_ring_split(g) : tn_split(g, M, N);
      int64_t nsplit_used = s.nsplit;
      TNArgs a;
      memset(&a, 0, sizeof(a));
      a.D = ws + lo.dz_off[cur];
      a.P = rec1 ? (const void*)x : P(l - 1);
      a.part = part;
      a.rows_per_batch = g.rows;
      a.rows_per_split = s.rows_per_split;
      a.split_stride = split_stride(g, (int64_t)M * N + M);
      if (rec1) {
        a.rec_W0 = d->weight[0];
        a.rec_w0_bstride = d->weights_batched ? (int64_t)F0 * C : 0;
        a.rec_b0 = d->bias[0];
        a.rec_b0_bstride = d->weights_batched ? F0 : 0;
      }
      a.M = M;
      a.N = N;
      a.p_vec = 0;
      a.w0 = d->w0;
      a.top = ta;
      dim3 grid((unsigned)(cdiv(M, TN_BM) * cdiv(N, TN_BN)), (unsigned)s.nsplit, (unsigned)g.nb);
      const int kcls = PREC != kPrecBF16 || !ring ? SIREN_KCLASS_DW_GEMM
                       : rec1                     ? SIREN_KCLASS_DW_RING_REC
                       : ring_t                   ? SIREN_KCLASS_DW_RING_TOP
                                                  : SIREN_KCLASS_DW_RING;
      tmark_begin(kcls, st);
      if constexpr (PREC == kPrecBF16) {
        const dim3 rg((unsigned)s.nsplit, (unsigned)g.nb);
        if (rec1) {
          switch (C) {
            case 1: hipLaunchKernelGGL((dw_ring_bf16_kernel<1>), rg, dim3(512), 0, st, a); break;
            case 2: hipLaunchKernelGGL((dw_ring_bf16_kernel<2>), rg, dim3(512), 0, st, a); break;
            case 3: hipLaunchKernelGGL((dw_ring_bf16_kernel<3>), rg, dim3(512), 0, st, a); break;
            default: hipLaunchKernelGGL((dw_ring_bf16_kernel<4>), rg, dim3(512), 0, st, a); break;
          }
        } else if (ring_t) {
          if (O == 1) hipLaunchKernelGGL((dw_ring_bf16_kernel<0, 1>), rg, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((dw_ring_bf16_kernel<0, 2>), rg, dim3(512), 0, st, a);
        } else if (ring)
          hipLaunchKernelGGL((dw_ring_bf16_kernel<0>), rg, dim3(512), 0, st, a);
        else if (is_top) hipLaunchKernelGGL((tn_dw_kernel<PREC, false, true>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((tn_dw_kernel<PREC, false>), grid, dim3(256), 0, st, a);
      } else if (g_f32_rows && jvp_tn2_ok(M, N)) {
        // fp32: jvp_tn2_kernel over the primal stream alone (S = 1: X = sin(P_{l-1}), D = dZ_l):
        // all 256 dW rows per workgroup, so each X element is formed once per launch
        JTNArgs j;
        memset(&j, 0, sizeof(j));
        const Split s2 = jtn2_split(g, g.rows, N);
        j.D = a.D;
        j.P = a.P;
        j.U = nullptr;
        j.part = part;
        j.N = g.rows;
        j.rows_per_split = s2.rows_per_split;
        j.split_stride = a.split_stride;
        j.S = 1;
        j.Su = 0;
        j.C = 0;
        j.M = M;
        j.Kin = N;
        j.w0 = d->w0;
        nsplit_used = s2.nsplit;
        hipLaunchKernelGGL((jvp_tn2_kernel<false>), dim3((unsigned)cdiv(N, JTN2_BN), (unsigned)s2.nsplit, (unsigned)g.nb),
                           dim3(512), 0, st, j);
      } else {
        hipLaunchKernelGGL((tn_dw_kernel<PREC, false>), grid, dim3(256), 0, st, a);
      }
      tmark_end(kcls, st);
      if ((rc = check_launch("tn_dw"))) return rc;
      if ((rc = launch_reduce(part, nsplit_used, a.split_stride, g.nb, (int64_t)M * N + M,
                              (int64_t)M * N, dW[l], db[l], st)))
        return rc;
      if (is_top &&
          (rc = launch_reduce(ta.partL, s.nsplit, ta.partL_stride, g.nb, (int64_t)O * M + O, (int64_t)O * M,
                              dW[g.L - 1], db[g.L - 1], st)))
        return rc;
    }
    {
      NTArgs a;
      memset(&a, 0, sizeof(a));
      a.A = ws + lo.dz_off[cur];
      a.W = saved + lo.wt_op_off[l];
      a.bias = nullptr;
      a.Paux = rec1 ? nullptr : P(l - 1);
      a.C = ws + lo.dz_off[cur ^ 1];
      a.rows_per_batch = g.rows;
      a.w_bstride = d->weights_batched ? (int64_t)M * N : 0;
      a.bias_bstride = 0;
      a.K = M;
      a.N = N;
      a.lda = M;
      a.a_vec = 0;
      a.w0 = d->w0;
      a.top = ta;
      a.stagger = g_dx_stagger ? 1 : 0;
      const int64_t bot_stride = split_stride(g, (int64_t)F0 * C + F0);
      if (is_bot) {
        a.bot.x = x;
        a.bot.W0 = d->weight[0];
        a.bot.w0_bstride = d->weights_batched ? (int64_t)F0 * C : 0;
        a.bot.b0 = d->bias[0];
        a.bot.b0_bstride = d->weights_batched ? F0 : 0;
        a.bot.part = part;
        a.bot.split_stride = bot_stride;
        a.bot.C = C;
      }
      if constexpr (PREC == kPrecBF16) {
        if (is_bot && ring_bot) {
          a.C = dx;  // [rows, C] f32, or not written
          rc = launch_dx_ring_bot(a, g.nb, C, dx != nullptr, rec1, SIREN_KCLASS_DX_RING_BOT, st);
        } else if (ring_t) {
          tmark_begin(SIREN_KCLASS_DX_RING_TOP, st);
          if (O == 1) hipLaunchKernelGGL((dx_ring_bf16_kernel<0, false, false, 1>), ring_grid(a, g.nb), dim3(512), 0, st, a);
          else hipLaunchKernelGGL((dx_ring_bf16_kernel<0, false, false, 2>), ring_grid(a, g.nb), dim3(512), 0, st, a);
          tmark_end(SIREN_KCLASS_DX_RING_TOP, st);
          rc = check_launch("dx_ring top");
        } else if (is_top && is_bot) rc = launch_nt<PREC, MODE_DX, true, true>(a, g.nb, SIREN_KCLASS_DX_GEMM, st);
        else if (is_top) rc = launch_nt<PREC, MODE_DX, true, false>(a, g.nb, SIREN_KCLASS_DX_GEMM, st);
        else if (is_bot) rc = launch_nt<PREC, MODE_DX, false, true>(a, g.nb, SIREN_KCLASS_DX_GEMM, st);
        else rc = launch_nt<PREC, MODE_DX>(a, g.nb, SIREN_KCLASS_DX_GEMM, st);
      } else {
        rc = launch_nt<PREC, MODE_DX>(a, g.nb, SIREN_KCLASS_DX_GEMM, st);
      }
      if (rc) return rc;
      if (is_bot) {
        const int64_t nslab = ring_bot ? ring_grid(a, g.nb).x : nt_grid(a, g.nb, PREC).x;
        if ((rc = launch_reduce(part, nslab, bot_stride, g.nb, (int64_t)F0 * C + F0, (int64_t)F0 * C, dW[0],
                                db[0], st)))
          return rc;
        return SIREN_OK;  // first layer done
      }
      cur ^= 1;
    }
  }
  if ((rc = flush())) return rc;
  // First layer.
  if (wide_input(d)) {
    const int F0 = d->dims[1], C = d->dims[0];
    const Split s = tn_split(g, F0, C);
    TNArgs a;
    a.D = ws + lo.dz_off[cur];
    a.P = x;
    a.part = part;
    a.rows_per_batch = g.rows;
    a.rows_per_split = s.rows_per_split;
    a.split_stride = split_stride(g, (int64_t)F0 * C + F0);
    a.M = F0;
    a.N = C;
    a.p_vec = (C % 4 == 0) && aligned16(x);
    dim3 grid((unsigned)(cdiv(F0, TN_BM) * cdiv(C, TN_BN)), (unsigned)s.nsplit, (unsigned)g.nb);
    hipLaunchKernelGGL((tn_dw_kernel<PREC, true>), grid, dim3(256), 0, st, a);
    if ((rc = check_launch("tn_dw first"))) return rc;
    if ((rc = launch_reduce(part, s.nsplit, a.split_stride, g.nb, (int64_t)F0 * C + F0,
                            (int64_t)F0 * C, dW[0], db[0], st)))
      return rc;
    if (dx) {
      NTArgs n;
      n.A = ws + lo.dz_off[cur];
      n.W = saved + lo.wt_op_off[0];
      n.bias = nullptr;
      n.Paux = nullptr;
      n.C = dx;
      n.rows_per_batch = g.rows;
      n.w_bstride = d->weights_batched ? (int64_t)F0 * C : 0;
      n.bias_bstride = 0;
      n.K = F0;
      n.N = C;
      n.lda = F0;
      n.a_vec = 0;
      n.w0 = d->w0;
      if ((rc = launch_nt<PREC, MODE_DXLIN>(n, g.nb, 0, st))) return rc;
    }
  } else {
    const Split s = valu_split(g);
    FirstBwdArgs a;
    memset(&a, 0, sizeof(a));
    a.dZ = ws + lo.dz_off[cur];
    a.x = x;
    a.ffB = d->ff_B;
    a.ffin = d->ff_B ? d->ff_in : 0;
    a.W = d->weight[0];
    a.dx = dx;
    a.part = part;
    a.rows_per_batch = g.rows;
    a.rows_per_split = s.rows_per_split;
    a.F = d->dims[1];
    a.C = d->dims[0];
    a.split_stride = split_stride(g, (int64_t)a.F * a.C + a.F);
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[1] * d->dims[0] : 0;
    if ((rc = dispatch_first_bwd<PREC>(a, s.nsplit, g.nb, st))) return rc;
    if ((rc = launch_reduce(part, s.nsplit, a.split_stride, g.nb, (int64_t)a.F * a.C + a.F,
                            (int64_t)a.F * a.C, dW[0], db[0], st)))
      return rc;
  }
  return SIREN_OK;
}

// ============================================================================================
// Analytic derivatives (tangent streams): layout and orchestration.
// saved = [prepared weights][P_l phase tensors, l = 0..L-2][U_l fp32 tangent planes, l = 0..L-2]
// ============================================================================================
struct JLayout {
  Layout base;             // prepared-weight offsets (w_op_off / wt_op_off / weights_bytes)
  int C, Su, S, Sb;        // tangents, stored U planes, forward streams, adjoint streams
  int64_t p_off[SIREN_MAX_LAYERS], u_off[SIREN_MAX_LAYERS];
  int64_t saved_bytes;
  int64_t d_off[2], raw_off, part_off, ws_bytes;
};

Split jtn_split(const Geo& g, int64_t stacked_rows, int M, int N) {
  const int64_t tiles = cdiv(M, 128) * cdiv(N, 128);
  return split_rows(stacked_rows, tiles, g.nb, 32);
}
Split jcol_split(const Geo& g) { return split_rows(g.rows, 1, g.nb, 64); }

JLayout jlayout_of(const siren_mlp_desc* d, int order) {
  const Geo g = geo_of(d);
  JLayout jl;
  memset(&jl, 0, sizeof(jl));
  jl.base = layout_of(d);
  jl.C = d->dims[0];
  jl.Su = jl.C + (order == SIREN_JVP_LAPLACE ? 1 : 0);
  jl.S = 1 + jl.Su;
  jl.Sb = 1 + jl.Su;  // adjoints [a_bar; u_bar^k (; V_bar)] mirror the forward streams
  int64_t off = jl.base.weights_bytes;
  for (int l = 0; l + 1 < g.L; ++l) {
    jl.p_off[l] = off;
    off = align_up(off + g.total * d->dims[l + 1] * g.phase_sz, 256);
  }
  for (int l = 0; l + 1 < g.L; ++l) {
    jl.u_off[l] = off;
    off = align_up(off + (int64_t)jl.Su * g.total * d->dims[l + 1] * 4, 256);
  }
  jl.saved_bytes = off;
  off = align_up(jl.base.weights_bytes, 256);  // workspace (prepared weights first when no saved)
  const int64_t act = (int64_t)jl.Sb * g.total * max_hidden(d);
  for (int k = 0; k < 2; ++k) {
    jl.d_off[k] = off;
    off = align_up(off + act * g.grad_sz, 256);
  }
  jl.raw_off = off;
  off = align_up(off + act * 4, 256);
  int64_t part = 0;
  for (int l = 1; l + 1 < g.L; ++l) {
    const int M = d->dims[l + 1], N = d->dims[l];
    const Split s = jtn_split(g, (int64_t)jl.Sb * g.rows, M, N);
    part = std::max(part, s.nsplit * split_stride(g, (int64_t)M * N + M));
  }
  {
    const Split s = jcol_split(g);
    const int F = d->dims[g.L - 1], O = d->dims[g.L];
    part = std::max(part, s.nsplit * split_stride(g, (int64_t)O * F + O));
    const int F0 = d->dims[1], C = d->dims[0];
    part = std::max(part, s.nsplit * split_stride(g, (int64_t)F0 * C + F0));
  }
  jl.part_off = off;
  off = align_up(off + part * 4, 256);
  jl.ws_bytes = off;
  return jl;
}

int jvp_check(const siren_mlp_desc* d, int order) {
  int rc = siren_mlp_check(d);
  if (rc) return rc;
  if (order != SIREN_JVP_GRADIENT && order != SIREN_JVP_LAPLACE && order != SIREN_JVP_JACOBIAN)
    return fail(SIREN_EINVAL, "derivative mode %d unsupported (1 gradient, 2 Laplacian, 3 Jacobian)", order);
  if (!d->outermost_linear) return fail(SIREN_EINVAL, "analytic derivatives need outermost_linear");
  if (d->dims[0] > 4) return fail(SIREN_EINVAL, "analytic derivatives support in_features <= 4");
  return SIREN_OK;
}

template <int PREC>
int jvp_forward_impl(const siren_mlp_desc* d, int order, const float* x, float* grad, float* lap,
                     char* saved, char* ws, hipStream_t st, const char* primal = nullptr) {
  const Geo g = geo_of(d);
  const JLayout jl = jlayout_of(d, order);
  char* base = saved ? saved : ws;
  int rc = prep_weights<PREC>(d, g, jl.base, base, st);
  if (rc) return rc;
  // without a saved buffer the per-layer tensors still need a home: use the saved layout inside
  // the workspace tail (jvp workspace queries include it in that case, see siren_jvp_workspace_bytes)
  char* store = saved ? saved : ws + jl.ws_bytes;
  // primal given: layer l's phases are the plain forward's saved P_l (siren_mlp_forward's layout),
  // and only the tangent streams run (stacked rows N .. S N)
  auto pptr = [&](int l) -> char* { return primal ? (char*)primal + jl.base.saved_off[l] : store + jl.p_off[l]; };
  {
    JFirstArgs a;
    a.x = x;
    a.W = d->weight[0];
    a.bias = d->bias[0];
    a.P = primal ? nullptr : store + jl.p_off[0];
    a.U = (float*)(store + jl.u_off[0]);
    a.N = g.rows;
    a.C = d->dims[0];
    a.F = d->dims[1];
    a.Su = jl.Su;
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[1] * d->dims[0] : 0;
    a.b_bstride = d->weights_batched ? d->dims[1] : 0;
    a.w0 = d->w0;
    hipLaunchKernelGGL(jvp_first_kernel<PREC>, dim3(grid1d(g.rows * a.F, std::max<int64_t>(1, 4096 / g.nb)), (unsigned)g.nb),
                       dim3(256), 0, st, a);
    if ((rc = check_launch("jvp_first"))) return rc;
  }
  for (int l = 1; l + 1 < g.L; ++l) {
    JNTArgs a;
    a.P = pptr(l - 1);
    a.U = (const float*)(store + jl.u_off[l - 1]);
    a.D = nullptr;
    a.W = PREC == kPrecBF16 ? (const void*)(base + jl.base.w_op_off[l]) : (const void*)d->weight[l];
    a.bias = d->bias[l];
    a.Pout = pptr(l);
    a.Uout = (float*)(store + jl.u_off[l]);
    a.N = g.rows;
    a.srow0 = primal ? g.rows : 0;
    a.S = jl.S;
    a.C = jl.C;
    a.lap = order == SIREN_JVP_LAPLACE;
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[l + 1] * d->dims[l] : 0;
    a.b_bstride = d->weights_batched ? d->dims[l + 1] : 0;
    a.K = d->dims[l];
    a.Nout = d->dims[l + 1];
    a.w0 = d->w0;
    if (PREC == kPrecF32 && primal && !a.lap && g_jvp_tan && jl.C >= 1 && jl.C <= 4 && a.Nout <= JADJ_BN &&
        a.K % JNT_KC == 0) {
      // the tangent streams only, stacked by row: one phase load and cosine per element
      JTanArgs t;
      t.P = a.P;
      t.U = a.U;
      t.W = a.W;
      t.Uout = a.Uout;
      t.N = g.rows;
      t.Su = jl.Su;
      t.w_bstride = a.w_bstride;
      t.K = a.K;
      t.Nout = a.Nout;
      t.w0 = a.w0;
      const dim3 tg((unsigned)cdiv(g.rows, JADJ_ROWS), (unsigned)g.nb);
      // (fp32 only: the primal stream is given by the fp32 forward alone, jvp_primal_check)
      constexpr int TP = kPrecF32;
      switch (jl.C) {
        case 1: hipLaunchKernelGGL((jvp_tan_kernel<TP, 1>), tg, dim3(512), 0, st, t); break;
        case 2: hipLaunchKernelGGL((jvp_tan_kernel<TP, 2>), tg, dim3(512), 0, st, t); break;
        case 3: hipLaunchKernelGGL((jvp_tan_kernel<TP, 3>), tg, dim3(512), 0, st, t); break;
        default: hipLaunchKernelGGL((jvp_tan_kernel<TP, 4>), tg, dim3(512), 0, st, t); break;
      }
      if ((rc = check_launch("jvp_tan"))) return rc;
      continue;
    }
    dim3 grid((unsigned)cdiv((int64_t)jl.S * g.rows - a.srow0, JNT_BM), (unsigned)cdiv(a.Nout, JNT_BN), (unsigned)g.nb);
    if (a.lap) hipLaunchKernelGGL((jvp_nt_kernel<PREC, JMODE_FWD, true>), grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((jvp_nt_kernel<PREC, JMODE_FWD>), grid, dim3(256), 0, st, a);
    if ((rc = check_launch("jvp_nt fwd"))) return rc;
  }
  {
    const int l = g.L - 1;
    JLastArgs a;
    a.P = pptr(l - 1);
    a.U = (const float*)(store + jl.u_off[l - 1]);
    a.W = d->weight[l];
    a.grad = grad;
    a.lap = order == SIREN_JVP_LAPLACE ? lap : nullptr;
    a.jac = order == SIREN_JVP_JACOBIAN;
    a.N = g.rows;
    a.C = jl.C;
    a.F = d->dims[l];
    a.O = d->dims[l + 1];
    a.Su = jl.Su;
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[l + 1] * d->dims[l] : 0;
    a.w0 = d->w0;
    hipLaunchKernelGGL(jvp_last_kernel<PREC>, dim3((unsigned)std::min<int64_t>(cdiv(g.rows, 8), 4096 / g.nb + 1), (unsigned)g.nb),
                       dim3(256), 0, st, a);
    if ((rc = check_launch("jvp_last"))) return rc;
  }
  return SIREN_OK;
}

// jvp_tn2_kernel (fp32 weight gradient of a hidden layer): dW of 256 rows (the layer's width M), input
// width a multiple of 4; option jvp_tn2 (default on)
bool jvp_tn2_ok(int M, int N) { return g_jvp_tn2 && M == 256 && N % 4 == 0; }
Split jtn2_split(const Geo& g, int64_t stacked_rows, int N) {
  const int64_t want = std::max<int64_t>(1, 256 / (cdiv(N, JTN2_BN) * g.nb));
  Split s;
  s.rows_per_split = std::max<int64_t>(JTN2_KC, align_up(cdiv(stacked_rows, want), JTN2_KC));
  s.nsplit = std::max<int64_t>(1, cdiv(stacked_rows, s.rows_per_split));
  return s;
}

// jvp_adj_kernel's shapes: 2..4 adjoint streams (gradient with C <= 3, Laplacian with C <= 2) and a
// layer below of at most 256 features (one column tile)
bool jvp_adj_fused(int S, int lap, int Nout) {
  return g_jvp_adj && S >= 2 && S <= 4 && !(lap && S < 3) && Nout <= JADJ_BN;
}

template <int PREC>
int jvp_backward_impl(const siren_mlp_desc* d, int order, const float* x, const float* dout,
                      const char* saved, char* ws, float* const* dW, float* const* db, float* dx, hipStream_t st,
                      const char* primal = nullptr) {
  const Geo g = geo_of(d);
  const JLayout jl = jlayout_of(d, order);
  auto pptr = [&](int l) -> const char* { return primal ? primal + jl.base.saved_off[l] : saved + jl.p_off[l]; };
  const int lapmode = order == SIREN_JVP_LAPLACE;
  float* part = (float*)(ws + jl.part_off);
  int rc = SIREN_OK;
  int cur = 0;
  {
    const int l = g.L - 1;
    const Split s = jcol_split(g);
    JCombArgs a;
    a.P = pptr(l - 1);
    a.U = (const float*)(saved + jl.u_off[l - 1]);
    a.raw = nullptr;
    a.gbar = lapmode ? nullptr : dout;
    a.lbar = lapmode ? dout : nullptr;
    a.WL = d->weight[l];
    a.D = ws + jl.d_off[cur];
    a.part = part;
    a.N = g.rows;
    a.rows_per_split = s.rows_per_split;
    a.C = jl.C;
    a.F = d->dims[l];
    a.O = d->dims[l + 1];
    a.Su = jl.Su;
    a.S = jl.Sb;
    a.top = 1;
    a.lap = lapmode;
    a.split_stride = split_stride(g, (int64_t)a.O * a.F + a.O);
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[l + 1] * d->dims[l] : 0;
    a.w0 = d->w0;
    a.jac = order == SIREN_JVP_JACOBIAN;
    if (a.jac)
      hipLaunchKernelGGL(jvp_combine_jac_kernel<PREC>, dim3((unsigned)s.nsplit, (unsigned)g.nb), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL(jvp_combine_kernel<PREC>, dim3((unsigned)s.nsplit, (unsigned)g.nb), dim3(256), 0, st, a);
    if ((rc = check_launch("jvp_combine top"))) return rc;
    if ((rc = launch_reduce(part, s.nsplit, a.split_stride, g.nb, (int64_t)a.O * a.F + a.O,
                            (int64_t)a.O * a.F, dW[l], db[l], st)))
      return rc;
  }
  for (int l = g.L - 2; l >= 1; --l) {
    const int M = d->dims[l + 1], N = d->dims[l];
    {
      const Split s = jtn_split(g, (int64_t)jl.Sb * g.rows, M, N);
      JTNArgs a;
      a.D = ws + jl.d_off[cur];
      a.P = pptr(l - 1);
      a.U = (const float*)(saved + jl.u_off[l - 1]);
      a.part = part;
      a.N = g.rows;
      a.rows_per_split = s.rows_per_split;
      a.split_stride = split_stride(g, (int64_t)M * N + M);
      a.S = jl.Sb;
      a.Su = jl.Su;
      a.C = jl.C;
      a.M = M;
      a.Kin = N;
      a.w0 = d->w0;
      if (PREC == kPrecF32 && jvp_tn2_ok(M, N)) {
        // fp32: all 256 dW rows per workgroup (jvp_tn2_kernel), with its own, smaller split count
        const Split s2 = jtn2_split(g, (int64_t)jl.Sb * g.rows, N);
        a.rows_per_split = s2.rows_per_split;
        dim3 grid2((unsigned)cdiv(N, JTN2_BN), (unsigned)s2.nsplit, (unsigned)g.nb);
        if (lapmode) hipLaunchKernelGGL((jvp_tn2_kernel<true>), grid2, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((jvp_tn2_kernel<false>), grid2, dim3(512), 0, st, a);
        if ((rc = check_launch("jvp_tn2"))) return rc;
        if ((rc = launch_reduce(part, s2.nsplit, a.split_stride, g.nb, (int64_t)M * N + M, (int64_t)M * N,
                                dW[l], db[l], st)))
          return rc;
      } else {
        dim3 grid((unsigned)(cdiv(M, 128) * cdiv(N, 128)), (unsigned)s.nsplit, (unsigned)g.nb);
        if (lapmode) hipLaunchKernelGGL((jvp_tn_kernel<PREC, true>), grid, dim3(256), 0, st, a);
        else hipLaunchKernelGGL((jvp_tn_kernel<PREC>), grid, dim3(256), 0, st, a);
        if ((rc = check_launch("jvp_tn"))) return rc;
        if ((rc = launch_reduce(part, s.nsplit, a.split_stride, g.nb, (int64_t)M * N + M, (int64_t)M * N,
                                dW[l], db[l], st)))
          return rc;
      }
    }
    if (jvp_adj_fused(jl.Sb, lapmode, N)) {
      // adjoint GEMM + combine in one launch (jvp_adj_kernel)
      JAdjArgs a;
      a.D = ws + jl.d_off[cur];
      a.W = saved + jl.base.wt_op_off[l];
      a.P = pptr(l - 1);
      a.U = (const float*)(saved + jl.u_off[l - 1]);
      a.Dout = ws + jl.d_off[cur ^ 1];
      a.N = g.rows;
      a.Su = jl.Su;
      a.w_bstride = d->weights_batched ? (int64_t)M * N : 0;
      a.K = M;
      a.Nout = N;
      a.w0 = d->w0;
      const dim3 grid((unsigned)cdiv(g.rows, JADJ_ROWS), (unsigned)g.nb);
      switch (jl.Sb * 2 + lapmode) {
        case 4: hipLaunchKernelGGL((jvp_adj_kernel<PREC, 2, false>), grid, dim3(512), 0, st, a); break;
        case 6: hipLaunchKernelGGL((jvp_adj_kernel<PREC, 3, false>), grid, dim3(512), 0, st, a); break;
        case 7: hipLaunchKernelGGL((jvp_adj_kernel<PREC, 3, true>), grid, dim3(512), 0, st, a); break;
        case 8: hipLaunchKernelGGL((jvp_adj_kernel<PREC, 4, false>), grid, dim3(512), 0, st, a); break;
        default: hipLaunchKernelGGL((jvp_adj_kernel<PREC, 4, true>), grid, dim3(512), 0, st, a); break;
      }
      if ((rc = check_launch("jvp_adj"))) return rc;
      cur ^= 1;
      continue;
    }
    {
      JNTArgs a;
      memset(&a, 0, sizeof(a));
      a.D = ws + jl.d_off[cur];
      a.W = saved + jl.base.wt_op_off[l];
      a.Uout = (float*)(ws + jl.raw_off);
      a.N = g.rows;
      a.S = jl.Sb;
      a.C = jl.C;
      a.w_bstride = d->weights_batched ? (int64_t)M * N : 0;
      a.K = M;
      a.Nout = N;
      a.w0 = d->w0;
      dim3 grid((unsigned)cdiv((int64_t)jl.Sb * g.rows, JNT_BM), (unsigned)cdiv(N, JNT_BN), (unsigned)g.nb);
      hipLaunchKernelGGL((jvp_nt_kernel<PREC, JMODE_BWD>), grid, dim3(256), 0, st, a);
      if ((rc = check_launch("jvp_nt bwd"))) return rc;
    }
    {
      const Split s = jcol_split(g);
      JCombArgs a;
      memset(&a, 0, sizeof(a));
      a.P = pptr(l - 1);
      a.U = (const float*)(saved + jl.u_off[l - 1]);
      a.raw = (const float*)(ws + jl.raw_off);
      a.D = ws + jl.d_off[cur ^ 1];
      a.N = g.rows;
      a.rows_per_split = s.rows_per_split;
      a.C = jl.C;
      a.F = N;
      a.Su = jl.Su;
      a.S = jl.Sb;
      a.top = 0;
      a.lap = lapmode;
      a.w0 = d->w0;
      hipLaunchKernelGGL(jvp_combine_kernel<PREC>, dim3((unsigned)s.nsplit, (unsigned)g.nb), dim3(256), 0, st, a);
      if ((rc = check_launch("jvp_combine"))) return rc;
      cur ^= 1;
    }
  }
  {
    const Split s = jcol_split(g);
    JFirstBwdArgs a;
    a.D = ws + jl.d_off[cur];
    a.x = x;
    a.W = d->weight[0];
    a.dx = dx;
    a.part = part;
    a.N = g.rows;
    a.rows_per_split = s.rows_per_split;
    a.C = d->dims[0];
    a.F = d->dims[1];
    a.S = jl.Sb;
    a.split_stride = split_stride(g, (int64_t)a.F * a.C + a.F);
    a.w_bstride = d->weights_batched ? (int64_t)d->dims[1] * d->dims[0] : 0;
    hipLaunchKernelGGL(jvp_first_bwd_kernel<PREC>, dim3((unsigned)s.nsplit, (unsigned)g.nb), dim3(256), 0, st, a);
    if ((rc = check_launch("jvp_first_bwd"))) return rc;
    if ((rc = launch_reduce(part, s.nsplit, a.split_stride, g.nb, (int64_t)a.F * a.C + a.F,
                            (int64_t)a.F * a.C, dW[0], db[0], st)))
      return rc;
    if (dx) {
      hipLaunchKernelGGL(jvp_first_dx_kernel<PREC>, dim3((unsigned)std::min<int64_t>(cdiv(g.rows, 8), 4096 / g.nb + 1), (unsigned)g.nb),
                         dim3(256), 0, st, a);
      if ((rc = check_launch("jvp_first_dx"))) return rc;
    }
  }
  return SIREN_OK;
}

}  // namespace

// ------------------------------------------------------------------ hypernetwork heads
namespace {
constexpr int HY_KCH = 512;  // K per split of the wide output layers' input gradient

int hyper_check(const siren_hyper_desc* d) {
  if (!d) return fail(SIREN_EINVAL, "null hyper descriptor");
  if (d->heads < 1 || d->heads > SIREN_HYPER_MAXG) return fail(SIREN_EINVAL, "hyper: %d heads (1..%d)", d->heads, SIREN_HYPER_MAXG);
  if (d->depth < 1 || d->depth > SIREN_HYPER_MAXD) return fail(SIREN_EINVAL, "hyper: depth %d (1..%d)", d->depth, SIREN_HYPER_MAXD);
  if (d->rows < 1 || d->in_features < 1 || d->hidden < 1) return fail(SIREN_EINVAL, "hyper: empty shape");
  for (int g = 0; g < d->heads; ++g) {
    if (d->out_features[g] < 1) return fail(SIREN_EINVAL, "hyper: head %d has no outputs", g);
    for (int l = 0; l <= d->depth; ++l)
      if (!d->weight[g * 5 + l] || !d->bias[g * 5 + l]) return fail(SIREN_EINVAL, "hyper: head %d layer %d null", g, l);
  }
  return SIREN_OK;
}
int64_t hyper_act(const siren_hyper_desc* d) { return (int64_t)d->rows * d->hidden; }
int hyper_nsplit(int n) { return (n + HY_KCH - 1) / HY_KCH; }
struct HyperWs {
  int64_t dz_off[2], part_off[SIREN_HYPER_MAXG], dzg_off, bytes;
};
HyperWs hyper_ws(const siren_hyper_desc* d) {
  HyperWs w;
  int64_t off = 0;
  const int64_t act = hyper_act(d) * 4 * d->heads;
  for (int k = 0; k < 2; ++k) {
    w.dz_off[k] = off;
    off = align_up(off + act, 256);
  }
  for (int g = 0; g < d->heads; ++g) {
    w.part_off[g] = off;
    off = align_up(off + (int64_t)hyper_nsplit(d->out_features[g]) * hyper_act(d) * 4, 256);
  }
  w.dzg_off = off;
  off = align_up(off + (int64_t)d->heads * d->rows * d->in_features * 4, 256);
  w.bytes = off;
  return w;
}
// tiles of one group (split: the number of K splits of HY_PART); BM 32 tiles (32 x 128) when every
// group has at most 32 rows, else 64 x 64
int hy_tiles(int M, int N, int split, int bm) { return (int)(cdiv(M, bm) * cdiv(N, 4096 / bm)) * split; }

template <int TA, int TB, int EPI>
int hy_launch(HyArgs& a, hipStream_t st) {
  // 32 x 128 tiles when every group has <= 32 rows and they still give >= 128 workgroups
  int bm = 32, t32 = 0;
  for (int g = 0; g < a.ng; ++g) {
    const HyGroup& G = a.g[g];
    if (G.M > 32) bm = 64;
    t32 += hy_tiles(G.M, G.N, EPI == HY_PART ? (G.K + G.ksplit - 1) / G.ksplit : 1, 32);
  }
  if (t32 < 128) bm = 64;
  int t = 0;
  for (int g = 0; g < a.ng; ++g) {
    HyGroup& G = a.g[g];
    G.tile0 = t;
    const int ns = EPI == HY_PART ? (G.K + G.ksplit - 1) / G.ksplit : 1;
    t += hy_tiles(G.M, G.N, ns, bm);
  }
  a.ntiles = t;
  if (bm == 32) hipLaunchKernelGGL((hy_gemm_kernel<TA, TB, EPI, 32>), dim3((unsigned)t), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((hy_gemm_kernel<TA, TB, EPI, 64>), dim3((unsigned)t), dim3(256), 0, st, a);
  return check_launch("hy_gemm");
}
}  // namespace

extern "C" {

int64_t siren_hyper_saved_bytes(const siren_hyper_desc* d) {
  if (hyper_check(d)) return -1;
  return (int64_t)d->heads * d->depth * hyper_act(d) * 4;
}

int64_t siren_hyper_workspace_bytes(const siren_hyper_desc* d) {
  if (hyper_check(d)) return -1;
  return hyper_ws(d).bytes;
}

int siren_hyper_forward(const siren_hyper_desc* d, const float* z, float* const* out, void* saved, int64_t saved_bytes,
                        void* stream) {
  int rc = hyper_check(d);
  if (rc) return rc;
  if (!z || !out || !saved) return fail(SIREN_EINVAL, "hyper forward: null argument");
  if (saved_bytes < siren_hyper_saved_bytes(d)) return fail(SIREN_ENOSPACE, "hyper forward: saved buffer too small");
  hipStream_t st = (hipStream_t)stream;
  const int G = d->heads, D = d->depth, B = d->rows, H = d->hidden;
  float* hs = (float*)saved;  // H_{l+1}[g] at hs + (g * D + l) * B * H
  auto hbuf = [&](int g, int l) { return hs + ((int64_t)g * D + l) * B * H; };
  for (int l = 0; l < D; ++l) {
    HyArgs a;
    memset(&a, 0, sizeof(a));
    a.ng = G;
    for (int g = 0; g < G; ++g) {
      HyGroup& q = a.g[g];
      const int K = l == 0 ? d->in_features : H;
      q.A = l == 0 ? z : hbuf(g, l - 1);
      q.lda = K;
      q.B = d->weight[g * 5 + l];
      q.ldb = K;
      q.bias = d->bias[g * 5 + l];
      q.C = hbuf(g, l);
      q.ldc = H;
      q.M = B;
      q.N = H;
      q.K = K;
    }
    if ((rc = hy_launch<0, 0, HY_BIAS_RELU>(a, st))) return rc;
  }
  HyArgs a;
  memset(&a, 0, sizeof(a));
  a.ng = G;
  for (int g = 0; g < G; ++g) {
    if (!out[g]) return fail(SIREN_EINVAL, "hyper forward: head %d null output", g);
    HyGroup& q = a.g[g];
    q.A = hbuf(g, D - 1);
    q.lda = H;
    q.B = d->weight[g * 5 + D];
    q.ldb = H;
    q.bias = d->bias[g * 5 + D];
    q.C = out[g];
    q.ldc = d->out_features[g];
    q.M = B;
    q.N = d->out_features[g];
    q.K = H;
  }
  return hy_launch<0, 0, HY_BIAS>(a, st);
}

int siren_hyper_backward(const siren_hyper_desc* d, const float* z, const float* const* dout, const void* saved,
                         int64_t saved_bytes, void* workspace, int64_t workspace_bytes, float* const* dW,
                         float* const* db, float* dz, void* stream) {
  int rc = hyper_check(d);
  if (rc) return rc;
  if (!z || !dout || !saved || !dW || !db) return fail(SIREN_EINVAL, "hyper backward: null argument");
  if (saved_bytes < siren_hyper_saved_bytes(d)) return fail(SIREN_ENOSPACE, "hyper backward: saved buffer too small");
  const HyperWs w = hyper_ws(d);
  if (!workspace || workspace_bytes < w.bytes) return fail(SIREN_ENOSPACE, "hyper backward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const int G = d->heads, D = d->depth, B = d->rows, H = d->hidden, IN = d->in_features;
  const float* hs = (const float*)saved;
  auto hbuf = [&](int g, int l) { return hs + ((int64_t)g * D + l) * B * H; };
  char* ws = (char*)workspace;
  auto dzbuf = [&](int k, int g) { return (float*)(ws + w.dz_off[k]) + (int64_t)g * B * H; };
  for (int g = 0; g < G; ++g)
    for (int l = 0; l <= D; ++l)
      if (!dW[g * 5 + l] || !db[g * 5 + l]) return fail(SIREN_EINVAL, "hyper backward: head %d layer %d null grad", g, l);
  // output layers: [dW | db] = dout^T [H_D | 1]
  {
    HyArgs a;
    memset(&a, 0, sizeof(a));
    a.ng = G;
    for (int g = 0; g < G; ++g) {
      HyGroup& q = a.g[g];
      q.A = dout[g];
      q.lda = d->out_features[g];
      q.B = hbuf(g, D - 1);
      q.ldb = H;
      q.C = dW[g * 5 + D];
      q.ldc = H;
      q.db = db[g * 5 + D];
      q.M = d->out_features[g];
      q.N = H;
      q.K = B;
    }
    if ((rc = hy_launch<1, 1, HY_DWDB>(a, st))) return rc;
  }
  // their input gradients dout W over K splits, then dZ_{D-1} = sum * (H_D > 0)
  {
    HyArgs a;
    memset(&a, 0, sizeof(a));
    a.ng = G;
    HyPartArgs r;
    memset(&r, 0, sizeof(r));
    r.ng = G;
    r.n = (int64_t)B * H;
    for (int g = 0; g < G; ++g) {
      HyGroup& q = a.g[g];
      q.A = dout[g];
      q.lda = d->out_features[g];
      q.B = d->weight[g * 5 + D];
      q.ldb = H;
      q.C = (float*)(ws + w.part_off[g]);
      q.ldc = H;
      q.M = B;
      q.N = H;
      q.K = d->out_features[g];
      q.ksplit = HY_KCH;
      r.part[g] = q.C;
      r.relu_out[g] = hbuf(g, D - 1);
      r.dz[g] = dzbuf(0, g);
      r.nsplit[g] = hyper_nsplit(d->out_features[g]);
    }
    if ((rc = hy_launch<0, 1, HY_PART>(a, st))) return rc;
    hipLaunchKernelGGL(hy_part_kernel, dim3((unsigned)cdiv(r.n, 256), (unsigned)G), dim3(256), 0, st, r);
    if ((rc = check_launch("hy_part"))) return rc;
  }
  int cur = 0;
  for (int l = D - 1; l >= 0; --l) {
    const int K = l == 0 ? IN : H;
    HyArgs a;
    memset(&a, 0, sizeof(a));
    a.ng = G;
    for (int g = 0; g < G; ++g) {
      HyGroup& q = a.g[g];
      q.A = dzbuf(cur, g);
      q.lda = H;
      q.B = l == 0 ? z : hbuf(g, l - 1);
      q.ldb = K;
      q.C = dW[g * 5 + l];
      q.ldc = K;
      q.db = db[g * 5 + l];
      q.M = H;
      q.N = K;
      q.K = B;
    }
    if ((rc = hy_launch<1, 1, HY_DWDB>(a, st))) return rc;
    if (l == 0 && !dz) break;
    HyArgs b;
    memset(&b, 0, sizeof(b));
    b.ng = G;
    for (int g = 0; g < G; ++g) {
      HyGroup& q = b.g[g];
      q.A = dzbuf(cur, g);
      q.lda = H;
      q.B = d->weight[g * 5 + l];
      q.ldb = K;
      q.M = B;
      q.N = K;
      q.K = H;
      if (l > 0) {
        q.aux = hbuf(g, l - 1);
        q.C = dzbuf(cur ^ 1, g);
        q.ldc = H;
      } else {
        q.C = (float*)(ws + w.dzg_off) + (int64_t)g * B * IN;
        q.ldc = IN;
      }
    }
    if (l > 0) {
      if ((rc = hy_launch<0, 1, HY_MASK>(b, st))) return rc;
      cur ^= 1;
    } else {
      if ((rc = hy_launch<0, 1, HY_PLAIN>(b, st))) return rc;
      HySumArgs sa;
      memset(&sa, 0, sizeof(sa));
      sa.ng = G;
      sa.n = (int64_t)B * IN;
      sa.out = dz;
      for (int g = 0; g < G; ++g) sa.src[g] = (const float*)(ws + w.dzg_off) + (int64_t)g * B * IN;
      hipLaunchKernelGGL(hy_sum_kernel, dim3((unsigned)cdiv(sa.n, 256)), dim3(256), 0, st, sa);
      if ((rc = check_launch("hy_sum"))) return rc;
    }
  }
  return SIREN_OK;
}

}  // extern "C"

namespace {
// ------------------------------------------------------------------ fp64 stack (siren_f64.hip)
struct F64Layout {
  int64_t z_off[SIREN_MAX_LAYERS];  // saved Z of each sine layer (-1: linear output layer)
  int64_t saved_bytes;
  int64_t h_off[2], dz_off[2], part_off, ws_bytes;
};

// split of the weight-gradient GEMM's row reduction: ~512 workgroups over the output tiles
void f64_split(const Geo& g, int M, int N, int64_t& nsplit, int64_t& per) {
  const int64_t tiles = cdiv(M, 64) * cdiv(N + 1, 64) * g.nb;
  nsplit = std::max<int64_t>(1, std::min<int64_t>(cdiv(512, tiles), cdiv(g.rows, 64)));
  per = align_up(cdiv(g.rows, nsplit), 16);
  nsplit = cdiv(g.rows, per);
}

F64Layout f64_layout(const siren_mlp_desc* d) {
  const Geo g = geo_of(d);
  F64Layout lo;
  int64_t off = 0, wmax = 0, part = 0;
  for (int l = 0; l < g.L; ++l) {
    const bool sine = l + 1 < g.L || !d->outermost_linear;
    lo.z_off[l] = sine ? off : -1;
    if (sine) off = align_up(off + g.total * d->dims[l + 1] * 8, 256);
    wmax = std::max<int64_t>(wmax, std::max(d->dims[l], d->dims[l + 1]));
    int64_t ns, per;
    f64_split(g, d->dims[l + 1], d->dims[l], ns, per);
    part = std::max<int64_t>(part, ns * g.nb * (int64_t)d->dims[l + 1] * (d->dims[l] + 1));
  }
  lo.saved_bytes = off;
  off = 0;
  for (int k = 0; k < 2; ++k) {
    lo.h_off[k] = off;
    off = align_up(off + g.total * wmax * 8, 256);
  }
  for (int k = 0; k < 2; ++k) {
    lo.dz_off[k] = off;
    off = align_up(off + g.total * wmax * 8, 256);
  }
  lo.part_off = off;
  off = align_up(off + part * 8, 256);
  lo.ws_bytes = off;
  return lo;
}

int f64_check(const siren_mlp_desc* d) {
  if (!d) return fail(SIREN_EINVAL, "null descriptor");
  const int L = d->num_layers;
  if (L < 1 || L > SIREN_MAX_LAYERS) return fail(SIREN_EINVAL, "num_layers=%d outside [1, %d]", L, SIREN_MAX_LAYERS);
  if (d->prec != SIREN_PREC_F64) return fail(SIREN_EINVAL, "fp64 entry point with precision %d", d->prec);
  if (d->batch < 1 || d->rows_per_batch < 1) return fail(SIREN_EINVAL, "empty input");
  if (d->batch > 65535) return fail(SIREN_EINVAL, "batch %lld > 65535", (long long)d->batch);
  for (int l = 0; l <= L; ++l)
    if (d->dims[l] < 1 || d->dims[l] > 65536) return fail(SIREN_EINVAL, "dims[%d]=%d unsupported", l, d->dims[l]);
  for (int l = 0; l < L; ++l)
    if (!d->weight[l] || !d->bias[l]) return fail(SIREN_EINVAL, "layer %d: null weight/bias", l);
  if (d->ff_B) return fail(SIREN_EINVAL, "fp64: no fused Fourier-feature input");
  return SIREN_OK;
}

template <int TA, int TB, int EPI>
int f64_launch(const F64Args& a, int64_t z, hipStream_t st) {
  const dim3 grid((unsigned)cdiv(a.M, 64), (unsigned)cdiv(EPI == F64_DW ? a.N + 1 : a.N, 64), (unsigned)z);
  hipLaunchKernelGGL((f64_gemm_kernel<TA, TB, EPI>), grid, dim3(256), 0, st, a);
  return check_launch("f64_gemm");
}

}  // namespace

extern "C" {

int64_t siren_mlp64_saved_bytes(const siren_mlp_desc* d) {
  if (f64_check(d)) return -1;
  return f64_layout(d).saved_bytes;
}

int64_t siren_mlp64_workspace_bytes(const siren_mlp_desc* d) {
  if (f64_check(d)) return -1;
  return f64_layout(d).ws_bytes;
}

int siren_mlp64_forward(const siren_mlp_desc* d, const double* x, double* y, void* saved, int64_t saved_bytes,
                        void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = f64_check(d);
  if (rc) return rc;
  if (!x || !y) return fail(SIREN_EINVAL, "fp64 forward: null x / y");
  const Geo g = geo_of(d);
  const F64Layout lo = f64_layout(d);
  if (saved && saved_bytes < lo.saved_bytes) return fail(SIREN_ENOSPACE, "fp64 forward: saved buffer too small");
  if (!workspace || workspace_bytes < lo.ws_bytes) return fail(SIREN_ENOSPACE, "fp64 forward: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const double* h = x;
  for (int l = 0; l < g.L; ++l) {
    const int K = d->dims[l], N = d->dims[l + 1];
    const bool last = l + 1 == g.L, sine = !last || !d->outermost_linear;
    F64Args a;
    memset(&a, 0, sizeof(a));
    a.A = h;
    a.B = (const double*)d->weight[l];
    a.bias = (const double*)d->bias[l];
    a.C = last ? y : (double*)(ws + lo.h_off[l & 1]);
    a.Zs = (saved && sine) ? (double*)((char*)saved + lo.z_off[l]) : nullptr;
    a.M = g.rows;
    a.N = N;
    a.K = K;
    a.lda = K;
    a.ldb = K;
    a.ldc = N;
    a.a_bs = g.rows * K;
    a.b_bs = d->weights_batched ? (int64_t)N * K : 0;
    a.bias_bs = d->weights_batched ? N : 0;
    a.c_bs = a.zs_bs = g.rows * N;
    a.nb = (int)g.nb;
    a.w0 = d->w0;
    rc = sine ? f64_launch<0, 0, F64_FWD_SINE>(a, g.nb, st) : f64_launch<0, 0, F64_FWD_LIN>(a, g.nb, st);
    if (rc) return rc;
    h = a.C;
  }
  return SIREN_OK;
}

int siren_mlp64_backward(const siren_mlp_desc* d, const double* x, const double* dy, const void* saved,
                         int64_t saved_bytes, void* workspace, int64_t workspace_bytes, double* const* dW,
                         double* const* db, double* dx, void* stream) {
  int rc = f64_check(d);
  if (rc) return rc;
  if (!x || !dy || !saved || !dW || !db) return fail(SIREN_EINVAL, "fp64 backward: null argument");
  const Geo g = geo_of(d);
  const F64Layout lo = f64_layout(d);
  if (saved_bytes < lo.saved_bytes) return fail(SIREN_ENOSPACE, "fp64 backward: saved buffer too small");
  if (!workspace || workspace_bytes < lo.ws_bytes) return fail(SIREN_ENOSPACE, "fp64 backward: workspace too small");
  for (int l = 0; l < g.L; ++l)
    if (!dW[l] || !db[l]) return fail(SIREN_EINVAL, "fp64 backward: layer %d null dW / db", l);
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  const char* sv = (const char*)saved;
  double* part = (double*)(ws + lo.part_off);
  // dZ of the output layer
  const double* dz = dy;
  if (!d->outermost_linear) {
    const int64_t n = g.total * d->dims[g.L];
    double* t = (double*)(ws + lo.dz_off[0]);
    hipLaunchKernelGGL(f64_top_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, dy,
                       (const double*)(sv + lo.z_off[g.L - 1]), t, n, (double)d->w0);
    if ((rc = check_launch("f64_top"))) return rc;
    dz = t;
  }
  for (int l = g.L - 1; l >= 0; --l) {
    const int M = d->dims[l + 1], N = d->dims[l];
    // [dW | db] = dZ_l^T [H_l | 1], H_l = sin(w0 Z_{l-1}) (x for l = 0)
    int64_t ns, per;
    f64_split(g, M, N, ns, per);
    F64Args w;
    memset(&w, 0, sizeof(w));
    w.A = dz;
    w.B = l == 0 ? x : (const double*)(sv + lo.z_off[l - 1]);
    w.Zp = l == 0 ? nullptr : w.B;
    w.C = part;
    w.M = M;
    w.N = N;
    w.K = g.rows;
    w.lda = M;
    w.ldb = N;
    w.ldc = N + 1;
    w.a_bs = g.rows * M;
    w.b_bs = g.rows * N;
    w.c_bs = (int64_t)M * (N + 1);
    w.k_per_split = per;
    w.nb = (int)g.nb;
    w.w0 = d->w0;
    if ((rc = f64_launch<1, 1, F64_DW>(w, ns * g.nb, st))) return rc;
    const int64_t nred = g.nb * (int64_t)M * (N + 1);
    hipLaunchKernelGGL(f64_reduce_kernel, dim3((unsigned)cdiv(nred, 256)), dim3(256), 0, st, (const double*)part,
                       dW[l], db[l], (int64_t)M, (int64_t)N, (int)g.nb, (int)ns);
    if ((rc = check_launch("f64_reduce"))) return rc;
    if (l == 0 && !dx) break;
    // dH_l = dZ_l W_l; dZ_{l-1} = dH_l w0 cos(w0 Z_{l-1}) (dx for l = 0)
    F64Args h;
    memset(&h, 0, sizeof(h));
    h.A = dz;
    h.B = (const double*)d->weight[l];
    h.M = g.rows;
    h.N = N;
    h.K = M;
    h.lda = M;
    h.ldb = N;
    h.ldc = N;
    h.a_bs = g.rows * M;
    h.b_bs = d->weights_batched ? (int64_t)M * N : 0;
    h.c_bs = h.zs_bs = g.rows * N;
    h.nb = (int)g.nb;
    h.w0 = d->w0;
    if (l == 0) {
      h.C = dx;
      if ((rc = f64_launch<0, 1, F64_DX>(h, g.nb, st))) return rc;
    } else {
      h.Zp = (const double*)(sv + lo.z_off[l - 1]);
      double* out = (double*)(ws + lo.dz_off[(dz == (const double*)(ws + lo.dz_off[0])) ? 1 : 0]);
      h.C = out;
      if ((rc = f64_launch<0, 1, F64_DH>(h, g.nb, st))) return rc;
      dz = out;
    }
  }
  return SIREN_OK;
}

int siren_mlp_check(const siren_mlp_desc* d) {
  if (!d) return fail(SIREN_EINVAL, "null descriptor");
  const int L = d->num_layers;
  if (L < 2 || L > SIREN_MAX_LAYERS)
    return fail(SIREN_EINVAL, "num_layers=%d outside [2, %d]", L, SIREN_MAX_LAYERS);
  if (d->prec != SIREN_PREC_F32 && d->prec != SIREN_PREC_BF16)
    return fail(SIREN_EINVAL, "unknown precision %d", d->prec);
  if (d->batch < 1 || d->rows_per_batch < 1)
    return fail(SIREN_EINVAL, "empty input (batch=%lld rows=%lld)", (long long)d->batch,
                (long long)d->rows_per_batch);
  if (d->batch > 65535) return fail(SIREN_EINVAL, "batch %lld > 65535", (long long)d->batch);
  const int kmax = 512;  // MFMA K bound of the GEMM kernels (fp32: two register chunks of 256)
  if (d->dims[0] < 1 || (wide_input(d) && first_kp(d) > kmax))
    return fail(SIREN_EINVAL, "in_features=%d unsupported (1..%d)", d->dims[0], kmax);
  if (d->dims[L] < 1 || d->dims[L] > 8)
    return fail(SIREN_EINVAL, "out_features=%d unsupported (1..8)", d->dims[L]);
  const int hmax = 512;
  for (int l = 1; l < L; ++l)
    if (d->dims[l] < 32 || d->dims[l] % 32 != 0 || d->dims[l] > hmax)
      return fail(SIREN_EINVAL, "hidden width dims[%d]=%d must be a multiple of 32 in [32, %d]",
                  l, d->dims[l], hmax);
  if (d->dims[0] > 4 && d->dims[1] > 512)
    return fail(SIREN_EINVAL, "in_features > 4 needs first hidden width <= 512");
  if ((int64_t)d->batch * d->rows_per_batch * (d->dims[1] / 8) >= (int64_t)1 << 31)
    return fail(SIREN_EINVAL, "too many rows for one call");
  for (int l = 0; l < L; ++l)
    if (!d->weight[l] || !d->bias[l]) return fail(SIREN_EINVAL, "layer %d: null weight/bias", l);
  for (int l = 1; l + 1 < L; ++l)
    if (!aligned16(d->weight[l])) return fail(SIREN_EINVAL, "layer %d weight not 16-B aligned", l);
  if (d->ff_B) {
    if (d->ff_in < 1 || d->ff_in > 4 || d->dims[0] % 2 || d->ff_in * (d->dims[0] / 2) > 32)
      return fail(SIREN_EINVAL, "fourier input: ff_in=%d raw coordinates (1..4) for %d features (even)", d->ff_in,
                  d->dims[0]);
    if (d->prec != SIREN_PREC_BF16 || !g_fused_forward || !g_fwd_reg || !fused_shape(d) || !fused_wide(d) || L < 3 ||
        d->dims[1] != 256)
      return fail(SIREN_EINVAL, "fourier input: needs the bf16 register-resident forward's wide first layer "
                                "(6..16 features, hidden 256)");
  }
  return SIREN_OK;
}

int64_t siren_mlp_saved_bytes(const siren_mlp_desc* d) {
  if (siren_mlp_check(d)) return -1;
  return layout_of(d).saved_bytes;
}

int64_t siren_mlp_workspace_bytes(const siren_mlp_desc* d) {
  if (siren_mlp_check(d)) return -1;
  return layout_of(d).ws_bytes;
}

int siren_mlp_forward(const siren_mlp_desc* d, const float* x, float* y, void* saved,
                      int64_t saved_bytes, void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = siren_mlp_check(d);
  if (rc) return rc;
  const Layout lo = layout_of(d);
  if (saved && saved_bytes < lo.saved_bytes)
    return fail(SIREN_ENOSPACE, "saved buffer %lld < %lld bytes", (long long)saved_bytes,
                (long long)lo.saved_bytes);
  if (workspace_bytes < lo.ws_bytes || !workspace)
    return fail(SIREN_ENOSPACE, "workspace %lld < %lld bytes", (long long)workspace_bytes,
                (long long)lo.ws_bytes);
  if (!x || !y) return fail(SIREN_EINVAL, "null x or y");
  hipStream_t st = (hipStream_t)stream;
  g_err.clear();
  if (d->prec == SIREN_PREC_BF16)
    return forward_impl<kPrecBF16>(d, x, y, (char*)saved, (char*)workspace, st);
  return forward_impl<kPrecF32>(d, x, y, (char*)saved, (char*)workspace, st);
}

int siren_mlp_backward(const siren_mlp_desc* d, const float* x, const float* dy, const void* saved,
                       int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                       float* const* dweight, float* const* dbias, float* dx, void* stream) {
  int rc = siren_mlp_check(d);
  if (rc) return rc;
  const Layout lo = layout_of(d);
  if (!saved || saved_bytes < lo.saved_bytes)
    return fail(SIREN_ENOSPACE, "saved buffer %lld < %lld bytes", (long long)saved_bytes,
                (long long)lo.saved_bytes);
  if (workspace_bytes < lo.ws_bytes || !workspace)
    return fail(SIREN_ENOSPACE, "workspace %lld < %lld bytes", (long long)workspace_bytes,
                (long long)lo.ws_bytes);
  if (!x || !dy || !dweight || !dbias) return fail(SIREN_EINVAL, "null argument");
  for (int l = 0; l < d->num_layers; ++l)
    if (!dweight[l] || !dbias[l]) return fail(SIREN_EINVAL, "layer %d: null gradient output", l);
  if (d->ff_B && dx) return fail(SIREN_EINVAL, "fourier input: no input gradient (dx must be NULL)");
  hipStream_t st = (hipStream_t)stream;
  g_err.clear();
  if (d->prec == SIREN_PREC_BF16)
    return backward_impl<kPrecBF16>(d, x, dy, (const char*)saved, (char*)workspace, dweight, dbias,
                                    dx, st);
  return backward_impl<kPrecF32>(d, x, dy, (const char*)saved, (char*)workspace, dweight, dbias, dx,
                                 st);
}

}  // extern "C"
namespace {
// Which forward carries a fused image loss: the bf16 register-resident forward (its output-layer
// epilogue, fused_fwd_reg_kernel<.., LOSS>) or the per-layer path's output kernel (last_fwd_kernel
// <.., LOSS>: fp32 mode, and bf16 shapes that are not the fused forward's); 0 = none applies.
int loss_path(const siren_mlp_desc* d) {
  const int O = d->dims[d->num_layers];
  if (!d->outermost_linear) return 0;
  const bool fused = d->prec == SIREN_PREC_BF16 && g_fused_forward && fused_shape(d);
  if (fused)
    return (g_fwd_reg && d->num_layers >= 3 && !g_freg_magic && (fused_wide(d) || O == 1)) ? 1 : 0;
  if (d->ff_B) return 0;  // (a Fourier-feature input is a register-forward form)
  return O <= 8 ? 2 : 0;
}

int loss_path_fail(const siren_mlp_desc* d) {
  if (!d->outermost_linear) return fail(SIREN_EINVAL, "fused loss: needs outermost_linear");
  if (g_freg_magic) return fail(SIREN_EINVAL, "fused loss: not with option freg_magic");
  return fail(SIREN_EINVAL, "fused loss: shape not supported (bf16 fused shapes: the register forward's "
                            "forms with 3+ layers and 1 output for 1..4 inputs; per-layer path: <= 8 outputs)");
}

// conv_fwd_k5_kernel in the stage-fill form of option conv_dma
template <int EPI>
void launch_conv_fwd_k5(dim3 grid, hipStream_t st, const ConvFArgs& a) {
  if (g_conv_dma == 2) hipLaunchKernelGGL((conv_fwd_k5_kernel<EPI, 2>), grid, dim3(512), 0, st, a);
  else if (g_conv_dma == 1) hipLaunchKernelGGL((conv_fwd_k5_kernel<EPI, 1>), grid, dim3(512), 0, st, a);
  else hipLaunchKernelGGL((conv_fwd_k5_kernel<EPI, 0>), grid, dim3(512), 0, st, a);
}
}  // namespace
extern "C" {

int siren_mlp_loss_check(const siren_mlp_desc* d, const siren_loss_desc* l) {
  int rc = siren_mlp_check(d);
  if (rc) return rc;
  if (!l) return fail(SIREN_EINVAL, "null loss descriptor");
  const int path = loss_path(d);
  if (!path) return loss_path_fail(d);
  if (!l->target || !l->dy || !l->loss || !l->loss_workspace)
    return fail(SIREN_EINVAL, "fused loss: null target / dy / loss / workspace");
  if (l->loss_workspace_bytes < siren_sse_workspace_bytes())
    return fail(SIREN_ENOSPACE, "fused loss: workspace %lld < %lld bytes", (long long)l->loss_workspace_bytes,
                (long long)siren_sse_workspace_bytes());
  if ((l->k0 == nullptr) != (l->mask == nullptr) || (l->k0 == nullptr) != (l->y_dc == nullptr))
    return fail(SIREN_EINVAL, "fused loss: k0, mask and y_dc are given together or not at all");
  if (l->hf && l->hf_len != d->rows_per_batch)
    return fail(SIREN_EINVAL, "fused loss: hf has %lld entries for %lld rows per weight set", (long long)l->hf_len,
                (long long)d->rows_per_batch);
  const Geo g = geo_of(d);
  const int64_t wgs = path == 1 ? std::min<int64_t>(cdiv(g.rows, FREG_WG_ROWS), std::max<int64_t>(1, 256 / g.nb)) * g.nb
                                : g.nb;  // (per-layer path: at most SSE_MAX_BLOCKS / nb workgroups per weight set)
  if (wgs > SSE_MAX_BLOCKS) return fail(SIREN_EINVAL, "fused loss: %lld workgroups > %d", (long long)wgs, SSE_MAX_BLOCKS);
  return SIREN_OK;
}

int siren_mlp_forward_loss(const siren_mlp_desc* d, const siren_loss_desc* l, const float* x, float* y, void* saved,
                           int64_t saved_bytes, void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = siren_mlp_loss_check(d, l);
  if (rc) return rc;
  const Layout lo = layout_of(d);
  if (saved && saved_bytes < lo.saved_bytes)
    return fail(SIREN_ENOSPACE, "saved buffer %lld < %lld bytes", (long long)saved_bytes, (long long)lo.saved_bytes);
  if (workspace_bytes < lo.ws_bytes || !workspace)
    return fail(SIREN_ENOSPACE, "workspace %lld < %lld bytes", (long long)workspace_bytes, (long long)lo.ws_bytes);
  if (!x || !y) return fail(SIREN_EINVAL, "null x or y");
  g_err.clear();
  const Geo g = geo_of(d);
  if (loss_path(d) == 1) {
    char* wbuf = saved ? (char*)saved : (char*)workspace;
    return fused_forward_reg(d, g, lo, x, y, (char*)saved, wbuf, (hipStream_t)stream, l);
  }
  if (d->prec == SIREN_PREC_BF16)
    return forward_impl<kPrecBF16>(d, x, y, (char*)saved, (char*)workspace, (hipStream_t)stream, l);
  return forward_impl<kPrecF32>(d, x, y, (char*)saved, (char*)workspace, (hipStream_t)stream, l);
}

int siren_mlp_backward_ex(const siren_mlp_desc* d, const float* x, const float* dy, const float* dy_scale,
                          const void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                          float* const* dweight, float* const* dbias, float* dx, void* stream) {
  int rc = siren_mlp_check(d);
  if (rc) return rc;
  const Layout lo = layout_of(d);
  if (!saved || saved_bytes < lo.saved_bytes)
    return fail(SIREN_ENOSPACE, "saved buffer %lld < %lld bytes", (long long)saved_bytes, (long long)lo.saved_bytes);
  if (workspace_bytes < lo.ws_bytes || !workspace)
    return fail(SIREN_ENOSPACE, "workspace %lld < %lld bytes", (long long)workspace_bytes, (long long)lo.ws_bytes);
  if (!x || !dy || !dweight || !dbias) return fail(SIREN_EINVAL, "null argument");
  for (int l = 0; l < d->num_layers; ++l)
    if (!dweight[l] || !dbias[l]) return fail(SIREN_EINVAL, "layer %d: null gradient output", l);
  if (d->ff_B && dx) return fail(SIREN_EINVAL, "fourier input: no input gradient (dx must be NULL)");
  hipStream_t st = (hipStream_t)stream;
  g_err.clear();
  if (d->prec == SIREN_PREC_BF16)
    return backward_impl<kPrecBF16>(d, x, dy, (const char*)saved, (char*)workspace, dweight, dbias, dx, st, dy_scale);
  return backward_impl<kPrecF32>(d, x, dy, (const char*)saved, (char*)workspace, dweight, dbias, dx, st, dy_scale);
}

int64_t siren_jvp_saved_bytes(const siren_mlp_desc* d, int order) {
  if (jvp_check(d, order)) return -1;
  return jlayout_of(d, order).saved_bytes;
}

int64_t siren_jvp_workspace_bytes(const siren_mlp_desc* d, int order) {
  if (jvp_check(d, order)) return -1;
  const JLayout jl = jlayout_of(d, order);
  return jl.ws_bytes + jl.saved_bytes;  // room for the per-layer tensors when no saved buffer is given
}

namespace {
// the plain forward's saved buffer as the primal stream of a jvp (fp32 mode: its phases are the
// jvp's fp32 phases; siren_mlp_forward's layout)
int jvp_primal_check(const siren_mlp_desc* d, const void* primal, int64_t primal_bytes) {
  if (!primal) return SIREN_OK;
  if (d->prec != SIREN_PREC_F32) return fail(SIREN_EINVAL, "jvp primal: fp32 mode only");
  if (!d->outermost_linear) return fail(SIREN_EINVAL, "jvp primal: needs outermost_linear");
  const Layout lo = layout_of(d);
  if (primal_bytes < lo.saved_bytes)
    return fail(SIREN_ENOSPACE, "jvp primal: saved buffer %lld < %lld bytes", (long long)primal_bytes,
                (long long)lo.saved_bytes);
  for (int l = 0; l + 1 < d->num_layers; ++l)
    if (lo.saved_off[l] < 0) return fail(SIREN_EINVAL, "jvp primal: layer %d phases not kept", l);
  return SIREN_OK;
}
}  // namespace

int siren_jvp_forward_ex(const siren_mlp_desc* d, int order, const float* x, float* grad, float* lap,
                         void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                         const void* primal, int64_t primal_bytes, void* stream) {
  int rc = jvp_check(d, order);
  if (rc) return rc;
  if ((rc = jvp_primal_check(d, primal, primal_bytes))) return rc;
  const JLayout jl = jlayout_of(d, order);
  if (saved && saved_bytes < jl.saved_bytes)
    return fail(SIREN_ENOSPACE, "saved buffer %lld < %lld bytes", (long long)saved_bytes, (long long)jl.saved_bytes);
  const int64_t need = saved ? jl.ws_bytes : jl.ws_bytes + jl.saved_bytes;
  if (!workspace || workspace_bytes < need)
    return fail(SIREN_ENOSPACE, "workspace %lld < %lld bytes", (long long)workspace_bytes, (long long)need);
  if (!x || !grad || (order == SIREN_JVP_LAPLACE && !lap)) return fail(SIREN_EINVAL, "null x/grad/lap");
  g_err.clear();
  hipStream_t st = (hipStream_t)stream;
  if (d->prec == SIREN_PREC_BF16)
    return jvp_forward_impl<kPrecBF16>(d, order, x, grad, lap, (char*)saved, (char*)workspace, st);
  return jvp_forward_impl<kPrecF32>(d, order, x, grad, lap, (char*)saved, (char*)workspace, st, (const char*)primal);
}

int siren_jvp_forward(const siren_mlp_desc* d, int order, const float* x, float* grad, float* lap,
                      void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                      void* stream) {
  return siren_jvp_forward_ex(d, order, x, grad, lap, saved, saved_bytes, workspace, workspace_bytes, nullptr, 0,
                              stream);
}

int siren_jvp_backward_ex(const siren_mlp_desc* d, int order, const float* x, const float* dgrad,
                          const void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                          float* const* dweight, float* const* dbias, float* dx, const void* primal,
                          int64_t primal_bytes, void* stream) {
  int rc = jvp_check(d, order);
  if (rc) return rc;
  if ((rc = jvp_primal_check(d, primal, primal_bytes))) return rc;
  const JLayout jl = jlayout_of(d, order);
  if (!saved || saved_bytes < jl.saved_bytes)
    return fail(SIREN_ENOSPACE, "saved buffer %lld < %lld bytes", (long long)saved_bytes, (long long)jl.saved_bytes);
  if (!workspace || workspace_bytes < jl.ws_bytes)
    return fail(SIREN_ENOSPACE, "workspace %lld < %lld bytes", (long long)workspace_bytes, (long long)jl.ws_bytes);
  if (!x || !dgrad || !dweight || !dbias) return fail(SIREN_EINVAL, "null argument");
  for (int l = 0; l < d->num_layers; ++l)
    if (!dweight[l] || !dbias[l]) return fail(SIREN_EINVAL, "layer %d: null gradient output", l);
  g_err.clear();
  hipStream_t st = (hipStream_t)stream;
  if (d->prec == SIREN_PREC_BF16)
    return jvp_backward_impl<kPrecBF16>(d, order, x, dgrad, (const char*)saved, (char*)workspace, dweight, dbias, dx, st);
  return jvp_backward_impl<kPrecF32>(d, order, x, dgrad, (const char*)saved, (char*)workspace, dweight, dbias, dx, st,
                                     (const char*)primal);
}

int siren_jvp_backward(const siren_mlp_desc* d, int order, const float* x, const float* dgrad,
                       const void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                       float* const* dweight, float* const* dbias, float* dx, void* stream) {
  return siren_jvp_backward_ex(d, order, x, dgrad, saved, saved_bytes, workspace, workspace_bytes, dweight, dbias, dx,
                               nullptr, 0, stream);
}

const char* siren_last_error(void) { return g_err.c_str(); }

int siren_timing_enable(int kernel_class, int max_launches) {
  siren_timing_disable();
  if (kernel_class <= 0 || max_launches <= 0) return SIREN_OK;
  g_timing.ev = new hipEvent_t[2 * (size_t)max_launches];
  for (int i = 0; i < 2 * max_launches; ++i) {
    if (hipEventCreate(&g_timing.ev[i]) != hipSuccess) {
      for (int k = 0; k < i; ++k) (void)hipEventDestroy(g_timing.ev[k]);
      delete[] g_timing.ev;
      g_timing = Timing();
      return fail(SIREN_ELAUNCH, "hipEventCreate failed");
    }
  }
  g_timing.cls = kernel_class;
  g_timing.cap = max_launches;
  g_timing.used = 0;
  return SIREN_OK;
}

int siren_timing_collect(double* total_ms, int64_t* launches) {
  double tot = 0.0;
  for (int i = 0; i < g_timing.used; ++i) {
    if (hipEventSynchronize(g_timing.ev[2 * i + 1]) != hipSuccess)
      return fail(SIREN_ELAUNCH, "hipEventSynchronize failed");
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, g_timing.ev[2 * i], g_timing.ev[2 * i + 1]) != hipSuccess)
      return fail(SIREN_ELAUNCH, "hipEventElapsedTime failed");
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = g_timing.used;
  return SIREN_OK;
}

void siren_timing_disable(void) {
  if (g_timing.ev) {
    for (int i = 0; i < 2 * g_timing.cap; ++i) (void)hipEventDestroy(g_timing.ev[i]);
    delete[] g_timing.ev;
  }
  g_timing = Timing();
}

int siren_adam_scalars_table(double* t, const float* table, int64_t n, float* out, void* stream) {
  if (!t || !table || n < 1 || !out) return fail(SIREN_EINVAL, "adam_scalars_table: null pointer or empty table");
  hipLaunchKernelGGL(adam_scalars_table_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, t, table, n, out);
  return check_launch("adam_scalars_table");
}

int siren_adam_scalars(double* t, double lr, double beta1, double beta2, float* out, void* stream) {
  if (!t || !out) return fail(SIREN_EINVAL, "adam_scalars: null pointer");
  hipLaunchKernelGGL(adam_scalars_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, t, lr, beta1, beta2, out);
  return check_launch("adam_scalars");
}

int64_t siren_sse_workspace_bytes(void) { return (int64_t)SSE_MAX_BLOCKS * 4 + 256; }

// ---------------------------------------------------------------- conv encoder epilogues
int64_t siren_enc_workspace_bytes(void) { return ENC_WS_FLOATS * 4 + 256; }

namespace {
// shared checks; fills the plane geometry and the block split of a [P, C] pass
int enc_setup(EncArgs& a, int64_t P, int C, void* ws, int64_t ws_bytes, bool need_ws, int64_t rows_per_block_min,
              const char* what) {
  memset(&a, 0, sizeof(a));
  if (P < 0 || C < 8 || C > ENC_MAXC || (C & (C - 1)) != 0)
    return fail(SIREN_EINVAL, "%s: C = %d must be a power of two in [8, %d] (P = %lld)", what, C, ENC_MAXC, (long long)P);
  if (need_ws && (!ws || ws_bytes < siren_enc_workspace_bytes()))
    return fail(SIREN_ENOSPACE, "%s: workspace %lld < %lld bytes", what, (long long)ws_bytes,
                (long long)siren_enc_workspace_bytes());
  a.P = P;
  a.C = C;
  a.part = (float*)ws;
  a.ticket = ws ? (unsigned*)((char*)ws + ENC_WS_FLOATS * 4) : nullptr;
  const int ppi = 256 / (C / 8);
  int64_t nblk = std::min<int64_t>(ENC_MAX_BLOCKS, std::max<int64_t>(1, cdiv(P, rows_per_block_min)));
  a.chunk = align_up(cdiv(std::max<int64_t>(P, 1), nblk), ppi);
  return SIREN_OK;
}
}  // namespace

int64_t siren_conv_wrw_workspace_bytes(int N, int H, int W) {
  const int64_t rows = (int64_t)N * H;
  const int64_t nsplit = std::max<int64_t>(1, std::min<int64_t>(25, rows));
  return nsplit * CW_SLAB * 4;
}

int siren_conv_wrw_k5(const void* x, const void* dy, int N, int H, int W, int C, float* dw, void* ws, int64_t ws_bytes,
                      void* stream) {
  if (C != CW_C || N < 1 || H < 1 || W < CW_PX || W % CW_PX != 0)
    return fail(SIREN_EINVAL, "conv_wrw_k5: needs C = %d and W a multiple of %d (C = %d, N = %d, H = %d, W = %d)", CW_C,
                CW_PX, C, N, H, W);
  if (!x || !dy || !dw) return fail(SIREN_EINVAL, "conv_wrw_k5: null pointer");
  const int64_t rows = (int64_t)N * H;
  const int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(25, rows));
  if (!ws || ws_bytes < (int64_t)nsplit * CW_SLAB * 4)
    return fail(SIREN_ENOSPACE, "conv_wrw_k5: workspace %lld < %lld bytes", (long long)ws_bytes,
                (long long)nsplit * CW_SLAB * 4);
  ConvWArgs a;
  memset(&a, 0, sizeof(a));
  a.x = (const bf16*)x;
  a.dy = (const bf16*)dy;
  a.part = (float*)ws;
  a.dw = dw;
  a.N = N;
  a.H = H;
  a.W = W;
  a.nsplit = nsplit;
  a.rows_per_split = cdiv(rows, nsplit);
  hipStream_t st = (hipStream_t)stream;
  const dim3 wg((unsigned)nsplit, CW_K, 2);
  if (g_wrw_dma >= 2 && W % (2 * CW_PX) == 0) hipLaunchKernelGGL((conv_wrw_k5_kernel<true, 2 * CW_PX>), wg, dim3(512), 0, st, a);
  else if (g_wrw_dma) hipLaunchKernelGGL((conv_wrw_k5_kernel<true>), wg, dim3(512), 0, st, a);
  else hipLaunchKernelGGL((conv_wrw_k5_kernel<false>), wg, dim3(512), 0, st, a);
  int rc = check_launch("conv_wrw_k5");
  if (rc) return rc;
  hipLaunchKernelGGL(conv_wrw_reduce_kernel, dim3((unsigned)cdiv(CW_SLAB, 256)), dim3(256), 0, st, a);
  return check_launch("conv_wrw_reduce");
}

int siren_conv_fwd_k5(const void* x, const void* w, const void* bias, int relu, void* y, int N, int H, int W, int C,
                      void* stream) {
  if (C != CW_C || W != CF_W || N < 1 || H < 2 || H % 2 != 0)
    return fail(SIREN_EINVAL, "conv_fwd_k5: needs C = %d, W = %d and H even (C = %d, N = %d, H = %d, W = %d)", CW_C,
                CF_W, C, N, H, W);
  if (!x || !w || !y) return fail(SIREN_EINVAL, "conv_fwd_k5: null pointer");
  ConvFArgs a;
  memset(&a, 0, sizeof(a));
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = (const bf16*)bias;
  a.y = (bf16*)y;
  a.N = N;
  a.H = H;
  a.relu = relu ? 1 : 0;
  launch_conv_fwd_k5<EPI_PLAIN>(dim3((unsigned)(N * (H / 2))), (hipStream_t)stream, a);
  return check_launch("conv_fwd_k5");
}

int siren_conv_fwd_k5_res(const void* x, const void* w, const void* cb, const void* t, void* a_out, void* out, int N,
                          int H, int W, int C, void* stream) {
  if (C != CW_C || W != CF_W || N < 1 || H < 2 || H % 2 != 0)
    return fail(SIREN_EINVAL, "conv_fwd_k5_res: needs C = %d, W = %d and H even (C = %d, N = %d, H = %d, W = %d)", CW_C,
                CF_W, C, N, H, W);
  if (!x || !w || !cb || !t || !a_out || !out) return fail(SIREN_EINVAL, "conv_fwd_k5_res: null pointer");
  ConvFArgs a;
  memset(&a, 0, sizeof(a));
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.y = (bf16*)a_out;
  a.N = N;
  a.H = H;
  a.g2 = (const bf16*)t;
  a.cb = (const bf16*)cb;
  a.y2 = (bf16*)out;
  launch_conv_fwd_k5<EPI_RESFWD>(dim3((unsigned)(N * (H / 2))), (hipStream_t)stream, a);
  return check_launch("conv_fwd_k5_res");
}

int siren_conv_dgrad_k5_fused(int mode, const void* dy, const void* wf, const void* g2, const void* m, const void* pa,
                              const void* cb, void* out, void* out2, float* db, int N, int H, int W, int C, void* ws,
                              int64_t ws_bytes, void* stream) {
  if (C != CW_C || W != CF_W || N < 1 || H < 2 || H % 2 != 0)
    return fail(SIREN_EINVAL, "conv_dgrad_k5_fused: needs C = %d, W = %d and H even (C = %d, N = %d, H = %d, W = %d)",
                CW_C, CF_W, C, N, H, W);
  if (mode != 1 && mode != 2) return fail(SIREN_EINVAL, "conv_dgrad_k5_fused: mode %d (1 relu, 2 residual tail)", mode);
  if (!dy || !wf || !m || !out || !db || (mode == 2 && (!g2 || !pa || !cb || !out2)))
    return fail(SIREN_EINVAL, "conv_dgrad_k5_fused: null pointer");
  const int64_t nblk = (int64_t)N * (H / 2);
  if (!ws || ws_bytes < nblk * CW_C * 4)
    return fail(SIREN_ENOSPACE, "conv_dgrad_k5_fused: workspace %lld < %lld bytes", (long long)ws_bytes,
                (long long)(nblk * CW_C * 4));
  ConvFArgs a;
  memset(&a, 0, sizeof(a));
  a.x = (const bf16*)dy;
  a.w = (const bf16*)wf;
  a.y = (bf16*)out;
  a.N = N;
  a.H = H;
  a.g2 = (const bf16*)g2;
  a.m = (const bf16*)m;
  a.pa = (const bf16*)pa;
  a.cb = (const bf16*)cb;
  a.y2 = (bf16*)out2;
  a.part = (float*)ws;
  hipStream_t st = (hipStream_t)stream;
  if (mode == 1) {
    launch_conv_fwd_k5<EPI_RELU>(dim3((unsigned)nblk), st, a);
  } else {
    launch_conv_fwd_k5<EPI_RES>(dim3((unsigned)nblk), st, a);
  }
  int rc = check_launch("conv_dgrad_k5_fused");
  if (rc) return rc;
  hipLaunchKernelGGL(conv_chan_reduce_kernel, dim3(CW_C), dim3(256), 0, st, (const float*)ws, (int)nblk, db);
  return check_launch("conv_chan_reduce");
}

}  // extern "C"
namespace {
// Native shapes of the generic encoder convolutions (siren_conv.hip conv_*_gen_kernel).
int conv_shape_check(int kind, int N, int H, int W, int CI, int CO, int KS) {
  if (N < 1 || H < 1) return fail(SIREN_EINVAL, "conv: empty input");
  if (KS != 3 && KS != 5 && KS != 7) return fail(SIREN_EINVAL, "conv: filter size %d not native (3, 5, 7)", KS);
  if (CI == 2) {  // conv_theta (conv_t_fwd_kernel / conv_t_wrw_kernel)
    if (CO < 32 || CO > 128 || CO % 32 != 0) return fail(SIREN_EINVAL, "conv (2 channels): %d output channels (32, 64, 96, 128)", CO);
    if (kind == 0 && W != CT_W) return fail(SIREN_EINVAL, "conv fwd (2 channels): needs W = %d (W = %d)", CT_W, W);
    if (kind != 0 && (W < CT_PX || W % CT_PX != 0)) return fail(SIREN_EINVAL, "conv wrw (2 channels): W = %d not a multiple of %d", W, CT_PX);
    return SIREN_OK;
  }
  if (CI != 64 && CI != 128) return fail(SIREN_EINVAL, "conv: %d input channels not native (2, 64, 128)", CI);
  if (kind == 0) {
    if (W != CF_W || H % 2 != 0) return fail(SIREN_EINVAL, "conv fwd: needs W = %d and H even (H = %d, W = %d)", CF_W, H, W);
    if (CO < 64 || CO % 64 != 0) return fail(SIREN_EINVAL, "conv fwd: %d output channels (a multiple of 64)", CO);
  } else {
    if (W < CW_PX || W % CW_PX != 0) return fail(SIREN_EINVAL, "conv wrw: W = %d not a multiple of %d", W, CW_PX);
    const int cow = CI == 64 ? 128 : 64;
    if (CO % cow != 0) return fail(SIREN_EINVAL, "conv wrw: %d output channels (a multiple of %d)", CO, cow);
  }
  return SIREN_OK;
}
// conv_theta weight gradient: splits of 64-pixel chunks (one workgroup each, ~3 per CU) and the
// partial slab of one split ([CO][32 NNT] floats)
int conv_t_nsplit(int N, int H, int W) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(768, (int64_t)N * H * (W / CT_PX)));
}
int64_t conv_t_slab(int CO, int KS) { return (int64_t)CO * 32 * ((KS * 16 + 31) / 32); }
int conv_wrw_nsplit(int N, int H, int CI, int CO, int KS) {
  const int64_t rows = (int64_t)N * H;
  const int64_t blocks = (int64_t)KS * (CO / (CI == 64 ? 128 : 64));
  return (int)std::max<int64_t>(1, std::min<int64_t>(rows, std::max<int64_t>(1, 256 / blocks)));
}
}  // namespace
extern "C" {

int siren_conv_check(int kind, int N, int H, int W, int CI, int CO, int KS) {
  return conv_shape_check(kind, N, H, W, CI, CO, KS);
}

int siren_conv_fwd(const void* x, const void* w, const void* bias, int relu, void* y, int N, int H, int W, int CI,
                   int CO, int KS, void* stream) {
  int rc = conv_shape_check(0, N, H, W, CI, CO, KS);
  if (rc) return rc;
  if (!x || !w || !y) return fail(SIREN_EINVAL, "conv fwd: null pointer");
  ConvGArgs a;
  memset(&a, 0, sizeof(a));
  a.x = (const bf16*)x;
  a.w = (const bf16*)w;
  a.bias = (const bf16*)bias;
  a.y = (bf16*)y;
  a.N = N;
  a.H = H;
  a.W = W;
  a.CO = CO;
  a.relu = relu ? 1 : 0;
  hipStream_t st = (hipStream_t)stream;
  if (CI == 2) {
    ConvTArgs t;
    memset(&t, 0, sizeof(t));
    t.x = a.x;
    t.w = a.w;
    t.bias = a.bias;
    t.y = a.y;
    t.N = N;
    t.H = H;
    t.W = W;
    t.CO = CO;
    t.relu = a.relu;
    t.rows_per_block = CT_RPB;
    const dim3 tg((unsigned)cdiv((int64_t)N * H, CT_RPB));
#define SIREN_CT(K)                                                                              \
  switch (CO / 32) {                                                                             \
    case 1: hipLaunchKernelGGL((conv_t_fwd_kernel<K, 1>), tg, dim3(256), 0, st, t); break;      \
    case 2: hipLaunchKernelGGL((conv_t_fwd_kernel<K, 2>), tg, dim3(256), 0, st, t); break;      \
    case 3: hipLaunchKernelGGL((conv_t_fwd_kernel<K, 3>), tg, dim3(256), 0, st, t); break;      \
    default: hipLaunchKernelGGL((conv_t_fwd_kernel<K, 4>), tg, dim3(256), 0, st, t); break;     \
  }
    if (KS == 3) { SIREN_CT(3) }
    else if (KS == 5) { SIREN_CT(5) }
    else { SIREN_CT(7) }
#undef SIREN_CT
    return check_launch("conv_t_fwd");
  }
  const bool big = KS <= 5 && CO % 128 == 0;  // 128-channel tiles (the 7x7 stages need 64 to fit in LDS)
  const dim3 grid((unsigned)(N * (H / 2)), (unsigned)(CO / (big ? 128 : 64)));
#define SIREN_CF(K, C, T)                                                                           \
  do {                                                                                              \
    if (g_conv_dma == 2) hipLaunchKernelGGL((conv_fwd_gen_kernel<K, C, T, true>), grid, dim3(512), 0, st, a); \
    else hipLaunchKernelGGL((conv_fwd_gen_kernel<K, C, T, false>), grid, dim3(512), 0, st, a);      \
  } while (0)
  if (KS == 3) {
    if (CI == 64) { if (big) SIREN_CF(3, 64, 128); else SIREN_CF(3, 64, 64); }
    else { if (big) SIREN_CF(3, 128, 128); else SIREN_CF(3, 128, 64); }
  } else if (KS == 5) {
    if (CI == 64) { if (big) SIREN_CF(5, 64, 128); else SIREN_CF(5, 64, 64); }
    else { if (big) SIREN_CF(5, 128, 128); else SIREN_CF(5, 128, 64); }
  } else {
    if (CI == 64) SIREN_CF(7, 64, 64);
    else SIREN_CF(7, 128, 64);
  }
#undef SIREN_CF
  return check_launch("conv_fwd_gen");
}

int64_t siren_conv_wrw_ws_bytes(int N, int H, int W, int CI, int CO, int KS) {
  if (conv_shape_check(1, N, H, W, CI, CO, KS)) return -1;
  if (CI == 2) return (int64_t)conv_t_nsplit(N, H, W) * conv_t_slab(CO, KS) * 4;
  return (int64_t)conv_wrw_nsplit(N, H, CI, CO, KS) * KS * KS * CO * CI * 4;
}

int siren_conv_wrw(const void* x, const void* dy, int N, int H, int W, int CI, int CO, int KS, float* dw, void* ws,
                   int64_t ws_bytes, void* stream) {
  int rc = conv_shape_check(1, N, H, W, CI, CO, KS);
  if (rc) return rc;
  if (!x || !dy || !dw) return fail(SIREN_EINVAL, "conv wrw: null pointer");
  if (CI == 2) {
    const int ns = conv_t_nsplit(N, H, W);
    const int64_t need = (int64_t)ns * conv_t_slab(CO, KS) * 4;
    if (!ws || ws_bytes < need) return fail(SIREN_ENOSPACE, "conv wrw: workspace %lld < %lld bytes", (long long)ws_bytes, (long long)need);
    ConvTArgs t;
    memset(&t, 0, sizeof(t));
    t.x = (const bf16*)x;
    t.dy = (const bf16*)dy;
    t.part = (float*)ws;
    t.dw = dw;
    t.N = N;
    t.H = H;
    t.W = W;
    t.CO = CO;
    t.nsplit = ns;
    t.chunks_per_split = cdiv((int64_t)N * H * (W / CT_PX), ns);
    hipStream_t st = (hipStream_t)stream;
    const dim3 rg((unsigned)cdiv((int64_t)CO * KS * KS * 2, 16));
#define SIREN_CTW(K)                                                                               \
  {                                                                                                \
    switch (CO / 32) {                                                                             \
      case 1: hipLaunchKernelGGL((conv_t_wrw_kernel<K, 1>), dim3(ns), dim3(256), 0, st, t); break; \
      case 2: hipLaunchKernelGGL((conv_t_wrw_kernel<K, 2>), dim3(ns), dim3(256), 0, st, t); break; \
      case 3: hipLaunchKernelGGL((conv_t_wrw_kernel<K, 3>), dim3(ns), dim3(256), 0, st, t); break; \
      default: hipLaunchKernelGGL((conv_t_wrw_kernel<K, 4>), dim3(ns), dim3(256), 0, st, t); break; \
    }                                                                                              \
    if ((rc = check_launch("conv_t_wrw"))) return rc;                                              \
    hipLaunchKernelGGL((conv_t_wrw_reduce_kernel<K>), rg, dim3(256), 0, st, t);                    \
  }
    if (KS == 3) SIREN_CTW(3)
    else if (KS == 5) SIREN_CTW(5)
    else SIREN_CTW(7)
#undef SIREN_CTW
    return check_launch("conv_t_wrw_reduce");
  }
  const int nsplit = conv_wrw_nsplit(N, H, CI, CO, KS);
  const int64_t need = (int64_t)nsplit * KS * KS * CO * CI * 4;
  if (!ws || ws_bytes < need) return fail(SIREN_ENOSPACE, "conv wrw: workspace %lld < %lld bytes", (long long)ws_bytes, (long long)need);
  ConvGArgs a;
  memset(&a, 0, sizeof(a));
  a.x = (const bf16*)x;
  a.dy = (const bf16*)dy;
  a.part = (float*)ws;
  a.dw = dw;
  a.N = N;
  a.H = H;
  a.W = W;
  a.CO = CO;
  a.nsplit = nsplit;
  a.rows_per_split = cdiv((int64_t)N * H, nsplit);
  hipStream_t st = (hipStream_t)stream;
  const int cow = CI == 64 ? 128 : 64;
  const dim3 grid((unsigned)nsplit, (unsigned)KS, (unsigned)(CO / cow));
  const int64_t slab = (int64_t)KS * KS * CO * CI;
  const dim3 rgrid((unsigned)cdiv(slab, 256));
#define SIREN_CW(K, C, B)                                                               \
  {                                                                                      \
    if (g_wrw_dma == 3 && W % 128 == 0)                                                  \
      hipLaunchKernelGGL((conv_wrw_gen_kernel<K, C, B, true>), grid, dim3(512), 0, st, a); \
    else                                                                                 \
      hipLaunchKernelGGL((conv_wrw_gen_kernel<K, C, B>), grid, dim3(512), 0, st, a);      \
    if ((rc = check_launch("conv_wrw_gen"))) return rc;                                  \
    hipLaunchKernelGGL((conv_wrw_gen_reduce_kernel<K, C>), rgrid, dim3(256), 0, st, a);   \
  }
  if (KS == 3) { if (CI == 64) SIREN_CW(3, 64, 4) else SIREN_CW(3, 128, 2) }
  else if (KS == 5) { if (CI == 64) SIREN_CW(5, 64, 4) else SIREN_CW(5, 128, 2) }
  else { if (CI == 64) SIREN_CW(7, 64, 4) else SIREN_CW(7, 128, 2) }
#undef SIREN_CW
  return check_launch("conv_wrw_gen_reduce");
}

int64_t siren_sumsq_workspace_bytes(int64_t total) {
  return 256 + (int64_t)std::max<int64_t>(1, cdiv(total, SUMSQ_CHUNK)) * 4;
}

namespace {
int sumsq_setup(SumsqArgs& a, int n, const float* const* src, const int64_t* numel) {
  if (n < 1 || n > SUMSQ_MAX) return fail(SIREN_EINVAL, "sumsq: %d tensors (1..%d)", n, SUMSQ_MAX);
  if (!src || !numel) return fail(SIREN_EINVAL, "sumsq: null table");
  memset(&a, 0, sizeof(a));
  a.n = n;
  int64_t t = 0;
  for (int i = 0; i < n; ++i) {
    if (!src[i] || numel[i] < 0) return fail(SIREN_EINVAL, "sumsq: tensor %d", i);
    a.src[i] = src[i];
    a.begin[i] = t;
    t += numel[i];
  }
  a.begin[n] = t;
  return SIREN_OK;
}
}  // namespace

int siren_sumsq_forward(int n, const float* const* src, const int64_t* numel, float* out, void* ws, int64_t ws_bytes,
                        void* stream) {
  SumsqArgs a;
  int rc = sumsq_setup(a, n, src, numel);
  if (rc) return rc;
  if (!out || !ws || ws_bytes < siren_sumsq_workspace_bytes(a.begin[n]))
    return fail(SIREN_ENOSPACE, "sumsq: workspace (zeroed, siren_sumsq_workspace_bytes) missing or small");
  a.counter = (unsigned*)ws;
  a.part = (float*)((char*)ws + 256);
  a.out = out;
  const int64_t nb = std::max<int64_t>(1, cdiv(a.begin[n], SUMSQ_CHUNK));
  hipLaunchKernelGGL(sumsq_fwd_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("sumsq_fwd");
}

int siren_sumsq_backward(int n, const float* const* src, const int64_t* numel, const float* g, float* const* dst,
                         void* stream) {
  SumsqArgs a;
  int rc = sumsq_setup(a, n, src, numel);
  if (rc) return rc;
  if (!g || !dst) return fail(SIREN_EINVAL, "sumsq backward: null argument");
  for (int i = 0; i < n; ++i) {
    if (!dst[i]) return fail(SIREN_EINVAL, "sumsq backward: null output %d", i);
    a.dst[i] = dst[i];
  }
  a.g = g;
  if (a.begin[n] == 0) return SIREN_OK;
  hipLaunchKernelGGL(sumsq_bwd_kernel, dim3((unsigned)cdiv(a.begin[n], 256)), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("sumsq_bwd");
}

int siren_enc_prep(int n, const float* const* w, const float* const* b, const int64_t* geom, void* const* wb,
                   void* const* wf, void* const* bb, void* stream) {
  if (n < 1 || n > ENC_PREP_MAX) return fail(SIREN_EINVAL, "enc_prep: %d filters (1..%d)", n, ENC_PREP_MAX);
  if (!w || !geom || !wb) return fail(SIREN_EINVAL, "enc_prep: null table");
  EncPrepArgs a;
  memset(&a, 0, sizeof(a));
  a.nseg = n;
  int64_t t = 0;
  for (int i = 0; i < n; ++i) {
    EncPrepSeg& g = a.seg[i];
    const int64_t* q = geom + 7 * i;
    g.co = (int)q[0];
    g.ci = (int)q[1];
    g.k = (int)q[2];
    g.s_co = q[3];
    g.s_ci = q[4];
    g.s_kh = q[5];
    g.s_kw = q[6];
    if (g.co < 1 || g.ci < 1 || g.k < 1) return fail(SIREN_EINVAL, "enc_prep: filter %d shape", i);
    g.w = w[i];
    g.b = b ? b[i] : nullptr;
    g.wb = (bf16*)wb[i];
    g.wf = wf ? (bf16*)wf[i] : nullptr;
    g.bb = bb ? (bf16*)bb[i] : nullptr;
    if (!g.w || !g.wb || (g.bb && !g.b)) return fail(SIREN_EINVAL, "enc_prep: filter %d null pointer", i);
    g.begin = t;
    t += (int64_t)g.co * g.ci * g.k * g.k + (g.bb ? g.co : 0);
  }
  a.total = t;
  hipLaunchKernelGGL(enc_prep_kernel, dim3((unsigned)cdiv(t, 256)), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("enc_prep");
}

int siren_enc_relu_bwd(const void* g1, const void* g2, const void* y, void* out, float* db, int64_t P, int C, void* ws,
                       int64_t ws_bytes, void* stream) {
  EncArgs a;
  int rc = enc_setup(a, P, C, ws, ws_bytes, db != nullptr, 512, "enc_relu_bwd");
  if (rc) return rc;
  if (!g1 || !y || !out) return fail(SIREN_EINVAL, "enc_relu_bwd: null plane");
  if (P == 0) return SIREN_OK;
  a.g1 = (const bf16*)g1;
  a.g2 = (const bf16*)g2;
  a.y = (const bf16*)y;
  a.out = (bf16*)out;
  a.db = db;
  hipLaunchKernelGGL(enc_relu_bwd_kernel, dim3((unsigned)cdiv(P, a.chunk)), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("enc_relu_bwd");
}

int siren_enc_bias_relu(void* y, const void* cb, int64_t P, int C, void* stream) {
  EncArgs a;
  int rc = enc_setup(a, P, C, nullptr, 0, false, 512, "enc_bias_relu");
  if (rc) return rc;
  if (!y) return fail(SIREN_EINVAL, "enc_bias_relu: null plane");
  if (P == 0) return SIREN_OK;
  a.out = (bf16*)y;
  a.cb = (const bf16*)cb;
  hipLaunchKernelGGL(enc_bias_relu_kernel, dim3((unsigned)std::min<int64_t>(cdiv(P * C / 8, 256), 8192)), dim3(256), 0,
                     (hipStream_t)stream, a);
  return check_launch("enc_bias_relu");
}

int siren_enc_res_fwd(const void* a_pre, const void* cb, const void* x, void* out, int64_t P, int C, void* stream) {
  EncArgs a;
  int rc = enc_setup(a, P, C, nullptr, 0, false, 512, "enc_res_fwd");
  if (rc) return rc;
  if (!a_pre || !x || !out) return fail(SIREN_EINVAL, "enc_res_fwd: null plane");
  if (P == 0) return SIREN_OK;
  a.cb = (const bf16*)cb;
  a.a = (const bf16*)a_pre;
  a.g1 = (const bf16*)x;
  a.out = (bf16*)out;
  hipLaunchKernelGGL(enc_res_fwd_kernel, dim3((unsigned)std::min<int64_t>(cdiv(P * C / 8, 256), 8192)), dim3(256), 0,
                     (hipStream_t)stream, a);
  return check_launch("enc_res_fwd");
}

int siren_enc_res_bwd(const void* g1, const void* g2, const void* out, const void* a_pre, const void* cb, void* gskip,
                      void* ga, float* db, int64_t P, int C, void* ws, int64_t ws_bytes, void* stream) {
  EncArgs a;
  int rc = enc_setup(a, P, C, ws, ws_bytes, db != nullptr, 512, "enc_res_bwd");
  if (rc) return rc;
  if (!g1 || !out || !a_pre || !gskip || !ga) return fail(SIREN_EINVAL, "enc_res_bwd: null plane");
  if (P == 0) return SIREN_OK;
  a.g1 = (const bf16*)g1;
  a.g2 = (const bf16*)g2;
  a.y = (const bf16*)out;
  a.a = (const bf16*)a_pre;
  a.cb = (const bf16*)cb;
  a.out = (bf16*)gskip;
  a.out2 = (bf16*)ga;
  a.db = db;
  hipLaunchKernelGGL(enc_res_bwd_kernel, dim3((unsigned)cdiv(P, a.chunk)), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("enc_res_bwd");
}

int siren_enc_pixfc_fwd(const void* a_pre, const void* cb, const float* w, const float* bias, float* e, int B,
                        int64_t P, int C, void* ws, int64_t ws_bytes, void* stream) {
  EncArgs a;
  // chunks of >= 512 pixels, at most ENC_MAX_BLOCKS blocks over the B images (32 x 32 at C4's 128^2)
  const int64_t min_rows = std::max<int64_t>(512, cdiv(std::max<int64_t>(P, 1), std::max<int64_t>(1, ENC_MAX_BLOCKS / std::max(B, 1))));
  int rc = enc_setup(a, P, C, ws, ws_bytes, true, min_rows, "enc_pixfc_fwd");
  if (rc) return rc;
  if (!a_pre || !w || !bias || !e || B < 1) return fail(SIREN_EINVAL, "enc_pixfc_fwd: null pointer or B < 1");
  const int64_t nchunk = cdiv(P, a.chunk);
  if (nchunk * B > ENC_MAX_BLOCKS || (int64_t)B * C > ENC_WS_FLOATS)
    return fail(SIREN_EINVAL, "enc_pixfc_fwd: %lld blocks > %d", (long long)(nchunk * B), ENC_MAX_BLOCKS);
  if (P == 0) return fail(SIREN_EINVAL, "enc_pixfc_fwd: no pixels");
  a.a = (const bf16*)a_pre;
  a.cb = (const bf16*)cb;
  a.w = w;
  a.bias = bias;
  a.e = e;
  a.B = B;
  hipLaunchKernelGGL(enc_pixfc_fwd_kernel, dim3((unsigned)nchunk, (unsigned)B), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("enc_pixfc_fwd");
}

int siren_enc_pixfc_bwd(const float* g, const void* a_pre, const void* cb, const float* w, void* ga, float* db,
                        float* gw, int B, int64_t P, int C, void* ws, int64_t ws_bytes, void* stream) {
  EncArgs a;
  int rc = enc_setup(a, P, C, ws, ws_bytes, true, 32, "enc_pixfc_bwd");  // 512 blocks at 128^2 (128: 177 us, C4)
  if (rc) return rc;
  if (!g || !a_pre || !w || !ga || !db || !gw || B < 1) return fail(SIREN_EINVAL, "enc_pixfc_bwd: null pointer or B < 1");
  if (P == 0) return fail(SIREN_EINVAL, "enc_pixfc_bwd: no pixels");
  a.gin = g;
  a.a = (const bf16*)a_pre;
  a.cb = (const bf16*)cb;
  a.w = w;
  a.out = (bf16*)ga;
  a.db = db;
  a.e = gw;
  a.B = B;
  hipLaunchKernelGGL(enc_pixfc_bwd_kernel, dim3((unsigned)cdiv(P, a.chunk)), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("enc_pixfc_bwd");
}

int siren_sse_forward(const float* pred, const float* tgt, const float* mask, int64_t n, int64_t mask_n,
                      float weight, float* d, float* loss, void* workspace, int64_t ws_bytes, void* stream) {
  if (n < 0 || !loss || (n > 0 && (!pred || !tgt || !d)) || (mask && mask_n <= 0))
    return fail(SIREN_EINVAL, "sse_forward: bad arguments (n=%lld, mask_n=%lld)", (long long)n, (long long)mask_n);
  if (!workspace || ws_bytes < siren_sse_workspace_bytes())
    return fail(SIREN_EINVAL, "sse_forward: workspace of %lld bytes, need %lld", (long long)ws_bytes,
                (long long)siren_sse_workspace_bytes());
  SseFwdArgs a;
  a.pred = pred;
  a.tgt = tgt;
  a.mask = mask;
  a.d = d;
  a.loss = loss;
  a.partial = (float*)workspace;
  a.counter = (unsigned*)((char*)workspace + SSE_MAX_BLOCKS * 4);
  a.n = n;
  a.mask_n = mask ? mask_n : 1;
  a.weight = weight;
  // 16 elements per thread: few enough blocks that the hand-off counter (one agent-scope add per
  // block, all on one address) stays off the critical path (262144 elements: 64 blocks)
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(SSE_MAX_BLOCKS, cdiv(n, 16 * SSE_THREADS)));
  hipLaunchKernelGGL(sse_fwd_kernel, dim3(blocks), dim3(SSE_THREADS), 0, (hipStream_t)stream, a);
  return check_launch("sse_forward");
}

int siren_sse_backward(const float* d, const float* mask, int64_t n, int64_t mask_n, const float* g, float scale,
                       float* out, void* stream) {
  if (n < 0 || (n > 0 && (!d || !g || !out)) || (mask && mask_n <= 0))
    return fail(SIREN_EINVAL, "sse_backward: bad arguments (n=%lld, mask_n=%lld)", (long long)n, (long long)mask_n);
  if (n == 0) return SIREN_OK;
  SseBwdArgs a;
  a.d = d;
  a.mask = mask;
  a.g = g;
  a.out = out;
  a.n = n;
  a.mask_n = mask ? mask_n : 1;
  a.scale = scale;
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, cdiv(n, 4 * SSE_THREADS)));
  hipLaunchKernelGGL(sse_bwd_kernel, dim3(blocks), dim3(SSE_THREADS), 0, (hipStream_t)stream, a);
  return check_launch("sse_backward");
}

int siren_dc_forward(const float* pred, const float* k0, const float* mask, int64_t batch, int64_t npix,
                     int channels, float noise, float* out, void* stream) {
  if (batch < 0 || npix < 0 || channels < 1 || channels > KS_MAXC || (batch * npix > 0 && (!pred || !k0 || !mask || !out)))
    return fail(SIREN_EINVAL, "dc_forward: bad arguments (batch=%lld, npix=%lld, channels=%d)", (long long)batch,
                (long long)npix, channels);
  if (batch * npix == 0) return SIREN_OK;
  DcArgs a{pred, k0, mask, out, batch, npix, channels, noise, 0};
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, cdiv(batch * npix, KS_THREADS)));
  hipLaunchKernelGGL(dc_kernel, dim3(blocks), dim3(KS_THREADS), 0, (hipStream_t)stream, a);
  return check_launch("dc_forward");
}

int siren_dc_backward(const float* g, const float* mask, int64_t batch, int64_t npix, int channels, float noise,
                      float* dpred, void* stream) {
  if (batch < 0 || npix < 0 || channels < 1 || channels > KS_MAXC || (batch * npix > 0 && (!g || !mask || !dpred)))
    return fail(SIREN_EINVAL, "dc_backward: bad arguments");
  if (batch * npix == 0) return SIREN_OK;
  DcArgs a{g, nullptr, mask, dpred, batch, npix, channels, noise, 1};
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, cdiv(batch * npix, KS_THREADS)));
  hipLaunchKernelGGL(dc_kernel, dim3(blocks), dim3(KS_THREADS), 0, (hipStream_t)stream, a);
  return check_launch("dc_backward");
}

int siren_kspace_sse_forward(const float* pred, const float* k0, const float* mask, const float* tgt,
                             const float* hf, int64_t batch, int64_t npix, int channels, float noise, float weight,
                             float* d, float* loss, void* workspace, int64_t ws_bytes, void* stream) {
  if (batch < 0 || npix < 0 || channels < 1 || channels > KS_MAXC || !loss || (!k0) != (!mask) ||
      (batch * npix > 0 && (!pred || !tgt || !d)))
    return fail(SIREN_EINVAL, "kspace_sse_forward: bad arguments (batch=%lld, npix=%lld, channels=%d)",
                (long long)batch, (long long)npix, channels);
  if (!workspace || ws_bytes < siren_sse_workspace_bytes())
    return fail(SIREN_EINVAL, "kspace_sse_forward: workspace of %lld bytes, need %lld", (long long)ws_bytes,
                (long long)siren_sse_workspace_bytes());
  KsseFwdArgs a{pred, k0, mask, tgt, hf, d, loss, (float*)workspace,
                (unsigned*)((char*)workspace + SSE_MAX_BLOCKS * 4), batch, npix, channels, noise, weight};
  // 8 coordinates per thread: few blocks for the hand-off counter (32 x 16384 coordinates: 256)
  const unsigned blocks =
      (unsigned)std::max<int64_t>(1, std::min<int64_t>(KS_MAX_BLOCKS, cdiv(batch * npix, 8 * KS_THREADS)));
  hipLaunchKernelGGL(ksse_fwd_kernel, dim3(blocks), dim3(KS_THREADS), 0, (hipStream_t)stream, a);
  return check_launch("kspace_sse_forward");
}

int siren_kspace_sse_backward(const float* d, const float* mask, const float* hf, int64_t batch, int64_t npix,
                              int channels, float noise, const float* g, float scale, float* dpred, void* stream) {
  if (batch < 0 || npix < 0 || channels < 1 || channels > KS_MAXC || (batch * npix > 0 && (!d || !g || !dpred)))
    return fail(SIREN_EINVAL, "kspace_sse_backward: bad arguments");
  if (batch * npix == 0) return SIREN_OK;
  KsseBwdArgs a{d, mask, hf, g, dpred, batch, npix, channels, noise, scale};
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, cdiv(batch * npix, KS_THREADS)));
  hipLaunchKernelGGL(ksse_bwd_kernel, dim3(blocks), dim3(KS_THREADS), 0, (hipStream_t)stream, a);
  return check_launch("kspace_sse_backward");
}

int siren_fourier_features(const float* x, const float* B, int64_t rows, int cin, int m, float* out, void* stream) {
  if (rows < 0 || cin < 1 || m < 1 || (rows > 0 && (!x || !B || !out)))
    return fail(SIREN_EINVAL, "fourier_features: bad arguments (rows=%lld, cin=%d, m=%d)", (long long)rows, cin, m);
  if (rows == 0) return SIREN_OK;
  FourierArgs a{x, B, out, rows, cin, m};
  const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(4096, cdiv(rows * m, KS_THREADS)));
  hipLaunchKernelGGL(fourier_kernel, dim3(blocks), dim3(KS_THREADS), 0, (hipStream_t)stream, a);
  return check_launch("fourier_features");
}

int siren_sincos_f32(const float* x, float* s, float* c, int64_t n, int impl, void* stream) {
  if (n < 0 || (impl != 0 && impl != 1) || (n > 0 && (!x || !s || !c)))
    return fail(SIREN_EINVAL, "sincos_f32: bad arguments (n=%lld, impl=%d)", (long long)n, impl);
  if (n == 0) return SIREN_OK;
  hipLaunchKernelGGL(sincos_probe_kernel, dim3(grid1d(n, 4096)), dim3(256), 0, (hipStream_t)stream, x, s, c, n, impl);
  return check_launch("sincos_f32");
}

int64_t siren_adam_num_blocks(const siren_adam_desc* d) {
  if (!d || d->num_tensors <= 0 || d->num_tensors > SIREN_ADAM_MAX_TENSORS) return 0;
  int64_t maxn = 0;
  for (int t = 0; t < d->num_tensors; ++t) maxn = std::max(maxn, d->numel[t]);
  return maxn > 0 ? (int64_t)grid1d(maxn, 1024) * d->num_tensors : 0;
}

int siren_adam_step(const siren_adam_desc* d, void* stream) {
  if (!d || d->num_tensors < 0 || d->num_tensors > SIREN_ADAM_MAX_TENSORS)
    return fail(SIREN_EINVAL, "adam: num_tensors outside [0, %d]", SIREN_ADAM_MAX_TENSORS);
  if (d->num_tensors == 0) return SIREN_OK;
  AdamArgs a;
  memset(&a, 0, sizeof(a));
  int64_t maxn = 0;
  for (int t = 0; t < d->num_tensors; ++t) {
    if (!d->param[t] || !d->grad[t] || !d->exp_avg[t] || !d->exp_avg_sq[t] || d->numel[t] < 0)
      return fail(SIREN_EINVAL, "adam: tensor %d has a null pointer or negative size", t);
    a.param[t] = d->param[t];
    a.grad[t] = d->grad[t];
    a.exp_avg[t] = d->exp_avg[t];
    a.exp_avg_sq[t] = d->exp_avg_sq[t];
    a.numel[t] = d->numel[t];
    maxn = std::max(maxn, d->numel[t]);
  }
  a.one_minus_beta1 = d->one_minus_beta1;
  a.beta2 = d->beta2;
  a.one_minus_beta2 = d->one_minus_beta2;
  a.eps = d->eps;
  a.weight_decay = d->weight_decay;
  a.step = d->step_size;
  a.bc2_sqrt = d->bias_correction2_sqrt;
  a.dev = d->dev_scalars;
  a.steps = d->dev_steps;
  a.table = d->dev_table;
  a.table_n = d->table_n;
  if (a.steps && (!a.table || a.table_n < 1)) return fail(SIREN_EINVAL, "adam: dev_steps without a table");
  a.maximize = d->maximize;
  if (maxn == 0) {
    if (a.steps) return fail(SIREN_EINVAL, "adam: dev_steps with no elements (the counters would not advance)");
    return SIREN_OK;
  }
  hipLaunchKernelGGL(adam_kernel, dim3(grid1d(maxn, 1024), (unsigned)d->num_tensors), dim3(256), 0,
                     (hipStream_t)stream, a);
  return check_launch("adam");
}

int siren_config_set(const char* key, int64_t value) {
  if (key && strcmp(key, "fused_forward") == 0 && (value == 0 || value == 1)) {
    g_fused_forward = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "fused_backward") == 0 && (value == 0 || value == 1)) {
    g_fused_backward = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "ring_output_fusion") == 0 && (value == 0 || value == 1)) {
    g_ring_top = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "fuse_output_layer") == 0 && (value == 0 || value == 1)) {
    g_fuse_top = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "fused_forward_pipe") == 0 && (value == 0 || value == 1)) {
    g_fwd_pipe = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "freg_magic") == 0 && (value == 0 || value == 1)) {
    g_freg_magic = value != 0;
    return 0;
  }
  if (key && strcmp(key, "fused_forward_reg") == 0 && (value == 0 || value == 1)) {
    g_fwd_reg = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "bwd_ring") == 0 && (value == 0 || value == 1)) {
    g_bwd_ring = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "dw_ring") == 0 && (value == 0 || value == 1)) {
    g_dw_ring = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "dx_ring") == 0 && (value == 0 || value == 1)) {
    g_dx_ring = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "debug_pair_roles") == 0 && value >= 0 && value <= 3) {
    g_pair_roles = (int)value;
    return SIREN_OK;
  }
  if (key && strcmp(key, "dx_stagger") == 0 && (value == 0 || value == 1)) {
    g_dx_stagger = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "pair_tail_reduce") == 0 && (value == 0 || value == 1)) {
    g_tail_reduce = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "jvp_adj") == 0 && (value == 0 || value == 1)) {
    g_jvp_adj = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "wrw_dma") == 0 && value >= 0 && value <= 3) {
    g_wrw_dma = (int)value;
    return SIREN_OK;
  }
  if (key && strcmp(key, "conv_dma") == 0 && value >= 0 && value <= 2) {
    g_conv_dma = (int)value;
    return SIREN_OK;
  }
  if (key && strcmp(key, "f32_rows") == 0 && (value == 0 || value == 1)) {
    g_f32_rows = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "jvp_tan") == 0 && (value == 0 || value == 1)) {
    g_jvp_tan = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "jvp_tn2") == 0 && (value == 0 || value == 1)) {
    g_jvp_tn2 = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "pair_ring") == 0 && (value == 0 || value == 1)) {
    g_pair_ring = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "debug_keep_p0") == 0 && (value == 0 || value == 1)) {
    g_keep_p0 = value != 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "debug_ring_profile") == 0) {  // device pointer or 0
    g_ring_prof = (long long*)(intptr_t)value;
    g_ring_prof_n = 0;
    return SIREN_OK;
  }
  if (key && strcmp(key, "debug_fwd_skip") == 0 && value >= 0 && value <= 31) {
    g_fwd_dbg = (int)value;
    return SIREN_OK;
  }
  if (key && strcmp(key, "debug_fused_profile") == 0) {  // device pointer or 0
    g_fused_prof = (long long*)(intptr_t)value;
    return SIREN_OK;
  }
  return fail(SIREN_EINVAL, "unknown option %s=%lld", key ? key : "(null)", (long long)value);
}

int64_t siren_config_get(const char* key) {
  if (key && strcmp(key, "fused_forward") == 0) return g_fused_forward ? 1 : 0;
  if (key && strcmp(key, "fused_backward") == 0) return g_fused_backward ? 1 : 0;
  if (key && strcmp(key, "fuse_output_layer") == 0) return g_fuse_top ? 1 : 0;
  if (key && strcmp(key, "ring_output_fusion") == 0) return g_ring_top ? 1 : 0;
  if (key && strcmp(key, "dx_ring") == 0) return g_dx_ring ? 1 : 0;
  if (key && strcmp(key, "dw_ring") == 0) return g_dw_ring ? 1 : 0;
  if (key && strcmp(key, "bwd_ring") == 0) return g_bwd_ring ? 1 : 0;
  if (key && strcmp(key, "pair_tail_reduce") == 0) return g_tail_reduce ? 1 : 0;
  if (key && strcmp(key, "jvp_adj") == 0) return g_jvp_adj ? 1 : 0;
  if (key && strcmp(key, "jvp_tn2") == 0) return g_jvp_tn2 ? 1 : 0;
  if (key && strcmp(key, "jvp_tan") == 0) return g_jvp_tan ? 1 : 0;
  if (key && strcmp(key, "f32_rows") == 0) return g_f32_rows ? 1 : 0;
  if (key && strcmp(key, "conv_dma") == 0) return g_conv_dma;
  if (key && strcmp(key, "wrw_dma") == 0) return g_wrw_dma;
  if (key && strcmp(key, "dx_stagger") == 0) return g_dx_stagger ? 1 : 0;
  if (key && strcmp(key, "pair_ring") == 0) return g_pair_ring ? 1 : 0;
  if (key && strcmp(key, "debug_keep_p0") == 0) return g_keep_p0 ? 1 : 0;
  if (key && strcmp(key, "fused_forward_pipe") == 0) return g_fwd_pipe ? 1 : 0;
  if (key && strcmp(key, "fused_forward_reg") == 0) return g_fwd_reg ? 1 : 0;
  if (key && strcmp(key, "freg_magic") == 0) return g_freg_magic ? 1 : 0;
  return -1;
}

const char* siren_version(void) {
  static char buf[128];
  snprintf(buf, sizeof(buf), "siren_mri_amd gfx950 hip %d.%d", HIP_VERSION_MAJOR, HIP_VERSION_MINOR);
  return buf;
}

}  // extern "C"
