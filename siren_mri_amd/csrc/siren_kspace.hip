// siren_kspace.hip — the k-space epilogue of the hypernetwork SIREN (configs 4/5) on gfx950:
// data consistency (data_consistency.py:8-48) and image_mse's masked k-space SSE
// (loss_functions.py:66-101, utils.py:25-40), on the SIREN's own output layout.
//
//   pred, tgt, y, d : [B, N, C]  (C channels per coordinate: SingleBVPNet's output rows)
//   k0, mask        : [B, C, N]  (NCHW planes: the reference's img_sparse / dc_mask)
//   hf              : [N]        (the 128x128 high-frequency mask, pixel n = i W + j), optional
//
// The reference permutes k0 and mask to [B, N, C] (two copies) before the DC arithmetic, and
// image_mse views model_out / gt as [B, C, H, W] (lin2img), which the SSE then reads strided;
// here every kernel reads the planes where they lie, and the SSE runs on [B, N, C] directly (the
// loss is a sum; only the mask index depends on the layout). With DC folded into the SSE, the
// fused pair is one forward launch (loss + the saved residual) and one backward launch that
// writes dL/dpred (the DC's backward included), instead of the ~10 PyTorch launches of
// permute / arithmetic / lin2img / sum and their backward.
#include "siren_common.h"

namespace siren {

constexpr int KS_THREADS = 256;
constexpr int KS_MAX_BLOCKS = 1024;
constexpr int KS_MAXC = 8;

struct DcArgs {
  const float* pred;   // [B, N, C] forward input / backward upstream gradient
  const float* k0;     // [B, C, N]
  const float* mask;   // [B, C, N]
  float* out;          // [B, N, C]
  int64_t batch, npix;
  int C;
  float noise;
  int backward;        // 0: out = DC(pred); 1: out = dc_coef(mask) * pred (pred = upstream gradient)
};

__global__ __launch_bounds__(KS_THREADS) void dc_kernel(DcArgs a) {
  const int64_t nq = a.batch * a.npix;
  const int64_t stride = (int64_t)gridDim.x * KS_THREADS;
  for (int64_t q = (int64_t)blockIdx.x * KS_THREADS + threadIdx.x; q < nq; q += stride) {
    const int64_t b = q / a.npix, n = q - b * a.npix;
    for (int c = 0; c < a.C; ++c) {
      const int64_t e = q * a.C + c, pl = (b * a.C + c) * a.npix + n;
      const float m = a.mask[pl];
      a.out[e] = a.backward ? __fmul_rn(dc_coef(m, a.noise), a.pred[e]) : dc_value(a.pred[e], a.k0[pl], m, a.noise);
    }
  }
}

struct KsseFwdArgs {
  const float* pred;   // [B, N, C]
  const float* k0;     // [B, C, N] (null: no data consistency)
  const float* mask;   // [B, C, N]
  const float* tgt;    // [B, N, C]
  const float* hf;     // [N] (null: no mask)
  float* d;            // [B, N, C] hf (DC(pred) - tgt), kept for the backward
  float* loss;         // [1]
  float* partial;      // [KS_MAX_BLOCKS] per-block sums (workspace)
  unsigned* counter;   // zero between launches (the last block resets it)
  int64_t batch, npix;
  int C;
  float noise, weight;
};

// Per-thread sums over a fixed grid-stride order, a fixed block tree, and the last block adds the
// block sums in index order (the hand-off of sse_fwd_kernel, siren_loss.hip): deterministic.
__global__ __launch_bounds__(KS_THREADS) void ksse_fwd_kernel(KsseFwdArgs a) {
  __shared__ float red[KS_THREADS / 64];
  __shared__ unsigned ticket;
  float acc = 0.f;
  const int64_t nq = a.batch * a.npix;
  const int64_t stride = (int64_t)gridDim.x * KS_THREADS;
  for (int64_t q = (int64_t)blockIdx.x * KS_THREADS + threadIdx.x; q < nq; q += stride) {
    const int64_t b = q / a.npix, n = q - b * a.npix;
    const float h = a.hf ? a.hf[n] : 1.f;
    for (int c = 0; c < a.C; ++c) {
      const int64_t e = q * a.C + c;
      float y = a.pred[e];
      if (a.k0) {
        const int64_t pl = (b * a.C + c) * a.npix + n;
        y = dc_value(y, a.k0[pl], a.mask[pl], a.noise);
      }
      const float dd = __fmul_rn(h, __fsub_rn(y, a.tgt[e]));
      a.d[e] = dd;
      acc = fmaf(dd, dd, acc);
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < KS_THREADS / 64; ++w) s += red[w];
    __hip_atomic_store(a.partial + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ticket = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (ticket != gridDim.x - 1) return;
  float s = 0.f;
  for (unsigned b = threadIdx.x; b < gridDim.x; b += KS_THREADS)
    s += __hip_atomic_load(a.partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s = wave_sum(s);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < KS_THREADS / 64; ++w) tot += red[w];
    a.loss[0] = tot * a.weight;
    __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct KsseBwdArgs {
  const float* d;      // [B, N, C]
  const float* mask;   // [B, C, N] (null: no data consistency)
  const float* hf;     // [N] or null
  const float* g;      // [1] upstream gradient of the loss
  float* out;          // [B, N, C] dL / dpred
  int64_t batch, npix;
  int C;
  float noise, scale;  // scale = 2 weight
};

__global__ __launch_bounds__(KS_THREADS) void ksse_bwd_kernel(KsseBwdArgs a) {
  const float k = a.g[0] * a.scale;
  const int64_t nq = a.batch * a.npix;
  const int64_t stride = (int64_t)gridDim.x * KS_THREADS;
  for (int64_t q = (int64_t)blockIdx.x * KS_THREADS + threadIdx.x; q < nq; q += stride) {
    const int64_t b = q / a.npix, n = q - b * a.npix;
    const float h = a.hf ? a.hf[n] : 1.f;
    for (int c = 0; c < a.C; ++c) {
      const int64_t e = q * a.C + c;
      float v = h * (a.d[e] * k);
      if (a.mask) v *= dc_coef(a.mask[(b * a.C + c) * a.npix + n], a.noise);
      a.out[e] = v;
    }
  }
}

// Gaussian Fourier features (features.py:31-41): out[r] = [sin(2 pi x_r B), cos(2 pi x_r B)],
// x [rows, cin], B [cin, m], out [rows, 2 m]; one launch for the reference's matmul, scale, sin,
// cos and cat. The argument is formed as the reference does (x B, then times 2 pi, fp32) and the
// accurate sinf / cosf take it (|2 pi x B| reaches hundreds of radians at scale 21).
struct FourierArgs {
  const float* x;
  const float* B;
  float* out;
  int64_t rows;
  int cin, m;
};

__global__ __launch_bounds__(KS_THREADS) void fourier_kernel(FourierArgs a) {
  const int64_t n = a.rows * a.m;
  const int64_t stride = (int64_t)gridDim.x * KS_THREADS;
  for (int64_t q = (int64_t)blockIdx.x * KS_THREADS + threadIdx.x; q < n; q += stride) {
    const int64_t r = q / a.m;
    const int k = (int)(q - r * a.m);
    float z = 0.f;
    for (int c = 0; c < a.cin; ++c) z = fmaf(a.x[r * a.cin + c], a.B[c * a.m + k], z);
    const float arg = __fmul_rn(6.2831854820251465f, z);  // (float)(2 pi), as 2 * np.pi * z in fp32
    // the sin / cos of siren_common.h ff_feature (Cody-Waite + minimax, one reduction for both):
    // the features the register forward forms in its first layer from the raw coordinates are then
    // bit-identical to these, so the fused and the materialised paths compute the same network
    float sv, cv;
    if (__builtin_expect(__builtin_fabsf(arg) < kFFPolyRange, 1)) {
      float sn, cs;
      int qd;
      sincos_poly(arg, sn, cs, qd);
      sv = (qd & 1) ? cs : sn;
      sv = (qd & 2) ? -sv : sv;
      cv = ((qd + 1) & 1) ? cs : sn;
      cv = ((qd + 1) & 2) ? -cv : cv;
    } else {
      sv = sin_f32(arg);
      cv = cos_f32(arg);
    }
    a.out[r * 2 * a.m + k] = sv;
    a.out[r * 2 * a.m + a.m + k] = cv;
  }
}

}  // namespace siren
