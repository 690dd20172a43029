// siren_encoder.hip — the elementwise and reduction work around the convolutions of configs 4/5's
// conv encoder (ConvImgEncoder, modules.py:340-380; Conv2dResBlock, modules.py:433-450) in bf16,
// channels-last (NHWC: a [P, C] row-major plane, P = N H W pixels, C channels innermost).
//
// The convolutions themselves are MIOpen's (the input gradient as a forward convolution with the
// flipped, transposed filter; the weight gradient alone). Around them the autograd chain of the
// reference launches, per layer, a ReLU, a ReLU mask in the backward, a bias-gradient reduction and
// the residual adds as separate passes over 134 MB planes (C4: 32 x 128^2 x 128 bf16); here they
// are folded into one pass each:
//
//   enc_relu_bwd     g = (g1 [+ g2]) * (y > 0) -> bf16, db[c] = sum_p g        (ReLU + bias grad)
//   enc_res_fwd      out = relu(relu(a) + x)                                (res block tail)
//   enc_res_bwd      s = (g1 [+ g2]) * (out > 0), ga = s * (a > 0), db[c] = sum_p ga
//   enc_pixfc_fwd    e[b][c] = sum_p relu(a[b][p][c]) w[p] + bias           (relu_2 + fc over pixels)
//   enc_pixfc_bwd    ga[b][p][c] = (a > 0) g[b][c] w[p], db[c] = sum ga, gw[p] = sum_bc g relu(a)
//
// Thread mapping: a thread owns 8 channels (16 bytes) of one pixel, C / 8 threads per pixel.
// Channel sums are per-thread fp32 partials over a block's pixels, summed over the block in a fixed
// order, then over the blocks by the last block to finish (ticket in the workspace, re-armed by
// that block): deterministic, one launch.
#include "siren_common.h"

namespace siren {

constexpr int ENC_MAX_BLOCKS = 1024;
constexpr int ENC_MAXC = 256;
// workspace: partial sums [ENC_MAX_BLOCKS][ENC_MAXC] (pixfc_fwd: [blocks][B][C] <= the same), then
// the ticket
constexpr int64_t ENC_WS_FLOATS = (int64_t)ENC_MAX_BLOCKS * ENC_MAXC;

struct EncArgs {
  const bf16* g1;     // incoming gradient (or a / x operands, see each kernel)
  const bf16* g2;     // second gradient summand, or null
  const bf16* y;      // mask source: y > 0
  const bf16* a;      // pre-activation (res_fwd / res_bwd / pixfc)
  bf16* out;          // bf16 result plane
  bf16* out2;         // second bf16 result plane (res_bwd: ga)
  float* db;          // [C] channel sums (null: not wanted)
  const float* w;     // pixfc: [P_img] weights
  const float* gin;   // pixfc_bwd: [B][C] incoming gradient
  float* e;           // pixfc_fwd: [B][C] output; pixfc_bwd: gw [P_img]
  const float* bias;  // pixfc_fwd: [1] device scalar added to every output
  float* part;        // workspace partials
  unsigned* ticket;   // workspace ticket
  int64_t P;          // pixels of the plane (pixfc: per image)
  int64_t chunk;      // pixels per block (a multiple of the pixels per iteration)
  int C, B;
};

DEV void load_bf16x8(const bf16* p, float (&v)[8]) {
  const bf16x8 t = *(const bf16x8*)p;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (float)t[e];
}

// The block's channel sums (acc: this thread's 8 channels at c0) into part[blk][C], then the
// last block to finish adds the blocks' rows in order into dst (C columns, or B * C for
// pixfc_fwd's [B][C] sums, each image's blocks only), plus *addend if given.
DEV void enc_block_sum(const EncArgs& a, const float (&acc)[8], int c0, int pix, int ppi, int ncol, float* dst,
                       const float* addend) {
  __shared__ float red[256 * 8];
  const int tid = threadIdx.x;
  // red[pix][c]: ppi rows of C (the block's pixel lanes)
#pragma unroll
  for (int e = 0; e < 8; ++e) red[pix * a.C + c0 + e] = acc[e];
  __syncthreads();
  const unsigned nblk = gridDim.x * gridDim.y;
  const unsigned blk = blockIdx.y * gridDim.x + blockIdx.x;
  const int nc = a.C;
  for (int c = tid; c < nc; c += 256) {
    float s = 0.f;
    for (int r = 0; r < ppi; ++r) s += red[r * nc + c];
    __hip_atomic_store(a.part + (int64_t)blk * nc + c, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // every writing wave's stores complete before the barrier (a release fence covers the issuing
  // wave's own stores only), so the ticket below is taken after all of this block's partials
  __threadfence();
  __shared__ unsigned last;
  __syncthreads();
  if (tid == 0) {
    last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1;
  }
  __syncthreads();
  if (!last) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  // ncol output columns: column k sums part[b][k % nc] over the blocks b whose rows carry it
  // (every block for the channel sums; blocks of image k / nc for pixfc_fwd)
  for (int k = tid; k < ncol; k += 256) {
    float s = 0.f;
    if (ncol == nc) {
      for (unsigned b = 0; b < nblk; ++b)
        s += __hip_atomic_load(a.part + (int64_t)b * nc + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const int img = k / nc, c = k - img * nc;
      for (unsigned b = 0; b < gridDim.x; ++b)
        s += __hip_atomic_load(a.part + ((int64_t)img * gridDim.x + b) * nc + c, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    dst[k] = addend ? s + *addend : s;
  }
  if (tid == 0) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// g = (g1 [+ g2]) * (y > 0) -> out; db = channel sums of g (as stored, bf16-rounded)
__global__ __launch_bounds__(256) void enc_relu_bwd_kernel(EncArgs a) {
  const int tpp = a.C / 8, ppi = 256 / tpp;
  const int pix = threadIdx.x / tpp, c0 = 8 * (threadIdx.x % tpp);
  const int64_t p0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t p1 = p0 + a.chunk < a.P ? p0 + a.chunk : a.P;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int64_t p = p0 + pix; p < p1; p += ppi) {
    const int64_t off = p * a.C + c0;
    float g[8], m[8];
    load_bf16x8(a.g1 + off, g);
    if (a.g2) {
      float g2[8];
      load_bf16x8(a.g2 + off, g2);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] += g2[e];
    }
    load_bf16x8(a.y + off, m);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = (bf16)(m[e] > 0.f ? g[e] : 0.f);
      acc[e] += (float)o[e];
    }
    *(bf16x8*)(a.out + off) = o;
  }
  if (a.db) enc_block_sum(a, acc, c0, pix, ppi, a.C, a.db, nullptr);
}

// out = relu(relu(a) + x), x = g1 (the block input)
__global__ __launch_bounds__(256) void enc_res_fwd_kernel(EncArgs a) {
  const int64_t n8 = a.P * a.C / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8], x[8];
    load_bf16x8(a.a + 8 * i, v);
    load_bf16x8(a.g1 + 8 * i, x);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // relu(a) + x rounded to bf16 first (the reference chain's add output), then the ReLU
      const float s = (float)(bf16)(fmaxf(v[e], 0.f) + x[e]);
      o[e] = (bf16)fmaxf(s, 0.f);
    }
    *(bf16x8*)(a.out + 8 * i) = o;
  }
}

// s = (g1 [+ g2]) * (out > 0) -> out (the skip's gradient); ga = s * (a > 0) -> out2; db = sum ga
__global__ __launch_bounds__(256) void enc_res_bwd_kernel(EncArgs a) {
  const int tpp = a.C / 8, ppi = 256 / tpp;
  const int pix = threadIdx.x / tpp, c0 = 8 * (threadIdx.x % tpp);
  const int64_t p0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t p1 = p0 + a.chunk < a.P ? p0 + a.chunk : a.P;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int64_t p = p0 + pix; p < p1; p += ppi) {
    const int64_t off = p * a.C + c0;
    float g[8], mo[8], ma[8];
    load_bf16x8(a.g1 + off, g);
    if (a.g2) {
      float g2[8];
      load_bf16x8(a.g2 + off, g2);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] += g2[e];
    }
    load_bf16x8(a.y + off, mo);
    load_bf16x8(a.a + off, ma);
    bf16x8 s, ga;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s[e] = (bf16)(mo[e] > 0.f ? g[e] : 0.f);
      ga[e] = ma[e] > 0.f ? s[e] : (bf16)0.f;
      acc[e] += (float)ga[e];
    }
    *(bf16x8*)(a.out + off) = s;
    *(bf16x8*)(a.out2 + off) = ga;
  }
  if (a.db) enc_block_sum(a, acc, c0, pix, ppi, a.C, a.db, nullptr);
}

// e[b][c] = sum_p relu(a[b][p][c]) w[p] + bias; grid (chunks, B)
__global__ __launch_bounds__(256) void enc_pixfc_fwd_kernel(EncArgs a) {
  const int tpp = a.C / 8, ppi = 256 / tpp;
  const int pix = threadIdx.x / tpp, c0 = 8 * (threadIdx.x % tpp);
  const int64_t b = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t p1 = p0 + a.chunk < a.P ? p0 + a.chunk : a.P;
  const bf16* src = a.a + b * a.P * a.C;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int64_t p = p0 + pix; p < p1; p += ppi) {
    float v[8];
    load_bf16x8(src + p * a.C + c0, v);
    const float wp = a.w[p];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = fmaf(fmaxf(v[e], 0.f), wp, acc[e]);
  }
  enc_block_sum(a, acc, c0, pix, ppi, a.B * a.C, a.e, a.bias);
}

// ga = (a > 0) g[b][c] w[p] -> out; db[c] = sum_{b,p} ga; gw[p] = sum_{b,c} g[b][c] relu(a[b][p][c]).
// One block per pixel chunk, looping over the images (gw needs every image of a pixel).
__global__ __launch_bounds__(256) void enc_pixfc_bwd_kernel(EncArgs a) {
  const int tpp = a.C / 8, ppi = 256 / tpp;
  const int pix = threadIdx.x / tpp, c0 = 8 * (threadIdx.x % tpp);
  const int64_t p0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t p1 = p0 + a.chunk < a.P ? p0 + a.chunk : a.P;
  float acc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  for (int64_t p = p0 + pix; p < p1; p += ppi) {
    const float wp = a.w[p];
    float gw = 0.f;
    for (int b = 0; b < a.B; ++b) {
      const int64_t off = ((int64_t)b * a.P + p) * a.C + c0;
      float v[8];
      load_bf16x8(a.a + off, v);
      const f32x4 g0 = *(const f32x4*)(a.gin + (int64_t)b * a.C + c0);
      const f32x4 g1 = *(const f32x4*)(a.gin + (int64_t)b * a.C + c0 + 4);
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = e < 4 ? g0[e] : g1[e - 4];
        o[e] = (bf16)(v[e] > 0.f ? g * wp : 0.f);
        acc[e] += (float)o[e];
        gw = fmaf(g, fmaxf(v[e], 0.f), gw);
      }
      *(bf16x8*)(a.out + off) = o;
    }
    // the pixel's tpp lanes (consecutive) add their channel groups
    for (int off = tpp / 2; off >= 1; off >>= 1) gw += __shfl_xor(gw, off, tpp);
    if (threadIdx.x % tpp == 0) a.e[p] = gw;
  }
  enc_block_sum(a, acc, c0, pix, ppi, a.C, a.db, nullptr);
}

}  // namespace siren
