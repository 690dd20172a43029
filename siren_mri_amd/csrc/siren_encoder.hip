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
//   enc_bias_relu    y = relu(y + cb)                                       (conv bias + ReLU)
//   enc_res_fwd      out = relu(relu(a + cb) + x)                           (res block tail)
//   enc_res_bwd      s = (g1 [+ g2]) * (out > 0), ga = s * (a + cb > 0), db[c] = sum_p ga
//   enc_pixfc_fwd    e[b][c] = sum_p relu(a[b][p][c] + cb[c]) w[p] + bias   (relu_2 + fc over pixels)
//   enc_pixfc_bwd    ga[b][p][c] = (a + cb > 0) g[b][c] w[p], db[c] = sum ga, gw[p] = sum_bc g relu(a + cb)
//
// The convolutions run without their bias (MIOpen adds it as a separate pass over the plane); cb
// is added here with the same bf16 rounding.
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
constexpr int ENC_U = 4;  // pixels per thread per iteration in the gradient passes
constexpr int ENC_UB = 8;  // images per thread per iteration in enc_pixfc_bwd_kernel

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
  const bf16* cb;     // [C] bias of the convolution that produced `a` (or y for bias_relu), or null:
                      // the pre-activation is bf16(a + cb[c]), the conv + bias-add chain's rounding
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

// the thread's 8 channel biases (zeros without a bias)
DEV void load_bias8(const bf16* cb, int c0, float (&b)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) b[e] = cb ? (float)cb[c0 + e] : 0.f;
}

// bf16(v + b): the separate bias add after a bias-free convolution
DEV void add_bias8(float (&v)[8], const float (&b)[8], bool on) {
  if (on) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)(bf16)(v[e] + b[e]);
  }
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
  // hand-off without an L2 write-back (siren_loss.hip, sse_fwd_kernel): write-through (relaxed
  // agent-scope = sc1) stores of the block's row drained by every writing lane, a barrier, then one
  // relaxed agent-scope ticket; the last block reads the rows with sc1 loads
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ unsigned last;
  __syncthreads();
  if (tid == 0) last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nblk - 1;
  __syncthreads();
  if (!last) return;
  // The rows are read 32 loads at a time before any is added (a chain of single sc1 loads made
  // this tail 0.2-0.5 ms; 8 at a time still left 64 load latencies in a row for 1,024 blocks), in a
  // fixed order: deterministic.
  auto ld = [](const float* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto sum_rows = [&](const float* src, unsigned b0, unsigned b1, int64_t stride) {
    float s = 0.f;
    unsigned b = b0;
    for (; b + 32 <= b1; b += 32) {
      float v[32];
#pragma unroll
      for (int k = 0; k < 32; ++k) v[k] = ld(src + (int64_t)(b + k) * stride);
#pragma unroll
      for (int k = 0; k < 32; ++k) s += v[k];
    }
    for (; b + 8 <= b1; b += 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ld(src + (int64_t)(b + k) * stride);
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; b < b1; ++b) s += ld(src + (int64_t)b * stride);
    return s;
  };
  if (ncol == nc) {
    // 256 / C threads per column, each a contiguous range of block rows, then those ranges in order
    const int tpc = 256 / nc, c = tid % nc, q = tid / nc;
    const unsigned per = (nblk + tpc - 1) / tpc;
    const unsigned b0 = q * per < nblk ? q * per : nblk, b1 = b0 + per < nblk ? b0 + per : nblk;
    const float s = sum_rows(a.part + c, b0, b1, nc);
    __syncthreads();
    red[tid] = s;
    __syncthreads();
    if (tid < nc) {
      float t = 0.f;
      for (int k = 0; k < tpc; ++k) t += red[k * nc + tid];
      dst[tid] = addend ? t + *addend : t;
    }
  } else {
    // pixfc_fwd: column k = (image, channel) sums that image's gridDim.x block rows
    for (int k = tid; k < ncol; k += 256) {
      const int img = k / nc, c = k - img * nc;
      const float s = sum_rows(a.part + (int64_t)img * gridDim.x * nc + c, 0, gridDim.x, nc);
      dst[k] = addend ? s + *addend : s;
    }
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
  // ENC_U pixels per thread per iteration, every load issued before the first store (more bytes
  // in flight: one pixel per iteration ran at ~3 TB/s)
  for (int64_t p = p0 + pix; p < p1; p += ENC_U * ppi) {
    float g[ENC_U][8], m[ENC_U][8];
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      const int64_t q = p + u * ppi;
      if (q < p1) {
        const int64_t off = q * a.C + c0;
        load_bf16x8(a.g1 + off, g[u]);
        if (a.g2) {
          float g2[8];
          load_bf16x8(a.g2 + off, g2);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[u][e] += g2[e];
        }
        load_bf16x8(a.y + off, m[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      const int64_t q = p + u * ppi;
      if (q < p1) {
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[e] = (bf16)(m[u][e] > 0.f ? g[u][e] : 0.f);
          acc[e] += (float)o[e];
        }
        *(bf16x8*)(a.out + q * a.C + c0) = o;
      }
    }
  }
  if (a.db) enc_block_sum(a, acc, c0, pix, ppi, a.C, a.db, nullptr);
}

// out = relu(relu(bf16(a + cb)) + x), x = g1 (the block input)
__global__ __launch_bounds__(256) void enc_res_fwd_kernel(EncArgs a) {
  const int64_t n8 = a.P * a.C / 8;
  // the grid stride is a multiple of C / 8, so a thread's channel group is fixed
  const int c0 = (int)((8 * ((int64_t)blockIdx.x * 256 + threadIdx.x)) % a.C);
  float bb[8];
  load_bias8(a.cb, c0, bb);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8], x[8];
    load_bf16x8(a.a + 8 * i, v);
    add_bias8(v, bb, a.cb != nullptr);
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

// y = relu(bf16(y + cb)) in place (a bias-free convolution's bias add and its ReLU, one pass)
__global__ __launch_bounds__(256) void enc_bias_relu_kernel(EncArgs a) {
  const int64_t n8 = a.P * a.C / 8;
  const int c0 = (int)((8 * ((int64_t)blockIdx.x * 256 + threadIdx.x)) % a.C);
  float bb[8];
  load_bias8(a.cb, c0, bb);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8];
    load_bf16x8(a.out + 8 * i, v);
    add_bias8(v, bb, a.cb != nullptr);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)fmaxf(v[e], 0.f);
    *(bf16x8*)(a.out + 8 * i) = o;
  }
}

// s = (g1 [+ g2]) * (out > 0) -> out (the skip's gradient); ga = s * (a > 0) -> out2; db = sum ga
__global__ __launch_bounds__(256) void enc_res_bwd_kernel(EncArgs a) {
  const int tpp = a.C / 8, ppi = 256 / tpp;
  const int pix = threadIdx.x / tpp, c0 = 8 * (threadIdx.x % tpp);
  const int64_t p0 = (int64_t)blockIdx.x * a.chunk;
  const int64_t p1 = p0 + a.chunk < a.P ? p0 + a.chunk : a.P;
  float acc[8], bb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  load_bias8(a.cb, c0, bb);
  for (int64_t p = p0 + pix; p < p1; p += ENC_U * ppi) {
    float g[ENC_U][8], mo[ENC_U][8], ma[ENC_U][8];
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      const int64_t q = p + u * ppi;
      if (q < p1) {
        const int64_t off = q * a.C + c0;
        load_bf16x8(a.g1 + off, g[u]);
        if (a.g2) {
          float g2[8];
          load_bf16x8(a.g2 + off, g2);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[u][e] += g2[e];
        }
        load_bf16x8(a.y + off, mo[u]);
        load_bf16x8(a.a + off, ma[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      const int64_t q = p + u * ppi;
      if (q < p1) {
        add_bias8(ma[u], bb, a.cb != nullptr);
        bf16x8 sk, ga;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          sk[e] = (bf16)(mo[u][e] > 0.f ? g[u][e] : 0.f);
          ga[e] = ma[u][e] > 0.f ? sk[e] : (bf16)0.f;
          acc[e] += (float)ga[e];
        }
        const int64_t off = q * a.C + c0;
        *(bf16x8*)(a.out + off) = sk;
        *(bf16x8*)(a.out2 + off) = ga;
      }
    }
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
  float acc[8], bb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  load_bias8(a.cb, c0, bb);
  // ENC_U pixels' loads in flight before the first is used (one at a time ran at ~1.9 TB/s); the
  // sums keep the pixel order
  for (int64_t p = p0 + pix; p < p1; p += ENC_U * ppi) {
    float v[ENC_U][8], wp[ENC_U];
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      const int64_t q = p + u * ppi;
      if (q < p1) {
        load_bf16x8(src + q * a.C + c0, v[u]);
        wp[u] = a.w[q];
      }
    }
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      if (p + u * ppi < p1) {
        add_bias8(v[u], bb, a.cb != nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(fmaxf(v[u][e], 0.f), wp[u], acc[e]);
      }
    }
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
  float acc[8], bb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  load_bias8(a.cb, c0, bb);
  for (int64_t p = p0 + pix; p < p1; p += ppi) {
    const float wp = a.w[p];
    float gw = 0.f;
    // ENC_UB images' loads issued before the first store (a store to out may alias the next load
    // for the compiler: one image at a time left every load's latency exposed, ~1.2 TB/s); the
    // sums keep the image order
    for (int b0 = 0; b0 < a.B; b0 += ENC_UB) {
      float v[ENC_UB][8];
      f32x4 g0[ENC_UB], g1[ENC_UB];
#pragma unroll
      for (int u = 0; u < ENC_UB; ++u) {
        const int b = b0 + u;
        if (b < a.B) {
          load_bf16x8(a.a + ((int64_t)b * a.P + p) * a.C + c0, v[u]);
          g0[u] = *(const f32x4*)(a.gin + (int64_t)b * a.C + c0);
          g1[u] = *(const f32x4*)(a.gin + (int64_t)b * a.C + c0 + 4);
        }
      }
#pragma unroll
      for (int u = 0; u < ENC_UB; ++u) {
        const int b = b0 + u;
        if (b < a.B) {
          add_bias8(v[u], bb, a.cb != nullptr);
          bf16x8 o;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float g = e < 4 ? g0[u][e] : g1[u][e - 4];
            o[e] = (bf16)(v[u][e] > 0.f ? g * wp : 0.f);
            acc[e] += (float)o[e];
            gw = fmaf(g, fmaxf(v[u][e], 0.f), gw);
          }
          *(bf16x8*)(a.out + ((int64_t)b * a.P + p) * a.C + c0) = o;
        }
      }
    }
    // the pixel's tpp lanes (consecutive) add their channel groups
    for (int off = tpp / 2; off >= 1; off >>= 1) gw += __shfl_xor(gw, off, tpp);
    if (threadIdx.x % tpp == 0) a.e[p] = gw;
  }
  enc_block_sum(a, acc, c0, pix, ppi, a.C, a.db, nullptr);
}

// The encoder's per-step operand preparation in one launch (round 5): every convolution's fp32
// filter -> its bf16 channels-last copy [co][kh][kw][ci], the flipped / transposed bf16 filter of
// its input gradient [ci][k - 1 - kh][k - 1 - kw][co] (when asked), and its bias -> bf16; the
// casts round to nearest even as torch's .to(torch.bfloat16). Replaces ~50 cast / flip / copy
// launches per C4 step.
constexpr int ENC_PREP_MAX = 32;
struct EncPrepSeg {
  const float* w;
  const float* b;
  bf16* wb;
  bf16* wf;  // or null
  bf16* bb;  // or null
  int co, ci, k;
  int64_t s_co, s_ci, s_kh, s_kw;  // element strides of w
  int64_t begin;                   // first flat index of this segment (filter elements, then bias)
};
struct EncPrepArgs {
  EncPrepSeg seg[ENC_PREP_MAX];
  int nseg;
  int64_t total;
};
__global__ __launch_bounds__(256) void enc_prep_kernel(EncPrepArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.total) return;
  int si = 0;
  while (si + 1 < a.nseg && i >= a.seg[si + 1].begin) ++si;
  const EncPrepSeg& g = a.seg[si];
  const int64_t e = i - g.begin;
  const int64_t nw = (int64_t)g.co * g.ci * g.k * g.k;
  if (e < nw) {
    // e in channels-last order: ((co k + kh) k + kw) ci + ci
    const int ci = (int)(e % g.ci);
    const int kw = (int)((e / g.ci) % g.k);
    const int kh = (int)((e / ((int64_t)g.ci * g.k)) % g.k);
    const int co = (int)(e / ((int64_t)g.ci * g.k * g.k));
    const bf16 v = (bf16)g.w[co * g.s_co + ci * g.s_ci + kh * g.s_kh + kw * g.s_kw];
    g.wb[e] = v;
    if (g.wf) g.wf[(((int64_t)ci * g.k + (g.k - 1 - kh)) * g.k + (g.k - 1 - kw)) * g.co + co] = v;
  } else if (g.bb && e < nw + g.co) {
    g.bb[e - nw] = (bf16)g.b[e - nw];
  }
}

// Sum of squares over a list of fp32 tensors (loss_functions.py:279-287 hypo_weight_loss's
// sum of torch.sum(w ** 2)) and its gradient 2 g w, each one launch over every tensor (round 5;
// ~45 pow / reduce / add / mul launches per C4 step before). Deterministic: fixed per-thread
// order, an LDS tree per block, the block partials added in block order by the last block.
constexpr int SUMSQ_MAX = 32;
constexpr int SUMSQ_CHUNK = 4096;  // elements per block
struct SumsqArgs {
  const float* src[SUMSQ_MAX];
  float* dst[SUMSQ_MAX];     // backward: 2 g src
  int64_t begin[SUMSQ_MAX + 1];
  int n;
  float* part;               // forward: [blocks] partials
  unsigned* counter;         // forward: zero between launches (the last block resets it)
  float* out;                // forward: the sum
  const float* g;            // backward: upstream gradient (device scalar)
};
DEV int sumsq_seg(const SumsqArgs& a, int64_t i) {
  int s = 0;
  while (s + 1 < a.n && i >= a.begin[s + 1]) ++s;
  return s;
}
__global__ __launch_bounds__(256) void sumsq_fwd_kernel(SumsqArgs a) {
  __shared__ float red[256];
  __shared__ bool last;
  const int64_t base = (int64_t)blockIdx.x * SUMSQ_CHUNK;
  float acc = 0.f;
  for (int k = 0; k < SUMSQ_CHUNK / 256; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    if (i < a.begin[a.n]) {
      const int s = sumsq_seg(a, i);
      const float v = a.src[s][i - a.begin[s]];
      acc = fmaf(v, v, acc);
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  // hand-off as enc_block_sum's: a write-through partial, drained, then one relaxed ticket
  if (threadIdx.x == 0) __hip_atomic_store(a.part + blockIdx.x, red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) last = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  // the last block: thread t adds partials t, t + 256, ... in order, then the same LDS tree
  float s = 0.f;
  for (unsigned b = threadIdx.x; b < gridDim.x; b += 256)
    s += __hip_atomic_load(a.part + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *a.out = red[0];
    __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__global__ __launch_bounds__(256) void sumsq_bwd_kernel(SumsqArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.begin[a.n]) return;
  const int s = sumsq_seg(a, i);
  const int64_t e = i - a.begin[s];
  a.dst[s][e] = 2.f * *a.g * a.src[s][e];
}

}  // namespace siren
