// siren_loss.hip — the k-space weighted SSE of image_mse (loss_functions.py:66-101) on gfx950:
//   forward : d = m (pred - tgt), loss = w sum d^2           (one launch, deterministic)
//   backward: dpred = m (d (g 2 w))                           (one launch; g = upstream scalar)
// The mask m (the high-frequency mask of utils.py:25-40, or none) broadcasts over the leading
// dimensions: element e uses m[e % mask_n]. Replaces the subtract / dot / scale / scale / multiply
// chain of the autograd path (six small launches) with two.
#include "siren_common.h"

namespace siren {

constexpr int SSE_THREADS = 256;
constexpr int SSE_MAX_BLOCKS = 1024;

struct SseFwdArgs {
  const float* pred;
  const float* tgt;
  const float* mask;   // null: no mask
  float* d;            // [n] m (pred - tgt), kept for the backward
  float* loss;         // [1]
  float* partial;      // [SSE_MAX_BLOCKS] per-block sums (workspace)
  unsigned* counter;   // zero between launches (the last block resets it)
  int64_t n, mask_n;
  float weight;
};

// Per-thread sums over a fixed grid-stride order, a fixed-order block tree, and the last block
// to finish adds the block sums in index order: the result does not depend on scheduling.
//
// Hand-off of the block sums (MI355X_MICROARCH.md, "Valid forms", the first row of the table of
// hand-offs measured with sc1 loads in place of the acquire). Every atomic below is RELAXED at
// agent scope; the ordering comes from the hardware path, not from the C++ memory model:
//   producer: one lane per block stores its sum write-through (relaxed agent-scope store =
//             global_store sc1), drains it with an explicit s_waitcnt vmcnt(0) (inline asm, so the
//             compiler cannot drop it), then takes a ticket with one agent-scope atomic add;
//   consumer: the block whose add returned gridDim.x - 1 reads every sum with sc1 loads (relaxed
//             agent-scope loads = global_load sc1, served from L2, never from a stale L1).
// This avoids the L2 write-back / invalidate of acq_rel fences (several us per launch). The
// partial/counter workspace is per (device, stream) on the host side, so two launches never share
// it concurrently.
__global__ __launch_bounds__(SSE_THREADS) void sse_fwd_kernel(SseFwdArgs a) {
  __shared__ float red[SSE_THREADS / 64];
  __shared__ unsigned ticket;
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * SSE_THREADS;
  const int64_t tid0 = (int64_t)blockIdx.x * SSE_THREADS + threadIdx.x;
  // 16-byte groups when every pointer and the mask period allow it, then the scalar tail
  const bool vec = ((((uintptr_t)a.pred | (uintptr_t)a.tgt | (uintptr_t)a.d | (uintptr_t)a.mask) & 15) == 0) &&
                   (!a.mask || a.mask_n % 4 == 0);
  const int64_t n4 = vec ? a.n / 4 : 0;
  for (int64_t q = tid0; q < n4; q += stride) {
    f32x4 v = ((const f32x4*)a.pred)[q] - ((const f32x4*)a.tgt)[q];
    if (a.mask) v = *(const f32x4*)(a.mask + (4 * q) % a.mask_n) * v;
    ((f32x4*)a.d)[q] = v;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = fmaf(v[j], v[j], acc);
  }
  for (int64_t e = 4 * n4 + tid0; e < a.n; e += stride) {
    float v = a.pred[e] - a.tgt[e];
    if (a.mask) v = a.mask[e % a.mask_n] * v;
    a.d[e] = v;
    acc = fmaf(v, v, acc);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < SSE_THREADS / 64; ++w) s += red[w];
    // hand-off without an L2 write-back (MI355X_MICROARCH.md, inter-workgroup visibility, first
    // form): write-through (sc1) store of the block sum, drained, then one agent-scope add; the
    // block whose add comes last reads every sum with sc1 loads
    __hip_atomic_store(a.partial + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ticket = __hip_atomic_fetch_add(a.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (ticket != gridDim.x - 1) return;
  // last block: thread t adds block sums t, t + 256, ... in order, then the same fixed tree
  float s = 0.f;
  for (unsigned b = threadIdx.x; b < gridDim.x; b += SSE_THREADS)
    s += __hip_atomic_load(a.partial + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s = wave_sum(s);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < SSE_THREADS / 64; ++w) tot += red[w];
    a.loss[0] = tot * a.weight;
    __hip_atomic_store(a.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

struct SseBwdArgs {
  const float* d;
  const float* mask;
  const float* g;      // [1] upstream gradient of the loss
  float* out;          // [n]
  int64_t n, mask_n;
  float scale;         // 2 w
};

__global__ __launch_bounds__(SSE_THREADS) void sse_bwd_kernel(SseBwdArgs a) {
  const float k = a.g[0] * a.scale;
  const int64_t stride = (int64_t)gridDim.x * SSE_THREADS;
  const int64_t tid0 = (int64_t)blockIdx.x * SSE_THREADS + threadIdx.x;
  const bool vec = ((((uintptr_t)a.d | (uintptr_t)a.out | (uintptr_t)a.mask) & 15) == 0) &&
                   (!a.mask || a.mask_n % 4 == 0);
  const int64_t n4 = vec ? a.n / 4 : 0;
  for (int64_t q = tid0; q < n4; q += stride) {
    f32x4 v = ((const f32x4*)a.d)[q] * k;
    if (a.mask) v = *(const f32x4*)(a.mask + (4 * q) % a.mask_n) * v;
    ((f32x4*)a.out)[q] = v;
  }
  for (int64_t e = 4 * n4 + tid0; e < a.n; e += stride) {
    float v = a.d[e] * k;
    if (a.mask) v = a.mask[e % a.mask_n] * v;
    a.out[e] = v;
  }
}

}  // namespace siren
