// siren_adam.hip — the Adam update of training.py:29,95 (torch.optim.Adam defaults, non-capturable
// foreach path on GPU) as ONE launch over every parameter tensor.
//
// Per element, in the order of torch's _multi_tensor_adam (fp32 "opmath", host scalars cast to
// float): g = grad (negated if maximize) (+ wd * param); m = lerp(m, g, 1 - beta1);
// v = v * beta2; v = v + (1 - beta2) * (g * g); d = sqrt(v) / bc2_sqrt + eps;
// param = param + step * (m / d), step = -lr / (1 - beta1^t), bc2_sqrt = sqrt(1 - beta2^t).
#include "siren_common.h"

namespace siren {

struct AdamArgs {
  float* param[SIREN_ADAM_MAX_TENSORS];
  const float* grad[SIREN_ADAM_MAX_TENSORS];
  float* exp_avg[SIREN_ADAM_MAX_TENSORS];
  float* exp_avg_sq[SIREN_ADAM_MAX_TENSORS];
  int64_t numel[SIREN_ADAM_MAX_TENSORS];
  float one_minus_beta1, beta2, one_minus_beta2, eps, weight_decay, step, bc2_sqrt;
  const float* dev;  // null, or device {step, bc2_sqrt} (graph-captured steps)
  double* steps;     // null, or one step counter per workgroup (graph-captured steps, table form)
  const float* table;
  int64_t table_n;
  int maximize;
};

// graph mode, table form: t += 1, out = the host-computed {step, bc2_sqrt} of step t (the last
// entry past the table's end: the host ends it where both bias corrections have reached 1)
__global__ void adam_scalars_table_kernel(double* t, const float* table, int64_t n, float* out) {
  const double tt = *t + 1.0;
  *t = tt;
  int64_t k = (int64_t)tt - 1;
  k = k < 0 ? 0 : k >= n ? n - 1 : k;
  out[0] = table[2 * k];
  out[1] = table[2 * k + 1];
}

__global__ void adam_scalars_kernel(double* t, double lr, double beta1, double beta2, float* out) {
  const double tt = *t + 1.0;
  *t = tt;
  out[0] = (float)((lr / (1.0 - pow(beta1, tt))) * -1.0);
  out[1] = (float)sqrt(1.0 - pow(beta2, tt));
}

DEV float torch_lerp(float self, float end, float w) {
  return fabsf(w) < 0.5f ? self + w * (end - self) : end - (end - self) * (1.f - w);
}

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  const int t = blockIdx.y;
  const int64_t n = a.numel[t];
  float* p = a.param[t];
  const float* gr = a.grad[t];
  float* m = a.exp_avg[t];
  float* v = a.exp_avg_sq[t];
  float step = a.dev ? a.dev[0] : a.step;
  float bc2_sqrt = a.dev ? a.dev[1] : a.bc2_sqrt;
  // table form: this workgroup's own counter (no other workgroup touches it, so the read-advance-
  // write needs no ordering between workgroups; the scalars kernel's launch is folded in here)
  const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
  double tnew = 0.0;
  if (a.steps) {
    tnew = a.steps[blk] + 1.0;
    int64_t k = (int64_t)tnew - 1;
    k = k < 0 ? 0 : k >= a.table_n ? a.table_n - 1 : k;
    step = a.table[2 * k];
    bc2_sqrt = a.table[2 * k + 1];
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float g = gr[i];
    if (a.maximize) g = -g;
    const float pv = p[i];
    if (a.weight_decay != 0.f) g = g + a.weight_decay * pv;
    const float mv = torch_lerp(m[i], g, a.one_minus_beta1);
    float vv = v[i] * a.beta2;
    vv = vv + a.one_minus_beta2 * (g * g);
    float d = sqrtf(vv) / bc2_sqrt;
    d = d + a.eps;
    m[i] = mv;
    v[i] = vv;
    p[i] = pv + step * (mv / d);
  }
  if (a.steps) {
    __syncthreads();  // every thread has read the counter
    if (threadIdx.x == 0) a.steps[blk] = tnew;
  }
}

}  // namespace siren
