/*
 * siren_mri_amd.h — C ABI of the MI355X (gfx950) SIREN SineLayer-stack library.
 *
 * The reference (jonbmartin/siren_mri) has no native ABI: its hot path is the Python
 * module stack modules.SingleBVPNet -> FCBlock -> MetaSequential(BatchLinear, Sine)
 * (modules.py:11-170) driven by training.train (training.py:19-146). This header is the
 * boundary the build puts underneath that Python API. Each entry point states which
 * reference interface it replaces.
 *
 * Conventions
 *  - Plain pointers to DEVICE memory (allocated by the caller, e.g. the PyTorch caching
 *    allocator); sizes in elements unless a name says bytes.
 *  - Row-major, contiguous tensors. "rows" = coordinates (batch * points).
 *  - Every call is asynchronous on `stream` (a hipStream_t passed as void*); no call
 *    allocates, frees or synchronises, so every call can be captured into a hipGraph.
 *  - Return value: 0 on success, a negative SIREN_E* code otherwise; the message is
 *    available from siren_last_error() (thread-local). No C++ exception crosses the ABI.
 */
#ifndef SIREN_MRI_AMD_H
#define SIREN_MRI_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIREN_MAX_LAYERS 16

/* Arithmetic modes of the layer stack. */
#define SIREN_PREC_F32  0 /* fp32 operands, exact-fp32 MFMA (v_mfma_f32_32x32x2_f32), libm sin/cos  */
#define SIREN_PREC_BF16 1 /* bf16 operands, fp32 accumulate, 16-bit phase storage, v_sin/v_cos     */
#define SIREN_PREC_F64  2 /* IEEE double throughout (siren_mlp64_*: double_precision=True)         */

/* Error codes. */
#define SIREN_OK 0
#define SIREN_EINVAL -1   /* unsupported shape / argument                       */
#define SIREN_ELAUNCH -2  /* a HIP launch failed (hipGetLastError)             */
#define SIREN_ENOSPACE -3 /* workspace or saved buffer too small               */

/*
 * Description of one SIREN MLP (an FCBlock with nonlinearity='sine').
 * Replaces modules.FCBlock.__init__/forward (modules.py:45-97) and the param routing of
 * torchmeta MetaSequential/get_subdict (torchmeta/modules/container.py:9-19, utils.py:4-11).
 *
 *   dims[0]           in_features (coords, or 2m Fourier features)
 *   dims[1..L-1]      hidden widths (multiples of 32; the MFMA layers need multiples of 32)
 *   dims[L]           out_features
 *   layer l computes  z = x_l W_l^T + b_l  (modules.py:25-26), then
 *                     h = sin(w0 * z)      (modules.py:38) for every layer except the last
 *                     one when outermost_linear != 0 (modules.py:78-79).
 *   weights_batched   0: weight[l] is [dims[l+1], dims[l]], shared by all rows
 *                     1: weight[l] is [batch, dims[l+1], dims[l]] (hypernetwork output,
 *                        meta_modules.py:42-54); bias[l] is then [batch, dims[l+1]]
 *   rows_per_batch    points per batch element; x is [batch * rows_per_batch, dims[0]]
 */
typedef struct siren_mlp_desc {
  int32_t num_layers;
  int32_t dims[SIREN_MAX_LAYERS + 1];
  int32_t outermost_linear;
  int32_t prec;
  int32_t weights_batched;
  float w0;
  int64_t batch;
  int64_t rows_per_batch;
  const float* weight[SIREN_MAX_LAYERS];
  const float* bias[SIREN_MAX_LAYERS];
  /* Fourier-feature input (features.py:21-41, applied by training.py:61-64 before the model)
   * computed in the first layer instead of materialised: when ff_B is non-NULL, x holds ff_in raw
   * coordinates per row and the first layer's dims[0] = 2m inputs are
   * cat(sin(2 pi x B), cos(2 pi x B)) with B = ff_B [ff_in][m]. bf16 mode, the register-resident
   * forward's wide first layer (dims[0] even, 6..16), ff_in 1..4; no input gradient (dx NULL). */
  const float* ff_B;
  int32_t ff_in;
} siren_mlp_desc;

/* Validates a descriptor; returns SIREN_OK or SIREN_EINVAL (message in siren_last_error). */
int siren_mlp_check(const siren_mlp_desc* d);

/*
 * fp64 stack: the reference's double_precision=True training (training.py:56-58, the model cast
 * to float64 with .double()). prec = SIREN_PREC_F64; weight[l] / bias[l] point to double arrays
 * and x, y, dy, dW, db, dx are double; any widths (dims 1..65536), shared or batched weights, sine
 * or linear output layer; no Fourier-feature input. Forward saves Z (the pre-activation, fp64) of
 * every sine layer in `saved` (siren_mlp64_saved_bytes; NULL for inference); the backward is
 * first-order (dW, db of every layer, dx when non-NULL), weight-gradient row reductions added
 * in a fixed split order (deterministic). Replaces FCBlock.forward / its autograd backward in
 * float64 (modules.py:16-27, 35-38, 92-97).
 */
int64_t siren_mlp64_saved_bytes(const siren_mlp_desc* d);
int64_t siren_mlp64_workspace_bytes(const siren_mlp_desc* d);
int siren_mlp64_forward(const siren_mlp_desc* d, const double* x, double* y, void* saved, int64_t saved_bytes,
                        void* workspace, int64_t workspace_bytes, void* stream);
int siren_mlp64_backward(const siren_mlp_desc* d, const double* x, const double* dy, const void* saved,
                         int64_t saved_bytes, void* workspace, int64_t workspace_bytes, double* const* dW,
                         double* const* db, double* dx, void* stream);

/* Bytes of the per-call "saved" buffer (the activations kept between forward and
 * backward: one phase tensor per sine layer). */
int64_t siren_mlp_saved_bytes(const siren_mlp_desc* d);

/* Bytes of scratch workspace a forward or backward call needs. */
int64_t siren_mlp_workspace_bytes(const siren_mlp_desc* d);

/*
 * Forward pass: y[rows, dims[L]] = FCBlock(x).
 * Replaces SingleBVPNet.forward -> FCBlock.forward (modules.py:146-164, 92-97) and the
 * per-layer BatchLinear.forward + Sine.forward (modules.py:16-27, 35-38).
 * `saved` may be NULL (inference: nothing is kept for backward).
 */
int siren_mlp_forward(const siren_mlp_desc* d, const float* x, float* y, void* saved,
                      int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                      void* stream);

/*
 * Backward pass from dy = dL/dy. Writes (overwrites) dweight[l], dbias[l] (same shapes as
 * weight[l], bias[l]) and, if dx != NULL, dx = dL/dx [rows, dims[0]].
 * Replaces the autograd MmBackward/AddBackward/MulBackward/SinBackward chain that
 * training.py:91 (train_loss.backward()) runs through the reference modules.
 */
int siren_mlp_backward(const siren_mlp_desc* d, const float* x, const float* dy,
                       const void* saved, int64_t saved_bytes, void* workspace,
                       int64_t workspace_bytes, float* const* dweight, float* const* dbias,
                       float* dx, void* stream);

/*
 * Forward with a fused image loss (replaces, in one launch, the SIREN
 * forward (modules.py:146-164), DataConsistencyInKspace (data_consistency.py:32-48) and
 * image_mse's masked k-space SSE (loss_functions.py:66-101, utils.py:25-40)). Rows are the
 * SIREN's [batch * rows_per_batch, O] outputs; for each element p = DC(y) (when k0 is given:
 * (1 - mask) y + mask k0, or the noisy form), d = hf (p - target) (hf indexed by the row within its
 * weight set), loss = weight * sum d^2 (deterministic order), y_dc = p and
 * dy = 2 weight hf d dDC/dy — dL/dy for a unit upstream gradient, which siren_mlp_backward_ex
 * scales by the device scalar dy_scale (the loss's upstream gradient) inside its output-layer
 * kernels. Where the loss runs (siren_mlp_loss_check): the bf16 register-resident forward's output
 * epilogue (its shapes with 3+ layers; one output for 1..4 inputs), or the per-layer path's output
 * kernel — fp32 mode (the reference's arithmetic) and bf16 shapes outside the register forward,
 * up to 8 outputs. outermost_linear only.
 */
typedef struct siren_loss_desc {
  const float* target;  /* [B * N, O]                                                  */
  const float* k0;      /* [B, O, N] k-space planes (NCHW), or NULL (no data consistency) */
  const float* mask;    /* [B, O, N] sampling mask, or NULL                             */
  const float* hf;      /* [N] high-frequency mask, or NULL                             */
  int64_t hf_len;       /* entries of hf (= rows_per_batch)                             */
  float noise;          /* DataConsistencyInKspace noise_lvl (0: noiseless)              */
  float weight;         /* image_mse's 1 / 128^2                                        */
  float* y_dc;          /* [B * N, O] DC(y) (with k0), or NULL                          */
  float* dy;            /* [B * N, O] dL/dy for a unit upstream gradient                */
  float* loss;          /* [1]                                                          */
  void* loss_workspace; /* siren_sse_workspace_bytes(), zero-initialised once, one per stream */
  int64_t loss_workspace_bytes;
} siren_loss_desc;
int siren_mlp_loss_check(const siren_mlp_desc* d, const siren_loss_desc* l);
int siren_mlp_forward_loss(const siren_mlp_desc* d, const siren_loss_desc* l, const float* x, float* y,
                           void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                           void* stream);
/* siren_mlp_backward with dL/dy = dy * (*dy_scale) (dy_scale: device pointer, NULL = 1). */
int siren_mlp_backward_ex(const siren_mlp_desc* d, const float* x, const float* dy, const float* dy_scale,
                          const void* saved, int64_t saved_bytes, void* workspace,
                          int64_t workspace_bytes, float* const* dweight, float* const* dbias,
                          float* dx, void* stream);

/*
 * Analytic spatial derivatives of the SIREN output w.r.t. its input (tangent streams carried
 * through the fused layers instead of an autograd graph). Replaces diff_operators.gradient
 * (diff_operators.py:39-43: grad[n][k] = sum_c dy_c/dx_k) and, with order 2, laplace
 * (diff_operators.py:27-36: lap[n] = sum_c sum_k d2y_c/dx_k2). Needs outermost_linear and
 * in_features <= 4. `saved` (may be NULL for order 2 / inference) keeps the per-layer phases and
 * tangents for siren_jvp_backward.
 * `order` selects the derivative (the same tangent streams): SIREN_JVP_GRADIENT writes
 * grad [rows, in_features]; SIREN_JVP_LAPLACE writes lap [rows] (grad is scratch of the gradient's
 * size); SIREN_JVP_JACOBIAN writes the per-channel Jacobian grad [rows, out_features, in_features]
 * (diff_operators.jacobian, diff_operators.py:46-59; and gradient() with grad_outputs that vary
 * across output channels, or any autograd double backward through the SIREN forward).
 */
#define SIREN_JVP_GRADIENT 1
#define SIREN_JVP_LAPLACE 2
#define SIREN_JVP_JACOBIAN 3
int64_t siren_jvp_saved_bytes(const siren_mlp_desc* d, int order);
int64_t siren_jvp_workspace_bytes(const siren_mlp_desc* d, int order);
int siren_jvp_forward(const siren_mlp_desc* d, int order, const float* x, float* grad, float* lap,
                      void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                      void* stream);

/*
 * Backward of a loss on the gradient (order 1), the Laplacian (order 2) or the Jacobian (order 3):
 * from dgrad = dL/dgrad [rows, in_features] (order 1), dL/dlap [rows] (order 2) or
 * dL/djac [rows, out_features, in_features] (order 3) writes
 * dweight/dbias (overwrite; the output bias gets zeros: it does not reach either derivative)
 * and, if dx != NULL, dx. These are the double / triple backward passes that
 * loss_functions.gradients_mse (loss_functions.py:330-335) and laplace_mse (:350-355) run
 * through autograd. `saved` must come from siren_jvp_forward with the same order.
 */
int siren_jvp_backward(const siren_mlp_desc* d, int order, const float* x, const float* dgrad,
                       const void* saved, int64_t saved_bytes, void* workspace,
                       int64_t workspace_bytes, float* const* dweight, float* const* dbias,
                       float* dx, void* stream);
/* The same two with `primal`: the saved buffer of a plain siren_mlp_forward of this stack on this x
 * (fp32 mode, outermost_linear; primal_bytes >= siren_mlp_saved_bytes). Its per-layer phases are the
 * primal stream, so only the tangent streams are computed (diff_operators.gradient of a model output
 * reuses the model's forward instead of repeating it); the backward reads the same phases, so
 * `primal` must stay unchanged between the two calls. NULL: as above. */
int siren_jvp_forward_ex(const siren_mlp_desc* d, int order, const float* x, float* grad, float* lap,
                         void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                         const void* primal, int64_t primal_bytes, void* stream);
int siren_jvp_backward_ex(const siren_mlp_desc* d, int order, const float* x, const float* dgrad,
                          const void* saved, int64_t saved_bytes, void* workspace, int64_t workspace_bytes,
                          float* const* dweight, float* const* dbias, float* dx, const void* primal,
                          int64_t primal_bytes, void* stream);

/*
 * Optional per-kernel-class timing, for benchmarks and profiling (not thread-safe; not for use
 * under hipGraph capture). While enabled, each launch of `kernel_class` is bracketed by a
 * hipEventRecord pair on the launch's stream (at most `max_launches` launches are recorded).
 * siren_timing_collect synchronises on the recorded events and returns the summed duration.
 */
#define SIREN_KCLASS_NONE 0
#define SIREN_KCLASS_FWD_GEMM 1 /* hidden-layer forward GEMM + bias/w0/phase epilogue     */
#define SIREN_KCLASS_DX_GEMM 2  /* hidden-layer input-gradient GEMM + cos-weighted epilogue */
#define SIREN_KCLASS_DW_GEMM 3  /* hidden-layer weight-gradient split-K GEMM               */
#define SIREN_KCLASS_FWD_FUSED 4 /* whole forward in one kernel (bf16, narrow in/out layers) */
#define SIREN_KCLASS_BWD_FUSED 5 /* a middle layer's input + weight gradients in one kernel   */
#define SIREN_KCLASS_DX_RING 6   /* dx_ring_bf16_kernel, middle layer                         */
#define SIREN_KCLASS_DW_RING 7   /* dw_ring_bf16_kernel, middle layer                         */
#define SIREN_KCLASS_DX_RING_BOT 8 /* dx_ring_bf16_kernel with the first layer folded in      */
#define SIREN_KCLASS_DW_RING_REC 9 /* dw_ring_bf16_kernel of layer 1 (P_0 rebuilt from x)     */
#define SIREN_KCLASS_DX_RING_TOP 10 /* dx_ring_bf16_kernel with the output layer folded in    */
#define SIREN_KCLASS_DW_RING_TOP 11 /* dw_ring_bf16_kernel with the output layer folded in    */
#define SIREN_KCLASS_PAIR_RING 12     /* pair_ring_bf16_kernel, middle layer (dx + dw roles)   */
#define SIREN_KCLASS_PAIR_RING_TOP 13 /* pair_ring_bf16_kernel, top layer + output layer        */
#define SIREN_KCLASS_PAIR_RING_BOT 14 /* pair_ring_bf16_kernel, layer 1 + first layer, P_0 rebuilt */
int siren_timing_enable(int kernel_class, int max_launches);
int siren_timing_collect(double* total_ms, int64_t* launches);
void siren_timing_disable(void);

/*
 * Adam step over up to SIREN_ADAM_MAX_TENSORS fp32 parameter tensors in one launch — the
 * optimizer of training.train (training.py:29, torch.optim.Adam with default flags). The host
 * passes the step-dependent scalars (torch's non-capturable convention):
 *   step_size = -lr / (1 - beta1^t),  bias_correction2_sqrt = sqrt(1 - beta2^t).
 * exp_avg / exp_avg_sq are updated in place, then param. amsgrad is not supported here.
 */
#define SIREN_ADAM_MAX_TENSORS 48
typedef struct siren_adam_desc {
  int32_t num_tensors;
  int32_t maximize;
  float lr, beta1, beta2, eps, weight_decay;
  float one_minus_beta1;         /* 1 - beta1, computed in double then rounded (as torch does) */
  float one_minus_beta2;         /* 1 - beta2, likewise */
  float step_size;               /* -lr / (1 - beta1^t) */
  float bias_correction2_sqrt;   /* sqrt(1 - beta2^t) */
  int64_t numel[SIREN_ADAM_MAX_TENSORS];
  float* param[SIREN_ADAM_MAX_TENSORS];
  const float* grad[SIREN_ADAM_MAX_TENSORS];
  float* exp_avg[SIREN_ADAM_MAX_TENSORS];
  float* exp_avg_sq[SIREN_ADAM_MAX_TENSORS];
  const float* dev_scalars;      /* NULL, or device {step_size, bias_correction2_sqrt} read by the
                                    kernel (written by siren_adam_scalars: hipGraph replays) */
  double* dev_steps;             /* NULL, or siren_adam_num_blocks(d) device step counters, all equal:
                                    each workgroup advances its own (t += 1) and reads its scalars
                                    from dev_table[t - 1] (hipGraph replays without the separate
                                    scalars launch); takes precedence over dev_scalars */
  const float* dev_table;        /* [table_n][2] {step_size, bias_correction2_sqrt} of t = 1 .. table_n,
                                    the last entry repeated past the end (as siren_adam_scalars_table) */
  int64_t table_n;
} siren_adam_desc;
int siren_adam_step(const siren_adam_desc* d, void* stream);
/* Workgroups of siren_adam_step's launch for this descriptor (the length of dev_steps). */
int64_t siren_adam_num_blocks(const siren_adam_desc* d);
/* Device-side bias corrections for graph-captured steps: *t += 1, then
 * out[0] = -(lr / (1 - beta1^t)), out[1] = sqrt(1 - beta2^t), computed in double and rounded to
 * float as the host path does (t, out: device pointers). One single-thread launch. */
int siren_adam_scalars(double* t, double lr, double beta1, double beta2, float* out, void* stream);
/* The same from a host-computed table ([n][2] {step_size, bias_correction2_sqrt} of t = 1 .. n, the
 * last entry repeated past the end): *t += 1, out = table[t - 1]. No pow in the launch. */
int siren_adam_scalars_table(double* t, const float* table, int64_t n, float* out, void* stream);

/*
 * Configs 4/5's conv encoder (modules.py:340-380, 433-450) in bf16 channels-last: the passes around
 * the (bias-free) convolutions, each one launch over a [P, C] plane (P pixels, C a power of two in
 * [8, 256]). cb is the producing convolution's bf16 bias ([C], or NULL): the pre-activation is
 * bf16(a + cb), the rounding of the conv + bias-add chain. Channel sums (db) are deterministic:
 * per-block partials in `ws` (siren_enc_workspace_bytes, zeroed once and left zeroed), added in
 * block order by the last block. g2 may be NULL.
 *   bias_relu: y = relu(bf16(y + cb)) in place                         (conv bias + ReLU)
 *   relu_bwd : out = (g1 + g2) * (y > 0) (bf16), db[c] = sum_p out     (ReLU backward + conv bias grad)
 *   res_fwd  : out = relu(relu(a + cb) + x)                            (Conv2dResBlock tail)
 *   res_bwd  : gskip = (g1 + g2) * (out > 0), ga = gskip * (a + cb > 0), db[c] = sum_p ga
 *   pixfc_fwd: e[b][c] = sum_p relu(a[b][p][c] + cb[c]) w[p] + *bias   (relu_2 + fc over pixels)
 *   pixfc_bwd: ga[b][p][c] = (a + cb > 0) g[b][c] w[p], db[c] = sum_{b,p} ga,
 *              gw[p] = sum_{b,c} g relu(a + cb)
 * (P is per image for pixfc; a is [B][P][C].) Replaces the autograd chain of ConvImgEncoder's
 * conv bias adds, ReLUs, residual adds, conv bias reductions and its Linear over the pixels.
 */
int64_t siren_enc_workspace_bytes(void);
/* Weight gradient of a 128 -> 128 channel, 5x5, stride-1, padding-2 convolution (Conv2dResBlock's,
 * modules.py:433-450) from bf16 NHWC x and dy ([N][H][W][128], W a multiple of 64) into fp32 dw
 * in the channels-last filter layout [co][kh][kw][ci]: split-K bf16-MFMA partials in ws
 * (siren_conv_wrw_workspace_bytes) added in split order (deterministic). Replaces the convolution
 * weight-gradient of the encoder's autograd chain. */
int64_t siren_conv_wrw_workspace_bytes(int N, int H, int W);
/* Forward convolution of the same shape, bf16 NHWC x [N][H][128][128] (H even) and filter w
 * [128 out][5][5][128 in] (channels-last) -> bf16 y, fp32 accumulation; with bias ([128] bf16)
 * y = bf16(bf16(acc) + bias) (then ReLU if relu), the rounding of the conv + bias-add chain. The
 * input gradient of such a convolution is this one on the flipped, transposed filter. Replaces
 * the encoder's MIOpen forward / input-gradient convolutions for this shape. */
int siren_conv_fwd_k5(const void* x, const void* w, const void* bias, int relu, void* y, int N, int H, int W, int C,
                      void* stream);
/* A residual block's second convolution with the block's tail in its epilogue (replaces
 * siren_conv_fwd_k5 + siren_enc_res_fwd, element for element): a_out = bf16(conv(x, w)) (bias-free,
 * kept for the backward), out = relu(bf16(relu(bf16(a_out + cb)) + t)), t the block input
 * (Conv2dResBlock.forward, modules.py:446-450). */
int siren_conv_fwd_k5_res(const void* x, const void* w, const void* cb, const void* t, void* a_out, void* out, int N,
                          int H, int W, int C, void* stream);
/* The input gradient of a residual-block convolution (siren_conv_fwd_k5 on the flipped, transposed
 * filter wf) with the encoder's next backward pass in its epilogue (replaces siren_conv_fwd_k5 +
 * siren_enc_relu_bwd / siren_enc_res_bwd; the arithmetic of those passes element for element):
 *   mode 1: out = bf16((g [+ g2]) * (m > 0)), db = channel sums of out        (a ReLU's backward)
 *   mode 2: out = bf16((g + g2) * (m > 0)) (skip gradient), out2 = out * (bf16(pa + cb) > 0),
 *           db = channel sums of out2                     (Conv2dResBlock's tail, modules.py:433-450)
 * with g = bf16(conv(dy, wf)). ws: N * H / 2 * 128 floats of partial sums (reduced in a fixed order
 * by a second launch: deterministic). Replaces the autograd ReLU / add backward of
 * modules.py:372-380,446-450 under the fused bf16 encoder node. */
int siren_conv_dgrad_k5_fused(int mode, const void* dy, const void* wf, const void* g2, const void* m, const void* pa,
                              const void* cb, void* out, void* out2, float* db, int N, int H, int W, int C, void* ws,
                              int64_t ws_bytes, void* stream);
int siren_conv_wrw_k5(const void* x, const void* dy, int N, int H, int W, int C, float* dw, void* ws, int64_t ws_bytes,
                      void* stream);
/* The encoder's other convolution shapes (round 5; ConvImgEncoder's cnn[0], modules.py:351 — 64 ->
 * 128 channels, 7x7 in configs 4/5 — its input gradient as a forward convolution of the flipped,
 * transposed filter, and the 3x3 forms), stride 1, 'same' padding, bf16 NHWC, fp32 accumulation:
 * filter size KS in {3, 5, 7}, CI in {2, 64, 128} input channels (2: conv_theta over the real /
 * imaginary k-space image, modules.py:359).
 *   siren_conv_fwd : y = conv(x, w) (+ bias, ReLU as siren_conv_fwd_k5); W = 128; CI 64/128: H
 *                    even, CO a multiple of 64; CI 2: CO in {32, 64, 96, 128}; w is [CO][KS][KS][CI].
 *   siren_conv_wrw : dw[CO][KS][KS][CI] (fp32) = the weight gradient of that convolution; CI 64/128:
 *                    W a multiple of 64, CO a multiple of 128 (CI 64) or 64 (CI 128); CI 2: W a
 *                    multiple of 64, CO in {32, 64, 96, 128}; split-K partials in ws
 *                    (siren_conv_wrw_ws_bytes) added in split order (deterministic).
 *   siren_conv_check: SIREN_OK when the shape (kind 0 forward, 1 weight gradient) runs natively;
 *                    the encoder falls back to MIOpen otherwise. */
int siren_conv_check(int kind, int N, int H, int W, int CI, int CO, int KS);
int siren_conv_fwd(const void* x, const void* w, const void* bias, int relu, void* y, int N, int H, int W, int CI,
                   int CO, int KS, void* stream);
int64_t siren_conv_wrw_ws_bytes(int N, int H, int W, int CI, int CO, int KS);
int siren_conv_wrw(const void* x, const void* dy, int N, int H, int W, int CI, int CO, int KS, float* dw, void* ws,
                   int64_t ws_bytes, void* stream);
/*
 * HyperNetwork heads (meta_modules.py:11-54; configs 4/5): `heads` ReLU FCBlocks (modules.py:40-119,
 * nonlinearity='relu', outermost_linear=True) on one shared latent z [rows][in_features]: per head
 * `depth` Linear + ReLU layers of width `hidden`, then a Linear to out_features[g]. Every head's layer
 * of one depth is one grouped fp32 GEMM launch (bias and ReLU in its epilogue). weight[g * 5 + d] /
 * bias[g * 5 + d] are the head's layer d (d = depth: the output layer), nn.Linear layout [out][in].
 *   forward : out[g] [rows][out_features[g]]; saved (siren_hyper_saved_bytes) keeps the ReLU outputs.
 *   backward: dW / db of every layer (same [g * 5 + d] indexing, [out][in] / [out]) and dz (the
 *             latent's gradient, summed over the heads in head order); deterministic.
 */
#define SIREN_HYPER_MAXG 32
#define SIREN_HYPER_MAXD 4
typedef struct siren_hyper_desc {
  int32_t heads, depth, rows, in_features, hidden;
  int32_t out_features[SIREN_HYPER_MAXG];
  const float* weight[SIREN_HYPER_MAXG * (SIREN_HYPER_MAXD + 1)];
  const float* bias[SIREN_HYPER_MAXG * (SIREN_HYPER_MAXD + 1)];
} siren_hyper_desc;
int64_t siren_hyper_saved_bytes(const siren_hyper_desc* d);
int64_t siren_hyper_workspace_bytes(const siren_hyper_desc* d);
int siren_hyper_forward(const siren_hyper_desc* d, const float* z, float* const* out, void* saved, int64_t saved_bytes,
                        void* stream);
int siren_hyper_backward(const siren_hyper_desc* d, const float* z, const float* const* dout, const void* saved,
                         int64_t saved_bytes, void* workspace, int64_t workspace_bytes, float* const* dW,
                         float* const* db, float* dz, void* stream);
/* The encoder's per-step operand preparation in one launch: for each of n (<= 32) convolutions,
 * geom[7 i ..] = {co, ci, k, stride_co, stride_ci, stride_kh, stride_kw} of the fp32 filter w[i]
 * (any strides); writes wb[i] = its bf16 channels-last copy [co][kh][kw][ci], wf[i] (wf or wf[i]
 * may be NULL) = the input gradient's bf16 filter [ci][k-1-kh][k-1-kw][co], and bb[i] (bb / bb[i]
 * may be NULL) = bf16 bias b[i] [co]; round to nearest even (torch's .to(torch.bfloat16)). */
int siren_enc_prep(int n, const float* const* w, const float* const* b, const int64_t* geom, void* const* wb,
                   void* const* wf, void* const* bb, void* stream);
/* Sum of squares over n (<= 32) fp32 tensors (hypo_weight_loss's sum of torch.sum(w ** 2),
 * loss_functions.py:279-287) into the device scalar out, deterministic; ws: zeroed once, left
 * zeroed, siren_sumsq_workspace_bytes(total elements). Backward: dst[i] = 2 g src[i] (g a device
 * scalar). */
int64_t siren_sumsq_workspace_bytes(int64_t total);
int siren_sumsq_forward(int n, const float* const* src, const int64_t* numel, float* out, void* ws, int64_t ws_bytes,
                        void* stream);
int siren_sumsq_backward(int n, const float* const* src, const int64_t* numel, const float* g, float* const* dst,
                         void* stream);
int siren_enc_relu_bwd(const void* g1, const void* g2, const void* y, void* out, float* db, int64_t P, int C, void* ws,
                       int64_t ws_bytes, void* stream);
int siren_enc_bias_relu(void* y, const void* cb, int64_t P, int C, void* stream);
int siren_enc_res_fwd(const void* a, const void* cb, const void* x, void* out, int64_t P, int C, void* stream);
int siren_enc_res_bwd(const void* g1, const void* g2, const void* out, const void* a, const void* cb, void* gskip,
                      void* ga, float* db, int64_t P, int C, void* ws, int64_t ws_bytes, void* stream);
int siren_enc_pixfc_fwd(const void* a, const void* cb, const float* w, const float* bias, float* e, int B, int64_t P,
                        int C, void* ws, int64_t ws_bytes, void* stream);
int siren_enc_pixfc_bwd(const float* g, const void* a, const void* cb, const float* w, void* ga, float* db, float* gw,
                        int B, int64_t P, int C, void* ws, int64_t ws_bytes, void* stream);

/*
 * Weighted sum of squared errors of image_mse (replaces loss_functions.py:66-101's
 *   diff = mask * (pred - gt); (diff.abs() ** 2).sum() * weight   and its autograd backward).
 * forward : d[e] = m[e % mask_n] (pred[e] - tgt[e]); *loss = weight * sum_e d[e]^2 (device
 *           scalar; deterministic summation order). mask may be NULL (no mask). `workspace` holds
 *           siren_sse_workspace_bytes() bytes, zero-filled before its first use and left zeroed by
 *           every call; one call at a time per workspace.
 * backward: out[e] = m[e % mask_n] (d[e] (g[0] scale)) with scale = 2 weight and g the upstream
 *           gradient (device scalar).
 * All pointers are device pointers of float32 data; stream is a hipStream_t (NULL = default).
 */
int64_t siren_sse_workspace_bytes(void);
int siren_sse_forward(const float* pred, const float* tgt, const float* mask, int64_t n, int64_t mask_n,
                      float weight, float* d, float* loss, void* workspace, int64_t ws_bytes, void* stream);
int siren_sse_backward(const float* d, const float* mask, int64_t n, int64_t mask_n, const float* g, float scale,
                       float* out, void* stream);

/*
 * k-space epilogue of the hypernetwork SIREN (configs 4/5) on the SIREN's output layout.
 *   pred, tgt, out, dpred, d : [batch, npix, channels] float32 (SingleBVPNet model_out rows)
 *   k0, mask                 : [batch, channels, npix] float32 (NCHW planes: img_sparse, dc_mask)
 *   hf                       : [npix] float32 per-pixel loss mask (the 128x128 high-frequency mask
 *                              1 - circle(r=20) of utils.py:25-40), or NULL
 * siren_dc_forward   replaces DataConsistencyInKspace.forward (data_consistency.py:32-48):
 *                    out = (1 - m) pred + m k0 (noise <= 0), (1 - m) pred + m (pred + noise k0) / (1 + noise)
 *                    (the reference's operation order, no contraction: bit-identical).
 * siren_dc_backward  its backward: dpred = g ((1 - m) [+ m / (1 + noise)]).
 * siren_kspace_sse_forward  image_mse (loss_functions.py:66-101) of DC(pred) (k0 and mask given) or
 *                    of pred (both NULL): d = hf (y - tgt), *loss = weight sum d^2 (deterministic
 *                    order); workspace as siren_sse_forward's (siren_sse_workspace_bytes()).
 * siren_kspace_sse_backward dL/dpred = g[0] scale hf d coef(m) (scale = 2 weight; coef = 1 without DC),
 *                    i.e. image_mse's and the data consistency's backward in one pass.
 */
int siren_dc_forward(const float* pred, const float* k0, const float* mask, int64_t batch, int64_t npix,
                     int channels, float noise, float* out, void* stream);
int siren_dc_backward(const float* g, const float* mask, int64_t batch, int64_t npix, int channels, float noise,
                      float* dpred, void* stream);
int siren_kspace_sse_forward(const float* pred, const float* k0, const float* mask, const float* tgt,
                             const float* hf, int64_t batch, int64_t npix, int channels, float noise, float weight,
                             float* d, float* loss, void* workspace, int64_t ws_bytes, void* stream);
int siren_kspace_sse_backward(const float* d, const float* mask, const float* hf, int64_t batch, int64_t npix,
                              int channels, float noise, const float* g, float scale, float* dpred, void* stream);

/*
 * Gaussian Fourier features (replaces GaussianFourierFeatureTransform.forward, features.py:31-41):
 * out [rows, 2 m] = cat(sin(2 pi x B), cos(2 pi x B)) for x [rows, cin], B [cin, m] (device float32),
 * one launch. Feeds the SIREN's wide first layer (5..16 inputs on the register-resident forward).
 */
int siren_fourier_features(const float* x, const float* B, int64_t rows, int cin, int m, float* out, void* stream);

/*
 * sin / cos of n fp32 radian arguments as the fp32 (SIREN_PREC_F32) kernels evaluate them
 * (impl 0: Cody-Waite reduction + minimax polynomials, siren_common.h sin_f32 / cos_f32) or through
 * OCML's sinf / cosf (impl 1). No reference counterpart: the accuracy probe behind the fp32 mode's
 * torch.sin / torch.cos replacement (modules.py:35-38), used by tests/test_gpu_sincos.py.
 */
int siren_sincos_f32(const float* x, float* s, float* c, int64_t n, int impl, void* stream);

/*
 * Process-wide execution options (no reference counterpart; used by tests and benchmarks to
 * compare code paths). Keys:
 *   "fused_forward"  1 (default): bf16 stacks of equal power-of-two hidden widths run their
 *                    forward as one kernel; 0: one kernel per layer.
 *   "fused_backward" 1 (default): bf16 backward folds the first layer's weight gradient into
 *                    the bottom hidden layer's input-gradient kernel (when no input gradient is
 *                    requested), and the output layer into the top hidden layer's kernels when
 *                    "fuse_output_layer" is 1 (default 0); 0: separate kernels.
 *   "ring_output_fusion"  1 (default): the output layer's backward runs inside the top 256x256
 *                    layer's ring kernels (bf16, outermost_linear, O <= 2); 0: last_bwd kernel.
 *   "dx_ring"        1 (default): 256x256 bf16 input-gradient layers use the 4-stage
 *                    load pipeline kernel; 0: the double-buffered one.
 *   "fused_forward_reg"  1 (default): the fused forward keeps every layer's activations in the
 *                    registers of the wave that owns the rows (weights streamed through an LDS
 *                    ring); 0: the LDS-staged fused forward below.
 *   "fused_forward_pipe"  1 (default): the LDS-staged fused forward overlaps one half-tile's MFMA
 *                    work with the other's epilogue; 0: the sequential single-kernel forward.
 *   "bwd_ring"       0 (default), 1: middle 256x256 bf16 layers compute both gradients in one
 *                    kernel (dZ and P read once); 0: separate input/weight-gradient kernels.
 *   "dw_ring"        1 (default): 256x256 bf16 weight-gradient layers use the ring kernel
 *                    (one full 256x256 partial per workgroup); 0: 128x128-tile split-K kernel.
 *   "pair_ring"      1 (default): a 256x256 bf16 layer whose two gradients both run on the ring
 *                    kernels computes them in ONE launch, on co-scheduled workgroup pairs that
 *                    stream the same tiles (one HBM read of dZ and P per pair); 0: two launches.
 *   "dx_stagger"     0 (default); 1: the middle/top input-gradient ring runs waves 4-7 one tile
 *                    late (epilogue from registers through a private staging tile; bit-identical,
 *                    measured 5-9 us/step slower).
 *   "pair_tail_reduce"  1 (default): a pair launch's weight-gradient workgroups also reduce the
 *                    previous pair launch's split-K slabs after their own rows (two slab buffers
 *                    alternate); 0: every pair launch is followed by a reduce_multi launch.
 *   "jvp_adj"        1 (default): the analytic-derivative backward (siren_jvp_backward*) runs each
 *                    hidden layer's adjoint GEMM with the adjoint combine in its epilogue (one
 *                    launch, the same formula to an fp32 ulp); 0: the GEMM and the combine as
 *                    two launches.
 *   "jvp_tn2"        1 (default): fp32 analytic-derivative weight gradients of 256-wide layers on
 *                    the all-rows tile kernel (X formed once per launch, double-buffered LDS);
 *                    0: the 128x128-tile kernel.
 *   "debug_pair_roles"  3 (default); 1 / 2 run only the input- / weight-gradient role of
 *                    pair_ring_bf16_kernel (timing experiments only: the gradients are then wrong).
 *   "jvp_tan"        1 (default): fp32 tangent streams of the 256-wide hidden layers on the
 *                    row-stacked tile (jvp_tan_kernel); 0: the stream-stacked GEMMs.
 *   "f32_rows"       1 (default): fp32 hidden layers' forward and input gradient on the
 *                    row-stacked tile, per-layer weight gradients on the all-rows tile; 0: the
 *                    128x128-tile kernels.
 *   "conv_dma"       2 (default): the encoder's forward / input-gradient convolutions (5x5 and
 *                    the other shapes) fill their stages by LDS-DMA with per-workgroup source
 *                    offsets; 1: LDS-DMA with per-stage offsets for the 5x5 ones, register staging
 *                    for the others; 0: register staging (all forms bit-identical).
 *   "wrw_dma"        2 (default): the 5x5 weight-gradient convolution's 128-pixel chunks (W a
 *                    multiple of 128, else 64) filled by LDS-DMA; 1: 64-pixel chunks by LDS-DMA;
 *                    0: 64-pixel chunks by register staging; 3: 2, and the other shapes' weight
 *                    gradients (cnn[0]'s 7x7, the 3x3 forms) in 128-pixel LDS-DMA chunks too
 *                    (all bit-identical).
 *   "debug_fused_profile"  device address of an int64 buffer [grid][4] that receives per-
 *                    workgroup cycle counts of the fused forward's phases, or 0 (off).
 * Returns SIREN_OK, or SIREN_EINVAL for an unknown key / value. Not thread-safe.
 */
int siren_config_set(const char* key, int64_t value);
int64_t siren_config_get(const char* key); /* -1 for an unknown key */

/* Thread-local message of the last failing call ("" if none). */
const char* siren_last_error(void);

/* Library build string (architecture, HIP version). */
const char* siren_version(void);

#ifdef __cplusplus
}
#endif

#endif /* SIREN_MRI_AMD_H */
