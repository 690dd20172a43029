// siren_common.h — shared device helpers for the gfx950 SIREN kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#define DEV __device__ __forceinline__

namespace siren {

// shape limits of the fused kernels (siren_fused.hip, siren_fwdreg.hip)
constexpr int FUSED_MAXC = 4;   // coordinate inputs of the narrow fused forms
constexpr int FUSED_MAXO = 8;   // outputs
constexpr int FUSED_MAXH = 14;  // hidden layers
// LDS address space (LDS-DMA destinations)
typedef __attribute__((address_space(3))) void lds_void;

constexpr float kInv2Pi = 0.15915494309189535f;
constexpr int kPrecF32 = 0;
constexpr int kPrecBF16 = 1;

typedef __bf16 bf16;
typedef bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 h16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Per-precision storage policy.
//  phase_t: what a sine layer keeps of its pre-activation between forward and backward.
//           F32 : p = w0*(xW^T+b) in radians (bit-faithful to modules.py:26,38).
//           BF16: p reduced mod 2pi and quantised to 16 bits of a revolution (resolution
//                 9.6e-5 rad); sin/cos are then single v_sin_f32/v_cos_f32 instructions
//                 (which take revolutions) and the tensor costs 2 B/element in HBM.
//  grad_t : storage of dL/dz between backward kernels.
//  op_t   : MFMA operand element.
template <int PREC> struct Prec;
#ifndef SIREN_F32_OCML
#define SIREN_F32_OCML 0
#endif

// fp32 sin / cos for the fp32 (reference-arithmetic) mode: 3-part Cody-Waite reduction by pi/2
// (FMA form, exact for |x| < ~1e5) and minimax polynomials on [-pi/4, pi/4], ~1-2 ulp. OCML's
// sinf/cosf inline a Payne-Hanek reduction at every call site: the tangent-stream GEMMs grew to
// 33 K instructions (1,300 64-bit multiplies, 400 alignbits, 700 branches) and ran 3x the time of
// the same GEMM without the operand math. Arguments past the Cody-Waite range take OCML's
// functions through a call (never on the SIREN path: |w0 z| stays far below 1e5 radians).
__attribute__((noinline)) __device__ float sin_f32_far(float x) { return sinf(x); }
__attribute__((noinline)) __device__ float cos_f32_far(float x) { return cosf(x); }
DEV void sincos_poly(float x, float& sn, float& cs, int& q) {
  const float k = __builtin_rintf(x * 0.636619772367581343f);  // round(x / (pi / 2))
  float r = fmaf(k, -1.57079637050628662109375f, x);
  r = fmaf(k, 4.371138828673793e-8f, r);
  r = fmaf(k, 1.7151245100058819e-15f, r);
  q = (int)k;
  const float t = r * r;
  float ps = fmaf(2.86567956e-6f, t, -1.98559923e-4f);
  ps = fmaf(ps, t, 8.33338592e-3f);
  ps = fmaf(ps, t, -1.66666672e-1f);
  sn = fmaf(ps * t, r, r);
  float pc = fmaf(2.44677067e-5f, t, -1.38877297e-3f);
  pc = fmaf(pc, t, 4.16666567e-2f);
  pc = fmaf(pc, t, -5.0e-1f);
  cs = fmaf(pc, t, 1.0f);
}
DEV float sin_f32(float x) {
  if (__builtin_expect(!(__builtin_fabsf(x) < 1.0e5f), 0)) return sin_f32_far(x);
  float sn, cs;
  int q;
  sincos_poly(x, sn, cs, q);
  const float v = (q & 1) ? cs : sn;
  return (q & 2) ? -v : v;
}
DEV float cos_f32(float x) {
  if (__builtin_expect(!(__builtin_fabsf(x) < 1.0e5f), 0)) return cos_f32_far(x);
  float sn, cs;
  int q;
  sincos_poly(x, sn, cs, q);
  const float v = (q & 1) ? sn : cs;
  return ((q + 1) & 2) ? -v : v;
}

// Range of Fourier-feature arguments (2 pi z, radians) over which both feature paths use
// sincos_poly: the FMA Cody-Waite reduction stays within 7e-8 absolute of sin / cos of the fp32
// argument up to 1e6 (measured against fp64; tests/test_gpu_fourier_input.py pins it).
constexpr float kFFPolyRange = 1.0e6f;

// Fourier feature f of a row (features.py:21-41): z = sum_c x[c] B[c][k] (fma chain from 0), k = f
// mod m, sin(2 pi z) for f < m, cos(2 pi z) for m <= f < 2m, 0 past 2m — bit-identical to
// siren_kspace.hip fourier_kernel (the same chain, argument and sincos_poly), so features formed
// here equal the materialised ones. There is no far-range path in the register forward (a call
// there would cost the kernel its register budget): the host takes the fused path only when
// 2 pi max_k sum_c |B[c][k]| < kFFPolyRange (coordinates in [-1, 1]; features.py), and an
// argument past the range anyway (coordinates outside [-1, 1]) yields NaN, never a silently
// different feature.
DEV float ff_feature(const float* xr, const float* B, int cin, int m, int f) {
  if (f >= 2 * m) return 0.f;
  const bool cosine = f >= m;
  const int k = cosine ? f - m : f;
  float z = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)  // (compile-time indices into the caller's register array; cin <= 4)
    if (c < cin) z = fmaf(xr[c], B[c * m + k], z);
  float sn, cs;
  int q;
  const float arg = __fmul_rn(6.2831854820251465f, z);
  sincos_poly(arg, sn, cs, q);
  q += cosine ? 1 : 0;  // cos x = sin(x + pi / 2): one quadrant on
  const float v = (q & 1) ? cs : sn;
  return __builtin_fabsf(arg) < kFFPolyRange ? ((q & 2) ? -v : v) : __builtin_nanf("");
}

template <> struct Prec<kPrecF32> {
  using phase_t = float;
  using grad_t = float;
  using op_t = float;
  static DEV phase_t enc(float p) { return p; }
  // phase of w0 * (z + b): the reference's sin(w0 * (xW^T + b)) argument (modules.py:26,38)
  static DEV phase_t encz(float z, float b, float w0) { return w0 * (z + b); }
  // sin_f32 / cos_f32 above (SIREN_F32_OCML=1 builds the OCML sinf / cosf instead, for A/B);
  // pinned against fp64 over |x| <= 2000 rad and past the Cody-Waite range by
  // tests/test_gpu_sincos.py through siren_sincos_f32
#if SIREN_F32_OCML
  static DEV float sinp(phase_t v) { return sinf(v); }
  static DEV float cosp(phase_t v) { return cosf(v); }
#else
  static DEV float sinp(phase_t v) { return sin_f32(v); }
  static DEV float cosp(phase_t v) { return cos_f32(v); }
#endif
  // sin / cos of an fp32 radian argument (the sine output layer, outermost_linear=False)
  static DEV float sinr(float x) { return sinp(x); }
  static DEV float cosr(float x) { return cosp(x); }
};

template <> struct Prec<kPrecBF16> {
  using phase_t = uint16_t;
  using grad_t = bf16;
  using op_t = bf16;
  static DEV phase_t enc(float p) {
    float r = p * kInv2Pi;
    r = r - floorf(r);
    return (uint16_t)((uint32_t)__builtin_rintf(r * 65536.0f) & 0xFFFFu);
  }
  // Phase of w0 * (z + b) in one FMA: round(z k + b k) with k = w0 * 2^16 / 2pi; the low 16 bits
  // of the two's-complement integer are the phase mod 2pi (valid for |w0 (z + b)| < 2^15 * 2pi * 2^15).
  static DEV float enck(float w0) { return w0 * (65536.0f * kInv2Pi); }
  static DEV phase_t encz(float z, float b, float w0) {
    const float k = enck(w0);
    return enc_scaled(z, b * k, k);
  }
  // the same with the bias already multiplied by k = enck(w0)
  // v_cvt_rpi_i32_f32 = floor(v + 0.5): one instruction for the round-and-convert (ties round up
  // instead of to even; every encoder and every recompute of a phase uses this same form)
  static DEV phase_t enc_scaled(float z, float bk, float k) {
    const float v = fmaf(z, k, bk);
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(v));
    return (uint16_t)r;
  }
  static DEV float rev(phase_t v) { return (float)v * (1.0f / 65536.0f); }
  // v_sin_f32 / v_cos_f32 take revolutions and reduce them exactly: the float with bits
  // 0x4300_0000 | v is 128 + v * 2^-16 (exact), one OR (or byte permute) instead of a convert and a
  // multiply. Measured on gfx950 over all 65536 phases: cos bit-identical to cos(rev(v)); sin
  // differs in 22 phases by less than 2^-24 absolute (tools/probe_sin.hip).
  static DEV float rev128(phase_t v) { return __builtin_bit_cast(float, 0x43000000u | (uint32_t)v); }
  static DEV float sinp(phase_t v) { return __builtin_amdgcn_sinf(rev128(v)); }
  static DEV float cosp(phase_t v) { return __builtin_amdgcn_cosf(rev128(v)); }
  static DEV float sinr(float x) {
    const float r = x * kInv2Pi;
    return __builtin_amdgcn_sinf(r - floorf(r));
  }
  static DEV float cosr(float x) {
    const float r = x * kInv2Pi;
    return __builtin_amdgcn_cosf(r - floorf(r));
  }
};

// Compile-time loop: fn(std::integral_constant<int, i>) for i in [B, E) (indices usable as
// template arguments, e.g. inline-asm immediate offsets).
template <int B, int E, typename Fn>
DEV void static_for(Fn&& fn) {
  if constexpr (B < E) {
    fn(std::integral_constant<int, B>{});
    static_for<B + 1, E>(fn);
  }
}

DEV float to_f32(float v) { return v; }
DEV float to_f32(bf16 v) { return (float)v; }

template <typename T> DEV T from_f32(float v);
template <> DEV float from_f32<float>(float v) { return v; }
template <> DEV bf16 from_f32<bf16>(float v) { return (bf16)v; }

DEV float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ds_read_b64_tr_b16: lane (4q+p) of each 16-lane group supplies the address of row q,
// columns 4p..4p+3 of a 4x16 block; lane i of the group receives column i of the 4 rows.
DEV s16x4 lds_read_tr16(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

// Two transposing reads (rows k..k+3 and k+4..k+7 of one 16-column block) -> one 8-element bf16
// MFMA operand. Whole-vector casts only: per-element bit_casts of the v4i16 result were lowered
// to a duplicating v_perm by hipcc 7.2 (wrong operands, no diagnostic).
DEV bf16x8 lds_read_tr16_pair(const void* lo_ptr, const void* hi_ptr) {
  const s16x4 lo = lds_read_tr16(lo_ptr);
  const s16x4 hi = lds_read_tr16(hi_ptr);
  const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// Raw buffer resource over [base, base + bytes): loads past the end return 0, stores past it are
// dropped (the ragged-tile handling of the ring and fused kernels).
DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0,
                                           (int)(bytes > 0x7fffffff ? 0x7fffffff : bytes), 0x00020000);
}

// Buffer stores whose data VGPRs are rewritten soon after them. Measured on MI355X
// (tools/det_p0.py, tools/det_wide.py, profiles/r3_store_hazard.txt): in the register-resident
// forward, under the ring's LDS-DMA traffic, a buffer_store_dwordx4 whose first data VGPR is
// rewritten by a VALU instruction shortly after the store (one to a few instructions later, as
// hipcc schedules it) sometimes stores the NEW value in lanes 12-15 of each 16-lane group: the
// store reads its data after issue, later than the documented one-wait-state hazard covers.
// Neither 16 s_nop wait states nor s_waitcnt expcnt(0) between the store and the write prevent it
// (the expcnt form only moved the failure: det_wide.py still caught it at C = 16, where the VALU
// write after the last hidden block's store is the output layer's fragment-address add). What
// does: the store having COMPLETED (s_waitcnt vmcnt) before its data VGPRs are written again.
// So each such store is followed by store_complete(data): an s_waitcnt vmcnt(0) that takes the
// store's data as an input operand, so the compiler keeps those registers unmodified (and nothing
// else allocated into them) until the store has completed. vmcnt counts in issue order, so the
// wait also covers older vector-memory operations (the ring DMA of the kernels is issued far
// enough ahead to have landed by then).
template <typename T>
DEV void store_complete(const T& data) {
  asm volatile("s_waitcnt vmcnt(0)" ::"v"(data));
}
// the same for two stores' data (the older one held until here)
template <typename T, typename U>
DEV void store_complete2(const T& data, const U& held) {
  asm volatile("s_waitcnt vmcnt(0)" ::"v"(data), "v"(held));
}
// The measured rule (tools/probe_store_hazard.hip): a store of more than 8 bytes
// reads its data VGPRs during the 2 wait states after its issue; a VALU write of them with 0 wait
// states in between corrupts lanes 8-15 of each 16-lane group, with 1 lanes 12-15, with 2 none
// (2.7e9 stores, with or without LDS-DMA or other stores in flight). hipcc 7.2 sometimes leaves a
// single wait state there. These stores carry their own `s_nop 1` (2 wait states) inside the asm
// statement that takes the data as input, so nothing can write those registers before it has
// passed — instead of waiting for the store to complete.
// SIREN_STORE_MOD: cache-policy modifiers of these stores (timing experiments, e.g. " nt")
#ifndef SIREN_STORE_MOD
#define SIREN_STORE_MOD ""
#endif
DEV void store_b128_ws2(const u32x4_t& v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen" SIREN_STORE_MOD "\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(r),
               "s"(soff)
               : "memory");
}
DEV void store_b32_ws2(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_store_dword %0, %1, %2, %3 offen\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(r), "s"(soff)
               : "memory");
}
#ifndef SIREN_STORE_EXPCNT
#define SIREN_STORE_EXPCNT 1
#endif
DEV void store_b128_sync(const u32x4_t& v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, 0);
#if SIREN_STORE_EXPCNT
  store_complete(v);
#endif
}
DEV void store_b32_sync(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, 0, 0);
#if SIREN_STORE_EXPCNT
  store_complete(v);
#endif
}
// The ring backward kernels (siren_gemm.hip) keep the compiler's buffer stores without the wait: a
// vmcnt(0) per store would drain their three-tile DMA ring. Their data registers stay untouched for
// 20-60 instructions after each store, and no run-to-run difference was ever observed there
// (tools/det_bwd.py, test_backward_deterministic). As inline asm (the compiler then reuses the data
// registers right after the asm) they differed in 5 of 5 runs: ~1e-1 without a wait, ~1e-3 with
// expcnt(0) (profiles/r3_store_hazard.txt) — the same hazard.
// Diagnostic builds: 0 builtin store (default), 1 store_b128_sync, 2 asm store without the wait,
// 3 builtin store + a separate expcnt(0).
#ifndef SIREN_GEMM_STORE
#define SIREN_GEMM_STORE 0
#endif
DEV void store_b128_gemm(const u32x4_t& v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
#if SIREN_GEMM_STORE == 1
  store_b128_sync(v, r, voff);
#elif SIREN_GEMM_STORE == 2
  asm volatile("buffer_store_dwordx4 %0, %1, %2, 0 offen" ::"v"(v), "v"(voff), "s"(r) : "memory");
#elif SIREN_GEMM_STORE == 3
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, 0);
  asm volatile("s_waitcnt expcnt(0)" ::: "memory");
#else
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, 0);
#endif
}
DEV void store_b32_gemm(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff) {
#if SIREN_GEMM_STORE == 1
  store_b32_sync(v, r, voff);
#elif SIREN_GEMM_STORE == 2
  asm volatile("buffer_store_dword %0, %1, %2, 0 offen" ::"v"(v), "v"(voff), "s"(r) : "memory");
#elif SIREN_GEMM_STORE == 3
  __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, 0, 0);
  asm volatile("s_waitcnt expcnt(0)" ::: "memory");
#else
  __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, 0, 0);
#endif
}

// The same transposing reads as inline asm, for kernels that also fill LDS by DMA
// (global_load_lds): hipcc 7.2's wait-count pass treats the ds_read_b64_tr_b16 builtin as possibly
// aliasing every LDS-DMA still in flight and puts an s_waitcnt vmcnt(0) in front of it, which
// drains the prefetch ring every iteration. The asm form is invisible to that pass, so the caller
// owns the LDS wait: issue the reads (tr16_issue), then tr16_wait(...) on every fragment (one
// s_waitcnt lgkmcnt(0) whose operands tie the fragments to it), then tr16_value.
struct TrFrag {
  s16x4 lo, hi;
};
DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
DEV void tr16_issue(TrFrag& f, const void* lo_ptr, const void* hi_ptr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.lo) : "v"(lds_addr(lo_ptr)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f.hi) : "v"(lds_addr(hi_ptr)));
}
template <int OFF>
DEV void tr16_read(s16x4& out, uint32_t vaddr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(out) : "v"(vaddr), "n"(OFF));
}
DEV bf16x8 tr16_value(const TrFrag& f) {
  const s16x8 v = __builtin_shufflevector(f.lo, f.hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

// Data consistency in k-space (data_consistency.py:8-48): (1 - m) p + m k0, or
// (1 - m) p + m (p + v k0) / (1 + v) (noisy), in the reference's operation order with no fused
// multiply-adds (bit-identical to PyTorch's elementwise chain); used by siren_kspace.hip and by the
// forward's fused output-layer loss (siren_fwdreg.hip).
DEV float dc_value(float p, float k, float m, float noise) {
  const float keep = __fmul_rn(__fsub_rn(1.f, m), p);
  if (noise > 0.f) {
    const float mix = __fdiv_rn(__fadd_rn(p, __fmul_rn(noise, k)), __fadd_rn(1.f, noise));
    return __fadd_rn(keep, __fmul_rn(m, mix));
  }
  return __fadd_rn(keep, __fmul_rn(m, k));
}
// d out / d pred of dc_value
DEV float dc_coef(float m, float noise) {
  const float keep = __fsub_rn(1.f, m);
  return noise > 0.f ? __fadd_rn(keep, __fdiv_rn(m, __fadd_rn(1.f, noise))) : keep;
}

}  // namespace siren
