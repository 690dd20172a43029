// siren_spair.hip — one 256x256 hidden layer's backward, split by feature halves (bf16, gfx950).
//
//   dZ_{l-1} = (dZ_l W_l) w0 cos(P_{l-1})        (input gradient)     modules.py:25-26,38 backward
//   dW_l = dZ_l^T sin(P_{l-1}), db_l = sum dZ_l   (weight gradient)
//
// The pair_ring kernel gives one workgroup of a pair the whole input gradient and the other the
// whole weight gradient, so all dZ_{l-1} stores come from half of the CUs, whose vector-memory
// write path (about one 64-byte write request per six clocks per CU) then bounds the launch.
// Here both workgroups of a pair do both gradients, each for half of the feature columns i of
// layer l's input:
//   * waves 0-3 (one per SIMD): dZ_{l-1}[:, i] for the half's 128 columns, 32 per wave, with the
//     wave's W_l^T rows in registers (transposed MFMA, B fragments = dZ_l rows from LDS), epilogue
//     w0 cos(P) in place over the staged phase codes, 64-byte row pieces stored per wave;
//   * waves 4-7: the half's dW_l[:, i] (256 x 128 fp32 partial in registers, 64 x 128 per wave,
//     transposing LDS reads) and db_l for the half's rows of dW, plus the sin(P) conversion of the
//     next tile's phase codes.
// Both workgroups stream the same 32-row tiles in the same order (workgroups b and b + 8 share
// an XCD under round-robin dispatch — speed only): dZ_l leaves HBM about once, each half of
// P_{l-1} once, and each CU writes half a tile of dZ_{l-1} per tile.
//
// LDS stage (one 32-row tile): D = dZ_l (32 x 256 bf16, 16 KB), P = the half's phase codes
// (32 x 128, 8 KB; the input gradient overwrites it in place), H = bf16 sin(P) (8 KB). 16-byte
// chunk c of row r sits at chunk c ^ s(r), s(r) = 4 (r & 3) + ((r >> 2) & 3): conflict-free for
// the row-fragment reads (16 rows of a ds_read_b128 lane group hit 16 distinct chunks) and for
// the transposing reads (4 rows x 2 chunks per half-wave on disjoint banks). Five stages (all of
// LDS: DMA issued three tiles ahead of the conversion, four ahead of the MFMAs, so three tiles
// of loads stay in flight per CU — a four-stage ring left the pure load stream at 3.6 TB/s);
// one barrier per tile.
#include <type_traits>

#include "siren_common.h"

namespace siren {

constexpr int SPAIR_BM = 32;
#ifndef SIREN_SPAIR_STAGES
#define SIREN_SPAIR_STAGES 4
#endif
constexpr int SPAIR_S = SIREN_SPAIR_STAGES;  // x 32 KB
constexpr int SPAIR_D = 32 * 256 * 2;
constexpr int SPAIR_P = 32 * 128 * 2;
constexpr int SPAIR_STAGE = SPAIR_D + 2 * SPAIR_P;

struct SpairArgs {
  const bf16* dZ;        // [rows, 256] dZ_l
  const uint16_t* P;     // [rows, 256] phase codes of layer l - 1
  const bf16* Wt;        // [nb][256 (in i)][256 (out o)] W_l^T
  bf16* dZo;             // [rows, 256] dZ_{l-1}
  float* part;           // [npair][nb][256 * 256 + 256] partial slabs (dW row-major, then db)
  int64_t split_stride;
  int64_t rows_per_batch;
  int64_t w_bstride;
  float w0;
};

DEV int spair_swz(int r) { return 4 * (r & 3) + ((r >> 2) & 3); }
DEV int spair_dimg(int r, int c) { return r * 512 + ((c ^ spair_swz(r)) << 4); }  // 32 chunks per row
DEV int spair_himg(int r, int c) { return r * 256 + ((c ^ spair_swz(r)) << 4); }  // 16 chunks per row

// LDS accesses to the DMA-filled stages as inline asm: hipcc 7.2's wait-count pass cannot tell a
// C++ access of `smem` from the LDS-DMA still landing in another stage and drains the whole
// vector-memory queue (vmcnt(0): the DMA just issued and earlier stores) before it. The caller
// owns the LDS waits (spair_lgkm*, which tie the loaded registers to the wait).
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
template <int OFF>
DEV void spair_rd128(u32x4_t& d, uint32_t va) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(va), "n"(OFF));
}
template <int OFF>
DEV void spair_rd64(u32x2_t& d, uint32_t va) {
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(d) : "v"(va), "n"(OFF));
}
template <int OFF>
DEV void spair_wr64(uint32_t va, u32x2_t v) {
  asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(va), "v"(v), "n"(OFF) : "memory");
}
template <int OFF>
DEV void spair_wr128(uint32_t va, u32x4_t v) {
  asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(va), "v"(v), "n"(OFF) : "memory");
}
template <int N>
DEV void spair_lgkm(u32x4_t& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

template <int N>
DEV void spair_vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
DEV void spair_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__global__ __launch_bounds__(512) void spair_mid_kernel(SpairArgs a) {
  using PT = Prec<kPrecBF16>;
#ifdef SIREN_SPAIR_DBG
  // timing builds only: 1 no dZ_{l-1} stores, 2 no input-gradient work, 4 no weight-gradient work
  constexpr int dbg = SIREN_SPAIR_DBG;
#else
  constexpr int dbg = 0;
#endif
  typedef __attribute__((address_space(3))) void lds_v;
  __shared__ __attribute__((aligned(16))) char smem[SPAIR_S * SPAIR_STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.x;
  const int64_t pair = (b & 7) | ((b >> 4) << 3);
  const int hf = (b >> 3) & 1;  // feature half: columns [128 hf, 128 hf + 128)
  const int64_t npair = gridDim.x >> 1;
  const int64_t batch = blockIdx.y;
  const int64_t rows = a.rows_per_batch;
  const int64_t rowbase = batch * rows;
  const int64_t ntiles = (rows + SPAIR_BM - 1) / SPAIR_BM;
  const int64_t tb = ntiles * pair / npair, te = ntiles * (pair + 1) / npair;
  const int64_t niter = te - tb;
  const bool dxw = wave < 4;

  auto nval = [&](int64_t t) -> int64_t {
    const int64_t n = rows - t * SPAIR_BM;
    return n < SPAIR_BM ? n : SPAIR_BM;
  };
  // ---- DMA of tile t into stage st: D (2 KB per wave), the half's P (1 KB per wave) ----
  uint32_t dvoff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int i = wave + 8 * j;
    const int r = 2 * i + (lane >> 5), pos = lane & 31;
    dvoff[j] = r * 512 + ((pos ^ spair_swz(r)) << 4);
  }
  uint32_t pvoff;
  {
    const int r = 4 * wave + (lane >> 4), pos = lane & 15;
    pvoff = r * 512 + ((16 * hf + (pos ^ spair_swz(r))) << 4);
  }
  auto dma = [&](int64_t t, int st) {
    char* base = smem + st * SPAIR_STAGE;
    const int64_t m0 = rowbase + t * SPAIR_BM, nv = nval(t);
    const __amdgpu_buffer_rsrc_t rD = make_rsrc(a.dZ + m0 * 256, nv * 512);
    const __amdgpu_buffer_rsrc_t rP = make_rsrc(a.P + m0 * 256, nv * 512);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rD, (lds_v*)(base + (wave + 8 * j) * 1024), 16, dvoff[j], 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rP, (lds_v*)(base + SPAIR_D + wave * 1024), 16, pvoff, 0, 0, 0);
  };

  // ================= waves 0-3: input gradient of the half =================
  const int r32 = lane & 31, kh = lane >> 5;
  const int wx = wave & 3;
  bf16x8 wf[16];
  if (dxw) {
    const bf16* Wb = a.Wt + batch * a.w_bstride + (int64_t)(128 * hf + 32 * wx + r32) * 256;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) wf[ks] = *(const bf16x8*)(Wb + 16 * ks + 8 * kh);
  }
  // epilogue groups: lane (r32, kh) holds half-local features 32 wx + 8 g + 4 kh + e
  int eoff[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) eoff[g] = SPAIR_D + spair_himg(r32, 4 * wx + g) + 8 * kh;
  // store pass: the wave's 4 chunks x 32 rows, pieces q = lane + 64 j -> row q / 4, chunk 4 wx + q % 4
  int soff[2];
  uint32_t goff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = lane + 64 * j, r = q >> 2, c = 4 * wx + (q & 3);
    soff[j] = SPAIR_D + spair_himg(r, c);
    goff[j] = r * 512 + (16 * hf + c) * 16;
  }
  // B-fragment reads: K step ks reads chunk 2 ks + kh of row r32 at position (2 ks + kh) ^ s(r32)
  // = 2 (ks ^ m) + (kh ^ (s & 1)), m = s >> 1: eight per-lane offsets (ks & 7), + 256 B for ks >= 8
  uint32_t boff[8];
  {
    const int sw = spair_swz(r32);
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) boff[jj] = r32 * 512 + 32 * (jj ^ (sw >> 1)) + 16 * (kh ^ (sw & 1));
  }
  const uint32_t smem_lds0 = lds_addr(smem);
  auto dx_tile = [&](int64_t t, int st) {
    const uint32_t sb = smem_lds0 + st * SPAIR_STAGE;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    constexpr int PF = 3;
    u32x4_t bq[4];
    auto bread = [&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      spair_rd128<256 * (ks >> 3)>(bq[ks & 3], sb + boff[ks & 7]);
    };
    static_for<0, PF>([&](auto c) { bread(c); });
    static_for<0, 16>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      if constexpr (ks + PF < 16) bread(std::integral_constant<int, ks + PF>{});
      if constexpr (ks + PF < 16) spair_lgkm<PF>(bq[ks & 3]);
      else spair_lgkm<15 - ks>(bq[ks & 3]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], __builtin_bit_cast(bf16x8, bq[ks & 3]), acc, 0, 0, 0);
    });
    // epilogue: dZ_{l-1} = acc w0 cos(P), in place over the phase codes (4 features per group)
    u32x2_t ph[4];
    spair_rd64<0>(ph[0], sb + eoff[0]);
    spair_rd64<0>(ph[1], sb + eoff[1]);
    spair_rd64<0>(ph[2], sb + eoff[2]);
    spair_rd64<0>(ph[3], sb + eoff[3]);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ph[0]), "+v"(ph[1]), "+v"(ph[2]), "+v"(ph[3]));
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const u16x4 pc = __builtin_bit_cast(u16x4, ph[g]);
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (bf16)((acc[4 * g + e] * PT::cosp(pc[e])) * a.w0);
      spair_wr64<0>(sb + eoff[g], __builtin_bit_cast(u32x2_t, v));
    }
    // the wave's 32 columns x 32 rows as 64-byte row pieces (its own writes: no barrier)
    u32x4_t sv[2];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    spair_rd128<0>(sv[0], sb + soff[0]);
    spair_rd128<0>(sv[1], sb + soff[1]);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(sv[0]), "+v"(sv[1]));
    const __amdgpu_buffer_rsrc_t rC = make_rsrc(a.dZo + (rowbase + t * SPAIR_BM) * 256, nval(t) * 512);
    if constexpr (!(dbg & 1))
#pragma unroll
      for (int j = 0; j < 2; ++j) __builtin_amdgcn_raw_buffer_store_b128(sv[j], rC, goff[j], 0, 0);
  };

  // ================= waves 4-7: weight gradient of the half =================
  const int wm = wave & 3;  // dW rows [64 wm, +64), the half's 128 columns
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][jj][e] = 0.f;
  // transposing fragment reads: lane (g, q, p) of a 16-lane group g reads row nb + (0 | 4), 4
  // columns; K step 1 = + 16 rows (the swizzle repeats every 16 rows: D + 8192, H + 4096)
  const int gq = lane >> 4, tq = lane & 15, q4 = tq >> 2, p4 = tq & 3;
  uint32_t abase[2][2], bbase[4][2];
  {
    const int nb0 = 8 * (gq >> 1) + q4;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int nb = nb0 + 4 * u;
#pragma unroll
      for (int bm = 0; bm < 2; ++bm) {
        const int c = 64 * wm + 32 * bm + 16 * (gq & 1) + 4 * p4;
        abase[bm][u] = spair_dimg(nb, c >> 3) + (c & 7) * 2;
      }
#pragma unroll
      for (int bn = 0; bn < 4; ++bn) {
        const int c = 32 * bn + 16 * (gq & 1) + 4 * p4;
        bbase[bn][u] = SPAIR_D + SPAIR_P + spair_himg(nb, c >> 3) + (c & 7) * 2;
      }
    }
  }
  const uint32_t smem_lds = lds_addr(smem);
  // conversion and db: dw thread u takes chunks u and u + 256 of the half (row k >> 4, chunk k & 15)
  const int u = tid - 256;
  const int crow = (u & 255) >> 4, cch = u & 15;
  float dbacc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) dbacc[e] = 0.f;
  const uint32_t coff[2] = {(uint32_t)spair_himg(crow, cch), (uint32_t)spair_himg(crow + 16, cch)};
  const uint32_t dboff[2] = {(uint32_t)spair_dimg(crow, 16 * hf + cch), (uint32_t)spair_dimg(crow + 16, 16 * hf + cch)};
  auto convert = [&](int st) {
    const uint32_t sb = smem_lds + st * SPAIR_STAGE;
    u32x4_t pv[2];
    spair_rd128<SPAIR_D>(pv[0], sb + coff[0]);
    spair_rd128<SPAIR_D>(pv[1], sb + coff[1]);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pv[0]), "+v"(pv[1]));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const u16x8 ph = __builtin_bit_cast(u16x8, pv[j]);
      bf16x8 hv;
#pragma unroll
      for (int e = 0; e < 8; ++e) hv[e] = (bf16)PT::sinp(ph[e]);
      if (j == 0) spair_wr128<SPAIR_D + SPAIR_P>(sb + coff[0], __builtin_bit_cast(u32x4_t, hv));
      else spair_wr128<SPAIR_D + SPAIR_P>(sb + coff[1], __builtin_bit_cast(u32x4_t, hv));
    }
  };
  auto dbsum = [&](int st) {  // db over dW rows (= dZ_l columns) 128 hf + 8 cch .. + 8
    const uint32_t sb = smem_lds + st * SPAIR_STAGE;
    u32x4_t dv[2];
    spair_rd128<0>(dv[0], sb + dboff[0]);
    spair_rd128<0>(dv[1], sb + dboff[1]);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(dv[0]), "+v"(dv[1]));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16x8 d8 = __builtin_bit_cast(bf16x8, dv[j]);
#pragma unroll
      for (int e = 0; e < 8; ++e) dbacc[e] += (float)d8[e];
    }
  };
  auto dw_tile = [&](int st) {
    const uint32_t sb = smem_lds + st * SPAIR_STAGE;
    TrFrag fa[2][2], fb[2][4];
    // both K steps' fragment reads up front (24 transposing reads), counted waits per step; K step
    // 1 is + 16 rows (the swizzle repeats every 16 rows): every offset an immediate
#define SIREN_SP_TR(F, V, OFF)                                                                  \
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"((F).lo) : "v"((V)[0]), "n"(OFF)); \
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"((F).hi) : "v"((V)[1]), "n"(OFF));
    uint32_t va[2][2], vb[4][2];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      va[0][x] = sb + abase[0][x];
      va[1][x] = sb + abase[1][x];
#pragma unroll
      for (int bn = 0; bn < 4; ++bn) vb[bn][x] = sb + bbase[bn][x];
    }
    SIREN_SP_TR(fa[0][0], va[0], 0) SIREN_SP_TR(fa[0][1], va[1], 0)
    SIREN_SP_TR(fb[0][0], vb[0], 0) SIREN_SP_TR(fb[0][1], vb[1], 0)
    SIREN_SP_TR(fb[0][2], vb[2], 0) SIREN_SP_TR(fb[0][3], vb[3], 0)
    SIREN_SP_TR(fa[1][0], va[0], 8192) SIREN_SP_TR(fa[1][1], va[1], 8192)
    SIREN_SP_TR(fb[1][0], vb[0], 4096) SIREN_SP_TR(fb[1][1], vb[1], 4096)
    SIREN_SP_TR(fb[1][2], vb[2], 4096) SIREN_SP_TR(fb[1][3], vb[3], 4096)
#undef SIREN_SP_TR
    asm volatile("s_waitcnt lgkmcnt(12)"
                 : "+v"(fa[0][0].lo), "+v"(fa[0][0].hi), "+v"(fa[0][1].lo), "+v"(fa[0][1].hi), "+v"(fb[0][0].lo),
                   "+v"(fb[0][0].hi), "+v"(fb[0][1].lo), "+v"(fb[0][1].hi), "+v"(fb[0][2].lo), "+v"(fb[0][2].hi),
                   "+v"(fb[0][3].lo), "+v"(fb[0][3].hi));
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int bn = 0; bn < 4; ++bn)
        acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr16_value(fa[0][bm]), tr16_value(fb[0][bn]),
                                                              acc[bm][bn], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(fa[1][0].lo), "+v"(fa[1][0].hi), "+v"(fa[1][1].lo), "+v"(fa[1][1].hi), "+v"(fb[1][0].lo),
                   "+v"(fb[1][0].hi), "+v"(fb[1][1].lo), "+v"(fb[1][1].hi), "+v"(fb[1][2].lo), "+v"(fb[1][2].hi),
                   "+v"(fb[1][3].lo), "+v"(fb[1][3].hi));
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int bn = 0; bn < 4; ++bn)
        acc[bm][bn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tr16_value(fa[1][bm]), tr16_value(fb[1][bn]),
                                                              acc[bm][bn], 0, 0, 0);
  };

  // ================= the tile loop =================
  // DMA(k) is issued at iteration k - (S - 1) (prologue: tiles 0..S-2); the conversion of tile k
  // runs in iteration k - 1; at the barrier of iteration k, DMA(k + 1) has landed. VMEM ops per
  // wave younger than DMA(k + 1) then: DMA(k + 2 .. k + S - 2) = 3 (S - 3), plus the input-
  // gradient waves' stores of iterations k - (S - 2) .. k - 1 = 2 (S - 2).
  constexpr int YD = 3 * (SPAIR_S - 3), YX = YD + 2 * (SPAIR_S - 2);
  for (int s = 0; s < SPAIR_S - 1; ++s)
    if (s < niter) dma(tb + s, s);
  auto loop = [&](auto dx_tag) {
    constexpr bool DX = decltype(dx_tag)::value;
    if (niter > 0) {
      if (niter >= SPAIR_S - 1) spair_vmwait<3 * (SPAIR_S - 2)>();  // DMA(0) landed
      else spair_vmwait<0>();
      spair_barrier();
      if constexpr (!DX) convert(0);
    }
    for (int64_t k = 0; k < niter; ++k) {
      const int st = (int)(k % SPAIR_S);
      if (k + SPAIR_S - 2 < niter) {
        if (DX && k >= SPAIR_S - 2) spair_vmwait<YX>();
        else spair_vmwait<YD>();  // (early iterations: fewer stores issued yet)
      } else {
        spair_vmwait<0>();
      }
      spair_barrier();
      if (k + SPAIR_S - 1 < niter) dma(tb + k + SPAIR_S - 1, (int)((k + SPAIR_S - 1) % SPAIR_S));
      if constexpr (DX) {
        if constexpr (!(dbg & 2)) dx_tile(tb + k, st);
      } else if constexpr (!(dbg & 4)) {
        dw_tile(st);
        if (k + 1 < niter) convert((int)((k + 1) % SPAIR_S));
        dbsum(st);
      }
    }
    spair_vmwait<0>();
  };
  if (dxw) loop(std::true_type{});
  else loop(std::false_type{});

  // ================= partial slab of the pair: the half's columns of dW, its rows of db =================
  float* part = a.part + pair * a.split_stride + batch * (int64_t)(256 * 256 + 256);
  if (!dxw) {
#pragma unroll
    for (int bm = 0; bm < 2; ++bm)
#pragma unroll
      for (int bn = 0; bn < 4; ++bn) {
        const int col = 128 * hf + 32 * bn + (lane & 31);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = 64 * wm + 32 * bm + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          part[(int64_t)row * 256 + col] = acc[bm][bn][e];
        }
      }
  }
  __syncthreads();
  float* red = (float*)smem;  // [16 row slots][128]
  if (!dxw) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[crow * 128 + 8 * cch + e] = dbacc[e];
  }
  __syncthreads();
  if (tid < 128) {
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) sum += red[k * 128 + tid];
    part[256 * 256 + 128 * hf + tid] = sum;
  }
}

}  // namespace siren
