// fp32 FC on the bf16 matrix cores: the GraphConv FC of fc.hip
//
//   C[m, n] = act( sum_{k<K1} A1[m,k] W1[n,k] + sum_{k<K2} A2[m,k] W2[n,k] [+ C[m,n]] + bias[n] )
//
// (PyG 2.1 GraphConv lin_rel + lin_root + ReLU/dropout, arch.py:57-62, 75-80,
// 182-188; and, with W = a transposed weight, the input-gradient GEMMs of its
// backward) with fp32 operands and fp32 accumulation, evaluated through an
// EXACT three-way bf16 split instead of the fp32 MFMA.
//
// Why: gfx950 issues v_mfma_f32_32x32x16_bf16 at 512 MAC/clk/SIMD and
// v_mfma_f32_32x32x2_f32 at 32 (MI355X_MICROARCH.md, constants table).  Every
// fp32 value splits exactly into three bf16 terms, a = a0 + a1 + a2 with
// a0 = RNE_bf16(a), a1 = RNE_bf16(a - a0), a2 = a - a0 - a1 (8 + 8 + 8
// significant bits = the 24-bit fp32 significand; |a1| <= 2^-8 |a|,
// |a2| <= 2^-16 |a|, every subtraction exact).  The product keeps every term
// down to 2^-16 relative size:
//   a b = a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0) + d,
//   |d| = |a1 b2 + a2 b1 + a2 b2| <= 2^-23 |a b|,
// i.e. below the fp32 rounding of the product itself.  Each bf16 x bf16
// product is exact in fp32.  a0 b0 accumulates in its own fp32 accumulator
// (accH) and the five small products in another (accL), added once at the
// end, so the small terms' roundings sit 2^-8 below the main chain's.  Cost:
// 6 bf16 MFMAs = 6/16 of one fp32 MFMA.  Accuracy is fp32 GEMM accuracy
// (fp32 operands are never rounded); tests/test_gpu_fc.py measures it against
// fp64 beside the exact-fp32 kernel.  Not a bitwise contract: the bf16 MFMA's
// internal summation order is unspecified, so there is no CPU restatement of
// the bits (the exact-fp32 kernel, lpg_fc_f32, keeps that contract).
//
// Operands: A (activations) fp32 as in lpg_fc_f32, split in registers by the
// lane that feeds it to the MFMA; W pre-split once per call (lpg_split3_f32:
// three bf16 planes, weights are small) so only A costs VALU in the k loop.
// Two kernels, both on v_mfma_f32_16x16x32_bf16 (which holds a higher clock
// under DVFS on gfx950 than 32x32x16) with 128 x 128 output tiles of four
// 32 x 128 wave strips: fc_x3_wide (the default: buffer_load ... lds staging)
// and fc_fwd_x3_16 (global_load_lds staging; takes operands fc_x3_wide cannot,
// and is the per-call alternative LPG_FC_KERNEL(1)).  Both:  k-tiles of BK = 32 staged by LDS-DMA
// (global_load_lds) into a 2-stage ring: A as 128-B fp32 rows (16-B chunk c of
// row r at c ^ ((r >> 1) & 7)), each W plane as 64-B bf16 rows (chunk c at
// c ^ ((r >> 2) & 3)); both make the ds_read_b128 fragment reads
// conflict-free.  80 KiB LDS per block (2 blocks per CU).  XCD-aware
// bijective block remap (each XCD walks contiguous m-tiles with all their
// n-tiles, so the A panel is re-read from that XCD's L2).
#include "common.h"
#include "fc_common.h"
#include "x3_split.h"

#include <cstdlib>
#include <type_traits>

#pragma clang fp contract(off)

namespace lpg {
namespace {

constexpr int BK = 32;

struct X3Args {
  int64_t M, N, K1, K2;
  const float *A1, *A2;
  const uint16_t *W1, *W2;  // three bf16 planes each, plane p at W + p * ps
  const float *bias;
  int64_t lda1, lda2, ldw1, ldw2, ps1, ps2;
  float *C;
  int64_t ldc;
  int64_t mt, nt;
  uint64_t seed;
  uint32_t drop_thresh;
  float drop_scale;
  int32_t accum;
  // fused heads (fc_fwd_x3_16 only): hw [hn][ldhw] fp32; per-(wave column tile, row) partial logits
  // to hpart [N / (TN * 16)][M][4]
  const float *hw;
  int64_t ldhw;
  int32_t hn;
  float *hpart;
  int64_t row_off;  // the dropout key of row m is row_keys[m] if given, else row_off + m (drop_row)
  int32_t store;    // 0: C is not written (LPG_FC_HEADS_ONLY: the logits are the only output)
  const int64_t *row_keys;
  // fused small-K weight gradient (fc_x3_wide WGK, lpg_fc_x3_relu_wgrad_f32): this GEMM's output g is the
  // gradient of a ReLU layer's output wy [M, N] whose inputs were [wx1 | wx2] (wk1 + wk2 <= 16 features,
  // conv1); each block writes the partial sums over its rows of dZ^T [wx1 | wx2 | 1], dZ = (wy > 0) ? g : 0,
  // to wpart[m-tile][k][n] (k < wk1 + wk2 + 1); g itself is not stored
  const float *wy, *wx1, *wx2;
  int64_t ldwy, ldwx1, ldwx2;
  int32_t wk1, wk2;
  float *wpart;
  // tile order of fc_x3_wide: 1 (the default) = n-split: the first half of the block ids (XCDs 0-3)
  // take n-tiles [0, nt/2) of every m-tile, the second half the rest -- an XCD's round of 64 blocks is
  // 16 m-tiles x 4 n-tiles, half of W and twice the A panels of the 8 x 8 order; 0 (the per-call kernel
  // choice 2, round 3's order) = each XCD walks contiguous m-tiles with all their n-tiles.  Past-L2
  // reads at 200 K x (1024 + 1024) -> 1024: 10.1 GB -> 6.7 GB per launch, 1-2 % faster
  // (profiles/r04_pmc_fc_x3_k2048_probe.json, r04_x3_order_ab.log)
  int32_t order;
  // "f16x2" operands (fc_x3_wide<..., F16 = true>): sa[m] = the power-of-2 scale of A row m (over both
  // k phases), sw[n] = that of W row n (both phases; W then holds two fp16 planes h, l of W * sw)
  const float *sa, *sw;
};

// dst plane p [rows, cols] (ldd) = term p of src (transposed: src is [cols, rows]).
// One thread per output pair (2 consecutive columns).
__global__ __launch_bounds__(256) void split3_planes(int64_t rows, int64_t cols, const float *__restrict__ src,
                                                     int64_t lds, int32_t transpose, uint16_t *__restrict__ dst,
                                                     int64_t ldd, int64_t ps) {
  const int64_t cp = (cols + 1) / 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < rows * cp; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cp, c = 2 * (i % cp);
    const bool two = c + 1 < cols;
    float x = transpose ? src[c * lds + r] : src[r * lds + c];
    float y = two ? (transpose ? src[(c + 1) * lds + r] : src[r * lds + c + 1]) : 0.f;
    const unsigned h = split_lvl(x, y), m = split_lvl(x, y), l = pk_bf16(x, y);
    uint16_t *d = dst + r * ldd + c;
    d[0] = (uint16_t)h;
    d[ps] = (uint16_t)m;
    d[2 * ps] = (uint16_t)l;
    if (two) {
      d[1] = (uint16_t)(h >> 16);
      d[ps + 1] = (uint16_t)(m >> 16);
      d[2 * ps + 1] = (uint16_t)(l >> 16);
    }
  }
}

// ---- f16x2 operand preparation (f16x2_scale, rowmax8, colfold_f32: fc_common.h) ---------------------
// sa[m] for the rows of [A1 | A2] (16-byte aligned rows, K1, K2 multiples of 4): one wave a row
__global__ __launch_bounds__(256) void rowscale_f32(int64_t M, int64_t K1, const float *__restrict__ A1, int64_t lda1,
                                                    int64_t K2, const float *__restrict__ A2, int64_t lda2,
                                                    float *__restrict__ sa) {
  const int lane = threadIdx.x & 63;
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < M; row += (int64_t)gridDim.x * 4) {
    float mx = 0.f;
    for (int ph = 0; ph < 2; ++ph) {
      const float *a = ph ? A2 : A1;
      const int64_t K = ph ? K2 : K1;
      if (!a || K == 0) continue;
      a += row * (ph ? lda2 : lda1);
      for (int64_t k = 4 * lane; k < K; k += 256) {
        const f32x4 v = *reinterpret_cast<const f32x4 *>(a + k);
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if (lane == 0) sa[row] = f16x2_scale(mx);
  }
}

// W for the f16x2 kernels: row r of [src1 | src2] (or column r of each with transpose) times its scale
// sw[r], as two fp16 planes h = RNE_f16(x s), l = RNE_f16(x s - h) at dst + p * ps; one block a row
__global__ __launch_bounds__(256) void split_f16x2_rows(int64_t rows, int64_t cols1, const float *__restrict__ src1,
                                                        int64_t lds1, int64_t cols2, const float *__restrict__ src2,
                                                        int64_t lds2, int32_t transpose, uint16_t *__restrict__ dst1,
                                                        int64_t ldd1, uint16_t *__restrict__ dst2, int64_t ldd2,
                                                        int64_t ps, float *__restrict__ sw) {
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    auto at = [&](int ph, int64_t c) {
      const float *src = ph ? src2 : src1;
      const int64_t ld = ph ? lds2 : lds1;
      return transpose ? src[c * ld + r] : src[r * ld + c];
    };
    float mx = 0.f;
    for (int ph = 0; ph < 2; ++ph)
      for (int64_t c = tid; c < (ph ? cols2 : cols1); c += 256) mx = fmaxf(mx, fabsf(at(ph, c)));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    const float sc = f16x2_scale(mx);
    for (int ph = 0; ph < 2; ++ph) {
      uint16_t *d = (ph ? dst2 : dst1) + r * (ph ? ldd2 : ldd1);
      for (int64_t c = tid; c < (ph ? cols2 : cols1); c += 256) {
        const float v = at(ph, c) * sc;
        const _Float16 h = (_Float16)v;
        const _Float16 l = (_Float16)sub_f32(v, (float)h);
        d[c] = __builtin_bit_cast(uint16_t, h);
        d[ps + c] = __builtin_bit_cast(uint16_t, l);
      }
    }
    if (tid == 0) sw[r] = sc;
  }
}

// sum over the 16 lanes of a DPP row (all lanes get it; fixed order): quad swaps, then the
// half-row and row mirrors -- VALU only (no LDS crossbar, no lgkmcnt waits)
__device__ __forceinline__ float sum16(float v) {
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));  // half mirror
  v = v + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));  // row mirror
  return v;
}

// ds_read_b128 serves a wave in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same
// +32, MI355X_MICROARCH.md §LDS): a fragment read (16 rows fr x one 16-B chunk per k group fg) is
// conflict-free when each group's 16 (row, chunk) pairs land on 16 distinct 4-bank slots.  These XOR
// maps give that for both images (searched over all linear maps of the row's low bits,
// tools/experiments/swz_search.py); the earlier (row >> 1) & 7 / (row >> 2) & 3 ones were 2-way
// conflicted on every fragment read (SQ_LDS_BANK_CONFLICT = half the LDS cycles).
__device__ __forceinline__ int swzA(int row, int chunk) {  // 128-B rows: 8 chunks
  return chunk ^ ((((row >> 1) & 1) << 2) | ((row >> 2) & 1));
}
__device__ __forceinline__ int swzW(int row, int chunk) { return chunk ^ (((row >> 2) & 1) << 1); }  // 64-B rows

// The same GEMM on v_mfma_f32_16x16x32_bf16 (MI355X_MICROARCH.md 'DVFS
// give-back' item 7: on random operands the chip holds a higher clock on this
// shape, ~1.12-1.15x the FLOP/s of 32x32x16 at equal cycles per FLOP).  One
// MFMA consumes a whole BK = 32 k-tile: lane group g = lane >> 4 feeds
// k = 8g .. 8g+7 (A: two 16-B chunks of its row, W: chunk g of each plane);
// LDS images: A as 128-B fp32 rows (16-B chunk c of row r at c ^ ((r >> 1) & 7)),
// each W plane as 64-B bf16 rows (chunk c at c ^ ((r >> 2) & 3)): 16 consecutive
// rows at one logical chunk land in 16 distinct bank slots.  Each wave owns
// (TM x TN) fragments of 16 x 16; output map col = lane & 15,
// row = 4 (lane >> 4) + r.
// HEADS: the fused-heads epilogue (lpg_fc_x3_heads_f32) is compiled only into the instantiations that
// use it, so the plain FC and input-gradient GEMMs carry none of its registers.
template <int WM, int WN, int TM, int TN, bool RELU, bool HEADS = false>
__global__ __launch_bounds__(64 * WM * WN, 2) void fc_fwd_x3_16(X3Args a) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
  constexpr int A_BYTES = BM * BK * 4, WP_BYTES = BN * BK * 2;
  constexpr int TILE_BYTES = A_BYTES + 3 * WP_BYTES;
  constexpr int PA = BM / 8 / NW;
  constexpr int PB = 3 * (BN / 16) / NW;
  static_assert(BM % (8 * NW) == 0 && (3 * BN / 16) % NW == 0, "tile rows must split into whole pieces per wave");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * TILE_BYTES];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);

  const float *srcA1[PA], *srcA2[PA];
  const uint16_t *srcW1[PB], *srcW2[PB];
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int row = (wave + NW * p) * 8 + (lane >> 3);
    int64_t gr = m0 + row;
    gr = gr < a.M ? gr : a.M - 1;
    const int off = swzA(row, lane & 7) * 4;
    srcA1[p] = a.A1 + gr * a.lda1 + off;
    srcA2[p] = a.A2 + gr * a.lda2 + off;
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int q = wave + NW * p, plane = q / (BN / 16);
    const int row = (q % (BN / 16)) * 16 + (lane >> 2);
    int64_t gn = n0 + row;
    gn = gn < a.N ? gn : a.N - 1;
    const int off = swzW(row, lane & 3) * 8;
    srcW1[p] = a.W1 + plane * a.ps1 + gn * a.ldw1 + off;
    srcW2[p] = a.W2 + plane * a.ps2 + gn * a.ldw2 + off;
  }
  auto stage = [&](int b, int t) {
    typedef __attribute__((address_space(3))) unsigned char lds_t;
    unsigned char *base = smem + b * TILE_BYTES;
    const bool p2 = t >= nk1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BK;
#pragma unroll
    for (int p = 0; p < PA; ++p)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>((p2 ? srcA2[p] : srcA1[p]) + k0),
                                       (lds_t *)(base + (wave + NW * p) * 1024), 16, 0, 0);
#pragma unroll
    for (int p = 0; p < PB; ++p)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>((p2 ? srcW2[p] : srcW1[p]) + k0),
                                       (lds_t *)(base + A_BYTES + (wave + NW * p) * 1024), 16, 0, 0);
  };

  f32x4 accH[TM][TN], accL[TM][TN];
  const f32x4 zero = {};
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) accH[i][j] = accL[i][j] = zero;

  const int fr = lane & 15, fg = lane >> 4;
  const int rA0 = wm * TM * 16 + fr, rB0 = wn * TN * 16 + fr;

  if (nk > 0) stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int b = 0;
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) stage(b ^ 1, t + 1);
    const unsigned char *T = smem + b * TILE_BYTES;
    auto ldb = [&](int j, bf16x8 (&bj)[3]) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bj[p] = *reinterpret_cast<const bf16x8 *>(T + A_BYTES + p * WP_BYTES + (rB0 + j * 16) * (BK * 2) +
                                                  swzW(rB0 + j * 16, fg) * 16);
    };
    auto mfma6 = [&](int i, int j, const Split3 &av, const bf16x8 (&bj)[3]) {
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av.l, bj[0], accL[i][j], 0, 0, 0);
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av.m, bj[1], accL[i][j], 0, 0, 0);
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av.h, bj[2], accL[i][j], 0, 0, 0);
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av.m, bj[0], accL[i][j], 0, 0, 0);
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av.h, bj[1], accL[i][j], 0, 0, 0);
      accH[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av.h, bj[0], accH[i][j], 0, 0, 0);
    };
    auto lda = [&](int i) {
      const unsigned char *ra = T + (rA0 + i * 16) * (BK * 4);
      return split3(*reinterpret_cast<const f32x4 *>(ra + swzA(rA0 + i * 16, 2 * fg) * 16),
                    *reinterpret_cast<const f32x4 *>(ra + swzA(rA0 + i * 16, 2 * fg + 1) * 16));
    };
    if constexpr (TN <= 4) {
      bf16x8 bv[TN][3];
#pragma unroll
      for (int j = 0; j < TN; ++j) ldb(j, bv[j]);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const Split3 av = lda(i);
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma6(i, j, av, bv[j]);
      }
    } else {  // wide wave tile (few A rows, many W columns): all A splits first, W streamed two fragments at a time
      Split3 av[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = lda(i);
#pragma unroll
      for (int j = 0; j < TN; j += 2) {
        bf16x8 b0[3], b1[3];
        ldb(j, b0);
        ldb(j + 1, b1);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          mfma6(i, j, av[i], b0);
          mfma6(i, j + 1, av[i], b1);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    b ^= 1;
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = accH[i][j] + accL[i][j];
  const int64_t mw = m0 + wm * TM * 16, nw = n0 + wn * TN * 16;
  if (a.accum) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int64_t col = nw + j * 16 + fr;
      col = col < a.N ? col : a.N - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int64_t row = mw + i * 16 + 4 * fg + r;
          row = row < a.M ? row : a.M - 1;
          acc[i][j][r] = acc[i][j][r] + a.C[row * a.ldc + col];
        }
    }
  }
  float hs[HEADS ? 4 : 1][TM][4];  // fused heads: this lane's partial logits [head][i][r]
  if constexpr (HEADS) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) hs[c][i][r] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = nw + j * 16 + fr;
    if (col >= a.N) continue;
    const float bb = a.bias ? a.bias[col] : 0.f;
    float hwv[HEADS ? 4 : 1];
    if constexpr (HEADS) {
#pragma unroll
      for (int c = 0; c < 4; ++c) hwv[c] = c < a.hn ? a.hw[c * a.ldhw + col] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = mw + i * 16 + 4 * fg + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r];
        if (a.bias) v = v + bb;
        if (RELU) v = (v < 0.f) ? 0.f : v;
        if (a.drop_thresh) v = drop_bits(a.seed, drop_row(a.row_keys, a.row_off, row, a.M), col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
        if (a.store) a.C[row * a.ldc + col] = v;
        if constexpr (HEADS) {
#pragma unroll
          for (int c = 0; c < 4; ++c) hs[c][i][r] = hs[c][i][r] + v * hwv[c];
        }
      }
    }
  }
  if constexpr (HEADS) {  // sum over the 16 lanes (columns) of each row group, fixed DPP order; lane fr = 0 writes
    const int64_t pidx = nw / (TN * 16);
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          hs[c][i][r] = c < a.hn ? sum16(hs[c][i][r]) : 0.f;
        }
    if (fr == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = mw + i * 16 + 4 * fg + r;
          if (row < a.M)
            *reinterpret_cast<f32x4 *>(a.hpart + (pidx * a.M + row) * 4) =
                f32x4{hs[0][i][r], hs[1][i][r], hs[2][i][r], hs[3][i][r]};
        }
    }
  }
}

// logits[m, c] = sum_t hpart[t][m][c] (t ascending) + hb[c]: the fused heads' fold
__global__ __launch_bounds__(256) void heads_fold(int64_t M, int64_t nparts, int32_t hn,
                                                  const float *__restrict__ hpart, const float *__restrict__ hb,
                                                  float *__restrict__ logits, int64_t ldl) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= M * hn) return;
  const int64_t m = i / hn;
  const int c = (int)(i % hn);
  float v = hpart[m * 4 + c];
  for (int64_t t = 1; t < nparts; ++t) v = v + hpart[(t * M + m) * 4 + c];
  if (hb) v = v + hb[c];
  logits[m * ldl + c] = v;
}

template <int WM, int WN, int TM, int TN, bool HEADS = false>
lpg_status launch_x3_16(X3Args a, bool relu, hipStream_t s) {
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16, NT = 64 * WM * WN;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_x3_f32: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_fwd_x3_16<WM, WN, TM, TN, true, HEADS>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((fc_fwd_x3_16<WM, WN, TM, TN, false, HEADS>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// ---- wide strips: fc_x3_wide (the default) -------------------------------------
//
// fc_fwd_x3_16 splits every A element once per block, so the split VALU per MFMA falls only as
// the block's N width grows; and its stage() spent ~6 VALU per LDS-DMA piece on 64-bit address
// arithmetic and phase selects (60 per k-tile, beside 88 of split).  fc_x3_wide: WM waves
// stacked along M, each owning a 16 x BN strip (BN = 16 TN): one A fragment split per k-tile
// feeds 6 TN MFMAs (TN = 16: 96).  Every DMA piece is a buffer_load ... lds through a
// descriptor per operand and phase (wave-uniform SGPRs), the lane's offset fixed for the whole
// loop and the k step in the scalar offset: no VALU per load, LDS destinations in M0 from SGPRs.
// Rows/columns past the edge are clamped (their outputs are never stored).  Same MFMA shape,
// k order and product sequence per output as fc_fwd_x3_16: the same C, bit for bit.
// Requires lda1 == lda2, ldw1 == ldw2, ps1 == ps2 (one offset set for both k phases; the host
// falls back to fc_fwd_x3_16 otherwise).
//
// F16 ("f16x2", round 5): A split in registers into two fp16 terms of (A row * sa[row]) and W given as
// two fp16 planes of (W row * sw[col]); per (i, j) three v_mfma_f32_16x16x32_f16 -- hh into accH, hl
// and lh into accL -- instead of six bf16 ones, and the sum rescaled by 1 / (sa sw) (powers of 2:
// exact) before the epilogue.  Representation error <= ~3 * 2^-22 of sum |a b| (a quarter of an fp32
// SGEMM's own; tools/experiments/split_error.py), half the matrix-core work.
#ifndef LPG_X3_EPI_NT
#define LPG_X3_EPI_NT 0
#endif
// the epilogue's streamed operands (the addend, the stored output, the conv1 fold's Y / C rows) as
// non-temporal accesses when LPG_X3_EPI_NT, as the bf16 kernels' epi_ld / epi_st (fc_bf16.hip).  Off: unlike
// there, the c2 step did not gain (fc_roofline 0.390 -> 0.385, profiles/r06_epi_nt_ab.log)
template <class T>
__device__ __forceinline__ T x3_ld(const T *p) {
  if constexpr (LPG_X3_EPI_NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <class T>
__device__ __forceinline__ void x3_st(T *p, T v) {
  if constexpr (LPG_X3_EPI_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int WM, int TM, int TN, int MINW, bool RELU, bool HEADS, bool WGK = false, bool F16 = false>
__global__ __launch_bounds__(64 * WM, MINW) void fc_x3_wide(X3Args a) {
  constexpr int NW = WM;
  constexpr int NP = F16 ? 2 : 3;  // W planes
  constexpr int BM = WM * TM * 16, BN = TN * 16;
  constexpr int A_BYTES = BM * BK * 4, WP_BYTES = BN * BK * 2;
  constexpr int TILE_BYTES = A_BYTES + NP * WP_BYTES;
  constexpr int SM_BYTES = 2 * (A_BYTES + 3 * WP_BYTES);  // both arithmetics: the epilogue images fit
  // DMA pieces of 1 KiB (one wave instruction): A pieces (8 rows x 128 B) first, then the W
  // pieces (16 rows x 64 B, plane by plane) -- piece q lands at q * 1 KiB of the tile image;
  // wave w moves pieces w, w + NW, ... (the last round partial when NW does not divide PT)
  constexpr int PA_T = BM / 8, PT = PA_T + NP * (BN / 16), PPW = (PT + NW - 1) / NW;
  static_assert(BM % 8 == 0 && BN % 16 == 0, "whole pieces");
  static_assert(TN % 2 == 0, "W fragments are consumed in pairs");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SM_BYTES];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + bid / 8;
#if defined(LPG_X3_TRAFFIC_PROBE)
  // probe builds only (tools/experiments/x3_traffic_probe.py; wrong results by design): every block
  // reads one W column slice (1: the A panels' traffic alone) or one A row panel (2: the W slices'
  // traffic alone), with the default schedule of the other operand
  const int64_t m0 = LPG_X3_TRAFFIC_PROBE == 2 ? 0 : (wgid / a.nt) * BM;
  const int64_t n0 = LPG_X3_TRAFFIC_PROBE == 1 ? 0 : (wgid % a.nt) * BN;
#else
  int64_t mi = wgid / a.nt, ni = wgid % a.nt;
  if (a.order == 1 && a.nt >= 2) {
    const int64_t nh = a.nt / 2, t0 = a.mt * nh;
    if (wgid < t0) {
      mi = wgid / nh;
      ni = wgid % nh;
    } else {
      mi = (wgid - t0) / (a.nt - nh);
      ni = nh + (wgid - t0) % (a.nt - nh);
    }
  } else if (a.order == 2 && a.nt % 4 == 0) {  // n-quarters: XCD pairs take a quarter of the n-tiles each
    const int64_t nq = a.nt / 4, tq = a.mt * nq, g = wgid / tq, w = wgid % tq;
    mi = w / nq;
    ni = g * nq + w % nq;
  }
  const int64_t m0 = mi * BM;
  const int64_t n0 = ni * BN;
#endif
  const int64_t mrows = a.M - m0 < BM ? a.M - m0 : BM;  // rows of this block (>= 1)
  const int64_t ncols = a.N - n0 < BN ? a.N - n0 : BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);

  // descriptors: A from row m0, W from column n0 (plane p at + p * ps); ranges cover exactly the
  // bytes the block reads, so a stray offset reads zeros instead of faulting (dma16)
  const int64_t kp1 = a.K1 > 0 ? a.K1 : BK, kp2 = a.K2 > 0 ? a.K2 : BK;
  const uint64_t pa1 = (uint64_t)(a.A1 + m0 * a.lda1), pw1 = (uint64_t)(a.W1 + n0 * a.ldw1);
  const uint64_t pa2 = a.A2 ? (uint64_t)(a.A2 + m0 * a.lda1) : pa1, pw2 = a.W2 ? (uint64_t)(a.W2 + n0 * a.ldw1) : pw1;
  const uint32_t na1 = (uint32_t)(((mrows - 1) * a.lda1 + kp1) * 4), na2 = (uint32_t)(((mrows - 1) * a.lda1 + kp2) * 4);
  const uint32_t nw1 = (uint32_t)(((NP - 1) * a.ps1 + (ncols - 1) * a.ldw1 + kp1) * 2);
  const uint32_t nw2 = (uint32_t)(((NP - 1) * a.ps1 + (ncols - 1) * a.ldw1 + kp2) * 2);
  uint32_t vo[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    const int q = wave + NW * p;
    if (q < PA_T) {
      const int row = q * 8 + (lane >> 3);
      const int64_t rc = row < mrows ? row : mrows - 1;  // rows past M feed outputs that are never stored
      vo[p] = (uint32_t)((rc * a.lda1 + swzA(row, lane & 7) * 4) * 4);
    } else {
      const int qw = q < PT ? q - PA_T : 0, plane = qw / (BN / 16);
      const int row = (qw % (BN / 16)) * 16 + (lane >> 2);
      const int64_t rc = row < ncols ? row : ncols - 1;
      vo[p] = (uint32_t)((plane * a.ps1 + rc * a.ldw1 + swzW(row, lane & 3) * 8) * 2);
    }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // the four descriptors (operand x k phase) once, in SGPRs: a stage selects, it does not rebuild
  const __amdgpu_buffer_rsrc_t rsa1 = dma_rsrc(pa1, na1), rsa2 = dma_rsrc(pa2, na2);
  const __amdgpu_buffer_rsrc_t rsw1 = dma_rsrc(pw1, nw1), rsw2 = dma_rsrc(pw2, nw2);
#else
  (void)pa2, (void)pw2, (void)na1, (void)na2, (void)nw1, (void)nw2;
#endif
  auto stage = [&](int b, int t) {
#if defined(__HIP_DEVICE_COMPILE__)
    const bool p2 = t >= nk1;
    const int kk = p2 ? t - nk1 : t;
    const __amdgpu_buffer_rsrc_t ra = p2 ? rsa2 : rsa1, rw = p2 ? rsw2 : rsw1;
    unsigned char *base = smem + b * TILE_BYTES;
#pragma unroll
    for (int p = 0; p < PPW; ++p) {
      const int q = wave + NW * p;  // wave-uniform
      if (PT % NW == 0 || q < PT) {
        if (q < PA_T)
          dma16r(ra, base + q * 1024, vo[p], kk * (BK * 4));
        else
          dma16r(rw, base + q * 1024, vo[p], kk * (BK * 2));
      }
    }
#else
    (void)b, (void)t;
#endif
  };

  f32x4 accH[TM][TN], accL[TM][TN];
  const f32x4 zero = {};
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) accH[i][j] = accL[i][j] = zero;

  const int fr = lane & 15, fg = lane >> 4;
  const int rA0 = wave * TM * 16 + fr;
  float sA[F16 ? TM : 1];  // F16: the scales of the A rows this lane splits
  // F16: the block's BM row scales and BN column scales in the last KiB of LDS (no tile, epilogue image or
  // WGK image reaches it), written here and read by the epilogue -- their load latency hidden under the
  // first tile's DMA instead of exposed after the last k-tile
  constexpr int SC_OFF = SM_BYTES - (BM + BN) * 4;
  static_assert(!F16 || (2 * TILE_BYTES <= SC_OFF && NW * TM * 16 * (BN + 4) * 4 + BM * 20 * 4 <= SC_OFF),
                "the scale slots clear the tile buffers and the epilogue images");
  float *const ssc = reinterpret_cast<float *>(smem + SC_OFF);  // [BM] row scales, then [BN] column scales
  if constexpr (F16) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t row = m0 + rA0 + i * 16;
      sA[i] = a.sa[row < a.M ? row : a.M - 1];
    }
    for (int q = tid; q < BM + BN; q += NW * 64) {
      const int64_t row = m0 + q, col = n0 + (q - BM);
      ssc[q] = q < BM ? a.sa[row < a.M ? row : a.M - 1] : a.sw[col < a.N ? col : a.N - 1];
    }
  }

  // the bias of this lane's output columns, loaded before the k loop (its latency hidden there instead of
  // exposed at the start of the epilogue, where it cost 2.5 % of a 200K-row launch: profiles/r06_epi_cost.log)
  float bpre[!WGK ? TN : 1];
  if constexpr (!WGK) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col = n0 + j * 16 + (lane & 15);
      bpre[j] = a.bias ? a.bias[col < a.N ? col : a.N - 1] : 0.f;
    }
  }
  if (nk > 0) stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  int b = 0;
  if constexpr (F16) {
    for (int t = 0; t < nk; ++t) {
      if (t + 1 < nk) stage(b ^ 1, t + 1);
      const unsigned char *T = smem + b * TILE_BYTES;
      Split2 av[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const unsigned char *ra = T + (rA0 + i * 16) * (BK * 4);
        av[i] = split2f16(*reinterpret_cast<const f32x4 *>(ra + swzA(rA0 + i * 16, 2 * fg) * 16),
                          *reinterpret_cast<const f32x4 *>(ra + swzA(rA0 + i * 16, 2 * fg + 1) * 16), sA[i]);
      }
      auto ldb = [&](int j, f16x8(&bj)[2]) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
          bj[p] = *reinterpret_cast<const f16x8 *>(T + A_BYTES + p * WP_BYTES + (j * 16 + fr) * (BK * 2) +
                                                   swzW(j * 16 + fr, fg) * 16);
      };
      auto mfma3 = [&](int i, int j, const f16x8(&bj)[2]) {
        accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i].l, bj[0], accL[i][j], 0, 0, 0);
        accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i].h, bj[1], accL[i][j], 0, 0, 0);
        accH[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[i].h, bj[0], accH[i][j], 0, 0, 0);
      };
      f16x8 c0[2], c1[2];
      ldb(0, c0);
      ldb(1, c1);
#pragma unroll
      for (int j = 0; j < TN; j += 2) {
        f16x8 n0_[2], n1_[2];
        if (j + 2 < TN) {
          ldb(j + 2, n0_);
          ldb(j + 3, n1_);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          mfma3(i, j, c0);
          mfma3(i, j + 1, c1);
        }
        if (j + 2 < TN) {
#pragma unroll
          for (int p = 0; p < 2; ++p) c0[p] = n0_[p], c1[p] = n1_[p];
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // tile t+1 landed; every wave done with tile t
      asm volatile("" ::: "memory");
      b ^= 1;
    }
  } else
  for (int t = 0; t < nk; ++t) {
    if (t + 1 < nk) stage(b ^ 1, t + 1);
    const unsigned char *T = smem + b * TILE_BYTES;
    Split3 av[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const unsigned char *ra = T + (rA0 + i * 16) * (BK * 4);
      av[i] = split3(*reinterpret_cast<const f32x4 *>(ra + swzA(rA0 + i * 16, 2 * fg) * 16),
                     *reinterpret_cast<const f32x4 *>(ra + swzA(rA0 + i * 16, 2 * fg + 1) * 16));
    }
    auto ldb = [&](int j, bf16x8(&bj)[3]) {
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bj[p] = *reinterpret_cast<const bf16x8 *>(T + A_BYTES + p * WP_BYTES + (j * 16 + fr) * (BK * 2) +
                                                  swzW(j * 16 + fr, fg) * 16);
    };
    auto mfma6 = [&](int i, int j, const bf16x8(&bj)[3]) {
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i].l, bj[0], accL[i][j], 0, 0, 0);
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i].m, bj[1], accL[i][j], 0, 0, 0);
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i].h, bj[2], accL[i][j], 0, 0, 0);
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i].m, bj[0], accL[i][j], 0, 0, 0);
      accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i].h, bj[1], accL[i][j], 0, 0, 0);
      accH[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i].h, bj[0], accH[i][j], 0, 0, 0);
    };
    // W fragments one pair ahead of the pair being multiplied
    bf16x8 c0[3], c1[3];
    ldb(0, c0);
    ldb(1, c1);
#pragma unroll
    for (int j = 0; j < TN; j += 2) {
      bf16x8 n0_[3], n1_[3];
      if (j + 2 < TN) {
        ldb(j + 2, n0_);
        ldb(j + 3, n1_);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        mfma6(i, j, c0);
        mfma6(i, j + 1, c1);
      }
      if (j + 2 < TN) {
#pragma unroll
        for (int p = 0; p < 3; ++p) c0[p] = n0_[p], c1[p] = n1_[p];
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile t+1 landed; every wave done with tile t
    asm volatile("" ::: "memory");
    b ^= 1;
  }

  const int64_t mw = m0 + wave * TM * 16, nw = n0;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = accH[i][j] + accL[i][j];
  if constexpr (F16) {  // undo the scales: output (row, col) times 1 / sa[row] times 1 / sw[col] (exact)
    // (as 4-vectors: packed multiplies, the same two roundings per element)
    f32x4 ia[TM];
    float iw[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const f32x4 s4 = *reinterpret_cast<const f32x4 *>(ssc + wave * TM * 16 + i * 16 + 4 * fg);
#pragma unroll
      for (int r = 0; r < 4; ++r) ia[i][r] = inv_pow2(s4[r]);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) iw[j] = inv_pow2(ssc[BM + j * 16 + fr]);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = acc[i][j] * ia[i] * f32x4{iw[j], iw[j], iw[j], iw[j]};
  }
  // fused heads (hn <= 3 here; the host routes hn = 4 to fc_fwd_x3_16): the store loops also put
  // each output into a per-wave LDS image (the tile buffers are free: every wave passed the last
  // k-tile's barrier), and a second pass reads them back column block by column block into this
  // lane's partial logits -- the same values in the same order as accumulating them in the store
  // loop, without 24 partial sums live beside the 64 outputs (that form spilled)
  constexpr int HC = HEADS ? 3 : 1;
  constexpr int HP = BN + 4;  // image row pitch (floats): rows 4 fg apart land 16 banks apart
  if constexpr (WGK) {
    // conv1's weight gradient folded into this input-gradient GEMM (the hidden layer's dZ W for the
    // conv1 output): the accumulators go to per-wave LDS images and the block's [BM][wk1 + wk2] input
    // rows beside them (x1 | x2 | 1 for the bias | zeros, KP floats a row); then each wave streams a
    // quarter of the block's rows -- the addend C and conv1's output Y read row by row, 512 contiguous
    // bytes per wave and row, U rows in flight -- forms dZ = (Y > 0) ? acc (+ C) : 0 for its lane's two
    // columns and advances their KP sums (v_pk_fma_f32); the four quarters are added in a fixed order.  One partial per (m-tile, k, n); g, the [M, N] gradient the separate pass re-read with Y,
    // is never stored.  (The first form loaded Y and C per accumulator register before the images,
    // one dependent 4-byte load after another: 2.94 ms against 1.76 for the plain launch at 200 K rows.)
    constexpr int KP = 20, U = 4;
    static_assert((NW * TM * 16 * HP + BM * KP) * 4 <= SM_BYTES, "images fit the tile buffers");
    float *const wimg = reinterpret_cast<float *>(smem);
    float *const xs = wimg + NW * TM * 16 * HP;
    const int ks = a.wk1 + a.wk2;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          wimg[wave * (TM * 16 * HP) + (i * 16 + 4 * fg + r) * HP + j * 16 + fr] = acc[i][j][r];
    for (int q = tid; q < BM * KP; q += NW * 64) {
      const int r = q / KP, k = q % KP;
      const int64_t row = m0 + r;
      float x = k == ks ? 1.f : 0.f;
      if (row < a.M && k < ks) x = k < a.wk1 ? a.wx1[row * a.ldwx1 + k] : a.wx2[row * a.ldwx2 + (k - a.wk1)];
      xs[q] = x;
    }
    __syncthreads();
    // wave q streams rows 32 q .. 32 q + 31 (wave-uniform, so the x rows are broadcast reads), lane l
    // columns 2 l and 2 l + 1: one x read serves four fmas, one 8-byte Y / C / d load two columns
    constexpr int RQ = BM / NW;
    static_assert(BN == 128 && RQ % (2 * U) == 0, "a wave row covers the 128 columns in pairs");
    const int64_t col0 = nw + 2 * lane;
    const bool cok0 = col0 < a.N;  // (N even: the pair is in or out together)
    const int64_t cc = cok0 ? col0 : a.N - 2;
    const bool acc_c = a.accum != 0;
    f32x2 s0[KP / 2], s1[KP / 2];
#pragma unroll
    for (int u = 0; u < KP / 2; ++u) s0[u] = s1[u] = f32x2{0.f, 0.f};
    // rows in groups of U, the next group's Y / C loads issued before the current group's arithmetic
    // (two register sets, alternating at compile time: a copy between them made hipcc wait first);
    // unconditional loads at clamped addresses (a conditional load became a branch with a vmcnt(0) at
    // its join), values selected after
    auto load = [&](int r0, f32x2 (&yv)[U], f32x2 (&cv)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = m0 + r0 + u;
        const bool ok = cok0 && row < a.M;
        const int64_t rr = row < a.M ? row : a.M - 1;
        const f32x2 y = x3_ld(reinterpret_cast<const f32x2 *>(a.wy + rr * a.ldwy + cc));
        const f32x2 cval = x3_ld(reinterpret_cast<const f32x2 *>(a.C + rr * a.ldc + cc));
        yv[u] = ok ? y : f32x2{0.f, 0.f};
        cv[u] = (ok && acc_c) ? cval : f32x2{0.f, 0.f};
      }
    };
    auto rows = [&](int r0, const f32x2 (&yv)[U], const f32x2 (&cv)[U]) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int lr = r0 + u;
        f32x2 d = *reinterpret_cast<const f32x2 *>(wimg + (lr / (TM * 16)) * (TM * 16 * HP) + (lr % (TM * 16)) * HP +
                                                   2 * lane);
        if (acc_c) d = d + cv[u];
        const float d0 = yv[u][0] > 0.f ? d[0] : 0.f, d1 = yv[u][1] > 0.f ? d[1] : 0.f;
        const f32x2 *xr = reinterpret_cast<const f32x2 *>(xs + lr * KP);
#pragma unroll
        for (int p = 0; p < KP / 2; ++p) {
          const f32x2 x = xr[p];
          s0[p] = __builtin_elementwise_fma(f32x2{d0, d0}, x, s0[p]);
          s1[p] = __builtin_elementwise_fma(f32x2{d1, d1}, x, s1[p]);
        }
      }
    };
    f32x2 ya[U], ca[U], yb[U], cb[U];
    load(wave * RQ, ya, ca);
    for (int r0 = wave * RQ; r0 < wave * RQ + RQ; r0 += 2 * U) {
      load(r0 + U, yb, cb);
      rows(r0, ya, ca);
      load(r0 + 2 * U, ya, ca);  // past the last group: rows of the next wave, never used (no branch)
      rows(r0 + U, yb, cb);
    }
    __syncthreads();  // the images are read: each wave's sums to LDS, added over the waves in order
    float *const hs = wimg;  // [wave][k][128 columns]
    static_assert(NW * KP * BN <= NW * TM * 16 * HP, "partial image fits the accumulator images");
#pragma unroll
    for (int p = 0; p < KP / 2; ++p)
#pragma unroll
      for (int e = 0; e < 2; ++e)
        *reinterpret_cast<f32x2 *>(hs + (wave * KP + 2 * p + e) * BN + 2 * lane) = f32x2{s0[p][e], s1[p][e]};
    __syncthreads();
    float *const pp = a.wpart + (m0 / BM) * (int64_t)(ks + 1) * a.N;
    for (int o = tid; o < (ks + 1) * BN; o += NW * 64) {
      const int k = o / BN, c = o % BN;
      float v = hs[k * BN + c];
#pragma unroll
      for (int q = 1; q < NW; ++q) v = v + hs[(q * KP + k) * BN + c];
      if (nw + c < a.N) pp[(int64_t)k * a.N + nw + c] = v;
    }
    return;
  }
  static_assert(!HEADS || NW * TM * 16 * HP * 4 <= SM_BYTES, "heads image fits the tile buffers");
  float *const himg = reinterpret_cast<float *>(smem) + wave * (TM * 16 * HP) + 4 * fg * HP + fr;
  auto hput = [&](int i, int r, int j, float v) {
    if constexpr (HEADS) himg[(i * 16 + r) * HP + j * 16] = v;
  };
  if (mw + TM * 16 <= a.M && nw + BN <= a.N) {
    // interior wave tile (wave-uniform): no per-element bounds, one C row pointer per (i, r) with
    // the column step j * 16 as the store's immediate offset, the dropout row keys computed once
    // per row (the per-element forms cost ~24 VALU incl. 6 v_mul_lo_u32 and a branch per output)
    float *const c0 = a.C + (mw + 4 * fg) * a.ldc + nw + fr;
    auto rp = [&](int i, int r) -> float * { return c0 + (i * 16 + r) * a.ldc; };
    if (a.accum) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = acc[i][j][r] + x3_ld(rp(i, r) + j * 16);
    }
    auto body = [&](auto bias_c, auto drop_c) {
      constexpr bool BIAS = decltype(bias_c)::value, DROP = decltype(drop_c)::value;
      // dropout: lanes fr = 2c and 2c + 1 hold the column pair c of the same four rows; the even lane
      // hashes rows 0-1 of the pair, the odd lane rows 2-3, and one DPP swap of adjacent lanes hands
      // each its partner's two -- two row keys and two pair hashes per lane and fragment, not four
      const int odd = fr & 1;
      uint32_t rk[TM][2];
      if constexpr (DROP) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            rk[i][h] = drop_row_key(a.seed, drop_row(a.row_keys, a.row_off, mw + i * 16 + 4 * fg + 2 * odd + h, a.M));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t col = nw + j * 16 + fr;
        float bb = 0.f;
        if constexpr (BIAS) bb = !WGK ? bpre[j] : a.bias[col];
        const uint32_t ck = drop_col_key(col);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          uint32_t hr[4] = {0u, 0u, 0u, 0u};  // the pair hash of row 4 fg + r
          if constexpr (DROP) {
            const uint32_t h0 = drop_hash_k(rk[i][0], ck), h1 = drop_hash_k(rk[i][1], ck);
            const uint32_t p0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)h0, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
            const uint32_t p1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)h1, 0xB1, 0xF, 0xF, false);
            hr[0] = odd ? p0 : h0;
            hr[1] = odd ? p1 : h1;
            hr[2] = odd ? h0 : p0;
            hr[3] = odd ? h1 : p1;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[i][j][r];
            if constexpr (BIAS) v = v + bb;
            if (RELU) v = (v < 0.f) ? 0.f : v;
            if constexpr (DROP) v = drop_half(hr[r], fr) >= a.drop_thresh ? v * a.drop_scale : 0.f;
            if (!HEADS || a.store) x3_st(rp(i, r) + j * 16, v);
            hput(i, r, j, v);
          }
        }
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    if (a.bias) {
      if (a.drop_thresh) body(T_{}, T_{}); else body(T_{}, F_{});
    } else {
      if (a.drop_thresh) body(F_{}, T_{}); else body(F_{}, F_{});
    }
  } else {  // edge wave tile: per-element bounds (same arithmetic, same bits)
    if (a.accum) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int64_t col = nw + j * 16 + fr;
        col = col < a.N ? col : a.N - 1;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            int64_t row = mw + i * 16 + 4 * fg + r;
            row = row < a.M ? row : a.M - 1;
            acc[i][j][r] = acc[i][j][r] + a.C[row * a.ldc + col];
          }
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col = nw + j * 16 + fr;
      if (col >= a.N) continue;
      const float bb = a.bias ? a.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = mw + i * 16 + 4 * fg + r;
          if (row >= a.M) continue;
          float v = acc[i][j][r];
          if (a.bias) v = v + bb;
          if (RELU) v = (v < 0.f) ? 0.f : v;
          if (a.drop_thresh) v = drop_bits(a.seed, drop_row(a.row_keys, a.row_off, row, a.M), col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
          if (!HEADS || a.store) a.C[row * a.ldc + col] = v;
          hput(i, r, j, v);
        }
    }
  }
  if constexpr (HEADS) {
    // this lane's partial logits [head][i][r] over its columns j * 16 + fr (columns past N and heads
    // past hn get zero weights; image entries never written belong to rows / columns never stored)
    float hs[HC][TM][4];
#pragma unroll
    for (int c = 0; c < HC; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) hs[c][i][r] = 0.f;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t col = nw + j * 16 + fr;
      const bool cok = col < a.N;
      float hwv[HC];
#pragma unroll
      for (int c = 0; c < HC; ++c) {
        const float w = a.hw[(c < a.hn ? c : a.hn - 1) * a.ldhw + (cok ? col : a.N - 1)];
        hwv[c] = (c < a.hn && cok) ? w : 0.f;
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = cok ? himg[(i * 16 + r) * HP + j * 16] : 0.f;
#pragma unroll
          for (int c = 0; c < HC; ++c) hs[c][i][r] = hs[c][i][r] + v * hwv[c];
        }
    }
    // sum over the 16 lanes (columns) of each row group, fixed DPP order; lane fr = 0 writes
    const int64_t pidx = nw / BN;
#pragma unroll
    for (int c = 0; c < HC; ++c)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) hs[c][i][r] = sum16(hs[c][i][r]);  // heads past hn sum zeros
    if (fr == 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = mw + i * 16 + 4 * fg + r;
          if (row < a.M)
            *reinterpret_cast<f32x4 *>(a.hpart + (pidx * a.M + row) * 4) =
                f32x4{hs[0][i][r], hs[1][i][r], hs[2][i][r], 0.f};
        }
    }
  }
}

// whether fc_x3_wide can take these operands (one offset set for both phases, 32-bit offsets)
bool wide_ok(const X3Args &a, int64_t BM, int64_t BN) {
  if (a.K1 > 0 && a.K2 > 0 && (a.lda1 != a.lda2 || a.ldw1 != a.ldw2 || a.ps1 != a.ps2)) return false;
  if (a.K1 == 0) return false;  // (the phase-1 operands carry the strides)
  const int64_t K = a.K1 > a.K2 ? a.K1 : a.K2;
  return (BM * a.lda1 + K) * 4 < ((int64_t)1 << 31) && (2 * a.ps1 + BN * a.ldw1 + K) * 2 < ((int64_t)1 << 31);
}

template <int WM, int TM, int TN, int MINW, bool HEADS = false, bool WGK = false, bool F16 = false>
lpg_status launch_x3_wide(X3Args a, bool relu, hipStream_t s) {
  constexpr int BM = WM * TM * 16, BN = TN * 16, NT = 64 * WM;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_x3_f32: grid too large");
  LPG_REQUIRE(!F16 || (a.sa && a.sw), "lpg_fc_f16x2: the row scales are missing");
  if constexpr (WGK) {
    hipLaunchKernelGGL((fc_x3_wide<WM, TM, TN, MINW, false, false, true, F16>), dim3((unsigned)nwg), dim3(NT), 0, s,
                       a);
    LPG_HIP(hipGetLastError());
    return LPG_OK;
  }
  if (relu)
    hipLaunchKernelGGL((fc_x3_wide<WM, TM, TN, MINW, true, HEADS, false, F16>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((fc_x3_wide<WM, TM, TN, MINW, false, HEADS, false, F16>), dim3((unsigned)nwg), dim3(NT), 0, s,
                       a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// ---- weight gradient dW = G^T X on the same arithmetic -----------------------
//
// dW[n, k] = sum_r G[r, n] X[r, k] (G = dZ [R, N], X = the layer input [R, K]:
// the lin_rel / lin_root weight gradients of GraphConv, torch Linear layout).
// Both operands are r-major, so a lane's 8 consecutive MFMA k (= rows r) of
// one output row n are 8 separate dwords: the LDS image keeps the natural
// 512-B rows (32 r-rows x 128 columns per operand and k-tile, LDS-DMA, no
// swizzle needed: a ds_read_b32's two 32-lane halves each read 32 consecutive
// dwords of one row -- conflict-free), each lane reads its 8 values with
// ds_read_b32 and splits them (three bf16 terms, as above) in registers.
// The output (N x K, 64 tiles at 1024^2) is far too small to fill 256 CUs, so
// R is split into S contiguous ranges (whole 32-row chunks); block (tile, s)
// writes its partial tile to workspace[s], and a fold kernel adds the S
// partials in s order (deterministic, no atomics).  Rows past R are DMA'd
// from a zeroed 512-B row at the end of the workspace.
constexpr int WG_T = 128;  // output tile (n and k)

// The weight-gradient kernel: each thread loads three columns' 8 consecutive rows of G or X (one
// dword per row through a buffer descriptor over the block's R range: rows past R read zeros, no
// branch; a wave's 64 lanes read 256 contiguous bytes of a row), splits each column's 8 values into
// three bf16x8 (k = the 8 rows) and writes them with ds_write_b128 into plane images laid out for
// the MFMA ([column][32 rows] bf16, 64-B rows, chunk c at c ^ ((col >> 2) & 3): the fc kernel's
// W-plane image, read conflict-free by 16 consecutive columns); 8 waves (4 x 2, 64 x 64 each,
// 16x16x32) read b128 fragments.  A 256 (n) x 128 (k) output tile per 512-thread block, one block
// per CU, and TWO plane buffers (2 x 72 KiB).  A split-then-multiply form (round 1's cooperative
// kernel) keeps both waves of a SIMD in the same phase, so the split VALU and the MFMAs never
// overlap.  Here chunk c + 1 is split into the other buffer in the same iteration as chunk c's
// MFMAs, one unit after each fragment row (the loop is unrolled by two so the buffers are
// compile-time distinct), and each unit's chunk c + 2 loads go out right behind its split; one
// barrier per chunk.  Each G element is split once per 128 k-columns and each X element once per
// 256 n-columns: 1.375 split VALU per MFMA, the same for every wave.  (Round 2's loader gave waves
// 0-3 G and waves 4-7 X with 6-7 repeating 4-5's work, 1.83 per MFMA on every SIMD, and issued a
// chunk's loads one fragment row before their use: 189 / 211 TF/s at R = 100 / 200 K against 197 /
// 218 for the balanced tasks, profiles/r03_wgrad_bal.log.)
//
// F16 (f16x2, round 5): G column n and X column k times their power-of-2 column scales sG[n], sX[k]
// (lpg_colscale_f32), split into two fp16 terms; three v_mfma_f32_16x16x32_f16 per fragment pair
// (hh into accH, hl + lh into accL) and the partial tile times 1 / (sG sX) (exact) at the store.
template <bool F16 = false>
__global__ __launch_bounds__(512, 1) void wgrad_x3w(int64_t R, int64_t N, int64_t K, const float *__restrict__ G,
                                                    int64_t ldg, const float *__restrict__ X, int64_t ldx,
                                                    float *__restrict__ part, int64_t nt, int64_t kt,
                                                    int64_t chunks_per_split, const float *__restrict__ sG,
                                                    const float *__restrict__ sX) {
  constexpr int GC = 256, XC = 128;               // tile columns of G (n) and X (k)
  constexpr int GP = GC * 32 * 2, XP = XC * 32 * 2;  // one plane image: columns x 32 rows x bf16
  constexpr int NPL = F16 ? 2 : 3;                // planes per operand
  constexpr int BUFB = NPL * GP + NPL * XP;       // one buffer: G planes, then X planes (72 / 48 KiB)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUFB];

  const int64_t nwg = (int64_t)gridDim.x, xcd = (int64_t)blockIdx.x % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t bid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (int64_t)blockIdx.x / 8;
  const int64_t tiles = nt * kt;
  const int64_t s = bid / tiles, tile = bid % tiles;
  const int64_t n0 = (tile / kt) * GC, k0 = (tile % kt) * XC;
  const int64_t nchunks = (R + 31) / 32;
  const int64_t c0 = s * chunks_per_split;
  const int64_t c1 = c0 + chunks_per_split < nchunks ? c0 + chunks_per_split : nchunks;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // loader tasks, the same for every thread (so every SIMD carries the same split VALU, whichever
  // waves it hosts): three split units of 8 rows (rg * 8 .. + 7, rg = tid >> 7) per chunk -- unit 0
  // G column gc, unit 1 G column 128 + gc, unit 2 X column gc (gc = tid & 127): 24 elements per
  // lane, every G and X element split once per block and chunk (G once per 128 k-columns, X once
  // per 256 n-columns).  Each unit has its own 8 registers: its next chunk's loads are issued as
  // soon as it has been split, a whole multiply ahead of their use.
  const int gc = tid & 127, rg = tid >> 7;
  // columns past the edge are clamped (their outputs are never stored)
  const int64_t col_u[3] = {n0 + gc < N ? n0 + gc : N - 1, n0 + 128 + gc < N ? n0 + 128 + gc : N - 1,
                            k0 + gc < K ? k0 + gc : K - 1};
  // descriptors from row c0 * 32 (rows past R out of range: zeros, no branch)
  const float *gbase = G + c0 * 32 * ldg + n0, *xbase = X + c0 * 32 * ldx + k0;
  const int64_t gleft = (R - c0 * 32) * ldg * 4, xleft = (R - c0 * 32) * ldx * 4;
  const uint32_t gbytes = (uint32_t)(gleft < 0x7fffffff ? gleft : 0x7fffffff);
  const uint32_t xbytes = (uint32_t)(xleft < 0x7fffffff ? xleft : 0x7fffffff);
  float raw[3][8];
  auto load_unit = [&](int u, int64_t c) {  // c clamped to the last chunk: a spare re-load at the end, no branch
    c = c < c1 ? c : c1 - 1;
    const bool isg = u < 2;
    const int64_t ld = isg ? ldg : ldx;
    const int voff = (int)((col_u[u] - (isg ? n0 : k0)) * 4 + rg * 8 * ld * 4);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      raw[u][e] = buf_load1(isg ? gbase : xbase, isg ? gbytes : xbytes, voff, (int)(((c - c0) * 32 + e) * ld * 4));
  };
  auto load = [&](int64_t c) {
#pragma unroll
    for (int u = 0; u < 3; ++u) load_unit(u, c);
  };
  float su[F16 ? 3 : 1];  // F16: the scales of this thread's three columns
  if constexpr (F16) {
#pragma unroll
    for (int u = 0; u < 3; ++u) su[u] = u < 2 ? sG[col_u[u]] : sX[col_u[u]];
  }
  auto split_col = [&](unsigned char *buf, int u) {  // unit u's 8 rows -> three bf16x8 (F16: two f16x8)
    const int col = u == 1 ? 128 + gc : gc, pl = u < 2 ? GP : XP;
    unsigned char *dst = buf + (u < 2 ? 0 : NPL * GP) + col * 64 + swzW(col, rg) * 16;
    if constexpr (F16) {
      const Split2 t = split2f16(f32x4{raw[u][0], raw[u][1], raw[u][2], raw[u][3]},
                                 f32x4{raw[u][4], raw[u][5], raw[u][6], raw[u][7]}, su[u]);
      *reinterpret_cast<f16x8 *>(dst) = t.h;
      *reinterpret_cast<f16x8 *>(dst + pl) = t.l;
    } else {
      const Split3 t = split3(f32x4{raw[u][0], raw[u][1], raw[u][2], raw[u][3]},
                              f32x4{raw[u][4], raw[u][5], raw[u][6], raw[u][7]});
      *reinterpret_cast<bf16x8 *>(dst) = t.h;
      *reinterpret_cast<bf16x8 *>(dst + pl) = t.m;
      *reinterpret_cast<bf16x8 *>(dst + 2 * pl) = t.l;
    }
  };

  const int wm = wave >> 1, wn = wave & 1;  // 4 (n) x 2 (k) waves of 64 x 64
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 accH[4][4], accL[4][4];
  const f32x4 zero = {};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) accH[i][j] = accL[i][j] = zero;
  auto frag = [&](const unsigned char *im, int plane, int col, bf16x8(&f)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const bf16x8 *>(im + p * plane + col * 64 + swzW(col, fg) * 16);
  };
  auto frag16 = [&](const unsigned char *im, int plane, int col, f16x8(&f)[2]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) f[p] = *reinterpret_cast<const f16x8 *>(im + p * plane + col * 64 + swzW(col, fg) * 16);
  };
  // multiply the chunk in buf; with `next`, split unit i - 1 of the next chunk (raw) into it after
  // fragment row i - 1's 24 MFMAs and issue that unit's loads of chunk `cload` (in source order, so
  // the VALU lands between MFMA groups)
  // (`split` a std::integral_constant: a runtime `next != nullptr` test -- hipcc cannot prove an LDS
  // pointer non-null -- put a branch around every split, and at each join the waitcnt pass assumed
  // the path without the other units' loads and waited for all of them)
  auto multiply = [&](const unsigned char *buf, unsigned char *next, int64_t cload, auto split) {
    if constexpr (F16) {
      f16x8 bv[4][2];
#pragma unroll
      for (int j = 0; j < 4; ++j) frag16(buf + 2 * GP, XP, wn * 64 + j * 16 + fr, bv[j]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (decltype(split)::value && i > 0) {
          split_col(next, i - 1);
          __builtin_amdgcn_sched_barrier(0);
          load_unit(i - 1, cload);
        }
        f16x8 av[2];
        frag16(buf, GP, wm * 64 + i * 16 + fr, av);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[1], bv[j][0], accL[i][j], 0, 0, 0);
          accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[0], bv[j][1], accL[i][j], 0, 0, 0);
          accH[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[0], bv[j][0], accH[i][j], 0, 0, 0);
        }
      }
      return;
    } else {
    bf16x8 bv[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) frag(buf + 3 * GP, XP, wn * 64 + j * 16 + fr, bv[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (decltype(split)::value && i > 0) {
        split_col(next, i - 1);
        // the unit's registers are free only once its split has read them: a load hoisted above
        // the split made hipcc copy the in-flight values out first, and wait for every load to do so
        __builtin_amdgcn_sched_barrier(0);
        load_unit(i - 1, cload);
      }
      bf16x8 av[3];
      frag(buf, GP, wm * 64 + i * 16 + fr, av);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[2], bv[j][0], accL[i][j], 0, 0, 0);
        accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1], bv[j][1], accL[i][j], 0, 0, 0);
        accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv[j][2], accL[i][j], 0, 0, 0);
        accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1], bv[j][0], accL[i][j], 0, 0, 0);
        accL[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv[j][1], accL[i][j], 0, 0, 0);
        accH[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv[j][0], accH[i][j], 0, 0, 0);
      }
    }
    }
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  unsigned char *const B0 = smem, *const B1 = smem + BUFB;
  // prologue: chunk c0 split into B0, chunk c0 + 1's loads in flight
  load(c0);
#pragma unroll
  for (int u = 0; u < 3; ++u) split_col(B0, u);
  load(c0 + 1);
  sync();
  // half-iteration (chunk c in one buffer, chunk c+1's loads landed or landing): multiply it, split
  // c+1 into the other buffer unit by unit, each unit's c+2 loads issued behind its split, barrier.
  // Past the end the split writes B0 with a spare chunk nobody reads.
  int64_t c = c0;
  for (; c + 1 < c1; c += 2) {
    multiply(B0, B1, c + 2, std::true_type{});
    sync();
    multiply(B1, B0, c + 3, std::true_type{});
    sync();
  }
  if (c < c1) multiply(B0, nullptr, 0, std::false_type{});  // odd count: the last chunk sits in B0

  float *P = part + s * N * K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t col = k0 + wn * 64 + j * 16 + fr;
    if (col >= K) continue;
    const float ix = F16 ? inv_pow2(sX[col]) : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = n0 + wm * 64 + i * 16 + 4 * fg + r;
        if (row < N) {
          float v = accH[i][j][r] + accL[i][j][r];
          if constexpr (F16) v = v * inv_pow2(sG[row]) * ix;
          P[row * K + col] = v;
        }
      }
  }
}

// per-column maxima of |G| (N, ldg multiples of 4, 16-byte aligned rows): block (column block of 1024,
// row chunk of rc) -- a thread's 4 columns as float4 over the chunk, eight rows in flight -- then one
// integer atomicMax per column on the bits (|x| >= 0: the uint order is the float order, NaN above
// every number): the same maxima whatever the order, so deterministic
__global__ __launch_bounds__(256) void colmax_f32(int64_t R, int64_t N, const float *__restrict__ G, int64_t ldg,
                                                  int64_t rc, unsigned *__restrict__ mbits) {
  const int64_t c4 = ((int64_t)blockIdx.y * 256 + threadIdx.x) * 4, chunk = blockIdx.x;  // x: row chunks (any R)
  if (c4 >= N) return;
  const int64_t r0 = chunk * rc, r1 = r0 + rc < R ? r0 + rc : R;
  f32x4 m = {0.f, 0.f, 0.f, 0.f};
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4 *>(G + (r + u) * ldg + c4);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], fabsf(v[u][e]));
  }
  for (; r < r1; ++r) {
    const f32x4 v = *reinterpret_cast<const f32x4 *>(G + r * ldg + c4);
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], fabsf(v[e]));
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) atomicMax(mbits + c4 + e, __float_as_uint(m[e]));
}

__global__ __launch_bounds__(256) void colscale_f32(int64_t N, const unsigned *__restrict__ mbits,
                                                    float *__restrict__ scale) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col < N) scale[col] = f16x2_scale(mbits ? __uint_as_float(mbits[col]) : 0.f);
}

// Row AND column maxima of |G| in one read (an operand that is both a row-scaled GEMM A operand and a
// column-scaled weight-gradient operand: the layer inputs, dZ, S^T dZ).  colmax_f32's blocks (column
// block of 1024, row chunk of rc <= 256, sixteen rows in flight); a thread's four |x| of each of
// eight rows reduce to one value per row, the eight rows over the wave's 64 lanes in a halving
// butterfly (each exchange halves the values a lane carries: 4 + 2 + 1 + 1 + 1 + 1 shuffles for
// eight rows, not 48), the four waves through LDS.  One column block (N <= 1024): the row's scale
// stored directly; else an integer atomicMax per (row, column block) into rbits.  The chunk's column
// maxima go to cpart[chunk][N] with plain stores (an atomicMax per column and chunk cost a third of
// the sweep: hundreds of chunks hit each column's address) and colfold_f32 folds them.
__global__ __launch_bounds__(256) void rowcolmax_f32(int64_t R, int64_t N, const float *__restrict__ G, int64_t ldg,
                                                     int64_t rc, float *__restrict__ cpart,
                                                     unsigned *__restrict__ rbits, float *__restrict__ rscale) {
  __shared__ float red[4][256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // blockIdx.x: the row chunk (the x dimension takes any R), blockIdx.y: the 1024-column block
  const int64_t c4 = ((int64_t)blockIdx.y * 256 + tid) * 4, r0 = (int64_t)blockIdx.x * rc;
  const int64_t r1 = r0 + rc < R ? r0 + rc : R;
  const bool col_ok = c4 < N;
  const int slot = rowmax8_slot(lane);
  f32x4 m = {0.f, 0.f, 0.f, 0.f};
  auto load8 = [&](int64_t r, f32x4(&v)[8]) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[u] = (col_ok && r + u < r1) ? *reinterpret_cast<const f32x4 *>(G + (r + u) * ldg + c4) : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // the next eight rows' loads issued before this eight's reduction: sixteen rows in flight
  f32x4 v[8], nv[8];
  load8(r0, v);
  for (int64_t r = r0; r < r1; r += 8) {
    if (r + 8 < r1) load8(r + 8, nv);
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float a0 = fabsf(v[u][0]), a1 = fabsf(v[u][1]), a2 = fabsf(v[u][2]), a3 = fabsf(v[u][3]);
      m[0] = fmaxf(m[0], a0);
      m[1] = fmaxf(m[1], a1);
      m[2] = fmaxf(m[2], a2);
      m[3] = fmaxf(m[3], a3);
      x[u] = fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
    }
    const float w = rowmax8(x, lane);
    if ((lane & 7) == 0) red[wave][r - r0 + slot] = w;  // (rows past r1 write zeros into unused slots)
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = nv[u];
  }
  if (col_ok) *reinterpret_cast<f32x4 *>(cpart + (int64_t)blockIdx.x * N + c4) = m;
  __syncthreads();
  if (tid < r1 - r0) {
    const float mx = fmaxf(fmaxf(red[0][tid], red[1][tid]), fmaxf(red[2][tid], red[3][tid]));
    if (rscale)
      rscale[r0 + tid] = f16x2_scale(mx);
    else
      atomicMax(rbits + r0 + tid, __float_as_uint(mx));
  }
}

// dW[n, k] = sum_s part[s][n, k], s ascending (fixed order), float4 per thread
__global__ __launch_bounds__(256) void wgrad_fold(int64_t N, int64_t K, int64_t S, const float *__restrict__ part,
                                                  float *__restrict__ dW, int64_t lddw) {
  const int64_t i4 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t k4 = K / 4;
  if (i4 >= N * k4) return;
  const int64_t n = i4 / k4, k = (i4 % k4) * 4;
  float4 acc = *reinterpret_cast<const float4 *>(part + n * K + k);
  for (int64_t s = 1; s < S; ++s) {
    const float4 v = *reinterpret_cast<const float4 *>(part + s * N * K + n * K + k);
    acc.x = acc.x + v.x;
    acc.y = acc.y + v.y;
    acc.z = acc.z + v.z;
    acc.w = acc.w + v.w;
  }
  *reinterpret_cast<float4 *>(dW + n * lddw + k) = acc;
}

// The R split of the x3 weight gradient: a function of the shape only (no environment or global
// state), so a given (R, N, K) always folds its partials in the same order -- the same dW bits.
int64_t wgrad_splits(int64_t R, int64_t N, int64_t K) {
  // one block per CU, one round: the kernel's 256 x 128 tiles times S row ranges = the CU count.  Round 6
  // (tools/experiments/wgrad_split_ab.py, profiles/r06_wgrad_split_ab.log): at N = K = 1024 S = 8 (256
  // blocks) runs R = 100 K / 200 K in 0.69 / 1.25 ms against 0.74 / 1.30 for the former 1024 blocks (four
  // rounds, 4x the partial tiles to fold) and 0.80 / 1.52 for a round and a half
  const int64_t tiles = ((N + 255) / 256) * ((K + 127) / 128);
  const int64_t nchunks = (R + 31) / 32;
  const int64_t cus = device_cus();
  int64_t S = (cus + tiles - 1) / tiles;
  const int64_t maxS = nchunks / 8 > 1 ? nchunks / 8 : 1;  // >= 8 chunks (256 rows) per split
  if (S > maxS) S = maxS;
  if (S > 64) S = 64;
  return S < 1 ? 1 : S;
}

// FC kernel choice, per call in flags bits 8-11 (LPG_FC_KERNEL(k), include/lpgnn.h): 0 = fc_x3_wide
// <4,2,8,2> in the n-split tile order when wide_ok (else 1), 1 = fc_fwd_x3_16 <4,1,2,8>, 2 = fc_x3_wide
// in round 3's contiguous-m tile order, 3 = fc_x3_wide in the n-quarter order (XCD pairs take a quarter
// of the n-tiles each; X3Args::order).  Same MFMA shape, k order and product
// sequence per output: the same C, bit for bit.  (tools/experiments/exp_wide.py at the c2 shapes:
// 207-221 TF/s for the wide form, +3-6 % over fc_fwd_x3_16.)
constexpr int kX3Kernels = 3;

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" lpg_status lpg_rowscale_f32(int64_t M, int64_t K1, const float *A1, int64_t lda1, int64_t K2,
                                       const float *A2, int64_t lda2, float *scale, void *stream) {
  LPG_REQUIRE(M >= 0 && K1 >= 0 && K2 >= 0, "lpg_rowscale_f32: negative size");
  if (M == 0) return LPG_OK;
  LPG_REQUIRE(scale && (K1 == 0 || A1) && (K2 == 0 || A2), "lpg_rowscale_f32: NULL pointer");
  LPG_REQUIRE(K1 % 4 == 0 && K2 % 4 == 0 && (K1 == 0 || (lda1 >= K1 && lda1 % 4 == 0 && aligned16(A1))) &&
                  (K2 == 0 || (lda2 >= K2 && lda2 % 4 == 0 && aligned16(A2))),
              "lpg_rowscale_f32: K and leading dimensions multiples of 4 floats, rows 16-byte aligned");
  int64_t blocks = (M + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(rowscale_f32, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), M, K1,
                     K1 ? A1 : nullptr, lda1, K2, K2 ? A2 : nullptr, lda2, scale);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_split_f16x2(int64_t rows, int64_t cols1, const float *src1, int64_t lds1, int64_t cols2,
                                      const float *src2, int64_t lds2, int32_t transpose, uint16_t *dst1,
                                      int64_t ldd1, uint16_t *dst2, int64_t ldd2, int64_t plane_stride, float *scale,
                                      void *stream) {
  LPG_REQUIRE(rows >= 0 && cols1 >= 0 && cols2 >= 0, "lpg_split_f16x2: negative size");
  if (rows == 0) return LPG_OK;
  LPG_REQUIRE(scale && (cols1 == 0 || (src1 && dst1)) && (cols2 == 0 || (src2 && dst2)), "lpg_split_f16x2: NULL pointer");
  LPG_REQUIRE((cols1 == 0 || (lds1 >= (transpose ? rows : cols1) && ldd1 >= cols1 && plane_stride >= rows * ldd1)) &&
                  (cols2 == 0 || (lds2 >= (transpose ? rows : cols2) && ldd2 >= cols2 && plane_stride >= rows * ldd2)),
              "lpg_split_f16x2: bad leading dimension / plane stride");
  int64_t blocks = rows < 16384 ? rows : 16384;
  hipLaunchKernelGGL(split_f16x2_rows, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), rows, cols1, src1,
                     lds1, cols2, src2, lds2, transpose, dst1, ldd1, dst2, ldd2, plane_stride, scale);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_split3_f32(int64_t rows, int64_t cols, const float *src, int64_t lds, int32_t transpose,
                                     uint16_t *dst, int64_t ldd, int64_t plane_stride, void *stream) {
  LPG_REQUIRE(rows >= 0 && cols >= 0, "lpg_split3_f32: negative size");
  if (rows == 0 || cols == 0) return LPG_OK;
  LPG_REQUIRE(src && dst, "lpg_split3_f32: NULL pointer");
  LPG_REQUIRE(lds >= (transpose ? rows : cols) && ldd >= cols && plane_stride >= rows * ldd,
              "lpg_split3_f32: bad leading dimension / plane stride");
  int64_t blocks = (rows * ((cols + 1) / 2) + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(split3_planes, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), rows, cols, src, lds,
                     transpose, dst, ldd, plane_stride);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

static lpg_status x3_args(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                          const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                          int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *bias,
                          float *C, int64_t ldc, int32_t flags, float dropout_p, uint64_t seed,
                          int64_t row_offset, const int64_t *row_keys, X3Args *out) {
  const bool heads_only = flags & LPG_FC_HEADS_ONLY;
  LPG_REQUIRE((C != nullptr || (heads_only && !(flags & LPG_FC_ACCUMULATE))) && ldc >= N, "lpg_fc_x3_f32: bad C/ldc");
  LPG_REQUIRE(K1 % BK == 0 && K2 % BK == 0, "lpg_fc_x3_f32: K1, K2 must be multiples of %d (zero-pad)", BK);
  LPG_REQUIRE(K1 == 0 || (A1 && W1 && lda1 >= K1 && ldw1 >= K1 && ps1 >= N * ldw1), "lpg_fc_x3_f32: bad A1/W1");
  LPG_REQUIRE(K2 == 0 || (A2 && W2 && lda2 >= K2 && ldw2 >= K2 && ps2 >= N * ldw2), "lpg_fc_x3_f32: bad A2/W2");
  LPG_REQUIRE(lda1 % 4 == 0 && ldw1 % 8 == 0 && ps1 % 8 == 0 &&
                  (K2 == 0 || (lda2 % 4 == 0 && ldw2 % 8 == 0 && ps2 % 8 == 0)) &&
                  (K1 == 0 || (aligned16(A1) && aligned16(W1))) && (K2 == 0 || (aligned16(A2) && aligned16(W2))),
              "lpg_fc_x3_f32: A rows must be 16-byte aligned (lda multiple of 4), W planes 16-byte aligned "
              "(ldw and plane stride multiples of 8)");
  LPG_REQUIRE((flags & ~0xf07) == 0 && ((flags >> 8) & 15) <= kX3Kernels, "lpg_fc_x3_f32: unknown flags 0x%x", flags);
  LPG_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "lpg_fc_x3_f32: dropout_p %g not in [0, 1)", (double)dropout_p);
  *out = X3Args{M, N, K1, K2, A1, A2, W1, W2, bias, lda1, lda2, ldw1, ldw2, ps1, ps2, C, ldc, 0, 0, seed, 0u, 1.f,
                (flags >> 1) & 1};
  dropout_params(dropout_p, &out->drop_thresh, &out->drop_scale);
  out->row_off = row_offset;
  out->row_keys = row_keys;
  out->store = heads_only ? 0 : 1;
  return LPG_OK;
}

// the plain FC of both arithmetics: x3 (sa == nullptr) or f16x2 (sa, sw: the row scales; W two fp16 planes)
static lpg_status fc_x3_plain(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const uint16_t *W1,
                              int64_t ldw1, int64_t ps1, int64_t K2, const float *A2, int64_t lda2,
                              const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *sa, const float *sw,
                              const float *bias, float *C, int64_t ldc, int32_t flags, float dropout_p, uint64_t seed,
                              int64_t row_offset, const int64_t *row_keys, void *stream) {
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "lpg_fc_x3_f32: negative size");
  if (M == 0 || N == 0) return LPG_OK;
  LPG_REQUIRE(!(flags & LPG_FC_HEADS_ONLY), "lpg_fc_x3_f32: LPG_FC_HEADS_ONLY needs the heads entry");
  X3Args a;
  const lpg_status st = x3_args(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, bias, C, ldc, flags,
                                dropout_p, seed, row_offset, row_keys, &a);
  if (st != LPG_OK) return st;
  hipStream_t s = as_stream(stream);
  const bool relu = flags & 1;
  const int kern = (flags >> 8) & 15;
  a.order = kern == 2 ? 0 : kern == 3 ? 2 : 1;
  if (sa) {
    LPG_REQUIRE(sw, "lpg_fc_f16x2_f32: sw is NULL");
    if (!wide_ok(a, 128, 128)) {
      set_error("lpg_fc_f16x2_f32: operands the wide kernel does not take (lda1 == lda2, ldw1 == ldw2, ps1 == ps2)");
      return LPG_ERR_UNSUPPORTED;
    }
    a.sa = sa;
    a.sw = sw;
    return launch_x3_wide<4, 2, 8, 2, false, false, true>(a, relu, s);
  }
  if (kern != 1 && wide_ok(a, 128, 128)) return launch_x3_wide<4, 2, 8, 2>(a, relu, s);
  return launch_x3_16<4, 1, 2, 8>(a, relu, s);
}

extern "C" lpg_status lpg_fc_x3_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                    const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                                    int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *bias,
                                    float *C, int64_t ldc, int32_t flags, float dropout_p, uint64_t seed,
                                    int64_t row_offset, const int64_t *row_keys, void *stream) {
  return fc_x3_plain(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, nullptr, nullptr, bias, C, ldc,
                     flags, dropout_p, seed, row_offset, row_keys, stream);
}

extern "C" lpg_status lpg_fc_f16x2_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                       const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                                       int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *sa,
                                       const float *sw, const float *bias, float *C, int64_t ldc, int32_t flags,
                                       float dropout_p, uint64_t seed, int64_t row_offset, const int64_t *row_keys,
                                       void *stream) {
  LPG_REQUIRE(sa && sw, "lpg_fc_f16x2_f32: NULL row scales");
  return fc_x3_plain(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, sa, sw, bias, C, ldc, flags,
                     dropout_p, seed, row_offset, row_keys, stream);
}

extern "C" int64_t lpg_fc_x3_heads_workspace_bytes(int64_t M, int64_t N) {
  if (M <= 0 || N <= 0) return 0;
  return ((N + 127) / 128) * M * 4 * (int64_t)sizeof(float);
}

static lpg_status fc_x3_heads(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const uint16_t *W1,
                              int64_t ldw1, int64_t ps1, int64_t K2, const float *A2, int64_t lda2,
                              const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *sa, const float *sw,
                              const float *bias, float *C, int64_t ldc, int32_t flags, float dropout_p, uint64_t seed,
                              int64_t row_offset, const int64_t *row_keys, int32_t hn, const float *hw, int64_t ldhw,
                              const float *hb, float *logits, int64_t ldl, void *workspace, void *stream) {
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "lpg_fc_x3_heads_f32: negative size");
  if (M == 0) return LPG_OK;
  LPG_REQUIRE(N > 0, "lpg_fc_x3_heads_f32: N must be positive");
  LPG_REQUIRE(hn >= 1 && hn <= 4, "lpg_fc_x3_heads_f32: %d heads outputs not in [1, 4]", (int)hn);
  LPG_REQUIRE(hw && ldhw >= N && logits && ldl >= hn, "lpg_fc_x3_heads_f32: bad head weight / logits");
  LPG_REQUIRE(workspace && aligned16(workspace), "lpg_fc_x3_heads_f32: workspace missing or not 16-byte aligned");
  X3Args a;
  const lpg_status st = x3_args(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, bias, C, ldc, flags,
                                dropout_p, seed, row_offset, row_keys, &a);
  if (st != LPG_OK) return st;
  a.hw = hw;
  a.ldhw = ldhw;
  a.hn = hn;
  a.hpart = reinterpret_cast<float *>(workspace);
  hipStream_t s = as_stream(stream);
  // one partial per (128-column tile, row); fc_x3_wide carries three head slots, so hn = 4 (and the
  // per-call alternative) takes fc_fwd_x3_16 -- the same C, bit for bit
  lpg_status r;
  a.order = ((flags >> 8) & 15) == 2 ? 0 : ((flags >> 8) & 15) == 3 ? 2 : 1;
  if (sa) {
    LPG_REQUIRE(sw, "lpg_fc_f16x2_heads_f32: sw is NULL");
    if (!(hn <= 3 && wide_ok(a, 128, 128))) {
      set_error("lpg_fc_f16x2_heads_f32: operands the wide kernel does not take (hn <= 3, one offset set)");
      return LPG_ERR_UNSUPPORTED;
    }
    a.sa = sa;
    a.sw = sw;
    r = launch_x3_wide<4, 2, 8, 2, true, false, true>(a, flags & 1, s);
  } else if (hn <= 3 && ((flags >> 8) & 15) != 1 && wide_ok(a, 128, 128))
    r = launch_x3_wide<4, 2, 8, 2, true>(a, flags & 1, s);
  else
    r = launch_x3_16<4, 1, 2, 8, true>(a, flags & 1, s);
  if (r != LPG_OK) return r;
  const int64_t nparts = (N + 127) / 128;
  hipLaunchKernelGGL(heads_fold, dim3((unsigned)((M * hn + 255) / 256)), dim3(256), 0, s, M, nparts, hn,
                     a.hpart, hb, logits, ldl);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_fc_x3_heads_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                          const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                                          int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2,
                                          const float *bias, float *C, int64_t ldc, int32_t flags, float dropout_p,
                                          uint64_t seed, int64_t row_offset, const int64_t *row_keys,
                                          int32_t hn, const float *hw,
                                          int64_t ldhw, const float *hb,
                                          float *logits, int64_t ldl, void *workspace, void *stream) {
  return fc_x3_heads(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, nullptr, nullptr, bias, C, ldc,
                     flags, dropout_p, seed, row_offset, row_keys, hn, hw, ldhw, hb, logits, ldl, workspace, stream);
}

extern "C" lpg_status lpg_fc_f16x2_heads_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                             const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2,
                                             const float *A2, int64_t lda2, const uint16_t *W2, int64_t ldw2,
                                             int64_t ps2, const float *sa, const float *sw, const float *bias,
                                             float *C, int64_t ldc, int32_t flags, float dropout_p, uint64_t seed,
                                             int64_t row_offset, const int64_t *row_keys, int32_t hn, const float *hw,
                                             int64_t ldhw, const float *hb, float *logits, int64_t ldl,
                                             void *workspace, void *stream) {
  LPG_REQUIRE(sa && sw, "lpg_fc_f16x2_heads_f32: NULL row scales");
  return fc_x3_heads(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, sa, sw, bias, C, ldc, flags,
                     dropout_p, seed, row_offset, row_keys, hn, hw, ldhw, hb, logits, ldl, workspace, stream);
}

extern "C" int64_t lpg_wgrad_x3_workspace_bytes(int64_t R, int64_t N, int64_t K) {
  if (R <= 0 || N <= 0 || K <= 0) return 0;
  return wgrad_splits(R, N, K) * N * K * (int64_t)sizeof(float) + 512;  // + the zero row
}

static lpg_status wgrad_x3_impl(int64_t R, int64_t N, int64_t K, const float *G, int64_t ldg, const float *X,
                                int64_t ldx, const float *sG, const float *sX, float *dW, int64_t lddw,
                                void *workspace, void *stream) {
  LPG_REQUIRE(R >= 0 && N >= 0 && K >= 0, "lpg_wgrad_x3_f32: negative size");
  LPG_REQUIRE(!sG == !sX, "lpg_wgrad_f16x2_f32: both column scales or neither");
  if (N == 0 || K == 0) return LPG_OK;
  LPG_REQUIRE(dW && lddw >= K && lddw % 4 == 0 && aligned16(dW), "lpg_wgrad_x3_f32: bad dW/lddw");
  if (R == 0) {
    LPG_HIP(hipMemset2DAsync(dW, lddw * sizeof(float), 0, K * sizeof(float), N, as_stream(stream)));
    return LPG_OK;
  }
  LPG_REQUIRE(G && X && workspace, "lpg_wgrad_x3_f32: NULL pointer");
  LPG_REQUIRE(N % 4 == 0 && K % 4 == 0 && ldg >= N && ldx >= K && ldg % 4 == 0 && ldx % 4 == 0 && aligned16(G) &&
                  aligned16(X) && aligned16(workspace),
              "lpg_wgrad_x3_f32: N, K and leading dimensions must be multiples of 4 floats, buffers 16-byte aligned");
  float *part = reinterpret_cast<float *>(workspace);
  hipStream_t st = as_stream(stream);
  const int64_t S = wgrad_splits(R, N, K);
  const int64_t nchunks = (R + 31) / 32;
  const int64_t cps = (nchunks + S - 1) / S;
  const int64_t S_used = (nchunks + cps - 1) / cps;
  // one R range's byte offsets must fit the buffer descriptors' 31 bits (a range of R / S rows: at
  // S <= 64 that is R * ld beyond 3e10 elements, 137 GB per operand)
  LPG_REQUIRE((cps * 32 + 40) * (ldg > ldx ? ldg : ldx) * 4 < ((int64_t)1 << 31),
              "lpg_wgrad_x3_f32: an R range of %lld rows x %lld floats exceeds 2 GiB", (long long)(cps * 32),
              (long long)(ldg > ldx ? ldg : ldx));
  const int64_t ntw = (N + 255) / 256, ktw = (K + 127) / 128;  // 256 x 128 tiles
  const int64_t nbw = S_used * ntw * ktw;
  LPG_REQUIRE(nbw < (int64_t)1 << 31, "lpg_wgrad_x3_f32: grid too large");
  if (sG)
    hipLaunchKernelGGL(wgrad_x3w<true>, dim3((unsigned)nbw), dim3(512), 0, st, R, N, K, G, ldg, X, ldx, part, ntw,
                       ktw, cps, sG, sX);
  else
    hipLaunchKernelGGL(wgrad_x3w<false>, dim3((unsigned)nbw), dim3(512), 0, st, R, N, K, G, ldg, X, ldx, part, ntw,
                       ktw, cps, nullptr, nullptr);
  LPG_HIP(hipGetLastError());
  const int64_t n4 = N * (K / 4);
  hipLaunchKernelGGL(wgrad_fold, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, N, K, S_used, part, dW, lddw);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_wgrad_x3_f32(int64_t R, int64_t N, int64_t K, const float *G, int64_t ldg, const float *X,
                                       int64_t ldx, float *dW, int64_t lddw, void *workspace, void *stream) {
  return wgrad_x3_impl(R, N, K, G, ldg, X, ldx, nullptr, nullptr, dW, lddw, workspace, stream);
}

extern "C" lpg_status lpg_wgrad_f16x2_f32(int64_t R, int64_t N, int64_t K, const float *G, int64_t ldg,
                                          const float *X, int64_t ldx, const float *sG, const float *sX, float *dW,
                                          int64_t lddw, void *workspace, void *stream) {
  LPG_REQUIRE(sG && sX, "lpg_wgrad_f16x2_f32: NULL column scales");
  return wgrad_x3_impl(R, N, K, G, ldg, X, ldx, sG, sX, dW, lddw, workspace, stream);
}

constexpr int64_t kColChunk = 256;  // rows per column-max block

extern "C" int64_t lpg_colscale_workspace_bytes(int64_t R, int64_t N) {
  if (R <= 0 || N <= 0) return 0;
  return N * (int64_t)sizeof(unsigned);
}

extern "C" lpg_status lpg_colscale_f32(int64_t R, int64_t N, const float *G, int64_t ldg, float *scale,
                                       void *workspace, void *stream) {
  LPG_REQUIRE(R >= 0 && N >= 0, "lpg_colscale_f32: negative size");
  if (N == 0) return LPG_OK;
  LPG_REQUIRE(scale && workspace, "lpg_colscale_f32: NULL pointer");
  LPG_REQUIRE(R == 0 || (G && ldg >= N && N % 4 == 0 && ldg % 4 == 0 && aligned16(G)),
              "lpg_colscale_f32: N and ldg multiples of 4 floats, G 16-byte aligned");
  hipStream_t st = as_stream(stream);
  unsigned *mbits = static_cast<unsigned *>(workspace);
  LPG_HIP(hipMemsetAsync(mbits, 0, N * sizeof(unsigned), st));
  const int64_t chunks = (R + kColChunk - 1) / kColChunk;
  LPG_REQUIRE(chunks < ((int64_t)1 << 31), "lpg_colscale_f32: too many rows");
  if (chunks > 0) {
    hipLaunchKernelGGL(colmax_f32, dim3((unsigned)chunks, (unsigned)((N + 1023) / 1024)), dim3(256), 0, st, R, N, G,
                       ldg, kColChunk, mbits);
    LPG_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(colscale_f32, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, N, mbits, scale);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

#ifndef LPG_ROWCOL_CHUNK
#define LPG_ROWCOL_CHUNK 256
#endif
constexpr int64_t kRowColChunk = LPG_ROWCOL_CHUNK;  // rows per block of the combined sweep (<= 256)
static_assert(kRowColChunk % 8 == 0 && kRowColChunk <= 256, "rowcolmax_f32's LDS holds 256 rows");

extern "C" int64_t lpg_rowcolscale_workspace_bytes(int64_t R, int64_t N) {
  if (R <= 0 || N <= 0) return 0;
  const int64_t chunks = (R + kRowColChunk - 1) / kRowColChunk;
  return (chunks * N + (N > 1024 ? R : 0)) * (int64_t)sizeof(float);
}

extern "C" lpg_status lpg_rowcolscale_f32(int64_t R, int64_t N, const float *G, int64_t ldg, float *rscale,
                                          float *cscale, void *workspace, void *stream) {
  LPG_REQUIRE(R >= 0 && N >= 0, "lpg_rowcolscale_f32: negative size");
  if (R == 0 || N == 0) {  // no maxima: every scale is the all-zero one (colscale_f32 on no bits)
    hipStream_t st = as_stream(stream);
    if (N > 0 && cscale)
      hipLaunchKernelGGL(colscale_f32, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, N, nullptr, cscale);
    if (R > 0 && rscale)
      hipLaunchKernelGGL(colscale_f32, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, st, R, nullptr, rscale);
    LPG_HIP(hipGetLastError());
    return LPG_OK;
  }
  LPG_REQUIRE(rscale && cscale && workspace && G, "lpg_rowcolscale_f32: NULL pointer");
  LPG_REQUIRE(ldg >= N && N % 4 == 0 && ldg % 4 == 0 && aligned16(G) && aligned16(workspace),
              "lpg_rowcolscale_f32: N and ldg multiples of 4 floats, G and the workspace 16-byte aligned");
  hipStream_t st = as_stream(stream);
  const int64_t chunks = (R + kRowColChunk - 1) / kRowColChunk;
  LPG_REQUIRE(chunks < ((int64_t)1 << 31), "lpg_rowcolscale_f32: too many rows");
  float *cpart = static_cast<float *>(workspace);
  unsigned *rbits = N > 1024 ? reinterpret_cast<unsigned *>(cpart + chunks * N) : nullptr;
  if (rbits) LPG_HIP(hipMemsetAsync(rbits, 0, R * sizeof(unsigned), st));
  hipLaunchKernelGGL(rowcolmax_f32, dim3((unsigned)chunks, (unsigned)((N + 1023) / 1024)), dim3(256), 0, st, R, N, G,
                     ldg, kRowColChunk, cpart, rbits, rbits ? nullptr : rscale);
  LPG_HIP(hipGetLastError());
  hipLaunchKernelGGL(colfold_f32, dim3((unsigned)((N + 63) / 64)), dim3(256), 0, st, chunks, N, cpart, cscale);
  LPG_HIP(hipGetLastError());
  if (rbits) {
    hipLaunchKernelGGL(colscale_f32, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, st, R, rbits, rscale);
    LPG_HIP(hipGetLastError());
  }
  return LPG_OK;
}

// ---- the conv1 weight gradient folded into the input-gradient GEMM ----------
extern "C" int64_t lpg_fc_x3_relu_wgrad_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K < 1 || K > 16) return 0;
  return smallk_fold_floats((M + 127) / 128, K + 1, N) * (int64_t)sizeof(float);
}

static lpg_status fc_x3_relu_wgrad(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                   const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                                   int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *sa,
                                   const float *sw, const float *C, int64_t ldc, int32_t flags, const float *Y,
                                   int64_t ldy, int64_t ks1, const float *X1, int64_t ldx1, int64_t ks2,
                                   const float *X2, int64_t ldx2, float *dW1, float *dW2, float *db, void *workspace,
                                   void *stream) {
  const char *name = sa ? "lpg_fc_f16x2_relu_wgrad_f32" : "lpg_fc_x3_relu_wgrad_f32";
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "%s: negative size", name);
  LPG_REQUIRE((flags & ~LPG_FC_ACCUMULATE) == 0, "%s: only the accumulate flag is accepted, got 0x%x", name, flags);
  LPG_REQUIRE(ks1 >= 0 && ks2 >= 0 && ks1 + ks2 >= 1 && ks1 + ks2 <= 16, "%s: need 1 <= ks1 + ks2 <= 16", name);
  LPG_REQUIRE(Y && ldy >= N && (ks1 == 0 || (X1 && ldx1 >= ks1)) && (ks2 == 0 || (X2 && ldx2 >= ks2)),
              "%s: bad Y / X1 / X2", name);
  LPG_REQUIRE(!(flags & LPG_FC_ACCUMULATE) || (C && ldc >= N), "%s: the accumulate flag needs C", name);
  LPG_REQUIRE(N % 2 == 0 && ldy % 2 == 0 && (reinterpret_cast<uintptr_t>(Y) & 7) == 0 &&
                  (!(flags & LPG_FC_ACCUMULATE) || (ldc % 2 == 0 && (reinterpret_cast<uintptr_t>(C) & 7) == 0)),
              "%s: N and the leading dimensions of Y and C even, Y and C 8-byte aligned (column pairs)", name);
  const int64_t ks = ks1 + ks2;
  hipStream_t s = as_stream(stream);
  if (M == 0 || N == 0) {
    if (dW1 && N * ks1) LPG_HIP(hipMemsetAsync(dW1, 0, sizeof(float) * N * ks1, s));
    if (dW2 && N * ks2) LPG_HIP(hipMemsetAsync(dW2, 0, sizeof(float) * N * ks2, s));
    if (db && N) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, s));
    return LPG_OK;
  }
  LPG_REQUIRE(workspace && aligned16(workspace), "%s: workspace missing or not 16-byte aligned", name);
  X3Args a;
  // (C is only read -- the addend -- and never written here; without the flag Y, whose alignment was
  // checked above, stands in for it whatever C the caller passed)
  const bool acc = (flags & LPG_FC_ACCUMULATE) != 0;
  const lpg_status st = x3_args(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, nullptr,
                                const_cast<float *>(acc ? C : Y), acc ? ldc : ldy, flags, 0.f, 0, 0, nullptr, &a);
  if (st != LPG_OK) return st;
  a.store = 0;
  LPG_REQUIRE(wide_ok(a, 128, 128), "%s: operands the wide kernel does not take (lda1 == lda2, ldw1 == ldw2, "
              "ps1 == ps2, 32-bit offsets)", name);
  a.wy = Y;
  a.ldwy = ldy;
  a.wx1 = X1;
  a.ldwx1 = ldx1;
  a.wx2 = X2;
  a.ldwx2 = ldx2;
  a.wk1 = (int32_t)ks1;
  a.wk2 = (int32_t)ks2;
  float *part = static_cast<float *>(workspace);
  a.wpart = part;
  a.order = 1;
  lpg_status r;
  if (sa) {
    LPG_REQUIRE(sw, "%s: sw is NULL", name);
    a.sa = sa;
    a.sw = sw;
    r = launch_x3_wide<4, 2, 8, 2, false, true, true>(a, false, s);
  } else {
    r = launch_x3_wide<4, 2, 8, 2, false, true>(a, false, s);
  }
  if (r != LPG_OK) return r;
  const int64_t mt = (M + 127) / 128;
  return smallk_fold(mt, N, (int)ks1, (int)ks, part, part + mt * (ks + 1) * N, dW1, dW2, db, s);
}

extern "C" lpg_status lpg_fc_x3_relu_wgrad_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                               const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2,
                                               const float *A2, int64_t lda2, const uint16_t *W2, int64_t ldw2,
                                               int64_t ps2, const float *C, int64_t ldc, int32_t flags, const float *Y,
                                               int64_t ldy, int64_t ks1, const float *X1, int64_t ldx1, int64_t ks2,
                                               const float *X2, int64_t ldx2, float *dW1, float *dW2, float *db,
                                               void *workspace, void *stream) {
  return fc_x3_relu_wgrad(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, nullptr, nullptr, C, ldc,
                          flags, Y, ldy, ks1, X1, ldx1, ks2, X2, ldx2, dW1, dW2, db, workspace, stream);
}

extern "C" lpg_status lpg_fc_f16x2_relu_wgrad_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                                  const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2,
                                                  const float *A2, int64_t lda2, const uint16_t *W2, int64_t ldw2,
                                                  int64_t ps2, const float *sa, const float *sw, const float *C,
                                                  int64_t ldc, int32_t flags, const float *Y, int64_t ldy, int64_t ks1,
                                                  const float *X1, int64_t ldx1, int64_t ks2, const float *X2,
                                                  int64_t ldx2, float *dW1, float *dW2, float *db, void *workspace,
                                                  void *stream) {
  LPG_REQUIRE(sa && sw, "lpg_fc_f16x2_relu_wgrad_f32: NULL row scales");
  return fc_x3_relu_wgrad(M, N, K1, A1, lda1, W1, ldw1, ps1, K2, A2, lda2, W2, ldw2, ps2, sa, sw, C, ldc, flags, Y,
                          ldy, ks1, X1, ldx1, ks2, X2, ldx2, dW1, dW2, db, workspace, stream);
}
