// bf16 variant of the fused GraphConv FC (the c5 "dense-FC-heavy, bf16 MFMA"
// configuration, BASELINE.json configs[4]):
//
//   C[m, n] = bf16( act( sum_k A1[m,k] W1[n,k] + sum_k A2[m,k] W2[n,k] + bias[n] ) )
//
// A, W bf16 (K contiguous), fp32 accumulation on v_mfma_f32_16x16x32_bf16,
// bias fp32, ReLU + the fused counter-based dropout of fc.hip, one RNE
// rounding to bf16 on the store.  No bitwise contract here (bf16 inputs): the
// tests compare against an fp32 GEMM of the same bf16-rounded operands.
//
// Tiling: 512 threads = 8 waves (2 x 4), 256 x 256 output tile, each wave
// 128 x 64 = 8 x 4 fragments of 16 x 16 (128 accumulator registers); small M
// (< 4096 rows) uses 4 waves on 128 x 128.  (A 128 x 128 tile needs 128 B/clk
// per CU of L2->CU bandwidth at the MFMA rate and measured 27 % MFMA-busy; the
// 256 x 256 tile halves the staged bytes per MFMA.)  K-tile
// BK = 64 (one 128-B row per tile row), staged global -> LDS directly by
// global_load_lds_dwordx4 (each wave-instruction writes 1 KiB = 8 rows
// lane-linearly), two buffers, one barrier per k-tile: the next tile's DMA is
// in flight while the current one feeds the MFMAs.  LDS image per row: 8
// 16-B chunks, chunk c stored at c ^ ((row >> 1) & 7) -- applied on the DMA
// SOURCE address (the destination must stay lane-linear) and on the
// ds_read_b128 fragment reads, so the 16 rows a read quarter-wave touches land
// in 16 distinct 16-B bank groups.  XCD-aware bijective block remap as in fc.hip.
#include "common.h"
#include "fc_common.h"

#include <type_traits>

namespace lpg {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int BK = 64;

struct FcB16Args {
  int64_t M, N, K1, K2;
  const uint16_t *A1, *A2, *W1, *W2;
  const float *bias;
  int64_t lda1, lda2, ldw1, ldw2;
  uint16_t *C;
  int64_t ldc;
  int64_t mt, nt;
  uint64_t seed;
  uint32_t drop_thresh;
  float drop_scale;
  int32_t accum;  // flags bit 1: C holds a bf16 addend, C = bf16(act(A1 W1^T + A2 W2^T + C + bias))
  // lpg_fc_bf16_relu_bwd: the ReLU + dropout backward of the layer whose output is `my`, applied to
  // the stored bf16 result: C = (my > 0) ? bf16(C * mscale) : 0 (nullptr: off)
  const uint16_t *my;
  int64_t ldy;
  float mscale;
  int64_t row_off;  // the dropout key of row m is row_keys[m] if given, else row_off + m (drop_row)
  const int64_t *row_keys;
  // fc_bf16_p's tile order: 1 (the default choice) = n-split (the first half of the block ids -- XCDs
  // 0-3 -- take n-tiles [0, nt/2) of every m-tile, the second half the rest: an XCD's round reads half
  // of W and twice the A panels); 0 (choices 3 and 4) = each XCD walks contiguous m-tiles with all
  // their n-tiles
  int32_t order;
  // 1-bit ReLU masks of a bf16 layer output Y, one byte per 8 columns (bit e of byte t of row m:
  // Y[m, 8 t + e] > 0): `mo` is written by a forward ReLU FC's store loop beside C, `mi` replaces the
  // Y rows `my` of the folded ReLU backward (lpg_fc_bf16_relu_bwd_bits): 1/16 of the bytes of Y
  uint8_t *mo;
  int64_t ldmo;
  const uint8_t *mi;
  int64_t ldmi;
  // the folded ReLU backward's bias column sums (lpg_fc_bf16_relu_bwd*_db; fc_bf16_p only): the stored
  // dZ's sums per 64-row chunk of the launch's rows into lpg_colsum_bf16's partial image [ceil(M / 64)][N]
  float *cs;
};


__device__ __forceinline__ uint16_t to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

#ifndef LPG_EPI_NT
#define LPG_EPI_NT 1
#endif
// The epilogue's streamed tiles -- the addend in, the output out -- as non-temporal accesses (round 6): they
// are touched once, and as ordinary accesses they displaced the A / W panels the concurrent blocks share
// in L2.  c5 step 64.2 -> 63.2 ms, fc_roofline 0.470 -> 0.482 (profiles/r06_epi_nt_ab.log); the same bits.
typedef unsigned int epi_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 epi_ld(const uint16_t *p) {
  if constexpr (LPG_EPI_NT) {
    const epi_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const epi_u32x4 *>(p));
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  return *reinterpret_cast<const uint4 *>(p);
}
__device__ __forceinline__ void epi_st(uint16_t *p, uint4 v) {
  if constexpr (LPG_EPI_NT) __builtin_nontemporal_store(epi_u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<epi_u32x4 *>(p));
  else *reinterpret_cast<uint4 *>(p) = v;
}

// The 16-bit storage type of a kernel instance: bf16 (the c5 path) or fp16 (the reference's --fp16
// inference mode, val.py:269: model.half()).  Same layouts, tiles and epilogues; only the MFMA
// (v_mfma_f32_16x16x32_bf16 / _f16, the same operand layout and rate on gfx950) and the conversions
// differ.  lo / hi: element 0 / 1 of a packed pair; pack: RNE of a pair (v_cvt_pk_bf16_f32 /
// v_cvt_pk_f16_f32); rne: RNE of one value.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
struct EBf16 {
  static constexpr bool kBf16 = true;
  typedef bf16x8 v8;
  __device__ static __forceinline__ float lo(uint32_t w) { return __uint_as_float(w << 16); }
  __device__ static __forceinline__ float hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
  __device__ static __forceinline__ uint32_t pack(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
  }
  __device__ static __forceinline__ uint16_t rne(float f) { return to_bf16_rne(f); }
  __device__ static __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
struct EF16 {
  static constexpr bool kBf16 = false;
  typedef f16x8 v8;
  __device__ static __forceinline__ float lo(uint32_t w) { return (float)__builtin_bit_cast(_Float16, (uint16_t)w); }
  __device__ static __forceinline__ float hi(uint32_t w) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
  }
  __device__ static __forceinline__ uint32_t pack(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, f16x2));
  }
  __device__ static __forceinline__ uint16_t rne(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
  __device__ static __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

// The folded ReLU/dropout backward on 8 stored bf16 values: relu_bwd_pk_bf16 (fc_common.h) per
// pair -- the arithmetic and instructions of lpg_relu_bwd_colsum_bf16, so the same bits.
__device__ __forceinline__ uint4 relu_bwd8(uint4 g, uint4 y, float scale) {
  return make_uint4(relu_bwd_pk_bf16(g.x, y.x, scale), relu_bwd_pk_bf16(g.y, y.y, scale),
                    relu_bwd_pk_bf16(g.z, y.z, scale), relu_bwd_pk_bf16(g.w, y.w, scale));
}

// bit e set iff 16-bit bf16 value e of the 8 in v is > 0 (sign clear, nonzero, not NaN): the y > 0.f
// test of relu_bwd_pk_bf16 on the stored value
__device__ __forceinline__ uint32_t pos_bits8(uint4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t b = 0u;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    b |= ((((w[p] & 0xffffu) - 1u) & 0xffffu) < 0x7f80u ? 1u : 0u) << (2 * p);
    b |= ((((w[p] >> 16) - 1u) & 0xffffu) < 0x7f80u ? 1u : 0u) << (2 * p + 1);
  }
  return b;
}

// relu_bwd8 with the mask as bits (pos_bits8 of the stored Y): the same product and rounding per pair,
// so the same bits as relu_bwd8 on Y
__device__ __forceinline__ uint32_t relu_bwd_pk_bits(uint32_t g, uint32_t b2, float scale) {
  const lpg_f32x2 gf = {__uint_as_float(g << 16), __uint_as_float(g & 0xffff0000u)};
  const uint32_t pk = __builtin_bit_cast(uint32_t, __builtin_convertvector(gf * lpg_f32x2{scale, scale}, lpg_bf16x2));
  return ((b2 & 1u) ? (pk & 0xffffu) : 0u) | ((b2 & 2u) ? (pk & 0xffff0000u) : 0u);
}
// The ReLU mask bytes of one row's 8 consecutive 16-B chunks, one byte per lane on 8 consecutive lanes
// (lane % 8 = the chunk: every store loop here has 8 chunks per row), gathered into the group's first
// lane by three DPP steps (pair swap, quad swap, half-row mirror) and stored as one 8-byte word; a group
// that crosses N (or an unaligned mask row) stores byte by byte.  Every lane of the wave must call it.
template <class A>
__device__ __forceinline__ void store_mask8(const A &a, int lane, uint32_t b, bool ok, int64_t row, int64_t col) {
  const int sh = 8 * (lane & 3);
  uint32_t lo = ok && !(lane & 4) ? (b << sh) : 0u, hi = ok && (lane & 4) ? (b << sh) : 0u;
  lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
  hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0xB1, 0xF, 0xF, false);
  lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
  hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x4E, 0xF, 0xF, false);
  lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x141, 0xF, 0xF, false);  // row_half_mirror
  hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x141, 0xF, 0xF, false);
  const int64_t col0 = col - (int64_t)(lane & 7) * 8;
  uint8_t *const p0 = a.mo + row * a.ldmo + col0 / 8;
  const bool whole = row < a.M && col0 + 64 <= a.N && (reinterpret_cast<uintptr_t>(p0) & 7) == 0;
  if (whole) {
    if ((lane & 7) == 0) *reinterpret_cast<uint2 *>(p0) = make_uint2(lo, hi);
  } else if (ok) {
    a.mo[row * a.ldmo + col / 8] = (uint8_t)b;
  }
}

__device__ __forceinline__ uint4 relu_bwd8_bits(uint4 g, uint32_t b, float scale) {
  return make_uint4(relu_bwd_pk_bits(g.x, b, scale), relu_bwd_pk_bits(g.y, b >> 2, scale),
                    relu_bwd_pk_bits(g.z, b >> 4, scale), relu_bwd_pk_bits(g.w, b >> 6, scale));
}

// The mask rows (Y) of a wave's store loop, issued together after the accumulators are in the
// image: one memory latency per epilogue instead of one per 16-B chunk (a dependent load inside
// the store loop cost ~0.3 ms per c5 launch).  Out-of-range chunks read as zeros (never stored).
template <int SIT, int CPR>
__device__ __forceinline__ void load_mask_rows(const FcB16Args &a, int lane, int64_t wrow0, int64_t wcol0,
                                               uint4 (&yv)[SIT]) {
#pragma unroll
  for (int it = 0; it < SIT; ++it) {
    const int q = it * 64 + lane;
    const int lr = q / CPR, ch = q % CPR;
    const int64_t row = wrow0 + lr, col = wcol0 + ch * 8;
    const bool ok = row < a.M && col < a.N;
    if (a.mi)  // the mask byte of the chunk's 8 columns in .x
      yv[it] = make_uint4(ok ? (uint32_t)a.mi[row * a.ldmi + col / 8] : 0u, 0u, 0u, 0u);
    else
      yv[it] = ok ? *reinterpret_cast<const uint4 *>(a.my + row * a.ldy + col) : make_uint4(0u, 0u, 0u, 0u);
  }
}

// Epilogue shared by the bf16 FC kernels: wave `wave` owns the FM*16 x FN*16
// output block at (wrow0, wcol0); C/D map of 16x16x32: col = lane & 15, row =
// 4 * (lane >> 4) + r.  `smem` must be free (every wave past its last tile read).
template <class E, int FM, int FN, bool RELU>
__device__ __forceinline__ void epilogue_bf16(const FcB16Args &a, f32x4 (&acc)[FM][FN], unsigned char *smem,
                                              int wave, int lane, int64_t wrow0, int64_t wcol0) {
  constexpr int EP_PITCH = FN * 16 * 2 + 16;  // epilogue image row pitch (bytes, 16-B aligned)
  const int fr = lane & 15, fq = lane >> 4;
  if (a.N % 8 == 0 && a.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(a.C) & 15) == 0) {
    // Through LDS (the staging buffers are free after the last barrier): each
    // wave writes its FM*16 x FN*16 bf16 tile row-major (padded pitch), then
    // stores it as 16-B chunks, 8 lanes per 128-B row segment -- one
    // global_store_dwordx4 per 8 outputs instead of one 2-byte store each.
    unsigned char *img = smem + wave * (FM * 16 * EP_PITCH);
    constexpr int CPR = FN * 16 / 8;  // 16-B chunks per row
    static_assert(CPR == 8, "store_mask8: a row's 8 chunks on 8 consecutive lanes");
    if (a.accum) {  // the addend tile, coalesced 16-B loads into the same image
#pragma unroll
      for (int it = 0; it < FM * 16 * CPR / 64; ++it) {
        const int q = it * 64 + lane;
        const int lr = q / CPR, ch = q % CPR;
        const int64_t row = wrow0 + lr < a.M ? wrow0 + lr : a.M - 1, col = wcol0 + ch * 8;
        if (col < a.N) *reinterpret_cast<uint4 *>(img + lr * EP_PITCH + ch * 16) = epi_ld(a.C + row * a.ldc + col);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    // the element loop with the addend / dropout choices made once (uniform branches per element
    // cost more than the arithmetic), RNE to bf16 in pairs by v_cvt_pk_bf16_f32
    // rows outer, columns inner: a row's dropout key (drop_row: possibly a load) is made once and dies
    // after its FN columns; the bias and column keys of the lane's FN columns stay in registers
    float bb[FN];
    uint32_t ck[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = wcol0 + j * 16 + fr;
      bb[j] = (a.bias && col < a.N) ? a.bias[col] : 0.f;
      ck[j] = drop_col_key(col);
    }
    auto body = [&](auto acc_c, auto drop_c) {
      constexpr bool ACC = decltype(acc_c)::value, DROP = decltype(drop_c)::value;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; r += 2) {
          const int lr = i * 16 + fq * 4 + r;
          const uint32_t rk0 = DROP ? drop_row_key(a.seed, drop_row(a.row_keys, a.row_off, wrow0 + lr, a.M)) : 0u;
          const uint32_t rk1 = DROP ? drop_row_key(a.seed, drop_row(a.row_keys, a.row_off, wrow0 + lr + 1, a.M)) : 0u;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            float v[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              v[h] = acc[i][j][r + h];
              if constexpr (ACC)
                v[h] = v[h] + E::lo(*reinterpret_cast<const uint16_t *>(img + (lr + h) * EP_PITCH + (j * 16 + fr) * 2));
              v[h] = v[h] + bb[j];
              if (RELU) v[h] = v[h] < 0.f ? 0.f : v[h];
              if constexpr (DROP)
                v[h] = drop_half(drop_hash_k(h ? rk1 : rk0, ck[j]), fr) >= a.drop_thresh ? v[h] * a.drop_scale : 0.f;
            }
            const uint32_t pk = E::pack(v[0], v[1]);
            *reinterpret_cast<uint16_t *>(img + lr * EP_PITCH + (j * 16 + fr) * 2) = (uint16_t)pk;
            *reinterpret_cast<uint16_t *>(img + (lr + 1) * EP_PITCH + (j * 16 + fr) * 2) = (uint16_t)(pk >> 16);
          }
        }
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    const bool drop = RELU && a.drop_thresh;
    if (a.accum) {
      if (drop) body(T_{}, T_{}); else body(T_{}, F_{});
    } else {
      if (drop) body(F_{}, T_{}); else body(F_{}, F_{});
    }
    constexpr int SIT = FM * 16 * CPR / 64;
    uint4 yv[SIT];
    if (E::kBf16 && (a.my || a.mi)) load_mask_rows<SIT, CPR>(a, lane, wrow0, wcol0, yv);  // all in flight before the first use
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int q = it * 64 + lane;
      const int lr = q / CPR, ch = q % CPR;
      const int64_t row = wrow0 + lr, col = wcol0 + ch * 8;
      uint4 v = *reinterpret_cast<const uint4 *>(img + lr * EP_PITCH + ch * 16);
      const bool ok = row < a.M && col < a.N;
      if (ok) {
        if constexpr (E::kBf16) {  // (the folded ReLU backward: bf16 training only)
          if (a.mi) v = relu_bwd8_bits(v, yv[it].x, a.mscale);
          else if (a.my) v = relu_bwd8(v, yv[it], a.mscale);
        }
        epi_st(a.C + row * a.ldc + col, v);
      }
      if (E::kBf16 && a.mo) store_mask8(a, lane, pos_bits8(v), ok, row, col);  // the layer's ReLU mask
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int64_t col = wcol0 + j * 16 + fr;
    if (col >= a.N) continue;
    const float bb = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = wrow0 + i * 16 + fq * 4 + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r];
        if (a.accum) v = v + E::lo(a.C[row * a.ldc + col]);
        v = v + bb;
        if (RELU) v = v < 0.f ? 0.f : v;
        if (a.drop_thresh) v = drop_bits(a.seed, drop_row(a.row_keys, a.row_off, row, a.M), col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
        a.C[row * a.ldc + col] = E::rne(v);
      }
    }
  }
}

// Epilogue of the transposed-fragment form (fc_bf16_p with TRO: the MFMA is issued as W x A^T,
// so the 16x16 C/D map puts output ROW 16 i + (lane & 15) on the lane and four CONSECUTIVE
// columns 16 j + 4 (lane >> 4) + r in its registers): every lane packs its four outputs into one
// 8-byte store (and loads a 4-wide addend the same way) -- no LDS image, no barrier, and the
// dropout row key is computed once per fragment row.  Same arithmetic per element as
// epilogue_bf16 (addend, + bias (0 without one), ReLU, dropout, RNE), so the same bits.
template <class E, int FM, int FN, bool RELU>
__device__ __forceinline__ void epilogue_bf16_t(const FcB16Args &a, f32x4 (&acc)[FM][FN], int lane, int64_t wrow0,
                                                int64_t wcol0) {
  const int fr = lane & 15, fq = lane >> 4;
  const int64_t c0 = wcol0 + 4 * fq;  // this lane's first column of fragment j = 0
  if (wrow0 + FM * 16 <= a.M && wcol0 + FN * 16 <= a.N && a.ldc % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(a.C) & 7) == 0) {
    uint16_t *const rp0 = a.C + (wrow0 + fr) * a.ldc + c0;  // fragment row i at + 16 i ldc (uniform step)
    float bb[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) bb[j][r] = a.bias ? a.bias[c0 + j * 16 + r] : 0.f;
    auto body = [&](auto acc_c, auto drop_c) {
      constexpr bool ACC = decltype(acc_c)::value, DROP = decltype(drop_c)::value;
      constexpr int IH = FM / 2;  // addend loads in two halves of IH fragment rows (register budget)
      uint32_t ck[FN][2];  // column-pair keys of the lane's columns c0 + 16 j + {0,1} and {2,3}
      if constexpr (DROP) {
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int q = 0; q < 2; ++q) ck[j][q] = drop_col_key(c0 + j * 16 + 2 * q);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        uint2 ad[IH][FN];
        if constexpr (ACC) {
#pragma unroll
          for (int ii = 0; ii < IH; ++ii)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              ad[ii][j] = *reinterpret_cast<const uint2 *>(rp0 + (h * IH + ii) * 16 * a.ldc + j * 16);
        }
#pragma unroll
        for (int ii = 0; ii < IH; ++ii) {
          const int i = h * IH + ii;
          const uint32_t rk = DROP ? drop_row_key(a.seed, drop_row(a.row_keys, a.row_off, wrow0 + i * 16 + fr, a.M)) : 0u;
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            float v[4];
            uint32_t hp[2] = {0u, 0u};
            if constexpr (DROP) hp[0] = drop_hash_k(rk, ck[j][0]), hp[1] = drop_hash_k(rk, ck[j][1]);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] = acc[i][j][r];
              if constexpr (ACC) {
                const uint32_t w = r < 2 ? ad[ii][j].x : ad[ii][j].y;
                v[r] = v[r] + ((r & 1) ? E::hi(w) : E::lo(w));
              }
              v[r] = v[r] + bb[j][r];
              if (RELU) v[r] = v[r] < 0.f ? 0.f : v[r];
              if constexpr (DROP) v[r] = drop_half(hp[r >> 1], r) >= a.drop_thresh ? v[r] * a.drop_scale : 0.f;
            }
            const uint32_t lo = E::pack(v[0], v[1]);
            const uint32_t hi = E::pack(v[2], v[3]);
            *reinterpret_cast<uint2 *>(rp0 + i * 16 * a.ldc + j * 16) = uint2{lo, hi};
          }
        }
      }
    };
    using T_ = std::true_type;
    using F_ = std::false_type;
    const bool drop = RELU && a.drop_thresh;
    if (a.accum) {
      if (drop) body(T_{}, T_{}); else body(T_{}, F_{});
    } else {
      if (drop) body(F_{}, T_{}); else body(F_{}, F_{});
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int64_t row = wrow0 + i * 16 + fr;
    if (row >= a.M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t col = c0 + j * 16 + r;
        if (col >= a.N) continue;
        float v = acc[i][j][r];
        if (a.accum) v = v + E::lo(a.C[row * a.ldc + col]);
        v = v + (a.bias ? a.bias[col] : 0.f);
        if (RELU) v = v < 0.f ? 0.f : v;
        if (RELU && a.drop_thresh) v = drop_bits(a.seed, drop_row(a.row_keys, a.row_off, row, a.M), col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
        a.C[row * a.ldc + col] = E::rne(v);
      }
  }
}

// ... then summed down the wave's two 64-row chunks: lanes 0-31 take chunk 0, 32-63 chunk 1, a
// column pair each, rows in order from 0.f -- relu_bwd_colsum_bf16_p1's blocks, order and fp32 sums
// (bwd.hip), so lpg_colsum_bf16's fold of the image gives its bits.  Rows past M hold +0 (their mask
// is 0) and are not read.
template <int FM, int FN>
__device__ __forceinline__ void colsum_chunks(const FcB16Args &a, const unsigned char *img, int lane, int64_t wrow0,
                                              int64_t wcol0) {
  constexpr int EP_PITCH = FN * 16 * 2 + 16;
  static_assert(FM * 16 == 128 && FN * 16 == 64, "two 64-row chunks of 32 column pairs per wave");
  const int h = lane >> 5, cp = lane & 31;
  const int64_t r0 = wrow0 + 64 * h, col = wcol0 + 2 * cp;
  if (r0 >= a.M || col >= a.N) return;
  const int64_t nr = a.M - r0 < 64 ? a.M - r0 : 64;
  const unsigned char *ip = img + 64 * h * EP_PITCH + cp * 4;
  float s0 = 0.f, s1 = 0.f;
  auto add = [&](int r) {
    const uint32_t w = *reinterpret_cast<const uint32_t *>(ip + r * EP_PITCH);
    s0 = s0 + __uint_as_float(w << 16);
    s1 = s1 + __uint_as_float(w & 0xffff0000u);
  };
  if (nr == 64) {
#pragma unroll 16
    for (int r = 0; r < 64; ++r) add(r);
  } else {
    for (int r = 0; r < (int)nr; ++r) add(r);
  }
  *reinterpret_cast<float2 *>(a.cs + (r0 / 64) * a.N + col) = make_float2(s0, s1);
}

// Transposed fragments through the LDS image (fc_bf16_p with TRO = 2): the lane's four
// consecutive columns go to the image as one ds_write_b64 (ds_read_b64 for the addend) instead
// of four 2-byte accesses, then the rows leave as 16-byte stores as in epilogue_bf16.  Image
// pitch 144 B: the 64 lanes' 8-byte accesses of one (i, j) are bank-conflict free.
template <class E, int FM, int FN, bool RELU>
__device__ __forceinline__ void epilogue_bf16_ti(const FcB16Args &a, f32x4 (&acc)[FM][FN], unsigned char *smem,
                                                 int wave, int lane, int64_t wrow0, int64_t wcol0) {
  constexpr int EP_PITCH = FN * 16 * 2 + 16;
  const int fr = lane & 15, fq = lane >> 4;
  if (!(a.N % 8 == 0 && a.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(a.C) & 15) == 0)) {
    epilogue_bf16_t<E, FM, FN, RELU>(a, acc, lane, wrow0, wcol0);  // its per-element path
    return;
  }
  unsigned char *img = smem + wave * (FM * 16 * EP_PITCH);
  constexpr int CPR = FN * 16 / 8;  // 16-B chunks per row
  static_assert(CPR == 8, "store_mask8: a row's 8 chunks on 8 consecutive lanes");
  if (a.accum) {  // the addend tile, coalesced 16-B loads into the image
#pragma unroll
    for (int it = 0; it < FM * 16 * CPR / 64; ++it) {
      const int q = it * 64 + lane;
      const int lr = q / CPR, ch = q % CPR;
      const int64_t row = wrow0 + lr < a.M ? wrow0 + lr : a.M - 1, col = wcol0 + ch * 8;
      if (col < a.N)
        *reinterpret_cast<uint4 *>(img + lr * EP_PITCH + ch * 16) = epi_ld(a.C + row * a.ldc + col);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  const int64_t c0 = wcol0 + 4 * fq;
  float bb[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bb[j][r] = (a.bias && c0 + j * 16 + r < a.N) ? a.bias[c0 + j * 16 + r] : 0.f;
  // the folded ReLU backward's mask rows, issued as the accumulators drain into the image (after
  // fragment row i, the VGPRs of acc[i] take the next loads): their latency runs under the image writes
  constexpr int SIT = FM * 16 * CPR / 64, SPI = (SIT + FM - 1) / FM;
  uint4 yv[SIT];
  auto load_y = [&](int it) {
    const int q = it * 64 + lane;
    const int lr = q / CPR, ch = q % CPR;
    const int64_t row = wrow0 + lr, col = wcol0 + ch * 8;
    const bool ok = row < a.M && col < a.N;
    if (a.mi)  // the mask byte of the chunk's 8 columns in .x
      yv[it] = make_uint4(ok ? (uint32_t)a.mi[row * a.ldmi + col / 8] : 0u, 0u, 0u, 0u);
    else
      yv[it] = ok ? *reinterpret_cast<const uint4 *>(a.my + row * a.ldy + col) : make_uint4(0u, 0u, 0u, 0u);
  };
  auto body = [&](auto acc_c, auto drop_c) {
    constexpr bool ACC = decltype(acc_c)::value, DROP = decltype(drop_c)::value;
    uint32_t ck[FN][2];
    if constexpr (DROP) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int q = 0; q < 2; ++q) ck[j][q] = drop_col_key(c0 + j * 16 + 2 * q);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const uint32_t rk = DROP ? drop_row_key(a.seed, drop_row(a.row_keys, a.row_off, wrow0 + i * 16 + fr, a.M)) : 0u;
      unsigned char *ip = img + (i * 16 + fr) * EP_PITCH + fq * 8;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        uint2 ad = {0u, 0u};
        if constexpr (ACC) ad = *reinterpret_cast<const uint2 *>(ip + j * 32);
        float v[4];
        uint32_t hp[2] = {0u, 0u};
        if constexpr (DROP) hp[0] = drop_hash_k(rk, ck[j][0]), hp[1] = drop_hash_k(rk, ck[j][1]);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[i][j][r];
          if constexpr (ACC) {
            const uint32_t w = r < 2 ? ad.x : ad.y;
            v[r] = v[r] + ((r & 1) ? E::hi(w) : E::lo(w));
          }
          v[r] = v[r] + bb[j][r];
          if (RELU) v[r] = v[r] < 0.f ? 0.f : v[r];
          if constexpr (DROP) v[r] = drop_half(hp[r >> 1], r) >= a.drop_thresh ? v[r] * a.drop_scale : 0.f;
        }
        const uint32_t lo = E::pack(v[0], v[1]);
        const uint32_t hi = E::pack(v[2], v[3]);
        *reinterpret_cast<uint2 *>(ip + j * 32) = uint2{lo, hi};
      }
      if (E::kBf16 && (a.my || a.mi)) {
#pragma unroll
        for (int u = 0; u < SPI; ++u)
          if (i * SPI + u < SIT) load_y(i * SPI + u);
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const bool drop = RELU && a.drop_thresh;
  if (a.accum) {
    if (drop) body(T_{}, T_{}); else body(T_{}, F_{});
  } else {
    if (drop) body(F_{}, T_{}); else body(F_{}, F_{});
  }
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (E::kBf16 && (a.my || a.mi)) {  // masked: every chunk formed first (one wait for the mask rows), then the stores back to back
    uint4 v[SIT];
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int q = it * 64 + lane;
      const int lr = q / CPR, ch = q % CPR;
      const uint4 g = *reinterpret_cast<const uint4 *>(img + lr * EP_PITCH + ch * 16);
      v[it] = a.mi ? relu_bwd8_bits(g, yv[it].x, a.mscale) : relu_bwd8(g, yv[it], a.mscale);
    }
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int q = it * 64 + lane;
      const int lr = q / CPR, ch = q % CPR;
      const int64_t row = wrow0 + lr, col = wcol0 + ch * 8;
      if (row < a.M && col < a.N) epi_st(a.C + row * a.ldc + col, v[it]);
    }
    if (a.cs) {  // the bias column sums of the stored dZ: each lane's own image chunks overwritten by dZ, ...
#pragma unroll
      for (int it = 0; it < SIT; ++it) {
        const int q = it * 64 + lane;
        *reinterpret_cast<uint4 *>(img + (q / CPR) * EP_PITCH + (q % CPR) * 16) = v[it];
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      colsum_chunks<FM, FN>(a, img, lane, wrow0, wcol0);
    }
    return;
  }
#pragma unroll
  for (int it = 0; it < SIT; ++it) {
    const int q = it * 64 + lane;
    const int lr = q / CPR, ch = q % CPR;
    const int64_t row = wrow0 + lr, col = wcol0 + ch * 8;
    const uint4 v = *reinterpret_cast<const uint4 *>(img + lr * EP_PITCH + ch * 16);
    const bool ok = row < a.M && col < a.N;
    if (ok) epi_st(a.C + row * a.ldc + col, v);
    if (E::kBf16 && a.mo) store_mask8(a, lane, pos_bits8(v), ok, row, col);  // the layer's ReLU mask
  }
}

// WM x WN waves, each owning FM x FN fragments of 16 x 16.
template <class E, int WM, int WN, int FM, int FN, bool RELU>
__global__ __launch_bounds__(64 * WM * WN) void fc_fwd_bf16(FcB16Args a) {
  typedef typename E::v8 v8;
  constexpr int NW = WM * WN;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int TILE_BYTES = (BM + BN) * BK * 2;  // one buffer: A tile then W tile
  constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW;  // 1-KiB DMA pieces per wave per k-tile
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows must split into whole pieces per wave");
  constexpr int EP_PITCH = FN * 16 * 2 + 16;                   // epilogue image row pitch (bytes, 16-B aligned)
  constexpr int EP_BYTES = NW * FM * 16 * EP_PITCH;
  constexpr int SMEM = 2 * TILE_BYTES > EP_BYTES ? 2 * TILE_BYTES : EP_BYTES;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);

  // DMA of k-tile t into buffer b: pieces of 8 rows x 128 B (one
  // wave-instruction each); wave w moves pieces w, w+NW, ... of A and of W.
  // Lane i of a piece lands at row 8*piece + i/8, physical chunk i%8, so it
  // fetches logical chunk swz().
  auto stage = [&](int b, int t) {
    const bool p2 = t >= nk1;
    const uint16_t *A = p2 ? a.A2 : a.A1;
    const uint16_t *W = p2 ? a.W2 : a.W1;
    const int64_t lda = p2 ? a.lda2 : a.lda1, ldw = p2 ? a.ldw2 : a.ldw1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BK;
    unsigned char *base = smem + b * TILE_BYTES;
    typedef __attribute__((address_space(3))) unsigned char lds_t;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int piece = wave + NW * p;
      const int row = piece * 8 + (lane >> 3);
      int64_t gr = m0 + row;
      gr = gr < a.M ? gr : a.M - 1;  // rows past M feed outputs that are never stored
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(A + gr * lda + k0 + swz(row, lane & 7) * 8),
                                       (lds_t *)(base + piece * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int piece = wave + NW * p;
      const int row = piece * 8 + (lane >> 3);
      int64_t gn = n0 + row;
      gn = gn < a.N ? gn : a.N - 1;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(W + gn * ldw + k0 + swz(row, lane & 7) * 8),
                                       (lds_t *)(base + BM * BK * 2 + piece * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment rows this lane reads: A rows wm*FM*16 + 16i + (lane&15), W rows wn*FN*16 + 16j + (lane&15)
  const int fr = lane & 15, fq = lane >> 4;

  if (nk > 0) stage(0, 0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    if (t + 1 < nk) stage(b ^ 1, t + 1);
    const unsigned char *As = smem + b * TILE_BYTES;
    const unsigned char *Bs = As + BM * BK * 2;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const int chunk = s * 4 + fq;  // k = 32 s + 8 fq .. +7
      v8 av[FM], bv[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * FM * 16 + i * 16 + fr;
        av[i] = *reinterpret_cast<const v8 *>(As + row * 128 + swz(row, chunk) * 16);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * FN * 16 + j * 16 + fr;
        bv[j] = *reinterpret_cast<const v8 *>(Bs + row * 128 + swz(row, chunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = E::mma(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();  // the DMA of tile t+1 has landed (vmcnt(0)) and every wave is done reading tile t
  }

  epilogue_bf16<E, FM, FN, RELU>(a, acc, smem, wave, lane, m0 + wm * FM * 16, n0 + wn * FN * 16);
}

// ---- pipelined kernel with buffer_load ... lds staging (the default) -------
//
// fc_bf16_p: same tile image as fc_fwd_bf16 (8 waves of 128 x 64), three
// changes in the k loop and one in the epilogue.
// (1) Staging: every 1-KiB DMA piece is a buffer_load ... lds through one
//     descriptor per operand and phase (wave-uniform SGPRs), the lane's offset
//     (row + swizzled chunk) fixed for the whole loop and the k step in the
//     scalar offset -- no 64-bit address arithmetic and no row clamps per load
//     (rows past M / N are past the descriptor's range and read zeros).
// (2) The barrier sits in the middle of a k-tile:  read F1 (second 32-k
//     half of tile t)  ->  MFMAs of F0  ->  barrier  ->  DMA of tile t+2 into
//     the buffer just released  ->  read F0 of tile t+1  ->  MFMAs of F1.
//     Every fragment read is issued one 32-k step ahead of the MFMAs that
//     consume it (two fragment register sets), and the DMA of a tile has the
//     MFMAs of one whole tile to land.
// (3) The reads and DMA pieces are placed one per MFMA (sched_group_barrier)
//     and waves 4-7 run at s_setprio 1.
// (4) Transposed fragments: the MFMA is issued as W x A^T, so the 16x16 C/D
//     map puts one output row on the lane and four consecutive columns in its
//     registers (epilogue_bf16_ti: 8-byte LDS image accesses).  Bitwise the
//     untransposed kernel (the MFMA sums the same exact products).
// Requires lda1 == lda2 and ldw1 == ldw2 (one offset set for both k phases);
// the host falls back to fc_fwd_bf16 otherwise.  (A 4-wave 128 x 128-per-wave
// form -- 256 accumulators, one wave per SIMD -- measured 670-790 TF/s and
// spilled; it is gone, see the spill rule in the header.)
#ifdef LPG_PHASE_PROBE
// experiments build only (tools/experiments/phase_probe.py): per-block phase timestamps of
// fc_bf16_p -- start, first tile landed, k loop done, epilogue done -- as s_memrealtime (100 MHz)
// and s_memtime (core clock), written by lane 0 of wave 0 with vector stores
__device__ uint64_t *lpg_probe_buf;
#define LPG_PROBE(i)                                                                               \
  do {                                                                                             \
    if (lpg_probe_buf && tid == 0) {                                                               \
      lpg_probe_buf[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();                      \
      lpg_probe_buf[blockIdx.x * 8 + 4 + (i)] = __builtin_amdgcn_s_memtime();                      \
    }                                                                                              \
  } while (0)
#else
#define LPG_PROBE(i) do { } while (0)
#endif

template <class E, int WM, int WN, int FM, int FN, bool RELU>
__global__ __launch_bounds__(64 * WM * WN, 1) void fc_bf16_p(FcB16Args a) {
  typedef typename E::v8 v8;
  constexpr bool SCHED = true, PRIO = true;
  constexpr int NW = WM * WN;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int A_BYTES = BM * BK * 2, TILE_BYTES = A_BYTES + BN * BK * 2;
  constexpr int PA = BM / 8, PT = PA + BN / 8, PPW = PT / NW;  // 1-KiB pieces: A, total, per wave
  static_assert(PA % NW == 0 && PT % NW == 0, "whole pieces per wave");
  constexpr int EP_BYTES = NW * FM * 16 * (FN * 16 * 2 + 16);
  constexpr int SMEM = 2 * TILE_BYTES > EP_BYTES ? 2 * TILE_BYTES : EP_BYTES;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + bid / 8;
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
  const int64_t mrows = a.M - m0 < BM ? a.M - m0 : BM;
  const int64_t ncols = a.N - n0 < BN ? a.N - n0 : BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);
  LPG_PROBE(0);

  // descriptors from row m0 of A / row n0 of W; a range ends after the block's last row, so the
  // offsets of rows past M (N) -- row * ld * 2 >= (rows - 1) * ld * 2 + K * 2 -- read zeros
  const int64_t kp1 = a.K1 > 0 ? a.K1 : BK, kp2 = a.K2 > 0 ? a.K2 : BK;
  const uint64_t pa1 = (uint64_t)(a.A1 + m0 * a.lda1), pw1 = (uint64_t)(a.W1 + n0 * a.ldw1);
  const uint64_t pa2 = a.A2 ? (uint64_t)(a.A2 + m0 * a.lda1) : pa1, pw2 = a.W2 ? (uint64_t)(a.W2 + n0 * a.ldw1) : pw1;
  const uint32_t na1 = (uint32_t)(((mrows - 1) * a.lda1 + kp1) * 2), na2 = (uint32_t)(((mrows - 1) * a.lda1 + kp2) * 2);
  const uint32_t nw1 = (uint32_t)(((ncols - 1) * a.ldw1 + kp1) * 2), nw2 = (uint32_t)(((ncols - 1) * a.ldw1 + kp2) * 2);
  // piece q = wave + NW p: rows 8 (q mod PA) .. +7 of A (q < PA) or W; lane i lands at row
  // 8 q' + i / 8, physical chunk i % 8, so it fetches logical chunk swz(row, i % 8)
  uint32_t vo[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    const int q = wave + NW * p;
    const int row = (q < PA ? q : q - PA) * 8 + (lane >> 3);
    vo[p] = (uint32_t)((row * (q < PA ? a.lda1 : a.ldw1) + swz(row, lane & 7) * 8) * 2);
  }
  // t >= nk: no tile -- the same instructions with an empty range (zeros land in a buffer nobody
  // reads again), so the loop body stays one basic block for the scheduler
  auto stage = [&](int b, int t) {
    const bool ok = t < nk;
    t = ok ? t : nk - 1;
    const bool p2 = t >= nk1;
    const int kk = p2 ? t - nk1 : t;
    unsigned char *base = smem + b * TILE_BYTES;
    const uint32_t na = ok ? (p2 ? na2 : na1) : 0u, nw = ok ? (p2 ? nw2 : nw1) : 0u;
#pragma unroll
    for (int p = 0; p < PPW; ++p) {
      const int q = wave + NW * p;  // A pieces for p < PA / NW (compile-time per p)
      if (p < PA / NW)
        dma16(p2 ? pa2 : pa1, na, base + q * 1024, vo[p], kk * (BK * 2));
      else
        dma16(p2 ? pw2 : pw1, nw, base + q * 1024, vo[p], kk * (BK * 2));
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto rd = [&](int b, int s, v8(&av)[FM], v8(&bv)[FN]) {  // 32-k step s (0, 1) of buffer b
    const unsigned char *As = smem + b * TILE_BYTES;
    const unsigned char *Bs = As + A_BYTES;
    const int chunk = s * 4 + fq;  // k = 32 s + 8 fq .. +7
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * FM * 16 + i * 16 + fr;
      av[i] = *reinterpret_cast<const v8 *>(As + row * 128 + swz(row, chunk) * 16);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * FN * 16 + j * 16 + fr;
      bv[j] = *reinterpret_cast<const v8 *>(Bs + row * 128 + swz(row, chunk) * 16);
    }
  };
  auto mma = [&](const v8(&av)[FM], const v8(&bv)[FN]) {  // W x A^T (transposed fragments)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[i][j] = E::mma(bv[j], av[i], acc[i][j]);
  };
  auto barrier = [&]() {  // this wave's DMA landed and its fragment reads returned; then all waves
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  v8 a0[FM], b0[FN], a1[FM], b1[FN];
  if (PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);  // the later-dispatched half (wave-uniform)
  if (nk > 0) {
    stage(0, 0);
    barrier();
    LPG_PROBE(1);
    if (nk > 1) stage(1, 1);
    rd(0, 0, a0, b0);
  }
  // the last tile is peeled: inside the loop every path has the same reads in flight, so the
  // compiler's lgkmcnt waits before mma(a1, b1) only cover a1 / b1 (with a conditional barrier the
  // join made them wait for most of the next tile's F0 reads too)
  constexpr int NR = FM + FN, NM = FM * FN;
  for (int t = 0; t + 1 < nk; ++t) {
    const int b = t & 1;
    rd(b, 1, a1, b1);
    mma(a0, b0);
    if constexpr (SCHED) {  // the F1 reads one per MFMA from the top, the rest MFMAs
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
    }
    barrier();  // tile t + 1 landed everywhere; every wave is done reading buffer b
    stage(b, t + 2);
    rd(b ^ 1, 0, a0, b0);
    mma(a1, b1);
    if constexpr (SCHED) {  // DMA pieces, then the next tile's F0 reads, one per MFMA
#pragma unroll
      for (int k = 0; k < PPW; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      if constexpr (NM > PPW + NR) __builtin_amdgcn_sched_group_barrier(0x008, NM - PPW - NR, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (nk > 0) {
    rd((nk - 1) & 1, 1, a1, b1);
    mma(a0, b0);
    mma(a1, b1);
  }
  // the epilogue image reuses the tile buffers: the last (empty-range) DMA has landed, every wave
  // is past its reads
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  LPG_PROBE(2);
  epilogue_bf16_ti<E, FM, FN, RELU>(a, acc, smem, wave, lane, m0 + wm * FM * 16, n0 + wn * FN * 16);
#ifdef LPG_PHASE_PROBE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (probe build: the epilogue's stores done)
  LPG_PROBE(3);
#endif
}

// ---- fc_bf16_q: two blocks per CU, 128 x 256 tiles, one LDS stage ---------------
//
// fc_bf16_p's single 8-wave block per CU runs its epilogue (the addend read and the output stores,
// HBM-bound when every CU stores at once) with the MFMA pipe idle.  Here a block is 4 waves side by
// side in n (each wave the same 128 x 64 fragment set: the same MFMA chain per output, so the same bits
// as every other choice), the tile 128 x 256, and ONE 48 KiB LDS stage: with the epilogue image
// (4 x 128 x 144 B) the block takes 74 KiB, so two blocks share a CU and one block's epilogue and DMA
// waits run beside the other's MFMAs.  Per 64-k tile: the tile landed (wait + barrier) -> both 32-k
// fragment sets read into registers -> barrier -> the next tile's DMA into the same buffer -> the 2 x 32
// MFMAs (the DMA lands under them).  1.5 x the staged bytes per MFMA of the 256 x 256 tile.
template <class E, int WM, int WN, int FM, int FN, bool RELU>
__global__ __launch_bounds__(64 * WM * WN, 2) void fc_bf16_q(FcB16Args a) {
  typedef typename E::v8 v8;
  constexpr int NW = WM * WN;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int A_BYTES = BM * BK * 2, TILE_BYTES = A_BYTES + BN * BK * 2;
  constexpr int PA = BM / 8, PT = PA + BN / 8, PPW = PT / NW;
  static_assert(PA % NW == 0 && PT % NW == 0, "whole pieces per wave");
  constexpr int EP_BYTES = NW * FM * 16 * (FN * 16 * 2 + 16);
  constexpr int SMEM = TILE_BYTES > EP_BYTES ? TILE_BYTES : EP_BYTES;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + bid / 8;
  int64_t mi = wgid / a.nt, ni = wgid % a.nt;
  if (a.order == 1 && a.nt >= 2) {  // n-split, as fc_bf16_p
    const int64_t nh = a.nt / 2, t0 = a.mt * nh;
    if (wgid < t0) {
      mi = wgid / nh;
      ni = wgid % nh;
    } else {
      mi = (wgid - t0) / (a.nt - nh);
      ni = nh + (wgid - t0) % (a.nt - nh);
    }
  }
  const int64_t m0 = mi * BM, n0 = ni * BN;
  const int64_t mrows = a.M - m0 < BM ? a.M - m0 : BM;
  const int64_t ncols = a.N - n0 < BN ? a.N - n0 : BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);

  const int64_t kp1 = a.K1 > 0 ? a.K1 : BK, kp2 = a.K2 > 0 ? a.K2 : BK;
  const uint64_t pa1 = (uint64_t)(a.A1 + m0 * a.lda1), pw1 = (uint64_t)(a.W1 + n0 * a.ldw1);
  const uint64_t pa2 = a.A2 ? (uint64_t)(a.A2 + m0 * a.lda1) : pa1, pw2 = a.W2 ? (uint64_t)(a.W2 + n0 * a.ldw1) : pw1;
  const uint32_t na1 = (uint32_t)(((mrows - 1) * a.lda1 + kp1) * 2), na2 = (uint32_t)(((mrows - 1) * a.lda1 + kp2) * 2);
  const uint32_t nw1 = (uint32_t)(((ncols - 1) * a.ldw1 + kp1) * 2), nw2 = (uint32_t)(((ncols - 1) * a.ldw1 + kp2) * 2);
  // piece p of a wave covers rows (wave + NW p) * 8 + lane / 8 of its operand: the swizzle depends on
  // the row only through (row / 2) & 7, the same for every p (NW even), so one voffset per operand and
  // the piece's row step in the (scalar) base address and record count -- 2 VGPRs, not PPW.
  static_assert(NW % 2 == 0, "piece swizzle independent of p");
  const int rowa = wave * 8 + (lane >> 3);
  const uint32_t voa = (uint32_t)((rowa * a.lda1 + swz(rowa, lane & 7) * 8) * 2);
  const uint32_t vow = (uint32_t)((rowa * a.ldw1 + swz(rowa, lane & 7) * 8) * 2);
  auto stage = [&](int t) {
    const bool p2 = t >= nk1;
    const int kk = p2 ? t - nk1 : t;
    const uint64_t ba = p2 ? pa2 : pa1, bw = p2 ? pw2 : pw1;
    const int64_t ra = p2 ? na2 : na1, rw = p2 ? nw2 : nw1;
#pragma unroll
    for (int p = 0; p < PPW; ++p) {
      const int q = wave + NW * p;
      const bool isa = p < PA / NW;
      const int64_t step = (int64_t)NW * 8 * 2 * (isa ? p : p - PA / NW) * (isa ? a.lda1 : a.ldw1);
      const int64_t left = (isa ? ra : rw) - step;
      dma16((isa ? ba : bw) + step, left > 0 ? (uint32_t)left : 0u, smem + q * 1024, isa ? voa : vow, kk * (BK * 2));
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
  auto rd = [&](int st, v8(&av)[FM], v8(&bv)[FN]) {
    const unsigned char *As = smem;
    const unsigned char *Bs = As + A_BYTES;
    const int chunk = st * 4 + fq;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * FM * 16 + i * 16 + fr;
      av[i] = *reinterpret_cast<const v8 *>(As + row * 128 + swz(row, chunk) * 16);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * FN * 16 + j * 16 + fr;
      bv[j] = *reinterpret_cast<const v8 *>(Bs + row * 128 + swz(row, chunk) * 16);
    }
  };
  auto mma = [&](const v8(&av)[FM], const v8(&bv)[FN]) {  // W x A^T (transposed fragments), as fc_bf16_p
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[i][j] = E::mma(bv[j], av[i], acc[i][j]);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  v8 a0[FM], b0[FN], a1[FM], b1[FN];
  if (nk > 0) stage(0);
  for (int t = 0; t < nk; ++t) {
    barrier();  // tile t landed everywhere
    rd(0, a0, b0);
    rd(1, a1, b1);
    barrier();  // every wave holds its fragments: the buffer is free
    if (t + 1 < nk) stage(t + 1);
    mma(a0, b0);
    mma(a1, b1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int elane = lane;  // opaque: keeps the epilogue's lane-derived addresses from living across the loop
  asm volatile("" : "+v"(elane));
  epilogue_bf16_ti<E, FM, FN, RELU>(a, acc, smem, wave, elane, m0 + wm * FM * 16, n0 + wn * FN * 16);
}

// ---- fc_bf16_sk: the pipelined kernel, persistent and stream-K -----------------
//
// One resident block per CU (G blocks) walks a contiguous range of the launch's (tile, k-tile)
// iterations -- W = tiles x nk split into G nearly equal ranges -- instead of one tile per block.
// Two costs of the one-tile-per-block grid go: (1) the partial last round (c5's 200 K rows are 24.4
// rounds of 256 x 256 tiles, 100 K rows 12.2; fp16 inference at N = 1024 6.1) -- every block now does
// W / G iterations; (2) the blocks' epilogues no longer start together, so their output stores
// (HBM-bound when 256 CUs store at once) spread over other blocks' k loops.
// A range boundary inside a tile splits its k loop: the block whose range ENDS in tile t computes
// t's first k-tiles FIRST (before its whole tiles), writes the fp32 accumulators to a partial slot
// and publishes a flag; the block whose range STARTS in t continues from those accumulators LAST,
// then runs the epilogue.  The accumulation order of every output is the one-block kernel's (the
// same MFMA chain, carried exactly through memory), so every kernel choice keeps giving the same
// bits.  Hand-off: plain partial stores, every wave drains, barrier, one lane's agent-scope release
// and relaxed agent-scope flag store; the consumer's one lane polls relaxed (bounded, s_sleep),
// fences acquire at agent scope, then the block reads.  A consumer whose flag never comes (its
// producer not resident) computes the whole tile itself -- the same bits, never a hang.
struct SkArgs {
  int64_t T;       // tiles (mt * nt)
  int32_t G;       // persistent blocks (a multiple of 8)
  int32_t spin;    // poll budget of a consumer before it computes the whole tile
  uint32_t *flags; // [G + 1], zeroed before the launch: flags[v] = 1 once slot v holds a partial
  float *part;     // [G + 1] slots of NW x FM x FN x 64 float4
};

// EPI: the epilogue flavours compiled into an instance (the others' fields are nulled at compile time,
// so their code and registers go): 0 = plain / addend / dropout, 1 = the folded ReLU backward (Y or its
// bits, with the bias column sums), 2 = the ReLU mask output
//
// Register budget: fc_bf16_p's body takes 255 VGPRs and ~60 SGPRs; inside a loop every argument it
// reads would stay live across the epilogue (SGPR spills into VGPRs).  So each piece re-reads the
// arguments from the kernarg segment through a laundered pointer (s_load per piece, nothing
// loop-invariant to hoist), and every lane-dependent address derives from a laundered lane id.
template <class E, int WM, int WN, int FM, int FN, bool RELU, int EPI>
__global__ __launch_bounds__(64 * WM * WN, 1) void fc_bf16_sk(FcB16Args a_arg, SkArgs sk_arg) {
  typedef typename E::v8 v8;
  typedef __attribute__((address_space(4))) const char kchar;
  constexpr int NW = WM * WN;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int A_BYTES = BM * BK * 2, TILE_BYTES = A_BYTES + BN * BK * 2;
  constexpr int PA = BM / 8, PT = PA + BN / 8, PPW = PT / NW;
  static_assert(PA % NW == 0 && PT % NW == 0, "whole pieces per wave");
  static_assert(sizeof(FcB16Args) % 8 == 0, "SkArgs follows FcB16Args in the kernarg segment");
  constexpr int EP_BYTES = NW * FM * 16 * (FN * 16 * 2 + 16);
  constexpr int SMEM = 2 * TILE_BYTES > EP_BYTES ? 2 * TILE_BYTES : EP_BYTES;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];
  (void)a_arg;
  (void)sk_arg;
#if defined(__HIP_DEVICE_COMPILE__)
  // the arguments through a laundered kernarg pointer: re-read where used (before the k loop, again
  // before the epilogue), so no field is live across the other phase
  auto args = [&]() {
    kchar *kp = (kchar *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    FcB16Args a = *(__attribute__((address_space(4))) const FcB16Args *)kp;
    if constexpr (EPI != 1) a.my = nullptr, a.mi = nullptr, a.cs = nullptr;
    if constexpr (EPI != 2) a.mo = nullptr;
    if constexpr (EPI == 1) a.bias = nullptr, a.drop_thresh = 0u;  // (the folded backward has neither)
    return a;
  };
  auto skargs = [&]() {
    kchar *kp = (kchar *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(kp));
    return *(__attribute__((address_space(4))) const SkArgs *)(kp + sizeof(FcB16Args));
  };

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  volatile uint32_t *word = reinterpret_cast<volatile uint32_t *>(smem);
  f32x4 acc[FM][FN];

  // The range's pieces in one loop (one copy of the k loop and of the epilogue): piece 0 -- if the
  // range ends inside a tile -- is that tile's first k-tiles, a partial for block v + 1; then the
  // whole tiles; last -- if the range starts inside a tile -- that tile's remaining k-tiles, from
  // block v - 1's partial.
  for (int q = 0;; ++q) {
    const FcB16Args a = args();
    const SkArgs sk = skargs();
    int ln = tid & 63;
    asm volatile("" : "+v"(ln));
    const int fr = ln & 15, fq = ln >> 4;

    // 32-bit index math (the host checks the iteration count); XCD-contiguous ranges: the blocks of
    // one XCD (blockIdx % 8) take neighbouring ranges
    const int nk1 = (int)(a.K1 / BK), nk = nk1 + (int)(a.K2 / BK);
    const int G = sk.G, W = (int)sk.T * nk;
    const int bid = (int)blockIdx.x, v = (bid % 8) * (G / 8) + bid / 8;
    const int s = (int)((int64_t)W * v / G), e = (int)((int64_t)W * (v + 1) / G);  // e - s >= nk
    const bool producer = e % nk != 0, consumer = s % nk != 0;
    const int t_first = (s + nk - 1) / nk, t_end = e / nk;  // whole tiles [t_first, t_end)
    const int npieces = (producer ? 1 : 0) + (t_end - t_first) + (consumer ? 1 : 0);
    if (q >= npieces) break;
    const bool is_prod = producer && q == 0, is_cons = consumer && q == npieces - 1;
    const int t = is_prod ? t_end : is_cons ? s / nk : t_first + q - (producer ? 1 : 0);

    // tile t -> (m0, n0) in fc_bf16_p's n-split order (t = its wgid; the host sets order 1)
    const int mt = (int)a.mt, nt = (int)a.nt;
    int mi = t / nt, ni = t % nt;
    if (nt >= 2) {
      const int nh = nt / 2, t0 = mt * nh;
      if (t < t0) {
        mi = t / nh;
        ni = t % nh;
      } else {
        mi = (t - t0) / (nt - nh);
        ni = nh + (t - t0) % (nt - nh);
      }
    }
    const int64_t m0 = (int64_t)mi * BM, n0 = (int64_t)ni * BN;
    const int ke = is_prod ? e % nk : nk;
    auto slot = [&](int sl) {
      return reinterpret_cast<f32x4 *>(sk.part) + ((int64_t)(sl * NW + wave) * (FM * FN)) * 64 + ln;
    };

    // the carried accumulators, or zeros
    int kb = 0;
    bool have = false;
    if (is_cons) {
      __syncthreads();  // smem free (the last epilogue's image reads are done)
      if (tid == 0) {
        uint32_t got = 0u;
        for (int i = 0; i < sk.spin; ++i) {
          if (__hip_atomic_load(sk.flags + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u) {
            got = 1u;
            break;
          }
          __builtin_amdgcn_s_sleep(8);
        }
        if (got) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        *word = got;
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __syncthreads();
      have = *word != 0u;  // (a producer that never published: the whole tile here, the same bits)
      kb = have ? s % nk : 0;
    }
    if (have) {
      const f32x4 *P = slot(v);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = P[(i * FN + j) * 64];
    } else {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // k-tiles [kb, ke) (fc_bf16_p's pipeline: barrier mid-tile, reads one 32-k step ahead, DMA pieces
    // and reads placed one per MFMA)
    {
      // the lane's DMA offsets: piece p of an operand is 8 NW rows past piece p - 1, so one offset per
      // operand plus a scalar step per piece (two VGPRs instead of PPW; laundered per stage so they are
      // not hoisted back into PPW registers)
      const int rowA = wave * 8 + (ln >> 3);
      const uint32_t voA = (uint32_t)((rowA * a.lda1 + swz(rowA, ln & 7) * 8) * 2);
      const uint32_t voW = (uint32_t)((rowA * a.ldw1 + swz(rowA, ln & 7) * 8) * 2);
      const uint32_t stepA = (uint32_t)(NW * 8 * a.lda1 * 2), stepW = (uint32_t)(NW * 8 * a.ldw1 * 2);
      const int64_t kp1 = a.K1 > 0 ? a.K1 : BK, kp2 = a.K2 > 0 ? a.K2 : BK;
      const int64_t mrows = a.M - m0 < BM ? a.M - m0 : BM;
      const int64_t ncols = a.N - n0 < BN ? a.N - n0 : BN;
      const uint64_t pa1 = (uint64_t)(a.A1 + m0 * a.lda1), pw1 = (uint64_t)(a.W1 + n0 * a.ldw1);
      const uint64_t pa2 = a.A2 ? (uint64_t)(a.A2 + m0 * a.lda1) : pa1;
      const uint64_t pw2 = a.W2 ? (uint64_t)(a.W2 + n0 * a.ldw1) : pw1;
      const uint32_t na1 = (uint32_t)(((mrows - 1) * a.lda1 + kp1) * 2), na2 = (uint32_t)(((mrows - 1) * a.lda1 + kp2) * 2);
      const uint32_t nw1 = (uint32_t)(((ncols - 1) * a.ldw1 + kp1) * 2), nw2 = (uint32_t)(((ncols - 1) * a.ldw1 + kp2) * 2);
      auto stage = [&](int b, int tk) {
        const bool ok = tk < ke;
        tk = ok ? tk : ke - 1;
        const bool p2 = tk >= nk1;
        const int kk = p2 ? tk - nk1 : tk;
        unsigned char *base = smem + b * TILE_BYTES;
        const uint32_t na = ok ? (p2 ? na2 : na1) : 0u, nw = ok ? (p2 ? nw2 : nw1) : 0u;
        uint32_t oa = voA, ow = voW;
        asm volatile("" : "+v"(oa), "+v"(ow));
#pragma unroll
        for (int p = 0; p < PPW; ++p) {
          const int qq = wave + NW * p;
          if (p < PA / NW)
            dma16(p2 ? pa2 : pa1, na, base + qq * 1024, oa + (uint32_t)p * stepA, kk * (BK * 2));
          else
            dma16(p2 ? pw2 : pw1, nw, base + qq * 1024, ow + (uint32_t)(p - PA / NW) * stepW, kk * (BK * 2));
        }
      };
      auto rd = [&](int b, int st, v8(&av)[FM], v8(&bv)[FN]) {
        const unsigned char *As = smem + b * TILE_BYTES;
        const unsigned char *Bs = As + A_BYTES;
        const int chunk = st * 4 + fq;
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int row = wm * FM * 16 + i * 16 + fr;
          av[i] = *reinterpret_cast<const v8 *>(As + row * 128 + swz(row, chunk) * 16);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = wn * FN * 16 + j * 16 + fr;
          bv[j] = *reinterpret_cast<const v8 *>(Bs + row * 128 + swz(row, chunk) * 16);
        }
      };
      auto mma = [&](const v8(&av)[FM], const v8(&bv)[FN]) {
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
          for (int i = 0; i < FM; ++i) acc[i][j] = E::mma(bv[j], av[i], acc[i][j]);
      };
      auto barrier = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      };
      constexpr int NR = FM + FN, NM = FM * FN;
      const int n = ke - kb;
      v8 a0[FM], b0[FN], a1[FM], b1[FN];
      __syncthreads();  // the previous piece's epilogue / partial reads of smem are done everywhere
      stage(0, kb);
      barrier();
      if (n > 1) stage(1, kb + 1);
      rd(0, 0, a0, b0);
      for (int j = 0; j + 1 < n; ++j) {
        const int b = j & 1;
        rd(b, 1, a1, b1);
        mma(a0, b0);
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
        barrier();
        stage(b, kb + j + 2);
        rd(b ^ 1, 0, a0, b0);
        mma(a1, b1);
#pragma unroll
        for (int k = 0; k < PPW; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
#pragma unroll
        for (int k = 0; k < NR; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
        if constexpr (NM > PPW + NR) __builtin_amdgcn_sched_group_barrier(0x008, NM - PPW - NR, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      rd((n - 1) & 1, 1, a1, b1);
      mma(a0, b0);
      mma(a1, b1);
      __builtin_amdgcn_sched_barrier(0);  // nothing of the epilogue moves up beside the last MFMAs
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
    }

    if (is_prod) {  // the partial for block v + 1: stores drained by every wave, then one release + flag
      const SkArgs sk2 = skargs();
      f32x4 *P = reinterpret_cast<f32x4 *>(sk2.part) + ((int64_t)((v + 1) * NW + wave) * (FM * FN)) * 64 + (tid & 63);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) P[(i * FN + j) * 64] = acc[i][j];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(sk2.flags + v + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      int ln2 = tid & 63;
      asm volatile("" : "+v"(ln2));
      epilogue_bf16_ti<E, FM, FN, RELU>(args(), acc, smem, wave, ln2, m0 + wm * FM * 16, n0 + wn * FN * 16);
    }
  }
#endif
}

// ---- weight gradient dW = G^T X in bf16 (fp32 out) ---------------------------
//
// dW[n, k] = sum_r G[r, n] X[r, k] (G = dZ [R, N], X = the layer input [R, K],
// both bf16, row-major; dW fp32 [N, K], the torch Linear weight layout): the
// lin_rel / lin_root weight gradients of the c5 bf16 model's backward
// (reference train.py:128 loss.backward() through GraphConv's Linears).  Both
// operands are r-major while the MFMA wants 8 consecutive r per lane, so the
// tiles are staged row-major by LDS-DMA (G rows of 256 n, X rows of 256 k:
// 512-B rows) and the fragments are read with ds_read_b64_tr_b16, the gfx950
// transposing LDS read (per 16-lane group: 4 rows x 16 columns in, lane i gets
// column i): two reads give a lane its 8 consecutive r of one column.  Image:
// 32-B segment s of row r stored at s ^ f(r), f(r) = (r & 3) | ((r & 8) >> 1),
// so the 8 rows one 32-lane half reads (r0 .. r0+3 and r0+8 .. r0+11) land on
// 8 distinct bank groups (conflict-free); the DMA source addresses carry the
// inverse map (the LDS destination stays lane-linear).  R-tiles of 64 rows,
// two buffers, the fc_bf16_p pipeline (barrier mid-tile).  Output tile
// 256 x 256; the 2048 x 2048 weights are only 64 tiles, so R is split into S
// contiguous ranges (XCD-aware: one range's tiles run on one XCD and share its
// rows in L2), partial tiles to a workspace, folded in range order:
// deterministic, no atomics.  Each range's descriptor is rebased per R-tile,
// so rows past the range (and past R) read zeros.
struct WgB16Args {
  int64_t R, N, K;
  const uint16_t *G, *X;
  int64_t ldg, ldx;
  float *P;  // partials: range s at P + s * ps, [N, ldp]
  int64_t ldp, ps;
  int64_t nt, kt, S, rows_per_split;
};

constexpr int WG_BR = 64;  // rows per R-tile

// dma16 as inline asm (the same buffer_load_dwordx4 ... lds, M0 = the LDS destination): hipcc
// then does not track the DMA and inserts no s_waitcnt vmcnt before the ds_read_tr16 reads of the
// OTHER stage buffer (it cannot tell the intrinsic's LDS address from the DMA's and waited for the
// DMA just issued before every read that followed it); every DMA of wgrad_bf16 goes through here
// (the kernel has no other M0 user), and its barriers wait vmcnt(0) themselves
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16_asm(uint64_t p, uint32_t n, unsigned char *lds, uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(3))) unsigned char lds_u8;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0, (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
  const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_u8 *)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m), "v"(voff), "s"(rs)
               : "memory", "m0");
#endif
}
#pragma clang diagnostic pop

__device__ __forceinline__ int wg_f(int r) { return (r & 3) | ((r & 8) >> 1); }

template <int WM, int WN, int FM, int FN>
__global__ __launch_bounds__(64 * WM * WN, 1) void wgrad_bf16(WgB16Args a) {
  constexpr bool SCHED = true;
  constexpr int NW = WM * WN;
  constexpr int BN = WM * FM * 16, BKC = WN * FN * 16;  // output rows (n) x columns (k)
  static_assert(BN == 256 && BKC == 256, "512-B image rows");
  constexpr int ROWB = 512, G_BYTES = WG_BR * ROWB, TILE_BYTES = 2 * G_BYTES;
  constexpr int PG = G_BYTES / 1024, PT = 2 * PG, PPW = PT / NW;  // pieces of 2 rows
  static_assert(PG % NW == 0, "whole pieces per wave");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * TILE_BYTES];

  const int64_t nwg = (int64_t)gridDim.x, bx = blockIdx.x;
  const int64_t xcd = bx % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t bid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + bx / 8;
  const int64_t tiles = a.nt * a.kt;
  const int64_t s = bid / tiles, tile = bid % tiles;
  const int64_t n0 = (tile / a.kt) * BN, k0 = (tile % a.kt) * BKC;
  const int64_t r0 = s * a.rows_per_split;
  const int64_t r1 = r0 + a.rows_per_split < a.R ? r0 + a.rows_per_split : a.R;
  const int nk = r1 > r0 ? (int)((r1 - r0 + WG_BR - 1) / WG_BR) : 0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // piece q = wave + NW p: rows 2 (q mod PG), +1 of G (q < PG) or X; lane i lands at row
  // 2 q' + i / 32, physical 16-B chunk c = i % 32, logical chunk c ^ (f(row) << 1)
  uint32_t vo[PPW];
#pragma unroll
  for (int p = 0; p < PPW; ++p) {
    const int q = wave + NW * p;
    const int row = (q < PG ? q : q - PG) * 2 + (lane >> 5), c = lane & 31;
    vo[p] = (uint32_t)((row * (q < PG ? a.ldg : a.ldx) + (c ^ (wg_f(row) << 1)) * 8) * 2);
  }
  auto stage = [&](int b, int t) {  // t >= nk: empty ranges (zeros into a buffer nobody reads again)
    unsigned char *base = smem + b * TILE_BYTES;
    const int64_t rt = r0 + (int64_t)t * WG_BR;
    const int64_t left = r1 > rt ? r1 - rt : 0;
    // the ranges end at the last row's last column of the tile (not n0 / k0 elements past it), so
    // a ragged column tile reads nothing past the end of G / X (its lanes past N / K read zeros)
    const int64_t gw = a.N - n0 < 256 ? a.N - n0 : 256, xw = a.K - k0 < 256 ? a.K - k0 : 256;
    const int64_t gb = left > 0 ? ((left - 1) * a.ldg + gw) * 2 : 0, xb = left > 0 ? ((left - 1) * a.ldx + xw) * 2 : 0;
    const uint32_t ng = (uint32_t)(gb < 0x7fffffff ? gb : 0x7fffffff), nx = (uint32_t)(xb < 0x7fffffff ? xb : 0x7fffffff);
    const uint64_t pg = (uint64_t)(a.G + rt * a.ldg + n0), px = (uint64_t)(a.X + rt * a.ldx + k0);
#pragma unroll
    for (int p = 0; p < PPW; ++p) {
      const int q = wave + NW * p;
      if (p < PG / NW)
        dma16_asm(pg, ng, base + q * 1024, vo[p]);
      else
        dma16_asm(px, nx, base + q * 1024, vo[p]);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed fragment reads: lane 16g + 4qq + pp supplies row 32 s + 8 g + 4 h + qq, columns
  // 16 c + 4 pp .. +3 of the 16-column block c; f(row) = qq | ((g & 1) << 2) for every s, h
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int fl = qq | ((g & 1) << 2);
  const int lane_off = (8 * g + qq) * ROWB + 8 * pp;
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  auto tr2 = [&](const unsigned char *img, int off) {  // rows +0..3 and +4..7 -> 8 consecutive r
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(img + off));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(img + off + 4 * ROWB));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
  };
  auto rd = [&](int b, int st, bf16x8(&av)[FM], bf16x8(&bv)[FN]) {
    // fl laundered per call: the 12 fragment addresses are recomputed (a few VALU) instead of
    // being hoisted out of the loop as 12 more live VGPRs (which spilled)
    int flv = fl;
    asm volatile("" : "+v"(flv));
    const unsigned char *Gs = smem + b * TILE_BYTES + st * 32 * ROWB + lane_off;
    const unsigned char *Xs = Gs + G_BYTES;
#pragma unroll
    for (int i = 0; i < FM; ++i) av[i] = tr2(Gs, ((wm * FM + i) ^ flv) * 32);
#pragma unroll
    for (int j = 0; j < FN; ++j) bv[j] = tr2(Xs, ((wn * FN + j) ^ flv) * 32);
  };
  auto mma = [&](const bf16x8(&av)[FM], const bf16x8(&bv)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  bf16x8 a0[FM], b0[FN], a1[FM], b1[FN];
  if (nk > 0) {
    stage(0, 0);
    barrier();
    if (nk > 1) stage(1, 1);
    rd(0, 0, a0, b0);
  }
  constexpr int NR = 2 * (FM + FN), NM = FM * FN;  // transposed reads (two per fragment), MFMAs
  for (int t = 0; t + 1 < nk; ++t) {  // last tile peeled, as in fc_bf16_p
    const int b = t & 1;
    rd(b, 1, a1, b1);
    mma(a0, b0);
    if constexpr (SCHED) {
#pragma unroll
      for (int k = 0; k < NR && k < NM; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      if constexpr (NR < NM) __builtin_amdgcn_sched_group_barrier(0x008, NM - NR, 0);
    }
    barrier();
    stage(b, t + 2);
    rd(b ^ 1, 0, a0, b0);
    mma(a1, b1);
    if constexpr (SCHED) {
#pragma unroll
      for (int k = 0; k < PPW; ++k) {  // (the asm DMAs are not schedulable units: they keep their place)
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (PPW + k < NM) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
      if constexpr (NM > PPW + NR) __builtin_amdgcn_sched_group_barrier(0x008, NM - PPW - NR, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (nk > 0) {
    rd((nk - 1) & 1, 1, a1, b1);
    mma(a0, b0);
    mma(a1, b1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last (empty) DMA lands before the wave ends

  float *P = a.P + s * a.ps;
  const int fr = lane & 15;
  // D map: row (n) = 4 * (lane >> 4) + r, col (k) = lane & 15
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int64_t col = k0 + wn * FN * 16 + j * 16 + fr;
    if (col >= a.K) continue;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = n0 + wm * FM * 16 + i * 16 + 4 * g + r;
        if (row < a.N) P[row * a.ldp + col] = acc[i][j][r];
      }
  }
}

// dW = sum_s part[s] in range order (s = 0 first): the deterministic fold of wgrad_bf16
__global__ __launch_bounds__(256) void wgrad_bf16_fold(int64_t N, int64_t K, int64_t S, const float *__restrict__ part,
                                                       float *__restrict__ dW, int64_t lddw) {
  const int64_t kq = K / 4, tot = N * kq;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < tot; i += (int64_t)gridDim.x * 256) {
    const int64_t n = i / kq, k = (i % kq) * 4;
    f32x4 v = *reinterpret_cast<const f32x4 *>(part + n * K + k);
    for (int64_t s = 1; s < S; ++s) v = v + *reinterpret_cast<const f32x4 *>(part + s * N * K + n * K + k);
    *reinterpret_cast<f32x4 *>(dW + n * lddw + k) = v;
  }
}

template <class E, int WM, int WN, int FM, int FN>
lpg_status launch_bf16(FcB16Args a, bool relu, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_bf16: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_fwd_bf16<E, WM, WN, FM, FN, true>), dim3((unsigned)nwg), dim3(64 * WM * WN), 0, s, a);
  else
    hipLaunchKernelGGL((fc_fwd_bf16<E, WM, WN, FM, FN, false>), dim3((unsigned)nwg), dim3(64 * WM * WN), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

template <class E, int WM, int WN, int FM, int FN>
lpg_status launch_bf16_p(FcB16Args a, bool relu, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_bf16: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_bf16_p<E, WM, WN, FM, FN, true>), dim3((unsigned)nwg), dim3(64 * WM * WN), 0, s, a);
  else
    hipLaunchKernelGGL((fc_bf16_p<E, WM, WN, FM, FN, false>), dim3((unsigned)nwg), dim3(64 * WM * WN), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// fc_bf16_sk's workspace: the flags ([G + 1] words at the start, padded to 16 B, zeroed per launch), then
// G + 1 partial slots of one 256 x 256 fp32 tile each
constexpr int64_t kSkSlotBytes = 256 * 256 * 4;
inline int sk_blocks() { return device_cus() / 8 * 8; }
inline int64_t sk_flag_bytes(int G) { return ((int64_t)(G + 1) * 4 + 255) / 256 * 256; }
inline int64_t sk_workspace_bytes() { return sk_flag_bytes(sk_blocks()) + (int64_t)(sk_blocks() + 1) * kSkSlotBytes; }

// whether fc_bf16_sk can take the call: a large enough 16-byte aligned workspace and at least one
// 256 x 256 tile per persistent block (so every range covers a whole tile: no chain of partials)
bool sk_ok(const FcB16Args &a, const void *ws, int64_t ws_bytes) {
  // (the mask flavours -- the folded ReLU backward, the ReLU mask output -- do not fit the register
  // budget of the persistent form yet: they run the one-tile-per-block kernel)
  if (a.my || a.mi || a.cs || a.mo) return false;
  const int G = sk_blocks();
  const int64_t T = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  return ws && aligned16(ws) && G >= 8 && T >= G && (a.K1 + a.K2) / BK >= 1 && ws_bytes >= sk_workspace_bytes() &&
         T * ((a.K1 + a.K2) / BK) < ((int64_t)1 << 31) / 1024;  // 32-bit iteration index math in the kernel
}

template <class E, int WM, int WN, int FM, int FN>
lpg_status launch_bf16_sk(FcB16Args a, bool relu, hipStream_t s, void *ws) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  static_assert(BM * BN * 4 == kSkSlotBytes, "one slot per 256 x 256 tile");
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int G = sk_blocks();
  SkArgs sk{a.mt * a.nt, G, 1 << 16, static_cast<uint32_t *>(ws),
            reinterpret_cast<float *>(static_cast<unsigned char *>(ws) + sk_flag_bytes(G))};
  LPG_HIP(hipMemsetAsync(ws, 0, sk_flag_bytes(G), s));
  const dim3 grid((unsigned)G), block(64 * WM * WN);
  if (relu)
    hipLaunchKernelGGL((fc_bf16_sk<E, WM, WN, FM, FN, true, 0>), grid, block, 0, s, a, sk);
  else
    hipLaunchKernelGGL((fc_bf16_sk<E, WM, WN, FM, FN, false, 0>), grid, block, 0, s, a, sk);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

template <class E, int WM, int WN, int FM, int FN>
lpg_status launch_bf16_q(FcB16Args a, bool relu, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_bf16: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_bf16_q<E, WM, WN, FM, FN, true>), dim3((unsigned)nwg), dim3(64 * WM * WN), 0, s, a);
  else
    hipLaunchKernelGGL((fc_bf16_q<E, WM, WN, FM, FN, false>), dim3((unsigned)nwg), dim3(64 * WM * WN), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// whether fc_bf16_p can take these operands: one offset set for both k phases, 32-bit offsets
bool p_ok(const FcB16Args &a) {
  if (a.K1 == 0) return false;
  if (a.K2 > 0 && (a.lda1 != a.lda2 || a.ldw1 != a.ldw2)) return false;
  const int64_t K = a.K1 > a.K2 ? a.K1 : a.K2;
  return (256 * a.lda1 + K) * 2 < ((int64_t)1 << 31) && (256 * a.ldw1 + K) * 2 < ((int64_t)1 << 31);
}

// Kernel choice, per call in flags bits 8-11 (LPG_FC_KERNEL(k), include/lpgnn.h): 0 = by shape
// (128 x 128 below 4096 rows, else the pipelined kernel when p_ok, else 256 x 256), 1 = fc_fwd_bf16
// 128 x 128 (4 waves), 2 = fc_fwd_bf16 256 x 256 (8 waves), 3 = fc_bf16_p (falls back to 2 when
// !p_ok), 4 / 5 = choice 0 with fc_bf16_p in the m-major / n-quarter tile order (FcB16Args::order; the default
// runs the n-split order: 1020-1225 vs 1020-1202 TF/s at the c5 shapes, profiles/r04_bf16_order_ab.log).
// Every choice computes the same bits.  Measured at the c5 shapes
// (profiles/r02_kbench_bf16.log, r02_kbench_fck10.log): fc_bf16_p 1212-1300 TF/s vs hipBLASLt
// 1248-1268, fc_fwd_bf16 256^2 1033; wgrad_bf16 1172-1222 vs hipBLASLt's bf16-output GEMM 924-1004.
// 6 = the persistent stream-K form (fc_bf16_sk) when the call carries its workspace (lpg_fc16), else
// choice 0.  (Not the default: 15-25 % slower than choice 0 at the c5 / fp16-inference shapes,
// profiles/r05_sk_ab.log -- each XCD's 32 resident blocks walk ranges 24 tiles apart, so the A panels
// the one-tile grid's concurrent blocks share in L2 are fetched once per block.)
// 7 = fc_bf16_q (two 4-wave blocks per CU on 128 x 256 tiles, one LDS stage) when p_ok, else choice 0.
constexpr int kKernels = 7;

int64_t wgrad_bf16_rows(int64_t R, int64_t N, int64_t K, int64_t *S_out) {
  const int64_t tiles = ((N + 255) / 256) * ((K + 255) / 256);
  // one block per CU, one round (round 6: the c5 step 64.3-65.0 -> 63.9-64.1 ms against two rounds,
  // profiles/r06_wgrad_bf16_split_ab.log -- half the partial tiles to fold, no second-round ramp)
  const int64_t cus = device_cus();
  int64_t S = (cus + tiles / 2) / tiles;
  const int64_t smax = (R + 511) / 512;
  S = S < smax ? S : smax;
  S = S < 1 ? 1 : S;
  int64_t rows = (R + S - 1) / S;
  rows = ((rows + WG_BR - 1) / WG_BR) * WG_BR;
  rows = rows < WG_BR ? WG_BR : rows;
  S = R > 0 ? (R + rows - 1) / rows : 1;
  *S_out = S;
  return rows;
}

}  // namespace
}  // namespace lpg

namespace lpg {
namespace {
template <class E>
lpg_status fc_bf16_dispatch(FcB16Args a, bool relu, hipStream_t s, int variant, int64_t *cs_rows = nullptr,
                             void *skws = nullptr, int64_t skws_bytes = 0);

// dst[c, r] = src[r, c] for bf16 through a 64 x 64 LDS tile, 16-byte global accesses both ways
// (the input gradients' W^T; torch's strided copy ran these at ~0.5 TB/s).  R, C multiples of 8.
__global__ __launch_bounds__(256) void transpose_bf16(int64_t R, int64_t C, const uint16_t *__restrict__ src,
                                                      int64_t lds, uint16_t *__restrict__ dst, int64_t ldd) {
  constexpr int P = 64 + 8;  // tile pitch (elements): 144-B rows, 16-B aligned
  __shared__ __attribute__((aligned(16))) uint16_t t[64 * P];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + 256 * k, row = q >> 3, ch = q & 7;
    const int64_t r = r0 + row, c = c0 + ch * 8;
    const uint4 v = (r < R && c < C) ? *reinterpret_cast<const uint4 *>(src + r * lds + c) : make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<uint4 *>(t + row * P + ch * 8) = v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = threadIdx.x + 256 * k, col = q >> 3, rch = q & 7;
    const int64_t c = c0 + col, r = r0 + rch * 8;
    if (c < C && r < R) {
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        w[e] = (uint32_t)t[(rch * 8 + 2 * e) * P + col] | ((uint32_t)t[(rch * 8 + 2 * e + 1) * P + col] << 16);
      *reinterpret_cast<uint4 *>(dst + c * ldd + r) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// conv1 in bf16 (c5): K1 + K2 <= 16 LP features, so the launch is the [M, N] bf16 output write
// (the MFMA kernel ran it on K zero-padded to 64 + 64: 0.44 ms per c5 step).  The block's rows of
// [A1 | A2] are staged once in LDS as fp32, a thread's 4 columns of weights live in registers as
// column pairs (v_pk_fma_f32); each output is one fp32 fma chain over the exact bf16 x bf16 products
// of the A1 part, the A2 part's chain added to it, then epilogue_bf16's order: + addend, + bias,
// ReLU, dropout (the shared mask hash, row key drop_row(m)), RNE to bf16.  The MFMA kernel sums the
// same exact products in its own order, so the two agree to fp32 summation order (tolerance).
constexpr int kSmallKRowsB = 64;

template <class E, int K1, int K2, bool RELU>
__global__ __launch_bounds__(256) void fc_smallk_bf16(FcB16Args a, int64_t S) {
  static_assert(K1 % 4 == 0 && K2 % 4 == 0 && K1 >= 4, "small-K kernel: K1, K2 multiples of 4");
  constexpr int KT = K1 + K2;
  constexpr int AE = kSmallKRowsB * KT / 256;  // staged values per thread per chunk
  // rows [s M / S, (s + 1) M / S) per block (a resident grid: no tail round), in chunks whose rows
  // are staged double-buffered, a chunk ahead, every load of a chunk in flight together
  __shared__ __attribute__((aligned(16))) float sx[2][kSmallKRowsB * KT];
  const int64_t sb = blockIdx.y;
  const int64_t rb = sb * a.M / S, re = (sb + 1) * a.M / S;
  if (re <= rb) return;  // (block-uniform)
  const int nch = (int)((re - rb + kSmallKRowsB - 1) / kSmallKRowsB);
  uint32_t xr_next[AE];  // raw: converted when stored, so nothing waits for the loads before then
  auto load_x = [&](int64_t r0) {
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      const int i = threadIdx.x + 256 * j, r = i / KT, k = i % KT;
      const int64_t m = r0 + r < re ? r0 + r : re - 1;  // rows past re are never stored
      xr_next[j] = k < K1 ? a.A1[m * a.lda1 + k] : a.A2[m * a.lda2 + (k - K1)];
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int j = 0; j < AE; ++j) sx[buf][threadIdx.x + 256 * j] = E::lo(xr_next[j]);
  };
  const int64_t c = (int64_t)blockIdx.x * 1024 + (int64_t)threadIdx.x * 4;
  const bool col_ok = c < a.N;
  const int64_t cc = col_ok ? c : 0;  // (lanes past N compute column 0 and store nothing)
  f32x2 wp1[2][K1], wp2[2][K2 > 0 ? K2 : 1], bp[2];
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
#pragma unroll
    for (int k = 0; k < K1; ++k)
      wp1[jp][k] = f32x2{E::lo(a.W1[(cc + 2 * jp) * a.ldw1 + k]), E::lo(a.W1[(cc + 2 * jp + 1) * a.ldw1 + k])};
#pragma unroll
    for (int k = 0; k < K2; ++k)
      wp2[jp][k] = f32x2{E::lo(a.W2[(cc + 2 * jp) * a.ldw2 + k]), E::lo(a.W2[(cc + 2 * jp + 1) * a.ldw2 + k])};
    bp[jp] = a.bias ? f32x2{a.bias[cc + 2 * jp], a.bias[cc + 2 * jp + 1]} : f32x2{0.f, 0.f};
  }
  load_x(rb);
  store_x(0);
  __syncthreads();
  if (nch > 1) load_x(rb + kSmallKRowsB);
  auto rows = [&](auto acc_c, auto drop_c) {
    constexpr bool ACC = decltype(acc_c)::value, DROP = decltype(drop_c)::value;
    uint32_t ck[4];
    if constexpr (DROP) {
#pragma unroll
      for (int j = 0; j < 4; ++j) ck[j] = drop_col_key(c + j);
    }
    for (int ch = 0; ch < nch; ++ch) {
      const int64_t r0 = rb + (int64_t)ch * kSmallKRowsB;
      const int64_t r1 = r0 + kSmallKRowsB < re ? r0 + kSmallKRowsB : re;
      const float *xb = sx[ch & 1];
      if (col_ok) {
        for (int64_t m = r0; m < r1; ++m) {
          const float *xr = xb + (m - r0) * KT;
          uint2 add = make_uint2(0u, 0u);
          if constexpr (ACC) add = *reinterpret_cast<const uint2 *>(a.C + m * a.ldc + c);
          const uint32_t rk = DROP ? drop_row_key(a.seed, drop_row(a.row_keys, a.row_off, m, a.M)) : 0u;
          uint32_t out[2];
#pragma unroll
          for (int jp = 0; jp < 2; ++jp) {
            f32x2 t = {0.f, 0.f};
#pragma unroll
            for (int k = 0; k < K1; ++k) t = __builtin_elementwise_fma(f32x2{xr[k], xr[k]}, wp1[jp][k], t);
            if constexpr (K2 > 0) {
              f32x2 p2 = {0.f, 0.f};
#pragma unroll
              for (int k = 0; k < K2; ++k) p2 = __builtin_elementwise_fma(f32x2{xr[K1 + k], xr[K1 + k]}, wp2[jp][k], p2);
              t = t + p2;
            }
            if constexpr (ACC) {
              const uint32_t w = jp ? add.y : add.x;
              t = t + f32x2{E::lo(w), E::hi(w)};
            }
            t = t + bp[jp];
            const uint32_t hp = DROP ? drop_hash_k(rk, ck[2 * jp]) : 0u;  // columns c + 2 jp, c + 2 jp + 1
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              float v = t[e];
              if (RELU) v = v < 0.f ? 0.f : v;
              if constexpr (DROP) v = drop_half(hp, e) >= a.drop_thresh ? v * a.drop_scale : 0.f;
              t[e] = v;
            }
            out[jp] = E::pack(t[0], t[1]);
          }
          *reinterpret_cast<uint2 *>(a.C + m * a.ldc + c) = make_uint2(out[0], out[1]);
          if (E::kBf16 && a.mo) {  // the layer's ReLU mask: this lane's 4 columns and its pair lane's 4 (N % 8 == 0)
            const uint32_t nib = pos_bits8(make_uint4(out[0], out[1], 0u, 0u)) & 0xfu;
            const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)nib, 0xB1, 0xF, 0xF, false);
            if ((threadIdx.x & 1) == 0) a.mo[m * a.ldmo + c / 8] = (uint8_t)(nib | (other << 4));
          }
        }
      }
      if (ch + 1 < nch) {  // the next chunk's rows (loaded a chunk ago) into the other buffer
        store_x((ch + 1) & 1);
        lds_barrier();  // (not __syncthreads: its fence would wait for the stores in flight)
        if (ch + 2 < nch) load_x(r0 + 2 * kSmallKRowsB);
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const bool drop = RELU && a.drop_thresh;
  if (a.accum) {
    if (drop) rows(T_{}, T_{}); else rows(T_{}, F_{});
  } else {
    if (drop) rows(F_{}, T_{}); else rows(F_{}, F_{});
  }
}

template <class E, int K1, int K2>
lpg_status launch_smallk_bf16(const FcB16Args &a, bool relu, hipStream_t s) {
  const int64_t ncg = (a.N + 1023) / 1024, chunks = (a.M + kSmallKRowsB - 1) / kSmallKRowsB;
  auto kern = relu ? fc_smallk_bf16<E, K1, K2, true> : fc_smallk_bf16<E, K1, K2, false>;
  int64_t S = resident_blocks(kern, 256) / ncg;  // the resident blocks, shared by the column groups
  S = S < chunks ? S : chunks;
  S = S < 1 ? 1 : S;
  const dim3 grid((unsigned)ncg, (unsigned)S);
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, a, S);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// The small-K shapes (4 <= K1, K1 + K2 <= 16, multiples of 4; N, ldc multiples of 4, C 8-byte
// aligned); false if not covered
template <class E>
bool try_smallk_bf16(const FcB16Args &a, bool relu, hipStream_t s, lpg_status *st) {
  if (a.K1 < 4 || a.K1 + a.K2 > 16 || a.K1 % 4 || a.K2 % 4 || a.N % 4 || a.ldc % 4 ||
      (reinterpret_cast<uintptr_t>(a.C) & 7))
    return false;
  if ((a.N + 1023) / 1024 >= 65536) return false;
  switch (a.K1 * 100 + a.K2) {
#define LPG_SKB(X, Y) case X * 100 + Y: *st = launch_smallk_bf16<E, X, Y>(a, relu, s); return true;
    LPG_SKB(4, 0) LPG_SKB(4, 4) LPG_SKB(4, 8) LPG_SKB(4, 12) LPG_SKB(8, 0) LPG_SKB(8, 4) LPG_SKB(8, 8)
    LPG_SKB(12, 0) LPG_SKB(12, 4) LPG_SKB(16, 0)
#undef LPG_SKB
  }
  return false;
}
}  // namespace
}  // namespace lpg

using namespace lpg;

#ifdef LPG_PHASE_PROBE
extern "C" lpg_status lpg_debug_set_probe(void *p) {
  LPG_HIP(hipMemcpyToSymbol(HIP_SYMBOL(lpg_probe_buf), &p, sizeof(p)));
  return LPG_OK;
}
#endif

template <class E>
static lpg_status fc16_entry(const char *name, int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                  const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2,
                                  const uint16_t *W2, int64_t ldw2, const float *bias, uint16_t *C, int64_t ldc,
                                  int32_t flags, float dropout_p, uint64_t seed, int64_t row_offset,
                                  const int64_t *row_keys, void *stream, uint8_t *mask = nullptr,
                                  int64_t ldm = 0, void *skws = nullptr, int64_t skws_bytes = 0) {
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "%s: negative size", name);
  if (M == 0 || N == 0) return LPG_OK;
  LPG_REQUIRE(C != nullptr && ldc >= N, "%s: bad C/ldc", name);
  LPG_REQUIRE(K1 == 0 || (A1 && W1 && lda1 >= K1 && ldw1 >= K1), "%s: bad A1/W1", name);
  LPG_REQUIRE(K2 == 0 || (A2 && W2 && lda2 >= K2 && ldw2 >= K2), "%s: bad A2/W2", name);
  const int kernel = (flags >> 8) & 15;
  LPG_REQUIRE((flags & ~0xf03) == 0 && kernel <= kKernels, "%s: unknown flags 0x%x", name, flags);
  LPG_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "%s: dropout_p %g not in [0, 1)", name, (double)dropout_p);
  FcB16Args a{M, N, K1, K2, A1, A2, W1, W2, bias, lda1, lda2, ldw1, ldw2, C, ldc, 0, 0, seed, 0u, 1.f, (flags >> 1) & 1,
              nullptr, 0, 1.f, row_offset, row_keys};
  dropout_params(dropout_p, &a.drop_thresh, &a.drop_scale);
  if (mask) {  // the ReLU mask beside C: only the 16-byte-chunk store loops write it
    LPG_REQUIRE((flags & LPG_FC_RELU) && N % 8 == 0 && ldc % 8 == 0 && aligned16(C) && ldm >= N / 8,
                "%s: the mask output needs the ReLU flag, N and ldc multiples of 8, C 16-byte aligned, ldm >= N / 8",
                name);
    a.mo = mask;
    a.ldmo = ldm;
  }
  lpg_status st;
  if (try_smallk_bf16<E>(a, flags & 1, as_stream(stream), &st)) return st;  // conv1: narrow LP features
  LPG_REQUIRE(K1 % BK == 0 && K2 % BK == 0,
              "%s: K1, K2 must be multiples of %d (zero-pad) unless 4 <= K1, K1 + K2 <= 16 (multiples of 4) "
              "and N, ldc are multiples of 4", name, BK);
  LPG_REQUIRE(lda1 % 8 == 0 && ldw1 % 8 == 0 && (K2 == 0 || (lda2 % 8 == 0 && ldw2 % 8 == 0)) &&
                  (K1 == 0 || (aligned16(A1) && aligned16(W1))) && (K2 == 0 || (aligned16(A2) && aligned16(W2))),
              "%s: A/W must be 16-byte aligned with leading dimensions multiple of 8", name);
  return fc_bf16_dispatch<E>(a, flags & 1, as_stream(stream), kernel, nullptr, skws, skws_bytes);
}

extern "C" lpg_status lpg_fc_bf16(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                  const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2,
                                  const uint16_t *W2, int64_t ldw2, const float *bias, uint16_t *C, int64_t ldc,
                                  int32_t flags, float dropout_p, uint64_t seed, int64_t row_offset,
                                  const int64_t *row_keys, void *stream) {
  return fc16_entry<EBf16>("lpg_fc_bf16", M, N, K1, A1, lda1, W1, ldw1, K2, A2, lda2, W2, ldw2, bias, C, ldc, flags,
                           dropout_p, seed, row_offset, row_keys, stream);
}

// lpg_fc_bf16 with the ReLU layer's 1-bit output mask beside C (mask[m][t] bit e: C[m, 8 t + e] > 0),
// the input of lpg_fc_bf16_relu_bwd_bits in the backward of the layer this output feeds
extern "C" lpg_status lpg_fc_bf16_mask(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                       const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2,
                                       int64_t lda2, const uint16_t *W2, int64_t ldw2, const float *bias, uint16_t *C,
                                       int64_t ldc, int32_t flags, float dropout_p, uint64_t seed, int64_t row_offset,
                                       const int64_t *row_keys, uint8_t *mask, int64_t ldm, void *stream) {
  LPG_REQUIRE(mask != nullptr, "lpg_fc_bf16_mask: NULL mask");
  return fc16_entry<EBf16>("lpg_fc_bf16_mask", M, N, K1, A1, lda1, W1, ldw1, K2, A2, lda2, W2, ldw2, bias, C, ldc,
                           flags, dropout_p, seed, row_offset, row_keys, stream, mask, ldm);
}

// fp16 storage (the reference's --fp16 inference: model.half(), batch_to(half=True); val.py:269,
// utils.py:909-915): the bf16 entry's kernels on v_mfma_f32_16x16x32_f16, fp32 accumulation, fp32 bias,
// one RNE rounding to fp16 per output
extern "C" lpg_status lpg_fc_f16(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                 const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2,
                                 const uint16_t *W2, int64_t ldw2, const float *bias, uint16_t *C, int64_t ldc,
                                 int32_t flags, float dropout_p, uint64_t seed, int64_t row_offset,
                                 const int64_t *row_keys, void *stream) {
  return fc16_entry<EF16>("lpg_fc_f16", M, N, K1, A1, lda1, W1, ldw1, K2, A2, lda2, W2, ldw2, bias, C, ldc, flags,
                          dropout_p, seed, row_offset, row_keys, stream);
}

// The input gradient of a layer whose input went through the previous layer's ReLU + dropout,
// with that backward folded into the store: C = (Y > 0) ? bf16(bf16(G1 W1^T + G2 W2^T [+ C]) * scale) : 0
// -- bit for bit lpg_fc_bf16 followed by lpg_relu_bwd_colsum_bf16(C, Y, scale) (whose bias column
// sums the caller takes from lpg_colsum_bf16 on C).  Saves the separate pass's read of C and
// write of dZ (c5: 2 x [rows, 2048] bf16 per layer input).
static lpg_status relu_bwd_entry(const char *name, int64_t M, int64_t N, int64_t K1, const uint16_t *A1,
                                 int64_t lda1, const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2,
                                 int64_t lda2, const uint16_t *W2, int64_t ldw2, uint16_t *C, int64_t ldc,
                                 int32_t flags, const uint16_t *Y, int64_t ldy, const uint8_t *mask, int64_t ldm,
                                 float scale, void *stream, float *db = nullptr, void *workspace = nullptr,
                                 void *skws = nullptr, int64_t skws_bytes = 0) {
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "%s: negative size", name);
  if (db) {
    LPG_REQUIRE(workspace && aligned16(workspace), "%s: db needs a 16-byte aligned workspace", name);
    if (M == 0 && N > 0) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, as_stream(stream)));
  }
  if (M == 0 || N == 0) return LPG_OK;
  LPG_REQUIRE(C != nullptr && ldc >= N && (Y ? ldy >= N : (mask != nullptr && ldm >= N / 8)),
              "%s: bad C/ldc or Y/ldy (mask/ldm)", name);
  LPG_REQUIRE(N % 8 == 0 && ldc % 8 == 0 && aligned16(C) && (!Y || (ldy % 8 == 0 && aligned16(Y))),
              "%s: N, ldc, ldy must be multiples of 8, C and Y 16-byte aligned", name);
  LPG_REQUIRE(K1 % BK == 0 && K2 % BK == 0, "%s: K1, K2 must be multiples of %d", name, BK);
  LPG_REQUIRE(K1 == 0 || (A1 && W1 && lda1 >= K1 && ldw1 >= K1), "%s: bad A1/W1", name);
  LPG_REQUIRE(K2 == 0 || (A2 && W2 && lda2 >= K2 && ldw2 >= K2), "%s: bad A2/W2", name);
  LPG_REQUIRE(lda1 % 8 == 0 && ldw1 % 8 == 0 && (K2 == 0 || (lda2 % 8 == 0 && ldw2 % 8 == 0)) &&
                  (K1 == 0 || (aligned16(A1) && aligned16(W1))) && (K2 == 0 || (aligned16(A2) && aligned16(W2))),
              "%s: A/W must be 16-byte aligned with leading dimensions multiple of 8", name);
  const int kernel = (flags >> 8) & 15;
  LPG_REQUIRE((flags & ~0xf02) == 0 && kernel <= kKernels,
              "%s: only the accumulate flag (2) and a kernel choice are accepted, got 0x%x", name, flags);
  FcB16Args a{M, N, K1, K2, A1, A2, W1, W2, nullptr, lda1, lda2, ldw1, ldw2, C, ldc, 0, 0, 0, 0u, 1.f, (flags >> 1) & 1,
              Y, ldy, scale};
  if (!Y) {
    a.mi = mask;
    a.ldmi = ldm;
  }
  hipStream_t s = as_stream(stream);
  a.cs = db ? static_cast<float *>(workspace) : nullptr;
  int64_t cs_rows = 0;
  const lpg_status st = fc_bf16_dispatch<EBf16>(a, false, s, kernel, &cs_rows, skws, skws_bytes);  // (every kernel's epilogue takes the fold)
  if (st != LPG_OK || !db) return st;
  return colsum_bf16_from(M, N, C, ldc, cs_rows, static_cast<float *>(workspace), db, s);
}

extern "C" lpg_status lpg_fc_bf16_relu_bwd(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                           const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2,
                                           int64_t lda2, const uint16_t *W2, int64_t ldw2, uint16_t *C, int64_t ldc,
                                           int32_t flags, const uint16_t *Y, int64_t ldy, float scale, void *stream) {
  LPG_REQUIRE(Y != nullptr || M == 0 || N == 0, "lpg_fc_bf16_relu_bwd: NULL Y");
  return relu_bwd_entry("lpg_fc_bf16_relu_bwd", M, N, K1, A1, lda1, W1, ldw1, K2, A2, lda2, W2, ldw2, C, ldc, flags,
                        Y, ldy, nullptr, 0, scale, stream);
}

// lpg_fc_bf16_relu_bwd with the previous layer's ReLU as its 1-bit mask (lpg_fc_bf16_mask's output)
// instead of its output Y: the same bits, 1/16 of the mask bytes
extern "C" lpg_status lpg_fc_bf16_relu_bwd_bits(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                                const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2,
                                                int64_t lda2, const uint16_t *W2, int64_t ldw2, uint16_t *C,
                                                int64_t ldc, int32_t flags, const uint8_t *mask, int64_t ldm,
                                                float scale, void *stream) {
  LPG_REQUIRE(mask != nullptr || M == 0 || N == 0, "lpg_fc_bf16_relu_bwd_bits: NULL mask");
  return relu_bwd_entry("lpg_fc_bf16_relu_bwd_bits", M, N, K1, A1, lda1, W1, ldw1, K2, A2, lda2, W2, ldw2, C, ldc,
                        flags, nullptr, 0, mask, ldm, scale, stream);
}

// ... and the bias column sums of the stored dZ, db [N] fp32 (the bits of lpg_colsum_bf16 on C): from the
// store loop's registers where the pipelined kernel runs (no second read of C), else by the colsum pass.
// workspace: lpg_relu_bwd_colsum_workspace_bytes(M, N)
extern "C" lpg_status lpg_fc_bf16_relu_bwd_db(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                              const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2,
                                              int64_t lda2, const uint16_t *W2, int64_t ldw2, uint16_t *C, int64_t ldc,
                                              int32_t flags, const uint16_t *Y, int64_t ldy, float scale, float *db,
                                              void *workspace, void *stream) {
  LPG_REQUIRE((Y != nullptr || M == 0 || N == 0) && db != nullptr, "lpg_fc_bf16_relu_bwd_db: NULL Y or db");
  return relu_bwd_entry("lpg_fc_bf16_relu_bwd_db", M, N, K1, A1, lda1, W1, ldw1, K2, A2, lda2, W2, ldw2, C, ldc,
                        flags, Y, ldy, nullptr, 0, scale, stream, db, workspace);
}

extern "C" lpg_status lpg_fc_bf16_relu_bwd_bits_db(int64_t M, int64_t N, int64_t K1, const uint16_t *A1,
                                                   int64_t lda1, const uint16_t *W1, int64_t ldw1, int64_t K2,
                                                   const uint16_t *A2, int64_t lda2, const uint16_t *W2, int64_t ldw2,
                                                   uint16_t *C, int64_t ldc, int32_t flags, const uint8_t *mask,
                                                   int64_t ldm, float scale, float *db, void *workspace,
                                                   void *stream) {
  LPG_REQUIRE((mask != nullptr || M == 0 || N == 0) && db != nullptr, "lpg_fc_bf16_relu_bwd_bits_db: NULL mask or db");
  return relu_bwd_entry("lpg_fc_bf16_relu_bwd_bits_db", M, N, K1, A1, lda1, W1, ldw1, K2, A2, lda2, W2, ldw2, C, ldc,
                        flags, nullptr, 0, mask, ldm, scale, stream, db, workspace);
}

extern "C" int64_t lpg_fc16_workspace_bytes(void) { return sk_workspace_bytes(); }

extern "C" lpg_status lpg_fc16(const lpg_fc16_call *c, void *workspace, int64_t workspace_bytes, void *stream) {
  LPG_REQUIRE(c != nullptr, "lpg_fc16: NULL call");
  LPG_REQUIRE(c->dtype == 0 || c->dtype == 1, "lpg_fc16: dtype %d (0 = bf16, 1 = fp16)", c->dtype);
  LPG_REQUIRE(!workspace || workspace_bytes >= sk_workspace_bytes(), "lpg_fc16: workspace of %lld bytes, need %lld",
              (long long)workspace_bytes, (long long)sk_workspace_bytes());
  if (c->Y || c->mask_in) {
    LPG_REQUIRE(c->dtype == 0, "lpg_fc16: the folded ReLU backward is a bf16 training path");
    LPG_REQUIRE(!(c->Y && c->mask_in), "lpg_fc16: Y or mask_in, not both");
    return relu_bwd_entry(c->db ? (c->Y ? "lpg_fc_bf16_relu_bwd_db" : "lpg_fc_bf16_relu_bwd_bits_db")
                                : (c->Y ? "lpg_fc_bf16_relu_bwd" : "lpg_fc_bf16_relu_bwd_bits"),
                          c->M, c->N, c->K1, c->A1, c->lda1, c->W1, c->ldw1, c->K2, c->A2, c->lda2, c->W2, c->ldw2,
                          c->C, c->ldc, c->flags, c->Y, c->ldy, c->mask_in, c->ldmi, c->scale, stream, c->db,
                          c->db_workspace, workspace, workspace_bytes);
  }
  if (c->dtype == 1) {
    LPG_REQUIRE(!c->mask_out, "lpg_fc16: the ReLU mask output is a bf16 training path");
    return fc16_entry<EF16>("lpg_fc_f16", c->M, c->N, c->K1, c->A1, c->lda1, c->W1, c->ldw1, c->K2, c->A2, c->lda2,
                            c->W2, c->ldw2, c->bias, c->C, c->ldc, c->flags, c->dropout_p, c->seed, c->row_offset,
                            c->row_keys, stream, nullptr, 0, workspace, workspace_bytes);
  }
  return fc16_entry<EBf16>(c->mask_out ? "lpg_fc_bf16_mask" : "lpg_fc_bf16", c->M, c->N, c->K1, c->A1, c->lda1, c->W1,
                           c->ldw1, c->K2, c->A2, c->lda2, c->W2, c->ldw2, c->bias, c->C, c->ldc, c->flags,
                           c->dropout_p, c->seed, c->row_offset, c->row_keys, stream, c->mask_out, c->ldmo, workspace,
                           workspace_bytes);
}

namespace lpg {
namespace {
// rows [r, M) of a as their own call: operands, output, mask rows and dropout keys offset by r
FcB16Args rows_from(const FcB16Args &a, int64_t r) {
  FcB16Args t = a;
  t.M = a.M - r;
  t.A1 = a.A1 ? a.A1 + r * a.lda1 : nullptr;
  t.A2 = a.A2 ? a.A2 + r * a.lda2 : nullptr;
  t.C = a.C + r * a.ldc;
  t.my = a.my ? a.my + r * a.ldy : nullptr;
  t.mo = a.mo ? a.mo + r * a.ldmo : nullptr;
  t.mi = a.mi ? a.mi + r * a.ldmi : nullptr;
  t.row_off = a.row_off + r;
  t.row_keys = a.row_keys ? a.row_keys + r : nullptr;
  t.cs = nullptr;
  return t;
}

template <class E>
// cs_rows: the leading rows whose column-sum partials the launches wrote (a.cs: fc_bf16_p's epilogue
// only; the other kernels never see a.cs)
lpg_status fc_bf16_dispatch(FcB16Args a, bool relu, hipStream_t s, int kernel, int64_t *cs_rows, void *skws,
                             int64_t skws_bytes) {
  if (cs_rows) *cs_rows = 0;
  float *const cs = a.cs;
  a.cs = nullptr;
  if (kernel == 1 || (kernel == 0 && a.M < 4096)) return launch_bf16<E, 2, 2, 4, 4>(a, relu, s);  // 128 x 128
  if (kernel == 7 && p_ok(a)) {  // two 4-wave blocks per CU, 128 x 256 tiles, n-split order
    a.order = 1;
    a.cs = cs;
    if (cs_rows && cs) *cs_rows = a.M;
    return launch_bf16_q<E, 1, 4, 8, 4>(a, relu, s);
  }
  if (kernel == 6 && p_ok(a) && sk_ok(a, skws, skws_bytes)) {
    // the persistent stream-K form of the pipelined kernel (with a workspace), n-split tile order --
    // measured 15-25 % slower than the default at the c5 and fp16-inference shapes
    // (profiles/r05_sk_ab.log): a per-call choice, not the default
    a.order = 1;
    a.cs = cs;
    if (cs_rows && cs) *cs_rows = a.M;
    return launch_bf16_sk<E, 2, 4, 8, 4>(a, relu, s, skws);
  }
  if ((kernel == 0 || kernel >= 3) && p_ok(a)) {
    a.order = kernel == 0 || kernel == 6 ? 1 : kernel == 5 ? 2 : 0;  // the default in the n-split order (1-2 % at the c5 shapes)
    if (kernel == 0 || kernel == 4 || kernel == 5 || kernel == 6) {
      // The last round of 256 x 256 tiles (one block per CU) is usually partial: c5's 200 K rows are 24
      // rounds + 41 % of one, 100 K rows 12 + 21 %, and the CUs without a tile idle for a whole block
      // time.  Those rows run as a second launch on 128 x 128 tiles (4 x the blocks, 2 per CU) -- the
      // same per-element arithmetic, so the same bits (kernels are interchangeable, LPG_FC_KERNEL).
      const int64_t nt = (a.N + 255) / 256;
      const int64_t per_round = (int64_t)(device_cus() / (nt > 0 ? nt : 1)) * 256;
      if (per_round >= 256) {
        const int64_t full = a.M / per_round * per_round, tail = a.M - full;
        if (full > 0 && tail > 0 && 2 * tail <= per_round) {
          FcB16Args h = a;
          h.M = full;
          h.cs = cs;
          const lpg_status st = launch_bf16_p<E, 2, 4, 8, 4>(h, relu, s);
          if (st != LPG_OK) return st;
          if (cs_rows && cs) *cs_rows = full;
          return launch_bf16<E, 2, 2, 4, 4>(rows_from(a, full), relu, s);
        }
      }
    }
    a.cs = cs;
    if (cs_rows && cs) *cs_rows = a.M;
    return launch_bf16_p<E, 2, 4, 8, 4>(a, relu, s);
  }
  return launch_bf16<E, 2, 4, 8, 4>(a, relu, s);  // 256 x 256, BK 64, 2 buffers
}
}  // namespace
}  // namespace lpg

extern "C" lpg_status lpg_transpose_bf16(int64_t R, int64_t C, const uint16_t *src, int64_t lds, uint16_t *dst,
                                         int64_t ldd, void *stream) {
  LPG_REQUIRE(R >= 0 && C >= 0, "lpg_transpose_bf16: negative size");
  if (R == 0 || C == 0) return LPG_OK;
  LPG_REQUIRE(src && dst && R % 8 == 0 && C % 8 == 0 && lds >= C && ldd >= R && lds % 8 == 0 && ldd % 8 == 0 &&
                  aligned16(src) && aligned16(dst),
              "lpg_transpose_bf16: R, C, lds, ldd must be multiples of 8 (lds >= C, ldd >= R), buffers 16-byte aligned");
  const dim3 grid((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64));
  LPG_REQUIRE((R + 63) / 64 < 65536, "lpg_transpose_bf16: too many rows");
  hipLaunchKernelGGL(transpose_bf16, grid, dim3(256), 0, as_stream(stream), R, C, src, lds, dst, ldd);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" int64_t lpg_wgrad_bf16_workspace_bytes(int64_t R, int64_t N, int64_t K) {
  if (R < 0 || N <= 0 || K <= 0) return 0;
  int64_t S;
  wgrad_bf16_rows(R, N, K, &S);
  return S > 1 ? S * N * K * 4 : 0;
}

extern "C" lpg_status lpg_wgrad_bf16(int64_t R, int64_t N, int64_t K, const uint16_t *G, int64_t ldg,
                                     const uint16_t *X, int64_t ldx, float *dW, int64_t lddw, void *workspace,
                                     void *stream) {
  LPG_REQUIRE(R >= 0 && N >= 0 && K >= 0, "lpg_wgrad_bf16: negative size");
  if (N == 0 || K == 0) return LPG_OK;
  LPG_REQUIRE(N % 8 == 0 && K % 8 == 0 && ldg % 8 == 0 && ldx % 8 == 0 && ldg >= N && ldx >= K &&
                  ldg < ((int64_t)1 << 24) && ldx < ((int64_t)1 << 24),
              "lpg_wgrad_bf16: N, K, ldg, ldx must be multiples of 8 (ldg >= N, ldx >= K)");
  LPG_REQUIRE(R == 0 || (G && X && aligned16(G) && aligned16(X)), "lpg_wgrad_bf16: G/X must be 16-byte aligned");
  LPG_REQUIRE(dW && aligned16(dW) && lddw >= K && lddw % 4 == 0, "lpg_wgrad_bf16: bad dW/lddw");
  int64_t S;
  const int64_t rows = wgrad_bf16_rows(R, N, K, &S);
  LPG_REQUIRE(S == 1 || (workspace && aligned16(workspace)), "lpg_wgrad_bf16: workspace required (16-B aligned)");
  WgB16Args w{R, N, K, G, X, ldg, ldx, S > 1 ? static_cast<float *>(workspace) : dW, S > 1 ? K : lddw, N * K,
              (N + 255) / 256, (K + 255) / 256, S, rows};
  const int64_t nwg = w.nt * w.kt * S;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_wgrad_bf16: grid too large");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL((wgrad_bf16<2, 4, 8, 4>), dim3((unsigned)nwg), dim3(512), 0, s, w);
  LPG_HIP(hipGetLastError());
  if (S > 1) {
    const int64_t tot = N * (K / 4);
    const int64_t blocks = (tot + 255) / 256 < 4096 ? (tot + 255) / 256 : 4096;
    hipLaunchKernelGGL(wgrad_bf16_fold, dim3((unsigned)blocks), dim3(256), 0, s, N, K, S,
                       static_cast<const float *>(workspace), dW, lddw);
    LPG_HIP(hipGetLastError());
  }
  return LPG_OK;
}
