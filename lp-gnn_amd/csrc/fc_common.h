// Device helpers shared by the FC kernels (fc.hip, fc_bf16.hip, fc_x3.hip):
// the fused-dropout mask function must be one definition, since the backward
// of every FC variant relies on "kept <=> stored output > 0".
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "lpgnn.h"

namespace lpg {

// Counter-based dropout mask over (seed, row, column pair): one round of the 32-bit "lowbias32"
// integer hash per row and one per (row, column pair); the pair's hash carries 16 bits for each of
// its two columns (low half: the even column, high half: the odd one), kept iff those bits >=
// the 16-bit threshold round(p * 2^16) (dropout_params; the drop rate is within 2^-17 of p, and the
// kept values are scaled by the reciprocal of the kept rate, 2^16 / (2^16 - threshold)).
// Stateless, so the backward pass never needs the mask (the kept set is exactly where the stored
// output is > 0).  One hash per two outputs: the hash's two quarter-rate v_mul_lo_u32 were most of
// a dropout epilogue's VALU (round 3: 1.56 VALU per MFMA in the bf16 FC with dropout, 0.37
// without).  32-bit on purpose: 64-bit multiplies are multi-instruction on CDNA.
// oracle/dropout_ref.py restates this function; every FC kernel draws the same mask through it.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// The dropout key of output row `row`: row_keys[row] when the caller gives one key per row (the
// global node ids of a partition's rows, in any order) or row_off + row (a contiguous slice); rows at
// or past M are never stored and key as row_off + row (no load past the key array).
__device__ __forceinline__ int64_t drop_row(const int64_t *row_keys, int64_t row_off, int64_t row, int64_t M) {
  return (row_keys != nullptr && row < M) ? row_keys[row] : row_off + row;
}

// The mask split into its row and column-pair keys, for epilogues that hold a few rows and a few
// columns per lane: the pair hash of (key, col) is drop_hash_k(drop_row_key(seed, key), drop_col_key(col)),
// the same for col = 2c and 2c + 1; drop_half picks a column's 16 bits out of it.
__device__ __forceinline__ uint32_t drop_row_key(uint64_t seed, int64_t key) {
  return lowbias32((uint32_t)key ^ (uint32_t)seed) ^ (uint32_t)(seed >> 32);
}
__device__ __forceinline__ uint32_t drop_col_key(int64_t col) { return (uint32_t)(col >> 1) * 0x9e3779b9u; }
__device__ __forceinline__ uint32_t drop_hash_k(uint32_t rk, uint32_t ck) { return lowbias32(rk ^ ck); }
__device__ __forceinline__ uint32_t drop_half(uint32_t h, int64_t col) { return (col & 1) ? (h >> 16) : (h & 0xffffu); }
// element form (fallback epilogues): the 16 mask bits of (key, col)
__device__ __forceinline__ uint32_t drop_bits(uint64_t seed, int64_t key, int64_t col) {
  return drop_half(drop_hash_k(drop_row_key(seed, key), drop_col_key(col)), col);
}

// 16 B per lane, buffer_load_dwordx4 ... lds into M0 = lds (lane-linear): the descriptor over
// [p, p + n) is built from readfirstlane'd values, so it stays in SGPRs (a select between two
// descriptors went to VGPRs and turned every load into a waterfall loop); the lane offset is
// voff, the step soff (scalar); offsets at or past n read zeros
__device__ __forceinline__ void dma16(uint64_t p, uint32_t n, unsigned char *lds, uint32_t voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef __attribute__((address_space(3))) void lds_v;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0, (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_v *)lds, 16, voff, soff, 0, 0);
#endif
}

#if defined(__HIP_DEVICE_COMPILE__)
// dma16 split in two: the descriptor once (outside a k loop: wave-uniform SGPRs, no v_readfirstlane
// per piece), the piece with it
__device__ __forceinline__ __amdgpu_buffer_rsrc_t dma_rsrc(uint64_t p, uint32_t n) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(n), 0x00020000);
}
__device__ __forceinline__ void dma16r(__amdgpu_buffer_rsrc_t rs, unsigned char *lds, uint32_t voff, int soff) {
  typedef __attribute__((address_space(3))) void lds_v;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_v *)lds, 16, voff, soff, 0, 0);
}
#endif

// The ReLU/dropout backward of two packed bf16 values (element 0 in the low half):
// (y > 0) ? RNE_bf16(g * scale) : 0 per element, on the packed datapath -- one v_pk_mul_f32 and one
// v_cvt_pk_bf16_f32 per pair.  Shared by lpg_relu_bwd_colsum_bf16 (bwd.hip) and the folded form in
// the bf16 FC epilogue (fc_bf16.hip), so the two give the same bits for every input, NaN included.
typedef float lpg_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 lpg_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t relu_bwd_pk_bf16(uint32_t g, uint32_t y, float scale) {
  const lpg_f32x2 gf = {__uint_as_float(g << 16), __uint_as_float(g & 0xffff0000u)};
  const uint32_t pk = __builtin_bit_cast(uint32_t, __builtin_convertvector(gf * lpg_f32x2{scale, scale}, lpg_bf16x2));
  const float y0 = __uint_as_float(y << 16), y1 = __uint_as_float(y & 0xffff0000u);
  return (y0 > 0.f ? (pk & 0xffffu) : 0u) | (y1 > 0.f ? (pk & 0xffff0000u) : 0u);
}

// A workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, then
// s_barrier.  __syncthreads() also carries a release fence, i.e. s_waitcnt vmcnt(0): every
// global load and store the wave has in flight -- a streaming kernel that stages rows in LDS
// drained its prefetched loads (and its stores) at each such barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// bwd.hip: the fold of a small-K weight-gradient partial image [nblk][K + 1][N] into dW1 [N, K1],
// dW2 [N, K - K1], db [N] (block order); the part + segment floats it needs
int64_t smallk_fold_floats(int64_t nblk, int64_t KR, int64_t N);
lpg_status smallk_fold(int64_t nblk, int64_t N, int K1, int K, const float *part, float *seg, float *dW1, float *dW2,
                       float *db, hipStream_t s);

// bwd.hip: db [N] of a bf16 dZ [M, N] from lpg_colsum_bf16's partial image `part` (its workspace), the
// chunks of rows [0, r0) already written by a producer (fc_bf16_p's folded ReLU backward), the rest
// summed from g; the bits of lpg_colsum_bf16
lpg_status colsum_bf16_from(int64_t M, int64_t N, const uint16_t *g, int64_t ldg, int64_t r0, float *part, float *db,
                            hipStream_t s);

// Host-side dropout threshold / scale shared by the FC entry points.
inline void dropout_params(float p, uint32_t *thresh, float *scale) {
  *thresh = 0u;
  *scale = 1.f;
  if (p > 0.f) {
    const double th = (double)p * 65536.0 + 0.5;  // round(p * 2^16), in [1, 65535]
    *thresh = th >= 65535.0 ? 65535u : (uint32_t)(th < 1.0 ? 1.0 : th);
    // kept values x 2^16 / (2^16 - thresh): the reciprocal of the rate actually kept, so E[out]
    // is exact whatever rounding the 16-bit threshold took (lpgnn.fc.dropout_scale mirrors it)
    *scale = 65536.f / (float)(65536u - *thresh);
  }
}

// ---- f16x2 operand scales (fc_x3.hip's f16x2 kernels; the maxima come from lpg_rowcolscale_f32 or from
// the producing kernel's own stores: fc_smallk_f32, heads_bwd_p1) ----
// ---- f16x2 operand preparation ---------------------------------------------------
// The power-of-2 scale that puts a row's largest |x| in [2^14, 2^15): 2^(15 - e) for max = f 2^e,
// f in [0.5, 1); 1 for a non-finite row (NaN / Inf propagate through the split as in fp32); for an
// all-zero row the largest scale, 2^115, so the scale of two operands' rows side by side is the
// smaller of their own (the host combines cached per-operand scales that way).  e is clamped to
// [-100, 120] so the scale and its inverse stay normal fp32 numbers.
__device__ __forceinline__ float f16x2_scale(float mx) {
  if (mx == 0.f) return ldexpf(1.f, 115);
  if (!(mx > 0.f) || !(mx <= 3.4e38f)) return 1.f;
  int e;
  frexpf(mx, &e);
  e = e < -100 ? -100 : (e > 120 ? 120 : e);
  return ldexpf(1.f, 15 - e);
}

// 1 / s for a scale of f16x2_scale (a power of two in [2^-105, 2^115], so 1 / s is a normal power of
// two): the exponent reflected about 0 by one integer subtract -- the bits of the IEEE division, which
// costs ~10 VALU (v_div_scale / v_rcp / v_div_fmas / v_div_fixup) per call
__device__ __forceinline__ float inv_pow2(float s) { return __uint_as_float(0x7f000000u - __float_as_uint(s)); }

// Eight rows' values x[0..7] (one per row, this lane's part) -> their maxima over the wave's 64 lanes in
// a halving butterfly: each exchange halves what a lane carries (4 + 2 + 1 exchanges, then a 3-step
// all-reduce inside eight lanes); lane l ends with row ((l >> 5) & 1) * 4 + ((l >> 4) & 1) * 2 +
// ((l >> 3) & 1)'s maximum.  No LDS traffic: the 32- and 16-lane exchanges are gfx950's
// v_permlane32_swap / v_permlane16_swap (a swap of rows 0-3 of the upper half with rows 4-7 of the lower
// half leaves every lane its own value and its partner's in the two results: one swap + one max per
// pair), the 8-lane one a DPP row rotation, the rest DPP (half-mirror, quad permutations).  (As
// __shfl_xor these were ten ds_bpermute per eight rows.)
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float rowmax8(const float (&x)[8], int lane) {
  float y[4], z[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // lanes 0-31 end with rows 0-3, lanes 32-63 with rows 4-7
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x[i]), __float_as_uint(x[i + 4]), false, false);
    y[i] = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // odd 16-lane rows end with the odd pair
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(y[i]), __float_as_uint(y[i + 2]), false, false);
    z[i] = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
  const bool b3 = (lane & 8) != 0;  // lanes 8-15 of each 16 keep z[1], and take the other half's z[1]
  float w = fmaxf(b3 ? z[1] : z[0], dpp_f32<0x128>(b3 ? z[0] : z[1]));  // row_ror:8 = lane ^ 8 in a row
  w = fmaxf(w, dpp_f32<0x141>(w));                                      // row_half_mirror: i <-> 7 - i
  w = fmaxf(w, dpp_f32<0xB1>(w));                                       // quad_perm [1,0,3,2]
  return fmaxf(w, dpp_f32<0x4E>(w));                                    // quad_perm [2,3,0,1]
}
__device__ __forceinline__ int rowmax8_slot(int lane) {
  return ((lane & 32) ? 4 : 0) + ((lane & 16) ? 2 : 0) + ((lane & 8) ? 1 : 0);
}

namespace {
typedef float lpg_cf32x4 __attribute__((ext_vector_type(4)));
// scale[n] from the chunks' column maxima part[c][n]: a block per 64 columns, its 256 threads 16
// float4 column groups x 16 chunk strides (loads independent, unrolled), then the 16 folded in LDS
__global__ __launch_bounds__(256) void colfold_f32(int64_t chunks, int64_t N, const float *__restrict__ part,
                                                   float *__restrict__ scale) {
  __shared__ lpg_cf32x4 red[16][16];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int64_t c4 = (int64_t)blockIdx.x * 64 + tx * 4;
  lpg_cf32x4 m = {0.f, 0.f, 0.f, 0.f};
  if (c4 < N) {
#pragma unroll 8
    for (int64_t c = ty; c < chunks; c += 16) {
      const lpg_cf32x4 v = *reinterpret_cast<const lpg_cf32x4 *>(part + c * N + c4);
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], v[e]);
    }
  }
  red[ty][tx] = m;
  __syncthreads();
  if (ty == 0 && c4 < N) {
#pragma unroll
    for (int k = 1; k < 16; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], red[k][tx][e]);
#pragma unroll
    for (int e = 0; e < 4; ++e) scale[c4 + e] = f16x2_scale(m[e]);
  }
}
}  // namespace

}  // namespace lpg
