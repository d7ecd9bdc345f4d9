// Device helpers of the fp32-on-bf16 ("x3") kernels (fc_x3.hip, wgrad_x3q.hip): vector types, the
// exact three-way bf16 split (fc_x3.hip's header comment) and a raw 4-B buffer load.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lpg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned pk_bf16(float x, float y) {  // v_cvt_pk_bf16_f32: RNE, x in the low half
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{x, y}, bf16x2));
}

// exact residual x - h as one v_sub_f32: kept out of the SLP vectorizer's reach, which paired
// the two subtractions of a level into v_pk_add_f32 -- an issue-cost anti-lever beside MFMAs
// (MI355X_MICROARCH.md, 'price of one filler beside MFMAs')
__device__ __forceinline__ float sub_f32(float x, float h) {
  float r;
  asm("v_sub_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(h));
  return r;
}

// one split level of a pair: the packed RNE bf16 terms; the exact residuals are left in x, y
__device__ __forceinline__ unsigned split_lvl(float &x, float &y) {
  const unsigned p = pk_bf16(x, y);
  x = sub_f32(x, __uint_as_float(p << 16));
  y = sub_f32(y, __uint_as_float(p & 0xffff0000u));
  return p;
}

struct Split3 {
  bf16x8 h, m, l;
};

// 8 consecutive k (lo = k 0..3, hi = k 4..7) -> the three bf16x8 MFMA operands
__device__ __forceinline__ Split3 split3(f32x4 lo, f32x4 hi) {
  u32x4 H, Mi, L;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float x = i < 2 ? lo[2 * i] : hi[2 * i - 4], y = i < 2 ? lo[2 * i + 1] : hi[2 * i - 3];
    H[i] = split_lvl(x, y);
    Mi[i] = split_lvl(x, y);
    L[i] = pk_bf16(x, y);
  }
  return Split3{__builtin_bit_cast(bf16x8, H), __builtin_bit_cast(bf16x8, Mi), __builtin_bit_cast(bf16x8, L)};
}

// ---- "f16x2": two fp16 planes per operand after a power-of-2 row scale (fc_x3.hip, F16 kernels) ----
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

struct Split2 {
  f16x8 h, l;
};

// 8 consecutive k of one row, times the row's scale s (a power of 2: exact), as h = RNE_f16(x s) and
// l = RNE_f16(x s - h) (the residual exact in fp32): |x s - h - l| <= 2^-22 |x s| while |x s| >= 2^-3,
// and <= 2^-25 below (fp16 subnormals); the scale puts the row's largest |x| in [2^14, 2^15)
//
// Per pair of k, four mixed-precision FMAs and nothing else: h = fma_mix(x, s, 0) rounded to fp16 (lo
// half, then the next x into the hi half), l = fma_mix(x, s, -h) with h read as fp16 from its half --
// x s - h computed exactly inside the FMA and rounded once, the same RNE_f16 of the exact residual
// the f32 multiply / convert / subtract / convert chain gave (x s is exact: s a power of 2; x s - h
// is exact in fp32), in 2 instructions per element instead of 5.
__device__ __forceinline__ void split_pair_f16(float x0, float x1, float s, uint32_t &h, uint32_t &l) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h), "=&v"(l)
      : "v"(x0), "v"(x1), "v"(s));
}

__device__ __forceinline__ Split2 split2f16(f32x4 lo, f32x4 hi, float s) {
  u32x4 H, L;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = i < 2 ? lo[2 * i] : hi[2 * i - 4], x1 = i < 2 ? lo[2 * i + 1] : hi[2 * i - 3];
    uint32_t h, l;
    split_pair_f16(x0, x1, s, h, l);
    H[i] = h;
    L[i] = l;
  }
  return Split2{__builtin_bit_cast(f16x8, H), __builtin_bit_cast(f16x8, L)};
}

// 4-B raw buffer load (v# in SGPRs: base and size wave-uniform): offsets at or past `nbytes` return
// zeros, with no branch and no compare in the kernel
__device__ __forceinline__ float buf_load1(const float *base, uint32_t nbytes, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), (short)0, (int)nbytes, 0x00020000);
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, soff, 0));
#else
  return 0.f;
#endif
}

}  // namespace
}  // namespace lpg
