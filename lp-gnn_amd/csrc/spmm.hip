// CSR SpMM for the bipartite cons<->var message passing of GCN_FC on gfx950.
//
// Replaces torch_sparse 0.6.12 `spmm_sum` (csrc/spmm.cpp SPMMSum, CPU loop in
// csrc/cpu/spmm_cpu.cpp, CUDA spmm_kernel in csrc/cuda/spmm_cuda.cu), reached
// from the reference through PyG GraphConv.message_and_aggregate at
// arch.py:75-80 (both directions) and from SPMMSum::backward during
// loss.backward() (train.py:128).
//
// Numerics: per output element the sum runs over the row's edges in CSR
// order, acc = acc + (val * x) with the product rounded before the add
// (this file is compiled with -ffp-contract=off and the pragma below), which
// is exactly torch_sparse's CPU loop; the results are bitwise equal to it and
// to oracle/spmm_ref.c.  No atomics anywhere.
//
// Mapping (CDNA4, wave64): one wave owns one destination row and a slice of
// its columns.  In the fp32 wide kernel lane l holds columns
// c0 + q*256 + 4l .. +3 for q < NV, so each source-row gather is NV fully
// coalesced 1 KiB wave-instructions (global_load_dwordx4).  The row's
// (col, val) pairs are fetched 64 at a time, one per lane, and broadcast with
// v_readlane (wave-uniform -> the gather base is a scalar).  U edges are
// gathered before any of them is accumulated, so U*NV 16-byte loads per lane
// are in flight (4 rows in flight per wave at F = 1024).
#include "common.h"

#pragma clang fp contract(off)

namespace lpg {
namespace {

constexpr int kBlock = 256;            // 4 waves
constexpr int kWavesPerBlock = kBlock / 64;

__device__ __forceinline__ int bcast_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ float bcast_f(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

__device__ __forceinline__ void axpy4(float4 &acc, float v, const float4 &x) {
  acc.x = acc.x + v * x.x;
  acc.y = acc.y + v * x.y;
  acc.z = acc.z + v * x.z;
  acc.w = acc.w + v * x.w;
}

// Heavy rows (degree > thresh; SpMM skew, e.g. a dense LP constraint): one block per heavy row
// and column slice, its 4 waves on interleaved 64-column pieces (lane l of wave w holds columns
// c0 + 256 q + 64 w + l, q < NV: one float per lane, every gather a contiguous 256 B), HU edges
// gathered ahead (HU = 32, the next 64-edge chunk's indices prefetched).  The row's chain is split over 4x the waves of a (row, slice) wave, every
// element still summed over the row's edges in CSR order (bitwise the same result), so a
// 6 000-edge row no longer sets the kernel's tail.
// All (heavy row, slice) units sit at the head of plane 0 (longest rows first: the host passes the
// rows by decreasing degree), so every long chain starts at the beginning of the launch instead of
// when its slice's plane is dispatched; the same block ids in the other planes exit at once.
struct HeavyRows {
  const int32_t *rows;  // heavy row ids (rows with degree > thresh), longest first
  int64_t blocks;       // = number of heavy rows
  int64_t thresh;       // the main waves skip rows with more edges than this
  int64_t slices;       // column slices of the launch (set by the launcher)
};

template <int NV, int HU>
__device__ __forceinline__ void spmm_f32_heavy_row(int64_t row, int64_t c0, int wave,
                                                   const int64_t *__restrict__ rowptr,
                                                   const int32_t *__restrict__ col, const float *__restrict__ val,
                                                   const float *__restrict__ X, int64_t ldx, float *__restrict__ Y,
                                                   int64_t ldy, int64_t F) {
  const int lane = threadIdx.x & 63;
  const int64_t cw = c0 + wave * 64 + lane;
  bool ok[NV];
  float acc[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) ok[q] = cw + q * 256 < F, acc[q] = 0.f;
  const float *Xs = X + cw;
  int64_t e = rowptr[row];
  const int64_t end = rowptr[row + 1];
  // the next 64-edge chunk's (col, val) are fetched while this chunk's gathers are in flight
  int cn = 0;
  float vn = 0.f;
  if (e + lane < end) {
    cn = col[e + lane];
    vn = val[e + lane];
  }
  while (e < end) {
    const int n = (int)(end - e < 64 ? end - e : 64);
    const int cl = cn;
    const float vl = vn;
    if (e + 64 + lane < end) {
      cn = col[e + 64 + lane];
      vn = val[e + 64 + lane];
    }
    int j = 0;
    for (; j + HU <= n; j += HU) {
      float xv[HU][NV];
#pragma unroll
      for (int k = 0; k < HU; ++k) {
        const float *xr = Xs + (int64_t)bcast_i(cl, j + k) * ldx;
#pragma unroll
        for (int q = 0; q < NV; ++q) xv[k][q] = ok[q] ? xr[q * 256] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < HU; ++k) {
        const float v = bcast_f(vl, j + k);
#pragma unroll
        for (int q = 0; q < NV; ++q) acc[q] = acc[q] + v * xv[k][q];
      }
    }
    for (; j < n; ++j) {
      const float *xr = Xs + (int64_t)bcast_i(cl, j) * ldx;
      const float v = bcast_f(vl, j);
#pragma unroll
      for (int q = 0; q < NV; ++q) acc[q] = acc[q] + v * (ok[q] ? xr[q * 256] : 0.f);
    }
    e += n;
  }
  float *yr = Y + row * ldy + cw;
#pragma unroll
  for (int q = 0; q < NV; ++q)
    if (ok[q]) yr[q * 256] = acc[q];
}

// ---------------------------------------------------------------- fp32 wide
// REMB: the chunk's last n mod U edges are gathered together too (predicated per edge, wave-uniform)
// instead of one dependent load at a time: a row of 20 edges costs 3 memory round trips, not 6,
// and rows shorter than U (most rows of a skewed LP) one.  Same edges, same order: same bits.
template <int NV, int U, bool FULL, bool REMB = true>
__global__ __launch_bounds__(kBlock) void spmm_f32_rowwave(
    int64_t n_rows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const float *__restrict__ val, const float *__restrict__ X, int64_t ldx,
    float *__restrict__ Y, int64_t ldy, int64_t F, HeavyRows hv) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t hb = hv.blocks * hv.slices;
  if ((int64_t)blockIdx.x < hb) {  // heavy (row, slice) units: all at the head of plane 0
    if (blockIdx.y != 0) return;
    // 32-bit division (the 64-bit expansion uses v_fmamk_f32, which the no-FMA ISA guard rejects)
    const uint32_t hs = (uint32_t)hv.slices, bxu = blockIdx.x;
    const int64_t hr = bxu / hs, sl = bxu % hs;
    spmm_f32_heavy_row<NV, 32>(hv.rows[hr], sl * (NV * 256), wave, rowptr, col, val, X, ldx, Y, ldy, F);
    return;
  }
  const int64_t row = ((int64_t)blockIdx.x - hb) * kWavesPerBlock + wave;
  if (row >= n_rows) return;
  if (rowptr[row + 1] - rowptr[row] > hv.thresh) return;  // a heavy row: done by the units above
  const int64_t c0 = (int64_t)blockIdx.y * (NV * 256);

  bool ok[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) ok[q] = FULL || (c0 + q * 256 + lane * 4 < F);

  float4 acc[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);

  const float *Xs = X + c0 + lane * 4;
  int64_t e = rowptr[row];
  const int64_t end = rowptr[row + 1];
  while (e < end) {
    const int n = (int)(end - e < 64 ? end - e : 64);
    int cl = 0;
    float vl = 0.f;
    if (lane < n) {
      cl = col[e + lane];
      vl = val[e + lane];
    }
    int j = 0;
    for (; j + U <= n; j += U) {
      float4 xv[U][NV];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const float *xr = Xs + (int64_t)bcast_i(cl, j + k) * ldx;
#pragma unroll
        for (int q = 0; q < NV; ++q)
          xv[k][q] = ok[q] ? *reinterpret_cast<const float4 *>(xr + q * 256) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const float v = bcast_f(vl, j + k);
#pragma unroll
        for (int q = 0; q < NV; ++q) axpy4(acc[q], v, xv[k][q]);
      }
    }
    if (REMB && j < n) {
      const int rem = n - j;  // 1 .. U-1, wave-uniform
      float4 xv[U][NV];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (k < rem) {
          const float *xr = Xs + (int64_t)bcast_i(cl, j + k) * ldx;
#pragma unroll
          for (int q = 0; q < NV; ++q)
            xv[k][q] = ok[q] ? *reinterpret_cast<const float4 *>(xr + q * 256) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (k < rem) {
          const float v = bcast_f(vl, j + k);
#pragma unroll
          for (int q = 0; q < NV; ++q) axpy4(acc[q], v, xv[k][q]);
        }
      }
      j = n;
    }
    for (; j < n; ++j) {
      const float *xr = Xs + (int64_t)bcast_i(cl, j) * ldx;
      const float v = bcast_f(vl, j);
      float4 xv[NV];
#pragma unroll
      for (int q = 0; q < NV; ++q)
        xv[q] = ok[q] ? *reinterpret_cast<const float4 *>(xr + q * 256) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < NV; ++q) axpy4(acc[q], v, xv[q]);
    }
    e += n;
  }

  float *yr = Y + row * ldy + c0 + lane * 4;
#pragma unroll
  for (int q = 0; q < NV; ++q)
    if (ok[q]) *reinterpret_cast<float4 *>(yr + q * 256) = acc[q];
}

// ------------------------------------------------------- fp32 narrow slices
// For gathered tables far above the 256 MiB Infinity Cache (c4: a [4M, 1024] fp32 table is 16 GB, a
// 256-column slice still 4 GB): one wave per (row, 64*CW-column slice), lane l holding columns
// c0 + CW*l .. +CW-1 (CW = 2: 512 B per gather, CW = 1: 256 B), so a slice of the table is 2-4x
// smaller than at 256 columns.  Same edge order, the chunk remainder gathered together: the same bits.
#ifndef LPG_SPMM_NT
#define LPG_SPMM_NT 1
#endif
// The wide kernels' output rows (written once) as non-temporal stores (round 6), so they do not displace
// the gathered source slice the launch keeps in L2 / MALL: c2 step 15.67 -> 15.60 ms, c5 62.15 -> 61.96 on
// one box (profiles/r06_epi_nt_ab.log); the same bits.
typedef float spmm_f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int spmm_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_out(float *p, float v) {
  if constexpr (LPG_SPMM_NT) __builtin_nontemporal_store(v, p); else *p = v;
}
__device__ __forceinline__ void st_out(float *p, float2 v) {
  if constexpr (LPG_SPMM_NT) __builtin_nontemporal_store(spmm_f32x2{v.x, v.y}, reinterpret_cast<spmm_f32x2 *>(p));
  else *reinterpret_cast<float2 *>(p) = v;
}
__device__ __forceinline__ void st_out(void *p, uint2 v) {
  if constexpr (LPG_SPMM_NT) __builtin_nontemporal_store(spmm_u32x2{v.x, v.y}, reinterpret_cast<spmm_u32x2 *>(p));
  else *reinterpret_cast<uint2 *>(p) = v;
}

template <int CW> struct VecF;
template <> struct VecF<1> { typedef float T; };
template <> struct VecF<2> { typedef float2 T; };

__device__ __forceinline__ void axpyv(float &acc, float v, float x) { acc = acc + v * x; }
__device__ __forceinline__ void axpyv(float2 &acc, float v, float2 x) {
  acc.x = acc.x + v * x.x;
  acc.y = acc.y + v * x.y;
}
__device__ __forceinline__ void zerov(float &a) { a = 0.f; }
__device__ __forceinline__ void zerov(float2 &a) { a = make_float2(0.f, 0.f); }

template <int CW, int U>
__global__ __launch_bounds__(kBlock) void spmm_f32_rowslim(int64_t n_rows, const int64_t *__restrict__ rowptr,
                                                           const int32_t *__restrict__ col,
                                                           const float *__restrict__ val, const float *__restrict__ X,
                                                           int64_t ldx, float *__restrict__ Y, int64_t ldy, int64_t F) {
  typedef typename VecF<CW>::T V;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t row = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (row >= n_rows) return;
  const int64_t c0 = (int64_t)blockIdx.y * (64 * CW);
  const bool ok = c0 + lane * CW < F;
  V acc;
  zerov(acc);
  const float *Xs = X + c0 + lane * CW;
  int64_t e = rowptr[row];
  const int64_t end = rowptr[row + 1];
  while (e < end) {
    const int n = (int)(end - e < 64 ? end - e : 64);
    int cl = 0;
    float vl = 0.f;
    if (lane < n) {
      cl = col[e + lane];
      vl = val[e + lane];
    }
    int j = 0;
    for (; j + U <= n; j += U) {
      V xv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (ok) xv[k] = *reinterpret_cast<const V *>(Xs + (int64_t)bcast_i(cl, j + k) * ldx); else zerov(xv[k]);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) axpyv(acc, bcast_f(vl, j + k), xv[k]);
    }
    if (j < n) {
      const int rem = n - j;  // wave-uniform
      V xv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (k < rem) {
          if (ok) xv[k] = *reinterpret_cast<const V *>(Xs + (int64_t)bcast_i(cl, j + k) * ldx); else zerov(xv[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (k < rem) axpyv(acc, bcast_f(vl, j + k), xv[k]);
    }
    e += n;
  }
  if (ok) st_out(Y + row * ldy + c0 + lane * CW, acc);
}

// ------------------------------------------------------------------- narrow
// F <= FW <= 64 (conv1's input, F = 8): FW lanes per row, 256/FW rows per block, one output element
// per lane, its sum over the row's edges in CSR order (acc = acc + v*x, product rounded first), one
// rounding to the storage type at the end.  L: the storage -- NF32 (fp32) or N16<E> (bf16 / fp16).
//
// HEAVY: the launch's first hv.blocks blocks are heavy-row units, one block per row with more than
// hv.thresh edges (a skewed LP's dense constraints, up to thousands of edges; longest first).  One FW-lane
// group walking such a row is one long dependent chain of memory round trips (round 5: 1.05 ms for the
// skewed conv1 launch against 0.03 ms on the uniform graph).  The unit splits the row into chunks of
// CH = 192 * kNarrowPer / FW edges.  Waves 1-3 (192 loader lanes, kNarrowPer products each) gather a
// chunk -- X[col, f] and the rounded product v*x, with the NEXT chunk's (col, val) already in flight --
// into one of two LDS buffers, column-major (lane f's products contiguous, rows padded by 4 floats so the
// 16-B reads of the FW summing lanes fall in distinct banks), while lane f < F of wave 0 adds the
// previous chunk's products into its accumulator in CSR order (four per 16-B LDS read).  One barrier
// per chunk.  The same products in the same order: the same bits as the FW-lane loop.
constexpr int kNarrowPer = 16;      // products per loader lane per chunk
constexpr int kNarrowLoaders = 192;  // waves 1..3

struct NF32 {
  typedef float T;
  __device__ static __forceinline__ float get(float x) { return x; }
  __device__ static __forceinline__ float put(float a) { return a; }
};
template <class E> struct N16 {
  typedef uint16_t T;
  __device__ static __forceinline__ float get(uint16_t h) { return E::lo(h); }
  __device__ static __forceinline__ uint16_t put(float a) { return E::rne(a); }
};

template <class L, int FW>
__device__ __forceinline__ void narrow_heavy_row(int64_t row, const int64_t *__restrict__ rowptr,
                                                 const int32_t *__restrict__ col, const float *__restrict__ val,
                                                 const typename L::T *__restrict__ X, int64_t ldx,
                                                 typename L::T *__restrict__ Y, int64_t ldy, int64_t F) {
  constexpr int EPI = kNarrowLoaders / FW;  // edges per loader step
  constexpr int CH = EPI * kNarrowPer;       // edges per chunk
  constexpr int LD = CH + 4;                 // a column's stride in the LDS image
  __shared__ __attribute__((aligned(16))) float prod[2][FW * LD];
  const int t = threadIdx.x;
  const int64_t e0 = rowptr[row];
  const int64_t end = rowptr[row + 1];
  const int nch = (int)((end - e0 + CH - 1) / CH);
  if (t >= 64) {  // loaders
    const int l = t - 64;
    const int f = l % FW;    // this lane's column (192 is a multiple of FW)
    const int le0 = l / FW;  // this lane's first edge of a chunk; then every EPI-th
    const bool act = f < F;
    int c[kNarrowPer];
    float v[kNarrowPer];
    auto fetch = [&](int64_t cb) {  // chunk base cb: its (col, val)
#pragma unroll
      for (int i = 0; i < kNarrowPer; ++i) {
        const int64_t e = cb + le0 + i * EPI;
        c[i] = e < end ? col[e] : 0;
        v[i] = e < end ? val[e] : 0.f;
      }
    };
    fetch(e0);
    for (int k = 0; k <= nch; ++k) {
      if (k < nch) {
        const int64_t cb = e0 + (int64_t)k * CH;
        float x[kNarrowPer];
#pragma unroll
        for (int i = 0; i < kNarrowPer; ++i)
          x[i] = (act && cb + le0 + i * EPI < end) ? L::get(X[(int64_t)c[i] * ldx + f]) : 0.f;
        float p[kNarrowPer];
#pragma unroll
        for (int i = 0; i < kNarrowPer; ++i) p[i] = v[i] * x[i];
        if (k + 1 < nch) fetch(cb + CH);  // the next chunk's indices in flight under this chunk's stores
        float *buf = prod[k & 1] + f * LD;
#pragma unroll
        for (int i = 0; i < kNarrowPer; ++i)
          if (act && cb + le0 + i * EPI < end) buf[le0 + i * EPI] = p[i];
      }
      __syncthreads();
    }
  } else {  // wave 0: lane t < F sums the previous chunk while the loaders fill the next
    const bool act = t < FW && t < F;
    float acc = 0.f;
    for (int k = 0; k <= nch; ++k) {
      if (k > 0 && act) {
        const int n = (int)(end - (e0 + (int64_t)(k - 1) * CH) < CH ? end - (e0 + (int64_t)(k - 1) * CH) : CH);
        const float *buf = prod[(k - 1) & 1] + t * LD;
        int j = 0;
#pragma unroll 4
        for (; j + 4 <= n; j += 4) {
          const float4 q = *reinterpret_cast<const float4 *>(buf + j);
          acc = acc + q.x;
          acc = acc + q.y;
          acc = acc + q.z;
          acc = acc + q.w;
        }
        for (; j < n; ++j) acc = acc + buf[j];
      }
      __syncthreads();
    }
    if (act) Y[row * ldy + t] = L::put(acc);
  }
}

template <class L, int FW, int U, bool HEAVY>
__global__ __launch_bounds__(kBlock) void spmm_narrow(
    int64_t n_rows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const float *__restrict__ val, const typename L::T *__restrict__ X, int64_t ldx,
    typename L::T *__restrict__ Y, int64_t ldy, int64_t F, HeavyRows hv) {
  constexpr int RPB = kBlock / FW;
  int64_t blk = blockIdx.x;
  if constexpr (HEAVY) {
    if (blk < hv.blocks) {
      narrow_heavy_row<L, FW>(hv.rows[blk], rowptr, col, val, X, ldx, Y, ldy, F);
      return;
    }
    blk -= hv.blocks;
  }
  const int sub = threadIdx.x % FW;
  const int64_t row = blk * RPB + threadIdx.x / FW;
  if (row >= n_rows) return;
  int64_t e = rowptr[row];
  const int64_t end = rowptr[row + 1];
  if (HEAVY && end - e > hv.thresh) return;  // a heavy row: done by its unit above
  const bool active = sub < F;
  const typename L::T *Xs = X + sub;
  float acc = 0.f;
  for (; e + U <= end; e += U) {
    int c[U];
    float v[U], x[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      c[k] = col[e + k];
      v[k] = val[e + k];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) x[k] = active ? L::get(Xs[(int64_t)c[k] * ldx]) : 0.f;
#pragma unroll
    for (int k = 0; k < U; ++k) acc = acc + v[k] * x[k];
  }
  for (; e < end; ++e) {
    const float x = active ? L::get(Xs[(int64_t)col[e] * ldx]) : 0.f;
    acc = acc + val[e] * x;
  }
  if (active) Y[row * ldy + sub] = L::put(acc);
}

// ------------------------------------------------------------- fp32 generic
// Any F / stride / alignment: one wave per row, lane strides the columns.
__global__ __launch_bounds__(kBlock) void spmm_f32_generic(
    int64_t n_rows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const float *__restrict__ val, const float *__restrict__ X, int64_t ldx,
    float *__restrict__ Y, int64_t ldy, int64_t F) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const int64_t beg = rowptr[row], end = rowptr[row + 1];
  for (int64_t c = lane; c < F; c += 64) {
    float acc = 0.f;
    for (int64_t e = beg; e < end; ++e) acc = acc + val[e] * X[(int64_t)col[e] * ldx + c];
    Y[row * ldy + c] = acc;
  }
}

// ------------------------------------------------------------------ bf16
__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

__device__ __forceinline__ uint32_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x0040u;  // keep NaN a NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

// The 16-bit storage of a kernel instance: bf16 (c5) or fp16 (the reference's --fp16 inference,
// val.py:269: SparseTensor.half() and model.half()).  lo / hi: element 0 / 1 of a packed pair as
// fp32 (exact); pack: RNE of a pair; rne: RNE of one value.  The accumulation is fp32 either way,
// rounded once per output (torch_sparse's CUDA spmm_sum accumulates in the storage type; the fp32
// sum here is the more accurate one -- DESIGN.md §5).
struct SBf16 {
  __device__ static __forceinline__ float lo(uint32_t w) { return bf16_to_f32(w & 0xffffu); }
  __device__ static __forceinline__ float hi(uint32_t w) { return bf16_to_f32(w >> 16); }
  __device__ static __forceinline__ uint32_t pack(float a, float b) {
    return f32_to_bf16_rne(a) | (f32_to_bf16_rne(b) << 16);
  }
  __device__ static __forceinline__ uint16_t rne(float f) { return (uint16_t)f32_to_bf16_rne(f); }
};
struct SF16 {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  __device__ static __forceinline__ float lo(uint32_t w) { return (float)__builtin_bit_cast(_Float16, (uint16_t)w); }
  __device__ static __forceinline__ float hi(uint32_t w) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
  }
  __device__ static __forceinline__ uint32_t pack(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{a, b}, h2));
  }
  __device__ static __forceinline__ uint16_t rne(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
};

template <class E>
__device__ __forceinline__ void axpy8_bf16(float (&acc)[8], float v, const uint4 &x) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    acc[2 * i] = acc[2 * i] + v * E::lo(w[i]);
    acc[2 * i + 1] = acc[2 * i + 1] + v * E::hi(w[i]);
  }
}

// bf16 heavy rows (degree > thresh): one block per (heavy row, 512-column piece) at the head of plane 0
// of a 512-column spmm_bf16_rowwave launch, wave w on columns
// c0 + 128 w + 2 l, +1 (4-B gathers, 256 B per wave-instruction), 32 gathers in flight and the next
// 64-edge chunk's indices prefetched -- 4x the waves on one long row's chain, each element still
// summed in CSR order (the same bits).
template <class E>
__device__ __forceinline__ void spmm_bf16_heavy_row(int64_t row, int64_t c0, int wave,
                                                    const int64_t *__restrict__ rowptr,
                                                    const int32_t *__restrict__ col, const float *__restrict__ val,
                                                    const uint16_t *__restrict__ X, int64_t ldx,
                                                    uint16_t *__restrict__ Y, int64_t ldy, int64_t F) {
  constexpr int HU = 32;
  const int lane = threadIdx.x & 63;
  const int64_t cw = c0 + wave * 128 + lane * 2;
  const bool ok = cw < F;
  float a0 = 0.f, a1 = 0.f;
  const uint16_t *Xs = X + cw;
  int64_t e = rowptr[row];
  const int64_t end = rowptr[row + 1];
  int cn = 0;
  float vn = 0.f;
  if (e + lane < end) {
    cn = col[e + lane];
    vn = val[e + lane];
  }
  while (e < end) {
    const int n = (int)(end - e < 64 ? end - e : 64);
    const int cl = cn;
    const float vl = vn;
    if (e + 64 + lane < end) {
      cn = col[e + 64 + lane];
      vn = val[e + 64 + lane];
    }
    int j = 0;
    for (; j + HU <= n; j += HU) {  // full batches: no predication (uniform branches around loads
      uint32_t xv[HU];              // made the waitcnt pass serialise them)
#pragma unroll
      for (int k = 0; k < HU; ++k)
        xv[k] = ok ? *reinterpret_cast<const uint32_t *>(Xs + (int64_t)bcast_i(cl, j + k) * ldx) : 0u;
#pragma unroll
      for (int k = 0; k < HU; ++k) {
        const float v = bcast_f(vl, j + k);
        a0 = a0 + v * E::lo(xv[k]);
        a1 = a1 + v * E::hi(xv[k]);
      }
    }
    if (j < n) {
      const int rem = n - j;  // wave-uniform, < HU
      uint32_t xv[HU];
#pragma unroll
      for (int k = 0; k < HU; ++k)
        if (k < rem) xv[k] = ok ? *reinterpret_cast<const uint32_t *>(Xs + (int64_t)bcast_i(cl, j + k) * ldx) : 0u;
#pragma unroll
      for (int k = 0; k < HU; ++k)
        if (k < rem) {
          const float v = bcast_f(vl, j + k);
          a0 = a0 + v * E::lo(xv[k]);
          a1 = a1 + v * E::hi(xv[k]);
        }
    }
    e += n;
  }
  if (ok) *reinterpret_cast<uint32_t *>(Y + row * ldy + cw) = E::pack(a0, a1);
}

// Lane l holds columns c0 + q*512 + 8l .. +7 (16 bytes) for q < NV.  HEAVY (NV = 1): the launch's
// leading blocks of plane 0 are heavy (row, 512-column) units, as in spmm_f32_rowwave.
template <class E, int NV, int U, bool FULL, bool HEAVY = false>
__global__ __launch_bounds__(kBlock) void spmm_bf16_rowwave(
    int64_t n_rows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const float *__restrict__ val, const uint16_t *__restrict__ X, int64_t ldx,
    uint16_t *__restrict__ Y, int64_t ldy, int64_t F, HeavyRows hv) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t hb = HEAVY ? hv.blocks * hv.slices : 0;
  if constexpr (HEAVY) {
    if ((int64_t)blockIdx.x < hb) {
      if (blockIdx.y != 0) return;
      const uint32_t hs = (uint32_t)hv.slices, bxu = blockIdx.x;
      spmm_bf16_heavy_row<E>(hv.rows[bxu / hs], (int64_t)(bxu % hs) * 512, wave, rowptr, col, val, X, ldx, Y, ldy, F);
      return;
    }
  }
  const int64_t row = ((int64_t)blockIdx.x - hb) * kWavesPerBlock + wave;
  if (row >= n_rows) return;
  if (HEAVY && rowptr[row + 1] - rowptr[row] > hv.thresh) return;  // a heavy row: done by the units above
  const int64_t c0 = (int64_t)blockIdx.y * (NV * 512);
  bool ok[NV];
#pragma unroll
  for (int q = 0; q < NV; ++q) ok[q] = FULL || (c0 + q * 512 + lane * 8 < F);
  float acc[NV][8];
#pragma unroll
  for (int q = 0; q < NV; ++q)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[q][i] = 0.f;

  const uint16_t *Xs = X + c0 + lane * 8;
  int64_t e = rowptr[row];
  const int64_t end = rowptr[row + 1];
  while (e < end) {
    const int n = (int)(end - e < 64 ? end - e : 64);
    int cl = 0;
    float vl = 0.f;
    if (lane < n) {
      cl = col[e + lane];
      vl = val[e + lane];
    }
    int j = 0;
    for (; j + U <= n; j += U) {
      uint4 xv[U][NV];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint16_t *xr = Xs + (int64_t)bcast_i(cl, j + k) * ldx;
#pragma unroll
        for (int q = 0; q < NV; ++q)
          xv[k][q] = ok[q] ? *reinterpret_cast<const uint4 *>(xr + q * 512) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const float v = bcast_f(vl, j + k);
#pragma unroll
        for (int q = 0; q < NV; ++q) axpy8_bf16<E>(acc[q], v, xv[k][q]);
      }
    }
    for (; j < n; ++j) {
      const uint16_t *xr = Xs + (int64_t)bcast_i(cl, j) * ldx;
      const float v = bcast_f(vl, j);
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const uint4 xv = ok[q] ? *reinterpret_cast<const uint4 *>(xr + q * 512) : make_uint4(0, 0, 0, 0);
        axpy8_bf16<E>(acc[q], v, xv);
      }
    }
    e += n;
  }
  uint16_t *yr = Y + row * ldy + c0 + lane * 8;
#pragma unroll
  for (int q = 0; q < NV; ++q) {
    if (!ok[q]) continue;
    uint4 o;
    o.x = E::pack(acc[q][0], acc[q][1]);
    o.y = E::pack(acc[q][2], acc[q][3]);
    o.z = E::pack(acc[q][4], acc[q][5]);
    o.w = E::pack(acc[q][6], acc[q][7]);
    *reinterpret_cast<uint4 *>(yr + q * 512) = o;
  }
}

// bf16 narrow slices: one wave per (row, 256-column slice), lane l holding columns c0 + 4l .. +3
// (8-B gathers, 512 B per wave-instruction), fp32 accumulation, one RNE rounding -- the bf16 twin of
// spmm_f32_rowslim (a slice of the c5 [200K, 2048] bf16 table is 102 MB instead of the whole 820 MB),
// the chunk remainder gathered together.  Same edge order: the same bits as spmm_bf16_rowwave.
template <class E, int U>
__global__ __launch_bounds__(kBlock) void spmm_bf16_rowslim(int64_t n_rows, const int64_t *__restrict__ rowptr,
                                                            const int32_t *__restrict__ col,
                                                            const float *__restrict__ val,
                                                            const uint16_t *__restrict__ X, int64_t ldx,
                                                            uint16_t *__restrict__ Y, int64_t ldy, int64_t F) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t row = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (row >= n_rows) return;
  const int64_t c0 = (int64_t)blockIdx.y * 256;
  const bool ok = c0 + lane * 4 < F;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const uint16_t *Xs = X + c0 + lane * 4;
  auto axpy = [&](float v, uint2 x) {
    acc[0] = acc[0] + v * E::lo(x.x);
    acc[1] = acc[1] + v * E::hi(x.x);
    acc[2] = acc[2] + v * E::lo(x.y);
    acc[3] = acc[3] + v * E::hi(x.y);
  };
  int64_t e = rowptr[row];
  const int64_t end = rowptr[row + 1];
  while (e < end) {
    const int n = (int)(end - e < 64 ? end - e : 64);
    int cl = 0;
    float vl = 0.f;
    if (lane < n) {
      cl = col[e + lane];
      vl = val[e + lane];
    }
    int j = 0;
    for (; j + U <= n; j += U) {
      uint2 xv[U];
#pragma unroll
      for (int k = 0; k < U; ++k)
        xv[k] = ok ? *reinterpret_cast<const uint2 *>(Xs + (int64_t)bcast_i(cl, j + k) * ldx) : make_uint2(0, 0);
#pragma unroll
      for (int k = 0; k < U; ++k) axpy(bcast_f(vl, j + k), xv[k]);
    }
    if (j < n) {
      const int rem = n - j;  // wave-uniform
      uint2 xv[U];
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (k < rem)
          xv[k] = ok ? *reinterpret_cast<const uint2 *>(Xs + (int64_t)bcast_i(cl, j + k) * ldx) : make_uint2(0, 0);
#pragma unroll
      for (int k = 0; k < U; ++k)
        if (k < rem) axpy(bcast_f(vl, j + k), xv[k]);
    }
    e += n;
  }
  if (ok) {
    uint2 o;
    o.x = E::pack(acc[0], acc[1]);
    o.y = E::pack(acc[2], acc[3]);
    st_out(Y + row * ldy + c0 + lane * 4, o);
  }
}

template <class E>
__global__ __launch_bounds__(kBlock) void spmm_bf16_generic(
    int64_t n_rows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const float *__restrict__ val, const uint16_t *__restrict__ X, int64_t ldx,
    uint16_t *__restrict__ Y, int64_t ldy, int64_t F) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const int64_t beg = rowptr[row], end = rowptr[row + 1];
  for (int64_t c = lane; c < F; c += 64) {
    float acc = 0.f;
    for (int64_t e = beg; e < end; ++e) acc = acc + val[e] * E::lo(X[(int64_t)col[e] * ldx + c]);
    Y[row * ldy + c] = E::rne(acc);
  }
}

// Tuning is per call (lpg_spmm_*_tuned): slice width and gather depth; every choice gives the same
// bits.  (The fp32 rowwave kernel gathers a chunk's remainder together; the bf16 kernel keeps one
// by one: batched, it measured 7-55 % slower.)
lpg_status check_tuning(int64_t slice_cols, int32_t depth) {
  LPG_REQUIRE(slice_cols == 0 || slice_cols == 64 || slice_cols == 128 || slice_cols == 256 || slice_cols == 512 ||
                  slice_cols == 1024,
              "lpg_spmm_*_tuned: slice_cols must be 0 (auto), 64, 128, 256, 512 or 1024, got %lld",
              (long long)slice_cols);
  LPG_REQUIRE(depth == 0 || depth == 8 || depth == 16 || depth == 32, "lpg_spmm_*_tuned: depth %d not in {0, 8, 16, 32}",
              (int)depth);
  return LPG_OK;
}

lpg_status check_csr(const lpg_csr *A) {
  LPG_REQUIRE(A != nullptr, "lpg_spmm: A is NULL");
  LPG_REQUIRE(A->n_rows >= 0 && A->n_cols >= 0 && A->nnz >= 0, "lpg_spmm: negative CSR size");
  LPG_REQUIRE(A->n_rows == 0 || A->rowptr != nullptr, "lpg_spmm: rowptr is NULL");
  LPG_REQUIRE(A->nnz == 0 || (A->col != nullptr && A->val != nullptr), "lpg_spmm: col/val is NULL");
  LPG_REQUIRE(A->n_cols <= INT32_MAX, "lpg_spmm: n_cols exceeds int32 column index");
  return LPG_OK;
}

template <class K, class... Args>
lpg_status launch(K kernel, dim3 grid, hipStream_t s, Args... args) {
  hipLaunchKernelGGL(kernel, grid, dim3(kBlock), 0, s, args...);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

template <int NV, int U>
lpg_status launch_wide_f32(const lpg_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                           int64_t F, hipStream_t s, HeavyRows hv) {
  const int64_t W = NV * 256;
  const int64_t slices = (F + W - 1) / W;
  hv.slices = slices;
  const int64_t nblk = (A->n_rows + kWavesPerBlock - 1) / kWavesPerBlock + hv.blocks * slices;
  LPG_REQUIRE(nblk < ((int64_t)1 << 31), "lpg_spmm_f32: grid too large");
  dim3 grid((unsigned)nblk, (unsigned)slices);
  if (F % W == 0)
    return launch(spmm_f32_rowwave<NV, U, true>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx,
                  Y, ldy, F, hv);
  return launch(spmm_f32_rowwave<NV, U, false>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y,
                ldy, F, hv);
}

template <class L, int FW>
lpg_status launch_narrow_fw(const lpg_csr *A, const typename L::T *X, int64_t ldx, typename L::T *Y, int64_t ldy,
                            int64_t F, HeavyRows hv, hipStream_t s) {
  constexpr int RPB = kBlock / FW;
  const int64_t nblk = (A->n_rows + RPB - 1) / RPB + hv.blocks;
  LPG_REQUIRE(nblk < ((int64_t)1 << 31), "lpg_spmm: grid too large");
  dim3 grid((unsigned)nblk);
  if (hv.blocks > 0)
    return launch(spmm_narrow<L, FW, 4, true>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F, hv);
  return launch(spmm_narrow<L, FW, 4, false>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F, hv);
}

// F <= 64: FW = the next power of 2 >= F lanes per row
template <class L>
lpg_status launch_narrow(const lpg_csr *A, const typename L::T *X, int64_t ldx, typename L::T *Y, int64_t ldy,
                         int64_t F, HeavyRows hv, hipStream_t s) {
  if (F <= 1) return launch_narrow_fw<L, 1>(A, X, ldx, Y, ldy, F, hv, s);
  if (F <= 2) return launch_narrow_fw<L, 2>(A, X, ldx, Y, ldy, F, hv, s);
  if (F <= 4) return launch_narrow_fw<L, 4>(A, X, ldx, Y, ldy, F, hv, s);
  if (F <= 8) return launch_narrow_fw<L, 8>(A, X, ldx, Y, ldy, F, hv, s);
  if (F <= 16) return launch_narrow_fw<L, 16>(A, X, ldx, Y, ldy, F, hv, s);
  if (F <= 32) return launch_narrow_fw<L, 32>(A, X, ldx, Y, ldy, F, hv, s);
  return launch_narrow_fw<L, 64>(A, X, ldx, Y, ldy, F, hv, s);
}

template <class E, int NV, int U>
lpg_status launch_wide_bf16(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy,
                            int64_t F, hipStream_t s) {
  const int64_t W = NV * 512;
  const int64_t slices = (F + W - 1) / W;
  dim3 grid((unsigned)((A->n_rows + kWavesPerBlock - 1) / kWavesPerBlock), (unsigned)slices);
  const HeavyRows none{nullptr, 0, INT64_MAX, 1};
  if (F % W == 0)
    return launch(spmm_bf16_rowwave<E, NV, U, true>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx,
                  Y, ldy, F, none);
  return launch(spmm_bf16_rowwave<E, NV, U, false>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx,
                Y, ldy, F, none);
}

// 512-column slices with the heavy rows split off (heavy units first in plane 0)
template <class E>
lpg_status launch_bf16_heavy(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy,
                             int64_t F, HeavyRows hv, hipStream_t s) {
  hv.slices = (F + 511) / 512;
  const int64_t nblk = (A->n_rows + kWavesPerBlock - 1) / kWavesPerBlock + hv.blocks * hv.slices;
  LPG_REQUIRE(nblk < ((int64_t)1 << 31), "lpg_spmm_bf16: grid too large");
  dim3 grid((unsigned)nblk, (unsigned)hv.slices);
  if (F % 512 == 0)
    return launch(spmm_bf16_rowwave<E, 1, 8, true, true>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y,
                  ldy, F, hv);
  return launch(spmm_bf16_rowwave<E, 1, 8, false, true>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y,
                ldy, F, hv);
}

}  // namespace
}  // namespace lpg

using namespace lpg;

static lpg_status spmm_f32_impl(const lpg_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                                HeavyRows hv, int64_t slice_cols, int32_t depth, void *stream) {
  lpg_status st = check_csr(A);
  if (st != LPG_OK) return st;
  st = check_tuning(slice_cols, depth);
  if (st != LPG_OK) return st;
  LPG_REQUIRE(F >= 0, "lpg_spmm_f32: F < 0");
  LPG_REQUIRE(ldx >= F && ldy >= F, "lpg_spmm_f32: ldx/ldy smaller than F");
  if (A->n_rows == 0 || F == 0) return LPG_OK;
  LPG_REQUIRE(Y != nullptr, "lpg_spmm_f32: Y is NULL");
  LPG_REQUIRE(A->nnz == 0 || X != nullptr, "lpg_spmm_f32: X is NULL");
  hipStream_t s = as_stream(stream);

  if (F <= 64) return launch_narrow<NF32>(A, X, ldx, Y, ldy, F, hv, s);
  const bool vec = (F % 4 == 0) && (ldx % 4 == 0) && (ldy % 4 == 0) && aligned16(X) && aligned16(Y);
  if (!vec) {
    dim3 grid((unsigned)((A->n_rows + kWavesPerBlock - 1) / kWavesPerBlock));
    return launch(spmm_f32_generic, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F);
  }
  int64_t W = slice_cols;
  // auto: 256-column slices (one float4 per lane).  Slices run in order
  // (blockIdx.y major), so only a quarter-width source table is being
  // gathered at a time and stays resident in the 256 MiB Infinity Cache;
  // measured ~3 % faster than full-width rows at c2 (profiles/r01_kbench*).
  // auto: 128-column slices (2 floats per lane, 512-B gathers; measured 0.95 / 0.99 of the edge-gather
  // roofline at c2 vs 0.93 / 0.94 at 256, profiles/r02_kbench_spmm_big.log) unless heavy rows are split
  // off, which the 256-column form does
  if (W == 0) W = hv.blocks == 0 ? 128 : 256;
  // auto depth: 8 edges in flight per batch (round 3, profiles/r03_kbench_spmmdepth.log, same box:
  // c2 cons<-vars 0.975 at 8 vs 0.967 at 16, vars<-cons 0.980 vs 0.927; depth 32 0.52-0.71; round 2
  // had measured 16 ahead for cons<-vars, 0.947 vs 0.913; the heavy-row split already used 8)
  const int U = depth != 0 ? depth : 8;
  if ((W == 64 || W == 128) && hv.blocks == 0) {  // narrow slices (no heavy-row split in this form)
    dim3 grid((unsigned)((A->n_rows + kWavesPerBlock - 1) / kWavesPerBlock), (unsigned)((F + W - 1) / W));
    if (W == 128)
      return U == 16 ? launch(spmm_f32_rowslim<2, 16>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F)
                     : launch(spmm_f32_rowslim<2, 8>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F);
    return U == 16 ? launch(spmm_f32_rowslim<1, 16>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F)
                   : launch(spmm_f32_rowslim<1, 8>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F);
  }
  if (W == 64 || W == 128) W = 256;
  if (W == 256) {
    if (U == 16) return launch_wide_f32<1, 16>(A, X, ldx, Y, ldy, F, s, hv);
    if (U == 32) return launch_wide_f32<1, 32>(A, X, ldx, Y, ldy, F, s, hv);
    return launch_wide_f32<1, 8>(A, X, ldx, Y, ldy, F, s, hv);
  }
  if (W == 512) {
    if (U == 16) return launch_wide_f32<2, 16>(A, X, ldx, Y, ldy, F, s, hv);
    return launch_wide_f32<2, 8>(A, X, ldx, Y, ldy, F, s, hv);
  }
  return launch_wide_f32<4, 4>(A, X, ldx, Y, ldy, F, s, hv);
}

extern "C" lpg_status lpg_spmm_f32(const lpg_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                                   int64_t F, void *stream) {
  return spmm_f32_impl(A, X, ldx, Y, ldy, F, HeavyRows{nullptr, 0, INT64_MAX, 1}, 0, 0, stream);
}

extern "C" lpg_status lpg_spmm_f32_tuned(const lpg_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                                         int64_t F, const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh,
                                         int64_t slice_cols, int32_t depth, void *stream) {
  LPG_REQUIRE(n_heavy >= 0 && thresh >= 0, "lpg_spmm_f32_tuned: negative n_heavy / thresh");
  LPG_REQUIRE(n_heavy == 0 || heavy_rows != nullptr, "lpg_spmm_f32_tuned: heavy_rows is NULL");
  LPG_REQUIRE(A != nullptr && n_heavy <= A->n_rows, "lpg_spmm_f32_tuned: more heavy rows than rows");
  return spmm_f32_impl(A, X, ldx, Y, ldy, F, HeavyRows{heavy_rows, n_heavy, n_heavy ? thresh : INT64_MAX, 1},
                       slice_cols, depth, stream);
}

extern "C" lpg_status lpg_spmm_f32_heavy(const lpg_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                                         int64_t F, const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh,
                                         void *stream) {
  LPG_REQUIRE(n_heavy >= 0 && thresh >= 0, "lpg_spmm_f32_heavy: negative n_heavy / thresh");
  LPG_REQUIRE(n_heavy == 0 || heavy_rows != nullptr, "lpg_spmm_f32_heavy: heavy_rows is NULL");
  LPG_REQUIRE(A != nullptr && n_heavy <= A->n_rows, "lpg_spmm_f32_heavy: more heavy rows than rows");
  return spmm_f32_impl(A, X, ldx, Y, ldy, F, HeavyRows{heavy_rows, n_heavy, n_heavy ? thresh : INT64_MAX, 1}, 0, 0,
                       stream);
}

template <class E>
static lpg_status spmm_bf16_impl(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy,
                                 int64_t F, HeavyRows hv, int64_t slice_cols, int32_t depth, void *stream) {
  lpg_status st = check_csr(A);
  if (st != LPG_OK) return st;
  st = check_tuning(slice_cols, depth);
  if (st != LPG_OK) return st;
  LPG_REQUIRE(F >= 0, "lpg_spmm_bf16: F < 0");
  LPG_REQUIRE(ldx >= F && ldy >= F, "lpg_spmm_bf16: ldx/ldy smaller than F");
  if (A->n_rows == 0 || F == 0) return LPG_OK;
  LPG_REQUIRE(Y != nullptr, "lpg_spmm_bf16: Y is NULL");
  LPG_REQUIRE(A->nnz == 0 || X != nullptr, "lpg_spmm_bf16: X is NULL");
  hipStream_t s = as_stream(stream);
  const bool vec = (F % 8 == 0) && (ldx % 8 == 0) && (ldy % 8 == 0) && aligned16(X) && aligned16(Y);
  if (F <= 64) return launch_narrow<N16<E>>(A, X, ldx, Y, ldy, F, hv, s);  // any alignment
  if (!vec || F < 256) {
    dim3 grid((unsigned)((A->n_rows + kWavesPerBlock - 1) / kWavesPerBlock));
    return launch(spmm_bf16_generic<E>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F);
  }
  // slice width: slice_cols (256 = spmm_bf16_rowslim, 512 / 1024 / 2048 = rowwave with 1 / 2 / 4
  // 16-B pieces per lane); auto = 256 (c5: 0.92 / 0.97 of the edge-gather roofline vs 0.88 / 0.91 for
  // whole 2048-column rows, profiles/r02_kbench_spmm16.log); with heavy rows split off, 512-column slices
// (spmm_bf16_rowwave<1, 8> + heavy units: a skewed LP's mostly one-edge rows want few, wide wave tasks)
  if (hv.blocks > 0) return launch_bf16_heavy<E>(A, X, ldx, Y, ldy, F, hv, s);
  const int64_t W = slice_cols == 0 ? 256 : slice_cols;
  if (W <= 256) {
    const int64_t nblk = (A->n_rows + kWavesPerBlock - 1) / kWavesPerBlock;
    LPG_REQUIRE(nblk < ((int64_t)1 << 31), "lpg_spmm_bf16: grid too large");
    dim3 grid((unsigned)nblk, (unsigned)((F + 255) / 256));
    // auto depth 8 (c5 cons<-vars 0.970 of the edge-gather roofline at 8 vs 0.903 at 16, vars<-cons
    // 0.970 vs 0.807: profiles/r03_kbench_spmmdepth.log)
    const int U = depth != 0 ? depth : 8;
    if (U == 16) return launch(spmm_bf16_rowslim<E, 16>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F);
    return launch(spmm_bf16_rowslim<E, 8>, grid, s, A->n_rows, A->rowptr, A->col, A->val, X, ldx, Y, ldy, F);
  }
  if (W == 512 || F <= 512) return launch_wide_bf16<E, 1, 8>(A, X, ldx, Y, ldy, F, s);
  if (W == 1024 || F <= 1024) return launch_wide_bf16<E, 2, 8>(A, X, ldx, Y, ldy, F, s);
  return launch_wide_bf16<E, 4, 4>(A, X, ldx, Y, ldy, F, s);
}

extern "C" lpg_status lpg_spmm_bf16(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y,
                                    int64_t ldy, int64_t F, void *stream) {
  return spmm_bf16_impl<SBf16>(A, X, ldx, Y, ldy, F, HeavyRows{nullptr, 0, INT64_MAX, 1}, 0, 0, stream);
}

extern "C" lpg_status lpg_spmm_bf16_tuned(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy,
                                          int64_t F, const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh,
                                          int64_t slice_cols, int32_t depth, void *stream) {
  LPG_REQUIRE(n_heavy >= 0 && thresh >= 0, "lpg_spmm_bf16_tuned: negative n_heavy / thresh");
  LPG_REQUIRE(n_heavy == 0 || heavy_rows != nullptr, "lpg_spmm_bf16_tuned: heavy_rows is NULL");
  LPG_REQUIRE(A != nullptr && n_heavy <= A->n_rows, "lpg_spmm_bf16_tuned: more heavy rows than rows");
  return spmm_bf16_impl<SBf16>(A, X, ldx, Y, ldy, F, HeavyRows{heavy_rows, n_heavy, n_heavy ? thresh : INT64_MAX, 1},
                        slice_cols, depth, stream);
}

extern "C" lpg_status lpg_spmm_bf16_heavy(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y,
                                          int64_t ldy, int64_t F, const int32_t *heavy_rows, int64_t n_heavy,
                                          int64_t thresh, void *stream) {
  LPG_REQUIRE(n_heavy >= 0 && thresh >= 0, "lpg_spmm_bf16_heavy: negative n_heavy / thresh");
  LPG_REQUIRE(n_heavy == 0 || heavy_rows != nullptr, "lpg_spmm_bf16_heavy: heavy_rows is NULL");
  LPG_REQUIRE(A != nullptr && n_heavy <= A->n_rows, "lpg_spmm_bf16_heavy: more heavy rows than rows");
  return spmm_bf16_impl<SBf16>(A, X, ldx, Y, ldy, F, HeavyRows{heavy_rows, n_heavy, n_heavy ? thresh : INT64_MAX, 1}, 0, 0,
                        stream);
}

// fp16 storage (the reference's --fp16 inference: SparseTensor.half() and model.half(), utils.py:909-915,
// val.py:269): the bf16 kernels with fp16 conversions -- fp32 accumulation in CSR edge order, one RNE
// rounding to fp16 per output.  Edge values stay fp32 (batch_to(half=True) rounds them to fp16
// first, lpgnn.data), so the products are those of fp16 values.
extern "C" lpg_status lpg_spmm_f16(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy,
                                   int64_t F, void *stream) {
  return spmm_bf16_impl<SF16>(A, X, ldx, Y, ldy, F, HeavyRows{nullptr, 0, INT64_MAX, 1}, 0, 0, stream);
}

extern "C" lpg_status lpg_spmm_f16_tuned(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy,
                                         int64_t F, const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh,
                                         int64_t slice_cols, int32_t depth, void *stream) {
  LPG_REQUIRE(n_heavy >= 0 && thresh >= 0, "lpg_spmm_f16_tuned: negative n_heavy / thresh");
  LPG_REQUIRE(n_heavy == 0 || heavy_rows != nullptr, "lpg_spmm_f16_tuned: heavy_rows is NULL");
  LPG_REQUIRE(A != nullptr && n_heavy <= A->n_rows, "lpg_spmm_f16_tuned: more heavy rows than rows");
  return spmm_bf16_impl<SF16>(A, X, ldx, Y, ldy, F, HeavyRows{heavy_rows, n_heavy, n_heavy ? thresh : INT64_MAX, 1},
                              slice_cols, depth, stream);
}
