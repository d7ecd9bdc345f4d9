// Memory-bound pieces of the GraphConv / head backward (train.py:128 loss.backward()
// through arch.py:57-62, 182-191), fused so each large gradient is streamed once:
//
//   lpg_relu_bwd_colsum_f32   dZ = (Y > 0) ? dY * scale : 0   (ReLU + fused dropout backward)
//                             and db = sum_m dZ[m, :]          (lin_rel.bias grad) in the same pass
//   lpg_wgrad_smallk_f32      dW1 = dZ^T A1, dW2 = dZ^T A2 for small K (conv1: K1 = K2 = 8 LP features)
//   lpg_relu_wgrad_smallk_f32 the same from (g, y) with the ReLU/dropout backward and db fused (dZ never stored)
//   lpg_linear_small_bwd_f32  the heads' backward (N = 3 outputs): dH = G W, dW = G^T H, db = sum G
//
// plus the c5 (bf16) twins and the bf16 heads' forward.  Row-block kernels: a block owns a range
// of rows and 16 B of columns per thread, streams its rows with the next group's loads issued
// before the current group's arithmetic, and writes one row of per-block partial sums.  The
// partials are then added in a fixed order -- a fold into kFold segment sums (many blocks,
// coalesced), then a short final pass -- so results are deterministic run to run, with no atomics.
#include "common.h"
#include "fc_common.h"

#include <type_traits>

#pragma clang fp contract(off)

namespace lpg {
namespace {

constexpr int kT = 256;
constexpr int kRowsColsum = 64;
#ifndef LPG_HEADS_U_F32
#define LPG_HEADS_U_F32 8
#endif
#ifndef LPG_HEADS_U_BF16
#define LPG_HEADS_U_BF16 8
#endif
#ifndef LPG_HEADS_U_SC
#define LPG_HEADS_U_SC 4
#endif
#ifndef LPG_HEADS_RB
#define LPG_HEADS_RB 128
#endif
constexpr int kRowsLinear = LPG_HEADS_RB;  // heads_bwd_p1 rows per block (64-row column-sum chunks)
constexpr int kMaxSmallK = 16;
constexpr int kSmallNMax = 4;
constexpr int64_t kFold = 64;

__device__ __forceinline__ float4 relu_scale(float4 g, float4 y, float scale) {
  float4 o;
  o.x = y.x > 0.f ? g.x * scale : 0.f;
  o.y = y.y > 0.f ? g.y * scale : 0.f;
  o.z = y.z > 0.f ? g.z * scale : 0.f;
  o.w = y.w > 0.f ? g.w * scale : 0.f;
  return o;
}

__device__ __forceinline__ void add4(float4 &s, float4 o) {
  s.x = s.x + o.x; s.y = s.y + o.y; s.z = s.z + o.z; s.w = s.w + o.w;
}

__global__ __launch_bounds__(kT) void relu_bwd_colsum_p1(int64_t M, int64_t N, const float *__restrict__ g,
                                                         int64_t ldg, const float *__restrict__ y, int64_t ldy,
                                                         float scale, float *__restrict__ out, int64_t ldo,
                                                         float *__restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowsColsum;
  const int64_t r1 = r0 + kRowsColsum < M ? r0 + kRowsColsum : M;
  for (int64_t c = (int64_t)threadIdx.x * 4; c < N; c += kT * 4) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t m = r0;
    for (; m + 4 <= r1; m += 4) {
      float4 gv[4], yv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        gv[u] = *reinterpret_cast<const float4 *>(g + (m + u) * ldg + c);
        yv[u] = *reinterpret_cast<const float4 *>(y + (m + u) * ldy + c);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 o = relu_scale(gv[u], yv[u], scale);
        *reinterpret_cast<float4 *>(out + (m + u) * ldo + c) = o;
        add4(s, o);
      }
    }
    for (; m < r1; ++m) {
      const float4 o = relu_scale(*reinterpret_cast<const float4 *>(g + m * ldg + c),
                                  *reinterpret_cast<const float4 *>(y + m * ldy + c), scale);
      *reinterpret_cast<float4 *>(out + m * ldo + c) = o;
      add4(s, o);
    }
    if (part) *reinterpret_cast<float4 *>(part + (int64_t)blockIdx.x * N + c) = s;
  }
}

// bf16 twin (c5 path): g, y, out bf16; db fp32.  8 columns per thread (16-B
// loads), 2048 per pass; dZ = RNE(bf16)(g * scale) where y > 0, the value
// torch's bf16 `g * scale` gives; db sums the rounded dZ in fp32.
__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {  // RNE, v_cvt_pk_bf16_f32
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(lpg_f32x2{lo, hi}, lpg_bf16x2));
}


// MASK = false (lpg_colsum_bf16): g already is dZ (the folded form, lpg_fc_bf16_relu_bwd) --
// only the column sums, same blocks and order, so the same db bits; y and out unused.
template <bool MASK>
__global__ __launch_bounds__(kT) void relu_bwd_colsum_bf16_p1(int64_t M, int64_t N, const uint16_t *__restrict__ g,
                                                              int64_t ldg, const uint16_t *__restrict__ y,
                                                              int64_t ldy, float scale, uint16_t *__restrict__ out,
                                                              int64_t ldo, float *__restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowsColsum;
  const int64_t r1 = r0 + kRowsColsum < M ? r0 + kRowsColsum : M;
  for (int64_t c = (int64_t)threadIdx.x * 8; c < N; c += kT * 8) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto row = [&](uint4 gv, uint4 yv, int64_t m) {
      const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w}, yw[4] = {yv.x, yv.y, yv.z, yv.w};
      uint32_t ow[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const uint32_t o = MASK ? relu_bwd_pk_bf16(gw[h], yw[h], scale) : gw[h];  // fc_common.h
        s[2 * h] = s[2 * h] + bf16_to_f32(o & 0xffffu);
        s[2 * h + 1] = s[2 * h + 1] + bf16_to_f32(o >> 16);
        ow[h] = o;
      }
      if constexpr (MASK) *reinterpret_cast<uint4 *>(out + m * ldo + c) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    };
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    int64_t m = r0;
    for (; m + 4 <= r1; m += 4) {
      uint4 gv[4], yv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        gv[u] = *reinterpret_cast<const uint4 *>(g + (m + u) * ldg + c);
        yv[u] = MASK ? *reinterpret_cast<const uint4 *>(y + (m + u) * ldy + c) : z4;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) row(gv[u], yv[u], m + u);
    }
    for (; m < r1; ++m)
      row(*reinterpret_cast<const uint4 *>(g + m * ldg + c),
          MASK ? *reinterpret_cast<const uint4 *>(y + m * ldy + c) : z4, m);
    if (part) {
      float *pp = part + (int64_t)blockIdx.x * N + c;
      *reinterpret_cast<float4 *>(pp) = make_float4(s[0], s[1], s[2], s[3]);
      *reinterpret_cast<float4 *>(pp + 4) = make_float4(s[4], s[5], s[6], s[7]);
    }
  }
}

// Fold stage: seg[s][i] = sum of part[b][i] over b in segment s of [0, nblk),
// in b order (grid: n / kT x kFold).
__global__ __launch_bounds__(kT) void fold_partials(int64_t nblk, int64_t n, const float *__restrict__ part,
                                                    float *__restrict__ seg) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const int64_t sg = blockIdx.y;
  const int64_t b0 = sg * nblk / kFold, b1 = (sg + 1) * nblk / kFold;
  float s = 0.f;
  int64_t b = b0;
  for (; b + 8 <= b1; b += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(b + u) * n + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s = s + v[u];
  }
  for (; b < b1; ++b) s = s + part[b * n + i];
  seg[sg * n + i] = s;
}

__device__ __forceinline__ float sum_rows(int64_t nrow, int64_t n, const float *__restrict__ img, int64_t i) {
  float s = 0.f;
  int64_t b = 0;
  for (; b + 8 <= nrow; b += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = img[(b + u) * n + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s = s + v[u];
  }
  for (; b < nrow; ++b) s = s + img[b * n + i];
  return s;
}

// out[i] = sum_b img[b][i]
__global__ __launch_bounds__(kT) void sum_partials(int64_t nrow, int64_t n, const float *__restrict__ img,
                                                   float *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = sum_rows(nrow, n, img, i);
}

// Reduces part [nblk][n] to the image the final pass sums: either part itself
// (few blocks) or the [kFold][n] segment sums in `seg`.  Returns its row count.
int64_t fold(int64_t nblk, int64_t n, const float *part, float *seg, const float **img, hipStream_t s) {
  if (nblk <= 2 * kFold) {
    *img = part;
    return nblk;
  }
  hipLaunchKernelGGL(fold_partials, dim3((unsigned)((n + kT - 1) / kT), (unsigned)kFold), dim3(kT), 0, s, nblk, n,
                     part, seg);
  *img = seg;
  return kFold;
}

int64_t fold_floats(int64_t nblk, int64_t n) { return (nblk + (nblk > 2 * kFold ? kFold : 0)) * n; }

// Weight gradients of a narrow-input FC (conv1: K = K1 + K2 <= 16 LP features):
//   part[s][k][n] = sum over block s's rows m of A[m][k] * dZ[m][n]   (k < K),
//   part[s][K][n] = sum_m dZ[m][n]                                    (the bias gradient row)
// dZ = the stored gradient, or with MASK (y > 0) ? g * scale : 0 from the output gradient g and the
// stored output y (bf16: relu_bwd_pk_bf16, the bits of relu_bwd_colsum_bf16 and of the folded
// store).  Grid (column groups of 1024 = 256 threads x 4 columns, S row ranges): block s owns rows
// [s M / S, (s + 1) M / S) -- every resident block the same share, the partial image [S][K + 1][N]
// independent of M -- walked in 64-row chunks whose [A1 | A2] rows are staged in LDS as fp32
// (double-buffered; the next chunk's values are loaded into registers a chunk ahead).  The
// gradient rows stream in groups of U, the next group's loads issued before the current group's
// FMAs (>= 128 B per lane in flight; hipcc otherwise interleaved them with the arithmetic and kept
// two loads in flight, 1.8 TB/s for bf16), accumulated as column pairs on v_pk_fma_f32.  (Weight
// gradients carry no bitwise contract: fma chains per block, folded in block order, checked against
// fp64 within the summation bound.)
constexpr int kChunk = 64;

template <bool BF> using G4 = typename std::conditional<BF, uint2, float4>::type;  // 4 gradient values

template <bool BF, bool MASK>
__device__ __forceinline__ void grad_pairs(G4<BF> g, G4<BF> y, float scale, lpg_f32x2 &z01, lpg_f32x2 &z23) {
  if constexpr (BF) {
    uint32_t a = g.x, b = g.y;
    if constexpr (MASK) {
      a = relu_bwd_pk_bf16(a, y.x, scale);
      b = relu_bwd_pk_bf16(b, y.y, scale);
    }
    z01 = lpg_f32x2{__uint_as_float(a << 16), __uint_as_float(a & 0xffff0000u)};
    z23 = lpg_f32x2{__uint_as_float(b << 16), __uint_as_float(b & 0xffff0000u)};
  } else {
    if constexpr (MASK) g = relu_scale(g, y, scale);
    z01 = lpg_f32x2{g.x, g.y};
    z23 = lpg_f32x2{g.z, g.w};
  }
}

template <int K, bool MASK, bool BF>
__global__ __launch_bounds__(kT) void wgrad_smallk_p1(int64_t M, int64_t N, const void *__restrict__ dzv, int64_t ldz,
                                                      const void *__restrict__ yv, int64_t ldy, float scale, int K1,
                                                      const void *__restrict__ A1v, int64_t lda1,
                                                      const void *__restrict__ A2v, int64_t lda2, int64_t S,
                                                      float *__restrict__ part) {
  using E = typename std::conditional<BF, uint16_t, float>::type;
  constexpr int KP = (K + 3) / 4 * 4;
  constexpr int KR = K + 1;
  constexpr int U = 128 / ((BF ? 8 : 16) * (MASK ? 2 : 1));  // rows per group: 128 B per lane in flight
  constexpr int AE = kChunk * KP / kT;                        // staged A values per thread per chunk
  static_assert(kChunk % (2 * U) == 0 && kChunk * KP % kT == 0, "chunk shape");
  __shared__ float4 sa[2][kChunk * KP / 4];
  const E *dz = static_cast<const E *>(dzv), *y = static_cast<const E *>(yv);
  const E *A1 = static_cast<const E *>(A1v), *A2 = static_cast<const E *>(A2v);
  const int64_t c = (int64_t)blockIdx.x * (kT * 4) + threadIdx.x * 4;
  const bool col_ok = c < N;
  const int64_t cl = col_ok ? c : N - 4;  // lanes past N load an in-range column (never accumulated)
  const int64_t sb = blockIdx.y;
  const int64_t rb = sb * M / S, re = (sb + 1) * M / S;
  if (re <= rb) {  // (block-uniform: no barrier is skipped by part of a block)
    if (col_ok)
      for (int k = 0; k < KR; ++k) *reinterpret_cast<float4 *>(part + (sb * KR + k) * N + c) = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  const int nch = (int)((re - rb + kChunk - 1) / kChunk);
  const int nfull = (int)((re - rb) / kChunk);

  // the next chunk's A values, raw (converted / zeroed when stored, so nothing waits for these
  // loads before the chunk boundary); addresses clamped in range, branchless
  E areg[AE];
  bool aok[AE];
  auto load_a = [&](int64_t r0) {
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      const int i = threadIdx.x + kT * j, r = i / KP, k = i % KP;
      const int64_t m = r0 + r < re ? r0 + r : re - 1;
      const int kk = k < K ? k : K - 1;
      areg[j] = kk < K1 ? A1[m * lda1 + kk] : A2[m * lda2 + (kk - K1)];
      aok[j] = r0 + r < re && k < K;
    }
  };
  auto store_a = [&](int buf) {
    float *sf = reinterpret_cast<float *>(sa[buf]);
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      float v;
      if constexpr (BF) v = bf16_to_f32(areg[j]); else v = areg[j];
      sf[threadIdx.x + kT * j] = aok[j] ? v : 0.f;
    }
  };
  // gradient rows in two register buffers: group g + 1 loads while group g is multiplied (a copy
  // from one buffer into the other made hipcc wait for the loads before the copy)
  G4<BF> gA[U], yA[U], gB[U], yB[U];
  auto issue = [&](G4<BF>(&gb)[U], G4<BF>(&yb)[U], int64_t m0) {  // rows past re: clamped, never used
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t m = m0 + u < re ? m0 + u : re - 1;
      gb[u] = *reinterpret_cast<const G4<BF> *>(dz + m * ldz + cl);
      if constexpr (MASK) yb[u] = *reinterpret_cast<const G4<BF> *>(y + m * ldy + cl);
    }
  };
  lpg_f32x2 acc[KR][2];
#pragma unroll
  for (int k = 0; k < KR; ++k) acc[k][0] = acc[k][1] = lpg_f32x2{0.f, 0.f};
  auto row = [&](G4<BF> gv, G4<BF> yv, const float4 *ar) {
    float a[KP];
#pragma unroll
    for (int q = 0; q < KP / 4; ++q) {
      const float4 v = ar[q];
      a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
    }
    lpg_f32x2 z01, z23;
    grad_pairs<BF, MASK>(gv, yv, scale, z01, z23);
    if (!col_ok) z01 = z23 = lpg_f32x2{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k) {
      acc[k][0] = __builtin_elementwise_fma(lpg_f32x2{a[k], a[k]}, z01, acc[k][0]);
      acc[k][1] = __builtin_elementwise_fma(lpg_f32x2{a[k], a[k]}, z23, acc[k][1]);
    }
    acc[K][0] = acc[K][0] + z01;
    acc[K][1] = acc[K][1] + z23;
  };
  auto group = [&](const G4<BF>(&gb)[U], const G4<BF>(&yb)[U], const float4 *sab, int rl) {
#pragma unroll
    for (int u = 0; u < U; ++u) row(gb[u], yb[u], sab + (rl + u) * (KP / 4));
  };

  load_a(rb);
  store_a(0);
  issue(gA, yA, rb);
  __syncthreads();
  if (nch > 1) load_a(rb + kChunk);
  // whole 64-row chunks: branch-free, one group always in flight
  for (int ch = 0; ch < nfull; ++ch) {
    const float4 *sab = sa[ch & 1];
    const int64_t cb = rb + (int64_t)ch * kChunk;
    for (int j = 0; j < kChunk / (2 * U); ++j) {
      issue(gB, yB, cb + (2 * j + 1) * U);
      __builtin_amdgcn_sched_barrier(0);
      group(gA, yA, sab, 2 * j * U);
      issue(gA, yA, cb + (2 * j + 2) * U);
      __builtin_amdgcn_sched_barrier(0);
      group(gB, yB, sab, (2 * j + 1) * U);
    }
    if (ch + 1 < nch) {  // the next chunk's A (loaded a chunk ago) into the other buffer
      store_a((ch + 1) & 1);
      lds_barrier();  // (not __syncthreads: its fence would drain the gradient loads in flight)
      if (ch + 2 < nch) load_a(cb + 2 * kChunk);
    }
  }
  // the partial last chunk: row by row (gA holds its first group)
  if (nfull < nch) {
    const float4 *sab = sa[nfull & 1];
    const int64_t cb = rb + (int64_t)nfull * kChunk;
    for (int64_t m0 = cb; m0 < re; m0 += U) {
      if (m0 != cb) issue(gA, yA, m0);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (m0 + u < re) row(gA[u], yA[u], sab + (int)(m0 - cb + u) * (KP / 4));
    }
  }
  if (col_ok) {
    float *pb = part + sb * KR * N + c;
#pragma unroll
    for (int k = 0; k < KR; ++k)
      *reinterpret_cast<float4 *>(pb + k * N) = make_float4(acc[k][0][0], acc[k][0][1], acc[k][1][0], acc[k][1][1]);
  }
}

// dW1[n][k] (k < K1), dW2[n][k - K1] (k < K) and db[n] (k = K) from the
// [KR][N] partial image
__global__ __launch_bounds__(kT) void wgrad_smallk_p2(int64_t nrow, int64_t N, int K, int KR, int K1,
                                                      const float *__restrict__ img, float *__restrict__ dW1,
                                                      float *__restrict__ dW2, float *__restrict__ db) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;  // over KR * N, i = k * N + n
  if (i >= (int64_t)KR * N) return;
  const float s = sum_rows(nrow, (int64_t)KR * N, img, i);
  const int k = (int)(i / N);
  const int64_t n = i % N;
  if (k < K1) {
    if (dW1) dW1[n * K1 + k] = s;
  } else if (k < K) {
    if (dW2) dW2[n * (K - K1) + (k - K1)] = s;
  } else if (db) {
    db[n] = s;
  }
}

// Backward of a Linear with few outputs (the heads lin_left / lin_right, N = 3, arch.py:190) over
// its input H [M, K] (fp32, or bf16 for the c5 model), G / W fp32:
//   dH[m, k] = sum_c G[m, c] W[c, k]        (written if dH != NULL; bf16: RNE)
//   dW[c, k] = sum_m G[m, c] H[m, k],  db[c] = sum_m G[m, c]     (per-block partials [N K + N])
// MASK (the fused heads + ReLU backward): H is the output Y of the previous layer's ReLU (+
// dropout) and dH leaves through that layer's ReLU/dropout backward -- the layer's dZ:
// fp32 (Y > 0) ? scale * dH : 0, bf16 relu_bwd_pk_bf16(RNE(dH), Y, scale) -- the bits of the
// separate relu_bwd_colsum pass over the plain dH.  party != NULL: the column sums of the stored
// dH per 64-row chunk in row order into the partial image [ceil(M / 64)][K] of relu_bwd_colsum
// (chunk j = rows [64 j, 64 j + 64)), so the same fold gives the same bits as that pass's db.
// A block owns 128 rows (2 chunks) and 16 B of columns per thread (fp32 4, bf16 8); its G rows are
// staged in LDS once (the per-row G loads were scalar loads, each waited for before its row:
// 4.4 TB/s), the H rows stream in groups of 8 with the next group's loads issued before the current
// group's arithmetic.
template <bool BF> using H16 = typename std::conditional<BF, uint4, float4>::type;

//
// SC (fp32, K a multiple of 1024 so every lane takes part in each k pass; f16x2 consumers of dZ): also
// the f16x2 scale of every stored dH row (rsc[m]; a block holds
// whole rows, so the row maximum is the block's: per group of eight rows a halving butterfly over the
// wave (rowmax8), the four waves through LDS) and the block's column maxima of |dH| (cpart[block][K],
// folded by colfold_f32) -- the scales lpg_rowcolscale_f32 would take from a second read of dZ.
template <int N, bool MASK, bool BF, bool STORE, bool SC = false>
__global__ __launch_bounds__(kT) void heads_bwd_p1(int64_t M, int64_t K, const float *__restrict__ G, int64_t ldg,
                                                   const float *__restrict__ W, const void *__restrict__ Hv,
                                                   int64_t ldh, void *__restrict__ dHv, int64_t lddh, float scale,
                                                   float *__restrict__ part, float *__restrict__ party,
                                                   float *__restrict__ rsc = nullptr, float *__restrict__ cpart = nullptr) {
  using E = typename std::conditional<BF, uint16_t, float>::type;
  constexpr int EPT = BF ? 8 : 4;  // columns per thread
  constexpr int P = EPT / 2;       // column pairs
  // rows per group (8: 128 B per lane in flight); the f16x2-scales form LPG_HEADS_U_SC (4: two groups per
  // eight-row maximum)
  constexpr int U = SC ? LPG_HEADS_U_SC : BF ? LPG_HEADS_U_BF16 : LPG_HEADS_U_F32;
  constexpr int RB = kRowsLinear;  // rows per block
  constexpr int CH = kRowsColsum;  // column-sum chunk
  static_assert(RB % CH == 0 && CH % (2 * U) == 0, "block shape");
  __shared__ float4 sg4[RB];
  __shared__ float rmx[SC ? kT / 64 : 1][SC ? RB : 1];  // SC: per wave, the rows' maxima of |dH|
  static_assert(!SC || (!BF && (U == 8 || U == 4)), "the f16x2 scales: fp32, groups of eight or four rows");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if constexpr (SC) {
    for (int i = threadIdx.x; i < (kT / 64) * RB; i += kT) rmx[i / RB][i % RB] = 0.f;
  }
  const E *H = static_cast<const E *>(Hv);
  E *dH = static_cast<E *>(dHv);
  const int64_t r0 = (int64_t)blockIdx.x * RB;
  const int64_t r1 = r0 + RB < M ? r0 + RB : M;
  if (threadIdx.x < RB) {
    const int64_t m = r0 + threadIdx.x;
    float gv[4] = {0.f, 0.f, 0.f, 0.f};
    if (m < r1) {
#pragma unroll
      for (int c = 0; c < N; ++c) gv[c] = G[m * ldg + c];
    }
    sg4[threadIdx.x] = make_float4(gv[0], gv[1], gv[2], gv[3]);
  }
  __syncthreads();
  const int64_t tot = N * K + N;
  float *pw = part + (int64_t)blockIdx.x * tot;  // [N][K], db[N]
  const int nfull = (int)((r1 - r0) / CH), nch = (int)((r1 - r0 + CH - 1) / CH);
  for (int64_t k = (int64_t)threadIdx.x * EPT; k < K; k += kT * EPT) {
    lpg_f32x2 w[N][P], acc[N][P], cs[P];
#pragma unroll
    for (int c = 0; c < N; ++c) {
#pragma unroll
      for (int q = 0; q < P; q += 2) {
        const float4 wv = *reinterpret_cast<const float4 *>(W + c * K + k + 2 * q);
        w[c][q] = lpg_f32x2{wv.x, wv.y};
        w[c][q + 1] = lpg_f32x2{wv.z, wv.w};
      }
#pragma unroll
      for (int q = 0; q < P; ++q) acc[c][q] = lpg_f32x2{0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < P; ++q) cs[q] = lpg_f32x2{0.f, 0.f};
    H16<BF> hA[U], hB[U];  // two register buffers: group g + 1 loading while group g is processed
    auto issue = [&](H16<BF>(&hb)[U], int64_t m0) {  // rows past r1: clamped, never used
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t m = m0 + u < r1 ? m0 + u : r1 - 1;
        hb[u] = *reinterpret_cast<const H16<BF> *>(H + m * ldh + k);
      }
    };
    lpg_f32x2 cmx[P];  // SC: the thread's column maxima of |dH| over the block's rows
#pragma unroll
    for (int q = 0; q < P; ++q) cmx[q] = lpg_f32x2{0.f, 0.f};
    auto row = [&](H16<BF> hv, int64_t m) -> float {
      lpg_f32x2 h[P];
      uint32_t hw[4] = {0u, 0u, 0u, 0u};
      if constexpr (BF) {
        hw[0] = hv.x; hw[1] = hv.y; hw[2] = hv.z; hw[3] = hv.w;
#pragma unroll
        for (int q = 0; q < P; ++q) h[q] = lpg_f32x2{__uint_as_float(hw[q] << 16), __uint_as_float(hw[q] & 0xffff0000u)};
      } else {
        h[0] = lpg_f32x2{hv.x, hv.y};
        h[1] = lpg_f32x2{hv.z, hv.w};
      }
      const float4 g4 = sg4[m - r0];
      const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
      lpg_f32x2 d[P];
#pragma unroll
      for (int q = 0; q < P; ++q) d[q] = lpg_f32x2{0.f, 0.f};
#pragma unroll
      for (int c = 0; c < N; ++c) {
        const lpg_f32x2 gc = {gv[c], gv[c]};
#pragma unroll
        for (int q = 0; q < P; ++q) {
          d[q] = __builtin_elementwise_fma(gc, w[c][q], d[q]);
          acc[c][q] = __builtin_elementwise_fma(gc, h[q], acc[c][q]);
        }
      }
      if constexpr (BF) {
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < P; ++q) {
          o[q] = pk_bf16(d[q][0], d[q][1]);
          if (MASK) o[q] = relu_bwd_pk_bf16(o[q], hw[q], scale);
          cs[q] = cs[q] + lpg_f32x2{__uint_as_float(o[q] << 16), __uint_as_float(o[q] & 0xffff0000u)};
        }
        if (STORE) *reinterpret_cast<uint4 *>(dH + m * lddh + k) = make_uint4(o[0], o[1], o[2], o[3]);
      } else {
        float o[4] = {d[0][0], d[0][1], d[1][0], d[1][1]};
        const float hv4[4] = {h[0][0], h[0][1], h[1][0], h[1][1]};
        if (MASK) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = hv4[e] > 0.f ? o[e] * scale : 0.f;
        }
        cs[0] = cs[0] + lpg_f32x2{o[0], o[1]};
        cs[1] = cs[1] + lpg_f32x2{o[2], o[3]};
        if (STORE) *reinterpret_cast<float4 *>(dH + m * lddh + k) = make_float4(o[0], o[1], o[2], o[3]);
        if constexpr (SC) {
          const float a0 = fabsf(o[0]), a1 = fabsf(o[1]), a2 = fabsf(o[2]), a3 = fabsf(o[3]);
          cmx[0] = lpg_f32x2{fmaxf(cmx[0][0], a0), fmaxf(cmx[0][1], a1)};
          cmx[1] = lpg_f32x2{fmaxf(cmx[1][0], a2), fmaxf(cmx[1][1], a3)};
          return fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
        }
      }
      return 0.f;
    };
    // SC: eight rows' lane maxima -> the rows' wave maxima (rows m0 .. m0 + 7 of the block) into rmx
    auto rows8 = [&](const float (&x)[8], int64_t m0) {
      if constexpr (SC) {
        const float w = rowmax8(x, lane);
        const int r = (int)(m0 - r0) + rowmax8_slot(lane);
        if ((lane & 7) == 0 && r < RB) rmx[wv][r] = fmaxf(rmx[wv][r], w);
      }
    };
    auto flush = [&](int ch) {  // the chunk's column sums into relu_bwd_colsum's partial image
      if (party) {
        float *py = party + (r0 / CH + ch) * K + k;
#pragma unroll
        for (int q = 0; q < P; q += 2)
          *reinterpret_cast<float4 *>(py + 2 * q) = make_float4(cs[q][0], cs[q][1], cs[q + 1][0], cs[q + 1][1]);
      }
#pragma unroll
      for (int q = 0; q < P; ++q) cs[q] = lpg_f32x2{0.f, 0.f};
    };
    issue(hA, r0);
    for (int ch = 0; ch < nfull; ++ch) {  // whole chunks: branch-free, one group always in flight
      const int64_t cb = r0 + (int64_t)ch * CH;
      for (int j = 0; j < CH / (2 * U); ++j) {
        issue(hB, cb + (2 * j + 1) * U);
        __builtin_amdgcn_sched_barrier(0);
        float xm[8];  // (SC) the eight rows' lane maxima: one group of eight, or the two groups of four
        if constexpr (SC) {
#pragma unroll
          for (int u = 0; u < U; ++u) xm[u] = row(hA[u], cb + 2 * j * U + u);
          if constexpr (U == 8) rows8(xm, cb + 2 * j * U);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u) row(hA[u], cb + 2 * j * U + u);
        }
        issue(hA, cb + (2 * j + 2) * U);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SC) {
#pragma unroll
          for (int u = 0; u < U; ++u) xm[(U == 4 ? 4 : 0) + u] = row(hB[u], cb + (2 * j + 1) * U + u);
          rows8(xm, cb + (U == 4 ? 2 * j : 2 * j + 1) * U);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u) row(hB[u], cb + (2 * j + 1) * U + u);
        }
      }
      flush(ch);
    }
    if (nfull < nch) {  // the partial last chunk, row by row (hA holds its first group)
      const int64_t cb = r0 + (int64_t)nfull * CH;
      for (int64_t m0 = cb; m0 < r1; m0 += (SC ? 8 : U)) {
        if (m0 != cb) issue(hA, m0);
        if constexpr (SC) {
          float xm[8];
#pragma unroll
          for (int u = 0; u < U; ++u) xm[u] = m0 + u < r1 ? row(hA[u], m0 + u) : 0.f;
          if constexpr (U == 4) {  // the second group of four
            issue(hB, m0 + 4);
#pragma unroll
            for (int u = 0; u < 4; ++u) xm[4 + u] = m0 + 4 + u < r1 ? row(hB[u], m0 + 4 + u) : 0.f;
          }
          rows8(xm, m0);
        } else {
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (m0 + u < r1) row(hA[u], m0 + u);
        }
      }
      flush(nfull);
    }
#pragma unroll
    for (int c = 0; c < N; ++c)
#pragma unroll
      for (int q = 0; q < P; q += 2)
        *reinterpret_cast<float4 *>(pw + c * K + k + 2 * q) =
            make_float4(acc[c][q][0], acc[c][q][1], acc[c][q + 1][0], acc[c][q + 1][1]);
    if constexpr (SC)
      *reinterpret_cast<float4 *>(cpart + (int64_t)blockIdx.x * K + k) = make_float4(cmx[0][0], cmx[0][1], cmx[1][0], cmx[1][1]);
  }
  if constexpr (SC) {  // the rows' maxima over the four waves (and every k pass): the row scales
    __syncthreads();
    if (threadIdx.x < RB && r0 + threadIdx.x < r1) {
      float mx = rmx[0][threadIdx.x];
#pragma unroll
      for (int w = 1; w < kT / 64; ++w) mx = fmaxf(mx, rmx[w][threadIdx.x]);
      rsc[r0 + threadIdx.x] = f16x2_scale(mx);
    }
  }
  if (threadIdx.x == 0) {  // db = sum_m G[m, c] in row order
    float sg[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t m = r0; m < r1; ++m) {
      const float4 g4 = sg4[m - r0];
      sg[0] = sg[0] + g4.x; sg[1] = sg[1] + g4.y; sg[2] = sg[2] + g4.z; sg[3] = sg[3] + g4.w;
    }
#pragma unroll
    for (int c = 0; c < N; ++c) pw[N * K + c] = sg[c];
  }
}

__global__ __launch_bounds__(kT) void linear_small_bwd_p2(int64_t nrow, int64_t K, int N, int64_t tot,
                                                          const float *__restrict__ img, float *__restrict__ dW,
                                                          float *__restrict__ db, float *__restrict__ dbY) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;  // over N*K + N (+ K)
  if (i >= tot) return;
  const float s = sum_rows(nrow, tot, img, i);
  if (i < (int64_t)N * K) {
    if (dW) dW[i] = s;
  } else if (i < (int64_t)N * K + N) {
    if (db) db[i - (int64_t)N * K] = s;
  } else if (dbY) {
    dbY[i - (int64_t)N * K - N] = s;
  }
}

// ---- bf16 (c5) narrow kernels: conv1's weight gradients and the heads (N = 3) ----------------


// The heads' forward in bf16 (c5): out[m, c] = RNE_bf16(sum_k H[m, k] W[c, k] + b[c]) for N <= 4,
// one streaming pass over H.  A wave takes RW rows at a time; lane l holds the 8-column chunks
// l, l + 64, ... (KC of them; their weights stay in registers), sums its products per (row, c),
// then a butterfly over the 64 lanes.  The MFMA kernel on N padded to 64 (0.36 ms per c5 step)
// sums the same exact bf16 x bf16 products in another order: tolerance, not bits.
constexpr int kRowsPerWaveFwd = 4;

// F16: fp16 storage of H and out (the reference's --fp16 inference, val.py:269), same sums.
__device__ __forceinline__ float f16_to_f32(uint32_t h) { return (float)__builtin_bit_cast(_Float16, (uint16_t)h); }

template <bool F16, int N, int KC>
__global__ __launch_bounds__(256) void linear_small_fwd_bf16(int64_t M, int64_t K, const uint16_t *__restrict__ H,
                                                             int64_t ldh, const float *__restrict__ W,
                                                             const float *__restrict__ bias,
                                                             uint16_t *__restrict__ out, int64_t ldo) {
  constexpr int RW = kRowsPerWaveFwd;
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nwave = (int64_t)gridDim.x * 4;
  float w[KC][N][8];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) {
    const int64_t k = (int64_t)kc * 512 + lane * 8;
#pragma unroll
    for (int c = 0; c < N; ++c) {
      float4 w0 = make_float4(0.f, 0.f, 0.f, 0.f), w1 = w0;
      if (k < K) {
        w0 = *reinterpret_cast<const float4 *>(W + c * K + k);
        w1 = *reinterpret_cast<const float4 *>(W + c * K + k + 4);
      }
      w[kc][c][0] = w0.x; w[kc][c][1] = w0.y; w[kc][c][2] = w0.z; w[kc][c][3] = w0.w;
      w[kc][c][4] = w1.x; w[kc][c][5] = w1.y; w[kc][c][6] = w1.z; w[kc][c][7] = w1.w;
    }
  }
  float b[N];
#pragma unroll
  for (int c = 0; c < N; ++c) b[c] = bias ? bias[c] : 0.f;
  for (int64_t m0 = wave * RW; m0 < M; m0 += nwave * RW) {
    uint4 hv[RW][KC];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int64_t m = m0 + r < M ? m0 + r : M - 1;  // clamped rows are never stored
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const int64_t k = (int64_t)kc * 512 + lane * 8;
        hv[r][kc] = k < K ? *reinterpret_cast<const uint4 *>(H + m * ldh + k) : make_uint4(0u, 0u, 0u, 0u);
      }
    }
    float p[RW][N];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
#pragma unroll
      for (int c = 0; c < N; ++c) p[r][c] = 0.f;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const uint32_t hw[4] = {hv[r][kc].x, hv[r][kc].y, hv[r][kc].z, hv[r][kc].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float h0 = F16 ? f16_to_f32(hw[e] & 0xffffu) : bf16_to_f32(hw[e] & 0xffffu);
          const float h1 = F16 ? f16_to_f32(hw[e] >> 16) : bf16_to_f32(hw[e] >> 16);
#pragma unroll
          for (int c = 0; c < N; ++c)
            p[r][c] = __builtin_fmaf(h1, w[kc][c][2 * e + 1], __builtin_fmaf(h0, w[kc][c][2 * e], p[r][c]));
        }
      }
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1)
#pragma unroll
      for (int r = 0; r < RW; ++r)
#pragma unroll
        for (int c = 0; c < N; ++c) p[r][c] = p[r][c] + __shfl_xor(p[r][c], s, 64);
#pragma unroll
    for (int r = 0; r < RW; ++r)
#pragma unroll
      for (int c = 0; c < N; ++c)
        if (lane == r * N + c && m0 + r < M)
          out[(m0 + r) * ldo + c] = F16 ? __builtin_bit_cast(uint16_t, (_Float16)(p[r][c] + b[c]))
                                        : (uint16_t)pk_bf16(p[r][c] + b[c], 0.f);
  }
}

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" int64_t lpg_relu_bwd_colsum_workspace_bytes(int64_t M, int64_t N) {
  if (M < 0 || N < 0) return -1;
  return fold_floats((M + kRowsColsum - 1) / kRowsColsum, N) * (int64_t)sizeof(float);
}

extern "C" lpg_status lpg_relu_bwd_colsum_f32(int64_t M, int64_t N, const float *g, int64_t ldg, const float *y,
                                              int64_t ldy, float scale, float *out, int64_t ldo, float *db,
                                              void *workspace, void *stream) {
  LPG_REQUIRE(M >= 0 && N >= 0, "lpg_relu_bwd_colsum_f32: negative size");
  if (M == 0 || N == 0) {
    if (db && N > 0) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, as_stream(stream)));
    return LPG_OK;
  }
  LPG_REQUIRE(g && y && out, "lpg_relu_bwd_colsum_f32: NULL pointer");
  LPG_REQUIRE(N % 4 == 0 && ldg % 4 == 0 && ldy % 4 == 0 && ldo % 4 == 0 && aligned16(g) && aligned16(y) &&
                  aligned16(out),
              "lpg_relu_bwd_colsum_f32: N / leading dims must be multiples of 4, buffers 16-byte aligned");
  LPG_REQUIRE(db == nullptr || (workspace && aligned16(workspace)), "lpg_relu_bwd_colsum_f32: db needs a workspace");
  hipStream_t s = as_stream(stream);
  const int64_t nblk = (M + kRowsColsum - 1) / kRowsColsum;
  float *part = db ? static_cast<float *>(workspace) : nullptr;
  hipLaunchKernelGGL(relu_bwd_colsum_p1, dim3((unsigned)nblk), dim3(kT), 0, s, M, N, g, ldg, y, ldy, scale, out, ldo,
                     part);
  LPG_HIP(hipGetLastError());
  if (db) {
    const float *img;
    const int64_t nrow = fold(nblk, N, part, part + nblk * N, &img, s);
    hipLaunchKernelGGL(sum_partials, dim3((unsigned)((N + kT - 1) / kT)), dim3(kT), 0, s, nrow, N, img, db);
    LPG_HIP(hipGetLastError());
  }
  return LPG_OK;
}

extern "C" lpg_status lpg_relu_bwd_colsum_bf16(int64_t M, int64_t N, const uint16_t *g, int64_t ldg, const uint16_t *y,
                                               int64_t ldy, float scale, uint16_t *out, int64_t ldo, float *db,
                                               void *workspace, void *stream) {
  LPG_REQUIRE(M >= 0 && N >= 0, "lpg_relu_bwd_colsum_bf16: negative size");
  if (M == 0 || N == 0) {
    if (db && N > 0) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, as_stream(stream)));
    return LPG_OK;
  }
  LPG_REQUIRE(g && y && out, "lpg_relu_bwd_colsum_bf16: NULL pointer");
  LPG_REQUIRE(N % 8 == 0 && ldg % 8 == 0 && ldy % 8 == 0 && ldo % 8 == 0 && aligned16(g) && aligned16(y) &&
                  aligned16(out),
              "lpg_relu_bwd_colsum_bf16: N / leading dims must be multiples of 8, buffers 16-byte aligned");
  LPG_REQUIRE(db == nullptr || (workspace && aligned16(workspace)), "lpg_relu_bwd_colsum_bf16: db needs a workspace");
  hipStream_t s = as_stream(stream);
  const int64_t nblk = (M + kRowsColsum - 1) / kRowsColsum;
  float *part = db ? static_cast<float *>(workspace) : nullptr;
  hipLaunchKernelGGL(relu_bwd_colsum_bf16_p1<true>, dim3((unsigned)nblk), dim3(kT), 0, s, M, N, g, ldg, y, ldy, scale,
                     out, ldo, part);
  LPG_HIP(hipGetLastError());
  if (db) {
    const float *img;
    const int64_t nrow = fold(nblk, N, part, part + nblk * N, &img, s);
    hipLaunchKernelGGL(sum_partials, dim3((unsigned)((N + kT - 1) / kT)), dim3(kT), 0, s, nrow, N, img, db);
    LPG_HIP(hipGetLastError());
  }
  return LPG_OK;
}

// db = column sums of a bf16 dZ that already went through its ReLU / dropout backward (the
// folded form, lpg_fc_bf16_relu_bwd): the blocks, partials and fold of lpg_relu_bwd_colsum_bf16,
// so db is bitwise what that kernel returns for the same dZ.  Workspace:
// lpg_relu_bwd_colsum_workspace_bytes(M, N).
extern "C" lpg_status lpg_colsum_bf16(int64_t M, int64_t N, const uint16_t *g, int64_t ldg, float *db,
                                      void *workspace, void *stream) {
  LPG_REQUIRE(M >= 0 && N >= 0, "lpg_colsum_bf16: negative size");
  LPG_REQUIRE(db != nullptr || N == 0, "lpg_colsum_bf16: NULL db");
  if (M == 0 || N == 0) {
    if (N > 0) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, as_stream(stream)));
    return LPG_OK;
  }
  LPG_REQUIRE(g && workspace && aligned16(workspace), "lpg_colsum_bf16: NULL pointer or unaligned workspace");
  LPG_REQUIRE(N % 8 == 0 && ldg % 8 == 0 && aligned16(g),
              "lpg_colsum_bf16: N / ldg must be multiples of 8, g 16-byte aligned");
  hipStream_t s = as_stream(stream);
  const int64_t nblk = (M + kRowsColsum - 1) / kRowsColsum;
  float *part = static_cast<float *>(workspace);
  hipLaunchKernelGGL(relu_bwd_colsum_bf16_p1<false>, dim3((unsigned)nblk), dim3(kT), 0, s, M, N, g, ldg,
                     (const uint16_t *)nullptr, (int64_t)0, 1.f, (uint16_t *)nullptr, (int64_t)0, part);
  LPG_HIP(hipGetLastError());
  const float *img;
  const int64_t nrow = fold(nblk, N, part, part + nblk * N, &img, s);
  hipLaunchKernelGGL(sum_partials, dim3((unsigned)((N + kT - 1) / kT)), dim3(kT), 0, s, nrow, N, img, db);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

namespace lpg {
namespace {

// wgrad_smallk_p1's row ranges: the resident blocks shared by the column groups, at least one
// chunk of rows each and at most kWgSplits (the partial image [S][K + 1][N]; the workspace is
// sized for the most a launch can use)
constexpr int64_t kWgSplits = 512;
int64_t wgrad_smallk_splits(int64_t M) {
  const int64_t s = (M + kChunk - 1) / kChunk;
  return s < 1 ? 1 : (s > kWgSplits ? kWgSplits : s);
}

template <bool BF>
lpg_status wgrad_smallk(int64_t M, int64_t N, const void *dz, int64_t ldz, const void *y, int64_t ldy, float scale,
                        int64_t K1, const void *A1, int64_t lda1, int64_t K2, const void *A2, int64_t lda2,
                        float *dW1, float *dW2, float *db, void *workspace, void *stream, const char *name) {
  const int64_t K = K1 + K2;
  const bool mask = y != nullptr;
  const uintptr_t al = BF ? 7 : 15;  // 4 gradient values per load: 8 B (bf16) / 16 B (fp32)
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0 && K >= 1 && K <= kMaxSmallK, "%s: need 1 <= K1 + K2 <= %d",
              name, kMaxSmallK);
  LPG_REQUIRE(dz && workspace && (K1 == 0 || A1) && (K2 == 0 || A2), "%s: NULL pointer", name);
  LPG_REQUIRE((K1 == 0 || lda1 >= K1) && (K2 == 0 || lda2 >= K2), "%s: bad lda", name);
  LPG_REQUIRE(N % 4 == 0 && ldz % 4 == 0 && (reinterpret_cast<uintptr_t>(dz) & al) == 0 && aligned16(workspace) &&
                  (!mask || (ldy % 4 == 0 && (reinterpret_cast<uintptr_t>(y) & al) == 0)),
              "%s: N / leading dims multiples of 4, gradient / output aligned to 4 elements, workspace 16-byte aligned",
              name);
  hipStream_t s = as_stream(stream);
  if (M == 0 || N == 0) {
    if (dW1 && N * K1) LPG_HIP(hipMemsetAsync(dW1, 0, sizeof(float) * N * K1, s));
    if (dW2 && N * K2) LPG_HIP(hipMemsetAsync(dW2, 0, sizeof(float) * N * K2, s));
    if (db && N) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, s));
    return LPG_OK;
  }
  const int64_t KR = K + 1;
  float *part = static_cast<float *>(workspace);
  const int k1 = (int)K1;
  const int64_t ncg = (N + kT * 4 - 1) / (kT * 4);
  LPG_REQUIRE(ncg < 65536, "%s: N too large", name);
  auto splits = [&](auto kern) {
    const int64_t r = resident_blocks(kern, kT) / ncg, smax = wgrad_smallk_splits(M);
    return r < 1 ? (int64_t)1 : (r < smax ? r : smax);
  };
  int64_t S = 1;
  switch (K * 2 + (mask ? 1 : 0)) {
#define LPG_WG(KK)                                                                                      \
  case 2 * KK:                                                                                          \
    S = splits(wgrad_smallk_p1<KK, false, BF>);                                                         \
    hipLaunchKernelGGL((wgrad_smallk_p1<KK, false, BF>), dim3((unsigned)ncg, (unsigned)S), dim3(kT), 0, s, M, N, \
                       dz, ldz, y, ldy, scale, k1, A1, lda1, A2, lda2, S, part);                       \
    break;                                                                                              \
  case 2 * KK + 1:                                                                                      \
    S = splits(wgrad_smallk_p1<KK, true, BF>);                                                          \
    hipLaunchKernelGGL((wgrad_smallk_p1<KK, true, BF>), dim3((unsigned)ncg, (unsigned)S), dim3(kT), 0, s, M, N,  \
                       dz, ldz, y, ldy, scale, k1, A1, lda1, A2, lda2, S, part);                       \
    break;
    LPG_WG(1) LPG_WG(2) LPG_WG(3) LPG_WG(4) LPG_WG(5) LPG_WG(6) LPG_WG(7) LPG_WG(8)
    LPG_WG(9) LPG_WG(10) LPG_WG(11) LPG_WG(12) LPG_WG(13) LPG_WG(14) LPG_WG(15) LPG_WG(16)
#undef LPG_WG
  }
  LPG_HIP(hipGetLastError());
  const float *img;
  const int64_t nrow = fold(S, KR * N, part, part + S * KR * N, &img, s);
  hipLaunchKernelGGL(wgrad_smallk_p2, dim3((unsigned)((KR * N + kT - 1) / kT)), dim3(kT), 0, s, nrow, N, (int)K,
                     (int)KR, k1, img, dW1, dW2, db);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

}  // namespace

// The fold of a small-K weight-gradient partial image [nblk][K + 1][N] (rows = blocks of rows) into
// dW1 [N, K1], dW2 [N, K - K1], db [N] in block order -- wgrad_smallk's tail, shared with the x3 FC's
// fused conv1 weight gradient (fc_x3.hip, lpg_fc_x3_relu_wgrad_f32).  seg: smallk_fold_floats floats
// after part (the segment sums).
int64_t smallk_fold_floats(int64_t nblk, int64_t KR, int64_t N) { return fold_floats(nblk, KR * N); }

lpg_status smallk_fold(int64_t nblk, int64_t N, int K1, int K, const float *part, float *seg, float *dW1, float *dW2,
                       float *db, hipStream_t s) {
  const int64_t KR = K + 1;
  const float *img;
  const int64_t nrow = fold(nblk, KR * N, part, seg, &img, s);
  hipLaunchKernelGGL(wgrad_smallk_p2, dim3((unsigned)((KR * N + kT - 1) / kT)), dim3(kT), 0, s, nrow, N, K, (int)KR,
                     K1, img, dW1, dW2, db);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// db of a bf16 dZ [M, N] whose partial image [ceil(M / 64)][N] (lpg_colsum_bf16's, in `part`, the
// workspace of lpg_relu_bwd_colsum_workspace_bytes) a producer already filled for rows [0, r0) --
// the folded ReLU backward of fc_bf16_p (fc_bf16.hip) -- rows [r0, M) summed here from g by
// relu_bwd_colsum_bf16_p1 (r0 a multiple of the 64-row chunk), then lpg_colsum_bf16's fold: db is
// bitwise what lpg_colsum_bf16 returns for the same dZ.
lpg_status colsum_bf16_from(int64_t M, int64_t N, const uint16_t *g, int64_t ldg, int64_t r0, float *part, float *db,
                            hipStream_t s) {
  LPG_REQUIRE(r0 >= 0 && r0 <= M && (r0 % kRowsColsum == 0 || r0 == M), "colsum_bf16_from: bad r0 %lld",
              (long long)r0);
  const int64_t nblk = (M + kRowsColsum - 1) / kRowsColsum;
  if (r0 < M) {
    const int64_t b0 = r0 / kRowsColsum;
    hipLaunchKernelGGL(relu_bwd_colsum_bf16_p1<false>, dim3((unsigned)(nblk - b0)), dim3(kT), 0, s, M - r0, N,
                       g + r0 * ldg, ldg, (const uint16_t *)nullptr, (int64_t)0, 1.f, (uint16_t *)nullptr, (int64_t)0,
                       part + b0 * N);
    LPG_HIP(hipGetLastError());
  }
  const float *img;
  const int64_t nrow = fold(nblk, N, part, part + nblk * N, &img, s);
  hipLaunchKernelGGL(sum_partials, dim3((unsigned)((N + kT - 1) / kT)), dim3(kT), 0, s, nrow, N, img, db);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

namespace {
int64_t heads_bwd_floats(int64_t M, int64_t K, int64_t N) {
  const int64_t nblk = (M + kRowsLinear - 1) / kRowsLinear, nchunk = (M + kRowsColsum - 1) / kRowsColsum;
  return fold_floats(nblk, N * K + N) + fold_floats(nchunk, K);
}

// The heads' backward (heads_bwd_p1) for both dtypes: dW / db through the [nblk][N K + N] image,
// dbY through relu_bwd_colsum's [ceil(M / 64)][K] image and its fold + final pass.
template <bool BF>
lpg_status heads_bwd(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg, const float *W, const void *H,
                     int64_t ldh, void *dH, int64_t lddh, float scale, float *dW, float *db, float *dbY, bool mask,
                     void *workspace, void *stream, const char *what, float *rscale = nullptr,
                     float *cscale = nullptr, float *cpart = nullptr) {
  constexpr int EPT = BF ? 8 : 4;
  LPG_REQUIRE(M >= 0 && K >= 0 && N >= 1 && N <= kSmallNMax, "%s: need 1 <= N <= %d", what, kSmallNMax);
  LPG_REQUIRE(K % EPT == 0 && ldh % EPT == 0 && (dH == nullptr || lddh % EPT == 0) && ldg >= N,
              "%s: K and leading dims must be multiples of %d", what, EPT);
  LPG_REQUIRE(G && W && H && workspace && (dH || !mask), "%s: NULL pointer", what);
  LPG_REQUIRE(aligned16(W) && aligned16(H) && (dH == nullptr || aligned16(dH)) && aligned16(workspace),
              "%s: W/H/dH/workspace must be 16-byte aligned", what);
  hipStream_t s = as_stream(stream);
  const int64_t nblk = (M + kRowsLinear - 1) / kRowsLinear, nchunk = (M + kRowsColsum - 1) / kRowsColsum;
  if (nblk == 0 || K == 0) {
    if (dW && N * K) LPG_HIP(hipMemsetAsync(dW, 0, sizeof(float) * N * K, s));
    if (dbY && K) LPG_HIP(hipMemsetAsync(dbY, 0, sizeof(float) * K, s));
    if (nblk == 0) {
      if (db) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, s));
      return LPG_OK;
    }
  }
  LPG_REQUIRE(nblk < ((int64_t)1 << 31), "%s: too many rows", what);
  const int64_t tot = N * K + N;
  float *part = static_cast<float *>(workspace);
  float *party = part + fold_floats(nblk, tot);
  float *py = dbY ? party : nullptr;
  const dim3 grid((unsigned)nblk), block(kT);
  const bool sc = rscale != nullptr;
  if (sc) {
    LPG_REQUIRE(!BF && mask && cscale && cpart && aligned16(cpart) && K % 4 == 0,
                "%s: the f16x2 scales need the fp32 masked form, cscale and a 16-byte aligned partial buffer", what);
  }
#define LPG_HB(NN)                                                                                                \
  if (sc && !BF)                                                                                                  \
    hipLaunchKernelGGL((heads_bwd_p1<NN, true, false, true, true>), grid, block, 0, s, M, K, G, ldg, W, H, ldh, dH,  \
                       lddh, scale, part, py, rscale, cpart);                                                     \
  else if (mask)                                                                                                  \
    hipLaunchKernelGGL((heads_bwd_p1<NN, true, BF, true>), grid, block, 0, s, M, K, G, ldg, W, H, ldh, dH, lddh,   \
                       scale, part, py);                                                                          \
  else if (dH)                                                                                                    \
    hipLaunchKernelGGL((heads_bwd_p1<NN, false, BF, true>), grid, block, 0, s, M, K, G, ldg, W, H, ldh, dH, lddh,  \
                       scale, part, py);                                                                          \
  else                                                                                                            \
    hipLaunchKernelGGL((heads_bwd_p1<NN, false, BF, false>), grid, block, 0, s, M, K, G, ldg, W, H, ldh, dH, lddh, \
                       scale, part, py);
  switch (N) {
    case 1: LPG_HB(1) break;
    case 2: LPG_HB(2) break;
    case 3: LPG_HB(3) break;
    default: LPG_HB(4)
  }
#undef LPG_HB
  LPG_HIP(hipGetLastError());
  if (sc) {
    hipLaunchKernelGGL(colfold_f32, dim3((unsigned)((K + 63) / 64)), dim3(256), 0, s, nblk, K, cpart, cscale);
    LPG_HIP(hipGetLastError());
  }
  const float *img;
  const int64_t nrow = fold(nblk, tot, part, part + nblk * tot, &img, s);
  hipLaunchKernelGGL(linear_small_bwd_p2, dim3((unsigned)((tot + kT - 1) / kT)), dim3(kT), 0, s, nrow, K, (int)N, tot,
                     img, dW, db, (float *)nullptr);
  LPG_HIP(hipGetLastError());
  if (dbY && K) {  // the fold and final pass of relu_bwd_colsum over the same 64-row partials
    const float *imy;
    const int64_t nry = fold(nchunk, K, party, party + nchunk * K, &imy, s);
    hipLaunchKernelGGL(sum_partials, dim3((unsigned)((K + kT - 1) / kT)), dim3(kT), 0, s, nry, K, imy, dbY);
    LPG_HIP(hipGetLastError());
  }
  return LPG_OK;
}

}  // namespace
}  // namespace lpg

extern "C" int64_t lpg_wgrad_smallk_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return -1;
  return fold_floats(wgrad_smallk_splits(M), (K + 1) * N) * (int64_t)sizeof(float);
}

extern "C" lpg_status lpg_wgrad_smallk_f32(int64_t M, int64_t N, const float *dz, int64_t ldz, int64_t K1,
                                           const float *A1, int64_t lda1, int64_t K2, const float *A2, int64_t lda2,
                                           float *dW1, float *dW2, void *workspace, void *stream) {
  return wgrad_smallk<false>(M, N, dz, ldz, nullptr, 0, 1.f, K1, A1, lda1, K2, A2, lda2, dW1, dW2, nullptr, workspace,
                             stream, "lpg_wgrad_smallk_f32");
}

extern "C" lpg_status lpg_relu_wgrad_smallk_f32(int64_t M, int64_t N, const float *g, int64_t ldg, const float *y,
                                                int64_t ldy, float scale, int64_t K1, const float *A1, int64_t lda1,
                                                int64_t K2, const float *A2, int64_t lda2, float *dW1, float *dW2,
                                                float *db, void *workspace, void *stream) {
  LPG_REQUIRE(y != nullptr, "lpg_relu_wgrad_smallk_f32: NULL output");
  return wgrad_smallk<false>(M, N, g, ldg, y, ldy, scale, K1, A1, lda1, K2, A2, lda2, dW1, dW2, db, workspace, stream,
                             "lpg_relu_wgrad_smallk_f32");
}

// conv1's weight gradients in bf16 from one read of the gradient: dW1 = dZ^T A1, dW2 = dZ^T A2,
// db = sum_m dZ (fp32 out).  y == NULL: g already is dZ (the folded ReLU backward of the next
// layer's input gradient); else dZ = (y > 0) ? RNE_bf16(g * scale) : 0 on the fly (never stored).
// Workspace: lpg_wgrad_smallk_workspace_bytes(M, N, K1 + K2).
extern "C" lpg_status lpg_relu_wgrad_smallk_bf16(int64_t M, int64_t N, const uint16_t *g, int64_t ldg,
                                                 const uint16_t *y, int64_t ldy, float scale, int64_t K1,
                                                 const uint16_t *A1, int64_t lda1, int64_t K2, const uint16_t *A2,
                                                 int64_t lda2, float *dW1, float *dW2, float *db, void *workspace,
                                                 void *stream) {
  return wgrad_smallk<true>(M, N, g, ldg, y, ldy, scale, K1, A1, lda1, K2, A2, lda2, dW1, dW2, db, workspace, stream,
                            "lpg_relu_wgrad_smallk_bf16");
}

extern "C" int64_t lpg_linear_small_bwd_workspace_bytes(int64_t M, int64_t K, int64_t N) {
  if (M < 0 || K < 0 || N < 0) return -1;
  return heads_bwd_floats(M, K, N) * (int64_t)sizeof(float);
}

extern "C" lpg_status lpg_linear_small_bwd_f32(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg,
                                               const float *W, const float *H, int64_t ldh, float *dH, int64_t lddh,
                                               float *dW, float *db, void *workspace, void *stream) {
  return heads_bwd<false>(M, K, N, G, ldg, W, H, ldh, dH, lddh, 1.f, dW, db, nullptr, false, workspace, stream,
                          "lpg_linear_small_bwd_f32");
}

extern "C" lpg_status lpg_heads_relu_bwd_f32(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg,
                                             const float *W, const float *Y, int64_t ldy, float scale, float *dZ,
                                             int64_t lddz, float *dW, float *db, float *dbY, void *workspace,
                                             void *stream) {
  LPG_REQUIRE(dZ != nullptr, "lpg_heads_relu_bwd_f32: NULL dZ");
  return heads_bwd<false>(M, K, N, G, ldg, W, Y, ldy, dZ, lddz, scale, dW, db, dbY, true, workspace, stream,
                          "lpg_heads_relu_bwd_f32");
}

// lpg_heads_relu_bwd_f32 that also returns dZ's f16x2 scales (rscale [M], cscale [K]: the values
// lpg_rowcolscale_f32 gives on dZ) from the stores themselves; cpart: lpg_heads_scales_workspace_bytes.
extern "C" int64_t lpg_heads_scales_workspace_bytes(int64_t M, int64_t K) {
  if (M <= 0 || K <= 0) return 0;
  const int64_t own = ((M + kRowsLinear - 1) / kRowsLinear) * K * (int64_t)sizeof(float);
  const int64_t sweep = lpg_rowcolscale_workspace_bytes(M, K);  // (the K % 1024 != 0 route)
  return own > sweep ? own : sweep;
}

extern "C" lpg_status lpg_heads_relu_bwd_scales_f32(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg,
                                                    const float *W, const float *Y, int64_t ldy, float scale,
                                                    float *dZ, int64_t lddz, float *dW, float *db, float *dbY,
                                                    float *rscale, float *cscale, void *scale_ws, void *workspace,
                                                    void *stream) {
  LPG_REQUIRE(dZ != nullptr && rscale != nullptr, "lpg_heads_relu_bwd_scales_f32: NULL dZ / rscale");
  if (M == 0 || K == 0) {  // no rows: lpg_rowcolscale_f32's empty-operand scales
    const lpg_status st = heads_bwd<false>(M, K, N, G, ldg, W, Y, ldy, dZ, lddz, scale, dW, db, dbY, true, workspace,
                                           stream, "lpg_heads_relu_bwd_scales_f32");
    if (st != LPG_OK) return st;
    return lpg_rowcolscale_f32(M, K, nullptr, K, rscale, cscale, nullptr, stream);
  }
  if (K % (kT * 4) != 0) {  // a k pass with idle lanes cannot run the rows' butterfly: the pass, then a sweep
    const lpg_status st = heads_bwd<false>(M, K, N, G, ldg, W, Y, ldy, dZ, lddz, scale, dW, db, dbY, true, workspace,
                                           stream, "lpg_heads_relu_bwd_scales_f32");
    if (st != LPG_OK) return st;
    return lpg_rowcolscale_f32(M, K, dZ, lddz, rscale, cscale, scale_ws, stream);
  }
  return heads_bwd<false>(M, K, N, G, ldg, W, Y, ldy, dZ, lddz, scale, dW, db, dbY, true, workspace, stream,
                          "lpg_heads_relu_bwd_scales_f32", rscale, cscale, static_cast<float *>(scale_ws));
}

extern "C" int64_t lpg_heads_bwd_bf16_workspace_bytes(int64_t M, int64_t K, int64_t N) {
  if (M < 0 || K < 0 || N < 0) return -1;
  return heads_bwd_floats(M, K, N) * (int64_t)sizeof(float);
}

// The heads' backward in bf16 (G [M, N] and W [N, K] fp32 holding the bf16 model's values, H the
// layer output [M, K] bf16): dH (bf16; mask != 0: through the layer's ReLU/dropout backward, the
// layer's dZ), dW, db, and (dbY != NULL) the column sums of the stored dH -- bitwise
// lpg_colsum_bf16 on it.  Workspace: lpg_heads_bwd_bf16_workspace_bytes(M, K, N).
extern "C" lpg_status lpg_heads_bwd_bf16(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg, const float *W,
                                         const uint16_t *H, int64_t ldh, int32_t mask, float scale, uint16_t *dH,
                                         int64_t lddh, float *dW, float *db, float *dbY, void *workspace,
                                         void *stream) {
  LPG_REQUIRE(dH != nullptr, "lpg_heads_bwd_bf16: NULL dH");
  return heads_bwd<true>(M, K, N, G, ldg, W, H, ldh, dH, lddh, scale, dW, db, dbY, mask != 0, workspace, stream,
                         "lpg_heads_bwd_bf16");
}

// The heads' forward in bf16: out[m, c] = RNE_bf16(sum_k H[m, k] W[c, k] + bias[c]), N <= 4,
// K <= 2048 (W fp32 holding the bf16 model's values; out bf16 [M, N] with leading dim ldo).
template <bool F16>
static lpg_status linear_small_fwd16(const char *what, int64_t M, int64_t K, int64_t N, const uint16_t *H, int64_t ldh,
                                     const float *W, const float *bias, uint16_t *out, int64_t ldo, void *stream) {
  LPG_REQUIRE(M >= 0 && K >= 8 && K <= 2048 && K % 8 == 0 && N >= 1 && N <= kSmallNMax,
              "%s: need 1 <= N <= %d and 8 <= K <= 2048, K %% 8 == 0", what, kSmallNMax);
  if (M == 0) return LPG_OK;
  LPG_REQUIRE(H && W && out && ldh >= K && ldh % 8 == 0 && ldo >= N && aligned16(H) && aligned16(W),
              "%s: bad H/W/out (H, W 16-byte aligned, ldh a multiple of 8)", what);
  const int64_t waves = (M + kRowsPerWaveFwd - 1) / kRowsPerWaveFwd;
  int64_t blocks = (waves + 3) / 4;
  blocks = blocks < 4096 ? blocks : 4096;
  const int kc = (int)((K + 511) / 512);
  hipStream_t s = as_stream(stream);
#define LPG_LF(NN, KC) \
  hipLaunchKernelGGL((linear_small_fwd_bf16<F16, NN, KC>), dim3((unsigned)blocks), dim3(256), 0, s, M, K, H, ldh, W, bias, out, ldo)
#define LPG_LFN(NN)          \
  switch (kc) {              \
    case 1: LPG_LF(NN, 1); break; \
    case 2: LPG_LF(NN, 2); break; \
    case 3: LPG_LF(NN, 3); break; \
    default: LPG_LF(NN, 4);  \
  }
  switch (N) {
    case 1: LPG_LFN(1) break;
    case 2: LPG_LFN(2) break;
    case 3: LPG_LFN(3) break;
    default: LPG_LFN(4)
  }
#undef LPG_LFN
#undef LPG_LF
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_linear_small_fwd_bf16(int64_t M, int64_t K, int64_t N, const uint16_t *H, int64_t ldh,
                                                const float *W, const float *bias, uint16_t *out, int64_t ldo,
                                                void *stream) {
  return linear_small_fwd16<false>("lpg_linear_small_fwd_bf16", M, K, N, H, ldh, W, bias, out, ldo, stream);
}

// ... and with fp16 H / out (the --fp16 model's heads, lin_left / lin_right, arch.py:190): W, bias fp32 holding
// the fp16 model's values; out = RNE_fp16 of the fp32 sum + bias
extern "C" lpg_status lpg_linear_small_fwd_f16(int64_t M, int64_t K, int64_t N, const uint16_t *H, int64_t ldh,
                                               const float *W, const float *bias, uint16_t *out, int64_t ldo,
                                               void *stream) {
  return linear_small_fwd16<true>("lpg_linear_small_fwd_f16", M, K, N, H, ldh, W, bias, out, ldo, stream);
}
