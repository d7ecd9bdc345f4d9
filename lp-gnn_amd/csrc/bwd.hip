// Memory-bound pieces of the GraphConv / head backward (train.py:128 loss.backward()
// through arch.py:57-62, 182-191), fused so each large gradient is streamed once:
//
//   lpg_relu_bwd_colsum_f32   dZ = (Y > 0) ? dY * scale : 0   (ReLU + fused dropout backward)
//                             and db = sum_m dZ[m, :]          (lin_rel.bias grad) in the same pass
//   lpg_wgrad_smallk_f32      dW1 = dZ^T A1, dW2 = dZ^T A2 for small K (conv1: K1 = K2 = 8 LP features)
//   lpg_relu_wgrad_smallk_f32 the same from (g, y) with the ReLU/dropout backward and db fused (dZ never stored)
//   lpg_linear_small_bwd_f32  the heads' backward (N = 3 outputs): dH = G W, dW = G^T H, db = sum G
//
// All are row-block kernels: a block owns R consecutive rows and all columns
// (256 threads x float4 = 1024 columns per pass, rows unrolled by 4 so each
// thread keeps 4+ loads in flight), and writes one row of per-block partial
// sums.  The partials are then added in a fixed order -- a fold into
// kFold segment sums (many blocks, coalesced), then a short final pass --
// so results are deterministic run to run, with no atomics.
#include "common.h"
#include "fc_common.h"

#pragma clang fp contract(off)

namespace lpg {
namespace {

constexpr int kT = 256;
constexpr int kRowsColsum = 64;
#ifndef LPG_WGRAD_ROWS
#define LPG_WGRAD_ROWS 256
#endif
#ifndef LPG_WGRAD_UNROLL
#define LPG_WGRAD_UNROLL 8  // rows of dZ (or g, y) in flight per thread; 4 -> 8 measured 0.61 -> 0.36 ms at 200K rows
#endif
constexpr int kRowsWgrad = LPG_WGRAD_ROWS;
constexpr int kUnrollWgrad = LPG_WGRAD_UNROLL;
#ifndef LPG_LINEAR_UNROLL
#define LPG_LINEAR_UNROLL 4
#endif
#ifndef LPG_LINEAR_ROWS
#define LPG_LINEAR_ROWS 128
#endif
constexpr int kRowsLinear = LPG_LINEAR_ROWS;
constexpr int kUnrollLinear = LPG_LINEAR_UNROLL;
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

// part[b][k][n] = sum over the block's rows of A[m][k] * dZ[m][n], k < K = K1 + K2.
// The block's [A1 | A2] rows are staged once into LDS ([row][KP], zero-padded
// to KP = K rounded up to 4) and read back as broadcast b128 loads.  (Weight
// gradients carry no bitwise contract: fused multiply-adds, checked against
// fp64 within the summation bound.)  With MASK the kernel reads the output
// gradient g and the stored output y instead of dZ and applies the ReLU /
// dropout backward on the fly, dZ = (y > 0) ? g * scale : 0, adding a K-th
// partial row for the bias gradient -- conv1 (whose inputs need no gradient)
// never materialises dZ.
template <int K, bool MASK>
__global__ __launch_bounds__(kT) void wgrad_smallk_p1(int64_t M, int64_t N, const float *__restrict__ dz,
                                                      int64_t ldz, const float *__restrict__ y, int64_t ldy,
                                                      float scale, int K1, const float *__restrict__ A1,
                                                      int64_t lda1, const float *__restrict__ A2, int64_t lda2,
                                                      float *__restrict__ part) {
  constexpr int KP = (K + 3) / 4 * 4;
  constexpr int KR = K + (MASK ? 1 : 0);  // partial rows per block
  __shared__ float4 sa[kRowsWgrad * KP / 4];
  const int64_t r0 = (int64_t)blockIdx.x * kRowsWgrad;
  const int64_t r1 = r0 + kRowsWgrad < M ? r0 + kRowsWgrad : M;
  float *sf = reinterpret_cast<float *>(sa);
  for (int i = threadIdx.x; i < kRowsWgrad * KP; i += kT) {
    const int r = i / KP, k = i % KP;
    const int64_t m = r0 + r;
    float v = 0.f;
    if (m < r1 && k < K) v = k < K1 ? A1[m * lda1 + k] : A2[m * lda2 + (k - K1)];
    sf[i] = v;
  }
  __syncthreads();
  for (int64_t c = (int64_t)threadIdx.x * 4; c < N; c += kT * 4) {
    float4 acc[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    auto row = [&](int r, float4 z) {
      float a[KP];
#pragma unroll
      for (int q = 0; q < KP / 4; ++q) {
        const float4 v = sa[r * (KP / 4) + q];
        a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        acc[k].x = __builtin_fmaf(a[k], z.x, acc[k].x); acc[k].y = __builtin_fmaf(a[k], z.y, acc[k].y);
        acc[k].z = __builtin_fmaf(a[k], z.z, acc[k].z); acc[k].w = __builtin_fmaf(a[k], z.w, acc[k].w);
      }
      if (MASK) add4(acc[KR - 1], z);
    };
    auto load_z = [&](int64_t m) {
      const float4 g = *reinterpret_cast<const float4 *>(dz + m * ldz + c);
      if (!MASK) return g;
      return relu_scale(g, *reinterpret_cast<const float4 *>(y + m * ldy + c), scale);
    };
    const int nr = (int)(r1 - r0);
    int r = 0;
    for (; r + kUnrollWgrad <= nr; r += kUnrollWgrad) {
      float4 z[kUnrollWgrad];
#pragma unroll
      for (int u = 0; u < kUnrollWgrad; ++u) z[u] = load_z(r0 + r + u);
#pragma unroll
      for (int u = 0; u < kUnrollWgrad; ++u) row(r + u, z[u]);
    }
    for (; r < nr; ++r) row(r, load_z(r0 + r));
    float *pb = part + (int64_t)blockIdx.x * KR * N;
#pragma unroll
    for (int k = 0; k < KR; ++k) *reinterpret_cast<float4 *>(pb + k * N + c) = acc[k];
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

// Backward of a Linear with few outputs (the heads, N = 3, arch.py:190):
//   dH[m, k] = sum_c G[m, c] W[c, k]        (written if dH != NULL)
//   dW[c, k] = sum_m G[m, c] H[m, k],  db[c] = sum_m G[m, c]
// Pass 1 streams H once, writes dH and the block's partial [dW | db] row.
// MASK (lpg_heads_relu_bwd_f32): H is the output Y of the previous layer's
// ReLU (+ dropout), and the gradient leaves already through that layer's
// ReLU/dropout backward: dH[m, k] = Y[m, k] > 0 ? scale * sum_c G W : 0 (the
// layer's dZ), plus its bias gradient dbY[k] = sum_m dH[m, k] as K more
// partial columns -- the pass relu_bwd_colsum would make over dH and Y again.
template <int N, bool MASK>
__global__ __launch_bounds__(kT) void linear_small_bwd_p1(int64_t M, int64_t K, const float *__restrict__ G,
                                                          int64_t ldg, const float *__restrict__ W,
                                                          const float *__restrict__ H, int64_t ldh,
                                                          float *__restrict__ dH, int64_t lddh, float scale,
                                                          float *__restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowsLinear;
  const int64_t r1 = r0 + kRowsLinear < M ? r0 + kRowsLinear : M;
  const int64_t tot = N * K + N + (MASK ? K : 0);
  float *pw = part + (int64_t)blockIdx.x * tot;  // [N][K], db[N], (MASK) dbY[K]
  // db = sum_m G[m, c] in row order, accumulated beside the rows' other work by every thread (the
  // same sums; thread 0 stores them) -- a separate loop after it was 128 dependent loads per block
  float sg[N];
#pragma unroll
  for (int c = 0; c < N; ++c) sg[c] = 0.f;
  bool first = true;
  for (int64_t k = (int64_t)threadIdx.x * 4; k < K; k += kT * 4) {
    float4 w[N], acc[N];
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int c = 0; c < N; ++c) {
      w[c] = *reinterpret_cast<const float4 *>(W + c * K + k);
      acc[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    auto row = [&](int64_t m, float4 h) {
      float4 d = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int c = 0; c < N; ++c) {
        const float gc = G[m * ldg + c];
        if (first) sg[c] = sg[c] + gc;
        d.x = d.x + gc * w[c].x; d.y = d.y + gc * w[c].y; d.z = d.z + gc * w[c].z; d.w = d.w + gc * w[c].w;
        acc[c].x = acc[c].x + gc * h.x; acc[c].y = acc[c].y + gc * h.y;
        acc[c].z = acc[c].z + gc * h.z; acc[c].w = acc[c].w + gc * h.w;
      }
      if (MASK) {
        d.x = h.x > 0.f ? d.x * scale : 0.f;
        d.y = h.y > 0.f ? d.y * scale : 0.f;
        d.z = h.z > 0.f ? d.z * scale : 0.f;
        d.w = h.w > 0.f ? d.w * scale : 0.f;
        cs.x = cs.x + d.x; cs.y = cs.y + d.y; cs.z = cs.z + d.z; cs.w = cs.w + d.w;
      }
      if (dH) *reinterpret_cast<float4 *>(dH + m * lddh + k) = d;
    };
    int64_t m = r0;
    for (; m + kUnrollLinear <= r1; m += kUnrollLinear) {
      float4 h[kUnrollLinear];
#pragma unroll
      for (int u = 0; u < kUnrollLinear; ++u) h[u] = *reinterpret_cast<const float4 *>(H + (m + u) * ldh + k);
#pragma unroll
      for (int u = 0; u < kUnrollLinear; ++u) row(m + u, h[u]);
    }
    for (; m < r1; ++m) row(m, *reinterpret_cast<const float4 *>(H + m * ldh + k));
#pragma unroll
    for (int c = 0; c < N; ++c) *reinterpret_cast<float4 *>(pw + c * K + k) = acc[c];
    if (MASK) *reinterpret_cast<float4 *>(pw + N * K + N + k) = cs;
    first = false;
  }
  if (threadIdx.x == 0) {
    if (first) {  // (no column pass ran on this thread: K == 0)
      for (int64_t m = r0; m < r1; ++m)
#pragma unroll
        for (int c = 0; c < N; ++c) sg[c] = sg[c] + G[m * ldg + c];
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

extern "C" int64_t lpg_wgrad_smallk_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return -1;
  return fold_floats((M + kRowsWgrad - 1) / kRowsWgrad, (K + 1) * N) * (int64_t)sizeof(float);
}

namespace lpg {
namespace {

lpg_status wgrad_smallk(int64_t M, int64_t N, const float *dz, int64_t ldz, const float *y, int64_t ldy, float scale,
                        int64_t K1, const float *A1, int64_t lda1, int64_t K2, const float *A2, int64_t lda2,
                        float *dW1, float *dW2, float *db, void *workspace, void *stream, const char *name) {
  const int64_t K = K1 + K2;
  const bool mask = y != nullptr;
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0 && K >= 1 && K <= kMaxSmallK, "%s: need 1 <= K1 + K2 <= %d",
              name, kMaxSmallK);
  LPG_REQUIRE(dz && workspace && (K1 == 0 || A1) && (K2 == 0 || A2), "%s: NULL pointer", name);
  LPG_REQUIRE(N % 4 == 0 && ldz % 4 == 0 && aligned16(dz) && aligned16(workspace) &&
                  (!mask || (ldy % 4 == 0 && aligned16(y))),
              "%s: N / leading dims multiples of 4, gradient / output / workspace 16-byte aligned", name);
  hipStream_t s = as_stream(stream);
  if (M == 0 || N == 0) {
    if (dW1 && N * K1) LPG_HIP(hipMemsetAsync(dW1, 0, sizeof(float) * N * K1, s));
    if (dW2 && N * K2) LPG_HIP(hipMemsetAsync(dW2, 0, sizeof(float) * N * K2, s));
    if (db && N) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, s));
    return LPG_OK;
  }
  const int64_t nblk = (M + kRowsWgrad - 1) / kRowsWgrad;
  const int64_t KR = K + (mask ? 1 : 0);
  float *part = static_cast<float *>(workspace);
  const int k1 = (int)K1;
  const dim3 grid((unsigned)nblk), block(kT);
  switch (K * 2 + (mask ? 1 : 0)) {
#define LPG_WG(KK)                                                                                                  \
  case 2 * KK:                                                                                                      \
    hipLaunchKernelGGL((wgrad_smallk_p1<KK, false>), grid, block, 0, s, M, N, dz, ldz, y, ldy, scale, k1, A1, lda1, \
                       A2, lda2, part);                                                                             \
    break;                                                                                                          \
  case 2 * KK + 1:                                                                                                  \
    hipLaunchKernelGGL((wgrad_smallk_p1<KK, true>), grid, block, 0, s, M, N, dz, ldz, y, ldy, scale, k1, A1, lda1,  \
                       A2, lda2, part);                                                                             \
    break;
    LPG_WG(1) LPG_WG(2) LPG_WG(3) LPG_WG(4) LPG_WG(5) LPG_WG(6) LPG_WG(7) LPG_WG(8)
    LPG_WG(9) LPG_WG(10) LPG_WG(11) LPG_WG(12) LPG_WG(13) LPG_WG(14) LPG_WG(15) LPG_WG(16)
#undef LPG_WG
  }
  LPG_HIP(hipGetLastError());
  const float *img;
  const int64_t nrow = fold(nblk, KR * N, part, part + nblk * KR * N, &img, s);
  hipLaunchKernelGGL(wgrad_smallk_p2, dim3((unsigned)((KR * N + kT - 1) / kT)), dim3(kT), 0, s, nrow, N, (int)K,
                     (int)KR, k1, img, dW1, dW2, db);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

}  // namespace
}  // namespace lpg

extern "C" lpg_status lpg_wgrad_smallk_f32(int64_t M, int64_t N, const float *dz, int64_t ldz, int64_t K1,
                                           const float *A1, int64_t lda1, int64_t K2, const float *A2, int64_t lda2,
                                           float *dW1, float *dW2, void *workspace, void *stream) {
  return wgrad_smallk(M, N, dz, ldz, nullptr, 0, 1.f, K1, A1, lda1, K2, A2, lda2, dW1, dW2, nullptr, workspace,
                      stream, "lpg_wgrad_smallk_f32");
}

extern "C" lpg_status lpg_relu_wgrad_smallk_f32(int64_t M, int64_t N, const float *g, int64_t ldg, const float *y,
                                                int64_t ldy, float scale, int64_t K1, const float *A1, int64_t lda1,
                                                int64_t K2, const float *A2, int64_t lda2, float *dW1, float *dW2,
                                                float *db, void *workspace, void *stream) {
  LPG_REQUIRE(y != nullptr, "lpg_relu_wgrad_smallk_f32: NULL output");
  return wgrad_smallk(M, N, g, ldg, y, ldy, scale, K1, A1, lda1, K2, A2, lda2, dW1, dW2, db, workspace, stream,
                      "lpg_relu_wgrad_smallk_f32");
}

namespace lpg {
namespace {

lpg_status linear_small_bwd(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg, const float *W,
                            const float *H, int64_t ldh, float *dH, int64_t lddh, float scale, float *dW, float *db,
                            float *dbY, bool mask, void *workspace, void *stream, const char *what) {
  LPG_REQUIRE(M >= 0 && K >= 0 && N >= 1 && N <= kSmallNMax, "%s: need 1 <= N <= %d", what, kSmallNMax);
  LPG_REQUIRE(K % 4 == 0 && ldh % 4 == 0 && (dH == nullptr || lddh % 4 == 0),
              "%s: K and leading dims must be multiples of 4", what);
  LPG_REQUIRE(G && W && H && workspace, "%s: NULL pointer", what);
  LPG_REQUIRE(aligned16(W) && aligned16(H) && (dH == nullptr || aligned16(dH)) && aligned16(workspace),
              "%s: W/H/dH/workspace must be 16-byte aligned", what);
  hipStream_t s = as_stream(stream);
  const int64_t nblk = (M + kRowsLinear - 1) / kRowsLinear;
  if (nblk == 0) {
    if (dW) LPG_HIP(hipMemsetAsync(dW, 0, sizeof(float) * N * K, s));
    if (db) LPG_HIP(hipMemsetAsync(db, 0, sizeof(float) * N, s));
    if (dbY) LPG_HIP(hipMemsetAsync(dbY, 0, sizeof(float) * K, s));
    return LPG_OK;
  }
  float *part = static_cast<float *>(workspace);
  const dim3 grid((unsigned)nblk), block(kT);
#define LPG_LSB(NN)                                                                                               \
  if (mask)                                                                                                       \
    hipLaunchKernelGGL((linear_small_bwd_p1<NN, true>), grid, block, 0, s, M, K, G, ldg, W, H, ldh, dH, lddh,     \
                       scale, part);                                                                              \
  else                                                                                                            \
    hipLaunchKernelGGL((linear_small_bwd_p1<NN, false>), grid, block, 0, s, M, K, G, ldg, W, H, ldh, dH, lddh,    \
                       scale, part);
  switch (N) {
    case 1: LPG_LSB(1) break;
    case 2: LPG_LSB(2) break;
    case 3: LPG_LSB(3) break;
    default: LPG_LSB(4)
  }
#undef LPG_LSB
  LPG_HIP(hipGetLastError());
  const int64_t tot = N * K + N + (mask ? K : 0);
  const float *img;
  const int64_t nrow = fold(nblk, tot, part, part + nblk * tot, &img, s);
  hipLaunchKernelGGL(linear_small_bwd_p2, dim3((unsigned)((tot + kT - 1) / kT)), dim3(kT), 0, s, nrow, K, (int)N, tot,
                     img, dW, db, dbY);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

}  // namespace
}  // namespace lpg

extern "C" int64_t lpg_linear_small_bwd_workspace_bytes(int64_t M, int64_t K, int64_t N) {
  if (M < 0 || K < 0 || N < 0) return -1;
  return fold_floats((M + kRowsLinear - 1) / kRowsLinear, N * K + N + K) * (int64_t)sizeof(float);
}

extern "C" lpg_status lpg_linear_small_bwd_f32(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg,
                                               const float *W, const float *H, int64_t ldh, float *dH, int64_t lddh,
                                               float *dW, float *db, void *workspace, void *stream) {
  return linear_small_bwd(M, K, N, G, ldg, W, H, ldh, dH, lddh, 1.f, dW, db, nullptr, false, workspace, stream,
                          "lpg_linear_small_bwd_f32");
}

extern "C" lpg_status lpg_heads_relu_bwd_f32(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg,
                                             const float *W, const float *Y, int64_t ldy, float scale, float *dZ,
                                             int64_t lddz, float *dW, float *db, float *dbY, void *workspace,
                                             void *stream) {
  LPG_REQUIRE(dZ != nullptr, "lpg_heads_relu_bwd_f32: NULL dZ");
  return linear_small_bwd(M, K, N, G, ldg, W, Y, ldy, dZ, lddz, scale, dW, db, dbY, true, workspace, stream,
                          "lpg_heads_relu_bwd_f32");
}
