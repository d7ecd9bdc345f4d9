// Weighted cross entropy of the balanced loss (train.py:39-46 via
// nn.CrossEntropyLoss(weight=w), mean reduction, ignore_index = -100):
//
//   CE = sum_i w[y_i] (lse(x_i) - x_i[y_i]) / sum_i w[y_i]     (rows with y_i = -100 skipped)
//   dCE/dx_i = w[y_i] / sum_j w[y_j] * (softmax(x_i) - onehot(y_i))
//
// torch's CUDA nll_loss with class weights reduces in ONE workgroup (measured
// 75-165 us per call at 100-200 K rows); here one thread per row, per-block
// partials (sum w*l, sum w) and a one-block fold in a fixed order
// (deterministic), C <= 4 classes.  An out-of-range label makes the loss NaN
// (the caller's NaN check, train.py:126, then trips; torch raises a device
// assert).  The backward reads the logits again (C floats per row) and the
// device-side sum of weights: no host synchronisation anywhere.
#include "common.h"

namespace lpg {
namespace {

constexpr int kCeT = 256;

__device__ __forceinline__ void ce_row(int64_t C, const float *x, int64_t y, const float *w, float &wl, float &ww,
                                       float (&p)[4], bool &valid) {
  float v[4];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    v[c] = c < C ? x[c] : -INFINITY;
    mx = v[c] > mx ? v[c] : mx;
  }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    p[c] = c < C ? expf(v[c] - mx) : 0.f;
    se = se + p[c];
  }
  const float lse = mx + logf(se);
#pragma unroll
  for (int c = 0; c < 4; ++c) p[c] = p[c] / se;
  valid = y != -100;
  if (!valid) {
    wl = 0.f;
    ww = 0.f;
  } else if (y < 0 || y >= C) {
    wl = NAN;
    ww = NAN;
  } else {
    const float wy = w ? w[y] : 1.f;
    float xy = v[0];
#pragma unroll
    for (int c = 1; c < 4; ++c) xy = (int64_t)c == y ? v[c] : xy;
    wl = wy * (lse - xy);
    ww = wy;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = v + __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kCeT) void ce_fwd_p1(int64_t M, int64_t C, const float *__restrict__ x, int64_t ldx,
                                                  const int64_t *__restrict__ y, const float *__restrict__ w,
                                                  float *__restrict__ part) {
  const int64_t i = (int64_t)blockIdx.x * kCeT + threadIdx.x;
  float wl = 0.f, ww = 0.f;
  if (i < M) {
    float p[4];
    bool valid;
    ce_row(C, x + i * ldx, y[i], w, wl, ww, p, valid);
  }
  wl = wave_sum(wl);
  ww = wave_sum(ww);
  __shared__ float s[2][kCeT / 64];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s[0][wv] = wl;
    s[1][wv] = ww;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int k = 0; k < kCeT / 64; ++k) {
      a = a + s[0][k];
      b = b + s[1][k];
    }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
}

// one block: thread t sums partials t, t + 256, ... in order, then a fixed tree
__global__ __launch_bounds__(kCeT) void ce_fwd_p2(int64_t nblk, const float *__restrict__ part, float coef,
                                                  float *__restrict__ loss, float *__restrict__ wsum) {
  float a = 0.f, b = 0.f;
  for (int64_t k = threadIdx.x; k < nblk; k += kCeT) {
    a = a + part[2 * k];
    b = b + part[2 * k + 1];
  }
  __shared__ float s[2][kCeT];
  s[0][threadIdx.x] = a;
  s[1][threadIdx.x] = b;
  __syncthreads();
  for (int h = kCeT / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      s[0][threadIdx.x] = s[0][threadIdx.x] + s[0][threadIdx.x + h];
      s[1][threadIdx.x] = s[1][threadIdx.x] + s[1][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    *loss = coef * (s[0][0] / s[1][0]);
    *wsum = s[1][0];
  }
}

__global__ __launch_bounds__(kCeT) void ce_bwd(int64_t M, int64_t C, const float *__restrict__ x, int64_t ldx,
                                               const int64_t *__restrict__ y, const float *__restrict__ w,
                                               const float *__restrict__ wsum, const float *__restrict__ gout,
                                               float coef, float *__restrict__ dx, int64_t lddx) {
  const int64_t i = (int64_t)blockIdx.x * kCeT + threadIdx.x;
  if (i >= M) return;
  float p[4], wl, ww;
  bool valid;
  const int64_t yi = y[i];
  ce_row(C, x + i * ldx, yi, w, wl, ww, p, valid);
  const float s = valid ? (gout ? *gout : 1.f) * coef * (ww / *wsum) : 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (c < C) dx[i * lddx + c] = s * (p[c] - ((int64_t)c == yi ? 1.f : 0.f));
}

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" int64_t lpg_weighted_ce_workspace_bytes(int64_t M) {
  return M <= 0 ? 8 : ((M + kCeT - 1) / kCeT) * 2 * (int64_t)sizeof(float);
}

extern "C" lpg_status lpg_weighted_ce_fwd_f32(int64_t M, int64_t C, const float *x, int64_t ldx, const int64_t *y,
                                              const float *w, float coef, float *loss, float *wsum, void *workspace,
                                              void *stream) {
  LPG_REQUIRE(M >= 0 && C >= 1 && C <= 4 && ldx >= C, "lpg_weighted_ce_fwd_f32: need 1 <= C <= 4, ldx >= C");
  LPG_REQUIRE(loss && wsum && workspace && (M == 0 || (x && y)), "lpg_weighted_ce_fwd_f32: NULL pointer");
  hipStream_t s = as_stream(stream);
  const int64_t nblk = M == 0 ? 1 : (M + kCeT - 1) / kCeT;
  LPG_REQUIRE(nblk < (int64_t)1 << 31, "lpg_weighted_ce_fwd_f32: too many rows");
  float *part = static_cast<float *>(workspace);
  if (M == 0) {
    LPG_HIP(hipMemsetAsync(part, 0, 2 * sizeof(float), s));  // 0 / 0 = NaN, as torch's mean over no rows
  } else {
    hipLaunchKernelGGL(ce_fwd_p1, dim3((unsigned)nblk), dim3(kCeT), 0, s, M, C, x, ldx, y, w, part);
    LPG_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(ce_fwd_p2, dim3(1), dim3(kCeT), 0, s, nblk, part, coef, loss, wsum);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_weighted_ce_bwd_f32(int64_t M, int64_t C, const float *x, int64_t ldx, const int64_t *y,
                                              const float *w, const float *wsum, const float *gout, float coef,
                                              float *dx, int64_t lddx, void *stream) {
  LPG_REQUIRE(M >= 0 && C >= 1 && C <= 4 && ldx >= C && lddx >= C, "lpg_weighted_ce_bwd_f32: bad shapes");
  if (M == 0) return LPG_OK;
  LPG_REQUIRE(x && y && wsum && dx, "lpg_weighted_ce_bwd_f32: NULL pointer");
  hipLaunchKernelGGL(ce_bwd, dim3((unsigned)((M + kCeT - 1) / kCeT)), dim3(kCeT), 0, as_stream(stream), M, C, x, ldx,
                     y, w, wsum, gout, coef, dx, lddx);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

namespace lpg {
namespace {
constexpr int kCntBlocks = 256;

// Per-class label counts (3 classes): one partial triple per block, summed by one block in
// block order -- integers, so the result is exact; no atomics.
__global__ __launch_bounds__(256) void class_counts_p1(int64_t M, const int64_t *__restrict__ y,
                                                       int64_t *__restrict__ part) {
  __shared__ int64_t red[3][256];
  int64_t c0 = 0, c1 = 0, c2 = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < M; i += (int64_t)gridDim.x * 256) {
    const int64_t v = y[i];
    c0 += v == 0;
    c1 += v == 1;
    c2 += v == 2;
  }
  red[0][threadIdx.x] = c0;
  red[1][threadIdx.x] = c1;
  red[2][threadIdx.x] = c2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int c = 0; c < 3; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3) part[blockIdx.x * 3 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ __launch_bounds__(256) void class_counts_p2(int nblk, const int64_t *__restrict__ part,
                                                       int64_t *__restrict__ counts, float *__restrict__ weights,
                                                       int32_t merge_lu) {
  __shared__ int64_t red[3][256];
#pragma unroll
  for (int c = 0; c < 3; ++c) red[c][threadIdx.x] = (int)threadIdx.x < nblk ? part[threadIdx.x * 3 + c] : 0;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int c = 0; c < 3; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3 && counts) counts[threadIdx.x] = red[threadIdx.x][0];
  if (threadIdx.x == 0 && weights) {
    // labels_to_balanced_weights (utils.py:286-299): w[c] = N / count_c (int64 true division, i.e.
    // float32 operands, correctly rounded) for present classes, 0 otherwise; unless exactly two
    // classes are present, w0 = w2 = (w0 + w2) / 2 (merge_lu)
    const int64_t c0 = red[0][0], c1 = red[1][0], c2 = red[2][0];
    const float n = (float)(c0 + c1 + c2);
    float w0 = c0 > 0 ? n / (float)c0 : 0.f, w2 = c2 > 0 ? n / (float)c2 : 0.f;
    const float w1 = c1 > 0 ? n / (float)c1 : 0.f;
    if (merge_lu && (c0 > 0) + (c1 > 0) + (c2 > 0) != 2) w0 = w2 = (w0 + w2) / 2.f;
    weights[0] = w0, weights[1] = w1, weights[2] = w2;
  }
}
}  // namespace
}  // namespace lpg

extern "C" int64_t lpg_class_counts_workspace_bytes(int64_t M) {
  (void)M;
  return (int64_t)kCntBlocks * 3 * (int64_t)sizeof(int64_t);
}

extern "C" lpg_status lpg_class_counts3(int64_t M, const int64_t *y, int64_t *counts, void *workspace, void *stream) {
  LPG_REQUIRE(M >= 0, "lpg_class_counts3: negative size");
  LPG_REQUIRE(counts && workspace && (M == 0 || y), "lpg_class_counts3: NULL pointer");
  hipStream_t s = as_stream(stream);
  const int64_t want = (M + 256 * 8 - 1) / (256 * 8);
  const int nblk = (int)(want < 1 ? 1 : (want > kCntBlocks ? kCntBlocks : want));
  int64_t *part = static_cast<int64_t *>(workspace);
  hipLaunchKernelGGL(class_counts_p1, dim3(nblk), dim3(256), 0, s, M, y, part);
  LPG_HIP(hipGetLastError());
  hipLaunchKernelGGL(class_counts_p2, dim3(1), dim3(256), 0, s, nblk, part, counts, (float *)nullptr, 0);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_balanced_weights3(int64_t M, const int64_t *y, int32_t merge_lu, float *weights,
                                            void *workspace, void *stream) {
  LPG_REQUIRE(M >= 0, "lpg_balanced_weights3: negative size");
  LPG_REQUIRE(weights && workspace && (M == 0 || y), "lpg_balanced_weights3: NULL pointer");
  hipStream_t s = as_stream(stream);
  const int64_t want = (M + 256 * 8 - 1) / (256 * 8);
  const int nblk = (int)(want < 1 ? 1 : (want > kCntBlocks ? kCntBlocks : want));
  int64_t *part = static_cast<int64_t *>(workspace);
  hipLaunchKernelGGL(class_counts_p1, dim3(nblk), dim3(256), 0, s, M, y, part);
  LPG_HIP(hipGetLastError());
  hipLaunchKernelGGL(class_counts_p2, dim3(1), dim3(256), 0, s, nblk, part, (int64_t *)nullptr, weights,
                     merge_lu ? 1 : 0);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}
