/*
 * ORACLE -- test infrastructure only (see spmm_ref.c header).
 *
 * Bitwise restatement of the dense FC order used by lpg_fc_f32:
 * PyG 2.1 GraphConv after propagate, out = lin_rel(agg) + lin_root(x_dst)
 * (arch.py:57-62, 75-80), ReLU (arch.py:182, 188), and the heads
 * lin_left/lin_right (arch.py:190), evaluated as ONE fp32 fma chain per
 * output in k order (agg part then x_dst part) from +0, then + bias, then
 * ReLU as (v < 0 ? 0 : v).  torch.nn.functional.linear on CPU (MKL) is the
 * reference's own evaluation; it sums in an unspecified blocked order, so it
 * agrees with this chain to fp32 rounding only (tests report both).
 *
 * Loop order m -> k -> n keeps each output's chain in k order while the
 * inner loop vectorises across n (W is transposed once per call).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static void transpose(const float *W, int64_t ldw, int64_t N, int64_t K, float *Wt) {
  for (int64_t n = 0; n < N; ++n)
    for (int64_t k = 0; k < K; ++k) Wt[k * N + n] = W[n * ldw + k];
}

void oracle_fc_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const float *W1, int64_t ldw1,
                   int64_t K2, const float *A2, int64_t lda2, const float *W2, int64_t ldw2, const float *bias,
                   float *C, int64_t ldc, int relu, int nthreads) {
  float *W1t = (float *)malloc(sizeof(float) * (size_t)(K1 * N + 1));
  float *W2t = (float *)malloc(sizeof(float) * (size_t)(K2 * N + 1));
  transpose(W1, ldw1, N, K1, W1t);
  transpose(W2, ldw2, N, K2, W2t);
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
  for (int64_t m = 0; m < M; ++m) {
    float *c = C + m * ldc;
    for (int64_t n = 0; n < N; ++n) c[n] = 0.0f;
    for (int64_t k = 0; k < K1; ++k) {
      const float a = A1[m * lda1 + k];
      const float *w = W1t + k * N;
      for (int64_t n = 0; n < N; ++n) c[n] = fmaf(a, w[n], c[n]);
    }
    for (int64_t k = 0; k < K2; ++k) {
      const float a = A2[m * lda2 + k];
      const float *w = W2t + k * N;
      for (int64_t n = 0; n < N; ++n) c[n] = fmaf(a, w[n], c[n]);
    }
    if (bias)
      for (int64_t n = 0; n < N; ++n) c[n] = c[n] + bias[n];
    if (relu)
      for (int64_t n = 0; n < N; ++n) c[n] = (c[n] < 0.0f) ? 0.0f : c[n];
  }
  free(W1t);
  free(W2t);
}
