/*
 * ORACLE -- test infrastructure only (see spmm_ref.c header).
 *
 * Bitwise restatement of the dense FC order used by lpg_fc_f32:
 * PyG 2.1 GraphConv after propagate, out = lin_rel(agg) + lin_root(x_dst)
 * (arch.py:57-62, 75-80), ReLU (arch.py:182, 188), and the heads
 * lin_left/lin_right (arch.py:190), evaluated in a fixed blocked k order
 * (see phase()) then + P (lpg_fc_f32's accumulate flag), then + bias,
 * then ReLU as (v < 0 ? 0 : v).  torch.nn.functional.linear on CPU (MKL) is the
 * reference's own evaluation; it sums in an unspecified blocked order, so it
 * agrees with this chain to fp32 rounding only (tests report both).
 *
 * Loop order m -> k -> n keeps each output's chains in the contract's order while the
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

/* The order of lpg_fc_f32 (fc.hip header): each part (A1 over K1, then A2
 * over K2) is cut into blocks of FC_NB = 128 k (the last one shorter); a
 * block's products form ONE fma chain from +0 whose k are visited in groups
 * of 8 consecutive k (the last group zero-padded -- exact no-ops, skipped
 * here), inside a group in the order 0,4,1,5,2,6,3,7; block sums are added
 * in order into the running total (+0 initially).
 * out = total [+ P] + bias, then ReLU. */
#define FC_NB 128

static int64_t pik(int64_t i) { return (i & ~7) + (i & 1) * 4 + ((i >> 1) & 3); }

static void phase(const float *A, int64_t lda, const float *Wt, int64_t N, int64_t K, int64_t m, float *tot,
                  float *part) {
  for (int64_t k0 = 0; k0 < K; k0 += FC_NB) {
    const int64_t kb = K - k0 < FC_NB ? K - k0 : FC_NB;
    for (int64_t n = 0; n < N; ++n) part[n] = 0.0f;
    for (int64_t i = 0; i < (kb + 7) / 8 * 8; ++i) {
      const int64_t k = k0 + pik(i);
      if (k >= k0 + kb) continue;
      const float a = A[m * lda + k];
      const float *w = Wt + k * N;
      for (int64_t n = 0; n < N; ++n) part[n] = fmaf(a, w[n], part[n]);
    }
    for (int64_t n = 0; n < N; ++n) tot[n] = tot[n] + part[n];
  }
}

void oracle_fc_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const float *W1, int64_t ldw1,
                   int64_t K2, const float *A2, int64_t lda2, const float *W2, int64_t ldw2, const float *bias,
                   float *C, int64_t ldc, const float *P, int64_t ldp, int relu, int nthreads) {
  float *W1t = (float *)malloc(sizeof(float) * (size_t)(K1 * N + 1));
  float *W2t = (float *)malloc(sizeof(float) * (size_t)(K2 * N + 1));
  transpose(W1, ldw1, N, K1, W1t);
  transpose(W2, ldw2, N, K2, W2t);
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
  {
    float *part = (float *)malloc(sizeof(float) * (size_t)(N + 1));
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
    for (int64_t m = 0; m < M; ++m) {
      float *c = C + m * ldc;
      for (int64_t n = 0; n < N; ++n) c[n] = 0.0f;
      phase(A1, lda1, W1t, N, K1, m, c, part);
      phase(A2, lda2, W2t, N, K2, m, c, part);
      if (P) /* accumulate flag: the re-associated GraphConv's S (x W_rel^T) */
        for (int64_t n = 0; n < N; ++n) c[n] = c[n] + P[m * ldp + n];
      if (bias)
        for (int64_t n = 0; n < N; ++n) c[n] = c[n] + bias[n];
      if (relu)
        for (int64_t n = 0; n < N; ++n) c[n] = (c[n] < 0.0f) ? 0.0f : c[n];
    }
    free(part);
  }
  free(W1t);
  free(W2t);
}
