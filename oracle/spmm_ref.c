/*
 * ORACLE -- test infrastructure only.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / the timed CPU baseline -- never as the product path.
 *
 * CPU restatement of torch_sparse 0.6.12 `spmm_sum` (upstream, not vendored
 * under /root/reference; pinned by readme.md:51 "torch-sparse==0.6.12"):
 * csrc/cpu/spmm_cpu.cpp `spmm_cpu(rowptr, col, value, mat, "sum")`:
 *
 *   at::parallel_for over output rows m:
 *     vals[k] = 0                                  (Reducer<SUM>::init)
 *     for e in [rowptr[m], rowptr[m+1]):           (CSR order)
 *       for k in [0, K): vals[k] += value[e] * mat[col[e]*K + k]
 *     out[m*K + k] = vals[k]                       (Reducer<SUM>::write)
 *
 * reached from the reference at arch.py:75-80 through PyG 2.1
 * GraphConv.message_and_aggregate -> torch_sparse.matmul(adj_t, x, 'add'),
 * and (backward, train.py:128) SPMMSum::backward = the same loop on the CSC
 * view (colptr, row[csr2csc], value[csr2csc]) = CSR of the transpose.
 *
 * Built with -ffp-contract=off: the product is rounded before the add, as in
 * the upstream build (x86-64, no -mfma).  Parallelising over rows and
 * vectorising over k keep the per-element order, so any thread count gives
 * the same bits.  Parity status: the restated loop is pinned against the
 * reference's own call sites only (no golden vectors exist upstream or in
 * /root/reference -- SURVEY.md §8c); see DESIGN.md "Parity".
 */
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

void oracle_spmm_f32(int64_t M, const int64_t *rowptr, const int32_t *col, const float *val,
                     const float *X, int64_t ldx, int64_t F, float *Y, int64_t ldy, int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
#endif
  for (int64_t m = 0; m < M; ++m) {
    float *y = Y + m * ldy;
    for (int64_t k = 0; k < F; ++k) y[k] = 0.0f;
    for (int64_t e = rowptr[m]; e < rowptr[m + 1]; ++e) {
      const float v = val[e];
      const float *x = X + (int64_t)col[e] * ldx;
      for (int64_t k = 0; k < F; ++k) y[k] = y[k] + v * x[k];
    }
  }
}

static inline float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x0040u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

/* bf16 storage, fp32 accumulation in the same order, one rounding at the end
 * (the contract of lpg_spmm_bf16; config c5). */
void oracle_spmm_bf16(int64_t M, const int64_t *rowptr, const int32_t *col, const float *val,
                      const uint16_t *X, int64_t ldx, int64_t F, uint16_t *Y, int64_t ldy, int nthreads) {
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
  {
    float *acc = NULL;
    /* per-thread accumulator row */
    acc = (float *)__builtin_alloca(sizeof(float) * (size_t)(F > 0 ? F : 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
    for (int64_t m = 0; m < M; ++m) {
      for (int64_t k = 0; k < F; ++k) acc[k] = 0.0f;
      for (int64_t e = rowptr[m]; e < rowptr[m + 1]; ++e) {
        const float v = val[e];
        const uint16_t *x = X + (int64_t)col[e] * ldx;
        for (int64_t k = 0; k < F; ++k) acc[k] = acc[k] + v * bf16_to_f32(x[k]);
      }
      for (int64_t k = 0; k < F; ++k) Y[m * ldy + k] = f32_to_bf16_rne(acc[k]);
    }
  }
}

int oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
