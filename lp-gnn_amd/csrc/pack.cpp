// Host dual-CSR pack: COO edges of A (rows = constraints, cols = variables)
// -> CSR(A) and CSR(A^T), columns ascending within every row.
//
// Replaces, for one graph, torch_sparse's SparseTensor.from_edge_index
// (called at dataset.py:301-304: sorts by row*N + col, builds rowptr) and
// SparseTensor.t() (called at arch.py:71 every layer: csr2csc = argsort of
// col*M + row).  Both orders are reproduced exactly, so the per-row edge
// order -- and with it the floating-point summation order of spmm_sum -- is
// the reference's.  O(nnz + m + n) plus a per-row sort of the columns.
#include <algorithm>
#include <vector>

#include "common.h"

using namespace lpg;

extern "C" lpg_status lpg_csr_pack_host(const int64_t *row, const int64_t *col, const float *val,
                                        int64_t nnz, int64_t m, int64_t n, int64_t *a_rowptr,
                                        int32_t *a_col, float *a_val, int64_t *at_rowptr,
                                        int32_t *at_col, float *at_val) {
  LPG_REQUIRE(nnz >= 0 && m >= 0 && n >= 0, "lpg_csr_pack_host: negative size");
  LPG_REQUIRE(m <= INT32_MAX && n <= INT32_MAX, "lpg_csr_pack_host: m/n exceed int32 indices");
  LPG_REQUIRE(a_rowptr && at_rowptr, "lpg_csr_pack_host: rowptr output is NULL");
  LPG_REQUIRE(nnz == 0 || (row && col && val && a_col && a_val && at_col && at_val),
              "lpg_csr_pack_host: NULL edge buffer");

  std::vector<int64_t> cnt_r(m + 1, 0), cnt_c(n + 1, 0);
  for (int64_t e = 0; e < nnz; ++e) {
    const int64_t r = row[e], c = col[e];
    LPG_REQUIRE(r >= 0 && r < m, "lpg_csr_pack_host: row[%lld]=%lld out of [0,%lld)", (long long)e,
                (long long)r, (long long)m);
    LPG_REQUIRE(c >= 0 && c < n, "lpg_csr_pack_host: col[%lld]=%lld out of [0,%lld)", (long long)e,
                (long long)c, (long long)n);
    ++cnt_r[r + 1];
    ++cnt_c[c + 1];
  }
  for (int64_t i = 0; i < m; ++i) cnt_r[i + 1] += cnt_r[i];
  for (int64_t j = 0; j < n; ++j) cnt_c[j + 1] += cnt_c[j];
  std::copy(cnt_r.begin(), cnt_r.end(), a_rowptr);
  std::copy(cnt_c.begin(), cnt_c.end(), at_rowptr);

  // CSR(A): bucket by row (stable), then sort each row by column.
  std::vector<int64_t> perm(nnz);
  {
    std::vector<int64_t> cur(cnt_r.begin(), cnt_r.end() - 1);
    for (int64_t e = 0; e < nnz; ++e) perm[cur[row[e]]++] = e;
  }
  for (int64_t i = 0; i < m; ++i) {
    auto b = perm.begin() + a_rowptr[i], en = perm.begin() + a_rowptr[i + 1];
    std::sort(b, en, [&](int64_t x, int64_t y) { return col[x] < col[y]; });
    for (auto it = b; it != en; ++it) {
      if (it != b && col[*it] == col[*(it - 1)]) {
        set_error("lpg_csr_pack_host: duplicate edge (%lld, %lld); coalesce first (dataset.py:252)",
                  (long long)i, (long long)col[*it]);
        return LPG_ERR_INVALID;
      }
    }
  }
  for (int64_t p = 0; p < nnz; ++p) {
    a_col[p] = (int32_t)col[perm[p]];
    a_val[p] = val[perm[p]];
  }
  // CSR(A^T): walk CSR(A) in (row, col) order and bucket by col -> rows ascending.
  {
    std::vector<int64_t> cur(cnt_c.begin(), cnt_c.end() - 1);
    for (int64_t i = 0; i < m; ++i)
      for (int64_t p = a_rowptr[i]; p < a_rowptr[i + 1]; ++p) {
        const int64_t q = cur[a_col[p]]++;
        at_col[q] = (int32_t)i;
        at_val[q] = a_val[p];
      }
  }
  clear_error();
  return LPG_OK;
}
