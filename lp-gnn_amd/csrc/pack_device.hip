// Device dual-CSR pack: the GPU counterpart of lpg_csr_pack_host (pack.cpp),
// same output bit for bit.  SURVEY.md §8f rank 1: the reference rebuilds the
// CSR in DataLoader workers every graph load (dataset.py:250-252, 296-304)
// and re-derives the transpose every layer (arch.py:71); here both
// orientations are built once on the device from the COO edge list.
//
// Algorithm: two stable LSD radix sorts (rocPRIM, header-only, ROCm 7.2) of
// composite keys row*n+col and col*m+row carrying the edge id, then
// per-row lower_bound for rowptr.  Out-of-range indices and duplicate
// (row, col) pairs are counted into the first 16 bytes of the workspace
// (two int64 counters) -- the stream-ordered analogue of the host pack's
// LPG_ERR_INVALID; the Python wrapper reads them after the pack.
#include <rocprim/device/device_radix_sort.hpp>

#include "common.h"

namespace lpg {
namespace {

constexpr int kThreads = 256;

inline unsigned blocks_for(int64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

__global__ void make_row_keys(const int64_t *__restrict__ row, const int64_t *__restrict__ col, int64_t nnz,
                              int64_t m, int64_t n, uint64_t *__restrict__ keys, int32_t *__restrict__ ids,
                              unsigned long long *__restrict__ bad) {
  const int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (e >= nnz) return;
  int64_t r = row[e], c = col[e];
  if (r < 0 || r >= m || c < 0 || c >= n) {
    atomicAdd(bad, 1ull);
    r = m - 1;  // keep the sort well defined; the result is flagged invalid
    c = n - 1;
  }
  keys[e] = (uint64_t)r * (uint64_t)n + (uint64_t)c;
  ids[e] = (int32_t)e;
}

// After sort 1: keys sorted by (row, col).  Emit CSR(A) col/val and the
// transposed keys col*m + row, carrying the CSR(A) position.
__global__ void emit_a(const uint64_t *__restrict__ skeys, const int32_t *__restrict__ perm,
                       const float *__restrict__ val, int64_t nnz, int64_t m, int64_t n,
                       int32_t *__restrict__ a_col, float *__restrict__ a_val, uint64_t *__restrict__ tkeys,
                       int32_t *__restrict__ pos, unsigned long long *__restrict__ dup) {
  const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (p >= nnz) return;
  const uint64_t k = skeys[p];
  const uint64_t r = k / (uint64_t)n, c = k % (uint64_t)n;
  if (p > 0 && skeys[p - 1] == k) atomicAdd(dup, 1ull);
  a_col[p] = (int32_t)c;
  a_val[p] = val[perm[p]];
  tkeys[p] = c * (uint64_t)m + r;
  pos[p] = (int32_t)p;
}

__global__ void emit_at(const uint64_t *__restrict__ skeys, const int32_t *__restrict__ perm,
                        const float *__restrict__ a_val, int64_t nnz, int64_t m, int32_t *__restrict__ at_col,
                        float *__restrict__ at_val) {
  const int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (p >= nnz) return;
  at_col[p] = (int32_t)(skeys[p] % (uint64_t)m);
  at_val[p] = a_val[perm[p]];
}

// rowptr[r] = first p with skeys[p] >= r * stride  (r in [0, rows]).
__global__ void rowptr_lower_bound(const uint64_t *__restrict__ skeys, int64_t nnz, int64_t rows,
                                   uint64_t stride, int64_t *__restrict__ rowptr) {
  const int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (r > rows) return;
  const uint64_t target = (uint64_t)r * stride;
  int64_t lo = 0, hi = nnz;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (skeys[mid] < target) lo = mid + 1; else hi = mid;
  }
  rowptr[r] = lo;
}

int end_bit_for(uint64_t max_key) {
  int b = 1;
  while (b < 64 && (max_key >> b) != 0) ++b;
  return b;
}

struct Layout {
  size_t flags, keys_a, keys_b, ids_a, ids_b, tmp, tmp_bytes, total;
};

inline size_t up16(size_t x) { return (x + 15) & ~size_t(15); }

Layout layout(int64_t nnz, int64_t m, int64_t n) {
  Layout L{};
  size_t off = 0;
  L.flags = off; off += 16;
  L.keys_a = off; off = up16(off + sizeof(uint64_t) * (size_t)nnz);
  L.keys_b = off; off = up16(off + sizeof(uint64_t) * (size_t)nnz);
  L.ids_a = off; off = up16(off + sizeof(int32_t) * (size_t)nnz);
  L.ids_b = off; off = up16(off + sizeof(int32_t) * (size_t)nnz);
  size_t t1 = 0, t2 = 0;
  const uint64_t mk = (uint64_t)(m > 0 ? m : 1) * (uint64_t)(n > 0 ? n : 1);
  (void)rocprim::radix_sort_pairs(nullptr, t1, (uint64_t *)nullptr, (uint64_t *)nullptr, (int32_t *)nullptr,
                            (int32_t *)nullptr, (size_t)nnz, 0, end_bit_for(mk));
  (void)rocprim::radix_sort_pairs(nullptr, t2, (uint64_t *)nullptr, (uint64_t *)nullptr, (int32_t *)nullptr,
                            (int32_t *)nullptr, (size_t)nnz, 0, end_bit_for(mk));
  L.tmp = off;
  L.tmp_bytes = t1 > t2 ? t1 : t2;
  off = up16(off + L.tmp_bytes);
  L.total = off;
  return L;
}

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" int64_t lpg_csr_pack_workspace_bytes(int64_t nnz, int64_t m, int64_t n) {
  if (nnz < 0 || m < 0 || n < 0) return -1;
  return (int64_t)layout(nnz, m, n).total;
}

extern "C" lpg_status lpg_csr_pack_f32(const int64_t *row, const int64_t *col, const float *val, int64_t nnz,
                                       int64_t m, int64_t n, int64_t *a_rowptr, int32_t *a_col, float *a_val,
                                       int64_t *at_rowptr, int32_t *at_col, float *at_val, void *workspace,
                                       void *stream) {
  LPG_REQUIRE(nnz >= 0 && m >= 0 && n >= 0, "lpg_csr_pack_f32: negative size");
  LPG_REQUIRE(m <= INT32_MAX && n <= INT32_MAX && nnz <= INT32_MAX,
              "lpg_csr_pack_f32: sizes exceed int32 indices");
  LPG_REQUIRE(a_rowptr && at_rowptr && workspace, "lpg_csr_pack_f32: NULL rowptr/workspace");
  LPG_REQUIRE(nnz == 0 || (row && col && val && a_col && a_val && at_col && at_val),
              "lpg_csr_pack_f32: NULL edge buffer");
  LPG_REQUIRE(lpg::aligned16(workspace), "lpg_csr_pack_f32: workspace must be 16-byte aligned");
  hipStream_t s = as_stream(stream);
  const Layout L = layout(nnz, m, n);
  char *ws = static_cast<char *>(workspace);
  auto *flags = reinterpret_cast<unsigned long long *>(ws + L.flags);
  LPG_HIP(hipMemsetAsync(flags, 0, 16, s));
  if (nnz == 0) {
    LPG_HIP(hipMemsetAsync(a_rowptr, 0, sizeof(int64_t) * (size_t)(m + 1), s));
    LPG_HIP(hipMemsetAsync(at_rowptr, 0, sizeof(int64_t) * (size_t)(n + 1), s));
    return LPG_OK;
  }
  auto *ka = reinterpret_cast<uint64_t *>(ws + L.keys_a);
  auto *kb = reinterpret_cast<uint64_t *>(ws + L.keys_b);
  auto *ia = reinterpret_cast<int32_t *>(ws + L.ids_a);
  auto *ib = reinterpret_cast<int32_t *>(ws + L.ids_b);
  void *tmp = ws + L.tmp;
  size_t tmp_bytes = L.tmp_bytes;
  const int eb = end_bit_for((uint64_t)m * (uint64_t)n);

  hipLaunchKernelGGL(make_row_keys, dim3(blocks_for(nnz)), dim3(kThreads), 0, s, row, col, nnz, m, n, ka, ia,
                     flags);
  LPG_HIP(hipGetLastError());
  LPG_HIP(rocprim::radix_sort_pairs(tmp, tmp_bytes, ka, kb, ia, ib, (size_t)nnz, 0, eb, s));
  // kb/ib: sorted by (row, col).  Reuse ka/ia for the transposed keys.
  hipLaunchKernelGGL(emit_a, dim3(blocks_for(nnz)), dim3(kThreads), 0, s, kb, ib, val, nnz, m, n, a_col, a_val,
                     ka, ia, flags + 1);
  LPG_HIP(hipGetLastError());
  hipLaunchKernelGGL(rowptr_lower_bound, dim3(blocks_for(m + 1)), dim3(kThreads), 0, s, kb, nnz, m,
                     (uint64_t)n, a_rowptr);
  LPG_HIP(hipGetLastError());
  tmp_bytes = L.tmp_bytes;
  LPG_HIP(rocprim::radix_sort_pairs(tmp, tmp_bytes, ka, kb, ia, ib, (size_t)nnz, 0, eb, s));
  hipLaunchKernelGGL(emit_at, dim3(blocks_for(nnz)), dim3(kThreads), 0, s, kb, ib, a_val, nnz, m, at_col,
                     at_val);
  LPG_HIP(hipGetLastError());
  hipLaunchKernelGGL(rowptr_lower_bound, dim3(blocks_for(n + 1)), dim3(kThreads), 0, s, kb, nnz, n,
                     (uint64_t)m, at_rowptr);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}
