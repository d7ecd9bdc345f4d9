// k-hop neighbour sampling on the device: the MI355X counterpart of the
// NeighborLoader collate path the reference uses for graphs above the
// MyToBipartite threshold (train.py:111-116, val.py:22-27; PyG 2.1
// NeighborLoader -> torch_sparse 0.6.12 ``neighbor_sample``, restated in
// oracle/model_ref.py:neighbor_sample).
//
// Graph: CSC of the homogeneous (undirected) LP graph -- colptr [N+1] int64,
// row [E] int64 = source of each in-edge of node v in colptr[v]..colptr[v+1),
// sorted by source (PyG to_csc).  Sampled node lists are int64 global ids;
// `local` [N] (int64, -1 = not sampled) and `first` [N] (uint64, all ones)
// are per-graph scratch the caller keeps and this file restores.
//
// One hop: count (min(fanout, deg) per frontier node) -> exclusive scan ->
// fill candidates (frontier order, then CSC order, or Floyd's sampling
// order) -> first-appearance dedupe (atomicMin of the candidate position, a
// deterministic result) -> scan of the "new" flags -> assign local ids in
// candidate order.  That is exactly the sequential insertion order of
// neighbor_sample, so with fanout -1 the node list, and the induced edge list
// (directed=False: every in-edge of every sampled node whose source is
// sampled, by destination then CSC order), match it element for element.
#include <rocprim/device/device_scan.hpp>

#include "common.h"

namespace lpg {
namespace {

constexpr int kT = 256;
constexpr int kMaxFanout = 256;

inline unsigned blocks_for(int64_t n, int per = kT) { return (unsigned)((n + per - 1) / per); }

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// uniform integer in [0, bound) for draw j of node v
__device__ __forceinline__ int64_t draw(uint64_t seed, int64_t v, int64_t j, int64_t bound) {
  const uint64_t h = mix64(seed + 0x9e3779b97f4a7c15ull * (uint64_t)(v + 1) + mix64((uint64_t)j + 0x632be59bd9b4e019ull));
  return (int64_t)(h % (uint64_t)bound);
}

__global__ __launch_bounds__(kT) void count_kernel(int64_t nf, const int64_t *__restrict__ frontier,
                                                   const int64_t *__restrict__ colptr, int64_t fanout,
                                                   int64_t *__restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= nf) return;
  const int64_t v = frontier[i];
  const int64_t deg = colptr[v + 1] - colptr[v];
  counts[i] = (fanout < 0 || fanout >= deg) ? deg : fanout;
}

// One wave per frontier node.  Full neighbourhoods are copied by the wave;
// sampled ones follow Floyd's algorithm (torch_sparse's without-replacement
// loop): for j = deg-k .. deg-1 draw t in [0, j]; if t was already chosen take
// j instead.  The chosen list lives in registers across the wave (lane l
// holds entries l, l+64, ...), membership is one compare per slot + __any.
__global__ __launch_bounds__(kT) void fill_kernel(int64_t nf, int64_t base, const int64_t *__restrict__ frontier,
                                                  const int64_t *__restrict__ colptr,
                                                  const int64_t *__restrict__ row, int64_t fanout, uint64_t seed,
                                                  const int64_t *__restrict__ offsets, int64_t *__restrict__ cand,
                                                  int64_t *__restrict__ cand_edge, int64_t *__restrict__ cand_dst) {
  constexpr int kSlots = kMaxFanout / 64;
  const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int64_t i = (int64_t)blockIdx.x * (kT / 64) + wv;
  if (i >= nf) return;
  const int64_t v = frontier[i];
  const int64_t c0 = colptr[v], deg = colptr[v + 1] - c0;
  const int64_t o = offsets[i];
  if (fanout < 0 || fanout >= deg) {
    for (int64_t e = lane; e < deg; e += 64) {
      cand[o + e] = row[c0 + e];
      cand_edge[o + e] = c0 + e;
      cand_dst[o + e] = base + i;
    }
    return;
  }
  int64_t mine[kSlots];
#pragma unroll
  for (int r = 0; r < kSlots; ++r) mine[r] = -1;
  for (int64_t j = deg - fanout, q = 0; j < deg; ++j, ++q) {
    int64_t t = draw(seed, v, j, j + 1);
    bool hit = false;
#pragma unroll
    for (int r = 0; r < kSlots; ++r) hit |= mine[r] == t;
    if (__any(hit)) t = j;  // wave-uniform
#pragma unroll
    for (int r = 0; r < kSlots; ++r)
      if (q == r * 64 + lane) mine[r] = t;
    if (lane == 0) {
      cand[o + q] = row[c0 + t];
      cand_edge[o + q] = c0 + t;
      cand_dst[o + q] = base + i;
    }
  }
}

__global__ __launch_bounds__(kT) void first_kernel(int64_t nc, const int64_t *__restrict__ cand,
                                                   const int64_t *__restrict__ local,
                                                   unsigned long long *__restrict__ first) {
  const int64_t p = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (p >= nc) return;
  const int64_t v = cand[p];
  if (local[v] < 0) atomicMin(first + v, (unsigned long long)p);
}

__global__ __launch_bounds__(kT) void flag_kernel(int64_t nc, const int64_t *__restrict__ cand,
                                                  const int64_t *__restrict__ local,
                                                  const unsigned long long *__restrict__ first,
                                                  int64_t *__restrict__ flag) {
  const int64_t p = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (p >= nc) return;
  const int64_t v = cand[p];
  flag[p] = (local[v] < 0 && first[v] == (unsigned long long)p) ? 1 : 0;
}

// rank = exclusive scan of flag ([nc + 1]); the new node's slot in this
// hop's chunk is rank[p], its local id base + rank[p]
__global__ __launch_bounds__(kT) void assign_kernel(int64_t nc, int64_t base, const int64_t *__restrict__ cand,
                                                    const int64_t *__restrict__ flag,
                                                    const int64_t *__restrict__ rank, int64_t *__restrict__ nodes,
                                                    int64_t *__restrict__ local,
                                                    unsigned long long *__restrict__ first) {
  const int64_t p = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (p >= nc) return;
  const int64_t v = cand[p];
  if (flag[p]) {
    nodes[rank[p]] = v;
    local[v] = base + rank[p];
  }
  first[v] = ~0ull;
}

__global__ __launch_bounds__(kT) void cand_local_kernel(int64_t nc, const int64_t *__restrict__ cand,
                                                        const int64_t *__restrict__ local,
                                                        int64_t *__restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (p < nc) out[p] = local[cand[p]];
}

// One wave per sampled node: number of in-edges whose source is sampled.
__global__ __launch_bounds__(kT) void induced_count_kernel(int64_t ns, const int64_t *__restrict__ nodes,
                                                           const int64_t *__restrict__ colptr,
                                                           const int64_t *__restrict__ row,
                                                           const int64_t *__restrict__ local,
                                                           int64_t *__restrict__ counts) {
  const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int64_t i = (int64_t)blockIdx.x * (kT / 64) + wv;
  if (i >= ns) return;
  const int64_t v = nodes[i];
  const int64_t c0 = colptr[v], c1 = colptr[v + 1];
  int64_t cnt = 0;
  for (int64_t e = c0 + lane; e - lane < c1; e += 64) {
    const bool in = e < c1 && local[row[e]] >= 0;
    cnt += __popcll(__ballot(in));
  }
  if (lane == 0) counts[i] = cnt;
}

// Ordered compaction per wave (ballot + mbcnt): CSC order is kept.
__global__ __launch_bounds__(kT) void induced_fill_kernel(int64_t ns, const int64_t *__restrict__ nodes,
                                                          const int64_t *__restrict__ colptr,
                                                          const int64_t *__restrict__ row,
                                                          const int64_t *__restrict__ local,
                                                          const int64_t *__restrict__ offsets,
                                                          int64_t *__restrict__ out_row, int64_t *__restrict__ out_col,
                                                          int64_t *__restrict__ out_edge) {
  const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int64_t i = (int64_t)blockIdx.x * (kT / 64) + wv;
  if (i >= ns) return;
  const int64_t v = nodes[i];
  const int64_t c0 = colptr[v], c1 = colptr[v + 1];
  int64_t o = offsets[i];
  for (int64_t e = c0 + lane; e - lane < c1; e += 64) {
    const int64_t lu = e < c1 ? local[row[e]] : -1;
    const bool in = lu >= 0;
    const uint64_t mask = __ballot(in);
    const int before = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
    if (in) {
      out_row[o + before] = lu;
      out_col[o + before] = i;
      out_edge[o + before] = e;
    }
    o += __popcll(mask);
  }
}

__global__ __launch_bounds__(kT) void reset_kernel(int64_t ns, const int64_t *__restrict__ nodes,
                                                   int64_t *__restrict__ local) {
  const int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x;
  if (i < ns) local[nodes[i]] = -1;
}

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" int64_t lpg_scan_i64_workspace_bytes(int64_t n) {
  if (n < 0) return -1;
  size_t bytes = 0;
  if (rocprim::inclusive_scan(nullptr, bytes, (const int64_t *)nullptr, (int64_t *)nullptr, (size_t)n,
                              rocprim::plus<int64_t>()) != hipSuccess)
    return -1;
  return (int64_t)bytes;
}

extern "C" lpg_status lpg_scan_i64(const int64_t *in, int64_t n, int64_t *out, void *workspace,
                                   int64_t workspace_bytes, void *stream) {
  LPG_REQUIRE(n >= 0 && out, "lpg_scan_i64: bad arguments");
  hipStream_t s = as_stream(stream);
  LPG_HIP(hipMemsetAsync(out, 0, sizeof(int64_t), s));
  if (n == 0) return LPG_OK;
  LPG_REQUIRE(in && workspace, "lpg_scan_i64: NULL pointer");
  size_t bytes = (size_t)workspace_bytes;
  LPG_HIP(rocprim::inclusive_scan(workspace, bytes, in, out + 1, (size_t)n, rocprim::plus<int64_t>(), s));
  return LPG_OK;
}

extern "C" lpg_status lpg_sample_count(const int64_t *frontier, int64_t nf, const int64_t *colptr, int64_t fanout,
                                       int64_t *counts, void *stream) {
  LPG_REQUIRE(nf >= 0, "lpg_sample_count: nf < 0");
  LPG_REQUIRE(fanout <= kMaxFanout, "lpg_sample_count: fanout %lld > %d", (long long)fanout, kMaxFanout);
  if (nf == 0) return LPG_OK;
  LPG_REQUIRE(frontier && colptr && counts, "lpg_sample_count: NULL pointer");
  hipLaunchKernelGGL(count_kernel, dim3(blocks_for(nf)), dim3(kT), 0, as_stream(stream), nf, frontier, colptr, fanout,
                     counts);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_sample_fill(const int64_t *frontier, int64_t nf, int64_t base, const int64_t *colptr,
                                      const int64_t *row, int64_t fanout, uint64_t seed, const int64_t *offsets,
                                      int64_t *cand, int64_t *cand_edge, int64_t *cand_dst, void *stream) {
  LPG_REQUIRE(nf >= 0 && fanout <= kMaxFanout, "lpg_sample_fill: bad nf / fanout");
  if (nf == 0) return LPG_OK;
  LPG_REQUIRE(frontier && colptr && row && offsets && cand && cand_edge && cand_dst, "lpg_sample_fill: NULL pointer");
  hipLaunchKernelGGL(fill_kernel, dim3(blocks_for(nf, kT / 64)), dim3(kT), 0, as_stream(stream), nf, base, frontier,
                     colptr, row, fanout, seed, offsets, cand, cand_edge, cand_dst);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_sample_dedupe(const int64_t *cand, int64_t nc, const int64_t *local, uint64_t *first,
                                        int64_t *flag, void *stream) {
  LPG_REQUIRE(nc >= 0, "lpg_sample_dedupe: nc < 0");
  if (nc == 0) return LPG_OK;
  LPG_REQUIRE(cand && local && first && flag, "lpg_sample_dedupe: NULL pointer");
  hipStream_t s = as_stream(stream);
  auto *f = reinterpret_cast<unsigned long long *>(first);
  hipLaunchKernelGGL(first_kernel, dim3(blocks_for(nc)), dim3(kT), 0, s, nc, cand, local, f);
  hipLaunchKernelGGL(flag_kernel, dim3(blocks_for(nc)), dim3(kT), 0, s, nc, cand, local, f, flag);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_sample_assign(const int64_t *cand, int64_t nc, int64_t base, const int64_t *flag,
                                        const int64_t *rank, int64_t *nodes, int64_t *local, uint64_t *first,
                                        void *stream) {
  LPG_REQUIRE(nc >= 0 && base >= 0, "lpg_sample_assign: bad sizes");
  if (nc == 0) return LPG_OK;
  LPG_REQUIRE(cand && flag && rank && nodes && local && first, "lpg_sample_assign: NULL pointer");
  hipLaunchKernelGGL(assign_kernel, dim3(blocks_for(nc)), dim3(kT), 0, as_stream(stream), nc, base, cand, flag, rank,
                     nodes, local, reinterpret_cast<unsigned long long *>(first));
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_sample_local_ids(const int64_t *cand, int64_t nc, const int64_t *local, int64_t *out,
                                           void *stream) {
  LPG_REQUIRE(nc >= 0, "lpg_sample_local_ids: nc < 0");
  if (nc == 0) return LPG_OK;
  LPG_REQUIRE(cand && local && out, "lpg_sample_local_ids: NULL pointer");
  hipLaunchKernelGGL(cand_local_kernel, dim3(blocks_for(nc)), dim3(kT), 0, as_stream(stream), nc, cand, local, out);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_induced_count(const int64_t *nodes, int64_t ns, const int64_t *colptr, const int64_t *row,
                                        const int64_t *local, int64_t *counts, void *stream) {
  LPG_REQUIRE(ns >= 0, "lpg_induced_count: ns < 0");
  if (ns == 0) return LPG_OK;
  LPG_REQUIRE(nodes && colptr && row && local && counts, "lpg_induced_count: NULL pointer");
  hipLaunchKernelGGL(induced_count_kernel, dim3(blocks_for(ns, kT / 64)), dim3(kT), 0, as_stream(stream), ns, nodes,
                     colptr, row, local, counts);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_induced_fill(const int64_t *nodes, int64_t ns, const int64_t *colptr, const int64_t *row,
                                       const int64_t *local, const int64_t *offsets, int64_t *out_row,
                                       int64_t *out_col, int64_t *out_edge, void *stream) {
  LPG_REQUIRE(ns >= 0, "lpg_induced_fill: ns < 0");
  if (ns == 0) return LPG_OK;
  LPG_REQUIRE(nodes && colptr && row && local && offsets && out_row && out_col && out_edge,
              "lpg_induced_fill: NULL pointer");
  hipLaunchKernelGGL(induced_fill_kernel, dim3(blocks_for(ns, kT / 64)), dim3(kT), 0, as_stream(stream), ns, nodes,
                     colptr, row, local, offsets, out_row, out_col, out_edge);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_sample_reset(const int64_t *nodes, int64_t ns, int64_t *local, void *stream) {
  LPG_REQUIRE(ns >= 0, "lpg_sample_reset: ns < 0");
  if (ns == 0) return LPG_OK;
  LPG_REQUIRE(nodes && local, "lpg_sample_reset: NULL pointer");
  hipLaunchKernelGGL(reset_kernel, dim3(blocks_for(ns)), dim3(kT), 0, as_stream(stream), ns, nodes, local);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}
