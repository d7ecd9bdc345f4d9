// Basis labels from per-node logits: inference_gnn (val.py:106-124), the post-processing of the
// reference's one timed GNN path (scripts/pred_basis.py:113-118, 169-173):
//
//   P = softmax(logits) (NaN -> 0); the m nodes with the largest P[:, 1] are basic (label 1);
//   every other node takes argmax(P[i, 0], P[i, 2]) -> 0 or 2 (0 on a tie: argmax's first maximum).
//
// torch's topk(m) over 300 K values (k = 100 K) sorts; here the m-th largest P[:, 1] is found by a
// three-pass radix select on the float bits (P[:, 1] >= 0, so the bits order like the values):
// 12 + 12 + 8 bits, one LDS histogram per block per pass merged with integer atomics (exact, the
// same counts whatever the order).  Every block of a pass re-derives the previous passes' bin
// choice from the merged histogram (a 4096-bin suffix scan, a few microseconds), block 0 records it
// for the later kernels.  Nodes above the threshold value are basic; of the nodes equal to it, the
// lowest indices are taken (torch.topk leaves that choice unspecified: per-block tie counts, a
// one-block scan, a ballot prefix inside the block).  Six launches, no host synchronisation,
// deterministic.
#include "common.h"

namespace lpg {
namespace {

constexpr int kBT = 256;     // threads per block, one node per thread
constexpr int kB1 = 4096;    // pass-1 bins: key bits 31..20
constexpr int kB2 = 4096;    // pass-2 bins: key bits 19..8
constexpr int kB3 = 256;     // pass-3 bins: key bits 7..0

struct SelState {  // written by block 0 of each pass
  uint32_t b1, b2, thr;
  int64_t need1, need2, need_eq;
};

// workspace: [SelState (64 B)] [h1 kB1 u32] [h2 kB2 u32] [h3 kB3 u32] [keys total u32] [ties nblocks u32]
// [side total u8]
struct Ws {
  SelState *st;
  uint32_t *h1, *h2, *h3, *keys, *ties;
  uint8_t *side;
};

__host__ __device__ inline Ws carve(void *w, int64_t total) {
  unsigned char *p = reinterpret_cast<unsigned char *>(w);
  Ws r;
  r.st = reinterpret_cast<SelState *>(p);
  p += 64;
  r.h1 = reinterpret_cast<uint32_t *>(p);
  r.h2 = r.h1 + kB1;
  r.h3 = r.h2 + kB2;
  r.keys = r.h3 + kB3;
  r.ties = r.keys + total;
  const int64_t nb = (total + kBT - 1) / kBT;
  r.side = reinterpret_cast<uint8_t *>(r.ties + nb);
  return r;
}

int64_t ws_bytes(int64_t total) {
  const int64_t nb = (total + kBT - 1) / kBT;
  return 64 + 4 * (kB1 + kB2 + kB3) + 4 * total + 4 * nb + total + 16;
}

// the bin holding the `need`-th largest key (need >= 1) of a histogram with `nbins` bins (bins ordered
// like the keys), and how many keys of that bin are still needed; every thread gets the answer
__device__ void select_bin(const uint32_t *__restrict__ h, int nbins, int64_t need, uint32_t &bin, int64_t &rest) {
  __shared__ int64_t sc[kBT];
  __shared__ uint32_t s_bin;
  __shared__ int64_t s_rest;
  const int t = threadIdx.x, per = nbins / kBT;
  int64_t local = 0;
  for (int i = 0; i < per; ++i) local += h[t * per + i];
  // above[t] = sum over threads t' > t (inclusive scan over the reversed thread order, then shifted)
  const int r = kBT - 1 - t;
  sc[r] = local;
  __syncthreads();
  for (int o = 1; o < kBT; o <<= 1) {
    const int64_t v = r >= o ? sc[r - o] : 0;
    __syncthreads();
    sc[r] += v;
    __syncthreads();
  }
  const int64_t above = sc[r] - local;
  if (above < need && need <= above + local) {
    int64_t acc = above;
    for (int i = per - 1; i >= 0; --i) {
      const int64_t c = h[t * per + i];
      if (acc + c >= need) {
        s_bin = (uint32_t)(t * per + i);
        s_rest = need - acc;
        break;
      }
      acc += c;
    }
  }
  __syncthreads();
  bin = s_bin;
  rest = s_rest;
}

// LDS histogram of (key >> shift) & (nbins - 1) over the keys whose bits above `shift + log2(nbins)`
// equal `prefix` (match_shift = 32: every key), merged into h with integer atomics (non-empty bins only)
__device__ void block_hist(const uint32_t *__restrict__ keys, int64_t total, int shift, int nbins, int match_shift,
                           uint32_t prefix, uint32_t *__restrict__ h) {
  __shared__ uint32_t lh[kB1];
  for (int i = threadIdx.x; i < nbins; i += kBT) lh[i] = 0u;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kBT + threadIdx.x;
  if (i < total) {
    const uint32_t k = keys[i];
    if (match_shift >= 32 || (k >> match_shift) == prefix) atomicAdd(&lh[(k >> shift) & (uint32_t)(nbins - 1)], 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbins; b += kBT)
    if (lh[b]) atomicAdd(&h[b], lh[b]);
}

// F16: fp16 logits (the reference's --fp16 inference): softmax computed in fp32 and rounded to fp16,
// as torch's half softmax stores it; the selection and the argmax then see the fp16 probabilities
// (ties among them go to the lower index / to class 0, torch.argmax's first maximum)
template <bool F16>
__global__ __launch_bounds__(kBT) void basis_keys(int64_t total, const void *__restrict__ logits_v, int64_t ldl,
                                                  Ws w) {
  const int64_t i = (int64_t)blockIdx.x * kBT + threadIdx.x;
  if (i < total) {
    float x0, x1, x2;
    if constexpr (F16) {
      const uint16_t *x = static_cast<const uint16_t *>(logits_v) + i * ldl;
      x0 = (float)__builtin_bit_cast(_Float16, x[0]);
      x1 = (float)__builtin_bit_cast(_Float16, x[1]);
      x2 = (float)__builtin_bit_cast(_Float16, x[2]);
    } else {
      const float *x = static_cast<const float *>(logits_v) + i * ldl;
      x0 = x[0], x1 = x[1], x2 = x[2];
    }
    float mx = x0 > x1 ? x0 : x1;
    mx = x2 > mx ? x2 : mx;
    const float e0 = expf(x0 - mx), e1 = expf(x1 - mx), e2 = expf(x2 - mx);
    const float s = e0 + e1 + e2;
    float p0 = e0 / s, p1 = e1 / s, p2 = e2 / s;
    if constexpr (F16) {
      p0 = (float)(_Float16)p0;
      p1 = (float)(_Float16)p1;
      p2 = (float)(_Float16)p2;
    }
    p0 = p0 != p0 ? 0.f : p0;  // pr[isnan(pr)] = 0
    p1 = p1 != p1 ? 0.f : p1;
    p2 = p2 != p2 ? 0.f : p2;
    w.keys[i] = __float_as_uint(p1) & 0x7fffffffu;  // >= 0 (a -0 would order as +0)
    w.side[i] = p0 >= p2 ? 0 : 2;
  }
  block_hist(w.keys, total, 20, kB1, 32, 0u, w.h1);
}

__global__ __launch_bounds__(kBT) void basis_pass2(int64_t total, int64_t m, Ws w) {
  uint32_t b1;
  int64_t need1;
  select_bin(w.h1, kB1, m, b1, need1);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.st->b1 = b1;
    w.st->need1 = need1;
  }
  block_hist(w.keys, total, 8, kB2, 20, b1, w.h2);
}

__global__ __launch_bounds__(kBT) void basis_pass3(int64_t total, Ws w) {
  const uint32_t b1 = w.st->b1;
  uint32_t b2;
  int64_t need2;
  select_bin(w.h2, kB2, w.st->need1, b2, need2);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.st->b2 = b2;
    w.st->need2 = need2;
  }
  block_hist(w.keys, total, 0, kB3, 8, (b1 << 12) | b2, w.h3);
}

// the threshold value and, per block, how many keys equal it
__global__ __launch_bounds__(kBT) void basis_ties(int64_t total, Ws w) {
  uint32_t b3;
  int64_t need3;
  select_bin(w.h3, kB3, w.st->need2, b3, need3);
  const uint32_t thr = (w.st->b1 << 20) | (w.st->b2 << 8) | b3;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.st->thr = thr;
    w.st->need_eq = need3;
  }
  __shared__ uint32_t cnt;
  if (threadIdx.x == 0) cnt = 0u;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * kBT + threadIdx.x;
  if (i < total && w.keys[i] == thr) atomicAdd(&cnt, 1u);
  __syncthreads();
  if (threadIdx.x == 0) w.ties[blockIdx.x] = cnt;
}

// ties[b] -> the number of threshold ties in the blocks before b (exclusive prefix, in place): one
// block, each thread a contiguous run of blocks
__global__ __launch_bounds__(1024) void basis_tie_scan(int64_t nb, Ws w) {
  __shared__ int64_t sc[1024];
  const int t = threadIdx.x;
  const int64_t per = (nb + 1023) / 1024, b0 = t * per, b1 = b0 + per < nb ? b0 + per : nb;
  int64_t local = 0;
  for (int64_t b = b0; b < b1; ++b) local += w.ties[b];
  sc[t] = local;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int64_t v = t >= o ? sc[t - o] : 0;
    __syncthreads();
    sc[t] += v;
    __syncthreads();
  }
  int64_t run = sc[t] - local;
  for (int64_t b = b0; b < b1; ++b) {
    const uint32_t c = w.ties[b];
    w.ties[b] = (uint32_t)run;  // < 2^31 nodes per call (host check)
    run += c;
  }
}

// labels: 1 above the threshold and for the first need_eq keys equal to it (by node index), else the
// argmax over {0, 2}.  With `select` false (m = 0) no node is basic.
__global__ __launch_bounds__(kBT) void basis_labels(int64_t total, int32_t select, Ws w, int64_t *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * kBT + threadIdx.x;
  const uint32_t thr = select ? w.st->thr : 0xffffffffu;
  const int64_t need_eq = select ? w.st->need_eq : 0;
  const uint32_t k = i < total ? w.keys[i] : 0u;
  const bool eq = select && i < total && k == thr;
  __shared__ uint32_t wcnt[kBT / 64];
  const uint64_t bal = __ballot(eq);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) wcnt[wv] = (uint32_t)__popcll(bal);
  __syncthreads();
  int64_t rank = (select ? (int64_t)w.ties[blockIdx.x] : 0) + (int64_t)__popcll(bal & ((1ull << lane) - 1ull));
  for (int v = 0; v < wv; ++v) rank += wcnt[v];
  if (i < total) out[i] = (select && (k > thr || (eq && rank < need_eq))) ? 1 : (int64_t)w.side[i];
}

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" int64_t lpg_basis_labels_workspace_bytes(int64_t total) { return total < 0 ? 0 : ws_bytes(total); }

template <bool F16>
static lpg_status basis_labels(int64_t total, int64_t m, const void *logits, int64_t ldl, int64_t *labels,
                                           void *workspace, void *stream) {
  LPG_REQUIRE(total >= 0 && m >= 0 && m <= total, "lpg_basis_labels: need 0 <= m <= total (m %lld, total %lld)",
              (long long)m, (long long)total);
  if (total == 0) return LPG_OK;
  LPG_REQUIRE(logits && labels && workspace && ldl >= 3, "lpg_basis_labels: NULL pointer or ldl < 3");
  LPG_REQUIRE(aligned16(workspace), "lpg_basis_labels: workspace not 16-byte aligned");
  LPG_REQUIRE(total < ((int64_t)1 << 31), "lpg_basis_labels: too many nodes");
  hipStream_t s = as_stream(stream);
  const Ws w = carve(workspace, total);
  const unsigned nb = (unsigned)((total + kBT - 1) / kBT);
  LPG_HIP(hipMemsetAsync(w.h1, 0, 4 * (kB1 + kB2 + kB3), s));
  hipLaunchKernelGGL(basis_keys<F16>, dim3(nb), dim3(kBT), 0, s, total, logits, ldl, w);
  if (m > 0) {
    hipLaunchKernelGGL(basis_pass2, dim3(nb), dim3(kBT), 0, s, total, m, w);
    hipLaunchKernelGGL(basis_pass3, dim3(nb), dim3(kBT), 0, s, total, w);
    hipLaunchKernelGGL(basis_ties, dim3(nb), dim3(kBT), 0, s, total, w);
    hipLaunchKernelGGL(basis_tie_scan, dim3(1), dim3(1024), 0, s, (int64_t)nb, w);
  }
  hipLaunchKernelGGL(basis_labels, dim3(nb), dim3(kBT), 0, s, total, (int32_t)(m > 0), w, labels);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_basis_labels_f32(int64_t total, int64_t m, const float *logits, int64_t ldl, int64_t *labels,
                                           void *workspace, void *stream) {
  return basis_labels<false>(total, m, logits, ldl, labels, workspace, stream);
}

// inference_gnn on fp16 logits (val.py:106-124 under the reference's --fp16: a half softmax); same
// workspace as lpg_basis_labels_f32
extern "C" lpg_status lpg_basis_labels_f16(int64_t total, int64_t m, const uint16_t *logits, int64_t ldl,
                                           int64_t *labels, void *workspace, void *stream) {
  return basis_labels<true>(total, m, logits, ldl, labels, workspace, stream);
}
