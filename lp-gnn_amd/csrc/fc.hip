// Dense per-node FC of GraphConv on fp32 MFMA (gfx950), fused:
//
//   C[m, n] = act( sum_{k<K1} A1[m,k] W1[n,k] + sum_{k<K2} A2[m,k] W2[n,k] + bias[n] )
//
// = PyG 2.1 GraphConv.forward after propagate:  lin_rel(agg) + lin_root(x_dst)
// (arch.py:57-62, 75-80) with the ReLU of arch.py:182/188 as the epilogue,
// and -- with K2 = 0, no ReLU -- the heads lin_left / lin_right (arch.py:190).
// The concat [agg | x_dst] is never materialised: the k loop walks A1 then A2.
//
// Numerics (the parity contract, mirrored by oracle/fc_ref.c): blocked k
// order.  Each part (A1, W1) over K1, then (A2, W2) over K2, is cut into
// k-tiles of BK = 32 (the last one zero-padded: fma(0, 0, p) = p exactly);
// a tile's products form ONE fp32 fma chain in k order from +0 --
// v_mfma_f32_32x32x2_f32 is bit-for-bit such a chain, k0 then k1 of each
// pair (MI355X_MICROARCH.md §Matrix cores) -- and the tile sums are added in
// tile order into the running total (+0 initially); then + bias, then ReLU
// as (v < 0 ? 0 : v).  The blocking keeps the rounding error at the level
// of MKL's blocked sgemm (~(32 + K/32) ulps worst case instead of K).
//
// Tiling: 256 threads = 4 waves; BM x BN output tile, BK = 32; A and W tiles
// staged global -> registers -> LDS ([row][BK+1] fp32, conflict-free column
// reads), double-buffered with one barrier per k-tile; each wave owns
// TM x TN blocks of 32x32 (16 accumulator VGPRs each).  Blocks are remapped
// so that each XCD walks a contiguous range of m-tiles with all their
// n-tiles (the A panel is then re-read from that XCD's L2).
#include "common.h"

#pragma clang fp contract(off)

namespace lpg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int NB = 32;  // numerics block: k-tile length of one fma chain (the parity contract)

struct FcArgs {
  int64_t M, N, K1, K2;
  const float *A1, *A2, *W1, *W2, *bias;
  int64_t lda1, lda2, ldw1, ldw2;
  float *C;
  int64_t ldc;
  int64_t mt, nt;  // tiles
  // fused dropout (after the ReLU): keep element (row, col) iff
  // hash(seed, row * N + col) >= drop_thresh; kept values are scaled.
  uint64_t seed;
  uint32_t drop_thresh;  // 0 = no dropout
  float drop_scale;
  // flags bit 1: C holds an addend on entry, C = act(A1 W1^T + A2 W2^T + C + bias);
  // each element is read and rewritten by the lane that owns it
  int32_t accum;
};

// Counter-based dropout RNG over (seed, row, col): two rounds of the 32-bit
// "lowbias32" integer hash, the inner one keyed by the row only (so a lane
// reuses it across its columns).  Stateless, so the backward pass never needs
// the mask (the kept set is exactly where the stored output is > 0).  32-bit
// on purpose: 64-bit multiplies are multi-instruction on CDNA and made the
// epilogue ~10% of a hidden-layer FC.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, int64_t row, int64_t col) {
  const uint32_t hr = lowbias32((uint32_t)row ^ (uint32_t)seed);
  return lowbias32(hr ^ ((uint32_t)col * 0x9e3779b9u) ^ (uint32_t)(seed >> 32));
}

__device__ __forceinline__ float epilogue(const FcArgs &a, float v, float b, int64_t row, int64_t col, bool relu) {
  if (a.bias) v = v + b;
  if (relu) v = (v < 0.f) ? 0.f : v;
  if (a.drop_thresh) v = drop_hash(a.seed, row, col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
  return v;
}

// Branch-free load of 4 consecutive k of row r of X (R rows, K columns):
// the address is clamped into range.  Rows >= R only feed outputs that are
// never stored, so they are left as whatever row R-1 holds; k >= K is zeroed
// later (sstore), only in the partial last k-tile of a phase.  (A conditional
// load -- or a select right after it -- makes hipcc wait vmcnt per load.)
__device__ __forceinline__ float4 load_k4(const float *X, int64_t ld, int64_t R, int64_t K, int64_t r, int64_t k) {
  const int64_t rr = r < R ? r : R - 1;
  const int64_t kk = k < K ? k : K - 4;
  return *reinterpret_cast<const float4 *>(X + rr * ld + kk);
}

// flags bit 1 (accumulate): acc[i][j][r] += C at the lane's 32x32-MFMA output
// positions, every load issued before the first store (C is read and then
// rewritten in place, so loads cannot be moved past stores by the compiler).
// Rows/cols past the edge load a clamped in-range element (never stored).
template <int TM, int TN, typename Acc>
__device__ __forceinline__ void add_c32(const FcArgs &a, Acc (&acc)[TM][TN], int64_t mw, int64_t nw, int lane) {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int64_t col = nw + j * 32 + (lane & 31);
    col = col < a.N ? col : a.N - 1;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int64_t row = mw + i * 32 + 4 * (lane >> 5) + (r & 3) + 8 * (r >> 2);
        row = row < a.M ? row : a.M - 1;
        acc[i][j][r] = acc[i][j][r] + a.C[row * a.ldc + col];
      }
  }
}

// WAVES_M x WAVES_N waves, each owning TM x TN blocks of 32x32; BK = staging
// k-tile (a multiple of the numerics block NB; chains restart every NB).
template <int WAVES_M, int WAVES_N, int TM, int TN, int BK, bool RELU>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void fc_fwd_f32(FcArgs a) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int BM = WAVES_M * TM * 32;
  constexpr int BN = WAVES_N * TN * 32;
  constexpr int LDK = BK + 1;
  constexpr int C4 = BK / 4;         // float4 chunks per staged row
  constexpr int LA = BM * C4 / NT;  // float4 loads per thread per k-tile
  constexpr int LB = BN * C4 / NT;
  static_assert(BK % NB == 0, "BK must be a multiple of NB");
  static_assert(LA >= 1 && LB >= 1 && BM * C4 % NT == 0 && BN * C4 % NT == 0, "tile/thread mismatch");
  __shared__ float smem[2 * (BM + BN) * LDK];
  // buffer b: A tile at smem + b*(BM+BN)*LDK, W tile right after it
  auto As = [&](int b) { return smem + b * (BM + BN) * LDK; };
  auto Bs = [&](int b) { return smem + b * (BM + BN) * LDK + BM * LDK; };

  // XCD-aware bijective remap of the 1-D grid.
  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  // Two uniform phases of k-tiles: (A1, W1) over K1, then (A2, W2) over K2,
  // each zero-padded to a multiple of BK (zeros are exact no-ops in the chain).
  const int nk1 = (int)((a.K1 + BK - 1) / BK);
  const int nk = nk1 + (int)((a.K2 + BK - 1) / BK);

  // acc: running total over k-tiles; each k-tile's 32 products are summed
  // in their own chain (part, from +0) and then added to acc in tile order.
  f32x16 acc[TM][TN];
  const f32x16 zero = {};
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero;

  float4 ra[LA], rb[LB];
  auto gload = [&](int t) {
    const bool p2 = t >= nk1;  // wave-uniform phase select
    const float *A = p2 ? a.A2 : a.A1;
    const float *W = p2 ? a.W2 : a.W1;
    const int64_t lda = p2 ? a.lda2 : a.lda1, ldw = p2 ? a.ldw2 : a.ldw1, Kp = p2 ? a.K2 : a.K1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BK;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + NT * i;
      ra[i] = load_k4(A, lda, a.M, Kp, m0 + idx / C4, k0 + (idx % C4) * 4);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + NT * i;
      rb[i] = load_k4(W, ldw, a.N, Kp, n0 + idx / C4, k0 + (idx % C4) * 4);
    }
  };
  auto sstore = [&](int buf, int t) {
    const bool p2 = t >= nk1;
    const int64_t Kp = p2 ? a.K2 : a.K1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BK;
    if (k0 + BK > Kp) {  // wave-uniform: partial k-tile, zero k >= Kp in both operands
#pragma unroll
      for (int i = 0; i < LA; ++i)
        if (k0 + ((tid + NT * i) % C4) * 4 >= Kp) ra[i] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < LB; ++i)
        if (k0 + ((tid + NT * i) % C4) * 4 >= Kp) rb[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + NT * i;
      float *p = As(buf) + (idx / C4) * LDK + (idx % C4) * 4;
      p[0] = ra[i].x; p[1] = ra[i].y; p[2] = ra[i].z; p[3] = ra[i].w;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + NT * i;
      float *p = Bs(buf) + (idx / C4) * LDK + (idx % C4) * 4;
      p[0] = rb[i].x; p[1] = rb[i].y; p[2] = rb[i].z; p[3] = rb[i].w;
    }
  };

  gload(0);
  sstore(0, 0);
  __syncthreads();
  const int fr = lane & 31, fk = lane >> 5;
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    if (t + 1 < nk) gload(t + 1);
    const float *Ab = As(buf) + (wm * TM * 32 + fr) * LDK + fk;
    const float *Bb = Bs(buf) + (wn * TN * 32 + fr) * LDK + fk;
    f32x16 part[TM][TN];
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = Ab[i * 32 * LDK + 2 * s];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = Bb[j * 32 * LDK + 2 * s];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], s % (NB / 2) == 0 ? zero : part[i][j],
                                                             0, 0, 0);
      if (s % (NB / 2) == NB / 2 - 1) {  // end of a numerics block: fold into the total
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = acc[i][j] + part[i][j];
      }
    }
    if (t + 1 < nk) sstore(buf ^ 1, t + 1);
    __syncthreads();
  }

  // Epilogue: C/D map of the 32x32 MFMA: col = lane & 31,
  // row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5).
  if (a.accum) add_c32<TM, TN>(a, acc, m0 + wm * TM * 32, n0 + wn * TN * 32, lane);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
    if (col >= a.N) continue;
    const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t rbase = m0 + wm * TM * 32 + i * 32 + 4 * (lane >> 5);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < a.M) a.C[row * a.ldc + col] = epilogue(a, acc[i][j][r], b, row, col, RELU);
      }
    }
  }
}

// Same contract on v_mfma_f32_16x16x4_f32 (lane l: A[l&15][k = l>>4],
// B[k = l>>4][l&15]; C/D col = l&15, row = 4*(l>>4) + r).  The staged tiles
// are stored k-permuted inside each 32-wide k-block -- position (k&3)*8 + k/4,
// rows padded to 36 floats -- so one conflict-free ds_read_b128 gives a lane
// its operand for 4 consecutive MFMA k-steps.  Chains and block sums are the
// same as fc_fwd_f32 (bitwise identical results).
template <int WAVES_M, int WAVES_N, int TM, int TN, bool RELU>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void fc_fwd_f32_m16(FcArgs a) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int BM = WAVES_M * TM * 16;
  constexpr int BN = WAVES_N * TN * 16;
  constexpr int BKs = 32;            // staging k-tile = one numerics block
  constexpr int LDK = 36;            // padded row (floats), 16-B aligned
  constexpr int C4 = BKs / 4;
  constexpr int LA = BM * C4 / NT;
  constexpr int LB = BN * C4 / NT;
  static_assert(LA >= 1 && LB >= 1 && BM * C4 % NT == 0 && BN * C4 % NT == 0, "tile/thread mismatch");
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDK];
  auto As = [&](int b) { return smem + b * (BM + BN) * LDK; };
  auto Bs = [&](int b) { return smem + b * (BM + BN) * LDK + BM * LDK; };

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int nk1 = (int)((a.K1 + BKs - 1) / BKs);
  const int nk = nk1 + (int)((a.K2 + BKs - 1) / BKs);

  f32x4v acc[TM][TN];
  const f32x4v zero = {};
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero;

  float4 ra[LA], rb[LB];
  auto gload = [&](int t) {
    const bool p2 = t >= nk1;
    const float *A = p2 ? a.A2 : a.A1;
    const float *W = p2 ? a.W2 : a.W1;
    const int64_t lda = p2 ? a.lda2 : a.lda1, ldw = p2 ? a.ldw2 : a.ldw1, Kp = p2 ? a.K2 : a.K1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BKs;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int idx = tid + NT * i;
      ra[i] = load_k4(A, lda, a.M, Kp, m0 + idx / C4, k0 + (idx % C4) * 4);
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int idx = tid + NT * i;
      rb[i] = load_k4(W, ldw, a.N, Kp, n0 + idx / C4, k0 + (idx % C4) * 4);
    }
  };
  // k = 4c + h  ->  position h*8 + c
  auto put = [&](float *base, int idx, const float4 &v) {
    float *p = base + (idx / C4) * LDK + (idx % C4);
    p[0] = v.x; p[8] = v.y; p[16] = v.z; p[24] = v.w;
  };
  auto sstore = [&](int buf, int t) {
    const bool p2 = t >= nk1;
    const int64_t Kp = p2 ? a.K2 : a.K1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BKs;
    if (k0 + BKs > Kp) {
#pragma unroll
      for (int i = 0; i < LA; ++i)
        if (k0 + ((tid + NT * i) % C4) * 4 >= Kp) ra[i] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < LB; ++i)
        if (k0 + ((tid + NT * i) % C4) * 4 >= Kp) rb[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < LA; ++i) put(As(buf), tid + NT * i, ra[i]);
#pragma unroll
    for (int i = 0; i < LB; ++i) put(Bs(buf), tid + NT * i, rb[i]);
  };

  gload(0);
  sstore(0, 0);
  __syncthreads();
  const int fr = lane & 15, fh = lane >> 4;
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    if (t + 1 < nk) gload(t + 1);
    const float *Ab = As(buf) + (wm * TM * 16 + fr) * LDK + fh * 8;
    const float *Bb = Bs(buf) + (wn * TN * 16 + fr) * LDK + fh * 8;
    f32x4v part[TM][TN];
#pragma unroll
    for (int half = 0; half < 2; ++half) {  // k-steps 4*half .. 4*half+3 of this block
      f32x4v av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = *reinterpret_cast<const f32x4v *>(Ab + i * 16 * LDK + 4 * half);
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = *reinterpret_cast<const f32x4v *>(Bb + j * 16 * LDK + 4 * half);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            part[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][u], bv[j][u],
                                                             (half == 0 && u == 0) ? zero : part[i][j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = acc[i][j] + part[i][j];
    if (t + 1 < nk) sstore(buf ^ 1, t + 1);
    __syncthreads();
  }

  if (a.accum) {  // addends first, all loads in flight before the first store
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int64_t col = n0 + wn * TN * 16 + j * 16 + (lane & 15);
      col = col < a.N ? col : a.N - 1;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int64_t row = m0 + wm * TM * 16 + i * 16 + 4 * (lane >> 4) + r;
          row = row < a.M ? row : a.M - 1;
          acc[i][j][r] = acc[i][j][r] + a.C[row * a.ldc + col];
        }
    }
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = n0 + wn * TN * 16 + j * 16 + (lane & 15);
    if (col >= a.N) continue;
    const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t rbase = m0 + wm * TM * 16 + i * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = rbase + r;
        if (row < a.M) a.C[row * a.ldc + col] = epilogue(a, acc[i][j][r], b, row, col, RELU);
      }
    }
  }
}

// add_knowledge for one side (arch.py:129-141), bitwise torch-CPU semantics:
//   n = sqrt(fma(x2, x2, fma(x1, x1, x0 * x0)))      (torch.linalg.vector_norm, CPU)
//   y = x / max(n, 1e-12) * 10                          (F.normalize(x) * 10)
//   y0 -= bound where feas[:, -3] != 0;  y2 -= bound where feas[:, -1] != 0
__global__ __launch_bounds__(256) void knowledge_f32(int64_t M, const float *__restrict__ logit, int64_t ldl,
                                                     const float *__restrict__ feas, int64_t ldf, int64_t fcols,
                                                     float bound, float *__restrict__ out, int64_t ldo) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const float x0 = logit[m * ldl], x1 = logit[m * ldl + 1], x2 = logit[m * ldl + 2];
  const float nrm = sqrtf(__builtin_fmaf(x2, x2, __builtin_fmaf(x1, x1, x0 * x0)));
  const float d = nrm < 1e-12f ? 1e-12f : nrm;
  float y0 = x0 / d * 10.f, y1 = x1 / d * 10.f, y2 = x2 / d * 10.f;
  if (feas[m * ldf + fcols - 3] != 0.f) y0 = y0 - bound;
  if (feas[m * ldf + fcols - 1] != 0.f) y2 = y2 - bound;
  out[m * ldo] = y0;
  out[m * ldo + 1] = y1;
  out[m * ldo + 2] = y2;
}

// dZ = (Y > 0) ? g * scale : 0 -- backward of ReLU followed by dropout
// (Y is the stored post-dropout output, so Y > 0 <=> kept and ReLU-active).
__global__ __launch_bounds__(256) void relu_dropout_bwd_f32(int64_t n4, const float4 *__restrict__ g,
                                                            const float4 *__restrict__ y, float scale,
                                                            float4 *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 gv = g[i], yv = y[i];
    float4 o;
    o.x = yv.x > 0.f ? gv.x * scale : 0.f;
    o.y = yv.y > 0.f ? gv.y * scale : 0.f;
    o.z = yv.z > 0.f ? gv.z * scale : 0.f;
    o.w = yv.w > 0.f ? gv.w * scale : 0.f;
    out[i] = o;
  }
}

template <int WM, int WN, int TM, int TN, int BK>
lpg_status launch_fc(const FcArgs &a0, bool relu, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = 64 * WM * WN;
  FcArgs a = a0;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_f32: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_fwd_f32<WM, WN, TM, TN, BK, true>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((fc_fwd_f32<WM, WN, TM, TN, BK, false>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

template <int WM, int WN, int TM, int TN>
lpg_status launch_fc16(const FcArgs &a0, bool relu, hipStream_t s) {
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16, NT = 64 * WM * WN;
  FcArgs a = a0;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_f32: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_fwd_f32_m16<WM, WN, TM, TN, true>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((fc_fwd_f32_m16<WM, WN, TM, TN, false>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// Narrow-input FC (conv1: K1 = K2 = 8 LP features, arch.py:170): the output
// write is the whole cost, so no MFMA tile -- each thread holds the weights of
// 4 output columns in registers and streams rows (A values are block-uniform
// scalar loads).  Same numerics as the tiled kernels: with K1, K2 <= NB each
// part is ONE k-tile, i.e. one fma chain from +0 in k order, the tile sums
// are added into +0 in order, then bias and ReLU -- bitwise identical.
constexpr int kSmallKRows = 64;

template <int K>
__device__ __forceinline__ void load_row_k(float (&x)[K > 0 ? K : 1], const float *A, int64_t ld, int64_t m) {
#pragma unroll
  for (int k = 0; k < K; k += 4) {
    const float4 v = *reinterpret_cast<const float4 *>(A + m * ld + k);
    x[k] = v.x; x[k + 1] = v.y; x[k + 2] = v.z; x[k + 3] = v.w;
  }
}

template <int K1, int K2, bool RELU>
__global__ __launch_bounds__(256) void fc_smallk_f32(FcArgs a) {
  static_assert(K1 % 4 == 0 && K2 % 4 == 0 && K1 >= 4, "small-K kernel: K1, K2 multiples of 4");
  constexpr int KT = K1 + K2;
  // the block's rows of [A1 | A2] staged once in LDS (coalesced), so the row
  // loop never waits on a global load; every lane then reads the same row
  // values (LDS broadcast)
  __shared__ __attribute__((aligned(16))) float sx[kSmallKRows * KT];
  const int64_t r0 = (int64_t)blockIdx.x * kSmallKRows;
  const int64_t r1 = r0 + kSmallKRows < a.M ? r0 + kSmallKRows : a.M;
  for (int i = threadIdx.x; i < kSmallKRows * KT; i += 256) {
    const int r = i / KT, k = i % KT;
    const int64_t m = r0 + r < r1 ? r0 + r : r1 - 1;  // rows past r1 are never stored
    sx[i] = k < K1 ? a.A1[m * a.lda1 + k] : a.A2[m * a.lda2 + (k - K1)];
  }
  __syncthreads();
  const int64_t c = (int64_t)blockIdx.y * 1024 + (int64_t)threadIdx.x * 4;
  if (c >= a.N) return;
  float w1[4][K1], w2[4][K2 > 0 ? K2 : 1], b[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    load_row_k<K1>(w1[j], a.W1, a.ldw1, c + j);
    load_row_k<K2>(w2[j], a.W2, a.ldw2, c + j);
    b[j] = a.bias ? a.bias[c + j] : 0.f;
  }
  f32x2 wp1[2][K1], wp2[2][K2 > 0 ? K2 : 1];  // column pairs (0,1), (2,3), packed once
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
#pragma unroll
    for (int k = 0; k < K1; ++k) wp1[jp][k] = f32x2{w1[2 * jp][k], w1[2 * jp + 1][k]};
#pragma unroll
    for (int k = 0; k < K2; ++k) wp2[jp][k] = f32x2{w2[2 * jp][k], w2[2 * jp + 1][k]};
  }
  for (int64_t m = r0; m < r1; ++m) {
    const float *xr = sx + (m - r0) * KT;
    float o[4];
    // columns in pairs: one v_pk_fma_f32 advances two independent chains
    // (a true fma per element -- the same bits as the scalar chains)
#pragma unroll
    for (int j = 0; j < 4; j += 2) {
      f32x2 p1 = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k < K1; ++k) p1 = __builtin_elementwise_fma(f32x2{xr[k], xr[k]}, wp1[j / 2][k], p1);
      f32x2 t = f32x2{0.f, 0.f} + p1;
      if (K2 > 0) {
        f32x2 p2 = {0.f, 0.f};
#pragma unroll
        for (int k = 0; k < K2; ++k) p2 = __builtin_elementwise_fma(f32x2{xr[K1 + k], xr[K1 + k]}, wp2[j / 2][k], p2);
        t = t + p2;
      }
      if (a.accum) t = t + f32x2{a.C[m * a.ldc + c + j], a.C[m * a.ldc + c + j + 1]};
      o[j] = epilogue(a, t[0], b[j], m, c + j, RELU);
      o[j + 1] = epilogue(a, t[1], b[j + 1], m, c + j + 1, RELU);
    }
    *reinterpret_cast<float4 *>(a.C + m * a.ldc + c) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

template <int K1, int K2>
lpg_status launch_smallk(const FcArgs &a, bool relu, hipStream_t s) {
  const dim3 grid((unsigned)((a.M + kSmallKRows - 1) / kSmallKRows), (unsigned)((a.N + 1023) / 1024));
  if (relu)
    hipLaunchKernelGGL((fc_smallk_f32<K1, K2, true>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((fc_smallk_f32<K1, K2, false>), grid, dim3(256), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// K1, K2 multiples of 4, 4 <= K1, K1 + K2 <= 16; returns false if not covered
bool try_smallk(const FcArgs &a, bool relu, hipStream_t s, lpg_status *st) {
  if (a.K1 < 4 || a.K1 + a.K2 > 16 || a.N % 4 || a.ldc % 4 || !aligned16(a.C)) return false;
  if (a.M >= ((int64_t)1 << 31) * kSmallKRows) return false;
  switch (a.K1 * 100 + a.K2) {
#define LPG_SK(X, Y) case X * 100 + Y: *st = launch_smallk<X, Y>(a, relu, s); return true;
    LPG_SK(4, 0) LPG_SK(4, 4) LPG_SK(4, 8) LPG_SK(4, 12) LPG_SK(8, 0) LPG_SK(8, 4) LPG_SK(8, 8)
    LPG_SK(12, 0) LPG_SK(12, 4) LPG_SK(16, 0)
#undef LPG_SK
  }
  return false;
}

// Same contract staged by global_load_lds (LDS-DMA, no register round trip,
// no ds_write pass): K1, K2 multiples of BK = 32.  LDS image: unpadded
// 128-B rows (32 fp32 of k), 16-B chunk c of row r stored at c ^ ((r >> 1) & 7)
// -- applied on the DMA source address (the DMA destination is lane-linear)
// and on the operand reads.  A wave-instruction moves 8 rows (1 KiB); two
// buffers, one barrier per k-tile, the next tile's DMA in flight under the
// current tile's MFMAs.  Operand reads are ds_read_b32 with a 2-way bank
// conflict (rows r and r+16), one per MFMA.
__device__ __forceinline__ int swz8(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int WAVES_M, int WAVES_N, int TM, int TN, bool RELU>
__global__ __launch_bounds__(64 * WAVES_M * WAVES_N) void fc_fwd_f32_glds(FcArgs a) {
  constexpr int NW = WAVES_M * WAVES_N;
  constexpr int BM = WAVES_M * TM * 32, BN = WAVES_N * TN * 32, BK = 32;
  constexpr int TILE_BYTES = (BM + BN) * BK * 4;
  constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW;
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows must split into whole pieces per wave");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * TILE_BYTES];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);

  // per-lane source rows, clamped once (rows past M / N feed outputs never stored)
  const float *srcA1[PA], *srcA2[PA], *srcW1[PB], *srcW2[PB];
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int row = (wave + NW * p) * 8 + (lane >> 3);
    int64_t gr = m0 + row;
    gr = gr < a.M ? gr : a.M - 1;
    const int off = swz8(row, lane & 7) * 4;
    srcA1[p] = a.A1 + gr * a.lda1 + off;
    srcA2[p] = a.A2 + gr * a.lda2 + off;
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int row = (wave + NW * p) * 8 + (lane >> 3);
    int64_t gn = n0 + row;
    gn = gn < a.N ? gn : a.N - 1;
    const int off = swz8(row, lane & 7) * 4;
    srcW1[p] = a.W1 + gn * a.ldw1 + off;
    srcW2[p] = a.W2 + gn * a.ldw2 + off;
  }
  auto stage = [&](int b, int t) {
    typedef __attribute__((address_space(3))) unsigned char lds_t;
    unsigned char *base = smem + b * TILE_BYTES;
    const bool p2 = t >= nk1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BK;
#pragma unroll
    for (int p = 0; p < PA; ++p)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>((p2 ? srcA2[p] : srcA1[p]) + k0),
                                       (lds_t *)(base + (wave + NW * p) * 1024), 16, 0, 0);
#pragma unroll
    for (int p = 0; p < PB; ++p)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>((p2 ? srcW2[p] : srcW1[p]) + k0),
                                       (lds_t *)(base + BM * BK * 4 + (wave + NW * p) * 1024), 16, 0, 0);
  };

  f32x16 acc[TM][TN];
  const f32x16 zero = {};
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero;

  const int fr = lane & 31, fk = lane >> 5;
  // Tile t-1's sums are folded into acc lazily, block by block, right before
  // tile t's first MFMA overwrites that block's sum register: the fold then
  // sits between MFMAs instead of stalling behind the tile's last one.  Same
  // order as fc_fwd_f32 (acc += tile t-1, then tile t).
  f32x16 part[TM][TN];
  if (nk > 0) stage(0, 0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    if (t + 1 < nk) stage(b ^ 1, t + 1);
    const unsigned char *As = smem + b * TILE_BYTES;
    const unsigned char *Bs = As + BM * BK * 4;
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int k = 2 * s + fk;
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * TM * 32 + i * 32 + fr;
        av[i] = *reinterpret_cast<const float *>(As + row * 128 + swz8(row, k >> 2) * 16 + (k & 3) * 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * TN * 32 + j * 32 + fr;
        bv[j] = *reinterpret_cast<const float *>(Bs + row * 128 + swz8(row, k >> 2) * 16 + (k & 3) * 4);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (s == 0) {
            if (t > 0) acc[i][j] = acc[i][j] + part[i][j];
            part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], zero, 0, 0, 0);
          } else {
            part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], part[i][j], 0, 0, 0);
          }
        }
    }
    __syncthreads();  // DMA of tile t+1 landed (vmcnt(0)); every wave done reading tile t
  }
  if (nk > 0) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = acc[i][j] + part[i][j];
  }
  if (a.accum) add_c32<TM, TN>(a, acc, m0 + wm * TM * 32, n0 + wn * TN * 32, lane);

#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
    if (col >= a.N) continue;
    const float b = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t rbase = m0 + wm * TM * 32 + i * 32 + 4 * (lane >> 5);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < a.M) a.C[row * a.ldc + col] = epilogue(a, acc[i][j][r], b, row, col, RELU);
      }
    }
  }
}

template <int WM, int WN, int TM, int TN>
lpg_status launch_fc_glds(const FcArgs &a0, bool relu, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = 64 * WM * WN;
  FcArgs a = a0;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_f32: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_fwd_f32_glds<WM, WN, TM, TN, true>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((fc_fwd_f32_glds<WM, WN, TM, TN, false>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

int g_fc_variant = 0;  // lpg_fc_set_variant; 0 = default tile

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" lpg_status lpg_fc_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const float *W1,
                                 int64_t ldw1, int64_t K2, const float *A2, int64_t lda2, const float *W2,
                                 int64_t ldw2, const float *bias, float *C, int64_t ldc, int32_t flags,
                                 float dropout_p, uint64_t seed, void *stream) {
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "lpg_fc_f32: negative size");
  if (M == 0 || N == 0) return LPG_OK;
  LPG_REQUIRE(C != nullptr && ldc >= N, "lpg_fc_f32: bad C/ldc");
  LPG_REQUIRE(K1 == 0 || (A1 && W1 && lda1 >= K1 && ldw1 >= K1), "lpg_fc_f32: bad A1/W1");
  LPG_REQUIRE(K2 == 0 || (A2 && W2 && lda2 >= K2 && ldw2 >= K2), "lpg_fc_f32: bad A2/W2");
  LPG_REQUIRE(K1 % 4 == 0 && K2 % 4 == 0 && lda1 % 4 == 0 && ldw1 % 4 == 0 && (K2 == 0 || (lda2 % 4 == 0 && ldw2 % 4 == 0)),
              "lpg_fc_f32: K and leading dimensions must be multiples of 4 floats");
  LPG_REQUIRE(aligned16(A1) && aligned16(W1) && (K2 == 0 || (aligned16(A2) && aligned16(W2))),
              "lpg_fc_f32: A/W must be 16-byte aligned");
  LPG_REQUIRE((flags & ~3) == 0, "lpg_fc_f32: unknown flags 0x%x", flags);
  LPG_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "lpg_fc_f32: dropout_p %g not in [0, 1)", (double)dropout_p);
  FcArgs a{M, N, K1, K2, A1, A2, W1, W2, bias, lda1, lda2, ldw1, ldw2, C, ldc, 0, 0, seed, 0u, 1.f, (flags >> 1) & 1};
  if (dropout_p > 0.f) {
    const double th = (double)dropout_p * 4294967296.0;
    a.drop_thresh = th >= 4294967295.0 ? 4294967295u : (uint32_t)(th < 1.0 ? 1.0 : th);
    a.drop_scale = 1.f / (1.f - dropout_p);
  }
  hipStream_t s = as_stream(stream);
  const bool relu = flags & 1;
  lpg_status st;
  if (try_smallk(a, relu, s, &st)) return st;                // conv1: narrow LP features
  if (N <= 32) return launch_fc<4, 1, 1, 1, 32>(a, relu, s);  // heads (N = 3): 128 x 32 tiles
  switch (g_fc_variant) {
    case 1: return launch_fc<4, 2, 2, 2, 32>(a, relu, s);  // 256 x 128, 8 waves
    case 2: return launch_fc<2, 4, 2, 2, 32>(a, relu, s);  // 128 x 256, 8 waves
    case 3: return launch_fc<2, 2, 2, 2, 64>(a, relu, s);  // 128 x 128, BK 64 (1 block / CU)
    case 4: return launch_fc16<2, 2, 4, 4>(a, relu, s);    // 16x16x4 MFMA, 128 x 128
    case 5: return launch_fc16<2, 2, 4, 8>(a, relu, s);    // 16x16x4 MFMA, 128 x 256
    case 6: return launch_fc16<4, 2, 4, 4>(a, relu, s);    // 16x16x4 MFMA, 256 x 128, 8 waves
    case 7:
      if (K1 % 32 == 0 && K2 % 32 == 0) return launch_fc_glds<2, 2, 2, 2>(a, relu, s);  // LDS-DMA staging
      return launch_fc<2, 2, 2, 2, 32>(a, relu, s);
    case 8:
      if (K1 % 32 == 0 && K2 % 32 == 0) return launch_fc_glds<2, 4, 2, 2>(a, relu, s);  // 128 x 256, 8 waves
      return launch_fc<2, 2, 2, 2, 32>(a, relu, s);
    default: return launch_fc<2, 2, 2, 2, 32>(a, relu, s); // 128 x 128, BK 32, 2 blocks / CU
  }
}

extern "C" lpg_status lpg_relu_dropout_bwd_f32(int64_t n, const float *g, const float *y, float scale, float *out,
                                                void *stream) {
  LPG_REQUIRE(n >= 0, "lpg_relu_dropout_bwd_f32: n < 0");
  if (n == 0) return LPG_OK;
  LPG_REQUIRE(g && y && out, "lpg_relu_dropout_bwd_f32: NULL pointer");
  LPG_REQUIRE(n % 4 == 0 && aligned16(g) && aligned16(y) && aligned16(out),
              "lpg_relu_dropout_bwd_f32: n must be a multiple of 4 and buffers 16-byte aligned");
  const int64_t n4 = n / 4;
  int64_t blocks = (n4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(relu_dropout_bwd_f32, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), n4,
                     reinterpret_cast<const float4 *>(g), reinterpret_cast<const float4 *>(y), scale,
                     reinterpret_cast<float4 *>(out));
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

extern "C" lpg_status lpg_fc_set_variant(int32_t v) {
  LPG_REQUIRE(v >= 0 && v <= 8, "lpg_fc_set_variant: variant %d not in [0, 8]", v);
  g_fc_variant = v;
  return LPG_OK;
}

extern "C" lpg_status lpg_knowledge_f32(int64_t M, const float *logit, int64_t ldl, const float *feas, int64_t ldf,
                                        int64_t feas_cols, float bound, float *out, int64_t ldo, void *stream) {
  LPG_REQUIRE(M >= 0, "lpg_knowledge_f32: M < 0");
  if (M == 0) return LPG_OK;
  LPG_REQUIRE(logit && feas && out, "lpg_knowledge_f32: NULL pointer");
  LPG_REQUIRE(ldl >= 3 && ldo >= 3 && feas_cols >= 3 && ldf >= feas_cols, "lpg_knowledge_f32: bad shapes");
  hipLaunchKernelGGL(knowledge_f32, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, as_stream(stream), M, logit,
                     ldl, feas, ldf, feas_cols, bound, out, ldo);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}
