// bf16 variant of the fused GraphConv FC (the c5 "dense-FC-heavy, bf16 MFMA"
// configuration, BASELINE.json configs[4]):
//
//   C[m, n] = bf16( act( sum_k A1[m,k] W1[n,k] + sum_k A2[m,k] W2[n,k] + bias[n] ) )
//
// A, W bf16 (K contiguous), fp32 accumulation on v_mfma_f32_16x16x32_bf16,
// bias fp32, ReLU + the fused counter-based dropout of fc.hip, one RNE
// rounding to bf16 on the store.  No bitwise contract here (bf16 inputs): the
// tests compare against an fp32 GEMM of the same bf16-rounded operands.
//
// Tiling: 256 threads = 4 waves (2 x 2), 128 x 128 output tile, each wave
// 64 x 64 = 4 x 4 fragments of 16 x 16 (64 accumulator registers).  K-tile
// BK = 64 (one 128-B row per tile row), staged global -> LDS directly by
// global_load_lds_dwordx4 (each wave-instruction writes 1 KiB = 8 rows
// lane-linearly), two buffers, one barrier per k-tile: the next tile's DMA is
// in flight while the current one feeds the MFMAs.  LDS image per row: 8
// 16-B chunks, chunk c stored at c ^ ((row >> 1) & 7) -- applied on the DMA
// SOURCE address (the destination must stay lane-linear) and on the
// ds_read_b128 fragment reads, so the 16 rows a read quarter-wave touches land
// in 16 distinct 16-B bank groups.  XCD-aware bijective block remap as in fc.hip.
#include "common.h"

namespace lpg {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = (BM + BN) * BK * 2;  // one buffer: A tile then W tile

struct FcB16Args {
  int64_t M, N, K1, K2;
  const uint16_t *A1, *A2, *W1, *W2;
  const float *bias;
  int64_t lda1, lda2, ldw1, ldw2;
  uint16_t *C;
  int64_t ldc;
  int64_t mt, nt;
  uint64_t seed;
  uint32_t drop_thresh;
  float drop_scale;
};

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Same mask function as fc.hip's fp32 epilogue.
__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, int64_t row, int64_t col) {
  const uint32_t hr = lowbias32((uint32_t)row ^ (uint32_t)seed);
  return lowbias32(hr ^ ((uint32_t)col * 0x9e3779b9u) ^ (uint32_t)(seed >> 32));
}

__device__ __forceinline__ uint16_t to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <bool RELU>
__global__ __launch_bounds__(NT) void fc_fwd_bf16(FcB16Args a) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * TILE_BYTES];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);

  // DMA of k-tile t into buffer b: 16 + 16 pieces of 8 rows x 128 B; wave w
  // moves pieces w, w+4, w+8, w+12 of A and of W.  Lane i of a piece lands at
  // row 8*piece + i/8, physical chunk i%8, so it fetches logical chunk swz().
  auto stage = [&](int b, int t) {
    const bool p2 = t >= nk1;
    const uint16_t *A = p2 ? a.A2 : a.A1;
    const uint16_t *W = p2 ? a.W2 : a.W1;
    const int64_t lda = p2 ? a.lda2 : a.lda1, ldw = p2 ? a.ldw2 : a.ldw1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BK;
    unsigned char *base = smem + b * TILE_BYTES;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int piece = wave + 4 * p;
      const int row = piece * 8 + (lane >> 3);
      const int chunk = swz(row, lane & 7);
      int64_t gr = m0 + row;
      gr = gr < a.M ? gr : a.M - 1;  // rows past M feed outputs that are never stored
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(A + gr * lda + k0 + chunk * 8),
                                       reinterpret_cast<__attribute__((address_space(3))) void *>(
                                           (__attribute__((address_space(3))) unsigned char *)(base + piece * 1024)),
                                       16, 0, 0);
      int64_t gn = n0 + row;
      gn = gn < a.N ? gn : a.N - 1;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(W + gn * ldw + k0 + chunk * 8),
                                       reinterpret_cast<__attribute__((address_space(3))) void *>(
                                           (__attribute__((address_space(3))) unsigned char *)(base + BM * BK * 2 +
                                                                                               piece * 1024)),
                                       16, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment rows this lane reads: A rows wm*64 + 16i + (lane&15), W rows wn*64 + 16j + (lane&15)
  const int fr = lane & 15, fq = lane >> 4;

  if (nk > 0) stage(0, 0);
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int b = t & 1;
    if (t + 1 < nk) stage(b ^ 1, t + 1);
    const unsigned char *As = smem + b * TILE_BYTES;
    const unsigned char *Bs = As + BM * BK * 2;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const int chunk = s * 4 + fq;  // k = 32 s + 8 fq .. +7
      bf16x8 av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        av[i] = *reinterpret_cast<const bf16x8 *>(As + row * 128 + swz(row, chunk) * 16);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + j * 16 + fr;
        bv[j] = *reinterpret_cast<const bf16x8 *>(Bs + row * 128 + swz(row, chunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();  // the DMA of tile t+1 has landed (vmcnt(0)) and every wave is done reading tile t
  }

  // Epilogue: C/D map of 16x16x32: col = lane & 15, row = 4 * (lane >> 4) + r.
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t col = n0 + wn * 64 + j * 16 + fr;
    if (col >= a.N) continue;
    const float bb = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * 64 + i * 16 + fq * 4 + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r];
        if (a.bias) v = v + bb;
        if (RELU) v = v < 0.f ? 0.f : v;
        if (a.drop_thresh) v = drop_hash(a.seed, row, col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
        a.C[row * a.ldc + col] = to_bf16_rne(v);
      }
    }
  }
}

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" lpg_status lpg_fc_bf16(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                  const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2,
                                  const uint16_t *W2, int64_t ldw2, const float *bias, uint16_t *C, int64_t ldc,
                                  int32_t flags, float dropout_p, uint64_t seed, void *stream) {
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "lpg_fc_bf16: negative size");
  if (M == 0 || N == 0) return LPG_OK;
  LPG_REQUIRE(C != nullptr && ldc >= N, "lpg_fc_bf16: bad C/ldc");
  LPG_REQUIRE(K1 % BK == 0 && K2 % BK == 0, "lpg_fc_bf16: K1, K2 must be multiples of %d (pad the features)", BK);
  LPG_REQUIRE(K1 == 0 || (A1 && W1 && lda1 >= K1 && ldw1 >= K1), "lpg_fc_bf16: bad A1/W1");
  LPG_REQUIRE(K2 == 0 || (A2 && W2 && lda2 >= K2 && ldw2 >= K2), "lpg_fc_bf16: bad A2/W2");
  LPG_REQUIRE(lda1 % 8 == 0 && ldw1 % 8 == 0 && (K2 == 0 || (lda2 % 8 == 0 && ldw2 % 8 == 0)) &&
                  (K1 == 0 || (aligned16(A1) && aligned16(W1))) && (K2 == 0 || (aligned16(A2) && aligned16(W2))),
              "lpg_fc_bf16: A/W must be 16-byte aligned with leading dimensions multiple of 8");
  LPG_REQUIRE((flags & ~1) == 0, "lpg_fc_bf16: unknown flags 0x%x", flags);
  LPG_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "lpg_fc_bf16: dropout_p %g not in [0, 1)", (double)dropout_p);
  FcB16Args a{M, N, K1, K2, A1, A2, W1, W2, bias, lda1, lda2, ldw1, ldw2, C, ldc, 0, 0, seed, 0u, 1.f};
  if (dropout_p > 0.f) {
    const double th = (double)dropout_p * 4294967296.0;
    a.drop_thresh = th >= 4294967295.0 ? 4294967295u : (uint32_t)(th < 1.0 ? 1.0 : th);
    a.drop_scale = 1.f / (1.f - dropout_p);
  }
  a.mt = (M + BM - 1) / BM;
  a.nt = (N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_bf16: grid too large");
  hipStream_t s = as_stream(stream);
  if (flags & 1)
    hipLaunchKernelGGL(fc_fwd_bf16<true>, dim3((unsigned)nwg), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL(fc_fwd_bf16<false>, dim3((unsigned)nwg), dim3(NT), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}
