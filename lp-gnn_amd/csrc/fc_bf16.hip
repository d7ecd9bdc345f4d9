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
// Tiling: 512 threads = 8 waves (2 x 4), 256 x 256 output tile, each wave
// 128 x 64 = 8 x 4 fragments of 16 x 16 (128 accumulator registers); small M
// (< 4096 rows) uses 4 waves on 128 x 128.  (A 128 x 128 tile needs 128 B/clk
// per CU of L2->CU bandwidth at the MFMA rate and measured 27 % MFMA-busy; the
// 256 x 256 tile halves the staged bytes per MFMA.)  K-tile
// BK = 64 (one 128-B row per tile row), staged global -> LDS directly by
// global_load_lds_dwordx4 (each wave-instruction writes 1 KiB = 8 rows
// lane-linearly), two buffers, one barrier per k-tile: the next tile's DMA is
// in flight while the current one feeds the MFMAs.  LDS image per row: 8
// 16-B chunks, chunk c stored at c ^ ((row >> 1) & 7) -- applied on the DMA
// SOURCE address (the destination must stay lane-linear) and on the
// ds_read_b128 fragment reads, so the 16 rows a read quarter-wave touches land
// in 16 distinct 16-B bank groups.  XCD-aware bijective block remap as in fc.hip.
#include "common.h"
#include "fc_common.h"

namespace lpg {
namespace {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;

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
  int32_t accum;  // flags bit 1: C holds a bf16 addend, C = bf16(act(A1 W1^T + A2 W2^T + C + bias))
};

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ uint16_t to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// WM x WN waves, each owning FM x FN fragments of 16 x 16.
template <int WM, int WN, int FM, int FN, bool RELU>
__global__ __launch_bounds__(64 * WM * WN) void fc_fwd_bf16(FcB16Args a) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int TILE_BYTES = (BM + BN) * BK * 2;  // one buffer: A tile then W tile
  constexpr int PA = BM / 8 / NW, PB = BN / 8 / NW;  // 1-KiB DMA pieces per wave per k-tile
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows must split into whole pieces per wave");
  constexpr int EP_PITCH = FN * 16 * 2 + 16;                   // epilogue image row pitch (bytes, 16-B aligned)
  constexpr int EP_BYTES = NW * FM * 16 * EP_PITCH;
  constexpr int SMEM = 2 * TILE_BYTES > EP_BYTES ? 2 * TILE_BYTES : EP_BYTES;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);

  // DMA of k-tile t into buffer b: pieces of 8 rows x 128 B (one
  // wave-instruction each); wave w moves pieces w, w+NW, ... of A and of W.
  // Lane i of a piece lands at row 8*piece + i/8, physical chunk i%8, so it
  // fetches logical chunk swz().
  auto stage = [&](int b, int t) {
    const bool p2 = t >= nk1;
    const uint16_t *A = p2 ? a.A2 : a.A1;
    const uint16_t *W = p2 ? a.W2 : a.W1;
    const int64_t lda = p2 ? a.lda2 : a.lda1, ldw = p2 ? a.ldw2 : a.ldw1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BK;
    unsigned char *base = smem + b * TILE_BYTES;
    typedef __attribute__((address_space(3))) unsigned char lds_t;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int piece = wave + NW * p;
      const int row = piece * 8 + (lane >> 3);
      int64_t gr = m0 + row;
      gr = gr < a.M ? gr : a.M - 1;  // rows past M feed outputs that are never stored
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(A + gr * lda + k0 + swz(row, lane & 7) * 8),
                                       (lds_t *)(base + piece * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int piece = wave + NW * p;
      const int row = piece * 8 + (lane >> 3);
      int64_t gn = n0 + row;
      gn = gn < a.N ? gn : a.N - 1;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(W + gn * ldw + k0 + swz(row, lane & 7) * 8),
                                       (lds_t *)(base + BM * BK * 2 + piece * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment rows this lane reads: A rows wm*FM*16 + 16i + (lane&15), W rows wn*FN*16 + 16j + (lane&15)
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
      bf16x8 av[FM], bv[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * FM * 16 + i * 16 + fr;
        av[i] = *reinterpret_cast<const bf16x8 *>(As + row * 128 + swz(row, chunk) * 16);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * FN * 16 + j * 16 + fr;
        bv[j] = *reinterpret_cast<const bf16x8 *>(Bs + row * 128 + swz(row, chunk) * 16);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();  // the DMA of tile t+1 has landed (vmcnt(0)) and every wave is done reading tile t
  }

  // Epilogue: C/D map of 16x16x32: col = lane & 15, row = 4 * (lane >> 4) + r.
  const int64_t wrow0 = m0 + wm * FM * 16, wcol0 = n0 + wn * FN * 16;
  if (a.N % 8 == 0 && a.ldc % 8 == 0 && (reinterpret_cast<uintptr_t>(a.C) & 15) == 0) {
    // Through LDS (the staging buffers are free after the last barrier): each
    // wave writes its FM*16 x FN*16 bf16 tile row-major (padded pitch), then
    // stores it as 16-B chunks, 8 lanes per 128-B row segment -- one
    // global_store_dwordx4 per 8 outputs instead of one 2-byte store each.
    unsigned char *img = smem + wave * (FM * 16 * EP_PITCH);
    constexpr int CPR = FN * 16 / 8;  // 16-B chunks per row
    if (a.accum) {  // the addend tile, coalesced 16-B loads into the same image
#pragma unroll
      for (int it = 0; it < FM * 16 * CPR / 64; ++it) {
        const int q = it * 64 + lane;
        const int lr = q / CPR, ch = q % CPR;
        const int64_t row = wrow0 + lr < a.M ? wrow0 + lr : a.M - 1, col = wcol0 + ch * 8;
        if (col < a.N)
          *reinterpret_cast<uint4 *>(img + lr * EP_PITCH + ch * 16) =
              *reinterpret_cast<const uint4 *>(a.C + row * a.ldc + col);
      }
      __builtin_amdgcn_wave_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int64_t col = wcol0 + j * 16 + fr;
      const float bb = (a.bias && col < a.N) ? a.bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = i * 16 + fq * 4 + r;
          float v = acc[i][j][r];
          if (a.accum) v = v + bf16_to_f32(*reinterpret_cast<const uint16_t *>(img + lr * EP_PITCH + (j * 16 + fr) * 2));
          v = v + bb;
          if (RELU) v = v < 0.f ? 0.f : v;
          if (a.drop_thresh) v = drop_hash(a.seed, wrow0 + lr, col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
          *reinterpret_cast<uint16_t *>(img + lr * EP_PITCH + (j * 16 + fr) * 2) = to_bf16_rne(v);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int it = 0; it < FM * 16 * CPR / 64; ++it) {
      const int q = it * 64 + lane;
      const int lr = q / CPR, ch = q % CPR;
      const int64_t row = wrow0 + lr, col = wcol0 + ch * 8;
      const uint4 v = *reinterpret_cast<const uint4 *>(img + lr * EP_PITCH + ch * 16);
      if (row < a.M && col < a.N) *reinterpret_cast<uint4 *>(a.C + row * a.ldc + col) = v;
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int64_t col = wcol0 + j * 16 + fr;
    if (col >= a.N) continue;
    const float bb = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = wrow0 + i * 16 + fq * 4 + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r];
        if (a.accum) v = v + bf16_to_f32(a.C[row * a.ldc + col]);
        v = v + bb;
        if (RELU) v = v < 0.f ? 0.f : v;
        if (a.drop_thresh) v = drop_hash(a.seed, row, col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
        a.C[row * a.ldc + col] = to_bf16_rne(v);
      }
    }
  }
}

// Deeper pipeline, 256 x 256 tile (8 waves, 2 x 4, 8 x 4 fragments each):
// BK = 32 (64-B rows), THREE LDS buffers of 32 KiB, the DMA of tile t+2 issued
// while tile t feeds the MFMAs and tile t+1 still in flight across the
// barrier.  A raw s_barrier with a counted vmcnt (this wave's 4 pieces of the
// newest tile may stay outstanding) replaces __syncthreads(), whose fence
// would wait for every DMA (vmcnt(0)).  LDS image per 64-B row: 4 16-B
// chunks, chunk c stored at c ^ ((row >> 2) & 3) (16 consecutive rows of one
// fragment read then cover all 16 bank groups).
__device__ __forceinline__ int swz32(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }

template <bool RELU>
__global__ __launch_bounds__(512) void fc_fwd_bf16_p3(FcB16Args a) {
  constexpr int WM = 2, WN = 4, FM = 8, FN = 4, NW = 8, BKP = 32;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;        // 256 x 256
  constexpr int ROWB = BKP * 2;                               // 64-B rows
  constexpr int TILE_BYTES = (BM + BN) * ROWB;                // 32 KiB
  constexpr int PA = BM * ROWB / 1024 / NW, PB = BN * ROWB / 1024 / NW;  // 2 + 2 pieces per wave
  __shared__ __attribute__((aligned(1024))) unsigned char smem[3 * TILE_BYTES];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nk1 = (int)(a.K1 / BKP);
  const int nk = nk1 + (int)(a.K2 / BKP);

  // piece = 16 rows x 64 B; lane i -> row 16*piece + i/4, physical chunk i%4
  auto stage = [&](int b, int t) {
    const bool p2 = t >= nk1;
    const uint16_t *A = p2 ? a.A2 : a.A1;
    const uint16_t *W = p2 ? a.W2 : a.W1;
    const int64_t lda = p2 ? a.lda2 : a.lda1, ldw = p2 ? a.ldw2 : a.ldw1;
    const int64_t k0 = (int64_t)(p2 ? t - nk1 : t) * BKP;
    unsigned char *base = smem + b * TILE_BYTES;
    typedef __attribute__((address_space(3))) unsigned char lds_t;
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int piece = wave + NW * p;
      const int row = piece * 16 + (lane >> 2);
      int64_t gr = m0 + row;
      gr = gr < a.M ? gr : a.M - 1;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(A + gr * lda + k0 + swz32(row, lane & 3) * 8),
                                       (lds_t *)(base + piece * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int piece = wave + NW * p;
      const int row = piece * 16 + (lane >> 2);
      int64_t gn = n0 + row;
      gn = gn < a.N ? gn : a.N - 1;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(W + gn * ldw + k0 + swz32(row, lane & 3) * 8),
                                       (lds_t *)(base + BM * ROWB + piece * 1024), 16, 0, 0);
    }
  };
  auto barrier_keep_newest = [&]() {  // this wave's DMA of all but the newest tile has landed
    asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto barrier_all = [&]() {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  static_assert(PA + PB == 4, "vmcnt(4) above counts this wave's pieces of one tile");

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;

  if (nk > 0) stage(0, 0);
  if (nk > 1) {
    stage(1, 1);
    barrier_keep_newest();
  } else {
    barrier_all();
  }
  int b = 0;
  for (int t = 0; t < nk; ++t) {
    const bool more = t + 2 < nk;
    if (more) stage(b == 0 ? 2 : b - 1, t + 2);  // buffer (t + 2) % 3: read last in iteration t - 1
    const unsigned char *As = smem + b * TILE_BYTES;
    const unsigned char *Bs = As + BM * ROWB;
    bf16x8 av[FM], bv[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * FM * 16 + i * 16 + fr;
      av[i] = *reinterpret_cast<const bf16x8 *>(As + row * ROWB + swz32(row, fq) * 16);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * FN * 16 + j * 16 + fr;
      bv[j] = *reinterpret_cast<const bf16x8 *>(Bs + row * ROWB + swz32(row, fq) * 16);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    if (more)
      barrier_keep_newest();  // tile t+1 landed, t+2 may still be in flight
    else
      barrier_all();
    b = b == 2 ? 0 : b + 1;
  }

#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int64_t col = n0 + wn * FN * 16 + j * 16 + fr;
    if (col >= a.N) continue;
    const float bb = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = m0 + wm * FM * 16 + i * 16 + fq * 4 + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r];
        if (a.accum) v = v + bf16_to_f32(a.C[row * a.ldc + col]);
        if (a.bias) v = v + bb;
        if (RELU) v = v < 0.f ? 0.f : v;
        if (a.drop_thresh) v = drop_hash(a.seed, row, col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
        a.C[row * a.ldc + col] = to_bf16_rne(v);
      }
    }
  }
}

template <int WM, int WN, int FM, int FN>
lpg_status launch_bf16(FcB16Args a, bool relu, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_bf16: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_fwd_bf16<WM, WN, FM, FN, true>), dim3((unsigned)nwg), dim3(64 * WM * WN), 0, s, a);
  else
    hipLaunchKernelGGL((fc_fwd_bf16<WM, WN, FM, FN, false>), dim3((unsigned)nwg), dim3(64 * WM * WN), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

lpg_status launch_bf16_p3(FcB16Args a, bool relu, hipStream_t s) {
  a.mt = (a.M + 255) / 256;
  a.nt = (a.N + 255) / 256;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_bf16: grid too large");
  if (relu)
    hipLaunchKernelGGL(fc_fwd_bf16_p3<true>, dim3((unsigned)nwg), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL(fc_fwd_bf16_p3<false>, dim3((unsigned)nwg), dim3(512), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

int g_bf16_variant = 0;  // lpg_fc_bf16_set_variant: 0 = by size, 1 = 128 x 128, 2 = 256^2 2-buffer, 3 = 256^2 3-buffer

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
  LPG_REQUIRE((flags & ~3) == 0, "lpg_fc_bf16: unknown flags 0x%x", flags);
  LPG_REQUIRE(dropout_p >= 0.f && dropout_p < 1.f, "lpg_fc_bf16: dropout_p %g not in [0, 1)", (double)dropout_p);
  FcB16Args a{M, N, K1, K2, A1, A2, W1, W2, bias, lda1, lda2, ldw1, ldw2, C, ldc, 0, 0, seed, 0u, 1.f, (flags >> 1) & 1};
  if (dropout_p > 0.f) {
    const double th = (double)dropout_p * 4294967296.0;
    a.drop_thresh = th >= 4294967295.0 ? 4294967295u : (uint32_t)(th < 1.0 ? 1.0 : th);
    a.drop_scale = 1.f / (1.f - dropout_p);
  }
  hipStream_t s = as_stream(stream);
  const bool relu = flags & 1;
  if (g_bf16_variant == 1 || (g_bf16_variant == 0 && M < 4096))
    return launch_bf16<2, 2, 4, 4>(a, relu, s);  // 128 x 128
  if (g_bf16_variant == 3) return launch_bf16_p3(a, relu, s);  // 256 x 256, BK 32, 3 buffers
  return launch_bf16<2, 4, 8, 4>(a, relu, s);    // 256 x 256, BK 64, 2 buffers
}

extern "C" lpg_status lpg_fc_bf16_set_variant(int32_t v) {
  LPG_REQUIRE(v >= 0 && v <= 3, "lpg_fc_bf16_set_variant: variant %d not in [0, 3]", v);
  g_bf16_variant = v;
  return LPG_OK;
}
