// EXPERIMENT (not in the product build; DESIGN.md 4.2b "x3 weight gradient on 256 x 256 tiles"): it was
// built as lp-gnn_amd/csrc/wgrad_x3q.hip with a launcher (wgrad_x3q_launch below, splits from
// wgrad_x3q_splits) called from lpg_wgrad_x3_f32 under LPGNN_WGRAD_KERNEL=1, measured against
// wgrad_x3w by tools/experiments/gpu_r03q{1,2,3}.sh and dropped.
//
// x3 weight gradient on 256 x 256 output tiles: dW[n, k] = sum_r G[r, n] X[r, k] in fp32 through
// the exact three-way bf16 split (fc_x3.hip's header), the lin_rel / lin_root weight gradients of
// GraphConv (arch.py:57-62, 75-80) in the fp32 training step (train.py:128).
//
// Why a second form beside wgrad_x3w (fc_x3.hip): that kernel's 256 x 128 tile of eight 64 x 64
// wave tiles keeps a0 b0 and the five small products in separate accumulators, so 128 of a wave's
// 256 registers hold accumulators and the tile cannot grow; per 16x16x32 MFMA it pays 1.375 split
// VALU and 0.25 fragment reads.  Here ONE accumulator per output takes all six products (small terms
// first), which halves the accumulator registers, and four waves of 128 x 128 (one wave per SIMD,
// accumulators in AGPRs) cover a 256 x 256 tile on v_mfma_f32_32x32x16_bf16: per 32 x 32 x 16
// MFMA (twice the work of a 16x16x32) 0.92 split VALU and 0.25 fragment reads -- 0.67x the split
// work and 0.5x the fragment reads per FLOP.  Accuracy: every product term is the same as in
// wgrad_x3w (dropped terms <= 2^-23 |ab|); the accumulation rounds six times per 16 rows (the
// MFMA's internal sum of 16 exact products, then the add into the accumulator) where wgrad_x3w
// rounds once per 32 rows on its main chain -- still fewer roundings than an fp32 FMA chain (one
// per row), and within tests/test_gpu_x3.py's fp64 bound.
//
// Chunks of 16 rows (the MFMA's k): every thread loads four 8-row units per chunk (G columns
// lc and 128 + lc, X columns lc and 128 + lc, lc = tid >> 1, rows 8 (tid & 1) .. + 7 of the
// chunk) through a raw buffer descriptor over the block's R range (rows past R read zeros), splits
// each unit into three bf16x8 and writes them into plane images laid out for the MFMA: per plane
// [256 columns][16 rows] bf16, 32-B column rows whose two 16-B halves swap on odd 8-column groups
// (conflict-free ds_read_b128 over the 32 consecutive columns a lane group reads, and
// conflict-free ds_write_b128 over the 4 columns x 2 halves of an 8-lane store group).  Two plane
// buffers (2 x 48 KiB): chunk c + 1 is split into the other buffer unit by unit between chunk c's
// fragment rows, each unit's chunk c + 2 loads issued right behind its split; one barrier per
// chunk.  R is split into S contiguous ranges (partial tiles folded in s order by wgrad_fold:
// deterministic, no atomics).
#include "common.h"
#include "x3_split.h"

#include <type_traits>

#pragma clang fp contract(off)

namespace lpg {
namespace {

constexpr int Q_T = 256;                 // output tile (n and k)
constexpr int Q_R = 16;                  // rows per chunk (the MFMA's k)
constexpr int Q_PL = Q_T * Q_R * 2;      // one plane image: 256 columns x 16 rows bf16 (8 KiB)
constexpr int Q_BUF = 6 * Q_PL;          // one buffer: three G planes, then three X planes (48 KiB)

// byte offset of (column, 8-row half) in a plane image
__device__ __forceinline__ int qoff(int col, int h) { return col * 32 + ((h ^ ((col >> 3) & 1)) << 4); }

__global__ __launch_bounds__(256, 1) void wgrad_x3q(int64_t R, int64_t N, int64_t K, const float *__restrict__ G,
                                                    int64_t ldg, const float *__restrict__ X, int64_t ldx,
                                                    float *__restrict__ part, int64_t nt, int64_t kt,
                                                    int64_t chunks_per_split) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * Q_BUF];

  // XCD-aware bijective remap: each XCD walks a contiguous range of (split, tile) ids
  const int64_t nwg = (int64_t)gridDim.x, xcd = (int64_t)blockIdx.x % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t bid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (int64_t)blockIdx.x / 8;
  const int64_t tiles = nt * kt;
  const int64_t s = bid / tiles, tile = bid % tiles;
  const int64_t n0 = (tile / kt) * Q_T, k0 = (tile % kt) * Q_T;
  const int64_t nchunks = (R + Q_R - 1) / Q_R;
  const int64_t c0 = s * chunks_per_split;
  const int64_t c1 = c0 + chunks_per_split < nchunks ? c0 + chunks_per_split : nchunks;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lc = tid >> 1, hf = tid & 1;
  // columns past the edge are clamped (their outputs are never stored)
  const int64_t col_u[4] = {n0 + lc < N ? n0 + lc : N - 1, n0 + 128 + lc < N ? n0 + 128 + lc : N - 1,
                            k0 + lc < K ? k0 + lc : K - 1, k0 + 128 + lc < K ? k0 + 128 + lc : K - 1};
  const float *gbase = G + c0 * Q_R * ldg + n0, *xbase = X + c0 * Q_R * ldx + k0;
  const int64_t gleft = (R - c0 * Q_R) * ldg * 4, xleft = (R - c0 * Q_R) * ldx * 4;
  const uint32_t gbytes = (uint32_t)(gleft < 0x7fffffff ? gleft : 0x7fffffff);
  const uint32_t xbytes = (uint32_t)(xleft < 0x7fffffff ? xleft : 0x7fffffff);
  float raw[4][8];
  auto load_unit = [&](int u, int64_t c) {  // c clamped to the last chunk: a spare re-load at the end, no branch
    c = c < c1 ? c : c1 - 1;
    const bool isg = u < 2;
    const int64_t ld = isg ? ldg : ldx;
    const int voff = (int)((col_u[u] - (isg ? n0 : k0)) * 4 + hf * 8 * ld * 4);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      raw[u][e] = buf_load1(isg ? gbase : xbase, isg ? gbytes : xbytes, voff, (int)(((c - c0) * Q_R + e) * ld * 4));
  };
  auto split_unit = [&](unsigned char *buf, int u) {  // unit u's 8 rows -> three bf16x8 in the plane images
    const Split3 t = split3(f32x4{raw[u][0], raw[u][1], raw[u][2], raw[u][3]},
                            f32x4{raw[u][4], raw[u][5], raw[u][6], raw[u][7]});
    unsigned char *dst = buf + (u < 2 ? 0 : 3 * Q_PL) + qoff((u & 1) * 128 + lc, hf);
    *reinterpret_cast<bf16x8 *>(dst) = t.h;
    *reinterpret_cast<bf16x8 *>(dst + Q_PL) = t.m;
    *reinterpret_cast<bf16x8 *>(dst + 2 * Q_PL) = t.l;
  };

  const int wn = wave >> 1, wk = wave & 1;  // 2 (n) x 2 (k) waves of 128 x 128
  const int fc = lane & 31, fh = lane >> 5;  // MFMA operand: column fc of the fragment, rows 8 fh .. + 7
  f32x16 acc[4][4];
  const f32x16 zero = {};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = zero;
  auto frag = [&](const unsigned char *im, int col, bf16x8(&f)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const bf16x8 *>(im + p * Q_PL + qoff(col, fh));
  };
  // multiply the chunk in buf; with `split`, split unit i of the next chunk (raw) into `next` during
  // fragment row i's 24 MFMAs and issue that unit's loads of chunk `cload` (a compile-time choice:
  // see wgrad_x3w on the runtime test it replaces).  One wave per SIMD: nothing else fills the
  // matrix pipe while this wave issues VALU, so each row is one scheduling region whose order is
  // pinned (sched_group_barrier): the next row's A fragments read first, then MFMA / 2 VALU pairs
  // (the split: 44 VALU per unit, each pair inside one MFMA's 32 cycles), the unit's three plane
  // stores, its eight loads (after the VALU that read its registers), the row's last MFMAs.
  auto multiply = [&](const unsigned char *buf, unsigned char *next, int64_t cload, auto split) {
    constexpr bool SPLIT = decltype(split)::value;
    bf16x8 bv[4][3], av[2][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) frag(buf + 3 * Q_PL, wk * 128 + j * 32 + fc, bv[j]);
    frag(buf, wn * 128 + fc, av[0]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8(&a)[3] = av[i & 1];
      if (i < 3) frag(buf, wn * 128 + (i + 1) * 32 + fc, av[(i + 1) & 1]);
      if constexpr (SPLIT) {
        split_unit(next, i);
        load_unit(i, cload);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], bv[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bv[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bv[j][2], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], bv[j][0], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bv[j][1], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], bv[j][0], acc[i][j], 0, 0, 0);
      }
      if (i < 3) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);  // next row's fragment reads
      if constexpr (SPLIT) {
#pragma unroll
        for (int k = 0; k < 22; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
        }
        __builtin_amdgcn_sched_group_barrier(0x200, 3, 0);  // plane stores
        __builtin_amdgcn_sched_group_barrier(0x020, 8, 0);  // next loads of the unit
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  unsigned char *const B0 = smem, *const B1 = smem + Q_BUF;
  // prologue: chunk c0 split into B0, chunk c0 + 1's loads in flight
#pragma unroll
  for (int u = 0; u < 4; ++u) load_unit(u, c0);
#pragma unroll
  for (int u = 0; u < 4; ++u) split_unit(B0, u);
#pragma unroll
  for (int u = 0; u < 4; ++u) load_unit(u, c0 + 1);
  sync();
  int64_t c = c0;
  for (; c + 1 < c1; c += 2) {
    multiply(B0, B1, c + 2, std::true_type{});
    sync();
    multiply(B1, B0, c + 3, std::true_type{});
    sync();
  }
  if (c < c1) multiply(B0, nullptr, 0, std::false_type{});  // odd count: the last chunk sits in B0

  // D layout of the 32 x 32 MFMA: column fc, row 8 (v >> 2) + 4 fh + (v & 3)
  float *P = part + s * N * K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t col = k0 + wk * 128 + j * 32 + fc;
    if (col >= K) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int64_t row = n0 + wn * 128 + i * 32 + 8 * (v >> 2) + 4 * fh + (v & 3);
        if (row < N) P[row * K + col] = acc[i][j][v];
      }
  }
}

}  // namespace

// R splits of the 256 x 256 form: >= 2 blocks per CU over the grid (one block per CU at a time),
// >= 8 chunks (128 rows) per split, at most 64
int64_t wgrad_x3q_splits(int64_t R, int64_t N, int64_t K) {
  const int64_t tiles = ((N + Q_T - 1) / Q_T) * ((K + Q_T - 1) / Q_T);
  const int64_t nchunks = (R + Q_R - 1) / Q_R;
  const int64_t want = 2 * (int64_t)device_cus();
  int64_t S = (want + tiles - 1) / tiles;
  const int64_t maxS = nchunks / 8 > 1 ? nchunks / 8 : 1;
  if (S > maxS) S = maxS;
  if (S > 64) S = 64;
  return S < 1 ? 1 : S;
}

int64_t wgrad_x3q_chunk_rows() { return Q_R; }

lpg_status wgrad_x3q_launch(int64_t R, int64_t N, int64_t K, const float *G, int64_t ldg, const float *X, int64_t ldx,
                            float *part, int64_t S_used, int64_t cps, hipStream_t st) {
  const int64_t nt = (N + Q_T - 1) / Q_T, kt = (K + Q_T - 1) / Q_T;
  const int64_t nb = S_used * nt * kt;
  LPG_REQUIRE(nb < (int64_t)1 << 31, "lpg_wgrad_x3_f32: grid too large");
  hipLaunchKernelGGL(wgrad_x3q, dim3((unsigned)nb), dim3(256), 0, st, R, N, K, G, ldg, X, ldx, part, nt, kt, cps);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

}  // namespace lpg
