// Dense per-node FC of GraphConv on fp32 MFMA (gfx950), fused:
//
//   C[m, n] = act( sum_{k<K1} A1[m,k] W1[n,k] + sum_{k<K2} A2[m,k] W2[n,k] [+ C[m,n]] + bias[n] )
//
// = PyG 2.1 GraphConv.forward after propagate:  lin_rel(agg) + lin_root(x_dst)
// (arch.py:57-62, 75-80) with the ReLU of arch.py:182/188 as the epilogue,
// and -- with K2 = 0, no ReLU -- the heads lin_left / lin_right (arch.py:190).
// The concat [agg | x_dst] is never materialised: the k loop walks A1 then A2.
// [+ C]: the accumulate flag (re-associated GraphConv, lpgnn/conv.py).
//
// Numerics (the parity contract, mirrored by oracle/fc_ref.c): each part
// (A1, W1) over K1, then (A2, W2) over K2, is cut into numerics blocks of
// NB = 128 k (the last one shorter; zero padding: fma(0, 0, s) = s exactly,
// the chain is never -0).  A block's products form ONE fp32 fma chain from
// +0, its k visited in groups of 8 consecutive k, inside a group in the
// order 0,4,1,5,2,6,3,7; the block sums are added in order into the running
// total (+0 initially); then + C (accumulate), + bias, ReLU as
// (v < 0 ? 0 : v), dropout.  The group order is what v_mfma_f32_32x32x2_f32
// -- bit-for-bit an fma chain, k0 then k1 of its pair (MI355X_MICROARCH.md
// §Matrix cores) -- sees when a lane's 16-B LDS read of 4 consecutive k
// feeds 4 MFMA steps and the two lane halves hold k and k + 4.  The blocks
// keep the rounding error at the level of MKL's blocked sgemm (one chain of
// K = 2048 drifted past the 1e-4 logit tolerance); 128-k blocks cost one
// fold (64 adds per wave) per 4 k-tiles.
//
// Tiling (fc_fwd_f32): 4 waves (2 x 2), 128 x 128 output tile, each wave
// 2 x 2 blocks of 32x32 (64 accumulators in AGPRs).  A and W k-tiles of
// BK = 32 are staged global -> LDS by global_load_lds (LDS-DMA, no register
// round trip) into an NS-stage ring, the DMA of the next tile in flight under
// the current tile's MFMAs; one barrier per k-tile.  LDS image: 16-B chunk c
// of row r at c ^ ((r >> 1) & 7) (128-B rows), which makes the ds_read_b128
// operand reads conflict-free for the b128 lane groups; the next k-group's
// operands are read halfway through the current group's 16 MFMAs.  Two
// blocks per CU (64 KiB LDS each).  Blocks are remapped so that each XCD
// walks a contiguous range of m-tiles with all their n-tiles (the A panel is
// re-read from that XCD's L2).  K1, K2 multiples of 32 (the host pads).
#include "common.h"
#include "fc_common.h"

#include <type_traits>

#pragma clang fp contract(off)

namespace lpg {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int NB = 128;  // numerics block: k per fma chain (the parity contract), a multiple of every BK


struct FcArgs {
  int64_t M, N, K1, K2;
  const float *A1, *A2, *W1, *W2, *bias;
  int64_t lda1, lda2, ldw1, ldw2;
  float *C;
  int64_t ldc;
  int64_t mt, nt;  // tiles
  // fused dropout (after the ReLU): keep element (row, col) iff its 16 mask bits
  // drop_bits(seed, key(row), col) >= drop_thresh (fc_common.h); kept values are scaled.
  uint64_t seed;
  uint32_t drop_thresh;  // 0 = no dropout
  float drop_scale;
  // flags bit 1: C holds an addend on entry, C = act(A1 W1^T + A2 W2^T + C + bias);
  // each element is read and rewritten by the lane that owns it
  int32_t accum;
  // the dropout key of row m is row_keys[m] if given, else row_off + m (the global node id when C holds
  // a slice of the rows; drop_row, fc_common.h)
  int64_t row_off;
  const int64_t *row_keys;
  // fc_smallk_f32<..., SC>: the f16x2 row scales of C (rsc[m], N <= 1024) and the blocks' column maxima
  // of |C| (cpart[row split][N], folded by colfold_f32) from the stores themselves
  float *rsc;
  float *cpart;
};

__device__ __forceinline__ float epilogue(const FcArgs &a, float v, float b, int64_t row, int64_t col, bool relu) {
  if (a.bias) v = v + b;
  if (relu) v = (v < 0.f) ? 0.f : v;
  if (a.drop_thresh) v = drop_bits(a.seed, drop_row(a.row_keys, a.row_off, row, a.M), col) >= a.drop_thresh ? v * a.drop_scale : 0.f;
  return v;
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

// The tiled FC (see the header): lane half fk of the 32x32x2 MFMA holds
// k = 8q + 4fk + u at step u of k-group q.  BK-deep k-tiles (32 or 64; 256-B
// rows use the swizzle c ^ (r & 15)), NS-stage ring (NS - 1 tiles in flight).
// K1, K2 multiples of BK.
template <int BK>
__device__ __forceinline__ int swzk(int row, int chunk) {
  return BK == 32 ? chunk ^ ((row >> 1) & 7) : chunk ^ (row & 15);
}

template <int WM, int WN, int TM, int TN, int BK, int NS, bool RELU>
__global__ __launch_bounds__(64 * WM * WN) void fc_fwd_f32(FcArgs a) {
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  constexpr int NW = WM * WN;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int ROWB = BK * 4, CPR = ROWB / 16, RPP = 1024 / ROWB;  // row bytes, chunks/row, rows/piece
  constexpr int TILE_BYTES = (BM + BN) * ROWB;
  constexpr int PA = BM / RPP / NW, PB = BN / RPP / NW;
  constexpr int NQ = BK / 8;
  static_assert(BK == 32 || BK == 64, "BK 32 or 64");
  static_assert(BM % (RPP * NW) == 0 && BN % (RPP * NW) == 0, "tile rows must split into whole pieces per wave");
  static_assert(NS == 2 || NS == 3, "2 or 3 stages");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NS * TILE_BYTES];

  const int64_t nwg = a.mt * a.nt;
  const int64_t bid = blockIdx.x;
  const int64_t xcd = bid % 8, q8 = nwg / 8, rr = nwg % 8;
  const int64_t wgid = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + bid / 8;
  const int64_t m0 = (wgid / a.nt) * BM;
  const int64_t n0 = (wgid % a.nt) * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nk1 = (int)(a.K1 / BK);
  const int nk = nk1 + (int)(a.K2 / BK);

  const float *srcA1[PA], *srcA2[PA], *srcW1[PB], *srcW2[PB];
#pragma unroll
  for (int p = 0; p < PA; ++p) {
    const int row = (wave + NW * p) * RPP + lane / CPR;
    int64_t gr = m0 + row;
    gr = gr < a.M ? gr : a.M - 1;
    const int off = swzk<BK>(row, lane % CPR) * 4;
    srcA1[p] = a.A1 + gr * a.lda1 + off;
    srcA2[p] = a.A2 + gr * a.lda2 + off;
  }
#pragma unroll
  for (int p = 0; p < PB; ++p) {
    const int row = (wave + NW * p) * RPP + lane / CPR;
    int64_t gn = n0 + row;
    gn = gn < a.N ? gn : a.N - 1;
    const int off = swzk<BK>(row, lane % CPR) * 4;
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
                                       (lds_t *)(base + BM * ROWB + (wave + NW * p) * 1024), 16, 0, 0);
  };
  auto barrier_keep = [&](bool keep_newest) {
    if (keep_newest)
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(PA + PB) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // acc: running total over numerics blocks; each block's products form their
  // own chain (part, from +0), added to acc in block order at the start of
  // the next block (part starts at +0: the first fold is +0 + +0)
  f32x16 acc[TM][TN], part[TM][TN];
  const f32x16 zero = {};
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = part[i][j] = zero;

  const int fr = lane & 31, fk = lane >> 5;
  int offA[TM], offB[TN];  // byte offset of the lane's row in a tile image
#pragma unroll
  for (int i = 0; i < TM; ++i) offA[i] = (wm * TM * 32 + i * 32 + fr) * ROWB;
#pragma unroll
  for (int j = 0; j < TN; ++j) offB[j] = BM * ROWB + (wn * TN * 32 + j * 32 + fr) * ROWB;
  const int rA0 = wm * TM * 32 + fr, rB0 = wn * TN * 32 + fr;

  if (nk > 0) stage(0, 0);
  if (NS == 3 && nk > 1) stage(1, 1);
  barrier_keep(NS == 3 && nk > 1);
  constexpr int FOLD = NB / BK;  // k-tiles per numerics block
  int b = 0;
  for (int t = 0; t < nk; ++t) {
    const bool more = t + NS - 1 < nk;
    if (more) stage(b == 0 ? NS - 1 : b - 1, t + NS - 1);  // buffer (t + NS - 1) % NS, read last in t - 1
    const unsigned char *T = smem + b * TILE_BYTES;
    f32x4v av[2][TM], bv[2][TN];
    auto lread = [&](int slot, int q) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        av[slot][i] = *reinterpret_cast<const f32x4v *>(T + offA[i] + swzk<BK>(rA0 + i * 32, 2 * q + fk) * 16);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[slot][j] = *reinterpret_cast<const f32x4v *>(T + offB[j] + swzk<BK>(rB0 + j * 32, 2 * q + fk) * 16);
    };
    const int tp = t < nk1 ? t : t - nk1;  // k-tile index within its part
    if (tp % FOLD == 0) {  // a numerics block starts (they restart in each part): fold, restart the chain
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = acc[i][j] + part[i][j];
          part[i][j] = zero;
        }
    }
    lread(0, 0);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      // the next group's reads are issued halfway through this group's MFMAs (kept
      // there by the scheduling fences): half a group of MFMAs covers their latency
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u == 2 && q + 1 < NQ) {
          __builtin_amdgcn_sched_barrier(0);
          lread((q + 1) & 1, q + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            part[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[q & 1][i][u], bv[q & 1][j][u], part[i][j], 0, 0, 0);
      }
    }
    barrier_keep(NS == 3 && more);  // tile t+1 landed; every wave done with tile t
    b = b == NS - 1 ? 0 : b + 1;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = acc[i][j] + part[i][j];
  if (a.accum) add_c32<TM, TN>(a, acc, m0 + wm * TM * 32, n0 + wn * TN * 32, lane);

#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int64_t col = n0 + wn * TN * 32 + j * 32 + (lane & 31);
    if (col >= a.N) continue;
    const float bb = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t rbase = m0 + wm * TM * 32 + i * 32 + 4 * (lane >> 5);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = rbase + (r & 3) + 8 * (r >> 2);
        if (row < a.M) a.C[row * a.ldc + col] = epilogue(a, acc[i][j][r], bb, row, col, RELU);
      }
    }
  }
}

template <int WM, int WN, int TM, int TN, int BK, int NS>
lpg_status launch_fc(const FcArgs &a0, bool relu, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32, NT = 64 * WM * WN;
  FcArgs a = a0;
  a.mt = (a.M + BM - 1) / BM;
  a.nt = (a.N + BN - 1) / BN;
  const int64_t nwg = a.mt * a.nt;
  LPG_REQUIRE(nwg < (int64_t)1 << 31, "lpg_fc_f32: grid too large");
  if (relu)
    hipLaunchKernelGGL((fc_fwd_f32<WM, WN, TM, TN, BK, NS, true>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL((fc_fwd_f32<WM, WN, TM, TN, BK, NS, false>), dim3((unsigned)nwg), dim3(NT), 0, s, a);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
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

// add_knowledge on fp16 logits (the reference's --fp16 inference: model.half() makes the heads' outputs
// fp16 and arch.py:129-141 runs in half precision), every stored intermediate rounded to fp16 as torch's
// half ops do (each computes in fp32 and rounds once):
//   n = RNE16(sqrt(fma(x2, x2, fma(x1, x1, x0 * x0))))   (x.norm(dim=1), fp32 accumulation)
//   d = max(n, RNE16(1e-12) = 0)                        (clamp_min(eps) of a half tensor)
//   y = RNE16(RNE16(x / d) * 10)                         (F.normalize(x) * 10)
//   y0 = RNE16(y0 - bound) where feas[:, -3] != 0; y2 likewise where feas[:, -1] != 0
// (a zero row gives 0 / 0 = NaN, as torch's half path does -- the reference's own comment at arch.py:133).
__device__ __forceinline__ float rne16(float v) { return (float)(_Float16)v; }

__global__ __launch_bounds__(256) void knowledge_f16(int64_t M, const uint16_t *__restrict__ logit, int64_t ldl,
                                                     const float *__restrict__ feas, int64_t ldf, int64_t fcols,
                                                     float bound, uint16_t *__restrict__ out, int64_t ldo) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  float x[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) x[c] = (float)__builtin_bit_cast(_Float16, logit[m * ldl + c]);
  const float nrm = rne16(sqrtf(__builtin_fmaf(x[2], x[2], __builtin_fmaf(x[1], x[1], x[0] * x[0]))));
  const float d = nrm > 0.f ? nrm : 0.f;
  float y[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) y[c] = rne16(rne16(x[c] / d) * 10.f);
  if (feas[m * ldf + fcols - 3] != 0.f) y[0] = rne16(y[0] - bound);
  if (feas[m * ldf + fcols - 1] != 0.f) y[2] = rne16(y[2] - bound);
#pragma unroll
  for (int c = 0; c < 3; ++c) out[m * ldo + c] = __builtin_bit_cast(uint16_t, (_Float16)y[c]);
}

// backward of y = normalize(x) * 10 (the mask subtractions have unit derivative), torch autograd's
// formula for F.normalize (arch.py:134-135):
//   dx = 10 (g / d - x (x . g) / d^3) where n > 1e-12, else 10 g / d   (d = max(n, 1e-12))
__global__ __launch_bounds__(256) void knowledge_bwd_f32(int64_t M, const float *__restrict__ logit, int64_t ldl,
                                                         const float *__restrict__ g, int64_t ldg,
                                                         float *__restrict__ dx, int64_t lddx) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const float x[3] = {logit[m * ldl], logit[m * ldl + 1], logit[m * ldl + 2]};
  const float gv[3] = {g[m * ldg], g[m * ldg + 1], g[m * ldg + 2]};
  const float nrm = sqrtf(__builtin_fmaf(x[2], x[2], __builtin_fmaf(x[1], x[1], x[0] * x[0])));
  const float d = nrm < 1e-12f ? 1e-12f : nrm;
  const float xg = x[0] * gv[0] + x[1] * gv[1] + x[2] * gv[2];
  const float d3 = d * d * d;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    dx[m * lddx + c] = nrm > 1e-12f ? 10.f * (gv[c] / d - x[c] * xg / d3) : 10.f * gv[c] / d;
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

// Narrow-input FC (conv1: K1 = K2 = 8 LP features, arch.py:170): the output
// write is the whole cost, so no MFMA tile -- each thread holds the weights of
// 4 output columns in registers and streams rows (staged in LDS, read as
// broadcasts).  Same numerics as the tiled kernel: each part is one numerics
// block (K <= 16 < NB), a chain from +0 in the contract's group-of-8 order
// (pik), added into the +0 total in order -- bitwise identical.
// Position i of a part's chain -> k: groups of 8, inside a group 0,4,1,5,2,6,3,7.
__host__ __device__ constexpr int pik(int i) { return (i & ~7) + (i & 1) * 4 + ((i >> 1) & 3); }
#ifndef LPG_SMALLK_ROWS
#define LPG_SMALLK_ROWS 64
#endif
constexpr int kSmallKRows = LPG_SMALLK_ROWS;

template <int K>
__device__ __forceinline__ void load_row_k(float (&x)[K > 0 ? K : 1], const float *A, int64_t ld, int64_t m) {
#pragma unroll
  for (int k = 0; k < K; k += 4) {
    const float4 v = *reinterpret_cast<const float4 *>(A + m * ld + k);
    x[k] = v.x; x[k + 1] = v.y; x[k + 2] = v.z; x[k + 3] = v.w;
  }
}

template <int K1, int K2, bool RELU, bool SC = false>
__global__ __launch_bounds__(256) void fc_smallk_f32(FcArgs a, int64_t S) {
  static_assert(K1 % 4 == 0 && K2 % 4 == 0 && K1 >= 4, "small-K kernel: K1, K2 multiples of 4");
  constexpr int KT = K1 + K2;
  constexpr int AE = kSmallKRows * KT / 256;  // staged values per thread per chunk
  // Block (column group, s) owns rows [s M / S, (s + 1) M / S) (the grid is about what stays
  // resident, so there is no tail round), walked in chunks of kSmallKRows rows whose [A1 | A2]
  // rows are staged in LDS (double-buffered; the next chunk's values are loaded a chunk ahead,
  // every load of a chunk in flight together -- one at a time the staging cost a memory latency
  // per value); every lane then reads the same row values (LDS broadcast)
  __shared__ __attribute__((aligned(16))) float sx[2][kSmallKRows * KT];
  __shared__ float rmx[SC ? 2 : 1][SC ? 4 : 1][SC ? kSmallKRows : 1];  // SC: per chunk parity and wave
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float cmx[4] = {0.f, 0.f, 0.f, 0.f};  // SC: the thread's column maxima of |C|
  const int64_t sb = blockIdx.y;
  const int64_t rb = sb * a.M / S, re = (sb + 1) * a.M / S;
  if (re <= rb) return;  // (block-uniform)
  const int nch = (int)((re - rb + kSmallKRows - 1) / kSmallKRows);
  float xr_next[AE];
  auto load_x = [&](int64_t r0) {
#pragma unroll
    for (int j = 0; j < AE; ++j) {
      const int i = threadIdx.x + 256 * j, r = i / KT, k = i % KT;
      const int64_t m = r0 + r < re ? r0 + r : re - 1;  // rows past re are never stored
      xr_next[j] = k < K1 ? a.A1[m * a.lda1 + k] : a.A2[m * a.lda2 + (k - K1)];
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int j = 0; j < AE; ++j) sx[buf][threadIdx.x + 256 * j] = xr_next[j];
  };
  const int64_t c = (int64_t)blockIdx.x * 1024 + (int64_t)threadIdx.x * 4;
  const bool col_ok = c < a.N;
  const int64_t cc = col_ok ? c : 0;  // (lanes past N compute column 0 and store nothing)
  float w1[4][K1], w2[4][K2 > 0 ? K2 : 1], b[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    load_row_k<K1>(w1[j], a.W1, a.ldw1, cc + j);
    load_row_k<K2>(w2[j], a.W2, a.ldw2, cc + j);
    b[j] = a.bias ? a.bias[cc + j] : 0.f;
  }
  f32x2 wp1[2][K1], wp2[2][K2 > 0 ? K2 : 1];  // column pairs (0,1), (2,3), packed once
#pragma unroll
  for (int jp = 0; jp < 2; ++jp) {
#pragma unroll
    for (int k = 0; k < K1; ++k) wp1[jp][k] = f32x2{w1[2 * jp][k], w1[2 * jp + 1][k]};
#pragma unroll
    for (int k = 0; k < K2; ++k) wp2[jp][k] = f32x2{w2[2 * jp][k], w2[2 * jp + 1][k]};
  }
  load_x(rb);
  store_x(0);
  __syncthreads();
  if (nch > 1) load_x(rb + kSmallKRows);
  // the row loop with the addend / bias / dropout choices made once per launch (uniform branches
  // per element cost more than the arithmetic of this write-bound kernel); the dropout column keys
  // once per thread, the row key once per row, one hash per column pair -- the mask bits of drop_bits
  auto rows = [&](auto acc_c, auto bias_c, auto drop_c) {
    constexpr bool ACC = decltype(acc_c)::value, BIAS = decltype(bias_c)::value, DROP = decltype(drop_c)::value;
    uint32_t ck[4];
    if constexpr (DROP) {
#pragma unroll
      for (int j = 0; j < 4; ++j) ck[j] = drop_col_key(c + j);
    }
    for (int ch = 0; ch < nch; ++ch) {
      const int64_t r0 = rb + (int64_t)ch * kSmallKRows;
      const int64_t r1 = r0 + kSmallKRows < re ? r0 + kSmallKRows : re;
      const float *xb = sx[ch & 1];
      // one row: its outputs computed and stored; returns the lane's max |output| (SC)
      auto one_row = [&](int64_t m) -> float {
          const float *xr = xb + (m - r0) * KT;
          const uint32_t rk = DROP ? drop_row_key(a.seed, drop_row(a.row_keys, a.row_off, m, a.M)) : 0u;
          float o[4];
          // columns in pairs: one v_pk_fma_f32 advances two independent chains
          // (a true fma per element -- the same bits as the scalar chains)
#pragma unroll
          for (int j = 0; j < 4; j += 2) {
            // each part (<= 16 k) is one numerics block: its own chain from +0, then added to the total
            f32x2 p1 = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < (K1 + 7) / 8 * 8; ++i) {
              const int k = pik(i);
              if (k < K1) p1 = __builtin_elementwise_fma(f32x2{xr[k], xr[k]}, wp1[j / 2][k], p1);
            }
            f32x2 t = f32x2{0.f, 0.f} + p1;
            if (K2 > 0) {
              f32x2 p2 = {0.f, 0.f};
#pragma unroll
              for (int i = 0; i < (K2 + 7) / 8 * 8; ++i) {
                const int k = pik(i);
                if (k < K2) p2 = __builtin_elementwise_fma(f32x2{xr[K1 + k], xr[K1 + k]}, wp2[j / 2][k], p2);
              }
              t = t + p2;
            }
            if constexpr (ACC) t = t + f32x2{a.C[m * a.ldc + c + j], a.C[m * a.ldc + c + j + 1]};
            const uint32_t hp = DROP ? drop_hash_k(rk, ck[j]) : 0u;  // columns c + j, c + j + 1: one pair
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              float v = t[e];
              if constexpr (BIAS) v = v + b[j + e];
              if (RELU) v = (v < 0.f) ? 0.f : v;
              if constexpr (DROP) v = drop_half(hp, e) >= a.drop_thresh ? v * a.drop_scale : 0.f;
              o[j + e] = v;
            }
          }
          *reinterpret_cast<float4 *>(a.C + m * a.ldc + c) = make_float4(o[0], o[1], o[2], o[3]);
          if constexpr (SC) {
#pragma unroll
            for (int e = 0; e < 4; ++e) cmx[e] = fmaxf(cmx[e], fabsf(o[e]));
            return fmaxf(fmaxf(fabsf(o[0]), fabsf(o[1])), fmaxf(fabsf(o[2]), fabsf(o[3])));
          }
          return 0.f;
      };
      if constexpr (SC) {
        // groups of eight rows, every lane taking part in the butterfly (lanes past N contribute 0)
        for (int64_t m8 = r0; m8 < r1; m8 += 8) {
          float xm[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) xm[u] = (col_ok && m8 + u < r1) ? one_row(m8 + u) : 0.f;
          const float w = rowmax8(xm, lane);
          if ((lane & 7) == 0) rmx[ch & 1][wv][(int)(m8 - r0) + rowmax8_slot(lane)] = w;
        }
        lds_barrier();
        if (threadIdx.x < r1 - r0) {  // the chunk's row scales (one column group: whole rows here)
          const float mx = fmaxf(fmaxf(rmx[ch & 1][0][threadIdx.x], rmx[ch & 1][1][threadIdx.x]),
                                 fmaxf(rmx[ch & 1][2][threadIdx.x], rmx[ch & 1][3][threadIdx.x]));
          a.rsc[r0 + threadIdx.x] = f16x2_scale(mx);
        }
      } else if (col_ok) {
        for (int64_t m = r0; m < r1; ++m) one_row(m);
      }
      if (ch + 1 < nch) {  // the next chunk's rows (loaded a chunk ago) into the other buffer
        store_x((ch + 1) & 1);
        lds_barrier();  // (not __syncthreads: its fence would wait for the stores in flight)
        if (ch + 2 < nch) load_x(r0 + 2 * kSmallKRows);
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  const bool acc = a.accum, bias = a.bias != nullptr, drop = a.drop_thresh != 0;
  if constexpr (SC) {  // (conv1's forms: bias, no addend, no dropout)
    if (bias) rows(F_{}, T_{}, F_{}); else rows(F_{}, F_{}, F_{});
    if (col_ok) *reinterpret_cast<float4 *>(a.cpart + sb * a.N + c) = make_float4(cmx[0], cmx[1], cmx[2], cmx[3]);
    return;
  }
  if (acc) {
    if (bias) { if (drop) rows(T_{}, T_{}, T_{}); else rows(T_{}, T_{}, F_{}); }
    else { if (drop) rows(T_{}, F_{}, T_{}); else rows(T_{}, F_{}, F_{}); }
  } else {
    if (bias) { if (drop) rows(F_{}, T_{}, T_{}); else rows(F_{}, T_{}, F_{}); }
    else { if (drop) rows(F_{}, F_{}, T_{}); else rows(F_{}, F_{}, F_{}); }
  }
}

// row ranges of the small-K kernels: the blocks that stay resident, shared by the column
// groups, at least one chunk of rows each
inline int64_t smallk_splits(int64_t M, int64_t ncg, int64_t resident) {
  int64_t s = resident / (ncg > 0 ? ncg : 1);
  const int64_t chunks = (M + kSmallKRows - 1) / kSmallKRows;
  s = s < chunks ? s : chunks;
  return s < 1 ? 1 : s;
}

template <int K1, int K2>
lpg_status launch_smallk(const FcArgs &a, bool relu, hipStream_t s, float *cscale = nullptr) {
  const int64_t ncg = (a.N + 1023) / 1024;
  if (a.rsc) {  // the f16x2 scales of C from the stores (one column group), then the column fold
    auto kern = relu ? fc_smallk_f32<K1, K2, true, true> : fc_smallk_f32<K1, K2, false, true>;
    const int64_t S = smallk_splits(a.M, ncg, resident_blocks(kern, 256));
    hipLaunchKernelGGL(kern, dim3(1u, (unsigned)S), dim3(256), 0, s, a, S);
    LPG_HIP(hipGetLastError());
    hipLaunchKernelGGL(colfold_f32, dim3((unsigned)((a.N + 63) / 64)), dim3(256), 0, s, S, a.N, a.cpart, cscale);
    LPG_HIP(hipGetLastError());
    return LPG_OK;
  }
  auto kern = relu ? fc_smallk_f32<K1, K2, true> : fc_smallk_f32<K1, K2, false>;
  const int64_t S = smallk_splits(a.M, ncg, resident_blocks(kern, 256));
  const dim3 grid((unsigned)ncg, (unsigned)S);
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, a, S);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

// K1, K2 multiples of 4, 4 <= K1, K1 + K2 <= 16; returns false if not covered
bool try_smallk(const FcArgs &a, bool relu, hipStream_t s, lpg_status *st, float *cscale = nullptr) {
  if (a.K1 < 4 || a.K1 + a.K2 > 16 || a.N % 4 || a.ldc % 4 || !aligned16(a.C)) return false;
  if ((a.N + 1023) / 1024 >= 65536) return false;
  if (a.rsc && (a.N > 1024 || a.accum || a.drop_thresh != 0)) return false;
  switch (a.K1 * 100 + a.K2) {
#define LPG_SK(X, Y) case X * 100 + Y: *st = launch_smallk<X, Y>(a, relu, s, cscale); return true;
    LPG_SK(4, 0) LPG_SK(4, 4) LPG_SK(4, 8) LPG_SK(4, 12) LPG_SK(8, 0) LPG_SK(8, 4) LPG_SK(8, 8)
    LPG_SK(12, 0) LPG_SK(12, 4) LPG_SK(16, 0)
#undef LPG_SK
  }
  return false;
}

}  // namespace
}  // namespace lpg

using namespace lpg;

extern "C" lpg_status lpg_fc_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const float *W1,
                                 int64_t ldw1, int64_t K2, const float *A2, int64_t lda2, const float *W2,
                                 int64_t ldw2, const float *bias, float *C, int64_t ldc, int32_t flags,
                                 float dropout_p, uint64_t seed, int64_t row_offset,
                                 const int64_t *row_keys, void *stream) {
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
  FcArgs a{M, N, K1, K2, A1, A2, W1, W2, bias, lda1, lda2, ldw1, ldw2, C, ldc, 0, 0, seed, 0u, 1.f, (flags >> 1) & 1,
           row_offset, row_keys};
  dropout_params(dropout_p, &a.drop_thresh, &a.drop_scale);
  hipStream_t s = as_stream(stream);
  const bool relu = flags & 1;
  lpg_status st;
  if (try_smallk(a, relu, s, &st)) return st;  // conv1: narrow LP features
  LPG_REQUIRE(K1 % 32 == 0 && K2 % 32 == 0,
              "lpg_fc_f32: K1, K2 must be multiples of 32 (zero-pad) unless 4 <= K1, K1 + K2 <= 16 and N %% 4 == 0");
  if (N <= 32) return launch_fc<4, 1, 1, 1, 32, 2>(a, relu, s);  // heads (N = 3): 128 x 32 tiles
  // 128 x 128, 64 KiB: 2 blocks / CU.  (A 3-stage ring, BK = 64, 128 x 256 and 256 x 128 tiles of
  // the same kernel gave the same bits and ran 4-20 % slower; they are not shipped.)
  return launch_fc<2, 2, 2, 2, 32, 2>(a, relu, s);
}

// conv1's narrow FC (the small-K kernel) that also returns C's f16x2 scales from its own stores (the
// next layer's f16x2 GEMMs take C as a row-scaled A operand and a column-scaled weight-gradient
// operand): rscale [M], cscale [N], the values lpg_rowcolscale_f32 gives on C.  LPG_ERR_UNSUPPORTED
// unless the small-K kernel applies with N <= 1024, no addend and no dropout.
extern "C" int64_t lpg_fc_smallk_scales_workspace_bytes(int64_t M, int64_t N) {
  if (M <= 0 || N <= 0) return 0;
  return ((M + kSmallKRows - 1) / kSmallKRows) * N * (int64_t)sizeof(float);
}

extern "C" lpg_status lpg_fc_smallk_scales_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                               const float *W1, int64_t ldw1, int64_t K2, const float *A2,
                                               int64_t lda2, const float *W2, int64_t ldw2, const float *bias,
                                               float *C, int64_t ldc, int32_t flags, float *rscale, float *cscale,
                                               void *scale_ws, void *stream) {
  LPG_REQUIRE(M >= 0 && N >= 0 && K1 >= 0 && K2 >= 0, "lpg_fc_smallk_scales_f32: negative size");
  if (M == 0 || N == 0) return LPG_OK;
  LPG_REQUIRE(C != nullptr && ldc >= N && rscale && cscale && scale_ws && aligned16(scale_ws),
              "lpg_fc_smallk_scales_f32: bad C / scale buffers");
  LPG_REQUIRE(K1 == 0 || (A1 && W1 && lda1 >= K1 && ldw1 >= K1), "lpg_fc_smallk_scales_f32: bad A1/W1");
  LPG_REQUIRE(K2 == 0 || (A2 && W2 && lda2 >= K2 && ldw2 >= K2), "lpg_fc_smallk_scales_f32: bad A2/W2");
  LPG_REQUIRE(K1 % 4 == 0 && K2 % 4 == 0 && lda1 % 4 == 0 && ldw1 % 4 == 0 && (K2 == 0 || (lda2 % 4 == 0 && ldw2 % 4 == 0)),
              "lpg_fc_smallk_scales_f32: K and leading dimensions must be multiples of 4 floats");
  LPG_REQUIRE(aligned16(A1) && aligned16(W1) && (K2 == 0 || (aligned16(A2) && aligned16(W2))),
              "lpg_fc_smallk_scales_f32: A/W must be 16-byte aligned");
  LPG_REQUIRE((flags & ~1) == 0, "lpg_fc_smallk_scales_f32: only the ReLU flag (no addend) 0x%x", flags);
  FcArgs a{M, N, K1, K2, A1, A2, W1, W2, bias, lda1, lda2, ldw1, ldw2, C, ldc, 0, 0, 0u, 0u, 1.f, 0, 0, nullptr};
  a.rsc = rscale;
  a.cpart = static_cast<float *>(scale_ws);
  lpg_status st;
  if (try_smallk(a, flags & 1, as_stream(stream), &st, cscale)) return st;
  set_error("lpg_fc_smallk_scales_f32: the small-K kernel does not take these operands (K1 >= 4, K1 + K2 <= 16, "
            "N <= 1024, N and ldc multiples of 4, C 16-byte aligned)");
  return LPG_ERR_UNSUPPORTED;
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

extern "C" lpg_status lpg_knowledge_bwd_f32(int64_t M, const float *logit, int64_t ldl, const float *g, int64_t ldg,
                                            float *dx, int64_t lddx, void *stream) {
  LPG_REQUIRE(M >= 0, "lpg_knowledge_bwd_f32: M < 0");
  if (M == 0) return LPG_OK;
  LPG_REQUIRE(logit && g && dx, "lpg_knowledge_bwd_f32: NULL pointer");
  LPG_REQUIRE(ldl >= 3 && ldg >= 3 && lddx >= 3, "lpg_knowledge_bwd_f32: bad shapes");
  hipLaunchKernelGGL(knowledge_bwd_f32, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, as_stream(stream), M, logit,
                     ldl, g, ldg, dx, lddx);
  LPG_HIP(hipGetLastError());
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

extern "C" lpg_status lpg_knowledge_f16(int64_t M, const uint16_t *logit, int64_t ldl, const float *feas, int64_t ldf,
                                        int64_t feas_cols, float bound, uint16_t *out, int64_t ldo, void *stream) {
  LPG_REQUIRE(M >= 0, "lpg_knowledge_f16: M < 0");
  if (M == 0) return LPG_OK;
  LPG_REQUIRE(logit && feas && out, "lpg_knowledge_f16: NULL pointer");
  LPG_REQUIRE(ldl >= 3 && ldo >= 3 && feas_cols >= 3 && ldf >= feas_cols, "lpg_knowledge_f16: bad shapes");
  hipLaunchKernelGGL(knowledge_f16, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, as_stream(stream), M, logit,
                     ldl, feas, ldf, feas_cols, bound, out, ldo);
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}
