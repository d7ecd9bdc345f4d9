/*
 * lpgnn.h — C ABI of liblpgnn_hip.so, the MI355X (gfx950) hot path of the
 * LP basis-prediction GNN (vbdai/lp-gnn, GCN_FC).
 *
 * The library replaces the native op the reference reaches through PyG:
 *
 *   arch.py:75-80  GraphConv(...)(x, adj_t)            (PyG 2.1 GraphConv, aggr='add')
 *     -> torch_sparse.matmul(adj_t, x[0], reduce='add')  (torch_sparse 0.6.12 matmul.py)
 *     -> torch.ops.torch_sparse.spmm_sum(row, rowptr, col, value, colptr, csr2csc, mat)
 *        (torch_sparse 0.6.12 csrc/spmm.cpp SPMMSum; CPU csrc/cpu/spmm_cpu.cpp)
 *
 * and the COO->CSR / CSR->CSC conversions of the batch boundary:
 *
 *   dataset.py:301-304  SparseTensor.from_edge_index(edge_index_l2r, edge_attr, (ncons, nvars))
 *   arch.py:71          edge_index.t()   (csr2csc permutation, every layer)
 *
 * Conventions (all entry points):
 *   - plain C types only; every buffer is caller-owned; device pointers are
 *     hipMalloc'd (or torch) memory on the current device; the library never
 *     allocates on the hot path.
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream); all
 *     device work is stream-ordered and the calls are re-entrant.
 *   - return value: LPG_OK or an error code; lpg_last_error() gives a
 *     thread-local message (the C analogue of TORCH_CHECK's RuntimeError).
 *   - determinism: no atomics on any floating-point path; results are
 *     bitwise identical run to run and equal to the sequential CPU loop of
 *     torch_sparse spmm_cpu (per-row edge order, product rounded then added).
 */
#ifndef LPGNN_H
#define LPGNN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t lpg_status;
#define LPG_OK 0
#define LPG_ERR_INVALID 1     /* bad argument / shape / alignment            */
#define LPG_ERR_HIP 2         /* a HIP runtime call failed                     */
#define LPG_ERR_UNSUPPORTED 3 /* valid request this build does not implement   */

/* One orientation of the bipartite adjacency, CSR with sorted columns.
 * Row i of the destination side gathers rows col[rowptr[i]..rowptr[i+1]) of
 * the source feature matrix, weighted by val[].  (torch_sparse SparseStorage:
 * rowptr/col/value; rows = destination nodes of the message direction.) */
typedef struct lpg_csr {
  int64_t n_rows;         /* destination nodes                               */
  int64_t n_cols;         /* source nodes (rows of X)                        */
  int64_t nnz;            /* edges                                           */
  const int64_t *rowptr;  /* [n_rows+1]                                      */
  const int32_t *col;     /* [nnz], ascending within each row                */
  const float *val;       /* [nnz], scaled A_ij (dataset.py:235-236)         */
} lpg_csr;

/* ---- errors / build info ------------------------------------------------ */
const char *lpg_last_error(void);
/* "gfx950" + build flags; never NULL. */
const char *lpg_build_info(void);

/* ---- dual-CSR pack (replaces from_edge_index + .t()) --------------------- */

/* Host pack.  Input: COO edges of A (rows = constraints, cols = variables)
 * as produced by MyToBipartite (dataset.py:296-304): int64 row/col, f32 val,
 * any order, no duplicate (row, col) pairs.  Output (caller-allocated host
 * buffers): CSR(A) [m rows] and CSR(A^T) [n rows], columns ascending within
 * each row, i.e. torch_sparse's from_edge_index order and its csr2csc order
 * (SparseTensor.t()).  Duplicates -> LPG_ERR_INVALID. */
lpg_status lpg_csr_pack_host(const int64_t *row, const int64_t *col, const float *val,
                             int64_t nnz, int64_t m, int64_t n,
                             int64_t *a_rowptr, int32_t *a_col, float *a_val,
                             int64_t *at_rowptr, int32_t *at_col, float *at_val);

/* Device pack: same contract and bit-identical output, all pointers device
 * memory, stream-ordered (no host sync).  `workspace` (16-byte aligned) must
 * hold lpg_csr_pack_workspace_bytes(nnz, m, n) bytes.  Because validation
 * cannot return through the status without a sync, the first 16 bytes of the
 * workspace receive two int64 counters after the pack: [0] edges with an
 * out-of-range index, [1] duplicate (row, col) pairs.  Non-zero => the
 * output is undefined and the caller must report LPG_ERR_INVALID itself. */
int64_t lpg_csr_pack_workspace_bytes(int64_t nnz, int64_t m, int64_t n);
lpg_status lpg_csr_pack_f32(const int64_t *row, const int64_t *col, const float *val,
                            int64_t nnz, int64_t m, int64_t n,
                            int64_t *a_rowptr, int32_t *a_col, float *a_val,
                            int64_t *at_rowptr, int32_t *at_col, float *at_val,
                            void *workspace, void *stream);

/* ---- SpMM (replaces torch_sparse spmm_sum, forward and backward) --------- */

/* Y[i, 0:F] = sum_{e in row i} val[e] * X[col[e], 0:F]   (Y overwritten).
 * X: [A->n_cols, >= F] row stride ldx floats; Y: [A->n_rows, >= F] stride ldy.
 * fp32 storage and accumulation, sequential edge order per row.
 * The backward of spmm(A, X) w.r.t. X is spmm(A^T, dY): call this entry on
 * the other orientation (torch_sparse SPMMSum::backward). */
lpg_status lpg_spmm_f32(const lpg_csr *A, const float *X, int64_t ldx,
                        float *Y, int64_t ldy, int64_t F, void *stream);
/* lpg_spmm_f32[_heavy] with explicit per-call tuning (benchmarks / tests; no
 * global state): heavy_rows / n_heavy / thresh as lpg_spmm_f32_heavy (NULL, 0,
 * 0 = none); slice_cols = columns of F one wave task covers (0 = auto, or 64,
 * 128, 256, 512, 1024; the slices run plane by plane, so a narrower slice
 * keeps the gathered source slice resident in the 256 MiB Infinity Cache),
 * depth = edges gathered ahead per wave (0 = auto, 8, 16, 32).  Every choice
 * gives bitwise lpg_spmm_f32's result (the per-element summation order is
 * always the row's CSR order). */
lpg_status lpg_spmm_f32_tuned(const lpg_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                              const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh, int64_t slice_cols,
                              int32_t depth, void *stream);

/* lpg_spmm_f32 with degree-aware scheduling for skewed rows: heavy_rows
 * (device int32 [n_heavy]) must list exactly the rows of A with more than
 * `thresh` edges (longest first is fastest).  Those rows run as (row,
 * 64-column) wave units, all at the head of the launch, instead of (row,
 * 128/256-column) units, so a long constraint row's sequential chain is
 * spread over 4x the waves and starts first; every element is still summed
 * over its row's edges in CSR order -- the result is bitwise lpg_spmm_f32's.
 * F < 256 and unaligned shapes ignore the list.  Same fwd/bwd use as
 * lpg_spmm_f32 (torch_sparse spmm_sum / SPMMSum). */
lpg_status lpg_spmm_f32_heavy(const lpg_csr *A, const float *X, int64_t ldx,
                              float *Y, int64_t ldy, int64_t F,
                              const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh,
                              void *stream);

/* ---- multi-GPU: the row-partitioned SpMM (SURVEY.md §8b "Multi-GPU", §8e) ---------------------
 *
 * One rank per GPU holds a block of constraint rows and the variables they touch (boundary
 * variables: touched by >= 2 ranks).  vars<-cons over the local edges gives full sums for the
 * variables only this rank touches and partial sums for the boundary ones; these entries sum the
 * boundary rows over the ranks with one RCCL all-reduce of a dense [n_boundary, F] buffer, so every
 * rank ends with the full sums of the boundary rows it holds (the same bits on every rank).  The
 * communicator is RCCL's (rccl.h's ncclComm_t), made here from a unique id that rank 0 draws and the
 * caller distributes (any side channel: torch.distributed, MPI, a file).  RCCL is resolved at run
 * time (the copy the process already loaded first), so only these entries need it.
 * Replaces nothing in the reference (no distributed code: train.py:81-82); lpgnn.partition's
 * Python exchange is the sparse owner form of the same sum. */
typedef struct ncclComm *ncclComm_t; /* as rccl.h */
#define LPG_COMM_ID_BYTES 128        /* NCCL_UNIQUE_ID_BYTES */
/* a fresh unique id into id[LPG_COMM_ID_BYTES] (host memory), on ONE rank */
lpg_status lpg_comm_unique_id(void *id);
/* this rank's communicator over nranks ranks on the current device (collective: every rank calls it
 * with the same id) */
lpg_status lpg_comm_init(ncclComm_t *comm, int32_t nranks, const void *id, int32_t rank);
lpg_status lpg_comm_destroy(ncclComm_t comm);
lpg_status lpg_comm_info(ncclComm_t comm, int32_t *nranks, int32_t *rank);

/* Its two halves, for a caller that runs the collective itself (MPI, another RCCL wrapper): pack
 * copies the mapped rows of Y into boundary_buf in boundary order (zero rows for -1); unpack copies
 * boundary_buf's rows back into the mapped rows.  Stream-ordered, no collective. */
lpg_status lpg_boundary_pack_f32(const float *Y, int64_t ldy, int64_t rows, int64_t F, int64_t n_boundary,
                                 const int32_t *boundary_map, float *boundary_buf, void *stream);
lpg_status lpg_boundary_unpack_f32(float *Y, int64_t ldy, int64_t rows, int64_t F, int64_t n_boundary,
                                   const int32_t *boundary_map, const float *boundary_buf, void *stream);
/* The boundary exchange alone: boundary_map (device int32 [n_boundary], the same global boundary
 * order on every rank) gives the row of Y holding boundary variable b on this rank, or -1 when this
 * rank does not touch it; boundary_buf: device fp32 [n_boundary, F] workspace.  Packs those rows
 * (zero rows for -1), all-reduces (sum) the buffer over comm on `stream`, and writes the sums back
 * into the mapped rows; other rows of Y are untouched.  Collective: every rank calls it with the same
 * n_boundary and F.  Entries of boundary_map outside [0, rows) count as -1. */
lpg_status lpg_boundary_allreduce_f32(float *Y, int64_t ldy, int64_t rows, int64_t F, int64_t n_boundary,
                                      const int32_t *boundary_map, float *boundary_buf, ncclComm_t comm,
                                      void *stream);
/* lpg_spmm_f32(A, X) on this rank's local CSR (rows = local variables for vars<-cons), then
 * lpg_boundary_allreduce_f32 on its rows.  The backward w.r.t. X of a partitioned cons<-vars product
 * is this entry on A^T; cons<-vars itself needs no exchange (lpg_spmm_f32). */
lpg_status lpg_spmm_partitioned_f32(const lpg_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy, int64_t F,
                                    int64_t n_boundary, const int32_t *boundary_map, float *boundary_buf,
                                    ncclComm_t comm, void *stream);

/* Same, bf16 storage (uint16 bit patterns) with fp32 accumulation; the
 * accumulated row is rounded to bf16 once (round-to-nearest-even). */
lpg_status lpg_spmm_bf16(const lpg_csr *A, const uint16_t *X, int64_t ldx,
                         uint16_t *Y, int64_t ldy, int64_t F, void *stream);
/* ... with per-call tuning as lpg_spmm_f32_tuned (slice_cols 0 = auto = 256,
 * 256, 512, 1024; depth for the 256-column form); bitwise lpg_spmm_bf16's. */
lpg_status lpg_spmm_bf16_tuned(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy, int64_t F,
                               const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh, int64_t slice_cols,
                               int32_t depth, void *stream);
/* ... and its degree-aware form (heavy_rows as lpg_spmm_f32_heavy; the heavy
 * units are (row, 128-column) waves); bitwise lpg_spmm_bf16's result. */
lpg_status lpg_spmm_bf16_heavy(const lpg_csr *A, const uint16_t *X, int64_t ldx,
                               uint16_t *Y, int64_t ldy, int64_t F,
                               const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh,
                               void *stream);
/* fp16 storage (the reference's --fp16 inference mode: model.half() and the batch's
 * SparseTensor.half(), val.py:269, utils.py:909-915): X, Y fp16 bit patterns, edge values fp32 (holding
 * the fp16-rounded values), fp32 accumulation in CSR edge order, one RNE rounding to fp16 per output
 * (torch_sparse 0.6.12's CUDA spmm_sum accumulates in the storage type; the fp32 sum is the more
 * accurate).  Layout rules, tuning and kernels as lpg_spmm_bf16(_tuned). */
lpg_status lpg_spmm_f16(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy, int64_t F,
                        void *stream);
lpg_status lpg_spmm_f16_tuned(const lpg_csr *A, const uint16_t *X, int64_t ldx, uint16_t *Y, int64_t ldy, int64_t F,
                              const int32_t *heavy_rows, int64_t n_heavy, int64_t thresh, int64_t slice_cols,
                              int32_t depth, void *stream);

/* ---- dense FC (replaces GraphConv's lin_rel + lin_root + ReLU) ----------- */

/* FC flags (lpg_fc_f32, lpg_fc_x3_f32, lpg_fc_x3_heads_f32, lpg_fc_bf16,
 * lpg_fc_bf16_relu_bwd): bit 0 = ReLU (+ fused dropout), bit 1 = accumulate,
 * bits 8-11 = kernel choice, 0 = by shape.  Every kernel choice of one entry
 * computes the same bits (the tests compare them); the choice exists so that
 * benchmarks and tests can pick a kernel per call, without global state.
 *   lpg_fc_x3_f32 / _heads: 1 = fc_fwd_x3_16 (global_load_lds staging), 2 = the default kernel
 *     in round 3's tile order (each XCD walks contiguous m-tiles with all their n-tiles; the default
 *     is the n-split order: half the XCDs take the first half of the n-tiles), 3 = the default kernel
 *     in the n-quarter order (XCD pairs take a quarter of the n-tiles each);
 *   lpg_fc_bf16 / _relu_bwd: 1 = 128 x 128 tiles, 2 = 256 x 256 tiles,
 *     3 = the pipelined 256 x 256 kernel (the default from 4096 rows, there in the n-split tile
 *     order), 4 / 5 = the default choice with the pipelined kernel in the m-major / n-quarter
 *     tile order, 6 = the persistent stream-K form (lpg_fc16 with a workspace only), 7 = two 4-wave
 *     blocks per CU on 128 x 256 tiles with one LDS stage (fc_bf16_q; measured 3-10 % slower than
 *     the default, profiles/r05_q_ab.log). */
#define LPG_FC_RELU 1
#define LPG_FC_ACCUMULATE 2
#define LPG_FC_HEADS_ONLY 4 /* lpg_fc_x3_heads_f32 only: C is not written (the logits are the only output;
                             * with LPG_FC_ACCUMULATE C still supplies the addend, else C may be NULL):
                             * the no-grad forward of the last layer, whose output feeds only the heads */
#define LPG_FC_KERNEL(k) ((int32_t)(k) << 8)

/* C[m, n] = act( sum_{k<K1} A1[m,k] W1[n,k] + sum_{k<K2} A2[m,k] W2[n,k] + bias[n] )
 *
 * PyG 2.1 GraphConv.forward after propagate, as built at arch.py:57-62 and
 * applied at arch.py:75-80: lin_rel(agg) + lin_root(x_dst), with W in the
 * torch Linear layout [out, in] (A1 = agg, W1 = lin_rel.weight, bias =
 * lin_rel.bias, A2 = x_dst, W2 = lin_root.weight).  With K2 = 0 it is a plain
 * Linear (heads lin_left / lin_right, arch.py:175-176, 190).
 * flags: bit 0 = ReLU epilogue (arch.py:182, 188); bit 1 = accumulate: C
 * holds an addend P on entry and C = act(A1 W1^T + A2 W2^T + P + bias), in
 * place (GraphConv re-associated as lin_root(x_dst) + S (x_src W_rel^T) + b,
 * with S (x_src W_rel^T) computed by lpg_fc_f32 + lpg_spmm_f32 into C first).
 * bias may be NULL.
 * dropout_p > 0 fuses F.dropout after the ReLU (arch.py:186-188, training):
 * element (m, n) is kept iff its 16 mask bits -- half of the 32-bit
 * lowbias32 hash of (seed, key(m), n / 2): the low half for even n, the high
 * half for odd n -- are >= round(dropout_p * 2^16), and kept values are
 * scaled by 1 / (1 - dropout_p) (oracle/dropout_ref.py restates the mask).  The mask is never stored: the
 * kept set is exactly where the output is > 0.  The hash keys row m as
 * row_keys[m] when row_keys != NULL (device int64 [M]: the global node id of
 * every row, e.g. a partition's owned variables, which need not be
 * contiguous), else as row_offset + m: a caller computing a slice of a larger
 * node set (the row partition, lpgnn/partition.py) passes the slice's global
 * ids, so every node's mask is the one a single-GPU run would draw.
 * Row-major fp32, leading dimensions in floats; A/W leading dimensions
 * multiples of 4, A/W 16-byte aligned; K1 and K2 multiples of 32 (zero-pad:
 * padded k are exact no-ops), except for the narrow-input kernel (4 <= K1,
 * K1 + K2 <= 16, K multiples of 4, N and ldc multiples of 4) -- otherwise
 * LPG_ERR_INVALID.
 * Numerics (bitwise reproducible, see oracle/fc_ref.c): each part (A1 over
 * K1, then A2 over K2) is cut into blocks of 128 k (the last one shorter); a
 * block's products form one fp32 fma chain from +0, its k visited in groups
 * of 8 consecutive k, inside a group in the order 0,4,1,5,2,6,3,7 (the
 * 32x32x2 MFMA operand order of the tiled kernel); the block sums are added
 * in order into the running total (+0 initially), then + P (accumulate),
 * then + bias, then ReLU. */
lpg_status lpg_fc_f32(int64_t M, int64_t N,
                      int64_t K1, const float *A1, int64_t lda1, const float *W1, int64_t ldw1,
                      int64_t K2, const float *A2, int64_t lda2, const float *W2, int64_t ldw2,
                      const float *bias, float *C, int64_t ldc, int32_t flags,
                      float dropout_p, uint64_t seed, int64_t row_offset, const int64_t *row_keys, void *stream);
/* lpg_fc_f32's small-K form (conv1: 4 <= K1, K1 + K2 <= 16) that also returns C's f16x2 scales from
 * its own stores (rscale [M], cscale [N]: the values lpg_rowcolscale_f32 gives on C); flags: the ReLU
 * bit only (no addend, no dropout), N <= 1024; scale_ws lpg_fc_smallk_scales_workspace_bytes(M, N)
 * bytes, 16-byte aligned.  LPG_ERR_UNSUPPORTED when the small-K kernel does not take the operands. */
int64_t lpg_fc_smallk_scales_workspace_bytes(int64_t M, int64_t N);
lpg_status lpg_fc_smallk_scales_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const float *W1,
                                    int64_t ldw1, int64_t K2, const float *A2, int64_t lda2, const float *W2,
                                    int64_t ldw2, const float *bias, float *C, int64_t ldc, int32_t flags,
                                    float *rscale, float *cscale, void *scale_ws, void *stream);

/* fp32 FC on the bf16 matrix cores (same operation and epilogue as
 * lpg_fc_f32; also the input-gradient GEMMs dZ W of its backward, with W
 * given transposed).  A1/A2 fp32 as in lpg_fc_f32 (K1, K2 multiples of 32,
 * lda multiples of 4, 16-byte aligned); W1/W2 PRE-SPLIT by lpg_split3_f32
 * into three bf16 planes (plane p at W + p * ps, [N, K] with leading
 * dimension ldw, ldw and ps multiples of 8, 16-byte aligned).  Each fp32
 * operand is split exactly, a = a0 + a1 + a2 (bf16 terms, RNE), and the
 * product keeps the six terms down to 2^-16 relative size (the three dropped
 * terms are <= 2^-23 |a b|, below the fp32 rounding of the product);
 * bf16 x bf16 products are exact and accumulate in fp32 (a0 b0 and the small
 * terms in separate accumulators).  fp32-GEMM accuracy at 6/16 of the fp32
 * MFMA cost; not bitwise reproducible on the CPU (the bf16 MFMA's internal
 * summation order is unspecified) -- lpg_fc_f32 keeps the bitwise contract.
 * flags, bias, dropout as lpg_fc_f32. */
lpg_status lpg_fc_x3_f32(int64_t M, int64_t N,
                         int64_t K1, const float *A1, int64_t lda1, const uint16_t *W1, int64_t ldw1, int64_t ps1,
                         int64_t K2, const float *A2, int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2,
                         const float *bias, float *C, int64_t ldc, int32_t flags,
                         float dropout_p, uint64_t seed, int64_t row_offset, const int64_t *row_keys, void *stream);

/* The exact three-way bf16 split of an fp32 matrix for lpg_fc_x3_f32:
 * plane p of dst ([rows, cols], leading dimension ldd, plane p at
 * dst + p * plane_stride) holds term p of S, S = src ([rows, cols], lds) or,
 * with transpose != 0, S = src^T (src [cols, rows]).  t0 = RNE_bf16(x),
 * t1 = RNE_bf16(x - t0), t2 = RNE_bf16(x - t0 - t1) = x - t0 - t1 exactly. */
lpg_status lpg_split3_f32(int64_t rows, int64_t cols, const float *src, int64_t lds, int32_t transpose,
                          uint16_t *dst, int64_t ldd, int64_t plane_stride, void *stream);

/* lpg_fc_x3_f32 with the heads fused into its epilogue: besides C, writes
 * logits[m, c] = sum_n C[m, n] hw[c, n] + hb[c] for c < hn (hn <= 4; hw
 * [hn, ldhw] fp32, hb may be NULL) -- lin_left / lin_right (arch.py:175-176,
 * 190) applied to the last hidden layer's output (arch.py:184-188) without
 * re-reading it.  Each 128-column tile's partial sums go to `workspace`
 * (lpg_fc_x3_heads_workspace_bytes(M, N) bytes, 16-byte aligned) and are added
 * in column order: deterministic, fp32-rounding-equal to the separate Linear
 * (not bitwise: a different summation order). */
int64_t lpg_fc_x3_heads_workspace_bytes(int64_t M, int64_t N);
lpg_status lpg_fc_x3_heads_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                               const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                               int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *bias,
                               float *C, int64_t ldc, int32_t flags, float dropout_p, uint64_t seed,
                               int64_t row_offset, const int64_t *row_keys, int32_t hn, const float *hw, int64_t ldhw,
                               const float *hb, float *logits, int64_t ldl, void *workspace, void *stream);

/* An input-gradient GEMM of lpg_fc_x3_f32 (same A / W / K / lda / ldw / plane arguments; flags: only
 * LPG_FC_ACCUMULATE, C then holding the addend, read and never written) whose result g [M, N] is the
 * gradient of a ReLU layer's output Y [M, N] (ldy) computed from ks1 + ks2 <= 16 input features
 * X1 [M, ks1], X2 [M, ks2] -- conv1 of GCN_FC (arch.py:170, 181-182), no dropout: instead of storing g,
 * the epilogue forms dZ = (Y > 0) ? g : 0 and each 128-row tile writes its partial sums of
 * dZ^T [X1 | X2 | 1] to the workspace, folded in tile order into that layer's weight gradients
 *   dW1 [N, ks1] = dZ^T X1,  dW2 [N, ks2] = dZ^T X2,  db [N] = sum_m dZ   (any of them may be NULL)
 * -- the gradient never makes the round trip through HBM that lpg_relu_wgrad_smallk_f32 reads back.
 * Tolerance-level like every weight gradient here (fp32 fma chains per tile, tiles folded in order;
 * deterministic).  Needs the wide x3 kernel's operand rules (lda1 == lda2, ldw1 == ldw2, ps1 == ps2)
 * -- otherwise LPG_ERR_INVALID and the caller takes the two-pass route.  Workspace:
 * lpg_fc_x3_relu_wgrad_workspace_bytes(M, N, ks1 + ks2), 16-byte aligned. */
int64_t lpg_fc_x3_relu_wgrad_workspace_bytes(int64_t M, int64_t N, int64_t K);
lpg_status lpg_fc_x3_relu_wgrad_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                    const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                                    int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *C,
                                    int64_t ldc, int32_t flags, const float *Y, int64_t ldy, int64_t ks1,
                                    const float *X1, int64_t ldx1, int64_t ks2, const float *X2, int64_t ldx2,
                                    float *dW1, float *dW2, float *db, void *workspace, void *stream);

/* ---- f16x2: the same three entries on two fp16 terms per operand (the default arithmetic, round 5) ----
 * Each row of [A1 | A2] is multiplied by a power of two sa[m] (lpg_rowscale_f32: its largest |x| lands
 * in [2^14, 2^15)) and split in registers into h = RNE_f16(x sa), l = RNE_f16(x sa - h); W is given as
 * two fp16 planes of [W1 | W2] rows times their own power of two sw[n] (lpg_split_f16x2: plane 0 = h,
 * plane 1 = l, at W + p * ps).  Per (m, n): hh + (hl + lh) in fp32 (three v_mfma_f32_16x16x32_f16,
 * half x3's six), then times 1 / (sa[m] sw[n]) (exact) and the same epilogue.  Representation error
 * <= ~3 * 2^-22 of sum |a b| -- a quarter of an fp32 SGEMM's own error (tools/experiments/
 * split_error.py); per-row scales keep every row's relative accuracy whatever the spread between rows.
 * The other arguments and rules are the x3 entries'; operands the wide kernel does not take (lda1 !=
 * lda2, ldw1 != ldw2, ps1 != ps2; heads hn = 4) return LPG_ERR_UNSUPPORTED and the caller runs x3. */
lpg_status lpg_rowscale_f32(int64_t M, int64_t K1, const float *A1, int64_t lda1, int64_t K2, const float *A2,
                            int64_t lda2, float *scale, void *stream);
/* rows of [src1 | src2] (columns with transpose != 0) times their shared scale, as two fp16 planes each:
 * dst1 / dst2 [rows, ldd] with plane 1 at + plane_stride, zero columns past cols left to the caller. */
lpg_status lpg_split_f16x2(int64_t rows, int64_t cols1, const float *src1, int64_t lds1, int64_t cols2,
                           const float *src2, int64_t lds2, int32_t transpose, uint16_t *dst1, int64_t ldd1,
                           uint16_t *dst2, int64_t ldd2, int64_t plane_stride, float *scale, void *stream);
lpg_status lpg_fc_f16x2_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const uint16_t *W1,
                            int64_t ldw1, int64_t ps1, int64_t K2, const float *A2, int64_t lda2, const uint16_t *W2,
                            int64_t ldw2, int64_t ps2, const float *sa, const float *sw, const float *bias, float *C,
                            int64_t ldc, int32_t flags, float dropout_p, uint64_t seed, int64_t row_offset,
                            const int64_t *row_keys, void *stream);
lpg_status lpg_fc_f16x2_heads_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                  const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                                  int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *sa,
                                  const float *sw, const float *bias, float *C, int64_t ldc, int32_t flags,
                                  float dropout_p, uint64_t seed, int64_t row_offset, const int64_t *row_keys,
                                  int32_t hn, const float *hw, int64_t ldhw, const float *hb, float *logits,
                                  int64_t ldl, void *workspace, void *stream);
lpg_status lpg_fc_f16x2_relu_wgrad_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1,
                                       const uint16_t *W1, int64_t ldw1, int64_t ps1, int64_t K2, const float *A2,
                                       int64_t lda2, const uint16_t *W2, int64_t ldw2, int64_t ps2, const float *sa,
                                       const float *sw, const float *C, int64_t ldc, int32_t flags, const float *Y,
                                       int64_t ldy, int64_t ks1, const float *X1, int64_t ldx1, int64_t ks2,
                                       const float *X2, int64_t ldx2, float *dW1, float *dW2, float *db,
                                       void *workspace, void *stream);

/* Weight gradient on the same arithmetic: dW[n, k] = sum_r G[r, n] X[r, k]
 * (G = dZ [R, N], ldg; X = the layer input [R, K], ldx; dW [N, K], lddw, the
 * torch Linear weight layout) -- the lin_rel / lin_root weight gradients of
 * GraphConv's backward.  N, K and the leading dimensions multiples of 4
 * floats, buffers 16-byte aligned.  R is split into contiguous ranges whose
 * partial products go to `workspace` (lpg_wgrad_x3_workspace_bytes(R, N, K)
 * bytes, 16-byte aligned) and are added in a fixed order: deterministic. */
int64_t lpg_wgrad_x3_workspace_bytes(int64_t R, int64_t N, int64_t K);
lpg_status lpg_wgrad_x3_f32(int64_t R, int64_t N, int64_t K, const float *G, int64_t ldg, const float *X,
                            int64_t ldx, float *dW, int64_t lddw, void *workspace, void *stream);
/* The weight gradient in f16x2: G column n and X column k times their power-of-2 column scales sG[n],
 * sX[k] (lpg_colscale_f32: each column's largest |x| over the R rows in [2^14, 2^15)), two fp16 terms
 * each, three products; otherwise lpg_wgrad_x3_f32 (same workspace, deterministic fold). */
lpg_status lpg_wgrad_f16x2_f32(int64_t R, int64_t N, int64_t K, const float *G, int64_t ldg, const float *X,
                               int64_t ldx, const float *sG, const float *sX, float *dW, int64_t lddw,
                               void *workspace, void *stream);
int64_t lpg_colscale_workspace_bytes(int64_t R, int64_t N);
lpg_status lpg_colscale_f32(int64_t R, int64_t N, const float *G, int64_t ldg, float *scale, void *workspace,
                            void *stream);
/* Both scales of one operand in one read (the same values as lpg_rowscale_f32 on G alone and
 * lpg_colscale_f32): rscale [R], cscale [N]; workspace lpg_rowcolscale_workspace_bytes(R, N) bytes. */
int64_t lpg_rowcolscale_workspace_bytes(int64_t R, int64_t N);
lpg_status lpg_rowcolscale_f32(int64_t R, int64_t N, const float *G, int64_t ldg, float *rscale, float *cscale,
                               void *workspace, void *stream);

/* Backward of ReLU (+ fused dropout): out[i] = y[i] > 0 ? g[i] * scale : 0,
 * y = the stored lpg_fc_f32 output, scale = 1/(1-p) (1 without dropout).
 * n a multiple of 4, buffers 16-byte aligned; out may alias g. */
lpg_status lpg_relu_dropout_bwd_f32(int64_t n, const float *g, const float *y, float scale, float *out,
                                    void *stream);

/* Same with the bias gradient fused: Y/out [M, N] row-major (ldy/ldo, N and
 * strides multiples of 4), and db[n] = sum_m out[m, n] when db != NULL
 * (deterministic two-pass column sum through `workspace`,
 * lpg_relu_bwd_colsum_workspace_bytes(M, N) bytes, 16-byte aligned). */
int64_t lpg_relu_bwd_colsum_workspace_bytes(int64_t M, int64_t N);
lpg_status lpg_relu_bwd_colsum_f32(int64_t M, int64_t N, const float *g, int64_t ldg, const float *y,
                                   int64_t ldy, float scale, float *out, int64_t ldo, float *db,
                                   void *workspace, void *stream);

/* bf16 twin (c5 path): g, y, out bf16 (uint16), N and leading dims multiples
 * of 8; dZ = bf16(g * scale) where y > 0; db (fp32) = column sums of dZ.
 * Workspace: lpg_relu_bwd_colsum_workspace_bytes(M, N). */
lpg_status lpg_relu_bwd_colsum_bf16(int64_t M, int64_t N, const uint16_t *g, int64_t ldg, const uint16_t *y,
                                    int64_t ldy, float scale, uint16_t *out, int64_t ldo, float *db,
                                    void *workspace, void *stream);
/* Column sums only (db[n] = sum_m g[m, n], fp32) of a bf16 dZ that already went
 * through its ReLU / dropout backward -- the output of lpg_fc_bf16_relu_bwd.
 * Same blocks and fold as lpg_relu_bwd_colsum_bf16, so the same db bits for the
 * same dZ.  Replaces the bias-gradient half of that pass in the folded c5
 * backward (torch's `db = dZ.sum(0)` of the Linear, arch.py:57-62 via
 * train.py:128 loss.backward()).  Workspace: lpg_relu_bwd_colsum_workspace_bytes. */
lpg_status lpg_colsum_bf16(int64_t M, int64_t N, const uint16_t *g, int64_t ldg, float *db, void *workspace,
                           void *stream);

/* Weight gradients of a GraphConv whose inputs are narrow (conv1: the 8 LP
 * features, arch.py:170): dW1 = dZ^T A1 [N, K1], dW2 = dZ^T A2 [N, K2], in the
 * torch weight layout, 1 <= K1 + K2 <= 16; dZ [M, N] read once; deterministic
 * two-pass reduction (lpg_wgrad_smallk_workspace_bytes(M, N, K1 + K2)). */
int64_t lpg_wgrad_smallk_workspace_bytes(int64_t M, int64_t N, int64_t K);
lpg_status lpg_wgrad_smallk_f32(int64_t M, int64_t N, const float *dz, int64_t ldz,
                                int64_t K1, const float *A1, int64_t lda1, int64_t K2, const float *A2, int64_t lda2,
                                float *dW1, float *dW2, void *workspace, void *stream);
/* Same with the ReLU/dropout backward fused: dZ = (y > 0) ? g * scale : 0 is
 * formed on the fly from the output gradient g and the stored output y (never
 * written), and db[n] = sum_m dZ[m, n] when db != NULL.  For layers whose
 * inputs need no gradient (conv1).  Same workspace size. */
lpg_status lpg_relu_wgrad_smallk_f32(int64_t M, int64_t N, const float *g, int64_t ldg, const float *y, int64_t ldy,
                                     float scale, int64_t K1, const float *A1, int64_t lda1, int64_t K2,
                                     const float *A2, int64_t lda2, float *dW1, float *dW2, float *db,
                                     void *workspace, void *stream);

/* bf16 variant (c5 configuration, BASELINE.json configs[4]): A1/A2/W1/W2
 * bf16 bit patterns (uint16), K1 and K2 multiples of 64 (zero-pad), leading
 * dims multiples of 8 and 16-byte aligned; fp32 accumulation on
 * v_mfma_f32_16x16x32_bf16, fp32 bias, same epilogue (ReLU, fused dropout
 * with the same mask function), C stored as bf16 (round to nearest even).
 * flags as lpg_fc_f32 (bit 1: C holds a bf16 addend, added in fp32 before
 * the bias).  Narrow inputs (conv1's LP features: 4 <= K1, K1 + K2 <= 16,
 * multiples of 4, N and ldc multiples of 4, C 8-byte aligned; no padding)
 * run a streaming kernel: one fp32 fma chain per output over the exact
 * bf16 products, the same epilogue -- equal to the MFMA kernel on the padded
 * operands up to fp32 summation order. */
lpg_status lpg_fc_bf16(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1, const uint16_t *W1,
                       int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2, const uint16_t *W2, int64_t ldw2,
                       const float *bias, uint16_t *C, int64_t ldc, int32_t flags, float dropout_p, uint64_t seed,
                       int64_t row_offset, const int64_t *row_keys, void *stream);
/* The same FC with fp16 storage (--fp16 inference, val.py:269): A/W/C fp16 bit patterns on
 * v_mfma_f32_16x16x32_f16 (the bf16 kernels' tiles and epilogues), fp32 accumulation and bias,
 * one RNE rounding to fp16 per output.  Arguments as lpg_fc_bf16. */
lpg_status lpg_fc_f16(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1, const uint16_t *W1,
                      int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2, const uint16_t *W2, int64_t ldw2,
                      const float *bias, uint16_t *C, int64_t ldc, int32_t flags, float dropout_p, uint64_t seed,
                      int64_t row_offset, const int64_t *row_keys, void *stream);
/* dst[c, r] = src[r, c] for bf16 [R, C] (R, C, lds, ldd multiples of 8, 16-byte
 * aligned): the transposed weights the c5 input gradients multiply by
 * (dX = dZ W of a Linear, arch.py:57-62 through train.py:128). */
lpg_status lpg_transpose_bf16(int64_t R, int64_t C, const uint16_t *src, int64_t lds, uint16_t *dst, int64_t ldd,
                              void *stream);

/* The input gradient of a GraphConv layer whose input is the previous layer's
 * ReLU + dropout output Y, with that layer's ReLU/dropout backward folded into
 * the store (c5 backward, train.py:128 through arch.py:185-188's
 * conv -> dropout -> ReLU):
 *   C = (Y > 0) ? bf16(bf16(A1 W1^T + A2 W2^T [+ C]) * scale) : 0
 * bit for bit lpg_fc_bf16 (no bias, no ReLU) followed by
 * lpg_relu_bwd_colsum_bf16(C, Y, scale) -- without that pass's read of C and
 * write of dZ.  flags: bit 1 (C holds a bf16 addend) and the kernel choice.  N, ldc, ldy
 * multiples of 8, C and Y 16-byte aligned; other requirements as lpg_fc_bf16. */
lpg_status lpg_fc_bf16_relu_bwd(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2,
                                const uint16_t *W2, int64_t ldw2, uint16_t *C, int64_t ldc, int32_t flags,
                                const uint16_t *Y, int64_t ldy, float scale, void *stream);

/* lpg_fc_bf16 (ReLU flag required) that also writes the output's 1-bit ReLU mask: mask[m * ldm + t]
 * bit e = (C[m, 8 t + e] > 0), ldm >= N / 8; N, ldc multiples of 8, C 16-byte aligned.  The bf16
 * layer's backward then folds its ReLU/dropout backward from the bits (lpg_fc_bf16_relu_bwd_bits)
 * instead of re-reading the layer output (c5: 51 MB instead of 819 MB per 200 K x 2048 launch). */
lpg_status lpg_fc_bf16_mask(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1, const uint16_t *W1,
                            int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2, const uint16_t *W2,
                            int64_t ldw2, const float *bias, uint16_t *C, int64_t ldc, int32_t flags, float dropout_p,
                            uint64_t seed, int64_t row_offset, const int64_t *row_keys, uint8_t *mask, int64_t ldm,
                            void *stream);

/* lpg_fc_bf16_relu_bwd with the previous layer's ReLU as lpg_fc_bf16_mask's bits instead of its
 * output Y: the same bits. */
lpg_status lpg_fc_bf16_relu_bwd_bits(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                     const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2,
                                     const uint16_t *W2, int64_t ldw2, uint16_t *C, int64_t ldc, int32_t flags,
                                     const uint8_t *mask, int64_t ldm, float scale, void *stream);

/* lpg_fc_bf16_relu_bwd / lpg_fc_bf16_relu_bwd_bits that also return the bias gradient of the layer
 * whose ReLU they fold, db[n] = sum_m C[m, n] (fp32): bitwise lpg_colsum_bf16 on the stored C (its
 * 64-row chunks, in-chunk order and fold), the chunk sums taken in the pipelined kernel's store loop
 * -- no second pass over C where that kernel runs (c5: the 819 MB re-read of a 200 K x 2048 dZ).
 * workspace: lpg_relu_bwd_colsum_workspace_bytes(M, N), 16-byte aligned; M = 0 zeroes db. */
lpg_status lpg_fc_bf16_relu_bwd_db(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                   const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2, int64_t lda2,
                                   const uint16_t *W2, int64_t ldw2, uint16_t *C, int64_t ldc, int32_t flags,
                                   const uint16_t *Y, int64_t ldy, float scale, float *db, void *workspace,
                                   void *stream);
lpg_status lpg_fc_bf16_relu_bwd_bits_db(int64_t M, int64_t N, int64_t K1, const uint16_t *A1, int64_t lda1,
                                        const uint16_t *W1, int64_t ldw1, int64_t K2, const uint16_t *A2,
                                        int64_t lda2, const uint16_t *W2, int64_t ldw2, uint16_t *C, int64_t ldc,
                                        int32_t flags, const uint8_t *mask, int64_t ldm, float scale, float *db,
                                        void *workspace, void *stream);

/* Every 16-bit FC form above in one call, with the workspace of the persistent stream-K kernel
 * (fc_bf16_sk): G = (CUs rounded down to a multiple of 8) resident blocks split the call's
 * (tile, k-tile) iterations into G nearly equal ranges, a tile cut by a range boundary carrying its
 * fp32 accumulators from one block to the next through `workspace` -- no partial last round of
 * 256 x 256 tiles and no chip-wide burst of epilogue stores, the same bits as the per-call entries
 * (the same MFMA chain per output).  It applies when the call has at least G tiles and the
 * pipelined kernel takes its operands; otherwise the call runs exactly as the per-call entry would.
 * Which entry the call stands for:
 *   dtype 0 (bf16) / 1 (fp16);  Y or mask_in set: lpg_fc_bf16_relu_bwd[_bits] (flags: accumulate +
 *   kernel only; bias / dropout unused; scale), with db: ..._db (db_workspace as there);  else
 *   lpg_fc_bf16 / lpg_fc_f16, with mask_out: lpg_fc_bf16_mask.
 * workspace: lpg_fc16_workspace_bytes() bytes, 16-byte aligned (NULL = the per-call entry's path);
 * LPG_FC_KERNEL(6) selects the stream-K form; every other choice runs as the per-call entry.  The
 * form is a measured alternative, not the default: 15-25 % slower than choice 0 at the c5 and
 * fp16-inference shapes (profiles/r05_sk_ab.log). */
typedef struct lpg_fc16_call {
  int32_t dtype, flags;
  int64_t M, N, K1, K2;
  const uint16_t *A1, *W1, *A2, *W2;
  int64_t lda1, ldw1, lda2, ldw2;
  const float *bias;
  uint16_t *C;
  int64_t ldc;
  float dropout_p;
  uint64_t seed;
  int64_t row_offset;
  const int64_t *row_keys;
  uint8_t *mask_out;
  int64_t ldmo;
  const uint16_t *Y;
  int64_t ldy;
  const uint8_t *mask_in;
  int64_t ldmi;
  float scale;
  float *db;
  void *db_workspace;
} lpg_fc16_call;
int64_t lpg_fc16_workspace_bytes(void);
lpg_status lpg_fc16(const lpg_fc16_call *call, void *workspace, int64_t workspace_bytes, void *stream);

/* bf16 weight gradient (c5 backward, reference train.py:128 loss.backward()
 * through GraphConv's lin_rel / lin_root): dW[n, k] = sum_r G[r, n] X[r, k],
 * G = dZ [R, N] and X = the layer input [R, K] as bf16 bit patterns
 * (row-major, leading dimensions ldg / ldx; N, K, ldg, ldx multiples of 8,
 * 16-byte aligned), fp32 accumulation on v_mfma_f32_16x16x32_bf16, dW fp32
 * [N, K] (lddw a multiple of 4, 16-byte aligned) -- the fp32 master-weight
 * gradient, never rounded to bf16.  Replaces torch's (G^T @ X).float() on
 * hipBLASLt (a bf16-rounded product).  R is split into contiguous ranges
 * whose partial products go to `workspace` (lpg_wgrad_bf16_workspace_bytes
 * bytes, 16-byte aligned; 0 bytes = not needed) and are added in range
 * order: deterministic. */
int64_t lpg_wgrad_bf16_workspace_bytes(int64_t R, int64_t N, int64_t K);
lpg_status lpg_wgrad_bf16(int64_t R, int64_t N, int64_t K, const uint16_t *G, int64_t ldg, const uint16_t *X,
                          int64_t ldx, float *dW, int64_t lddw, void *workspace, void *stream);

/* Backward of a Linear with 1 <= N <= 4 outputs (the heads lin_left /
 * lin_right, arch.py:175-176, 190; torch Linear backward):
 *   dH = G W (skipped if dH == NULL), dW = G^T H, db = sum_m G[m, :].
 * G [M, N] (ldg), W [N, K] contiguous, H [M, K] (ldh).  Deterministic
 * two-pass reduction through `workspace` (16-byte aligned,
 * lpg_linear_small_bwd_workspace_bytes(M, K, N) bytes). */
int64_t lpg_linear_small_bwd_workspace_bytes(int64_t M, int64_t K, int64_t N);
lpg_status lpg_linear_small_bwd_f32(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg,
                                    const float *W, const float *H, int64_t ldh, float *dH, int64_t lddh,
                                    float *dW, float *db, void *workspace, void *stream);

/* The heads' backward fused with the ReLU/dropout backward of the layer that
 * produced their input (GCN_FC: the last hidden layer's output Y feeds
 * lin_left / lin_right, arch.py:186-190): one pass over Y,
 *   dZ[m, k] = Y[m, k] > 0 ? scale * sum_c G[m, c] W[c, k] : 0   (the layer's dZ),
 *   dW = G^T Y, db = sum_m G[m, :], dbY[k] = sum_m dZ[m, k]       (the layer's bias gradient),
 * 1 <= N <= 4; db / dbY may be NULL; workspace lpg_linear_small_bwd_workspace_bytes(M, K, N). */
lpg_status lpg_heads_relu_bwd_f32(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg, const float *W,
                                  const float *Y, int64_t ldy, float scale, float *dZ, int64_t lddz, float *dW,
                                  float *db, float *dbY, void *workspace, void *stream);
/* The same, also returning dZ's f16x2 scales from its own stores (rscale [M], cscale [K]: the values
 * lpg_rowcolscale_f32 gives on dZ, without reading it again when K is a multiple of 1024; other K: the
 * pass, then that sweep); K a multiple of 4, scale_ws
 * lpg_heads_scales_workspace_bytes(M, K) bytes, 16-byte aligned. */
int64_t lpg_heads_scales_workspace_bytes(int64_t M, int64_t K);
lpg_status lpg_heads_relu_bwd_scales_f32(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg,
                                         const float *W, const float *Y, int64_t ldy, float scale, float *dZ,
                                         int64_t lddz, float *dW, float *db, float *dbY, float *rscale,
                                         float *cscale, void *scale_ws, void *workspace, void *stream);

/* bf16 twin of lpg_relu_wgrad_smallk_f32 (c5 conv1, arch.py:170 through
 * train.py:128): g, y, A1, A2 bf16 bit patterns; dW1, dW2, db fp32.  y == NULL:
 * g already is dZ (the next layer's input gradient folded this layer's ReLU /
 * dropout backward into its store, lpg_fc_bf16_relu_bwd); else dZ = (y > 0) ?
 * RNE_bf16(g * scale) : 0 on the fly (the bits of lpg_relu_bwd_colsum_bf16).
 * One read of the gradient gives dW1, dW2 and db (db may be NULL).  N, ldg,
 * ldy multiples of 4, g / y 8-byte aligned; workspace
 * lpg_wgrad_smallk_workspace_bytes(M, N, K1 + K2), 16-byte aligned. */
lpg_status lpg_relu_wgrad_smallk_bf16(int64_t M, int64_t N, const uint16_t *g, int64_t ldg, const uint16_t *y,
                                      int64_t ldy, float scale, int64_t K1, const uint16_t *A1, int64_t lda1,
                                      int64_t K2, const uint16_t *A2, int64_t lda2, float *dW1, float *dW2, float *db,
                                      void *workspace, void *stream);

/* The heads' forward in bf16 (lin_left / lin_right of the c5 model,
 * arch.py:175-176, 190): out[m, c] = RNE_bf16(sum_k H[m, k] W[c, k] + bias[c])
 * for 1 <= N <= 4, 8 <= K <= 2048 (K, ldh multiples of 8; H bf16 and W fp32
 * holding the bf16 weights, both 16-byte aligned; bias fp32 or NULL; out bf16
 * [M, N], leading dimension ldo).  One streaming pass over H; the MFMA FC on N
 * zero-padded to 64 sums the same exact products in another order. */
lpg_status lpg_linear_small_fwd_bf16(int64_t M, int64_t K, int64_t N, const uint16_t *H, int64_t ldh, const float *W,
                                     const float *bias, uint16_t *out, int64_t ldo, void *stream);
/* ... with fp16 H / out (the --fp16 model's heads): out = RNE_fp16(fp32 sum + bias). */
lpg_status lpg_linear_small_fwd_f16(int64_t M, int64_t K, int64_t N, const uint16_t *H, int64_t ldh, const float *W,
                                    const float *bias, uint16_t *out, int64_t ldo, void *stream);

/* The heads' backward in bf16, one pass over the layer output H [M, K] (bf16):
 *   dH[m, k] = RNE_bf16(sum_c G[m, c] W[c, k]); with mask != 0 through the
 *              producing layer's ReLU/dropout backward, (H > 0) ? RNE_bf16(dH * scale) : 0
 *              (the layer's dZ, bitwise lpg_fc_bf16 + lpg_relu_bwd_colsum_bf16's rule);
 *   dW = G^T H (fp32 [N, K]), db = sum_m G[m, :]  (db may be NULL),
 *   dbY[k] = sum_m dH[m, k] when dbY != NULL: bitwise lpg_colsum_bf16 on the stored dH.
 * G [M, N] fp32 (ldg >= N), W [N, K] fp32 contiguous (the bf16 weights), 1 <= N <= 4;
 * K, ldh, lddh multiples of 8, W / H / dH 16-byte aligned; workspace
 * lpg_heads_bwd_bf16_workspace_bytes(M, K, N), 16-byte aligned. */
int64_t lpg_heads_bwd_bf16_workspace_bytes(int64_t M, int64_t K, int64_t N);
lpg_status lpg_heads_bwd_bf16(int64_t M, int64_t K, int64_t N, const float *G, int64_t ldg, const float *W,
                              const uint16_t *H, int64_t ldh, int32_t mask, float scale, uint16_t *dH, int64_t lddh,
                              float *dW, float *db, float *dbY, void *workspace, void *stream);

/* ---- balanced loss (train.py:39-46) ---------------------------------------- */

/* nn.CrossEntropyLoss(weight=w)(x, y) * coef (mean reduction, ignore_index
 * -100) for C <= 4 classes: loss[0] = coef * sum_i w[y_i] l_i / sum_i w[y_i],
 * wsum[0] = sum_i w[y_i] (device scalars; kept for the backward).  w may be
 * NULL (unit weights).  Deterministic fixed-order reduction through
 * `workspace` (lpg_weighted_ce_workspace_bytes(M)).  An out-of-range label
 * makes the loss NaN. */
/* Class counts of the balanced loss's weights (utils.py:286-299
 * labels_to_balanced_weights, which counts by torch.unique): counts[c] =
 * #{i : y[i] == c} for c = 0, 1, 2 (int64; other values are not counted),
 * exact, no atomics, no host sync.  Workspace:
 * lpg_class_counts_workspace_bytes(M). */
int64_t lpg_class_counts_workspace_bytes(int64_t M);
lpg_status lpg_class_counts3(int64_t M, const int64_t *y, int64_t *counts, void *workspace, void *stream);
/* The balanced loss's class weights themselves (utils.py:286-299 labels_to_balanced_weights, on the
 * device, no host sync): weights[c] = N / count_c (float32 operands, correctly rounded) for the
 * present classes of y (labels 0, 1, 2), 0 otherwise; with merge_lu and other than exactly two
 * classes present, weights[0] = weights[2] = (weights[0] + weights[2]) / 2.  The counting pass of
 * lpg_class_counts3 plus the formula in its fold (one launch fewer than ~13 elementwise ops).
 * Workspace: lpg_class_counts_workspace_bytes(M). */
lpg_status lpg_balanced_weights3(int64_t M, const int64_t *y, int32_t merge_lu, float *weights, void *workspace,
                                 void *stream);

int64_t lpg_weighted_ce_workspace_bytes(int64_t M);
lpg_status lpg_weighted_ce_fwd_f32(int64_t M, int64_t C, const float *x, int64_t ldx, const int64_t *y,
                                   const float *w, float coef, float *loss, float *wsum, void *workspace,
                                   void *stream);
/* dx[i, c] = gout[0] * coef * w[y_i] / wsum[0] * (softmax(x_i)_c - [c == y_i]) (gout may be NULL: 1). */
lpg_status lpg_weighted_ce_bwd_f32(int64_t M, int64_t C, const float *x, int64_t ldx, const int64_t *y,
                                   const float *w, const float *wsum, const float *gout, float coef,
                                   float *dx, int64_t lddx, void *stream);

/* ---- basis labels (inference_gnn, val.py:106-124) -------------------------- */

/* labels[i] for i < total from logits [total, 3] (stride ldl): P = softmax(logits) with NaN -> 0;
 * the m nodes with the largest P[:, 1] get 1 (of the nodes equal to the m-th largest value, the
 * lowest indices; torch.topk leaves that choice open), every other node argmax(P[i,0], P[i,2])
 * (0 on a tie).  Replaces the softmax / topk / argmax chain of val.py:106-118 (the reference's
 * timed post-processing, scripts/pred_basis.py:117).  0 <= m <= total.  Exact radix select on the
 * float bits, no host sync, deterministic.  Workspace: lpg_basis_labels_workspace_bytes(total),
 * 16-byte aligned. */
int64_t lpg_basis_labels_workspace_bytes(int64_t total);
lpg_status lpg_basis_labels_f32(int64_t total, int64_t m, const float *logits, int64_t ldl, int64_t *labels,
                                void *workspace, void *stream);
/* ... on fp16 logits (--fp16 inference): P computed in fp32 and rounded to fp16 (torch's half softmax
 * stores it so); the selection and argmax see the fp16 values.  Same workspace. */
lpg_status lpg_basis_labels_f16(int64_t total, int64_t m, const uint16_t *logits, int64_t ldl, int64_t *labels,
                                void *workspace, void *stream);

/* add_knowledge for one side (arch.py:129-141): out = normalize(logit) * 10,
 * then out[:,0] -= bound where feas[:, cols-3] != 0 (infinite lower bound)
 * and out[:,2] -= bound where feas[:, cols-1] != 0 (infinite upper bound).
 * logit/out [M, 3] (strides ldl/ldo), feas [M, feas_cols] (stride ldf).
 * Bitwise torch-CPU F.normalize semantics (norm = sqrt(fma(x2,x2,fma(x1,x1,x0*x0)))). */
lpg_status lpg_knowledge_f32(int64_t M, const float *logit, int64_t ldl, const float *feas, int64_t ldf,
                             int64_t feas_cols, float bound, float *out, int64_t ldo, void *stream);
/* ... on fp16 logits / out (--fp16 inference: arch.py:129-141 in half precision), each stored
 * intermediate rounded to fp16 as torch's half ops do: n = RNE16(sqrt(...)), d = max(n, 0),
 * y = RNE16(RNE16(x / d) * 10), masked y = RNE16(y - bound).  feas fp32. */
lpg_status lpg_knowledge_f16(int64_t M, const uint16_t *logit, int64_t ldl, const float *feas, int64_t ldf,
                             int64_t feas_cols, float bound, uint16_t *out, int64_t ldo, void *stream);
/* Its backward (autograd of F.normalize(x) * 10, arch.py:134-135; the bound subtractions pass g
 * through): dx = 10 (g / d - x (x . g) / d^3) where |x| > 1e-12, else 10 g / d (d = max(|x|, 1e-12)),
 * logit / g / dx [M, 3] with row strides ldl / ldg / lddx.  One pass instead of torch's ~12 kernels. */
lpg_status lpg_knowledge_bwd_f32(int64_t M, const float *logit, int64_t ldl, const float *g, int64_t ldg, float *dx,
                                 int64_t lddx, void *stream);

/* ---- k-hop neighbour sampling (NeighborLoader collate, train.py:111-116,
 * val.py:22-27; replaces torch_sparse 0.6.12 neighbor_sample) -------------
 * Graph = CSC of the homogeneous LP graph: colptr [N+1], row [E] (sources of
 * node v's in-edges, sorted).  All ids int64.  `local` [N] must hold -1 and
 * `first` [N] all ones (UINT64_MAX) between batches; the calls below restore
 * them (lpg_sample_reset for `local`).  A hop is
 *   count -> lpg_scan_i64 -> fill -> dedupe -> lpg_scan_i64(flag) -> assign;
 * node ids are assigned in first-appearance order (frontier order, then
 * neighbour order) exactly as neighbor_sample's sequential insertion.
 * fanout < 0 = all neighbours; fanout <= 256. */
int64_t lpg_scan_i64_workspace_bytes(int64_t n);
/* out [n + 1]: out[0] = 0, out[i + 1] = in[0] + ... + in[i] */
lpg_status lpg_scan_i64(const int64_t *in, int64_t n, int64_t *out, void *workspace, int64_t workspace_bytes,
                        void *stream);
lpg_status lpg_sample_count(const int64_t *frontier, int64_t nf, const int64_t *colptr, int64_t fanout,
                            int64_t *counts, void *stream);
/* candidates of frontier node i go to [offsets[i], offsets[i+1]); cand_dst =
 * base + i (the frontier node's local id), cand_edge = CSC position */
lpg_status lpg_sample_fill(const int64_t *frontier, int64_t nf, int64_t base, const int64_t *colptr,
                           const int64_t *row, int64_t fanout, uint64_t seed, const int64_t *offsets,
                           int64_t *cand, int64_t *cand_edge, int64_t *cand_dst, void *stream);
/* flag[p] = 1 iff cand[p] is unsampled and p is its first appearance */
lpg_status lpg_sample_dedupe(const int64_t *cand, int64_t nc, const int64_t *local, uint64_t *first,
                             int64_t *flag, void *stream);
/* where flag[p]: nodes[rank[p]] = cand[p] (this hop's chunk) and
 * local[cand[p]] = base + rank[p] (its local id) */
lpg_status lpg_sample_assign(const int64_t *cand, int64_t nc, int64_t base, const int64_t *flag,
                             const int64_t *rank, int64_t *nodes, int64_t *local, uint64_t *first, void *stream);
/* out[p] = local[cand[p]] (directed=True edge rows) */
lpg_status lpg_sample_local_ids(const int64_t *cand, int64_t nc, const int64_t *local, int64_t *out, void *stream);
/* directed=False: edges of the subgraph induced on nodes[0..ns) --
 * per destination i, in CSC order: (row = local[src], col = i, edge = CSC pos) */
lpg_status lpg_induced_count(const int64_t *nodes, int64_t ns, const int64_t *colptr, const int64_t *row,
                             const int64_t *local, int64_t *counts, void *stream);
lpg_status lpg_induced_fill(const int64_t *nodes, int64_t ns, const int64_t *colptr, const int64_t *row,
                            const int64_t *local, const int64_t *offsets, int64_t *out_row, int64_t *out_col,
                            int64_t *out_edge, void *stream);
lpg_status lpg_sample_reset(const int64_t *nodes, int64_t ns, int64_t *local, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LPGNN_H */
