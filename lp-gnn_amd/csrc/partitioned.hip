// The row-partitioned SpMM with its boundary exchange inside the library (SURVEY.md §8b "Multi-GPU",
// §8e): lpg_spmm_partitioned_f32 and the RCCL communicator entries of include/lpgnn.h.
//
// One rank per GPU holds a block of constraint rows and the variables they touch.  The vars<-cons
// direction over the local edges gives full sums for the variables only this rank touches and
// partial sums for the boundary variables (touched by >= 2 ranks).  The boundary rows are packed into
// a dense [n_boundary, F] buffer in GLOBAL boundary order (zero rows for the boundary variables this
// rank does not touch), summed over the ranks by one RCCL all-reduce over xGMI, and unpacked back
// into the local rows: every rank ends with the full sums of exactly the boundary rows it holds --
// the same values on every rank (an all-reduce hands every rank the same reduced buffer).  The
// reverse direction (cons<-vars) needs no exchange, so it is plain lpg_spmm_f32; the backward of
// this entry is this entry on the other orientation (torch_sparse SPMMSum::backward).
//
// lpgnn.partition's Python exchange is the sparse owner form of the same sum (all_to_all of only the
// rows that cross); this is the dense survey form with the collective in native code, callable
// from any host language that can hold an ncclComm_t.
//
// RCCL is resolved at run time (dlopen, reusing the copy the process already loaded -- torch's, when
// the caller is a torch process), so the library has no link-time dependency on it and loads on a
// host without RCCL; only the communicator entries need it.
#include <dlfcn.h>

#include <cstring>
#include <mutex>

#include "common.h"

namespace lpg {
namespace {

// ---- RCCL, resolved once -----------------------------------------------------------------------
// The subset of rccl.h this file calls (same ABI: ncclResult_t / ncclDataType_t / ncclRedOp_t are
// C enums passed as int; ncclUniqueId is 128 bytes passed by value).
struct UniqueId {
  char internal[LPG_COMM_ID_BYTES];
};
struct Rccl {
  void *h = nullptr;
  int (*get_unique_id)(UniqueId *) = nullptr;
  int (*comm_init_rank)(ncclComm_t *, int, UniqueId, int) = nullptr;
  int (*comm_destroy)(ncclComm_t) = nullptr;
  int (*comm_count)(ncclComm_t, int *) = nullptr;
  int (*comm_user_rank)(ncclComm_t, int *) = nullptr;
  int (*all_reduce)(const void *, void *, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  const char *(*error_string)(int) = nullptr;
  bool ok = false;
  char why[256] = "";
};
constexpr int kNcclFloat32 = 7, kNcclSum = 0;

const Rccl &rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // the copy already in the process first (torch's libtorch_hip pulls in librccl.so.1), else the
    // system's
    const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char *n : names)
      if ((r.h = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL)) != nullptr) break;
    for (const char *n : names)
      if (!r.h && (r.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
    if (!r.h) {
      snprintf(r.why, sizeof(r.why), "RCCL not loadable: %s", dlerror());
      return;
    }
    auto sym = [&](const char *s) {
      void *p = dlsym(r.h, s);
      if (!p && !r.why[0]) snprintf(r.why, sizeof(r.why), "RCCL lacks %s", s);
      return p;
    };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
    r.comm_count = reinterpret_cast<decltype(r.comm_count)>(sym("ncclCommCount"));
    r.comm_user_rank = reinterpret_cast<decltype(r.comm_user_rank)>(sym("ncclCommUserRank"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    r.ok = !r.why[0];
  });
  return r;
}

#define LPG_RCCL_LOADED(R)                      \
  do {                                          \
    if (!(R).ok) {                              \
      ::lpg::set_error("%s", (R).why);          \
      return LPG_ERR_UNSUPPORTED;               \
    }                                           \
  } while (0)

#define LPG_NCCL(R, call)                                                                        \
  do {                                                                                           \
    const int _r = (call);                                                                       \
    if (_r != 0) {                                                                               \
      ::lpg::set_error("%s failed: %s", #call, (R).error_string ? (R).error_string(_r) : "?"); \
      return LPG_ERR_HIP;                                                                        \
    }                                                                                            \
  } while (0)

// ---- boundary pack / unpack (HBM-bound row copies) ------------------------------------------------
// Block b' handles boundary rows b = b', b' + grid, ...; its threads stride the F columns, 16 bytes a
// lane when every row start is 16-byte aligned (vec), else 4.  A map entry outside [0, rows) is a
// boundary variable this rank does not hold: pack writes a zero row, unpack skips it.
template <bool VEC>
__global__ __launch_bounds__(256) void boundary_pack(const float *__restrict__ Y, int64_t ldy, int64_t rows,
                                                     const int32_t *__restrict__ map, int64_t nb, int64_t F,
                                                     float *__restrict__ buf) {
  for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const int32_t r = map[b];
    const bool here = r >= 0 && r < rows;
    float *dst = buf + b * F;
    const float *src = Y + (here ? r : 0) * ldy;
    if constexpr (VEC) {
      for (int64_t c = threadIdx.x * 4; c < F; c += 1024) {
        const float4 v = here ? *reinterpret_cast<const float4 *>(src + c) : make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4 *>(dst + c) = v;
      }
    } else {
      for (int64_t c = threadIdx.x; c < F; c += 256) dst[c] = here ? src[c] : 0.f;
    }
  }
}

template <bool VEC>
__global__ __launch_bounds__(256) void boundary_unpack(float *__restrict__ Y, int64_t ldy, int64_t rows,
                                                       const int32_t *__restrict__ map, int64_t nb, int64_t F,
                                                       const float *__restrict__ buf) {
  for (int64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const int32_t r = map[b];
    if (r < 0 || r >= rows) continue;
    float *dst = Y + (int64_t)r * ldy;
    const float *src = buf + b * F;
    if constexpr (VEC) {
      for (int64_t c = threadIdx.x * 4; c < F; c += 1024)
        *reinterpret_cast<float4 *>(dst + c) = *reinterpret_cast<const float4 *>(src + c);
    } else {
      for (int64_t c = threadIdx.x; c < F; c += 256) dst[c] = src[c];
    }
  }
}

lpg_status launch_boundary(bool pack, float *Y, int64_t ldy, int64_t rows, const int32_t *map, int64_t nb, int64_t F,
                           float *buf, hipStream_t s) {
  if (nb == 0 || F == 0) return LPG_OK;
  const bool vec = F % 4 == 0 && ldy % 4 == 0 && aligned16(Y) && aligned16(buf);
  const int64_t grid = nb < 8 * (int64_t)device_cus() ? nb : 8 * (int64_t)device_cus();
  if (pack) {
    if (vec)
      hipLaunchKernelGGL(boundary_pack<true>, dim3((unsigned)grid), dim3(256), 0, s, Y, ldy, rows, map, nb, F, buf);
    else
      hipLaunchKernelGGL(boundary_pack<false>, dim3((unsigned)grid), dim3(256), 0, s, Y, ldy, rows, map, nb, F, buf);
  } else {
    if (vec)
      hipLaunchKernelGGL(boundary_unpack<true>, dim3((unsigned)grid), dim3(256), 0, s, Y, ldy, rows, map, nb, F, buf);
    else
      hipLaunchKernelGGL(boundary_unpack<false>, dim3((unsigned)grid), dim3(256), 0, s, Y, ldy, rows, map, nb, F,
                         buf);
  }
  LPG_HIP(hipGetLastError());
  return LPG_OK;
}

}  // namespace
}  // namespace lpg

// ---- C ABI ------------------------------------------------------------------------------------------
extern "C" lpg_status lpg_comm_unique_id(void *id) {
  lpg::clear_error();
  LPG_REQUIRE(id != nullptr, "lpg_comm_unique_id: id is NULL");
  const lpg::Rccl &r = lpg::rccl();
  LPG_RCCL_LOADED(r);
  lpg::UniqueId u;
  LPG_NCCL(r, r.get_unique_id(&u));
  memcpy(id, u.internal, LPG_COMM_ID_BYTES);
  return LPG_OK;
}

extern "C" lpg_status lpg_comm_init(ncclComm_t *comm, int32_t nranks, const void *id, int32_t rank) {
  lpg::clear_error();
  LPG_REQUIRE(comm != nullptr && id != nullptr, "lpg_comm_init: comm / id is NULL");
  LPG_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "lpg_comm_init: rank %d of %d", rank, nranks);
  const lpg::Rccl &r = lpg::rccl();
  LPG_RCCL_LOADED(r);
  lpg::UniqueId u;
  memcpy(u.internal, id, LPG_COMM_ID_BYTES);
  *comm = nullptr;
  LPG_NCCL(r, r.comm_init_rank(comm, nranks, u, rank));
  return LPG_OK;
}

extern "C" lpg_status lpg_comm_destroy(ncclComm_t comm) {
  lpg::clear_error();
  if (comm == nullptr) return LPG_OK;
  const lpg::Rccl &r = lpg::rccl();
  LPG_RCCL_LOADED(r);
  LPG_NCCL(r, r.comm_destroy(comm));
  return LPG_OK;
}

extern "C" lpg_status lpg_comm_info(ncclComm_t comm, int32_t *nranks, int32_t *rank) {
  lpg::clear_error();
  LPG_REQUIRE(comm != nullptr && nranks != nullptr && rank != nullptr, "lpg_comm_info: NULL argument");
  const lpg::Rccl &r = lpg::rccl();
  LPG_RCCL_LOADED(r);
  int n = 0, k = 0;
  LPG_NCCL(r, r.comm_count(comm, &n));
  LPG_NCCL(r, r.comm_user_rank(comm, &k));
  *nranks = n;
  *rank = k;
  return LPG_OK;
}

extern "C" lpg_status lpg_boundary_pack_f32(const float *Y, int64_t ldy, int64_t rows, int64_t F, int64_t n_boundary,
                                            const int32_t *boundary_map, float *boundary_buf, void *stream) {
  lpg::clear_error();
  LPG_REQUIRE(F >= 0 && rows >= 0 && n_boundary >= 0 && ldy >= F, "lpg_boundary_pack_f32: bad shape");
  if (n_boundary == 0 || F == 0) return LPG_OK;
  LPG_REQUIRE((Y != nullptr || rows == 0) && boundary_map != nullptr && boundary_buf != nullptr,
              "lpg_boundary_pack_f32: NULL argument");
  return lpg::launch_boundary(true, const_cast<float *>(Y), ldy, rows, boundary_map, n_boundary, F, boundary_buf,
                              lpg::as_stream(stream));
}

extern "C" lpg_status lpg_boundary_unpack_f32(float *Y, int64_t ldy, int64_t rows, int64_t F, int64_t n_boundary,
                                              const int32_t *boundary_map, const float *boundary_buf, void *stream) {
  lpg::clear_error();
  LPG_REQUIRE(F >= 0 && rows >= 0 && n_boundary >= 0 && ldy >= F, "lpg_boundary_unpack_f32: bad shape");
  if (n_boundary == 0 || F == 0) return LPG_OK;
  LPG_REQUIRE((Y != nullptr || rows == 0) && boundary_map != nullptr && boundary_buf != nullptr,
              "lpg_boundary_unpack_f32: NULL argument");
  return lpg::launch_boundary(false, Y, ldy, rows, boundary_map, n_boundary, F, const_cast<float *>(boundary_buf),
                              lpg::as_stream(stream));
}

extern "C" lpg_status lpg_boundary_allreduce_f32(float *Y, int64_t ldy, int64_t rows, int64_t F, int64_t n_boundary,
                                                 const int32_t *boundary_map, float *boundary_buf, ncclComm_t comm,
                                                 void *stream) {
  lpg::clear_error();
  LPG_REQUIRE(F >= 0 && rows >= 0 && n_boundary >= 0 && ldy >= F, "lpg_boundary_allreduce_f32: bad shape");
  if (n_boundary == 0 || F == 0) return LPG_OK;  // no collective: every rank must agree on n_boundary
  LPG_REQUIRE(Y != nullptr || rows == 0, "lpg_boundary_allreduce_f32: Y is NULL");
  LPG_REQUIRE(boundary_map != nullptr && boundary_buf != nullptr && comm != nullptr,
              "lpg_boundary_allreduce_f32: NULL map / buffer / comm");
  const lpg::Rccl &r = lpg::rccl();
  LPG_RCCL_LOADED(r);
  hipStream_t s = lpg::as_stream(stream);
  lpg_status st = lpg::launch_boundary(true, Y, ldy, rows, boundary_map, n_boundary, F, boundary_buf, s);
  if (st != LPG_OK) return st;
  LPG_NCCL(r, r.all_reduce(boundary_buf, boundary_buf, (size_t)(n_boundary * F), lpg::kNcclFloat32, lpg::kNcclSum,
                           comm, s));
  return lpg::launch_boundary(false, Y, ldy, rows, boundary_map, n_boundary, F, boundary_buf, s);
}

extern "C" lpg_status lpg_spmm_partitioned_f32(const lpg_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                                               int64_t F, int64_t n_boundary, const int32_t *boundary_map,
                                               float *boundary_buf, ncclComm_t comm, void *stream) {
  lpg::clear_error();
  LPG_REQUIRE(A != nullptr, "lpg_spmm_partitioned_f32: A is NULL");
  // the local SpMM first (its own validation), then the boundary rows' sum over the ranks
  const lpg_status st = lpg_spmm_f32(A, X, ldx, Y, ldy, F, stream);
  if (st != LPG_OK) return st;
  return lpg_boundary_allreduce_f32(Y, ldy, A->n_rows, F, n_boundary, boundary_map, boundary_buf, comm, stream);
}
