// Host-side sanitizer harness (ASan + UBSan): the C-ABI library's host code (csrc/pack.cpp,
// csrc/abi.cpp) and the oracle's C restatement (oracle/spmm_ref.c, oracle/fc_ref.c) on random
// and edge-case inputs, built by `make -C tools/sanitize` with -fsanitize=address,undefined and
// run by tests/test_sanitize.py.  The GPU kernels are not covered here (no GPU sanitizer on the
// pool); what is checked is every host loop that indexes caller buffers.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "lpgnn.h"

extern "C" {
void oracle_spmm_f32(int64_t M, const int64_t *rowptr, const int32_t *col, const float *val, const float *X,
                     int64_t ldx, int64_t F, float *Y, int64_t ldy, int nthreads);
void oracle_spmm_bf16(int64_t M, const int64_t *rowptr, const int32_t *col, const float *val, const uint16_t *X,
                      int64_t ldx, int64_t F, uint16_t *Y, int64_t ldy, int nthreads);
void oracle_fc_f32(int64_t M, int64_t N, int64_t K1, const float *A1, int64_t lda1, const float *W1, int64_t ldw1,
                   int64_t K2, const float *A2, int64_t lda2, const float *W2, int64_t ldw2, const float *bias,
                   float *C, int64_t ldc, const float *P, int64_t ldp, int relu, int nthreads);
}

static int fails = 0;
#define CHECK(c, ...)                   \
  do {                                  \
    if (!(c)) {                         \
      std::fprintf(stderr, __VA_ARGS__); \
      std::fprintf(stderr, "\n");       \
      ++fails;                          \
    }                                   \
  } while (0)

// exact-size heap buffers so ASan sees any overrun of the caller's allocation
template <class T>
static T *buf(size_t n) {
  return static_cast<T *>(std::malloc(sizeof(T) * (n ? n : 1)));
}

static void pack_case(int64_t m, int64_t n, int64_t nnz, std::mt19937_64 &rng) {
  // distinct (row, col) pairs
  std::vector<int64_t> keys;
  std::uniform_int_distribution<int64_t> dk(0, m * n - 1);
  while ((int64_t)keys.size() < nnz) keys.push_back(dk(rng));
  std::sort(keys.begin(), keys.end());
  keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
  std::shuffle(keys.begin(), keys.end(), rng);
  const int64_t e = (int64_t)keys.size();
  int64_t *row = buf<int64_t>(e), *col = buf<int64_t>(e);
  float *val = buf<float>(e);
  for (int64_t i = 0; i < e; ++i) {
    row[i] = keys[i] / n;
    col[i] = keys[i] % n;
    val[i] = (float)(i % 7) - 3.f;
  }
  int64_t *arp = buf<int64_t>(m + 1), *atrp = buf<int64_t>(n + 1);
  int32_t *ac = buf<int32_t>(e), *atc = buf<int32_t>(e);
  float *av = buf<float>(e), *atv = buf<float>(e);
  const lpg_status st = lpg_csr_pack_host(row, col, val, e, m, n, arp, ac, av, atrp, atc, atv);
  CHECK(st == LPG_OK, "pack %lld x %lld nnz %lld: status %d (%s)", (long long)m, (long long)n, (long long)e, st,
        lpg_last_error());
  if (st == LPG_OK) {
    CHECK(arp[m] == e && atrp[n] == e, "pack: rowptr totals");
    for (int64_t r = 0; r < m; ++r)
      for (int64_t p = arp[r] + 1; p < arp[r + 1]; ++p) CHECK(ac[p - 1] < ac[p], "pack: row %lld unsorted", (long long)r);
    for (int64_t c = 0; c < n; ++c)
      for (int64_t p = atrp[c] + 1; p < atrp[c + 1]; ++p)
        CHECK(atc[p - 1] < atc[p], "pack: column %lld unsorted", (long long)c);
    // the oracle SpMM on both orientations (F = 3, strided)
    const int64_t F = 3, ld = 5;
    float *X = buf<float>(n * ld), *Y = buf<float>(m * ld), *XT = buf<float>(m * ld), *YT = buf<float>(n * ld);
    for (int64_t i = 0; i < n * ld; ++i) X[i] = (float)((i * 37) % 11) - 5.f;
    for (int64_t i = 0; i < m * ld; ++i) XT[i] = (float)((i * 13) % 9) - 4.f;
    oracle_spmm_f32(m, arp, ac, av, X, ld, F, Y, ld, 2);
    oracle_spmm_f32(n, atrp, atc, atv, XT, ld, F, YT, ld, 2);
    uint16_t *Xb = buf<uint16_t>(n * ld), *Yb = buf<uint16_t>(m * ld);
    for (int64_t i = 0; i < n * ld; ++i) Xb[i] = (uint16_t)(0x3f80 + (i % 5));
    oracle_spmm_bf16(m, arp, ac, av, Xb, ld, F, Yb, ld, 2);
    std::free(X), std::free(Y), std::free(XT), std::free(YT), std::free(Xb), std::free(Yb);
  }
  // a duplicate edge and an out-of-range column are rejected, never read past the buffers
  if (e >= 2) {
    const int64_t keep = col[1];
    row[1] = row[0], col[1] = col[0];
    CHECK(lpg_csr_pack_host(row, col, val, e, m, n, arp, ac, av, atrp, atc, atv) == LPG_ERR_INVALID,
          "pack: duplicate accepted");
    col[1] = n;
    CHECK(lpg_csr_pack_host(row, col, val, e, m, n, arp, ac, av, atrp, atc, atv) == LPG_ERR_INVALID,
          "pack: column n accepted");
    col[1] = keep;
  }
  std::free(row), std::free(col), std::free(val), std::free(arp), std::free(atrp);
  std::free(ac), std::free(atc), std::free(av), std::free(atv);
}

static void fc_case(int64_t M, int64_t N, int64_t K1, int64_t K2, bool add) {
  const int64_t lda = K1 + 3, ldb = K2 + 1, ldc = N + 2;
  float *A1 = buf<float>(M * lda), *W1 = buf<float>(N * K1), *A2 = buf<float>(M * ldb), *W2 = buf<float>(N * K2);
  float *b = buf<float>(N), *C = buf<float>(M * ldc), *P = buf<float>(M * ldc);
  for (int64_t i = 0; i < M * lda; ++i) A1[i] = std::sin((float)i);
  for (int64_t i = 0; i < N * K1; ++i) W1[i] = std::cos((float)i);
  for (int64_t i = 0; i < M * ldb; ++i) A2[i] = 0.5f * std::sin(0.3f * (float)i);
  for (int64_t i = 0; i < N * K2; ++i) W2[i] = 0.25f * std::cos(0.7f * (float)i);
  for (int64_t i = 0; i < N; ++i) b[i] = 0.1f * (float)i;
  for (int64_t i = 0; i < M * ldc; ++i) P[i] = 1.f;
  oracle_fc_f32(M, N, K1, A1, lda, W1, K1, K2, A2, ldb, W2, K2, b, C, ldc, add ? P : nullptr, ldc, 1, 2);
  for (int64_t m = 0; m < M; ++m)
    for (int64_t n = 0; n < N; ++n) CHECK(std::isfinite(C[m * ldc + n]) && C[m * ldc + n] >= 0.f, "fc: bad output");
  std::free(A1), std::free(W1), std::free(A2), std::free(W2), std::free(b), std::free(C), std::free(P);
}

int main() {
  std::mt19937_64 rng(7);
  const int64_t shapes[][3] = {{1, 1, 1}, {0, 5, 0}, {5, 0, 0}, {7, 9, 0}, {3, 4, 12}, {40, 70, 500},
                               {1, 300, 300}, {300, 1, 200}, {257, 129, 4000}};
  for (auto &s : shapes) pack_case(s[0], s[1], s[2], rng);
  // invalid arguments return an error without touching memory
  CHECK(lpg_csr_pack_host(nullptr, nullptr, nullptr, -1, 1, 1, nullptr, nullptr, nullptr, nullptr, nullptr,
                          nullptr) == LPG_ERR_INVALID,
        "pack: negative nnz accepted");
  CHECK(std::strlen(lpg_last_error()) > 0 && std::strlen(lpg_build_info()) > 0, "error / build strings");
  const int64_t fcs[][4] = {{1, 1, 1, 0}, {5, 3, 130, 0}, {33, 17, 8, 8}, {70, 129, 256, 40}, {2, 4, 0, 9}};
  for (auto &s : fcs) {
    fc_case(s[0], s[1], s[2], s[3], false);
    fc_case(s[0], s[1], s[2], s[3], true);
  }
  std::printf("host sanitizer checks: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
