// Sustained bf16 MFMA rate of this MI355X under load: a bare v_mfma_f32_16x16x32_bf16 loop on
// random operands held in registers (no memory traffic in the loop), every SIMD busy, run for
// >= 2 s of back-to-back launches before the timed launches (MI355X_MICROARCH.md 'DVFS
// give-back' items 1, 6, 7).  Reports TFLOP/s from HIP events and the in-kernel clock
// (delta s_memtime / delta s_memrealtime x 100 MHz, median over workgroups, stamps written to a
// buffer of their own).  The x3 / bf16 GEMMs of the step are compared against this rate
// (DESIGN.md §4.2b): it is the ceiling the 2.5 PF spec figure does not describe on this part.
//
//   hipcc --offload-arch=gfx950 -O3 -o mfma_peak mfma_peak.hip && ./mfma_peak
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((__vector_size__(8 * sizeof(__bf16)))) __bf16 bf16x8;
typedef __attribute__((__vector_size__(4 * sizeof(float)))) float f32x4;

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

// NACC independent accumulators per wave; `iters` rounds of NACC MFMAs.  NREAD > 0: every round
// reads the NEXT round's NREAD B operands from LDS (ds_read_b128, the address stepping with the
// round; in flight under this round's MFMAs), the MFMAs cycling through the current ones -- the operand traffic a GEMM's inner loop carries (the x3 FC reads
// 0.29 fragments per MFMA, the bf16 FC 0.375)
template <int NACC, int NREAD = 0>
__global__ __launch_bounds__(256) void mfma_loop(const unsigned *__restrict__ seed, int iters, float *__restrict__ out,
                                                 unsigned long long *__restrict__ stamps) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  // random bf16 operands (finite, |x| in [2^-4, 2^4)) from a per-lane hash
  unsigned h = seed[0] ^ (unsigned)gid * 0x9e3779b9u;
  auto next = [&]() {
    h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
    return h;
  };
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    const unsigned ra = next(), rb = next();
    a[i] = (__bf16)__uint_as_float(((ra & 0x807fffffu) | (0x7bu + (ra >> 29)) << 23));
    b[i] = (__bf16)__uint_as_float(((rb & 0x807fffffu) | (0x7bu + (rb >> 29)) << 23));
  }
  f32x4 acc[NACC];
  // distinct starting values: identical chains (same operands, same start) would be merged by the compiler
  for (int j = 0; j < NACC; ++j) {
    f32x4 v;
    for (int e = 0; e < 4; ++e) v[e] = __uint_as_float(0x3f800000u | (next() >> 9));
    acc[j] = v;
  }
  __shared__ bf16x8 lds[4][8][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if constexpr (NREAD > 0) {
    for (int q = 0; q < 8; ++q) {
      bf16x8 v;
      for (int i = 0; i < 8; ++i) {
        const unsigned r = next();
        v[i] = (__bf16)__uint_as_float(((r & 0x807fffffu) | (0x7bu + (r >> 29)) << 23));
      }
      lds[wave][q][lane] = v;
    }
    __syncthreads();
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  bf16x8 cur[NREAD > 0 ? NREAD : 1];
  if constexpr (NREAD > 0) {
#pragma unroll
    for (int r = 0; r < NREAD; ++r) cur[r] = lds[wave][r & 7][lane];
  }
  for (int it = 0; it < iters; ++it) {
    if constexpr (NREAD > 0) {  // next round's operands in flight under this round's MFMAs
      bf16x8 nxt[NREAD];
#pragma unroll
      for (int r = 0; r < NREAD; ++r) nxt[r] = lds[wave][(it + 1 + r) & 7][lane];
#pragma unroll
      for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, cur[j % NREAD], acc[j], 0, 0, 0);
#pragma unroll
      for (int r = 0; r < NREAD; ++r) cur[r] = nxt[r];
    } else {
#pragma unroll
      for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[gid] = s;
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t1 - t0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main(int argc, char **argv) {
  const double warm_s = argc > 1 ? std::atof(argv[1]) : 3.0;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  unsigned *seed;
  float *out;
  unsigned long long *stamps;
  const int max_blocks = cus * 8;
  CHECK(hipMalloc(&seed, 4));
  CHECK(hipMalloc(&out, sizeof(float) * 256 * max_blocks));
  CHECK(hipMalloc(&stamps, sizeof(unsigned long long) * 2 * max_blocks));
  const unsigned s0 = 12345u;
  CHECK(hipMemcpy(seed, &s0, 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::printf("{\"device\": \"%s\", \"cus\": %d, \"runs\": [\n", prop.name, cus);
  // blocks of 4 waves: 1 block/CU = one wave per SIMD, 2 = two waves per SIMD
  const int iters = 20000;
  bool first = true;
  struct V { int wps, nread; };
  for (V v : {V{1, 0}, V{2, 0}, V{2, 4}, V{2, 6}}) {
    const int wps = v.wps;
    const int blocks = cus * wps;
    auto kern = v.nread == 0 ? mfma_loop<16, 0> : v.nread == 4 ? mfma_loop<16, 4> : mfma_loop<16, 6>;
    const double flop = 2.0 * 16 * 16 * 32 * 16.0 * iters * blocks * 4;  // NACC = 16 per wave
    // warm: back-to-back launches for warm_s seconds
    float ms = 0.f;
    double spent = 0.0;
    while (spent < warm_s * 1000.0) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, seed, iters, out, stamps);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      spent += ms;
    }
    std::vector<float> t;
    std::vector<double> ghz;
    for (int rep = 0; rep < 10; ++rep) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, seed, iters, out, stamps);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
      std::vector<unsigned long long> st(2 * blocks);
      CHECK(hipMemcpy(st.data(), stamps, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost));
      std::vector<double> g(blocks);
      for (int bI = 0; bI < blocks; ++bI) g[bI] = (double)st[2 * bI] / (double)st[2 * bI + 1] * 0.1;  // GHz
      std::nth_element(g.begin(), g.begin() + blocks / 2, g.end());
      ghz.push_back(g[blocks / 2]);
    }
    std::sort(t.begin(), t.end());
    std::sort(ghz.begin(), ghz.end());
    const double med = t[t.size() / 2];
    std::printf("%s {\"waves_per_simd\": %d, \"lds_reads_per_16_mfma\": %d, \"median_ms\": %.3f, \"tflops\": %.1f, \"frac_of_2500\": %.3f, "
                "\"in_kernel_ghz\": %.3f}",
                first ? " " : ",\n ", wps, v.nread, med, flop / med / 1e9, flop / med / 1e9 / 2500.0, ghz[ghz.size() / 2]);
    first = false;
  }
  std::printf("\n]}\n");
  return 0;
}
