// Ceiling probe for libgsync's Σg² at ResNet-50 size (25.56 M fp32 = 102 MB,
// inside the 256 MiB Infinity Cache, read back to back): how fast does a plain
// grid of float4 lanes read the same bytes, with no chunk map, no descriptors,
// no tensor boundaries?  Timed as the plan launch timer times the library's
// kernels: hipExtLaunchKernel's start / stop events (the kernel itself, no
// packet on the stream), 50 back-to-back launches, average and median.
// Cases: one-shot grids (one group of G 1 Ki-element chunks per workgroup, as
// the chunk engine's streaming ops), resident grid-stride grids (2,048 and
// 1,024 workgroups, as its capped reductions), cached or non-temporal loads,
// with or without the reduction epilogue (block reduce through LDS + one store
// per workgroup).  One JSON line per case.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// G float4 per lane per iteration (G Ki elements per workgroup), grid-stride
template <int G, bool NT, bool RED>
__global__ void __launch_bounds__(256) rd(const f4* __restrict__ x, int64_t n4, float* __restrict__ part) {
  __shared__ float s[4];
  float acc = 0.f;
  const int64_t step = (int64_t)gridDim.x * 256 * G;
  for (int64_t base = (int64_t)blockIdx.x * 256 * G; base < n4; base += step) {
    f4 v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t i = base + (int64_t)g * 256 + threadIdx.x;
      v[g] = i < n4 ? ld<NT>(x + i) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int g = 0; g < G; ++g) acc += v[g].x * v[g].x + v[g].y * v[g].y + v[g].z * v[g].z + v[g].w * v[g].w;
  }
  if constexpr (RED) {
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
  } else {
    if (acc == 12345.f) part[blockIdx.x] = acc;  // keeps the loads; never true here
  }
}

int main() {
  const int64_t n = 25557032 / 1024 * 1024;  // ResNet-50's parameters, whole 1 Ki chunks
  const int64_t n4 = n / 4;
  f4* x;
  float* part;
  if (hipMalloc(&x, n * 4) || hipMalloc(&part, 65536 * 4)) return 1;
  hipMemset(x, 0, n * 4);
  hipEvent_t a[50], b[50];
  for (int i = 0; i < 50; ++i) {
    hipEventCreate(&a[i]);
    hipEventCreate(&b[i]);
  }
  struct Case {
    const char* name;
    int grid;
    float avg, med;
  };
  std::vector<Case> cs;
  for (int round = 0; round < 2; ++round) {
#define CASE(NAME, G, NT, RED, GRID)                                                                          \
  do {                                                                                                        \
    const int grid = (GRID) ? (GRID) : (int)((n4 + 256 * (G) - 1) / (256 * (G)));                            \
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((rd<G, NT, RED>), dim3(grid), dim3(256), 0, 0, x, n4, part); \
    for (int i = 0; i < 50; ++i)                                                                              \
      hipExtLaunchKernelGGL((rd<G, NT, RED>), dim3(grid), dim3(256), 0, 0, a[i], b[i], 0, x, n4, part);      \
    hipDeviceSynchronize();                                                                                   \
    std::vector<float> t(50);                                                                                 \
    for (int i = 0; i < 50; ++i) hipEventElapsedTime(&t[i], a[i], b[i]);                                      \
    float s = 0.f;                                                                                            \
    for (float v : t) s += v;                                                                                 \
    std::sort(t.begin(), t.end());                                                                            \
    cs.push_back({NAME, grid, s / 50, t[25]});                                                                \
  } while (0)
    CASE("oneshot_g1", 1, false, false, 0);
    CASE("oneshot_g2", 2, false, false, 0);
    CASE("oneshot_g4", 4, false, false, 0);
    CASE("oneshot_g8", 8, false, false, 0);
    CASE("oneshot_g2_nt", 2, true, false, 0);
    CASE("oneshot_g4_nt", 4, true, false, 0);
    CASE("oneshot_g2_red", 2, false, true, 0);
    CASE("stride2k_g2", 2, false, false, 2048);
    CASE("stride2k_g4", 4, false, false, 2048);
    CASE("stride2k_g2_red", 2, false, true, 2048);
    CASE("stride2k_g2_nt_red", 2, true, true, 2048);
    CASE("stride1k_g4_red", 4, false, true, 1024);
    CASE("stride1783_g2_red", 2, false, true, 1783);
#undef CASE
  }
  for (auto& c : cs) {
    const double gbps = 4.0 * n / (c.avg * 1e-3) / 1e9;
    printf("{\"case\": \"%s\", \"elems\": %lld, \"grid\": %d, \"avg_us\": %.2f, \"median_us\": %.2f, \"GBps\": %.1f, "
           "\"frac\": %.4f}\n",
           c.name, (long long)n, c.grid, c.avg * 1e3, c.med * 1e3, gbps, gbps / 8000.0);
  }
  hipFree(x);
  hipFree(part);
  return 0;
}
