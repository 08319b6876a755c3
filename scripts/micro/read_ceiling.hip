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
// per workgroup), with the chunk engine's dependent scalar loads ahead of
// every iteration's data loads (rd_tab), with its two-level in-kernel combine
// as the epilogue (rd_ticket), and with a polling combiner (rd_poll, checked
// against the host's double sum).  The buffer holds hashed non-zero
// values (the first run read zeros).  One JSON line per case.
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
    if (acc == 12345.f) part[blockIdx.x] = acc;  // keeps the loads; (almost) never true
  }
}

// The same grid-stride read, but every iteration first reads its group's place
// through DEP dependent scalar loads, as the chunk engine does (chunk-table
// entry, then the tensor's offset): tab[g] = g, off[t] = t * 256 * G float4s
#define CONST_AS __attribute__((address_space(4)))
template <int G, bool NT, int DEP>
__global__ void __launch_bounds__(256) rd_tab(const f4* __restrict__ x, int64_t n4, float* __restrict__ part,
                                              const int* tab, const int64_t* off) {
  __shared__ float s[4];
  float acc = 0.f;
  const int64_t ngroups = (n4 + 256 * G - 1) / (256 * G);
  for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int t = ((const CONST_AS int*)tab)[g];
    const int64_t base = DEP >= 2 ? ((const CONST_AS int64_t*)off)[t] : (int64_t)t * 256 * G;
    f4 v[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int64_t i = base + (int64_t)j * 256 + threadIdx.x;
      v[j] = i < n4 ? ld<NT>(x + i) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < G; ++j) acc += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = s[0] + s[1] + s[2] + s[3];
}

// rd_tab<..., 2> with the chunk engine's in-kernel combine instead of the plain
// store: the two-level ticket over R = 64 groups (gs_engine.h chunk_kernel: an
// agent-scope store of the partial, vmcnt(0), an atomic add on the group's
// counter; the group's last arriver folds the group, publishes its sum and
// arrives on the top counter; the last group folds the 64 sums).
template <bool NT>
__global__ void __launch_bounds__(256) rd_ticket(const f4* __restrict__ x, int64_t n4, float* __restrict__ part,
                                                 const int* tab, const int64_t* off, uint32_t* ticket,
                                                 float* out) {
  __shared__ float s[4];
  __shared__ int s_role;
  constexpr int G = 2, R = 64, kStride = 32;
  float acc = 0.f;
  const int64_t ngroups = (n4 + 256 * G - 1) / (256 * G);
  for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int t = ((const CONST_AS int*)tab)[g];
    const int64_t base = ((const CONST_AS int64_t*)off)[t];
    f4 v[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int64_t i = base + (int64_t)j * 256 + threadIdx.x;
      v[j] = i < n4 ? ld<NT>(x + i) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < G; ++j) acc += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  const float r = s[0] + s[1] + s[2] + s[3];
  const int k = blockIdx.x & (R - 1);
  const int grid = gridDim.x;
  uint32_t* top = &ticket[R * kStride];
  float* gsums = reinterpret_cast<float*>(ticket + (R + 1) * kStride);
  if (threadIdx.x == 0) {
    const uint32_t ng = (uint32_t)((grid - 1 - k) / R + 1);
    __hip_atomic_store(&part[blockIdx.x], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t tk = __hip_atomic_fetch_add(&ticket[k * kStride], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_role = tk == ng - 1;
  }
  __syncthreads();
  if (!s_role) return;
  float v = 0.f;
  for (int i = k + R * (int)threadIdx.x; i < grid; i += R * 256)
    v += __hip_atomic_load(&part[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float gsum = s[0] + s[1] + s[2] + s[3];
    __hip_atomic_store(&ticket[k * kStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&gsums[k * kStride], gsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t tk = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_role = tk == (uint32_t)(grid < R ? grid : R) - 1 ? 2 : 0;
  }
  __syncthreads();
  if (s_role != 2 || threadIdx.x >= 64) return;
  float t = 0.f;
  for (int j = threadIdx.x; j < (grid < R ? grid : R); j += 64)
    t += __hip_atomic_load(&gsums[j * kStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = wave_sum(t);
  if (threadIdx.x == 0) {
    out[0] = t;
    __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The same with a polling combiner instead of the last-arriver hand-offs:
// every other workgroup stores its partial (sc1), drains it and adds to its
// group's counter without waiting for the add (64 counters, one 128-B line
// each); workgroup 0, after its own data, polls the 64 counters (one per lane
// of wave 0, sc1 loads) until every group has arrived, re-arms them and folds
// all partials in a fixed order.  The spin is bounded (kPollMax polls, then
// the result is NaN) so that a lost arrival cannot hang the GPU.
constexpr int kPollMax = 1 << 22;
template <bool NT>
__global__ void __launch_bounds__(256) rd_poll(const f4* __restrict__ x, int64_t n4, float* __restrict__ part,
                                               const int* tab, const int64_t* off, uint32_t* ticket, float* out) {
  __shared__ float s[4];
  __shared__ int s_ok;
  constexpr int G = 2, R = 64, kStride = 32;
  float acc = 0.f;
  const int64_t ngroups = (n4 + 256 * G - 1) / (256 * G);
  for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int t = ((const CONST_AS int*)tab)[g];
    const int64_t base = ((const CONST_AS int64_t*)off)[t];
    f4 v[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int64_t i = base + (int64_t)j * 256 + threadIdx.x;
      v[j] = i < n4 ? ld<NT>(x + i) : f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int j = 0; j < G; ++j) acc += v[j].x * v[j].x + v[j].y * v[j].y + v[j].z * v[j].z + v[j].w * v[j].w;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  const float r = s[0] + s[1] + s[2] + s[3];
  const int grid = gridDim.x;
  if (blockIdx.x != 0) {
    if (threadIdx.x == 0) {
      __hip_atomic_store(&part[blockIdx.x], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&ticket[(blockIdx.x & (R - 1)) * kStride], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (threadIdx.x < 64) {
    const int j = threadIdx.x;
    const uint32_t want = j < grid ? (uint32_t)((grid - 1 - j) / R + 1) - (j == 0 ? 1u : 0u) : 0u;
    int ok = 0;
    for (int it = 0; it < kPollMax; ++it) {
      const uint32_t c = __hip_atomic_load(&ticket[j * kStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all(c >= want)) {
        ok = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(&ticket[j * kStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (j == 0) s_ok = ok;
  }
  __syncthreads();
  float v = 0.f;
  for (int i = threadIdx.x; i < grid; i += 256)
    v += i == 0 ? r : __hip_atomic_load(&part[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = s_ok ? s[0] + s[1] + s[2] + s[3] : __builtin_nanf("");
}

__global__ void fill_tab(int* tab, int64_t* off, int64_t ng, int G) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < ng; i += (int64_t)gridDim.x * 256) {
    tab[i] = (int)i;
    off[i] = i * 256 * G;
  }
}

// non-zero, incompressible-looking contents (an integer hash of the index)
__global__ void fill(float* x, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint32_t h = (uint32_t)i * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    x[i] = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * 0.02f;
  }
}

int main() {
  const int64_t n = 25557032 / 1024 * 1024;  // ResNet-50's parameters, whole 1 Ki chunks
  const int64_t n4 = n / 4;
  f4* x;
  float* part;
  if (hipMalloc(&x, n * 4) || hipMalloc(&part, 65536 * 4)) return 1;
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (float*)x, n);
  hipDeviceSynchronize();
  int* tab;
  int64_t* off;
  const int64_t ng2 = (n4 + 511) / 512;
  if (hipMalloc(&tab, ng2 * 4) || hipMalloc(&off, ng2 * 8)) return 1;
  hipLaunchKernelGGL(fill_tab, dim3(256), dim3(256), 0, 0, tab, off, ng2, 2);
  hipDeviceSynchronize();
  uint32_t* ticket;
  float* outv;
  if (hipMalloc(&ticket, 64 * 1024) || hipMalloc(&outv, 64)) return 1;
  hipMemset(ticket, 0, 64 * 1024);
  double ref = 0.0;
  {
    std::vector<float> h(n);
    hipMemcpy(h.data(), x, n * 4, hipMemcpyDeviceToHost);
    for (float v : h) ref += (double)v * v;
  }
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
#define TCASE(NAME, NT, DEP)                                                                                  \
  do {                                                                                                        \
    for (int i = 0; i < 3; ++i)                                                                               \
      hipLaunchKernelGGL((rd_tab<2, NT, DEP>), dim3(2048), dim3(256), 0, 0, x, n4, part, tab, off);           \
    for (int i = 0; i < 50; ++i)                                                                              \
      hipExtLaunchKernelGGL((rd_tab<2, NT, DEP>), dim3(2048), dim3(256), 0, 0, a[i], b[i], 0, x, n4, part, tab, \
                            off);                                                                             \
    hipDeviceSynchronize();                                                                                   \
    std::vector<float> t(50);                                                                                 \
    for (int i = 0; i < 50; ++i) hipEventElapsedTime(&t[i], a[i], b[i]);                                      \
    float s = 0.f;                                                                                            \
    for (float v : t) s += v;                                                                                 \
    std::sort(t.begin(), t.end());                                                                            \
    cs.push_back({NAME, 2048, s / 50, t[25]});                                                                \
  } while (0)
#define KCASE(NAME, NT)                                                                                       \
  do {                                                                                                        \
    for (int i = 0; i < 3; ++i)                                                                               \
      hipLaunchKernelGGL((rd_ticket<NT>), dim3(2048), dim3(256), 0, 0, x, n4, part, tab, off, ticket, outv);  \
    for (int i = 0; i < 50; ++i)                                                                              \
      hipExtLaunchKernelGGL((rd_ticket<NT>), dim3(2048), dim3(256), 0, 0, a[i], b[i], 0, x, n4, part, tab, off, \
                            ticket, outv);                                                                    \
    hipDeviceSynchronize();                                                                                   \
    std::vector<float> t(50);                                                                                 \
    for (int i = 0; i < 50; ++i) hipEventElapsedTime(&t[i], a[i], b[i]);                                      \
    float s = 0.f;                                                                                            \
    for (float v : t) s += v;                                                                                 \
    std::sort(t.begin(), t.end());                                                                            \
    cs.push_back({NAME, 2048, s / 50, t[25]});                                                                \
  } while (0)
#define PCASE(NAME, NT)                                                                                       \
  do {                                                                                                        \
    for (int i = 0; i < 3; ++i)                                                                               \
      hipLaunchKernelGGL((rd_poll<NT>), dim3(2048), dim3(256), 0, 0, x, n4, part, tab, off, ticket, outv);    \
    for (int i = 0; i < 50; ++i)                                                                              \
      hipExtLaunchKernelGGL((rd_poll<NT>), dim3(2048), dim3(256), 0, 0, a[i], b[i], 0, x, n4, part, tab, off, \
                            ticket, outv);                                                                    \
    if (hipDeviceSynchronize() != hipSuccess) return 2;                                                       \
    std::vector<float> t(50);                                                                                 \
    for (int i = 0; i < 50; ++i) hipEventElapsedTime(&t[i], a[i], b[i]);                                      \
    float s = 0.f;                                                                                            \
    for (float v : t) s += v;                                                                                 \
    std::sort(t.begin(), t.end());                                                                            \
    cs.push_back({NAME, 2048, s / 50, t[25]});                                                                \
    float o = 0.f;                                                                                            \
    hipMemcpy(&o, outv, 4, hipMemcpyDeviceToHost);                                                            \
    printf("{\"check\": \"%s\", \"sum\": %.6e, \"ref\": %.6e}\n", NAME, o, ref);                            \
  } while (0)
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
    TCASE("stride2k_g2_red_tab1", false, 1);
    TCASE("stride2k_g2_red_tab2", false, 2);
    TCASE("stride2k_g2_nt_red_tab1", true, 1);
    TCASE("stride2k_g2_nt_red_tab2", true, 2);
    KCASE("stride2k_g2_tab2_ticket", false);
    KCASE("stride2k_g2_nt_tab2_ticket", true);
    PCASE("stride2k_g2_tab2_poll", false);
    PCASE("stride2k_g2_nt_tab2_poll", true);
#undef CASE
#undef PCASE
#undef KCASE
#undef TCASE
  }
  for (auto& c : cs) {
    const double gbps = 4.0 * n / (c.avg * 1e-3) / 1e9;
    printf("{\"case\": \"%s\", \"elems\": %lld, \"grid\": %d, \"avg_us\": %.2f, \"median_us\": %.2f, \"GBps\": %.1f, "
           "\"frac\": %.4f}\n",
           c.name, (long long)n, c.grid, c.avg * 1e3, c.med * 1e3, gbps, gbps / 8000.0);
  }
  hipFree(x);
  hipFree(part);
  hipFree(tab);
  hipFree(off);
  hipFree(ticket);
  hipFree(outv);
  return 0;
}
