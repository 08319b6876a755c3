// Descriptor-chain probe for the chunk engine's short kernels: the fp32 -> bf16
// conversion of cvt_width.hip (4 elements per lane, G accesses in flight, one group
// per workgroup), preceded by D dependent scalar loads through the constant
// address space, as chunk_kernel reads its chunk map (t, code) and then the tensor
// descriptor (stream pointer) before the first data load.  D = 0 / 1 / 2; also a
// persistent grid (4 workgroups per CU) that prefetches the next group's
// descriptors while the current group's data is in flight (PF = 1).  ResNet-50 and
// ResNet-152 x 2 element counts.  One JSON line per case.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));
#define CONST_AS __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ T cload(const T* p, int64_t i) { return ((const CONST_AS T*)(p))[i]; }

__device__ __forceinline__ uint32_t bf(float f) {
  uint32_t u = __float_as_uint(f);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

struct Desc { const float* x; uint16_t* y; };

template <int G, int D>
__global__ void __launch_bounds__(256) chain(const int* map, const Desc* descs, const float* x0, uint16_t* y0,
                                              int64_t n_groups) {
  for (int64_t grp = blockIdx.x; grp < n_groups; grp += gridDim.x) {
    const float* x = x0;
    uint16_t* y = y0;
    int64_t g = grp;
    if constexpr (D >= 1) g = cload(map, grp);            // the chunk map: group -> (tensor, offset)
    if constexpr (D >= 2) {                                // the tensor descriptor: stream pointers
      x = (const float*)cload((const uint64_t*)descs, 2 * (g & 1));
      y = (uint16_t*)cload((const uint64_t*)descs, 2 * (g & 1) + 1);
    }
    const int64_t base = g * 256 * 4 * G;
    f4 a[G];
#pragma unroll
    for (int j = 0; j < G; ++j) a[j] = *(const f4*)(x + base + (j * 256 + threadIdx.x) * 4);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      u2 v;
      v.x = bf(a[j].x) | (bf(a[j].y) << 16);
      v.y = bf(a[j].z) | (bf(a[j].w) << 16);
      __builtin_nontemporal_store(v, (u2*)(y + base + (j * 256 + threadIdx.x) * 4));
    }
  }
}

// persistent grid, next group's descriptors fetched before this group's data is used
template <int G>
__global__ void __launch_bounds__(256) chain_pf(const int* map, const Desc* descs, int64_t n_groups) {
  int64_t grp = blockIdx.x;
  if (grp >= n_groups) return;
  int64_t g = cload(map, grp);
  const float* x = (const float*)cload((const uint64_t*)descs, 2 * (g & 1));
  uint16_t* y = (uint16_t*)cload((const uint64_t*)descs, 2 * (g & 1) + 1);
  while (true) {
    const int64_t base = g * 256 * 4 * G;
    f4 a[G];
#pragma unroll
    for (int j = 0; j < G; ++j) a[j] = *(const f4*)(x + base + (j * 256 + threadIdx.x) * 4);
    const int64_t nxt = grp + gridDim.x;
    int64_t g2 = 0;
    const float* x2 = nullptr;
    uint16_t* y2 = nullptr;
    if (nxt < n_groups) {
      g2 = cload(map, nxt);
      x2 = (const float*)cload((const uint64_t*)descs, 2 * (g2 & 1));
      y2 = (uint16_t*)cload((const uint64_t*)descs, 2 * (g2 & 1) + 1);
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      u2 v;
      v.x = bf(a[j].x) | (bf(a[j].y) << 16);
      v.y = bf(a[j].z) | (bf(a[j].w) << 16);
      __builtin_nontemporal_store(v, (u2*)(y + base + (j * 256 + threadIdx.x) * 4));
    }
    if (nxt >= n_groups) break;
    grp = nxt; g = g2; x = x2; y = y2;
  }
}

template <class K>
static float time_ms(K launch, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch();
  float tot = 0.f;
  for (int i = 0; i < iters; ++i) {
    hipEventRecord(a, 0); launch(); hipEventRecord(b, 0); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); tot += ms;
  }
  hipEventDestroy(a); hipEventDestroy(b);
  return tot / iters;
}

int main() {
  constexpr int G = 8;
  const int64_t per = 256 * 4 * G;
  const int64_t sizes[] = {25557032 / per * per, 120385616 / per * per};
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int64_t n : sizes) {
    const int64_t ng = n / per;
    float* x; uint16_t* y; int* map; Desc* descs;
    if (hipMalloc(&x, n * 4) || hipMalloc(&y, n * 2) || hipMalloc(&map, ng * 4) || hipMalloc(&descs, 2 * sizeof(Desc))) {
      printf("alloc failed\n"); return 1;
    }
    hipMemset(x, 0, n * 4);
    std::vector<int> h(ng);
    for (int64_t i = 0; i < ng; ++i) h[i] = (int)i;
    hipMemcpy(map, h.data(), ng * 4, hipMemcpyHostToDevice);
    Desc hd[2] = {{x, y}, {x, y}};
    hipMemcpy(descs, hd, sizeof(hd), hipMemcpyHostToDevice);
    const double bytes = 6.0 * n;
    struct C { const char* name; float ms; };
    std::vector<C> cs;
    cs.push_back({"d0", time_ms([&] { chain<G, 0><<<ng, 256>>>(map, descs, x, y, ng); }, 20)});
    cs.push_back({"d1", time_ms([&] { chain<G, 1><<<ng, 256>>>(map, descs, x, y, ng); }, 20)});
    cs.push_back({"d2", time_ms([&] { chain<G, 2><<<ng, 256>>>(map, descs, x, y, ng); }, 20)});
    for (int per_cu : {4, 8, 16}) {
      const int grid = (int)std::min<int64_t>(ng, (int64_t)cus * per_cu);
      char* nm = new char[32];
      snprintf(nm, 32, "d2_persistent_%d", per_cu);
      cs.push_back({nm, time_ms([&] { chain<G, 2><<<grid, 256>>>(map, descs, x, y, ng); }, 20)});
      nm = new char[32];
      snprintf(nm, 32, "d2_prefetch_%d", per_cu);
      cs.push_back({nm, time_ms([&] { chain_pf<G><<<grid, 256>>>(map, descs, ng); }, 20)});
    }
    for (auto& c : cs)
      printf("{\"case\": \"%s\", \"elems\": %lld, \"avg_ms\": %.5f, \"frac\": %.4f}\n", c.name, (long long)n, c.ms,
             bytes / (c.ms * 1e-3) / 1e9 / 8000.0);
    hipFree(x); hipFree(y); hipFree(map); hipFree(descs);
  }
  return 0;
}
