// Store-width probe for the 16-bit pack (fp32 -> bf16, the bf16 bucket / ZeRO
// cast): does a lane that moves 8 elements (two 16-B loads, ONE 16-B store) beat
// the chunk engine's 4 elements (one 16-B load, one 8-B store)?  Also bf16 -> bf16
// (8-B vs 16-B loads and stores).  Grid-stride streaming, 256-thread workgroups,
// non-temporal stores as libgsync's kernels; > 256 MiB working sets (beyond the
// Infinity Cache) and a ResNet-50-sized one.  Prints one JSON line per case.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t bf(float f) {
  uint32_t u = __float_as_uint(f);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ uint32_t pk(float a, float b) { return bf(a) | (bf(b) << 16); }

// W = elements per lane per access (4 or 8); G = accesses in flight per lane
template <int W, int G>
__global__ void __launch_bounds__(256) cvt(const float* __restrict__ x, uint16_t* __restrict__ y, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * 256 * W * G;
  for (int64_t base = ((int64_t)blockIdx.x * 256 * G) * W; base < n; base += step) {
    f4 a[G][W / 4];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t e = base + ((int64_t)g * 256 + threadIdx.x) * W;
#pragma unroll
      for (int h = 0; h < W / 4; ++h) a[g][h] = *(const f4*)(x + e + 4 * h);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t e = base + ((int64_t)g * 256 + threadIdx.x) * W;
      if constexpr (W == 4) {
        u2 v; v.x = pk(a[g][0].x, a[g][0].y); v.y = pk(a[g][0].z, a[g][0].w);
        __builtin_nontemporal_store(v, (u2*)(y + e));
      } else {
        u4 v; v.x = pk(a[g][0].x, a[g][0].y); v.y = pk(a[g][0].z, a[g][0].w);
        v.z = pk(a[g][1].x, a[g][1].y); v.w = pk(a[g][1].z, a[g][1].w);
        __builtin_nontemporal_store(v, (u4*)(y + e));
      }
    }
  }
}

// bf16 -> bf16 copy x 1/ws (the ZeRO bucket pack): W = 4 (8-B) or 8 (16-B) per access
template <int W, int G>
__global__ void __launch_bounds__(256) cp16(const uint16_t* __restrict__ x, uint16_t* __restrict__ y, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * 256 * W * G;
  for (int64_t base = ((int64_t)blockIdx.x * 256 * G) * W; base < n; base += step) {
    if constexpr (W == 4) {
      u2 a[G];
#pragma unroll
      for (int g = 0; g < G; ++g) a[g] = *(const u2*)(x + base + ((int64_t)g * 256 + threadIdx.x) * W);
#pragma unroll
      for (int g = 0; g < G; ++g) __builtin_nontemporal_store(a[g], (u2*)(y + base + ((int64_t)g * 256 + threadIdx.x) * W));
    } else {
      u4 a[G];
#pragma unroll
      for (int g = 0; g < G; ++g) a[g] = *(const u4*)(x + base + ((int64_t)g * 256 + threadIdx.x) * W);
#pragma unroll
      for (int g = 0; g < G; ++g) __builtin_nontemporal_store(a[g], (u4*)(y + base + ((int64_t)g * 256 + threadIdx.x) * W));
    }
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
  const int64_t sizes[] = {25557032 / 1024 * 1024, 120385616 / 1024 * 1024};  // ResNet-50, ResNet-152 x 2
  for (int64_t n : sizes) {
    float* x; uint16_t* y; uint16_t* x16;
    if (hipMalloc(&x, n * 4) || hipMalloc(&y, n * 2) || hipMalloc(&x16, n * 2)) { printf("alloc failed\n"); return 1; }
    hipMemset(x, 0, n * 4); hipMemset(x16, 0, n * 2);
    for (int grid : {2048, 8192, 0}) {
      auto g_of = [&](int per) { return grid ? grid : (int)std::min<int64_t>(65536, (n + per - 1) / per); };
      struct Case { const char* name; float ms; double bytes; };
      std::vector<Case> cs;
      int g4 = g_of(256 * 4 * 2), g8 = g_of(256 * 8 * 2);
      cs.push_back({"cvt_w4_g2", time_ms([&] { cvt<4, 2><<<g4, 256>>>(x, y, n); }, 20), 6.0 * n});
      cs.push_back({"cvt_w8_g2", time_ms([&] { cvt<8, 2><<<g8, 256>>>(x, y, n); }, 20), 6.0 * n});
      cs.push_back({"cvt_w4_g4", time_ms([&] { cvt<4, 4><<<g_of(256 * 16), 256>>>(x, y, n); }, 20), 6.0 * n});
      cs.push_back({"cvt_w8_g1", time_ms([&] { cvt<8, 1><<<g_of(256 * 8), 256>>>(x, y, n); }, 20), 6.0 * n});
      cs.push_back({"cp16_w4_g2", time_ms([&] { cp16<4, 2><<<g4, 256>>>(x16, y, n); }, 20), 4.0 * n});
      cs.push_back({"cp16_w8_g2", time_ms([&] { cp16<8, 2><<<g8, 256>>>(x16, y, n); }, 20), 4.0 * n});
      cs.push_back({"cp16_w4_g4", time_ms([&] { cp16<4, 4><<<g_of(256 * 16), 256>>>(x16, y, n); }, 20), 4.0 * n});
      for (auto& c : cs)
        printf("{\"case\": \"%s\", \"elems\": %lld, \"grid\": %d, \"avg_ms\": %.5f, \"GBps\": %.1f, \"frac\": %.4f}\n", c.name,
               (long long)n, grid, c.ms, c.bytes / (c.ms * 1e-3) / 1e9, c.bytes / (c.ms * 1e-3) / 1e9 / 8000.0);
    }
    hipFree(x); hipFree(y); hipFree(x16);
  }
  return 0;
}
