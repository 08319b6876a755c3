// Streaming scale-copy shapes at the grad-sync sizes, to locate the gap between
// libgsync's pack (one resident wave of looping workgroups) and HIP's own D2D
// copy at Infinity-Cache-resident sizes (profiles/r1n_ab_interleave_ceiling.jsonl:
// 4.8 vs 6.7 TB/s at 25.6 M fp32).  Not product code.
//   hipcc -O3 --offload-arch=gfx950 scripts/copy_micro.hip -o scripts/build/copy_micro
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kB = 256;

// one shot: K float4 per lane, no loop, grid covers the array
template <int K>
__global__ void __launch_bounds__(kB) copy_grid(const f4* __restrict__ s, f4* __restrict__ d, long n4, float a) {
  const long base = static_cast<long>(blockIdx.x) * kB * K + threadIdx.x;
  f4 v[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const long i = base + j * kB;
    if (i < n4) v[j] = s[i];
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const long i = base + j * kB;
    if (i < n4) d[i] = v[j] * a;
  }
}

// resident grid, chunks of kB*ILP float4 taken round-robin (the interleaved sweep)
template <int ILP>
__global__ void __launch_bounds__(kB) copy_persist(const f4* __restrict__ s, f4* __restrict__ d, long n4, float a) {
  for (long c = blockIdx.x; c * kB * ILP < n4; c += gridDim.x) {
    const long base = c * kB * ILP + threadIdx.x;
    f4 v[ILP];
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      const long i = base + j * kB;
      if (i < n4) v[j] = s[i];
    }
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      const long i = base + j * kB;
      if (i < n4) d[i] = v[j] * a;
    }
  }
}

// the same resident grid with non-temporal stores (libgsync's GS_NT_STORE=1)
template <int ILP>
__global__ void __launch_bounds__(kB) copy_persist_nt(const f4* __restrict__ s, f4* __restrict__ d, long n4, float a) {
  for (long c = blockIdx.x; c * kB * ILP < n4; c += gridDim.x) {
    const long base = c * kB * ILP + threadIdx.x;
    f4 v[ILP];
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      const long i = base + j * kB;
      if (i < n4) v[j] = s[i];
    }
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      const long i = base + j * kB;
      if (i < n4) __builtin_nontemporal_store(v[j] * a, &d[i]);
    }
  }
}

// resident grid behind a 3-deep dependent descriptor chain per workgroup
// (task -> segment -> pointer), as libgsync's single-segment tasks
__global__ void __launch_bounds__(kB) copy_persist_desc(const int* __restrict__ task_seg,
                                                        const int* __restrict__ seg_tensor,
                                                        const f4* const* __restrict__ ptrs, f4* __restrict__ d,
                                                        long n4, float a) {
  const int sg = task_seg[blockIdx.x];
  const int t = seg_tensor[sg];
  const f4* s = ptrs[t];
  constexpr int ILP = 4;
  for (long c = blockIdx.x; c * kB * ILP < n4; c += gridDim.x) {
    const long base = c * kB * ILP + threadIdx.x;
    f4 v[ILP];
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      const long i = base + j * kB;
      if (i < n4) v[j] = s[i];
    }
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      const long i = base + j * kB;
      if (i < n4) __builtin_nontemporal_store(v[j] * a, &d[i]);
    }
  }
}

// non-constant source data (a hash of the index): an all-zero buffer streams
// faster than real data through the memory system
__global__ void fill_hash(f4* p, long n4) {
  const long i = static_cast<long>(blockIdx.x) * kB + threadIdx.x;
  if (i >= n4) return;
  unsigned h = static_cast<unsigned>(i) * 2654435761u;
  f4 v;
  v.x = static_cast<float>(h & 0xffff) * 1e-4f;
  v.y = static_cast<float>(h >> 16) * 1e-4f;
  v.z = static_cast<float>((h ^ 0x5bd1e995u) & 0xffff) * 1e-4f;
  v.w = static_cast<float>((h * 31u) >> 16) * 1e-4f;
  p[i] = v;
}

template <class F>
static float timed(F f, hipEvent_t* ev, int reps) {
  for (int i = 0; i < 5; ++i) f();
  std::vector<float> ms(reps);
  for (int i = 0; i < reps; ++i) {
    (void)hipEventRecord(ev[0], 0);
    f();
    (void)hipEventRecord(ev[1], 0);
    (void)hipEventSynchronize(ev[1]);
    (void)hipEventElapsedTime(&ms[i], ev[0], ev[1]);
  }
  std::sort(ms.begin(), ms.end());
  return ms[reps / 2];
}

int main() {
  const long sizes[] = {25557032L, 60192808L, 120385616L};
  hipEvent_t ev[2];
  CK(hipEventCreate(&ev[0]));
  CK(hipEventCreate(&ev[1]));
  for (long n : sizes) {
    const long n4 = n / 4;
    const size_t bytes = static_cast<size_t>(n4) * 16;
    f4 *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    fill_hash<<<(n4 + kB - 1) / kB, kB>>>(s, n4);
    fill_hash<<<(n4 + kB - 1) / kB, kB>>>(d, n4);
    CK(hipDeviceSynchronize());
    const double alg = 2.0 * bytes;
    auto rate = [&](float ms) { return alg / (ms * 1e-3) / 1e9; };
    printf("{\"elements\": %ld, \"bytes\": %.0f", n, alg);
    float t = timed([&] { (void)hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }, ev, 30);
    printf(", \"hipMemcpy_D2D\": %.0f", rate(t));
#define GRID(K)                                                                                         \
  t = timed([&] { copy_grid<K><<<(n4 + kB * K - 1) / (kB * K), kB>>>(s, d, n4, 0.5f); }, ev, 30); \
  printf(", \"grid_k%d\": %.0f", K, rate(t));
    GRID(1) GRID(2) GRID(4) GRID(8)
#define PERSIST(ILP, G)                                                              \
  t = timed([&] { copy_persist<ILP><<<G, kB>>>(s, d, n4, 0.5f); }, ev, 30); \
  printf(", \"persist_ilp%d_g%d\": %.0f", ILP, G, rate(t));
    PERSIST(4, 1024) PERSIST(4, 1920) PERSIST(4, 2048) PERSIST(4, 4096) PERSIST(2, 2048) PERSIST(2, 4096)
    PERSIST(1, 8192)
    t = timed([&] { copy_persist_nt<4><<<1920, kB>>>(s, d, n4, 0.5f); }, ev, 30);
    printf(", \"persist_nt_ilp4_g1920\": %.0f", rate(t));
    t = timed([&] { copy_persist_nt<2><<<4096, kB>>>(s, d, n4, 0.5f); }, ev, 30);
    printf(", \"persist_nt_ilp2_g4096\": %.0f", rate(t));
    {
      int *ts, *st;
      const f4** pt;
      CK(hipMalloc(&ts, 65536 * sizeof(int)));
      CK(hipMalloc(&st, sizeof(int)));
      CK(hipMalloc(&pt, sizeof(f4*)));
      CK(hipMemset(ts, 0, 65536 * sizeof(int)));
      CK(hipMemset(st, 0, sizeof(int)));
      CK(hipMemcpy(pt, &s, sizeof(f4*), hipMemcpyHostToDevice));
      t = timed([&] { copy_persist_desc<<<1920, kB>>>(ts, st, pt, d, n4, 0.5f); }, ev, 30);
      printf(", \"persist_desc_nt_ilp4_g1920\": %.0f", rate(t));
      CK(hipFree(ts));
      CK(hipFree(st));
      CK(hipFree(pt));
    }
    CK(hipGetLastError());
    printf("}\n");
    fflush(stdout);
    CK(hipFree(s));
    CK(hipFree(d));
  }
  return 0;
}
