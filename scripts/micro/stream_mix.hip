// Ceiling probe for the update kernels beyond the Infinity Cache: how fast does
// a plain grid of float4 lanes stream the same read / write mix as the fused
// SGD (p, g, momentum read; p, momentum written in place = 3R2W, 20 B/elem) and
// the fp32 Adam (4R3W, 28 B/elem), next to copy (1R1W) and a read-only sum (1R),
// with no chunk map, no descriptors, no tensor boundaries?  Loads cached or
// non-temporal, stores non-temporal or plain, G accesses in flight per lane,
// one-shot grid (one G-group per workgroup, as libgsync's chunk engine) or a
// resident grid-stride grid.  ResNet-152 x 2 elements (120.4 M, 2.4 GB per SGD
// launch: > 9x the 256 MiB cache), back-to-back launches timed by an event pair
// each (the beyond_ic harness's conditions).  One JSON line per case.  With case
// names as arguments: only those cases on the one-shot grid, each kernel timed
// by its own start / stop events (bench.py's live ceiling for the update rows).
// The cvt* cases are the 16-bit pack / unpack rows' mixes (bf16 -> bf16 4 B/elem,
// fp32 -> bf16 and bf16 -> fp32 6 B/elem); a bf16 source runs on 240.8 M elements
// (481 MB, past the cache as the fp32 sets are).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// R streams read (s[0..R-1]); the first W of them written back in place.
// SM: issue the loads stream-major (all G accesses of stream 0, then stream 1, ...)
// instead of access-major (every stream of access 0, then access 1, ...)
template <int R, int W, int G, bool NTL, bool NTS, bool SM = false>
__global__ void __launch_bounds__(256) mix(f4* __restrict__ s0, f4* __restrict__ s1, f4* __restrict__ s2,
                                          f4* __restrict__ s3, int64_t n4, float* __restrict__ part) {
  f4* s[4] = {s0, s1, s2, s3};
  const int64_t step = (int64_t)gridDim.x * 256 * G;
  float acc = 0.f;
  for (int64_t base = (int64_t)blockIdx.x * 256 * G; base < n4; base += step) {
    f4 v[G][R];
    if constexpr (SM) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int64_t i = base + (int64_t)g * 256 + threadIdx.x;
          v[g][r] = i < n4 ? ld<NTL>(s[r] + i) : f4{0.f, 0.f, 0.f, 0.f};
        }
      }
    } else {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int64_t i = base + (int64_t)g * 256 + threadIdx.x;
#pragma unroll
        for (int r = 0; r < R; ++r) v[g][r] = i < n4 ? ld<NTL>(s[r] + i) : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t i = base + (int64_t)g * 256 + threadIdx.x;
      if constexpr (W == 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) acc += v[g][r].x + v[g][r].y + v[g][r].z + v[g][r].w;
      } else if (i < n4) {
        if constexpr (R == 1) {
          st<NTS>(s[1] + i, v[g][0]);  // copy: s0 -> s1
        } else if constexpr (R == 3) {
          const f4 m = v[g][2] * 0.9f + v[g][1];  // SGD: buf = mu buf + g; p -= lr buf
          st<NTS>(s[2] + i, m);
          st<NTS>(s[0] + i, v[g][0] - 1e-6f * m);
        } else {
          const f4 m = v[g][2] * 0.9f + v[g][1] * 0.1f;  // Adam-shaped: m, v, p
          const f4 q = v[g][3] * 0.999f + v[g][1] * v[g][1] * 0.001f;
          st<NTS>(s[2] + i, m);
          st<NTS>(s[3] + i, q);
          st<NTS>(s[0] + i, v[g][0] - 1e-6f * m / (q + 1e-8f));
        }
      }
    }
  }
  if constexpr (W == 0) {
    if (acc == 12345.f) part[blockIdx.x] = acc;  // keeps the loads; never true for zeros
  }
}

// The 16-bit rows' mixes (bench.py's pack_bf16, pack_f32_to_bf16, unpack_bf16_to_f32):
// n elements of IN bytes read from src, converted, n elements of OUT bytes written
// to dst (non-temporal stores, as copy_*), E elements per lane access (4: libgsync's
// unit, 8-B bf16 accesses; 8: 16-B bf16 accesses), G accesses in flight per lane.
// fp32 -> bf16 rounds to nearest even, bf16 -> fp32 is exact.
template <int E, int IN>
struct Vec;
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
template <> struct Vec<4, 2> { typedef u2v T; };
template <> struct Vec<8, 2> { typedef u4v T; };
template <> struct Vec<4, 4> { typedef u4v T; };
template <> struct Vec<8, 4> { struct T { u4v a, b; }; };

__device__ __forceinline__ uint32_t bf16_rne(uint32_t u) { return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16; }

template <int E, int IN, bool NT>
__device__ __forceinline__ void ld_units(const void* p, int64_t i, uint32_t (&w)[E]) {
  typedef typename Vec<E, IN>::T V;
  const V* q = reinterpret_cast<const V*>(static_cast<const char*>(p) + i * IN);
  V v;
  if constexpr (IN == 4 && E == 8) {
    v.a = NT ? __builtin_nontemporal_load(&q->a) : q->a;
    v.b = NT ? __builtin_nontemporal_load(&q->b) : q->b;
  } else {
    v = NT ? __builtin_nontemporal_load(q) : *q;
  }
  if constexpr (IN == 4) {  // fp32 words
    const uint32_t* u = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
    for (int k = 0; k < E; ++k) w[k] = u[k];
  } else {  // packed bf16 pairs -> fp32 bit patterns
    const uint32_t* u = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
    for (int k = 0; k < E / 2; ++k) {
      w[2 * k] = u[k] << 16;
      w[2 * k + 1] = u[k] & 0xffff0000u;
    }
  }
}

template <int E, int OUT>
__device__ __forceinline__ void st_units(void* p, int64_t i, const uint32_t (&w)[E]) {
  typedef typename Vec<E, OUT>::T V;
  V v;
  uint32_t* u = reinterpret_cast<uint32_t*>(&v);
  if constexpr (OUT == 4) {
#pragma unroll
    for (int k = 0; k < E; ++k) u[k] = w[k];
  } else {
#pragma unroll
    for (int k = 0; k < E / 2; ++k) u[k] = bf16_rne(w[2 * k]) | (bf16_rne(w[2 * k + 1]) << 16);
  }
  V* q = reinterpret_cast<V*>(static_cast<char*>(p) + i * OUT);
  if constexpr (OUT == 4 && E == 8) {
    __builtin_nontemporal_store(v.a, &q->a);
    __builtin_nontemporal_store(v.b, &q->b);
  } else {
    __builtin_nontemporal_store(v, q);
  }
}

template <int IN, int OUT, int E, int G, bool NTL>
__global__ void __launch_bounds__(256) cvt(const void* __restrict__ src, void* __restrict__ dst, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * 256 * G * E;
  for (int64_t base = (int64_t)blockIdx.x * 256 * G * E; base < n; base += step) {
    uint32_t w[G][E];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t i = base + ((int64_t)g * 256 + threadIdx.x) * E;
      if (i < n) ld_units<E, IN, NTL>(src, i, w[g]);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t i = base + ((int64_t)g * 256 + threadIdx.x) * E;
      if (i < n) st_units<E, OUT>(dst, i, w[g]);
    }
  }
}

// launch(a, b): a null pair = a plain launch; else the kernel carries a / b as its
// own start / stop events (hipExtLaunchKernel, as libgsync's plan launch timer
// times its kernels) — the mode with case names on the command line; without
// them, an event pair of packets around each launch (the committed r4 runs)
static bool g_ext = false;
template <class K>
static float time_ms(K launch, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) launch(nullptr, nullptr);
  float tot = 0.f;
  for (int i = 0; i < iters; ++i) {
    if (g_ext) {
      launch(a, b);
    } else {
      hipEventRecord(a, 0);
      launch(nullptr, nullptr);
      hipEventRecord(b, 0);
    }
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    tot += ms;
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return tot / iters;
}

int main(int argc, char** argv) {
  // optional: case names to run (only those, grid 0 and both rounds), ext-event timing
  std::vector<std::string> only(argv + 1, argv + argc);
  g_ext = !only.empty();
  auto wanted = [&](const char* name, int gridc) {
    if (only.empty()) return true;
    if (gridc != 0) return false;
    for (auto& o : only)
      if (o == name) return true;
    return false;
  };
  const int64_t n = 120385616 / 1024 * 1024;  // ResNet-152 x 2, whole 1 Ki chunks
  const int64_t n4 = n / 4;
  // the 16-bit-source mixes run on twice the elements (n16): a 240 MB bf16 source would
  // sit in the 256 MiB Infinity Cache, a 481 MB one does not (bench.py's 16-bit rows the same)
  const int64_t n16 = 2 * n;
  f4* s[4];
  for (auto& p : s) {
    if (hipMalloc(&p, n16 * 4)) {
      printf("alloc failed\n");
      return 1;
    }
    hipMemset(p, 0, n16 * 4);
  }
  float* part;
  if (hipMalloc(&part, 65536 * 4)) return 1;
  struct Case {
    const char* name;
    double bytes_per_elem;
    float ms;
    int grid;
    int64_t elems = 0;  // 0: n
  };
  std::vector<Case> cs;
  for (int round = 0; round < 2; ++round) {
    for (int gridc : {0, 2048, 8192}) {
      auto g_of = [&](int G) { return gridc ? gridc : (int)std::min<int64_t>(1 << 30, (n4 + 256 * G - 1) / (256 * G)); };
#define CASE(NAME, BPE, R, W, G, NTL, NTS, ...)                                                                      \
  if (wanted(NAME, gridc))                                                                                           \
  cs.push_back({NAME, BPE,                                                                                           \
                time_ms([&](hipEvent_t ea, hipEvent_t eb) {                                                          \
                  if (ea)                                                                                            \
                    hipExtLaunchKernelGGL((mix<R, W, G, NTL, NTS, ##__VA_ARGS__>), dim3(g_of(G)), dim3(256), 0, 0,   \
                                          ea, eb, 0, s[0], s[1], s[2], s[3], n4, part);                              \
                  else                                                                                               \
                    mix<R, W, G, NTL, NTS, ##__VA_ARGS__><<<g_of(G), 256>>>(s[0], s[1], s[2], s[3], n4, part);       \
                }, 20),                                                                                              \
                gridc})
      CASE("read_sum_g4", 4, 1, 0, 4, false, true);
      CASE("read_sum_g4_ntl", 4, 1, 0, 4, true, true);
      CASE("copy_g4", 8, 1, 1, 4, false, true);
      CASE("copy_g4_ntl", 8, 1, 1, 4, true, true);
      CASE("sgd3r2w_g2", 20, 3, 2, 2, false, true);
      CASE("sgd3r2w_g4", 20, 3, 2, 4, false, true);
      CASE("sgd3r2w_g4_ntl", 20, 3, 2, 4, true, true);
      CASE("sgd3r2w_g4_plainst", 20, 3, 2, 4, false, false);
      CASE("sgd3r2w_g4_ntl_plainst", 20, 3, 2, 4, true, false);
      CASE("sgd3r2w_g8", 20, 3, 2, 8, false, true);
      CASE("adam4r3w_g4", 28, 4, 3, 4, false, true);
      CASE("adam4r3w_g4_ntl", 28, 4, 3, 4, true, true);
      CASE("sgd3r2w_g4_ntl_streammajor", 20, 3, 2, 4, true, true, true);
      CASE("sgd3r2w_g2_ntl_streammajor", 20, 3, 2, 2, true, true, true);
      CASE("adam4r3w_g4_ntl_streammajor", 28, 4, 3, 4, true, true, true);
#undef CASE
      // 16-bit mixes: src s[0], dst s[1]
      auto g16 = [&](int64_t m, int E, int G) {
        return gridc ? gridc : (int)std::min<int64_t>(1 << 30, (m + 256 * G * E - 1) / (256 * G * E));
      };
#define CVT(NAME, BPE, IN, OUT, E, G, NTL)                                                                           \
  if (wanted(NAME, gridc)) {                                                                                         \
    const int64_t m = IN == 2 ? n16 : n;                                                                             \
    cs.push_back({NAME, BPE,                                                                                         \
                  time_ms([&](hipEvent_t ea, hipEvent_t eb) {                                                        \
                    if (ea)                                                                                          \
                      hipExtLaunchKernelGGL((cvt<IN, OUT, E, G, NTL>), dim3(g16(m, E, G)), dim3(256), 0, 0, ea, eb,  \
                                            0, (const void*)s[0], (void*)s[1], m);                                   \
                    else                                                                                             \
                      cvt<IN, OUT, E, G, NTL><<<g16(m, E, G), 256>>>(s[0], s[1], m);                                 \
                  }, 20),                                                                                            \
                  gridc, m});                                                                                        \
  }
      CVT("cvt16_16_e4", 4, 2, 2, 4, 4, false);
      CVT("cvt16_16_e8", 4, 2, 2, 8, 4, false);
      CVT("cvt16_16_e8_ntl", 4, 2, 2, 8, 4, true);
      CVT("cvt32_16_e4", 6, 4, 2, 4, 4, false);
      CVT("cvt32_16_e8", 6, 4, 2, 8, 4, false);
      CVT("cvt32_16_e4_ntl", 6, 4, 2, 4, 4, true);
      CVT("cvt16_32_e4", 6, 2, 4, 4, 4, false);
      CVT("cvt16_32_e8", 6, 2, 4, 8, 4, false);
      CVT("cvt16_32_e8_ntl", 6, 2, 4, 8, 4, true);
#undef CVT
    }
  }
  for (auto& c : cs) {
    const int64_t m = c.elems ? c.elems : n;
    const double gbps = c.bytes_per_elem * m / (c.ms * 1e-3) / 1e9;
    printf("{\"case\": \"%s\", \"elems\": %lld, \"grid\": %d, \"avg_ms\": %.5f, \"GBps\": %.1f, \"frac\": %.4f}\n", c.name,
           (long long)m, c.grid, c.ms, gbps, gbps / 8000.0);
  }
  for (auto& p : s) hipFree(p);
  hipFree(part);
  return 0;
}
