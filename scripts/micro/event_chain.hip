// Stream-packet probe for libgsync's short dependent chains (the exposed
// end-of-backward tail: pack -> collective -> unpack; configs[3]'s clip path:
// Σg² -> 64-float all-reduce -> update).  A chain of K kernels on one stream,
// queued behind a spin kernel so that host enqueue never paces it, timed by an
// event pair around the chain.  Variants: plain launches; each launch followed
// by hipEventRecord of a timing-disabled event (what every plan launch did to
// keep `last_event`); of a timing event; the same event attached to the launch
// itself (hipExtLaunchKernel's stop event; its start event; both); a
// cross-stream wait on an event recorded long before.  Kernels: a 1-workgroup no-op (pure dispatch) and a
// 12.8 MB copy (3.2 M floats: a ZeRO N=8 shard).  One JSON line per case.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void spin(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}

__global__ void noop(float* p) {
  if (threadIdx.x == 0 && p[0] == 12345.f) p[1] = 1.f;
}

typedef float f4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) copy4(const f4* __restrict__ x, f4* __restrict__ y, int64_t n4) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) y[i] = x[i];
}

enum Mode { PLAIN = 0, REC_NOTIME = 1, REC_TIME = 2, EXT_NOTIME = 3, EXT_TIME = 4, XWAIT = 5, EXT_START = 6,
            EXT_BOTH = 7 };
static const char* kModeName[] = {"plain", "record_notiming", "record_timing", "ext_stop_notiming",
                                  "ext_stop_timing", "cross_stream_wait", "ext_start_timing", "ext_start_stop_timing"};

int main() {
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int64_t n = 3200000;
  float *x, *y, *tiny;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&tiny, 64));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMemset(tiny, 0, 64));
  hipEvent_t a, b, ev_nt, ev_t, ev_x, ev_s;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventCreateWithFlags(&ev_nt, hipEventDisableTiming));
  CK(hipEventCreate(&ev_t));
  CK(hipEventCreateWithFlags(&ev_x, hipEventDisableTiming));
  CK(hipEventCreate(&ev_s));
  // spin calibration: ~150 us of clock64 at any clock
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 1000000LL);
  CK(hipEventRecord(a, s));
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 1000000LL);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms_cal = 0.f;
  CK(hipEventElapsedTime(&ms_cal, a, b));
  const long long cycles = (long long)(1000000.0 * 0.15 / std::max(ms_cal, 1e-3f));
  const int grid_copy = 2048;
  for (int kernel = 0; kernel < 2; ++kernel) {
    for (int K : {1, 3}) {
      for (int mode = 0; mode < 8; ++mode) {
        std::vector<float> t;
        for (int it = 0; it < 60; ++it) {
          CK(hipEventRecord(ev_x, s2));  // long done by the time s reaches its wait
          hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, cycles);
          CK(hipEventRecord(a, s));
          for (int k = 0; k < K; ++k) {
            if (mode == XWAIT) CK(hipStreamWaitEvent(s, ev_x, 0));
            hipEvent_t stop = mode == EXT_NOTIME ? ev_nt : (mode == EXT_TIME || mode == EXT_BOTH) ? ev_t : nullptr;
            hipEvent_t start = (mode == EXT_START || mode == EXT_BOTH) ? ev_s : nullptr;
            if (kernel == 0) {
              if (stop || start) hipExtLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s, start, stop, 0, tiny);
              else hipLaunchKernelGGL(noop, dim3(1), dim3(64), 0, s, tiny);
            } else {
              if (stop || start)
                hipExtLaunchKernelGGL(copy4, dim3(grid_copy), dim3(256), 0, s, start, stop, 0, (const f4*)x,
                                      (f4*)y, n / 4);
              else
                hipLaunchKernelGGL(copy4, dim3(grid_copy), dim3(256), 0, s, (const f4*)x, (f4*)y, n / 4);
            }
            if (mode == REC_NOTIME) CK(hipEventRecord(ev_nt, s));
            if (mode == REC_TIME) CK(hipEventRecord(ev_t, s));
          }
          CK(hipEventRecord(b, s));
          CK(hipEventSynchronize(b));
          float ms = 0.f;
          CK(hipEventElapsedTime(&ms, a, b));
          if (it >= 10) t.push_back(ms * 1000.f);
        }
        std::sort(t.begin(), t.end());
        printf("{\"kernel\": \"%s\", \"chain\": %d, \"mode\": \"%s\", \"median_us\": %.2f, \"p10_us\": %.2f, "
               "\"p90_us\": %.2f}\n",
               kernel == 0 ? "noop_1wg" : "copy_12.8MB", K, kModeName[mode], t[t.size() / 2], t[t.size() / 10],
               t[t.size() * 9 / 10]);
        fflush(stdout);
      }
    }
  }
  return 0;
}
