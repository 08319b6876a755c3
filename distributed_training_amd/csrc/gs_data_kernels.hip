// gfx950 kernel of the input step: the whole uint8 image
// set stays resident in HBM ([N, H, W, C], CIFAR-10 train = 153.6 MB) and one
// launch per batch gathers the sampled images and applies Pad -> hflip ->
// crop -> ToTensor (x / 255) (+ bf16 cast), writing the training tensor in
// NCHW or NHWC, with the labels gathered alongside.  Replaces the reference's
// per-sample PIL transforms + default_collate + H2D copy
// (R:resnet/pytorch_ddp/ddp_train.py:25-48, 62-63).
//
// HBM-bound streaming: per sample C*oh*ow*(1 + 4) bytes (uint8 read, f32
// write).  Each lane produces 4 consecutive output elements and stores them
// with one 16-B (f32) / 8-B (bf16) access; the uint8 reads are byte gathers
// served from L2 (a sample's 3 KiB image is touched by 12 lanes at most per
// row).  The per-sample params (index, flip, top, left) arrive as one small
// device array.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gs_common.h"

namespace gs {
namespace {

#define HIP_RET(expr)                                                               \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    if (_e != hipSuccess)                                                           \
      return fail(GS_EHIP, std::string(#expr " failed: ") + hipGetErrorString(_e)); \
  } while (0)

typedef float gf4 __attribute__((ext_vector_type(4)));
typedef uint32_t gu2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint16_t to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7FC0;
  return static_cast<uint16_t>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

template <int LAYOUT>
__device__ __forceinline__ float elem(const ImageAugArgs& a, int64_t e, int64_t per) {
  const int64_t b = e / per;
  const int64_t k = e - b * per;
  int c, y, x;
  if constexpr (LAYOUT == GS_LAYOUT_NCHW) {
    x = static_cast<int>(k % a.out_w);
    y = static_cast<int>((k / a.out_w) % a.out_h);
    c = static_cast<int>(k / (static_cast<int64_t>(a.out_w) * a.out_h));
  } else {
    c = static_cast<int>(k % a.C);
    x = static_cast<int>((k / a.C) % a.out_w);
    y = static_cast<int>(k / (static_cast<int64_t>(a.C) * a.out_w));
  }
  const int4 p = reinterpret_cast<const int4*>(a.params)[b];
  if (p.x < 0 || p.x >= a.n_src) return 0.f;  // never read outside the image set
  return aug_pixel(a.src, p.x, a.H, a.W, a.C, a.pad, p.y, p.z, p.w, c, y, x);
}

template <int LAYOUT, int DT>
__global__ void __launch_bounds__(256) augment_kernel(ImageAugArgs a, int64_t total, bool vec) {
  const int64_t per = static_cast<int64_t>(a.C) * a.out_h * a.out_w;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  const int64_t gid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (a.out_labels && gid < a.B) {
    const int idx = reinterpret_cast<const int4*>(a.params)[gid].x;
    a.out_labels[gid] = (a.labels && idx >= 0 && idx < a.n_src) ? a.labels[idx] : 0;
  }
  for (int64_t q = gid; q * 4 < total; q += stride) {
    const int64_t e = q * 4;
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (e + i < total) ? elem<LAYOUT>(a, e + i, per) : 0.f;
    if constexpr (DT == GS_F32) {
      float* o = static_cast<float*>(a.out) + e;
      if (vec && e + 4 <= total) {
        gf4 w;
        w.x = v[0]; w.y = v[1]; w.z = v[2]; w.w = v[3];
        *reinterpret_cast<gf4*>(o) = w;
      } else {
        for (int i = 0; i < 4; ++i)
          if (e + i < total) o[i] = v[i];
      }
    } else {
      uint16_t* o = static_cast<uint16_t*>(a.out) + e;
      if (vec && e + 4 <= total) {
        gu2 w;
        w.x = static_cast<uint32_t>(to_bf16(v[0])) | (static_cast<uint32_t>(to_bf16(v[1])) << 16);
        w.y = static_cast<uint32_t>(to_bf16(v[2])) | (static_cast<uint32_t>(to_bf16(v[3])) << 16);
        *reinterpret_cast<gu2*>(o) = w;
      } else {
        for (int i = 0; i < 4; ++i)
          if (e + i < total) o[i] = to_bf16(v[i]);
      }
    }
  }
}

// One workgroup per sample (grid-stride over samples): the sample's uint8
// image is staged in LDS with coalesced 16-B loads, then every lane builds
// 4 consecutive output elements from LDS (32-bit index math only) and writes
// them with one 16-B / 8-B store.  Used when the image fits the LDS budget
// (CIFAR: 3 KiB); larger images take augment_kernel (L2-served gathers).
constexpr int kAugLdsBytes = 48 * 1024;

template <int LAYOUT, int DT>
__global__ void __launch_bounds__(256) augment_lds_kernel(ImageAugArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_img[];
  const int img_bytes = a.H * a.W * a.C;
  const int per = a.C * a.out_h * a.out_w;
  const int quads = per >> 2;  // per % 4 == 0 (host checks)
  const int wp = a.W + 2 * a.pad;
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    const int4 p = reinterpret_cast<const int4*>(a.params)[b];
    const bool ok = p.x >= 0 && p.x < a.n_src;
    if (threadIdx.x == 0 && a.out_labels) a.out_labels[b] = (ok && a.labels) ? a.labels[p.x] : 0;
    __syncthreads();  // previous sample's LDS reads are done
    if (ok) {
      const uint8_t* src = a.src + static_cast<int64_t>(p.x) * img_bytes;
      for (int o = threadIdx.x * 16; o < img_bytes; o += 256 * 16)
        *reinterpret_cast<uint4*>(s_img + o) = *reinterpret_cast<const uint4*>(src + o);
    }
    __syncthreads();
    for (int q = threadIdx.x; q < quads; q += 256) {
      const int k0 = q << 2;
      // (c, y, x) of the quad's first element, then step through the layout's order
      int c, y, x;
      if constexpr (LAYOUT == GS_LAYOUT_NCHW) {
        x = k0 % a.out_w;
        const int r = k0 / a.out_w;
        y = r % a.out_h;
        c = r / a.out_h;
      } else {
        c = k0 % a.C;
        const int pix = k0 / a.C;
        x = pix % a.out_w;
        y = pix / a.out_w;
      }
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int px = p.y ? (wp - 1 - (x + p.w)) : (x + p.w);
        const int sy = y + p.z - a.pad, sx = px - a.pad;
        v[i] = (ok && sy >= 0 && sy < a.H && sx >= 0 && sx < a.W)
                   ? static_cast<float>(s_img[(sy * a.W + sx) * a.C + c]) / 255.f
                   : 0.f;
        if constexpr (LAYOUT == GS_LAYOUT_NCHW) {
          if (++x == a.out_w) { x = 0; if (++y == a.out_h) { y = 0; ++c; } }
        } else {
          if (++c == a.C) { c = 0; if (++x == a.out_w) { x = 0; ++y; } }
        }
      }
      const int64_t e = b * per + k0;
      if constexpr (DT == GS_F32) {
        gf4 w;
        w.x = v[0]; w.y = v[1]; w.z = v[2]; w.w = v[3];
        *reinterpret_cast<gf4*>(static_cast<float*>(a.out) + e) = w;
      } else {
        gu2 w;
        w.x = static_cast<uint32_t>(to_bf16(v[0])) | (static_cast<uint32_t>(to_bf16(v[1])) << 16);
        w.y = static_cast<uint32_t>(to_bf16(v[2])) | (static_cast<uint32_t>(to_bf16(v[3])) << 16);
        *reinterpret_cast<gu2*>(static_cast<uint16_t*>(a.out) + e) = w;
      }
    }
  }
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) (void)hipSetDevice(dev);
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

int hip_image_augment(int device, const ImageAugArgs& a, void* stream) {
  DeviceGuard g(device);
  const int64_t total = a.B * a.C * a.out_h * a.out_w;
  const int64_t quads = (total + 3) / 4;
  const int blocks = static_cast<int>(std::max<int64_t>(
      (a.B + 255) / 256, std::min<int64_t>((quads + 255) / 256, 8192)));
  const bool vec = (reinterpret_cast<uintptr_t>(a.out) & 15u) == 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t img_bytes = static_cast<int64_t>(a.H) * a.W * a.C;
  const int64_t per = static_cast<int64_t>(a.C) * a.out_h * a.out_w;
  if (vec && img_bytes <= kAugLdsBytes && img_bytes % 16 == 0 && per % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(a.src) & 15u) == 0) {
    const int g2 = static_cast<int>(std::min<int64_t>(a.B, 65535));
    const size_t lds = static_cast<size_t>(img_bytes);
    if (a.layout == GS_LAYOUT_NCHW) {
      if (a.out_dtype == GS_F32)
        hipLaunchKernelGGL((augment_lds_kernel<GS_LAYOUT_NCHW, GS_F32>), dim3(g2), dim3(256), lds, s, a);
      else
        hipLaunchKernelGGL((augment_lds_kernel<GS_LAYOUT_NCHW, GS_BF16>), dim3(g2), dim3(256), lds, s, a);
    } else {
      if (a.out_dtype == GS_F32)
        hipLaunchKernelGGL((augment_lds_kernel<GS_LAYOUT_NHWC, GS_F32>), dim3(g2), dim3(256), lds, s, a);
      else
        hipLaunchKernelGGL((augment_lds_kernel<GS_LAYOUT_NHWC, GS_BF16>), dim3(g2), dim3(256), lds, s, a);
    }
    HIP_RET(hipGetLastError());
    return GS_OK;
  }
  if (a.layout == GS_LAYOUT_NCHW) {
    if (a.out_dtype == GS_F32)
      hipLaunchKernelGGL((augment_kernel<GS_LAYOUT_NCHW, GS_F32>), dim3(blocks), dim3(256), 0, s, a, total, vec);
    else
      hipLaunchKernelGGL((augment_kernel<GS_LAYOUT_NCHW, GS_BF16>), dim3(blocks), dim3(256), 0, s, a, total, vec);
  } else {
    if (a.out_dtype == GS_F32)
      hipLaunchKernelGGL((augment_kernel<GS_LAYOUT_NHWC, GS_F32>), dim3(blocks), dim3(256), 0, s, a, total, vec);
    else
      hipLaunchKernelGGL((augment_kernel<GS_LAYOUT_NHWC, GS_BF16>), dim3(blocks), dim3(256), 0, s, a, total, vec);
  }
  HIP_RET(hipGetLastError());
  return GS_OK;
}

}  // namespace gs
