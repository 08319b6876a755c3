// The gfx950 streaming engine of libgsync, shared by the kernel translation units
// (gs_kernels.hip: pack / unpack / reductions / plan memory; gs_update_kernels.hip:
// the fused SGD / Adam updates — two TUs so hipcc compiles them in parallel).
// Device code: include from .hip sources only.
//
// All of them are HBM-streaming kernels (no MFMA: nothing here is a
// contraction).  One engine serves every op (chunk_kernel): a plan lays its
// tensors end to end in a virtual element space cut into 1 Ki-element chunks;
// a 256-thread workgroup (4 wave64) takes G consecutive chunks per iteration
// and grid-strides.  A group inside one tensor streams from a wave-uniform
// (SGPR) base with G 16-B (fp32) / 8-B (16-bit) accesses per lane in flight;
// chunks where tensors meet (tensor tails, runs of BN weights / biases) stage
// the span's descriptors in LDS and resolve each lane's tensor there.
//
// Arithmetic is written with explicit fmaf and compiled with
// -ffp-contract=off so that the host restatement (oracle/gs_oracle.c) and
// the host backend (gs_host.cpp) reproduce it bit for bit.

#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "gs_common.h"

namespace gs {

namespace {

#define HIP_RET(expr)                                                                 \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      return fail(GS_EHIP, std::string(#expr " failed: ") + hipGetErrorString(_e));   \
  } while (0)

// ---------------------------------------------------------------- dtype I/O
__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}
// round-to-nearest-even; NaN -> 0x7FC0 (c10::BFloat16 round_to_nearest_even)
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7FC0;
  return static_cast<uint16_t>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float f16_to_f32(uint16_t h) {
  _Float16 x;
  __builtin_memcpy(&x, &h, 2);
  return static_cast<float>(x);
}
// fp32 -> fp16, round-to-nearest-even of the fp32 VALUE (torch: opmath in fp32,
// then the cast).  The empty asm pins f as an fp32 register value: without it
// LLVM folds the producing fma / mul into v_fma_mixlo_f16, which rounds the
// exact result once, straight to fp16 — a different fp16 wherever the fp32
// rounding lands on an fp16 tie (ZeRO fp16 params, fp16 buckets, fp16 unscale;
// found as master.half() != the fp16 param in test_colossal_low_level_zero_fp16_gpu)
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
  __asm__("" : "+v"(f));
  _Float16 x = static_cast<_Float16>(f);
  uint16_t h;
  __builtin_memcpy(&h, &x, 2);
  return h;
}

template <int DT>
__device__ __forceinline__ float to_f32(uint16_t h) {
  if constexpr (DT == GS_BF16) return bf16_to_f32(h);
  else return f16_to_f32(h);
}
template <int DT>
__device__ __forceinline__ uint16_t from_f32(float f) {
  if constexpr (DT == GS_BF16) return f32_to_bf16(f);
  else return f32_to_f16(f);
}
// value as it would read back after a store in DT (used for norms / casts)
template <int DT>
__device__ __forceinline__ float round_to(float f) {
  if constexpr (DT == GS_F32) return f;
  else return to_f32<DT>(from_f32<DT>(f));
}

// Plan pointers are read from a table, so the compiler only sees generic
// pointers and would emit flat_* accesses; every buffer here is device
// global memory, so accesses go through address_space(1) (global_*) with
// native 16-B / 8-B vector types.
typedef float gf4 __attribute__((ext_vector_type(4)));
typedef uint32_t gu2 __attribute__((ext_vector_type(2)));
typedef uint32_t gu4 __attribute__((ext_vector_type(4)));
#define GLOBAL_AS __attribute__((address_space(1)))

template <class T>
__device__ __forceinline__ const GLOBAL_AS T* gptr(const void* p) {
  return (const GLOBAL_AS T*)(p);
}
template <class T>
__device__ __forceinline__ GLOBAL_AS T* gptr_w(void* p) {
  return (GLOBAL_AS T*)(p);
}

// Load / store policy (measured)
// * The update's read-once gradient stream takes non-temporal loads unless a Σg²
//   pass of the plan read it just before and it fits the Infinity Cache (in-step
//   ResNet-50 SGD 0.786 -> 0.805-0.816 of 8 TB/s; beyond the cache 0.709 -> 0.729;
//   the clip path's update right behind its Σg² 0.770 -> 0.740 with NT loads:
//   profiles/r4/r4c_nt_instep.jsonl).  The parameter / optimizer-state streams keep
//   cached loads: NT there cost every in-step configuration measured (ResNet-50 SGD
//   0.79 -> 0.70, Adam 0.82 -> 0.73, ResNet-152 SGD 0.83 -> 0.74, r4e_nt_state.jsonl).
// * Every store is non-temporal (written once, read by another kernel much later).
constexpr int64_t kInfinityCacheBytes = 256ll << 20;

// A stream read once takes non-temporal loads when it is larger than the
// Infinity Cache: none of it can still be resident from its producer, and the NT
// path streams faster (a plain read-only float4 sum beyond the cache: 0.84-0.87
// of 8 TB/s NT vs 0.72-0.76 cached, scripts/micro/stream_mix.hip,
// profiles/r4/r4p_stream_mix_*.jsonl).  At or below the cache size the pack's
// source and the unpack's flat buffer stay cached: NT cost them 5-16 % there
// (r4r).  The Σg² kernels follow the same size rule.  Below the cache size the
// better choice depends on the producer: right after libgsync's unpack wrote the
// grads with non-temporal stores, NT Σg² loads ran the clip path 0.72 -> 0.80 at
// ResNet-50 (profiles/r4/r4s_chain.jsonl); inside configs[3]'s real ZeRO step,
// after RCCL wrote the shard, they cost 10 % (12.9 -> 14.2 us, r4v), and on the
// bench's resident grads 2-5 % (r4u).  The DDP clip chain has a better answer
// than NT loads, the Σg² folded into the unpack (fuse_grad_norm_into).
// GS_NT_READ_ONCE / GS_NT_SQNORM (environment): 0 never, 1 always, 2 the size rule
// (default) — tests/test_clip_fold.py checks that no policy changes a bit.
// hint (gs_plan_set_read_hint, Σg² only): 1 non-temporal, 2 cached, 0 the size
// rule; an explicit environment policy wins over it
inline bool nt_read_once(int64_t stream_bytes, bool sqnorm = false, int hint = 0) {
  static const int policy = [] {
    const char* e = std::getenv("GS_NT_READ_ONCE");
    return e ? std::atoi(e) : 2;
  }();
  static const int policy_sq = [] {
    const char* e = std::getenv("GS_NT_SQNORM");
    return e ? std::atoi(e) : 2;
  }();
  const int pol = sqnorm ? policy_sq : policy;
  if (pol != 2) return pol != 0;
  if (hint == 1 || hint == 2) return hint == 1;
  return stream_bytes > kInfinityCacheBytes;
}
inline int dtype_bytes(int dt) { return dt == GS_F32 ? 4 : 2; }
// in-kernel combine of chunk-engine reductions (two-level ticket over R groups)
// instead of the combine_partials launch (0); GS_RED_FUSE=<R> in the environment
// overrides (tests/test_clip_fold.py).  A single-counter ticket measured slower
// than the launch (r2c).
#ifndef GS_RED_FUSE
#define GS_RED_FUSE 64
#endif
#ifndef GS_RED_FUSE_GRID
#define GS_RED_FUSE_GRID 2048  // workgroups of a fused reduction (r2z2 sweep: 2048 < 4096 < 8192)
#endif
constexpr int kRedSyncWords = (2 * kRedMaxGroups + 1) * kRedSyncStride;
constexpr int kRedFuseMaxGrid = 8192;  // above this a group's counter sees too many arrivals
// chunks per workgroup iteration (chunk-map engine), per op: profiles/r2*_kernels_*.jsonl,
// r3d (fp32 -> 16-bit pack: 8 > 2 = 4 > 1), r4k (ZeRO's bf16 -> bf16 pack: 4 > 2 > 8 > 1)
#ifndef GS_G_PACK
#define GS_G_PACK 1     // fp32 bucket
#endif
#ifndef GS_G_PACK16
#define GS_G_PACK16 8   // fp32 grads -> 16-bit bucket
#endif
#ifndef GS_G_PACK16_16
#define GS_G_PACK16_16 4  // 16-bit grads -> 16-bit bucket, ZeRO's bf16 pack
#endif
#ifndef GS_G_UNPACK
#define GS_G_UNPACK 2
#endif
#ifndef GS_G_RED
#define GS_G_RED 2
#endif
#ifndef GS_G_SGD
#define GS_G_SGD 2
#endif
#ifndef GS_G_ADAM
#define GS_G_ADAM 4
#endif
// 256-thread workgroups are admitted 8 per CU only while the kernel uses <= 80
// SGPRs (MI355X_MICROARCH.md, residency); cap the allocation there
#define GS_SGPR_ATTR __attribute__((amdgpu_num_sgpr(80)))

template <bool NT = false, class V>
__device__ __forceinline__ V vload(const GLOBAL_AS V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <class V>
__device__ __forceinline__ void vstore(GLOBAL_AS V* p, V v) {
  __builtin_nontemporal_store(v, p);
}

// load N (4 or 8) consecutive elements [e, e+N) of a tensor with n elements;
// e is a multiple of N.  fp32: N/4 16-B loads; 16-bit: one 8-B (N=4) or
// 16-B (N=8) load.  `vec`: the tensor base is 16-B aligned.
template <int DT, int N, bool NT = false>
__device__ __forceinline__ void loadN(const void* base, int64_t e, int64_t n, bool vec,
                                      float (&x)[N]) {
  static_assert(N == 4 || N == 8, "4 or 8 elements per lane");
  if constexpr (DT == GS_F32) {
    const GLOBAL_AS float* p = gptr<float>(base) + e;
    if (vec && e + N <= n) {
#pragma unroll
      for (int h = 0; h < N / 4; ++h) {
        const gf4 v = vload<NT>((const GLOBAL_AS gf4*)(p + 4 * h));
        x[4 * h + 0] = v.x; x[4 * h + 1] = v.y; x[4 * h + 2] = v.z; x[4 * h + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) x[i] = (e + i < n) ? p[i] : 0.f;
    }
  } else {
    const GLOBAL_AS uint16_t* p = gptr<uint16_t>(base) + e;
    if (vec && e + N <= n) {
      uint32_t w[N / 2];
      if constexpr (N == 8) {
        const gu4 v = vload<NT>((const GLOBAL_AS gu4*)p);
        w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
      } else {
        const gu2 v = vload<NT>((const GLOBAL_AS gu2*)p);
        w[0] = v.x; w[1] = v.y;
      }
#pragma unroll
      for (int k = 0; k < N / 2; ++k) {
        x[2 * k] = to_f32<DT>(static_cast<uint16_t>(w[k] & 0xffffu));
        x[2 * k + 1] = to_f32<DT>(static_cast<uint16_t>(w[k] >> 16));
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) x[i] = (e + i < n) ? to_f32<DT>(p[i]) : 0.f;
    }
  }
}

template <int DT, int N>
__device__ __forceinline__ void storeN(void* base, int64_t e, int64_t n, bool vec,
                                       const float (&x)[N]) {
  static_assert(N == 4 || N == 8, "4 or 8 elements per lane");
  if constexpr (DT == GS_F32) {
    GLOBAL_AS float* p = gptr_w<float>(base) + e;
    if (vec && e + N <= n) {
#pragma unroll
      for (int h = 0; h < N / 4; ++h) {
        gf4 v;
        v.x = x[4 * h + 0]; v.y = x[4 * h + 1]; v.z = x[4 * h + 2]; v.w = x[4 * h + 3];
        vstore((GLOBAL_AS gf4*)(p + 4 * h), v);
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (e + i < n) p[i] = x[i];
    }
  } else {
    GLOBAL_AS uint16_t* p = gptr_w<uint16_t>(base) + e;
    if (vec && e + N <= n) {
      uint32_t w[N / 2];
#pragma unroll
      for (int k = 0; k < N / 2; ++k)
        w[k] = static_cast<uint32_t>(from_f32<DT>(x[2 * k])) |
               (static_cast<uint32_t>(from_f32<DT>(x[2 * k + 1])) << 16);
      if constexpr (N == 8) {
        gu4 v;
        v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3];
        vstore((GLOBAL_AS gu4*)p, v);
      } else {
        gu2 v;
        v.x = w[0]; v.y = w[1];
        vstore((GLOBAL_AS gu2*)p, v);
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (e + i < n) p[i] = from_f32<DT>(x[i]);
    }
  }
}

// Full-chunk access of the chunk-map engine: `base` is wave-uniform (SGPRs),
// e0 the uniform element index of the chunk inside the tensor and `lo` the
// lane's 32-bit element offset; everything is in range and 16-B aligned, so
// the access is one global_load/store with an SGPR base and a VGPR offset.
template <int DT>
__device__ __forceinline__ const void* elem_at(const void* base, int64_t e0) {
  return static_cast<const char*>(base) + e0 * (DT == GS_F32 ? 4 : 2);
}
template <int DT, bool NT = false>
__device__ __forceinline__ void load4F(const void* base, uint32_t lo, float (&x)[4]) {
  if constexpr (DT == GS_F32) {
    const gf4 v = vload<NT>((const GLOBAL_AS gf4*)(gptr<float>(base) + lo));
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  } else {
    const gu2 v = vload<NT>((const GLOBAL_AS gu2*)(gptr<uint16_t>(base) + lo));
    x[0] = to_f32<DT>(static_cast<uint16_t>(v.x & 0xffffu));
    x[1] = to_f32<DT>(static_cast<uint16_t>(v.x >> 16));
    x[2] = to_f32<DT>(static_cast<uint16_t>(v.y & 0xffffu));
    x[3] = to_f32<DT>(static_cast<uint16_t>(v.y >> 16));
  }
}
template <int DT>
__device__ __forceinline__ void store4F(void* base, uint32_t lo, const float (&x)[4]) {
  if constexpr (DT == GS_F32) {
    gf4 v;
    v.x = x[0]; v.y = x[1]; v.z = x[2]; v.w = x[3];
    vstore((GLOBAL_AS gf4*)(gptr_w<float>(base) + lo), v);
  } else {
    gu2 v;
    v.x = static_cast<uint32_t>(from_f32<DT>(x[0])) | (static_cast<uint32_t>(from_f32<DT>(x[1])) << 16);
    v.y = static_cast<uint32_t>(from_f32<DT>(x[2])) | (static_cast<uint32_t>(from_f32<DT>(x[3])) << 16);
    vstore((GLOBAL_AS gu2*)(gptr_w<uint16_t>(base) + lo), v);
  }
}
// F = full-chunk fast path (above); otherwise element e0 + lo of a tensor of
// n elements with the bounds / alignment checks of loadN / storeN
template <int DT, int N, bool F, bool NT = false>
__device__ __forceinline__ void ld(const void* base, int64_t e0, uint32_t lo, int64_t n, bool vec,
                                   float (&x)[N]) {
  if constexpr (F) {
    static_assert(N == 4, "the chunk engine moves 4 elements per lane-access");
    load4F<DT, NT>(elem_at<DT>(base, e0), lo, x);
  } else {
    loadN<DT, N, NT>(base, e0 + lo, n, vec, x);
  }
}
template <int DT, int N, bool F>
__device__ __forceinline__ void st(void* base, int64_t e0, uint32_t lo, int64_t n, bool vec,
                                   const float (&x)[N]) {
  if constexpr (F) {
    static_assert(N == 4, "the chunk engine moves 4 elements per lane-access");
    store4F<DT>(const_cast<void*>(elem_at<DT>(base, e0)), lo, x);
  } else {
    storeN<DT, N>(base, e0 + lo, n, vec, x);
  }
}

__device__ __forceinline__ void* slot_ptr(const PlanArgs& P, int slot, int t) {
  return P.ptrs[static_cast<int64_t>(slot) * P.n + t];
}
__device__ __forceinline__ bool slot_vec(const PlanArgs& P, int slot, int t) {
  return (P.align[t] >> slot) & 1u;
}

// ------------------------------------------------------- wave/block reduce
// DPP wave reduction (GFX9 DPP, all in VALU — no LDS crossbar): quad swaps,
// half-row and row mirrors give every lane its row-of-16 total, row_bcast:15
// folds rows 0->1 and 2->3, row_bcast:31 folds row 1 into rows 2-3, so lane
// 63 holds the wave total; v_readlane broadcasts it.  A fixed tree:
// deterministic.  Lanes of rows a DPP op does not write keep `id`.
template <int Ctrl, int RowMask, bool MAX>
__device__ __forceinline__ float dpp_op(float v, float id) {
  const int s = __builtin_amdgcn_update_dpp(__float_as_int(id), __float_as_int(v), Ctrl, RowMask, 0xF, false);
  const float t = __int_as_float(s);
  return MAX ? fmaxf(v, t) : v + t;
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce(float v) {
  const float id = MAX ? -INFINITY : 0.f;
  v = dpp_op<0xB1, 0xF, MAX>(v, id);   // quad_perm [1,0,3,2]
  v = dpp_op<0x4E, 0xF, MAX>(v, id);   // quad_perm [2,3,0,1]
  v = dpp_op<0x141, 0xF, MAX>(v, id);  // row_half_mirror
  v = dpp_op<0x140, 0xF, MAX>(v, id);  // row_mirror
  v = dpp_op<0x142, 0xA, MAX>(v, id);  // row_bcast:15 into rows 1, 3
  v = dpp_op<0x143, 0xC, MAX>(v, id);  // row_bcast:31 into rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
__device__ __forceinline__ float wave_sum(float v) { return wave_reduce<false>(v); }
__device__ __forceinline__ float wave_max(float v) { return wave_reduce<true>(v); }
// block of kBlock threads; result valid in thread 0
template <bool MAX>
__device__ __forceinline__ float block_reduce(float v) {
  __shared__ float s_red[kBlock / 64];
  v = MAX ? wave_max(v) : wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) s_red[w] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0) {
    r = s_red[0];
#pragma unroll
    for (int i = 1; i < kBlock / 64; ++i) r = MAX ? fmaxf(r, s_red[i]) : r + s_red[i];
  }
  __syncthreads();
  return r;
}

// ------------------------------------------------------------- the engine
// Everything a unit needs about its tensor, staged once per task in LDS
// (one entry per segment of the task) instead of re-read from the global
// tables for every unit.
struct TV {
  void* ptr[GS_PLAN_SLOTS];
  int64_t numel;
  int64_t off;
  uint32_t align;
  int32_t pad;
  __device__ __forceinline__ bool vec(int slot) const { return (align >> slot) & 1u; }
};

// Op contract:
//   struct Frag;                             registers for one unit (4 elements)
//   load_hyper(Op&) overload (optional)      step-varying hyper-parameters from device memory
//   bool active() const;                     uniform early-out (found_inf skip)
//   void load(const TV&, e, Frag&)           issue the unit's loads
//   void apply(const TV&, e, Frag&, acc)     compute + store (+ reduction)
//   static constexpr int kRed = 0 (none) | 1 (sum) | 2 (max); float* partials
//   static constexpr int kKind = GS_OP_* (tags the launch timer's records)
// default: hyper-parameters travel in the kernel arguments
template <class Op>
__device__ __forceinline__ void load_hyper(Op&) {}

// The plan tables are read-only for the whole launch: reading them through
// the constant address space lets the uniform descriptor loads of a
// single-segment task go to the scalar unit (s_load), with no LDS round trip
// and no barrier before the first data load.
#define CONST_AS __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ T cload(const T* p, int64_t i) {
  return ((const CONST_AS T*)(p))[i];
}

// Descriptor of tensor t as `op` addresses it: logical slot k is table row
// op.phys(k), so single-stream ops read their runtime slot as the constant
// logical slot 0.  (A runtime index into TV::ptr made the compiler spill the
// descriptor to scratch and reload the stream pointer into VGPRs, turning
// every access into per-lane 64-bit addressing.)  SCALAR: wave-uniform t,
// loaded through the constant address space (s_load).
template <bool SCALAR, class Op>
__device__ __forceinline__ TV load_tv(const Op& op, const PlanArgs& P, int t) {
  TV v;
  const uint32_t a = SCALAR ? cload(P.align, t) : P.align[t];
  uint32_t bits = 0;
#pragma unroll
  for (int s = 0; s < GS_PLAN_SLOTS; ++s) {
    const int64_t r = static_cast<int64_t>(op.phys(s)) * P.n + t;
    v.ptr[s] = SCALAR ? cload(P.ptrs, r) : P.ptrs[r];
    bits |= ((a >> op.phys(s)) & 1u) << s;
  }
  v.align = bits;
  v.numel = SCALAR ? cload(P.numel, t) : P.numel[t];
  v.off = SCALAR ? cload(P.off, t) : P.off[t];
  v.pad = 0;
  return v;
}

// deterministic combine of the per-workgroup partials (fixed order): 1024
// threads, thread t folds the float4s t, t+1024, ... (8 16-B loads issued
// before the first add: up to 32 Ki partials — the uncapped unpack + Σg² grid
// of a ResNet-50 — in one round trip), the < 4 trailing partials go to threads
// 0-2, then a fixed-tree block reduction
constexpr int kCombineBlock = 1024;
template <bool MAX>
__global__ void __launch_bounds__(kCombineBlock) combine_partials(const float* partials, int n,
                                                                  float* out, int accumulate) {
  __shared__ float s_red[kCombineBlock / 64];
  float v = 0.f;
  const int n4 = n >> 2;
  const float4* p4 = reinterpret_cast<const float4*>(partials);  // hipMalloc'd: 16-B aligned
  for (int i = threadIdx.x; i < n4; i += 8 * kCombineBlock) {
    float4 x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      x[u] = (i + u * kCombineBlock < n4) ? p4[i + u * kCombineBlock] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (i + u * kCombineBlock < n4) {
        v = MAX ? fmaxf(v, x[u].x) : v + x[u].x;
        v = MAX ? fmaxf(v, x[u].y) : v + x[u].y;
        v = MAX ? fmaxf(v, x[u].z) : v + x[u].z;
        v = MAX ? fmaxf(v, x[u].w) : v + x[u].w;
      }
    }
  }
  if (static_cast<int>(threadIdx.x) < (n & 3)) {
    const float x = partials[4 * n4 + threadIdx.x];
    v = MAX ? fmaxf(v, x) : v + x;
  }
  v = MAX ? wave_max(v) : wave_sum(v);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = s_red[0];
#pragma unroll
    for (int w = 1; w < kCombineBlock / 64; ++w) r = MAX ? fmaxf(r, s_red[w]) : r + s_red[w];
    if (MAX) out[0] = accumulate ? fmaxf(out[0], r) : r;
    else out[0] = accumulate ? out[0] + r : r;
  }
}

// ------------------------------------------------------- chunk-map engine
// (layout: gs_common.h).  A workgroup takes G consecutive 1 Ki-element chunks
// per iteration and grid-strides.  A group wholly inside one tensor whose
// streams are all 16-B aligned runs the op's F = true path: the descriptor
// comes through scalar loads and every lane issues G 16-B accesses per stream
// (SGPR base + 32-bit VGPR offset) before the first use, with no bounds or
// alignment branches.  Other groups go chunk by chunk: a full chunk the same
// way with one access per lane, a mixed chunk (tensor tails, runs of small
// tensors) by a per-lane binary search over voff and the checked path.
// Reductions write one partial per workgroup; the grid is capped for them so
// that the combine reads few partials (combine_partials, fixed order).
template <class Op>
__device__ __forceinline__ void chunk_mixed(const Op& op, const PlanArgs& P, int t0, int span, int64_t c,
                                            float& acc) {
  const int64_t e = c * kChunkElems + static_cast<int>(threadIdx.x) * kUnit;
  int lo = t0, hi = t0 + span - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (P.voff[mid] <= e) lo = mid; else hi = mid - 1;
  }
  const int64_t local = e - P.voff[lo];
  if (local < 0 || local >= P.numel[lo]) return;  // alignment gap between tensors
  const TV v = load_tv<false>(op, P, lo);
  typename Op::Frag f;
  op.template load<false>(v, local, 0u, f);
  op.template apply<false>(v, local, 0u, f, acc);
}

// The same with the span's descriptors staged in LDS (the north star's "LDS
// staging for small-tensor gather"): the first `span` lanes each load one
// tensor's extent [voff, voff + numel) and its descriptor (stream pointers,
// alignment bits) into LDS, then every lane binary-searches LDS instead of
// chasing log2(span) dependent global loads and reads its tensor's descriptor
// from LDS instead of gathering it.  Runs of small tensors (BN weights /
// biases, tensor tails) are the chunks this serves; spans above kMixedStage
// (runs of tiny or empty tensors) keep the global path.  The caller's branch
// is uniform across the workgroup (the chunk's code), so the barriers are too.
// Measured: profiles/r2mlds/ (tiny tensors pack -15 %, R50 neutral).
constexpr int kMixedStage = 64;  // tensors per mixed chunk staged (5 KB of LDS)
template <class Op>
__device__ __forceinline__ void chunk_mixed_lds(const Op& op, const PlanArgs& P, int t0, int span, int64_t c,
                                                float& acc, int64_t* s_lo, int64_t* s_hi, TV* s_tv) {
  __syncthreads();  // the previous mixed chunk's lanes are done with the stage
  if (static_cast<int>(threadIdx.x) < span) {
    const int t = t0 + static_cast<int>(threadIdx.x);
    const TV d = load_tv<false>(op, P, t);
    s_lo[threadIdx.x] = P.voff[t];
    s_hi[threadIdx.x] = P.voff[t] + d.numel;
    s_tv[threadIdx.x] = d;
  }
  __syncthreads();
  const int64_t e = c * kChunkElems + static_cast<int>(threadIdx.x) * kUnit;
  int lo = 0, hi = span - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s_lo[mid] <= e) lo = mid; else hi = mid - 1;
  }
  const int64_t local = e - s_lo[lo];
  if (local < 0 || e >= s_hi[lo]) return;  // alignment gap between tensors
  const TV v = s_tv[lo];
  typename Op::Frag f;
  op.template load<false>(v, local, 0u, f);
  op.template apply<false>(v, local, 0u, f, acc);
}

template <int G, class Op>
__device__ __forceinline__ void chunk_full(const Op& op, const PlanArgs& P, int t, int64_t c0, float& acc) {
  // G chunks c0 .. c0+G-1, all inside tensor t
  const TV v = load_tv<true>(op, P, t);
  const int64_t e0 = c0 * kChunkElems - cload(P.voff, t);
  const uint32_t tid = threadIdx.x;
  typename Op::Frag f[G];
  if (op.fast_ok(v)) {
#pragma unroll
    for (int j = 0; j < G; ++j) op.template load<true>(v, e0, j * kChunkElems + tid * kUnit, f[j]);
#pragma unroll
    for (int j = 0; j < G; ++j) op.template apply<true>(v, e0, j * kChunkElems + tid * kUnit, f[j], acc);
  } else {
    // a stream is not 16-B aligned: the checked path over the same range
#pragma unroll
    for (int j = 0; j < G; ++j) op.template load<false>(v, e0 + j * kChunkElems + tid * kUnit, 0u, f[j]);
#pragma unroll
    for (int j = 0; j < G; ++j) op.template apply<false>(v, e0 + j * kChunkElems + tid * kUnit, 0u, f[j], acc);
  }
}

template <class Op>
__global__ void __launch_bounds__(kBlock) GS_SGPR_ATTR chunk_kernel(PlanArgs P, Op op) {
  static_assert(Op::kN == kUnit, "the chunk engine moves 4 elements per lane-access");
  constexpr int G = Op::kG;
  static_assert(G == 1 || G == 2 || G == 4 || G == 8, "group of 1, 2, 4 or 8 chunks");
  float acc = 0.f;
  load_hyper(op);            // uniform: graph-replayable lr / bias corrections, clip coefficient
  if (!op.active()) return;  // uniform across the grid
  __shared__ int64_t s_lo[kMixedStage], s_hi[kMixedStage];  // mixed chunks: the span's extents
  __shared__ TV s_tv[kMixedStage];                            // ... and descriptors
  const int64_t n_groups = (static_cast<int64_t>(P.n_chunks) + G - 1) / G;
  const int* cw = &P.chunks[0].t0;  // [t0, code] pairs
  for (int64_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
    const int64_t c0 = g * G;
    const int t = cload(cw, 2 * c0);
    const int code = cload(cw, 2 * c0 + 1);
    if constexpr (G > 1) {
      // the whole group inside one tensor: first and last chunk full in t
      if (code == 0 && c0 + G <= P.n_chunks && cload(cw, 2 * (c0 + G - 1)) == t &&
          cload(cw, 2 * (c0 + G - 1) + 1) == 0) {
        chunk_full<G>(op, P, t, c0, acc);
        continue;
      }
    }
    for (int j = 0; j < G; ++j) {
      const int64_t c = c0 + j;
      if (c >= P.n_chunks) break;
      const int tj = j == 0 ? t : cload(cw, 2 * c);
      const int cj = j == 0 ? code : cload(cw, 2 * c + 1);
      if (cj == 0) chunk_full<1>(op, P, tj, c, acc);
      else if (cj > 0 && cj <= kMixedStage) chunk_mixed_lds(op, P, tj, cj, c, acc, s_lo, s_hi, s_tv);
      else if (cj > 0) chunk_mixed(op, P, tj, cj, c, acc);
    }
  }
  if constexpr (Op::kRed != 0) {
    constexpr bool MAX = Op::kRed == 2;
    const float r = block_reduce<MAX>(acc);
    if (!P.red_fuse) {
      // raw (gs_sqnorm_partial_out on a small plan): the partial goes straight to the
      // caller's buffer, stream-ordered for its consumer; else to the combine's input
      if (threadIdx.x == 0) (P.red_raw ? P.red_out : op.partials)[blockIdx.x] = r;
      // ... and workgroup 0 zeroes the buffer's slots past the grid: a sharded caller
      // sums the whole buffer across ranks whose partial counts may differ
      if (P.red_raw && blockIdx.x == 0)
        for (int i = static_cast<int>(gridDim.x + threadIdx.x); i < GS_RED_PARTIALS; i += kBlock) P.red_out[i] = 0.f;
      return;
    }
    // In-kernel combine, two-level ticket.  Workgroup b belongs to group
    // b mod R (R = P.red_fuse, a power of two <= kRedMaxGroups; with R a
    // multiple of 8 a group's workgroups share the round-robin XCD of their
    // dispatch: speed only, nothing assumes it).  Each group has its own
    // arrival counter on its own 128-B line, so no device-scope word sees
    // more than grid/R arrivals (one word serialises them at ~12 ns each —
    // MI355X_MICROARCH.md "fanin"; the single-counter form measured 2.4 TB/s,
    // r2c).  The partial goes out write-through (agent-scope store), the
    // storing wave drains it (vmcnt(0)), then arrives; the group's last
    // arriver folds the group's partials (agent-scope loads) in block order,
    // publishes the group sum the same way and arrives on the top counter;
    // the last group folds the R group sums in group order.  Every counter is
    // re-armed by its last arriver.  The result depends only on the grid and
    // R, not on arrival order: deterministic, so ranks reducing identical
    // grads agree bit for bit.  Hand-off form: MI355X_MICROARCH.md's table,
    // row 1 (sc1 stores, vmcnt(0), atomic add, sc1 loads), no fences.
    constexpr int kStride = kRedSyncStride;
    __shared__ int s_role;  // 0: done, 1: group leader, 2: also the last group
    const int R = P.red_fuse;
    const int k = static_cast<int>(blockIdx.x) & (R - 1);
    const int grid = static_cast<int>(gridDim.x);
    const int n_groups = grid < R ? grid : R;
    uint32_t* top = &P.ticket[kRedMaxGroups * kStride];
    float* gsums = reinterpret_cast<float*>(P.ticket + (kRedMaxGroups + 1) * kStride);
    // gs_sqnorm_partial_out: the caller's slots past the group count read 0 (as in the raw form)
    if (P.red_groups_only && P.red_out && blockIdx.x == 0)
      for (int i = n_groups + static_cast<int>(threadIdx.x); i < GS_RED_PARTIALS; i += kBlock) P.red_out[i] = 0.f;
    if (threadIdx.x == 0) {
      const uint32_t ng = static_cast<uint32_t>((grid - 1 - k) / R + 1);
      __hip_atomic_store(&op.partials[blockIdx.x], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t tk = __hip_atomic_fetch_add(&P.ticket[k * kStride], 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
      s_role = tk == ng - 1;
    }
    __syncthreads();
    if (!s_role) return;  // uniform within the workgroup
    float v = 0.f;
    for (int i = k + R * static_cast<int>(threadIdx.x); i < grid; i += R * kBlock) {
      const float x = __hip_atomic_load(&op.partials[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v = MAX ? fmaxf(v, x) : v + x;
    }
    const float gsum = block_reduce<MAX>(v);
    if (threadIdx.x == 0) {
      __hip_atomic_store(&P.ticket[k * kStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gsums[k * kStride], gsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (P.red_groups_only) {
        // gs_sqnorm_partial: the group sums are the result; the clipped update
        // on this plan folds them (clip_multiplier), no top-level hand-off.
        // gs_sqnorm_partial_out: also contiguous in caller memory (a stream-
        // ordered consumer: the ranks' all-reduce, then the update)
        if (P.red_out) P.red_out[k] = gsum;
        s_role = 0;
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t tk = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_role = tk == static_cast<uint32_t>(n_groups) - 1 ? 2 : 0;
      }
    }
    __syncthreads();
    if (s_role != 2 || threadIdx.x >= 64) return;
    // the last group: wave 0 folds the group sums (lane j: group j, j + 64, ...)
    float t = 0.f;
    for (int j = static_cast<int>(threadIdx.x); j < n_groups; j += 64) {
      const float x = __hip_atomic_load(&gsums[j * kStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t = MAX ? fmaxf(t, x) : t + x;
    }
    const float tot = MAX ? wave_max(t) : wave_sum(t);
    if (threadIdx.x == 0) {
      float* out = P.red_out;
      if (MAX) out[0] = P.red_acc ? fmaxf(out[0], tot) : tot;
      else out[0] = P.red_acc ? out[0] + tot : tot;
      __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// reductions: at most Op::kRedGrid workgroups (= partials for the combine:
// 8 Ki for the read-only Σg² / inf checks, uncapped for the unpack that
// carries a fused Σg²; profiles/r2e_red.jsonl); GS_RED_GRID in the environment
// overrides (tests/test_clip_fold.py: the folded clip stays bit-identical)
int red_grid_cap(int op_default) {
  static const int v = [] {
    const char* e = std::getenv("GS_RED_GRID");
    return e ? std::max(1, std::min(std::atoi(e), kGridLimit)) : 0;
  }();
  return v > 0 ? v : op_default;
}
// in-kernel combine groups (0 = the combine_partials launch); GS_RED_FUSE=<R>
int red_fuse_groups() {
  static const int v = [] {
    const char* e = std::getenv("GS_RED_FUSE");
    int r = e ? std::atoi(e) : GS_RED_FUSE;
    if (r <= 0) return 0;
    int p2 = 1;
    while (p2 < r && p2 < kRedMaxGroups) p2 <<= 1;
    return p2;
  }();
  return v;
}
// ---------------------------------------------------------------- ops
template <int DT>
__device__ __forceinline__ char* flat_at(void* flat, int64_t off) {
  return static_cast<char*>(flat) + off * (DT == GS_F32 ? 4 : 2);
}

// Op access convention: load<F> / apply<F>(tv, e0, lo, frag[, acc]) handle the
// 4 (or kN) elements starting at element e0 + lo of tensor tv.  F = true is
// the chunk engine's full-chunk path (e0 wave-uniform, no bounds checks, every
// stream 16-B aligned: `fast_ok` says when a tensor qualifies); F = false is
// the general path with bounds / alignment checks (lo = 0 there).

// MODE (GS_SCALE_NONE / _MUL / _DIV) is a template parameter: a runtime mode
// left a uniform branch and the unused IEEE-division path inside every
// lane-step of the streaming loop
// NT: non-temporal loads of the source (a read-once stream above the cache size, nt_read_once)
// G2: a small plan into an fp32 bucket takes groups of 2 chunks (pack_group_small)
template <int N, int SD, int FD, int MODE, bool NT = false, bool G2 = false>
struct PackOp {
  static constexpr int kN = N;
  static constexpr int kG = FD == GS_F32 ? (G2 ? 2 : GS_G_PACK) : (SD == GS_F32 ? GS_G_PACK16 : GS_G_PACK16_16);
  static constexpr int kRed = 0;
  static constexpr int kRedGrid = kGridLimit;
  static constexpr int kRedFuseGrid = GS_RED_FUSE_GRID;
  static constexpr int kKind = GS_OP_PACK;
  float* partials = nullptr;
  int slot;
  void* flat;
  bool flat_vec;
  float s;
  struct Frag { float x[N]; };
  // logical slot 0 = the op's table row `slot` (descriptor loads, gs_kernels.hip: load_tv)
  __device__ int phys(int k) const { return k == 0 ? slot : k; }
  __device__ bool active() const { return true; }
  __device__ bool fast_ok(const TV& v) const {
    return flat_vec && (v.off % 4) == 0 && (v.ptr[0] == nullptr || v.vec(0));
  }
  template <bool F>
  __device__ void load(const TV& v, int64_t e0, uint32_t lo, Frag& f) const {
    const void* src = v.ptr[0];
    if (src == nullptr) {  // unused parameter (find_unused_parameters): pack zeros
      for (int i = 0; i < N; ++i) f.x[i] = 0.f;
      return;
    }
    ld<SD, N, F, NT>(src, e0, lo, v.numel, v.vec(0), f.x);
  }
  template <bool F>
  __device__ void apply(const TV& v, int64_t e0, uint32_t lo, Frag& f, float&) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float x = f.x[i];
      if constexpr (MODE == GS_SCALE_MUL) {
        x = x * s;
      } else if constexpr (MODE == GS_SCALE_DIV) {
        // bf16_compress_hook order: round to the bucket dtype, then divide
        x = round_to<FD>(x) / s;
      }
      f.x[i] = x;
    }
    st<FD, N, F>(flat_at<FD>(flat, v.off), e0, lo, v.numel, flat_vec && (v.off % N) == 0, f.x);
  }
};

// RED = 1: Σ dst² of the written values (fused grad-norm); RED = 2: non-finite
// flag of the written values (fused AMP inf check, max-combined into the flag)
// NT: non-temporal loads of the flat buffer (above the cache size, nt_read_once)
template <int N, int FD, int DD, int RED = 1, bool NT = false>
struct UnpackOp {
  static constexpr int kN = N;
  static constexpr int kG = GS_G_UNPACK;
  static constexpr int kRed = RED;
  static constexpr int kRedGrid = kGridLimit;
  static constexpr int kRedFuseGrid = 8192;  // its fused Σg² / inf check: <= 2 groups per workgroup (r4l)
  static constexpr int kKind = GS_OP_UNPACK;
  float* partials = nullptr;
  bool want_red;
  const void* flat;
  bool flat_vec;
  int slot;
  struct Frag { float x[N]; };
  // logical slot 0 = the op's table row `slot` (descriptor loads, gs_kernels.hip: load_tv)
  __device__ int phys(int k) const { return k == 0 ? slot : k; }
  __device__ bool active() const { return true; }
  __device__ bool fast_ok(const TV& v) const {
    return flat_vec && (v.off % 4) == 0 && (v.ptr[0] == nullptr || v.vec(0));
  }
  template <bool F>
  __device__ void load(const TV& v, int64_t e0, uint32_t lo, Frag& f) const {
    ld<FD, N, F, NT>(flat_at<FD>(const_cast<void*>(flat), v.off), e0, lo, v.numel,
                     flat_vec && (v.off % N) == 0, f.x);
  }
  template <bool F>
  __device__ void apply(const TV& v, int64_t e0, uint32_t lo, Frag& f, float& acc) const {
    void* dst = v.ptr[0];
    if (dst == nullptr) return;  // unused parameter: grad left untouched
    st<DD, N, F>(dst, e0, lo, v.numel, v.vec(0), f.x);
    if (want_red) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const float r = round_to<DD>(f.x[i]);
        if constexpr (RED == 1) acc = fmaf(r, r, acc);
        else if ((F || e0 + lo + i < v.numel) && !isfinite(r)) acc = 1.f;
      }
    }
  }
};

template <int N, int DT>
struct ScaleOp {
  static constexpr int kN = N;
  static constexpr int kG = GS_G_UNPACK;
  static constexpr int kRed = 0;
  static constexpr int kRedGrid = kGridLimit;
  static constexpr int kRedFuseGrid = GS_RED_FUSE_GRID;
  static constexpr int kKind = GS_OP_SCALE;
  float* partials = nullptr;
  int slot;
  float s;
  int mode;
  struct Frag { float x[N]; };
  // logical slot 0 = the op's table row `slot` (descriptor loads, gs_kernels.hip: load_tv)
  __device__ int phys(int k) const { return k == 0 ? slot : k; }
  __device__ bool active() const { return true; }
  __device__ bool fast_ok(const TV& v) const { return v.vec(0); }
  template <bool F>
  __device__ void load(const TV& v, int64_t e0, uint32_t lo, Frag& f) const {
    ld<DT, N, F>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.x);
  }
  template <bool F>
  __device__ void apply(const TV& v, int64_t e0, uint32_t lo, Frag& f, float&) const {
#pragma unroll
    for (int i = 0; i < N; ++i) f.x[i] = (mode == GS_SCALE_DIV) ? f.x[i] / s : f.x[i] * s;
    st<DT, N, F>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.x);
  }
};

// NT: non-temporal loads (a read-once stream larger than the Infinity Cache,
// nt_read_once below).  G: chunks per group (the raw partials of a small plan take
// 8: one group per workgroup, every access of the workgroup in flight at once)
template <int N, int DT, bool NT = false, int G = GS_G_RED>
struct SqnormOp {
  static constexpr int kN = N;
  static constexpr int kG = G;
  static constexpr int kRed = 1;
  static constexpr int kRedGrid = 8192;
  static constexpr int kRedFuseGrid = GS_RED_FUSE_GRID;
  static constexpr int kKind = GS_OP_SQNORM;
  float* partials = nullptr;
  int slot;
  struct Frag { float x[N]; };
  // logical slot 0 = the op's table row `slot` (descriptor loads, gs_kernels.hip: load_tv)
  __device__ int phys(int k) const { return k == 0 ? slot : k; }
  __device__ bool active() const { return true; }
  __device__ bool fast_ok(const TV& v) const { return v.vec(0); }
  template <bool F>
  __device__ void load(const TV& v, int64_t e0, uint32_t lo, Frag& f) const {
    ld<DT, N, F, NT>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.x);
  }
  template <bool F>
  __device__ void apply(const TV&, int64_t, uint32_t, Frag& f, float& acc) const {
#pragma unroll
    for (int i = 0; i < N; ++i) acc = fmaf(f.x[i], f.x[i], acc);
  }
};

// Σ x (debug bucket checksums)
template <int N, int DT>
struct SumOp {
  static constexpr int kN = N;
  static constexpr int kG = GS_G_RED;
  static constexpr int kRed = 1;
  static constexpr int kRedGrid = 8192;
  static constexpr int kRedFuseGrid = GS_RED_FUSE_GRID;
  static constexpr int kKind = GS_OP_SUM;
  float* partials = nullptr;
  int slot;
  struct Frag { float x[N]; };
  __device__ int phys(int k) const { return k == 0 ? slot : k; }
  __device__ bool active() const { return true; }
  __device__ bool fast_ok(const TV& v) const { return v.vec(0); }
  template <bool F>
  __device__ void load(const TV& v, int64_t e0, uint32_t lo, Frag& f) const {
    ld<DT, N, F>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.x);
  }
  template <bool F>
  __device__ void apply(const TV&, int64_t, uint32_t, Frag& f, float& acc) const {
#pragma unroll
    for (int i = 0; i < N; ++i) acc += f.x[i];
  }
};

template <int N, int DT>
struct UnscaleOp {
  static constexpr int kN = N;
  static constexpr int kG = GS_G_RED;
  static constexpr int kRed = 2;
  static constexpr int kRedGrid = 8192;
  static constexpr int kRedFuseGrid = GS_RED_FUSE_GRID;
  static constexpr int kKind = GS_OP_UNSCALE;
  float* partials = nullptr;
  int slot;
  const float* inv;  // nullable
  struct Frag { float x[N]; };
  // logical slot 0 = the op's table row `slot` (descriptor loads, gs_kernels.hip: load_tv)
  __device__ int phys(int k) const { return k == 0 ? slot : k; }
  __device__ bool active() const { return true; }
  __device__ bool fast_ok(const TV& v) const { return v.vec(0); }
  template <bool F>
  __device__ void load(const TV& v, int64_t e0, uint32_t lo, Frag& f) const {
    ld<DT, N, F>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.x);
  }
  template <bool F>
  __device__ void apply(const TV& v, int64_t e0, uint32_t lo, Frag& f, float& acc) const {
#pragma unroll
    for (int i = 0; i < N; ++i)
      if ((F || e0 + lo + i < v.numel) && !isfinite(f.x[i])) acc = 1.f;
    if (inv) {
      const float s = *inv;
      if (s != 1.f) {
#pragma unroll
        for (int i = 0; i < N; ++i) f.x[i] = f.x[i] * s;
        st<DT, N, F>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.x);
      }
    }
  }
};

// clip_grad_norm_'s scale pass (gs_clip_scale): x *= the clip coefficient, which every
// workgroup forms itself from the plan's Σg² partial sums (clip_multiplier, as the
// clipped updates fold them: no combine and no coefficient launch between the Σg²
// pass and this one).  A coefficient of exactly 1 leaves every element as it is
// (x * 1 == x, NaN and -0 included), so the grid then exits before any access.
// NT: non-temporal loads of the grads (above the cache size, nt_read_once: the Σg² pass
// before it could not leave them in the cache either)
template <int N, int DT, bool NT = false>
struct ClipScaleOp {
  static constexpr int kN = N;
  static constexpr int kG = GS_G_UNPACK;
  static constexpr int kRed = 0;
  static constexpr int kRedGrid = kGridLimit;
  static constexpr int kRedFuseGrid = GS_RED_FUSE_GRID;
  static constexpr int kKind = GS_OP_SCALE;
  float* partials = nullptr;
  int slot;
  ClipArgs clip{};
  float gsv = 1.f;
  struct Frag { float x[N]; };
  __device__ int phys(int k) const { return k == 0 ? slot : k; }
  __device__ bool active() const { return gsv != 1.f; }  // uniform; a NaN coefficient scales
  __device__ bool fast_ok(const TV& v) const { return v.vec(0); }
  template <bool F>
  __device__ void load(const TV& v, int64_t e0, uint32_t lo, Frag& f) const {
    ld<DT, N, F, NT>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.x);
  }
  template <bool F>
  __device__ void apply(const TV& v, int64_t e0, uint32_t lo, Frag& f, float&) const {
#pragma unroll
    for (int i = 0; i < N; ++i) f.x[i] = f.x[i] * gsv;
    st<DT, N, F>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.x);
  }
};

// SGD: slots 0 = p (f32), 1 = g (GD), 2 = momentum buffer (f32), 3 = low-precision copy (LD)
// NTG: non-temporal loads of the grad (the load policy above; p and the state stay cached)
template <int N, int GD, int LD, bool NTG = true>
struct SgdOp {
  static constexpr int kN = N;
  static constexpr int kG = GS_G_SGD;
  static constexpr int kRed = 0;
  static constexpr int kRedGrid = kGridLimit;
  static constexpr int kRedFuseGrid = GS_RED_FUSE_GRID;
  static constexpr int kKind = GS_OP_SGD;
  float* partials = nullptr;
  SgdHyper h;
  const float* gscale;
  const float* found_inf;
  const float* hyper = nullptr;  // [lr] in device memory (gs_plan_set_hyper_source)
  ClipArgs clip{};               // folded clip (clip_on), gs_plan_set_clip
  bool clip_on = false;
  bool use_gs = false;           // the grad multiplier gsv applies (set by load_hyper)
  float gsv = 1.f;
  struct Frag { float p[N], g[N], b[N]; };
  __device__ int phys(int k) const { return k; }
  __device__ bool active() const { return found_inf == nullptr || *found_inf == 0.f; }
  __device__ bool fast_ok(const TV& v) const {
    return v.vec(0) && v.vec(1) && (h.mom == 0.f || v.vec(2)) && (LD < 0 || v.vec(3));
  }
  template <bool F>
  __device__ void load(const TV& v, int64_t e0, uint32_t lo, Frag& f) const {
    ld<GS_F32, N, F>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.p);
    ld<GD, N, F, NTG>(v.ptr[1], e0, lo, v.numel, v.vec(1), f.g);
    if (h.mom != 0.f && !h.first) ld<GS_F32, N, F>(v.ptr[2], e0, lo, v.numel, v.vec(2), f.b);
  }
  template <bool F>
  __device__ void apply(const TV& v, int64_t e0, uint32_t lo, Frag& f, float&) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float g = f.g[i];
      if (use_gs) g = g * gsv;                      // clip_grad_norm_ / unscale: grads *= coef
      if (h.maximize) g = -g;
      if (h.wd != 0.f) g = fmaf(h.wd, f.p[i], g);   // grad.add(param, alpha=wd)
      float d = g;
      if (h.mom != 0.f) {
        // buf = clone(g) on the first step, else buf.mul_(mom).add_(g, alpha=1-damp)
        const float b = h.first ? g : fmaf(h.omd, g, f.b[i] * h.mom);
        f.b[i] = b;
        d = h.nesterov ? fmaf(h.mom, b, g) : b;     // g.add(buf, alpha=mom)
      }
      f.p[i] = fmaf(-h.lr, d, f.p[i]);              // param.add_(d, alpha=-lr)
    }
    st<GS_F32, N, F>(v.ptr[0], e0, lo, v.numel, v.vec(0), f.p);
    if (h.mom != 0.f) st<GS_F32, N, F>(v.ptr[2], e0, lo, v.numel, v.vec(2), f.b);
    if constexpr (LD >= 0) st<LD, N, F>(v.ptr[3], e0, lo, v.numel, v.vec(3), f.p);
  }
};

// Adam/AdamW: slots 0 = p, 1 = g, 2 = exp_avg, 3 = exp_avg_sq, 4 = low-precision copy
template <int N, int GD, int LD, bool NTG = true>
struct AdamOp {
  static constexpr int kN = N;
  static constexpr int kG = GS_G_ADAM;
  static constexpr int kRed = 0;
  static constexpr int kRedGrid = kGridLimit;
  static constexpr int kRedFuseGrid = GS_RED_FUSE_GRID;
  static constexpr int kKind = GS_OP_ADAM;
  float* partials = nullptr;
  AdamHyper h;
  const float* gscale;
  const float* found_inf;
  const float* hyper = nullptr;  // [step_size, bc2_sqrt, 1 - lr*wd] in device memory
  ClipArgs clip{};               // folded clip (clip_on), gs_plan_set_clip
  bool clip_on = false;
  bool use_gs = false;           // the grad multiplier gsv applies (set by load_hyper)
  float gsv = 1.f;
  struct Frag { float p[N], g[N], m[N], v[N]; };
  __device__ int phys(int k) const { return k; }
  __device__ bool active() const { return found_inf == nullptr || *found_inf == 0.f; }
  __device__ bool fast_ok(const TV& tv) const {
    return tv.vec(0) && tv.vec(1) && tv.vec(2) && tv.vec(3) && (LD < 0 || tv.vec(4));
  }
  template <bool F>
  __device__ void load(const TV& tv, int64_t e0, uint32_t lo, Frag& f) const {
    ld<GS_F32, N, F>(tv.ptr[0], e0, lo, tv.numel, tv.vec(0), f.p);
    ld<GD, N, F, NTG>(tv.ptr[1], e0, lo, tv.numel, tv.vec(1), f.g);
    ld<GS_F32, N, F>(tv.ptr[2], e0, lo, tv.numel, tv.vec(2), f.m);
    ld<GS_F32, N, F>(tv.ptr[3], e0, lo, tv.numel, tv.vec(3), f.v);
  }
  template <bool F>
  __device__ void apply(const TV& tv, int64_t e0, uint32_t lo, Frag& f, float&) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      float g = f.g[i];
      if (use_gs) g = g * gsv;
      if (h.maximize) g = -g;
      float p = f.p[i];
      if (h.wd != 0.f) {
        if (h.adamw) p = p * h.decay;                       // param.mul_(1 - lr*wd)
        else g = fmaf(h.wd, p, g);                          // grad.add(param, alpha=wd)
      }
      const float m = fmaf(h.w1, g - f.m[i], f.m[i]);       // exp_avg.lerp_(g, 1-b1)  (w<0.5)
      const float v = fmaf(h.w2 * g, g, f.v[i] * h.b2);     // mul_(b2).addcmul_(g, g, 1-b2)
      const float denom = sqrtf(v) / h.bc2s + h.eps;        // sqrt(v)/bc2_sqrt + eps
      p = fmaf(h.step_size, m / denom, p);                  // addcdiv_(m, denom, -lr/bc1)
      f.p[i] = p; f.m[i] = m; f.v[i] = v;
    }
    st<GS_F32, N, F>(tv.ptr[0], e0, lo, tv.numel, tv.vec(0), f.p);
    st<GS_F32, N, F>(tv.ptr[2], e0, lo, tv.numel, tv.vec(2), f.m);
    st<GS_F32, N, F>(tv.ptr[3], e0, lo, tv.numel, tv.vec(3), f.v);
    if constexpr (LD >= 0) st<LD, N, F>(tv.ptr[4], e0, lo, tv.numel, tv.vec(4), f.p);
  }
};

// The update's grad multiplier, formed once per workgroup (uniform): *gscale
// (AMP unscale / a precomputed clip coefficient) or, with a folded clip, the
// clip coefficient itself — from a finished Σg² or from the Σg² kernel's group
// sums (lane j reads group j and the wave folds them: the fused combine's own
// last step, so the result is bit-identical to gs_sqnorm's), then exactly
// clip_coef_kernel's arithmetic.  Workgroup 0 publishes [Σg², coef, norm].
__device__ __forceinline__ float clip_multiplier(const ClipArgs& c, const float* gscale) {
  // wave 0 forms the coefficient, the workgroup reads it from LDS: one wave per
  // workgroup reads the partial sums (every wave of every workgroup re-reading the
  // same lines of L2 was the fold's cost).  Called uniformly by the whole workgroup.
  __shared__ float s_coef;
  if (threadIdx.x < 64) {
    float sq;
    if (c.groups > 0) {
      // lane l: partials l, l + 64, ... in order (<= GS_RED_PARTIALS), then the tree;
      // for <= 64 group sums exactly the fused combine's last step.  All loads are
      // issued before the first add (one memory round trip, not one per partial);
      // an absent partial adds +0 (the partials are sums of squares: never -0)
      constexpr int kPer = GS_RED_PARTIALS / 64;
      const int l = static_cast<int>(threadIdx.x);
      float v[kPer];
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int j = l + 64 * k;
        v[k] = j < c.groups ? c.sq[j * c.stride] : 0.f;
      }
      float x = 0.f;
#pragma unroll
      for (int k = 0; k < kPer; ++k) x = x + v[k];
      sq = wave_sum(0.f + x);
    } else {
      sq = c.sq[0];
    }
    const float s = gscale ? *gscale : 1.f;
    if (gscale) sq = sq * (s * s);                    // the norm of the unscaled grads
    sq = sq * c.sq_mul;
    const float nrm = sqrtf(sq);
    float coef = c.max_norm / (nrm + c.eps);
    coef = c.torch_clamp ? (coef >= 1.f ? 1.f : coef) : (coef < 1.f ? coef : 1.f);
    if (gscale) coef = coef * s;
    coef = coef * c.coef_mul;
    if (threadIdx.x == 0) {
      s_coef = coef;
      if (c.out && blockIdx.x == 0) {
        c.out[0] = sq;
        c.out[1] = coef;
        c.out[2] = nrm;
      }
    }
  }
  __syncthreads();
  return s_coef;
}
template <class Op>
__device__ __forceinline__ void load_grad_multiplier(Op& op) {
  op.use_gs = op.gscale != nullptr || op.clip_on;
  op.gsv = op.clip_on ? clip_multiplier(op.clip, op.gscale) : (op.gscale ? *op.gscale : 1.f);
}
template <int N, int DT, bool NT>
__device__ __forceinline__ void load_hyper(ClipScaleOp<N, DT, NT>& op) {
  op.gsv = clip_multiplier(op.clip, nullptr);
}
template <int N, int GD, int LD, bool NTG>
__device__ __forceinline__ void load_hyper(SgdOp<N, GD, LD, NTG>& op) {
  if (op.hyper) {
    op.h.lr = op.hyper[0];
    if (op.h.first < 0) op.h.first = op.hyper[1] != 0.f;  // device first-step flag (AMP skips)
  }
  load_grad_multiplier(op);
}
template <int N, int GD, int LD, bool NTG>
__device__ __forceinline__ void load_hyper(AdamOp<N, GD, LD, NTG>& op) {
  if (op.hyper) {
    op.h.step_size = op.hyper[0];
    op.h.bc2s = op.hyper[1];
    op.h.decay = op.hyper[2];
  }
  load_grad_multiplier(op);
}

__global__ void clip_coef_kernel(const float* sq, float max_norm, float eps, float* coef,
                                 float* norm) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float nrm = sqrtf(sq[0]);
    if (norm) norm[0] = nrm;
    const float c = max_norm / (nrm + eps);
    coef[0] = c < 1.f ? c : 1.f;
  }
}

// ------------------------------------------------------------- launching
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
      (void)hipSetDevice(dev);
    } else {
      prev = -1;
    }
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// The plan launch timer (gs_plan_timer_enable) takes the kernel's own start and
// end: hipExtLaunchKernel's events, written by the dispatch itself, instead of two
// event packets queued around it, whose own processing added ~3 µs to every timed
// launch (a fifth of a 17 µs Σg² kernel, profiles/r4/r4i_timer_ext.jsonl).

// groups_only (gs_sqnorm_partial): the fused reduction stops at its R group
// sums, which stay in the plan for the next clipped update (p->red_groups);
// groups_only = 2 (raw, gs_sqnorm_partial_out on a small plan): a balanced grid of
// <= GS_RED_PARTIALS workgroups, each writing its partial to red_out
// the raw form: groups of GS_G_RED chunks, at most kRawWorkgroups workgroups (= partials,
// <= GS_RED_PARTIALS), each the same number of groups; plans of up to 4 Ki chunks
#ifndef GS_RAW_WORKGROUPS
#define GS_RAW_WORKGROUPS 1024  // 256 / 512 / 1024 / 2048: 7.1 / 4.7-5.1 / 4.4-4.5 / 4.3-4.4 µs (r5g)
#endif
constexpr int kRawWorkgroups = GS_RAW_WORKGROUPS;
static_assert(kRawWorkgroups <= GS_RED_PARTIALS, "raw partials fit the caller's buffer");
constexpr int64_t kRawChunksMax = 4096;
template <class Op>
int launch(gs_plan* p, Op op, void* stream, float* red_out = nullptr, int accumulate = 0,
           int groups_only = 0) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p->n == 0 || p->segs.empty()) {
    if (Op::kRed != 0 && red_out && !accumulate) HIP_RET(hipMemsetAsync(red_out, 0, 4, s));
    return GS_OK;
  }
  {
    GsRange r("gs_plan_flush");
    GS_TRY_RET(hip_plan_flush(p, stream));
  }
  GsRange r_launch("gs_kernel_launch");
  op.partials = p->d_partials;
  const bool capturing = stream_capturing(s);
  // one-shot events (the bucketer's timeline) take the launch; the timer ring skips it
  const bool once = !capturing && (p->once_start != nullptr || p->once_stop != nullptr);
  const int nslots = (capturing || once) ? 0 : static_cast<int>(p->timer_ev.size() / 2);
  const int tk = p->timer_next;
  hipEvent_t ev0 = once ? static_cast<hipEvent_t>(p->once_start)
                        : nslots ? static_cast<hipEvent_t>(p->timer_ev[2 * tk]) : nullptr;
  hipEvent_t ev1 = once ? static_cast<hipEvent_t>(p->once_stop)
                        : nslots ? static_cast<hipEvent_t>(p->timer_ev[2 * tk + 1]) : nullptr;
  p->once_start = p->once_stop = nullptr;
  // a collective deferred its watchdog mark to this launch (gs_allreduce_marked,
  // gs_bucketer_set_mark_consumer): the kernel's own stop event carries it when the
  // launch has none of its own, else a packet follows the launch
  gs_comm* wc = (!capturing && p->watch_comm) ? static_cast<gs_comm*>(p->watch_comm) : nullptr;
  void* wev = nullptr;
  int wtake = 0;
  if (wc) {
    p->watch_comm = nullptr;
    wtake = comm_mark_take(wc, &wev);
  }
  const bool wcarry = wtake && wev && ev1 == nullptr;
  if (wcarry) ev1 = static_cast<hipEvent_t>(wev);
  const bool ext = once || nslots || wcarry;
  bool fused = false;
  int grid = 1;
  {
    const int64_t groups = (static_cast<int64_t>(p->chunks.size()) + Op::kG - 1) / Op::kG;
    const bool red = Op::kRed != 0 && (red_out || groups_only);
    // a streaming op carrying a reduction (the unpack's Σg² / inf check) runs one group
    // per workgroup; up to 16 Ki groups (a ResNet-50 gradient, any DDP bucket) it
    // combines in-kernel on an 8 Ki grid rather than through a second launch
    // (profiles/r4/r4l_red_grid.jsonl: ResNet-50 0.70 -> 0.78; ResNet-152 x 2 stays
    // uncapped + combine launch, 0.76 vs 0.71)
    const int op_cap = (Op::kRedGrid == kGridLimit && groups <= 2 * kRedFuseMaxGrid) ? kRedFuseMaxGrid
                                                                                       : Op::kRedGrid;
    int cap = red ? std::min(p->grid_cap, red_grid_cap(op_cap)) : p->grid_cap;
    // groups_only is asked for only when the ordinary reduction would fuse too
    // (hip_sqnorm_partial), so both fold the same R group sums of the same grid
    const bool raw = red && groups_only == 2;
    fused = red && !raw && (groups_only || (cap <= kRedFuseMaxGrid && red_fuse_groups() > 0));
    if (fused) cap = std::min(cap, red_grid_cap(Op::kRedFuseGrid));
    // any fused reduction overwrites the group sums a gs_sqnorm_partial left
    if (fused && !groups_only) p->red_valid = false;
    grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(groups, cap)));
    if (raw) {
      // every workgroup the same number of groups (grid-stride over a balanced grid)
      const int64_t per = (groups + kRawWorkgroups - 1) / kRawWorkgroups;
      grid = static_cast<int>(std::max<int64_t>(1, (groups + per - 1) / per));
    }
    PlanArgs a = p->args();
    a.red_out = Op::kRed != 0 ? red_out : nullptr;  // groups_only: the contiguous group sums (nullable)
    a.red_acc = accumulate;
    a.red_fuse = fused ? red_fuse_groups() : 0;
    a.red_groups_only = groups_only ? 1 : 0;
    a.red_raw = raw ? 1 : 0;
    if (groups_only) p->red_groups = raw ? grid : std::min(grid, red_fuse_groups());
    a.ticket = reinterpret_cast<uint32_t*>(p->d_partials + kGridLimit);  // kRedSyncWords, zero between launches
    const bool combine = Op::kRed != 0 && red_out && !fused && !raw;
    if (ext)
      hipExtLaunchKernelGGL((chunk_kernel<Op>), dim3(grid), dim3(kBlock), 0, s, ev0, combine ? nullptr : ev1, 0, a,
                            op);
    else
      hipLaunchKernelGGL((chunk_kernel<Op>), dim3(grid), dim3(kBlock), 0, s, a, op);
  }
  HIP_RET(hipGetLastError());
  if constexpr (Op::kRed != 0) {
    if (red_out && !fused && groups_only != 2) {
      if (ext)
        hipExtLaunchKernelGGL((combine_partials<Op::kRed == 2>), dim3(1), dim3(kCombineBlock), 0, s, nullptr, ev1, 0,
                              (const float*)p->d_partials, grid, red_out, accumulate);
      else
        hipLaunchKernelGGL((combine_partials<Op::kRed == 2>), dim3(1), dim3(kCombineBlock), 0, s,
                           (const float*)p->d_partials, grid, red_out, accumulate);
      HIP_RET(hipGetLastError());
    }
  }
  if (wtake) {
    if (wev && !wcarry) HIP_RET(hipEventRecord(static_cast<hipEvent_t>(wev), s));
    GS_TRY_RET(comm_mark_commit(wc, wev, stream, p));
  }
  if (nslots) {
    p->timer_kind[tk] = Op::kKind;
    p->timer_next = (tk + 1) % nslots;
    p->timer_count = std::min(p->timer_count + 1, nslots);
  }
  // No event packet after the launch: each one cost ~4.7 µs of stream time on every
  // dependent chain (scripts/micro/event_chain.hip, profiles/r5/r5a_event_chain.jsonl).
  // A launch on another stream orders itself after this one (hip_plan_flush); release
  // synchronises before freeing.
  p->last_stream = stream;
  p->last_captured = capturing;
  return GS_OK;
}

bool flat_aligned(const void* flat) { return (reinterpret_cast<uintptr_t>(flat) & 15u) == 0; }

}  // namespace

#define GS_DISPATCH_FLOAT(DT, NAME, ...)                        \
  switch (DT) {                                                 \
    case GS_F32: { constexpr int NAME = GS_F32; __VA_ARGS__; break; }   \
    case GS_BF16: { constexpr int NAME = GS_BF16; __VA_ARGS__; break; } \
    case GS_F16: { constexpr int NAME = GS_F16; __VA_ARGS__; break; }   \
    default: return fail(GS_EINVAL, "unsupported floating dtype");      \
  }

#define GS_DISPATCH_LOWP(DT, NAME, ...)                                  \
  switch (DT) {                                                          \
    case -1: { constexpr int NAME = -1; __VA_ARGS__; break; }            \
    case GS_BF16: { constexpr int NAME = GS_BF16; __VA_ARGS__; break; }  \
    case GS_F16: { constexpr int NAME = GS_F16; __VA_ARGS__; break; }    \
    default: return fail(GS_EINVAL, "unsupported low-precision dtype");  \
  }

}  // namespace gs
