// Input step of the CIFAR configuration: the reference's
// data pipeline, restated so that the images live in HBM and one gfx950
// kernel per batch produces the training tensor.
//
// Reference pipeline (R:resnet/pytorch_ddp/ddp_train.py:25-48, torchvision
// 0.15.2 as pinned in R:resnet/pytorch_ddp/requirements.txt; torchvision is
// not installed here, its published algorithm is restated):
//   DistributedSampler(dataset)   shuffle=True, seed=0, drop_last=False
//     (T:utils/data/distributed.py:107-138): randperm(n, manual_seed(seed+epoch)),
//     pad by repeating the head to ceil(n/ws)*ws, take [rank::ws]
//   Pad(4) -> RandomHorizontalFlip() -> RandomCrop(32) -> ToTensor()
//     flip  : torch.rand(1) < 0.5                      (one draw / sample)
//     crop  : i = randint(0, H+8-32+1), j = randint(0, W+8-32+1)
//             (two draws / sample, none when the padded image equals the crop)
//     ToTensor: uint8 HWC -> float32 CHW, x / 255
//   DataLoader(num_workers=0): draws come from torch's global CPU generator in
//   sampler order, after one int64 random_() per iterator (the base seed,
//   T:utils/data/dataloader.py _BaseDataLoaderIter.__init__).
//
// torch's CPU generator is MT19937 (ATen/core/MT19937RNGEngine.h):
// manual_seed(s) = init_genrand(uint32(s)) with left = 1, next = 0; rand(1) of
// float32 = (u32 & 0xFFFFFF) * 2^-24; randint(lo, hi) with hi-lo < 2^32 =
// lo + u32 % (hi-lo); randperm(n) (n < 2^32/20) = forward Fisher-Yates with
// z = u32 % (n - i).  gs_rng_draw_u32 advances torch's own serialized state
// (torch.get_rng_state(), 5056 bytes: u64 seed | i32 left | i32 seeded |
// u64 next | u64 state[624] | normal-sample caches), so the loader consumes
// the global generator exactly as the reference's DataLoader does.
#include <algorithm>
#include <cmath>

#include "gs_common.h"

namespace gs {
namespace {

constexpr int kMtN = 624;
constexpr int kMtM = 397;
constexpr int64_t kTorchRngStateBytes = 5056;
constexpr int64_t kOffLeft = 8, kOffNext = 16, kOffState = 24;

struct Mt19937 {
  uint32_t s[kMtN];
  int32_t left = 1;
  uint64_t next = 0;

  void seed(uint64_t sd) {
    s[0] = static_cast<uint32_t>(sd & 0xffffffffu);
    for (int j = 1; j < kMtN; ++j) s[j] = 1812433253u * (s[j - 1] ^ (s[j - 1] >> 30)) + j;
    left = 1;
    next = 0;
  }
  void twist() {
    for (int i = 0; i < kMtN; ++i) {
      const uint32_t y = (s[i] & 0x80000000u) | (s[(i + 1) % kMtN] & 0x7fffffffu);
      s[i] = s[(i + kMtM) % kMtN] ^ (y >> 1) ^ ((s[(i + 1) % kMtN] & 1u) ? 0x9908b0dfu : 0u);
    }
    left = kMtN;
    next = 0;
  }
  uint32_t operator()() {
    if (--left == 0) twist();
    uint32_t y = s[next++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
};

int load_torch_state(const uint8_t* st, int64_t bytes, Mt19937* m) {
  GS_CHECK_ARG(st != nullptr, "rng state is NULL");
  GS_CHECK_ARG(bytes == kTorchRngStateBytes,
               "rng state must be torch.get_rng_state() of a CPU generator (5056 bytes)");
  int32_t left;
  uint64_t next;
  std::memcpy(&left, st + kOffLeft, 4);
  std::memcpy(&next, st + kOffNext, 8);
  GS_CHECK_ARG(left >= 1 && left <= kMtN && next <= static_cast<uint64_t>(kMtN),
               "rng state is not an MT19937 state");
  m->left = left;
  m->next = next;
  for (int i = 0; i < kMtN; ++i) {
    uint64_t v;
    std::memcpy(&v, st + kOffState + 8 * i, 8);
    m->s[i] = static_cast<uint32_t>(v);
  }
  return GS_OK;
}

void store_torch_state(const Mt19937& m, uint8_t* st) {
  std::memcpy(st + kOffLeft, &m.left, 4);
  std::memcpy(st + kOffNext, &m.next, 8);
  for (int i = 0; i < kMtN; ++i) {
    const uint64_t v = m.s[i];
    std::memcpy(st + kOffState + 8 * i, &v, 8);
  }
}

inline uint16_t f32_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7FC0;
  return static_cast<uint16_t>((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

int host_image_augment(const ImageAugArgs& a) {
  const int64_t per = static_cast<int64_t>(a.C) * a.out_h * a.out_w;
  for (int64_t b = 0; b < a.B; ++b) {
    const int32_t* pr = a.params + 4 * b;
    const int64_t idx = pr[0];
    if (a.out_labels) a.out_labels[b] = a.labels ? a.labels[idx] : 0;
    for (int64_t k = 0; k < per; ++k) {
      int c, y, x;
      if (a.layout == GS_LAYOUT_NCHW) {
        x = static_cast<int>(k % a.out_w);
        y = static_cast<int>((k / a.out_w) % a.out_h);
        c = static_cast<int>(k / (static_cast<int64_t>(a.out_w) * a.out_h));
      } else {
        c = static_cast<int>(k % a.C);
        x = static_cast<int>((k / a.C) % a.out_w);
        y = static_cast<int>(k / (static_cast<int64_t>(a.C) * a.out_w));
      }
      const float v = aug_pixel(a.src, idx, a.H, a.W, a.C, a.pad, pr[1], pr[2], pr[3], c, y, x);
      const int64_t o = b * per + k;
      if (a.out_dtype == GS_F32) static_cast<float*>(a.out)[o] = v;
      else static_cast<uint16_t*>(a.out)[o] = f32_to_bf16(v);
    }
  }
  return GS_OK;
}

}  // namespace
}  // namespace gs

using namespace gs;

extern "C" {

int gs_rng_state_bytes(void) { return static_cast<int>(kTorchRngStateBytes); }

int gs_rng_draw_u32(uint8_t* state, int64_t state_bytes, int64_t n, uint32_t* out) {
  GS_CHECK_ARG(n >= 0 && (n == 0 || out != nullptr), "gs_rng_draw_u32: bad output");
  Mt19937 m;
  GS_TRY_RET(load_torch_state(state, state_bytes, &m));
  for (int64_t i = 0; i < n; ++i) out[i] = m();
  store_torch_state(m, state);
  return GS_OK;
}

int gs_randperm(uint64_t seed, int64_t n, int64_t* out) {
  GS_CHECK_ARG(n >= 0 && (n == 0 || out != nullptr), "gs_randperm: bad output");
  GS_CHECK_ARG(n < static_cast<int64_t>(0xffffffffu / 20),
               "gs_randperm: n beyond torch's 32-bit Fisher-Yates branch");
  Mt19937 m;
  m.seed(seed);
  for (int64_t i = 0; i < n; ++i) out[i] = i;
  for (int64_t i = 0; i + 1 < n; ++i) {
    const int64_t z = static_cast<int64_t>(m() % static_cast<uint32_t>(n - i));
    std::swap(out[i], out[z + i]);
  }
  return GS_OK;
}

int gs_distributed_sampler_indices(int64_t n, int num_replicas, int rank, int shuffle, uint64_t seed,
                                   int64_t epoch, int drop_last, int64_t* out, int64_t cap,
                                   int64_t* count) {
  GS_CHECK_ARG(n >= 0 && num_replicas >= 1 && count != nullptr, "gs_distributed_sampler_indices: bad argument");
  GS_CHECK_ARG(rank >= 0 && rank < num_replicas,
               "Invalid rank " + std::to_string(rank) + ", rank should be in the interval [0, " +
                   std::to_string(num_replicas - 1) + "]");
  int64_t num_samples;
  if (drop_last && n % num_replicas != 0)
    num_samples = (n - num_replicas + num_replicas - 1) / num_replicas;  // ceil((n - ws) / ws)
  else
    num_samples = (n + num_replicas - 1) / num_replicas;
  if (num_samples < 0) num_samples = 0;
  const int64_t total = num_samples * num_replicas;
  *count = num_samples;
  if (out == nullptr) return GS_OK;  // size query
  GS_CHECK_ARG(cap >= num_samples, "gs_distributed_sampler_indices: output too small");
  std::vector<int64_t> idx(static_cast<size_t>(n));
  if (shuffle) GS_TRY_RET(gs_randperm(seed + static_cast<uint64_t>(epoch), n, idx.data()));
  else
    for (int64_t i = 0; i < n; ++i) idx[i] = i;
  // pad by repeating the (shuffled) head, or cut the tail (drop_last)
  std::vector<int64_t> full(static_cast<size_t>(total));
  for (int64_t i = 0; i < total; ++i) {
    GS_CHECK_ARG(n > 0, "gs_distributed_sampler_indices: empty dataset with samples requested");
    full[i] = idx[i % n];
  }
  for (int64_t k = 0; k < num_samples; ++k) out[k] = full[rank + k * num_replicas];
  return GS_OK;
}

int gs_crop_flip_params(const int64_t* indices, int64_t B, int in_h, int in_w, int pad, int out_h,
                        int out_w, int flip, uint8_t* rng_state, int64_t state_bytes,
                        int32_t* params) {
  GS_CHECK_ARG(B >= 0 && (B == 0 || (indices && params)), "gs_crop_flip_params: NULL argument");
  GS_CHECK_ARG(pad >= 0 && in_h > 0 && in_w > 0 && out_h > 0 && out_w > 0, "gs_crop_flip_params: bad geometry");
  const int hp = in_h + 2 * pad, wp = in_w + 2 * pad;
  // RandomCrop.get_params raises "Required crop size ... is larger than input image size"
  GS_CHECK_ARG(out_h <= hp && out_w <= wp, "Required crop size is larger than the (padded) input image size");
  const bool draws_crop = !(hp == out_h && wp == out_w);
  const bool draws = flip || draws_crop;
  Mt19937 m;
  if (draws) GS_TRY_RET(load_torch_state(rng_state, state_bytes, &m));
  for (int64_t b = 0; b < B; ++b) {
    int32_t f = 0, top = 0, left = 0;
    if (flip) f = (m() & 0xFFFFFFu) < (1u << 23);  // float(u & 0xFFFFFF) * 2^-24 < 0.5
    if (draws_crop) {
      top = static_cast<int32_t>(m() % static_cast<uint32_t>(hp - out_h + 1));
      left = static_cast<int32_t>(m() % static_cast<uint32_t>(wp - out_w + 1));
    }
    params[4 * b + 0] = static_cast<int32_t>(indices[b]);
    params[4 * b + 1] = f;
    params[4 * b + 2] = top;
    params[4 * b + 3] = left;
  }
  if (draws) store_torch_state(m, rng_state);
  return GS_OK;
}

int gs_image_augment(int device_kind, int device, const uint8_t* src, const int64_t* labels, int64_t n_src,
                     int H, int W, int C, int pad, int out_h, int out_w, const int32_t* params, int64_t B,
                     void* out, int out_dtype, int out_layout, int64_t* out_labels, void* stream) {
  GS_CHECK_ARG(device_kind == GS_DEV_HOST || device_kind == GS_DEV_HIP, "gs_image_augment: bad device_kind");
  GS_CHECK_ARG(B >= 0 && n_src >= 0 && H > 0 && W > 0 && C > 0 && pad >= 0 && out_h > 0 && out_w > 0,
               "gs_image_augment: bad geometry");
  GS_CHECK_ARG(out_h <= H + 2 * pad && out_w <= W + 2 * pad, "gs_image_augment: crop larger than padded image");
  GS_CHECK_ARG(out_dtype == GS_F32 || out_dtype == GS_BF16, "gs_image_augment: out dtype must be f32 or bf16");
  GS_CHECK_ARG(out_layout == GS_LAYOUT_NCHW || out_layout == GS_LAYOUT_NHWC, "gs_image_augment: bad layout");
  if (B == 0) return GS_OK;
  GS_CHECK_ARG(src && params && out, "gs_image_augment: NULL buffer");
  ImageAugArgs a{src, labels, n_src, H, W, C, pad, out_h, out_w, params, B, out, out_dtype, out_layout, out_labels};
  if (device_kind == GS_DEV_HOST) {
    // host params are readable: bounds-check every sample (the device path
    // trusts the caller, which validated the same params before the upload)
    for (int64_t b = 0; b < B; ++b) {
      const int32_t* p = params + 4 * b;
      GS_CHECK_ARG(p[0] >= 0 && p[0] < n_src, "gs_image_augment: sample index out of range");
      GS_CHECK_ARG(p[2] >= 0 && p[2] + out_h <= H + 2 * pad && p[3] >= 0 && p[3] + out_w <= W + 2 * pad,
                   "gs_image_augment: crop offset out of range");
    }
    return host_image_augment(a);
  }
  if (hip_device_count() <= device) return fail(GS_ENODEV, "gs_image_augment: HIP device not available");
  return hip_image_augment(device, a, stream);
}

}  // extern "C"
