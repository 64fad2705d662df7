// Training-image augmentation on the GPU (SURVEY 8(f) "GPU input pipeline"): the
// reference's per-image transform chain of lib/dataset.py:106-117 after the resize,
//   RandomHorizontalFlip(0.5) -> ColorJitter(0.2, 0.2, 0.2, 0.01) -> ToTensor
//   -> Normalize((0.5,) * 3, (0.5,) * 3),
// applied to a batch of decoded, resized uint8 HWC images already in HBM and written as the
// step's fp32 NCHW [-1, 1] input.  The jitter follows torchvision's tensor formulation
// (functional_tensor: _blend, rgb_to_grayscale, _rgb2hsv / _hsv2rgb) in fp32; the random
// parameters (flip, the op order fn_idx and the four factors) are drawn on the host in
// torchvision's call order and passed per image (pggan_amd/data.py).
//
// Three launches per batch: (1) flip + the ops before contrast, per-block partial sums of
// the grayscale image (contrast blends with the mean of the image as it is at that point);
// (2) one block per image sums its partials in a fixed order (deterministic mean);
// (3) contrast + the ops after it + normalize, in place.  HBM bound: 3 B read + 12 B
// written + 12 B read + 12 B written per pixel.
#include <hip/hip_runtime.h>

#include "common.h"

namespace {

constexpr int AUG_PPT = 4;                 // pixels per thread (one 12-byte source run)
constexpr int AUG_BLOCK = 256;
constexpr int AUG_PSTRIDE = 12;            // floats per image in the parameter table

struct AugP {
  float flip, b, c, s, h;
  float c1, s1;   // 1 - contrast, 1 - saturation (rounded from double on the host, as in _blend)
  int order[4];   // torchvision fn_idx: 0 brightness, 1 contrast, 2 saturation, 3 hue
};

__device__ __forceinline__ AugP aug_params(const float* params, int img) {
  const float* q = params + img * AUG_PSTRIDE;
  AugP p;
  p.flip = q[0]; p.b = q[1]; p.c = q[2]; p.s = q[3]; p.h = q[4];
  p.c1 = q[9]; p.s1 = q[10];
#pragma unroll
  for (int k = 0; k < 4; ++k) p.order[k] = (int)q[5 + k];
  return p;
}

__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }
// torchvision rgb_to_grayscale (float input): 0.2989 r + 0.587 g + 0.114 b
__device__ __forceinline__ float gray(float r, float g, float b) {
  return 0.2989f * r + 0.587f * g + 0.114f * b;
}
// _blend(img1, img2, ratio) = (ratio * img1 + (1 - ratio) * img2).clamp(0, 1)
__device__ __forceinline__ float blend(float a, float o, float f, float f1) { return clamp01(f * a + f1 * o); }

// adjust_hue (functional_tensor): _rgb2hsv, h = (h + hue) % 1, _hsv2rgb
__device__ __forceinline__ void hue_shift(float& r, float& g, float& b, float hf) {
  const float maxc = fmaxf(fmaxf(r, g), b), minc = fminf(fminf(r, g), b);
  const bool eqc = maxc == minc;
  const float cr = maxc - minc;
  const float s = cr / (eqc ? 1.f : maxc);
  const float crd = eqc ? 1.f : cr;
  const float rc = (maxc - r) / crd, gc = (maxc - g) / crd, bc = (maxc - b) / crd;
  const float hr = maxc == r ? bc - gc : 0.f;
  const float hg = (maxc == g && maxc != r) ? 2.f + rc - bc : 0.f;
  const float hb = (maxc != g && maxc != r) ? 4.f + gc - rc : 0.f;
  float h = hr + hg + hb;
  h = fmodf(h / 6.f + 1.f, 1.f);
  h = h + hf;
  h = h - floorf(h);                    // Python / torch remainder by 1.0
  const float v = maxc;
  const float fi = floorf(h * 6.f);
  const float f = h * 6.f - fi;
  int i = (int)fi % 6;
  if (i < 0) i += 6;
  const float p = clamp01(v * (1.f - s));
  const float q = clamp01(v * (1.f - s * f));
  const float t = clamp01(v * (1.f - s * (1.f - f)));
  switch (i) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

// ops k0 <= k < k1 of the image's order; op 1 (contrast) uses `mean`
__device__ __forceinline__ void apply_ops(const AugP& P, int k0, int k1, float mean, float& r, float& g,
                                          float& b) {
  for (int k = k0; k < k1; ++k) {
    switch (P.order[k]) {
      case 0: r = clamp01(P.b * r); g = clamp01(P.b * g); b = clamp01(P.b * b); break;
      case 1: r = blend(r, mean, P.c, P.c1); g = blend(g, mean, P.c, P.c1); b = blend(b, mean, P.c, P.c1); break;
      case 2: {
        const float l = gray(r, g, b);
        r = blend(r, l, P.s, P.s1); g = blend(g, l, P.s, P.s1); b = blend(b, l, P.s, P.s1);
        break;
      }
      default: hue_shift(r, g, b, P.h); break;
    }
  }
}

__device__ __forceinline__ int contrast_pos(const AugP& P) {
  int k = 0;
  while (k < 4 && P.order[k] != 1) ++k;
  return k;
}

// stage 1: grid (nblk, B); dst planes hold the pre-contrast values (already flipped)
__global__ __launch_bounds__(AUG_BLOCK) void aug_stage1(const unsigned char* src, float* dst,
                                                        const float* params, float* part, int H,
                                                        int W) {
  const int img = blockIdx.y;
  const AugP P = aug_params(params, img);
  const int kc = contrast_pos(P);
  const size_t hw = (size_t)H * W;
  const size_t q = ((size_t)blockIdx.x * AUG_BLOCK + threadIdx.x) * AUG_PPT;   // first pixel
  float gsum = 0.f;
  if (q < hw) {
    const int y = (int)(q / W), x = (int)(q % W);
    const bool flip = P.flip != 0.f;
    // dst pixels x..x+3 come from x..x+3, or mirrored from W-4-x..W-1-x (one 12-B run)
    const int sx = flip ? W - AUG_PPT - x : x;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + ((size_t)img * hw + (size_t)y * W + sx) * 3);
    uint32_t w[3] = {s32[0], s32[1], s32[2]};
    const unsigned char* by = reinterpret_cast<const unsigned char*>(w);
    float o[3][AUG_PPT];
#pragma unroll
    for (int j = 0; j < AUG_PPT; ++j) {
      const int sj = flip ? AUG_PPT - 1 - j : j;
      float r = by[3 * sj] / 255.f, g = by[3 * sj + 1] / 255.f, b = by[3 * sj + 2] / 255.f;
      apply_ops(P, 0, kc, 0.f, r, g, b);
      gsum += gray(r, g, b);
      o[0][j] = r; o[1][j] = g; o[2][j] = b;
    }
    float* d = dst + (size_t)img * 3 * hw + q;
#pragma unroll
    for (int c = 0; c < 3; ++c)
      *reinterpret_cast<float4*>(d + c * hw) = make_float4(o[c][0], o[c][1], o[c][2], o[c][3]);
  }
  // block sum in a fixed order (deterministic)
  __shared__ float red[AUG_BLOCK];
  red[threadIdx.x] = gsum;
  __syncthreads();
  for (int st = AUG_BLOCK / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)img * gridDim.x + blockIdx.x] = red[0];
}

// stage 2: one block per image: mean of the grayscale image from the partials
__global__ __launch_bounds__(AUG_BLOCK) void aug_stage2(const float* part, int nblk, float* mean,
                                                        float inv_hw) {
  const int img = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < nblk; i += AUG_BLOCK) s += part[(size_t)img * nblk + i];
  __shared__ float red[AUG_BLOCK];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = AUG_BLOCK / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) mean[img] = red[0] * inv_hw;
}

// stage 3: contrast + the ops after it, then Normalize((0.5,)*3, (0.5,)*3), in place
__global__ __launch_bounds__(AUG_BLOCK) void aug_stage3(float* dst, const float* params,
                                                        const float* mean, int H, int W) {
  const int img = blockIdx.y;
  const AugP P = aug_params(params, img);
  const int kc = contrast_pos(P);
  const float m = mean[img];
  const size_t hw = (size_t)H * W;
  const size_t q = ((size_t)blockIdx.x * AUG_BLOCK + threadIdx.x) * AUG_PPT;
  if (q >= hw) return;
  float* d = dst + (size_t)img * 3 * hw + q;
  float4 v[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) v[c] = *reinterpret_cast<const float4*>(d + c * hw);
  float o[3][AUG_PPT] = {{v[0].x, v[0].y, v[0].z, v[0].w},
                         {v[1].x, v[1].y, v[1].z, v[1].w},
                         {v[2].x, v[2].y, v[2].z, v[2].w}};
#pragma unroll
  for (int j = 0; j < AUG_PPT; ++j) {
    float r = o[0][j], g = o[1][j], b = o[2][j];
    apply_ops(P, kc, 4, m, r, g, b);
    o[0][j] = (r - 0.5f) / 0.5f; o[1][j] = (g - 0.5f) / 0.5f; o[2][j] = (b - 0.5f) / 0.5f;
  }
#pragma unroll
  for (int c = 0; c < 3; ++c)
    *reinterpret_cast<float4*>(d + c * hw) = make_float4(o[c][0], o[c][1], o[c][2], o[c][3]);
}

int aug_nblk(int H, int W) { return pg_cdiv(H * W / AUG_PPT, AUG_BLOCK); }

}  // namespace

extern "C" {

size_t pg_augment_workspace_bytes(int B, int H, int W) {
  return ((size_t)B * aug_nblk(H, W) + B) * sizeof(float);
}

int pg_augment_u8(int B, int H, int W, const void* src, const float* params, float* ws,
                  size_t ws_bytes, float* dst, void* stream) {
  PG_CHECK_ARG(src && params && ws && dst && B > 0 && H > 0 && W > 0, "augment: bad args");
  PG_CHECK_ARG(W % AUG_PPT == 0, "augment: W (%d) must be a multiple of %d", W, AUG_PPT);
  PG_CHECK_ARG(((uintptr_t)src & 3) == 0 && ((uintptr_t)dst & 15) == 0,
               "augment: src must be 4-byte and dst 16-byte aligned");
  PG_CHECK_ARG(ws_bytes >= pg_augment_workspace_bytes(B, H, W), "augment: workspace too small");
  const int nblk = aug_nblk(H, W);
  hipStream_t st = (hipStream_t)stream;
  float* part = ws;
  float* mean = ws + (size_t)B * nblk;
  hipLaunchKernelGGL(aug_stage1, dim3(nblk, B), dim3(AUG_BLOCK), 0, st,
                     reinterpret_cast<const unsigned char*>(src), dst, params, part, H, W);
  PG_LAUNCH_CHECK();
  hipLaunchKernelGGL(aug_stage2, dim3(B), dim3(AUG_BLOCK), 0, st, part, nblk, mean,
                     1.f / ((float)H * (float)W));
  PG_LAUNCH_CHECK();
  hipLaunchKernelGGL(aug_stage3, dim3(nblk, B), dim3(AUG_BLOCK), 0, st, dst, params, mean, H, W);
  PG_LAUNCH_CHECK();
  return PG_OK;
}

}  // extern "C"
