// Training-image augmentation on the GPU (SURVEY 8(f) "GPU input pipeline"): the
// reference's per-image transform chain of lib/dataset.py:106-117 after the resize,
//   RandomHorizontalFlip(0.5) -> ColorJitter(0.2, 0.2, 0.2, 0.01) -> ToTensor
//   -> Normalize((0.5,) * 3, (0.5,) * 3),
// applied to a batch of decoded, resized uint8 HWC images already in HBM and written as the
// step's fp32 NCHW [-1, 1] input.  The reference runs ColorJitter on the PIL image
// (torchvision's functional_pil: ImageEnhance.Brightness / Contrast / Color and a uint8
// shift of PIL's HSV hue band), so every op here is PIL's uint8 arithmetic, operation for
// operation (libImaging Blend / Convert as restated and checked exhaustively in
// oracle/augment_oracle.py): each op rounds to uint8 before the next, the grayscale is
// PIL's L = (19595 R + 38470 G + 7471 B + 2^15) >> 16, the contrast mean is
// int(sum(L) / N + 0.5) in double, the float / double mix of PIL's HSV conversions is kept
// (and fp contraction is off), so the output is byte-identical to the reference transform.
// The random parameters (flip, the op order fn_idx and the four factors) are drawn on the
// host in torchvision's call order and passed per image (pggan_amd/data.py).
//
// Three launches per batch: (1) flip + the ops before contrast into a uint8 workspace image,
// per-block integer sums of L (contrast blends with the mean of the image as it is at that
// point); (2) one block per image: the integer mean; (3) contrast + the ops after it +
// ToTensor + Normalize.  HBM bound: 3 B read + 3 B written + 3 B read + 12 B written per pixel.
#include <hip/hip_runtime.h>

#include "common.h"

#pragma clang fp contract(off)   // and -ffp-contract=off for this file (Makefile)

namespace {

constexpr int AUG_PPT = 4;                 // pixels per thread (one 12-byte source run)
constexpr int AUG_BLOCK = 256;
constexpr int AUG_PSTRIDE = 12;            // floats per image in the parameter table

struct AugP {
  float b, c, s;  // enhance factors (Image.blend's float alpha)
  int flip;
  int hue;        // uint8 shift of the H band: np.uint8(hue_factor * 255) (trunc, wrap)
  int order[4];   // torchvision fn_idx: 0 brightness, 1 contrast, 2 saturation, 3 hue
};

__device__ __forceinline__ AugP aug_params(const float* params, int img) {
  const float* q = params + img * AUG_PSTRIDE;
  AugP p;
  p.flip = q[0] != 0.f;
  p.b = q[1]; p.c = q[2]; p.s = q[3];
  // hue_factor * 255 in double (a Python float times 255), truncated, wrapped to uint8
  p.hue = (int)(long long)((double)q[4] * 255.0) & 255;
#pragma unroll
  for (int k = 0; k < 4; ++k) p.order[k] = (int)q[5 + k];
  return p;
}

// Image.blend(in1, in2, alpha) per byte (libImaging/Blend.c): float arithmetic
// in1 + alpha * (in2 - in1), truncated to uint8; clipped to [0, 255] outside 0 <= alpha <= 1
__device__ __forceinline__ int blend8(int a, int b, float alpha) {
  const float t = __fadd_rn((float)a, __fmul_rn(alpha, (float)(b - a)));
  if (alpha >= 0.f && alpha <= 1.f) return (int)t;
  if (t <= 0.f) return 0;
  if (t >= 255.f) return 255;
  return (int)t;
}
// RGB -> L (libImaging/Convert.c, ITU-R 601-2 in 16.16 fixed point, rounded)
__device__ __forceinline__ int luma8(int r, int g, int b) {
  return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16;
}
__device__ __forceinline__ int clip8(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

// RGB -> HSV (libImaging/Convert.c rgb2hsv_row): float ratios, the hue offsets and the wrap
// in double, truncation to uint8
__device__ __forceinline__ void rgb2hsv8(int r, int g, int b, int& uh, int& us, int& uv) {
  const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
  uv = maxc;
  if (minc == maxc) {
    uh = 0;
    us = 0;
    return;
  }
  const float cr = (float)(maxc - minc);
  const float s = __fdiv_rn(cr, (float)maxc);
  const float rc = __fdiv_rn((float)(maxc - r), cr);
  const float gc = __fdiv_rn((float)(maxc - g), cr);
  const float bc = __fdiv_rn((float)(maxc - b), cr);
  float h;
  if (r == maxc) h = __fsub_rn(bc, gc);
  else if (g == maxc) h = (float)(__dsub_rn(__dadd_rn(2.0, (double)rc), (double)bc));
  else h = (float)(__dsub_rn(__dadd_rn(4.0, (double)gc), (double)rc));
  h = (float)fmod(__dadd_rn(__ddiv_rn((double)h, 6.0), 1.0), 1.0);
  uh = clip8((int)__dmul_rn((double)h, 255.0));
  us = clip8((int)__dmul_rn((double)s, 255.0));
}

// C round(): half away from zero (the arguments here are >= 0)
__device__ __forceinline__ int round_half_up(double x) { return (int)floor(__dadd_rn(x, 0.5)); }

// HSV -> RGB (libImaging/Convert.c hsv2rgb)
__device__ __forceinline__ void hsv2rgb8(int h, int s, int v, int& r, int& g, int& b) {
  if (s == 0) {
    r = g = b = v;
    return;
  }
  const double h6 = __ddiv_rn(__dmul_rn((double)(float)h, 6.0), 255.0);
  const int i = (int)floor(h6);
  const float f = (float)__dsub_rn(h6, (double)(float)i);
  const float fs = (float)__ddiv_rn((double)(float)s, 255.0);
  const double vf = (double)(float)v;
  const int p = clip8(round_half_up(__dmul_rn(vf, __dsub_rn(1.0, (double)fs))));
  const int q = clip8(round_half_up(__dmul_rn(vf, __dsub_rn(1.0, (double)__fmul_rn(fs, f)))));
  const int t = clip8(round_half_up(__dmul_rn(vf, __dsub_rn(1.0, __dmul_rn((double)fs,
                                                                           __dsub_rn(1.0, (double)f))))));
  switch (i % 6) {
    case 0: r = v; g = t; b = p; break;
    case 1: r = q; g = v; b = p; break;
    case 2: r = p; g = v; b = t; break;
    case 3: r = p; g = q; b = v; break;
    case 4: r = t; g = p; b = v; break;
    default: r = v; g = p; b = q; break;
  }
}

// ops k0 <= k < k1 of the image's order on one uint8 pixel; op 1 (contrast) blends with the
// image's integer L mean
__device__ __forceinline__ void apply_ops(const AugP& P, int k0, int k1, int mean, int& r, int& g,
                                          int& b) {
  for (int k = k0; k < k1; ++k) {
    switch (P.order[k]) {
      case 0:   // ImageEnhance.Brightness: blend(black, img, f)
        r = blend8(0, r, P.b); g = blend8(0, g, P.b); b = blend8(0, b, P.b);
        break;
      case 1:   // ImageEnhance.Contrast: blend(mean gray, img, f)
        r = blend8(mean, r, P.c); g = blend8(mean, g, P.c); b = blend8(mean, b, P.c);
        break;
      case 2: {  // ImageEnhance.Color: blend(L(img) as RGB, img, f)
        const int l = luma8(r, g, b);
        r = blend8(l, r, P.s); g = blend8(l, g, P.s); b = blend8(l, b, P.s);
        break;
      }
      default: {  // adjust_hue: RGB -> HSV, H += shift (uint8 wrap), HSV -> RGB
        int h, s, v;
        rgb2hsv8(r, g, b, h, s, v);
        hsv2rgb8((h + P.hue) & 255, s, v, r, g, b);
        break;
      }
    }
  }
}

__device__ __forceinline__ int contrast_pos(const AugP& P) {
  int k = 0;
  while (k < 4 && P.order[k] != 1) ++k;
  return k;
}

// stage 1: grid (nblk, B); mid holds the pre-contrast uint8 image (already flipped)
__global__ __launch_bounds__(AUG_BLOCK) void aug_stage1(const unsigned char* src, unsigned char* mid,
                                                        const float* params, unsigned* part, int H,
                                                        int W) {
  const int img = blockIdx.y;
  const AugP P = aug_params(params, img);
  const int kc = contrast_pos(P);
  const size_t hw = (size_t)H * W;
  const size_t q = ((size_t)blockIdx.x * AUG_BLOCK + threadIdx.x) * AUG_PPT;   // first pixel
  unsigned lsum = 0;
  if (q < hw) {
    const int y = (int)(q / W), x = (int)(q % W);
    // dst pixels x..x+3 come from x..x+3, or mirrored from W-4-x..W-1-x (one 12-B run)
    const int sx = P.flip ? W - AUG_PPT - x : x;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + ((size_t)img * hw + (size_t)y * W + sx) * 3);
    uint32_t w[3] = {s32[0], s32[1], s32[2]};
    const unsigned char* by = reinterpret_cast<const unsigned char*>(w);
    uint32_t o[3] = {0u, 0u, 0u};
    unsigned char* ob = reinterpret_cast<unsigned char*>(o);
#pragma unroll
    for (int j = 0; j < AUG_PPT; ++j) {
      const int sj = P.flip ? AUG_PPT - 1 - j : j;
      int r = by[3 * sj], g = by[3 * sj + 1], b = by[3 * sj + 2];
      apply_ops(P, 0, kc, 0, r, g, b);
      lsum += (unsigned)luma8(r, g, b);
      ob[3 * j] = (unsigned char)r; ob[3 * j + 1] = (unsigned char)g; ob[3 * j + 2] = (unsigned char)b;
    }
    uint32_t* d = reinterpret_cast<uint32_t*>(mid + ((size_t)img * hw + q) * 3);
    d[0] = o[0]; d[1] = o[1]; d[2] = o[2];
  }
  // integer block sum (exact, any order)
  __shared__ unsigned red[AUG_BLOCK];
  red[threadIdx.x] = lsum;
  __syncthreads();
  for (int st = AUG_BLOCK / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[(size_t)img * gridDim.x + blockIdx.x] = red[0];
}

// stage 2: one block per image: ImageStat mean of L (sum / count in double), int(m + 0.5)
__global__ __launch_bounds__(AUG_BLOCK) void aug_stage2(const unsigned* part, int nblk, int* mean,
                                                        double npix) {
  const int img = blockIdx.x;
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < nblk; i += AUG_BLOCK) s += part[(size_t)img * nblk + i];
  __shared__ unsigned long long red[AUG_BLOCK];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int st = AUG_BLOCK / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) mean[img] = (int)__dadd_rn(__ddiv_rn((double)red[0], npix), 0.5);
}

// stage 3: contrast + the ops after it, ToTensor (x / 255) and Normalize((x - 0.5) / 0.5)
__global__ __launch_bounds__(AUG_BLOCK) void aug_stage3(const unsigned char* mid, float* dst,
                                                        const float* params, const int* mean, int H,
                                                        int W) {
  const int img = blockIdx.y;
  const AugP P = aug_params(params, img);
  const int kc = contrast_pos(P);
  const int m = mean[img];
  const size_t hw = (size_t)H * W;
  const size_t q = ((size_t)blockIdx.x * AUG_BLOCK + threadIdx.x) * AUG_PPT;
  if (q >= hw) return;
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(mid + ((size_t)img * hw + q) * 3);
  uint32_t w[3] = {s32[0], s32[1], s32[2]};
  const unsigned char* by = reinterpret_cast<const unsigned char*>(w);
  float o[3][AUG_PPT];
#pragma unroll
  for (int j = 0; j < AUG_PPT; ++j) {
    int r = by[3 * j], g = by[3 * j + 1], b = by[3 * j + 2];
    apply_ops(P, kc, 4, m, r, g, b);
    o[0][j] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)r, 255.f), 0.5f), 0.5f);
    o[1][j] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)g, 255.f), 0.5f), 0.5f);
    o[2][j] = __fdiv_rn(__fsub_rn(__fdiv_rn((float)b, 255.f), 0.5f), 0.5f);
  }
  float* d = dst + (size_t)img * 3 * hw + q;
#pragma unroll
  for (int c = 0; c < 3; ++c)
    *reinterpret_cast<float4*>(d + c * hw) = make_float4(o[c][0], o[c][1], o[c][2], o[c][3]);
}

int aug_nblk(int H, int W) { return pg_cdiv(H * W / AUG_PPT, AUG_BLOCK); }

size_t aug_mid_bytes(int B, int H, int W) { return ((size_t)B * H * W * 3 + 15) & ~(size_t)15; }

}  // namespace

extern "C" {

size_t pg_augment_workspace_bytes(int B, int H, int W) {
  return aug_mid_bytes(B, H, W) + ((size_t)B * aug_nblk(H, W) + B) * sizeof(unsigned);
}

int pg_augment_u8(int B, int H, int W, const void* src, const float* params, float* ws,
                  size_t ws_bytes, float* dst, void* stream) {
  PG_CHECK_ARG(src && params && ws && dst && B > 0 && H > 0 && W > 0, "augment: bad args");
  PG_CHECK_ARG(W % AUG_PPT == 0, "augment: W (%d) must be a multiple of %d", W, AUG_PPT);
  PG_CHECK_ARG(((uintptr_t)src & 3) == 0 && ((uintptr_t)dst & 15) == 0 && ((uintptr_t)ws & 15) == 0,
               "augment: src must be 4-byte, dst and ws 16-byte aligned");
  PG_CHECK_ARG(ws_bytes >= pg_augment_workspace_bytes(B, H, W), "augment: workspace too small");
  const int nblk = aug_nblk(H, W);
  hipStream_t st = (hipStream_t)stream;
  unsigned char* mid = reinterpret_cast<unsigned char*>(ws);
  unsigned* part = reinterpret_cast<unsigned*>(mid + aug_mid_bytes(B, H, W));
  int* mean = reinterpret_cast<int*>(part + (size_t)B * nblk);
  PG_KLAUNCH(aug_stage1, dim3(nblk, B), dim3(AUG_BLOCK), 0, st,
                     reinterpret_cast<const unsigned char*>(src), mid, params, part, H, W);
  PG_LAUNCH_CHECK();
  PG_KLAUNCH(aug_stage2, dim3(B), dim3(AUG_BLOCK), 0, st, part, nblk, mean,
                     (double)H * (double)W);
  PG_LAUNCH_CHECK();
  PG_KLAUNCH(aug_stage3, dim3(nblk, B), dim3(AUG_BLOCK), 0, st, mid, dst, params, mean, H, W);
  PG_LAUNCH_CHECK();
  return PG_OK;
}

}  // extern "C"
