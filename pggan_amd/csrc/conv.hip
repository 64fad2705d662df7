// Equalized-LR 3x3 convolution on gfx950 MFMA: forward / dgrad / R1-tangent
// (one kernel, conv3x3_kernel) and the weight gradient (wgrad3x3_kernel).
//
// Forward = implicit GEMM over an LDS-staged spatial halo tile:
//   M = output pixels of a TH x TW (x NB images) tile, N = output channels (BN),
//   K = 9 taps x Cin, walked in chunks of CK input channels.
// Per chunk the workgroup stages the (TH+2)x(TW+2) NHWC halo (optionally read
// through a nearest x2 upsample) and the BN x (9*CK) weight slab in LDS, then
// every wave issues MFMAs whose A fragment is 8 consecutive channels of one halo
// pixel shifted by the tap and whose B fragment is 8 consecutive (tap,cin) of
// one output channel: one 16-byte ds_read each.
//   bf16: v_mfma_f32_16x16x32_bf16 (one per fragment pair)
//   f32 : v_mfma_f32_16x16x4_f32 x 8 with the k index permuted so lane group g
//         owns k = 8g..8g+7 (same LDS reads as bf16; exact fp32)
// Epilogue: accumulators -> LDS tile -> bias / leaky-relu / 2x2 pool / lrelu'
// mask / accumulate -> coalesced channel-vector stores.
// Reference: lib/layers.py:58-89 (conv*c incl. bias), lib/blocks.py:113-201.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

struct ConvParams {
  const void* x;
  const void* w;
  const float* bias;
  const void* aux;
  void* y;
  void* y2;
  int B, H, W, Hin, Win;
  int cin_p, cout, cout_p;
  int x_cs, y_cs, aux_cs, y2_cs;
  int flags;
  float slope, out_scale;
  int NB, TH, TW, tiles_x, tiles_y;
  int CK, KS, nchunks;
  int pixb, wrowb, halo_bytes;
  // split-K: blockIdx.z sums chunks [z*cps, (z+1)*cps) into fp32 slab z of ws
  float* ws;
  int cps;
  size_t slab;   // elements per slab = B*H*W*cout_p
  // PG_CONV_X_BITS: sign bits masking the input on load ([B][H][W][xb_cs bytes], conv res)
  const unsigned char* xbits;
  int xb_cs;
  int lg_tx, lg_ty;   // conv_hr: log2 of the tile counts along x and y
  int xcd_remap;      // conv3x3_kernel: XCD-aware workgroup order
  int diag;           // conv_hr: timing diagnostics (PG_HR_DIAG), 0 in every real launch
  int tpw;            // conv_hr 8-wave LDS-DMA tile: tiles per workgroup (> 1: persistent form)
  // PG_CONV_RGBW (conv_hr EF tiles): fromRGB weight gradient of the conv result
  const float* rimg;  // fp32 NCHW [B][3][H][W]
  float* rdw;         // [cout][3], accumulated
  float* rdb;         // [cout], accumulated
  float* scratch;     // det_commit scratch of the stream
  float rscale;
  // PG_CONV_RGBD: fromRGB input gradient of the conv result
  const float* rw;    // fromRGB weights [cout][3]
  float* gimg;        // fp32 NCHW [B][3][H][W], written
  float* norms;       // [B] per-sample squared norms, accumulated (or NULL)
  float f2;           // gimg = f2 * W^T gz
  // PG_CONV_RGBO: the toRGB output of the conv result (rw = toRGB weights [3][cout], gimg = the
  // image written, f2 = its He constant)
  const float* rb;    // toRGB bias [3]
};

// the RGBW operands of the next conv_hr launch on this host thread (pg_conv3x3_rgbw)
struct RgbwArgs {
  const float* img = nullptr;
  float* dw = nullptr;
  float* db = nullptr;
  float* scratch = nullptr;
  float s = 0.f;
  // RGBD
  const float* rw = nullptr;
  float* gimg = nullptr;
  float* norms = nullptr;
  float f = 0.f;
  // RGBO (rw, gimg, f as above)
  const float* rb = nullptr;
};
static thread_local RgbwArgs g_rgbw;

int cinp_of(int c) { return c <= 16 ? ((c + 7) & ~7) : ((c + 31) & ~31); }
__device__ __forceinline__ int cinp_of_dev(int c) { return c <= 16 ? ((c + 7) & ~7) : ((c + 31) & ~31); }

struct TileCfg {
  int BM, BN, NB, TH, TW;
};

TileCfg pick_tile(int H, int W, int BM, int BN) {
  TileCfg t;
  t.BM = BM;
  t.BN = BN;
  t.TW = W < 16 ? W : 16;
  t.TH = BM / t.TW;
  if (t.TH > H) t.TH = H;
  t.NB = BM / (t.TH * t.TW);
  return t;
}

template <typename T>
struct Frag;

template <>
struct Frag<bf16_t> {
  bf16x8_t v;
  __device__ __forceinline__ void load(const char* p) {
    v = *reinterpret_cast<const bf16x8_t*>(p);
  }
  static __device__ __forceinline__ void mma(const Frag& a, const Frag& b, f32x4_t& acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
  }
};

template <>
struct Frag<float> {
  f32x4_t lo, hi;
  __device__ __forceinline__ void load(const char* p) {
    lo = *reinterpret_cast<const f32x4_t*>(p);
    hi = *reinterpret_cast<const f32x4_t*>(p + 16);
  }
  static __device__ __forceinline__ void mma(const Frag& a, const Frag& b, f32x4_t& acc) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[i], b.lo[i], acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[i], b.hi[i], acc, 0, 0, 0);
  }
};

// waves along M of the 64-output-channel compile-time tiles (the 16^2 / 32^2 split-K convs):
// 2 -> four waves of 64 x 32 outputs, 4 -> eight waves of 32 x 32 (half the accumulators and
// staging registers per wave, two waves per SIMD): 16^2 512 -> 512 20.7 -> 19.1 us per launch
// at B = 4, 27.6 -> 25.2 at B = 8, step 10.084 -> 10.030 ms (profiles/r6_c64_waves_ab.txt)
#ifndef PG_C64_WM
#define PG_C64_WM 4
#endif

// CKC > 0: the channel chunk is fixed at compile time (CKC == p.CK), so the k-step loop
// unrolls and each k-step's tap / channel offset is a constant (the 4x4..64x64 convs at
// 256-512 channels are otherwise bound by that per-k-step index arithmetic)
template <typename T, int BM, int BN, int WM, int WN, int MAXV, bool TR, int CKC = 0, int TWC = 0,
          int THC = 0>
__global__ __launch_bounds__(64 * WM * WN) void conv3x3_kernel(ConvParams p) {
  // geometry: compile-time where the launch fixes it (TWC/THC/CKC > 0), else from p
  constexpr int SZ = (int)sizeof(T);
  const int cTW = TWC > 0 ? TWC : p.TW, cTH = THC > 0 ? THC : p.TH;
  const int cNB = TWC > 0 ? BM / (TWC * THC) : p.NB;
  const int cCK = CKC > 0 ? CKC : p.CK;
  const int cKS = CKC > 0 ? (9 * CKC + 31) / 32 : p.KS;
  const int cpixb = CKC > 0 ? CKC * SZ + (CKC * SZ >= 64 ? (SZ == 2 ? 32 : 16) : 0) : p.pixb;
  const int cwrowb = CKC > 0 ? cKS * 32 * SZ + (SZ == 2 ? 32 : 16) : p.wrowb;
  const int chalo = (CKC > 0 && TWC > 0) ? ((cNB * (cTH + 2) * (cTW + 2) * cpixb + 15) & ~15) : p.halo_bytes;
  constexpr int MT = BM / WM / 16;
  constexpr int NT = BN / WN / 16;
  static_assert(WM * WN == 4 || WM * WN == 8, "4 or 8 waves");
  constexpr int NTHR = 64 * WM * WN;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int g = lane >> 4, r = lane & 15;

  // XCD-aware block order (as in wgrad_bf16_kernel): every XCD owns a contiguous range of
  // logical (tile, cout block, K chunk) ids, so the workgroups that share a K chunk's
  // weights and halos run behind one L2 instead of pulling them through all eight
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (p.xcd_remap) {
    const int ox = gridDim.x, oy = gridDim.y;
    const int n = ox * oy * gridDim.z;
    const int h = bx + ox * (by + oy * bz);
    const int xcd = h & 7, slot = h >> 3, q = n >> 3, rr = n & 7;
    const int Lg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + slot;
    bx = Lg % ox;
    by = (Lg / ox) % oy;
    bz = Lg / (ox * oy);
  }
  int t = bx;
  const int tx0 = (t % p.tiles_x) * cTW;
  t /= p.tiles_x;
  const int ty0 = (t % p.tiles_y) * cTH;
  t /= p.tiles_y;
  const int b0 = t * cNB;
  const int n0 = by * BN;

  const int TW2 = cTW + 2;
  const int HW2 = (cTH + 2) * TW2;
  const int npix_halo = cNB * HW2;
  char* halo = smem;
  char* wl = smem + chalo;

  int hoff[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int pm = wm * (BM / WM) + mt * 16 + r;
    const int tx = pm % cTW, ty = (pm / cTW) % cTH, nb = pm / (cTW * cTH);
    hoff[mt] = ((nb * (cTH + 2) + ty) * TW2 + tx) * cpixb;
  }

  f32x4_t acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const bool ups = (p.flags & PG_CONV_UPS_IN) != 0;
  const int vpp = cCK * (int)sizeof(T) / 16;  // 16-byte vectors per halo pixel / per tap
  const int ntap_pad = cKS * 32 / cCK;
  constexpr int EPV = 16 / (int)sizeof(T);     // elements per 16-byte vector

  // Staging plan, computed once: this thread's 16-byte vectors of the halo tile and of
  // the weight slab (element offset in x / w without the chunk's channel base, -1 = zero
  // fill) and their LDS byte offsets.  Each chunk is then fetched into registers one
  // chunk ahead (issued before the MFMAs of the current chunk, written to LDS after).
  int soff[MAXV], loff[MAXV];
  unsigned wmask = 0;
  const int nhv = npix_halo * vpp;
  const int ntot = nhv + BN * ntap_pad * vpp;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    const int i = tid + NTHR * j;
    soff[j] = -1;
    loff[j] = -1;
    if (i < nhv) {
      const int hp = i / vpp, v = i - hp * vpp;
      const int nb = hp / HW2, rem = hp - nb * HW2;
      const int hy = rem / TW2, hx = rem - hy * TW2;
      const int b = b0 + nb, yy = ty0 + hy - 1, xx = tx0 + hx - 1;
      loff[j] = hp * cpixb + v * 16;
      if (b < p.B && yy >= 0 && yy < p.H && xx >= 0 && xx < p.W) {
        const int sy = ups ? (yy >> 1) : yy, sx = ups ? (xx >> 1) : xx;
        soff[j] = (int)((((size_t)b * p.Hin + sy) * p.Win + sx) * p.x_cs + v * EPV);
      }
    } else if (i < ntot) {
      const int iw = i - nhv;
      const int row = iw / (ntap_pad * vpp), rem = iw - row * (ntap_pad * vpp);
      const int tap = rem / vpp, v = rem - tap * vpp;
      const int n = n0 + row;
      loff[j] = chalo + row * cwrowb + tap * cCK * (int)sizeof(T) + v * 16;
      wmask |= 1u << j;
      if (tap < 9 && n < p.cout_p) soff[j] = (n * 9 + tap) * p.cin_p + v * EPV;
    }
  }
  const T* xs = reinterpret_cast<const T*>(p.x);
  const T* wsrc = reinterpret_cast<const T*>(p.w);
  u32x4_t buf[MAXV];
  auto prefetch = [&](int c0) {
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
      // branch-free (clamped address; the zero fill is applied at the LDS write): a load
      // under a per-lane branch, or a select right after it, makes hipcc wait for it
      const T* base = ((wmask >> j) & 1u) ? wsrc : xs;
      buf[j] = *reinterpret_cast<const u32x4_t*>(base + (soff[j] >= 0 ? soff[j] + c0 : 0));
    }
  };

  const int ch_begin = bz * p.cps;
  const int ch_end = min(p.nchunks, ch_begin + p.cps);
  if (ch_begin < ch_end) prefetch(ch_begin * cCK);
  for (int ch = ch_begin; ch < ch_end; ++ch) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
      if (loff[j] >= 0)
        *reinterpret_cast<u32x4_t*>(smem + loff[j]) = soff[j] >= 0 ? buf[j] : u32x4_t{0u, 0u, 0u, 0u};
    __syncthreads();
    if (ch + 1 < ch_end) prefetch((ch + 1) * cCK);
    auto kstep = [&](int ks) {
      const int CKr = cCK;
      const int k0 = ks * 32 + 8 * g;
      int tap = k0 / CKr;
      const int c = k0 - tap * CKr;
      if (tap > 8) tap = 8;  // padded taps: weights are zero, read real data
      const int toff = ((tap / 3) * TW2 + (tap % 3)) * cpixb + c * (int)sizeof(T);
      Frag<T> bfr[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        bfr[nt].load(wl + (wn * (BN / WN) + nt * 16 + r) * cwrowb + k0 * (int)sizeof(T));
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        Frag<T> afr;
        afr.load(halo + hoff[mt] + toff);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          if constexpr (TR)
            Frag<T>::mma(bfr[nt], afr, acc[mt][nt]);   // D[cout][pixel]
          else
            Frag<T>::mma(afr, bfr[nt], acc[mt][nt]);   // D[pixel][cout]
        }
      }
    };
    if constexpr (CKC > 0) {
#pragma unroll
      for (int ks = 0; ks < (9 * CKC + 31) / 32; ++ks) kstep(ks);
    } else {
      for (int ks = 0; ks < cKS; ++ks) kstep(ks);
    }
  }

  if constexpr (TR) {
    // ---- direct epilogue: lane holds 4 consecutive output channels of one pixel, so a
    // wave-instruction writes 16 pixels x 4 lane-groups x 8 B = whole pixel rows
    const bool has_bias = !p.ws && (p.flags & PG_CONV_BIAS) != 0;
    const bool do_lrelu = !p.ws && (p.flags & PG_CONV_LRELU) != 0;
    if (p.flags & PG_CONV_PIXNORM) {
      // PixelNorm over the cout channels of each pixel (WN == 1, n0 == 0, cout_p <= BN)
      T* y = reinterpret_cast<T*>(p.y);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int pm = wm * (BM / WM) + mt * 16 + r;
        const int tx = pm % cTW, ty = (pm / cTW) % cTH, nb = pm / (cTW * cTH);
        const int b = b0 + nb;
        const size_t pix = ((size_t)b * p.H + ty0 + ty) * p.W + tx0 + tx;
        float v[NT][4];
        float ss = 0.f;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int n = nt * 16 + 4 * g + j;
            float u = acc[mt][nt][j] + ((has_bias && n < p.cout) ? p.bias[n] : 0.f);
            if (do_lrelu) u = lrelu_f(u, p.slope);
            if constexpr (sizeof(T) == 2) u = bf2f(f2bf(u));   // as stored
            v[nt][j] = n < p.cout ? u : 0.f;
            ss += v[nt][j] * v[nt][j];
          }
        ss += __shfl_xor(ss, 16, 64);
        ss += __shfl_xor(ss, 32, 64);
        const float rn = rsqrtf(ss / (float)p.cout + 1e-8f);
        if (b >= p.B) continue;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int n = nt * 16 + 4 * g;
          if (n >= p.cout) continue;
          float o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = v[nt][j] * rn;
          Ty<T>::st4(y + pix * p.y_cs + n, o);
        }
        if (p.y2 && g == 0) reinterpret_cast<float*>(p.y2)[pix] = rn;
      }
      return;
    }
    const bool do_mask = (p.flags & PG_CONV_MASK) != 0;
    const bool do_acc = (p.flags & PG_CONV_ACCUM) != 0;
    const bool pool = !p.ws && (p.flags & PG_CONV_POOL) != 0;
    T* y = reinterpret_cast<T*>(p.y);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + wn * (BN / WN) + nt * 16 + 4 * g;
      const bool nok = n < p.cout;
      float bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[j] = (has_bias && nok) ? p.bias[n + j] : 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int pm = wm * (BM / WM) + mt * 16 + r;
        const int tx = pm % cTW, ty = (pm / cTW) % cTH, nb = pm / (cTW * cTH);
        const int b = b0 + nb;
        const size_t pix = ((size_t)b * p.H + ty0 + ty) * p.W + tx0 + tx;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = acc[mt][nt][j] + bv[j];
          if (do_lrelu) v[j] = lrelu_f(v[j], p.slope);
        }
        if (p.ws) {
          if (b < p.B && n < p.cout_p)
            *reinterpret_cast<f32x4_t*>(p.ws + bz * p.slab + pix * p.cout_p + n) =
                f32x4_t{v[0], v[1], v[2], v[3]};
          continue;
        }
        if (!pool) {
          if (b < p.B && nok) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] *= p.out_scale;
            if (do_mask) {
              float a[4];
              Ty<T>::ld4(reinterpret_cast<const T*>(p.aux) + pix * p.aux_cs + n, a);
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] *= lmask_f(a[j], p.slope);
            }
            T* dst = y + pix * p.y_cs + n;
            if (do_acc) {
              float o[4];
              Ty<T>::ld4(dst, o);
#pragma unroll
              for (int j = 0; j < 4; ++j) v[j] += o[j];
            }
            Ty<T>::st4(dst, v);
          }
        } else {
          if (p.y2 && b < p.B && nok && !(cTW >= 16 && (mt & 1)))
            Ty<T>::st4(reinterpret_cast<T*>(p.y2) + pix * p.y2_cs + n, v);
          // 2x2 sum: horizontal partner = lane ^ 1; vertical = lane ^ TW (TW < 16) or the
          // next 16-pixel subtile (TW == 16, handled when mt is the even row)
          float h[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) h[j] = v[j] + __shfl_xor(v[j], 1, 64);
          if (cTW < 16) {
#pragma unroll
            for (int j = 0; j < 4; ++j) h[j] += __shfl_xor(h[j], cTW, 64);
          } else {
            if (mt & 1) continue;
            if (mt + 1 < MT) {
              float u[4];
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                u[j] = acc[mt + 1][nt][j] + bv[j];
                if (do_lrelu) u[j] = lrelu_f(u[j], p.slope);
              }
              if (p.y2 && b < p.B && nok)
                Ty<T>::st4(reinterpret_cast<T*>(p.y2) + (pix + p.W) * p.y2_cs + n, u);
#pragma unroll
              for (int j = 0; j < 4; ++j) h[j] += u[j] + __shfl_xor(u[j], 1, 64);
            }
          }
          if ((tx & 1) == 0 && (ty & 1) == 0 && b < p.B && nok) {
            const size_t op = ((size_t)b * (p.H >> 1) + ((ty0 + ty) >> 1)) * (p.W >> 1) +
                              ((tx0 + tx) >> 1);
#pragma unroll
            for (int j = 0; j < 4; ++j) h[j] *= p.out_scale;
            T* dst = y + op * p.y_cs + n;
            if (do_acc) {
              float o[4];
              Ty<T>::ld4(dst, o);
#pragma unroll
              for (int j = 0; j < 4; ++j) h[j] += o[j];
            }
            Ty<T>::st4(dst, h);
          }
        }
      }
    }
    return;
  }

  // ---- epilogue: accumulators -> LDS tile [BM][BN+4] fp32 (bias, lrelu applied)
  __syncthreads();
  float* ot = reinterpret_cast<float*>(smem);
  constexpr int ORS = BN + 4;
  const bool has_bias = !p.ws && (p.flags & PG_CONV_BIAS) != 0;   // split-K: raw sums
  const bool do_lrelu = !p.ws && (p.flags & PG_CONV_LRELU) != 0;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int nl = wn * (BN / WN) + nt * 16 + r;
    const int n = n0 + nl;
    const float bv = (has_bias && n < p.cout) ? p.bias[n] : 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pm = wm * (BM / WM) + mt * 16 + 4 * g + j;
        float v = acc[mt][nt][j] + bv;
        if (do_lrelu) v = lrelu_f(v, p.slope);
        ot[pm * ORS + nl] = v;
      }
    }
  }
  __syncthreads();

  constexpr int NV = BN / 4;
  const bool do_mask = (p.flags & PG_CONV_MASK) != 0;
  const bool do_acc = (p.flags & PG_CONV_ACCUM) != 0;
  T* y = reinterpret_cast<T*>(p.y);
  if (p.ws) {   // split-K partial: raw fp32 sums to this split's slab, [pixel][cout_p]
    float* slab = p.ws + bz * p.slab;
    for (int i = tid; i < BM * NV; i += NTHR) {
      const int pm = i / NV, cv = (i - pm * NV) * 4;
      const int n = n0 + cv;
      if (n >= p.cout_p) continue;
      const int tx = pm % cTW, ty = (pm / cTW) % cTH, nb = pm / (cTW * cTH);
      const int b = b0 + nb;
      if (b >= p.B) continue;
      const size_t pix = ((size_t)b * p.H + ty0 + ty) * p.W + tx0 + tx;
      *reinterpret_cast<f32x4_t*>(slab + pix * p.cout_p + n) =
          *reinterpret_cast<const f32x4_t*>(ot + pm * ORS + cv);
    }
  } else if (!(p.flags & PG_CONV_POOL)) {
    for (int i = tid; i < BM * NV; i += NTHR) {
      const int pm = i / NV, cv = (i - pm * NV) * 4;
      const int n = n0 + cv;
      if (n >= p.cout) continue;
      const int tx = pm % cTW, ty = (pm / cTW) % cTH, nb = pm / (cTW * cTH);
      const int b = b0 + nb;
      if (b >= p.B) continue;
      const size_t pix = ((size_t)b * p.H + ty0 + ty) * p.W + tx0 + tx;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = ot[pm * ORS + cv + q] * p.out_scale;
      if (do_mask) {
        float a[4];
        Ty<T>::ld4(reinterpret_cast<const T*>(p.aux) + pix * p.aux_cs + n, a);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] *= lmask_f(a[q], p.slope);
      }
      T* dst = y + pix * p.y_cs + n;
      if (do_acc) {
        float o[4];
        Ty<T>::ld4(dst, o);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += o[q];
      }
      Ty<T>::st4(dst, v);
    }
  } else {
    const int PTW = cTW >> 1, PTH = cTH >> 1;
    const int Ho = p.H >> 1, Wo = p.W >> 1;
    T* y2 = reinterpret_cast<T*>(p.y2);
    for (int i = tid; i < (BM / 4) * NV; i += NTHR) {
      const int pp = i / NV, cv = (i - pp * NV) * 4;
      const int n = n0 + cv;
      if (n >= p.cout) continue;
      const int ptx = pp % PTW, pty = (pp / PTW) % PTH, nb = pp / (PTW * PTH);
      const int b = b0 + nb;
      if (b >= p.B) continue;
      const int pm00 = (nb * cTH + 2 * pty) * cTW + 2 * ptx;
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        v[q] = ot[pm00 * ORS + cv + q] + ot[(pm00 + 1) * ORS + cv + q] +
               ot[(pm00 + cTW) * ORS + cv + q] + ot[(pm00 + cTW + 1) * ORS + cv + q];
      if (y2) {
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 2; ++dx) {
            const size_t fpix = ((size_t)b * p.H + ty0 + 2 * pty + dy) * p.W + tx0 + 2 * ptx + dx;
            float f[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) f[q] = ot[(pm00 + dy * cTW + dx) * ORS + cv + q];
            Ty<T>::st4(y2 + fpix * p.y2_cs + n, f);
          }
      }
      const size_t pix = ((size_t)b * Ho + (ty0 >> 1) + pty) * Wo + (tx0 >> 1) + ptx;
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] *= p.out_scale;
      T* dst = y + pix * p.y_cs + n;
      if (do_acc) {
        float o[4];
        Ty<T>::ld4(dst, o);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += o[q];
      }
      Ty<T>::st4(dst, v);
    }
  }
}

// Split-K reduction + epilogue: y = out_scale * post(sum_z slab_z + bias) with the same
// flag semantics as conv3x3_kernel's epilogue (bias, lrelu, 2x2 pool (+ y2), mask, accum).
// PIXNORM (no pool / mask / accumulate): one wave per pixel, the wave's lanes hold all
// cout channels (4 per lane and round); bias, leaky relu, bf16 rounding as stored, then
// y = v * r with r = rsqrt(mean_c v^2 + 1e-8) (lib/layers.py:8-14), r to y2 (fp32 per pixel)
template <typename T>
__device__ void splitk_pixnorm(const ConvParams& p, int splits) {
  const int lane = threadIdx.x & 63;
  const int npix = p.B * p.H * p.W;
  const int pix = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (pix >= npix) return;   // wave-uniform
  constexpr int MAXR = 4;    // cout <= 1024
  float v[MAXR][4];
  float ss = 0.f;
#pragma unroll
  for (int rr = 0; rr < MAXR; ++rr) {
    const int c = (rr * 64 + lane) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) v[rr][q] = 0.f;
    if (c >= p.cout) continue;
    const float* src = p.ws + (size_t)pix * p.cout_p + c;
    float a[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] = (p.flags & PG_CONV_BIAS) ? p.bias[c + q] : 0.f;
    for (int z = 0; z < splits; ++z) {
      const f32x4_t t = *reinterpret_cast<const f32x4_t*>(src + z * p.slab);
#pragma unroll
      for (int q = 0; q < 4; ++q) a[q] += t[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float u = (p.flags & PG_CONV_LRELU) ? lrelu_f(a[q], p.slope) : a[q];
      if constexpr (sizeof(T) == 2) u = bf2f(f2bf(u));
      v[rr][q] = u;
      ss += u * u;
    }
  }
  ss = wave_sum(ss);
  const float rn = rsqrtf(ss / (float)p.cout + 1e-8f);
  T* y = reinterpret_cast<T*>(p.y);
#pragma unroll
  for (int rr = 0; rr < MAXR; ++rr) {
    const int c = (rr * 64 + lane) * 4;
    if (c >= p.cout) continue;
    float o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = v[rr][q] * rn;
    Ty<T>::st4(y + (size_t)pix * p.y_cs + c, o);
  }
  if (p.y2 && lane == 0) reinterpret_cast<float*>(p.y2)[pix] = rn;
}

template <typename T>
__global__ void conv_splitk_epilogue(ConvParams p, int splits) {
  if (p.flags & PG_CONV_PIXNORM) {
    splitk_pixnorm<T>(p, splits);
    return;
  }
  const int nv = p.cout >> 2;
  const bool pool = (p.flags & PG_CONV_POOL) != 0;
  const int Ho = pool ? p.H >> 1 : p.H, Wo = pool ? p.W >> 1 : p.W;
  const size_t n = (size_t)p.B * Ho * Wo * nv;
  T* y = reinterpret_cast<T*>(p.y);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % nv) * 4;
    const size_t op = i / nv;
    const int xo = (int)(op % Wo), yo = (int)((op / Wo) % Ho), b = (int)(op / ((size_t)Wo * Ho));
    float bsv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bsv[q] = (p.flags & PG_CONV_BIAS) ? p.bias[c + q] : 0.f;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    const int np = pool ? 4 : 1;
    for (int k = 0; k < np; ++k) {
      const int yy = pool ? 2 * yo + (k >> 1) : yo, xx = pool ? 2 * xo + (k & 1) : xo;
      const size_t pix = ((size_t)b * p.H + yy) * p.W + xx;
      float a[4] = {bsv[0], bsv[1], bsv[2], bsv[3]};
      const float* src = p.ws + pix * p.cout_p + c;
      int z = 0;
      // 4 slabs per round: the loads are issued together (one memory latency per round),
      // the sum stays in slab order
      for (; z + 4 <= splits; z += 4) {
        f32x4_t t[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) t[u] = *reinterpret_cast<const f32x4_t*>(src + (z + u) * p.slab);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int q = 0; q < 4; ++q) a[q] += t[u][q];
      }
      for (; z < splits; ++z) {
        const f32x4_t t = *reinterpret_cast<const f32x4_t*>(src + z * p.slab);
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] += t[q];
      }
      if (p.flags & PG_CONV_LRELU)
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = lrelu_f(a[q], p.slope);
      if (pool && p.y2) Ty<T>::st4(reinterpret_cast<T*>(p.y2) + pix * p.y2_cs + c, a);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += a[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] *= p.out_scale;
    if (p.flags & PG_CONV_MASK) {
      float m[4];
      Ty<T>::ld4(reinterpret_cast<const T*>(p.aux) + op * p.aux_cs + c, m);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] *= lmask_f(m[q], p.slope);
    }
    T* dst = y + op * p.y_cs + c;
    if (p.flags & PG_CONV_ACCUM) {
      float o[4];
      Ty<T>::ld4(dst, o);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += o[q];
    }
    Ty<T>::st4(dst, v);
  }
}

// --------------------------------------------------------------------------
// Weight gradient: dW[o][c][tap] += scale * sum_p gz[p][o] * x[p + off(tap)][c]
// One workgroup = 32 output channels x 32 input channels x 9 taps, walking a
// contiguous range of spatial pixel tiles (split over blockIdx.z); each split writes
// its partial sums to a workspace slab (summed in slab order by wgrad_slab_reduce), or, with
// one split, adds them to dw directly.  MFMA v_mfma_f32_16x16x4_f32 with
// K = pixels: A[o][p] and B[p][c] are one ds_read_b32 each from the
// pixel-major LDS tiles (exact fp32; bf16 inputs are widened on staging).
// --------------------------------------------------------------------------
struct WgParams {
  const void* x;
  const void* gz;
  float* dw;
  float* db;
  float* ws;       // split slabs [splits][cout*cin*9 + cout], or NULL (one split: direct)
  size_t slab;
  int B, H, W, Hin, Win;
  int cin, cout, x_cs, gz_cs;
  int ups;
  float scale;
  int NB, TH, TW, tiles_x, tiles_y, ntiles, tiles_per_split;
};

constexpr int WG_BO = 32, WG_BC = 32, WG_BP = 128, WG_RS = 33;

template <typename T>
__global__ __launch_bounds__(256) void wgrad3x3_kernel(WgParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* gzl = reinterpret_cast<float*>(smem);  // [WG_BP][WG_RS]
  float* hal = gzl + WG_BP * WG_RS;               // [NB*(TH+2)*(TW+2)][WG_RS]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int o0 = blockIdx.x * WG_BO, cc0 = blockIdx.y * WG_BC;
  const int om = (wid >> 1) * 16, cn = (wid & 1) * 16;
  const int TW2 = p.TW + 2, HW2 = (p.TH + 2) * TW2;
  const T* x = reinterpret_cast<const T*>(p.x);
  const T* gz = reinterpret_cast<const T*>(p.gz);

  f32x4_t acc[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) acc[q] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;   // bias gradient of output channel o0 + tid (c-tile 0 only)
  const bool do_db = p.db && blockIdx.y == 0 && tid < WG_BO;

  const int t_begin = blockIdx.z * p.tiles_per_split;
  const int t_end = min(p.ntiles, t_begin + p.tiles_per_split);
  for (int t = t_begin; t < t_end; ++t) {
    int tt = t;
    const int tx0 = (tt % p.tiles_x) * p.TW;
    tt /= p.tiles_x;
    const int ty0 = (tt % p.tiles_y) * p.TH;
    tt /= p.tiles_y;
    const int b0 = tt * p.NB;
    __syncthreads();
    // gz tile: WG_BP pixels x 32 output channels
    for (int i = tid; i < WG_BP * WG_BO; i += 256) {
      const int pm = i / WG_BO, oc = i - pm * WG_BO;
      const int tx = pm % p.TW, ty = (pm / p.TW) % p.TH, nb = pm / (p.TW * p.TH);
      const int b = b0 + nb, o = o0 + oc;
      float v = 0.f;
      if (b < p.B && o < p.cout)
        v = Ty<T>::ld(gz + (((size_t)b * p.H + ty0 + ty) * p.W + tx0 + tx) * p.gz_cs + o);
      gzl[pm * WG_RS + oc] = v;
    }
    // x halo: NB*(TH+2)*(TW+2) pixels x 32 input channels
    for (int i = tid; i < p.NB * HW2 * WG_BC; i += 256) {
      const int hp = i / WG_BC, ci = i - hp * WG_BC;
      const int nb = hp / HW2, rem = hp - nb * HW2;
      const int hy = rem / TW2, hx = rem - hy * TW2;
      const int b = b0 + nb, yy = ty0 + hy - 1, xx = tx0 + hx - 1, c = cc0 + ci;
      float v = 0.f;
      if (b < p.B && c < p.cin && yy >= 0 && yy < p.H && xx >= 0 && xx < p.W) {
        const int sy = p.ups ? (yy >> 1) : yy, sx = p.ups ? (xx >> 1) : xx;
        v = Ty<T>::ld(x + (((size_t)b * p.Hin + sy) * p.Win + sx) * p.x_cs + c);
      }
      hal[hp * WG_RS + ci] = v;
    }
    __syncthreads();
    if (do_db)
      for (int pm = 0; pm < WG_BP; ++pm) bsum += gzl[pm * WG_RS + tid];
    for (int k0 = 0; k0 < WG_BP; k0 += 4) {
      const int pm = k0 + g;
      const int tx = pm % p.TW, ty = (pm / p.TW) % p.TH, nb = pm / (p.TW * p.TH);
      const int hbase = (nb * (p.TH + 2) + ty) * TW2 + tx;
      const float a = gzl[pm * WG_RS + om + r];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const float bb = hal[(hbase + (tap / 3) * TW2 + (tap % 3)) * WG_RS + cn + r];
        acc[tap] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb, acc[tap], 0, 0, 0);
      }
    }
  }
  float* slab = p.ws ? p.ws + blockIdx.z * p.slab : nullptr;
  if (do_db && o0 + tid < p.cout) {
    if (slab) slab[(size_t)p.cout * p.cin * 9 + o0 + tid] = bsum;
    else p.db[o0 + tid] += bsum * p.scale;   // one split: the sole writer
  }
  // acc[tap][j]: row (o) = om + 4g + j, col (c) = cn + r
  const int c = cc0 + cn + r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = o0 + om + 4 * g + j;
    if (o < p.cout && c < p.cin) {
      const size_t e = ((size_t)o * p.cin + c) * 9;
      if (slab) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) slab[e + tap] = acc[tap][j];
      } else {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) p.dw[e + tap] += acc[tap][j] * p.scale;
      }
    }
  }
}

// the fp32 weight gradient's split of the pixel tiles (enough workgroups to fill the chip)
static int wgrad_f32_splits(const pg_conv_desc* d, int* tiles_per_split) {
  TileCfg tc = pick_tile(d->H, d->W, WG_BP, 32);
  const int ntiles = pg_cdiv(d->B, tc.NB) * (d->W / tc.TW) * (d->H / tc.TH);
  const int ot = pg_cdiv(d->cout, WG_BO), ct = pg_cdiv(d->cin, WG_BC);
  int splits = pg_cdiv(2048, ot * ct);
  if (splits > ntiles) splits = ntiles;
  if (splits < 1) splits = 1;
  *tiles_per_split = pg_cdiv(ntiles, splits);
  return pg_cdiv(ntiles, *tiles_per_split);
}
static size_t wgrad_f32_ws_bytes(const pg_conv_desc* d) {
  int tps;
  const int splits = wgrad_f32_splits(d, &tps);
  return splits > 1 ? (size_t)splits * ((size_t)d->cout * d->cin * 9 + d->cout) * sizeof(float) : 0;
}

// --------------------------------------------------------------------------
// bf16 weight gradient on v_mfma_f32_16x16x32_bf16.  GEMM view: M = cout,
// N = 9 taps x cin, K = pixels.  Both operands are staged pixel-major in LDS
// ([pixel][o] and the [halo pixel][c] tile) and the k-contiguous fragments are
// read with ds_read_b64_tr_b16 (gfx950 transposed read: 16 lanes fetch a 4-row x
// 16-column block, lane i receives column i), whose per-lane row addresses also
// apply the 3x3 tap shift.  A wave owns MO x NC 16x16 (o, c) blocks for all 9
// taps; KW waves split the pixel k-steps and are reduced through LDS.
//
// Pipeline: the global loads of pixel tile t+1 are issued into registers before
// the MFMAs of tile t (one LDS buffer, two barriers per tile), so every resident
// workgroup keeps a tile of loads in flight.  The bias gradient is summed from
// the staged gz registers (no extra LDS pass).
//
// Reduction over pixel splits (blockIdx.z), chosen on the host:
//   WG_DIRECT : one split -> plain coalesced read-modify-write of dw / db
//   WG_SLABS  : split z writes an fp32 partial slab of the workspace; a second
//               kernel sums the slabs into dw / db in slab order
// (no workspace for the slabs -> the plan falls back to one split: results never depend on
// the order workgroups finish)
// Writes go through a per-wave LDS transpose so that each wave instruction covers
// contiguous [c][tap] runs of one OIHW row.
// --------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4_t;
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;

__device__ __forceinline__ bf16x8_t tr_read8(const bf16_t* lo, const bf16_t* hi) {
  bf16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)lo);
  bf16x4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)hi);
  return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

enum { WG_DIRECT = 0, WG_SLABS = 1 };

struct WgBParams {
  const bf16_t* x;
  const bf16_t* gz;
  float* dw;
  float* db;
  float* ws;       // WG_SLABS: [splits][slab] fp32, slab = cout*cin*9 + cout
  size_t slab;
  int mode;
  int B, H, W, Hin, Win;
  int cin, cout, x_cs, gz_cs;
  int ups;
  float scale;
  int NB, TH, TW, tiles_x, tiles_y, ntiles, tiles_per_split;
  int GZS, HS, halo_elems, hpad;
  int lg_tx, lg_ty;   // log2 of tiles_x / tiles_y, -1 when not a power of two
  // PG_CONV_GZ_BITS: gz at half resolution, masked by lrelu'(gzb) at full resolution
  const unsigned char* gzb;
  int gzb_cs;
  float slope;
  int xcd_remap;      // XCD-aware workgroup order (see the kernel prologue)
};

// pixels per staged tile: 128, or 256 (16x16) for the wide tiles at W >= 16 (half the
// per-tile staging / barrier overhead per MFMA)
constexpr int WGB_BP = 128;
constexpr int wgb_maxhalo(int bp) { return bp == 128 ? 288 : 18 * 18; }   // pick_tile geometry

__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

#ifndef PG_WG_PRE_ALL
#define PG_WG_PRE_ALL 1
#endif
template <int MO, int NC, int WMO, int WNC, int PD, int WPE, bool GZB, int BP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
void wgrad_bf16_kernel(WgBParams p) {
  // precomputed per-lane staging offsets + shifts for the tile origin (every tile when
  // PG_WG_PRE_ALL; the 64-bit per-load address math of the other form put each wide-tile
  // halo load behind its own branch, ~600 instructions of staging per 72 MFMAs)
  constexpr bool PRE = PG_WG_PRE_ALL || MO < 4;
  constexpr int KW = 4 / (WMO * WNC);
  constexpr int BO = WMO * MO * 16, BC = WNC * NC * 16;
  constexpr int GV = BO / 8, HV = BC / 8;
  constexpr int NGZ = BP * GV / 256;                      // gz vectors per thread
  constexpr int NH = (wgb_maxhalo(BP) * HV + 255) / 256;  // halo vectors per thread (max)
  static_assert(NGZ * 256 == BP * GV, "gz staging must tile the workgroup");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* gzl = reinterpret_cast<bf16_t*>(smem);
  // row r of a tile lives at r*S + (r/8)*64 elements: with S = 16 (mod 32) elements the
  // transposed fragment reads are bank-conflict free (tools/lds_banks.py)
  // halo rows: BC = 16 unpadded, plus p.hpad elements per 8 rows (64 for 16- and 8-wide
  // tiles, 0 for 4x4): 1 LDS cycle per 32-lane group on the tap-shifted reads at 16x8
  // tiles, was 2 with 48-byte rows (tools/lds_banks.py wgrad_halo)
  constexpr int GZS = BO + (BO > 16 ? 16 : 0), HS = BC == 16 ? 16 : BC + 16;
  const int hpad = p.hpad;
  auto grow = [](int r) { return r * GZS + (r >> 3) * 64; };
  auto hrow = [hpad](int r) { return r * HS + (r >> 3) * hpad; };
  bf16_t* hal = gzl + grow(BP);
  const int hscr = hrow(p.halo_elems);   // 16-B scratch slot behind the halo (see store_tile)
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid % KW, wmn = wid / KW;
  const int wo = wmn / WNC, wc = wmn % WNC;
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pq = i16 & 3;
  // XCD-aware block order: consecutive workgroups go to different XCDs (8, round robin),
  // so the ot x ct workgroups of one pixel split (which stage the same gz / x tiles) would
  // each pull them through a different L2.  Remap so every XCD owns a contiguous range of
  // logical ids (bijective for any grid size): a split's workgroups share one L2.
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (p.xcd_remap) {
    const int ox = gridDim.x, oy = gridDim.y;
    const int n = ox * oy * gridDim.z;
    const int h = bx + ox * (by + oy * bz);
    const int xcd = h & 7, slot = h >> 3, q = n >> 3, rr = n & 7;
    const int L = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + slot;
    bx = L % ox;
    by = (L / ox) % oy;
    bz = L / (ox * oy);
  }
  const int o0 = bx * BO, c0 = by * BC;
  const int TW2 = p.TW + 2, HW2 = (p.TH + 2) * TW2;
  const int nhalo = p.halo_elems * HV;

  f32x4_t acc[MO][NC][9];
#pragma unroll
  for (int a = 0; a < MO; ++a)
#pragma unroll
    for (int b = 0; b < NC; ++b)
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[a][b][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const bool do_db = p.db && by == 0;
  float bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs[e] = 0.f;

  // per-thread staging plan (fixed across tiles; TH, TW even so the upsample's floor
  // shift splits over tile origin + offset): gz element k -> (pixel offset, image),
  // halo element k -> packed (image, hy, hx, channel vector) or -1
  constexpr bool gz_bits = GZB;   // gz = up2(g) * lrelu'(bits) (PG_CONV_GZ_BITS)
  const int gH = gz_bits ? p.H >> 1 : p.H, gW = gz_bits ? p.W >> 1 : p.W;
  int gzrel[NGZ], gznb[NGZ], hpk[NH], gbrel[NGZ], hrel[NH];
#pragma unroll
  for (int k = 0; k < NGZ; ++k) {
    const int i = tid + k * 256;
    const int pm = i / GV, v = i - pm * GV;
    const int tx = pm % p.TW, ty = (pm / p.TW) % p.TH, nb = pm / (p.TW * p.TH);
    const int gs = gz_bits ? 1 : 0;
    gzrel[k] = ((nb * gH + (ty >> gs)) * gW + (tx >> gs)) * p.gz_cs + 8 * v;
    gbrel[k] = ((nb * p.H + ty) * p.W + tx) * p.gzb_cs + ((o0 + 8 * v) >> 3);
    gznb[k] = (o0 + 8 * v < p.cout) ? nb : 1 << 20;
  }
#pragma unroll
  for (int k = 0; k < NH; ++k) {
    const int i = tid + k * 256;
    hpk[k] = -1;
    if (i < nhalo) {
      const int hp = i / HV, v = i - hp * HV;
      const int nb = hp / HW2, rem = hp - nb * HW2;
      const int hy = rem / TW2, hx = rem - hy * TW2;
      if (c0 + 8 * v < p.x_cs) hpk[k] = (nb << 24) | (hy << 16) | (hx << 8) | v;
    }
    // element offset from the tile's input origin (tile origins are even, so the
    // upsample's floor shift splits: (t0 + h - 1) >> 1 = t0 / 2 + ((h - 1) >> 1))
    const int pk = hpk[k] < 0 ? 0 : hpk[k];
    const int ys = p.ups ? 1 : 0;
    if constexpr (PRE) hrel[k] = (((pk >> 24) * p.Hin + ((((pk >> 16) & 0xff) - 1) >> ys)) * p.Win +
               ((((pk >> 8) & 0xff) - 1) >> ys)) * p.x_cs + 8 * (pk & 0xff);
  }
  // ok masks of a loaded tile: bit k of gz vector k / halo vector k (zero fill at the
  // LDS write, so the loaded registers are not touched before then)
  auto load_tile = [&](int t, u32x4_t (&rg)[NGZ], u32x4_t (&rh)[NH], int (&rb)[NGZ],
                       unsigned& gok, unsigned& hok) {
    // tile -> origin (wave-uniform, scalar; shifts where the tile counts are powers of 2)
    constexpr bool sh = PRE;
    const int tx0 = (sh && p.lg_tx >= 0 ? (t & (p.tiles_x - 1)) : t % p.tiles_x) * p.TW;
    const int tt = sh && p.lg_tx >= 0 ? t >> p.lg_tx : t / p.tiles_x;
    const int ty0 = (sh && p.lg_ty >= 0 ? (tt & (p.tiles_y - 1)) : tt % p.tiles_y) * p.TH;
    const int b0 = (sh && p.lg_ty >= 0 ? tt >> p.lg_ty : tt / p.tiles_y) * p.NB;
    const int gs = gz_bits ? 1 : 0;
    gok = 0;
    hok = 0;
    const bf16_t* gzt = p.gz + (((size_t)b0 * gH + (ty0 >> gs)) * gW + (tx0 >> gs)) * p.gz_cs + o0;
    const unsigned char* gbt =
        gz_bits ? p.gzb + (((size_t)b0 * p.H + ty0) * p.W + tx0) * p.gzb_cs : nullptr;
#pragma unroll
    for (int k = 0; k < NGZ; ++k) {
      // branch-free, as in conv_hr's fetch_halo: clamped address, zero fill at the LDS write
      const bool ok = b0 + gznb[k] < p.B;
      rg[k] = *reinterpret_cast<const u32x4_t*>(ok ? gzt + gzrel[k] : p.gz);
      if constexpr (gz_bits) rb[k] = *(ok ? gbt + gbrel[k] : p.gzb);
      gok |= (ok ? 1u : 0u) << k;
    }
    const int ys = p.ups ? 1 : 0;
    // the tile's input origin (scalar) + the lane's precomputed offset
    const bf16_t* xt = PRE ? p.x + c0 + (((size_t)b0 * p.Hin + (ty0 >> ys)) * p.Win + (tx0 >> ys)) * p.x_cs
                              : p.x;
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      const int pk = hpk[k];
      const int yy = ty0 + ((pk >> 16) & 0xff) - 1, xx = tx0 + ((pk >> 8) & 0xff) - 1;
      const bool ok = pk >= 0 && b0 + (pk >> 24) < p.B && (unsigned)yy < (unsigned)p.H &&
                      (unsigned)xx < (unsigned)p.W;
      if constexpr (PRE) {   // precomputed offsets (A/B: -7..-13 % at 1024^2)
        rh[k] = *reinterpret_cast<const u32x4_t*>(ok ? xt + hrel[k] : p.x);
      } else {                  // wide tiles: registers are tighter than VALU (+2 % the other way)
        rh[k] = *reinterpret_cast<const u32x4_t*>(
            ok ? p.x + c0 + (((size_t)(b0 + (pk >> 24)) * p.Hin + (yy >> ys)) * p.Win + (xx >> ys)) * p.x_cs +
                     8 * (pk & 0xff)
               : p.x);
      }
      hok |= (ok ? 1u : 0u) << k;
    }
  };
  auto store_tile = [&](const u32x4_t (&rg0)[NGZ], const u32x4_t (&rh)[NH], const int (&rb)[NGZ],
                        unsigned gok, unsigned hok) {
#pragma unroll
    for (int k = 0; k < NGZ; ++k) {
      const int i = tid + k * 256;
      const int pm = i / GV, v = i - pm * GV;
      const bool ok = (gok >> k) & 1u;
      u32x4_t rg = ok ? rg0[k] : u32x4_t{0u, 0u, 0u, 0u};
      if (gz_bits && ok && rb[k] != 0xff) {   // up2(g) * lrelu'(bits), rounded as the unfused gz
        const int m = rb[k];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float a = bf_lo(rg[e]), c = bf_hi(rg[e]);
          if (!((m >> (2 * e)) & 1)) a *= p.slope;
          if (!((m >> (2 * e + 1)) & 1)) c *= p.slope;
          rg[e] = pack_bf16x2(a, c);
        }
      }
      *reinterpret_cast<u32x4_t*>(gzl + grow(pm) + 8 * v) = rg;
      if (do_db) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bs[2 * e] += bf_lo(rg[e]);
          bs[2 * e + 1] += bf_hi(rg[e]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NH; ++k) {
      // branch-free: lanes past the halo write a scratch slot behind it (an exec-masked
      // store block here made the compiler drain every prefetched tile, vmcnt(0), once per
      // PD tiles)
      const int i = tid + k * 256;
      const int hp = i / HV, v = i - hp * HV;
      const int off = i < nhalo ? hrow(hp) + 8 * v : hscr;
      *reinterpret_cast<u32x4_t*>(hal + off) = ((hok >> k) & 1u) ? rh[k] : u32x4_t{0u, 0u, 0u, 0u};
    }
  };
  // halo rows of this lane's two k-rows for each k-step the wave owns (tile-invariant)
  constexpr int KSW = (BP / 32) / KW;
  int hAo[KSW], hBo[KSW];
#pragma unroll
  for (int j = 0; j < KSW; ++j) {
    const int ks = wk + j * KW;
    const int rA = ks * 32 + 8 * g + q, rB = rA + 4;
    const int txA = rA % p.TW, tyA = (rA / p.TW) % p.TH, nbA = rA / (p.TW * p.TH);
    const int txB = rB % p.TW, tyB = (rB / p.TW) % p.TH, nbB = rB / (p.TW * p.TH);
    hAo[j] = (nbA * (p.TH + 2) + tyA) * TW2 + txA;
    hBo[j] = (nbB * (p.TH + 2) + tyB) * TW2 + txB;
  }
  auto compute_tile = [&]() {
#pragma unroll
    for (int j = 0; j < KSW; ++j) {
      const int ks = wk + j * KW;
      const int rA = ks * 32 + 8 * g + q, rB = rA + 4;   // tile pixels of this lane's rows
      bf16x8_t A[MO];
#pragma unroll
      for (int mo = 0; mo < MO; ++mo) {
        const int ol = (wo * MO + mo) * 16 + 4 * pq;
        A[mo] = tr_read8(gzl + grow(rA) + ol, gzl + grow(rB) + ol);
      }
      const int hA = hAo[j], hB = hBo[j];
      auto readB = [&](int tap, int nc) {
        const int toff = (tap / 3) * TW2 + (tap % 3);
        const int cl = (wc * NC + nc) * 16 + 4 * pq;
        return tr_read8(hal + hrow(hA + toff) + cl, hal + hrow(hB + toff) + cl);
      };
      // software-pipelined: the B fragment of the next (tap, nc) is read before the MFMAs
      // of the current one, so they never wait on a read issued just before them
      bf16x8_t Bc = readB(0, 0);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
#pragma unroll
        for (int nc = 0; nc < NC; ++nc) {
          const bool last = tap == 8 && nc == NC - 1;
          const bf16x8_t Bn = last ? Bc : (nc + 1 < NC ? readB(tap, nc + 1) : readB(tap + 1, 0));
          // keep the read ahead of these MFMAs (wide tiles; A/B: -2..-12 % there, +15 % at
          // MO = 1 where one MFMA per read cannot cover it)
          if constexpr (MO >= 4) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int mo = 0; mo < MO; ++mo)
            acc[mo][nc][tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[mo], Bc, acc[mo][nc][tap],
                                                                       0, 0, 0);
          if constexpr (MO >= 4) __builtin_amdgcn_sched_barrier(0);
          Bc = Bn;
        }
      }
    }
  };

  // PD tiles of global loads in flight: tile t+PD is fetched into the register set that
  // tile t just left, right after it was written to LDS
  u32x4_t rg[PD][NGZ], rh[PD][NH];
  int rb[PD][NGZ];
  unsigned gokr[PD], hokr[PD];
  const int t_begin = bz * p.tiles_per_split;
  const int t_end = min(p.ntiles, t_begin + p.tiles_per_split);
  // tiles past the end re-load the last tile (never stored): no branch around the loads
#pragma unroll
  for (int d = 0; d < PD; ++d)
    load_tile(min(t_begin + d, t_end - 1), rg[d], rh[d], rb[d], gokr[d], hokr[d]);
  // the staging stores and loads run unconditionally (tiles past the end store zeros and
  // skip their MFMAs), so the compiler's load counting stays exact across the back edge
  // and PD tiles of loads really stay in flight (a branch around them cost a full vmcnt(0)
  // drain per PD tiles)
  for (int t = t_begin; t < t_end; t += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      const bool live = t + d < t_end;
      __syncthreads();   // the previous tile's fragments have been read
      store_tile(rg[d], rh[d], rb[d], live ? gokr[d] : 0u, live ? hokr[d] : 0u);
      __syncthreads();
      load_tile(min(t + d + PD, t_end - 1), rg[d], rh[d], rb[d], gokr[d], hokr[d]);
      if (live) compute_tile();   // no global memory access inside: the counting stays exact
    }
  }

  float* red = reinterpret_cast<float*>(smem);
  // ---- bias gradient: thread tid holds channel group v = tid % GV (256 % GV == 0)
  if (do_db) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[tid * 8 + e] = bs[e];
    __syncthreads();
    if (tid < BO && o0 + tid < p.cout) {
      const int v = tid >> 3, e = tid & 7;
      float s = 0.f;
      for (int r = v; r < 256; r += GV) s += red[r * 8 + e];
      const int o = o0 + tid;
      if (p.mode == WG_SLABS)
        p.ws[bz * p.slab + (size_t)p.cout * p.cin * 9 + o] = s;
      else   // WG_DIRECT: sole writer, one add like a read-modify-write (see the dW epilogue)
        atomicAdd(p.db + o, s * p.scale);
    }
  }
  // ---- epilogue, one (mo, nc) 16x16x9 block per round: every wave dumps its partial
  // accumulators to LDS in output order ([wave][o][c][tap]: the lane's 16x16 MFMA
  // fragment holds c = lane & 15, o = 4 * (lane >> 4) + j); all 256 threads then sum the
  // KW partials of each (o, c, tap) from consecutive words (conflict free; the former
  // [tap][lane][j] image put the 9 taps a lane group reads 256 words apart, on one bank:
  // ~45 % of the kernel's LDS cycles were conflicts) and write [o][c][tap] runs contiguously.
  float* slab = p.mode == WG_SLABS ? p.ws + bz * p.slab : nullptr;
#pragma unroll 1
  for (int r = 0; r < MO * NC; ++r) {
    const int a = r / NC, b = r % NC;
    __syncthreads();
    float* mine = red + (size_t)wid * 2304 + ((lane >> 4) * 64 + (lane & 15)) * 9;
#pragma unroll
    for (int mo = 0; mo < MO; ++mo)
#pragma unroll
      for (int nc = 0; nc < NC; ++nc)
        if (mo == a && nc == b) {
#pragma unroll
          for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int j = 0; j < 4; ++j) mine[j * 16 * 9 + t] = acc[mo][nc][t][j];
        }
    __syncthreads();
    constexpr int NOUT = (4 / KW) * 2304;   // outputs of this round (per wmn: 16 o x 16 c x 9)
    constexpr int NPT = NOUT / 256;
    float v[NPT];
    int offs[NPT];
#pragma unroll
    for (int k2 = 0; k2 < NPT; ++k2) {
      const int e = tid + 256 * k2;
      const int m = e / 2304, rem = e - m * 2304;
      const int ol = rem / 144, rem2 = rem - ol * 144;
      const int cl = rem2 / 9, tap = rem2 - cl * 9;
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < KW; ++k) sum += red[(size_t)(m * KW + k) * 2304 + rem];
      const int mwo = m / WNC, mwc = m % WNC;
      const int o = o0 + (mwo * MO + a) * 16 + ol;
      const int c = c0 + (mwc * NC + b) * 16 + cl;
      v[k2] = sum;
      offs[k2] = (o < p.cout && c < p.cin) ? (o * p.cin + c) * 9 + tap : -1;
    }
    if (p.mode == WG_DIRECT) {
      // one fp32 add per element into dW.  WG_DIRECT: this workgroup is the only writer in
      // the launch, so the (no-return, fire-and-forget) atomic performs the same single
      // add old + v*scale as a read-modify-write, without a dependent load round trip per
      // round (the order of adds into dW across launches stays stream order)
#pragma unroll
      for (int k2 = 0; k2 < NPT; ++k2)
        if (offs[k2] >= 0) atomicAdd(p.dw + offs[k2], v[k2] * p.scale);
    } else {
#pragma unroll
      for (int k2 = 0; k2 < NPT; ++k2)
        if (offs[k2] >= 0) slab[offs[k2]] = v[k2];
    }
  }
}

// Sum the split slabs (slab order, deterministic): block x covers 64 consecutive outputs with
// G slab groups (a wave each: 256 contiguous bytes of one slab per load); wave g sums slabs
// [g*spg, (g+1)*spg) with 4 loads in flight, the G group sums are added in group order through
// LDS and added once to dw / db.  G is picked per shape (wgrad_reduce_groups) so the launch has
// ~512 x 256 threads in flight like the former 2-D grid, which added its y-partials with fp32
// atomics (order-dependent results, tools/repro_probe.py).
template <int G>
__global__ __launch_bounds__(64 * G) void wgrad_slab_reduce(const float* ws, size_t slab, int splits,
                                                            int nw, float* dw, float* db, float scale) {
  __shared__ float part[G][64];
  const int l = threadIdx.x & 63, g = threadIdx.x >> 6;
  const size_t i = (size_t)blockIdx.x * 64 + l;
  const int spg = (splits + G - 1) / G;
  const int s0 = g * spg, s1 = min(splits, s0 + spg);
  float s = 0.f;
  if (i < slab) {
    int k = s0;
    // 16 loads in flight per round, summed in slab order (the narrow layers' 512-1024 splits
    // over 16 waves per block: 4 loads per round left a 16-round latency chain, ~18 us)
    for (; k + 16 <= s1; k += 16) {
      float t[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) t[u] = ws[(size_t)(k + u) * slab + i];
#pragma unroll
      for (int u = 0; u < 16; ++u) s += t[u];
    }
    for (; k + 4 <= s1; k += 4) {
      float t[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = ws[(size_t)(k + u) * slab + i];
#pragma unroll
      for (int u = 0; u < 4; ++u) s += t[u];
    }
    for (; k < s1; ++k) s += ws[(size_t)k * slab + i];
  }
  part[g][l] = s;
  __syncthreads();
  if (g != 0 || i >= slab) return;
  float t = part[0][l];
#pragma unroll
  for (int q = 1; q < G; ++q) t += part[q][l];
  float* dst = i < (size_t)nw ? dw + i : (db ? db + (i - nw) : nullptr);
  if (dst) *dst += t * scale;
}

// groups per block of wgrad_slab_reduce: enough blocks x groups for ~2048 waves in flight
static int wgrad_reduce_groups(size_t slab, int splits) {
  const long nblk = (long)((slab + 63) / 64);
  int g = 1;
  while (g < 16 && nblk * g < 2048 && g * 2 <= splits) g *= 2;
  return g;
}

static void launch_slab_reduce(const float* ws, size_t slab, int splits, int nw, float* dw, float* db,
                               float scale, hipStream_t st) {
  const dim3 grid((unsigned)pg_cdiv((long long)slab, 64));
  switch (wgrad_reduce_groups(slab, splits)) {
    case 1: PG_KLAUNCH(wgrad_slab_reduce<1>, grid, dim3(64), 0, st, ws, slab, splits, nw, dw, db, scale); break;
    case 2: PG_KLAUNCH(wgrad_slab_reduce<2>, grid, dim3(128), 0, st, ws, slab, splits, nw, dw, db, scale); break;
    case 4: PG_KLAUNCH(wgrad_slab_reduce<4>, grid, dim3(256), 0, st, ws, slab, splits, nw, dw, db, scale); break;
    case 8: PG_KLAUNCH(wgrad_slab_reduce<8>, grid, dim3(512), 0, st, ws, slab, splits, nw, dw, db, scale); break;
    default: PG_KLAUNCH(wgrad_slab_reduce<16>, grid, dim3(1024), 0, st, ws, slab, splits, nw, dw, db, scale); break;
  }
}

// The same sum, thread = 4 consecutive outputs: one 16-byte load per slab, RSP of them issued
// before any is summed (the 4-byte form above kept 4 loads in flight per thread, ~9 KiB per CU:
// latency bound at 1.2 TB/s).  Slabs are still summed in slab order into one register per
// output, then added once to dw / db: the result is bitwise the form above's (gridDim.y == 1).
// slab % 4 == 0 and nw % 4 == 0 (cout, cin multiples of 8), so a vector never straddles dw / db.
constexpr int RSP = 16;
__global__ __launch_bounds__(64) void wgrad_slab_reduce4(const float* ws, size_t slab, int splits,
                                                         int nw, float* dw, float* db, float scale) {
  const size_t i = ((size_t)blockIdx.x * 64 + threadIdx.x) * 4;
  if (i >= slab) return;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < splits; k += RSP) {
    f32x4_t t[RSP];
#pragma unroll
    for (int u = 0; u < RSP; ++u)
      if (k + u < splits) t[u] = *reinterpret_cast<const f32x4_t*>(ws + (size_t)(k + u) * slab + i);
#pragma unroll
    for (int u = 0; u < RSP; ++u)
      if (k + u < splits) {
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += t[u][e];
      }
  }
  float* dst = i < (size_t)nw ? dw + i : (db ? db + (i - nw) : nullptr);
  if (!dst) return;
#pragma unroll
  for (int e = 0; e < 4; ++e) dst[e] += s[e] * scale;
}

struct WgbPlan {
  int MO, NC, WMO, WNC, BP;
  int ot, ct, splits, tiles_per_split, ntiles;
  TileCfg tc;
  size_t slab;
};

bool wgrad_dma_ok(const pg_conv_desc* d, const WgbPlan& pl);

WgbPlan wgrad_bf16_plan(const pg_conv_desc* d) {
  WgbPlan pl;
  const int co = d->cout, ci = d->cin;
  pl.MO = co <= 16 ? 1 : co <= 32 ? 2 : 4;
  pl.NC = 1;
  pl.WMO = 1;
  // two 16-channel halves of a 32-channel input slice per workgroup (waves split the
  // channels, the gz tile is staged once for both): A/B -5..-22 % at 32^2-256^2 for
  // cin > 32; below 32^2 the single-half tile is faster (the LDS-DMA kernel, which needs
  // WNC = 2, measured 28.6 vs 24.1 us at 16^2 512 -> 512)
  pl.WNC = ci <= 16 ? 1 : (ci <= 32 || d->W >= 32) ? 2 : 1;
  // ... unless the single-half tiles overflow one round of workgroups (the 513-channel
  // minibatch-stddev conv at 4^2: 8 x 33 = 264 > 256 ran as two rounds, 29.6 us vs 15.8)
  if (pl.WNC == 1 && ci > 16 && pg_cdiv(co, co <= 16 ? 16 : co <= 32 ? 32 : 64) * pg_cdiv(ci, 16) > 256)
    pl.WNC = 2;
  const int BO = pl.WMO * pl.MO * 16, BC = pl.WNC * pl.NC * 16;
  // 128-pixel tiles (256-pixel ones measured -6..-10 % for the single-half tile at 32^2-128^2,
  // where the two-half tile is faster still, and +50 % with two halves: spills)
  pl.BP = WGB_BP;
  pl.tc = pick_tile(d->H, d->W, pl.BP, 32);
  pl.ntiles = pg_cdiv(d->B, pl.tc.NB) * (d->W / pl.tc.TW) * (d->H / pl.tc.TH);
  pl.ot = pg_cdiv(co, BO);
  pl.ct = pg_cdiv(ci, BC);
  const int base = pl.ot * pl.ct;
  // >= 256 workgroups without a split when the output tiles allow it; otherwise split
  // the pixels up to ~1024 workgroups, keeping >= 2 tiles per split
  // wide (MO = 4) tiles run one workgroup per CU with 4 tiles of loads in flight: one
  // wave of workgroups; the HBM-bound narrow ones use ~4 per CU
  // (tools/wg_target_sweep.sh: 512 for the narrow tiles, 80.9 -> 59.2 us at 512^2 32->32,
  // 86 -> 79 at 1024^2 16->16, 108 -> 99 at 1024^2 16->32: half the slab traffic)
  // wide: 192 rather than one workgroup per CU (256): the weight gradients run on the side
  // stream beside the input-gradient chain, and leaving a quarter of the CUs to the main
  // stream's launches measured +0.2-0.6 % per step in 5 of 5 interleaved rounds (128: -2.6 %;
  // profiles/r5_dp_ab.txt section 9)
  int target = pl.MO >= 4 ? 192 : 512;   // narrow: 384 measured slower (r5_dp_ab.txt section 10)
  // the LDS-DMA narrow tiles (tools/wg_target_dma.sh): (2,2) at 512^2 in one round of
  // workgroups (8 waves at 164 VGPRs: one workgroup per CU), 51.0 -> 48.8 us at 32->32;
  // (1,1) at 1024^2 with ~4 per CU, 74.3 -> 62.7 us at 16->16
  if (pl.MO < 4) {
    pl.tiles_per_split = 1;
    if (wgrad_dma_ok(d, pl)) {
      if (pl.MO == 2 && pl.WNC == 2) target = 256;
      else if (pl.MO == 1 && pl.WNC == 1) target = 1024;
    }
  }
  int splits = base >= 256 ? 1 : pg_cdiv(target, base);
  const int max_splits = pl.ntiles / 2 > 1 ? pl.ntiles / 2 : 1;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  pl.tiles_per_split = pg_cdiv(pl.ntiles, splits);
  pl.splits = pg_cdiv(pl.ntiles, pl.tiles_per_split);
  pl.slab = (size_t)co * ci * 9 + co;
  return pl;
}

size_t wgrad_bf16_ws_bytes(const pg_conv_desc* d) {
  WgbPlan pl = wgrad_bf16_plan(d);
  return pl.splits > 1 ? pl.splits * pl.slab * sizeof(float) : 0;
}

// The second launch of the WG_SLABS mode: the split partials summed into dw / db
int wgrad_slab_finish(const pg_conv_desc* d, const WgbPlan& pl, int mode, const float* ws, float* dw,
                      float* db, float scale, hipStream_t st) {
  if (mode != WG_SLABS) return PG_OK;
  if (pl.slab >= 65536 && pl.slab % 4 == 0 && ((uintptr_t)ws & 15) == 0) {
    // wide layers (>= 256 blocks of 64 threads): vector form, one thread sums every split
    PG_KLAUNCH(wgrad_slab_reduce4, dim3((unsigned)pg_cdiv((long long)pl.slab / 4, 64)), dim3(64), 0, st,
                       ws, pl.slab, pl.splits, d->cout * d->cin * 9, dw, db, scale);
    PG_LAUNCH_CHECK();
    return PG_OK;
  }
  launch_slab_reduce(ws, pl.slab, pl.splits, d->cout * d->cin * 9, dw, db, scale, st);
  PG_LAUNCH_CHECK();
  return PG_OK;
}

// the LDS-DMA weight gradient of the wide layers (wgrad_dma.inc)
bool wgrad_dma_ok(const pg_conv_desc* d, const WgbPlan& pl);
int launch_wgrad_dma(const pg_conv_desc* d, const WgbPlan& pl, const void* x, const void* gz, float scale,
                     float* dw, float* db, float* ws, size_t ws_bytes, hipStream_t st, const void* gzbits);

template <int MO, int NC, int WMO, int WNC, int PD, int WPE, bool GZB = false, int BP = WGB_BP>
int launch_wgrad_bf16(const pg_conv_desc* d, const WgbPlan& pl, const void* x, const void* gz,
                      float scale, float* dw, float* db, float* ws, size_t ws_bytes,
                      hipStream_t st, const void* gzbits) {
  constexpr int BO = WMO * MO * 16, BC = WNC * NC * 16;
  WgBParams p;
  p.x = (const bf16_t*)x; p.gz = (const bf16_t*)gz; p.dw = dw; p.db = db;
  p.B = d->B; p.H = d->H; p.W = d->W;
  p.ups = (d->flags & PG_CONV_UPS_IN) ? 1 : 0;
  p.Hin = p.ups ? d->H / 2 : d->H;
  p.Win = p.ups ? d->W / 2 : d->W;
  p.cin = d->cin; p.cout = d->cout; p.x_cs = d->x_cs; p.gz_cs = d->y_cs;
  p.scale = scale;
  p.NB = pl.tc.NB; p.TH = pl.tc.TH; p.TW = pl.tc.TW;
  p.tiles_x = d->W / pl.tc.TW;
  p.tiles_y = d->H / pl.tc.TH;
  auto lg2 = [](int v) { int l = 0; while ((1 << l) < v) ++l; return (1 << l) == v ? l : -1; };
  p.lg_tx = lg2(p.tiles_x);
  p.lg_ty = lg2(p.tiles_y);
  p.ntiles = pl.ntiles;
  p.tiles_per_split = pl.tiles_per_split;
  p.GZS = BO + (BO > 16 ? 16 : 0);
  p.HS = BC == 16 ? 16 : BC + 16;
  p.hpad = pl.tc.TW >= 8 ? 64 : 0;
  p.halo_elems = pl.tc.NB * (pl.tc.TH + 2) * (pl.tc.TW + 2);
  p.gzb = (d->flags & PG_CONV_GZ_BITS) ? reinterpret_cast<const unsigned char*>(gzbits) : nullptr;
  p.gzb_cs = d->xb_cs;
  p.slope = d->slope;
  p.xcd_remap = 1;
  PG_CHECK_ARG(!p.gzb || (d->xb_cs * 8 >= d->cout && pl.tc.TH % 2 == 0 && pl.tc.TW % 2 == 0),
               "wgrad_bf16: GZ_BITS needs gzbits with >= cout/8 bytes per pixel");
  PG_CHECK_ARG(pl.BP == BP && p.halo_elems <= wgb_maxhalo(BP), "wgrad_bf16: halo %d > %d", p.halo_elems,
               wgb_maxhalo(BP));
  p.slab = pl.slab;
  p.ws = nullptr;
  // wgrad_bf16_dispatch re-plans to one split when the workspace cannot hold the slabs
  PG_CHECK_ARG(pl.splits == 1 || (ws && ws_bytes >= pl.splits * pl.slab * sizeof(float)),
               "wgrad: split plan without its workspace");
  p.mode = pl.splits == 1 ? WG_DIRECT : WG_SLABS;
  if (p.mode == WG_SLABS) p.ws = ws;
  // + 16 B: store_tile's scratch slot behind the halo
  int lds = (BP * p.GZS + (BP / 8) * 64 + p.halo_elems * p.HS + (p.halo_elems / 8 + 1) * p.hpad) * 2 + 16;
  const int need = 4 * 9 * 64 * 4 * 4;   // epilogue dump of one (mo, nc) block per wave
  if (need > lds) lds = need;
  PG_CHECK_ARG(lds <= 160 * 1024, "wgrad_bf16: LDS %d too large", lds);
  PG_LDS_ATTR((wgrad_bf16_kernel<MO, NC, WMO, WNC, PD, WPE, GZB, BP>), 160 * 1024);
  PG_KLAUNCH((wgrad_bf16_kernel<MO, NC, WMO, WNC, PD, WPE, GZB, BP>), dim3(pl.ot, pl.ct, pl.splits),
                     dim3(256), lds, st, p);
  PG_LAUNCH_CHECK();
  return wgrad_slab_finish(d, pl, p.mode, ws, dw, db, scale, st);
}

// GZ_BITS variants: the tiles of the discriminator's conv b weight gradient at the levels
// that keep sign bits (1024^2: cout 32 -> MO 2; 512^2: cout 64, cin 32 -> MO 4, WNC 2)
constexpr bool wgrad_gzb_ok(int MO, int WNC, int PD, int WPE) {
  return (MO == 2 && WNC == 1 && PD == 2 && WPE == 2) || (MO == 4 && PD == 4 && WPE == 1) ||
         (MO == 1 && PD == 2);
}

int wgrad_bf16_dispatch(const pg_conv_desc* d, const void* x, const void* gz, float scale,
                        float* dw, float* db, float* ws, size_t ws_bytes, hipStream_t st,
                        const void* gzbits = nullptr) {
  PG_CHECK_ARG(!(d->flags & PG_CONV_GZ_BITS) || gzbits, "wgrad_bf16: GZ_BITS without gzbits");
  PG_CHECK_ARG(d->cout % 8 == 0 && d->x_cs % 8 == 0 && d->y_cs % 8 == 0,
               "wgrad_bf16: cout (%d) and channel strides must be multiples of 8", d->cout);
  WgbPlan pl = wgrad_bf16_plan(d);
  if (pl.splits > 1 && !(ws && ws_bytes >= pl.splits * pl.slab * sizeof(float))) {
    pl.splits = 1;   // no room for the slabs: one split (WG_DIRECT), deterministic
    pl.tiles_per_split = pl.ntiles;
  }
  if (wgrad_dma_ok(d, pl)) return launch_wgrad_dma(d, pl, x, gz, scale, dw, db, ws, ws_bytes, st, gzbits);
  // (prefetch depth, waves per SIMD) from the round-1 sweep
  const int pd = pl.MO >= 4 ? 4 : 2, wpe = pl.MO >= 4 ? 1 : (pl.MO * pl.WNC >= 2 ? 2 : 3);
  const bool gzb = (d->flags & PG_CONV_GZ_BITS) != 0;
#define PG_WGB(a, b, c, e, PD, WPE)                                                        \
  if (pl.MO == a && pl.NC == b && pl.WMO == c && pl.WNC == e && pd == PD && wpe == WPE) {  \
    if constexpr (wgrad_gzb_ok(a, e, PD, WPE)) {                                           \
      if (gzb)                                                                             \
        return launch_wgrad_bf16<a, b, c, e, PD, WPE, true>(d, pl, x, gz, scale, dw, db,   \
                                                            ws, ws_bytes, st, gzbits);     \
    }                                                                                      \
    PG_CHECK_ARG(!gzb, "wgrad_bf16: GZ_BITS not instantiated for this tile");              \
    return launch_wgrad_bf16<a, b, c, e, PD, WPE, false>(d, pl, x, gz, scale, dw, db, ws,  \
                                                         ws_bytes, st, gzbits);            \
  }
  PG_WGB(1, 1, 1, 1, 2, 3)
  PG_WGB(1, 1, 1, 2, 2, 2)
  PG_WGB(2, 1, 1, 1, 2, 2)
  PG_WGB(2, 1, 1, 2, 2, 2)
  PG_WGB(4, 1, 1, 1, 4, 1)
  PG_WGB(4, 1, 1, 2, 4, 1)
#undef PG_WGB
  PG_CHECK_ARG(false, "wgrad_bf16: no kernel for plan");
  return PG_ERR_ARG;
}

// --------------------------------------------------------------------------
template <typename T>
__global__ void pack_kernel(int mode, int cout, int cin, int rows, int kin, const float* w,
                            float scale, T* out) {
  // fwd:   out[o][tap][c]  (rows = cout_p, kin = cin_p)
  // dgrad: out[c][tap][o]  (rows = cin padded to 16, kin = cinp(cout)); W flipped
  const size_t total = (size_t)rows * 9 * kin;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(i % kin);
    const int tap = (int)((i / kin) % 9);
    const int row = (int)(i / ((size_t)kin * 9));
    float v = 0.f;
    if (mode == PG_PACK_FWD) {
      if (row < cout && k < cin) v = w[((size_t)row * cin + k) * 9 + tap] * scale;
    } else {
      if (row < cin && k < cout) v = w[((size_t)k * cin + row) * 9 + (8 - tap)] * scale;
    }
    Ty<T>::st(out + i, v);
  }
}

// One launch for all conv weights of a net.  Block (x, item): a 32(o) x 32(c) x 9 tile of
// W staged in LDS (rows read contiguously), then written in the fwd layout (c fastest) and
// the flipped dgrad layout (o fastest), both coalesced; zero padding included.
template <typename T>
__global__ __launch_bounds__(256) void pack_batch_kernel(const pg_pack_item* items) {
  const pg_pack_item it = items[blockIdx.y];
  const int cout = it.cout, cin = it.cin;
  const int rf = (cout + 15) & ~15, kf = cinp_of_dev(cin);   // fwd   [rf][9][kf]
  const int rd = (cin + 15) & ~15, kd = cinp_of_dev(cout);   // dgrad [rd][9][kd]
  const int O = rf > kd ? rf : kd, C = kf > rd ? kf : rd;
  const int tc = (C + 31) / 32;
  if ((int)blockIdx.x >= ((O + 31) / 32) * tc) return;
  const int o0 = (blockIdx.x / tc) * 32, c0 = (blockIdx.x % tc) * 32;
  __shared__ float s[32][32 * 9 + 1];
  const int tid = threadIdx.x;
  if ((cin & 3) == 0 && ((uintptr_t)it.w & 15) == 0) {
    // 16-byte loads: a row segment (o, c0..c0+31) is 288 contiguous floats at a multiple of 4
#pragma unroll 3
    for (int i = tid; i < 32 * 72; i += 256) {
      const int ol = i / 72, j = (i - ol * 72) * 4;
      const int o = o0 + ol;
      f32x4_t v = f32x4_t{0.f, 0.f, 0.f, 0.f};
      if (o < cout && c0 + j / 9 < cin)   // cin % 4 == 0: a 4-group never straddles cin
        v = *reinterpret_cast<const f32x4_t*>(it.w + ((size_t)o * cin + c0) * 9 + j);
#pragma unroll
      for (int k = 0; k < 4; ++k) s[ol][j + k] = (c0 + (j + k) / 9 < cin) ? v[k] * it.scale : 0.f;
    }
  } else {
    for (int i = tid; i < 32 * 288; i += 256) {
      const int ol = i / 288, j = i - ol * 288;
      const int o = o0 + ol, c = c0 + j / 9;
      s[ol][j] = (o < cout && c < cin) ? it.w[((size_t)o * cin + c0) * 9 + j] * it.scale : 0.f;
    }
  }
  __syncthreads();
  T* fwd = reinterpret_cast<T*>(it.fwd);
  T* dg = reinterpret_cast<T*>(it.dgrad);
  // 4 consecutive fastest-axis elements per store (kf, kd, rf, rd are multiples of 16, so a
  // group of 4 is wholly inside or outside the padded range and 8/16-byte aligned)
  for (int i = tid; i < 8 * 288; i += 256) {
    const int cq = i & 7, tap = (i >> 3) % 9, ol = i / 72;
    const int o = o0 + ol, c = c0 + 4 * cq;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = s[ol][(4 * cq + k) * 9 + tap];
    if (o < rf && c < kf) Ty<T>::st4(fwd + ((size_t)o * 9 + tap) * kf + c, v);
  }
  for (int i = tid; i < 8 * 288; i += 256) {
    const int oq = i & 7, tap = (i >> 3) % 9, cl = i / 72;
    const int o = o0 + 4 * oq, c = c0 + cl;
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = s[4 * oq + k][cl * 9 + 8 - tap];
    if (c < rd && o < kd) Ty<T>::st4(dg + ((size_t)c * 9 + tap) * kd + o, v);
  }
  if (c0 == 0 && tid < 32 && o0 + tid < cout)
    it.bias_scaled[o0 + tid] = it.bias ? it.bias[o0 + tid] * it.scale : 0.f;
}

// db[c] += scale * sum_p g[p][c]: block totals summed over blocks in block order (det_commit)
template <typename T>
__global__ __launch_bounds__(256) void bias_grad_kernel(int npix, int C, int cs, const T* g, float scale,
                                                        float* db, int pix_per_block, float* scratch) {
  __shared__ float red[256];
  __shared__ float tot[1024];   // C <= 1024 totals, then det_commit's tmp
  const int p0 = blockIdx.x * pix_per_block;
  const int p1 = min(npix, p0 + pix_per_block);
  if (C <= 256 && (256 % C) == 0) {
    const int ppi = 256 / C;  // pixels per iteration
    const int c = threadIdx.x % C, pi = threadIdx.x / C;
    float s = 0.f;
    for (int pp = p0 + pi; pp < p1; pp += ppi) s += Ty<T>::ld(g + (size_t)pp * cs + c);
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x < C) {
      float t = 0.f;
      for (int q = 0; q < ppi; ++q) t += red[q * C + threadIdx.x];
      tot[threadIdx.x] = t;
    }
  } else {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float s = 0.f;
      for (int pp = p0; pp < p1; ++pp) s += Ty<T>::ld(g + (size_t)pp * cs + c);
      tot[c] = s;
    }
  }
  __syncthreads();
  det_commit(tot, C, scratch, tot, [&](int c, float t) { db[c] += t * scale; });
}

void conv_tile_for(int cout, int* BM, int* BN, int W = 16) {
  const int cout_p = (cout + 15) & ~15;
  if (cout_p >= 64) { *BM = 128; *BN = 64; }
  else if (cout_p >= 32) { *BM = W >= 16 ? 256 : 128; *BN = 32; }
  else { *BM = W >= 16 ? 256 : 128; *BN = 16; }
}

// split-K factor: spread the channel chunks of small-spatial / wide convs (4x4..16x16 at
// 512 channels launch only 8..64 output tiles) over enough workgroups to fill the chip
int conv_splits(const pg_conv_desc* d) {
  int BM, BN;
  conv_tile_for(d->cout, &BM, &BN, d->W);
  TileCfg tc = pick_tile(d->H, d->W, BM, BN);
  const int cout_p = (d->cout + 15) & ~15;
  const int base = pg_cdiv(d->B, tc.NB) * (d->W / tc.TW) * (d->H / tc.TH) * pg_cdiv(cout_p, BN);
  const int cin_p = cinp_of(d->cin);
  const int nch = cin_p / (cin_p < 32 ? cin_p : 32);
  // round-2 split sweep; round 5: min_base 128 -> 256 splits the 16^2 512 -> 512 convs of the
  // merged passes (B = 8: 128 tiles) in two, 31.2 -> 27.1 us per launch with the epilogue
  // (profiles/r5_lowres_tiles.txt)
  constexpr int min_base = 256, target = 256;
  if (base >= min_base || nch < 4) return 1;
  int sp = pg_cdiv(target, base);
  if (sp > nch) sp = nch;
  const int cps = pg_cdiv(nch, sp);
  return pg_cdiv(nch, cps);
}

size_t conv_ws_bytes(const pg_conv_desc* d) {
  const int sp = conv_splits(d);
  if (sp <= 1) return 0;
  return (size_t)sp * d->B * d->H * d->W * ((d->cout + 15) & ~15) * sizeof(float);
}

template <typename T, int BM, int BN, int WM, int WN, int MAXV, bool TR, int CKC = 0, int TWC = 0,
          int THC = 0>
int launch_conv(const pg_conv_desc* d, const void* x, const void* wpk, const float* bias,
                const void* aux, void* y, void* y2, void* ws, size_t ws_bytes, hipStream_t st) {
  TileCfg tc = pick_tile(d->H, d->W, BM, BN);
  ConvParams p;
  p.x = x; p.w = wpk; p.bias = bias; p.aux = aux; p.y = y; p.y2 = y2;
  p.B = d->B; p.H = d->H; p.W = d->W;
  const bool ups = (d->flags & PG_CONV_UPS_IN) != 0;
  p.Hin = ups ? d->H / 2 : d->H;
  p.Win = ups ? d->W / 2 : d->W;
  p.cin_p = cinp_of(d->cin);
  p.cout = d->cout;
  p.cout_p = (d->cout + 15) & ~15;
  p.x_cs = d->x_cs; p.y_cs = d->y_cs; p.aux_cs = d->aux_cs; p.y2_cs = d->y2_cs;
  p.flags = d->flags; p.slope = d->slope; p.out_scale = d->out_scale;
  p.NB = tc.NB; p.TH = tc.TH; p.TW = tc.TW;
  p.tiles_x = d->W / tc.TW;
  p.tiles_y = d->H / tc.TH;
  // channels per chunk: 32 (bf16) / 16 (f32) keeps the staged chunk at 64 B per halo pixel
  const int ck_max = sizeof(T) == 4 ? 16 : 32;
  p.CK = p.cin_p < ck_max ? p.cin_p : ck_max;
  p.KS = (9 * p.CK + 31) / 32;
  p.nchunks = p.cin_p / p.CK;
  const int pb = p.CK * (int)sizeof(T);
  // bf16: paddings that make the b128 fragment reads conflict-free (tools/lds_banks.py)
  p.pixb = pb + (pb >= 64 ? (sizeof(T) == 2 ? 32 : 16) : 0);
  p.wrowb = p.KS * 32 * (int)sizeof(T) + (sizeof(T) == 2 ? 32 : 16);
  p.halo_bytes = (tc.NB * (tc.TH + 2) * (tc.TW + 2) * p.pixb + 15) & ~15;
  const int main_bytes = p.halo_bytes + BN * p.wrowb;
  const int epi_bytes = TR ? 0 : BM * (BN + 4) * 4;
  const int lds = main_bytes > epi_bytes ? main_bytes : epi_bytes;
  PG_CHECK_ARG(lds <= 160 * 1024, "conv3x3: LDS %d bytes too large", lds);
  PG_CHECK_ARG(CKC == 0 || CKC == p.CK, "conv3x3: compile-time chunk %d != %d", CKC, p.CK);
  PG_CHECK_ARG(TWC == 0 || (TWC == tc.TW && THC == tc.TH), "conv3x3: compile-time tile %dx%d != %dx%d",
               TWC, THC, tc.TW, tc.TH);
  {
    const int vpp = p.CK * (int)sizeof(T) / 16;
    const int ntot = tc.NB * (tc.TH + 2) * (tc.TW + 2) * vpp + BN * (p.KS * 32 / p.CK) * vpp;
    PG_CHECK_ARG(ntot <= 64 * WM * WN * MAXV, "conv3x3: %d staged vectors exceed %d per block", ntot,
                 64 * WM * WN * MAXV);
    (void)0;
  }
  int splits = 1;
  const size_t need = conv_ws_bytes(d);
  if (need && ws && ws_bytes >= need) splits = conv_splits(d);
  p.ws = splits > 1 ? (float*)ws : nullptr;
  p.cps = pg_cdiv(p.nchunks, splits);
  p.slab = (size_t)d->B * d->H * d->W * p.cout_p;
  p.xcd_remap = 1;
  dim3 grid(pg_cdiv(d->B, tc.NB) * p.tiles_x * p.tiles_y, p.cout_p / BN + (p.cout_p % BN ? 1 : 0),
            splits);
  PG_LDS_ATTR((conv3x3_kernel<T, BM, BN, WM, WN, MAXV, TR, CKC, TWC, THC>), 160 * 1024);
  PG_KLAUNCH((conv3x3_kernel<T, BM, BN, WM, WN, MAXV, TR, CKC, TWC, THC>), grid, dim3(64 * WM * WN), lds,
             st, p);
  if (splits > 1) {
    const bool pool = (d->flags & PG_CONV_POOL) != 0;
    const size_t n = (size_t)d->B * (pool ? d->H / 2 : d->H) * (pool ? d->W / 2 : d->W) * (d->cout / 4);
    int blocks = (int)((n + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    if (d->flags & PG_CONV_PIXNORM) {   // one wave per pixel
      PG_CHECK_ARG(d->cout <= 1024 && d->cout % 4 == 0, "conv3x3: split-K PixelNorm needs cout %% 4 == 0, <= 1024");
      blocks = pg_cdiv(d->B * d->H * d->W, 4);
    }
    PG_KLAUNCH(conv_splitk_epilogue<T>, dim3(blocks), dim3(256), 0, st, p, splits);
  }
  PG_LAUNCH_CHECK();
  return PG_OK;
}

// staged 16-byte vectors per thread for one chunk (halo tile + weight slab)
template <typename T>
int conv_vectors_per_thread(const pg_conv_desc* d, int BM, int BN) {
  TileCfg tc = pick_tile(d->H, d->W, BM, BN);
  const int cin_p = cinp_of(d->cin);
  const int ck_max = sizeof(T) == 4 ? 16 : 32;
  const int CK = cin_p < ck_max ? cin_p : ck_max;
  const int KS = (9 * CK + 31) / 32;
  const int vpp = CK * (int)sizeof(T) / 16;
  const int ntot = tc.NB * (tc.TH + 2) * (tc.TW + 2) * vpp + BN * (KS * 32 / CK) * vpp;
  return pg_cdiv(ntot, 256);
}

template <typename T, int BM, int BN>
int launch_tr(const pg_conv_desc* d, const void* x, const void* wpk, const float* bias,
              const void* aux, void* y, void* y2, void* ws, size_t wsb, hipStream_t st) {
  // fewest staging registers that fit -> highest occupancy for the HBM-bound high-res convs
  const int v = conv_vectors_per_thread<T>(d, BM, BN);
  if (v <= 4) return launch_conv<T, BM, BN, 4, 1, 4, true>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
  if (v <= 8) return launch_conv<T, BM, BN, 4, 1, 8, true>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
  return launch_conv<T, BM, BN, 4, 1, 12, true>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
}

#include "conv_hr.inc"
#include "conv_lr.inc"
#include "wgrad_dma.inc"


// Which fused epilogues the kernel the dispatcher picks supports.
template <typename T>
bool conv_supported(const pg_conv_desc* d, size_t wsb) {
  constexpr int BITS = PG_CONV_Y2_BITS | PG_CONV_AUX_BITS | PG_CONV_X_BITS;
  if (d->flags & PG_CONV_RGBO) {   // the EF tiles 0 / 5 (16 / 32 channels), PixelNorm forward
    if constexpr (sizeof(T) != 2) return false;
    constexpr int PN = PG_CONV_PIXNORM | PG_CONV_LRELU | PG_CONV_BIAS;
    if (d->flags != (PN | PG_CONV_RGBO) || !conv_hr_ok(d)) return false;
    const int t = conv_hr_tile(d);
    return (t == 0 && d->cout == 16) || (t == 5 && d->cout == 32);
  }
  if (d->flags & (PG_CONV_RGBW | PG_CONV_RGBD)) {   // the EF tiles 0 / 5 (16 / 32 channels)
    if constexpr (sizeof(T) != 2) return false;
    const int rf = d->flags & (PG_CONV_RGBW | PG_CONV_RGBD);
    if (rf == (PG_CONV_RGBW | PG_CONV_RGBD)) return false;
    if (d->flags != (rf | PG_CONV_MASK | PG_CONV_AUX_BITS) || !conv_hr_ok(d)) return false;
    if ((d->flags & PG_CONV_RGBD) && d->B > 16) return false;
    const int t = conv_hr_tile(d);
    return (t == 0 && d->cout == 16) || (t == 5 && d->cout == 32);
  }
  if (d->flags & PG_CONV_PNBWD) {   // conv_hr epilogue, [cout][pixel] tiles of <= 32 channels
    if constexpr (sizeof(T) != 2) return false;
    if (d->flags & (BITS | PG_CONV_BIAS | PG_CONV_MASK | PG_CONV_ACCUM | PG_CONV_PIXNORM))
      return false;
    // after a 2x2 pool: the 32-channel tiles (their swap epilogue; y and r at pooled resolution)
    if ((d->flags & PG_CONV_POOL) && (d->cout != 32 || conv_hr_bn(d) != 32)) return false;
    return conv_hr_ok(d) && ((d->cout + 15) & ~15) <= conv_hr_bn(d) && conv_hr_bn(d) <= 32 &&
           d->cout % 4 == 0;
  }
  if (d->flags & BITS) {
    if constexpr (sizeof(T) != 2) return false;
    if (!conv_hr_ok(d) || !conv_hr_mode_ok(d)) return false;
    if ((d->flags & PG_CONV_PIXNORM) && ((d->cout + 15) & ~15) > conv_hr_bn(d)) return false;
    return true;
  }
  if ((d->flags & PG_CONV_MASK) && (d->flags & PG_CONV_POOL)) return false;
  if (!(d->flags & PG_CONV_PIXNORM)) return true;
  if (d->flags & (PG_CONV_POOL | PG_CONV_MASK | PG_CONV_ACCUM)) return false;
  const int cout_p = (d->cout + 15) & ~15;
  if constexpr (sizeof(T) == 2) {
    if (conv_hr_ok(d)) return cout_p <= conv_hr_bn(d);
  }
  int BM, BN;
  conv_tile_for(d->cout, &BM, &BN, d->W);
  const size_t need = conv_ws_bytes(d);
  const bool split = need && wsb >= need && conv_splits(d) > 1;
  // in the split-K epilogue (bf16 step; the fp32 parity mode keeps PixelNorm separate)
  if (split) return sizeof(T) == 2 && BN == 64 && d->cout % 4 == 0 && d->cout <= 1024;
  return BN <= 32 && cout_p <= BN;   // [cout][pixel] variants, single pass
}

template <typename T>
int conv_dispatch(const pg_conv_desc* d, const void* x, const void* wpk, const float* bias,
                  const void* aux, void* y, void* y2, void* ws, size_t wsb, hipStream_t st,
                  const void* xbits = nullptr) {
  PG_CHECK_ARG(conv_supported<T>(d, wsb), "conv3x3_fwd: flags 0x%x not supported for cout %d at %dx%d",
               d->flags, d->cout, d->H, d->W);
  if constexpr (sizeof(T) == 2) {
    if (conv_lr_ok(d)) return conv_lr_dispatch(d, x, wpk, bias, aux, y, y2, st);
    if (conv_hr_ok(d)) return conv_hr_dispatch(d, x, wpk, bias, aux, y, y2, xbits, st);
  }
  int BM, BN;
  conv_tile_for(d->cout, &BM, &BN, d->W);
  // cout >= 64: [pixel][cout] MFMA + LDS-transposed epilogue; cout <= 32: [cout][pixel]
  // MFMA with the direct epilogue (whole pixel rows per store instruction)
  if (BN == 64) {
    if constexpr (sizeof(T) == 2) {
      if (cinp_of(d->cin) % 32 == 0) {   // chunk = 32 channels: compile-time k loop + tile
        const TileCfg tc = pick_tile(d->H, d->W, 128, 64);
#define PG_LC(tw, th)                                                                            \
  if (tc.TW == tw && tc.TH == th)                                                                \
    return launch_conv<T, 128, 64, PG_C64_WM, 2, 16 * 2 / PG_C64_WM, false, 32, tw, th>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
        PG_LC(4, 4)
        PG_LC(8, 8)
        PG_LC(16, 8)
#undef PG_LC
        return launch_conv<T, 128, 64, 2, 2, 16, false, 32>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
      }
    }
    return launch_conv<T, 128, 64, 2, 2, 16, false>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
  }
  if (BN == 32) {
    if (BM == 256) return launch_tr<T, 256, 32>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
    return launch_tr<T, 128, 32>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
  }
  if (BM == 256) return launch_tr<T, 256, 16>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
  return launch_tr<T, 128, 16>(d, x, wpk, bias, aux, y, y2, ws, wsb, st);
}

}  // namespace

extern "C" {

size_t pg_conv3x3_packed_elems(int mode, int cout, int cin) {
  if (mode == PG_PACK_FWD) return (size_t)((cout + 15) & ~15) * 9 * cinp_of(cin);
  return (size_t)((cin + 15) & ~15) * 9 * cinp_of(cout);
}

int pg_conv3x3_pack(int dtype, int mode, int cout, int cin, const float* w_oihw, float scale,
                    void* wpk, void* stream) {
  PG_CHECK_ARG(w_oihw && wpk && cout > 0 && cin > 0, "conv3x3_pack: bad args");
  int rows, kin;
  if (mode == PG_PACK_FWD) {
    rows = (cout + 15) & ~15;
    kin = cinp_of(cin);
  } else {
    rows = (cin + 15) & ~15;
    kin = cinp_of(cout);
  }
  const size_t total = (size_t)rows * 9 * kin;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == PG_F32)
    PG_KLAUNCH(pack_kernel<float>, dim3(blocks), dim3(256), 0, st, mode, cout, cin, rows,
                       kin, w_oihw, scale, (float*)wpk);
  else
    PG_KLAUNCH(pack_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, mode, cout, cin, rows,
                       kin, w_oihw, scale, (bf16_t*)wpk);
  PG_LAUNCH_CHECK();
  return PG_OK;
}

int pg_conv3x3_pack_batch(int dtype, int n, const pg_pack_item* items, int max_tiles,
                          void* stream) {
  PG_CHECK_ARG(items && n > 0 && n < 65536 && max_tiles > 0, "conv3x3_pack_batch: bad args");
  const dim3 grid(max_tiles, n);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == PG_F32)
    PG_KLAUNCH(pack_batch_kernel<float>, grid, dim3(256), 0, st, items);
  else
    PG_KLAUNCH(pack_batch_kernel<bf16_t>, grid, dim3(256), 0, st, items);
  PG_LAUNCH_CHECK();
  return PG_OK;
}

size_t pg_conv3x3_workspace_size(const pg_conv_desc* d) { return d ? conv_ws_bytes(d) : 0; }

int pg_conv3x3_fwd(int dtype, const pg_conv_desc* d, const void* x, const void* wpk,
                   const float* bias, const void* aux, void* y, void* y2, void* ws,
                   size_t ws_bytes, void* stream) {
  PG_CHECK_ARG(d && x && wpk && y, "conv3x3_fwd: null pointer");
  PG_CHECK_ARG(d->B > 0 && d->H >= 4 && d->W >= 4 && (d->H & (d->H - 1)) == 0 &&
                   (d->W & (d->W - 1)) == 0,
               "conv3x3_fwd: spatial %dx%d must be powers of two >= 4", d->H, d->W);
  PG_CHECK_ARG(d->cin > 0 && d->cout > 0 && d->cout % 4 == 0,
               "conv3x3_fwd: cout %d must be a multiple of 4", d->cout);
  PG_CHECK_ARG(d->x_cs >= cinp_of(d->cin) && d->x_cs % 8 == 0,
               "conv3x3_fwd: x channel stride %d < padded cin %d (or not a multiple of 8)", d->x_cs,
               cinp_of(d->cin));
  PG_CHECK_ARG(d->y_cs >= d->cout && d->y_cs % 4 == 0, "conv3x3_fwd: bad y channel stride");
  PG_CHECK_ARG(!(d->flags & PG_CONV_BIAS) || bias, "conv3x3_fwd: BIAS flag without bias");
  PG_CHECK_ARG(!(d->flags & PG_CONV_MASK) ||
                   (aux && (d->flags & PG_CONV_AUX_BITS ? d->aux_cs * 8 >= d->cout
                                                         : d->aux_cs >= d->cout)),
               "conv3x3_fwd: MASK flag without aux");
  PG_CHECK_ARG(!(d->flags & PG_CONV_Y2_BITS) || (y2 && d->y2_cs * 8 >= d->cout && d->y2_cs % 2 == 0),
               "conv3x3_fwd: Y2_BITS needs y2 with >= cout/8 bytes per pixel");
  PG_CHECK_ARG(!y2 || (d->flags & (PG_CONV_POOL | PG_CONV_PIXNORM | PG_CONV_PNBWD | PG_CONV_Y2_BITS)),
               "conv3x3_fwd: y2 only with POOL, PIXNORM, PNBWD or Y2_BITS");
  PG_CHECK_ARG(!(d->flags & PG_CONV_PNBWD) || (aux && y2 && d->aux_cs >= d->cout && d->aux_cs % 4 == 0),
               "conv3x3_fwd: PNBWD needs aux = y (aux_cs >= cout) and y2 = r");
  PG_CHECK_ARG(dtype == PG_F32 || dtype == PG_BF16, "conv3x3_fwd: bad dtype");
  PG_CHECK_ARG(!(d->flags & PG_CONV_X_BITS), "conv3x3_fwd: X_BITS needs pg_conv3x3_fwd_ex");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == PG_F32) return conv_dispatch<float>(d, x, wpk, bias, aux, y, y2, ws, ws_bytes, st);
  return conv_dispatch<bf16_t>(d, x, wpk, bias, aux, y, y2, ws, ws_bytes, st);
}

int pg_conv3x3_fwd_ex(int dtype, const pg_conv_desc* d, const void* x, const void* xbits,
                      const void* wpk, const float* bias, const void* aux, void* y, void* y2,
                      void* ws, size_t ws_bytes, void* stream) {
  if (!d || !(d->flags & PG_CONV_X_BITS))
    return pg_conv3x3_fwd(dtype, d, x, wpk, bias, aux, y, y2, ws, ws_bytes, stream);
  PG_CHECK_ARG(xbits && dtype == PG_BF16, "conv3x3_fwd_ex: X_BITS needs xbits (bf16)");
  PG_CHECK_ARG(x && wpk && y && d->cout % 4 == 0 && d->x_cs % 8 == 0 && d->y_cs >= d->cout,
               "conv3x3_fwd_ex: bad args");
  return conv_dispatch<bf16_t>(d, x, wpk, bias, aux, y, y2, ws, ws_bytes, (hipStream_t)stream, xbits);
}

int pg_conv3x3_rgbw(int dtype, const pg_conv_desc* d, const void* x, const void* wpk,
                    const void* aux, const float* img, float s, float* dw, float* db,
                    void* scratch, void* stream) {
  PG_CHECK_ARG(d && x && wpk && aux && img && dw && scratch, "conv3x3_rgbw: null pointer");
  PG_CHECK_ARG(dtype == PG_BF16 && (d->flags & PG_CONV_RGBW) && conv_supported<bf16_t>(d, 0),
               "conv3x3_rgbw: flags 0x%x not supported for %d -> %d at %dx%d", d->flags, d->cin,
               d->cout, d->H, d->W);
  PG_CHECK_ARG(d->x_cs >= cinp_of(d->cin) && d->x_cs % 8 == 0 && d->aux_cs * 8 >= d->cout,
               "conv3x3_rgbw: bad channel strides");
  PG_CHECK_ARG(pg_det_fits((size_t)256 * 8, (size_t)d->cout * 4), "conv3x3_rgbw: scratch too small");
  g_rgbw.img = img; g_rgbw.dw = dw; g_rgbw.db = db; g_rgbw.scratch = (float*)scratch; g_rgbw.s = s;
  const int rc = conv_dispatch<bf16_t>(d, x, wpk, nullptr, aux, nullptr, nullptr, nullptr, 0,
                                       (hipStream_t)stream);
  g_rgbw = RgbwArgs{};
  return rc;
}

int pg_conv3x3_rgbd(int dtype, const pg_conv_desc* d, const void* x, const void* wpk,
                    const void* aux, const float* w_rgb, float f, float* gimg, float* norms,
                    float* dw, float s, void* scratch, void* stream) {
  PG_CHECK_ARG(d && x && wpk && aux && w_rgb && gimg && scratch, "conv3x3_rgbd: null pointer");
  PG_CHECK_ARG(dtype == PG_BF16 && (d->flags & PG_CONV_RGBD) && conv_supported<bf16_t>(d, 0),
               "conv3x3_rgbd: flags 0x%x not supported for %d -> %d at %dx%d (B %d)", d->flags,
               d->cin, d->cout, d->H, d->W, d->B);
  PG_CHECK_ARG(d->x_cs >= cinp_of(d->cin) && d->x_cs % 8 == 0 && d->aux_cs * 8 >= d->cout,
               "conv3x3_rgbd: bad channel strides");
  PG_CHECK_ARG(pg_det_fits((size_t)256 * 8, (size_t)16 + d->cout * 4), "conv3x3_rgbd: scratch too small");
  g_rgbw = RgbwArgs{};
  g_rgbw.rw = w_rgb; g_rgbw.f = f; g_rgbw.gimg = gimg; g_rgbw.norms = norms; g_rgbw.dw = dw;
  g_rgbw.s = s; g_rgbw.scratch = (float*)scratch;
  const int rc = conv_dispatch<bf16_t>(d, x, wpk, nullptr, aux, nullptr, nullptr, nullptr, 0,
                                       (hipStream_t)stream);
  g_rgbw = RgbwArgs{};
  return rc;
}

int pg_conv3x3_rgbo(int dtype, const pg_conv_desc* d, const void* x, const void* wpk,
                    const float* bias, void* y, void* y2, const float* w_rgb, const float* b_rgb,
                    float c, float* img, void* stream) {
  PG_CHECK_ARG(d && x && wpk && bias && y && w_rgb && b_rgb && img, "conv3x3_rgbo: null pointer");
  PG_CHECK_ARG(dtype == PG_BF16 && (d->flags & PG_CONV_RGBO) && conv_supported<bf16_t>(d, 0),
               "conv3x3_rgbo: flags 0x%x not supported for %d -> %d at %dx%d", d->flags, d->cin,
               d->cout, d->H, d->W);
  PG_CHECK_ARG(d->x_cs >= cinp_of(d->cin) && d->x_cs % 8 == 0 && d->y_cs >= d->cout,
               "conv3x3_rgbo: bad channel strides");
  g_rgbw = RgbwArgs{};
  g_rgbw.rw = w_rgb; g_rgbw.rb = b_rgb; g_rgbw.f = c; g_rgbw.gimg = img;
  const int rc = conv_dispatch<bf16_t>(d, x, wpk, bias, nullptr, y, y2, nullptr, 0,
                                       (hipStream_t)stream);
  g_rgbw = RgbwArgs{};
  return rc;
}

int pg_conv3x3_supported(int dtype, const pg_conv_desc* d, size_t ws_bytes) {
  if (!d) return 0;
  return (dtype == PG_F32 ? conv_supported<float>(d, ws_bytes) : conv_supported<bf16_t>(d, ws_bytes))
             ? 1 : 0;
}

size_t pg_conv3x3_wgrad_workspace_size(int dtype, const pg_conv_desc* d) {
  if (!d) return 0;
  return dtype == PG_BF16 ? wgrad_bf16_ws_bytes(d) : wgrad_f32_ws_bytes(d);
}

int pg_conv3x3_wgrad(int dtype, const pg_conv_desc* d, const void* x, const void* gz, float scale,
                     float* dw, float* db, void* ws, size_t ws_bytes, void* stream) {
  PG_CHECK_ARG(d && x && gz && dw, "conv3x3_wgrad: null pointer");
  PG_CHECK_ARG(d->B > 0 && d->H >= 4 && d->W >= 4, "conv3x3_wgrad: bad spatial size");
  PG_CHECK_ARG(!(d->flags & PG_CONV_GZ_BITS), "conv3x3_wgrad: GZ_BITS needs pg_conv3x3_wgrad_ex");
  if (dtype == PG_BF16)
    return wgrad_bf16_dispatch(d, x, gz, scale, dw, db, (float*)ws, ws_bytes, (hipStream_t)stream);
  TileCfg tc = pick_tile(d->H, d->W, WG_BP, 32);
  WgParams p;
  p.x = x; p.gz = gz; p.dw = dw; p.db = db;
  p.B = d->B; p.H = d->H; p.W = d->W;
  p.ups = (d->flags & PG_CONV_UPS_IN) ? 1 : 0;
  p.Hin = p.ups ? d->H / 2 : d->H;
  p.Win = p.ups ? d->W / 2 : d->W;
  p.cin = d->cin; p.cout = d->cout; p.x_cs = d->x_cs; p.gz_cs = d->y_cs;
  p.scale = scale;
  p.NB = tc.NB; p.TH = tc.TH; p.TW = tc.TW;
  p.tiles_x = d->W / tc.TW;
  p.tiles_y = d->H / tc.TH;
  p.ntiles = pg_cdiv(d->B, tc.NB) * p.tiles_x * p.tiles_y;
  const int ot = pg_cdiv(d->cout, WG_BO), ct = pg_cdiv(d->cin, WG_BC);
  int splits = wgrad_f32_splits(d, &p.tiles_per_split);
  p.slab = (size_t)d->cout * d->cin * 9 + d->cout;
  p.ws = nullptr;
  if (splits > 1 && ws && ws_bytes >= splits * p.slab * sizeof(float)) {
    p.ws = (float*)ws;
  } else {   // no room for the slabs: one split (deterministic, slower)
    splits = 1;
    p.tiles_per_split = p.ntiles;
  }
  const int lds = (WG_BP * WG_RS + tc.NB * (tc.TH + 2) * (tc.TW + 2) * WG_RS) * 4;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid(ot, ct, splits);
  if (dtype == PG_F32)
    PG_KLAUNCH(wgrad3x3_kernel<float>, grid, dim3(256), lds, st, p);
  else
    PG_KLAUNCH(wgrad3x3_kernel<bf16_t>, grid, dim3(256), lds, st, p);
  if (p.ws)
    launch_slab_reduce(p.ws, p.slab, splits, d->cout * d->cin * 9, dw, db, scale, st);
  PG_LAUNCH_CHECK();
  return PG_OK;
}

int pg_conv3x3_wgrad_ex(int dtype, const pg_conv_desc* d, const void* x, const void* gz,
                        const void* gzbits, float scale, float* dw, float* db, void* ws,
                        size_t ws_bytes, void* stream) {
  if (!d || !(d->flags & PG_CONV_GZ_BITS))
    return pg_conv3x3_wgrad(dtype, d, x, gz, scale, dw, db, ws, ws_bytes, stream);
  PG_CHECK_ARG(x && gz && gzbits && dw && dtype == PG_BF16, "conv3x3_wgrad_ex: GZ_BITS needs gzbits (bf16)");
  PG_CHECK_ARG(d->B > 0 && d->H >= 4 && d->W >= 4 && d->H % 2 == 0 && d->W % 2 == 0,
               "conv3x3_wgrad_ex: bad spatial size");
  return wgrad_bf16_dispatch(d, x, gz, scale, dw, db, (float*)ws, ws_bytes, (hipStream_t)stream,
                             gzbits);
}

int pg_bias_grad(int dtype, int npix, int C, int cs, const void* g, float scale, float* db,
                 void* scratch, void* stream) {
  PG_CHECK_ARG(g && db && npix > 0 && C > 0 && C <= 1024 && cs >= C && scratch,
               "bias_grad: bad args (C <= 1024, scratch required)");
  int ppb = 256;
  int blocks = pg_cdiv(npix, ppb);
  int cap = (int)(pg_scratch_floats() / (size_t)C);
  if (cap > 2048) cap = 2048;
  if (blocks > cap) {
    blocks = cap;
    ppb = pg_cdiv(npix, blocks);
    blocks = pg_cdiv(npix, ppb);
  }
  hipStream_t st = (hipStream_t)stream;
  if (dtype == PG_F32)
    PG_KLAUNCH(bias_grad_kernel<float>, dim3(blocks), dim3(256), 0, st, npix, C, cs,
                       (const float*)g, scale, db, ppb, (float*)scratch);
  else
    PG_KLAUNCH(bias_grad_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, npix, C, cs,
                       (const bf16_t*)g, scale, db, ppb, (float*)scratch);
  PG_LAUNCH_CHECK();
  return PG_OK;
}

}  // extern "C"

// --------------------------------------------------------------------------
// Step plan: every 3x3 conv of G and D at one (stage, batch, dtype) with
// the kernel path each pass takes and the split-reduction workspace the step needs.
// Reference: the layer list of pggan/nets.py:53-119 (G), :164-239 (D) at scale_index.
namespace {
struct PlanLayer {
  char net, kind[8];
  int H, cin, cout, ups;
  int fwd_path, dgrad_path;   // 0 conv3x3 (split-K when ws > 0), 1 conv_hr tile t, 2 conv_lr
  int fwd_tile, dgrad_tile;
  size_t fwd_ws, dgrad_ws, wgrad_ws;
  int wg_MO, wg_WNC, wg_splits;
};
}  // namespace

struct pg_step_plan {
  int dtype, stage, batch;
  size_t ws_bytes;
  int n;
  PlanLayer layers[64];
};

namespace {
void plan_conv(int dtype, pg_conv_desc* d, int* path, int* tile, size_t* ws) {
  *ws = conv_ws_bytes(d);
  *path = 0;
  *tile = -1;
  if (dtype == PG_BF16) {
    if (conv_lr_ok(d)) { *path = 2; *ws = 0; return; }
    if (conv_hr_ok(d)) { *path = 1; *tile = conv_hr_tile(d); *ws = 0; }
  }
}
}  // namespace

extern "C" {

int pg_step_plan_create(int dtype, int n_depths, const int* depths, int stage, int batch,
                        pg_step_plan** out) {
  PG_CHECK_ARG(out && depths && stage >= 0 && stage + 1 <= n_depths && batch > 0 &&
                   (dtype == PG_F32 || dtype == PG_BF16),
               "step_plan_create: bad arguments");
  pg_step_plan* p = new pg_step_plan();
  p->dtype = dtype; p->stage = stage; p->batch = batch; p->ws_bytes = 0; p->n = 0;
  auto add = [&](char net, const char* kind, int H, int cin, int cout, int ups) {
    PlanLayer& L = p->layers[p->n++];
    L.net = net;
    snprintf(L.kind, sizeof(L.kind), "%s", kind);
    L.H = H; L.cin = cin; L.cout = cout; L.ups = ups;
    pg_conv_desc d{};
    d.B = batch; d.H = d.W = H; d.cin = cin; d.cout = cout;
    d.x_cs = cinp_of(cin); d.y_cs = (cout + 3) & ~3; d.flags = ups ? PG_CONV_UPS_IN : 0;
    plan_conv(dtype, &d, &L.fwd_path, &L.fwd_tile, &L.fwd_ws);
    pg_conv_desc g = d;   // input gradient: the transposed conv, cout -> cin channels
    g.cin = cout; g.cout = (cin + 3) & ~3; g.x_cs = cinp_of(cout); g.y_cs = g.cout; g.flags = 0;
    plan_conv(dtype, &g, &L.dgrad_path, &L.dgrad_tile, &L.dgrad_ws);
    L.wgrad_ws = dtype == PG_BF16 ? wgrad_bf16_ws_bytes(&d) : wgrad_f32_ws_bytes(&d);
    if (dtype == PG_BF16) {
      const WgbPlan w = wgrad_bf16_plan(&d);
      L.wg_MO = w.MO; L.wg_WNC = w.WNC; L.wg_splits = w.splits;
    } else {
      L.wg_MO = L.wg_WNC = 0; L.wg_splits = 1;
    }
    p->ws_bytes = std::max({p->ws_bytes, L.fwd_ws, L.dgrad_ws, L.wgrad_ws});
  };
  const int d0 = depths[0];
  add('G', "first", 4, d0, d0, 0);
  for (int i = 0; i < stage; ++i) {
    const int R = 8 << i;
    add('G', "a", R, depths[i], depths[i + 1], 1);
    add('G', "b", R, depths[i + 1], depths[i + 1], 0);
  }
  add('D', "mb", 4, d0 + 1, d0, 0);
  for (int i = 0; i < stage; ++i) {
    const int R = 8 << i;
    add('D', "a", R, depths[i + 1], depths[i + 1], 0);
    add('D', "b", R, depths[i + 1], depths[i], 0);
  }
  *out = p;
  return PG_OK;
}

size_t pg_step_plan_workspace_size(const pg_step_plan* plan) { return plan ? plan->ws_bytes : 0; }

int pg_step_plan_describe(const pg_step_plan* plan, char* buf, size_t len) {
  PG_CHECK_ARG(plan && buf && len > 0, "step_plan_describe: bad arguments");
  static const char* path[] = {"conv3x3", "conv_hr", "conv_lr"};
  size_t o = 0;
  auto put = [&](const char* fmt, auto... a) {
    if (o < len) o += snprintf(buf + o, len - o, fmt, a...);
  };
  put("stage %d batch %d dtype %s workspace %zu bytes\n", plan->stage, plan->batch,
      plan->dtype == PG_BF16 ? "bf16" : "f32", plan->ws_bytes);
  for (int i = 0; i < plan->n; ++i) {
    const PlanLayer& L = plan->layers[i];
    put("%c %-5s %4dx%-4d %3d->%-3d%s fwd %s", L.net, L.kind, L.H, L.H, L.cin, L.cout,
        L.ups ? " up2" : "    ", path[L.fwd_path]);
    if (L.fwd_path == 1) put("/t%d", L.fwd_tile);
    if (L.fwd_ws) put("/splitK");
    put("  dgrad %s", path[L.dgrad_path]);
    if (L.dgrad_path == 1) put("/t%d", L.dgrad_tile);
    if (L.dgrad_ws) put("/splitK");
    put("  wgrad MO%d WNC%d splits %d\n", L.wg_MO, L.wg_WNC, L.wg_splits);
  }
  return PG_OK;
}

void pg_step_plan_destroy(pg_step_plan* plan) { delete plan; }

}  // extern "C"
