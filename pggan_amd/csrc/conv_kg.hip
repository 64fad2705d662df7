// Wide bf16 3x3 convolutions on gfx950 (cout a multiple of 64, cin a multiple of 32, W a
// multiple of 16: the 32^2-256^2 levels of both nets, forward / input-gradient / R1 tangent):
// a K-grouped implicit GEMM.
//
//   tile      : TH rows x 16 columns of one image x 64 output channels per workgroup
//   waves     : 8 = two K-groups of four.  Wave (wr = wid & 3, kg = wid >> 2) owns rows
//               [wr*MT, wr*MT + MT) (MT = TH / 4) and all 64 channels (MT x 4 blocks of
//               v_mfma_f32_16x16x32_bf16, D[cout][pixel]) and computes the taps of each
//               32-channel chunk that belong to its K-group: taps 0-4 or 5-8, the halves
//               swapped every chunk, so both groups do 9 taps per two chunks.  Two waves per
//               SIMD with twice the per-wave tile of a one-group form at the same workgroup
//               tile: the k-loop probe (tools/kloop_probe.hip) runs 8 waves x (8x4 blocks) at
//               0.77 of the MFMA peak against 0.62-0.70 for 8 x (4x4) and 0.50 for the
//               4 x (2x4) of the 32^2 tile; the K-split is what makes the larger wave tile fit
//               the 256-workgroup grids of these levels.
//   staging   : each chunk's halo ((TH+2) x 18 pixels x 32 channels) and weight slab (64 x 9 x
//               32) go global -> LDS by buffer_load ... lds (no registers, no ds_write;
//               out-of-image halo pixels get an offset past the buffer range: the hardware
//               loads zeros), 16-B slots XOR-swizzled by bit 2 of the pixel column / weight row
//               (conflict-free fragment reads: tools/lds_banks.py); 3-slot ring (two chunks
//               in flight) when three slots fit in LDS, else two; one barrier per chunk.
//   reduction : the two groups' partial sums meet in LDS once per tile; afterwards group kg
//               holds output channels [32 kg, 32 kg + 32) of its rows (deterministic: one
//               fp32 add of the two partials).
//   epilogue  : bias, leaky ReLU, out_scale, lrelu' mask (bf16 aux), 2x2 pool (+ the pre-pool
//               copy in y2) per lane; the results are staged in LDS as [pixel][64 channels]
//               rows and written by whole 16-B pieces (8 pixel lines of 128 B per store
//               instruction); ACCUM and PixelNorm (sum of squares over a pixel's 8 lanes, r
//               to y2) are applied in that copy.
// Reference: lib/layers.py:58-89 (EqualizedConv2d incl. the bias x c), lib/blocks.py:113-201.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void kg_lds_t;

struct KgParams {
  const bf16_t* x;
  const bf16_t* w;
  const float* bias;
  const bf16_t* aux;
  bf16_t* y;
  void* y2;
  int B, H, W, Hin, Win;
  int cin_p, cout_p;
  int x_cs, y_cs, aux_cs, y2_cs;
  int flags;
  float slope, out_scale;
  int lg_tx, lg_ty;
  int xcd_remap;
  int diag;   // timing diagnostics (PG_KG_DIAG, wrong results): 1 no staging DMA, 4 no epilogue,
              // 8 / 16 contiguous weight / halo pieces (the feed with full-line requests)
};

// TH rows per tile; ONE: a single staging slot (LDS small enough for two workgroups per CU,
// each overlapping the other's staging and epilogue: the one- and two-chunk layers at >= 256^2)
template <int TH, bool ONE = false>
struct KgGeo {
  static constexpr int MT = TH / 4;
  static constexpr int HPIX = (TH + 2) * 18;
  static constexpr int HPIECES = (HPIX * 4 + 63) / 64;   // 1-KiB wave pieces (16 pixels)
  static constexpr int WPIECES = 64 * 9 * 4 / 64;         // 64 rows x 9 taps x 64 B
  static constexpr int NP = HPIECES + WPIECES;
  static constexpr int NPW = (NP + 7) / 8;                // pieces per wave (last round partial)
  static constexpr int HREG = HPIECES * 1024;
  static constexpr int SLOT = NP * 1024;
  static constexpr int NSLOT = ONE ? 1 : 3 * SLOT <= 160 * 1024 ? 3 : 2;
  static constexpr int XCH = 16 * MT * 1024;              // group exchange: 8 waves x MT x 2 KiB
  static constexpr int ORS = 144;                         // staged row: 64 ch + 16 B (banks)
  static constexpr int STG = TH * 16 * ORS;               // staged full-resolution rows
  static constexpr int STP = TH * 4 * ORS;                // staged pooled rows
  static constexpr int LDS0 = NSLOT * SLOT > XCH ? NSLOT * SLOT : XCH;
  static constexpr int LDS = LDS0 > STG + STP ? LDS0 : STG + STP;
  static_assert(NSLOT != 3 || NP % 8 == 0, "3-slot ring: the same DMA count in every wave");
  static_assert(LDS <= (ONE ? 80 : 160) * 1024, "conv_kg: LDS");
};

__device__ __forceinline__ int kg_swz(int x) { return ((x >> 2) & 1) << 1; }

// 16 B per lane global -> LDS (M0 + 16 * lane), untracked by the compiler (waited for by hand):
// the buffer resource from the base and byte range, scalar operands through readfirstlane
__device__ __forceinline__ void kg_dma16(const void* base, unsigned nrec, kg_lds_t* dst, unsigned voff,
                                         unsigned soff) {
  const size_t a = (size_t)base;
  const unsigned alo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned ahi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((size_t)ahi << 32) | alo), 0, __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
  soff = __builtin_amdgcn_readfirstlane(soff);
  const unsigned m0v = __builtin_amdgcn_readfirstlane((unsigned)(size_t)dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(m0v), "v"(voff), "s"(rs), "s"(soff) : "memory");
}

__device__ __forceinline__ float kg_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float kg_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

template <int TH, bool ONE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(ONE ? 4 : 2)))
void conv_kg_kernel(KgParams p) {
#if defined(__HIP_DEVICE_COMPILE__)
  using G = KgGeo<TH, ONE>;
  constexpr int MT = G::MT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid & 3, kg = wid >> 2;
  const int g = lane >> 4, r = lane & 15;

  // (pixel tile, output-channel block); with xcd_remap the hardware's round-robin dealing of
  // blocks over the 8 XCDs is undone so XCD k owns a contiguous band of logical ids (channel
  // block fastest): the tiles of one XCD share halos and every conv of a level reads rows the
  // same XCD's previous conv of that level wrote (speed only)
  int tile = blockIdx.x, cblk = blockIdx.y;
  if (p.xcd_remap) {
    const int gx = gridDim.x, gy = gridDim.y, n = gx * gy;
    const int h = blockIdx.x + gx * blockIdx.y;
    const int xcd = h & 7, slot = h >> 3, q = n >> 3, rr = n & 7;
    const int Lg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + slot;
    cblk = Lg % gy;
    tile = Lg / gy;
  }
  const int n0 = cblk * 64;
  const int tiles_x = 1 << p.lg_tx, tiles_y = 1 << p.lg_ty;
  const int tx0 = (tile & (tiles_x - 1)) * 16;
  const int ty0 = ((tile >> p.lg_tx) & (tiles_y - 1)) * TH;
  const int b = tile >> (p.lg_tx + p.lg_ty);
  const int ys = (p.flags & PG_CONV_UPS_IN) ? 1 : 0;
  const int nch = p.cin_p >> 5;

  // ---- DMA plan of this lane: byte offset of its 16 B in each of its pieces (the same for
  // every chunk; the chunk enters as the scalar channel offset)
  constexpr unsigned OOB = 0x7fff0000u;
  const unsigned x_nrec = (unsigned)((size_t)p.B * p.Hin * p.Win * p.x_cs * 2);
  const unsigned w_nrec = (unsigned)((size_t)p.cout_p * 9 * p.cin_p * 2);
  const unsigned img_off = (unsigned)b * (unsigned)(p.Hin * p.Win * p.x_cs * 2);
  auto piece_off = [&](int k, int lane) __attribute__((always_inline)) -> unsigned {
    const int q = wid + 8 * k;
    unsigned v = OOB;
    if (q < G::HPIECES) {
      const int sl = q * 64 + lane, P = sl >> 2;
      const int hy = P / 18, hx = P - hy * 18;
      const int j = (sl & 3) ^ kg_swz(hx);
      const int yy = ty0 + hy - 1, xx = tx0 + hx - 1;
      if (P < G::HPIX && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W)
        v = (unsigned)((((yy >> ys) * p.Win + (xx >> ys)) * p.x_cs + 8 * j) * 2);
      // feed diagnostic (PG_KG_DIAG & 16, wrong results): the same bytes as contiguous 1-KiB runs
      if (p.diag & 16) v = (unsigned)((((ty0 * p.Win + tx0) * p.x_cs) * 2 + sl * 16) & 0x3fffff);
    } else if (q < G::NP) {
      const int sl = (q - G::HPIECES) * 64 + lane, nr = sl / 36, sr = sl - nr * 36;
      const int tap = sr >> 2, j = (sr & 3) ^ kg_swz(nr);
      v = (unsigned)((((n0 + nr) * 9 + tap) * p.cin_p + 8 * j) * 2);
      // (PG_KG_DIAG & 8: the weight slab as one contiguous run, as a chunk-major packing gives)
      if (p.diag & 8) v = (unsigned)(n0 * 9 * p.cin_p * 2 + sl * 16);
    }
    return v;
  };
  // held in registers, except by the 8-row tile (its accumulators need them: recomputed at
  // each issue, ~15 VALU per piece against 288 MFMAs per chunk)
  constexpr bool HOLD = MT <= 4;
  unsigned voff[HOLD ? G::NPW : 1];
  if constexpr (HOLD) {
#pragma unroll
    for (int k = 0; k < G::NPW; ++k) voff[k] = piece_off(k, lane);
  }
  auto dma_chunk = [&](int c, int sl) __attribute__((always_inline)) {
    char* base = smem + sl * G::SLOT;
    // !HOLD: the lane index made opaque here, so the offsets are computed at the issue and not
    // hoisted out of the chunk loop (which is what spilled them)
    int ln = lane;
    if constexpr (!HOLD) asm volatile("" : "+v"(ln));
#pragma unroll
    for (int k = 0; k < G::NPW; ++k) {
      const int q = wid + 8 * k;   // wave-uniform
      if (q < G::HPIECES) {
        kg_dma16(p.x, x_nrec, (kg_lds_t*)(base + q * 1024), HOLD ? voff[HOLD ? k : 0] : piece_off(k, ln),
                 img_off + c * 64);
      } else if (q < G::NP) {
        kg_dma16(p.w, w_nrec, (kg_lds_t*)(base + q * 1024), HOLD ? voff[HOLD ? k : 0] : piece_off(k, ln), c * 64);
      }
    }
  };

  // ---- fragment addresses (bytes inside a slot): weight row r of block nt, tap t; halo row
  // wr*MT + mt + dy, column r + dx
  const int wlane = G::HREG + r * 576 + ((g ^ kg_swz(r)) << 4);
  int hl[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) hl[dx] = ((wr * MT) * 18 + r + dx) * 64 + ((g ^ kg_swz(r + dx)) << 4);

  f32x4_t acc[MT][4];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // taps [t0, t0 + ntap) of the chunk in slot base sb, one rolled iteration per tap (both
  // K-groups' tap ranges run the same code: two unrolled instances behind a branch kept the
  // registers of both live), software-pipelined: the next pixel block's halo fragment is read
  // before this block's MFMAs, the next tap's weight fragments right after their last use and
  // its first halo fragment with this tap's last block
  auto compute = [&](int t0, int ntap, const char* sb) __attribute__((always_inline)) {
    auto tap_base = [&](int t, const char*& wt, const char*& xt) __attribute__((always_inline)) {
      const int dy = (t * 11) >> 5, dx = t - 3 * dy;   // t / 3, t % 3 for t < 9
      const int h = dx == 0 ? hl[0] : dx == 1 ? hl[1] : hl[2];
      wt = sb + wlane + t * 64;
      xt = sb + h + dy * (18 * 64);
    };
    const char *wt, *xt;
    tap_base(t0, wt, xt);
    bf16x8_t wf[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) wf[nt] = *reinterpret_cast<const bf16x8_t*>(wt + nt * 16 * 576);
    bf16x8_t xf = *reinterpret_cast<const bf16x8_t*>(xt);
#pragma unroll 1
    for (int i = 0; i < ntap; ++i) {
      const int tn = t0 + (i + 1 < ntap ? i + 1 : i);
      const char *wn, *xn0;
      tap_base(tn, wn, xn0);
      bf16x8_t wnx[4];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const bool lastm = mt + 1 == MT;
        const bf16x8_t xn = *reinterpret_cast<const bf16x8_t*>(lastm ? xn0 : xt + (mt + 1) * (18 * 64));
        if constexpr (MT > 4) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nt], xf, acc[mt][nt], 0, 0, 0);
          if (lastm) wnx[nt] = *reinterpret_cast<const bf16x8_t*>(wn + nt * 16 * 576);
        }
        if constexpr (MT > 4) __builtin_amdgcn_sched_barrier(0);
        xf = xn;
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) wf[nt] = wnx[nt];
      xt = xn0;
    }
  };

  // ---- the chunk ring
  const bool dma_on = !(p.diag & 1);
  if (dma_on) dma_chunk(0, 0);
  if (dma_on && G::NSLOT == 3 && nch > 1) dma_chunk(1, 1);
  for (int c = 0; c < nch; ++c) {
    if constexpr (G::NSLOT == 3) {
      if (c + 1 < nch) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::NPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    // chunk c landed for every wave; every wave is done reading the slot refilled next
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr (G::NSLOT > 1) {
      const int ahead = G::NSLOT - 1;
      if (dma_on && c + ahead < nch) dma_chunk(c + ahead, (c + ahead) % G::NSLOT);
    } else if (c > 0) {
      // one slot: chunk c was issued after chunk c-1's reads (below); nothing to issue here
    }
    const char* sb = smem + (c % G::NSLOT) * G::SLOT;
    const bool lo = ((c & 1) ^ kg) == 0;   // this group's taps of chunk c: 0-4 or 5-8
    compute(lo ? 0 : 5, lo ? 5 : 4, sb);
    if constexpr (G::NSLOT == 1) {
      if (c + 1 < nch) {   // the only slot is free once every wave is past its reads
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (dma_on) dma_chunk(c + 1, 0);
      }
    }
  }

  // ---- epilogue operands: bias and the lrelu' mask of this wave's output half
  const int nbase = n0 + kg * 32;   // after the exchange: channels [nbase, nbase + 32)
  const bool do_bias = (p.flags & PG_CONV_BIAS) != 0, do_lrelu = (p.flags & PG_CONV_LRELU) != 0;
  const bool do_mask = (p.flags & PG_CONV_MASK) != 0, pool = (p.flags & PG_CONV_POOL) != 0;
  const bool do_acc = (p.flags & PG_CONV_ACCUM) != 0, do_pn = (p.flags & PG_CONV_PIXNORM) != 0;
  const size_t img = (size_t)b * p.H * p.W;
  float bv[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[h][j] = do_bias ? p.bias[nbase + h * 16 + 4 * g + j] : 0.f;
  // ---- the two K-groups' partial sums: wave (wr, kg) sends the other half's blocks to its
  // partner (wr, 1 - kg) and adds the partner's partial of its own half
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  {
    char* xo = smem + ((wr * 2 + (1 - kg)) * MT * 2) * 1024 + lane * 16;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        *reinterpret_cast<f32x4_t*>(xo + (mt * 2 + h) * 1024) = kg ? acc[mt][h] : acc[mt][2 + h];
  }
  __syncthreads();
  // the result of half h of row mt lands in acc[mt][h] (the other half's registers die here)
  {
    const char* xi = smem + ((wr * 2 + kg) * MT * 2) * 1024 + lane * 16;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4_t o = *reinterpret_cast<const f32x4_t*>(xi + (mt * 2 + h) * 1024);
        // both halves add group 0's partial + group 1's (fp32 add is commutative: the same sum)
        acc[mt][h] = (kg ? acc[mt][2 + h] : acc[mt][h]) + o;
      }
  }
  __syncthreads();   // the exchange region becomes the staging area
  if (p.diag & 4) return;
  u32x2_t am[MT][2];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      am[mt][h] = u32x2_t{0u, 0u};
      if (do_mask) {
        const int lp = (ty0 + wr * MT + mt) * p.W + tx0 + r;
        am[mt][h] = *reinterpret_cast<const u32x2_t*>(p.aux + img * p.aux_cs +
                                                       (unsigned)(lp * p.aux_cs + nbase + h * 16 + 4 * g));
      }
    }


  char* st = smem;                 // [TH*16 pixels][64 ch] rows (full resolution)
  char* stp = smem + G::STG;       // [TH*4 pixels][64 ch] rows (pooled)
  auto stage4 = [&](char* s, int pl, int h, const float (&o)[4]) {
    u32x2_t q;
    q[0] = pack_bf16x2(o[0], o[1]);
    q[1] = pack_bf16x2(o[2], o[3]);
    *reinterpret_cast<u32x2_t*>(s + pl * G::ORS + (kg * 2 + h) * 32 + g * 8) = q;
  };
  auto mask4 = [&](float (&v)[4], const u32x2_t& m) {
    v[0] *= lmask_f(kg_lo(m[0]), p.slope);
    v[1] *= lmask_f(kg_hi(m[0]), p.slope);
    v[2] *= lmask_f(kg_lo(m[1]), p.slope);
    v[3] *= lmask_f(kg_hi(m[1]), p.slope);
  };
  if (!pool) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = acc[mt][h][j] + bv[h][j];
          if (do_lrelu) v[j] = lrelu_f(v[j], p.slope);
          v[j] *= p.out_scale;
        }
        if (do_mask) mask4(v, am[mt][h]);
        stage4(st, (wr * MT + mt) * 16 + r, h, v);
      }
  } else {
    const bool keep = p.y2 != nullptr;   // the pre-pool activation as well
#pragma unroll
    for (int mt = 0; mt < MT; mt += 2)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float v[4], u[4], s[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = acc[mt][h][j] + bv[h][j];
          u[j] = acc[mt + 1][h][j] + bv[h][j];
          if (do_lrelu) {
            v[j] = lrelu_f(v[j], p.slope);
            u[j] = lrelu_f(u[j], p.slope);
          }
        }
        if (keep) {
          stage4(st, (wr * MT + mt) * 16 + r, h, v);
          stage4(st, (wr * MT + mt + 1) * 16 + r, h, u);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float sm = v[j] + u[j];
          s[j] = (sm + __shfl_xor(sm, 1, 64)) * p.out_scale;
        }
        if ((r & 1) == 0) stage4(stp, ((wr * MT + mt) >> 1) * 8 + (r >> 1), h, s);
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- copy-out: thread = 16 B (8 channels) of one staged pixel row
  auto copy_out = [&](auto NPXc, auto TCc, const char* s, bf16_t* dst0, int cs, int row0, int col0, int Wo,
                      bool accum, bool pn) __attribute__((always_inline)) {
    constexpr int NPX = decltype(NPXc)::value, TC = decltype(TCc)::value;
    constexpr int ITER = (NPX * 8 + 511) / 512;
#pragma unroll
    for (int k = 0; k < ITER; ++k) {
      const int i = tid + k * 512;
      if ((NPX * 8) % 512 != 0 && i >= NPX * 8) break;
      const int pl = i >> 3, sg = i & 7;
      u32x4_t v = *reinterpret_cast<const u32x4_t*>(s + pl * G::ORS + sg * 16);
      const int gp = (row0 + pl / TC) * Wo + col0 + pl % TC;
      bf16_t* dst = dst0 + (unsigned)(gp * cs + n0 + sg * 8);
      if (pn) {   // PixelNorm over the 64 channels = the 8 lanes of this pixel
        float ss = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) ss += kg_lo(v[e]) * kg_lo(v[e]) + kg_hi(v[e]) * kg_hi(v[e]);
        ss += __shfl_xor(ss, 1, 64);
        ss += __shfl_xor(ss, 2, 64);
        ss += __shfl_xor(ss, 4, 64);
        const float rn = rsqrtf(ss / 64.f + 1e-8f);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = pack_bf16x2(kg_lo(v[e]) * rn, kg_hi(v[e]) * rn);
        if (p.y2 && sg == 0) reinterpret_cast<float*>(p.y2)[img + gp] = rn;
      }
      if (accum) {
        const u32x4_t o = *reinterpret_cast<const u32x4_t*>(dst);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = pack_bf16x2(kg_lo(v[e]) + kg_lo(o[e]), kg_hi(v[e]) + kg_hi(o[e]));
      }
      *reinterpret_cast<u32x4_t*>(dst) = v;
    }
  };
  using NFULL = std::integral_constant<int, TH * 16>;
  using NPOOL = std::integral_constant<int, TH * 4>;
  using C16 = std::integral_constant<int, 16>;
  using C8 = std::integral_constant<int, 8>;
  if (!pool) {
    copy_out(NFULL{}, C16{}, st, p.y + img * p.y_cs, p.y_cs, ty0, tx0, p.W, do_acc, do_pn);
  } else {
    if (p.y2)
      copy_out(NFULL{}, C16{}, st, reinterpret_cast<bf16_t*>(p.y2) + img * p.y2_cs, p.y2_cs, ty0, tx0, p.W, false,
               false);
    copy_out(NPOOL{}, C8{}, stp, p.y + (img >> 2) * p.y_cs, p.y_cs, ty0 >> 1, tx0 >> 1, p.W >> 1, do_acc, false);
  }
#endif
}

template <int TH, bool ONE>
int launch_kg(const pg_conv_desc* d, const void* x, const void* wpk, const float* bias, const void* aux, void* y,
              void* y2, hipStream_t st) {
  using G = KgGeo<TH, ONE>;
  KgParams p{};
  p.x = (const bf16_t*)x; p.w = (const bf16_t*)wpk; p.bias = bias; p.aux = (const bf16_t*)aux;
  p.y = (bf16_t*)y; p.y2 = y2;
  p.B = d->B; p.H = d->H; p.W = d->W;
  const bool ups = (d->flags & PG_CONV_UPS_IN) != 0;
  p.Hin = ups ? d->H / 2 : d->H;
  p.Win = ups ? d->W / 2 : d->W;
  p.cin_p = (d->cin + 31) & ~31;
  p.cout_p = d->cout;
  p.x_cs = d->x_cs; p.y_cs = d->y_cs; p.aux_cs = d->aux_cs; p.y2_cs = d->y2_cs;
  p.flags = d->flags; p.slope = d->slope; p.out_scale = d->out_scale;
  p.lg_tx = 0;
  while ((1 << p.lg_tx) < d->W / 16) ++p.lg_tx;
  p.lg_ty = 0;
  while ((1 << p.lg_ty) < d->H / TH) ++p.lg_ty;
  static const int xcd = getenv("PG_KG_XCD") ? atoi(getenv("PG_KG_XCD")) : 1;   // A/B switch
  static const int diag = getenv("PG_KG_DIAG") ? atoi(getenv("PG_KG_DIAG")) : 0;   // timing only
  p.xcd_remap = xcd;
  p.diag = diag;
  PG_LDS_ATTR((conv_kg_kernel<TH, ONE>), G::LDS);
  const int ntiles = d->B * (d->W / 16) * (d->H / TH);
  PG_KLAUNCH((conv_kg_kernel<TH, ONE>), dim3(ntiles, d->cout / 64), dim3(512), G::LDS, st, p);
  PG_LAUNCH_CHECK();
  return PG_OK;
}

// The variant a conv takes: 0 none (conv_hr), 8 / 16 / 32 the two- or three-slot tiles of
// that many rows, -16 the one-slot 16-row tile (two workgroups per CU).  Measured (kbench,
// PG_KG=2 forces every eligible shape for A/B): the 16-row two-slot tile wins at 64^2 without
// pooling; at 128^2 and for the pooled 64^2 layers conv_hr's tiles are as fast or faster; the
// one- / two-chunk layers at >= 256^2 run one workgroup per CU with everything exposed in
// conv_hr, which the one-slot form overlaps.
// Whole-step A/B (profiles/r4_kg_ab.txt): neutral at C5 (350.7 vs 350.2 img/s with / without),
// slower at C3 (475.3 vs 480.9) and C4's shard (541.5 vs 548.3), so it is opt-in (PG_KG=1).
int kg_variant(const pg_conv_desc* d) {
  const char* env = getenv("PG_KG");   // read per call: the op tests switch it within a process
  const int mode = env ? atoi(env) : 0;
  if (!mode) return 0;
  const int cin_p = (d->cin + 31) & ~31;
  const bool pool = (d->flags & PG_CONV_POOL) != 0;
  if (mode == 2) return d->H >= 256 && cin_p <= 64 ? -16 : d->H >= 128 ? 32 : d->H >= 64 ? 16 : 8;
  // (with MASK the one-slot form is slower: its mask operands spill at 128 registers)
  if (d->H >= 256 && cin_p <= 64 && !(d->flags & PG_CONV_MASK)) return -16;
  if (d->H == 64 && !pool) return 16;
  return 0;
}
}  // namespace

// Whether conv_kg takes this bf16 conv (PG_KG=0, the default: never; 1: the shapes kg_variant
// picks; 2: every eligible shape; A/B runs).
bool conv_kg_ok(const pg_conv_desc* d) {
  const int v = kg_variant(d);
  if (!v) return false;
  constexpr int OK = PG_CONV_UPS_IN | PG_CONV_BIAS | PG_CONV_LRELU | PG_CONV_MASK | PG_CONV_POOL |
                     PG_CONV_ACCUM | PG_CONV_PIXNORM;
  if (d->flags & ~OK) return false;
  if ((d->flags & PG_CONV_MASK) && (d->flags & PG_CONV_POOL)) return false;
  if ((d->flags & PG_CONV_PIXNORM) && (d->cout != 64 || (d->flags & (PG_CONV_POOL | PG_CONV_MASK | PG_CONV_ACCUM))))
    return false;
  if (d->cout % 64 || d->cin % 32 || d->W % 16 || d->B <= 0) return false;
  const int th = v < 0 ? -v : v;
  if (d->H % th || d->H < th) return false;
  const int tx = d->W / 16, ty = d->H / th;
  if ((tx & (tx - 1)) || (ty & (ty - 1))) return false;
  if ((d->flags & PG_CONV_POOL) && (d->H & 1)) return false;
  if (d->x_cs % 8 || d->y_cs % 8 || ((d->flags & PG_CONV_MASK) && d->aux_cs % 4) ||
      ((d->flags & PG_CONV_POOL) && d->y2_cs % 8))
    return false;
  // enough workgroups for the chip (the 16^2 levels stay on the split-K kernel)
  if ((long)d->B * tx * ty * (d->cout / 64) < 256) return false;
  const bool ups = (d->flags & PG_CONV_UPS_IN) != 0;
  const size_t xin = (size_t)d->B * (ups ? d->H / 2 : d->H) * (ups ? d->W / 2 : d->W) * d->x_cs * 2;
  // out-of-image halo slots load with offset 0x7fff0000: it must be past the buffer's range
  return xin <= 0x7fff0000ull && (size_t)d->cout * 9 * d->cin * 2 < 0x7fff0000ull &&
         (size_t)d->H * d->W * std::max(d->y_cs, std::max(d->aux_cs, d->y2_cs)) < (1ull << 31);
}

int conv_kg_dispatch(const pg_conv_desc* d, const void* x, const void* wpk, const float* bias, const void* aux,
                     void* y, void* y2, hipStream_t st) {
  PG_CHECK_ARG(conv_kg_ok(d), "conv_kg: unsupported conv");
  switch (kg_variant(d)) {
    case 8: return launch_kg<8, false>(d, x, wpk, bias, aux, y, y2, st);
    case 16: return launch_kg<16, false>(d, x, wpk, bias, aux, y, y2, st);
    case -16: return launch_kg<16, true>(d, x, wpk, bias, aux, y, y2, st);
    default: return launch_kg<32, false>(d, x, wpk, bias, aux, y, y2, st);
  }
}
