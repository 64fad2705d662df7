// k-loop probe (GPU box): the MFMA + LDS-fragment-read loop of an implicit-GEMM conv tile
// with no global memory traffic, to find the structure that runs the matrix pipe closest to
// its peak.  Every workgroup fills its LDS once (random bf16), then runs `nch` chunks of
// KS k-steps; per k-step each wave reads NB A fragments + MB B fragments (ds_read_b128,
// contiguous 1 KiB per wave read: conflict-free) and issues MB x NB MFMAs.
//   MF = 16: v_mfma_f32_16x16x32_bf16 (k 32 per MFMA, 9 k-steps per 32-channel tap chunk)
//   MF = 32: v_mfma_f32_32x32x16_bf16 (k 16 per MFMA, 18 k-steps per chunk)
//   BAR: s_barrier after every chunk (the staging ring's hand-off); PIPE: the next k-step's
//   fragments read before this k-step's MFMAs (register double buffer)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/kloop_probe tools/kloop_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

template <int MF> struct Acc;
template <> struct Acc<16> { typedef f32x4_t T; };
template <> struct Acc<32> { typedef f32x16_t T; };

template <int MF>
__device__ __forceinline__ typename Acc<MF>::T mma(bf16x8_t a, bf16x8_t b, typename Acc<MF>::T c) {
  if constexpr (MF == 16) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

template <int MF, int NW, int MB, int NB, int KS, bool BAR, bool PIPE, int WPE>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(WPE)))
void kloop(float* out, int nch, int region_kib) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  // random-ish bf16 (not zero: zero operands let the chip hold a higher clock)
  for (int i = tid; i < region_kib * 256; i += NW * 64) {
    unsigned h = (unsigned)i * 2654435761u + blockIdx.x * 97u;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    const unsigned lo = 0x3c00u + (h & 0x3ffu), hi = 0x3c00u + ((h >> 16) & 0x3ffu);
    reinterpret_cast<unsigned*>(lds)[i] = (lo | (hi << 16)) ^ ((h & 0x80008000u));
  }
  __syncthreads();
  typedef typename Acc<MF>::T AT;
  AT acc[MB][NB];
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[m][n] = AT{};
  // A region: NB x KS KiB per wave (shared by all waves, as a weight slab); B region: the
  // pixel blocks of this wave
  const int wmask = region_kib / 2 - 1;   // KiB slots in each half (power of two)
  const char* A = lds;
  const char* Bb = lds + (region_kib / 2) * 1024;
  auto rdA = [&](int ks, int n) {
    return *reinterpret_cast<const bf16x8_t*>(A + (((ks * NB + n) & wmask) * 1024) + lane * 16);
  };
  auto rdB = [&](int ks, int m) {
    return *reinterpret_cast<const bf16x8_t*>(Bb + (((wid * MB * 3 + ks * 2 + m) & wmask) * 1024) + lane * 16);
  };
  for (int c = 0; c < nch; ++c) {
    if constexpr (PIPE) {
      bf16x8_t a[NB], b[MB];
#pragma unroll
      for (int n = 0; n < NB; ++n) a[n] = rdA(0, n);
#pragma unroll
      for (int m = 0; m < MB; ++m) b[m] = rdB(0, m);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8_t a2[NB], b2[MB];
        const int k1 = ks + 1 < KS ? ks + 1 : ks;
#pragma unroll
        for (int n = 0; n < NB; ++n) a2[n] = rdA(k1, n);
#pragma unroll
        for (int m = 0; m < MB; ++m) b2[m] = rdB(k1, m);
#pragma unroll
        for (int m = 0; m < MB; ++m)
#pragma unroll
          for (int n = 0; n < NB; ++n) acc[m][n] = mma<MF>(a[n], b[m], acc[m][n]);
#pragma unroll
        for (int n = 0; n < NB; ++n) a[n] = a2[n];
#pragma unroll
        for (int m = 0; m < MB; ++m) b[m] = b2[m];
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8_t a[NB], b[MB];
#pragma unroll
        for (int n = 0; n < NB; ++n) a[n] = rdA(ks, n);
#pragma unroll
        for (int m = 0; m < MB; ++m) b[m] = rdB(ks, m);
#pragma unroll
        for (int m = 0; m < MB; ++m)
#pragma unroll
          for (int n = 0; n < NB; ++n) acc[m][n] = mma<MF>(a[n], b[m], acc[m][n]);
      }
    }
    if constexpr (BAR) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
  float s = 0.f;
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int j = 0; j < (MF == 16 ? 4 : 16); ++j) s += acc[m][n][j];
  if (s == 12345.678f) out[blockIdx.x * NW * 64 + tid] = s;
}

template <int MF, int NW, int MB, int NB, int KS, bool BAR, bool PIPE, int WPE = 1>
void run(const char* name, float* out, int wg_per_cu, int lds_kib) {
  auto k = kloop<MF, NW, MB, NB, KS, BAR, PIPE, WPE>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  const int grid = 256 * wg_per_cu, nch = 64;
  const size_t lds = (size_t)lds_kib * 1024;
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k, NW * 64, lds));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), lds, 0, out, nch, lds_kib);
  CK(hipEventRecord(a));
  const int reps = 40;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), lds, 0, out, nch, lds_kib);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double kk = MF == 16 ? 32 : 16;
  const double flops = (double)reps * grid * NW * nch * KS * MB * NB * 2.0 * MF * MF * kk;
  const double us = ms * 1e3 / reps;
  printf("%-44s occ %d/CU  %8.1f us  %7.1f TF/s  (%.3f of 2.5 PF)\n", name, occ, us,
         flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 2.5e15);
  fflush(stdout);
}

int main() {
  float* out;
  CK(hipMalloc(&out, 1 << 24));
  // tile 3 today: 8 waves, 4x4 16x16 blocks (64 px x 64 co per wave), barrier per chunk
  run<16, 8, 4, 4, 9, true, false>("mf16 w8 4x4 bar", out, 1, 64);
  run<16, 8, 4, 4, 9, true, true>("mf16 w8 4x4 bar pipe", out, 1, 64);
  run<16, 4, 4, 4, 9, true, false>("mf16 w4 4x4 bar", out, 1, 64);
  run<16, 4, 4, 4, 9, true, true>("mf16 w4 4x4 bar pipe", out, 1, 64);
  run<16, 4, 4, 4, 9, true, false, 2>("mf16 w4 4x4 bar 2wg/cu", out, 2, 64);
  run<16, 8, 8, 4, 9, true, false>("mf16 w8 8x4 bar", out, 1, 64);
  run<16, 4, 8, 4, 9, true, false>("mf16 w4 8x4 bar", out, 1, 64);
  run<16, 4, 8, 4, 9, true, true>("mf16 w4 8x4 bar pipe", out, 1, 64);
  // small wave tiles (the 8^2-32^2 convs): 32 px x 64 co and 32 x 32 per wave
  run<16, 8, 2, 4, 9, true, false>("mf16 w8 2x4 bar", out, 1, 64);
  run<16, 4, 2, 4, 9, true, false>("mf16 w4 2x4 bar", out, 1, 64);
  run<16, 8, 2, 2, 9, true, false>("mf16 w8 2x2 bar", out, 1, 64);
  run<16, 8, 1, 4, 9, true, false>("mf16 w8 1x4 bar", out, 1, 64);
  run<16, 8, 4, 2, 9, true, false>("mf16 w8 4x2 bar", out, 1, 64);
  run<16, 8, 2, 4, 9, true, false, 2>("mf16 w8 2x4 bar 2wg/cu", out, 2, 64);
  // 32x32x16: 2x2 blocks = the same 64 x 64 per wave
  run<32, 8, 2, 2, 18, true, false>("mf32 w8 2x2 bar", out, 1, 64);
  run<32, 8, 2, 2, 18, true, true>("mf32 w8 2x2 bar pipe", out, 1, 64);
  run<32, 4, 2, 2, 18, true, false>("mf32 w4 2x2 bar", out, 1, 64);
  run<32, 4, 2, 2, 18, true, true>("mf32 w4 2x2 bar pipe", out, 1, 64);
  run<32, 4, 2, 2, 18, true, false, 2>("mf32 w4 2x2 bar 2wg/cu", out, 2, 64);
  run<32, 8, 4, 2, 18, true, false>("mf32 w8 4x2 bar", out, 1, 64);
  return 0;
}
