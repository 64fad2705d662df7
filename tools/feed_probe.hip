// Per-CU feed probe (GPU box): how many bytes per second one CU pulls from L2 with
// LDS-DMA (global_load_lds_dwordx4) vs ordinary 16-B register loads, as a function of the
// waves per workgroup and the 1-KiB wave loads each wave keeps in flight before it waits.
// One workgroup per CU (256), every workgroup streams a 2 MiB window shared by all of them
// (L2-resident after the first pass, like the conv tiles' halo and weight re-reads).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/feed_probe tools/feed_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

constexpr size_t WIN = 2u << 20;

// piece: contiguous bytes per lane group (1024 = one contiguous KiB per wave load; 64 = the
// conv tiles' halo pattern, 64 B of every `stride` bytes); win: the span the addresses wrap
// in (2 MiB: L2-resident; 512 MiB: beyond the MALL, every pass from HBM)
// (piece, stride, win: powers of two, so the address math is shifts and masks and the
// probe measures the memory path, not a 64-bit division per load)
__device__ __forceinline__ size_t paddr(size_t logical, int piece, int stride, size_t win) {
  const int lp = __builtin_ctz(piece), ls = __builtin_ctz(stride);
  return (((logical >> lp) << ls) | (logical & (size_t)(piece - 1))) & (win - 1);
}
template <int NW, int DEPTH, bool DMA>
__global__ __launch_bounds__(NW * 64) void feed(const char* __restrict__ src, int rounds,
                                                unsigned* __restrict__ sink, int piece, int stride,
                                                size_t win, int pair) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned acc = 0;
  // L2 case: every workgroup walks the same window from its own offset; HBM case (win >
  // 2 MiB): disjoint per-workgroup spans
  const size_t span = win > WIN ? (win / gridDim.x) * piece / stride : 8192;
  size_t off = (size_t)blockIdx.x * span + (size_t)wid * DEPTH * 1024;
  for (int it = 0; it < rounds; ++it) {
    if constexpr (DMA) {
#pragma unroll
      for (int k = 0; k < DEPTH; ++k) {
        const size_t o = (paddr(off + (size_t)k * 1024 + lane * 16, piece, stride, win) + ((pair & it) ? piece : 0)) & (win - 1);
        __builtin_amdgcn_global_load_lds((const void*)(src + o),
                                         (__attribute__((address_space(3))) void*)(lds + (wid * DEPTH + k) * 1024),
                                         16, 0, 0);
      }
      __syncthreads();
    } else {
      uint4 v[DEPTH];
#pragma unroll
      for (int k = 0; k < DEPTH; ++k) {
        const size_t o = (paddr(off + (size_t)k * 1024 + lane * 16, piece, stride, win) + ((pair & it) ? piece : 0)) & (win - 1);
        v[k] = *reinterpret_cast<const uint4*>(src + o);
      }
#pragma unroll
      for (int k = 0; k < DEPTH; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (!(pair & ~it & 1)) off += (size_t)NW * DEPTH * 1024;   // pair: advance after the odd round
  }
  if constexpr (DMA) acc = *reinterpret_cast<const unsigned*>(lds + lane * 16);
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;   // keeps the loads live
}

template <int NW, int DEPTH, bool DMA>
void run(const char* src, unsigned* sink, int piece = 1024, int stride = 1024, size_t win = WIN, int pair = 0) {
  // logical bytes per workgroup: 2 MiB, or its own disjoint span of the HBM window
  size_t lb = win > WIN ? (win / 256) * piece / stride : (2u << 20);
  if (lb < (512u << 10)) lb = 512u << 10;   // small windows (MALL-resident): wrap
  const int ncu = 256, rounds = (int)(lb / (NW * DEPTH * 1024));
  const int lds = DMA ? NW * DEPTH * 1024 : 0;
  CK(hipFuncSetAttribute((const void*)feed<NW, DEPTH, DMA>, hipFuncAttributeMaxDynamicSharedMemorySize,
                         160 * 1024));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((feed<NW, DEPTH, DMA>), dim3(ncu), dim3(NW * 64), lds, 0, src, rounds, sink, piece, stride, win, pair);
  CK(hipEventRecord(a));
  const int reps = 10;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((feed<NW, DEPTH, DMA>), dim3(ncu), dim3(NW * 64), lds, 0, src, rounds, sink, piece, stride, win, pair);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)reps * ncu * rounds * NW * DEPTH * 1024.0;
  printf("%s piece %4d stride %4d win %4zu MiB rounds %3d  %-4s waves %2d  KiB in flight/wave %2d  (/CU %3d)  %7.1f GB/s per CU  %6.2f TB/s total  %.1f us/launch\n",
         pair ? "pair" : "    ", piece, stride, win >> 20, rounds, DMA ? "dma" : "reg", NW, DEPTH, NW * DEPTH, bytes / (ms * 1e-3) / ncu / 1e9, bytes / (ms * 1e-3) / 1e12,
         ms * 1e3 / reps);
}

int main() {
  char* src; unsigned* sink;
  const size_t BIG = 512u << 20;
  CK(hipMalloc(&src, BIG + 4096)); CK(hipMalloc(&sink, 4096));
  CK(hipMemset(src, 1, BIG + 4096));
  run<4, 4, true>(src, sink);   run<4, 8, true>(src, sink);   run<4, 16, true>(src, sink);
  run<8, 4, true>(src, sink);   run<8, 8, true>(src, sink);   run<8, 16, true>(src, sink);
  run<16, 4, true>(src, sink);  run<16, 8, true>(src, sink);
  run<4, 4, false>(src, sink);  run<4, 8, false>(src, sink);  run<4, 16, false>(src, sink);
  run<8, 4, false>(src, sink);  run<8, 8, false>(src, sink);  run<8, 16, false>(src, sink);
  run<16, 4, false>(src, sink); run<16, 8, false>(src, sink);
  // the wide conv tiles' patterns: 64 B of every 256 / 512 B (a 32-channel chunk of a
  // 128- / 256-channel NHWC pixel), L2-resident and from HBM
  for (int st : {256, 512}) {
    run<8, 8, true>(src, sink, 64, st);  run<8, 8, false>(src, sink, 64, st);
    run<4, 16, true>(src, sink, 64, st);
  }
  // MALL-resident (32 MiB, past the 4 MiB L2 of an XCD, inside the 256 MiB MALL): what the
  // 32^2-256^2 activations (4-34 MB at B = 4) are when the next conv reads them
  const size_t MID = 32u << 20;
  run<8, 8, true>(src, sink, 1024, 1024, MID);  run<8, 8, false>(src, sink, 1024, 1024, MID);
  run<8, 8, true>(src, sink, 64, 256, MID);     run<8, 8, false>(src, sink, 64, 256, MID);
  run<8, 16, true>(src, sink, 64, 256, MID);    run<8, 16, true>(src, sink, 1024, 1024, MID);
  // pair: each 64-B piece's line-mate (the next chunk's 32 channels) read in the next
  // round, as consecutive channel chunks of one conv tile do
  run<8, 8, true>(src, sink, 64, 256, MID, 1);  run<8, 8, true>(src, sink, 64, 128, MID, 1);
  run<8, 8, true>(src, sink, 64, 256, WIN, 1);
  run<8, 8, true>(src, sink, 1024, 1024, BIG);  run<8, 8, false>(src, sink, 1024, 1024, BIG);
  run<8, 8, true>(src, sink, 64, 256, BIG);     run<8, 8, false>(src, sink, 64, 256, BIG);
  run<8, 16, true>(src, sink, 64, 256, BIG);
  CK(hipDeviceSynchronize());
  return 0;
}
