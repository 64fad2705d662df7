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

template <int NW, int DEPTH, bool DMA>
__global__ __launch_bounds__(NW * 64) void feed(const char* __restrict__ src, int rounds,
                                                unsigned* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned acc = 0;
  size_t off = ((size_t)blockIdx.x * 8192 + (size_t)wid * DEPTH * 1024) % WIN;
  for (int it = 0; it < rounds; ++it) {
    if constexpr (DMA) {
#pragma unroll
      for (int k = 0; k < DEPTH; ++k) {
        const size_t o = (off + (size_t)k * 1024) % WIN;
        __builtin_amdgcn_global_load_lds((const void*)(src + o + lane * 16),
                                         (__attribute__((address_space(3))) void*)(lds + (wid * DEPTH + k) * 1024),
                                         16, 0, 0);
      }
      __syncthreads();
    } else {
      uint4 v[DEPTH];
#pragma unroll
      for (int k = 0; k < DEPTH; ++k) {
        const size_t o = (off + (size_t)k * 1024) % WIN;
        v[k] = *reinterpret_cast<const uint4*>(src + o + lane * 16);
      }
#pragma unroll
      for (int k = 0; k < DEPTH; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    off = (off + (size_t)NW * DEPTH * 1024) % WIN;
  }
  if constexpr (DMA) acc = *reinterpret_cast<const unsigned*>(lds + lane * 16);
  if (acc == 0x12345678u) sink[blockIdx.x] = acc;   // keeps the loads live
}

template <int NW, int DEPTH, bool DMA>
void run(const char* src, unsigned* sink) {
  const int ncu = 256, rounds = 2048 / (NW * DEPTH) > 8 ? 2048 / (NW * DEPTH) : 8;
  const int lds = DMA ? NW * DEPTH * 1024 : 0;
  CK(hipFuncSetAttribute((const void*)feed<NW, DEPTH, DMA>, hipFuncAttributeMaxDynamicSharedMemorySize,
                         160 * 1024));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((feed<NW, DEPTH, DMA>), dim3(ncu), dim3(NW * 64), lds, 0, src, rounds, sink);
  CK(hipEventRecord(a));
  const int reps = 10;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((feed<NW, DEPTH, DMA>), dim3(ncu), dim3(NW * 64), lds, 0, src, rounds, sink);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
  const double bytes = (double)reps * ncu * rounds * NW * DEPTH * 1024.0;
  printf("%-4s waves %2d  KiB in flight/wave %2d  (/CU %3d)  %7.1f GB/s per CU  %6.2f TB/s total  %.1f us/launch\n",
         DMA ? "dma" : "reg", NW, DEPTH, NW * DEPTH, bytes / (ms * 1e-3) / ncu / 1e9, bytes / (ms * 1e-3) / 1e12,
         ms * 1e3 / reps);
}

int main() {
  char* src; unsigned* sink;
  CK(hipMalloc(&src, WIN + 4096)); CK(hipMalloc(&sink, 4096));
  CK(hipMemset(src, 1, WIN + 4096));
  run<4, 4, true>(src, sink);   run<4, 8, true>(src, sink);   run<4, 16, true>(src, sink);
  run<8, 4, true>(src, sink);   run<8, 8, true>(src, sink);   run<8, 16, true>(src, sink);
  run<16, 4, true>(src, sink);  run<16, 8, true>(src, sink);
  run<4, 4, false>(src, sink);  run<4, 8, false>(src, sink);  run<4, 16, false>(src, sink);
  run<8, 4, false>(src, sink);  run<8, 8, false>(src, sink);  run<8, 16, false>(src, sink);
  run<16, 4, false>(src, sink); run<16, 8, false>(src, sink);
  CK(hipDeviceSynchronize());
  return 0;
}
