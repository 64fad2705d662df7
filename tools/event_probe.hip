// What a cross-stream dependency costs the producing stream (DESIGN.md "Streams"): N short
// kernels on a main stream, each followed by a dependency the side stream waits on, in four
// forms:
//   plain   no dependency (the floor)
//   record  hipEventRecord after each kernel (the engine's form today: a marker packet)
//   bound   the event bound to the kernel itself (hipExtLaunchKernel's stopEvent)
//   (record / bound) x (side waits + runs a small kernel per event, or not)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/event_probe tools/event_probe.hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

// ~10 us of streaming over a 16 MiB buffer with 512 workgroups (vector loads / stores only)
__global__ void work(const float4* __restrict__ x, float4* __restrict__ y, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    float4 v = x[i];
    v.x = v.x * 1.0001f + 1.f;
    y[i] = v;
  }
}
__global__ void tiny(float* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.f;
}

int main() {
  const int N = 200, n = (16 << 20) / 16;
  float4 *x, *y;
  float* t;
  CK(hipMalloc(&x, (size_t)n * 16));
  CK(hipMalloc(&y, (size_t)n * 16));
  CK(hipMalloc(&t, 4096));
  CK(hipMemset(x, 0, (size_t)n * 16));
  hipStream_t main_s, side;
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  CK(hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&side, hipStreamNonBlocking, least));
  std::vector<hipEvent_t> ev(N);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const dim3 g(512), b(256);
  std::vector<hipEvent_t> evd(N);
  for (auto& e : evd) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  uint32_t* flag;
  CK(hipMalloc(&flag, 4));
  CK(hipMemset(flag, 0, 4));
  const char* names[] = {"plain", "record", "record+side", "bound", "bound+side",
                         "record+wait", "bound+wait", "recdflt+side", "value+side", "side-lag4", "side-nowait"};
  const int NM = 11;
  uint32_t tick = 0;
  for (int rep = 0; rep < 3; ++rep) {
    for (int mode = 0; mode < NM; ++mode) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, main_s));
      for (int i = 0; i < N; ++i) {
        const bool bound = mode == 3 || mode == 4 || mode == 6;
        if (bound) {
          void* args[] = {&x, &y, (void*)&n};
          CK(hipExtLaunchKernel((const void*)work, g, b, args, 0, main_s, nullptr, ev[i], 0));
        } else {
          hipLaunchKernelGGL(work, g, b, 0, main_s, x, y, n);
          if (mode == 1 || mode == 2 || mode == 5) CK(hipEventRecord(ev[i], main_s));
          if (mode == 7) CK(hipEventRecord(evd[i], main_s));
          if (mode == 9 && i % 4 == 3) CK(hipEventRecord(ev[i], main_s));
        }
        if (mode == 8) {
          ++tick;
          CK(hipStreamWriteValue32(main_s, flag, tick, 0));
          CK(hipStreamWaitValue32(side, flag, tick, hipStreamWaitValueGte, 0xffffffffu));
        }
        if (mode == 2 || mode == 4 || mode == 5 || mode == 6) CK(hipStreamWaitEvent(side, ev[i], 0));
        if (mode == 7) CK(hipStreamWaitEvent(side, evd[i], 0));
        if (mode == 9 && i % 4 == 3) CK(hipStreamWaitEvent(side, ev[i], 0));
        if (mode == 2 || mode == 4 || mode == 7 || mode == 8 || mode == 9 || mode == 10)
          hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, side, t);
      }
      CK(hipEventRecord(t1, main_s));
      CK(hipDeviceSynchronize());
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, t0, t1));
      printf("rep %d %-14s %8.2f us per kernel\n", rep, names[mode], 1000.f * ms / N);
    }
  }
  return 0;
}
