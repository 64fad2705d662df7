// Shared device helpers for the PGGAN gfx950 kernels.
//
// Storage dtypes: DT_F32 (parity mode) and DT_BF16 (perf mode, fp32 accumulate).
// Activations are NHWC with a channel stride (`cs`) that may exceed the logical
// channel count (the mbstd output is padded 513 -> 544 so the following conv
// sees a multiple of 32 input channels).  Images are NCHW fp32 (the reference's
// tensor layout at the API boundary).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

#include "../../include/pggan_hip.h"

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;

#define PG_WAVE 64

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }

// round-to-nearest-even; NaN stays NaN (v_cvt_pk_bf16_f32, one instruction per pair)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  bf16x2_t v;
  v[0] = (__bf16)a;
  v[1] = (__bf16)b;
  return __builtin_bit_cast(uint32_t, v);
}
// lrelu'-mask of 8 bf16 (one 16-B vector) by one sign-bit byte: element j keeps its value
// when bit j is set, else becomes round(x * slope) -- branch-free: the factor (1.0 or slope)
// is one bitfield insert from the bit sign-extended (x * 1.0 == x, so the kept elements
// round-trip exactly and the result equals the per-element branch)
__device__ __forceinline__ u32x4_t lrelu_mask_bf16x8(u32x4_t v, unsigned m, float slope) {
  const unsigned one = __float_as_uint(1.0f), sl = __float_as_uint(slope);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned ka = (unsigned)(((int)(m << (31 - 2 * i))) >> 31);       // bit 2i -> 0 / ~0
    const unsigned kc = (unsigned)(((int)(m << (30 - 2 * i))) >> 31);       // bit 2i+1
    const float fa = __uint_as_float((ka & one) | (~ka & sl));
    const float fc = __uint_as_float((kc & one) | (~kc & sl));
    v[i] = pack_bf16x2(__uint_as_float(v[i] << 16) * fa, __uint_as_float(v[i] & 0xffff0000u) * fc);
  }
  return v;
}
// The same mask with the factors from a 16-entry LDS table (entry e: 4 floats, (e >> j) & 1 ?
// 1.0 : slope): two 16-B reads per byte instead of a compare + select per element (the staging
// of the sign-bit input-gradient tiles is VALU-bound).  Bitwise the same result.
__device__ __forceinline__ u32x4_t lrelu_mask_bf16x8_lut(u32x4_t v, unsigned m, const char* lut) {
  typedef __attribute__((ext_vector_type(4))) float f4_t;
  const f4_t f0 = *reinterpret_cast<const f4_t*>(lut + ((m & 15u) << 4));
  const f4_t f1 = *reinterpret_cast<const f4_t*>(lut + (((m >> 4) & 15u) << 4));
  v[0] = pack_bf16x2(__uint_as_float(v[0] << 16) * f0[0], __uint_as_float(v[0] & 0xffff0000u) * f0[1]);
  v[1] = pack_bf16x2(__uint_as_float(v[1] << 16) * f0[2], __uint_as_float(v[1] & 0xffff0000u) * f0[3]);
  v[2] = pack_bf16x2(__uint_as_float(v[2] << 16) * f1[0], __uint_as_float(v[2] & 0xffff0000u) * f1[1]);
  v[3] = pack_bf16x2(__uint_as_float(v[3] << 16) * f1[2], __uint_as_float(v[3] & 0xffff0000u) * f1[3]);
  return v;
}
__device__ __forceinline__ bf16_t f2bf(float f) {
  const __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}

template <typename T> struct Ty;
template <> struct Ty<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
  // 4 consecutive elements
  static __device__ __forceinline__ void ld4(const float* p, float v[4]) {
    f32x4_t q = *reinterpret_cast<const f32x4_t*>(p);
    v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
  }
  static __device__ __forceinline__ void st4(float* p, const float v[4]) {
    f32x4_t q = {v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4_t*>(p) = q;
  }
};
template <> struct Ty<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
  static __device__ __forceinline__ void ld4(const bf16_t* p, float v[4]) {
    u32x2_t q = *reinterpret_cast<const u32x2_t*>(p);
    v[0] = __uint_as_float(q[0] << 16); v[1] = __uint_as_float(q[0] & 0xffff0000u);
    v[2] = __uint_as_float(q[1] << 16); v[3] = __uint_as_float(q[1] & 0xffff0000u);
  }
  static __device__ __forceinline__ void st4(bf16_t* p, const float v[4]) {
    u32x2_t q;
    q[0] = pack_bf16x2(v[0], v[1]);
    q[1] = pack_bf16x2(v[2], v[3]);
    *reinterpret_cast<u32x2_t*>(p) = q;
  }
};

// Image operand of the fromRGB kernels (NCHW fp32 [B][3][Ri][Ri]): x0, or per sample b the
// mix a[b] * x0 + c[b] * x1 (x1 / c may be NULL: a scaled image).  The gradient-penalty
// passes read the interpolated image eps x_real + (1 - eps) x_fake and the scaled input
// gradient through it instead of materialising them (pg_img_src in the C ABI).
struct ImgSrc {
  const float* x0;
  const float* x1;
  const float* a;
  const float* c;
  __host__ __device__ ImgSrc(const float* p = nullptr) : x0(p), x1(nullptr), a(nullptr), c(nullptr) {}
  __host__ ImgSrc(const pg_img_src& s) : x0(s.x0), x1(s.x1), a(s.a), c(s.c) {}
  __host__ __device__ explicit operator bool() const { return x0 != nullptr; }
  // separate roundings (no contraction): a * x0 + c * x1 as the reference's fp32 tensor ops
  __device__ __forceinline__ float mix(int b, float v0, float v1) const {
    float v = __fmul_rn(a[b], v0);
    if (x1) v = __fadd_rn(v, __fmul_rn(c[b], v1));
    return v;
  }
  __device__ __forceinline__ float at(int b, size_t i) const {
    if (!a) return x0[i];
    return mix(b, x0[i], x1 ? x1[i] : 0.f);
  }
  __device__ __forceinline__ float2 at2(int b, size_t i) const {
    const float2 u = *reinterpret_cast<const float2*>(x0 + i);
    if (!a) return u;
    const float2 t = x1 ? *reinterpret_cast<const float2*>(x1 + i) : make_float2(0.f, 0.f);
    return make_float2(mix(b, u.x, t.x), mix(b, u.y, t.y));
  }
};

__device__ __forceinline__ float lrelu_f(float v, float slope) { return v > 0.f ? v : v * slope; }
__device__ __forceinline__ float lmask_f(float y, float slope) { return y > 0.f ? 1.f : slope; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum; `red` must hold >= blockDim.x/64 floats; result valid in all threads
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// ---- deterministic cross-workgroup sums ------------------------------------
// The reductions whose result sums over workgroups (the 1x1 RGB weight gradients, the
// per-sample squared norms of the penalties, the bias gradient) used fp32 atomics: the order of
// the adds followed the order the workgroups finished, so two runs of the same step differed in
// the last bits (and a bf16 rounding downstream could amplify that, tools/repro_probe.py).
// Instead every workgroup stores its totals into the caller's scratch (pg_scratch_bytes, one per
// stream, zero-filled once) and the last workgroup to arrive sums them in workgroup order with a
// fixed split over its threads: the result depends only on the launch geometry.
// Hand-off (MI355X guide, Guideline 16 R1): the partials are stored write-through (sc1, relaxed
// agent-scope atomic stores) -> every wave's vmcnt(0) -> barrier -> one lane's relaxed agent
// ticket; the drawer of the last ticket acquires (agent) and reads the partials with sc1 loads,
// then returns the ticket to 0.  No release fence: an agent-scope release writes back the
// whole XCD L2's dirty lines (buffer_wbl2), once per workgroup -- with the main stream's convs
// writing beside these side-stream kernels that cost the 1x1 RGB weight gradient 84-175 us
// per launch (kernel trace, profiles/r5_v2_*).
// The write-through hand-off is validated on gfx950 (and holds on gfx942, same cache
// protocol); any other target gets the agent-scope release fence the memory model asks for.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#define PG_DET_RELEASE() __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent")
#else
#define PG_DET_RELEASE() ((void)0)
#endif
constexpr int PG_SCRATCH_HDR_FLOATS = 16;   // ticket word + padding (64 B)
__host__ __device__ constexpr size_t pg_scratch_floats() {
  return (PG_SCRATCH_BYTES / sizeof(float)) - PG_SCRATCH_HDR_FLOATS;
}
__host__ __device__ inline float* pg_scratch_partials(float* scratch) {
  return scratch + PG_SCRATCH_HDR_FLOATS;
}

// Every thread of every workgroup calls this last, uniformly.  tot: LDS, the workgroup's NA
// totals (visible to all threads: a __syncthreads() after writing them); tmp: LDS scratch of
// >= max(NA, 4 * blockDim.x) floats, may alias tot.  fin(q, total) runs once per q < NA in the
// last workgroup (the sum over workgroups 0..nb-1 in order, as groups of consecutive workgroups
// summed in group order).  nb * NA <= pg_scratch_floats() (checked by the host).
template <typename Fin>
__device__ __forceinline__ void det_commit(const float* tot, int NA, float* scratch, float* tmp,
                                           Fin fin) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const unsigned nb = gridDim.x * gridDim.y * gridDim.z;
  const unsigned bid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  unsigned* ticket = reinterpret_cast<unsigned*>(scratch);
  float* part = pg_scratch_partials(scratch);
  for (int q = tid; q < NA; q += nt)
    __hip_atomic_store(part + (size_t)bid * NA + q, tot[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PG_DET_RELEASE();
  __syncthreads();
  __shared__ unsigned det_last;
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    det_last = (t == nb - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (!det_last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // G groups of consecutive workgroups per output; items (q, g) spread over the threads
  int G = (4 * nt) / (NA > 0 ? NA : 1);
  G = G < 1 ? 1 : G > 64 ? 64 : G;
  if ((unsigned)G > nb) G = (int)nb;
  const unsigned per = (nb + G - 1) / G;
  for (int it = tid; it < NA * G; it += nt) {
    const int q = it % NA, g = it / NA;
    const unsigned b0 = g * per, b1 = b0 + per < nb ? b0 + per : nb;
    float s = 0.f;
    unsigned b = b0;
    for (; b + 8 <= b1; b += 8) {   // 8 loads in flight, summed in workgroup order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = __hip_atomic_load(part + (size_t)(b + u) * NA + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; b < b1; ++b)
      s += __hip_atomic_load(part + (size_t)b * NA + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tmp[it] = s;
  }
  __syncthreads();
  for (int q = tid; q < NA; q += nt) {
    float s = 0.f;
    for (int g = 0; g < G; ++g) s += tmp[g * NA + q];
    fin(q, s);
  }
  if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Segmented form: each workgroup contributes ONE value `v` (valid in thread 0) to output
// q = bid / (nb / nseg) (the workgroups of one output are a contiguous index range, e.g. the
// blocks of one sample); fin(q, total) for q < nseg in the last workgroup.  tmp: LDS of
// >= 4 * blockDim.x floats.  nb <= pg_scratch_floats(), nb % nseg == 0.
template <typename Fin>
__device__ __forceinline__ void det_commit_seg(float v, int nseg, float* scratch, float* tmp,
                                               Fin fin) {
  const int tid = threadIdx.x, nt = blockDim.x;
  const unsigned nb = gridDim.x * gridDim.y * gridDim.z;
  const unsigned bid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  unsigned* ticket = reinterpret_cast<unsigned*>(scratch);
  float* part = pg_scratch_partials(scratch);
  if (tid == 0) __hip_atomic_store(part + bid, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  PG_DET_RELEASE();
  __syncthreads();
  __shared__ unsigned det_last;
  if (tid == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    det_last = (t == nb - 1) ? 1u : 0u;
  }
  __syncthreads();
  if (!det_last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const unsigned seg = nb / nseg;
  int G = (4 * nt) / nseg;
  G = G < 1 ? 1 : G > 64 ? 64 : G;
  if ((unsigned)G > seg) G = (int)seg;
  const unsigned per = (seg + G - 1) / G;
  for (int it = tid; it < nseg * G; it += nt) {
    const int q = it % nseg, g = it / nseg;
    const unsigned j0 = g * per, j1 = j0 + per < seg ? j0 + per : seg;
    float* p = part + (size_t)q * seg;
    float s = 0.f;
    unsigned j = j0;
    for (; j + 8 <= j1; j += 8) {
      float w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = __hip_atomic_load(p + j + u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += w[u];
    }
    for (; j < j1; ++j) s += __hip_atomic_load(p + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tmp[it] = s;
  }
  __syncthreads();
  for (int q = tid; q < nseg; q += nt) {
    float s = 0.f;
    for (int g = 0; g < G; ++g) s += tmp[g * nseg + q];
    fin(q, s);
  }
  if (tid == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// host side: whether a launch of nb workgroups with na partials each fits the scratch
static inline bool pg_det_fits(size_t nb, size_t na) { return nb * na <= pg_scratch_floats(); }

// ---- error plumbing -------------------------------------------------------
void pg_set_error(const char* fmt, ...);

#define PG_CHECK_ARG(cond, ...)             \
  do {                                      \
    if (!(cond)) {                          \
      pg_set_error(__VA_ARGS__);            \
      return PG_ERR_ARG;                    \
    }                                       \
  } while (0)

// ---- launches and the launch recorder ---------------------------------------
// Every kernel launch of the library goes through PG_KLAUNCH -> pg_launch: the arguments are
// converted to the kernel's parameter types once, and the launch is a hipLaunchKernel over
// them.  While the calling host thread records (pg_record_begin .. pg_record_end), the launch
// is also appended to the recording -- function, geometry, stream and the converted argument
// tuple by value -- so pg_replay can issue the same sequence again from C++ on the same streams
// (the host enqueue of a ~380-launch training step without its Python layer, and without
// hipGraph's re-levelling of the two streams onto other hardware queues).
#include <functional>
#include <tuple>
#include <utility>

bool pg_recording();
void pg_record_push(std::function<hipError_t()> op);
extern "C" int pg_fill_zero(void* p, size_t bytes, void* stream);

template <typename... KArgs, size_t... I>
inline hipError_t pg_launch_tuple(void (*k)(KArgs...), dim3 g, dim3 b, unsigned lds, hipStream_t s,
                                  std::tuple<KArgs...>& t, std::index_sequence<I...>) {
  void* argv[sizeof...(KArgs) + 1] = {(void*)&std::get<I>(t)...};
  return hipLaunchKernel((const void*)k, g, b, argv, lds, s);
}

template <typename... KArgs, typename... Args>
inline void pg_launch(void (*k)(KArgs...), dim3 g, dim3 b, unsigned lds, hipStream_t s,
                      Args&&... args) {
  static_assert(sizeof...(KArgs) == sizeof...(Args), "pg_launch: kernel argument count");
  std::tuple<KArgs...> t{static_cast<KArgs>(std::forward<Args>(args))...};
  (void)pg_launch_tuple(k, g, b, lds, s, t, std::index_sequence_for<KArgs...>{});
  if (pg_recording())
    pg_record_push([=]() mutable {
      return pg_launch_tuple(k, g, b, lds, s, t, std::index_sequence_for<KArgs...>{});
    });
}
#define PG_KLAUNCH(K, G, B, L, S, ...) pg_launch((K), dim3(G), dim3(B), (L), (S), __VA_ARGS__)

#define PG_LAUNCH_CHECK()                                                       \
  do {                                                                          \
    hipError_t e_ = hipGetLastError();                                          \
    if (e_ != hipSuccess) {                                                     \
      pg_set_error("%s: HIP launch error: %s", __func__, hipGetErrorString(e_)); \
      return PG_ERR_HIP;                                                        \
    }                                                                           \
  } while (0)

static inline int pg_cdiv(int a, int b) { return (a + b - 1) / b; }

// Opt kernel `fn` (parenthesise template arguments) in to `bytes` of dynamic LDS on the
// current device, once per (call site, device): the attribute is per device, and a failed set
// is reported here with its reason instead of surfacing later as a bare launch error.
#define PG_LDS_ATTR(fn, bytes)                                                               \
  do {                                                                                       \
    static unsigned done_ = 0;                                                               \
    int dev_ = 0;                                                                            \
    (void)hipGetDevice(&dev_);                                                               \
    if (!((done_ >> (dev_ & 31)) & 1u)) {                                                    \
      const hipError_t e_ = hipFuncSetAttribute((const void*)(fn),                           \
                                                hipFuncAttributeMaxDynamicSharedMemorySize,  \
                                                (int)(bytes));                               \
      if (e_ != hipSuccess) {                                                                \
        pg_set_error("%s: %d B of dynamic LDS: %s", __func__, (int)(bytes),                  \
                     hipGetErrorString(e_));                                                 \
        return PG_ERR_HIP;                                                                   \
      }                                                                                      \
      done_ |= 1u << (dev_ & 31);                                                            \
    }                                                                                        \
  } while (0)
