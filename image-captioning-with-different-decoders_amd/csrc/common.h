// Shared device helpers for libcapmi (gfx950 only).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <algorithm>

#include "capmi.h"

#define CAPMI_LAUNCH_CHECK()                         \
  do {                                               \
    hipError_t e__ = hipGetLastError();              \
    if (e__ != hipSuccess) return (int)e__;          \
  } while (0)

#define CAPMI_REQUIRE(cond, code) \
  do {                            \
    if (!(cond)) return (code);   \
  } while (0)

// Kernel timing for bench.py's roofline (capmi_timing_arm, timing.hip): the next GEMM launch on this
// host thread takes these two events and records into them the dispatch's own start / end timestamps
// (hipExtLaunchKernel: the AQL packet's times, the ones rocprofv3 reports as the kernel duration),
// then the pair is disarmed. Unarmed, CAPMI_KLAUNCH is hipLaunchKernelGGL.
struct CapmiArmedEvents {
  hipEvent_t start, stop;
};
extern thread_local CapmiArmedEvents g_capmi_armed;
// the last kernel CAPMI_KLAUNCH launched on this host thread (capmi_last_launch_name: the instantiation a plan
// query names must be the one launched -- tests/test_gpu_plan_names.py)
extern thread_local const void* g_capmi_last_kernel;
#define CAPMI_KLAUNCH(kernel, grid, block, shmem, stream, ...)                                          \
  do {                                                                                                 \
    g_capmi_last_kernel = reinterpret_cast<const void*>(kernel);                                       \
    if (g_capmi_armed.start != nullptr) {                                                              \
      const CapmiArmedEvents ev__ = g_capmi_armed;                                                     \
      g_capmi_armed = CapmiArmedEvents{nullptr, nullptr};                                              \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, ev__.start, ev__.stop, 0, __VA_ARGS__); \
    } else {                                                                                           \
      hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                             \
    }                                                                                                  \
  } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

static inline unsigned cdiv(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide reduction over up to 1024 threads (blockDim multiple of 64); red = LDS[>= 16]
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 operator+(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ __forceinline__ float4 operator*(float4 a, float4 b) {
  return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w);
}
__device__ __forceinline__ float4 fma4(float4 a, float4 b, float4 c) {
  return make_float4(fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y), fmaf(a.z, b.z, c.z),
                     fmaf(a.w, b.w, c.w));
}
__device__ __forceinline__ float4 relu4(float4 a) {
  return make_float4(fmaxf(a.x, 0.f), fmaxf(a.y, 0.f), fmaxf(a.z, 0.f), fmaxf(a.w, 0.f));
}
// init + sum of the S split-K partial slabs p[s * slab], s = 0..S-1, added in slab order (the
// same rounding as a plain loop) but with up to 8 loads in flight instead of one
template <typename T>
__device__ __forceinline__ T slab_sum(const T* __restrict__ p, int S, long long slab, T acc) {
  int s = 0;
  for (; s + 8 <= S; s += 8) {
    T v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = p[(s + u) * slab];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = acc + v[u];
  }
  if (s + 4 <= S) {
    T v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = p[(s + u) * slab];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = acc + v[u];
    s += 4;
  }
  for (; s < S; ++s) acc = acc + p[s * slab];
  return acc;
}

__device__ __forceinline__ float dot4(float4 a, float4 b) {
  return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w;
}
