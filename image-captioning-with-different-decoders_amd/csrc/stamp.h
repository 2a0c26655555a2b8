// Diagnostic builds only (-DX3_STAMP=1, tools/stamps.py): per-workgroup phase timestamps of the x3 GEMM
// kernels. Lane 0 of each workgroup appends (event, s_memtime) records to a buffer of its own (a __device__
// array no other code reads; vector stores); the host copies it out with capmi_x3_stamps_read. In the real
// kernels (X3_STAMP unset) every macro below is empty.
#pragma once

// event codes (low 8 bits of the record's top 16; the next 8 bits carry a small argument)
enum : unsigned {
  kStStart = 1,     // kernel entry (s_memtime)
  kStRStart = 2,    // kernel entry (s_memrealtime, 100 MHz)
  kStSeg = 3,       // a tile segment starts; arg = k-tiles in it
  kStMain = 4,      // its main loop ended
  kStPub = 5,       // k-prefix partial published (stream-K producer)
  kStCons = 6,      // all partials consumed (stream-K owner)
  kStEpi = 7,       // epilogue ended
  kStEnd = 8,       // kernel exit (s_memtime)
  kStREnd = 9,      // kernel exit (s_memrealtime)
};

#if X3_STAMP
constexpr int kStampSlots = 64;
constexpr int kStampBlocks = 4096;
#define STAMP_BUFFER(name)                                                                          \
  __device__ unsigned long long name[kStampBlocks * kStampSlots];                                   \
  extern "C" int name##_read(void* dst, long long n) {                                              \
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(name), (size_t)n * 8, 0, hipMemcpyDeviceToHost); \
  }                                                                                                 \
  extern "C" int name##_clear(void) {                                                               \
    void* p = nullptr;                                                                              \
    hipError_t e = hipGetSymbolAddress(&p, HIP_SYMBOL(name));                                       \
    if (e != hipSuccess) return (int)e;                                                             \
    return (int)hipMemset(p, 0, sizeof(name));                                                      \
  }
#define STAMP_DECL int stamp_n__ = 0
#define STAMP_RAW(buf, ev, arg, t)                                                                    \
  do {                                                                                                \
    if (threadIdx.x == 0 && blockIdx.x < kStampBlocks && stamp_n__ < kStampSlots)                     \
      buf[blockIdx.x * kStampSlots + stamp_n__++] =                                                   \
          ((unsigned long long)((ev) | ((unsigned)(arg) << 8)) << 48) | ((unsigned long long)(t) & 0xffffffffffffull); \
  } while (0)
#define STAMP(buf, ev, arg) STAMP_RAW(buf, ev, arg, __builtin_amdgcn_s_memtime())
#define STAMP_REAL(buf, ev) STAMP_RAW(buf, ev, 0, __builtin_amdgcn_s_memrealtime())
#else
#define STAMP_BUFFER(name)
#define STAMP_DECL (void)0
#define STAMP(buf, ev, arg) (void)0
#define STAMP_REAL(buf, ev) (void)0
#endif
