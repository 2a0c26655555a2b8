// Short-k streaming fp32-accurate GEMM ("x3s", round 3): C[M][N] = A[M][64] . W[N][64]^T with the x3
// arithmetic of gemm_x3.hip (each fp32 operand split exactly into three bf16 terms, the six cross
// products above 2^-23 |a||b| accumulated in fp32 on v_mfma_f32_16x16x32_bf16). Replaces the K = 64
// Conv2d calls of torchvision's ResNet-101 layer1 (models/encoder.py:88-91: layer1.0 conv1 and
// downsample on the max-pooled stem, every layer1 conv3 on relu(bn2(y2))), which the 256-row tiled
// kernels ran at 0.28 of HBM: their output (N = 256: 4x the input bytes) is what
// bounds them, and a tile's k-loop is only two k-tiles, so a one-workgroup-per-CU kernel spends most
// of its time in the serial load -> MFMA -> store phases of one tile.
//
// Structure: 256 threads (4 waves), two persistent workgroups per CU. The whole weight (N x 64, three
// planes) sits in VGPRs for the run: wave w owns output columns [16 NCB w, 16 NCB (w + 1)) and holds
// their 6 NCB MFMA B fragments (N = 256: 96 VGPRs). The workgroup streams 64-row tiles (one BN
// statistics slice each): while tile t's MFMAs, stores and statistics run, the fp32 rows of tile
// t + grid are already in flight into registers; they are then BN-applied (optional prologue), split
// into three bf16 planes and written to the other half of a 2 x 24 KiB LDS double buffer; one
// barrier per tile. Epilogue: the store-only form (plain_epilogue: C = A.B, 32-bit row offsets per
// tile, the column block as an immediate), per-column (sum, sum of squares) of the 64 rows reduced
// across the wave's four row quads and written once per tile: no atomics, deterministic.
#include "gemm_args.h"

namespace {

constexpr int SBM = 64;   // rows per tile (= one 64-row BN statistics slice)
constexpr int SKD = 64;   // k (fixed)
constexpr int SNT = 256;  // threads
typedef __bf16 bf16x8_s __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_s __attribute__((ext_vector_type(4)));
typedef float f32x4_s __attribute__((ext_vector_type(4)));
constexpr unsigned kOOBs = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_s(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// bf16 offset of 8-element chunk c (0..7) of LDS row r (128-B rows): chunk slot c ^ ((r >> 1) & 7), so
// the 16-lane groups of the fragment reads (rows r0..r0+15, one chunk) hit 16 distinct 16-B slots mod
// 256 B (all 64 banks), and the split stores (two whole rows per 32 lanes) are conflict-free
__device__ __forceinline__ int soff(int r, int c) { return r * SKD + ((c ^ ((r >> 1) & 7)) << 3); }

__device__ __forceinline__ bf16x4_s cvt4s(float4 v) {
  bf16x4_s r;
  r.x = (__bf16)v.x;
  r.y = (__bf16)v.y;
  r.z = (__bf16)v.z;
  r.w = (__bf16)v.w;
  return r;
}

template <int NCB, bool PRO>
__global__ void __launch_bounds__(SNT) __attribute__((amdgpu_waves_per_eu(2)))
gemm_x3s_kernel(const capmi_gemm_problem P, long long lda, int tiles) {
  __shared__ __attribute__((aligned(16))) __bf16 As[2][3][SBM * SKD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int rl = lane & 15, c4 = lane >> 4;
  const int M = P.M, N = P.N;
  const int wc0 = wid * 16 * NCB;

  // the wave's weight fragments for the whole run: column 16 cb + rl of its block, k 32 kc + 8 c4 .. + 7
  bf16x8_s bw[NCB][2][3];
  {
    const long long plane = (long long)N * P.ldb;
    const auto rb = rsrc_s(P.B, (unsigned)(3 * plane * 2));
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb)
#pragma unroll
      for (int kc = 0; kc < 2; ++kc)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const unsigned off = (unsigned)((p * plane + (long long)(wc0 + 16 * cb + rl) * P.ldb + 32 * kc + 8 * c4) * 2);
          bw[cb][kc][p] = __builtin_bit_cast(bf16x8_s, __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0));
        }
  }
  // A slots: float4 s of this thread = row (tid >> 4) + 16 s, k 4 (tid & 15) .. + 3
  const int ak = (tid & 15) * 4, ar = tid >> 4;
  float4 sc = f4(1.f), sh = f4(0.f);
  if (PRO) {
    sc = *reinterpret_cast<const float4*>(P.in_scale + ak);
    sh = *reinterpret_cast<const float4*>(P.in_shift + ak);
  }
  const auto ra = rsrc_s(P.A, (unsigned)((long long)M * lda * 4));
  float4 areg[4];
  unsigned amsk = 0;
  auto load_a = [&](int t) {
    amsk = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int row = t * SBM + ar + 16 * s;
      const bool ok = t < tiles && row < M;
      areg[s] = __builtin_bit_cast(
          float4, __builtin_amdgcn_raw_buffer_load_b128(ra, ok ? (unsigned)(row * lda + ak) * 4u : kOOBs, 0, 0));
      amsk |= (unsigned)ok << s;
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float4 v = areg[s];
      if (PRO) v = relu4(fma4(v, sc, sh));
      if (!((amsk >> s) & 1u)) v = f4(0.f);  // rows past M: zeros (their outputs add nothing to the sums)
      const bf16x4_s h0 = cvt4s(v);
      const float4 r1 = make_float4(v.x - (float)h0.x, v.y - (float)h0.y, v.z - (float)h0.z, v.w - (float)h0.w);
      const bf16x4_s h1 = cvt4s(r1);
      const bf16x4_s h2 = cvt4s(make_float4(r1.x - (float)h1.x, r1.y - (float)h1.y, r1.z - (float)h1.z,
                                            r1.w - (float)h1.w));
      const int o = soff(ar + 16 * s, ak >> 3) + (ak & 4);
      *reinterpret_cast<bf16x4_s*>(&As[buf][0][o]) = h0;
      *reinterpret_cast<bf16x4_s*>(&As[buf][1][o]) = h1;
      *reinterpret_cast<bf16x4_s*>(&As[buf][2][o]) = h2;
    }
  };

  int t = blockIdx.x;  // (the host launches at most `tiles` workgroups)
  load_a(t);
  store_a(0);
  __syncthreads();
  const auto rc = rsrc_s(P.C, (unsigned)((long long)M * P.ldc * 4));
  const unsigned cbo = (unsigned)(wc0 + rl) * 4u;
  float* __restrict__ stats = P.stats;
  int buf = 0;
  for (; t < tiles; t += gridDim.x) {
    load_a(t + gridDim.x);  // past the last tile: zeros, never stored
    __builtin_amdgcn_sched_barrier(0);
    f32x4_s acc[4][NCB];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      bf16x8_s a[2][3];
#pragma unroll
      for (int kc = 0; kc < 2; ++kc)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          a[kc][p] = *reinterpret_cast<const bf16x8_s*>(&As[buf][p][soff(16 * rb + rl, 4 * kc + c4)]);
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        f32x4_s c = f32x4_s{0.f, 0.f, 0.f, 0.f};
        // smallest terms first into the fp32 accumulator, k-block by k-block
#pragma unroll
        for (int kc = 0; kc < 2; ++kc) {
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kc][1], bw[cb][kc][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kc][0], bw[cb][kc][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kc][2], bw[cb][kc][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kc][0], bw[cb][kc][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kc][1], bw[cb][kc][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kc][0], bw[cb][kc][0], c, 0, 0, 0);
        }
        acc[rb][cb] = c;
      }
    }
    // epilogue: lane holds rows 16 rb + 4 c4 + r of column 16 cb + rl of the wave's block
    unsigned roff[4][4];
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = t * SBM + 16 * rb + 4 * c4 + r;
        roff[rb][r] = row < M ? (unsigned)row * (unsigned)P.ldc * 4u : kOOBs;
      }
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[rb][cb][r];
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, roff[rb][r] + cbo + 64u * cb, 0, 0);
          s += v;
          q = fmaf(v, v, q);
        }
      if (stats != nullptr) {
        s += __shfl_xor(s, 16, 64);
        q += __shfl_xor(q, 16, 64);
        s += __shfl_xor(s, 32, 64);
        q += __shfl_xor(q, 32, 64);
        if (c4 == 0) {
          const long long o = ((long long)t * N + wc0 + 16 * cb + rl) * 2;
          *reinterpret_cast<float2*>(stats + o) = make_float2(s, q);
        }
      }
    }
    store_a(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
}

}  // namespace

int gemm_x3s_launch(const capmi_gemm_problem& p, long long lda, int tiles, int grid, hipStream_t s) {
  CAPMI_REQUIRE(grid >= 1 && grid <= tiles, CAPMI_EINVAL);
  const bool pro = p.in_scale != nullptr;
  const dim3 g(grid), b(SNT);
#define X3S_GO(NCB)                                                                    \
  do {                                                                                 \
    if (pro)                                                                           \
      CAPMI_KLAUNCH((gemm_x3s_kernel<NCB, true>), g, b, 0, s, p, lda, tiles);  \
    else                                                                      \
      CAPMI_KLAUNCH((gemm_x3s_kernel<NCB, false>), g, b, 0, s, p, lda, tiles); \
  } while (0)
  if (p.N == 64)
    X3S_GO(1);
  else if (p.N == 128)
    X3S_GO(2);
  else if (p.N == 256)
    X3S_GO(4);
  else
    return CAPMI_EINVAL;
#undef X3S_GO
  CAPMI_LAUNCH_CHECK();
  return 0;
}
