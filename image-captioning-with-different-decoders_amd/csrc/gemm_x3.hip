// fp32-accurate GEMM / implicit-GEMM convolution on the bf16 matrix cores ("x3"): every fp32
// operand is split EXACTLY into three bf16 terms, a = a0 + a1 + a2 (a0 = RNE(a), a1 = RNE(a - a0),
// a2 = a - a0 - a1; 8 + 8 + 8 significant bits cover the 24 of an fp32), and the product is
//   a.b = a0 b0 + (a0 b1 + a1 b0) + (a0 b2 + a1 b1 + a2 b0) + [a1 b2 + a2 b1 + a2 b2]
// where every bf16 x bf16 product is exact in fp32 and the bracketed terms, dropped, are below
// 2^-23 |a||b| together (|a1| <= 2^-8 |a|, |a2| <= 2^-16 |a|): the fp32 rounding level. The six kept
// products run on v_mfma_f32_32x32x16_bf16 (32 cycles per 32x32x16 on one SIMD, 16x the f32 MFMA
// rate), accumulated in fp32: 6 x 32 = 192 cycles per 32x32x16 against 8 x 64 = 512 for
// v_mfma_f32_32x32x2_f32, so the MFMA bound is 2.67x the fp32 matrix peak (420 TFLOP/s of fp32
// arithmetic). Accuracy equals the fp32 kernel's (tests/test_gpu_x3.py: |C - C64| against the fp64
// product, element-wise, at the fp32 kernel's tolerance). Replaces the Conv2d calls of torchvision's
// ResNet-101 (models/encoder.py:88-91,107) in the fp32 encoder forward.
//
// Operands: A fp32 (dense K-major rows, or the implicit im2col of an NHWC activation with the
// fused BN-apply + ReLU prologue of the previous BatchNorm); the split happens when a k-tile is
// written to LDS. B = the conv weight pre-split once into three bf16 planes [3][N][ldb]
// (capmi_split3_bf16; the weights are frozen, or re-split when they change).
// Tile 128 x BN (BN = 128 or 64), 512 threads = 8 waves as 4 rows x 2 columns (wave 32 x BN/2),
// BK = 32: per k-tile and wave 2 x (3 + 3 TN) ds_read_b128 feed 2 x 6 TN MFMAs. Two register
// stages (loads two k-tiles ahead), LDS double buffer (3 planes per operand, rows of 40 bf16 = 80 B:
// the 16-lane groups of ds_read_b128 hit 64 distinct banks). Epilogue, BN statistics per 64-row
// slice and the stream-K hand-off are those of gemm_nt.hip.
#include "gemm_args.h"
#include "stamp.h"

STAMP_BUFFER(capmi_x3_stamps)

#ifndef X3_VARIANT
#define X3_VARIANT 0
#endif

namespace {

constexpr int XBK = 32;       // fp32 k per k-tile
#ifndef X3_M16
#define X3_M16 1
#endif
#ifndef X3_SWZ
#define X3_SWZ X3_M16
#endif
// LDS row stride (bf16 elements). X3_SWZ (default): 64-B rows with x3p's 16-B chunk swizzle (chunk c
// of row r at c ^ ((r / 4) % 4)): the 8-B split stores of a wave (8 rows x 64 B) and the 16-lane
// ds_read_b128 groups both hit 64 distinct banks. Else 80-B padded rows (the reads conflict-free,
// the split stores 2-3-way conflicted: PMC lds_conflict 29 %, profiles/r02_pmc_sq.txt).
constexpr int XSB = X3_SWZ ? XBK : XBK + 8;
// X3_M16 (round 3, default): the MFMAs are v_mfma_f32_16x16x32_bf16 (one per 32-deep k-tile and
// 16 x 16 block; the chip holds a higher clock under them than under 32x32x16: gemm_x3p.hip), read
// as lane l -> row l % 16, chunk l / 16, conflict-free on the [0, 2, 3, 1][(row >> 2) & 3] chunk
// swizzle of 64-B rows (the split stores stay conflict-free: 16 lanes = two whole rows)
__device__ __forceinline__ int xoff(int row, int chunk) {  // bf16 offset of 8-element chunk `chunk` of `row`
  const int sw = X3_M16 ? ((0x1320 >> (4 * ((row >> 2) & 3))) & 3) : ((row >> 2) & 3);
  return row * XSB + ((X3_SWZ ? (chunk ^ sw) : chunk) << 3);
}
constexpr int XNT = 512;
typedef unsigned u32x4_x __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_x __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_x __attribute__((ext_vector_type(4)));
constexpr unsigned kOOBx = 0x80000000u;  // buffer offset past every operand: the load returns 0
constexpr int kSc1x = 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_x(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ bf16x4_x cvt4(float4 v) {
  bf16x4_x r;
  r.x = (__bf16)v.x;
  r.y = (__bf16)v.y;
  r.z = (__bf16)v.z;
  r.w = (__bf16)v.w;
  return r;
}
__device__ __forceinline__ float4 back4(bf16x4_x h) {
  return make_float4((float)h.x, (float)h.y, (float)h.z, (float)h.w);
}
__device__ __forceinline__ float4 sub4(float4 a, float4 b) {
  return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w);
}

template <int BN, int AMODE, bool PRO, bool SK>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
gemm_x3_kernel(const GemmArgs args) {
  constexpr int BM = 128, WM = 32, WN = BN / 2, TN = WN / 32;
  constexpr int NA = BM * XBK / 4 / XNT;        // fp32 float4 slots of A per thread (2)
  constexpr int NB = 3 * BN * (XBK / 8) / XNT;  // 16-B bf16 chunks of B per thread (3 or 1.5)
  static_assert(NA == 2, "tile");
  constexpr int NBr = (3 * BN * (XBK / 8) + XNT - 1) / XNT;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][3][BM * XSB];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][3][BN * XSB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm0 = (wid >> 1) * WM, wn0 = (wid & 1) * WN;
  STAMP_DECL;
  STAMP(capmi_x3_stamps, kStStart, 0);
  STAMP_REAL(capmi_x3_stamps, kStRStart);
  const int lr = lane & 31, lh = lane >> 5;
  const int kq = (tid & 7) * 4;  // k of this thread's A float4 inside a k-tile
  (void)NB;

  f32x16 acc[TN];
  constexpr int TN16 = WN / 16;      // 16x16x32: 2 x TN16 blocks per wave
  typedef float f32x4_x __attribute__((ext_vector_type(4)));
  f32x4_x acc4[2][TN16];

  auto mainloop = [&](const capmi_gemm_problem& P, int m0, int n0, int k_lo, int k_hi) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < TN16; ++j) acc4[i][j] = f32x4_x{0.f, 0.f, 0.f, 0.f};
    const int nkt = (k_hi - k_lo) / XBK;
    if (nkt <= 0) return;
    const int M = P.M, N = P.N;
    const int cH = P.cH, cW = P.cW, cCin = P.cCin, cKW = P.cKW;
    const unsigned a_bytes = AMODE == 2 ? (unsigned)((long long)P.cN * cH * cW * cCin * 4)
                                        : (unsigned)((long long)M * P.lda * 4);
    const auto ra = rsrc_x(P.A, a_bytes);
    const long long plane = (long long)N * P.ldb;  // bf16 elements per B plane
    const auto rb = rsrc_x(P.B, (unsigned)(3 * plane * 2));
    const float* __restrict__ isc = P.in_scale;
    const float* __restrict__ ish = P.in_shift;
    unsigned a_off[NA];
    int a_ih0[NA], a_iw0[NA];
    bool a_ok[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = m0 + ((tid + i * XNT) >> 3);
      a_ok[i] = row < M;
      if (AMODE == 0) {
        a_off[i] = a_ok[i] ? (unsigned)(((long long)row * P.lda + kq) * 4) : kOOBx;
        a_ih0[i] = a_iw0[i] = 0;
      } else {
        const int hw = P.cHo * P.cWo;
        const int rr = a_ok[i] ? row : 0;
        const int n = rr / hw, rem = rr - n * hw;
        const int oh = rem / P.cWo, ow = rem - oh * P.cWo;
        a_ih0[i] = oh * P.cStride - P.cPad;
        a_iw0[i] = ow * P.cStride - P.cPad;
        a_off[i] = (unsigned)(n * cH * cW);  // pixel index of the image's (0, 0)
      }
    }
    // B chunk c = tid + i * XNT: plane c / (4 BN), row (c / 4) % BN, k 8 (c % 4)
    unsigned b_off[NBr];
    int b_lds[NBr];
#pragma unroll
    for (int i = 0; i < NBr; ++i) {
      const int c = tid + i * XNT;
      const int p = c / (4 * BN), rem = c - p * 4 * BN, r = rem >> 2, kc = (rem & 3) * 8;
      const int n = n0 + r;
      const bool ok = c < 3 * BN * 4 && n < N;
      b_off[i] = ok ? (unsigned)((p * plane + (long long)n * P.ldb + kc) * 2) : kOOBx;
      b_lds[i] = c < 3 * BN * 4 ? (p * BN * XSB + xoff(r, kc >> 3)) : -1;
    }
    int c_ci = 0, c_kh = 0, c_kw = 0;  // conv k walk, advanced XBK per k-tile
    if (AMODE == 2) {
      const int kpos = k_lo / cCin;
      c_ci = k_lo - kpos * cCin;
      c_kh = kpos / cKW;
      c_kw = kpos - c_kh * cKW;
    }

    struct Stage {
      float4 a[NA];
      u32x4_x b[NBr];
      float4 sc, sh;
      unsigned am;
    };
    auto load_tile = [&](Stage& st, int kt) {
      const int k = k_lo + kt * XBK;
      const bool kok = k < k_hi;
      st.am = 0;
      if (AMODE == 0) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const bool ok = a_ok[i] && kok;
          st.a[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                                   ra, ok ? a_off[i] + (unsigned)k * 4 : kOOBx, 0, 0));
          st.am |= (unsigned)ok << i;
        }
      } else {
        const int ci = c_ci + kq;
        if (PRO) {
          st.sc = *reinterpret_cast<const float4*>(isc + ci);
          st.sh = *reinterpret_cast<const float4*>(ish + ci);
        }
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int ih = a_ih0[i] + c_kh, iw = a_iw0[i] + c_kw;
          const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
          const unsigned off = ((a_off[i] + (unsigned)(ih * cW + iw)) * (unsigned)cCin + (unsigned)ci) * 4u;
          st.a[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, ok ? off : kOOBx, 0, 0));
          st.am |= (unsigned)ok << i;
        }
        c_ci += XBK;
        if (c_ci >= cCin) {
          c_ci = 0;
          if (++c_kw == cKW) {
            c_kw = 0;
            ++c_kh;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NBr; ++i)
        st.b[i] = __builtin_amdgcn_raw_buffer_load_b128(rb, kok && b_off[i] != kOOBx ? b_off[i] + (unsigned)k * 2 : kOOBx,
                                                        0, 0);
    };
    auto store_tile = [&](const Stage& st, int buf) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        float4 v = st.a[i];
        if (PRO && AMODE == 2) {
          v = relu4(fma4(v, st.sc, st.sh));
          if (!((st.am >> i) & 1u)) v = f4(0.f);  // padding taps are zeros AFTER the BN apply
        }
        const bf16x4_x h0 = cvt4(v);
#if X3_VARIANT == 1  // A/B only: no split VALU (wrong results)
        const bf16x4_x h1 = h0, h2 = h0;
#else
        const float4 r1 = sub4(v, back4(h0));
        const bf16x4_x h1 = cvt4(r1);
        const bf16x4_x h2 = cvt4(sub4(r1, back4(h1)));
#endif
        const int o = xoff((tid + i * XNT) >> 3, kq >> 3) + (kq & 7);
        *reinterpret_cast<bf16x4_x*>(&As[buf][0][o]) = h0;
        *reinterpret_cast<bf16x4_x*>(&As[buf][1][o]) = h1;
        *reinterpret_cast<bf16x4_x*>(&As[buf][2][o]) = h2;
      }
#pragma unroll
      for (int i = 0; i < NBr; ++i)
        if ((3 * BN * 4) % XNT == 0 || b_lds[i] >= 0) *reinterpret_cast<u32x4_x*>(&Bs[buf][0][b_lds[i]]) = st.b[i];
    };
    auto compute = [&](int buf) {
      if constexpr (X3_M16) {
        const int c = lane >> 4, rl = lane & 15;
        bf16x8_x a[2][3], b[TN16][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int ao = xoff(wm0 + 16 * i + rl, c);
#pragma unroll
          for (int p = 0; p < 3; ++p) a[i][p] = *reinterpret_cast<const bf16x8_x*>(&As[buf][p][ao]);
        }
#pragma unroll
        for (int j = 0; j < TN16; ++j) {
          const int bo = xoff(wn0 + 16 * j + rl, c);
#pragma unroll
          for (int p = 0; p < 3; ++p) b[j][p] = *reinterpret_cast<const bf16x8_x*>(&Bs[buf][p][bo]);
        }
        // smallest terms first into the fp32 accumulator
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < TN16; ++j) {
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][1], acc4[i][j], 0, 0, 0);
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][2], acc4[i][j], 0, 0, 0);
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[j][0], acc4[i][j], 0, 0, 0);
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][1], acc4[i][j], 0, 0, 0);
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][0], acc4[i][j], 0, 0, 0);
            acc4[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][0], acc4[i][j], 0, 0, 0);
          }
        return;
      }
#pragma unroll
      for (int g = 0; g < XBK / 16; ++g) {
        bf16x8_x a[3], b[3][TN];
        const int ao = xoff(wm0 + lr, 2 * g + lh);
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8_x*>(&As[buf][p][ao]);
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            b[p][j] = *reinterpret_cast<const bf16x8_x*>(&Bs[buf][p][xoff(wn0 + 32 * j + lr, 2 * g + lh)]);
        // smallest terms first into the fp32 accumulator
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#if X3_VARIANT == 2  // A/B only: one product per pair (wrong results)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0][j], acc[j], 0, 0, 0);
          continue;
#endif
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1][j], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2][j], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0][j], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1][j], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0][j], acc[j], 0, 0, 0);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0][j], acc[j], 0, 0, 0);
        }
      }
    };
    auto kstep = [&](Stage& ld, const Stage& sv, int kt) {
      load_tile(ld, kt + 2);
      __builtin_amdgcn_sched_barrier(0);
      compute(kt & 1);
      store_tile(sv, (kt + 1) & 1);
      __syncthreads();
    };
    Stage s0, s1;
    s0.sc = s1.sc = f4(1.f);
    s0.sh = s1.sh = f4(0.f);
    load_tile(s0, 0);
    store_tile(s0, 0);
    load_tile(s1, 1);
    __syncthreads();
    // back edge only from the second k-step (gemm_nt.hip: keeps the prefetch two deep)
    int kt = 0;
    for (; kt + 1 < nkt; kt += 2) {
      kstep(s0, s1, kt);
      kstep(s1, s0, kt + 1);
    }
    if (kt < nkt) kstep(s0, s1, kt);
  };

  // epilogue (gemm_nt.hip's): alpha, bias, beta*C, relu, store, BN statistics per 64-row slice
  auto epilogue = [&](const capmi_gemm_problem& P, int tm, int tn) {
    const int M = P.M, N = P.N;
    const int m0 = tm * BM, n0 = tn * BN;
    const float alpha = P.alpha * (P.alpha_ptr ? *P.alpha_ptr : 1.f);
    float* C = P.C;
    const float beta = P.beta;
    const int relu = P.relu;
    const long long ldc = P.ldc, c_r1 = P.c_r1, c_s2 = P.c_s2;
    // per-lane column sums over this wave's 32 rows: TN columns per lane (32x32x16: lane column
    // 32 j + lane % 32) or TN16 (16x16x32: column 16 j + lane % 16); scol(j) is the wave-local column
    constexpr int NCOL = X3_M16 ? TN16 : TN;
    float csum[NCOL], csq[NCOL];
    auto scol = [&](int j) { return X3_M16 ? 16 * j + (lane & 15) : 32 * j + lr; };
    if constexpr (X3_M16) {
      const int rq = lane >> 4;
      if (args.plain_epi) {
        // store-only form (host: plain_epilogue): row offsets once per tile, column block as an
        // immediate offset; rows past M are dropped by the descriptor (their accumulators are 0)
        const auto rc = rsrc_x(C, (unsigned)((long long)M * ldc * 4));
        unsigned roff[2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wm0 + 16 * i + 4 * rq + r;
            roff[i][r] = row < M ? (unsigned)row * (unsigned)ldc * 4u : kOOBx;
          }
        const unsigned cb = (unsigned)(n0 + wn0 + (lane & 15)) * 4u;
        // + beta C: every C value loaded before the first store (interleaved, each load waited for the store
        // before it -- they may alias through the one descriptor -- a serial memory round trip per element)
        float cold[2][TN16][4];
        if (args.plain_epi == 2) {
#pragma unroll
          for (int j = 0; j < TN16; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                cold[i][j][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rc, roff[i][r] + cb + 64u * j, 0, 0));
        }
#pragma unroll
        for (int j = 0; j < TN16; ++j) {
          csum[j] = 0.f;
          csq[j] = 0.f;
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc4[i][j][r];
              if (args.plain_epi == 2) v = fmaf(beta, cold[i][j][r], v);  // (the general epilogue's fmaf, bit for bit)
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, roff[i][r] + cb + 64u * j, 0, 0);
              csum[j] += v;
              csq[j] = fmaf(v, v, csq[j]);
            }
        }
      } else
#pragma unroll
      for (int j = 0; j < TN16; ++j) {
        csum[j] = 0.f;
        csq[j] = 0.f;
        const int col = n0 + wn0 + scol(j);
        const bool cok = col < N;
        float bias = 0.f;
        if (cok) {
          if (P.bias) bias += P.bias[col];
          if (P.bias2) bias += P.bias2[col];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wm0 + 16 * i + 4 * rq + r;
            if (cok && row < M) {
              float* cp = C + remap(row, c_r1, ldc, c_s2) + col;
              float v = fmaf(acc4[i][j][r], alpha, bias);
              if (beta != 0.f) v = fmaf(beta, *cp, v);
              if (relu) v = fmaxf(v, 0.f);
              *cp = v;
              csum[j] += v;
              csq[j] = fmaf(v, v, csq[j]);
            }
          }
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        csum[j] = 0.f;
        csq[j] = 0.f;
        const int col = n0 + wn0 + 32 * j + lr;
        const bool cok = col < N;
        float bias = 0.f;
        if (cok) {
          if (P.bias) bias += P.bias[col];
          if (P.bias2) bias += P.bias2[col];
        }
  #pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (cok && row < M) {
            float* cp = C + remap(row, c_r1, ldc, c_s2) + col;
            float v = fmaf(acc[j][r], alpha, bias);
            if (beta != 0.f) v = fmaf(beta, *cp, v);
            if (relu) v = fmaxf(v, 0.f);
            *cp = v;
            csum[j] += v;
            csq[j] = fmaf(v, v, csq[j]);
          }
        }
      }
    }
    float* __restrict__ stats = P.stats;
    if (stats != nullptr) {
#pragma unroll
      for (int j = 0; j < NCOL; ++j) {
        if (X3_M16) {
          csum[j] += __shfl_xor(csum[j], 16, 64);
          csq[j] += __shfl_xor(csq[j], 16, 64);
        }
        csum[j] += __shfl_xor(csum[j], 32, 64);
        csq[j] += __shfl_xor(csq[j], 32, 64);
      }
      // wave rows 2s and 2s+1 share the tile's 64-row slice s
      float* red = reinterpret_cast<float*>(&As[0][0][0]);  // the k loop ended with a barrier
      if (X3_M16 ? (lane >> 4) == 0 : lh == 0) {
#pragma unroll
        for (int j = 0; j < NCOL; ++j) {
          red[(wid * 2 + 0) * WN + scol(j)] = csum[j];
          red[(wid * 2 + 1) * WN + scol(j)] = csq[j];
        }
      }
      __syncthreads();
      constexpr int NS = BM / 64;
      for (int c = tid; c < NS * BN; c += XNT) {
        const int sl = c / BN, cn = c % BN, wn = cn / WN, cc = cn % WN;
        const int w0 = (2 * sl) * 2 + wn, w1 = (2 * sl + 1) * 2 + wn;
        const float s = red[(w0 * 2 + 0) * WN + cc] + red[(w1 * 2 + 0) * WN + cc];
        const float q = red[(w0 * 2 + 1) * WN + cc] + red[(w1 * 2 + 1) * WN + cc];
        const int col = n0 + cn;
        if (col < N && m0 + 64 * sl < M) {
          const long long slice = (m0 >> 6) + sl;
          stats[(slice * N + col) * 2 + 0] = s;
          stats[(slice * N + col) * 2 + 1] = q;
        }
      }
      __syncthreads();  // LDS reused by the next tile (stream-K)
    }
  };

  if (!SK) {
    int bid = blockIdx.x;
    {  // XCD-aware remap (bijective for any grid size): consecutive tiles on one XCD
      const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = bid & 7;
      bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    }
    const capmi_gemm_problem& P = args.p[0];
    const int tiles_n = args.tiles_n[0];
    const int tn = bid % tiles_n, tm = bid / tiles_n;
    STAMP(capmi_x3_stamps, kStSeg, P.K / XBK);
    mainloop(P, tm * BM, tn * BN, 0, P.K);
    STAMP(capmi_x3_stamps, kStMain, 0);
    epilogue(P, tm, tn);
    STAMP(capmi_x3_stamps, kStEpi, 0);
    STAMP(capmi_x3_stamps, kStEnd, 0);
    STAMP_REAL(capmi_x3_stamps, kStREnd);
    return;
  }

  // stream-K over (tile, k-tile) units with XCD groups and the hybrid schedule: gemm_nt.hip's
  // hand-off protocol (sc1 write-through parking, drained, agent-scope flag; sc1 loads). The sc1 form
  // without fences (gemm_args.h) needs one workgroup per CU: the BN = 64 tile (72 KB of LDS, <= 168
  // VGPRs) fits two per CU, so it keeps the agent-scope release / acquire
  constexpr bool kFencedX = kSkFenced1 || BN == 64;
  const capmi_gemm_problem& P = args.p[0];
  const int nkt = args.sk_nkt, tiles_n = args.tiles_n[0];
  const long long ngrp = args.sk_groups, grp = blockIdx.x % ngrp;
  const long long T = args.sk_units / nkt, G = gridDim.x / ngrp, w = blockIdx.x / ngrp;
  if (args.sk_dp_tiles > 0) {
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = blockIdx.x & 7;
    const int pos = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (blockIdx.x >> 3);
    for (long long t = T + pos; t < T + args.sk_dp_tiles; t += nwg) {
      const int tm = (int)(t / tiles_n), tn = (int)(t % tiles_n);
      mainloop(P, tm * BM, tn * BN, 0, P.K);
      epilogue(P, tm, tn);
    }
  }
  const long long ub = grp * T / ngrp * nkt, U = ((grp + 1) * T / ngrp) * nkt - ub;
  const long long u0 = ub + w * U / G, u1 = ub + (w + 1) * U / G;
  constexpr int PART = BM * BN;
  int* flags = args.sk_flags;
  if (u0 >= u1) return;
  for (long long t = (u1 - 1) / nkt; t >= u0 / nkt; --t) {
    const long long tb = t * nkt;
    const int ks = (int)(max(u0, tb) - tb), ke = (int)(min(u1, tb + nkt) - tb);
    const int tm = (int)(t / tiles_n), tn = (int)(t % tiles_n);
    mainloop(P, tm * BM, tn * BN, ks * XBK, ke * XBK);
    if (ke < nkt) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.sk_part + (long long)blockIdx.x * PART, 0,
                                                        PART * 4, 0x00020000);
      if constexpr (X3_M16) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < TN16; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_x, acc4[i][j]), rs,
                                                   ((i * TN16 + j) * XNT + tid) * 16, 0, kSc1x);
      } else {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          u32x4_x v;
          v.x = __float_as_uint(acc[j][4 * q + 0]);
          v.y = __float_as_uint(acc[j][4 * q + 1]);
          v.z = __float_as_uint(acc[j][4 * q + 2]);
          v.w = __float_as_uint(acc[j][4 * q + 3]);
          __builtin_amdgcn_raw_buffer_store_b128(v, rs, ((j * 4 + q) * XNT + tid) * 16, 0, kSc1x);
        }
      }
      sk_publish<kFencedX>(flags + blockIdx.x, tid);
      continue;
    }
    if (ks > 0) {
      for (long long w2 = w - 1;; --w2) {
        const long long b2 = w2 * ngrp + grp;
        sk_consume<kFencedX>(flags + b2, flags + gridDim.x, tid);
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.sk_part + b2 * PART, 0, PART * 4, 0x00020000);
        if constexpr (X3_M16) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < TN16; ++j)
              acc4[i][j] += __builtin_bit_cast(
                  f32x4_x, __builtin_amdgcn_raw_buffer_load_b128(rs, ((i * TN16 + j) * XNT + tid) * 16, 0, kSc1x));
        } else {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const u32x4_x v = __builtin_amdgcn_raw_buffer_load_b128(rs, ((j * 4 + q) * XNT + tid) * 16, 0, kSc1x);
            acc[j][4 * q + 0] += __uint_as_float(v.x);
            acc[j][4 * q + 1] += __uint_as_float(v.y);
            acc[j][4 * q + 2] += __uint_as_float(v.z);
            acc[j][4 * q + 3] += __uint_as_float(v.w);
          }
        }
        if (ub + w2 * U / G <= tb) break;
      }
    }
    epilogue(P, tm, tn);
  }
}

template <int BN, bool SK>
void launch_x3(const GemmArgs& a, int amode, bool pro, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(XNT);
  if (amode == 2) {
    if (pro)
      CAPMI_KLAUNCH((gemm_x3_kernel<BN, 2, true, SK>), g, b, 0, s, a);
    else
      CAPMI_KLAUNCH((gemm_x3_kernel<BN, 2, false, SK>), g, b, 0, s, a);
  } else {  // dense A: no prologue (x3_plan)
    CAPMI_KLAUNCH((gemm_x3_kernel<BN, 0, false, SK>), g, b, 0, s, a);
  }
}

// in[n] fp32 -> out[3][n] bf16: the exact three-term split (RNE at each step)
__global__ void split3_bf16_kernel(const float4* __restrict__ in, long long n4, bf16x4_x* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const float4 v = in[i];
    const bf16x4_x h0 = cvt4(v);
    const float4 r1 = sub4(v, back4(h0));
    const bf16x4_x h1 = cvt4(r1);
    const bf16x4_x h2 = cvt4(sub4(r1, back4(h1)));
    out[i] = h0;
    out[n4 + i] = h1;
    out[2 * n4 + i] = h2;
  }
}

}  // namespace

int gemm_x3_launch(const GemmArgs& a, int amode, int bn, int blocks, hipStream_t s) {
  const bool pro = a.p[0].in_scale != nullptr;
  const bool sk = a.sk_workers > 0;
  if (bn == 128) {
    if (sk)
      launch_x3<128, true>(a, amode, pro, blocks, s);
    else
      launch_x3<128, false>(a, amode, pro, blocks, s);
  } else if (bn == 64) {
    if (sk)
      launch_x3<64, true>(a, amode, pro, blocks, s);
    else
      launch_x3<64, false>(a, amode, pro, blocks, s);
  } else {
    return CAPMI_EINVAL;
  }
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_split3_bf16(const float* in, long long n, void* out, void* stream) {
  CAPMI_REQUIRE(in && out && n >= 0 && n % 4 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(in) && ((reinterpret_cast<uintptr_t>(out) & 7u) == 0), CAPMI_EALIGN);
  if (n == 0) return 0;
  const long long n4 = n / 4;
  const unsigned blocks = (unsigned)std::min<long long>(std::max<long long>(cdiv(n4, 256), 1), 8192);
  hipLaunchKernelGGL(split3_bf16_kernel, dim3(blocks), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(in), n4, static_cast<bf16x4_x*>(out));
  CAPMI_LAUNCH_CHECK();
  return 0;
}
