// fp32 MFMA GEMM and implicit-GEMM convolution for gfx950.
//
// One kernel template serves every dense contraction of the training step:
//   * nn.Linear forward / dX / dW (models/attention.py:33-35,54-55,110-114,162-163,270,279)
//   * LSTMCell gate GEMMs (models/attention.py:108-109,277-278)
//   * all 104 Conv2d of torchvision ResNet-101 (models/encoder.py:88-91,107) as implicit
//     GEMMs over NHWC activations (k = (kh, kw, ci)), with the previous layer's
//     BatchNorm-apply + ReLU fused into the A-tile load and the BatchNorm(train)
//     batch statistics fused into the epilogue.
//
// Exact fp32: v_mfma_f32_32x32x2_f32 (gfx950 has no xf32); each 32x32 accumulator is a
// k-ordered fmaf chain. Tiles: 128x128x16 (4 waves of 64x64) for large problems,
// 64x64x16 (4 waves of 32x32) for the per-timestep decoder GEMMs (M = batch), which
// rely on split-K for parallelism; split partial slabs are summed by the consumer.
// Global->LDS staging is register-double-buffered: tile t+1 is loaded into registers
// while tile t is multiplied out of LDS, one barrier per K-tile.
#include <cstdlib>

#include "common.h"

#include "gemm_args.h"

constexpr int BK = 16;

template <int AMODE> struct APad { static constexpr int v = 2; };
template <> struct APad<1> { static constexpr int v = 4; };
template <> struct APad<3> { static constexpr int v = 4; };
template <int BMODE> struct BPad { static constexpr int v = 2; };
template <> struct BPad<1> { static constexpr int v = 4; };

// load 4 consecutive elements p[0..3] of which `n` (0..4) are in bounds
template <bool VEC>
__device__ __forceinline__ float4 load4(const float* p, int n) {
  if (VEC) {
    return n > 0 ? *reinterpret_cast<const float4*>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
  } else {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n > 0) v.x = p[0];
    if (n > 1) v.y = p[1];
    if (n > 2) v.z = p[2];
    if (n > 3) v.w = p[3];
    return v;
  }
}

template <int BM, int BN, int WM, int WN, int AMODE, int BMODE, bool VEC>
__global__ void __launch_bounds__(256) gemm_kernel(const GemmArgs args) {
  constexpr int NWN = BN / WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int SA = BM + APad<AMODE>::v;
  constexpr int SB = BN + BPad<BMODE>::v;
  // A slots per thread per K-tile: float4 slots for modes 0-2, scalars for mode 3
  constexpr int NA = (AMODE == 3) ? (BM * BK / 256) : (BM * BK / 4 / 256);
  constexpr int NB = BN * BK / 4 / 256;
  static_assert(NA >= 1 && NB >= 1, "tile too small");
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");

  __shared__ __attribute__((aligned(16))) float As[2][BK][SA];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][SB];
  __shared__ float red[4][2][32 * TN];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm0 = (wid / NWN) * WM, wn0 = (wid % NWN) * WN;

  int bid = blockIdx.x, pi = 0;
  while (pi + 1 < args.nprob && bid >= args.tiles_begin[pi + 1]) ++pi;
  const capmi_gemm_problem& P = args.p[pi];
  const int local = bid - args.tiles_begin[pi];
  const int tiles_n = args.tiles_n[pi], tiles_m = args.tiles_m[pi];
  const int tn = local % tiles_n;
  const int tm = (local / tiles_n) % tiles_m;
  const int z = local / (tiles_n * tiles_m);
  const int M = P.M, N = P.N, K = P.K;
  const int k_begin = z * args.kchunk[pi];
  const int k_end = min(K, k_begin + args.kchunk[pi]);
  const int nkt = k_end > k_begin ? (k_end - k_begin + BK - 1) / BK : 0;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-thread A-row precompute --------------------------------------------------
  const float* a_ptr[NA];
  int a_ih0[NA], a_iw0[NA];
  bool a_ok[NA];
  int a_kk[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int f = tid + i * 256;
    if (AMODE == 0 || AMODE == 2) {
      const int row = m0 + (f >> 2);
      a_kk[i] = (f & 3) * 4;
      a_ok[i] = row < M;
      if (AMODE == 0) {
        a_ptr[i] = P.A + (a_ok[i] ? remap(row, P.a_r1, P.lda, P.a_s2) : 0);
      } else {
        const int hw = P.cHo * P.cWo;
        const int n = row / hw, rem = row - n * hw;
        const int oh = rem / P.cWo, ow = rem - oh * P.cWo;
        a_ih0[i] = oh * P.cStride - P.cPad;
        a_iw0[i] = ow * P.cStride - P.cPad;
        a_ptr[i] = P.A + (long long)n * P.cH * P.cW * P.cCin;
      }
    } else if (AMODE == 1) {
      a_kk[i] = f / (BM / 4);
      const int m = m0 + (f % (BM / 4)) * 4;
      a_ok[i] = m < M;
      a_ptr[i] = P.A + m;
      a_ih0[i] = min(4, M - m);
    } else {  // AMODE 3: scalar gather, r = f % BM, kk = f / BM
      const int row = m0 + (f % BM);
      a_kk[i] = f / BM;
      a_ok[i] = row < M;
      const int hw = P.cHo * P.cWo;
      const int n = row / hw, rem = row - n * hw;
      const int oh = rem / P.cWo, ow = rem - oh * P.cWo;
      a_ih0[i] = oh * P.cStride - P.cPad;
      a_iw0[i] = ow * P.cStride - P.cPad;
      a_ptr[i] = P.A + (long long)n * P.cCin * P.cH * P.cW;
    }
  }
  // ---- per-thread B precompute ----------------------------------------------------
  const float* b_ptr[NB];
  int b_kk[NB], b_nv[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int f = tid + i * 256;
    if (BMODE == 0) {
      const int n = n0 + (f >> 2);
      b_kk[i] = (f & 3) * 4;
      b_nv[i] = n < N;
      b_ptr[i] = P.B + (n < N ? (long long)n * P.ldb : 0);
    } else {
      b_kk[i] = f / (BN / 4);
      const int n = n0 + (f % (BN / 4)) * 4;
      b_nv[i] = max(0, min(4, N - n));
      b_ptr[i] = P.B + (n < N ? n : 0);
    }
  }

  float4 ra[NA];
  float rs[NA];  // scalar staging for AMODE 3
  float4 rb[NB];

  auto load_tile = [&](int kt) {
    const int k0 = k_begin + kt * BK;
    if (AMODE == 0) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int k = k0 + a_kk[i];
        const int nv = a_ok[i] ? max(0, min(4, k_end - k)) : 0;
        ra[i] = load4<VEC>(a_ptr[i] + k, nv);
      }
    } else if (AMODE == 1) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int k = k0 + a_kk[i];
        const bool ok = a_ok[i] && k < k_end;
        ra[i] = load4<VEC>(a_ptr[i] + (ok ? remap(k, P.a_r1, P.lda, P.a_s2) : 0), ok ? a_ih0[i] : 0);
      }
    } else if (AMODE == 2) {
      const int kpos = k0 / P.cCin;
      const int ci0 = k0 - kpos * P.cCin;
      const int kh = kpos / P.cKW, kw = kpos - kh * P.cKW;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
        const bool ok = a_ok[i] && k0 < k_end && ih >= 0 && ih < P.cH && iw >= 0 && iw < P.cW;
        const int ci = ci0 + a_kk[i];
        float4 v = load4<true>(a_ptr[i] + ((long long)ih * P.cW + iw) * P.cCin + ci, ok ? 4 : 0);
        if (P.in_scale != nullptr && ok) {
          const float4 sc = *reinterpret_cast<const float4*>(P.in_scale + ci);
          const float4 sh = *reinterpret_cast<const float4*>(P.in_shift + ci);
          v = relu4(fma4(v, sc, sh));
        }
        ra[i] = v;
      }
    } else {  // AMODE 3
      const int khw = P.cKH * P.cKW;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int k = k0 + a_kk[i];
        float v = 0.f;
        if (a_ok[i] && k < k_end) {
          const int ci = k / khw, rem = k - ci * khw;
          const int kh = rem / P.cKW, kw = rem - kh * P.cKW;
          const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
          if (ih >= 0 && ih < P.cH && iw >= 0 && iw < P.cW) {
            v = a_ptr[i][((long long)ci * P.cH + ih) * P.cW + iw];
            if (P.in_scale != nullptr) v = fmaxf(fmaf(v, P.in_scale[ci], P.in_shift[ci]), 0.f);
          }
        }
        rs[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int k = k0 + b_kk[i];
      if (BMODE == 0) {
        const int nv = b_nv[i] ? max(0, min(4, k_end - k)) : 0;
        rb[i] = load4<VEC>(b_ptr[i] + k, nv);
      } else {
        const bool ok = k < k_end;
        rb[i] = load4<VEC>(b_ptr[i] + (ok ? (long long)k * P.ldb : 0), ok ? b_nv[i] : 0);
      }
    }
  };

  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int f = tid + i * 256;
      if (AMODE == 0 || AMODE == 2) {
        const int r = f >> 2, kq = a_kk[i];
        As[buf][kq + 0][r] = ra[i].x;
        As[buf][kq + 1][r] = ra[i].y;
        As[buf][kq + 2][r] = ra[i].z;
        As[buf][kq + 3][r] = ra[i].w;
      } else if (AMODE == 1) {
        *reinterpret_cast<float4*>(&As[buf][a_kk[i]][(f % (BM / 4)) * 4]) = ra[i];
      } else {
        As[buf][a_kk[i]][f % BM] = rs[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = tid + i * 256;
      if (BMODE == 0) {
        const int r = f >> 2, kq = b_kk[i];
        Bs[buf][kq + 0][r] = rb[i].x;
        Bs[buf][kq + 1][r] = rb[i].y;
        Bs[buf][kq + 2][r] = rb[i].z;
        Bs[buf][kq + 3][r] = rb[i].w;
      } else {
        *reinterpret_cast<float4*>(&Bs[buf][b_kk[i]][(f % (BN / 4)) * 4]) = rb[i];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int lr = lane & 31, lk = lane >> 5;
  if (nkt > 0) {
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nkt) load_tile(kt + 1);
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        float a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = As[buf][2 * kk + lk][wm0 + 32 * i + lr];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = Bs[buf][2 * kk + lk][wn0 + 32 * j + lr];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nkt) store_tile(buf ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue ---------------------------------------------------------------------
  const float alpha = P.alpha * (P.alpha_ptr ? *P.alpha_ptr : 1.f);
  float* Cz = P.C + (long long)z * P.c_split_stride;
  const bool want_stats = P.stats != nullptr;
  float csum[TN], csq[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    csum[j] = 0.f;
    csq[j] = 0.f;
    const int col = n0 + wn0 + 32 * j + lr;
    const bool cok = col < N;
    float bias = 0.f;
    if (z == 0 && cok) {
      if (P.bias) bias += P.bias[col];
      if (P.bias2) bias += P.bias2[col];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (cok && row < M) {
          float* cp = Cz + remap(row, P.c_r1, P.ldc, P.c_s2) + col;
          float v = fmaf(acc[i][j][r], alpha, bias);
          if (P.beta != 0.f) v = fmaf(P.beta, *cp, v);
          if (P.relu) v = fmaxf(v, 0.f);
          *cp = v;
          csum[j] += v;
          csq[j] = fmaf(v, v, csq[j]);
        }
      }
    }
  }
  if (want_stats) {
    // per-channel (sum, sumsq) per 64-row slice, as gemm_nt.hip
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      csum[j] += __shfl_xor(csum[j], 32, 64);
      csq[j] += __shfl_xor(csq[j], 32, 64);
    }
    if (WM == 64) {
      if (lk == 0) {
        const long long sl = (m0 + wm0) >> 6;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + wn0 + 32 * j + lr;
          if (col < N && m0 + wm0 < M) {
            P.stats[(sl * N + col) * 2 + 0] = csum[j];
            P.stats[(sl * N + col) * 2 + 1] = csq[j];
          }
        }
      }
    } else {
      if (lk == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          red[wid][0][32 * j + lr] = csum[j];
          red[wid][1][32 * j + lr] = csq[j];
        }
      }
      __syncthreads();
      constexpr int NWM = BM / WM;
      for (int c = tid; c < BN; c += 256) {
        const int wn = c / WN, cc = c % WN;
        float s = 0.f, q = 0.f;
        for (int w = 0; w < NWM; ++w) {
          s += red[w * NWN + wn][0][cc];
          q += red[w * NWN + wn][1][cc];
        }
        const int col = n0 + c;
        if (col < N) {
          P.stats[((long long)tm * N + col) * 2 + 0] = s;
          P.stats[((long long)tm * N + col) * 2 + 1] = q;
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int AMODE, int BMODE>
static int launch_t(const GemmArgs& a, bool vec, int blocks, hipStream_t s) {
  if (vec)
    CAPMI_KLAUNCH((gemm_kernel<BM, BN, WM, WN, AMODE, BMODE, true>), dim3(blocks), dim3(256), 0,
                       s, a);
  else
    CAPMI_KLAUNCH((gemm_kernel<BM, BN, WM, WN, AMODE, BMODE, false>), dim3(blocks), dim3(256),
                       0, s, a);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

template <int BM, int BN, int WM, int WN>
static int launch_mode(const GemmArgs& a, int amode, int bmode, bool vec, int blocks, hipStream_t s) {
  if (amode == 0 && bmode == 0) return launch_t<BM, BN, WM, WN, 0, 0>(a, vec, blocks, s);
  if (amode == 0 && bmode == 1) return launch_t<BM, BN, WM, WN, 0, 1>(a, vec, blocks, s);
  if (amode == 1 && bmode == 0) return launch_t<BM, BN, WM, WN, 1, 0>(a, vec, blocks, s);
  if (amode == 1 && bmode == 1) return launch_t<BM, BN, WM, WN, 1, 1>(a, vec, blocks, s);
  if (amode == 2 && bmode == 0) return launch_t<BM, BN, WM, WN, 2, 0>(a, true, blocks, s);
  if (amode == 3 && bmode == 0) return launch_t<BM, BN, WM, WN, 3, 0>(a, vec, blocks, s);
  return CAPMI_EINVAL;
}

extern "C" int capmi_gemm_stat_tiles(int M, int tile) {
  // statistics rows are always kept per 64-row slice, whatever tile ran (see capmi.h)
  (void)tile;
  return (M + 63) / 64;
}

static long long tiles_of(const capmi_gemm_problem* probs, int nprob, int bm, int bn) {
  long long t = 0;
  for (int i = 0; i < nprob; ++i)
    t += (long long)((probs[i].M + bm - 1) / bm) * ((probs[i].N + bn - 1) / bn) * probs[i].ksplit;
  return t;
}

namespace {
struct GemmPlan {
  GemmArgs a;
  int bm, bn;
  int nt = 256;  // threads per workgroup of the v2 kernel (512: CAPMI_TILE_128_W8)
  bool nt_ok, vec;
  long long total;  // workgroups of the data-parallel launch
};

int gemm_plan(const capmi_gemm_problem* probs, int nprob, int amode, int bmode, int tile, GemmPlan& g) {
  CAPMI_REQUIRE(probs != nullptr && nprob >= 1 && nprob <= CAPMI_MAX_GROUP, CAPMI_EINVAL);
  CAPMI_REQUIRE(amode >= 0 && amode <= 4 && bmode >= 0 && bmode <= 2, CAPMI_EINVAL);
  CAPMI_REQUIRE(bmode != 2 || amode == 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(tile >= CAPMI_TILE_128 && tile <= CAPMI_TILE_128_W8, CAPMI_EINVAL);
  CAPMI_REQUIRE(amode != 4 || bmode == 0, CAPMI_EINVAL);
  GemmArgs& a = g.a;
  memset(&a, 0, sizeof(a));
  a.nprob = nprob;
  bool vec = true;
  // v2 kernel eligible: row-major A (dense / conv) with B = W[N][K], or the transposed-staging
  // forms (A stored as k rows and/or B stored as k rows) of the backward GEMMs
  bool nt_ok = ((amode == 0 || amode == 2 || amode == 4) && bmode == 0) || ((amode == 0 || amode == 1) && bmode == 1) ||
               (amode == 1 && bmode == 2);
  int maxN = 0;
  for (int i = 0; i < nprob; ++i) {
    const capmi_gemm_problem& p = probs[i];
    CAPMI_REQUIRE(p.M >= 0 && p.N >= 0 && p.K >= 0 && p.ksplit >= 1, CAPMI_EINVAL);
    CAPMI_REQUIRE(p.A && p.B && p.C, CAPMI_EINVAL);
    CAPMI_REQUIRE(p.ksplit == 1 || p.c_split_stride > 0, CAPMI_EINVAL);
    CAPMI_REQUIRE(p.stats == nullptr || p.ksplit == 1, CAPMI_EINVAL);
    if (amode == 2) {
      CAPMI_REQUIRE(p.cCin % BK == 0 && p.cCin % 4 == 0, CAPMI_EALIGN);
      CAPMI_REQUIRE(p.K == p.cKH * p.cKW * p.cCin && p.M == p.cN * p.cHo * p.cWo, CAPMI_EINVAL);
      CAPMI_REQUIRE(aligned16(p.A), CAPMI_EALIGN);
      CAPMI_REQUIRE(p.in_scale == nullptr || (aligned16(p.in_scale) && aligned16(p.in_shift)),
                    CAPMI_EALIGN);
      CAPMI_REQUIRE(aligned16(p.B) && p.ldb % 4 == 0, CAPMI_EALIGN);
      nt_ok = nt_ok && p.cCin % 32 == 0;
    }
    if (amode == 4) {
      CAPMI_REQUIRE(p.cCin == 4 && p.K == p.cKH * p.cKW * 4 && p.M == p.cN * p.cHo * p.cWo, CAPMI_EINVAL);
      CAPMI_REQUIRE(aligned16(p.A) && aligned16(p.B) && p.ldb % 4 == 0 && p.in_scale == nullptr,
                    CAPMI_EALIGN);
    }
    if (bmode == 2) {
      // weight gradient of a conv: B[k = output pixel][n = (kh, kw, ci)] = X (implicit im2col)
      CAPMI_REQUIRE(p.cCin % 4 == 0 && p.N == p.cKH * p.cKW * p.cCin && p.K == p.cN * p.cHo * p.cWo,
                    CAPMI_EINVAL);
      CAPMI_REQUIRE(p.K < (1 << 24), CAPMI_ERANGE);
      CAPMI_REQUIRE(aligned16(p.B), CAPMI_EALIGN);
      CAPMI_REQUIRE(p.in_scale == nullptr || (aligned16(p.in_scale) && aligned16(p.in_shift)),
                    CAPMI_EALIGN);
    }
    if (amode == 3) {
      CAPMI_REQUIRE(p.K == p.cKH * p.cKW * p.cCin && p.M == p.cN * p.cHo * p.cWo, CAPMI_EINVAL);
    }
    if (amode == 0) {
      vec = vec && aligned16(p.A) && p.lda % 4 == 0 && p.K % 4 == 0 && (p.a_r1 <= 0 || p.a_s2 % 4 == 0);
    } else if (amode == 1) {
      vec = vec && aligned16(p.A) && p.lda % 4 == 0 && p.M % 4 == 0 && (p.a_r1 <= 0 || p.a_s2 % 4 == 0);
    }
    if (bmode == 0)
      vec = vec && aligned16(p.B) && p.ldb % 4 == 0 && p.K % 4 == 0;
    else if (bmode == 2)
      vec = vec && p.N % 4 == 0;
    else
      vec = vec && aligned16(p.B) && p.ldb % 4 == 0 && p.N % 4 == 0;
    a.p[i] = p;
    maxN = std::max(maxN, p.N);
  }
  nt_ok = nt_ok && (vec || ((amode == 2 || amode == 4) && bmode == 0));
  CAPMI_REQUIRE(bmode != 2 || nt_ok, CAPMI_EALIGN);  // no generic-kernel form of the im2col B
  int bm = 128, bn = 128;
  g.nt = 256;
  if (tile == CAPMI_TILE_128_W8) {  // 512-thread 128x128 form: forward modes of the v2 kernel only
    CAPMI_REQUIRE(nt_ok && bmode == 0 && (amode == 0 || amode == 2 || amode == 4), CAPMI_EINVAL);
    g.nt = 512;
    tile = CAPMI_TILE_128;
  }
  if (tile == CAPMI_TILE_64) {
    bm = bn = 64;
  } else if (tile == CAPMI_TILE_128x64) {
    bn = 64;
  } else if (tile == CAPMI_TILE_AUTO) {
    if (!nt_ok) {
      bm = bn = (tiles_of(probs, nprob, 128, 128) >= 256 ? 128 : 64);
    } else {
      // measured on the ResNet-101 / decoder shapes (tools/gemm_sweep.py): the 64x64 tile
      // (4 WGs per CU) is the fastest or within noise of it on every one of them
      bm = bn = 64;
    }
  }
  if (!nt_ok && bm != bn) bn = bm = 128;
  const int bk = nt_ok ? 32 : BK;
  long long total = 0;
  for (int i = 0; i < nprob; ++i) {
    const capmi_gemm_problem& p = probs[i];
    a.tiles_m[i] = (p.M + bm - 1) / bm;
    a.tiles_n[i] = (p.N + bn - 1) / bn;
    int kc = (p.K + p.ksplit - 1) / p.ksplit;
    kc = ((kc + bk - 1) / bk) * bk;
    a.kchunk[i] = kc > 0 ? kc : bk;
    a.tiles_begin[i] = (int)total;
    total += (long long)a.tiles_m[i] * a.tiles_n[i] * p.ksplit;
  }
  a.tiles_begin[nprob] = (int)total;
  CAPMI_REQUIRE(total < (1LL << 31), CAPMI_ERANGE);
  g.bm = bm;
  g.bn = bn;
  g.nt_ok = nt_ok;
  g.vec = vec;
  g.total = total;
  return 0;
}

int gemm_launch_dp(const GemmPlan& g, int amode, int bmode, hipStream_t s) {
  if (g.total == 0) return 0;
  if (g.nt_ok) return gemm_nt_launch(g.a, amode, bmode, g.bm, g.bn, (int)g.total, s, false, g.nt);
  if (g.bm == 128) return launch_mode<128, 128, 64, 64>(g.a, amode, bmode, g.vec, (int)g.total, s);
  return launch_mode<64, 64, 32, 32>(g.a, amode, bmode, g.vec, (int)g.total, s);
}

int cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// CUs the stream-K grids are sized for: cu_count(), or CAPMI_SK_CUS (A/B measurement: fewer
// persistent workers than CUs leave CUs free for the concurrently running decoder stream)
int sk_cus() {
  static const int n = [] {
    const char* e = getenv("CAPMI_SK_CUS");
    const int v = e ? atoi(e) : 0;
    return v > 0 && v < cu_count() ? v : cu_count();
  }();
  return n;
}

constexpr int kSkMaxWgPerCu = 4;
long long sk_flag_bytes(int cus) { return ((long long)(cus * kSkMaxWgPerCu + 1) * 4 + 255) / 256 * 256; }
}  // namespace

extern "C" int capmi_gemm(const capmi_gemm_problem* probs, int nprob, int amode, int bmode,
                          int tile, void* stream) {
  GemmPlan g;
  const int rc = gemm_plan(probs, nprob, amode, bmode, tile, g);
  if (rc) return rc;
  return gemm_launch_dp(g, amode, bmode, as_stream(stream));
}

extern "C" long long capmi_gemm_workspace_flag_bytes(void) { return sk_flag_bytes(cu_count()); }

namespace {
int flag_terms(int flags);
bool terms_mode_ok(int terms, int amode, int bmode);
}  // namespace

extern "C" int capmi_gemm_ex(const capmi_gemm_problem* probs, int nprob, int amode, int bmode, int tile, int flags,
                             void* stream) {
  const int terms = flag_terms(flags);
  CAPMI_REQUIRE(terms >= 0, CAPMI_EINVAL);
  if (terms == 0) return capmi_gemm(probs, nprob, amode, bmode, tile, stream);
  CAPMI_REQUIRE(terms_mode_ok(terms, amode, bmode) && tile != CAPMI_TILE_128_W8, CAPMI_EINVAL);
  GemmPlan g;
  const int rc = gemm_plan(probs, nprob, amode, bmode, tile, g);
  if (rc) return rc;
  bool split_ok = g.nt_ok && g.vec;
  for (int i = 0; i < nprob; ++i) split_ok = split_ok && probs[i].in_scale == nullptr;
  // shapes the split forms do not cover (unaligned / generic-kernel problems): the fp32 kernel
  if (!split_ok) return gemm_launch_dp(g, amode, bmode, as_stream(stream));
  if (g.total == 0) return 0;
  return gemm_nt_launch(g.a, amode, bmode, g.bm, g.bn, (int)g.total, as_stream(stream), terms);
}

extern "C" long long capmi_gemm_workspace_bytes(void) {
  const int cus = cu_count();
  // parked partials: (WGs per CU) * BM * BN floats per CU is 64 KB for 4 x 64x64 and for
  // 2 x 128x64, 128 KB for 2 x 128x128 and 1 x 256x128
  return sk_flag_bytes(cus) + (long long)cus * 128 * 1024;
}

namespace {
// XCD-grouped stream-K (gemm_nt.hip); CAPMI_SK_GROUPS=1 turns it off (A/B measurement)
bool sk_xcd_groups() {
  static const bool on = [] {
    const char* e = getenv("CAPMI_SK_GROUPS");
    return !(e && e[0] == '1' && e[1] == 0);
  }();
  return on;
}
// hybrid data-parallel + stream-K schedule (gemm_nt.hip); CAPMI_SK_HYBRID=0 turns it off (A/B)
bool sk_hybrid() {
  static const bool on = [] {
    const char* e = getenv("CAPMI_SK_HYBRID");
    return !(e && e[0] == '0' && e[1] == 0);
  }();
  return on;
}
// CAPMI_SK_OFF=1: data-parallel grids everywhere (A/B measurement: a persistent stream-K grid
// holds every CU until it ends, a data-parallel one frees CUs as its tiles retire)
bool sk_off() {
  static const bool off = [] {
    const char* e = getenv("CAPMI_SK_OFF");
    return e && e[0] == '1' && e[1] == 0;
  }();
  return off;
}
// the three-term conv weight gradients keep the fp32 wgrad tile rule (128x128 / 128x64, one workgroup per
// CU): fine-tune config 1633 -> 1647 img/s against 64x64 (fewer re-reads of dY and the im2col rows).
// CAPMI_X3_WGRAD_WIDE=0: 64x64 (A/B measurement)
bool x3_wgrad_wide() {
  static const bool on = [] {
    const char* e = getenv("CAPMI_X3_WGRAD_WIDE");
    return !(e && e[0] == '0' && e[1] == 0);
  }();
  return on;
}
// the encoder-sized three-term GEMMs that keep the fp32 tile rule instead of 64x64 (bit mask, A/B
// measurement; CAPMI_X3_KEEP_TILE): 1 the 1x1 weight gradients (k rows, K >= 8192 output pixels),
// 2 the 1x1 data gradients (M >= 8192 output pixels). The decoder's GEMMs stay below both bounds.
int x3_keep_tile() {
  static const int m = [] {
    const char* e = getenv("CAPMI_X3_KEEP_TILE");
    return e ? atoi(e) : 0;
  }();
  return m;
}
// the launch capmi_gemm_sk makes for a problem (shared by the launcher and the plan query)
int sk_decide(const capmi_gemm_problem* prob, int amode, int bmode, int tile, int terms, GemmPlan& g, bool& sk) {
  const bool bf16 = terms > 0;
  CAPMI_REQUIRE(prob != nullptr, CAPMI_EINVAL);
  const int nkt = (prob->K + 31) / 32;
  const bool automatic = tile == CAPMI_TILE_AUTO;
  // measured (tools/gemm_sweep.py, ResNet-101 shapes at batch 64): with >= 16 k-tiles per
  // output tile, stream-K over 128x64 tiles is the fastest form; below that the per-segment
  // pipeline fill outweighs the balance gain and 64x64 data-parallel wins
  if (automatic) tile = nkt >= 16 ? CAPMI_TILE_128x64 : CAPMI_TILE_64;
  // conv weight gradients (k = output pixels, always >= 16 k-tiles; tools/wgrad_tile_ab.py, with
  // the k-major LDS images): 128x128 for the wide 3x3 ones (Cout >= 256, N = 9*Cin >= 2048:
  // layer3/4, 1-7 % faster than 128x64), 128x64 for the rest (layer2 3x3 and the 1x1 ones: 128x128
  // is up to 2x slower there, 64x64 5-12 % slower)
  if (automatic && amode == CAPMI_A_MMAJOR && bmode == CAPMI_B_CONV_NHWC)
    tile = (prob->M >= 256 && prob->N >= 2048) ? CAPMI_TILE_128 : CAPMI_TILE_128x64;
  // three-term split staging: 64x64 everywhere (two workgroups per CU; the larger tiles hold one:
  // tools/dec_gemm_ab.py --tile, 5-20 % faster on every decoder GEMM at 64x64)
  const bool keep = (bmode == CAPMI_B_CONV_NHWC && x3_wgrad_wide()) ||
                    ((x3_keep_tile() & 1) && amode == CAPMI_A_MMAJOR && bmode == CAPMI_B_KROWS && prob->K >= 8192) ||
                    ((x3_keep_tile() & 2) && amode == CAPMI_A_KMAJOR && bmode == CAPMI_B_NMAJOR_W && prob->M >= 8192);
  if (automatic && terms == 3 && !keep) tile = CAPMI_TILE_64;
  int rc = gemm_plan(prob, 1, amode, bmode, tile, g);
  if (rc) return rc;
  // the 512-thread 128x128 form (tools/w8_ab.sh over all 19 encoder conv shapes, batch 64):
  // 2-12% faster wherever N >= 128 and either the k-loop is long (>= 16 k-tiles) or N <= 256;
  // slower for N = 64 (half the tile idle) and for N >= 512 with a short k-loop (64x64 keeps
  // 4 workgroups per CU to hide the epilogue)
  if (automatic && g.nt_ok && !bf16 && bmode == 0 && (amode == 0 || amode == 2 || amode == 4) &&
      prob->ksplit == 1 && prob->M >= 2048 && prob->N >= 128 && (nkt >= 16 || prob->N <= 256)) {
    rc = gemm_plan(prob, 1, amode, bmode, CAPMI_TILE_128_W8, g);
    if (rc) return rc;
  }
  const long long slots = (long long)sk_cus() * (g.nt == 512 ? 1 : gemm_nt_wg_per_cu(g.bm, g.bn, terms));
  const long long tiles = g.total;
  // short k-loops (< 16 k-tiles) stay data-parallel even in the hybrid form: splitting the last
  // rounds' tiles there cost 6-10 % on the layer1-3 1x1 shapes (tools/hybrid_ab.sh)
  sk = g.nt_ok && prob->ksplit == 1 && tiles > 0 && (!automatic || nkt >= 16);
  if (sk) {
    // stream-K only when the data-parallel grid would leave a costly partial last round
    const long long rounds = (tiles + slots - 1) / slots;
    sk = (double)tiles / (double)(rounds * slots) < 0.9;
  }
  if (sk_off()) sk = false;
  return 0;
}
}  // namespace

namespace {
// operand staging of the v2 kernel: 0 fp32, 1 bf16 (CAPMI_GEMM_BF16), 3 three-term split
// (CAPMI_GEMM_SPLIT3); -1 for any other flag combination
int flag_terms(int flags) {
  if (flags == 0) return 0;
  if (flags == CAPMI_GEMM_BF16) return 1;
  if (flags == CAPMI_GEMM_SPLIT3) return 3;
  return -1;
}
// the modes a split-staged (terms > 0) launch supports (gemm_nt.hip: gemm_nt_launch)
bool terms_mode_ok(int terms, int amode, int bmode) {
  if (terms == 0) return true;
  if (bmode == 0 && (amode == 2 || amode == 4)) return true;  // convs
  if (bmode == 2) return terms == 3 && amode == 1;             // conv weight gradients (three-term split)
  if (terms == 1 && bmode == 0) return amode == 0;
  return (amode == 0 && bmode <= 1) || (amode == 1 && bmode == 1);
}
int x3_plan(const capmi_gemm_problem* prob, int amode, int bmode, int tile, GemmArgs& a, int& bn, bool& sk,
            long long& total);
int x3p_plan(const capmi_gemm_problem* prob, int amode, int bmode, GemmArgs& a, bool& sk, long long& total,
             int& bk);
int x3d_plan(const capmi_gemm_problem* prob, int amode, int bmode, GemmArgs& a, bool& sk, long long& total);
int x3s_plan(const capmi_gemm_problem* prob, int amode, int bmode, long long& lda, int& tiles, int& grid);
int x3c_plan(const capmi_gemm_problem* prob, int amode, int bmode, int& tiles);
int x3w_plan(const capmi_gemm_problem* prob, int amode, int bmode, long long ws_floats, GemmArgs& a, int& S,
             long long& tiles);
// CAPMI_GEMM_BF16_IO's launch plan (shared by the launcher and capmi_gemm_sk_plan): the column tile bn (BM = 128),
// the LDS stages (1: the one-stage short-k form, 2) and stream-K
struct Bf16Plan {
  int bn, stages;
  bool sk;
  long long total;
};
Bf16Plan bf16_io_plan(const capmi_gemm_problem& p, int tile, bool have_ws) {
  // AUTO on a short k (K <= 256: the bf16 config's 1x1 c3 convs, layer1's K = 64 convs and downsample, the c1 of
  // layer1): 128x64 tiles, one LDS stage, four workgroups per CU, data-parallel (round 5: l3 c3 20.0 -> 17.1 us, l2 c3
  // 24.7 -> 18.4, l1 c3 33.3 -> 24.3; at K = 512 a tie and above it slower). Round 6: alone, the K = 256 convs on 128+
  // columns run faster on the DMA ring below (l3 c3 17.3 -> 16.0 us, ds2 29.3 -> 28.1), but in the pipelined config-5
  // step the one-stage form stays ahead (13330 -> 13365 img/s, three interleaved rounds, same box); CAPMI_BF16_ST1_K = k
  // moves the bound (A/B)
  static const int st1_k = [] {
    const char* e = getenv("CAPMI_BF16_ST1_K");
    return e ? atoi(e) : 256;
  }();
  const bool st1 = tile == CAPMI_TILE_AUTO && p.K <= st1_k;
  // AUTO on a grid of 128x128 tiles that fills at most half the CUs (layer4's 3136-row convs: 100 tiles):
  // 128x64 tiles, twice the workgroups (round 5: l4 3x3 53.2 -> 40.8 us, l4 c1 25.8 -> 18.9; the 400-tile
  // layer4 c3 / downsample and layer3's 196-tile grids stay at 128x128, where 128x64 measured slower)
  const bool narrow = tile == CAPMI_TILE_AUTO && 2 * cdiv(p.M, 128) * cdiv(p.N, 128) <= cu_count();
  Bf16Plan r;
  r.bn = (st1 || narrow || tile == CAPMI_TILE_128x64 || tile == CAPMI_TILE_64 || (tile == CAPMI_TILE_AUTO && p.N <= 64))
             ? 64 : 128;
  r.total = cdiv(p.M, 128) * cdiv(p.N, r.bn);
  const long long slots = (long long)sk_cus() * 2;
  const long long rounds = (r.total + slots - 1) / slots;
  // (round 3) stream-K for the bf16 convs only on CAPMI_BF16_SK=1: data-parallel grids measured faster in the
  // pipelined bf16 step (config 5)
  static const bool bf16_sk = [] {
    const char* e = getenv("CAPMI_BF16_SK");
    return e && e[0] == '1';
  }();
  r.sk = !st1 && bf16_sk && !sk_off() && have_ws && p.K / 64 >= 4 && (double)r.total / (double)(rounds * slots) < 0.9;
  // (round 6) data-parallel: the LDS-DMA ring (gemm_bf16.hip), four k-tiles deep at one workgroup per CU when the grid
  // is one round of tiles (layer3's 196-tile and layer4's 200-tile grids: l3 3x3 28.7 -> 23.4 us, l3 c1 15.8 -> 12.5,
  // l4 c1 17.5 -> 14.7), else two deep at two workgroups per CU (l2 3x3 25.3 -> 21.4, l1 3x3 35.6 -> 31.4, ds3 27.4 ->
  // 23.3, l4 c3 15.2 -> 13.1); CAPMI_BF16_STAGES = 2 / 4 forces one depth (A/B)
  static const int bf16_stages = [] {
    const char* e = getenv("CAPMI_BF16_STAGES");
    const int v = e ? atoi(e) : 0;
    return v == 2 || v == 4 ? v : 0;
  }();
  r.stages = st1 ? 1 : r.sk ? 2 : bf16_stages ? bf16_stages : r.total <= cu_count() ? 4 : 2;
  return r;
}
}  // namespace

extern "C" int capmi_gemm_sk_plan(const capmi_gemm_problem* prob, int amode, int bmode, int tile, int flags,
                                  int* bm, int* bn, int* stream_k, int* generic, int* threads) {
  GemmPlan g;
  bool sk = false;
  if (flags == CAPMI_GEMM_X3P) {
    GemmArgs a;
    long long total = 0;
    int bk = 32;
    const int rc = x3p_plan(prob, amode, bmode, a, sk, total, bk);
    if (rc) return rc;
    if (threads) *threads = 512;
    if (bm) *bm = 256;
    if (bn) *bn = 128;
    if (stream_k) *stream_k = sk ? 1 : 0;
    if (generic) *generic = bk;  // CAPMI_GEMM_X3P: the k-tile depth
    return 0;
  }
  if (flags == CAPMI_GEMM_X3D) {
    GemmArgs a;
    long long total = 0;
    const int rc = x3d_plan(prob, amode, bmode, a, sk, total);
    if (rc) return rc;
    if (threads) *threads = 512;
    if (bm) *bm = 256;
    if (bn) *bn = 128;
    if (stream_k) *stream_k = sk ? 1 : 0;
    if (generic) *generic = 32;
    return 0;
  }
  if (flags == CAPMI_GEMM_X3W || flags == (CAPMI_GEMM_X3W | CAPMI_GEMM_BF16)) {
    GemmArgs a;
    int S = 1;
    long long tiles = 0;
    const long long ws = (capmi_gemm_workspace_bytes() - capmi_gemm_workspace_flag_bytes()) / 4;
    const int rc = x3w_plan(prob, amode, bmode, ws, a, S, tiles);
    if (rc) return rc;
    if (threads) *threads = 512;
    if (bm) *bm = 256;
    if (bn) *bn = 128;
    if (stream_k) *stream_k = S > 1 ? 1 : 0;
    if (generic) *generic = S;  // CAPMI_GEMM_X3W: the k-splits
    return 0;
  }
  if (flags == CAPMI_GEMM_X3C) {
    int tiles = 0;
    const int rc = x3c_plan(prob, amode, bmode, tiles);
    if (rc) return rc;
    if (threads) *threads = 512;
    if (bm) *bm = 256;
    if (bn) *bn = 64;
    if (stream_k) *stream_k = 0;
    if (generic) *generic = tiles;
    return 0;
  }
  if (flags == CAPMI_GEMM_X3S) {
    long long lda = 0;
    int tiles = 0, grid = 0;
    const int rc = x3s_plan(prob, amode, bmode, lda, tiles, grid);
    if (rc) return rc;
    if (threads) *threads = 256;
    if (bm) *bm = 64;
    if (bn) *bn = prob->N;
    if (stream_k) *stream_k = 0;
    if (generic) *generic = grid;  // CAPMI_GEMM_X3S: the persistent grid
    return 0;
  }
  if (flags == CAPMI_GEMM_X3) {
    GemmArgs a;
    int xbn = 128;
    long long total = 0;
    const int rc = x3_plan(prob, amode, bmode, tile, a, xbn, sk, total);
    if (rc) return rc;
    if (threads) *threads = 512;
    if (bm) *bm = 128;
    if (bn) *bn = xbn;
    if (stream_k) *stream_k = sk ? 1 : 0;
    if (generic) *generic = 0;
    return 0;
  }
  if (flags == CAPMI_GEMM_BF16_IO) {  // (the launcher's own plan; stream-K assumes a workspace is passed)
    CAPMI_REQUIRE(prob != nullptr && bmode == CAPMI_B_NMAJOR_W &&
                      (amode == CAPMI_A_KMAJOR || amode == CAPMI_A_CONV_NHWC) && prob->K > 0 && prob->K % 64 == 0,
                  CAPMI_EINVAL);
    const Bf16Plan pl = bf16_io_plan(*prob, tile, true);
    if (threads) *threads = pl.stages >= 2 && !pl.sk && pl.bn == 128 ? 512 : 256;  // (gemm_bf16.hip: bf16_threads)
    if (bm) *bm = 128;
    if (bn) *bn = pl.bn;
    if (stream_k) *stream_k = pl.sk ? 1 : 0;
    if (generic) *generic = pl.stages;  // CAPMI_GEMM_BF16_IO: the LDS stages (1: the one-stage short-k form)
    return 0;
  }
  int terms = flag_terms(flags);
  CAPMI_REQUIRE(terms >= 0 && terms_mode_ok(terms, amode, bmode), CAPMI_EINVAL);
  int rc = sk_decide(prob, amode, bmode, tile, terms, g, sk);
  if (rc) return rc;
  if (terms > 0 && !(g.nt_ok && g.nt == 256 && (prob->in_scale == nullptr || amode == CAPMI_A_CONV_NHWC || bmode == CAPMI_B_CONV_NHWC))) {
    rc = sk_decide(prob, amode, bmode, tile, 0, g, sk);
    if (rc) return rc;
  }
  if (threads) *threads = g.nt_ok ? g.nt : 256;
  if (bm) *bm = g.bm;
  if (bn) *bn = g.bn;
  if (stream_k) *stream_k = sk ? 1 : 0;
  if (generic) *generic = g.nt_ok ? 0 : 1;
  return 0;
}

namespace {
// CAPMI_GEMM_BF16_IO: bf16 A / B / C (gemm_bf16.hip), plain conv / dense GEMM with BN statistics
int gemm_bf16_io(const capmi_gemm_problem* prob, int amode, int bmode, int tile, void* workspace,
                 long long ws_bytes, hipStream_t s) {
  CAPMI_REQUIRE(prob != nullptr, CAPMI_EINVAL);
  const capmi_gemm_problem& p = *prob;
  CAPMI_REQUIRE(bmode == CAPMI_B_NMAJOR_W && (amode == CAPMI_A_KMAJOR || amode == CAPMI_A_CONV_NHWC), CAPMI_EINVAL);
  CAPMI_REQUIRE(p.A && p.B && p.C && p.M >= 0 && p.N > 0 && p.K > 0 && p.K % 64 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(p.ksplit == 1 && !p.bias && !p.bias2 && !p.alpha_ptr && p.alpha == 1.f && p.beta == 0.f &&
                    !p.relu && p.a_r1 <= 0 && p.c_r1 <= 0,
                CAPMI_EINVAL);
  // no prologue: the bf16 conv input is materialised once per tensor (capmi_bn_relu_bf16)
  CAPMI_REQUIRE(p.in_scale == nullptr && p.in_shift == nullptr, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(p.A) && aligned16(p.B) && p.ldb % 8 == 0 && p.ldb >= p.K && p.ldc >= p.N, CAPMI_EALIGN);
  CAPMI_REQUIRE((long long)p.N * p.ldb * 2 < (1LL << 31), CAPMI_ERANGE);
  if (amode == CAPMI_A_CONV_NHWC) {
    CAPMI_REQUIRE(p.cCin % 64 == 0 && p.K == p.cKH * p.cKW * p.cCin && p.M == p.cN * p.cHo * p.cWo, CAPMI_EINVAL);
    CAPMI_REQUIRE((long long)p.cN * p.cH * p.cW * p.cCin * 2 < (1LL << 31), CAPMI_ERANGE);
  } else {
    CAPMI_REQUIRE(p.lda % 8 == 0 && p.lda >= p.K, CAPMI_EALIGN);
    CAPMI_REQUIRE((long long)p.M * p.lda * 2 < (1LL << 31), CAPMI_ERANGE);
  }
  if (p.M == 0) return 0;
  const Bf16Plan pl = bf16_io_plan(p, tile, workspace != nullptr);
  const int bm = 128, bn = pl.bn;
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  a.p[0] = p;
  a.tiles_m[0] = (int)cdiv(p.M, bm);
  a.tiles_n[0] = (int)cdiv(p.N, bn);
  a.plain_epi = plain_epilogue(p, bn);  // (bf16 C: the fp32 bound on M * ldc is the stricter one)
  if (p.ldc % 8 != 0 || !aligned16(p.C)) a.plain_epi = 0;  // (its 16-B row-chunk stores)
  const long long total = pl.total;
  a.tiles_begin[1] = (int)total;
  const int cus = cu_count();
  const long long slots = (long long)sk_cus() * 2;
  const int nkt = p.K / 64;
  if (!pl.sk) return gemm_bf16_launch(a, amode, bm, bn, (int)total, s, pl.stages);
  CAPMI_REQUIRE(aligned16(workspace), CAPMI_EINVAL);
  CAPMI_REQUIRE(ws_bytes >= capmi_gemm_workspace_bytes(), CAPMI_ERANGE);
  a.sk_nkt = nkt;
  a.sk_units = total * nkt;
  a.sk_workers = (int)std::min<long long>(slots, a.sk_units);
  a.sk_groups = sk_xcd_groups() && a.sk_workers % 8 == 0 && total >= 64 ? 8 : 1;
  a.sk_flags = static_cast<int*>(workspace);
  a.sk_part = reinterpret_cast<float*>(static_cast<char*>(workspace) + sk_flag_bytes(cus));
  return gemm_bf16_launch(a, amode, bm, bn, a.sk_workers, s, 2);
}
}  // namespace

namespace {
// CAPMI_SK_FAMILY_OFF = bit mask of the x3 kernel families launched data-parallel instead of stream-K
// (1 gemm_x3, 2 x3p, 4 x3d). Default 1 (round 3): in the pipelined step, where the decoder stream holds CUs
// a stream-K worker may wait on, gemm_x3 measured faster data-parallel (headline 5987-5995 -> 6035-6048,
// fine-tune 1775 -> 1795 img/s, one box; small grids excepted, x3_plan); x3p (-10 %) and x3d (-7 %) keep
// stream-K
bool sk_family_off(int bit) {
  static const int mask = [] {
    const char* e = getenv("CAPMI_SK_FAMILY_OFF");
    return e ? atoi(e) : 1;
  }();
  return (mask & bit) != 0;
}

// CAPMI_GEMM_X3: fp32 A x three-plane bf16 B (gemm_x3.hip), one 512-thread workgroup per CU
int x3_plan(const capmi_gemm_problem* prob, int amode, int bmode, int tile, GemmArgs& a, int& bn, bool& sk,
            long long& total) {
  CAPMI_REQUIRE(prob != nullptr, CAPMI_EINVAL);
  const capmi_gemm_problem& p = *prob;
  CAPMI_REQUIRE(bmode == CAPMI_B_NMAJOR_W && (amode == CAPMI_A_KMAJOR || amode == CAPMI_A_CONV_NHWC), CAPMI_EINVAL);
  CAPMI_REQUIRE(p.A && p.B && p.C && p.M >= 0 && p.N > 0 && p.K > 0 && p.K % 32 == 0 && p.ksplit == 1, CAPMI_EINVAL);
  // the prologue is the conv input's BN-apply + ReLU: dense A takes none
  CAPMI_REQUIRE(amode == CAPMI_A_CONV_NHWC || (!p.in_scale && !p.in_shift), CAPMI_EINVAL);
  CAPMI_REQUIRE((p.in_scale == nullptr) == (p.in_shift == nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE(p.stats == nullptr || p.c_r1 <= 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(p.A) && aligned16(p.B) && p.ldb % 8 == 0 && p.ldb >= p.K, CAPMI_EALIGN);
  CAPMI_REQUIRE(p.in_scale == nullptr || (aligned16(p.in_scale) && aligned16(p.in_shift)), CAPMI_EALIGN);
  CAPMI_REQUIRE(3LL * p.N * p.ldb * 2 < (1LL << 31), CAPMI_ERANGE);
  if (amode == CAPMI_A_CONV_NHWC) {
    CAPMI_REQUIRE(p.cCin % 32 == 0 && p.K == p.cKH * p.cKW * p.cCin && p.M == p.cN * p.cHo * p.cWo, CAPMI_EINVAL);
    CAPMI_REQUIRE((long long)p.cN * p.cH * p.cW * p.cCin * 4 < (1LL << 31), CAPMI_ERANGE);
  } else {
    CAPMI_REQUIRE(p.lda % 4 == 0 && p.lda >= p.K && p.a_r1 <= 0, CAPMI_EALIGN);
    CAPMI_REQUIRE((long long)p.M * p.lda * 4 < (1LL << 31), CAPMI_ERANGE);
  }
  bn = (tile == CAPMI_TILE_128x64 || tile == CAPMI_TILE_64 || (tile == CAPMI_TILE_AUTO && p.N <= 64)) ? 64 : 128;
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  a.p[0] = p;
  a.tiles_m[0] = (int)cdiv(p.M, 128);
  a.tiles_n[0] = (int)cdiv(p.N, bn);
  a.plain_epi = plain_epilogue(p, bn);
  total = (long long)a.tiles_m[0] * a.tiles_n[0];
  a.tiles_begin[1] = (int)total;
  const long long slots = sk_cus();
  const int nkt = p.K / 32;
  const long long rounds = (total + slots - 1) / slots;
  // (round 3) more than two rounds of tiles: data-parallel -- the hardware's dynamic dispatch beat the hybrid
  // schedule there (layer1 c1: 55 vs 69 us, layer1 3x3: 154 vs 156; CAPMI_SK_OFF A/B on one box)
  // with the family data-parallel (the default), grids under a quarter of the CUs keep stream-K: a few long-k
  // tiles would otherwise run on a few CUs and accumulate the whole k serially (conv grids are >= 100 tiles)
  sk = !sk_off() && (!sk_family_off(1) || total * 4 < slots) && total > 0 && nkt >= 8 && rounds <= 2 &&
       (double)total / (double)(rounds * slots) < 0.9;
  return 0;
}

// CAPMI_X3P_BK=32 forces the one-workgroup-per-CU form (A/B measurements)
bool x3p_force32() {
  static const bool f = [] {
    const char* e = getenv("CAPMI_X3P_BK");
    return e && e[0] == '3';
  }();
  return f;
}

// CAPMI_GEMM_X3P: three-plane A and B (gemm_x3p.hip), 256x128 tiles, 1-2 workgroups per CU
// Two forms: BK = 16 with two workgroups per CU (their DMA waits and barriers interleave) as a
// plain data-parallel grid when there are at least 2 x CUs tiles and they fill >= 70 % of the last
// round; otherwise BK = 32, one workgroup per CU, stream-K when the tile count leaves the chip
// under-filled (l3 c3, 392 tiles: 49 us stream-K vs 102 us as one 2-per-CU round).
int x3p_plan(const capmi_gemm_problem* prob, int amode, int bmode, GemmArgs& a, bool& sk, long long& total,
             int& bk) {
  CAPMI_REQUIRE(prob != nullptr, CAPMI_EINVAL);
  const capmi_gemm_problem& p = *prob;
  CAPMI_REQUIRE(bmode == CAPMI_B_NMAJOR_W && (amode == CAPMI_A_KMAJOR || amode == CAPMI_A_CONV_NHWC), CAPMI_EINVAL);
  CAPMI_REQUIRE(p.A && p.B && p.C && p.M >= 0 && p.N > 0 && p.K > 0 && p.K % 32 == 0 && p.ksplit == 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(!p.in_scale && !p.in_shift && p.a_r1 <= 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(p.stats == nullptr || p.c_r1 <= 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(p.A) && aligned16(p.B) && p.ldb % 8 == 0 && p.ldb >= p.K, CAPMI_EALIGN);
  CAPMI_REQUIRE(3LL * p.N * p.ldb * 2 < (1LL << 31), CAPMI_ERANGE);
  if (amode == CAPMI_A_CONV_NHWC) {
    CAPMI_REQUIRE(p.cCin % 32 == 0 && p.K == p.cKH * p.cKW * p.cCin && p.M == p.cN * p.cHo * p.cWo, CAPMI_EINVAL);
    CAPMI_REQUIRE(3LL * p.cN * p.cH * p.cW * p.cCin * 2 < (1LL << 31), CAPMI_ERANGE);
  } else {
    CAPMI_REQUIRE(p.lda % 8 == 0 && p.lda >= p.K, CAPMI_EALIGN);
    CAPMI_REQUIRE(3LL * p.M * p.lda * 2 < (1LL << 31), CAPMI_ERANGE);
  }
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  a.p[0] = p;
  a.tiles_m[0] = (int)cdiv(p.M, 256);
  a.tiles_n[0] = (int)cdiv(p.N, 128);
  {  // A/B knob: CAPMI_X3P_ORDER=col walks tiles column-major (an XCD's contiguous range shares B)
    static const int col = [] {
      const char* e = getenv("CAPMI_X3P_ORDER");
      return e && e[0] == 'c' ? 1 : 0;
    }();
    a.tile_cols_first = col;
  }
  a.plain_epi = plain_epilogue(p, 128);
  total = (long long)a.tiles_m[0] * a.tiles_n[0];
  a.tiles_begin[1] = (int)total;
  const long long slots2 = 2LL * sk_cus();
  const long long rounds2 = (total + slots2 - 1) / slots2;
  if (!x3p_force32() && total >= slots2 && (double)total / (double)(rounds2 * slots2) >= 0.7) {
    bk = 16;
    sk = false;
    return 0;
  }
  bk = 32;
  const long long slots = sk_cus();
  const int nkt = p.K / 32;
  const long long rounds = (total + slots - 1) / slots;
  sk = !sk_off() && !sk_family_off(2) && total > 0 && nkt >= 8 && (double)total / (double)(rounds * slots) < 0.9;
  return 0;
}

int gemm_x3p(const capmi_gemm_problem* prob, int amode, int bmode, void* workspace, long long ws_bytes,
             hipStream_t s) {
  GemmArgs a;
  bool sk = false;
  long long total = 0;
  int bk = 32;
  const int rc = x3p_plan(prob, amode, bmode, a, sk, total, bk);
  if (rc) return rc;
  if (prob->M == 0) return 0;
  if (!sk || workspace == nullptr) return gemm_x3p_launch(a, amode, bk, (int)total, s);
  CAPMI_REQUIRE(aligned16(workspace), CAPMI_EINVAL);
  CAPMI_REQUIRE(ws_bytes >= capmi_gemm_workspace_bytes(), CAPMI_ERANGE);
  const int cus = cu_count();
  const long long slots = sk_cus();
  a.sk_nkt = prob->K / bk;  // k-tiles of the x3p kernel
  a.sk_dp_tiles = sk_hybrid() && total >= 2 * slots ? (int)((total / slots - 1) * slots) : 0;
  a.sk_units = (total - a.sk_dp_tiles) * a.sk_nkt;
  a.sk_workers = (int)std::min<long long>(slots, a.sk_units);
  a.sk_groups = sk_xcd_groups() && a.sk_workers % 8 == 0 && total >= 64 ? 8 : 1;
  a.sk_flags = static_cast<int*>(workspace);
  a.sk_part = reinterpret_cast<float*>(static_cast<char*>(workspace) + sk_flag_bytes(cus));
  return gemm_x3p_launch(a, amode, bk, a.sk_workers, s);
}

// CAPMI_GEMM_X3D: fp32 A (+ BN prologue for convs) split in-kernel x three-plane B in the x3p k order
// (gemm_x3p.hip, ASPLIT): 256x128 tiles, 512 threads, k-tiles of 32, one workgroup per CU, stream-K
// when the tiles under-fill the chip
int x3d_plan(const capmi_gemm_problem* prob, int amode, int bmode, GemmArgs& a, bool& sk, long long& total) {
  CAPMI_REQUIRE(prob != nullptr, CAPMI_EINVAL);
  const capmi_gemm_problem& p = *prob;
  CAPMI_REQUIRE(bmode == CAPMI_B_NMAJOR_W && (amode == CAPMI_A_KMAJOR || amode == CAPMI_A_CONV_NHWC), CAPMI_EINVAL);
  CAPMI_REQUIRE(p.A && p.B && p.C && p.M >= 0 && p.N > 0 && p.K > 0 && p.K % 32 == 0 && p.ksplit == 1, CAPMI_EINVAL);
  // dense rows take the prologue when k is the channel (a 1x1 conv's input: lda == K)
  CAPMI_REQUIRE(amode == CAPMI_A_CONV_NHWC || (!p.in_scale && !p.in_shift) || p.lda == p.K, CAPMI_EINVAL);
  CAPMI_REQUIRE((p.in_scale == nullptr) == (p.in_shift == nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE(p.a_r1 <= 0 && (p.stats == nullptr || p.c_r1 <= 0), CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(p.A) && aligned16(p.B) && p.ldb % 8 == 0 && p.ldb >= p.K, CAPMI_EALIGN);
  CAPMI_REQUIRE(p.in_scale == nullptr || (aligned16(p.in_scale) && aligned16(p.in_shift)), CAPMI_EALIGN);
  CAPMI_REQUIRE(3LL * p.N * p.ldb * 2 < (1LL << 31), CAPMI_ERANGE);
  if (amode == CAPMI_A_CONV_NHWC) {
    CAPMI_REQUIRE(p.cCin % 32 == 0 && p.K == p.cKH * p.cKW * p.cCin && p.M == p.cN * p.cHo * p.cWo, CAPMI_EINVAL);
    CAPMI_REQUIRE((long long)p.cN * p.cH * p.cW * p.cCin * 4 < (1LL << 31), CAPMI_ERANGE);
  } else {
    CAPMI_REQUIRE(p.lda % 4 == 0 && p.lda >= p.K, CAPMI_EALIGN);
    CAPMI_REQUIRE((long long)p.M * p.lda * 4 < (1LL << 31), CAPMI_ERANGE);
  }
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  a.p[0] = p;
  a.tiles_m[0] = (int)cdiv(p.M, 256);
  a.tiles_n[0] = (int)cdiv(p.N, 128);
  a.plain_epi = plain_epilogue(p, 128);
  // the two-deep A pipeline (round 4, per-conv A/B at batch 64, one box): 4-9 % faster without the BN
  // prologue and on the conv-mode prologue above layer4's 3136 rows; 1-5 % slower on the dense-row prologue
  // (layer2/3 c3) and layer4's 3x3 -- those keep the one-deep loop. CAPMI_X3D_PIPE=0 / 1: off / on everywhere
  {
    static const int force = [] {
      const char* e = getenv("CAPMI_X3D_PIPE");
      return e ? atoi(e) : -1;
    }();
    const bool pro = p.in_scale != nullptr;
    a.x3d_pipe = force >= 0 ? force : (!pro || (amode == CAPMI_A_CONV_NHWC && p.M > 3136)) ? 1 : 0;
  }
  total = (long long)a.tiles_m[0] * a.tiles_n[0];
  a.tiles_begin[1] = (int)total;
  const long long slots = sk_cus();
  const int nkt = p.K / 32;
  const long long rounds = (total + slots - 1) / slots;
  sk = !sk_off() && !sk_family_off(4) && total > 0 && nkt >= 8 && (double)total / (double)(rounds * slots) < 0.9;
  // C = A.B + beta C (the fine-tune 1x1 data gradients accumulating into the block input's gradient): the
  // data-parallel form, whose epilogue loads each column block of C ahead of its stores (the stream-K forms sit
  // at the register cap and keep the interleaved load / store); CAPMI_X3D_BETA_SK=1 keeps stream-K (A/B)
  {
    static const bool beta_sk = [] {
      const char* e = getenv("CAPMI_X3D_BETA_SK");
      return e && e[0] == '1';
    }();
    if (a.plain_epi == 2 && !beta_sk) sk = false;
  }
  return 0;
}

int gemm_x3d(const capmi_gemm_problem* prob, int amode, int bmode, void* workspace, long long ws_bytes,
             hipStream_t s) {
  GemmArgs a;
  bool sk = false;
  long long total = 0;
  const int rc = x3d_plan(prob, amode, bmode, a, sk, total);
  if (rc) return rc;
  if (prob->M == 0) return 0;
  if (!sk || workspace == nullptr) return gemm_x3d_launch(a, amode, (int)total, s);
  CAPMI_REQUIRE(aligned16(workspace), CAPMI_EINVAL);
  CAPMI_REQUIRE(ws_bytes >= capmi_gemm_workspace_bytes(), CAPMI_ERANGE);
  const int cus = cu_count();
  const long long slots = sk_cus();
  a.sk_nkt = prob->K / 32;
  a.sk_dp_tiles = sk_hybrid() && total >= 2 * slots ? (int)((total / slots - 1) * slots) : 0;
  a.sk_units = (total - a.sk_dp_tiles) * a.sk_nkt;
  a.sk_workers = (int)std::min<long long>(slots, a.sk_units);
  a.sk_groups = sk_xcd_groups() && a.sk_workers % 8 == 0 && total >= 64 ? 8 : 1;
  a.sk_flags = static_cast<int*>(workspace);
  a.sk_part = reinterpret_cast<float*>(static_cast<char*>(workspace) + sk_flag_bytes(cus));
  return gemm_x3d_launch(a, amode, a.sk_workers, s);
}

// CAPMI_GEMM_X3W (gemm_x3w.hip): conv weight gradient dW = dY^T . im2col(X), both operands fp32 k rows (pixels),
// split in-kernel; 256 x 128 tiles, one workgroup per CU, the k range split S ways so that tiles x S fills the
// CUs once (S partial slabs in the workspace after the stream-K flags, summed by capmi_splitk_reduce's kernel)
int x3w_plan(const capmi_gemm_problem* prob, int amode, int bmode, long long ws_floats, GemmArgs& a, int& S,
             long long& tiles) {
  CAPMI_REQUIRE(prob != nullptr, CAPMI_EINVAL);
  const capmi_gemm_problem& p = *prob;
  CAPMI_REQUIRE(amode == CAPMI_A_MMAJOR && (bmode == CAPMI_B_KROWS || bmode == CAPMI_B_CONV_NHWC), CAPMI_EINVAL);
  // K = 0 is refused: the kernel would leave C untouched where C = beta C is the contract
  CAPMI_REQUIRE(p.A && p.B && p.C && p.M > 0 && p.N > 0 && p.K > 0 && p.ksplit == 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(!p.bias && !p.bias2 && !p.relu && !p.stats && p.a_r1 <= 0 && p.c_r1 <= 0, CAPMI_EINVAL);
  CAPMI_REQUIRE((p.in_scale == nullptr) == (p.in_shift == nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE(p.M % 4 == 0 && p.N % 4 == 0 && p.lda >= p.M && p.lda % 4 == 0 && p.ldc >= p.N, CAPMI_EALIGN);
  CAPMI_REQUIRE(aligned16(p.A) && aligned16(p.B), CAPMI_EALIGN);
  CAPMI_REQUIRE(p.in_scale == nullptr || (aligned16(p.in_scale) && aligned16(p.in_shift)), CAPMI_EALIGN);
  CAPMI_REQUIRE((long long)p.K * p.lda * 4 < (1LL << 31), CAPMI_ERANGE);
  if (bmode == CAPMI_B_CONV_NHWC) {
    CAPMI_REQUIRE(p.cCin % 4 == 0 && p.N == p.cKH * p.cKW * p.cCin && p.K == p.cN * p.cHo * p.cWo, CAPMI_EINVAL);
    CAPMI_REQUIRE((long long)p.cN * p.cH * p.cW * p.cCin * 4 < (1LL << 31), CAPMI_ERANGE);
    // the kernel advances each pixel walk by a 32-pixel k-tile with at most two wraps of the output row
    CAPMI_REQUIRE(p.cWo > 0 && p.cHo > 0 && 32 / p.cWo + 1 < 2 * p.cHo, CAPMI_ERANGE);
  } else {
    CAPMI_REQUIRE(p.ldb % 4 == 0 && p.ldb >= p.N, CAPMI_EALIGN);
    CAPMI_REQUIRE((long long)p.K * p.ldb * 4 < (1LL << 31), CAPMI_ERANGE);
  }
  memset(&a, 0, sizeof(a));
  a.nprob = 1;
  a.p[0] = p;
  a.tiles_m[0] = (int)cdiv(p.M, 256);
  a.tiles_n[0] = (int)cdiv(p.N, 128);
  a.plain_epi = plain_epilogue(p, 128);
  tiles = (long long)a.tiles_m[0] * a.tiles_n[0];
  a.tiles_begin[1] = (int)tiles;
  const long long nkt = std::max<long long>(1, (p.K + 31) / 32);
  // k-splits: one round of workgroups over the CUs, at least 4 k-tiles each, slabs within the workspace;
  // a k-split sums in fp32 partials, so the host requires alpha 1 / beta 0 for it (the weight gradients)
  const long long slab = (long long)p.M * a.tiles_n[0] * 128;
  long long s = std::max<long long>(1, std::min<long long>(sk_cus() / tiles, nkt / 4));
  s = std::min<long long>(s, ws_floats / slab);
  if (!(p.alpha == 1.f && p.beta == 0.f && p.alpha_ptr == nullptr)) s = 1;
  s = std::max<long long>(s, 1);
  const long long kc = (nkt + s - 1) / s;
  a.kchunk[0] = (int)kc;
  S = (int)((nkt + kc - 1) / kc);
  return 0;
}

int gemm_x3w(const capmi_gemm_problem* prob, int amode, int bmode, void* workspace, long long ws_bytes, hipStream_t s,
             int terms) {
  const int cus = cu_count();
  const long long part_floats =
      workspace != nullptr && ws_bytes > sk_flag_bytes(cus) ? (ws_bytes - sk_flag_bytes(cus)) / 4 : 0;
  GemmArgs a;
  int S = 1;
  long long tiles = 0;
  const int rc = x3w_plan(prob, amode, bmode, part_floats, a, S, tiles);
  if (rc) return rc;
  CAPMI_REQUIRE(workspace == nullptr || aligned16(workspace), CAPMI_EINVAL);
  if (S > 1) a.sk_part = reinterpret_cast<float*>(static_cast<char*>(workspace) + sk_flag_bytes(cus));
  int e = gemm_x3w_launch(a, bmode, (int)(tiles * S), s, terms);
  if (e || S == 1) return e;
  const int ldp = a.tiles_n[0] * 128;
  return capmi_splitk_reduce(a.sk_part, S, (long long)prob->M * ldp, prob->M, prob->N, ldp, nullptr, prob->C,
                             prob->ldc, s);
}

// CAPMI_GEMM_X3S (gemm_x3s.hip): K = 64, N in {64, 128, 256}, dense rows or a 1x1 / stride-1 conv input
// (optional prologue), store-only epilogue; grid = two persistent workgroups per CU over 64-row tiles
int x3s_plan(const capmi_gemm_problem* prob, int amode, int bmode, long long& lda, int& tiles, int& grid) {
  CAPMI_REQUIRE(prob != nullptr, CAPMI_EINVAL);
  const capmi_gemm_problem& p = *prob;
  CAPMI_REQUIRE(bmode == CAPMI_B_NMAJOR_W && (amode == CAPMI_A_KMAJOR || amode == CAPMI_A_CONV_NHWC), CAPMI_EINVAL);
  CAPMI_REQUIRE(p.A && p.B && p.C && p.M >= 0 && p.K == 64 && (p.N == 64 || p.N == 128 || p.N == 256), CAPMI_EINVAL);
  // the store-only epilogue is x3s's only form (independent of the CAPMI_X3_PLAIN_EPI A/B switch)
  CAPMI_REQUIRE(p.alpha == 1.f && p.alpha_ptr == nullptr && p.bias == nullptr && p.bias2 == nullptr && p.beta == 0.f &&
                    !p.relu && p.c_r1 <= 0 && p.ksplit == 1 && p.ldc >= p.N && (long long)p.M * p.ldc * 4 < (1LL << 31),
                CAPMI_EINVAL);
  CAPMI_REQUIRE(p.a_r1 <= 0 && (p.in_scale == nullptr) == (p.in_shift == nullptr), CAPMI_EINVAL);
  if (amode == CAPMI_A_CONV_NHWC) {
    CAPMI_REQUIRE(p.cKH == 1 && p.cKW == 1 && p.cStride == 1 && p.cPad == 0 && p.cCin == 64 && p.cHo == p.cH &&
                      p.cWo == p.cW && p.M == p.cN * p.cHo * p.cWo,
                  CAPMI_EINVAL);
    lda = p.cCin;
  } else {
    CAPMI_REQUIRE(p.in_scale == nullptr, CAPMI_EINVAL);
    lda = p.lda;
  }
  CAPMI_REQUIRE(aligned16(p.A) && aligned16(p.B) && lda % 4 == 0 && lda >= 64 && p.ldb % 8 == 0 && p.ldb >= 64,
                CAPMI_EALIGN);
  CAPMI_REQUIRE(p.in_scale == nullptr || (aligned16(p.in_scale) && aligned16(p.in_shift)), CAPMI_EALIGN);
  CAPMI_REQUIRE((reinterpret_cast<uintptr_t>(p.stats) & 7u) == 0, CAPMI_EALIGN);
  CAPMI_REQUIRE((long long)p.M * lda * 4 < (1LL << 31) && 3LL * p.N * p.ldb * 2 < (1LL << 31), CAPMI_ERANGE);
  tiles = (int)cdiv(p.M, 64);
  grid = (int)std::max<long long>(1, std::min<long long>(tiles, 2LL * cu_count()));
  return 0;
}

// CAPMI_GEMM_X3C (gemm_x3c.hip, round 4): the direct 3x3 conv for short channel axes (layer1)
int x3c_plan(const capmi_gemm_problem* prob, int amode, int bmode, int& tiles) {
  CAPMI_REQUIRE(prob != nullptr, CAPMI_EINVAL);
  const capmi_gemm_problem& p = *prob;
  CAPMI_REQUIRE(amode == CAPMI_A_CONV_NHWC && bmode == CAPMI_B_NMAJOR_W, CAPMI_EINVAL);
  CAPMI_REQUIRE(p.A && p.B && p.C && p.M >= 0 && p.N == 64 && p.ksplit == 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(p.cKH == 3 && p.cKW == 3 && p.cStride == 1 && p.cPad == 1 && p.cHo == p.cH && p.cWo == p.cW &&
                    p.cCin % 32 == 0 && p.K == 9 * p.cCin && p.M == p.cN * p.cH * p.cW &&
                    p.cW <= gemm_x3c_max_width(),
                CAPMI_EINVAL);
  CAPMI_REQUIRE(p.alpha == 1.f && p.alpha_ptr == nullptr && p.bias == nullptr && p.bias2 == nullptr && p.beta == 0.f &&
                    !p.relu && p.c_r1 <= 0 && p.a_r1 <= 0 && p.ldc >= p.N && (long long)p.M * p.ldc * 4 < (1LL << 31),
                CAPMI_EINVAL);
  CAPMI_REQUIRE((p.in_scale == nullptr) == (p.in_shift == nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(p.A) && aligned16(p.B) && p.ldb == p.K, CAPMI_EALIGN);
  CAPMI_REQUIRE(p.in_scale == nullptr || (aligned16(p.in_scale) && aligned16(p.in_shift)), CAPMI_EALIGN);
  CAPMI_REQUIRE((reinterpret_cast<uintptr_t>(p.stats) & 7u) == 0, CAPMI_EALIGN);
  CAPMI_REQUIRE((long long)p.cN * p.cH * p.cW * p.cCin * 4 < (1LL << 31) && 3LL * p.N * p.ldb * 2 < (1LL << 31),
                CAPMI_ERANGE);
  CAPMI_REQUIRE(gemm_x3c_band_fits(p), CAPMI_EINVAL);  // (e.g. many 1-row images per tile)
  tiles = (int)cdiv(p.M, 256);
  return 0;
}

int gemm_x3c(const capmi_gemm_problem* prob, int amode, int bmode, hipStream_t s) {
  int tiles = 0;
  const int rc = x3c_plan(prob, amode, bmode, tiles);
  if (rc) return rc;
  if (prob->M == 0) return 0;
  return gemm_x3c_launch(*prob, tiles, s);
}

int gemm_x3s(const capmi_gemm_problem* prob, int amode, int bmode, hipStream_t s) {
  long long lda = 0;
  int tiles = 0, grid = 0;
  const int rc = x3s_plan(prob, amode, bmode, lda, tiles, grid);
  if (rc) return rc;
  if (prob->M == 0) return 0;
  return gemm_x3s_launch(*prob, lda, tiles, grid, s);
}

int gemm_x3(const capmi_gemm_problem* prob, int amode, int bmode, int tile, void* workspace, long long ws_bytes,
            hipStream_t s) {
  GemmArgs a;
  int bn = 128;
  bool sk = false;
  long long total = 0;
  const int rc = x3_plan(prob, amode, bmode, tile, a, bn, sk, total);
  if (rc) return rc;
  if (prob->M == 0) return 0;
  if (!sk || workspace == nullptr) return gemm_x3_launch(a, amode, bn, (int)total, s);
  CAPMI_REQUIRE(aligned16(workspace), CAPMI_EINVAL);
  CAPMI_REQUIRE(ws_bytes >= capmi_gemm_workspace_bytes(), CAPMI_ERANGE);
  const int cus = cu_count();
  const long long slots = sk_cus();
  a.sk_nkt = prob->K / 32;
  a.sk_dp_tiles = sk_hybrid() && total >= 2 * slots ? (int)((total / slots - 1) * slots) : 0;
  a.sk_units = (total - a.sk_dp_tiles) * a.sk_nkt;
  a.sk_workers = (int)std::min<long long>(slots, a.sk_units);
  a.sk_groups = sk_xcd_groups() && a.sk_workers % 8 == 0 && total >= 64 ? 8 : 1;
  a.sk_flags = static_cast<int*>(workspace);
  a.sk_part = reinterpret_cast<float*>(static_cast<char*>(workspace) + sk_flag_bytes(cus));
  return gemm_x3_launch(a, amode, bn, a.sk_workers, s);
}
}  // namespace

extern "C" int capmi_gemm_sk_ex(const capmi_gemm_problem* prob, int amode, int bmode, int tile, int flags,
                                void* workspace, long long ws_bytes, void* stream) {
  GemmPlan g;
  bool sk = false;
  if (flags == CAPMI_GEMM_BF16_IO) return gemm_bf16_io(prob, amode, bmode, tile, workspace, ws_bytes, as_stream(stream));
  if (flags == CAPMI_GEMM_X3) return gemm_x3(prob, amode, bmode, tile, workspace, ws_bytes, as_stream(stream));
  if (flags == CAPMI_GEMM_X3P) return gemm_x3p(prob, amode, bmode, workspace, ws_bytes, as_stream(stream));
  if (flags == CAPMI_GEMM_X3D) return gemm_x3d(prob, amode, bmode, workspace, ws_bytes, as_stream(stream));
  if (flags == CAPMI_GEMM_X3S) return gemm_x3s(prob, amode, bmode, as_stream(stream));
  if (flags == CAPMI_GEMM_X3W) return gemm_x3w(prob, amode, bmode, workspace, ws_bytes, as_stream(stream), 3);
  if (flags == (CAPMI_GEMM_X3W | CAPMI_GEMM_BF16))  // (round 6, ABI 26) one bf16 term per operand: gemm_w16_kernel
    return gemm_x3w(prob, amode, bmode, workspace, ws_bytes, as_stream(stream), 1);
  if (flags == CAPMI_GEMM_X3C) return gemm_x3c(prob, amode, bmode, as_stream(stream));
  int terms = flag_terms(flags);
  CAPMI_REQUIRE(terms >= 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(terms_mode_ok(terms, amode, bmode), CAPMI_EINVAL);
  int rc = sk_decide(prob, amode, bmode, tile, terms, g, sk);
  if (rc) return rc;
  if (terms > 0 && !(g.nt_ok && g.nt == 256 && (prob->in_scale == nullptr || amode == CAPMI_A_CONV_NHWC || bmode == CAPMI_B_CONV_NHWC))) {
    // shapes the split forms do not cover (unaligned / generic-kernel problems): the fp32 kernel
    terms = 0;
    rc = sk_decide(prob, amode, bmode, tile, 0, g, sk);
    if (rc) return rc;
  }
  hipStream_t s = as_stream(stream);
  if (!sk) {
    if (g.total == 0) return 0;
    return terms ? gemm_nt_launch(g.a, amode, bmode, g.bm, g.bn, (int)g.total, s, terms)
                 : gemm_launch_dp(g, amode, bmode, s);
  }
  CAPMI_REQUIRE(workspace != nullptr && aligned16(workspace), CAPMI_EINVAL);
  CAPMI_REQUIRE(ws_bytes >= capmi_gemm_workspace_bytes(), CAPMI_ERANGE);
  const int cus = cu_count();
  const long long slots = (long long)sk_cus() * (g.nt == 512 ? 1 : gemm_nt_wg_per_cu(g.bm, g.bn, terms));
  GemmArgs& a = g.a;
  a.sk_nkt = (prob->K + 31) / 32;
  // hybrid: with more than two rounds of tiles, all but the last 1-2 rounds' worth run whole
  a.sk_dp_tiles = sk_hybrid() && g.total >= 2 * slots ? (int)((g.total / slots - 1) * slots) : 0;
  a.sk_units = (g.total - a.sk_dp_tiles) * a.sk_nkt;
  a.sk_workers = (int)std::min<long long>(slots, a.sk_units);
  a.sk_groups = sk_xcd_groups() && a.sk_workers % 8 == 0 && g.total >= 64 ? 8 : 1;
  a.sk_flags = static_cast<int*>(workspace);
  a.sk_part = reinterpret_cast<float*>(static_cast<char*>(workspace) + sk_flag_bytes(cus));
  return gemm_nt_launch(a, amode, bmode, g.bm, g.bn, a.sk_workers, s, terms, g.nt);
}

extern "C" int capmi_gemm_sk(const capmi_gemm_problem* prob, int amode, int bmode, int tile,
                             void* workspace, long long ws_bytes, void* stream) {
  return capmi_gemm_sk_ex(prob, amode, bmode, tile, 0, workspace, ws_bytes, stream);
}

// ------------------------------------------------------------------------------------
// split-K slab reduction and column sums (bias gradients)
// ------------------------------------------------------------------------------------
__global__ void splitk_reduce_kernel(const float* __restrict__ in, int S, long long slab, int rows,
                                     int cols, long long ld_in, const float* __restrict__ bias,
                                     float* __restrict__ out, long long ld_out) {
  const long long n = (long long)rows * cols;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / cols), c = (int)(i - (long long)r * cols);
    const float* p = in + r * ld_in + c;
    out[r * ld_out + c] = slab_sum(p, S, slab, bias ? bias[c] : 0.f);
  }
}

extern "C" int capmi_splitk_reduce(const float* in, int S, long long slab, int rows, int cols,
                                   long long ld_in, const float* bias, float* out,
                                   long long ld_out, void* stream) {
  CAPMI_REQUIRE(S >= 1 && rows >= 0 && cols >= 0, CAPMI_EINVAL);
  const long long n = (long long)rows * cols;
  if (n == 0) return 0;
  const unsigned blocks = (unsigned)std::min<long long>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), in, S,
                     slab, rows, cols, ld_in, bias, out, ld_out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// stage 1: work[g][c] = sum of rows [g*R, g*R+R) (64 columns x 4 row-lanes per WG, <= 64 groups);
// stage 2: out[c] = scale * sum_g work[g][c]
__global__ void colsum_stage1(const float* __restrict__ in, int rows, int cols, long long ld, int R,
                              float* __restrict__ work) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * R, r1 = min(rows, r0 + R);
  float s = 0.f;
  if (c < cols)
    for (int r = r0 + rl; r < r1; r += 4) s += in[(long long)r * ld + c];
  red[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && c < cols)
    work[(long long)blockIdx.y * cols + c] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

__global__ void colsum_stage2(const float* __restrict__ work, int nb, int cols, float scale,
                              float* __restrict__ out, int accumulate) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cols) return;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += work[(long long)b * cols + c];
  s *= scale;
  out[c] = accumulate ? out[c] + s : s;
}

extern "C" int capmi_colsum(const float* in, int rows, int cols, long long ld, float scale,
                            float* work, float* out, int accumulate, void* stream) {
  CAPMI_REQUIRE(rows >= 0 && cols >= 0, CAPMI_EINVAL);
  if (cols == 0) return 0;
  int R = std::max(64, (rows + CAPMI_COLSUM_GROUPS - 1) / CAPMI_COLSUM_GROUPS);
  R = (R + 3) & ~3;
  const int nb = rows > 0 ? (rows + R - 1) / R : 0;
  hipStream_t s = as_stream(stream);
  if (nb > 0)
    hipLaunchKernelGGL(colsum_stage1, dim3(cdiv(cols, 64), nb), dim3(256), 0, s, in, rows, cols, ld, R,
                       work);
  hipLaunchKernelGGL(colsum_stage2, dim3(cdiv(cols, 256)), dim3(256), 0, s, work, nb, cols, scale,
                     out, accumulate);
  CAPMI_LAUNCH_CHECK();
  return 0;
}
