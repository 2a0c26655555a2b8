// Backward of the fine-tuned ResNet-101 stages (EncoderAttention.fine_tune, models/encoder.py:112-121:
// layer2, layer3, layer4 get requires_grad; BASELINE config 4). The convolutions' data and weight
// gradients run on the implicit-GEMM kernels (gemm_nt.hip: dgrad = NHWC conv of dY with the
// flipped, transposed weights; wgrad = dY^T x implicit-im2col(X), BMODE 2). This file holds the
// memory-bound rest, all NHWC with float4 I/O:
//   * weight re-layouts for dgrad / gradient unpacking,
//   * zero-upsampling of a stride-2 conv's output gradient (the transposed conv becomes a
//     stride-1 conv),
//   * BatchNorm2d(train) backward split into a per-channel reduction (which also yields the
//     gamma/beta gradients) and an element-wise apply, with the ReLU mask recomputed from the
//     saved pre-BN conv output (in-block BN+ReLU) or from the saved block output (bottleneck tail),
//   * AdaptiveAvgPool2d backward (models/encoder.py:92,108).
// BN backward (autograd of F.batch_norm(training=True)): with x^ = (y - mean) * invstd over the
// N = rows samples of a channel, dz the gradient at the BN output,
//   dbeta = sum dz, dgamma = sum dz * x^,  dy = gamma*invstd * (dz - dbeta/N - x^ * dgamma/N).
#include "common.h"

// ---------------------------------------------------------------------------------
// weights
// ---------------------------------------------------------------------------------
// out[ci][kh][kw][co] = w[co][ci][KH-1-kh][KW-1-kw]: the B operand (W[N = Cin][K = (kh, kw, co)])
// of the data-gradient conv dX = conv(dY, flip(W)^T)
__global__ void conv_weight_pack_dgrad_kernel(const float* __restrict__ w, int Cout, int Cin, int KH, int KW,
                                              float* __restrict__ out) {
  const long long n = (long long)Cout * Cin * KH * KW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i % Cout);
    long long r = i / Cout;
    const int kw = (int)(r % KW);
    r /= KW;
    const int kh = (int)(r % KH);
    const int ci = (int)(r / KH);
    out[i] = w[(((long long)co * Cin + ci) * KH + (KH - 1 - kh)) * KW + (KW - 1 - kw)];
  }
}

extern "C" int capmi_conv_weight_pack_dgrad(const float* w, int Cout, int Cin, int KH, int KW, float* out,
                                            void* stream) {
  CAPMI_REQUIRE(w && out && Cout > 0 && Cin > 0 && KH > 0 && KW > 0, CAPMI_EINVAL);
  const long long n = (long long)Cout * Cin * KH * KW;
  hipLaunchKernelGGL(conv_weight_pack_dgrad_kernel, dim3(std::min<long long>(cdiv(n, 256), 8192)), dim3(256),
                     0, as_stream(stream), w, Cout, Cin, KH, KW, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// Sub-pixel data gradient of a 3x3 / stride-2 / pad-1 conv: input pixel (2i+ph, 2j+pw) receives
// dY[i+th][j+tw] * W[kh(th)][kw(tw)] with kh = 1 for ph = 0 (one tap) and kh = 2, 0 for th = 0, 1
// when ph = 1 (two taps); same along w. out[ci][th][tw][co] = w[co][ci][kh(th)][kw(tw)], the B
// operand of the parity class's (1|2)x(1|2) stride-1 pad-0 conv over dY.
__global__ void conv_weight_pack_dgrad_s2_kernel(const float* __restrict__ w, int Cout, int Cin, int ph, int pw,
                                                 float* __restrict__ out) {
  const int TH = ph + 1, TW = pw + 1;
  const long long n = (long long)Cout * Cin * TH * TW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(i % Cout);
    long long r = i / Cout;
    const int tw = (int)(r % TW);
    r /= TW;
    const int th = (int)(r % TH);
    const int ci = (int)(r / TH);
    const int kh = ph ? 2 - 2 * th : 1, kw = pw ? 2 - 2 * tw : 1;
    out[i] = w[(((long long)co * Cin + ci) * 3 + kh) * 3 + kw];
  }
}

extern "C" int capmi_conv_weight_pack_dgrad_s2(const float* w, int Cout, int Cin, int ph, int pw, float* out,
                                               void* stream) {
  CAPMI_REQUIRE(w && out && Cout > 0 && Cin > 0 && (ph == 0 || ph == 1) && (pw == 0 || pw == 1), CAPMI_EINVAL);
  const long long n = (long long)Cout * Cin * (ph + 1) * (pw + 1);
  hipLaunchKernelGGL(conv_weight_pack_dgrad_s2_kernel, dim3(std::min<long long>(cdiv(n, 256), 8192)), dim3(256),
                     0, as_stream(stream), w, Cout, Cin, ph, pw, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// The two packs above, re-ordered to the x3p conv k order and split, in one pass: the B operand of
// the x3d data gradient (CAPMI_GEMM_X3D), three bf16 planes out[3][Cin][T*Cout] (T = the taps of the
// dgrad conv) with k = ((co / 32) * T + tap) * 32 + co % 32 (gemm_x3p.hip: the taps of one
// 32-channel slice consecutive) and the exact three-term split of split3_bf16. ph < 0: the full
// flipped KHxKW kernel (stride 1); ph, pw in {0, 1}: the sub-pixel class of a 3x3 / stride-2 conv.
__global__ void conv_weight_pack_dgrad_x3_kernel(const float* __restrict__ w, int Cout, int Cin, int KH, int KW,
                                                 int ph, int pw, __bf16* __restrict__ out) {
  const int TH = ph < 0 ? KH : ph + 1, TW = ph < 0 ? KW : pw + 1, T = TH * TW;
  const long long K = (long long)T * Cout, n = (long long)Cin * K;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int ci = (int)(i / K);
    const int j = (int)(i - (long long)ci * K);
    const int slice = j / (T * 32), rem = j - slice * T * 32;
    const int tap = rem >> 5, co = slice * 32 + (rem & 31);
    const int th = tap / TW, tw = tap - th * TW;
    int kh, kw;
    if (ph < 0) {
      kh = KH - 1 - th;
      kw = KW - 1 - tw;
    } else {
      kh = ph ? 2 - 2 * th : 1;
      kw = pw ? 2 - 2 * tw : 1;
    }
    const float x = w[(((long long)co * Cin + ci) * KH + kh) * KW + kw];
    const __bf16 h0 = (__bf16)x;
    const float r1 = x - (float)h0;
    const __bf16 h1 = (__bf16)r1;
    out[i] = h0;
    out[n + i] = h1;
    out[2 * n + i] = (__bf16)(r1 - (float)h1);
  }
}

extern "C" int capmi_conv_weight_pack_dgrad_x3(const float* w, int Cout, int Cin, int KH, int KW, int ph, int pw,
                                               void* out, void* stream) {
  CAPMI_REQUIRE(w && out && Cout > 0 && Cin > 0 && KH > 0 && KW > 0 && Cout % 32 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(ph < 0 || (KH == 3 && KW == 3 && (ph == 0 || ph == 1) && (pw == 0 || pw == 1)), CAPMI_EINVAL);
  const long long T = ph < 0 ? (long long)KH * KW : (long long)(ph + 1) * (pw + 1);
  const long long n = T * Cout * Cin;
  CAPMI_REQUIRE(3 * n < (1LL << 31), CAPMI_ERANGE);
  hipLaunchKernelGGL(conv_weight_pack_dgrad_x3_kernel, dim3(std::min<long long>(cdiv(n, 256), 8192)), dim3(256),
                     0, as_stream(stream), w, Cout, Cin, KH, KW, ph, pw, static_cast<__bf16*>(out));
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// Round 5: every trainable conv's three-plane weight operands of a fine-tune step in ONE launch (the forward's
// B planes in the plain [Cout][KH][KW][Cin] or the x3p k order, the data gradients' transposed / flipped planes),
// instead of 2-3 latency-bound launches per conv (split3_bf16 + packs: ~250 launches per step). Block row y =
// job y (read once, uniform); the element map of each mode restates the per-conv kernels above exactly, and the
// split is split3_bf16's (RNE at each step), so the planes are bit-identical to the per-conv path.
__device__ __forceinline__ void wx3_store(__bf16* out, long long n, long long e, float x) {
  const __bf16 h0 = (__bf16)x;
  const float r1 = x - (float)h0;
  const __bf16 h1 = (__bf16)r1;
  out[e] = h0;
  out[n + e] = h1;
  out[2 * n + e] = (__bf16)(r1 - (float)h1);
}

__global__ void __launch_bounds__(256) weight_x3_batch_kernel(const capmi_wx3_job* __restrict__ jobs) {
  const capmi_wx3_job j = jobs[blockIdx.y];
  if (j.mode == CAPMI_WX3_DGRAD_T) {  // 1x1 transpose through LDS: 64 x 64 tiles, both sides row-contiguous
    __shared__ float tile[64][65];
    const int co_n = j.cout, ci_n = j.cin, tco = (co_n + 63) / 64, tci = (ci_n + 63) / 64;
    const long long n = (long long)co_n * ci_n;
    __bf16* __restrict__ out = static_cast<__bf16*>(j.out);
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int t = blockIdx.x; t < tco * tci; t += gridDim.x) {
      const int co0 = (t / tci) * 64, ci0 = (t % tci) * 64;
      __syncthreads();  // (the previous tile's reads are done)
#pragma unroll
      for (int i = 0; i < 16; ++i) {  // rows co0 + ty + 4 i, columns ci0 + tx: coalesced along ci
        const int co = co0 + ty + 4 * i, ci = ci0 + tx;
        tile[ty + 4 * i][tx] = co < co_n && ci < ci_n ? j.w[(long long)co * ci_n + ci] : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 16; ++i) {  // out[ci][co]: coalesced along co
        const int ci = ci0 + ty + 4 * i, co = co0 + tx;
        if (ci < ci_n && co < co_n) wx3_store(out, n, (long long)ci * co_n + co, tile[tx][ty + 4 * i]);
      }
    }
    return;
  }
  const int KH = j.kh, KW = j.kw;
  const int T = j.mode == CAPMI_WX3_DGRAD && j.ph >= 0 ? (j.ph + 1) * (j.pw + 1) : KH * KW;
  const int TW = j.mode == CAPMI_WX3_DGRAD && j.ph >= 0 ? j.pw + 1 : KW;
  const bool dg = j.mode == CAPMI_WX3_DGRAD || j.mode == CAPMI_WX3_DGRAD_T;
  const int R = dg ? j.cin : j.cout;  // rows of the B operand
  const int Kc = T * (dg ? j.cout : j.cin);  // its k extent
  const int n = R * Kc;                      // (< 2^31: the host checks)
  const float* __restrict__ w = j.w;
  __bf16* __restrict__ out = static_cast<__bf16*>(j.out);
  for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {  // 32-bit index math
    const int r = e / Kc;
    const int k = e - r * Kc;
    int co, ci, kh, kw;
    if (j.mode == CAPMI_WX3_FWD) {  // [Cout][KH][KW][Cin] (capmi_conv_weight_pack_pad, Cin >= 4)
      co = (int)r;
      const int tap = k / j.cin;
      ci = k - tap * j.cin;
      kh = tap / KW;
      kw = tap - kh * KW;
    } else if (j.mode == CAPMI_WX3_FWD_X3P) {  // (ci / 32, kh, kw, ci % 32): conv_weight_order_x3p
      co = (int)r;
      const int slice = k / (T * 32), rem = k - slice * T * 32, tap = rem >> 5;
      ci = slice * 32 + (rem & 31);
      kh = tap / KW;
      kw = tap - kh * KW;
    } else if (j.mode == CAPMI_WX3_DGRAD) {  // conv_weight_pack_dgrad_x3_kernel's map
      ci = (int)r;
      const int slice = k / (T * 32), rem = k - slice * T * 32, tap = rem >> 5;
      co = slice * 32 + (rem & 31);
      const int th = tap / TW, tw = tap - th * TW;
      if (j.ph < 0) {
        kh = KH - 1 - th;
        kw = KW - 1 - tw;
      } else {
        kh = j.ph ? 2 - 2 * th : 1;
        kw = j.pw ? 2 - 2 * tw : 1;
      }
    } else {  // CAPMI_WX3_DGRAD_T: 1x1, out[ci][co] = w[co][ci] (capmi_conv_weight_pack_dgrad at 1x1)
      ci = (int)r;
      co = k;
      kh = kw = 0;
    }
    wx3_store(out, n, e, w[(((long long)co * j.cin + ci) * KH + kh) * KW + kw]);
  }
}

extern "C" int capmi_weight_x3_batch(const capmi_wx3_job* jobs, int njobs, long long max_elems, void* stream) {
  CAPMI_REQUIRE(njobs >= 0 && njobs <= 65535 && (njobs == 0 || jobs) && max_elems >= 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(max_elems < (1LL << 31), CAPMI_ERANGE);
  if (njobs == 0 || max_elems == 0) return 0;
  // a grid row per job, sized so the largest job's threads take about 8 elements each (a fixed 64 blocks per
  // row left the 2.4M-element layer4 jobs at ~144 serial elements per thread); rows of smaller jobs end early
  const unsigned bx = (unsigned)std::min<long long>(std::max<long long>(cdiv(max_elems, 256 * 8), 1), 4096);
  hipLaunchKernelGGL(weight_x3_batch_kernel, dim3(bx, njobs), dim3(256), 0, as_stream(stream), jobs);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// out[co][ci][kh][kw] (= nn.Conv2d weight layout) from the GEMM layout g[co][kh][kw][ci]
__global__ void conv_weight_unpack_kernel(const float* __restrict__ g, int Cout, int Cin, int KH, int KW,
                                          float* __restrict__ out) {
  const long long n = (long long)Cout * Cin * KH * KW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int kw = (int)(i % KW);
    long long r = i / KW;
    const int kh = (int)(r % KH);
    r /= KH;
    const int ci = (int)(r % Cin);
    const int co = (int)(r / Cin);
    out[i] = g[(((long long)co * KH + kh) * KW + kw) * Cin + ci];
  }
}

extern "C" int capmi_conv_weight_unpack(const float* packed, int Cout, int Cin, int KH, int KW, float* out,
                                        void* stream) {
  CAPMI_REQUIRE(packed && out && Cout > 0 && Cin > 0 && KH > 0 && KW > 0, CAPMI_EINVAL);
  const long long n = (long long)Cout * Cin * KH * KW;
  hipLaunchKernelGGL(conv_weight_unpack_kernel, dim3(std::min<long long>(cdiv(n, 256), 8192)), dim3(256), 0,
                     as_stream(stream), packed, Cout, Cin, KH, KW, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------
// out (N,H,W,C) = dy (N,Ho,Wo,C) at even (h, w) positions, zero elsewhere
// ---------------------------------------------------------------------------------
__global__ void zero_upsample2_kernel(const float4* __restrict__ dy, int N, int Ho, int Wo, int C4, int H, int W,
                                      float4* __restrict__ out) {
  const long long n = (long long)N * H * W * C4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4);
    long long r = i / C4;
    const int w = (int)(r % W);
    r /= W;
    const int h = (int)(r % H);
    const int img = (int)(r / H);
    float4 v = f4(0.f);
    if (((h | w) & 1) == 0 && (h >> 1) < Ho && (w >> 1) < Wo)
      v = dy[(((long long)img * Ho + (h >> 1)) * Wo + (w >> 1)) * C4 + c];
    out[i] = v;
  }
}

extern "C" int capmi_zero_upsample2_nhwc(const float* dy, int N, int Ho, int Wo, int C, int H, int W, float* out,
                                         void* stream) {
  CAPMI_REQUIRE(dy && out && N > 0 && Ho > 0 && Wo > 0 && C > 0 && C % 4 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(H >= 2 * Ho - 1 && W >= 2 * Wo - 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(dy) && aligned16(out), CAPMI_EALIGN);
  const long long n = (long long)N * H * W * C / 4;
  hipLaunchKernelGGL(zero_upsample2_kernel, dim3(std::min<long long>(cdiv(n, 256), 16384)), dim3(256), 0,
                     as_stream(stream), (const float4*)dy, N, Ho, Wo, C / 4, H, W, (float4*)out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------
// BatchNorm2d(train) backward
// ---------------------------------------------------------------------------------
// dz = d * relu'(.) with the mask of the forward's ReLU:
//   CAPMI_BNB_RELU_Y   : in-block BN + ReLU, mask [fma(y, scale, shift) > 0] (the GEMM prologue's
//                        exact expression, so the mask matches the forward bit for bit);
//   CAPMI_BNB_RELU_OUT : bottleneck tail relu(bn3(y3) + residual), mask [out > 0] of the saved output.
__device__ __forceinline__ float4 bnb_dz(int mode, float4 d, float4 y, const float* __restrict__ msrc,
                                         long long i4, float4 sc, float4 sh) {
  float4 m;
  if (mode == CAPMI_BNB_RELU_OUT) {
    m = reinterpret_cast<const float4*>(msrc)[i4];
  } else {
    m = fma4(y, sc, sh);
  }
  d.x = m.x > 0.f ? d.x : 0.f;
  d.y = m.y > 0.f ? d.y : 0.f;
  d.z = m.z > 0.f ? d.z : 0.f;
  d.w = m.w > 0.f ? d.w : 0.f;
  return d;
}

// stage 1: block (cb, slab): CB float4 channel groups x RL row lanes; partial (sum dz, sum dz*(y-mean))
// per channel of the slab -> part[slab][c][2]
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(int mode, const float* __restrict__ d,
                                                            const float* __restrict__ y,
                                                            const float* __restrict__ msrc,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            const float* __restrict__ mean, long long rows, int C,
                                                            int CB, int rows_per_slab, float* __restrict__ part) {
  __shared__ float4 rs[256], rq[256];
  const int C4 = C / 4, RL = 256 / CB;
  const int cg = threadIdx.x % CB, rl = threadIdx.x / CB;
  const int c4 = blockIdx.x * CB + cg;
  const long long r0 = (long long)blockIdx.y * rows_per_slab;
  const long long r1 = min(rows, r0 + rows_per_slab);
  float4 s = f4(0.f), q = f4(0.f);
  if (c4 < C4) {
    const int c = c4 * 4;
    const float4 sc = *reinterpret_cast<const float4*>(scale + c);
    const float4 sh = *reinterpret_cast<const float4*>(shift + c);
    const float4 mu = *reinterpret_cast<const float4*>(mean + c);
#pragma unroll 4
    for (long long r = r0 + rl; r < r1; r += RL) {
      const long long i4 = r * C4 + c4;
      const float4 yv = reinterpret_cast<const float4*>(y)[i4];
      const float4 dz = bnb_dz(mode, reinterpret_cast<const float4*>(d)[i4], yv, msrc, i4, sc, sh);
      s = s + dz;
      const float4 xc = make_float4(yv.x - mu.x, yv.y - mu.y, yv.z - mu.z, yv.w - mu.w);
      q = fma4(dz, xc, q);
    }
  }
  rs[threadIdx.x] = s;
  rq[threadIdx.x] = q;
  __syncthreads();
  if (rl == 0 && c4 < C4) {
    for (int l = 1; l < RL; ++l) {
      s = s + rs[l * CB + cg];
      q = q + rq[l * CB + cg];
    }
    float* p = part + ((long long)blockIdx.y * C + c4 * 4) * 2;
    *reinterpret_cast<float4*>(p) = make_float4(s.x, q.x, s.y, q.y);
    *reinterpret_cast<float4*>(p + 4) = make_float4(s.z, q.z, s.w, q.w);
  }
}

// stage 2: block of 256 threads = BNB_FIN_CW channels x (256 / BNB_FIN_CW) slab lanes. Each lane
// sums its strided slabs in fp64 (all of its loads independent, so they are in flight together,
// instead of one thread walking up to 256 slabs with one dependent load each: 60 -> a few us per
// call), then a fixed-shape LDS tree adds the lanes: the result is deterministic run to run.
constexpr int BNB_FIN_CW = 16;
__global__ void __launch_bounds__(256) bn_bwd_finalize_kernel(const float* __restrict__ part, int slabs, int C,
                                                              long long count, const float* __restrict__ gamma,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ var, float eps,
                                                              float* dgamma, float* dbeta, int accumulate,
                                                              float* __restrict__ coef) {
  constexpr int SL = 256 / BNB_FIN_CW;
  __shared__ double ls[256], lq[256];
  const int cl = threadIdx.x % BNB_FIN_CW, lane = threadIdx.x / BNB_FIN_CW;
  const int c = blockIdx.x * BNB_FIN_CW + cl;
  double s = 0.0, q = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int k = lane; k < slabs; k += SL) {
      const float2 v = *reinterpret_cast<const float2*>(part + ((long long)k * C + c) * 2);
      s += v.x;
      q += v.y;
    }
  }
  ls[threadIdx.x] = s;
  lq[threadIdx.x] = q;
  __syncthreads();
#pragma unroll
  for (int st = SL / 2; st > 0; st >>= 1) {
    if (lane < st) {
      ls[threadIdx.x] += ls[threadIdx.x + st * BNB_FIN_CW];
      lq[threadIdx.x] += lq[threadIdx.x + st * BNB_FIN_CW];
    }
    __syncthreads();
  }
  if (lane != 0 || c >= C) return;
  s = ls[cl];
  q = lq[cl];
  const double inv = 1.0 / sqrt((double)var[c] + (double)eps);
  const double dg = q * inv, db = s;
  if (dgamma) dgamma[c] = accumulate ? dgamma[c] + (float)dg : (float)dg;
  if (dbeta) dbeta[c] = accumulate ? dbeta[c] + (float)db : (float)db;
  const double n = (double)count;
  const double k1 = (double)gamma[c] * inv;
  coef[c] = (float)k1;                      // gamma * invstd
  coef[C + c] = (float)(k1 * inv * dg / n); // multiplies (y - mean)
  coef[2 * C + c] = (float)(k1 * db / n);   // constant term
  coef[3 * C + c] = mean[c];
}

extern "C" int capmi_bn_bwd_reduce(int mode, const float* d, const float* y, const float* mask_src,
                                   const float* scale, const float* shift, const float* gamma,
                                   const float* save_mean, const float* save_var, float eps, long long rows,
                                   int C, float* dgamma, float* dbeta, int accumulate, float* coef, float* work,
                                   void* stream) {
  CAPMI_REQUIRE(mode == CAPMI_BNB_RELU_Y || mode == CAPMI_BNB_RELU_OUT, CAPMI_EINVAL);
  CAPMI_REQUIRE(d && y && gamma && save_mean && save_var && coef && work && rows > 0 && C > 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(mode != CAPMI_BNB_RELU_OUT || mask_src, CAPMI_EINVAL);
  CAPMI_REQUIRE(mode != CAPMI_BNB_RELU_Y || (scale && shift), CAPMI_EINVAL);
  CAPMI_REQUIRE(C % 4 == 0, CAPMI_ERANGE);
  CAPMI_REQUIRE(aligned16(d) && aligned16(y) && (!mask_src || aligned16(mask_src)) && aligned16(save_mean) &&
                    aligned16(work) && (!scale || (aligned16(scale) && aligned16(shift))),
                CAPMI_EALIGN);
  const int C4 = C / 4;
  const int CB = std::min(64, C4);
  const int gx = (C4 + CB - 1) / CB;
  long long slabs = std::min<long long>(CAPMI_BNB_MAX_SLABS, std::max<long long>(1, 2048 / gx));
  slabs = std::min<long long>(slabs, (rows + 31) / 32);
  const int per = (int)((rows + slabs - 1) / slabs);
  slabs = (rows + per - 1) / per;
  hipStream_t s = as_stream(stream);
  // mode RELU_OUT never reads scale/shift: pass the mean as a harmless valid pointer
  const float* sc = scale ? scale : save_mean;
  const float* sh = shift ? shift : save_mean;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(gx, (unsigned)slabs), dim3(256), 0, s, mode, d, y, mask_src, sc,
                     sh, save_mean, rows, C, CB, per, work);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(cdiv(C, BNB_FIN_CW)), dim3(256), 0, s, work, (int)slabs, C, rows,
                     gamma, save_mean, save_var, eps, dgamma, dbeta, accumulate, coef);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// dy = k1*dz - k2*(y - mean) - k0; dz_out (optional) = dz (the residual branch's gradient)
__global__ void bn_bwd_apply_kernel(int mode, const float4* __restrict__ d, const float4* __restrict__ y,
                                    const float* __restrict__ msrc, const float* __restrict__ scale,
                                    const float* __restrict__ shift, const float* __restrict__ coef, long long n4,
                                    int C4, float4* dy, float4* dz_out) {
  const int C = C4 * 4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const float4 yv = y[i];
    float4 sc = f4(0.f), sh = f4(0.f);
    if (mode == CAPMI_BNB_RELU_Y) {
      sc = *reinterpret_cast<const float4*>(scale + c);
      sh = *reinterpret_cast<const float4*>(shift + c);
    }
    const float4 dz = bnb_dz(mode, d[i], yv, msrc, i, sc, sh);
    const float4 k1 = *reinterpret_cast<const float4*>(coef + c);
    const float4 k2 = *reinterpret_cast<const float4*>(coef + C + c);
    const float4 k0 = *reinterpret_cast<const float4*>(coef + 2 * C + c);
    const float4 mu = *reinterpret_cast<const float4*>(coef + 3 * C + c);
    float4 r;
    r.x = fmaf(k1.x, dz.x, -fmaf(k2.x, yv.x - mu.x, k0.x));
    r.y = fmaf(k1.y, dz.y, -fmaf(k2.y, yv.y - mu.y, k0.y));
    r.z = fmaf(k1.z, dz.z, -fmaf(k2.z, yv.z - mu.z, k0.z));
    r.w = fmaf(k1.w, dz.w, -fmaf(k2.w, yv.w - mu.w, k0.w));
    if (dz_out) dz_out[i] = dz;
    dy[i] = r;
  }
}

extern "C" int capmi_bn_bwd_apply(int mode, const float* d, const float* y, const float* mask_src,
                                  const float* scale, const float* shift, const float* coef, long long rows, int C,
                                  float* dy, float* dz_out, void* stream) {
  CAPMI_REQUIRE(mode == CAPMI_BNB_RELU_Y || mode == CAPMI_BNB_RELU_OUT, CAPMI_EINVAL);
  CAPMI_REQUIRE(d && y && coef && dy && rows >= 0 && C > 0 && C % 4 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(mode != CAPMI_BNB_RELU_OUT || mask_src, CAPMI_EINVAL);
  CAPMI_REQUIRE(mode != CAPMI_BNB_RELU_Y || (scale && shift), CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(d) && aligned16(y) && aligned16(coef) && aligned16(dy) && (!dz_out || aligned16(dz_out)) &&
                    (!mask_src || aligned16(mask_src)) && (!scale || (aligned16(scale) && aligned16(shift))),
                CAPMI_EALIGN);
  const long long n4 = rows * C / 4;
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(std::min<long long>(cdiv(n4, 256), 16384)), dim3(256), 0,
                     as_stream(stream), mode, (const float4*)d, (const float4*)y, mask_src, scale, shift, coef,
                     n4, C / 4, (float4*)dy, (float4*)dz_out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------
// AdaptiveAvgPool2d backward on NHWC: din[n][h][w] = sum over the output cells whose window
// [floor(o*H/OH), ceil((o+1)*H/OH)) contains (h, w) of dout / window area
// ---------------------------------------------------------------------------------
__global__ void adaptive_avgpool_bwd_kernel(const float4* __restrict__ dout, int N, int H, int W, int C4, int OH,
                                            int OW, float4* __restrict__ din) {
  const long long n = (long long)N * H * W * C4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4);
    long long r = i / C4;
    const int w = (int)(r % W);
    r /= W;
    const int h = (int)(r % H);
    const int img = (int)(r / H);
    float4 acc = f4(0.f);
    const int oh_lo = max(0, (h * OH) / H - 1), oh_hi = min(OH - 1, ((h + 1) * OH + H - 1) / H);
    const int ow_lo = max(0, (w * OW) / W - 1), ow_hi = min(OW - 1, ((w + 1) * OW + W - 1) / W);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int h0 = (oh * H) / OH, h1 = ((oh + 1) * H + OH - 1) / OH;
      if (h < h0 || h >= h1) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int w0 = (ow * W) / OW, w1 = ((ow + 1) * W + OW - 1) / OW;
        if (w < w0 || w >= w1) continue;
        const float inv = 1.f / (float)((h1 - h0) * (w1 - w0));
        acc = fma4(dout[(((long long)img * OH + oh) * OW + ow) * C4 + c], f4(inv), acc);
      }
    }
    din[i] = acc;
  }
}

extern "C" int capmi_adaptive_avgpool_bwd_nhwc(const float* dout, int N, int H, int W, int C, int OH, int OW,
                                               float* din, void* stream) {
  CAPMI_REQUIRE(dout && din && N > 0 && H > 0 && W > 0 && OH > 0 && OW > 0 && C > 0 && C % 4 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(dout) && aligned16(din), CAPMI_EALIGN);
  const long long n = (long long)N * H * W * C / 4;
  hipLaunchKernelGGL(adaptive_avgpool_bwd_kernel, dim3(std::min<long long>(cdiv(n, 256), 16384)), dim3(256), 0,
                     as_stream(stream), (const float4*)dout, N, H, W, C / 4, OH, OW, (float4*)din);
  CAPMI_LAUNCH_CHECK();
  return 0;
}
