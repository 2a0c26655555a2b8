// ResNet-101 encoder kernels besides the conv GEMMs (gemm.hip):
// BatchNorm2d(train) finalize, bottleneck tail (BN-apply + residual + ReLU),
// conv1 tail (BN-apply + ReLU + 3x3/2 max-pool), AdaptiveAvgPool2d on NHWC, and the
// one-time conv weight repack. All activations NHWC, all memory-bound, float4 I/O.
//
// Reference: models/encoder.py:88-92 (resnet children()[:-2], AdaptiveAvgPool2d(14,14)),
// :107-110 (forward + permute to NHWC); BN in train mode because of
// models/attention.py:374 (encoder.train()).
#include "common.h"

__global__ void conv_weight_pack_kernel(const float* __restrict__ w, int Cout, int Cin, int KH,
                                        int KW, float* __restrict__ out) {
  const long long n = (long long)Cout * Cin * KH * KW;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    // i indexes the OUTPUT [co][kh][kw][ci]
    const int ci = (int)(i % Cin);
    long long r = i / Cin;
    const int kw = (int)(r % KW);
    r /= KW;
    const int kh = (int)(r % KH);
    const int co = (int)(r / KH);
    out[i] = w[(((long long)co * Cin + ci) * KH + kh) * KW + kw];
  }
}

extern "C" int capmi_conv_weight_pack(const float* w, int Cout, int Cin, int KH, int KW, float* out,
                                      void* stream) {
  CAPMI_REQUIRE(w && out && Cout > 0 && Cin > 0 && KH > 0 && KW > 0, CAPMI_EINVAL);
  const long long n = (long long)Cout * Cin * KH * KW;
  hipLaunchKernelGGL(conv_weight_pack_kernel, dim3(std::min<long long>(cdiv(n, 256), 8192)),
                     dim3(256), 0, as_stream(stream), w, Cout, Cin, KH, KW, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------
// BN finalize, two stages: (1) G slice-groups x 64 channels, fp64 partial sums per group;
// (2) per channel: combine the G partials, mean/var -> scale/shift, running stats.
// ---------------------------------------------------------------------------------
constexpr int BNF_MAXG = 32;

__global__ void bn_stats_stage1(const float* __restrict__ stats, int tiles, int C, int per_g,
                                double* __restrict__ part) {
  __shared__ double rs[4][64], rq[4][64];
  const int cl = threadIdx.x & 63, tl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int t0 = blockIdx.y * per_g, t1 = min(tiles, t0 + per_g);
  double s = 0.0, q = 0.0;
  if (c < C) {
    for (int t = t0 + tl; t < t1; t += 4) {
      const float2 v = *reinterpret_cast<const float2*>(stats + ((long long)t * C + c) * 2);
      s += v.x;
      q += v.y;
    }
  }
  rs[tl][cl] = s;
  rq[tl][cl] = q;
  __syncthreads();
  if (tl == 0 && c < C) {
    s = rs[0][cl] + rs[1][cl] + rs[2][cl] + rs[3][cl];
    q = rq[0][cl] + rq[1][cl] + rq[2][cl] + rq[3][cl];
    part[((long long)blockIdx.y * C + c) * 2 + 0] = s;
    part[((long long)blockIdx.y * C + c) * 2 + 1] = q;
  }
}

__global__ void bn_stats_stage2(const double* __restrict__ part, int G, int C, long long count,
                                const float* __restrict__ gamma, const float* __restrict__ beta,
                                float* running_mean, float* running_var, float momentum, float eps,
                                float* __restrict__ scale, float* __restrict__ shift,
                                float* save_mean, float* save_var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int g = 0; g < G; ++g) {
    s += part[((long long)g * C + c) * 2 + 0];
    q += part[((long long)g * C + c) * 2 + 1];
  }
  const double n = (double)count;
  const double mean = s / n;
  double var = q / n - mean * mean;
  if (var < 0) var = 0;
  const double inv = 1.0 / sqrt(var + (double)eps);
  const float sc = (float)((double)gamma[c] * inv);
  scale[c] = sc;
  shift[c] = (float)((double)beta[c] - mean * (double)sc);
  if (save_mean) save_mean[c] = (float)mean;
  if (save_var) save_var[c] = (float)var;
  if (running_mean) {
    const double unb = count > 1 ? var * n / (n - 1.0) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * (float)unb;
  }
}

extern "C" int capmi_bn_finalize(const float* stats, int tiles, int C, long long count,
                                 const float* gamma, const float* beta, float* running_mean,
                                 float* running_var, float momentum, float eps, float* scale,
                                 float* shift, float* save_mean, float* save_var, void* work,
                                 void* stream) {
  CAPMI_REQUIRE(stats && gamma && beta && scale && shift && work && tiles > 0 && C > 0 && count > 0,
                CAPMI_EINVAL);
  CAPMI_REQUIRE((running_mean == nullptr) == (running_var == nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE(((uintptr_t)stats & 7) == 0 && ((uintptr_t)work & 7) == 0, CAPMI_EALIGN);
  const int G = std::min(BNF_MAXG, std::max(1, (tiles + 31) / 32));
  const int per_g = (tiles + G - 1) / G;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(bn_stats_stage1, dim3(cdiv(C, 64), G), dim3(256), 0, s, stats, tiles, C, per_g,
                     (double*)work);
  hipLaunchKernelGGL(bn_stats_stage2, dim3(cdiv(C, 256)), dim3(256), 0, s, (const double*)work, G, C,
                     count, gamma, beta, running_mean, running_var, momentum, eps, scale, shift,
                     save_mean, save_var);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

__global__ void bn_eval_params_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                      const float* __restrict__ rm, const float* __restrict__ rv,
                                      int C, float eps, float* __restrict__ scale,
                                      float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float sc = gamma[c] / sqrtf(rv[c] + eps);
  scale[c] = sc;
  shift[c] = beta[c] - rm[c] * sc;
}

extern "C" int capmi_bn_eval_params(const float* gamma, const float* beta, const float* running_mean,
                                    const float* running_var, int C, float eps, float* scale,
                                    float* shift, void* stream) {
  CAPMI_REQUIRE(gamma && beta && running_mean && running_var && scale && shift && C > 0, CAPMI_EINVAL);
  hipLaunchKernelGGL(bn_eval_params_kernel, dim3(cdiv(C, 256)), dim3(256), 0, as_stream(stream), gamma,
                     beta, running_mean, running_var, C, eps, scale, shift);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------
// out = relu(y*s + b + (res_scale ? res*rs + rb : res))
// ---------------------------------------------------------------------------------
__global__ void bn_add_relu_kernel(const float4* __restrict__ y, const float* __restrict__ s,
                                   const float* __restrict__ b, const float4* __restrict__ res,
                                   const float* __restrict__ rs, const float* __restrict__ rb,
                                   float4* __restrict__ out, long long n4, int C4) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    const float4 sc = *reinterpret_cast<const float4*>(s + c);
    const float4 sh = *reinterpret_cast<const float4*>(b + c);
    float4 r = res[i];
    if (rs) r = fma4(r, *reinterpret_cast<const float4*>(rs + c), *reinterpret_cast<const float4*>(rb + c));
    out[i] = relu4(fma4(y[i], sc, sh) + r);
  }
}

extern "C" int capmi_bn_add_relu(const float* y, const float* s, const float* b, const float* res,
                                 const float* res_scale, const float* res_shift, float* out,
                                 long long rows, int C, void* stream) {
  CAPMI_REQUIRE(y && s && b && res && out && rows >= 0 && C > 0 && C % 4 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(y) && aligned16(res) && aligned16(out) && aligned16(s) && aligned16(b),
                CAPMI_EALIGN);
  const long long n4 = rows * C / 4;
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(bn_add_relu_kernel, dim3(std::min<long long>(cdiv(n4, 256), 8192)), dim3(256),
                     0, as_stream(stream), (const float4*)y, s, b, (const float4*)res, res_scale,
                     res_shift, (float4*)out, n4, C / 4);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------
// out = maxpool3x3/2/p1(relu(y*s + b)), NHWC
// ---------------------------------------------------------------------------------
__global__ void bn_relu_maxpool_kernel(const float* __restrict__ y, const float* __restrict__ s,
                                       const float* __restrict__ b, float* __restrict__ out, int N,
                                       int H, int W, int C, int Ho, int Wo) {
  const int C4 = C / 4;
  const long long n = (long long)N * Ho * Wo * C4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    long long r = i / C4;
    const int ow = (int)(r % Wo);
    r /= Wo;
    const int oh = (int)(r % Ho);
    const int nn = (int)(r / Ho);
    const float4 sc = *reinterpret_cast<const float4*>(s + c);
    const float4 sh = *reinterpret_cast<const float4*>(b + c);
    float4 m = f4(-INFINITY);
    for (int dh = 0; dh < 3; ++dh) {
      const int ih = oh * 2 - 1 + dh;
      if (ih < 0 || ih >= H) continue;
      for (int dw = 0; dw < 3; ++dw) {
        const int iw = ow * 2 - 1 + dw;
        if (iw < 0 || iw >= W) continue;
        const float4 v = relu4(fma4(
            *reinterpret_cast<const float4*>(y + (((long long)nn * H + ih) * W + iw) * C + c), sc, sh));
        m.x = fmaxf(m.x, v.x);
        m.y = fmaxf(m.y, v.y);
        m.z = fmaxf(m.z, v.z);
        m.w = fmaxf(m.w, v.w);
      }
    }
    *reinterpret_cast<float4*>(out + i * 4) = m;
  }
}

extern "C" int capmi_bn_relu_maxpool(const float* y, const float* s, const float* b, float* out,
                                     int N, int H, int W, int C, int Ho, int Wo, void* stream) {
  CAPMI_REQUIRE(y && s && b && out && C % 4 == 0 && N > 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(Ho == (H + 2 - 3) / 2 + 1 && Wo == (W + 2 - 3) / 2 + 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(y) && aligned16(out) && aligned16(s) && aligned16(b), CAPMI_EALIGN);
  const long long n = (long long)N * Ho * Wo * C / 4;
  hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3(std::min<long long>(cdiv(n, 256), 8192)),
                     dim3(256), 0, as_stream(stream), y, s, b, out, N, H, W, C, Ho, Wo);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------------
// AdaptiveAvgPool2d((OH,OW)) on NHWC (window [floor(i*H/OH), ceil((i+1)*H/OH)) )
// ---------------------------------------------------------------------------------
__global__ void adaptive_avgpool_nhwc_kernel(const float* __restrict__ in, int N, int H, int W,
                                             int C, int OH, int OW, float* __restrict__ out) {
  const int C4 = C / 4;
  const long long n = (long long)N * OH * OW * C4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C4) * 4;
    long long r = i / C4;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int nn = (int)(r / OH);
    const int h0 = (oh * H) / OH, h1 = ((oh + 1) * H + OH - 1) / OH;
    const int w0 = (ow * W) / OW, w1 = ((ow + 1) * W + OW - 1) / OW;
    float4 acc = f4(0.f);
    for (int ih = h0; ih < h1; ++ih)
      for (int iw = w0; iw < w1; ++iw)
        acc = acc + *reinterpret_cast<const float4*>(in + (((long long)nn * H + ih) * W + iw) * C + c);
    const float inv = 1.f / (float)((h1 - h0) * (w1 - w0));
    *reinterpret_cast<float4*>(out + i * 4) = acc * f4(inv);
  }
}

extern "C" int capmi_adaptive_avgpool_nhwc(const float* in, int N, int H, int W, int C, int OH,
                                           int OW, float* out, void* stream) {
  CAPMI_REQUIRE(in && out && C % 4 == 0 && N > 0 && H > 0 && W > 0 && OH > 0 && OW > 0,
                CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(in) && aligned16(out), CAPMI_EALIGN);
  const long long n = (long long)N * OH * OW * C / 4;
  hipLaunchKernelGGL(adaptive_avgpool_nhwc_kernel, dim3(std::min<long long>(cdiv(n, 256), 8192)),
                     dim3(256), 0, as_stream(stream), in, N, H, W, C, OH, OW, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}
