// Image preprocessing on the GPU: the reference's per-image CPU transform
// Resize((224, 224)) -> ToTensor -> Normalize(mean, std) (models/attention.py:296-301, applied in
// dataset.py:55-59 by DataLoader workers) as two kernels over a batch of decoded uint8 RGB images
// of any sizes. Only the JPEG decode stays on the host; the uint8 pixels (4x fewer bytes than the
// fp32 tensor) cross PCIe.
//
// Resize is torchvision's PIL path (Image.resize(size, BILINEAR), reducing_gap None), restated
// from Pillow's Resample.c so that the result is bit-identical to it:
//   * separable antialiasing triangle filter, support = max(1, in/out); per output index the taps
//     [xmin, xmin + xmax) and weights w = f((x + xmin - center + 0.5) / filterscale) normalised to
//     sum 1 in double (precompute_coeffs), then 22-bit fixed point (normalize_coeffs_8bpc);
//   * horizontal pass first, rounded to uint8 (clip8: (acc + 2^21) >> 22, clamped), then the
//     vertical pass over that intermediate, rounded to uint8 again;
// the double arithmetic is evaluated in Pillow's order with FMA contraction off. ToTensor +
// Normalize: (u8 / 255.f - mean[c]) / std[c] in fp32, as torchvision does it.
#include <cmath>

#include "common.h"

namespace {

constexpr int kPrec = 22;  // Pillow's PRECISION_BITS for 8-bit images (32 - 8 - 2)

// Pillow's precompute_coeffs + normalize_coeffs_8bpc for ONE output index `xx`: fills k[0..n)
// (fixed point) and returns the first source index; n = the tap count (<= kmax).
#pragma clang fp contract(off)
__device__ int resample_taps(int in_size, int out_size, int xx, int kmax, int* k, int* n) {
  const double scale = (double)(float)in_size / out_size;  // (in1 - in0) / outSize, box as floats
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;                 // bilinear support 1.0
  const double center = 0.0 + (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > kmax) xmax = kmax;  // never for kmax = 2*ceil(support)+1 (host-checked)
  double w[32];
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) {
    double t = (x + xmin - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    const double v = t < 1.0 ? 1.0 - t : 0.0;
    w[x] = v;
    ww += v;
  }
  for (int x = 0; x < xmax; ++x) {
    double v = w[x];
    if (ww != 0.0) v /= ww;
    k[x] = v < 0 ? (int)(-0.5 + v * (1 << kPrec)) : (int)(0.5 + v * (1 << kPrec));
  }
  *n = xmax;
  return xmin;
}
#pragma clang fp contract(on)

__device__ __forceinline__ unsigned char clip8(int acc) {
  const int v = acc >> kPrec;  // arithmetic shift: floor, as Pillow's lookup index
  return (unsigned char)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// horizontal pass: tmp[b][y][ox][c] (uint8) for every source row y of image b
__global__ void resize_h_kernel(const unsigned char* __restrict__ src, const long long* __restrict__ offs,
                                const int* __restrict__ hs, const int* __restrict__ ws, int OW, int Hmax, int kmax,
                                unsigned char* __restrict__ tmp) {
  const int b = blockIdx.z, y = blockIdx.y;
  const int H = hs[b], W = ws[b];
  if (y >= H) return;
  const unsigned char* row = src + offs[b] + (long long)y * W * 3;
  unsigned char* out = tmp + (((long long)b * Hmax + y) * OW) * 3;
  for (int ox = blockIdx.x * blockDim.x + threadIdx.x; ox < OW; ox += gridDim.x * blockDim.x) {
    int k[32], n;
    const int x0 = resample_taps(W, OW, ox, kmax, k, &n);
    int s0 = 1 << (kPrec - 1), s1 = s0, s2 = s0;
    for (int i = 0; i < n; ++i) {
      const unsigned char* p = row + (x0 + i) * 3;
      s0 += p[0] * k[i];
      s1 += p[1] * k[i];
      s2 += p[2] * k[i];
    }
    out[ox * 3 + 0] = clip8(s0);
    out[ox * 3 + 1] = clip8(s1);
    out[ox * 3 + 2] = clip8(s2);
  }
}

// vertical pass + ToTensor + Normalize: out[b][c][oy][ox] fp32
__global__ void resize_v_norm_kernel(const unsigned char* __restrict__ tmp, const int* __restrict__ hs, int OH,
                                     int OW, int Hmax, int kmax, float m0, float m1, float m2, float s0_,
                                     float s1_, float s2_, float* __restrict__ out) {
  const int b = blockIdx.z, oy = blockIdx.y;
  const int H = hs[b];
  int k[32], n;
  const int y0 = resample_taps(H, OH, oy, kmax, k, &n);
  const unsigned char* base = tmp + ((long long)b * Hmax) * OW * 3;
  const long long plane = (long long)OH * OW;
  float* ob = out + (long long)b * 3 * plane + (long long)oy * OW;
  for (int ox = blockIdx.x * blockDim.x + threadIdx.x; ox < OW; ox += gridDim.x * blockDim.x) {
    int a0 = 1 << (kPrec - 1), a1 = a0, a2 = a0;
    for (int i = 0; i < n; ++i) {
      const unsigned char* p = base + ((long long)(y0 + i) * OW + ox) * 3;
      a0 += p[0] * k[i];
      a1 += p[1] * k[i];
      a2 += p[2] * k[i];
    }
    ob[ox] = ((float)clip8(a0) / 255.f - m0) / s0_;
    ob[plane + ox] = ((float)clip8(a1) / 255.f - m1) / s1_;
    ob[2 * plane + ox] = ((float)clip8(a2) / 255.f - m2) / s2_;
  }
}

}  // namespace

extern "C" int capmi_resize_taps_max(int in_size, int out_size) {
  if (in_size <= 0 || out_size <= 0) return -CAPMI_EINVAL;
  const double scale = (double)in_size / out_size;
  const double support = scale < 1.0 ? 1.0 : scale;
  return (int)ceil(support) * 2 + 1;
}

extern "C" int capmi_resize_normalize_u8(const unsigned char* src, const long long* offsets, const int* heights,
                                         const int* widths, int B, int max_h, int max_w, int OH, int OW,
                                         const float* mean, const float* std, void* tmp, float* out,
                                         void* stream) {
  CAPMI_REQUIRE(src && offsets && heights && widths && mean && std && tmp && out, CAPMI_EINVAL);
  CAPMI_REQUIRE(B >= 0 && max_h > 0 && max_w > 0 && OH > 0 && OW > 0, CAPMI_EINVAL);
  if (B == 0) return 0;
  // taps per output index: the largest reduction factor over both axes and every image
  const int kmax = std::max(capmi_resize_taps_max(max_w, OW), capmi_resize_taps_max(max_h, OH));
  CAPMI_REQUIRE(kmax <= 32, CAPMI_ERANGE);  // reductions up to 15x
  CAPMI_REQUIRE(B <= 65535 && max_h <= 65535 && OH <= 65535, CAPMI_ERANGE);
  hipStream_t s = as_stream(stream);
  const int tx = std::min(256, OW);
  hipLaunchKernelGGL(resize_h_kernel, dim3(cdiv(OW, tx), max_h, B), dim3(tx), 0, s, src, offsets, heights, widths,
                     OW, max_h, kmax, static_cast<unsigned char*>(tmp));
  CAPMI_LAUNCH_CHECK();
  hipLaunchKernelGGL(resize_v_norm_kernel, dim3(cdiv(OW, tx), OH, B), dim3(tx), 0, s,
                     static_cast<const unsigned char*>(tmp), heights, OH, OW, max_h, kmax, mean[0], mean[1], mean[2],
                     std[0], std[1], std[2], out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}
