// Train-mode BatchNorm finalize: per-slice (Σ, Σx²) of a conv output -> scale / shift (+ batch mean / var,
// running-stat update), models/encoder.py:97-107 (torchvision BN in train mode, momentum 0.1, unbiased
// running variance). Round 4: one canonical fp64 summation order, independent of the launch shape, that
// the host can restate op for op (tests/test_gpu_bn_final.py).
//
// Canonical order for channel c over the T statistic slices (rows of stats[T][C][2]):
//   q_l = sum of slice t = l, l + 64, l + 128, ... in ascending t   (l = 0..63, fp64)
//   r_w = q_8w + q_8w+1 + ... + q_8w+7                                 (w = 0..7, in order)
//   sum = r_0 + r_1 + ... + r_7                                        (in order)
// Threads: a wave covers 8 channels x 8 slice lanes (one 64-B row segment per slice); the 64 lane groups
// l = 8 w + s of a channel are 8 (virtual) waves w x 8 lanes s.
#pragma once
#include "common.h"

constexpr int BNF_CG = 8;  // channels per finalize group

struct BnFinArgs {
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float* scale;
  float* shift;
  float* save_mean;
  float* save_var;
  float momentum, eps;
  long long count;
};

// every operation rounded on its own (no contraction into fma): the result is a function of the sums alone,
// reproducible by any IEEE implementation (tests/test_gpu_bn_final.py)
__device__ __forceinline__ void bnf_apply(const BnFinArgs& f, int c, double s, double q) {
#pragma clang fp contract(off)
  const double n = (double)f.count;
  const double mean = s / n;
  double var = q / n - mean * mean;
  if (var < 0) var = 0;
  const double inv = 1.0 / sqrt(var + (double)f.eps);
  const float sc = (float)((double)f.gamma[c] * inv);
  f.scale[c] = sc;
  f.shift[c] = (float)((double)f.beta[c] - mean * (double)sc);
  if (f.save_mean) f.save_mean[c] = (float)mean;
  if (f.save_var) f.save_var[c] = (float)var;
  if (f.running_mean) {
    const double unb = f.count > 1 ? var * n / (n - 1.0) : var;
    f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * (float)mean;
    f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unb;
  }
}

// Finalize channel group g (channels [8 g, 8 g + 8) below C) with the calling workgroup's NT threads.
// scratch: 72 x 8 double2 in LDS (9 KiB), free on entry; the workgroup meets three times.
template <int NT>
__device__ __forceinline__ void bnf_group(const BnFinArgs& f, const float* __restrict__ stats, int T, int C, int g,
                                          double2* scratch) {
  static_assert(NT % 64 == 0 && NT <= 512, "whole waves, at most 8");
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, cl = lane & 7, s = lane >> 3;
  const int c = g * BNF_CG + cl;
#pragma unroll
  for (int vw = w; vw < 8; vw += NT / 64) {
    const int l = vw * 8 + s;
    double sm = 0.0, sq = 0.0;
    if (c < C) {
      const float2* p = reinterpret_cast<const float2*>(stats) + c;
      int t = l;
      for (; t + 15 * 64 < T; t += 16 * 64) {  // 16 loads in flight, then the adds in slice order
        float2 v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = p[(long long)(t + 64 * u) * C];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          sm += v[u].x;
          sq += v[u].y;
        }
      }
      for (; t < T; t += 64) {
        const float2 v = p[(long long)t * C];
        sm += v.x;
        sq += v.y;
      }
    }
    scratch[l * BNF_CG + cl] = make_double2(sm, sq);
  }
  __syncthreads();
  if (tid < 64) {  // r_w for (w, channel) = (tid / 8, tid % 8): two serial chains of 8 instead of one of 64
    const int w8 = tid >> 3, cc = tid & 7;
    double sm = 0.0, sq = 0.0;
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      const double2 v = scratch[(8 * w8 + s8) * BNF_CG + cc];
      sm += v.x;
      sq += v.y;
    }
    scratch[(64 + w8) * BNF_CG + cc] = make_double2(sm, sq);
  }
  __syncthreads();
  if (tid < BNF_CG && g * BNF_CG + tid < C) {
    double sm = 0.0, sq = 0.0;
#pragma unroll
    for (int w8 = 0; w8 < 8; ++w8) {
      const double2 v = scratch[(64 + w8) * BNF_CG + tid];
      sm += v.x;
      sq += v.y;
    }
    bnf_apply(f, g * BNF_CG + tid, sm, sq);
  }
  __syncthreads();
}
