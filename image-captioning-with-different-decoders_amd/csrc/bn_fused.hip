// Train-mode BatchNorm finalize fused into the elementwise pass that consumes it (encoder
// forward, layer3/4 sizes). A BN of the conv stack is normally two launches on the encoder's
// critical path: capmi_bn_finalize (the per-slice (sum, sumsq) of the conv epilogue -> batch mean /
// var -> scale, shift, running stats; ~5 us, latency-bound) and the apply pass (BN + ReLU of the
// next conv's input, or the bottleneck tail). Here every workgroup owns a 32-channel group and a
// chunk of rows: it first finalizes its 32 channels itself from the slice statistics (redundantly
// per row chunk: <= 256 slices x 32 channels x 8 B = 64 KB of L2-resident reads), in fp64 and a
// fixed order, then applies them to its rows. The workgroups of row chunk 0 write scale / shift and
// update the running statistics (models/encoder.py:88-91: nn.BatchNorm2d in train mode, momentum
// 0.1, unbiased running variance) exactly once.
//
// ops (capmi.h: CAPMI_BNFA_*):
//   0 SPLIT3    y fp32 -> relu(bn(y)) split exactly into three bf16 planes out[3][rows*C] (x3p input)
//   1 ADD_RELU  y, res fp32 -> out = relu(bn(y) + res)          (identity-residual bottleneck tail)
//   2 RELU_BF16 y bf16 -> out bf16 = relu(bn(y)) (in place allowed; the bf16 conv input)
//   3 ADD_RELU_BF16 y, res bf16 -> out bf16 = relu(bn(y) + res)
// Arithmetic of the apply is that of bn_relu_split3 / bn_add_relu / bn_relu_bf16 / bn_add_relu_bf16;
// the finalize is bn_finalize_direct's formulas with a different (fixed) fp64 summation order.
#include "common.h"

namespace {

constexpr int FW = 32;         // channels per workgroup
constexpr int FS = 256 / FW;   // slice lanes per channel in the finalize

struct BnFin {
  const float* stats;
  int tiles, C;
  long long count;
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float momentum, eps;
  float* scale;
  float* shift;
};

__device__ __forceinline__ unsigned short bfbits(float x) { return __builtin_bit_cast(unsigned short, (__bf16)x); }
__device__ __forceinline__ float bfval(unsigned b16) { return __uint_as_float(b16 << 16); }

template <int OP>
__global__ void __launch_bounds__(256) bn_fin_apply_kernel(const BnFin f, const void* __restrict__ y_,
                                                           const void* __restrict__ res_, void* __restrict__ out_,
                                                           long long rows, int rows_per_chunk) {
  __shared__ double rs[FS][FW], rq[FS][FW];
  __shared__ float ssc[FW], ssh[FW];
  const int t = threadIdx.x, ch = t % FW, sl = t / FW;
  const int C = f.C, c0 = blockIdx.x * FW;
  // ---- finalize the workgroup's 32 channels (4 independent loads in flight per lane)
  {
    double s = 0.0, q = 0.0;
    const float* st = f.stats + (long long)(c0 + ch) * 2;
    for (int k = sl; k < f.tiles; k += 4 * FS) {
      float2 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = k + u * FS;
        v[u] = kk < f.tiles ? *reinterpret_cast<const float2*>(st + (long long)kk * C * 2) : make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s += v[u].x;
        q += v[u].y;
      }
    }
    rs[sl][ch] = s;
    rq[sl][ch] = q;
  }
  __syncthreads();
  if (t < FW) {
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int r = 0; r < FS; ++r) {
      s += rs[r][t];
      q += rq[r][t];
    }
    const int c = c0 + t;
    const double n = (double)f.count;
    const double mean = s / n;
    double var = q / n - mean * mean;
    if (var < 0) var = 0;
    const double inv = 1.0 / sqrt(var + (double)f.eps);
    const float sc = (float)((double)f.gamma[c] * inv);
    const float sh = (float)((double)f.beta[c] - mean * (double)sc);
    ssc[t] = sc;
    ssh[t] = sh;
    if (blockIdx.y == 0) {
      f.scale[c] = sc;
      f.shift[c] = sh;
      if (f.running_mean) {
        const double unb = f.count > 1 ? var * n / (n - 1.0) : var;
        f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * (float)mean;
        f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * (float)unb;
      }
    }
  }
  __syncthreads();
  // ---- apply to rows [r0, r1) x channels [c0, c0 + 32): 8 groups of 4 channels per row
  const long long r0 = (long long)blockIdx.y * rows_per_chunk;
  const long long r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
  const int g = t & 7, cl = 4 * g;
  const float s0 = ssc[cl], s1 = ssc[cl + 1], s2 = ssc[cl + 2], s3 = ssc[cl + 3];
  const float b0 = ssh[cl], b1 = ssh[cl + 1], b2 = ssh[cl + 2], b3 = ssh[cl + 3];
  for (long long r = r0 + (t >> 3); r < r1; r += 32) {
    const long long e = r * C + c0 + cl;  // element index of this thread's 4 channels
    if (OP == 0 || OP == 1) {
      const float4 v = *reinterpret_cast<const float4*>(static_cast<const float*>(y_) + e);
      float o[4] = {fmaf(v.x, s0, b0), fmaf(v.y, s1, b1), fmaf(v.z, s2, b2), fmaf(v.w, s3, b3)};
      if (OP == 1) {
        const float4 rr = *reinterpret_cast<const float4*>(static_cast<const float*>(res_) + e);
        o[0] += rr.x;
        o[1] += rr.y;
        o[2] += rr.z;
        o[3] += rr.w;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) o[u] = fmaxf(o[u], 0.f);
      if (OP == 1) {
        *reinterpret_cast<float4*>(static_cast<float*>(out_) + e) = make_float4(o[0], o[1], o[2], o[3]);
      } else {
        unsigned short h[3][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const __bf16 h0 = (__bf16)o[u];
          const float r1v = o[u] - (float)h0;
          const __bf16 h1 = (__bf16)r1v;
          const __bf16 h2 = (__bf16)(r1v - (float)h1);
          h[0][u] = __builtin_bit_cast(unsigned short, h0);
          h[1][u] = __builtin_bit_cast(unsigned short, h1);
          h[2][u] = __builtin_bit_cast(unsigned short, h2);
        }
        const long long plane = rows * C;
        unsigned long long* out = static_cast<unsigned long long*>(out_);
#pragma unroll
        for (int p = 0; p < 3; ++p)
          out[(p * plane + e) >> 2] = (unsigned long long)h[p][0] | ((unsigned long long)h[p][1] << 16) |
                                      ((unsigned long long)h[p][2] << 32) | ((unsigned long long)h[p][3] << 48);
      }
    } else {
      const uint2 v = *reinterpret_cast<const uint2*>(static_cast<const unsigned short*>(y_) + e);
      float o[4] = {fmaf(bfval(v.x & 0xffffu), s0, b0), fmaf(bfval(v.x >> 16), s1, b1),
                    fmaf(bfval(v.y & 0xffffu), s2, b2), fmaf(bfval(v.y >> 16), s3, b3)};
      if (OP == 3) {
        const uint2 rr = *reinterpret_cast<const uint2*>(static_cast<const unsigned short*>(res_) + e);
        o[0] += bfval(rr.x & 0xffffu);
        o[1] += bfval(rr.x >> 16);
        o[2] += bfval(rr.y & 0xffffu);
        o[3] += bfval(rr.y >> 16);
      }
      const unsigned lo = (unsigned)bfbits(fmaxf(o[0], 0.f)) | ((unsigned)bfbits(fmaxf(o[1], 0.f)) << 16);
      const unsigned hi = (unsigned)bfbits(fmaxf(o[2], 0.f)) | ((unsigned)bfbits(fmaxf(o[3], 0.f)) << 16);
      *reinterpret_cast<uint2*>(static_cast<unsigned short*>(out_) + e) = make_uint2(lo, hi);
    }
  }
}

// workgroups per launch (row chunks x channel groups); CAPMI_BNFA_BLOCKS overrides (A/B measurement)
int bnfa_blocks() {
  static const int n = [] {
    const char* e = getenv("CAPMI_BNFA_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : 512;
  }();
  return n;
}

}  // namespace

extern "C" int capmi_bn_finalize_apply(int op, const float* stats, int tiles, int C, long long count,
                                       const float* gamma, const float* beta, float* running_mean,
                                       float* running_var, float momentum, float eps, float* scale, float* shift,
                                       const void* y, const void* res, void* out, long long rows, void* stream) {
  CAPMI_REQUIRE(op >= 0 && op <= 3, CAPMI_EINVAL);
  CAPMI_REQUIRE(stats && gamma && beta && scale && shift && y && out && tiles > 0 && count > 0 && rows > 0,
                CAPMI_EINVAL);
  CAPMI_REQUIRE(C > 0 && C % FW == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(tiles <= CAPMI_BNFA_MAX_TILES, CAPMI_ERANGE);
  CAPMI_REQUIRE((running_mean == nullptr) == (running_var == nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE((op == 1 || op == 3) == (res != nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE(((uintptr_t)stats & 7) == 0 && aligned16(y) && aligned16(out) && (res == nullptr || aligned16(res)),
                CAPMI_EALIGN);
  const int groups = C / FW;
  const long long want = std::max<long long>(1, bnfa_blocks() / groups);
  long long chunk = cdiv(rows, want);
  chunk = cdiv(chunk, 32) * 32;  // whole 32-row passes
  const long long chunks = cdiv(rows, chunk);
  CAPMI_REQUIRE(chunk < (1LL << 31) && chunks < 65536, CAPMI_ERANGE);
  BnFin f{stats, tiles, C, count, gamma, beta, running_mean, running_var, momentum, eps, scale, shift};
  const dim3 g((unsigned)groups, (unsigned)chunks), b(256);
  hipStream_t s = as_stream(stream);
  switch (op) {
    case 0: hipLaunchKernelGGL(bn_fin_apply_kernel<0>, g, b, 0, s, f, y, res, out, rows, (int)chunk); break;
    case 1: hipLaunchKernelGGL(bn_fin_apply_kernel<1>, g, b, 0, s, f, y, res, out, rows, (int)chunk); break;
    case 2: hipLaunchKernelGGL(bn_fin_apply_kernel<2>, g, b, 0, s, f, y, res, out, rows, (int)chunk); break;
    default: hipLaunchKernelGGL(bn_fin_apply_kernel<3>, g, b, 0, s, f, y, res, out, rows, (int)chunk); break;
  }
  CAPMI_LAUNCH_CHECK();
  return 0;
}
