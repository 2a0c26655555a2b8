// Optimiser step: element-wise gradient clamp (train_utils.py:2-12) fused into Adam
// (torch.optim.Adam defaults: betas (0.9, 0.999), eps 1e-8, no weight decay;
// models/attention.py:352-355,423-430). One pass over the flat parameter/grad/state
// buffers: read p, g, m, v; write p, m, v (28 B / parameter, HBM-bound).
// The arithmetic follows torch's single-tensor path: m.lerp_(g, 1-b1),
// v.mul_(b2).addcmul_(g, g, 1-b2), p.addcdiv_(m, sqrt(v)/sqrt(bc2) + eps, -lr/bc1).
#include "common.h"

// Hyper-parameters arrive in double (Python floats) and are rounded to T exactly where torch
// rounds its Scalars: step_size = lr / bc1 and bc2_sqrt in double, then cast.
template <typename T>
__global__ void adam_clamp_kernel(T* __restrict__ p, const T* __restrict__ g, T* __restrict__ m,
                                  T* __restrict__ v, long long n, double lr, double beta1,
                                  double beta2, double eps, double bc1_h, double bc2s_h, double clip_d,
                                  const long long* __restrict__ step_dev) {
  double bc1 = bc1_h, bc2s = bc2s_h;
  if (step_dev != nullptr) {
    const double t = (double)(*step_dev);
    bc1 = 1.0 - pow(beta1, t);
    bc2s = sqrt(1.0 - pow(beta2, t));
  }
  const T step_size = (T)(lr / bc1), bc2_sqrt = (T)bc2s;
  const T w1 = (T)(1.0 - beta1), b2 = (T)beta2, w2 = (T)(1.0 - beta2), e = (T)eps, clip = (T)clip_d;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    T gi = g[i];
    gi = gi < -clip ? -clip : (gi > clip ? clip : gi);
    const T mi = m[i] + w1 * (gi - m[i]);  // lerp, weight < 0.5
    const T vi = v[i] * b2 + (w2 * gi) * gi;
    m[i] = mi;
    v[i] = vi;
    const T denom = sqrt(vi) / bc2_sqrt + e;
    p[i] = p[i] + (-step_size) * (mi / denom);
  }
}

template <typename T>
static int adam_launch(T* p, const T* g, T* m, T* v, long long n, double lr, double beta1,
                       double beta2, double eps, double bc1, double bc2_sqrt, double clip,
                       const long long* step_dev, void* stream) {
  CAPMI_REQUIRE(p && g && m && v && n >= 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(step_dev != nullptr || (bc1 > 0.0 && bc2_sqrt > 0.0), CAPMI_EINVAL);
  if (n == 0) return 0;
  hipLaunchKernelGGL(adam_clamp_kernel<T>, dim3(std::min<long long>(cdiv(n, 256), 8192)), dim3(256),
                     0, as_stream(stream), p, g, m, v, n, lr, beta1, beta2, eps, bc1, bc2_sqrt, clip,
                     step_dev);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_adam_clamp(float* p, const float* g, float* m, float* v, long long n, double lr,
                                double beta1, double beta2, double eps, double bc1, double bc2_sqrt,
                                double clip, const long long* step_dev, void* stream) {
  return adam_launch<float>(p, g, m, v, n, lr, beta1, beta2, eps, bc1, bc2_sqrt, clip, step_dev, stream);
}

extern "C" int capmi_adam_clamp_f64(double* p, const double* g, double* m, double* v, long long n,
                                    double lr, double beta1, double beta2, double eps, double bc1,
                                    double bc2_sqrt, double clip, const long long* step_dev,
                                    void* stream) {
  return adam_launch<double>(p, g, m, v, n, lr, beta1, beta2, eps, bc1, bc2_sqrt, clip, step_dev, stream);
}

__global__ void counter_add_kernel(long long* c, long long v) { *c += v; }

extern "C" int capmi_counter_add(long long* counter, long long v, void* stream) {
  CAPMI_REQUIRE(counter != nullptr, CAPMI_EINVAL);
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, as_stream(stream), counter, v);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// embedding gradient (nn.Embedding backward, models/attention.py:117,247): scatter-add of the
// embedding half of the LSTM input gradient, dx[t][b][0:M] -> demb[caps[b*L+t]]
__global__ void embed_scatter_add_kernel(const float* __restrict__ dx, long long ld_dx,
                                         const long long* __restrict__ caps, int B, int L, int T,
                                         const int* __restrict__ bt, int M, void* demb, int is_f64) {
  const long long n = (long long)T * B * M;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int mm = (int)(i % M);
    const long long tb = i / M;
    const int b = (int)(tb % B), t = (int)(tb / B);
    if (bt && b >= bt[t]) continue;
    const long long tok = caps[(long long)b * L + t];
    const float d = dx[tb * ld_dx + mm];
    if (is_f64)
      atomicAdd(reinterpret_cast<double*>(demb) + tok * M + mm, (double)d);
    else
      atomicAdd(reinterpret_cast<float*>(demb) + tok * M + mm, d);
  }
}

extern "C" int capmi_embed_scatter_add(const float* dx, long long ld_dx, const long long* caps,
                                       int B, int L, int T, const int* bt, int M, void* demb,
                                       int demb_is_f64, void* stream) {
  CAPMI_REQUIRE(dx && caps && demb && B > 0 && M > 0 && T >= 0 && T <= L, CAPMI_EINVAL);
  const long long n = (long long)T * B * M;
  if (n == 0) return 0;
  hipLaunchKernelGGL(embed_scatter_add_kernel, dim3(std::min<long long>(cdiv(n, 256), 4096)),
                     dim3(256), 0, as_stream(stream), dx, ld_dx, caps, B, L, T, bt, M, demb,
                     demb_is_f64);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" const char* capmi_strerror(int code) {
  switch (code) {
    case CAPMI_OK: return "ok";
    case CAPMI_EINVAL: return "capmi: invalid argument or shape";
    case CAPMI_EALIGN: return "capmi: pointer/stride alignment requirement not met";
    case CAPMI_ERANGE: return "capmi: size outside the supported range";
    default: return hipGetErrorString((hipError_t)code);
  }
}

extern "C" int capmi_abi_version(void) { return CAPMI_ABI_VERSION; }
