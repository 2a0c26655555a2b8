// Attention-decoder step kernels (forward + backward through time), loss kernels.
//
// Reference: models/attention.py
//   SoftAttention.forward                    :43-61   (ReLU score, softmax over the 196 slots)
//   AttentionDecoder.init_hidden_state       :151-164
//   AttentionDecoder.forward time loop       :260-281 (gate :270-271, LSTMCell :277-278, fc :279)
//   loss                                     :401-414 (CE over packed rows incl. pads, alpha reg)
//
// Layout: per-step tensors are time-major [t][b][...]; the API outputs predictions /
// alphas keep the reference's batch-major (B,T,V) / (B,T,P). Each kernel's grid has
// >= 256 workgroups at B = 64 so the 256 CUs are covered; reductions are per-wave
// (64-lane shuffles) then through LDS. The GEMM partial slabs of split-K launches are
// summed here, in the consumer, instead of in a separate reduction launch.
#include "common.h"

// --------------------------------------------------------------------------------------
__global__ void embed_gather_kernel(const void* __restrict__ emb, int is_f64, int M,
                                    const long long* __restrict__ caps, int B, int L, int T,
                                    float* __restrict__ out, long long ld_out) {
  const long long n = (long long)T * B * M;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(i % M);
    const long long tb = i / M;
    const int b = (int)(tb % B), t = (int)(tb / B);
    const long long tok = caps[(long long)b * L + t];
    const float v = is_f64 ? (float)reinterpret_cast<const double*>(emb)[tok * M + m]
                           : reinterpret_cast<const float*>(emb)[tok * M + m];
    out[tb * ld_out + m] = v;
  }
}

extern "C" int capmi_embed_gather(const void* emb, int emb_is_f64, int M, const long long* caps,
                                  int B, int L, int T, float* out, long long ld_out, void* stream) {
  CAPMI_REQUIRE(emb && caps && out && M > 0 && B > 0 && T >= 0 && T <= L, CAPMI_EINVAL);
  const long long n = (long long)T * B * M;
  if (n == 0) return 0;
  hipLaunchKernelGGL(embed_gather_kernel, dim3(std::min<long long>(cdiv(n, 256), 4096)), dim3(256),
                     0, as_stream(stream), emb, emb_is_f64, M, caps, B, L, T, out, ld_out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// dense (precomputed) word embeddings, e.g. BERT layer-11 features (models/attention.py:166-215,242-244):
// out[t][b][0:M] = emb[b][t][0:M], float4 per thread
__global__ void embed_dense_kernel(const float4* __restrict__ emb, int B, int Le, int M4, int T,
                                   float* __restrict__ out, long long ld_out) {
  const long long n = (long long)T * B * M4;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(i % M4);
    const long long tb = i / M4;
    const int b = (int)(tb % B), t = (int)(tb / B);
    *reinterpret_cast<float4*>(out + tb * ld_out + 4 * m) = emb[((long long)b * Le + t) * M4 + m];
  }
}

extern "C" int capmi_embed_dense(const float* emb, int B, int Le, int M, int T, float* out, long long ld_out,
                                 void* stream) {
  CAPMI_REQUIRE(emb && out && M > 0 && B > 0 && T >= 0 && T <= Le, CAPMI_EINVAL);
  CAPMI_REQUIRE(M % 4 == 0 && ld_out % 4 == 0 && aligned16(emb) && aligned16(out), CAPMI_EALIGN);
  const long long n = (long long)T * B * (M / 4);
  if (n == 0) return 0;
  hipLaunchKernelGGL(embed_dense_kernel, dim3(std::min<long long>(cdiv(n, 256), 4096)), dim3(256), 0,
                     as_stream(stream), reinterpret_cast<const float4*>(emb), B, Le, M / 4, T, out, ld_out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// --------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) mean_rows_kernel(const float* __restrict__ enc, int B, int P,
                                                        int E, float* __restrict__ out) {
  __shared__ float4 part[4][64];
  const int b = blockIdx.y, c4 = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + c4 * 4;
  float4 acc = f4(0.f);
  if (c < E) {
    const float* base = enc + (long long)b * P * E + c;
    for (int p = pg; p < P; p += 4) acc = acc + *reinterpret_cast<const float4*>(base + (long long)p * E);
  }
  part[pg][c4] = acc;
  __syncthreads();
  if (pg == 0 && c < E) {
    const float4 s = ((part[0][c4] + part[1][c4]) + part[2][c4]) + part[3][c4];
    const float inv = (float)P;
    *reinterpret_cast<float4*>(out + (long long)b * E + c) =
        make_float4(s.x / inv, s.y / inv, s.z / inv, s.w / inv);
  }
}

extern "C" int capmi_mean_rows(const float* enc, int B, int P, int E, float* out, void* stream) {
  CAPMI_REQUIRE(enc && out && B > 0 && P > 0 && E > 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(E % 4 == 0 && aligned16(enc) && aligned16(out), CAPMI_EALIGN);
  hipLaunchKernelGGL(mean_rows_kernel, dim3(cdiv(E, 256), B), dim3(256), 0, as_stream(stream), enc, B,
                     P, E, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// --------------------------------------------------------------------------------------
// score: e[b][p] = relu(att_enc[b][p][:] + ad[b][:]) . wf + bf      grid (P/PCH, B)
// --------------------------------------------------------------------------------------
constexpr int PCH = 28;  // slots per workgroup (7 per wave); 196 -> 7 chunks
// the per-timestep score forward and context backward (round 6): 13 slots per workgroup -- the bench's 49 distinct
// rows in 4 chunks, 256 workgroups at B = 64 instead of 128 (half the CUs idle, each reading twice the enc rows):
// per call in a graph (tools/dec_kernels.py) att_score_fwd 5.15 -> 3.91 us, att_ctx_bwd 10.96 -> 10.26 us; every
// row's dot product is one wave's in the same lane order, so the results are bit-identical
constexpr int PCH_T = 13;

__global__ void __launch_bounds__(256) att_score_fwd_kernel(
    const float* __restrict__ att_enc, const float* __restrict__ dec_part, int S, long long dec_slab,
    const float* __restrict__ bias_da, const float* __restrict__ wf, const float* __restrict__ bf,
    int B, int P, int A, float* __restrict__ e, float* __restrict__ att_dec_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* ad = smem;  // [A]
  const int b = blockIdx.y, p0 = blockIdx.x * PCH_T;
  for (int a = threadIdx.x; a < A; a += blockDim.x) {
    const float v = slab_sum(dec_part + (long long)b * A + a, S, dec_slab, bias_da ? bias_da[a] : 0.f);
    ad[a] = v;
    if (att_dec_out && blockIdx.x == 0) att_dec_out[(long long)b * A + a] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float b0 = bf ? bf[0] : 0.f;
  // a wave owns rows p0+wid, p0+wid+4, ... (ceil(PCH_T/4) of them): all their loads are issued before
  // any reduction, and the wave sums run interleaved
  constexpr int R = (PCH_T + 3) / 4;
  const int pend = min(P, p0 + PCH_T);
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int p = p0 + wid + 4 * r;
    acc[r] = 0.f;
    if (p < pend) {
      const float* row = att_enc + ((long long)b * P + p) * A;
      for (int a = lane * 4; a < A; a += 256) {
        const float4 x = *reinterpret_cast<const float4*>(row + a);
        const float4 d = *reinterpret_cast<const float4*>(ad + a);
        const float4 w = *reinterpret_cast<const float4*>(wf + a);
        acc[r] += dot4(relu4(x + d), w);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = wave_sum(acc[r]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int p = p0 + wid + 4 * r;
      if (p < pend) e[(long long)b * P + p] = acc[r] + b0;
    }
  }
}

extern "C" int capmi_att_score_fwd(const float* att_enc, const float* dec_part, int S,
                                   long long dec_slab, const float* bias_da, const float* wf,
                                   const float* bf, int B, int P, int A, float* e,
                                   float* att_dec_out, void* stream) {
  CAPMI_REQUIRE(att_enc && dec_part && wf && e && B > 0 && P > 0 && A > 0 && S >= 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(A % 4 == 0 && A <= 16384, CAPMI_ERANGE);
  CAPMI_REQUIRE(aligned16(att_enc) && aligned16(wf), CAPMI_EALIGN);
  hipLaunchKernelGGL(att_score_fwd_kernel, dim3(cdiv(P, PCH_T), B), dim3(256), A * sizeof(float),
                     as_stream(stream), att_enc, dec_part, S, dec_slab, bias_da, wf, bf, B, P, A, e,
                     att_dec_out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// --------------------------------------------------------------------------------------
// softmax over P + context + gate:  grid (E/ECH, B), 256 threads = 64 float4 cols x 4 p-groups
// --------------------------------------------------------------------------------------
constexpr int ECH = 256;

__global__ void __launch_bounds__(256) att_softmax_ctx_fwd_kernel(
    const float* __restrict__ e, const float* __restrict__ enc, int B, int P, int E, int bt,
    float* __restrict__ alpha_out, long long alpha_ld_b, float* __restrict__ awe_out,
    const float* __restrict__ gate_part, int S, long long gate_slab,
    const float* __restrict__ bias_fb, float* __restrict__ gate_out, float* __restrict__ x_out,
    long long ld_x) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* alpha = smem;                                   // [P]
  float4* part = reinterpret_cast<float4*>(smem + ((P + 3) & ~3));  // [4][64]
  __shared__ float red[16];
  const int b = blockIdx.y, tid = threadIdx.x;
  // softmax over the P scores of row b (every block recomputes; P is small)
  float m = -INFINITY;
  for (int p = tid; p < P; p += 256) {
    const float v = e[(long long)b * P + p];
    alpha[p] = v;
    m = fmaxf(m, v);
  }
  m = block_max(m, red);
  float s = 0.f;
  for (int p = tid; p < P; p += 256) {
    const float v = expf(alpha[p] - m);
    alpha[p] = v;
    s += v;
  }
  s = block_sum(s, red);
  const float inv = 1.f / s;
  for (int p = tid; p < P; p += 256) {
    const float a = alpha[p] * inv;
    alpha[p] = a;
    if (alpha_out && blockIdx.x == 0) alpha_out[(long long)b * alpha_ld_b + p] = b < bt ? a : 0.f;
  }
  __syncthreads();
  // context over this block's 256 columns
  const int c4 = tid & 63, pg = tid >> 6;
  const int c = blockIdx.x * ECH + c4 * 4;
  float4 acc = f4(0.f);
  if (c < E) {
    const float* base = enc + (long long)b * P * E + c;
#pragma unroll 8
    for (int p = pg; p < P; p += 4)
      acc = fma4(f4(alpha[p]), *reinterpret_cast<const float4*>(base + (long long)p * E), acc);
  }
  part[pg * 64 + c4] = acc;
  __syncthreads();
  if (pg == 0 && c < E) {
    float4 awe = part[c4];
    awe = awe + part[64 + c4];
    awe = awe + part[128 + c4];
    awe = awe + part[192 + c4];
    const long long o = (long long)b * E + c;
    if (awe_out) *reinterpret_cast<float4*>(awe_out + o) = awe;
    float4 xg = awe;
    if (gate_part) {
      float4 g = slab_sum(reinterpret_cast<const float4*>(gate_part + o), S, gate_slab / 4,
                          *reinterpret_cast<const float4*>(bias_fb + c));
      g = make_float4(sigmoidf_(g.x), sigmoidf_(g.y), sigmoidf_(g.z), sigmoidf_(g.w));
      if (gate_out) *reinterpret_cast<float4*>(gate_out + o) = g;
      xg = g * awe;
    }
    if (x_out) *reinterpret_cast<float4*>(x_out + (long long)b * ld_x + c) = xg;
  }
}

extern "C" int capmi_att_softmax_ctx_fwd(const float* e, const float* enc, int B, int P, int E,
                                         int bt, float* alpha_out, long long alpha_ld_b,
                                         float* awe_out, const float* gate_part, int S,
                                         long long gate_slab, const float* bias_fb,
                                         float* gate_out, float* x_out, long long ld_x,
                                         void* stream) {
  CAPMI_REQUIRE(e && enc && B > 0 && P > 0 && E > 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(E % 4 == 0 && P <= 8192, CAPMI_ERANGE);
  CAPMI_REQUIRE(aligned16(enc) && (!awe_out || aligned16(awe_out)) && (!gate_out || aligned16(gate_out)),
                CAPMI_EALIGN);
  CAPMI_REQUIRE(!x_out || (aligned16(x_out) && ld_x % 4 == 0), CAPMI_EALIGN);
  CAPMI_REQUIRE(!gate_part || (bias_fb && S >= 1 && aligned16(gate_part) && gate_slab % 4 == 0),
                CAPMI_EINVAL);
  const size_t sh = (((P + 3) & ~3) + 4 * 64 * 4) * sizeof(float);
  hipLaunchKernelGGL(att_softmax_ctx_fwd_kernel, dim3(cdiv(E, ECH), B), dim3(256), sh,
                     as_stream(stream), e, enc, B, P, E, bt, alpha_out, alpha_ld_b, awe_out,
                     gate_part, S, gate_slab, bias_fb, gate_out, x_out, ld_x);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// --------------------------------------------------------------------------------------
// LSTMCell pointwise (gate order i, f, g, o)
// --------------------------------------------------------------------------------------
__device__ __forceinline__ float sig_(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void lstm_cell_fwd_kernel(const float* __restrict__ part, int S, long long slab,
                                     const float* __restrict__ xemb,
                                     const float* __restrict__ hh_part, int S2, long long slab2,
                                     const float* __restrict__ c_prev, int B, int D,
                                     float* __restrict__ h_out, float* __restrict__ c_out,
                                     float* __restrict__ act_out) {
  const long long n = (long long)B * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(i % D), b = (int)(i / D);
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long long o = (long long)b * 4 * D + q * D + j;
      float v = slab_sum(part + o, S, slab, xemb ? xemb[o] : 0.f);
      g[q] = slab_sum(hh_part + o, S2, slab2, v);
    }
    const float ig = sig_(g[0]), fg = sig_(g[1]), cg = tanhf(g[2]), og = sig_(g[3]);
    const float c = fg * c_prev[i] + ig * cg;
    const float h = og * tanhf(c);
    c_out[i] = c;
    h_out[i] = h;
    const long long o = (long long)b * 4 * D + j;
    act_out[o] = ig;
    act_out[o + D] = fg;
    act_out[o + 2 * D] = cg;
    act_out[o + 3 * D] = og;
  }
}

extern "C" int capmi_lstm_cell_fwd(const float* part, int S, long long slab, const float* xemb,
                                   const float* hh_part, int S2, long long slab2,
                                   const float* c_prev, int B, int D, float* h_out, float* c_out,
                                   float* act_out, void* stream) {
  CAPMI_REQUIRE(c_prev && h_out && c_out && act_out && B > 0 && D > 0, CAPMI_EINVAL);
  CAPMI_REQUIRE((S == 0 || part) && (S2 == 0 || hh_part), CAPMI_EINVAL);
  const long long n = (long long)B * D;
  // one lane per (b, j), 64-lane workgroups: B*D = 32768 -> 512 WGs (all CUs busy)
  hipLaunchKernelGGL(lstm_cell_fwd_kernel, dim3(cdiv(n, 64)), dim3(64), 0, as_stream(stream),
                     part, S, slab, xemb, hh_part, S2, slab2, c_prev, B, D, h_out, c_out, act_out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// --------------------------------------------------------------------------------------
// dropout with a stateless counter hash (the mask is regenerated for the backward pass)
// --------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void dropout_kernel(const float* __restrict__ in, long long n, float p,
                               unsigned long long seed, const unsigned long long* __restrict__ seed_dev,
                               float scale, float* __restrict__ out) {
  if (seed_dev != nullptr) seed ^= splitmix64(*seed_dev);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const unsigned long long r = splitmix64(seed ^ splitmix64((unsigned long long)i));
    const float u = (float)(r >> 40) * (1.0f / 16777216.0f);
    out[i] = u >= p ? in[i] * scale : 0.f;
  }
}

extern "C" int capmi_dropout(const float* in, long long n, float p, unsigned long long seed,
                             const unsigned long long* seed_dev, float* out, void* stream) {
  CAPMI_REQUIRE(in && out && n >= 0 && p >= 0.f && p < 1.f, CAPMI_EINVAL);
  if (n == 0) return 0;
  hipLaunchKernelGGL(dropout_kernel, dim3(std::min<long long>(cdiv(n, 256), 4096)), dim3(256), 0,
                     as_stream(stream), in, n, p, seed, seed_dev, 1.f / (1.f - p), out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

__global__ void mask_rows_tb_kernel(float* x, const int* __restrict__ bt, int T, int B, int cols,
                                    long long ld, long long r1, long long s2) {
  const long long n = (long long)T * B * cols;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cols);
    const long long r = i / cols;
    const int b = (int)(r % B), t = (int)(r / B);
    if (b >= bt[t]) x[(r1 > 0 ? (r % r1) * ld + (r / r1) * s2 : r * ld) + c] = 0.f;
  }
}

extern "C" int capmi_mask_rows_tb(float* x, const int* bt, int T, int B, int cols, long long ld,
                                  long long r1, long long s2, void* stream) {
  CAPMI_REQUIRE(x && bt && T >= 0 && B > 0 && cols > 0, CAPMI_EINVAL);
  const long long n = (long long)T * B * cols;
  if (n == 0) return 0;
  hipLaunchKernelGGL(mask_rows_tb_kernel, dim3(std::min<long long>(cdiv(n, 256), 4096)), dim3(256),
                     0, as_stream(stream), x, bt, T, B, cols, ld, r1, s2);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// --------------------------------------------------------------------------------------
// Cross entropy over the (B,T,V) logits: one workgroup per row, online max/sum, then the
// gradient (softmax - onehot)/nrows in the same launch (the row is L2-hot).
// --------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) ce_fwd_bwd_kernel(
    const float* __restrict__ logits, const long long* __restrict__ caps, int B, int T, int L,
    int V, const int* __restrict__ bt, float inv_n, float* __restrict__ loss_rows,
    float* __restrict__ lse_out, float* __restrict__ dlogits, int tm, const float* __restrict__ gscale) {
  __shared__ float red[16];
  const int r = blockIdx.x;  // r = b*T + t
  const int b = r / T, t = r - b * T;
  const bool active = bt == nullptr || b < bt[t];
  const long long drow = tm ? ((long long)t * B + b) : r;
  if (!active) {
    if (threadIdx.x == 0) {
      loss_rows[r] = 0.f;
      if (lse_out) lse_out[r] = 0.f;
    }
    if (dlogits)
      for (int v = threadIdx.x; v < V; v += 256) dlogits[drow * V + v] = 0.f;
    return;
  }
  const float* x = logits + (long long)r * V;
  float m = -INFINITY, s = 0.f;
  for (int v = threadIdx.x; v < V; v += 256) {
    const float xv = x[v];
    if (xv > m) {
      s = s * expf(m - xv) + 1.f;
      m = xv;
    } else {
      s += expf(xv - m);
    }
  }
  const float gm = block_max(m, red);
  s = (m == -INFINITY) ? 0.f : s * expf(m - gm);
  s = block_sum(s, red);
  const float lse = gm + logf(s);
  const long long tgt = caps[(long long)b * L + t + 1];
  if (threadIdx.x == 0) {
    loss_rows[r] = lse - x[tgt];
    if (lse_out) lse_out[r] = lse;
  }
  if (dlogits) {
    const float g = (gscale ? *gscale : 1.f) * inv_n;
    for (int v = threadIdx.x; v < V; v += 256) {
      const float pv = expf(x[v] - lse);
      dlogits[drow * V + v] = (pv - (v == tgt ? 1.f : 0.f)) * g;
    }
  }
}

extern "C" int capmi_ce_fwd_bwd(const float* logits, const long long* caps, int B, int T, int L,
                                int V, const int* bt, int nrows, float* loss_rows, float* lse,
                                float* dlogits, int dl_time_major, const float* gscale,
                                void* stream) {
  CAPMI_REQUIRE(logits && caps && loss_rows && B > 0 && T > 0 && V > 0 && L > T && nrows > 0,
                CAPMI_EINVAL);
  hipLaunchKernelGGL(ce_fwd_bwd_kernel, dim3(B * T), dim3(256), 0, as_stream(stream), logits, caps,
                     B, T, L, V, bt, 1.f / (float)nrows, loss_rows, lse, dlogits, dl_time_major,
                     gscale);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// --------------------------------------------------------------------------------------
// alpha regulariser ((alpha_c - sum_t alpha)^2).mean() and its gradient; one thread per (b, p)
// --------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) alpha_reg_kernel(const float* __restrict__ alphas, int B,
                                                        int T, int P, float alpha_c,
                                                        float* __restrict__ reg_part,
                                                        float* __restrict__ dreg) {
  __shared__ float red[16];
  const int n = B * P;
  const float inv = 1.f / (float)n;
  const int i = blockIdx.x * 256 + threadIdx.x;
  float acc = 0.f;
  if (i < n) {
    const int b = i / P, p = i - b * P;
    const float* a = alphas + (long long)b * T * P + p;
    float s = 0.f;
    for (int t = 0; t < T; ++t) s += a[(long long)t * P];
    const float d = alpha_c - s;
    acc = d * d;
    if (dreg) dreg[i] = -2.f * d * inv;
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0 && reg_part) reg_part[blockIdx.x] = acc * inv;
}

extern "C" int capmi_alpha_reg_parts(int B, int P) { return (int)cdiv((long long)B * P, 256); }

extern "C" int capmi_alpha_reg(const float* alphas, int B, int T, int P, float alpha_c,
                               float* reg_part, float* dreg, void* stream) {
  CAPMI_REQUIRE(alphas && B > 0 && T > 0 && P > 0, CAPMI_EINVAL);
  hipLaunchKernelGGL(alpha_reg_kernel, dim3(cdiv((long long)B * P, 256)), dim3(256), 0,
                     as_stream(stream), alphas, B, T, P, alpha_c, reg_part, dreg);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

__global__ void __launch_bounds__(1024) loss_finalize_kernel(const float* __restrict__ rows, int n,
                                                             float inv_n, const float* __restrict__ reg,
                                                             int nreg, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += rows[i];
  s = block_sum(s, red);
  float r = 0.f;
  for (int i = threadIdx.x; i < nreg; i += blockDim.x) r += reg[i];
  r = block_sum(r, red);
  if (threadIdx.x == 0) out[0] = s * inv_n + r;
}

extern "C" int capmi_loss_finalize(const float* loss_rows, int n, int nrows, const float* reg_part,
                                   int nreg, float* out, void* stream) {
  CAPMI_REQUIRE(loss_rows && out && n > 0 && nrows > 0 && (nreg == 0 || reg_part), CAPMI_EINVAL);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(1024), 0, as_stream(stream), loss_rows, n,
                     1.f / (float)nrows, reg_part, nreg, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// ======================================================================================
// backward through time
// ======================================================================================
__global__ void lstm_cell_bwd_kernel(const float* __restrict__ dhd, const float* __restrict__ dh_part,
                                     int S, long long slab, const float* __restrict__ dc_in,
                                     const float* __restrict__ act, const float* __restrict__ c_prev,
                                     const float* __restrict__ c_cur, int B, int D, int bt,
                                     float* __restrict__ dgates, float* __restrict__ dc_out) {
  const long long n = (long long)B * D;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const int j = (int)(i % D), b = (int)(i / D);
    const long long o = (long long)b * 4 * D + j;
    if (b >= bt) {
      dgates[o] = 0.f;
      dgates[o + D] = 0.f;
      dgates[o + 2 * D] = 0.f;
      dgates[o + 3 * D] = 0.f;
      dc_out[i] = 0.f;
      continue;
    }
    const float dh = slab_sum(dh_part + i, S, slab, dhd ? dhd[i] : 0.f);
    float dc = dc_in ? dc_in[i] : 0.f;
    const float ig = act[o], fg = act[o + D], cg = act[o + 2 * D], og = act[o + 3 * D];
    const float tc = tanhf(c_cur[i]);
    const float d_o = dh * tc * og * (1.f - og);
    dc += dh * og * (1.f - tc * tc);
    const float d_i = dc * cg * ig * (1.f - ig);
    const float d_f = dc * c_prev[i] * fg * (1.f - fg);
    const float d_g = dc * ig * (1.f - cg * cg);
    dgates[o] = d_i;
    dgates[o + D] = d_f;
    dgates[o + 2 * D] = d_g;
    dgates[o + 3 * D] = d_o;
    dc_out[i] = dc * fg;
  }
}

extern "C" int capmi_lstm_cell_bwd(const float* dhd, const float* dh_part, int S, long long slab,
                                   const float* dc_in, const float* act, const float* c_prev,
                                   const float* c_cur, int B, int D, int bt, float* dgates,
                                   float* dc_out, void* stream) {
  CAPMI_REQUIRE(act && c_prev && c_cur && dgates && dc_out && B > 0 && D > 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(S == 0 || dh_part, CAPMI_EINVAL);
  const long long n = (long long)B * D;
  hipLaunchKernelGGL(lstm_cell_bwd_kernel, dim3(cdiv(n, 64)), dim3(64), 0, as_stream(stream), dhd,
                     dh_part, S, slab, dc_in, act, c_prev, c_cur, B, D, bt, dgates, dc_out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// d(awe_g) -> dawe (LDS), dgp, dalpha[b][p] = dawe . enc[b][p][:]        grid (P/PCH, B)
__global__ void __launch_bounds__(256) att_ctx_bwd_kernel(
    const float* __restrict__ part, int S, long long slab, const float* __restrict__ gate,
    const float* __restrict__ awe, const float* __restrict__ enc, int B, int P, int E,
    float* __restrict__ dgp, float* __restrict__ dalpha, float* __restrict__ dawe_out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* dawe = smem;  // [E]
  const int b = blockIdx.y, p0 = blockIdx.x * PCH_T;
  for (int c = threadIdx.x * 4; c < E; c += 1024) {
    const long long o = (long long)b * E + c;
    const float4 d = slab_sum(reinterpret_cast<const float4*>(part + slab + o), S - 1, slab / 4,
                              *reinterpret_cast<const float4*>(part + o));
    float4 dw = d;
    if (gate) {
      const float4 g = *reinterpret_cast<const float4*>(gate + o);
      dw = d * g;
      if (dgp && blockIdx.x == 0) {
        const float4 a = *reinterpret_cast<const float4*>(awe + o);
        float4 r;
        r.x = d.x * a.x * g.x * (1.f - g.x);
        r.y = d.y * a.y * g.y * (1.f - g.y);
        r.z = d.z * a.z * g.z * (1.f - g.z);
        r.w = d.w * a.w * g.w * (1.f - g.w);
        *reinterpret_cast<float4*>(dgp + o) = r;
      }
    }
    *reinterpret_cast<float4*>(dawe + c) = dw;
    if (dawe_out && blockIdx.x == 0) *reinterpret_cast<float4*>(dawe_out + o) = dw;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int p = p0 + wid; p < min(P, p0 + PCH_T); p += 4) {
    const float* row = enc + ((long long)b * P + p) * E;
    float acc = 0.f;
#pragma unroll 8
    for (int c = lane * 4; c < E; c += 256)
      acc += dot4(*reinterpret_cast<const float4*>(row + c), *reinterpret_cast<const float4*>(dawe + c));
    acc = wave_sum(acc);
    if (lane == 0) dalpha[(long long)b * P + p] = acc;
  }
}

// ---------------------------------------------------------------------------------
// Pixel-duplicated encoder features. The reference pools the 7x7 ResNet map to 14x14
// (models/encoder.py:92,108: AdaptiveAvgPool2d(14)); when the output side is a multiple d of the
// input side every pooled pixel IS one input pixel, repeated d x d times. The decoder then runs on
// the F*F distinct rows: softmax over the (F d)^2 positions equals the softmax over the distinct
// ones divided by d^2, and the context sum is unchanged.
// ---------------------------------------------------------------------------------
// ap[r][pi][pj] = aq[r][pi / d][pj / d] * scale   (rows r = b*T + t; scale = 1 / d^2)
__global__ void __launch_bounds__(256) att_alpha_expand_kernel(const float* __restrict__ aq, long long rows,
                                                               int F, int d, float scale,
                                                               float* __restrict__ ap) {
  const int S = F * d, P = S * S, Q = F * F;
  const long long n = rows * P;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long r = i / P;
    const int p = (int)(i - r * P), pi = p / S, pj = p - pi * S;
    ap[i] = aq[r * Q + (pi / d) * F + pj / d] * scale;
  }
}

// out[b][qi][qj] = in[b][qi d][qj d]: one representative of each duplicated group
__global__ void __launch_bounds__(256) att_dup_pick_kernel(const float* __restrict__ in, int B, int F, int d,
                                                           float* __restrict__ out) {
  const int S = F * d, Q = F * F;
  const long long n = (long long)B * Q;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long b = i / Q;
    const int q = (int)(i - b * Q), qi = q / F, qj = q - qi * F;
    out[i] = in[b * S * S + (long long)(qi * d) * S + qj * d];
  }
}

extern "C" int capmi_att_alpha_expand(const float* aq, long long rows, int F, int d, float* ap, void* stream) {
  CAPMI_REQUIRE(aq && ap && rows >= 0 && F > 0 && d > 0, CAPMI_EINVAL);
  const long long n = rows * (long long)(F * d) * (F * d);
  if (n == 0) return 0;
  hipLaunchKernelGGL(att_alpha_expand_kernel, dim3((unsigned)std::min<long long>(cdiv(n, 256), 4096)), dim3(256),
                     0, as_stream(stream), aq, rows, F, d, 1.0f / (float)(d * d), ap);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_att_dup_pick(const float* in, int B, int F, int d, float* out, void* stream) {
  CAPMI_REQUIRE(in && out && B >= 0 && F > 0 && d > 0, CAPMI_EINVAL);
  const long long n = (long long)B * F * F;
  if (n == 0) return 0;
  hipLaunchKernelGGL(att_dup_pick_kernel, dim3((unsigned)std::min<long long>(cdiv(n, 256), 4096)), dim3(256), 0,
                     as_stream(stream), in, B, F, d, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_att_ctx_bwd(const float* part, int S, long long slab, const float* gate,
                                 const float* awe, const float* enc, int B, int P, int E,
                                 float* dgp, float* dalpha, float* dawe_out, void* stream) {
  CAPMI_REQUIRE(part && enc && dalpha && B > 0 && P > 0 && E > 0 && S >= 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(!dawe_out || aligned16(dawe_out), CAPMI_EALIGN);
  CAPMI_REQUIRE(E % 4 == 0 && E <= 16384 && slab % 4 == 0, CAPMI_ERANGE);
  CAPMI_REQUIRE(aligned16(part) && aligned16(enc) && (!gate || aligned16(gate)) &&
                    (!awe || aligned16(awe)) && (!dgp || aligned16(dgp)),
                CAPMI_EALIGN);
  CAPMI_REQUIRE(!dgp || (gate && awe), CAPMI_EINVAL);
  hipLaunchKernelGGL(att_ctx_bwd_kernel, dim3(cdiv(P, PCH_T), B), dim3(256), E * sizeof(float),
                     as_stream(stream), part, S, slab, gate, awe, enc, B, P, E, dgp, dalpha, dawe_out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// gradient w.r.t. encoder_out through the context sums and the init-state mean (fine-tune only):
// denc[b][p][e] = sum_t alpha[b][t][p] * dawe[t][b][e] + dmean[b][e] / P      grid (P/8, B, E/1024)
constexpr int DIN_PB = 8;
__global__ void __launch_bounds__(256) att_enc_dinput_kernel(
    const float* __restrict__ alpha, long long alpha_ld_b, const float* __restrict__ dawe,
    const float* __restrict__ dmean, int B, int T, int P, int E, float* __restrict__ denc) {
  extern __shared__ float al[];  // [T][DIN_PB]
  const int b = blockIdx.y, p0 = blockIdx.x * DIN_PB;
  for (int i = threadIdx.x; i < T * DIN_PB; i += 256) {
    const int t = i / DIN_PB, j = i - t * DIN_PB;
    al[i] = p0 + j < P ? alpha[(long long)b * alpha_ld_b + (long long)t * P + p0 + j] : 0.f;
  }
  __syncthreads();
  const int e = (blockIdx.z * 256 + threadIdx.x) * 4;
  if (e >= E) return;
  float4 acc[DIN_PB];
#pragma unroll
  for (int j = 0; j < DIN_PB; ++j) acc[j] = f4(0.f);
  for (int t = 0; t < T; ++t) {
    const float4 d = *reinterpret_cast<const float4*>(dawe + ((long long)t * B + b) * E + e);
#pragma unroll
    for (int j = 0; j < DIN_PB; ++j) acc[j] = fma4(f4(al[t * DIN_PB + j]), d, acc[j]);
  }
  float4 dm = f4(0.f);
  if (dmean) dm = *reinterpret_cast<const float4*>(dmean + (long long)b * E + e) * f4(1.f / (float)P);
#pragma unroll
  for (int j = 0; j < DIN_PB; ++j)
    if (p0 + j < P) *reinterpret_cast<float4*>(denc + ((long long)b * P + p0 + j) * E + e) = acc[j] + dm;
}

extern "C" int capmi_att_enc_dinput(const float* alpha, long long alpha_ld_b, const float* dawe,
                                    const float* dmean, int B, int T, int P, int E, float* denc,
                                    void* stream) {
  CAPMI_REQUIRE(alpha && dawe && denc && B > 0 && T > 0 && P > 0 && E > 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(E % 4 == 0 && T <= 1024, CAPMI_ERANGE);
  CAPMI_REQUIRE(aligned16(dawe) && aligned16(denc) && (!dmean || aligned16(dmean)), CAPMI_EALIGN);
  hipLaunchKernelGGL(att_enc_dinput_kernel, dim3(cdiv(P, DIN_PB), B, cdiv(E, 1024)), dim3(256),
                     T * DIN_PB * sizeof(float), as_stream(stream), alpha, alpha_ld_b, dawe, dmean, B, T, P, E,
                     denc);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// softmax bwd + relu-score bwd -> de[b][p], dad[b][a]      grid (A/64, B), 64 cols x 4 p-groups
__global__ void __launch_bounds__(256) att_score_bwd_kernel(
    const float* __restrict__ dalpha, const float* __restrict__ dreg, long long dreg_ld_b,
    const float* __restrict__ alpha, long long alpha_ld_b, const float* __restrict__ att_enc,
    const float* __restrict__ att_dec, const float* __restrict__ wf, int B, int P, int A, int bt,
    float* __restrict__ de, float* __restrict__ dad) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* des = smem;  // [P]
  __shared__ float red[16];
  __shared__ float4 part4[256];
  const int b = blockIdx.y, tid = threadIdx.x;
  const bool active = b < bt;
  float s = 0.f;
  for (int p = tid; p < P; p += 256) {
    float da = dalpha[(long long)b * P + p];
    if (dreg) da += dreg[(long long)b * dreg_ld_b + p];
    const float al = alpha[(long long)b * alpha_ld_b + p];
    des[p] = da;
    s = fmaf(al, da, s);
  }
  s = block_sum(s, red);  // includes the barrier that publishes des
  for (int p = tid; p < P; p += 256) {
    const float al = alpha[(long long)b * alpha_ld_b + p];
    const float v = active ? al * (des[p] - s) : 0.f;
    des[p] = v;
    if (blockIdx.x == 0) de[(long long)b * P + p] = v;
  }
  __syncthreads();
  // d(att_dec)[b][a] = wf[a] * sum_p des[p] * [att_enc[b][p][a] + att_dec[b][a] > 0]:
  // 16 lanes x float4 cover the block's 64 columns, 16 p-groups stride over P
  const int c4 = tid & 15, pg = tid >> 4;
  const int a = blockIdx.x * 64 + c4 * 4;
  float4 acc = f4(0.f);
  if (a < A) {
    const float4 ad = *reinterpret_cast<const float4*>(att_dec + (long long)b * A + a);
    const float* base = att_enc + (long long)b * P * A + a;
#pragma unroll 4
    for (int p = pg; p < P; p += 16) {
      const float4 x = *reinterpret_cast<const float4*>(base + (long long)p * A) + ad;
      const float d = des[p];
      acc.x += x.x > 0.f ? d : 0.f;
      acc.y += x.y > 0.f ? d : 0.f;
      acc.z += x.z > 0.f ? d : 0.f;
      acc.w += x.w > 0.f ? d : 0.f;
    }
  }
  part4[pg * 16 + c4] = acc;
  __syncthreads();
  if (tid < 16 && blockIdx.x * 64 + tid * 4 < A) {
    float4 tot = part4[tid];
    for (int g = 1; g < 16; ++g) tot = tot + part4[g * 16 + tid];
    const int a0 = blockIdx.x * 64 + tid * 4;
    const float4 w = *reinterpret_cast<const float4*>(wf + a0);
    *reinterpret_cast<float4*>(dad + (long long)b * A + a0) = w * tot;
  }
}

extern "C" int capmi_att_score_bwd(const float* dalpha, const float* dreg, long long dreg_ld_b,
                                   const float* alpha, long long alpha_ld_b, const float* att_enc,
                                   const float* att_dec, const float* wf, int B, int P, int A,
                                   int bt, float* de, float* dad, void* stream) {
  CAPMI_REQUIRE(dalpha && alpha && att_enc && att_dec && wf && de && dad && B > 0 && P > 0 && A > 0,
                CAPMI_EINVAL);
  CAPMI_REQUIRE(P <= 16384 && A % 4 == 0, CAPMI_ERANGE);
  CAPMI_REQUIRE(aligned16(att_enc) && aligned16(att_dec) && aligned16(wf) && aligned16(dad), CAPMI_EALIGN);
  hipLaunchKernelGGL(att_score_bwd_kernel, dim3(cdiv(A, 64), B), dim3(256), P * sizeof(float),
                     as_stream(stream), dalpha, dreg, dreg_ld_b, alpha, alpha_ld_b, att_enc, att_dec,
                     wf, B, P, A, bt, de, dad);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

// hoisted d(att_enc) over all t + full_att weight/bias partials   grid (P/PCH, B)
// 256 threads = A/4 float4 columns x (256/(A/4)) p-groups; ad[t][b][:] cached in LDS
__global__ void __launch_bounds__(256) att_enc_grad_kernel(
    const float* __restrict__ de, const float* __restrict__ att_enc, const float* __restrict__ att_dec,
    const float* __restrict__ wf, int T, int B, int P, int A, float* __restrict__ datt_enc,
    float* __restrict__ wf_part, float* __restrict__ bf_part) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* ads = smem;                // [T][A]
  float* des = smem + (long long)T * A;  // [T][PCH]
  float* wred = des + T * PCH;      // [256][4]
  const int b = blockIdx.y, p0 = blockIdx.x * PCH, tid = threadIdx.x;
  const int np = min(PCH, P - p0);
  for (int i = tid; i < T * A; i += 256) {
    const int t = i / A, a = i - t * A;
    ads[i] = att_dec[((long long)t * B + b) * A + a];
  }
  for (int i = tid; i < T * PCH; i += 256) {
    const int t = i / PCH, pp = i - t * PCH;
    des[i] = pp < np ? de[((long long)t * B + b) * P + p0 + pp] : 0.f;
  }
  __syncthreads();
  const int A4 = A / 4;
  const int ngrp = 256 / A4 > 0 ? 256 / A4 : 1;
  float4 wacc = f4(0.f);
  for (int base = 0; base < A4; base += 256) {  // A4 may exceed 256 for large A
    const int c4 = base + (A4 >= 256 ? tid : tid % A4);
    const int pg = A4 >= 256 ? 0 : tid / A4;
    const int pstep = A4 >= 256 ? 1 : ngrp;
    if (c4 < A4 && pg < ngrp) {
      const int a = c4 * 4;
      const float4 w = *reinterpret_cast<const float4*>(wf + a);
      for (int pp = pg; pp < np; pp += pstep) {
        const long long o = ((long long)b * P + p0 + pp) * A + a;
        const float4 x = *reinterpret_cast<const float4*>(att_enc + o);
        float4 g = f4(0.f);
        for (int t = 0; t < T; ++t) {
          const float d = des[t * PCH + pp];
          const float4 s = x + *reinterpret_cast<const float4*>(ads + t * A + a);
          g.x += s.x > 0.f ? d : 0.f;
          g.y += s.y > 0.f ? d : 0.f;
          g.z += s.z > 0.f ? d : 0.f;
          g.w += s.w > 0.f ? d : 0.f;
          wacc = fma4(f4(d), relu4(s), wacc);
        }
        *reinterpret_cast<float4*>(datt_enc + o) = g * w;
      }
    }
  }
  // reduce wacc over p-groups sharing a column (only when A4 < 256)
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  if (A4 >= 256) {
    if (tid < A4) *reinterpret_cast<float4*>(wf_part + (long long)blk * A + tid * 4) = wacc;
  } else {
    reinterpret_cast<float4*>(wred)[tid] = wacc;
    __syncthreads();
    if (tid < A4) {
      float4 s = f4(0.f);
      for (int g = 0; g < ngrp; ++g) s = s + reinterpret_cast<float4*>(wred)[g * A4 + tid];
      *reinterpret_cast<float4*>(wf_part + (long long)blk * A + tid * 4) = s;
    }
  }
  if (tid == 0) {
    float s = 0.f;
    for (int i = 0; i < T * PCH; ++i) s += des[i];
    bf_part[blk] = s;
  }
}

extern "C" int capmi_att_enc_grad(const float* de, const float* att_enc, const float* att_dec,
                                  const float* wf, int T, int B, int P, int A, float* datt_enc,
                                  float* wf_part, float* bf_part, int* nblk_out, void* stream) {
  CAPMI_REQUIRE(de && att_enc && att_dec && wf && datt_enc && wf_part && bf_part && T > 0 && B > 0 &&
                    P > 0 && A > 0,
                CAPMI_EINVAL);
  CAPMI_REQUIRE(A % 4 == 0 && A / 4 <= 256, CAPMI_ERANGE);
  const size_t sh = ((size_t)T * A + T * PCH + 256 * 4) * sizeof(float);
  CAPMI_REQUIRE(sh <= 160 * 1024, CAPMI_ERANGE);
  const dim3 grid(cdiv(P, PCH), B);
  if (nblk_out) *nblk_out = (int)(grid.x * grid.y);
  if (sh > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)att_enc_grad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)sh);
  hipLaunchKernelGGL(att_enc_grad_kernel, grid, dim3(256), sh, as_stream(stream), de, att_enc,
                     att_dec, wf, T, B, P, A, datt_enc, wf_part, bf_part);
  CAPMI_LAUNCH_CHECK();
  return 0;
}
