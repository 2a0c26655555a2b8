// Fused kernels of the decoder's per-timestep recurrence (models/attention.py:260-281 and its
// autograd backward): three launches per timestep forward and three backward, where the generic
// path (decoder.hip + gemm_nt.hip) issues five each.
//
// Why: at B = 64 every per-step kernel is tiny (0.2-0.7 GFLOP), and a dispatch on the serialised
// decoder stream costs ~4 us however small the kernel (rocprofv3 trace: counter_add, colsum_stage2
// and splitk_reduce all take 4-5 us). The 240 per-step launches of a training step were ~2.3 ms of
// the decoder's 3.7 ms. What fuses:
//   * the split-K reduction of a GEMM and the pointwise op that consumes it (LSTM cell forward /
//     backward, the gate/context split of d(gate*awe), bias + sigmoid) run in the LAST workgroup to
//     finish a tile ("last arriver": the S partials are parked with write-through stores, one
//     agent-scope counter per tile, the last arriver adds them in split order -> deterministic);
//   * the LSTM's four gates of a hidden unit are made to land in one tile (gate-interleaved W rows,
//     16 units x 4 gates per 64-column tile) and in one lane (each wave covers all 64 columns), so
//     the cell runs in registers;
//   * W_hh h moves from the step's h-GEMM into the input GEMM (a second K segment), the score
//     is recomputed by every workgroup of the context kernel (no separate score launch), and the
//     score backward runs in the last workgroup of each row's context backward.
// MFMA (round 6): the fp32-accurate "x3" arithmetic of the other decoder GEMMs (CAPMI_GEMM_SPLIT3; gemm_x3.hip) --
// each fp32 fragment read from LDS is split exactly into three bf16 terms in registers, six products per 16 x 16 x 32
// block on v_mfma_f32_16x16x32_bf16 with fp32 accumulation (2.7x fewer MFMA cycles than v_mfma_f32_16x16x4_f32,
// whose fp32 products rounds 1-5 used here; error at or below the fp32 kernel's: tests/test_gpu_dstep.py).
#include "gemm_args.h"

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));
constexpr int DS_ROWS = 64;  // rows (batch) per tile
constexpr int DS_BK = 32;    // k per k-tile
constexpr int DS_LD = 36;    // LDS row stride in floats: 16-lane ds_read_b128 groups hit 64 banks
constexpr int kSc1d = 16;    // write-through / coherent cache policy of the parked partials
#ifndef DSTEP_SC1
#define DSTEP_SC1 1
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_d(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

struct DsArgs {
  capmi_dstep_seg seg[3];
  int kt_begin[4];  // first k-tile of segment i; kt_begin[nseg] = total k-tiles
  int nseg, M, N, S, gate_D, tiles_n;
  capmi_dstep_epi e;
  float* part;
  int* count;
};

__device__ __forceinline__ float sig_d(float x) { return 1.f / (1.f + expf(-x)); }

constexpr int DS_KG = 4;    // k-groups of four waves per workgroup (1024 threads)
constexpr int DS_KMAX = 4;  // k-tiles per k-group, all loaded up front (the host sizes S for it)

template <int NT, int EPI>
__global__ void __launch_bounds__(256 * DS_KG) dstep_gemm_kernel(const DsArgs a) {
  constexpr int NJ = NT / 16;             // 16-column MFMA tiles per wave (each wave: 16 rows x NT)
  constexpr int NW4 = NT * DS_BK / 4;     // float4 of one W k-tile
  constexpr int WPT = (NW4 + 255) / 256;  // ... per thread of a k-group
  constexpr int GBUF = (DS_ROWS + NT) * DS_LD;  // floats of one k-group's LDS tile (A rows, then W rows)
  static_assert(GBUF >= DS_ROWS * NT, "cross-group reduction reuses the staging tile");
  __shared__ __attribute__((aligned(16))) float lds[DS_KG * GBUF];
  __shared__ int last_flag;

  const int tid = threadIdx.x, grp = tid >> 8, t = tid & 255, lane = t & 63, w = t >> 6;
  const int S = a.S;
  const int s = blockIdx.x % S, tile = blockIdx.x / S;
  const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
  const int m0 = tm * DS_ROWS;
  const int M = a.M;
  const int KT = a.kt_begin[a.nseg];
  const int kt0 = (int)((long long)s * KT / S), n = (int)((long long)(s + 1) * KT / S) - kt0;
  // this k-group's k-tiles [g0, g0 + ng) of the workgroup's n; ngmax is uniform over the workgroup
  const int g0 = kt0 + n * grp / DS_KG, ng = kt0 + n * (grp + 1) / DS_KG - g0;
  const int ngmax = (n + DS_KG - 1) / DS_KG;
  float* As = lds + grp * GBUF;
  float* Ws = As + DS_ROWS * DS_LD;

  // staging: A rows ar, ar + 32 (16 B at k offset ak); W rows (t + 256 i) / 8
  const int ar = t >> 3, ak = (t & 7) * 4;
  long long wrow[WPT];
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    const int r = ((t + 256 * i) >> 3) % NT;
    wrow[i] = a.gate_D > 0 ? (long long)(r >> 4) * a.gate_D + tn * 16 + (r & 15) : (long long)tn * NT + r;
  }

  f32x4_t acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  struct Stage {
    float4 ra[2], rw[WPT];
  };
  auto load = [&](Stage& st, int gk) {
    // segment of this k-tile (selects, no dynamic indexing of the kernel-argument array)
    const int sg = (a.nseg > 1 && gk >= a.kt_begin[1]) ? ((a.nseg > 2 && gk >= a.kt_begin[2]) ? 2 : 1) : 0;
    const capmi_dstep_seg g = sg == 0 ? a.seg[0] : (sg == 1 ? a.seg[1] : a.seg[2]);
    const int kb = sg == 0 ? a.kt_begin[0] : (sg == 1 ? a.kt_begin[1] : a.kt_begin[2]);
    const int kk = (gk - kb) * DS_BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = m0 + ar + 32 * i;
      st.ra[i] = row < M ? *reinterpret_cast<const float4*>(g.A + row * g.lda + kk + ak) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < WPT; ++i)
      if (t + 256 * i < NW4)
        st.rw[i] = *reinterpret_cast<const float4*>(g.W + wrow[i] * g.ldw + kk + (((t + 256 * i) & 7) * 4));
  };
  auto store = [&](const Stage& st) {
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<float4*>(&As[(ar + 32 * i) * DS_LD + ak]) = st.ra[i];
#pragma unroll
    for (int i = 0; i < WPT; ++i)
      if (t + 256 * i < NW4)
        *reinterpret_cast<float4*>(&Ws[((t + 256 * i) >> 3) * DS_LD + ((t + 256 * i) & 7) * 4]) = st.rw[i];
  };
  // lane (q = lane/16, r = lane%16) reads k 8q .. 8q+7 of its row (the 16 x 16 x 32 bf16 operand layout; the same
  // k for A and W), splits the eight values into their three bf16 terms and runs the six products, smallest first
  typedef __bf16 bf16x8_d __attribute__((ext_vector_type(8)));
  typedef unsigned u32x4_d __attribute__((ext_vector_type(4)));
  auto split8 = [](const float4 v0, const float4 v1, bf16x8_d (&t)[3]) {
    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    u32x4_d w0, w1, w2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      unsigned wq[3];
      split3_pair(v[2 * q], v[2 * q + 1], wq);
      w0[q] = wq[0];
      w1[q] = wq[1];
      w2[q] = wq[2];
    }
    t[0] = __builtin_bit_cast(bf16x8_d, w0);
    t[1] = __builtin_bit_cast(bf16x8_d, w1);
    t[2] = __builtin_bit_cast(bf16x8_d, w2);
  };
  auto compute = [&]() {
    const int ko = 8 * (lane >> 4);
    bf16x8_d av[3];
    {
      const float* ar_ = &As[(16 * w + (lane & 15)) * DS_LD + ko];
      split8(*reinterpret_cast<const float4*>(ar_), *reinterpret_cast<const float4*>(ar_ + 4), av);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      bf16x8_d bv[3];
      const float* wr_ = &Ws[(16 * j + (lane & 15)) * DS_LD + ko];
      split8(*reinterpret_cast<const float4*>(wr_), *reinterpret_cast<const float4*>(wr_ + 4), bv);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1], bv[1], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv[2], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[2], bv[0], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv[1], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1], bv[0], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0], bv[0], acc[j], 0, 0, 0);
    }
  };
  // every k-tile of the group is requested before the first is multiplied: one memory round
  // trip per workgroup instead of one per two k-tiles
  Stage st[DS_KMAX];
#pragma unroll
  for (int i = 0; i < DS_KMAX; ++i)
    if (i < ng) load(st[i], g0 + i);
#pragma unroll
  for (int i = 0; i < DS_KMAX; ++i) {
    if (i < ngmax) {
      if (i < ng) store(st[i]);
      __syncthreads();
      if (i < ng) compute();
      __syncthreads();
    }
  }
  // k-groups 1.. hand their sums to group 0 (added in group order: deterministic)
  if (grp > 0) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      *reinterpret_cast<f32x4_t*>(&As[((w * NJ + j) * 64 + lane) * 4]) = acc[j];
  }
  __syncthreads();
  if (grp == 0) {
#pragma unroll
    for (int g = 1; g < DS_KG; ++g)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[j] += *reinterpret_cast<const f32x4_t*>(&lds[g * GBUF + ((w * NJ + j) * 64 + lane) * 4]);
  }

  if (S > 1) {
    // park this split's partial (lane-linear: the last arriver reads it back in the same layout)
    const long long tb = (long long)tile * S * (DS_ROWS * NT);
    if (grp == 0) {
      const auto rs = rsrc_d(a.part + tb + (long long)s * (DS_ROWS * NT), DS_ROWS * NT * 4);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        u32x4 v;
        v.x = __float_as_uint(acc[j][0]);
        v.y = __float_as_uint(acc[j][1]);
        v.z = __float_as_uint(acc[j][2]);
        v.w = __float_as_uint(acc[j][3]);
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, ((w * NJ + j) * 64 + lane) * 16, 0, kSc1d);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
      // DSTEP_SC1 (round 6): the hand-off form of MI355X_MICROARCH.md's "Valid forms besides Guideline 16", table
      // row 1: every partial byte stored and loaded with 16-B sc1 buffer ops, every storing wave
      // drained (vmcnt(0)) before the barrier above, ONE lane's relaxed agent-scope add for the workgroup, the
      // workgroup whose add returns S - 1 learns it is last and its other waves load after the barrier below; one
      // workgroup per CU (16 waves of 84-86 VGPRs: 5 waves per SIMD fit, a second workgroup's 4 do not).
      // DSTEP_SC1=0: acq_rel at agent scope (an L2 write-back per workgroup) and an acquire in the last arriver
      const int old = __hip_atomic_fetch_add(a.count + tile, 1, DSTEP_SC1 ? __ATOMIC_RELAXED : __ATOMIC_ACQ_REL,
                                             __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == S - 1;
      if (last) __hip_atomic_store(a.count + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = last;
    }
    __syncthreads();
    if (!last_flag || grp != 0) return;
    if (!DSTEP_SC1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the fenced form's acquire)
    const auto rt = rsrc_d(a.part + tb, (unsigned)(S * DS_ROWS * NT * 4));
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    int s2 = 0;
    for (; s2 + 8 <= S; s2 += 8) {
      f32x4_t v[8][NJ];
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          v[u][j] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rt, ((s2 + u) * DS_ROWS * NT + (w * NJ + j) * 64 * 4 + lane * 4) * 4, 0, kSc1d));
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] += v[u][j];
    }
    for (; s2 < S; ++s2)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[j] += __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rt, (s2 * DS_ROWS * NT + (w * NJ + j) * 64 * 4 + lane * 4) * 4, 0, kSc1d));
  } else if (grp != 0) {
    return;
  }

  // epilogue: lane holds rows 16w + 4(lane/16) + r (r < 4) of column 16j + lane%16 of tile j
  const capmi_dstep_epi& e = a.e;
  const int rbase = m0 + 16 * w + 4 * (lane >> 4);
  if (EPI == CAPMI_DSTEP_STORE2 || EPI == CAPMI_DSTEP_GATE_BWD) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = tn * NT + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + r;
        if (row >= M) continue;
        const float v = acc[j][r];
        if (EPI == CAPMI_DSTEP_STORE2) {
          if (col < e.nsplit) {
            e.out0[row * e.ld0 + col] = v + (e.bias0 ? e.bias0[col] : 0.f);
          } else {
            const int c1 = col - e.nsplit;
            const float x = v + (e.bias1 ? e.bias1[c1] : 0.f);
            e.out1[row * e.ld1 + c1] = e.act1 ? sigmoidf_(x) : x;
          }
        } else {
          const long long o = (long long)row * a.N + col;
          const float g = e.gate[o];
          e.dawe_out[o] = v * g;
          e.dgp[o] = v * e.awe[o] * g * (1.f - g);
        }
      }
    }
  } else if (EPI == CAPMI_DSTEP_LSTM_FWD) {
    // NT = 64, gate-interleaved: tile j = gate q of hidden unit 16 tn + lane%16
    const int D = e.D, u = tn * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = rbase + r;
      if (row >= M) continue;
      const long long o = (long long)row * 4 * D + u;
      float g[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) g[q] = acc[q & (NJ - 1)][r] + (e.xemb ? e.xemb[o + q * D] : 0.f);
      const float ig = sig_d(g[0]), fg = sig_d(g[1]), cg = tanhf(g[2]), og = sig_d(g[3]);
      const long long i = (long long)row * D + u;
      const float c = fg * e.c_prev[i] + ig * cg;
      e.c_out[i] = c;
      e.h_out[i] = og * tanhf(c);
      e.act_out[o] = ig;
      e.act_out[o + D] = fg;
      e.act_out[o + 2 * D] = cg;
      e.act_out[o + 3 * D] = og;
    }
  } else {  // LSTM_BWD: columns = hidden units
    const int D = e.D;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int u = tn * NT + 16 * j + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + r;
        if (row >= M) continue;
        const long long i = (long long)row * D + u, o = (long long)row * 4 * D + u;
        if (row >= e.bt) {
          e.dgates[o] = 0.f;
          e.dgates[o + D] = 0.f;
          e.dgates[o + 2 * D] = 0.f;
          e.dgates[o + 3 * D] = 0.f;
          e.dc_out[i] = 0.f;
          continue;
        }
        const float dh = acc[j][r] + (e.dhd ? e.dhd[i] : 0.f);
        float dc = e.dc_in ? e.dc_in[i] : 0.f;
        const float ig = e.act[o], fg = e.act[o + D], cg = e.act[o + 2 * D], og = e.act[o + 3 * D];
        const float tc = tanhf(e.c_cur[i]);
        const float d_o = dh * tc * og * (1.f - og);
        dc += dh * og * (1.f - tc * tc);
        e.dgates[o] = dc * cg * ig * (1.f - ig);
        e.dgates[o + D] = dc * e.c_prev[i] * fg * (1.f - fg);
        e.dgates[o + 2 * D] = dc * ig * (1.f - cg * cg);
        e.dgates[o + 3 * D] = d_o;
        e.dc_out[i] = dc * fg;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// score + softmax + context + gate, one timestep: grid (E / 512, B), 512 threads. Every workgroup
// of row b recomputes the P scores (same per-row sum order as att_score_fwd), so there is no score
// launch and no e[] round trip. The context's enc rows are requested together with the score rows
// (they do not depend on the softmax), so the kernel waits on memory about twice: ad, then
// att_enc + enc. Context: 128 float4 columns x 4 p-groups (att_softmax_ctx_fwd's order).
// ---------------------------------------------------------------------------------------------
constexpr int AF_T = 512, AF_ECH = 512, AF_R = 7;  // threads, columns per workgroup, score rows per wave (P <= 56)
constexpr int AF_CR = 14;                          // context rows per thread in flight (P <= 56)

__global__ void __launch_bounds__(AF_T) att_fwd_fused_kernel(
    const float* __restrict__ att_enc, const float* __restrict__ ad_in, int S_a, long long slab_a,
    const float* __restrict__ bias_da, float* __restrict__ ad_out, const float* __restrict__ wf,
    const float* __restrict__ bf, const float* __restrict__ enc, const float* __restrict__ gate_in, int S_g,
    long long slab_g, const float* __restrict__ bias_fb, float* __restrict__ gate_out, int B, int P, int A, int E,
    int bt, float* __restrict__ alpha_out, long long alpha_ld_b, float* __restrict__ awe_out,
    float* __restrict__ x_out, long long ld_x) {
  constexpr int C4 = AF_ECH / 4, PG = AF_T / C4;  // 128 columns x 4 p-groups
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* ad = smem;                                  // [A]
  float* al = smem + A;                              // [P] scores -> alphas
  float4* part = reinterpret_cast<float4*>(al + ((P + 3) & ~3));  // [PG][C4]
  __shared__ float red[16];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int c4 = tid % C4, pg = tid / C4;
  const int c = blockIdx.x * AF_ECH + c4 * 4;
  // context operand: rows pg, pg + 4, ... of this thread's column (issued first, used last)
  float4 ev[AF_CR];
#pragma unroll
  for (int r = 0; r < AF_CR; ++r) {
    const int p = pg + PG * r;
    ev[r] = (c < E && p < P) ? *reinterpret_cast<const float4*>(enc + ((long long)b * P + p) * E + c) : f4(0.f);
  }
  // att_dec: final, or bias + the S_a split-K partials of the h-GEMM (att_score_fwd's sum order)
  for (int i = tid; i < A; i += AF_T) {
    const long long o = (long long)b * A + i;
    const float v = S_a > 0 ? slab_sum(ad_in + o, S_a, slab_a, bias_da ? bias_da[i] : 0.f) : ad_in[o];
    ad[i] = v;
    if (ad_out && blockIdx.x == 0) ad_out[o] = v;
  }
  __syncthreads();
  const float b0 = bf ? bf[0] : 0.f;
  // scores: wave wid owns rows wid, wid + 8, ... (all loads in flight)
  float sc[AF_R];
#pragma unroll
  for (int r = 0; r < AF_R; ++r) sc[r] = 0.f;
  for (int i = lane * 4; i < A; i += 256) {
    const float4 d = *reinterpret_cast<const float4*>(ad + i);
    const float4 wv = *reinterpret_cast<const float4*>(wf + i);
    float4 x[AF_R];
#pragma unroll
    for (int r = 0; r < AF_R; ++r) {
      const int p = wid + 8 * r;
      x[r] = p < P ? *reinterpret_cast<const float4*>(att_enc + ((long long)b * P + p) * A + i) : f4(0.f);
    }
#pragma unroll
    for (int r = 0; r < AF_R; ++r) sc[r] += dot4(relu4(x[r] + d), wv);
  }
#pragma unroll
  for (int r = 0; r < AF_R; ++r) sc[r] = wave_sum(sc[r]);
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < AF_R; ++r)
      if (wid + 8 * r < P) al[wid + 8 * r] = sc[r] + b0;
  }
  __syncthreads();
  float m = -INFINITY;
  for (int p = tid; p < P; p += AF_T) m = fmaxf(m, al[p]);
  m = block_max(m, red);
  float s = 0.f;
  for (int p = tid; p < P; p += AF_T) {
    const float v = expf(al[p] - m);
    al[p] = v;
    s += v;
  }
  s = block_sum(s, red);
  const float inv = 1.f / s;
  for (int p = tid; p < P; p += AF_T) {
    const float v = al[p] * inv;
    al[p] = v;
    if (alpha_out && blockIdx.x == 0) alpha_out[(long long)b * alpha_ld_b + p] = b < bt ? v : 0.f;
  }
  __syncthreads();
  float4 acc = f4(0.f);
#pragma unroll
  for (int r = 0; r < AF_CR; ++r) {
    const int p = pg + PG * r;
    if (p < P) acc = fma4(f4(al[p]), ev[r], acc);
  }
  part[pg * C4 + c4] = acc;
  __syncthreads();
  if (pg == 0 && c < E) {
    float4 awe = part[c4];
#pragma unroll
    for (int g = 1; g < PG; ++g) awe = awe + part[g * C4 + c4];
    const long long o = (long long)b * E + c;
    if (awe_out) *reinterpret_cast<float4*>(awe_out + o) = awe;
    float4 gv;
    if (S_g > 0) {  // sigmoid(bias + partials): att_softmax_ctx_fwd's order
      gv = slab_sum(reinterpret_cast<const float4*>(gate_in + o), S_g, slab_g / 4,
                    *reinterpret_cast<const float4*>(bias_fb + c));
      gv = make_float4(sigmoidf_(gv.x), sigmoidf_(gv.y), sigmoidf_(gv.z), sigmoidf_(gv.w));
      if (gate_out) *reinterpret_cast<float4*>(gate_out + o) = gv;
    } else {
      gv = *reinterpret_cast<const float4*>(gate_in + o);
    }
    *reinterpret_cast<float4*>(x_out + (long long)b * ld_x + c) = gv * awe;
  }
}

// ---------------------------------------------------------------------------------------------
// context + softmax + score backward, one timestep: one 1024-thread workgroup per row b (no
// cross-workgroup step). d(gate*awe) is final (S = 0) or the S split-K partials of its GEMM, split
// into dawe = d * gate (LDS, and dawe_out) and dgp = d * awe * gate' as att_ctx_bwd does; then
// dalpha[p] = dawe . enc[b][p] (att_ctx_bwd's per-row order), the softmax backward with the
// regulariser term, and dad[a] = wf[a] sum_p de[p] [att_enc + att_dec > 0] in att_score_bwd's order
// (per column 16 p-groups, summed in group order). Bit-identical to att_ctx_bwd + att_score_bwd.
// ---------------------------------------------------------------------------------------------
constexpr int AB_T = 1024;

__global__ void __launch_bounds__(AB_T) att_bwd_fused_kernel(
    const float* __restrict__ dx, int S, long long slab, const float* __restrict__ gate,
    const float* __restrict__ awe, float* __restrict__ dgp, float* __restrict__ dawe_out,
    const float* __restrict__ enc, const float* __restrict__ alpha, long long alpha_ld_b,
    const float* __restrict__ dreg, long long dreg_ld_b, const float* __restrict__ att_enc,
    const float* __restrict__ att_dec, const float* __restrict__ wf, int B, int P, int A, int E, int bt,
    float* __restrict__ de, float* __restrict__ dad) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* dawe = smem;                          // [E]
  float* des = smem + E;                       // [P]
  float4* part4 = reinterpret_cast<float4*>(des + ((P + 3) & ~3));  // [16][64]
  __shared__ float red[16];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int c = tid * 4; c < E; c += AB_T * 4) {
    const long long o = (long long)b * E + c;
    float4 dw;
    if (S > 0) {
      const float4 d = slab_sum(reinterpret_cast<const float4*>(dx + slab + o), S - 1, slab / 4,
                                *reinterpret_cast<const float4*>(dx + o));
      dw = d;
      if (gate) {
        const float4 g = *reinterpret_cast<const float4*>(gate + o);
        dw = d * g;
        if (dgp) {
          const float4 a = *reinterpret_cast<const float4*>(awe + o);
          float4 r;
          r.x = d.x * a.x * g.x * (1.f - g.x);
          r.y = d.y * a.y * g.y * (1.f - g.y);
          r.z = d.z * a.z * g.z * (1.f - g.z);
          r.w = d.w * a.w * g.w * (1.f - g.w);
          *reinterpret_cast<float4*>(dgp + o) = r;
        }
      }
      if (dawe_out) *reinterpret_cast<float4*>(dawe_out + o) = dw;
    } else {
      dw = *reinterpret_cast<const float4*>(dx + o);
    }
    *reinterpret_cast<float4*>(dawe + c) = dw;
  }
  __syncthreads();
  // 16 waves, rows wid, wid + 16, ...: two rows' loads in flight per wave
  for (int p0 = wid; p0 < P; p0 += 32) {
    float acc[2] = {0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int p = p0 + 16 * r;
      if (p < P) {
        const float* row = enc + ((long long)b * P + p) * E;
#pragma unroll 8
        for (int c = lane * 4; c < E; c += 256)
          acc[r] += dot4(*reinterpret_cast<const float4*>(row + c), *reinterpret_cast<const float4*>(dawe + c));
      }
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) acc[r] = wave_sum(acc[r]);
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < 2; ++r)
        if (p0 + 16 * r < P) des[p0 + 16 * r] = acc[r];
    }
  }
  __syncthreads();
  const bool active = b < bt;
  float s = 0.f;
  for (int p = tid; p < P; p += AB_T) {
    float da = des[p];
    if (dreg) da += dreg[(long long)b * dreg_ld_b + p];
    des[p] = da;
    s = fmaf(alpha[(long long)b * alpha_ld_b + p], da, s);
  }
  s = block_sum(s, red);
  for (int p = tid; p < P; p += AB_T) {
    const float al = alpha[(long long)b * alpha_ld_b + p];
    const float v = active ? al * (des[p] - s) : 0.f;
    des[p] = v;
    de[(long long)b * P + p] = v;
  }
  __syncthreads();
  // 256 columns per pass: 64 float4 columns x 16 p-groups
  const int A4 = A / 4;
  for (int cb = 0; cb < A4; cb += 64) {
    const int c4 = cb + (tid & 63), pg = tid >> 6;
    float4 acc = f4(0.f);
    if (c4 < A4) {
      const float4 adv = *reinterpret_cast<const float4*>(att_dec + (long long)b * A + 4 * c4);
      const float* base = att_enc + (long long)b * P * A + 4 * c4;
#pragma unroll 4
      for (int p = pg; p < P; p += 16) {
        const float4 x = *reinterpret_cast<const float4*>(base + (long long)p * A) + adv;
        const float d = des[p];
        acc.x += x.x > 0.f ? d : 0.f;
        acc.y += x.y > 0.f ? d : 0.f;
        acc.z += x.z > 0.f ? d : 0.f;
        acc.w += x.w > 0.f ? d : 0.f;
      }
    }
    part4[pg * 64 + (tid & 63)] = acc;
    __syncthreads();
    if (tid < 64 && c4 < A4) {
      float4 tot = part4[tid];
      for (int g = 1; g < 16; ++g) tot = tot + part4[g * 64 + tid];
      *reinterpret_cast<float4*>(dad + (long long)b * A + 4 * c4) = *reinterpret_cast<const float4*>(wf + 4 * c4) * tot;
    }
    __syncthreads();
  }
}

template <int NT>
int launch_dstep(const DsArgs& a, int mode, int blocks, hipStream_t st) {
  const dim3 g(blocks), bl(256 * DS_KG);
  switch (mode) {
    case CAPMI_DSTEP_STORE2: hipLaunchKernelGGL((dstep_gemm_kernel<NT, CAPMI_DSTEP_STORE2>), g, bl, 0, st, a); break;
    case CAPMI_DSTEP_LSTM_FWD: hipLaunchKernelGGL((dstep_gemm_kernel<NT, CAPMI_DSTEP_LSTM_FWD>), g, bl, 0, st, a); break;
    case CAPMI_DSTEP_LSTM_BWD: hipLaunchKernelGGL((dstep_gemm_kernel<NT, CAPMI_DSTEP_LSTM_BWD>), g, bl, 0, st, a); break;
    default: hipLaunchKernelGGL((dstep_gemm_kernel<NT, CAPMI_DSTEP_GATE_BWD>), g, bl, 0, st, a); break;
  }
  return 0;
}

}  // namespace

extern "C" int capmi_dstep_gemm(const capmi_dstep_seg* segs, int nseg, int M, int N, int nt, int S, int gate_D,
                                const capmi_dstep_epi* epi, float* part, long long part_floats, int* counters,
                                int ncounters, void* stream) {
  CAPMI_REQUIRE(segs && epi && nseg >= 1 && nseg <= 3 && M > 0 && N > 0 && S >= 1, CAPMI_EINVAL);
  CAPMI_REQUIRE(nt == 16 || nt == 32 || nt == 64, CAPMI_EINVAL);
  CAPMI_REQUIRE(N % nt == 0, CAPMI_ERANGE);
  CAPMI_REQUIRE(epi->mode >= CAPMI_DSTEP_STORE2 && epi->mode <= CAPMI_DSTEP_GATE_BWD, CAPMI_EINVAL);
  DsArgs a{};
  int kt = 0;
  for (int i = 0; i < nseg; ++i) {
    const capmi_dstep_seg& g = segs[i];
    CAPMI_REQUIRE(g.A && g.W && g.K > 0, CAPMI_EINVAL);
    CAPMI_REQUIRE(g.K % DS_BK == 0, CAPMI_ERANGE);
    CAPMI_REQUIRE(aligned16(g.A) && aligned16(g.W) && g.lda % 4 == 0 && g.ldw % 4 == 0, CAPMI_EALIGN);
    CAPMI_REQUIRE(g.lda >= g.K && g.ldw >= g.K, CAPMI_EINVAL);
    a.seg[i] = g;
    a.kt_begin[i] = kt;
    kt += g.K / DS_BK;
  }
  a.kt_begin[nseg] = kt;
  for (int i = nseg + 1; i < 4; ++i) a.kt_begin[i] = kt;
  for (int i = nseg; i < 3; ++i) a.seg[i] = segs[0];
  S = std::min(std::max(S, (int)cdiv(kt, DS_KG * DS_KMAX)), kt);
  const int mode = epi->mode;
  if (mode == CAPMI_DSTEP_LSTM_FWD) {
    CAPMI_REQUIRE(nt == 64 && gate_D > 0 && gate_D % 16 == 0 && N == 4 * gate_D && epi->D == gate_D, CAPMI_EINVAL);
    CAPMI_REQUIRE(epi->c_prev && epi->h_out && epi->c_out && epi->act_out, CAPMI_EINVAL);
  } else {
    CAPMI_REQUIRE(gate_D == 0, CAPMI_EINVAL);
  }
  if (mode == CAPMI_DSTEP_STORE2)
    CAPMI_REQUIRE(epi->out0 && (epi->nsplit >= N || epi->out1) && epi->nsplit % nt == 0, CAPMI_EINVAL);
  if (mode == CAPMI_DSTEP_LSTM_BWD)
    CAPMI_REQUIRE(epi->D == N && epi->act && epi->c_prev && epi->c_cur && epi->dgates && epi->dc_out, CAPMI_EINVAL);
  if (mode == CAPMI_DSTEP_GATE_BWD) CAPMI_REQUIRE(epi->gate && epi->awe && epi->dawe_out && epi->dgp, CAPMI_EINVAL);
  a.nseg = nseg;
  a.M = M;
  a.N = N;
  a.S = S;
  a.gate_D = gate_D;
  a.tiles_n = gate_D > 0 ? gate_D / 16 : N / nt;
  const long long tiles = (long long)cdiv(M, DS_ROWS) * a.tiles_n;
  if (S > 1) {
    CAPMI_REQUIRE(part && counters && aligned16(part), CAPMI_EINVAL);
    CAPMI_REQUIRE(part_floats >= tiles * S * DS_ROWS * nt && ncounters >= tiles, CAPMI_ERANGE);
    CAPMI_REQUIRE((long long)S * DS_ROWS * nt * 4 < (1LL << 31), CAPMI_ERANGE);
  }
  a.e = *epi;
  a.part = part;
  a.count = counters;
  const long long blocks = tiles * S;
  CAPMI_REQUIRE(blocks < (1LL << 31), CAPMI_ERANGE);
  hipStream_t st = as_stream(stream);
  if (nt == 16)
    launch_dstep<16>(a, mode, (int)blocks, st);
  else if (nt == 32)
    launch_dstep<32>(a, mode, (int)blocks, st);
  else
    launch_dstep<64>(a, mode, (int)blocks, st);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_att_fwd_fused(const float* att_enc, const float* ad, int S_a, long long slab_a,
                                   const float* bias_da, float* ad_out, const float* wf, const float* bf,
                                   const float* enc, const float* gate, int S_g, long long slab_g, const float* bias_fb,
                                   float* gate_out, int B, int P, int A, int E, int bt, float* alpha_out,
                                   long long alpha_ld_b, float* awe_out, float* x_out, long long ld_x, void* stream) {
  CAPMI_REQUIRE(att_enc && ad && wf && enc && gate && x_out && B > 0 && P > 0 && A > 0 && E > 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(S_a >= 0 && S_g >= 0 && (S_g == 0 || (bias_fb && aligned16(bias_fb) && slab_g % 4 == 0)), CAPMI_EINVAL);
  CAPMI_REQUIRE(P <= 8 * AF_R && P <= 4 * AF_CR, CAPMI_ERANGE);
  CAPMI_REQUIRE(A % 4 == 0 && E % 4 == 0 && ld_x % 4 == 0 && A + P + 4 <= 16384, CAPMI_ERANGE);
  CAPMI_REQUIRE(aligned16(att_enc) && aligned16(ad) && aligned16(wf) && aligned16(enc) && aligned16(gate) &&
                    aligned16(x_out) && (!awe_out || aligned16(awe_out)),
                CAPMI_EALIGN);
  const size_t sh = (A + ((P + 3) & ~3) + AF_T * 4) * sizeof(float);
  hipLaunchKernelGGL(att_fwd_fused_kernel, dim3(cdiv(E, AF_ECH), B), dim3(AF_T), sh, as_stream(stream), att_enc,
                     ad, S_a, slab_a, bias_da, ad_out, wf, bf, enc, gate, S_g, slab_g, bias_fb, gate_out, B, P, A, E,
                     bt, alpha_out, alpha_ld_b, awe_out, x_out, ld_x);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_att_bwd_fused(const float* dx, int S, long long slab, const float* gate, const float* awe,
                                   float* dgp, float* dawe_out, const float* enc, const float* alpha,
                                   long long alpha_ld_b, const float* dreg, long long dreg_ld_b, const float* att_enc,
                                   const float* att_dec, const float* wf, int B, int P, int A, int E, int bt, float* de,
                                   float* dad, void* stream) {
  CAPMI_REQUIRE(dx && enc && alpha && att_enc && att_dec && wf && de && dad && B > 0 && P > 0 && A > 0 && E > 0 &&
                    S >= 0,
                CAPMI_EINVAL);
  CAPMI_REQUIRE(!dgp || (gate && awe), CAPMI_EINVAL);
  CAPMI_REQUIRE(A % 4 == 0 && E % 4 == 0 && slab % 4 == 0, CAPMI_ERANGE);
  CAPMI_REQUIRE(aligned16(dx) && aligned16(enc) && aligned16(att_enc) && aligned16(att_dec) && aligned16(wf) &&
                    aligned16(dad) && (!gate || aligned16(gate)) && (!awe || aligned16(awe)) &&
                    (!dgp || aligned16(dgp)) && (!dawe_out || aligned16(dawe_out)),
                CAPMI_EALIGN);
  const size_t sh = (E + ((P + 3) & ~3) + 16 * 64 * 4) * sizeof(float);
  CAPMI_REQUIRE(sh <= 64 * 1024, CAPMI_ERANGE);
  hipLaunchKernelGGL(att_bwd_fused_kernel, dim3(B), dim3(AB_T), sh, as_stream(stream), dx, S, slab, gate, awe, dgp,
                     dawe_out, enc, alpha, alpha_ld_b, dreg, dreg_ld_b, att_enc, att_dec, wf, B, P, A, E, bt, de, dad);
  CAPMI_LAUNCH_CHECK();
  return 0;
}
