// bf16-in / bf16-out implicit-GEMM convolution for the bf16 configuration (BASELINE config 5):
// activations and packed conv weights are bf16 in HBM, products on v_mfma_f32_32x32x16_bf16 with
// fp32 accumulation, the output rounded to bf16 (RNE) once, train-mode BN statistics in fp32 from
// the stored (rounded) values. Replaces the Conv2d calls of torchvision's ResNet-101
// (models/encoder.py:88-91,107) when the encoder runs in bf16.
//
// vs the fp32 kernel (gemm_nt.hip), whose structure (2x2 waves, two register prefetch stages,
// LDS double buffer, stream-K hand-off, XCD groups, slice statistics) it keeps:
//   * BK = 64 (K % 64 == 0: every ResNet conv but conv1, Cin % 64 == 0, so a k-tile never
//     straddles a (kh, kw) tap); one 16-B load = 8 consecutive k of one row;
//   * loads are raw buffer loads over the whole operand: a masked slot (padding tap, row >= M)
//     gets an offset past the buffer's end and reads zeros, so there is no select, no 64-bit
//     address arithmetic and no prologue VALU between the loads and the LDS stores (the BN
//     apply + ReLU of the conv input is materialised once per tensor: capmi_bn_relu_bf16);
//   * LDS rows of 72 bf16 (144 B): the 16-lane groups of ds_read_b128 / 8-lane groups of
//     ds_write_b128 hit 64 distinct banks; lane (r, h) reads k 16g+8h..+7 of row r, the operand
//     layout of the 32x32x16 bf16 MFMA;
//   * tiles 128x128 (wave 64x64: 4 MFMAs per 4 ds_read_b128) or 128x64;
//   * round 5: for K <= 256 a one-stage 128x64 form at four workgroups per CU (ST = 1 below), and the
//     store-only epilogue leaves through LDS as 16-B row chunks.
#include "gemm_args.h"

namespace {

constexpr int BKH = 64;      // k per tile (bf16 elements)
constexpr int SBH = BKH + 8;  // LDS row stride (elements)
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr unsigned kOOB = 0x80000000u;  // buffer offset past every operand: the load returns 0
constexpr int kSc1h = 16;
#ifndef BF16_SKIP  // timing-only builds (wrong results): 1 no C stores, 2 no MFMAs, 4 no operand loads
#define BF16_SKIP 0
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ unsigned short bf16_bits(float x) {
  return __builtin_bit_cast(unsigned short, (__bf16)x);  // RNE
}
__device__ __forceinline__ float bf16_val(unsigned short b) {
  return __uint_as_float((unsigned)b << 16);
}
__device__ __forceinline__ float lo_bf(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(unsigned w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ unsigned pack_bf(float lo, float hi) {
  return (unsigned)bf16_bits(lo) | ((unsigned)bf16_bits(hi) << 16);
}

// s_barrier once this wave has at most N vector-memory operations (the later k-tiles' DMA) outstanding
template <int N>
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// ST = LDS stages.
//  * ST = 1 (round 5, 128x64 data-parallel only): one LDS stage, one register stage ahead, four workgroups per CU --
//    the short-k 1x1 convs, where a tile's few k-tiles leave no steady state to pipeline and more resident tiles hide
//    the load latency instead.
//  * ST = 2 with stream-K (opt-in, CAPMI_BF16_SK=1): two register stages ahead, LDS double buffer, two workgroups per CU.
//  * ST = 2 or 4 data-parallel (round 6): an LDS-DMA ring of ST k-tiles, ST - 1 in flight. The operands go straight
//    from the buffer loads into LDS (buffer_load_dwordx4 ... lds: no staging registers, no ds_write), rows of 64 bf16
//    without padding: lane l of a wave-instruction fills 16-B slot l % 8 of row l / 8 of a 1 KiB block, and that
//    slot holds logical k-chunk (l % 8) ^ ((row / 2) % 8) (the swizzle is on the source address), so each 16-lane
//    group of the 32x32x16 ds_read_b128 (lane: row l % 32, chunk 2 g + l / 32) covers 64 distinct banks. One barrier
//    per k-tile, behind a counted vmcnt that leaves the later stages' DMA in flight. On 128-column tiles 512 threads
//    (waves 2 x 4, wave tile 64 x 32), so a SIMD holds two waves of a workgroup: 75 VGPRs instead of the register
//    form's 212, two workgroups per CU at ST = 2 (64 KiB of LDS each), one at ST = 4 (128 KiB).
// Otherwise 256 threads (waves 2 x 2, wave tile 64 x BN / 2).
constexpr bool bf16_dma(int ST, bool SK) { return ST >= 2 && !SK; }
constexpr int bf16_threads(int BN, int ST, bool SK) { return bf16_dma(ST, SK) && BN == 128 ? 512 : 256; }
constexpr int bf16_waves(int BM, int BN, int ST, bool SK) {  // waves per SIMD the LDS leaves room for
  return ST == 1 ? 4 : !bf16_dma(ST, SK) ? 2 : (160 * 1024 / (ST * (BM + BN) * 128)) * bf16_threads(BN, ST, SK) / 256;
}

template <int BM, int BN, int AMODE, bool SK, int ST>
__global__ void __launch_bounds__((bf16_threads(BN, ST, SK))) __attribute__((amdgpu_waves_per_eu(bf16_waves(BM, BN, ST, SK))))
gemm_bf16_kernel(const GemmArgs args) {
  constexpr int NT = bf16_threads(BN, ST, SK), WGN = NT / 128;  // waves along N (2 along M)
  constexpr int WM = BM / 2, WN = BN / WGN, TM = WM / 32, TN = WN / 32;
  constexpr int NA = BM * BKH / 8 / NT, NB = BN * BKH / 8 / NT;
  static_assert(NA >= 1 && NB >= 1 && WM == 64 && TN >= 1, "tile");
  constexpr bool DMA = bf16_dma(ST, SK);
  static_assert(!DMA || NA <= 4, "DMA offsets");
  constexpr int SB = DMA ? BKH : SBH;  // LDS row stride (elements)
  __shared__ __attribute__((aligned(1024))) __bf16 lds_tile[ST * (BM + BN) * SB];
  __bf16* const As = lds_tile;                 // [ST][BM * SB]
  __bf16* const Bs = lds_tile + ST * BM * SB;  // [ST][BN * SB]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm0 = (wid / WGN) * WM, wn0 = (wid % WGN) * WN;
  const int lr = lane & 31, lh = lane >> 5;
  // k offset of this thread's 16-B chunk inside a k-tile (its rows are (tid >> 3) + NT / 8 i: DMA swizzle (tid >> 4) % 8)
  const int kc = DMA ? (((tid & 7) ^ ((tid >> 4) & 7)) * 8) : (tid & 7) * 8;

  f32x16 acc[TM][TN];

  // operand walk of the current tile (set by begin_tile), the two register stages of the prefetch
  const capmi_gemm_problem& P0 = args.p[0];
  const unsigned a_bytes = AMODE == 2 ? (unsigned)((long long)P0.cN * P0.cH * P0.cW * P0.cCin * 2)
                                      : (unsigned)((long long)P0.M * P0.lda * 2);
  const auto ra = rsrc_of(P0.A, a_bytes);
  const auto rb = rsrc_of(P0.B, (unsigned)((long long)P0.N * P0.ldb * 2));
  unsigned a_off[NA];  // dense: byte offset of (row, kc); conv: element offset of the image
  int a_ih0[NA], a_iw0[NA];
  bool a_ok[NA];
  unsigned b_off[NB];
  int c_ci = 0, c_kh = 0, c_kw = 0;  // conv k walk, advanced BKH per k-tile
  int t_lo = 0, t_hi = 0;             // k range of the current tile
  struct Stage {
    u32x4_t ra[NA], rb[NB];
  };
  Stage s0, s1;

  auto begin_tile = [&](const capmi_gemm_problem& P, int m0, int n0, int k_lo, int k_hi) {
    const int M = P.M, N = P.N;
    t_lo = k_lo;
    t_hi = k_hi;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = m0 + ((tid + i * NT) >> 3);
      a_ok[i] = row < M;
      if (AMODE == 0) {
        a_off[i] = a_ok[i] ? (unsigned)(((long long)row * P.lda + kc) * 2) : kOOB;
        a_ih0[i] = a_iw0[i] = 0;
      } else {
        const int hw = P.cHo * P.cWo;
        const int rr = a_ok[i] ? row : 0;
        const int n = rr / hw, rem = rr - n * hw;
        const int oh = rem / P.cWo, ow = rem - oh * P.cWo;
        a_ih0[i] = oh * P.cStride - P.cPad;
        a_iw0[i] = ow * P.cStride - P.cPad;
        a_off[i] = (unsigned)(n * P.cH * P.cW);  // pixel index of the image's (0, 0)
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int n = n0 + ((tid + i * NT) >> 3);
      b_off[i] = n < N ? (unsigned)(((long long)n * P.ldb + kc) * 2) : kOOB;
    }
    if (AMODE == 2) {
      const int kpos = k_lo / P.cCin;
      c_ci = k_lo - kpos * P.cCin;
      c_kh = kpos / P.cKW;
      c_kw = kpos - c_kh * P.cKW;
    }
  };
  auto load_tile = [&](Stage& st, int kt) {
    const int k = t_lo + kt * BKH;
    const bool kok = k < t_hi;
    if (AMODE == 0) {
#pragma unroll
      for (int i = 0; i < NA; ++i)
        st.ra[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, kok && !(BF16_SKIP & 4) ? a_off[i] + (unsigned)k * 2 : kOOB, 0, 0);
    } else {
      const int cH = P0.cH, cW = P0.cW, cCin = P0.cCin;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int ih = a_ih0[i] + c_kh, iw = a_iw0[i] + c_kw;
        const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
        const unsigned off = ((a_off[i] + (unsigned)(ih * cW + iw)) * (unsigned)cCin + (unsigned)(c_ci + kc)) * 2u;
        st.ra[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, ok && !(BF16_SKIP & 4) ? off : kOOB, 0, 0);
      }
      c_ci += BKH;
      if (c_ci >= cCin) {
        c_ci = 0;
        if (++c_kw == P0.cKW) {
          c_kw = 0;
          ++c_kh;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      st.rb[i] = __builtin_amdgcn_raw_buffer_load_b128(rb, kok && !(BF16_SKIP & 4) ? b_off[i] + (unsigned)k * 2 : kOOB, 0, 0);
  };
  // DMA ring: k-tile kt of the current tile into LDS stage buf, NA + NB wave-instructions per wave whatever kt is
  // (past the k range every lane reads zeros), so the per-k-tile vmcnt count is a constant
  const int wdu = __builtin_amdgcn_readfirstlane(wid);  // wave-uniform: the LDS-DMA bases in SGPRs
  auto issue = [&](int kt, int buf) {
    const int k = t_lo + kt * BKH;
    const bool kok = k < t_hi && !(BF16_SKIP & 4);
    unsigned offa[4];
    if (AMODE == 0) {
#pragma unroll
      for (int i = 0; i < NA; ++i) offa[i] = kok ? a_off[i] + (unsigned)k * 2 : kOOB;
    } else {
      const int cH = P0.cH, cW = P0.cW, cCin = P0.cCin;
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int ih = a_ih0[i] + c_kh, iw = a_iw0[i] + c_kw;
        const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
        offa[i] = ok ? ((a_off[i] + (unsigned)(ih * cW + iw)) * (unsigned)cCin + (unsigned)(c_ci + kc)) * 2u : kOOB;
      }
      c_ci += BKH;
      if (c_ci >= cCin) {
        c_ci = 0;
        if (++c_kw == P0.cKW) {
          c_kw = 0;
          ++c_kh;
        }
      }
    }
    // row block wid + NT / 64 i: 8 rows x 128 B = 512 elements
    __bf16* const ab = lds_tile + buf * BM * SB + wdu * 512;
    __bf16* const bb = lds_tile + ST * BM * SB + buf * BN * SB + wdu * 512;
    // (the DMA builtin takes offsets from local arrays of literal size: an element of the captured b_off[NB] as
    // its argument loses the host launch stub)
    unsigned offb[4];
#pragma unroll
    for (int i = 0; i < NB; ++i) offb[i] = kok ? b_off[i] + (unsigned)k * 2 : kOOB;
#pragma unroll
    for (int i = 0; i < NA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(ab + i * NT * 8), 16,
                                               offa[i], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(bb + i * NT * 8), 16,
                                               offb[i], 0, 0, 0);
  };
  // the first k-tiles of a tile into the register stages (the DMA ring issues its own in the k-loop)
  auto prefetch = [&](const capmi_gemm_problem& P, int m0, int n0, int k_lo, int k_hi) {
    begin_tile(P, m0, n0, k_lo, k_hi);
    if (DMA) return;
    load_tile(s0, 0);
    if (ST == 2) load_tile(s1, 1);
  };
  auto store_tile = [&](const Stage& st, int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) *reinterpret_cast<u32x4_t*>(&As[buf * BM * SB + ((tid + i * NT) >> 3) * SB + kc]) = st.ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      *reinterpret_cast<u32x4_t*>(&Bs[buf * BN * SB + ((tid + i * NT) >> 3) * SB + kc]) = st.rb[i];
  };
  const int dsw = (lr >> 1) & 7;  // DMA ring: the swizzle of this lane's read rows (wm0 / wn0 + lr + 32 i)
  auto compute = [&](int buf) {
    const __bf16* Ah = &As[buf * BM * SB + (wm0 + lr) * SB + (DMA ? 0 : 8 * lh)];
    const __bf16* Bh = &Bs[buf * BN * SB + (wn0 + lr) * SB + (DMA ? 0 : 8 * lh)];
#pragma unroll
    for (int g = 0; g < BKH / 16; ++g) {
      bf16x8_t a[TM], b[TN];
      const int ko = DMA ? ((2 * g + lh) ^ dsw) * 8 : 16 * g;
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const bf16x8_t*>(Ah + 32 * i * SB + ko);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const bf16x8_t*>(Bh + 32 * j * SB + ko);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if (BF16_SKIP & 2)
            acc[i][j][0] += (float)a[i][0] * (float)b[j][1];
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  auto kstep = [&](Stage& ld, const Stage& sv, int kt) {
    load_tile(ld, kt + 2);
    compute(kt & 1);
    store_tile(sv, (kt + 1) & 1);
    __syncthreads();
  };
  // the k-loop of the prefetched tile (LDS free on entry: the previous k-loop ended on a barrier)
  auto mainloop = [&]() {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nkt = (t_hi - t_lo) / BKH;
    if (nkt <= 0) return;
    if constexpr (DMA) {  // LDS-DMA ring: k-tiles kt + 1 .. kt + ST - 2 stay in flight across the barrier
#pragma unroll
      for (int s = 0; s < ST - 1; ++s) issue(s, s);
      for (int kt = 0; kt < nkt; ++kt) {
        // this wave's DMA of k-tile kt done, every wave's (barrier); every wave past k-tile kt - 1's reads, so its
        // stage takes k-tile kt + ST - 1
        vm_barrier<(ST - 2) * (NA + NB)>();
        issue(kt + ST - 1, (kt + ST - 1) % ST);
        compute(kt % ST);
      }
      // the DMAs past the last k-tile drained and every wave's reads done before the epilogue stages C in LDS
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      return;
    }
    if (ST == 1) {  // one LDS stage, one register stage ahead
      for (int kt = 0; kt < nkt; ++kt) {
        store_tile(s0, 0);
        __syncthreads();
        load_tile(s0, kt + 1);
        compute(0);
        __syncthreads();
      }
      return;
    }
    store_tile(s0, 0);
    __syncthreads();
    // back edge only from the second k-step (see gemm_nt.hip: keeps the prefetch two deep)
    int kt = 0;
    for (; kt + 1 < nkt; kt += 2) {
      kstep(s0, s1, kt);
      kstep(s1, s0, kt + 1);
    }
    if (kt < nkt) kstep(s0, s1, kt);
  };

  // epilogue: round to bf16, store, per-channel (sum, sumsq) of the stored values per 64-row slice
  auto epilogue = [&](const capmi_gemm_problem& P, int tm, int tn) {
    const int M = P.M, N = P.N;
    const int m0 = tm * BM, n0 = tn * BN;
    unsigned short* C = reinterpret_cast<unsigned short*>(P.C);
    const long long ldc = P.ldc;
    float csum[TN], csq[TN];
    if (args.plain_epi == 1 && m0 + BM <= M) {
      // store-only form for a whole tile (round 3; host: plain_epilogue), through LDS since round 5: the rounded
      // tile is written row-major into LDS (row stride BN + 8 bf16: the two 4-row halves of a ds_write_b16 land on
      // disjoint banks), then leaves as 16-B row chunks, 4 rows x 256 B per store instruction instead of 2 x 64 B
      // per 2-B store (l3 c2 32.3 -> 30.3 us, l3 c3 19.9 -> 19.5)
      constexpr int ES = BN + 8;
      __bf16* E = lds_tile;
      static_assert(BM * ES <= ST * (BM + BN) * SB, "staging tile fits the LDS tile");
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        csum[j] = 0.f;
        csq[j] = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const unsigned short h = bf16_bits(acc[i][j][r]);
            const int rr = wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
            reinterpret_cast<unsigned short*>(E)[rr * ES + wn0 + 32 * j + lr] = h;
            const float v = bf16_val(h);
            csum[j] += v;
            csq[j] = fmaf(v, v, csq[j]);
          }
      }
      __syncthreads();
      const auto rc = rsrc_of(C, (unsigned)((long long)M * ldc * 2));
      constexpr int CPR = BN / 8;  // 16-B chunks per row
#pragma unroll
      for (int q = 0; q < BM * CPR / NT; ++q) {
        const int e = q * NT + tid, row = e / CPR, ch = e % CPR;
        const u32x4_t v = *reinterpret_cast<const u32x4_t*>(E + row * ES + ch * 8);
        if (!(BF16_SKIP & 1))
          __builtin_amdgcn_raw_buffer_store_b128(v, rc, (unsigned)(((long long)(m0 + row) * ldc + n0 + ch * 8) * 2), 0, 0);
      }
      __syncthreads();  // (the next k-loop's first LDS stores overwrite the staging tile)
    } else
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      csum[j] = 0.f;
      csq[j] = 0.f;
      const int col = n0 + wn0 + 32 * j + lr;
      const bool cok = col < N;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (cok && row < M) {
            const unsigned short h = bf16_bits(acc[i][j][r]);
            C[(long long)row * ldc + col] = h;
            const float v = bf16_val(h);
            csum[j] += v;
            csq[j] = fmaf(v, v, csq[j]);
          }
        }
      }
    }
    float* __restrict__ stats = P.stats;
    if (stats != nullptr) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        csum[j] += __shfl_xor(csum[j], 32, 64);
        csq[j] += __shfl_xor(csq[j], 32, 64);
      }
      if (lh == 0) {  // WM == 64: each wave row owns one 64-row slice
        const long long sl = (m0 + wm0) >> 6;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = n0 + wn0 + 32 * j + lr;
          if (col < N && m0 + wm0 < M) {
            stats[(sl * N + col) * 2 + 0] = csum[j];
            stats[(sl * N + col) * 2 + 1] = csq[j];
          }
        }
      }
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
    prefetch(P, tm * BM, tn * BN, 0, P.K);
    mainloop();
    epilogue(P, tm, tn);
    return;
  }

  // stream-K over (tile, k-tile) units, XCD groups: as gemm_nt.hip (the same hand-off protocol)
  const capmi_gemm_problem& P = args.p[0];
  const int nkt = args.sk_nkt, tiles_n = args.tiles_n[0];
  const long long ngrp = args.sk_groups, grp = blockIdx.x % ngrp;
  const long long T = args.sk_units / nkt, G = gridDim.x / ngrp, w = blockIdx.x / ngrp;
  const long long ub = grp * T / ngrp * nkt, U = ((grp + 1) * T / ngrp) * nkt - ub;
  const long long u0 = ub + w * U / G, u1 = ub + (w + 1) * U / G;
  if (u0 >= u1) return;
  constexpr int PART = BM * BN;
  int* flags = args.sk_flags;
  for (long long t = (u1 - 1) / nkt; t >= u0 / nkt; --t) {
    const long long tb = t * nkt;
    const int ks = (int)(max(u0, tb) - tb), ke = (int)(min(u1, tb + nkt) - tb);
    const int tm = (int)(t / tiles_n), tn = (int)(t % tiles_n);
    prefetch(P, tm * BM, tn * BN, ks * BKH, ke * BKH);
    mainloop();
    if (ke < nkt) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.sk_part + (long long)blockIdx.x * PART, 0,
                                                        PART * 4, 0x00020000);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            u32x4_t v;
            v.x = __float_as_uint(acc[i][j][4 * q + 0]);
            v.y = __float_as_uint(acc[i][j][4 * q + 1]);
            v.z = __float_as_uint(acc[i][j][4 * q + 2]);
            v.w = __float_as_uint(acc[i][j][4 * q + 3]);
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (((i * TN + j) * 4 + q) * NT + tid) * 16, 0, kSc1h);
          }
      sk_publish(flags + blockIdx.x, tid);
      continue;
    }
    if (ks > 0) {
      for (long long w2 = w - 1;; --w2) {
        const long long b2 = w2 * ngrp + grp;
        sk_consume(flags + b2, flags + gridDim.x, tid);
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.sk_part + b2 * PART, 0, PART * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(rs, (((i * TN + j) * 4 + q) * NT + tid) * 16, 0, kSc1h);
              acc[i][j][4 * q + 0] += __uint_as_float(v.x);
              acc[i][j][4 * q + 1] += __uint_as_float(v.y);
              acc[i][j][4 * q + 2] += __uint_as_float(v.z);
              acc[i][j][4 * q + 3] += __uint_as_float(v.w);
            }
        if (ub + w2 * U / G <= tb) break;
      }
    }
    epilogue(P, tm, tn);
  }
}

template <int BM, int BN>
void launch_bf16_sk(const GemmArgs& a, int amode, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(bf16_threads(BN, 2, true));
  if (amode == 2)
    CAPMI_KLAUNCH((gemm_bf16_kernel<BM, BN, 2, true, 2>), g, b, 0, s, a);
  else
    CAPMI_KLAUNCH((gemm_bf16_kernel<BM, BN, 0, true, 2>), g, b, 0, s, a);
}

template <int BM, int BN, int ST>
void launch_bf16_dma(const GemmArgs& a, int amode, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(bf16_threads(BN, ST, false));
  if (amode == 2)
    CAPMI_KLAUNCH((gemm_bf16_kernel<BM, BN, 2, false, ST>), g, b, 0, s, a);
  else
    CAPMI_KLAUNCH((gemm_bf16_kernel<BM, BN, 0, false, ST>), g, b, 0, s, a);
}

template <int BM, int BN>
void launch_bf16_st1(const GemmArgs& a, int amode, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(256);
  if (amode == 2)
    CAPMI_KLAUNCH((gemm_bf16_kernel<BM, BN, 2, false, 1>), g, b, 0, s, a);
  else
    CAPMI_KLAUNCH((gemm_bf16_kernel<BM, BN, 0, false, 1>), g, b, 0, s, a);
}

// ---- elementwise: the bf16 activations around the convs ---------------------------------------

// The two BN kernels below stream 16-B chunks (8 channels) of a [rows][C] bf16 tensor. The grid
// size in threads is a multiple of C/8 (host: C/8 divides 256), so a thread keeps ONE channel
// group for its whole grid-stride loop and holds its 8 scales / shifts in registers: per chunk one
// 16-B load per operand and one 16-B store, no index arithmetic beyond the stride.
__device__ __forceinline__ void load8(const float* __restrict__ p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// x = relu(y * scale[c] + shift[c]) (bf16 -> bf16): the materialised conv input
__global__ void __launch_bounds__(256) bn_relu_bf16_kernel(const uint4* __restrict__ y, const float* __restrict__ sc,
                                                           const float* __restrict__ sh, int n8, int C8,
                                                           uint4* __restrict__ x) {
  const int gt = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  const int c0 = (gt % C8) * 8;
  float s[8], b[8];
  load8(sc + c0, s);
  load8(sh + c0, b);
  for (int i = gt; i < n8; i += stride) {
    const uint4 v = y[i];
    const unsigned in[4] = {v.x, v.y, v.z, v.w};
    unsigned o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = pack_bf(fmaxf(fmaf(lo_bf(in[q]), s[2 * q], b[2 * q]), 0.f),
                     fmaxf(fmaf(hi_bf(in[q]), s[2 * q + 1], b[2 * q + 1]), 0.f));
    x[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// out = relu(y*s + b + res'), res' = res or res*rs + rb (downsample BN): the bottleneck tail
template <bool RBN>
__global__ void __launch_bounds__(256) bn_add_relu_bf16_kernel(const uint4* __restrict__ y, const float* __restrict__ s_,
                                                               const float* __restrict__ b_, const uint4* __restrict__ res,
                                                               const float* __restrict__ rs_, const float* __restrict__ rb_,
                                                               int n8, int C8, uint4* __restrict__ out) {
  const int gt = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  const int c0 = (gt % C8) * 8;
  float s[8], b[8], rs[8], rb[8];
  load8(s_ + c0, s);
  load8(b_ + c0, b);
  if (RBN) {
    load8(rs_ + c0, rs);
    load8(rb_ + c0, rb);
  }
  for (int i = gt; i < n8; i += stride) {
    const uint4 v = y[i], r = res[i];
    const unsigned yv[4] = {v.x, v.y, v.z, v.w}, rv[4] = {r.x, r.y, r.z, r.w};
    unsigned o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float r0 = lo_bf(rv[q]), r1 = hi_bf(rv[q]);
      if (RBN) {
        r0 = fmaf(r0, rs[2 * q], rb[2 * q]);
        r1 = fmaf(r1, rs[2 * q + 1], rb[2 * q + 1]);
      }
      o[q] = pack_bf(fmaxf(fmaf(lo_bf(yv[q]), s[2 * q], b[2 * q]) + r0, 0.f),
                     fmaxf(fmaf(hi_bf(yv[q]), s[2 * q + 1], b[2 * q + 1]) + r1, 0.f));
    }
    out[i] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// grid (in 256-thread blocks) for the channel-group kernels: enough blocks for every CU several
// times over; 256 % C8 == 0 keeps the thread count a multiple of C8
unsigned grid_c8(long long n8) { return (unsigned)std::min<long long>(std::max<long long>(cdiv(n8, 256), 1), 4096); }

// fp32 -> bf16 (RNE), n % 8 == 0
__global__ void f32_to_bf16_kernel(const float4* __restrict__ in, long long n8, uint4* __restrict__ out) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const float4 a = in[2 * i], c = in[2 * i + 1];
    out[i] = make_uint4((unsigned)bf16_bits(a.x) | ((unsigned)bf16_bits(a.y) << 16),
                        (unsigned)bf16_bits(a.z) | ((unsigned)bf16_bits(a.w) << 16),
                        (unsigned)bf16_bits(c.x) | ((unsigned)bf16_bits(c.y) << 16),
                        (unsigned)bf16_bits(c.z) | ((unsigned)bf16_bits(c.w) << 16));
  }
}

// AdaptiveAvgPool2d(OH, OW) of a bf16 NHWC map -> fp32 NHWC (the encoder output)
__global__ void adaptive_avgpool_bf16_kernel(const unsigned short* __restrict__ x, int N, int H, int W, int C,
                                             int OH, int OW, float* __restrict__ out) {
  const long long total = (long long)N * OH * OW * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    const int h0 = oh * H / OH, h1 = ((oh + 1) * H + OH - 1) / OH;
    const int w0 = ow * W / OW, w1 = ((ow + 1) * W + OW - 1) / OW;
    float acc = 0.f;
    for (int h = h0; h < h1; ++h)
      for (int w = w0; w < w1; ++w) acc += bf16_val(x[(((long long)n * H + h) * W + w) * C + c]);
    out[i] = acc / (float)((h1 - h0) * (w1 - w0));
  }
}

unsigned grid_for(long long n) { return (unsigned)std::min<long long>(std::max<long long>(cdiv(n, 256), 1), 8192); }

}  // namespace

int gemm_bf16_launch(const GemmArgs& a, int amode, int bm, int bn, int blocks, hipStream_t s, int stages) {
  if (bm != 128 || (bn != 64 && bn != 128)) return CAPMI_EINVAL;
  const bool sk = a.sk_workers > 0;
  if (stages == 1) {  // (data-parallel 128x64 only)
    if (bn != 64 || sk) return CAPMI_EINVAL;
    launch_bf16_st1<128, 64>(a, amode, blocks, s);
  } else if (sk) {  // (two register stages)
    if (stages != 2) return CAPMI_EINVAL;
    if (bn == 128)
      launch_bf16_sk<128, 128>(a, amode, blocks, s);
    else
      launch_bf16_sk<128, 64>(a, amode, blocks, s);
  } else if (stages == 2) {  // the data-parallel DMA ring
    if (bn == 128)
      launch_bf16_dma<128, 128, 2>(a, amode, blocks, s);
    else
      launch_bf16_dma<128, 64, 2>(a, amode, blocks, s);
  } else if (stages == 4) {
    if (bn == 128)
      launch_bf16_dma<128, 128, 4>(a, amode, blocks, s);
    else
      launch_bf16_dma<128, 64, 4>(a, amode, blocks, s);
  } else {
    return CAPMI_EINVAL;
  }
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_bn_relu_bf16(const void* y, const float* scale, const float* shift, long long rows, int C,
                                  void* x, void* stream) {
  CAPMI_REQUIRE(y && scale && shift && x && rows >= 0 && C > 0 && C % 8 == 0 && 256 % (C / 8) == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(y) && aligned16(x) && aligned16(scale) && aligned16(shift), CAPMI_EALIGN);
  const long long n8 = rows * C / 8;
  CAPMI_REQUIRE(n8 < (1LL << 31), CAPMI_ERANGE);
  if (n8 == 0) return 0;
  hipLaunchKernelGGL(bn_relu_bf16_kernel, dim3(grid_c8(n8)), dim3(256), 0, as_stream(stream),
                     static_cast<const uint4*>(y), scale, shift, (int)n8, C / 8, static_cast<uint4*>(x));
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_bn_add_relu_bf16(const void* y, const float* scale, const float* shift, const void* res,
                                      const float* res_scale, const float* res_shift, long long rows, int C,
                                      void* out, void* stream) {
  CAPMI_REQUIRE(y && scale && shift && res && out && rows >= 0 && C > 0 && C % 8 == 0 && 256 % (C / 8) == 0,
                CAPMI_EINVAL);
  CAPMI_REQUIRE((res_scale == nullptr) == (res_shift == nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(y) && aligned16(res) && aligned16(out) && aligned16(scale) && aligned16(shift) &&
                    (res_scale == nullptr || (aligned16(res_scale) && aligned16(res_shift))),
                CAPMI_EALIGN);
  const long long n8 = rows * C / 8;
  CAPMI_REQUIRE(n8 < (1LL << 31), CAPMI_ERANGE);
  if (n8 == 0) return 0;
  if (res_scale)
    hipLaunchKernelGGL(bn_add_relu_bf16_kernel<true>, dim3(grid_c8(n8)), dim3(256), 0, as_stream(stream),
                       static_cast<const uint4*>(y), scale, shift, static_cast<const uint4*>(res), res_scale,
                       res_shift, (int)n8, C / 8, static_cast<uint4*>(out));
  else
    hipLaunchKernelGGL(bn_add_relu_bf16_kernel<false>, dim3(grid_c8(n8)), dim3(256), 0, as_stream(stream),
                       static_cast<const uint4*>(y), scale, shift, static_cast<const uint4*>(res), res_scale,
                       res_shift, (int)n8, C / 8, static_cast<uint4*>(out));
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_f32_to_bf16(const float* in, long long n, void* out, void* stream) {
  CAPMI_REQUIRE(in && out && n >= 0 && n % 8 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(in) && aligned16(out), CAPMI_EALIGN);
  if (n == 0) return 0;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(grid_for(n / 8)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(in), n / 8, static_cast<uint4*>(out));
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_adaptive_avgpool_bf16(const void* x, int N, int H, int W, int C, int OH, int OW, float* out,
                                           void* stream) {
  CAPMI_REQUIRE(x && out && N >= 0 && H > 0 && W > 0 && C > 0 && OH > 0 && OW > 0, CAPMI_EINVAL);
  const long long total = (long long)N * OH * OW * C;
  if (total == 0) return 0;
  hipLaunchKernelGGL(adaptive_avgpool_bf16_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream),
                     static_cast<const unsigned short*>(x), N, H, W, C, OH, OW, out);
  CAPMI_LAUNCH_CHECK();
  return 0;
}
