// GEMM v2 for the case that dominates the step: A K-major (dense rows, or the implicit
// im2col of an NHWC activation) x B = W[N][K] (nn.Linear / packed conv weight), fp32 MFMA.
//
// vs the generic kernel (gemm.hip):
//   * BK = 32 and an LDS image in the operands' own [row][k] layout (row stride 36 floats),
//     so the global->LDS staging is float4 -> ds_write_b128 with no transpose;
//   * the k order inside each 8-wide k-group is permuted so one ds_read_b128 per lane feeds
//     four consecutive v_mfma_f32_32x32x2_f32: MFMA s of group g multiplies k = 8g+s (lanes
//     0-31) and k = 8g+4+s (lanes 32-63), and lane (i, h) reads row i, k 8g+4h..8g+4h+3.
//     Every k is used exactly once (A and B share the permutation), the 36-float stride
//     makes the b128 reads conflict-free (36*i mod 64 distinct over each 16-lane group);
//   * the next k-tile's global loads are only ISSUED at the top of a k-step (masked slots
//     read a valid dummy address); masking and the fused BN-apply+ReLU prologue are applied
//     when the registers are written to LDS, after the MFMAs, so load latency overlaps math;
//   * conv1 (Cin = 3) runs on an NHWC copy of the images padded to 4 channels (AMODE 4): a
//     float4 is one pixel, k = (kh, kw, c4);
//   * the conv's (kh, kw, ci) walk is incremental (no integer division in the k loop) and
//     every problem field is read once into registers before the loop;
//   * tile shapes 128x128 / 128x64 / 64x64 (4 waves, 2x2) so grids of the small-M layers
//     (ResNet layer3/layer4, M = 64*196 / 64*49) still fill 256 CUs with >= 2 WGs each;
//   * XCD-aware block order: consecutive tiles (same A rows) land on one XCD's L2;
//   * BMODE 2 (conv weight gradient dW = dY^T im2col(X)): B is the implicit im2col of an NHWC
//     input read as k rows (k = output pixel, n = (kh, kw, ci)), staged like BMODE 1; the
//     optional BN-apply+ReLU prologue then acts on B (the conv's input is relu(bn(y_prev))).
// Numerics: unchanged (exact fp32 fmaf chains, different k order than any CPU library).
#include "gemm_args.h"

namespace {

constexpr int BK2 = 32;
constexpr int S2 = BK2 + 4;  // LDS row stride in floats

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSc1 = 16;  // buffer-op aux bit: sc1 (write-through store / L1-bypassing load)

// buffer descriptor of one parked-partial slot (wave-uniform inputs only)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slot_rsrc(float* base, long long off_floats) {
  float* p = base + off_floats;
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, 256 * 1024, 0x00020000);
}

// q = a / b for 0 <= a < 2^24, b > 0, from a float reciprocal plus one correction step
__device__ __forceinline__ int fdivq(int a, int b, float inv_b) {
  int q = (int)((float)a * inv_b);
  const int r = a - q * b;
  q += r < 0 ? -1 : (r >= b ? 1 : 0);
  return q;
}

// resident workgroups per SIMD the register budget is sized for (== gemm_nt_wg_per_cu)
template <int BM, int BN>
constexpr int kWavesPerEu = (BM == 64 && BN == 64) ? 4 : 2;

// bf16 staging (BF = true): the fp32 operands are rounded to bf16 (RNE, v_cvt_pk_bf16_f32) when
// a k-tile is written to LDS, in natural k order with a 40-element (80 B) row stride; lane
// (r, h) reads 8 consecutive k (one ds_read_b128) at k = 16g + 8h of row r, the operand layout
// of v_mfma_f32_32x32x16_bf16 (32 cycles per MFMA instead of 64 per 32x32x2 f32 for 8x the k).
// 16 lanes x 16 B at stride 80 B touch 64 distinct banks. Accumulation stays fp32; the
// epilogue, BN statistics and stream-K hand-off are the fp32 kernel's.
constexpr int SB = BK2 + 8;  // bf16 LDS row stride (elements)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));


// the exact split of gemm_x3.hip: t0 = RNE(x), t1 = RNE(x - t0), t2 = x - t0 - t1 (exact in bf16)
template <int TERMS>
__device__ __forceinline__ void split_terms(float x, __bf16 (&t)[TERMS]) {
  t[0] = (__bf16)x;
  if (TERMS == 3) {
    const float r = x - (float)t[0];
    t[1 % TERMS] = (__bf16)r;
    t[2 % TERMS] = (__bf16)(r - (float)t[1 % TERMS]);
  }
}

// four consecutive k of one row -> TERMS planes (plane stride PL bf16 elements)
template <int TERMS, int PL>
__device__ __forceinline__ void store_row4(__bf16* dst, float4 v) {
  __bf16 t0[TERMS], t1[TERMS], t2[TERMS], t3[TERMS];
  split_terms<TERMS>(v.x, t0);
  split_terms<TERMS>(v.y, t1);
  split_terms<TERMS>(v.z, t2);
  split_terms<TERMS>(v.w, t3);
#pragma unroll
  for (int p = 0; p < TERMS; ++p) {
    bf16x4 h;
    h.x = t0[p];
    h.y = t1[p];
    h.z = t2[p];
    h.w = t3[p];
    *reinterpret_cast<bf16x4*>(dst + p * PL) = h;
  }
}

// k rows k, k+1 of four consecutive rows (v0: row k, v1: row k+1, one float per row) -> per plane
// four 32-bit stores at rows 0..3 (stride SB) of dst, k pair (k, k+1)
template <int TERMS, int PL>
__device__ __forceinline__ void store_kpair(__bf16* dst, float4 v0, float4 v1) {
  const float a[4] = {v0.x, v0.y, v0.z, v0.w}, b[4] = {v1.x, v1.y, v1.z, v1.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    __bf16 ta[TERMS], tb[TERMS];
    split_terms<TERMS>(a[e], ta);
    split_terms<TERMS>(b[e], tb);
#pragma unroll
    for (int p = 0; p < TERMS; ++p) {
      const unsigned w = (unsigned)__builtin_bit_cast(unsigned short, ta[p]) |
                         ((unsigned)__builtin_bit_cast(unsigned short, tb[p]) << 16);
      *reinterpret_cast<unsigned*>(dst + p * PL + e * SB) = w;
    }
  }
}

// NT threads = NT/64 waves as (NT/128) rows x 2 columns: 256 (the 2x2 form, every mode) or 512
// (128x128 tiles only, 4x2 waves of 32x64: one workgroup per CU moves a third fewer bytes per
// k-tile through L2 and LDS than two 128x64 workgroups; forward modes only)
// TERMS = 0: fp32 operands on v_mfma_f32_32x32x2_f32. TERMS = 1: both operands rounded to bf16
// when staged (the BF form above). TERMS = 3: both operands split EXACTLY into three bf16 terms when
// staged (a = a0 + a1 + a2, gemm_x3.hip's arithmetic: six cross products above 2^-23 |a||b| on the
// bf16 matrix cores, fp32-accurate), three LDS planes per operand. With TERMS > 0 a transposed
// operand (AMODE 1 / BMODE 1: k rows, m/n contiguous) is loaded as pairs of adjacent k rows and
// transposed at the LDS store (one 32-bit store = two k of one row per plane), so the MFMA loop
// reads [row][k] images with one ds_read_b128 per fragment in every mode.
template <int BM, int BN, int AMODE, int BMODE, bool PRO, bool SK, int TERMS, int NT>
__device__ __forceinline__ void gemm_nt_body(const GemmArgs& args) {
  constexpr bool BF = TERMS > 0;
  constexpr int TT = BF ? TERMS : 1;  // planes (array extents; the fp32 form never reads them)
  static_assert(TERMS == 0 || TERMS == 1 || TERMS == 3, "terms");
  static_assert(!BF || BMODE <= 2, "split staging: B = W[N][K], k rows or the wgrad im2col");
  static_assert(NT == 256 || (NT == 512 && BMODE == 0 && AMODE != 1 && !BF), "512-thread form: forward modes");
  constexpr int WR = NT / 128;  // wave rows
  constexpr int WM = BM / WR, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int NA = BM * BK2 / 4 / NT, NB = BN * BK2 / 4 / NT;
  static_assert(NA >= 1 && NB >= 1, "tile");
  static_assert(!BF || ((AMODE != 1 || NA % 2 == 0) && (BMODE == 0 || NB % 2 == 0)), "k-row pairs");
  // floats per tile row and buffer: the fp32 [m][k] image (S2), or TERMS bf16 planes of SB
  constexpr int ROWF = TERMS == 3 ? 3 * SB / 2 : S2;
  static_assert(TERMS != 1 || SB / 2 <= S2, "bf16 plane");
  constexpr int PLA = BM * SB, PLB = BN * SB;  // bf16 elements per plane
  __shared__ __attribute__((aligned(16))) float As[2][BM * ROWF];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * ROWF];
  // row strides of the k-major images of transposed operands (AMODE 1 / BMODE >= 1): BK2 rows of
  // BM (BN) + 8 floats fit the [m][k] image's BM * S2 for BM >= 64; the +8 puts the two half-waves'
  // rows (4 apart) on disjoint bank halves
  constexpr int SMA = BM + 8, SMB = BN + 8;
  static_assert(BK2 * SMA <= BM * ROWF && BK2 * SMB <= BN * ROWF, "k-major LDS image");

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm0 = (wid >> 1) * WM, wn0 = (wid & 1) * WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int kq = (tid & 7) * 4;

  f32x16 acc[TM][TN];

  // ---- main loop: acc = A[m0:m0+BM, k_lo:k_hi) * B[n0:n0+BN, k_lo:k_hi)^T ------------------
  auto mainloop = [&](const capmi_gemm_problem& P, int m0, int n0, int k_lo, int k_hi) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nkt = k_hi > k_lo ? (k_hi - k_lo + BK2 - 1) / BK2 : 0;
    if (nkt == 0) return;
    const int M = P.M, N = P.N;
    const float* __restrict__ Ag = P.A;
    const float* __restrict__ Bg = P.B;
    const long long ldb = P.ldb;
    // conv geometry, read once
    const int cH = P.cH, cW = P.cW, cCin = P.cCin, cKW = P.cKW;
    const float* __restrict__ isc = P.in_scale;
    const float* __restrict__ ish = P.in_shift;

    // staging slots. Row-major operands (k contiguous): float4 f -> (row f>>3, k 4*(f&7)).
    // Transposed operands (AMODE 1 / BMODE 1: stored as k rows, m/n contiguous): slot i of
    // thread tid holds the float4 at column group jq = tid%16 + 16*(i % (Q/16)) of k-row
    // tid/16 + 16*(i / (Q/16)) (16 lanes read 256 contiguous bytes of a k-row) and stores it
    // whole into a k-major LDS image [k][m]; the MFMA loop reads it back as four ds_read_b32
    // per four k. (Transposing at the store into the [m][k] image, four rotated scalar stores
    // per float4, was 20-25 % slower on the weight gradients: tools/wgrad_tile_ab.py.)
    constexpr int AQ = BM / 4, BQ = BN / 4;  // float4s per k-row of a transposed tile
    constexpr int AQ16 = AQ / 16, BQ16 = BQ / 16;
    long long a_base[NA];  // dense: row offset; conv: image base offset; transposed: column
    int a_ih0[NA], a_iw0[NA];
    bool a_ok[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int f = tid + i * NT;
      if (AMODE == 1) {
        if (BF) {  // slots 2j, 2j+1: k rows 2kp, 2kp+1 of column group jq (transposed at the store).
          // Lanes walk the 16 k pairs first: a wave's 32-bit LDS stores (row 4 jq + e, word kp) then
          // hit 64 distinct banks; its loads read 16 k rows x 64 contiguous bytes
          const int u = tid + (i >> 1) * NT;
          const int jq = u / (BK2 / 2), kp = u % (BK2 / 2);
          a_ok[i] = m0 + jq * 4 < M;
          a_base[i] = m0 + jq * 4;
          a_ih0[i] = 2 * kp + (i & 1);
          a_iw0[i] = jq;
          continue;
        }
        const int jq = (tid & 15) + 16 * (i % AQ16);
        const int m = m0 + jq * 4;
        a_ok[i] = m < M;  // M % 4 == 0
        a_base[i] = m;
        a_ih0[i] = (tid >> 4) + 16 * (i / AQ16);  // k within the tile
        a_iw0[i] = jq;
        continue;
      }
      const int row = m0 + (f >> 3);
      a_ok[i] = row < M;
      if (AMODE == 0) {
        a_base[i] = a_ok[i] ? remap(row, P.a_r1, P.lda, P.a_s2) : 0;
        a_ih0[i] = a_iw0[i] = 0;
      } else {
        const int hw = P.cHo * P.cWo;
        const int n = row / hw, rem = row - n * hw;
        const int oh = rem / P.cWo, ow = rem - oh * P.cWo;
        a_ih0[i] = oh * P.cStride - P.cPad;
        a_iw0[i] = ow * P.cStride - P.cPad;
        a_base[i] = (long long)n * cH * cW * cCin;
      }
    }
    long long b_base[NB];
    int b_k[NB];
    bool b_ok[NB];
    // BMODE 2 (wgrad): the n column (kh, kw, ci..ci+3) of a slot is fixed for the whole k loop
    int b_kh[NB], b_kw[NB], b_jq[NB];  // b_jq: column group of a k-row pair slot (split staging)
    float4 b_sc[NB], b_sh[NB];
    const int cWo = P.cWo, cHW = P.cHo * P.cWo, cStr = P.cStride, cPd = P.cPad;
    const float inv_hw = 1.f / (float)cHW, inv_wo = 1.f / (float)cWo;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = tid + i * NT;
      b_kh[i] = b_kw[i] = 0;
      b_sc[i] = f4(1.f);
      b_sh[i] = f4(0.f);
      b_jq[i] = 0;
      if (BMODE == 2) {
        // split staging: slots 2j, 2j+1 = k rows 2kp, 2kp+1 of column group jq (lanes along the k pairs)
        const int u = tid + (i >> 1) * NT;
        const int jq = BF ? u / (BK2 / 2) : (tid & 15) + 16 * (i % BQ16);
        b_jq[i] = jq;
        const int n = n0 + jq * 4;
        b_ok[i] = n < N;  // N % 4 == 0, Cin % 4 == 0: a float4 never straddles (kh, kw)
        const int nn = b_ok[i] ? n : 0;
        const int kpos = nn / cCin, ci = nn - kpos * cCin;
        b_kh[i] = kpos / cKW;
        b_kw[i] = kpos - b_kh[i] * cKW;
        b_base[i] = ci;
        b_k[i] = BF ? 2 * (u % (BK2 / 2)) + (i & 1) : (tid >> 4) + 16 * (i / BQ16);
        if (PRO) {
          b_sc[i] = *reinterpret_cast<const float4*>(isc + ci);
          b_sh[i] = *reinterpret_cast<const float4*>(ish + ci);
        }
        continue;
      }
      if (BMODE == 1 && BF) {
        const int u = tid + (i >> 1) * NT;
        const int jq = u / (BK2 / 2), kp = u % (BK2 / 2);
        b_ok[i] = n0 + jq * 4 < N;
        b_base[i] = n0 + jq * 4;
        b_k[i] = 2 * kp + (i & 1);
        b_jq[i] = jq;  // column group (the transposing store's row)
      } else if (BMODE == 1) {
        const int jq = (tid & 15) + 16 * (i % BQ16);
        const int n = n0 + jq * 4;
        b_ok[i] = n < N;  // N % 4 == 0
        b_base[i] = n;
        b_k[i] = (tid >> 4) + 16 * (i / BQ16);
      } else {
        const int n = n0 + (f >> 3);
        b_ok[i] = n < N;
        b_base[i] = b_ok[i] ? (long long)n * ldb : 0;
        b_k[i] = 0;
      }
    }
    // conv k walk: k = ((kh * KW) + kw) * Cin + ci, advanced by BK2 per k-tile
    int c_ci = 0, c_kh = 0, c_kw = 0;
    if (AMODE == 2) {
      const int kpos = k_lo / cCin;
      c_ci = k_lo - kpos * cCin;
      c_kh = kpos / cKW;
      c_kw = kpos - c_kh * cKW;
    }

    // Two register stages: the loads of k-tile t+2 are issued while tile t is multiplied out
    // of LDS and tile t+1 (loaded one k-step earlier) is written to the other LDS buffer, so
    // every global load has two k-steps of MFMA work to land.
    struct Stage {
      float4 ra[NA], rb[NB], sc, sh;
      unsigned am, bm;
    };
    auto load_tile = [&](Stage& st, int kt) {
      const int k = k_lo + kt * BK2 + kq;
      const bool kok = k < k_hi;  // K % 4 == 0: a float4 is all-in or all-out
      st.am = 0;
      st.bm = 0;
      if (AMODE == 0) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const bool ok = a_ok[i] && kok;
          st.ra[i] = *reinterpret_cast<const float4*>(Ag + (ok ? a_base[i] + k : 0));
          st.am |= (unsigned)ok << i;
        }
      } else if (AMODE == 1) {
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int kr = k_lo + kt * BK2 + a_ih0[i];
          const bool ok = a_ok[i] && kr < k_hi;
          const long long off = remap(kr, P.a_r1, P.lda, P.a_s2) + a_base[i];
          st.ra[i] = *reinterpret_cast<const float4*>(Ag + (ok ? off : 0));
          st.am |= (unsigned)ok << i;
        }
      } else if (AMODE == 4) {
        // NHWC4 (conv1): one float4 = the 4 (zero-padded) channels of one input pixel
        const int pos = k >> 2, kh = pos / cKW, kw = pos - kh * cKW;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int ih = a_ih0[i] + kh, iw = a_iw0[i] + kw;
          const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
          const long long off = a_base[i] + ((long long)(ih * cW + iw)) * 4;
          st.ra[i] = *reinterpret_cast<const float4*>(Ag + (ok ? off : 0));
          st.am |= (unsigned)ok << i;
        }
      } else {
        const int ci = c_ci + kq;
        if (PRO) {
          st.sc = *reinterpret_cast<const float4*>(isc + ci);
          st.sh = *reinterpret_cast<const float4*>(ish + ci);
        }
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          const int ih = a_ih0[i] + c_kh, iw = a_iw0[i] + c_kw;
          const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
          const long long off = a_base[i] + ((long long)(ih * cW + iw)) * cCin + ci;
          st.ra[i] = *reinterpret_cast<const float4*>(Ag + (ok ? off : 0));
          st.am |= (unsigned)ok << i;
        }
        c_ci += BK2;  // advance the (kh, kw, ci) walk to the next k-tile
        if (c_ci >= cCin) {
          c_ci = 0;
          if (++c_kw == cKW) {
            c_kw = 0;
            ++c_kh;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        if (BMODE == 2) {
          // k row = output pixel (img, oh, ow) of the forward conv; the column is (kh, kw, ci)
          const int kr = k_lo + kt * BK2 + b_k[i];
          const int img = fdivq(kr, cHW, inv_hw), rem = kr - img * cHW;
          const int oh = fdivq(rem, cWo, inv_wo), ow = rem - oh * cWo;
          const int ih = oh * cStr - cPd + b_kh[i], iw = ow * cStr - cPd + b_kw[i];
          const bool ok = b_ok[i] && kr < k_hi && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
          const long long off = (((long long)img * cH + ih) * cW + iw) * cCin + b_base[i];
          st.rb[i] = *reinterpret_cast<const float4*>(Bg + (ok ? off : 0));
          st.bm |= (unsigned)ok << i;
        } else if (BMODE == 1) {
          const int kr = k_lo + kt * BK2 + b_k[i];
          const bool ok = b_ok[i] && kr < k_hi;
          st.rb[i] = *reinterpret_cast<const float4*>(Bg + (ok ? (long long)kr * ldb + b_base[i] : 0));
          st.bm |= (unsigned)ok << i;
        } else {
          const bool ok = b_ok[i] && kok;
          st.rb[i] = *reinterpret_cast<const float4*>(Bg + (ok ? b_base[i] + k : 0));
          st.bm |= (unsigned)ok << i;
        }
      }
    };
    auto store_tile = [&](const Stage& st, int buf) {
      if (BF) {
        __bf16* Ah = reinterpret_cast<__bf16*>(As[buf]);
        __bf16* Bh = reinterpret_cast<__bf16*>(Bs[buf]);
        if (AMODE == 1) {
#pragma unroll
          for (int j = 0; j < NA / 2; ++j) {
            const float4 v0 = (st.am >> (2 * j)) & 1u ? st.ra[2 * j] : f4(0.f);
            const float4 v1 = (st.am >> (2 * j + 1)) & 1u ? st.ra[2 * j + 1] : f4(0.f);
            store_kpair<TT, PLA>(Ah + 4 * a_iw0[2 * j] * SB + a_ih0[2 * j], v0, v1);
          }
        } else {
#pragma unroll
          for (int i = 0; i < NA; ++i) {
            float4 v = st.ra[i];
            if (PRO && AMODE == 2) v = relu4(fma4(v, st.sc, st.sh));
            if (!((st.am >> i) & 1u)) v = f4(0.f);
            const int f = tid + i * NT;
            store_row4<TT, PLA>(Ah + (f >> 3) * SB + kq, v);
          }
        }
        if (BMODE >= 1) {
#pragma unroll
          for (int j = 0; j < NB / 2; ++j) {
            float4 v0 = st.rb[2 * j], v1 = st.rb[2 * j + 1];
            if (PRO && BMODE == 2) {  // the wgrad's BN-apply + ReLU prologue, then the padding zeros
              v0 = relu4(fma4(v0, b_sc[2 * j], b_sh[2 * j]));
              v1 = relu4(fma4(v1, b_sc[2 * j + 1], b_sh[2 * j + 1]));
            }
            if (!((st.bm >> (2 * j)) & 1u)) v0 = f4(0.f);
            if (!((st.bm >> (2 * j + 1)) & 1u)) v1 = f4(0.f);
            store_kpair<TT, PLB>(Bh + 4 * b_jq[2 * j] * SB + b_k[2 * j], v0, v1);
          }
        } else {
#pragma unroll
          for (int i = 0; i < NB; ++i) {
            float4 v = st.rb[i];
            if (!((st.bm >> i) & 1u)) v = f4(0.f);
            const int f = tid + i * NT;
            store_row4<TT, PLB>(Bh + (f >> 3) * SB + kq, v);
          }
        }
        return;
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        float4 v = st.ra[i];
        if (PRO && AMODE == 2) v = relu4(fma4(v, st.sc, st.sh));
        if (!((st.am >> i) & 1u)) v = f4(0.f);
        const int f = tid + i * NT;
        if (AMODE == 1) {
          // k-major LDS image [k][m] (row stride SMA): the float4 along m lands whole
          *reinterpret_cast<float4*>(&As[buf][((tid >> 4) + 16 * (i / AQ16)) * SMA + (i % AQ16 * 16 + (tid & 15)) * 4]) = v;
        } else {
          *reinterpret_cast<float4*>(&As[buf][(f >> 3) * S2 + kq]) = v;
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        float4 v = st.rb[i];
        if (PRO && BMODE == 2) v = relu4(fma4(v, b_sc[i], b_sh[i]));
        if (!((st.bm >> i) & 1u)) v = f4(0.f);
        const int f = tid + i * NT;
        if (BMODE >= 1) {
          *reinterpret_cast<float4*>(&Bs[buf][((tid >> 4) + 16 * (i / BQ16)) * SMB + (i % BQ16 * 16 + (tid & 15)) * 4]) = v;
        } else {
          *reinterpret_cast<float4*>(&Bs[buf][(f >> 3) * S2 + kq]) = v;
        }
      }
    };
    auto compute = [&](int buf) {
      if (BF) {
        const __bf16* Ah = reinterpret_cast<const __bf16*>(As[buf]) + (wm0 + lr) * SB + 8 * lh;
        const __bf16* Bh = reinterpret_cast<const __bf16*>(Bs[buf]) + (wn0 + lr) * SB + 8 * lh;
#pragma unroll
        for (int g = 0; g < BK2 / 16; ++g) {
          bf16x8 a[TT][TM], b[TT][TN];
#pragma unroll
          for (int p = 0; p < TT; ++p) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
              a[p][i] = *reinterpret_cast<const bf16x8*>(Ah + p * PLA + 32 * i * SB + 16 * g);
#pragma unroll
            for (int j = 0; j < TN; ++j)
              b[p][j] = *reinterpret_cast<const bf16x8*>(Bh + p * PLB + 32 * j * SB + 16 * g);
          }
          // TERMS 3: the six products smallest first (gemm_x3.hip), product-major so that the
          // TM x TN independent accumulators interleave between dependent MFMAs
          constexpr int NPROD = TERMS == 3 ? 6 : 1;
          constexpr int PA[6] = {1, 0, 2, 0, 1, 0}, PB[6] = {1, 2, 0, 1, 0, 0};
#pragma unroll
          for (int q = 6 - NPROD; q < 6; ++q)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
              for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[PA[q] % TT][i], b[PB[q] % TT][j], acc[i][j],
                                                                   0, 0, 0);
        }
        return;
      }
      // [m][k] images: lane (lr, lh) reads k = 8g + 4lh .. +3 of its row in one ds_read_b128;
      // k-major images ([k][m], transposed operands): the same four k as four ds_read_b32
      const float* Ab = AMODE == 1 ? As[buf] + 4 * lh * SMA + wm0 + lr : As[buf] + (wm0 + lr) * S2 + 4 * lh;
      const float* Bb = BMODE >= 1 ? Bs[buf] + 4 * lh * SMB + wn0 + lr : Bs[buf] + (wn0 + lr) * S2 + 4 * lh;
#pragma unroll
      for (int g = 0; g < BK2 / 8; ++g) {
        float4 a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if (AMODE == 1) {
            const float* q = Ab + 8 * g * SMA + 32 * i;
            a[i] = make_float4(q[0], q[SMA], q[2 * SMA], q[3 * SMA]);
          } else {
            a[i] = *reinterpret_cast<const float4*>(Ab + 32 * i * S2 + 8 * g);
          }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (BMODE >= 1) {
            const float* q = Bb + 8 * g * SMB + 32 * j;
            b[j] = make_float4(q[0], q[SMB], q[2 * SMB], q[3 * SMB]);
          } else {
            b[j] = *reinterpret_cast<const float4*>(Bb + 32 * j * S2 + 8 * g);
          }
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              const float av = s == 0 ? a[i].x : s == 1 ? a[i].y : s == 2 ? a[i].z : a[i].w;
              const float bv = s == 0 ? b[j].x : s == 1 ? b[j].y : s == 2 ? b[j].z : b[j].w;
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
            }
      }
    };
    // one k-step: issue loads of tile kt+2 into `ld`, multiply tile kt, park tile kt+1 (`sv`).
    // The loads and stores are unconditional (tiles past the end load masked dummies and park
    // zeros in the unused buffer): a branch around them makes the compiler's vmcnt merge at the
    // join wait for the loads just issued, i.e. it silently drops the second prefetch stage.
    // 512-thread form: a scheduling fence after the loads keeps them at the top of the k-step.
    // Without it the scheduler sinks them below most of the step's MFMAs (and then consumes
    // the A loads with the BN prologue right after issuing them, vmcnt(1) in the ISA), so the
    // "two k-steps ahead" prefetch had well under one step of MFMA work to land behind
    // (tools/fence_ab.sh: headline +1.5 %, dominant conv 88-90 -> 92-93 TF/s; the 256-thread
    // 128x64 form measured 2 % slower with it, so it is not fenced).
    auto kstep = [&](Stage& ld, const Stage& sv, int kt) {
      load_tile(ld, kt + 2);
      if (NT == 512) __builtin_amdgcn_sched_barrier(0);
      compute(kt & 1);
      store_tile(sv, (kt + 1) & 1);
      __syncthreads();
    };

    // 128x128 with the BN prologue cannot afford the second register stage (it would drop to
    // one wave per SIMD): it prefetches one tile ahead.
    constexpr bool DEEP = !(BM == 128 && BN == 128 && PRO && NT == 256);
    Stage s0, s1;
    s0.sc = s1.sc = f4(1.f);
    s0.sh = s1.sh = f4(0.f);
    load_tile(s0, 0);
    store_tile(s0, 0);
    if (DEEP) {
      load_tile(s1, 1);
      __syncthreads();
      // the back edge must only ever come from the second k-step: with a conditional second
      // step inside the loop, the header merges a path on which the first step's loads are
      // still in flight into the registers the next ds_reads overwrite, and the compiler waits
      // vmcnt(0) at the top of EVERY iteration (the second step's prefetch then has no time)
      int kt = 0;
      for (; kt + 1 < nkt; kt += 2) {
        kstep(s0, s1, kt);
        kstep(s1, s0, kt + 1);
      }
      if (kt < nkt) kstep(s0, s1, kt);
    } else {
      __syncthreads();
      for (int kt = 0; kt < nkt; ++kt) {
        load_tile(s0, kt + 1);
        compute(kt & 1);
        store_tile(s0, (kt + 1) & 1);
        __syncthreads();
      }
    }
  };

  // ---- epilogue: alpha, bias (split 0 only), beta*C, relu, store, BN statistics -------------
  auto epilogue = [&](const capmi_gemm_problem& P, int tm, int tn, int z) {
    const int M = P.M, N = P.N;
    const int m0 = tm * BM, n0 = tn * BN;
    const float alpha = P.alpha * (P.alpha_ptr ? *P.alpha_ptr : 1.f);
    float* Cz = P.C + (long long)z * P.c_split_stride;
    const float* bias1 = P.bias;
    const float* bias2 = P.bias2;
    const float beta = P.beta;
    const int relu = P.relu;
    const long long ldc = P.ldc, c_r1 = P.c_r1, c_s2 = P.c_s2;
    float csum[TN], csq[TN];
    // store-only form (round 3) for a whole tile of C = A.B (k-split slabs included): the decoder's
    // per-timestep GEMMs and the weight gradients. Uniform test on the problem; one 32-bit lane offset, the
    // row term of each accumulator register as a uniform soffset, the column block as an immediate
    const bool plain = alpha == 1.f && (z > 0 || (!bias1 && !bias2)) && beta == 0.f && !relu && c_r1 <= 0 &&
                       m0 + BM <= M && n0 + BN <= N && (long long)(m0 + BM) * ldc * 4 < (1LL << 31);
    if (plain) {
      const auto rc = __builtin_amdgcn_make_buffer_rsrc(Cz, 0, (int)((long long)(m0 + BM) * ldc * 4), 0x00020000);
      const unsigned lbase = (unsigned)(((m0 + wm0 + 4 * lh) * ldc + n0 + wn0 + lr) * 4);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        csum[j] = 0.f;
        csq[j] = 0.f;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = acc[i][j][r];  // fmaf(acc, 1, 0) == acc
            const int rr = 32 * i + (r & 3) + 8 * (r >> 2);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, lbase + 128u * j, (int)(rr * ldc * 4), 0);
            csum[j] += v;
            csq[j] = fmaf(v, v, csq[j]);
          }
      }
    } else
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      csum[j] = 0.f;
      csq[j] = 0.f;
      const int col = n0 + wn0 + 32 * j + lr;
      const bool cok = col < N;
      float bias = 0.f;
      if (z == 0 && cok) {
        if (bias1) bias += bias1[col];
        if (bias2) bias += bias2[col];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (cok && row < M) {
            float* cp = Cz + remap(row, c_r1, ldc, c_s2) + col;
            float v = fmaf(acc[i][j][r], alpha, bias);
            if (beta != 0.f) v = fmaf(beta, *cp, v);
            if (relu) v = fmaxf(v, 0.f);
            *cp = v;
            csum[j] += v;
            csq[j] = fmaf(v, v, csq[j]);
          }
        }
      }
    }
    float* __restrict__ stats = P.stats;
    if (stats != nullptr) {
      // per-channel (sum, sumsq) of the stored values per 64-row slice: stats[slice][col][2]
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        csum[j] += __shfl_xor(csum[j], 32, 64);
        csq[j] += __shfl_xor(csq[j], 32, 64);
      }
      if (WM == 64) {  // each wave row owns one slice
        if (lh == 0) {
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
      } else {  // WM == 32: wave rows 2s and 2s+1 share the tile's 64-row slice s
        float* red = As[0];  // the K loop ended with a barrier: LDS is free
        if (lh == 0) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            red[(wid * 2 + 0) * WN + 32 * j + lr] = csum[j];
            red[(wid * 2 + 1) * WN + 32 * j + lr] = csq[j];
          }
        }
        __syncthreads();
        constexpr int NS = BM / 64;  // 64-row slices per tile
        for (int c = tid; c < NS * BN; c += NT) {
          const int sl = c / BN, cn = c % BN, wn = cn / WN, cc = cn % WN;
          const int w0 = (2 * sl) * 2 + wn, w1 = (2 * sl + 1) * 2 + wn;  // wid = 2 * row + column
          const float s = red[(w0 * 2 + 0) * WN + cc] + red[(w1 * 2 + 0) * WN + cc];
          const float q = red[(w0 * 2 + 1) * WN + cc] + red[(w1 * 2 + 1) * WN + cc];
          const int col = n0 + cn;
          if (col < N && m0 + 64 * sl < M) {
            const long long slice = (m0 >> 6) + sl;
            stats[(slice * N + col) * 2 + 0] = s;
            stats[(slice * N + col) * 2 + 1] = q;
          }
        }
        __syncthreads();  // LDS reused by the next tile (stream-K)
      }
    }
  };

  if (!SK) {
    // ---- data-parallel: one tile (of one problem / k-split) per workgroup --------------------
    int bid = blockIdx.x;
    if (args.nprob == 1) {  // XCD-aware remap (bijective for any grid size)
      const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = bid & 7;
      bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    }
    int pi = 0;
    while (pi + 1 < args.nprob && bid >= args.tiles_begin[pi + 1]) ++pi;
    const capmi_gemm_problem& P = args.p[pi];
    const int local = bid - args.tiles_begin[pi];
    const int tiles_n = args.tiles_n[pi], tiles_m = args.tiles_m[pi];
    const int tn = local % tiles_n;
    const int tm = (local / tiles_n) % tiles_m;
    const int z = local / (tiles_n * tiles_m);
    const int k_begin = z * args.kchunk[pi];
    mainloop(P, tm * BM, tn * BN, k_begin, min(P.K, k_begin + args.kchunk[pi]));
    epilogue(P, tm, tn, z);
    return;
  }

  // ---- stream-K: worker w owns units [w*U/G, (w+1)*U/G) of the (tile, k-tile) space ------------
  // Tiles are visited from the last to the first: the first segment of a tile's range (its
  // k-prefix, owned by the lower-numbered neighbour) is computed at the START of that
  // worker's schedule and parked in its workspace slot; the worker owning the tile's k-end
  // visits it LAST, adds the parked partials of the lower-numbered contributors in a fixed
  // order (deterministic) and runs the epilogue. A worker only ever waits on lower-numbered
  // workgroups, which are dispatched before it.
  //
  // With sk_groups = 8 the tiles are cut into 8 contiguous ranges (consecutive tiles share A
  // rows) and the workers with blockIdx % 8 == x run stream-K over range x among themselves:
  // under the observed round-robin placement that is one XCD, whose 4 MB L2 then holds its
  // range's A rows instead of every XCD streaming all of them (speed only). A worker still
  // only waits on workers with a lower blockIdx (same group, earlier in the group's order).
  //
  // Hybrid (sk_dp_tiles > 0, grids of more than two rounds): the tiles after the first
  // T = sk_units / nkt are run whole, round-robin over the workers (XCD-aware: each round's
  // tiles are cut into 8 contiguous chunks, one per blockIdx % 8), before the worker's stream-K
  // segment; only the last one-to-two rounds' worth of tiles is balanced by stream-K.
  const capmi_gemm_problem& P = args.p[0];
  const int nkt = args.sk_nkt, tiles_n = args.tiles_n[0];
  const long long ngrp = args.sk_groups, grp = blockIdx.x % ngrp;
  const long long T = args.sk_units / nkt, G = gridDim.x / ngrp, w = blockIdx.x / ngrp;
  if (args.sk_dp_tiles > 0) {
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = blockIdx.x & 7;
    const int pos = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (blockIdx.x >> 3);
    for (long long t = T + pos; t < T + args.sk_dp_tiles; t += nwg) {
      const int tm = (int)(t / tiles_n), tn = (int)(t % tiles_n);
      mainloop(P, tm * BM, tn * BN, 0, P.K);
      epilogue(P, tm, tn, 0);
    }
  }
  const long long ub = grp * T / ngrp * nkt, U = ((grp + 1) * T / ngrp) * nkt - ub;
  const long long u0 = ub + w * U / G, u1 = ub + (w + 1) * U / G;
  if (u0 >= u1) return;
  constexpr int PART = BM * BN;
  int* flags = args.sk_flags;
  for (long long t = (u1 - 1) / nkt; t >= u0 / nkt; --t) {
    const long long tb = t * nkt;
    const int ks = (int)(max(u0, tb) - tb), ke = (int)(min(u1, tb + nkt) - tb);
    const int tm = (int)(t / tiles_n), tn = (int)(t % tiles_n);
    mainloop(P, tm * BM, tn * BN, ks * BK2, min(P.K, ke * BK2));
    if (ke < nkt) {  // k-prefix of a tile finished by a higher-numbered worker: park it
      // write-through (sc1) 16-B stores, every wave drains them, one lane raises the flag
      // with an agent-scope store: the hand-off needs no L2 write-back fence
      const auto rs = slot_rsrc(args.sk_part, (long long)blockIdx.x * PART);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            u32x4 v;
            v.x = __float_as_uint(acc[i][j][4 * q + 0]);
            v.y = __float_as_uint(acc[i][j][4 * q + 1]);
            v.z = __float_as_uint(acc[i][j][4 * q + 2]);
            v.w = __float_as_uint(acc[i][j][4 * q + 3]);
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (((i * TN + j) * 4 + q) * NT + tid) * 16, 0, kSc1);
          }
      sk_publish(flags + blockIdx.x, tid);
      continue;
    }
    if (ks > 0) {  // add the parked k-prefixes, nearest contributor first
      for (long long w2 = w - 1;; --w2) {
        const long long b2 = w2 * ngrp + grp;  // blockIdx of the contributor
        // (a timeout leaves b2's flag and raises the error word: capmi.kernels.sk_check, the host's
        // check that every flag word is zero between launches, raises and re-zeroes the workspace)
        sk_consume(flags + b2, flags + gridDim.x, tid);
        const auto rs = slot_rsrc(args.sk_part, b2 * PART);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
                  rs, (((i * TN + j) * 4 + q) * NT + tid) * 16, 0, kSc1);
              acc[i][j][4 * q + 0] += __uint_as_float(v.x);
              acc[i][j][4 * q + 1] += __uint_as_float(v.y);
              acc[i][j][4 * q + 2] += __uint_as_float(v.z);
              acc[i][j][4 * q + 3] += __uint_as_float(v.w);
            }
        if (ub + w2 * U / G <= tb) break;  // w2's range starts inside (or at) this tile
      }
    }
    epilogue(P, tm, tn, 0);
  }
}

template <int BM, int BN, int AMODE, int BMODE, bool PRO, bool SK, bool BF = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kWavesPerEu<BM, BN>)))
gemm_nt_kernel(const GemmArgs args) {
  gemm_nt_body<BM, BN, AMODE, BMODE, PRO, SK, BF ? 1 : 0, 256>(args);
}

// split-staged dense GEMMs (the decoder's, every layout it uses): TERMS 1 (bf16 operands) or 3
// (fp32-accurate three-term split); TERMS 3 holds three LDS planes per operand, so 64x64 tiles run
// two workgroups per CU and the larger ones one (gemm_nt_wg_per_cu)
template <int BM, int BN, int AMODE, int BMODE, bool SK, int TERMS, bool PRO = false>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(TERMS == 3 ? (BM == 64 && BN == 64 ? 2 : 1) : kWavesPerEu<BM, BN>)))
gemm_nts_kernel(const GemmArgs args) {
  gemm_nt_body<BM, BN, AMODE, BMODE, PRO, SK, TERMS, 256>(args);
}

template <int BM, int BN, bool SK, int TERMS>
void launch_nts(const GemmArgs& a, int amode, int bmode, bool pro, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(256);
  if (TERMS == 3 && amode == 2 && pro)  // conv with the BN-apply + ReLU prologue
    CAPMI_KLAUNCH((gemm_nts_kernel<BM, BN, TERMS == 3 ? 2 : 0, 0, SK, TERMS, TERMS == 3>), g, b, 0, s, a);
  else if (TERMS == 3 && amode == 2)  // conv (no prologue: the data gradients' dY)
    CAPMI_KLAUNCH((gemm_nts_kernel<BM, BN, TERMS == 3 ? 2 : 0, 0, SK, TERMS>), g, b, 0, s, a);
  else if (TERMS == 3 && amode == 4)  // conv1 on the NHWC4 images
    CAPMI_KLAUNCH((gemm_nts_kernel<BM, BN, TERMS == 3 ? 4 : 0, 0, SK, TERMS>), g, b, 0, s, a);
  else if (TERMS == 3 && bmode == 2 && pro)  // conv weight gradient, BN prologue on the im2col B
    CAPMI_KLAUNCH((gemm_nts_kernel<BM, BN, 1, TERMS == 3 ? 2 : 1, SK, TERMS, TERMS == 3>), g, b, 0, s, a);
  else if (TERMS == 3 && bmode == 2)
    CAPMI_KLAUNCH((gemm_nts_kernel<BM, BN, 1, TERMS == 3 ? 2 : 1, SK, TERMS>), g, b, 0, s, a);
  else if (amode == 0 && bmode == 0)
    CAPMI_KLAUNCH((gemm_nts_kernel<BM, BN, 0, 0, SK, TERMS>), g, b, 0, s, a);
  else if (amode == 0 && bmode == 1)
    CAPMI_KLAUNCH((gemm_nts_kernel<BM, BN, 0, 1, SK, TERMS>), g, b, 0, s, a);
  else
    CAPMI_KLAUNCH((gemm_nts_kernel<BM, BN, 1, 1, SK, TERMS>), g, b, 0, s, a);
}

template <int AMODE, bool PRO, bool SK>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
gemm_nt8_kernel(const GemmArgs args) {
  gemm_nt_body<128, 128, AMODE, 0, PRO, SK, 0, 512>(args);
}

template <bool SK>
void launch_nt8(const GemmArgs& a, int amode, bool pro, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(512);
  if (amode == 4)
    CAPMI_KLAUNCH((gemm_nt8_kernel<4, false, SK>), g, b, 0, s, a);
  else if (amode == 0)
    CAPMI_KLAUNCH((gemm_nt8_kernel<0, false, SK>), g, b, 0, s, a);
  else if (pro)
    CAPMI_KLAUNCH((gemm_nt8_kernel<2, true, SK>), g, b, 0, s, a);
  else
    CAPMI_KLAUNCH((gemm_nt8_kernel<2, false, SK>), g, b, 0, s, a);
}

template <int BM, int BN, bool SK>
void launch_sk_bf16(const GemmArgs& a, int amode, bool pro, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(256);
  if (amode == 4)
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 4, 0, false, SK, true>), g, b, 0, s, a);
  else if (amode == 0)
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 0, 0, false, SK, true>), g, b, 0, s, a);
  else if (pro)
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 2, 0, true, SK, true>), g, b, 0, s, a);
  else
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 2, 0, false, SK, true>), g, b, 0, s, a);
}

template <int BM, int BN, bool SK>
void launch_sk(const GemmArgs& a, int amode, int bmode, bool pro, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(256);
  if (bmode == 2) {  // weight gradient: A = dY stored as k rows, B = implicit im2col k rows
    if (pro)
      CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 1, 2, true, SK>), g, b, 0, s, a);
    else
      CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 1, 2, false, SK>), g, b, 0, s, a);
  } else if (bmode == 1) {
    if (amode == 1)
      CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 1, 1, false, SK>), g, b, 0, s, a);
    else
      CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 0, 1, false, SK>), g, b, 0, s, a);
  } else if (amode == 1) {
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 1, 0, false, SK>), g, b, 0, s, a);
  } else if (amode == 4) {
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 4, 0, false, SK>), g, b, 0, s, a);
  } else if (amode == 0) {
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 0, 0, false, SK>), g, b, 0, s, a);
  } else if (pro) {
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 2, 0, true, SK>), g, b, 0, s, a);
  } else {
    CAPMI_KLAUNCH((gemm_nt_kernel<BM, BN, 2, 0, false, SK>), g, b, 0, s, a);
  }
}

template <int BM, int BN>
int launch_bmbn(const GemmArgs& a, int amode, int bmode, bool pro, int terms, int blocks, hipStream_t s) {
  const bool bf16 = terms == 1 && bmode == 0 && amode != 1;  // the forward / conv bf16 forms
  if (terms > 0 && !bf16) {
    const bool conv3 = terms == 3 && bmode == 0 && (amode == 2 || amode == 4);
    const bool wgrad3 = terms == 3 && amode == 1 && bmode == 2;
    if (!((amode == 0 && bmode <= 1) || (amode == 1 && bmode == 1) || conv3 || wgrad3)) return CAPMI_EINVAL;
    if (pro && !((conv3 && amode == 2) || wgrad3)) return CAPMI_EINVAL;
    const bool sk = a.sk_workers > 0;
    if (terms == 3) {
      if (sk)
        launch_nts<BM, BN, true, 3>(a, amode, bmode, pro, blocks, s);
      else
        launch_nts<BM, BN, false, 3>(a, amode, bmode, pro, blocks, s);
    } else {
      if (sk)
        launch_nts<BM, BN, true, 1>(a, amode, bmode, pro, blocks, s);
      else
        launch_nts<BM, BN, false, 1>(a, amode, bmode, pro, blocks, s);
    }
  } else if (bf16) {
    if (a.sk_workers > 0)
      launch_sk_bf16<BM, BN, true>(a, amode, pro, blocks, s);
    else
      launch_sk_bf16<BM, BN, false>(a, amode, pro, blocks, s);
  } else if (a.sk_workers > 0)
    launch_sk<BM, BN, true>(a, amode, bmode, pro, blocks, s);
  else
    launch_sk<BM, BN, false>(a, amode, bmode, pro, blocks, s);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

}  // namespace

int gemm_nt_launch(const GemmArgs& a, int amode, int bmode, int bm, int bn, int blocks, hipStream_t s,
                   int terms, int nt) {
  const bool bf16 = terms > 0;
  bool pro = false;
  for (int i = 0; i < a.nprob; ++i) pro = pro || a.p[i].in_scale != nullptr;
  for (int i = 0; i < a.nprob; ++i)
    if (pro && a.p[i].in_scale == nullptr) return CAPMI_EINVAL;  // grouped: all or none
  if (pro && !((amode == 2 && bmode == 0) || (amode == 1 && bmode == 2))) return CAPMI_EINVAL;
  if (bmode == 2 && amode != 1) return CAPMI_EINVAL;
  if (terms != 0 && terms != 1 && terms != 3) return CAPMI_EINVAL;
  if (terms == 3 && !((amode == 0 && bmode <= 1) || (amode == 1 && bmode >= 1) ||
                      (bmode == 0 && (amode == 2 || (amode == 4 && !pro)))))
    return CAPMI_EINVAL;
  if (terms == 1 && !((bmode == 0 && amode != 1 && amode != 3) || (amode <= 1 && bmode == 1))) return CAPMI_EINVAL;
  if (nt == 512) {
    if (bm != 128 || bn != 128 || bf16 || bmode != 0 || !(amode == 0 || amode == 2 || amode == 4)) return CAPMI_EINVAL;
    if (a.sk_workers > 0)
      launch_nt8<true>(a, amode, pro, blocks, s);
    else
      launch_nt8<false>(a, amode, pro, blocks, s);
    CAPMI_LAUNCH_CHECK();
    return 0;
  }
  if (bm == 128 && bn == 128) return launch_bmbn<128, 128>(a, amode, bmode, pro, terms, blocks, s);
  if (bm == 128 && bn == 64) return launch_bmbn<128, 64>(a, amode, bmode, pro, terms, blocks, s);
  if (bm == 64 && bn == 64) return launch_bmbn<64, 64>(a, amode, bmode, pro, terms, blocks, s);
  return CAPMI_EINVAL;
}
