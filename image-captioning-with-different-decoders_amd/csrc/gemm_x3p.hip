// fp32-accurate GEMM / implicit-GEMM convolution with BOTH operands pre-split into three bf16
// planes ("x3p"; the arithmetic of gemm_x3.hip: six cross products above 2^-23 |a||b|, fp32
// accumulation on v_mfma_f32_32x32x16_bf16). The conv input relu(bn(y)) is split once per tensor
// by capmi_bn_relu_split3 (a 3x3 conv reads every input element nine times, a 1x1 conv with
// N = 1024 re-stages each A tile for eight column tiles: splitting in the GEMM repeated the VALU
// work that often), the weights once per weight version (capmi_split3_bf16).
//
// Structure: 256 x 128 tile, 512 threads = 8 waves as 4 (M) x 2 (N), wave tile 64 x 64 (2 x 2
// MFMA tiles: per 16-k chunk 6 + 6 ds_read_b128 feed 24 MFMAs), BK = 32. Staging is LDS-DMA
// (buffer_load_dwordx4 ... lds, no VGPRs, no ds_write): one wave-instruction moves 16 rows x 64 B
// of one plane into a lane-linear 1 KiB LDS block; the 16-B chunk of row r in slot s holds the
// logical k-chunk s ^ ((r >> 2) & 3) (the swizzle goes on the per-lane SOURCE address), so the
// 16-lane groups of ds_read_b128 hit 64 distinct banks. Padding taps and rows past M read zeros
// (buffer offsets past the descriptor's range). LDS double buffer (2 x 72 KiB, one array), one
// barrier per k-tile: the DMA of tile t+1 is issued before tile t is multiplied and retired by
// `vmcnt(0)` + the barrier that ends tile t. (Measured alternative: BK = 16 with three buffers and
// the DMA two tiles ahead behind a counted vmcnt -- the extra barrier per 32 k cost more than the
// deeper prefetch gained: layer3 3x3 101 us vs 85.) Epilogue (fp32 C, alpha/bias/beta/relu,
// per-64-row BN statistics: a wave's 64 rows are one slice) and the stream-K / hybrid schedule with
// the write-through hand-off are those of gemm_nt.hip.
#include "gemm_args.h"
#include "stamp.h"

STAMP_BUFFER(capmi_x3p_stamps)

namespace {

constexpr int PNT = 512;
typedef unsigned u32x4_p __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_p __attribute__((ext_vector_type(8)));
typedef float f32x4_p __attribute__((ext_vector_type(4)));
constexpr unsigned kOOBp = 0x80000000u;
constexpr int kSc1p = 16;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_p(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// BK = 32: 72 KiB per LDS buffer, one workgroup per CU; BK = 16: 36 KiB, two workgroups per CU (their
// barriers and DMA waits fall at different times, so one's MFMAs cover the other's stalls)
// tile: 256 x 128 (M x N)
template <int PBK>
struct X3pGeo {
  static constexpr int BM = 256, BN = 128;
  static constexpr int PROWB = PBK * 2;             // bytes per LDS row
  static constexpr int CPR = PBK / 8;               // 16-B chunks per row
  static constexpr int RPB = 1024 / PROWB;          // rows per 1 KiB LDS-DMA block (16 or 32)
  static constexpr int SWZ = 16 / CPR;              // swizzle period: chunk s of row r holds s ^ ((r / SWZ) % CPR)
  static constexpr int PA_BYTES = 3 * BM * PROWB;  // A planes of one k-tile
  static constexpr int PB_BYTES = 3 * BN * PROWB;
  static constexpr int PBUF = PA_BYTES + PB_BYTES;  // 72 / 36 KiB per buffer
  static constexpr int NAB = BM / RPB / 8;          // A row blocks per wave (2 / 1)
  static constexpr int NBB = BN / RPB;              // B row blocks (8 / 4): waves 0 .. NBB-1
  static constexpr int WPE = PBK == 16 ? 4 : 2;     // waves per SIMD: two workgroups per CU at BK = 16
};

#ifndef X3P_M16
#define X3P_M16 1
#endif
// MFMA shape (round 3): 32-deep k-tiles run v_mfma_f32_16x16x32_bf16 (X3P_M16, default) -- the same
// cycles per FLOP as 32x32x16, but MI355X holds a higher clock under a 16x16x32 stream (random data:
// ~1.12-1.15x the FLOP/s, MI355X_MICROARCH.md 'DVFS give-back' (7)); 16-deep k-tiles keep 32x32x16.
// LDS chunk swizzle of row r (physical 16-B slot of logical k-chunk c = c ^ swz(r)): for the 16x16x32
// reads (lane l: row l % 16, chunk l / 16) the slot pattern [0, 2, 3, 1][(r >> 2) & 3] makes every
// 16-lane group of ds_read_b128 hit 64 distinct banks; the 32x32x16 reads (lane l: row l % 32, chunk
// 2g + l / 32) use (r / SWZ) % CPR.
template <int PBK>
__device__ __forceinline__ int swz(int r) {
  if constexpr (PBK == 32 && X3P_M16)
    return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;
  else
    return (r / X3pGeo<PBK>::SWZ) % X3pGeo<PBK>::CPR;
}

// one 16x16x32 bf16 MFMA, c += a . b (round 5 measured the operand-swapped form, whose transposed accumulator
// blocks the epilogue can store 16 B per lane: 16 rows per store instead of 4 made the epilogue slower, 6.9k -> 10.6k
// cycles per 256 x 128 tile with the column statistics on DPP row sums; not kept)
__device__ __forceinline__ f32x4_p mf16(bf16x8_p a, bf16x8_p b, f32x4_p c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ASPLIT ("x3d"): A is the fp32 operand itself (dense, or the NHWC conv input with the optional BN-apply
// + ReLU prologue PRO), loaded to registers one k-tile ahead and split into the three swizzled LDS
// planes after the k-tile's MFMAs; B stays LDS-DMA. It replaces gemm_x3 (both operands through
// registers) and the separate split pass of x3p (BK = 32 only).
template <int AMODE, bool SK, int PBK, bool ASPLIT = false, bool PRO = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(X3pGeo<PBK>::WPE)))
gemm_x3p_kernel(const GemmArgs args) {
#if X3P_CLOCK  // diagnostic build only (tools/r04/run27.sh): the clock this workgroup ran at, by device printf
  const long long clk_t0 = __builtin_amdgcn_s_memtime(), clk_r0 = __builtin_amdgcn_s_memrealtime();
  auto clk_report = [&]() {
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x % 16 == 0)
      printf("x3pclk %d %lld %lld\n", (int)blockIdx.x, t1 - clk_t0, r1 - clk_r0);
  };
#else
  auto clk_report = [] {};
#endif
#if X3P_PRIO  // A/B: the second-dispatched half of the workgroup at issue priority 1 (MI355X_MICROARCH.md, item 4)
  if (threadIdx.x >= 256) __builtin_amdgcn_s_setprio(1);
#endif
  STAMP_DECL;
  STAMP(capmi_x3p_stamps, kStStart, 0);
  STAMP_REAL(capmi_x3p_stamps, kStRStart);
  static_assert(!ASPLIT || PBK == 32, "x3d: 32-deep k-tiles");
  static_assert(!PRO || ASPLIT, "prologue: x3d (conv, or dense rows whose k is the channel: 1x1 convs)");
  using G_ = X3pGeo<PBK>;
  constexpr int PBM = G_::BM, PBN = G_::BN;
  constexpr int JN = 64 / 16;    // 16x16x32: 16-column blocks per wave (wave tile 64 x 64)
  constexpr int JN32 = 64 / 32;  // 32x32x16: 32-column blocks per wave
  constexpr int PROWB = G_::PROWB, CPR = G_::CPR, RPB = G_::RPB;
  constexpr int PA_BYTES = G_::PA_BYTES, PBUF = G_::PBUF, NAB = G_::NAB, NBB = G_::NBB;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[2 * PBUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: LDS-DMA bases in SGPRs
  const int wm0 = (wid >> 1) * 64, wn0 = (wid & 1) * 64;  // waves as 4 x 2, wave tile 64 x 64
  const int lr = lane & 31, lh = lane >> 5;
  // DMA lane geometry: row lane / CPR of an RPB-row block, slot lane % CPR
  const int drow = lane / CPR, dslot = lane % CPR;

  constexpr bool M16 = PBK == 32 && X3P_M16;
  f32x16 acc[2][JN32];  // 32x32x16: wave tile 2 x JN32 blocks of 32 x 32
  f32x4_p acc4[4][JN];  // 16x16x32: wave tile 4 x JN blocks of 16 x 16

  auto mainloop = [&](const capmi_gemm_problem& P, int m0, int n0, int k_lo, int k_hi) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < JN32; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < JN; ++j) acc4[i][j] = f32x4_p{0.f, 0.f, 0.f, 0.f};
    const int nkt = (k_hi - k_lo) / PBK;
    if (nkt <= 0) return;
    const int M = P.M, N = P.N;
    const int cH = P.cH, cW = P.cW, cCin = P.cCin, cKW = P.cKW;
    const long long planeA = AMODE == 2 ? (long long)P.cN * cH * cW * cCin : (long long)M * P.lda;
    const long long planeB = (long long)N * P.ldb;
#ifndef X3P_PRICE
#define X3P_PRICE 0
#endif
#ifndef X3P_SKIP
#define X3P_SKIP 0
#endif
    // X3P_PRICE (timing-only builds): 1 = A descriptor with zero records (no A traffic), 2 = B, 3 = both
    const auto ra = rsrc_p(P.A, (X3P_PRICE & 1) ? 0u : (unsigned)(ASPLIT ? planeA * 4 : 3 * planeA * 2));
    const auto rb = rsrc_p(P.B, (X3P_PRICE & 2) ? 0u : (unsigned)(3 * planeB * 2));
    // x3d prologue: scale / shift through descriptors sized to the channel count (round 3):
    // a read past the last channel returns 0 instead of touching the next allocation
    const unsigned ss_bytes = PRO ? (unsigned)((AMODE == 2 ? cCin : P.K) * 4) : 0u;
    const auto rsc_p = rsrc_p(PRO ? (const void*)P.in_scale : P.B, ss_bytes);
    const auto rsh_p = rsrc_p(PRO ? (const void*)P.in_shift : P.B, ss_bytes);
    // this lane's two A rows (row blocks 2 wid, 2 wid + 1) and one B row (row block wid)
    // (arrays sized 2 >= NAB: a dependent bound in the nested lambda loses the host launch stub)
    unsigned a_base[2];  // dense: byte offset of (row, chunk) in plane 0; conv: pixel index of (n, 0, 0)
    int a_ih0[2], a_iw0[2], a_ch[2];
    bool a_ok[2];
#pragma unroll
    for (int i = 0; i < NAB; ++i) {
      const int r = (NAB * wid + i) * RPB + drow;
      const int row = m0 + r;
      a_ch[i] = dslot ^ swz<PBK>(r);
      a_ok[i] = row < M;
      if (AMODE == 0) {
        a_base[i] = (unsigned)(((long long)(a_ok[i] ? row : 0) * P.lda + a_ch[i] * 8) * 2);
        a_ih0[i] = a_iw0[i] = 0;
      } else {
        const int hw = P.cHo * P.cWo;
        const int rr = a_ok[i] ? row : 0;
        const int n = rr / hw, rem = rr - n * hw;
        const int oh = rem / P.cWo, ow = rem - oh * P.cWo;
        a_ih0[i] = oh * P.cStride - P.cPad;
        a_iw0[i] = ow * P.cStride - P.cPad;
        a_base[i] = (unsigned)(n * cH * cW);
      }
    }
    // B row block wid
    const bool bw = NBB == PNT / 64 || wid < NBB;  // (BK = 32: every wave issues one B row block)
    const int br = wid * RPB + drow;
    const int b_ch = dslot ^ swz<PBK>(br);
    const bool b_ok = bw && n0 + br < N;
    const unsigned b_base = (unsigned)(((long long)(b_ok ? n0 + br : 0) * P.ldb + b_ch * 8) * 2);
    // x3d: four fp32 float4 slots per thread, slot i = row (tid + 512 i) / 8, k 4 ((tid + 512 i) % 8)
    constexpr int NSA = ASPLIT ? PBM / 64 : 1;
    const int aq = tid & 7;
    unsigned s_base[NSA];
    int s_ih0[NSA], s_iw0[NSA];
    bool s_ok[NSA];
    int s_lds[NSA];  // byte offset of the slot's 8 B in plane 0 (swizzled chunk)
    if (ASPLIT) {
#pragma unroll
      for (int i = 0; i < NSA; ++i) {
        const int r = (tid + 512 * i) >> 3;
        const int row = m0 + r;
        s_ok[i] = row < M;
        s_lds[i] = r * PROWB + (((aq >> 1) ^ swz<PBK>(r)) << 4) + (aq & 1) * 8;
        if (AMODE == 0) {
          s_base[i] = (unsigned)(((long long)(s_ok[i] ? row : 0) * P.lda + aq * 4) * 4);
          s_ih0[i] = s_iw0[i] = 0;
        } else {
          const int hw = P.cHo * P.cWo;
          const int rr = s_ok[i] ? row : 0;
          const int n = rr / hw, rem = rr - n * hw;
          const int oh = rem / P.cWo, ow = rem - oh * P.cWo;
          s_ih0[i] = oh * P.cStride - P.cPad;
          s_iw0[i] = ow * P.cStride - P.cPad;
          s_base[i] = (unsigned)(n * cH * cW);
        }
      }
    }
    float4 areg[NSA];
    float4 a_sc = make_float4(1.f, 1.f, 1.f, 1.f), a_sh = make_float4(0.f, 0.f, 0.f, 0.f);
    unsigned a_msk = 0;
    // conv k order (ci / 32, kh, kw, ci % 32): the taps of one 32-channel slice are consecutive
    // k-tiles, so the input rows a tile re-reads for its KH*KW taps are re-read within KH*KW k-tiles
    // (L2-resident) instead of once per full sweep over Cin; the weights are packed to match
    // (capmi.kernels.pack_conv_weight_x3p)
    // k-tiles of 16 walk each (32-channel slice, tap) chunk in two halves (c_sub), so the packed
    // weight layout is the same for both depths
    constexpr int SUB = 32 / PBK;
    int c_ci = 0, c_kh = 0, c_kw = 0, c_sub = 0;
    if (AMODE == 2) {
      const int taps = cKW * P.cKH, kt0 = k_lo / PBK, kt32 = kt0 / SUB;
      const int tap = kt32 % taps;
      c_sub = kt0 % SUB;
      c_ci = (kt32 / taps) * 32;
      c_kh = tap / cKW;
      c_kw = tap - c_kh * cKW;
    }
    const unsigned pA2 = (unsigned)(planeA * 2), pB2 = (unsigned)(planeB * 2);

    // DMA of k-tile kt into buffer buf: 6 A + 3 B wave-instructions per wave
    auto issue = [&](int kt, int buf) {
#if X3P_SKIP & 1  // timing-only: no DMA
      return;
#endif
      const int k = k_lo + kt * PBK;
      const bool kok = k < k_hi;
      if (ASPLIT) {
        a_msk = 0;
        if (PRO && kok) {  // (past the last k-tile the walk is past Cin: no read)
          const unsigned ch = (unsigned)((AMODE == 2 ? c_ci : k) + aq * 4) * 4u;  // dense rows: channel = k
          a_sc = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsc_p, ch, 0, 0));
          a_sh = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsh_p, ch, 0, 0));
        }
#pragma unroll
        for (int i = 0; i < NSA; ++i) {
          unsigned off;
          bool ok;
          if (AMODE == 0) {
            ok = s_ok[i] && kok;
            off = s_base[i] + (unsigned)k * 4;
          } else {
            const int ih = s_ih0[i] + c_kh, iw = s_iw0[i] + c_kw;
            ok = s_ok[i] && kok && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
            off = ((s_base[i] + (unsigned)(ih * cW + iw)) * (unsigned)cCin + (unsigned)(c_ci + aq * 4)) * 4u;
          }
          areg[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, ok ? off : kOOBp, 0, 0));
          a_msk |= (unsigned)ok << i;
        }
      }
      // plane-0 byte offset of this lane's A piece and its out-of-range bit (kOOBp: padding taps, rows past M, k past
      // the end), combined per plane below without a branch (an exec-masked offset computation split the DMA issue
      // into basic blocks of its own, out of reach of the MFMA interleave)
      unsigned aoff[2], abad[2];
#pragma unroll
      for (int i = 0; i < NAB; ++i) {
        if (ASPLIT) break;
        if (AMODE == 0) {
          aoff[i] = a_base[i] + (unsigned)k * 2;
          abad[i] = a_ok[i] && kok ? 0u : kOOBp;
        } else {
          const int ih = a_ih0[i] + c_kh, iw = a_iw0[i] + c_kw;
          const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
          aoff[i] = ((a_base[i] + (unsigned)(ih * cW + iw)) * (unsigned)cCin + (unsigned)(c_ci + c_sub * PBK + a_ch[i] * 8)) * 2u;
          abad[i] = ok ? 0u : kOOBp;
        }
      }
      if (AMODE == 2 && ++c_sub == SUB) {
        c_sub = 0;
        if (++c_kw == cKW) {
          c_kw = 0;
          if (++c_kh == P.cKH) {
            c_kh = 0;
            c_ci += 32;
          }
        }
      }
      unsigned char* base = lds + buf * PBUF;
#pragma unroll
      for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int i = 0; i < (ASPLIT ? 0 : NAB); ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              ra, (lds_ptr_t)(base + p * PBM * PROWB + (NAB * wid + i) * RPB * PROWB), 16,
              PBK == 32 ? (aoff[i] + p * pA2) | abad[i] : (abad[i] ? kOOBp : aoff[i] + p * pA2), 0, 0, 0);
      if (bw) {
        const unsigned boff = b_base + (unsigned)k * 2, bbad = b_ok && kok ? 0u : kOOBp;
        // (BK = 16, at its 128-register cap, keeps the select form: the branch-free one spilled it)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(base + PA_BYTES + p * PBN * PROWB + wid * RPB * PROWB),
                                                   16, PBK == 32 ? (boff + p * pB2) | bbad : (bbad ? kOOBp : boff + p * pB2), 0, 0, 0);
      }
    };
    // x3d: fp32 A registers of one k-tile -> (prologue) -> three planes
    auto store_a_from = [&](int buf, const float4 (&ar)[NSA], float4 sc, float4 sh, unsigned msk) {
      if (!ASPLIT) return;
      unsigned char* base = lds + buf * PBUF;
#pragma unroll
      for (int i = 0; i < NSA; ++i) {
        float4 v = ar[i];
#if X3D_NOSPLIT  // timing-only builds: no prologue / split VALU, the raw bits stored (wrong results)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          *reinterpret_cast<uint2*>(base + p * PBM * PROWB + s_lds[i]) = make_uint2(__float_as_uint(v.x), __float_as_uint(v.z));
        continue;
#endif
        if (PRO) v = make_float4(fmaxf(fmaf(v.x, sc.x, sh.x), 0.f), fmaxf(fmaf(v.y, sc.y, sh.y), 0.f),
                                 fmaxf(fmaf(v.z, sc.z, sh.z), 0.f), fmaxf(fmaf(v.w, sc.w, sh.w), 0.f));
        if (!((msk >> i) & 1u)) v = make_float4(0.f, 0.f, 0.f, 0.f);  // padding taps: zeros AFTER the BN
        unsigned lo[3], hi[3];
        split3_pair(v.x, v.y, lo);
        split3_pair(v.z, v.w, hi);
#pragma unroll
        for (int p = 0; p < 3; ++p)
          *reinterpret_cast<uint2*>(base + p * PBM * PROWB + s_lds[i]) = make_uint2(lo[p], hi[p]);
      }
    };
    // x3d: the registers of the k-tile loaded by the last issue()
    auto store_a = [&](int buf) { store_a_from(buf, areg, a_sc, a_sh, a_msk); };
    auto compute = [&](int buf) {
      const unsigned char* A_ = lds + buf * PBUF;
      const unsigned char* B_ = A_ + PA_BYTES;
      if constexpr (M16) {
        // 16x16x32: lane l reads row (l % 16) of each 16-row block, k-chunk l / 16 (8 k of the 32);
        // all 24 fragments of the k-tile up front, then 16 blocks x 6 products
        bf16x8_p a[4][3], b[JN][3];
        const int c = lane >> 4, rl = lane & 15;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wm0 + 16 * i + rl;
          const int o = r * PROWB + ((c ^ swz<PBK>(r)) << 4);
#pragma unroll
          for (int p = 0; p < 3; ++p) a[i][p] = *reinterpret_cast<const bf16x8_p*>(A_ + p * PBM * PROWB + o);
        }
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int r = wn0 + 16 * j + rl;
          const int o = r * PROWB + ((c ^ swz<PBK>(r)) << 4);
#pragma unroll
          for (int p = 0; p < 3; ++p) b[j][p] = *reinterpret_cast<const bf16x8_p*>(B_ + p * PBN * PROWB + o);
        }
        // smallest terms first into each fp32 accumulator
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < JN; ++j) {
            acc4[i][j] = mf16(a[i][1], b[j][1], acc4[i][j]);
            acc4[i][j] = mf16(a[i][0], b[j][2], acc4[i][j]);
            acc4[i][j] = mf16(a[i][2], b[j][0], acc4[i][j]);
          }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < JN; ++j) {
            acc4[i][j] = mf16(a[i][0], b[j][1], acc4[i][j]);
            acc4[i][j] = mf16(a[i][1], b[j][0], acc4[i][j]);
            acc4[i][j] = mf16(a[i][0], b[j][0], acc4[i][j]);
          }
        return;
      }
      // every fragment of the k-tile is requested up front (2 x 12 ds_read_b128): the second
      // chunk's reads land while the first chunk's 24 MFMAs run
      bf16x8_p a[PBK / 16][2][3], b[PBK / 16][JN32][3];
#pragma unroll
      for (int g = 0; g < PBK / 16; ++g) {
        const int c = 2 * g + lh;  // logical 16-B chunk (8 k) this lane reads
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = wm0 + 32 * i + lr;
          const int o = r * PROWB + ((c ^ swz<PBK>(r)) << 4);
#if X3P_SKIP & 2  // timing-only: no LDS reads
#pragma unroll
          for (int p = 0; p < 3; ++p) a[g][i][p] = bf16x8_p{} + (__bf16)(float)(o + p);
#else
#pragma unroll
          for (int p = 0; p < 3; ++p) a[g][i][p] = *reinterpret_cast<const bf16x8_p*>(A_ + p * PBM * PROWB + o);
#endif
        }
#pragma unroll
        for (int j = 0; j < JN32; ++j) {
          const int r = wn0 + 32 * j + lr;
          const int o = r * PROWB + ((c ^ swz<PBK>(r)) << 4);
#if X3P_SKIP & 2
#pragma unroll
          for (int p = 0; p < 3; ++p) b[g][j][p] = bf16x8_p{} + (__bf16)(float)(o - p);
#else
#pragma unroll
          for (int p = 0; p < 3; ++p) b[g][j][p] = *reinterpret_cast<const bf16x8_p*>(B_ + p * PBN * PROWB + o);
#endif
        }
      }
#pragma unroll
      for (int g = 0; g < PBK / 16; ++g) {
        // smallest terms first into each fp32 accumulator
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < JN32; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[g][i][1], b[g][j][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[g][i][0], b[g][j][2], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[g][i][2], b[g][j][0], acc[i][j], 0, 0, 0);
          }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < JN32; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[g][i][0], b[g][j][1], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[g][i][1], b[g][j][0], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[g][i][0], b[g][j][0], acc[i][j], 0, 0, 0);
          }
      }
    };
#ifndef X3D_PIPE
#define X3D_PIPE 1
#endif
    // x3d staging helpers (round 4 pipelined loop, round 5 phase loop): B planes by LDS-DMA, A slots by register
    auto b_dma = [&](int kt, int buf) {  // B planes of tile kt (past the end: zeros) into buffer buf
      const int k = k_lo + kt * PBK;
      unsigned char* base = lds + buf * PBUF;
      if (bw) {
        const unsigned boff = b_base + (unsigned)k * 2, bbad = b_ok && k < k_hi ? 0u : kOOBp;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(base + PA_BYTES + p * PBN * PROWB + wid * RPB * PROWB),
                                                   16, (boff + p * pB2) | bbad, 0, 0, 0);
      }
    };
    auto a_load = [&](int kt, int i) {  // slot i of tile kt (the conv walk at tile kt)
      const int k = k_lo + kt * PBK;
      const bool kok = k < k_hi;
      unsigned off;
      bool ok;
      if (AMODE == 0) {
        ok = s_ok[i] && kok;
        off = s_base[i] + (unsigned)k * 4;
      } else {
        const int ih = s_ih0[i] + c_kh, iw = s_iw0[i] + c_kw;
        ok = s_ok[i] && kok && (unsigned)ih < (unsigned)cH && (unsigned)iw < (unsigned)cW;
        off = ((s_base[i] + (unsigned)(ih * cW + iw)) * (unsigned)cCin + (unsigned)(c_ci + aq * 4)) * 4u;
      }
      areg[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(ra, off | (ok ? 0u : kOOBp), 0, 0));
      a_msk = (a_msk & ~(1u << i)) | ((unsigned)ok << i);
    };
    auto a_next = [&](int kt) {  // after tile kt's four slots: its BN scale / shift, then the walk advances
      const int k = k_lo + kt * PBK;
      if (PRO) {  // always two loads (the step's vmcnt count relies on it); past the last k-tile the walk is
                  // past Cin: an out-of-range offset, zeros
        const unsigned ch = k < k_hi ? (unsigned)((AMODE == 2 ? c_ci : k) + aq * 4) * 4u : kOOBp;
        a_sc = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsc_p, ch, 0, 0));
        a_sh = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsh_p, ch, 0, 0));
      }
      if (AMODE == 2 && ++c_kw == cKW) {  // (32-deep k-tiles: one (channel slice, tap) chunk per tile)
        c_kw = 0;
        if (++c_kh == P.cKH) {
          c_kh = 0;
          c_ci += 32;
        }
      }
    };
    auto a_split = [&](int buf, int i) {  // slot i -> (prologue) -> three planes of buffer buf
      unsigned char* base = lds + buf * PBUF;
      float4 v = areg[i];
#if X3D_NOSPLIT  // timing-only builds (above)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        *reinterpret_cast<uint2*>(base + p * PBM * PROWB + s_lds[i]) = make_uint2(__float_as_uint(v.x), __float_as_uint(v.z));
      return;
#endif
      if (PRO) v = make_float4(fmaxf(fmaf(v.x, a_sc.x, a_sh.x), 0.f), fmaxf(fmaf(v.y, a_sc.y, a_sh.y), 0.f),
                               fmaxf(fmaf(v.z, a_sc.z, a_sh.z), 0.f), fmaxf(fmaf(v.w, a_sc.w, a_sh.w), 0.f));
      const bool keep = (a_msk >> i) & 1u;  // padding taps / rows past M: zeros AFTER the BN
      v.x = keep ? v.x : 0.f;
      v.y = keep ? v.y : 0.f;
      v.z = keep ? v.z : 0.f;
      v.w = keep ? v.w : 0.f;
      unsigned lo[3], hi[3];
      split3_pair(v.x, v.y, lo);
      split3_pair(v.z, v.w, hi);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        *reinterpret_cast<uint2*>(base + p * PBM * PROWB + s_lds[i]) = make_uint2(lo[p], hi[p]);
    };
// X3P_PHASE (round 5, default 2): x3p's k-loop places its one barrier after this many row blocks' MFMAs and
// issues the next-but-one tile's DMA behind it (see the x3p branch of mainloop); 0 = the round-4 loop
#ifndef X3P_PHASE
#define X3P_PHASE 2
#endif
    // the six products of row block i of a k-tile, smallest terms first per accumulator
    auto mm6 = [&](int i, const bf16x8_p (&a)[3], const bf16x8_p (&b)[JN][3]) {
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        acc4[i][j] = mf16(a[1], b[j][1], acc4[i][j]);
        acc4[i][j] = mf16(a[0], b[j][2], acc4[i][j]);
        acc4[i][j] = mf16(a[2], b[j][0], acc4[i][j]);
      }
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        acc4[i][j] = mf16(a[0], b[j][1], acc4[i][j]);
        acc4[i][j] = mf16(a[1], b[j][0], acc4[i][j]);
        acc4[i][j] = mf16(a[0], b[j][0], acc4[i][j]);
      }
    };
    if (ASPLIT && M16 && X3D_PIPE && args.x3d_pipe) {
      // x3d, round 4: A two k-tiles deep in ONE register set. During tile kt's MFMAs each of the thread's four
      // float4 slots is split into the other buffer for tile kt + 1 and at once reloaded with tile kt + 2's
      // (its BN scale / shift and the conv walk follow after the fourth slot): the A load has a whole k-tile to
      // land, and the split's VALU and ds_writes interleave with the MFMAs instead of standing between two
      // k-tiles with the load latency in front of them (the one-deep form: issue, MFMAs, wait, split, barrier)
      const int c16 = lane >> 4, rl16 = lane & 15;
      auto frag = [&](const unsigned char* plane, int r) {  // 16x16x32 fragment of row r, chunk c16
        return *reinterpret_cast<const bf16x8_p*>(plane + r * PROWB + ((c16 ^ swz<PBK>(r)) << 4));
      };
      auto step = [&](int kt, int buf) {
        b_dma(kt + 1, buf ^ 1);  // buffer buf ^ 1 was last read by the previous step (barrier since)
        const unsigned char* A_ = lds + buf * PBUF;
        const unsigned char* B_ = A_ + PA_BYTES;
        bf16x8_p b[JN][3], a[3];
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
          for (int p = 0; p < 3; ++p) b[j][p] = frag(B_ + p * PBN * PROWB, wn0 + 16 * j + rl16);
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = frag(A_ + p * PBM * PROWB, wm0 + rl16);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          bf16x8_p an[3];
          if (i + 1 < 4) {
#pragma unroll
            for (int p = 0; p < 3; ++p) an[p] = frag(A_ + p * PBM * PROWB, wm0 + 16 * (i + 1) + rl16);
          }
          __builtin_amdgcn_sched_barrier(0);
          a_split(buf ^ 1, i);
          a_load(kt + 2, i);
          if (i == 3) a_next(kt + 2);
          // per accumulator the six products smallest terms first (the one-deep form's order)
#pragma unroll
          for (int j = 0; j < JN; ++j) {
            acc4[i][j] = mf16(a[1], b[j][1], acc4[i][j]);
            acc4[i][j] = mf16(a[0], b[j][2], acc4[i][j]);
            acc4[i][j] = mf16(a[2], b[j][0], acc4[i][j]);
          }
#pragma unroll
          for (int j = 0; j < JN; ++j) {
            acc4[i][j] = mf16(a[0], b[j][1], acc4[i][j]);
            acc4[i][j] = mf16(a[1], b[j][0], acc4[i][j]);
            acc4[i][j] = mf16(a[0], b[j][0], acc4[i][j]);
          }
#pragma unroll
          for (int r = 0; r < 24; ++r) {  // one MFMA, then up to two VALU (the slot's split)
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (i + 1 < 4) {
#pragma unroll
            for (int p = 0; p < 3; ++p) a[p] = an[p];
          }
        }
        // the B DMA of tile kt + 1 was issued before the four A loads (and the two scale / shift loads) of
        // tile kt + 2: waiting until that many remain drains it
        if (PRO)
          asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __syncthreads();
      };
      // tile 0: A loaded, split into buffer 0 with its B planes; tile 1's A loaded; then one step per tile
      b_dma(0, 0);
#pragma unroll
      for (int i = 0; i < NSA; ++i) a_load(0, i);
      a_next(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < NSA; ++i) a_split(0, i);
#pragma unroll
      for (int i = 0; i < NSA; ++i) a_load(1, i);
      a_next(1);
      __syncthreads();
      for (int kt = 0; kt < nkt; ++kt) step(kt, kt & 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the loads and DMA past the end drained)
      __syncthreads();  // (the next tile's prologue rewrites buffer 0, which the last step may have read)
      return;
    }
    if (!ASPLIT && M16 && X3P_PHASE) {
      // x3p, round 5: the DMA of tile kt + 2 is issued right after the barrier that ends the reads of tile kt
      // (into the buffer those reads used), interleaved with the second half of tile kt's MFMAs, so each tile's
      // DMA has a whole k-tile to land; the one-barrier loop below issued it ahead of the reads and waited for
      // it at the hoisted barrier, ~40 % of a k-tile later
      issue(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      issue(1, 1);
      const int c = lane >> 4, rl = lane & 15;
      for (int kt = 0; kt < nkt; ++kt) {
        const unsigned char* A_ = lds + (kt & 1) * PBUF;
        const unsigned char* B_ = A_ + PA_BYTES;
        bf16x8_p a[4][3], b[JN][3];
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          const int r = wn0 + 16 * j + rl;
          const int o = r * PROWB + ((c ^ swz<PBK>(r)) << 4);
#pragma unroll
#if X3P_SKIP & 2  // timing-only: no LDS reads
          for (int p = 0; p < 3; ++p) b[j][p] = bf16x8_p{} + (__bf16)(float)(o - p);
#else
          for (int p = 0; p < 3; ++p) b[j][p] = *reinterpret_cast<const bf16x8_p*>(B_ + p * PBN * PROWB + o);
#endif
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = wm0 + 16 * i + rl;
          const int o = r * PROWB + ((c ^ swz<PBK>(r)) << 4);
#pragma unroll
#if X3P_SKIP & 2  // timing-only: no LDS reads
          for (int p = 0; p < 3; ++p) a[i][p] = bf16x8_p{} + (__bf16)(float)(o + p);
#else
          for (int p = 0; p < 3; ++p) a[i][p] = *reinterpret_cast<const bf16x8_p*>(A_ + p * PBM * PROWB + o);
#endif
        }
        // X3P_PHASE = row blocks multiplied before the barrier (1-3)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (i == X3P_PHASE) {
            __builtin_amdgcn_sched_barrier(0);
            // tile kt + 1 landed (this wave's DMA), this wave's reads of tile kt done; the barrier makes both hold
            // for every wave: buffer kt & 1 is free for tile kt + 2, buffer (kt + 1) & 1 readable
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            issue(kt + 2, kt & 1);  // (past the end: zeros, no memory traffic; keeps the DMA branch-free)
          }
          mm6(i, a[i], b);
        }
#pragma unroll
        for (int r = 0; r < 9; ++r) {  // the DMA pieces spread over the MFMAs after the barrier
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * (4 - X3P_PHASE), 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();  // (the next tile's prologue rewrites buffer 0, which the last k-tile may have read)
      return;
    }
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_a(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      issue(kt + 1, (kt + 1) & 1);  // past the end: OOB loads (zeros) into the idle buffer
      compute(kt & 1);
#if X3P_SKIP & 4  // timing-only: no barrier inside the k-loop
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      store_a((kt + 1) & 1);  // x3d: buffer (kt + 1) & 1 was last read by compute(kt - 1)
      __syncthreads();
#endif
    }
  };

  auto epilogue = [&](const capmi_gemm_problem& P, int tm, int tn) {
    const int M = P.M, N = P.N;
    const int m0 = tm * PBM, n0 = tn * PBN;
    const float alpha = P.alpha * (P.alpha_ptr ? *P.alpha_ptr : 1.f);
    float* C = P.C;
    const float beta = P.beta;
    const int relu = P.relu;
    const long long ldc = P.ldc, c_r1 = P.c_r1, c_s2 = P.c_s2;
    if constexpr (M16) {
      // 16x16 blocks: lane l holds rows 4 (l / 16) .. + 3 of column l % 16 of each block
      const int cl = lane & 15, rq = lane >> 4;
      float csum4[JN], csq4[JN];
      if (args.plain_epi) {
        // store-only form (host: plain_epilogue): 16 row offsets per lane computed once, the 64 stores
        // take the column block as an immediate offset; rows past M are dropped by the descriptor
        const auto rc = rsrc_p(C, (unsigned)((long long)M * ldc * 4));
        unsigned roff[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wm0 + 16 * i + 4 * rq + r;
            roff[i][r] = row < M ? (unsigned)row * (unsigned)ldc * 4u : kOOBp;
          }
        const unsigned cb = (unsigned)(n0 + wn0 + cl) * 4u;
        // + beta C (plain_epi 2): each column block's 16 C values loaded before its first store. Interleaved, each
        // load waited for the store before it (they may alias through the one descriptor): 64 serial round trips
        // to memory per lane -- the fine-tune 1x1 data gradients ran 92 us against 51 for the same GEMM shape.
        // (All 64 ahead of the stores spilled this kernel's registers.)
        // The stream-K forms sit at the 256-register cap and spill with those loads in flight: they keep the
        // interleaved form, and the planner runs beta problems data-parallel (x3d_plan).
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          csum4[j] = 0.f;
          csq4[j] = 0.f;
          float cold[4][4];
          if (!SK && args.plain_epi == 2) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                cold[i][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rc, roff[i][r] + cb + 64u * j, 0, 0));
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc4[i][j][r];
              if (args.plain_epi == 2)  // (the general epilogue's fmaf(beta, C, v), bit for bit)
                v = fmaf(beta, SK ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rc, roff[i][r] + cb + 64u * j, 0, 0))
                                  : cold[i][r], v);
              __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, roff[i][r] + cb + 64u * j, 0, 0);
              csum4[j] += v;
              csq4[j] = fmaf(v, v, csq4[j]);
            }
        }
      } else
#pragma unroll
      for (int j = 0; j < JN; ++j) {
        csum4[j] = 0.f;
        csq4[j] = 0.f;
        const int col = n0 + wn0 + 16 * j + cl;
        const bool cok = col < N;
        float bias = 0.f;
        if (cok) {
          if (P.bias) bias += P.bias[col];
          if (P.bias2) bias += P.bias2[col];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = m0 + wm0 + 16 * i + 4 * rq + r;
            if (cok && row < M) {
              float* cp = C + remap(row, c_r1, ldc, c_s2) + col;
              float v = fmaf(acc4[i][j][r], alpha, bias);
              if (beta != 0.f) v = fmaf(beta, *cp, v);
              if (relu) v = fmaxf(v, 0.f);
              *cp = v;
              csum4[j] += v;
              csq4[j] = fmaf(v, v, csq4[j]);
            }
          }
      }
      float* __restrict__ stats = P.stats;
      if (stats != nullptr) {
#pragma unroll
        for (int j = 0; j < JN; ++j) {
          csum4[j] += __shfl_xor(csum4[j], 16, 64);
          csq4[j] += __shfl_xor(csq4[j], 16, 64);
          csum4[j] += __shfl_xor(csum4[j], 32, 64);
          csq4[j] += __shfl_xor(csq4[j], 32, 64);
        }
        if (rq == 0) {  // the wave's 64 rows are one 64-row slice
          const long long sl = (m0 + wm0) >> 6;
#pragma unroll
          for (int j = 0; j < JN; ++j) {
            const int col = n0 + wn0 + 16 * j + cl;
            if (col < N && m0 + wm0 < M) {
              stats[(sl * N + col) * 2 + 0] = csum4[j];
              stats[(sl * N + col) * 2 + 1] = csq4[j];
            }
          }
        }
      }
      return;
    }
    float csum[JN32], csq[JN32];
#pragma unroll
    for (int j = 0; j < JN32; ++j) {
      csum[j] = 0.f;
      csq[j] = 0.f;
      const int col = n0 + wn0 + 32 * j + lr;
      const bool cok = col < N;
      float bias = 0.f;
      if (cok) {
        if (P.bias) bias += P.bias[col];
        if (P.bias2) bias += P.bias2[col];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
          if (cok && row < M) {
            float* cp = C + remap(row, c_r1, ldc, c_s2) + col;
            float v = fmaf(acc[i][j][r], alpha, bias);
            if (beta != 0.f) v = fmaf(beta, *cp, v);
            if (relu) v = fmaxf(v, 0.f);
            *cp = v;
            csum[j] += v;
            csq[j] = fmaf(v, v, csq[j]);
          }
        }
    }
    float* __restrict__ stats = P.stats;
    if (stats != nullptr) {
#pragma unroll
      for (int j = 0; j < JN32; ++j) {
        csum[j] += __shfl_xor(csum[j], 32, 64);
        csq[j] += __shfl_xor(csq[j], 32, 64);
      }
      if (lh == 0) {  // the wave's 64 rows are one 64-row slice
        const long long sl = (m0 + wm0) >> 6;
#pragma unroll
        for (int j = 0; j < JN32; ++j) {
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
    {
      const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = bid & 7;
      bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    }
    const capmi_gemm_problem& P = args.p[0];
    const int tiles_n = args.tiles_n[0];
    const int tiles_m = args.tiles_m[0];
    const int tn = args.tile_cols_first ? bid / tiles_m : bid % tiles_n;
    const int tm = args.tile_cols_first ? bid % tiles_m : bid / tiles_n;
    STAMP(capmi_x3p_stamps, kStSeg, P.K / PBK);
    mainloop(P, tm * PBM, tn * PBN, 0, P.K);
    STAMP(capmi_x3p_stamps, kStMain, 0);
    epilogue(P, tm, tn);
    STAMP(capmi_x3p_stamps, kStEpi, 0);
    clk_report();
    STAMP(capmi_x3p_stamps, kStEnd, 0);
    STAMP_REAL(capmi_x3p_stamps, kStREnd);
    return;
  }

  const capmi_gemm_problem& P = args.p[0];
  const int nkt = args.sk_nkt, tiles_n = args.tiles_n[0], tiles_m = args.tiles_m[0];
  const bool cf = args.tile_cols_first != 0;
  const long long ngrp = args.sk_groups, grp = blockIdx.x % ngrp;
  const long long T = args.sk_units / nkt, G = gridDim.x / ngrp, w = blockIdx.x / ngrp;
  const int nwg = gridDim.x;
  long long pos;
  {
    const int q = nwg >> 3, r = nwg & 7, x = blockIdx.x & 7;
    pos = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (blockIdx.x >> 3);
  }
  const long long ub = grp * T / ngrp * nkt, U = ((grp + 1) * T / ngrp) * nkt - ub;
  const long long u0 = ub + w * U / G, u1 = ub + (w + 1) * U / G;
  constexpr int PART = PBM * PBN;
  int* flags = args.sk_flags;
  // one segment loop (a single mainloop call site keeps the register allocation of the
  // data-parallel kernel): first the hybrid's whole tiles T + pos, T + pos + nwg, ..., then this
  // worker's stream-K tiles from the last to the first
  long long t_dp = T + pos, t_sk = u0 < u1 ? (u1 - 1) / nkt : -1;
  const long long t_sk_end = u0 / nkt;
  for (;;) {
    long long t;
    int ks, ke;
    if (t_dp < T + args.sk_dp_tiles) {
      t = t_dp;
      t_dp += nwg;
      ks = 0;
      ke = nkt;
    } else if (t_sk >= 0 && t_sk >= t_sk_end) {
      t = t_sk--;
      const long long tb = t * nkt;
      ks = (int)(max(u0, tb) - tb);
      ke = (int)(min(u1, tb + nkt) - tb);
    } else {
      break;
    }
    const long long tb = t * nkt;
    const int tm = cf ? (int)(t % tiles_m) : (int)(t / tiles_n), tn = cf ? (int)(t / tiles_m) : (int)(t % tiles_n);
    STAMP(capmi_x3p_stamps, kStSeg, ke - ks);
    mainloop(P, tm * PBM, tn * PBN, ks * PBK, ke * PBK);
    STAMP(capmi_x3p_stamps, kStMain, 0);
    if (ke < nkt) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.sk_part + (long long)blockIdx.x * PART, 0,
                                                        PART * 4, 0x00020000);
      if constexpr (M16) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < JN; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_p, acc4[i][j]), rs,
                                                   ((i * JN + j) * PNT + tid) * 16, 0, kSc1p);
      } else {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < JN32; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            u32x4_p v;
            v.x = __float_as_uint(acc[i][j][4 * q + 0]);
            v.y = __float_as_uint(acc[i][j][4 * q + 1]);
            v.z = __float_as_uint(acc[i][j][4 * q + 2]);
            v.w = __float_as_uint(acc[i][j][4 * q + 3]);
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (((i * JN32 + j) * 4 + q) * PNT + tid) * 16, 0, kSc1p);
          }
      }
      sk_publish<kSkFenced1>(flags + blockIdx.x, tid);
      STAMP(capmi_x3p_stamps, kStPub, 0);
      continue;
    }
    if (ks > 0) {
      for (long long w2 = w - 1;; --w2) {
        const long long b2 = w2 * ngrp + grp;
        sk_consume<kSkFenced1>(flags + b2, flags + gridDim.x, tid);
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(args.sk_part + b2 * PART, 0, PART * 4, 0x00020000);
        if constexpr (M16) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < JN; ++j)
              acc4[i][j] += __builtin_bit_cast(
                  f32x4_p, __builtin_amdgcn_raw_buffer_load_b128(rs, ((i * JN + j) * PNT + tid) * 16, 0, kSc1p));
        } else {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < JN32; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const u32x4_p v =
                  __builtin_amdgcn_raw_buffer_load_b128(rs, (((i * JN32 + j) * 4 + q) * PNT + tid) * 16, 0, kSc1p);
              acc[i][j][4 * q + 0] += __uint_as_float(v.x);
              acc[i][j][4 * q + 1] += __uint_as_float(v.y);
              acc[i][j][4 * q + 2] += __uint_as_float(v.z);
              acc[i][j][4 * q + 3] += __uint_as_float(v.w);
            }
        }
        if (ub + w2 * U / G <= tb) break;
      }
      STAMP(capmi_x3p_stamps, kStCons, 0);
    }
    epilogue(P, tm, tn);
    STAMP(capmi_x3p_stamps, kStEpi, 0);
  }
  clk_report();
  STAMP(capmi_x3p_stamps, kStEnd, 0);
  STAMP_REAL(capmi_x3p_stamps, kStREnd);
}

// x = relu(y * scale[c] + shift[c]) split into three bf16 planes out[p][i] (the x3p A operand)
__global__ void __launch_bounds__(256) bn_relu_split3_kernel(const float4* __restrict__ y, const float* __restrict__ sc,
                                                            const float* __restrict__ sh, long long n4, int C4,
                                                            unsigned long long* __restrict__ out, int relu_bn) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += stride) {
    float4 v = y[i];
    if (relu_bn) {
      const int c = (int)(i % C4) * 4;
      const float4 s = *reinterpret_cast<const float4*>(sc + c), b = *reinterpret_cast<const float4*>(sh + c);
      v = make_float4(fmaxf(fmaf(v.x, s.x, b.x), 0.f), fmaxf(fmaf(v.y, s.y, b.y), 0.f),
                      fmaxf(fmaf(v.z, s.z, b.z), 0.f), fmaxf(fmaf(v.w, s.w, b.w), 0.f));
    }
    unsigned lo[3], hi[3];
    split3_pair(v.x, v.y, lo);
    split3_pair(v.z, v.w, hi);
#pragma unroll
    for (int p = 0; p < 3; ++p) out[p * n4 + i] = (unsigned long long)lo[p] | ((unsigned long long)hi[p] << 32);
  }
}

}  // namespace

int gemm_x3d_launch(const GemmArgs& a, int amode, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(PNT);
  const bool sk = a.sk_workers > 0;
  const bool pro = a.p[0].in_scale != nullptr;
#define X3D_GO(M, S, PR) CAPMI_KLAUNCH((gemm_x3p_kernel<M, S, 32, true, PR>), g, b, 0, s, a)
  if (amode == 2) {
    if (pro) {
      if (sk) X3D_GO(2, true, true); else X3D_GO(2, false, true);
    } else {
      if (sk) X3D_GO(2, true, false); else X3D_GO(2, false, false);
    }
  } else if (pro) {  // 1x1 conv as dense rows with the BN prologue (round 3: no im2col address VALU)
    if (sk) X3D_GO(0, true, true); else X3D_GO(0, false, true);
  } else {
    if (sk) X3D_GO(0, true, false); else X3D_GO(0, false, false);
  }
#undef X3D_GO
  CAPMI_LAUNCH_CHECK();
  return 0;
}

int gemm_x3p_launch(const GemmArgs& a, int amode, int bk, int blocks, hipStream_t s) {
  const dim3 g(blocks), b(PNT);
  const bool sk = a.sk_workers > 0;
  // the two-workgroup form runs data-parallel grids only (its 128-VGPR budget has no room for
  // the stream-K hand-off)
  CAPMI_REQUIRE(bk == 32 || (bk == 16 && !sk), CAPMI_EINVAL);
#define X3P_GO(M, S, BK) CAPMI_KLAUNCH((gemm_x3p_kernel<M, S, BK>), g, b, 0, s, a)
  if (bk == 16) {
    if (amode == 2)
      X3P_GO(2, false, 16);
    else
      X3P_GO(0, false, 16);
  } else if (amode == 2) {
    if (sk)
      X3P_GO(2, true, 32);
    else
      X3P_GO(2, false, 32);
  } else {
    if (sk)
      X3P_GO(0, true, 32);
    else
      X3P_GO(0, false, 32);
  }
#undef X3P_GO
  CAPMI_LAUNCH_CHECK();
  return 0;
}

extern "C" int capmi_bn_relu_split3(const float* y, const float* scale, const float* shift, long long rows, int C,
                                    void* out, void* stream) {
  CAPMI_REQUIRE(y && out && rows >= 0 && C > 0 && C % 4 == 0, CAPMI_EINVAL);
  CAPMI_REQUIRE((scale == nullptr) == (shift == nullptr), CAPMI_EINVAL);
  CAPMI_REQUIRE(aligned16(y) && ((reinterpret_cast<uintptr_t>(out) & 7u) == 0) &&
                    (scale == nullptr || (aligned16(scale) && aligned16(shift))),
                CAPMI_EALIGN);
  const long long n4 = rows * C / 4;
  if (n4 == 0) return 0;
  const unsigned blocks = (unsigned)std::min<long long>(std::max<long long>(cdiv(n4, 256), 1), 8192);
  hipLaunchKernelGGL(bn_relu_split3_kernel, dim3(blocks), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const float4*>(y), scale, shift, n4, C / 4,
                     static_cast<unsigned long long*>(out), scale != nullptr ? 1 : 0);
  CAPMI_LAUNCH_CHECK();
  return 0;
}
