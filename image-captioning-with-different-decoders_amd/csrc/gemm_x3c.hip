// fp32-accurate DIRECT 3x3 convolution ("x3c", round 4): layer1's 3x3 / stride 1 / pad 1
// convs (Cin = Cout = 64 at 56 x 56) in the x3 arithmetic of gemm_x3.hip (operands split exactly into three
// bf16 terms, the six cross products above 2^-23 |a||b| accumulated in fp32 on v_mfma_f32_16x16x32_bf16).
// Replaces the layer1 conv2 of torchvision's Bottleneck (models/encoder.py:88-92, ResNet-101 children).
//
// The implicit-GEMM kernels split an input element once per TAP that reads it (nine times for a 3x3): on
// layer1's short channel axis that VALU work bounded gemm_x3 (7 VALU per MFMA, 26 % MFMA busy). Here a tile
// of 256 consecutive output pixels (row-major over images) stages the input rows those pixels touch -- the
// output rows they span plus one above and below, all W columns -- one 32-channel slice at a time: each input
// element is loaded, BN-applied (+ ReLU) and split ONCE per slice, into three swizzled bf16 planes in LDS.
// The nine taps then read their A fragments from that image at a per-lane pixel offset shifted by
// (kh - 1) rows and (kw - 1) columns. The band is staged in PADDED coordinates (each image's rows framed by a zero
// row above and below, each row by a zero column either side), so that shift is one uniform offset for every
// pixel and tap, with no validity test or select in the tap loop, while the weight's 64 x 32 tap block
// streams by LDS-DMA through a three-deep ring, in gemm_x3p's packed k order (ci / 32, kh, kw, ci % 32).
//
// k order, products and accumulator order are those of the x3p conv path (one workgroup per tile, 32-deep
// k-tiles) on the same split planes (tests/test_gpu_x3.py::test_x3c_direct_conv).
// 512 threads = 8 waves as 4 (64-row slices) x 2 (32 output channels); store-only epilogue.
#include "gemm_args.h"

namespace {

constexpr int CNT = 512;              // threads
constexpr int CBM = 256;              // output pixels per tile
constexpr int CBN = 64;               // output channels (the whole Cout)
constexpr int CW_MAX = 64;            // image width bound
constexpr int CPOS = 640;             // staged band positions (padded rows x (W + 2)); the host checks the bound
constexpr int CA_PLANE = CPOS * 64;   // 64 B per position per plane (32 bf16 channels)
constexpr int CB_PLANE = CBN * 64;    // the weight's 64 x 32 tap block, per plane
constexpr int CB_BUF = 3 * CB_PLANE;  // 12 KiB
constexpr int CB_NBUF = 3;            // weight ring: the DMA runs two taps ahead
constexpr int CPF = (CPOS * 8 + 511) / 512;  // float4 loads per thread to stage one slice of the band
typedef unsigned u32x4_c __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8_c __attribute__((ext_vector_type(8)));
typedef float f32x4_c __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_c;
constexpr unsigned kOOBc = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_c(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
// 16-B chunk c of staged position q sits in slot c ^ (2 ((q >> 2) & 1)). A fragment read's 16 lanes take 16
// consecutive positions starting ANYWHERE (the tap shift (kh - 1) (W + 2) + kw - 1 moves them), in
// ds_read_b128's lane groups {0-3, 12-15, 20-27} ... (MI355X_MICROARCH.md, LDS) with two chunks per group;
// position q starts at bank 16 (q % 4). This slot function keeps every group on 64 distinct banks for every
// starting position (an exhaustive check over the 64 shifts); where a lane group crosses an image row the
// padded band skips two positions, a 2-way conflict on one read in seven at W = 56. gemm_x3p's row swizzle,
// conflict-free for 16-aligned rows, is not (SQ: 37.6 % LDS bank conflicts, 119-121 us), nor was c ^ (q & 3)
__device__ __forceinline__ int apos_off(int q, int c) { return q * 64 + ((c ^ (((q >> 2) & 1) << 1)) << 4); }
// The workgroup barrier of the tap loop. __syncthreads() here compiled to `s_waitcnt vmcnt(0)` + s_barrier
// (its release fence waits for the LDS-DMA and the next slice's staging loads), so every tap drained the DMAs
// issued two taps ahead and the staging loads at once; this barrier waits only for the wave's LDS operations
// (its ds_writes / ds_reads), the counted `s_waitcnt vmcnt` before it retiring the DMA the next tap reads.
// The asm's memory clobber keeps the compiler from moving LDS accesses across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// weight rows: gemm_x3p's 16x16x32 swizzle (slot pattern [0, 2, 3, 1][(r >> 2) & 3])
__device__ __forceinline__ int bswz(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }

template <bool PRO>
__global__ void __launch_bounds__(CNT) __attribute__((amdgpu_waves_per_eu(2)))
gemm_x3c_kernel(const capmi_gemm_problem P) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[3 * CA_PLANE + CB_NBUF * CB_BUF];
  unsigned char* const Al = lds;
  unsigned char* const Bl = lds + 3 * CA_PLANE;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm0 = (wid >> 1) * 64, wn0 = (wid & 1) * 32;
  const int M = P.M, H = P.cH, W = P.cW, Cin = P.cCin;
  const int rows_all = P.cN * H;  // global input rows (image, ih)
  // padded coordinates: image n's rows -1 .. H are padded rows n (H + 2) .. n (H + 2) + H + 1, columns -1 .. W are
  // 0 .. W + 1; the padding is zeros, so every tap of every pixel reads a staged position (no validity test, no
  // select) at the uniform offset (kh - 1) (W + 2) + (kw - 1) from the pixel's centre
  const int Hp = H + 2, Wp = W + 2;
  // XCD-aware tile order (consecutive tiles -- overlapping bands -- on one XCD)
  int bid = blockIdx.x;
  {
    const int nwg = gridDim.x, q = nwg >> 3, r = nwg & 7, x = bid & 7;
    bid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
  }
  const int p0 = bid * CBM;
  auto prow = [&](int p) {  // padded centre row of output pixel p
    const int g = p / W, n = g / H;
    return n * Hp + (g - n * H) + 1;
  };
  const int rmin = prow(p0) - 1;                                 // first staged padded row
  const int npos = (prow(min(p0 + CBM, M) - 1) + 2 - rmin) * Wp;  // staged positions (<= CPOS: host)

  const auto rx = rsrc_c(P.A, (unsigned)((long long)rows_all * W * Cin * 4));
  const auto rb = rsrc_c(P.B, (unsigned)(3LL * CBN * P.ldb * 2));
  const unsigned ss_bytes = PRO ? (unsigned)(Cin * 4) : 0u;
  const auto rsc = rsrc_c(PRO ? (const void*)P.in_scale : P.B, ss_bytes);
  const auto rsh = rsrc_c(PRO ? (const void*)P.in_shift : P.B, ss_bytes);

  // this lane's fragment pixels: rows wm0 + 16 i + (lane & 15) of the tile, chunk lane >> 4; their centre
  // positions in the band (a pixel past M reads a position inside the band; its rows are zeroed in the epilogue)
  const int c16 = lane >> 4, r16 = lane & 15;
  int fq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = p0 + wm0 + 16 * i + r16;
    fq[i] = p < M ? (prow(p) - rmin) * Wp + (p % W) + 1 : Wp + 1;
  }

  // weight tap block DMA: waves 0-3 each move 16 rows x 64 B of each plane (rows 16 w + lane / 4, slot lane % 4)
  const int drow = lane >> 2, dslot = lane & 3;
  const bool bw = wid < 4;
  const int br = wid * 16 + drow;
  const unsigned b_base = (unsigned)(((long long)br * P.ldb + ((dslot ^ bswz(br)) * 8)) * 2);
  const unsigned pB2 = (unsigned)((long long)CBN * P.ldb * 2);
  auto b_dma = [&](int kt, int buf) {  // k-tile kt = slice * 9 + tap of the packed weight
    if (!bw) return;
    const unsigned off = b_base + (unsigned)(kt * 32) * 2u;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_c)(Bl + buf * CB_BUF + p * CB_PLANE + wid * 1024), 16,
                                               off + p * pB2, 0, 0, 0);
  };
  // input slice s of the band: float4 f = tid + 512 j is position f / 8 = tid / 8 + 64 j, channels 4 (f % 8) .. + 3.
  // Each slot's source offset (or none: padding / past the band) is found once per tile; a slice adds 128 B.
  // Loaded into registers one slice ahead, written as the three planes after the previous slice's last tap
  const int ch8 = (tid & 7) * 4;
  unsigned soff[CPF];
#pragma unroll
  for (int j = 0; j < CPF; ++j) {
    const int q = (tid >> 3) + 64 * j;
    const int br = q / Wp, c = q - br * Wp;
    const int R = rmin + br, n = R / Hp, ih = R - n * Hp - 1, iw = c - 1;
    const bool ok = q < npos && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W && n < P.cN;
    soff[j] = ok ? (unsigned)((((long long)(n * H + ih) * W + iw) * Cin + ch8) * 4) : kOOBc;
  }
  float4 pf[CPF];
  float4 pf_sc = make_float4(1.f, 1.f, 1.f, 1.f), pf_sh = make_float4(0.f, 0.f, 0.f, 0.f);
  auto stage_load = [&](int s) {
    if (PRO) {
      const unsigned ch = (unsigned)(s * 32 + ch8) * 4u;
      pf_sc = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsc, ch, 0, 0));
      pf_sh = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsh, ch, 0, 0));
    }
#pragma unroll
    for (int j = 0; j < CPF; ++j)
      pf[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rx, soff[j] == kOOBc ? kOOBc : soff[j] + (unsigned)s * 128u, 0, 0));
  };
  auto stage_write = [&]() {
#pragma unroll
    for (int j = 0; j < CPF; ++j) {
      const int q = (tid >> 3) + 64 * j;
      if (q >= npos) break;
      float4 x = pf[j];
      if (PRO) x = make_float4(fmaxf(fmaf(x.x, pf_sc.x, pf_sh.x), 0.f), fmaxf(fmaf(x.y, pf_sc.y, pf_sh.y), 0.f),
                               fmaxf(fmaf(x.z, pf_sc.z, pf_sh.z), 0.f), fmaxf(fmaf(x.w, pf_sc.w, pf_sh.w), 0.f));
      if (soff[j] == kOOBc) x = make_float4(0.f, 0.f, 0.f, 0.f);  // padding: zeros AFTER the BN
      unsigned lo[3], hi[3];
      split3_pair(x.x, x.y, lo);
      split3_pair(x.z, x.w, hi);
      const int c8 = tid & 7;
      const int o = apos_off(q, c8 >> 1) + (c8 & 1) * 8;
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<uint2*>(Al + p * CA_PLANE + o) = make_uint2(lo[p], hi[p]);
    }
  };

  f32x4_c acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_c{0.f, 0.f, 0.f, 0.f};
  const int nslice = Cin / 32, nkt = nslice * 9;
  // weight ring: tap kt's block in buffer kt % 3, its DMA issued two taps ahead (past the last tap: out of
  // range, zeros into a buffer nobody reads -- so the count of DMA wave-instructions in flight is fixed)
#pragma unroll
  for (int t = 0; t < CB_NBUF - 1; ++t) b_dma(t < nkt ? t : 1 << 20, t);
  int bcur = 0;  // kt % 3
  stage_load(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  stage_write();
  __syncthreads();
  int kt = 0;
  for (int s = 0; s < nslice; ++s) {
    for (int tap = 0; tap < 9; ++tap, ++kt) {
      const int buf = bcur;
      const int bnext = bcur == 0 ? 2 : bcur - 1;  // (kt + 2) % 3: last read by tap kt - 1
      b_dma(kt + 2 < nkt ? kt + 2 : 1 << 20, bnext);
      bcur = bcur == 2 ? 0 : bcur + 1;
      // (the vmcnt counts below rely on this order: the staging loads after this tap's DMA)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const bool pre = tap == 0 && s + 1 < nslice;
      if (pre) stage_load(s + 1);  // the next slice's band, into registers, while this slice's taps run
      const int kh = tap / 3, kw = tap - kh * 3;
      const int dq = (kh - 1) * Wp + (kw - 1);
      const unsigned char* B_ = Bl + buf * CB_BUF;
      bf16x8_c b[2][3];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn0 + 16 * j + r16;
#pragma unroll
        for (int p = 0; p < 3; ++p)
          b[j][p] = *reinterpret_cast<const bf16x8_c*>(B_ + p * CB_PLANE + r * 64 + ((c16 ^ bswz(r)) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int o = apos_off(fq[i] + dq, c16);
        bf16x8_c a[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) a[p] = *reinterpret_cast<const bf16x8_c*>(Al + p * CA_PLANE + o);
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // per accumulator the six products smallest terms first (x3p's order)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][2], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[j][0], acc[i][j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][0], acc[i][j], 0, 0, 0);
        }
      }
      // the next tap's weight block: issued before the later DMA (3 wave-instructions) and, in the slice's
      // first two taps, before the next slice's CPF (+ 2) staging loads
      if (tap <= 1 && s + 1 < nslice) {
        if (PRO)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 + CPF + 2) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 + CPF) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      }
      lds_barrier();
    }
    if (s + 1 < nslice) {  // every wave is past the slice's last tap (barrier above): the band is free
      stage_write();
      lds_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the DMAs past the last tap)

  // store-only epilogue (x3p's form): lane l holds rows 4 (l / 16) .. + 3 of column l % 16 of each 16x16 block;
  // rows past M are dropped by the descriptor and zeroed for the statistics
  const auto rc = rsrc_c(P.C, (unsigned)((long long)M * P.ldc * 4));
  const int cl = lane & 15, rq = lane >> 4;
  unsigned roff[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = p0 + wm0 + 16 * i + 4 * rq + r;
      roff[i][r] = row < M ? (unsigned)row * (unsigned)P.ldc * 4u : kOOBc;
    }
  float* __restrict__ stats = P.stats;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const unsigned cb = (unsigned)(wn0 + 16 * j + cl) * 4u;
    float cs = 0.f, cq = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // (a row past M read band data: its store is dropped by the descriptor, its value kept out of the sums)
        const float v = roff[i][r] == kOOBc ? 0.f : acc[i][j][r];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, roff[i][r] + cb, 0, 0);
        cs += v;
        cq = fmaf(v, v, cq);
      }
    if (stats != nullptr) {  // the wave's 64 rows are one 64-row slice (x3p's reduction order)
      cs += __shfl_xor(cs, 16, 64);
      cq += __shfl_xor(cq, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      cq += __shfl_xor(cq, 32, 64);
      if (rq == 0 && p0 + wm0 < M) {
        const long long sl = (p0 + wm0) >> 6;
        const int col = wn0 + 16 * j + cl;
        stats[(sl * CBN + col) * 2 + 0] = cs;
        stats[(sl * CBN + col) * 2 + 1] = cq;
      }
    }
  }
}

}  // namespace

int gemm_x3c_launch(const capmi_gemm_problem& p, int tiles, hipStream_t s) {
  const dim3 g(tiles), b(CNT);
  if (p.in_scale)
    CAPMI_KLAUNCH((gemm_x3c_kernel<true>), g, b, 0, s, p);
  else
    CAPMI_KLAUNCH((gemm_x3c_kernel<false>), g, b, 0, s, p);
  CAPMI_LAUNCH_CHECK();
  return 0;
}

int gemm_x3c_max_width() { return CW_MAX; }

// every tile's staged band (its padded rows x (W + 2)) fits the CPOS positions of LDS -- the kernel's npos, for
// each tile (a few hundred tiles; the host runs it once per plan)
bool gemm_x3c_band_fits(const capmi_gemm_problem& p) {
  const long long H = p.cH, W = p.cW, Hp = H + 2, Wp = W + 2, M = p.M;
  auto prow = [&](long long q) {
    const long long g = q / W, n = g / H;
    return n * Hp + (g - n * H) + 1;
  };
  for (long long p0 = 0; p0 < M; p0 += CBM) {
    const long long last = (p0 + CBM < M ? p0 + CBM : M) - 1;
    if ((prow(last) + 2 - (prow(p0) - 1)) * Wp > CPOS) return false;
  }
  return true;
}
