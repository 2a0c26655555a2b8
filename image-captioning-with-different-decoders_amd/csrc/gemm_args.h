// Launch descriptor shared by the GEMM kernels (gemm.hip, gemm_nt.hip).
#pragma once
#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct GemmArgs {
  capmi_gemm_problem p[CAPMI_MAX_GROUP];
  int tiles_begin[CAPMI_MAX_GROUP + 1];
  int tiles_m[CAPMI_MAX_GROUP];
  int tiles_n[CAPMI_MAX_GROUP];
  int kchunk[CAPMI_MAX_GROUP];
  int nprob;
  // stream-K (gemm_nt only, one problem, no k-split): 0 workers = data-parallel launch
  int sk_workers;
  int sk_nkt;            // k-tiles per output tile
  long long sk_units;    // stream-K tiles * sk_nkt
  int sk_dp_tiles;       // tiles after the stream-K ones, run whole by the workers first (a multiple of workers)
  int sk_groups;         // 1, or 8: tiles and workers split into blockIdx%8 groups (XCD-local)
  float* sk_part;        // [workers][BM*BN] parked k-prefix partials
  int* sk_flags;         // [workers + 1], zero between launches; [workers] = spin-timeout flag
  int tile_cols_first;   // x3p: tile t = (tm, tn) as tm = t % tiles_m, tn = t / tiles_m (column-major)
  // x3 kernels (gemm_x3 / x3p / x3d): the store-only epilogue applies (plain_epilogue() below): C = A.B
  // stored through one buffer descriptor with per-row 32-bit offsets computed once per tile -- no
  // per-element 64-bit address, bounds branch, alpha / bias / beta / relu (round 3)
  int plain_epi;
  // x3d (round 4): the two-deep A pipeline for this launch (the planner's rule, gemm.hip x3d_plan)
  int x3d_pipe;
};

// Exact three-term bf16 split of two fp32 values (the x3 arithmetic: h0 = RNE(e), h1 = RNE(e - h0),
// h2 = RNE(e - h0 - h1), every difference exact in fp32), packed: w[p] = (h_p(e1) << 16) | h_p(e0), one
// v_cvt_pk_bf16_f32 per term and pair (round 4: the scalar form converted one value per instruction and
// packed the pairs with v_or_b32_sdwa -- 12 VALU per element in x3d's A staging, 4.5 now)
typedef float capmi_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 capmi_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split3_pair(float e0, float e1, unsigned (&w)[3]) {
  const capmi_f32x2 e = {e0, e1};
  w[0] = __builtin_bit_cast(unsigned, __builtin_convertvector(e, capmi_bf16x2));
  const capmi_f32x2 r1 = e - capmi_f32x2{__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u)};
  w[1] = __builtin_bit_cast(unsigned, __builtin_convertvector(r1, capmi_bf16x2));
  const capmi_f32x2 r2 = r1 - capmi_f32x2{__uint_as_float(w[1] << 16), __uint_as_float(w[1] & 0xffff0000u)};
  w[2] = __builtin_bit_cast(unsigned, __builtin_convertvector(r2, capmi_bf16x2));
}

// Stream-K hand-off of a parked k-prefix partial. Two forms, both ordered without relying on cache-policy
// accidents (MI355X_MICROARCH.md, "Workgroup dispatch, XCD placement & inter-workgroup visibility"):
// * FENCED (round 4; the multi-workgroup-per-CU kernels gemm_nt / gemm_bf16): producer stores -> every wave's
//   vmcnt(0) -> barrier -> one lane's agent-scope release (buffer_wbl2) -> relaxed agent flag store; consumer: one
//   lane's relaxed poll -> agent-scope acquire (buffer_inv sc1) + vmcnt(0) -> barrier -> loads;
// * SC1 (round 5; the one-workgroup-per-CU kernels x3p / x3d / gemm_x3): the same sequence without the two fences,
//   which is the guide's measured-valid table row 1 ("Valid forms besides Guideline 16"): ONE lane of each storing
//   workgroup signals for ALL its stores with an sc1 flag store (a relaxed agent-scope atomic store) after every
//   storing wave's vmcnt(0) and a workgroup barrier; the consumer learns it by an sc1 poll (relaxed agent-scope
//   atomic load) and its other waves load after a barrier that wave joins; hipMalloc memory, one workgroup per CU;
//   every partial store and every partial load is a 16-B sc1 buffer access (kSc1 in the kernels). The release was
//   an L2 write-back of every dirty line of the XCD (the conv outputs these kernels have just stored) at each
//   hand-off, the acquire an L1 invalidate.
// Producer, called by EVERY thread after its partial stores.
template <bool kFenced = true>
__device__ __forceinline__ void sk_publish(int* flag, int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if constexpr (kFenced) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (ROCm 7.2 may drop the fence's own wait)
    }
    __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// Consumer, called by EVERY thread: one lane polls the producer's flag (relaxed, bounded: a timeout raises err and
// leaves the flag), re-arms it (and in the fenced form acquires at agent scope and waits for the invalidate); the
// workgroup barrier then orders every wave's partial loads after the poll.
template <bool kFenced = true>
__device__ __forceinline__ void sk_consume(int* flag, int* err, int tid) {
  if (tid == 0) {
    int spins = 0;
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 && ++spins < (1 << 22))
      __builtin_amdgcn_s_sleep(2);
    if (spins >= (1 << 22))  // never expected: raise the error word (capmi.kernels.sk_check)
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      __hip_atomic_store(flag, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (kFenced) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
}
// the form the one-workgroup-per-CU x3 kernels use (A/B: -DSK_SC1=0 keeps the fences)
#ifndef SK_SC1
#define SK_SC1 1
#endif
constexpr bool kSkFenced1 = SK_SC1 == 0;

__device__ __forceinline__ long long remap(long long r, long long r1, long long ld, long long s2) {
  return r1 > 0 ? (r % r1) * ld + (r / r1) * s2 : r * ld;
}

// Host: does problem p take the store-only epilogue of the x3 kernels with BN-wide column tiles?
// (C = A.B (+ beta C) exactly: no alpha / bias / relu / row remap; whole column tiles; C addressable with
// 32-bit byte offsets; rows past M read zeros in A, so their accumulators add nothing to the BN sums)
inline int plain_epilogue(const capmi_gemm_problem& p, int bn) {
  static const bool off = [] {  // CAPMI_X3_PLAIN_EPI=0: the general epilogue everywhere (A/B arm)
    const char* e = getenv("CAPMI_X3_PLAIN_EPI");
    return e && e[0] == '0';
  }();
  // 1: C = A.B; 2: C = A.B + beta C (read-modify-write through the same offsets; the fine-tune 1x1 data
  // gradients accumulate into the block input's gradient)
  const bool ok = !off && p.alpha == 1.f && p.alpha_ptr == nullptr && p.bias == nullptr && p.bias2 == nullptr &&
                  !p.relu && p.c_r1 <= 0 && p.ksplit == 1 && p.N % bn == 0 && p.ldc >= p.N &&
                  (long long)p.M * p.ldc * 4 < (1LL << 31);
  return ok ? (p.beta == 0.f ? 1 : 2) : 0;
}

// v2 kernel: A K-major dense / NHWC conv / NHWC4 conv1 / M-major (k rows), B = W[N][K] or k rows;
// BM x BN in {128x128, 128x64, 64x64}
int gemm_nt_launch(const GemmArgs& a, int amode, int bmode, int bm, int bn, int blocks, hipStream_t s,
                   int terms = 0, int nt = 256);
// bf16-in/bf16-out conv GEMM (gemm_bf16.hip): BM = 128, BN in {128, 64}, amode 0 (dense) / 2 (conv)
int gemm_bf16_launch(const GemmArgs& a, int amode, int bm, int bn, int blocks, hipStream_t s, int stages);
// fp32-accurate 3-way bf16 split GEMM (gemm_x3.hip): BM = 128, BN in {128, 64}, 512 threads,
// amode 0 (dense) / 2 (conv, optional prologue)
int gemm_x3_launch(const GemmArgs& a, int amode, int bn, int blocks, hipStream_t s);
// x3 with both operands pre-split (gemm_x3p.hip): 256x128 tiles, 512 threads, amode 0 / 2; k-tile depth
// bk (16: two workgroups per CU, data-parallel grids only; 32: one, stream-K capable) is the unit
// of GemmArgs::sk_nkt for it
int gemm_x3p_launch(const GemmArgs& a, int amode, int bk, int blocks, hipStream_t s);
// x3p with A fp32 split in-kernel ("x3d": register-staged A + optional conv BN prologue, LDS-DMA B)
int gemm_x3d_launch(const GemmArgs& a, int amode, int blocks, hipStream_t s);
// short-k streaming x3 GEMM (gemm_x3s.hip): K = 64, N in {64, 128, 256}, dense rows of lda floats
// (optional BN prologue), store-only epilogue; persistent grid over 64-row tiles
int gemm_x3s_launch(const capmi_gemm_problem& p, long long lda, int tiles, int grid, hipStream_t s);
// conv weight gradients (gemm_x3w.hip): A = dY fp32 k rows, B = fp32 k rows (bmode 1) or the NHWC conv input's
// implicit im2col (bmode 2), both split in-kernel; grid = tiles x S k-splits (a.kchunk[0] k-tiles each)
int gemm_x3w_launch(const GemmArgs& a, int bmode, int blocks, hipStream_t s, int terms);  // terms 3 (x3) or 1 (bf16)
// direct 3x3 conv (gemm_x3c.hip): N = 64, stride 1, pad 1, Cin % 32 == 0, W <= gemm_x3c_max_width(); one
// workgroup per 256-pixel tile
int gemm_x3c_launch(const capmi_gemm_problem& p, int tiles, hipStream_t s);
int gemm_x3c_max_width();
bool gemm_x3c_band_fits(const capmi_gemm_problem& p);
// resident workgroups per CU of the NT kernel for a tile shape (LDS / register bound)
// (terms 3: three bf16 LDS planes per operand, 60 KB for 64x64 and >= 90 KB for the larger tiles)
inline int gemm_nt_wg_per_cu(int bm, int bn, int terms = 0) {
  if (terms == 3) return bm == 64 && bn == 64 ? 2 : 1;
  return bm == 64 && bn == 64 ? 4 : 2;
}
