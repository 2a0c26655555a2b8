/*
 * capmi.h -- C ABI of libcapmi.so, the MI355X (gfx950) kernels behind the
 * 'attention' captioning training step of
 * SarahAlkhateeb/Image-Captioning-with-Different-Decoders.
 *
 * The reference has no native boundary: every device op is a PyTorch library
 * op called from Python. Each entry point below replaces the reference op(s)
 * cited next to it (file:line into the reference). Conventions:
 *   - plain device pointers (fp32 unless the name says f64), sizes as ints,
 *     the HIP stream as an opaque `void*` (hipStream_t), no torch types;
 *   - every call returns 0 on success, else a CAPMI_E* code or a hipError_t
 *     (>= 1000 is capmi's own, see capmi_strerror);
 *   - the library never allocates or frees device memory: every output and
 *     workspace is passed in by the caller (PyTorch's caching allocator);
 *   - launches only, no synchronisation: every call is safe inside a
 *     hipStreamBeginCapture / hipGraph.
 * Layouts: activations are NHWC (channels innermost); decoder per-step state
 * is time-major (T, B, ...); weights stay in their nn.Module layout except
 * the conv weights, which are packed once to [Cout][KH][KW][Cin].
 */
#ifndef CAPMI_H
#define CAPMI_H

#ifdef __cplusplus
extern "C" {
#endif

#define CAPMI_ABI_VERSION 26

#define CAPMI_OK 0
#define CAPMI_EINVAL 1001   /* bad shape / argument */
#define CAPMI_EALIGN 1002   /* pointer or stride not aligned as required */
#define CAPMI_ERANGE 1003   /* size outside what the kernel supports */

#define CAPMI_MAX_GROUP 4

/* ------------------------------------------------------------------------
 * GEMM / implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32).
 * C[M,N] = alpha * op(A)[M,K] * op(B)[K,N] (+ bias) (+ beta*C) (relu)
 * Replaces: nn.Linear forward/backward (models/attention.py:33-35,54-55,
 * 110-114,162-163,270,279), the LSTMCell gate GEMMs (:108-109,277-278) and
 * every Conv2d of torchvision's ResNet-101 (models/encoder.py:88-91,107).
 * ---------------------------------------------------------------------- */
enum capmi_amode {
  CAPMI_A_KMAJOR = 0,   /* A[m][k]: off(m) + k, off(r) = (r % a_r1)*lda + (r / a_r1)*a_s2 */
  CAPMI_A_MMAJOR = 1,   /* A[k][m]: off(k) + m  (i.e. A^T of a row-major matrix)          */
  CAPMI_A_CONV_NHWC = 2,/* implicit im2col of an NHWC input, k = (kh, kw, ci), Cin % 16 == 0 */
  CAPMI_A_CONV_NCHW = 3,/* implicit im2col of an NCHW input, k = (ci, kh, kw) (generic kernel) */
  CAPMI_A_CONV_NHWC4 = 4/* implicit im2col of an NHWC input padded to Cin = 4 (conv1 on capmi_image_nhwc4 output), k = (kh, kw, c4) */
};
enum capmi_bmode {
  CAPMI_B_NMAJOR_W = 0, /* B[k][n] = W[n][k] (nn.Linear weight / packed conv weight), ldb = row stride of W */
  CAPMI_B_KROWS = 1,    /* B[k][n] row-major, ldb = row stride */
  CAPMI_B_CONV_NHWC = 2 /* conv weight gradient: B[k][n] = implicit im2col of the NHWC input (conv geometry
                           fields), k = output pixel (img, oh, ow), n = (kh, kw, ci); A must be CAPMI_A_MMAJOR
                           (dY stored as [pixel][Cout]); C = dW[Cout][KH][KW][Cin]; in_scale/in_shift, when
                           set, are the BN-apply+ReLU prologue of the conv's input (Cin % 4 == 0) */
};
/* tile: 128x128, 64x64, 128x64, or AUTO (chosen from the grid size; what the encoder uses);
 * CAPMI_TILE_128_W8: 128x128 with 512-thread workgroups (8 waves, one workgroup per CU), forward
 * modes (A row-major / conv x W[N][K]) of capmi_gemm_sk only */
enum capmi_tile { CAPMI_TILE_128 = 0, CAPMI_TILE_64 = 1, CAPMI_TILE_128x64 = 2, CAPMI_TILE_AUTO = 3,
                  CAPMI_TILE_128_W8 = 4 };

typedef struct capmi_gemm_problem {
  int M, N, K;
  int ksplit;            /* >= 1. split z writes C + z*c_split_stride (raw partials, bias only on z = 0) */
  const float* A; long long lda, a_r1, a_s2;   /* a_r1 <= 0 means "no 2-level row remap" */
  const float* B; long long ldb;
  float* C; long long ldc, c_r1, c_s2, c_split_stride;
  const float* bias;     /* [N] or NULL */
  const float* bias2;    /* [N] or NULL (added as well: LSTM b_ih + b_hh) */
  const float* alpha_ptr;/* device scalar multiplying A*B, or NULL */
  float alpha, beta;     /* host scalars; beta != 0 reads C */
  int relu;
  float* stats;          /* NULL or [ceil(M/64)][N][2]: per 64-row slice (sum, sumsq) of the stored C (BN-train stats) */
  /* implicit-GEMM conv geometry (A = input activation, modes 2/3) */
  int cN, cH, cW, cCin, cKH, cKW, cStride, cPad, cHo, cWo;
  const float* in_scale; /* NULL or [Cin]: A element := relu(x*in_scale[ci] + in_shift[ci]) in-bounds (BN-apply+ReLU prologue) */
  const float* in_shift;
} capmi_gemm_problem;

int capmi_gemm(const capmi_gemm_problem* problems, int nprob, int amode, int bmode, int tile,
               void* stream);
/* rows of the statistics buffer capmi_gemm writes for M rows: ceil(M/64) (tile ignored) */
int capmi_gemm_stat_tiles(int M, int tile);
/* Stream-K form of capmi_gemm for ONE problem (every conv of the encoder, the decoder's hoisted
 * GEMMs and weight gradients): when the data-parallel grid would end in a partial round of
 * workgroups (e.g. 784 64x64 tiles on 1024 resident slots), the (tile, k-tile) iteration
 * space is instead split evenly over one persistent workgroup per resident slot; the k-prefix
 * of a tile shared by two workgroups is parked in `workspace` and added, in a fixed order, by
 * the workgroup that owns the tile's k-end (deterministic result). Same output contract
 * (alpha/bias/beta/relu/stats/prologue) as capmi_gemm; other cases launch capmi_gemm.
 * workspace: capmi_gemm_workspace_bytes() bytes, 16-B aligned, ZEROED by the caller once
 * before first use (the kernel leaves it reusable); one workspace per concurrently running
 * stream. */
long long capmi_gemm_workspace_bytes(void);
/* Bytes at the start of the stream-K workspace holding the hand-off flags and the spin-timeout
 * error word. Every one of these int32 words is zero between launches; a nonzero word after a
 * launch has completed means a hand-off timed out (result invalid): the host checks this at its
 * sync points (capmi.kernels.sk_check), raises, and re-zeroes the workspace. */
long long capmi_gemm_workspace_flag_bytes(void);
int capmi_gemm_sk(const capmi_gemm_problem* problem, int amode, int bmode, int tile, void* workspace,
                  long long ws_bytes, void* stream);
/* capmi_gemm_sk with flags: CAPMI_GEMM_BF16 = operands rounded to bf16 (RNE) when staged to LDS,
 * v_mfma_f32_32x32x16_bf16 with fp32 accumulation (the bf16 configs, BASELINE config 5); A row-major
 * (CAPMI_A_KMAJOR / CAPMI_A_CONV_NHWC / CAPMI_A_CONV_NHWC4) x B = W[N][K] (CAPMI_B_NMAJOR_W) only.
 * Inputs, outputs, statistics and the prologue stay fp32. */
#define CAPMI_GEMM_BF16 1
/* CAPMI_GEMM_BF16_IO (alone): A, B and C are bf16 buffers (the float* fields carry bf16 pointers;
 * leading dimensions in elements), v_mfma_f32_32x32x16_bf16 with fp32 accumulation, C rounded to bf16
 * (RNE) once, `stats` fp32 from the stored values. A = CAPMI_A_KMAJOR (lda % 8 == 0) or
 * CAPMI_A_CONV_NHWC (Cin % 64 == 0) x B = W[N][K] (CAPMI_B_NMAJOR_W, ldb % 8 == 0); K % 64 == 0;
 * alpha 1, beta 0, no bias / relu / ksplit, no prologue (the conv input is relu(bn(y)) materialised in bf16
 * by capmi_bn_relu_bf16). Tile 128x128, or 128x64 for CAPMI_TILE_128x64 / N <= 64. */
#define CAPMI_GEMM_BF16_IO 2
/* CAPMI_GEMM_X3 (alone): fp32-accurate GEMM on the bf16 matrix cores. A is fp32 (CAPMI_A_KMAJOR,
 * lda % 4 == 0, or CAPMI_A_CONV_NHWC, Cin % 32 == 0, with the optional BN-apply + ReLU prologue);
 * B is the fp32 weight W[N][K] pre-split by capmi_split3_bf16 into three bf16 planes [3][N][ldb]
 * (ldb % 8 == 0, ldb >= K; the B pointer is plane 0); K % 32 == 0; C, bias, alpha/beta, relu,
 * output row remap and `stats` as capmi_gemm; no ksplit. Each operand is split exactly into three
 * bf16 terms and the six cross products above 2^-23 |a||b| are accumulated in fp32 on
 * v_mfma_f32_32x32x16_bf16 (the dropped three are below the fp32 rounding level). Tile 128x128
 * (128x64 for CAPMI_TILE_128x64 / N <= 64), 512 threads, one workgroup per CU; stream-K as
 * capmi_gemm_sk. */
#define CAPMI_GEMM_X3 4
/* CAPMI_GEMM_X3P (alone): as CAPMI_GEMM_X3 with A pre-split too: the A pointer is plane 0 of three
 * bf16 planes (dense [3][M][lda], lda % 8 == 0; or the NHWC conv input [3][N*H*W][Cin], Cin % 32 ==
 * 0, from capmi_bn_relu_split3 / capmi_split3_bf16); no prologue. For a conv the k order of B is
 * (ci / 32, kh, kw, ci % 32) -- the KH*KW taps of a 32-channel slice consecutive, so a tile re-reads
 * its input rows within KH*KW k-tiles (L2-resident); 1x1 convs: the plain order. Tile 256x128,
 * 512 threads, LDS-DMA staging; k-tiles of 16 with two workgroups per CU (data-parallel grid)
 * when there are >= 2 x CUs tiles filling >= 70 % of the last round, else k-tiles of 32, one
 * workgroup per CU, stream-K as capmi_gemm_sk. */
#define CAPMI_GEMM_X3P 8
/* CAPMI_GEMM_X3D (alone): the CAPMI_GEMM_X3P kernel with A the fp32 operand itself (CAPMI_A_KMAJOR,
 * lda % 4 == 0, or CAPMI_A_CONV_NHWC, Cin % 32 == 0, with the optional BN-apply + ReLU prologue),
 * split into the three bf16 planes in-kernel while B (pre-split, x3p k order) is LDS-DMA staged;
 * 256x128 tiles, k-tiles of 32, one workgroup per CU, stream-K as capmi_gemm_sk. */
#define CAPMI_GEMM_X3D 32
/* CAPMI_GEMM_X3S (alone, ABI 17): the CAPMI_GEMM_X3 arithmetic for the short-k convs (layer1's K = 64):
 * K == 64, N in {64, 128, 256}; A fp32 dense rows (CAPMI_A_KMAJOR, lda % 4 == 0) or a 1x1 / stride-1 /
 * unpadded NHWC conv input with Cin == 64 (CAPMI_A_CONV_NHWC, optional BN-apply + ReLU prologue); B the
 * three bf16 planes of capmi_split3_bf16 (ldb % 8 == 0); C = A.B only (alpha 1, no bias / beta / relu /
 * remap / ksplit) with the optional `stats`. Persistent 256-thread workgroups (two per CU) stream 64-row
 * tiles with the weight held in registers; the workspace is not used (may be NULL). */
#define CAPMI_GEMM_X3S 64
/* CAPMI_GEMM_X3W (alone, ABI 19): the conv WEIGHT gradient in the CAPMI_GEMM_X3 arithmetic, C[M][N] =
 * sum_k A[k][m] B[k][n] with k = output pixel: A = dY fp32 (CAPMI_A_MMAJOR, [K][lda], lda % 4 == 0) and B =
 * the conv input fp32 as k rows (CAPMI_B_KROWS, [K][ldb]) or through its implicit im2col (CAPMI_B_CONV_NHWC,
 * n = (kh, kw, ci), the packed [Cout][KH][KW][Cin] weight order, Cin % 4 == 0), with the optional BN-apply +
 * ReLU prologue on B (in_scale / in_shift [Cin]; padding taps zero after it); M % 4 == 0, N % 4 == 0, K > 0; alpha /
 * beta only, no bias / relu / stats / ksplit. Both operands are split into three bf16 terms in the kernel and
 * read back transposed (ds_read_b64_tr_b16); 256x128 tiles, 512 threads, one workgroup per CU. With alpha 1
 * and beta 0 the pixel range is split over several workgroups whose partial slabs go to the workspace (as
 * capmi_gemm_sk's) and are summed in a fixed order (capmi_splitk_reduce); capmi_gemm_sk_plan reports the
 * split count in `generic`. (ABI 26) CAPMI_GEMM_X3W | CAPMI_GEMM_BF16: the same kernel with one term per operand --
 * each fp32 value rounded to bf16 (RNE), one product, fp32 accumulation: the CAPMI_GEMM_BF16 operand contract for
 * weight gradients (gemm_w16_kernel). */
#define CAPMI_GEMM_X3W 128
/* CAPMI_GEMM_X3C (alone, ABI 23): DIRECT 3x3 convolution in the CAPMI_GEMM_X3 arithmetic for short-channel
 * layers (layer1's 3x3): CAPMI_A_CONV_NHWC with KH = KW = 3, stride 1, pad 1, Cin % 32 == 0, W <= 64, the
 * optional BN-apply + ReLU prologue; N == 64; B = the weight's three bf16 planes in CAPMI_GEMM_X3P's packed k
 * order (ldb == K); C = A.B only (alpha 1, no bias / beta / relu / remap / ksplit) with the optional `stats`.
 * Each tile of 256 output pixels splits the input rows it touches once per 32-channel slice and reads the nine
 * taps from that image (the k order and products of CAPMI_GEMM_X3P). The workspace is not used (may be NULL). */
#define CAPMI_GEMM_X3C 256
/* CAPMI_GEMM_SPLIT3 (alone): fp32 A and B, both split exactly into three bf16 terms when staged to
 * LDS (the CAPMI_GEMM_X3 arithmetic with no pre-split operand: fp32-accurate on the bf16 matrix
 * cores). Dense modes only: CAPMI_A_KMAJOR x CAPMI_B_NMAJOR_W / CAPMI_B_KROWS and CAPMI_A_MMAJOR x
 * CAPMI_B_KROWS (the decoder's forward, data-gradient and weight-gradient GEMMs); K % 4 == 0, 16-B
 * aligned operands, M % 4 == 0 for CAPMI_A_MMAJOR, N % 4 == 0 for CAPMI_B_KROWS; no prologue, no
 * stats. Tiles 64x64 (two workgroups per CU), 128x64, 128x128 (one). Also accepted by
 * capmi_gemm_ex (grouped problems, ksplit). CAPMI_GEMM_BF16 accepts the same dense modes (bf16
 * operands, one product). A problem of these modes that the split forms do not cover (an operand
 * not 16-B aligned or a stride / size not a multiple of 4: the generic-kernel shapes) runs the fp32
 * kernel instead. */
#define CAPMI_GEMM_SPLIT3 16
/* capmi_gemm with flags 0 / CAPMI_GEMM_BF16 / CAPMI_GEMM_SPLIT3 (dense modes above; grouped problems,
 * ksplit and the epilogue as capmi_gemm). Replaces the decoder's per-timestep nn.Linear / LSTMCell
 * GEMMs (models/attention.py:55,270,277-278) and their backward. */
int capmi_gemm_ex(const capmi_gemm_problem* problems, int nprob, int amode, int bmode, int tile, int flags,
                  void* stream);
int capmi_gemm_sk_ex(const capmi_gemm_problem* problem, int amode, int bmode, int tile, int flags, void* workspace,
                     long long ws_bytes, void* stream);
/* the launch capmi_gemm_sk_ex(..., flags, ...) would make (no GPU work): tile bm x bn, stream_k 0/1,
 * generic = 1 when the problem falls back to the generic kernel (for CAPMI_GEMM_X3P: the k-tile
 * depth, 16 or 32), threads = workgroup size (256, or 512 for the CAPMI_TILE_128_W8 form AUTO picks
 * for wide convs). Used by the benchmark to attribute
 * time. Any out pointer may be NULL. */
int capmi_gemm_sk_plan(const capmi_gemm_problem* problem, int amode, int bmode, int tile, int flags, int* bm,
                       int* bn, int* stream_k, int* generic, int* threads);
/* (ABI 25) for CAPMI_GEMM_BF16_IO the plan is the launcher's own (generic = the LDS stages: 1 the one-stage short-k
 * form, 2 or 4 the data-parallel LDS-DMA ring, 2 with stream_k the register-staged stream-K form; stream_k as if a
 * workspace were passed; threads 512 for the 128-column DMA ring). The name of the last GEMM kernel instantiation this host thread launched (demangled,
 * without return type and parameters, as rocprofv3 lists it) into out[n]: what a plan query's name must equal.
 * Needs the HIP runtime's code-object registry (a GPU process). */
int capmi_last_launch_name(char* out, int n);

/* sum of S partial slabs: out[r][c] = sum_s in[s*slab + r*ld_in + c] (+ bias[c]); rows x cols */
int capmi_splitk_reduce(const float* in, int S, long long slab, int rows, int cols, long long ld_in,
                        const float* bias, float* out, long long ld_out, void* stream);
/* column sums of a rows x cols row-major matrix (bias gradients): out[c] = scale * sum_r in[r*ld + c].
 * work must hold CAPMI_COLSUM_GROUPS * cols floats. accumulate != 0 adds into out. */
#define CAPMI_COLSUM_GROUPS 64
int capmi_colsum(const float* in, int rows, int cols, long long ld, float scale, float* work,
                 float* out, int accumulate, void* stream);

/* ------------------------------------------------------------------------
 * ResNet-101 encoder pieces (models/encoder.py:88-110, BatchNorm in train
 * mode because the reference calls encoder.train(): models/attention.py:374).
 * ---------------------------------------------------------------------- */
/* [Cout][Cin][KH][KW] -> [Cout][KH][KW][Cin] */
int capmi_conv_weight_pack(const float* w, int Cout, int Cin, int KH, int KW, float* out, void* stream);
/* same, channels zero-padded to Cin_pad >= Cin: [Cout][KH][KW][Cin_pad] (conv1: Cin_pad = 4) */
int capmi_conv_weight_pack_pad(const float* w, int Cout, int Cin, int KH, int KW, int Cin_pad, float* out,
                               void* stream);
/* images NCHW (C <= 4) -> NHWC with 4 channels, zero padded (input of the CAPMI_A_CONV_NHWC4 conv1;
 * the reference's imgs tensor, models/attention.py:389 -> encoder(imgs)) */
int capmi_image_nhwc4(const float* in, int N, int C, int H, int W, float* out, void* stream);
/* BatchNorm2d(train) finalize from capmi_gemm stats: mean/var over `count` rows, then
 * scale = gamma*rsqrt(var+eps), shift = beta - mean*scale; running stats updated in place
 * (momentum, unbiased var) when running_mean != NULL. mean/var out (may be NULL). The fp64 sums run
 * in one canonical order (csrc/bn_final.h), reproducible op for op on the host.
 * work: unused since round 4 and may be NULL (kept in the signature; older callers pass
 * CAPMI_BN_WORK_DOUBLES(C) doubles). */
#define CAPMI_BN_WORK_DOUBLES(C) (64 + 64 * (long long)(C)) /* C <= 8192 */
int capmi_bn_finalize(const float* stats, int tiles, int C, long long count, const float* gamma,
                      const float* beta, float* running_mean, float* running_var, float momentum,
                      float eps, float* scale, float* shift, float* save_mean, float* save_var,
                      void* work, void* stream);
/* BatchNorm2d(eval): scale/shift from running statistics */
int capmi_bn_eval_params(const float* gamma, const float* beta, const float* running_mean,
                         const float* running_var, int C, float eps, float* scale, float* shift,
                         void* stream);
/* bf16 activations (the bf16 encoder of BASELINE config 5, capmi_gemm_sk_ex + CAPMI_GEMM_BF16_IO):
 * x = relu(y*scale[c] + shift[c]) on a bf16 NHWC tensor of rows x C (C % 8 == 0): the BN-apply+ReLU
 * of a conv input, materialised once (models/encoder.py:88-91 via torchvision's Bottleneck) */
int capmi_bn_relu_bf16(const void* y, const float* scale, const float* shift, long long rows, int C, void* x,
                       void* stream);
/* bf16 bottleneck tail: out = relu(y*s + b + (res_scale ? res*rs + rb : res)) */
int capmi_bn_add_relu_bf16(const void* y, const float* scale, const float* shift, const void* res,
                           const float* res_scale, const float* res_shift, long long rows, int C, void* out,
                           void* stream);
/* fp32 -> bf16 (RNE), n % 8 == 0 (layer1 input, packed conv weights) */
int capmi_f32_to_bf16(const float* in, long long n, void* out, void* stream);
/* AdaptiveAvgPool2d((OH, OW)) of a bf16 NHWC map -> fp32 NHWC (models/encoder.py:92,108-109) */
int capmi_adaptive_avgpool_bf16(const void* x, int N, int H, int W, int C, int OH, int OW, float* out,
                                void* stream);
/* Image preprocessing: Resize((OH, OW)) -> ToTensor -> Normalize(mean, std) of the
 * reference's transform (models/attention.py:296-301, dataset.py:55-59) for a batch of decoded RGB
 * uint8 HWC images of any sizes, bit-identical to torchvision's PIL path (Pillow's antialiased
 * bilinear resample, 22-bit fixed point, uint8 rounding after each pass). src: packed images,
 * image b at src + offsets[b] with heights[b] x widths[b] (device arrays); max_h/max_w bound them;
 * mean/std: 3 HOST floats each; tmp: B * max_h * OW * 3 bytes of scratch; out: (B, 3, OH, OW) fp32. */
int capmi_resize_normalize_u8(const unsigned char* src, const long long* offsets, const int* heights,
                              const int* widths, int B, int max_h, int max_w, int OH, int OW, const float* mean,
                              const float* std, void* tmp, float* out, void* stream);
/* taps per output index of that resample (2*ceil(max(1, in/out)) + 1); host-only helper */
int capmi_resize_taps_max(int in_size, int out_size);
/* Bottleneck tail: out = relu(y*s + b + (res_scale ? res*rs + rb : res)), NHWC, C % 4 == 0 */
int capmi_bn_add_relu(const float* y, const float* s, const float* b, const float* res,
                      const float* res_scale, const float* res_shift, float* out, long long rows,
                      int C, void* stream);
/* conv1 tail: out = maxpool3x3/2/p1(relu(y*s + b)), NHWC (models/encoder.py:90 children 1-3) */
int capmi_bn_relu_maxpool(const float* y, const float* s, const float* b, float* out, int N, int H,
                          int W, int C, int Ho, int Wo, void* stream);
/* AdaptiveAvgPool2d to (OH,OW) on NHWC, output NHWC (models/encoder.py:92,108-109) */
int capmi_adaptive_avgpool_nhwc(const float* in, int N, int H, int W, int C, int OH, int OW,
                                float* out, void* stream);

/* ------------------------------------------------------------------------
 * Encoder fine-tune backward (EncoderAttention.fine_tune, models/encoder.py:112-121: layer2-4
 * trainable; BASELINE config 4). Conv dgrad = capmi_gemm_sk over CAPMI_A_CONV_NHWC of dY with the
 * weights from capmi_conv_weight_pack_dgrad (stride 2: four parity-class GEMMs with the weights from
 * capmi_conv_weight_pack_dgrad_s2; capmi_zero_upsample2_nhwc is the older 4x-FLOP form); conv wgrad =
 * capmi_gemm_sk(CAPMI_A_MMAJOR, CAPMI_B_CONV_NHWC).
 * ---------------------------------------------------------------------------------------- */
/* out[ci][kh][kw][co] = w[co][ci][KH-1-kh][KW-1-kw] (B operand of the data-gradient conv) */
int capmi_conv_weight_pack_dgrad(const float* w, int Cout, int Cin, int KH, int KW, float* out, void* stream);
/* 3x3 / stride 2 / pad 1 conv, parity class (ph, pw) of the input grid: out[ci][th][tw][co] =
 * w[co][ci][kh][kw], kh = 1 (ph = 0) or 2 - 2*th (ph = 1, th in {0,1}), same for kw. The class's
 * data gradient is a (ph+1)x(pw+1) stride-1 pad-0 conv over dY written to rows (2i+ph, 2j+pw)
 * (sub-pixel form: 9 taps in total over the 4 classes instead of 36 on the zero-upsampled grid). */
int capmi_conv_weight_pack_dgrad_s2(const float* w, int Cout, int Cin, int ph, int pw, float* out, void* stream);
/* The two packs above in the x3p conv k order, split exactly into three bf16 planes (ABI 15): the B
 * operand of the CAPMI_GEMM_X3D data gradient. out[3][Cin][T*Cout] bf16, k = ((co/32)*T + tap)*32 +
 * co%32 with tap = th*TW + tw over the T = TH*TW taps; ph < 0: the flipped KHxKW kernel of
 * capmi_conv_weight_pack_dgrad, else parity class (ph, pw) of capmi_conv_weight_pack_dgrad_s2
 * (KH = KW = 3). Cout % 32 == 0. */
int capmi_conv_weight_pack_dgrad_x3(const float* w, int Cout, int Cin, int KH, int KW, int ph, int pw, void* out,
                                    void* stream);
/* Many conv weights' three-plane bf16 operands in one launch (ABI 24, the fine-tune step's weight
 * preparation). jobs: DEVICE array of njobs descriptors (read by the kernel, so it may be built once and
 * re-launched every step, e.g. from a captured graph), max_elems = the largest job's R * Kc (< 2^31; sizes
 * the grid); w = the nn.Conv2d weight [Cout][Cin][KH][KW] fp32, out =
 * three planes [3][R][Kc] bf16, the exact RNE split of capmi_split3_bf16, bit-identical to:
 *   CAPMI_WX3_FWD      R = Cout, Kc = KH*KW*Cin: split3 of capmi_conv_weight_pack_pad (Cin >= 4, unpadded)
 *   CAPMI_WX3_FWD_X3P  the same in the x3p conv k order (ci/32, kh, kw, ci%32); Cin % 32 == 0
 *   CAPMI_WX3_DGRAD    capmi_conv_weight_pack_dgrad_x3 with (ph, pw) (ph < 0: the flipped KHxKW kernel)
 *   CAPMI_WX3_DGRAD_T  KH = KW = 1: split3 of capmi_conv_weight_pack_dgrad (out[ci][co] = w[co][ci]) */
#define CAPMI_WX3_FWD 0
#define CAPMI_WX3_FWD_X3P 1
#define CAPMI_WX3_DGRAD 2
#define CAPMI_WX3_DGRAD_T 3
typedef struct {
  const float* w;
  void* out;
  int mode;
  int cout, cin, kh, kw;
  int ph, pw;
  int pad_;
} capmi_wx3_job;
int capmi_weight_x3_batch(const capmi_wx3_job* jobs, int njobs, long long max_elems, void* stream);
/* [Cout][KH][KW][Cin] (GEMM layout of a weight gradient) -> [Cout][Cin][KH][KW] (nn.Conv2d layout) */
int capmi_conv_weight_unpack(const float* packed, int Cout, int Cin, int KH, int KW, float* out, void* stream);
/* out (N,H,W,C) = dy (N,Ho,Wo,C) at even (h, w), zero elsewhere (stride-2 conv data gradient) */
int capmi_zero_upsample2_nhwc(const float* dy, int N, int Ho, int Wo, int C, int H, int W, float* out,
                              void* stream);
/* BatchNorm2d(train) backward, rows x C NHWC. dz = d * relu mask:
 *   CAPMI_BNB_RELU_Y   mask = [y*scale + shift > 0] (BN + ReLU inside a bottleneck),
 *   CAPMI_BNB_RELU_OUT mask = [mask_src > 0]        (mask_src = saved relu(bn3 + residual) output).
 * reduce: dbeta = sum dz, dgamma = sum dz*(y-mean)*invstd (written, or added when accumulate) and
 * coef[4][C] for apply; work >= CAPMI_BNB_WORK_FLOATS(C) floats. invstd = rsqrt(save_var + eps),
 * save_mean / save_var = the forward's batch statistics (capmi_bn_finalize outputs, biased var).
 * apply: dy = gamma*invstd*(dz - dbeta/N - x^*dgamma/N); dz_out = dz when non-NULL. */
#define CAPMI_BNB_RELU_Y 0
#define CAPMI_BNB_RELU_OUT 1
#define CAPMI_BNB_MAX_SLABS 256
#define CAPMI_BNB_WORK_FLOATS(C) (2LL * CAPMI_BNB_MAX_SLABS * (C))
int capmi_bn_bwd_reduce(int mode, const float* d, const float* y, const float* mask_src, const float* scale,
                        const float* shift, const float* gamma, const float* save_mean, const float* save_var,
                        float eps, long long rows, int C, float* dgamma, float* dbeta, int accumulate,
                        float* coef, float* work, void* stream);
int capmi_bn_bwd_apply(int mode, const float* d, const float* y, const float* mask_src, const float* scale,
                       const float* shift, const float* coef, long long rows, int C, float* dy, float* dz_out,
                       void* stream);
/* AdaptiveAvgPool2d backward, NHWC: din (N,H,W,C) from dout (N,OH,OW,C) */
int capmi_adaptive_avgpool_bwd_nhwc(const float* dout, int N, int H, int W, int C, int OH, int OW, float* din,
                                    void* stream);

/* ------------------------------------------------------------------------
 * Attention decoder (models/attention.py:43-61, 151-164, 218-284).
 * Per-step state is time-major: X[t][b][M+E], H[t][b][D], ...
 * ---------------------------------------------------------------------- */
/* out[t][b][0:M] (row stride ld_out) = emb[caps[b*L + t]] for t < T; emb fp32 or fp64 (emb_is_f64) */
int capmi_embed_gather(const void* emb, int emb_is_f64, int M, const long long* caps, int B, int L,
                       int T, float* out, long long ld_out, void* stream);
/* dense word embeddings (the BERT variant's per-caption features, :166-215,242-244; no gather):
 * out[t][b][0:M] (row stride ld_out) = emb[b][t][0:M] for t < T, emb (B, Le, M) fp32, M % 4 == 0 */
int capmi_embed_dense(const float* emb, int B, int Le, int M, int T, float* out, long long ld_out, void* stream);
/* out[b][e] = mean_p enc[b][p][e]  (encoder_out.mean(dim=1), :161) */
int capmi_mean_rows(const float* enc, int B, int P, int E, float* out, void* stream);
/* Soft-attention score (:54-58 without the softmax): ad = sum_s dec_part[s][b][:] + bias_da;
 * e[b][p] = relu(att_enc[b][p][:] + ad) . wf + bf. Writes ad to att_dec_out[b][:] if non-NULL. */
int capmi_att_score_fwd(const float* att_enc, const float* dec_part, int S, long long dec_slab,
                        const float* bias_da, const float* wf, const float* bf, int B, int P, int A,
                        float* e, float* att_dec_out, void* stream);
/* softmax over P (:58) + context (:59-60) + optional f_beta gate (:270-271).
 * alpha -> alpha_out[b*alpha_ld_b + p] (zeros for rows b >= bt); awe (ungated) -> awe_out[b][E];
 * gate = sigmoid(sum_s gate_part[s][b][:] + bias_fb) -> gate_out[b][E];
 * gated awe -> x_out[b*ld_x + e] (if x_out). gate_part == NULL: no gate. */
int capmi_att_softmax_ctx_fwd(const float* e, const float* enc, int B, int P, int E, int bt,
                              float* alpha_out, long long alpha_ld_b, float* awe_out,
                              const float* gate_part, int S, long long gate_slab,
                              const float* bias_fb, float* gate_out, float* x_out, long long ld_x,
                              void* stream);
/* LSTMCell (:108-109,277-278), gate order i,f,g,o. pre = sum_s part[s] + xemb + sum_s hh_part[s].
 * writes h_out, c_out [B][D], act_out [B][4D] = (sig i, sig f, tanh g, sig o) */
int capmi_lstm_cell_fwd(const float* part, int S, long long slab, const float* xemb,
                        const float* hh_part, int S2, long long slab2, const float* c_prev, int B,
                        int D, float* h_out, float* c_out, float* act_out, void* stream);
/* Dropout before fc (:107,279): out = in * keep/(1-p), keep = hash(seed', index) >= p with
 * seed' = seed ^ hash(*seed_dev) when seed_dev != NULL (a device counter: graph replays draw
 * fresh masks), else seed. The backward pass re-applies the same mask to the gradient. */
int capmi_dropout(const float* in, long long n, float p, unsigned long long seed,
                  const unsigned long long* seed_dev, float* out, void* stream);
/* *counter += v (one thread): advances the device step / seed counters inside a graph */
int capmi_counter_add(long long* counter, long long v, void* stream);
/* zero rows r of a (rows x cols) matrix, row r = t*B + b, where b >= bt[t] (ragged decode, :261) */
int capmi_mask_rows_tb(float* x, const int* bt, int T, int B, int cols, long long ld, long long r1,
                       long long s2, void* stream);

/* Loss (:401-414). rows r = b*T + t of logits (B,T,V); target = caps[b*L + t + 1].
 * loss_rows[r] = lse - x[target]; dlogits (if non-NULL) = (softmax - onehot) * (*gscale) / nrows,
 * written at row t*B + b (time-major) when dl_time_major else b*T + t. Rows with t >= T_b skipped. */
int capmi_ce_fwd_bwd(const float* logits, const long long* caps, int B, int T, int L, int V,
                     const int* bt, int nrows, float* loss_rows, float* lse, float* dlogits,
                     int dl_time_major, const float* gscale, void* stream);
/* alpha regulariser ((alpha_c - sum_t alpha)^2).mean() over (B,P), alphas (B,T,P):
 * reg_part[g] = sum over workgroup g's (b,p) of (alpha_c - sum_t alpha)^2 / (B*P), g < capmi_alpha_reg_parts(B,P);
 * dreg[b][p] = -2 (alpha_c - sum_t alpha) / (B*P). */
int capmi_alpha_reg_parts(int B, int P);
int capmi_alpha_reg(const float* alphas, int B, int T, int P, float alpha_c, float* reg_part,
                    float* dreg, void* stream);
/* loss = sum(loss_rows[0:n]) / nrows + sum(reg_part[0:nreg]) -> out[0] (one workgroup, deterministic) */
int capmi_loss_finalize(const float* loss_rows, int n, int nrows, const float* reg_part, int nreg,
                        float* out, void* stream);

/* ---- backward through time ---- */
/* dh = dhd[b][:] (already dropout-masked, may be NULL) + sum_s dh_part[s][b][:]; dc = dc_in (NULL=0)
 * -> dgates [B][4D] (pre-activation) and dc_out [B][D]; rows b >= bt produce zeros. */
int capmi_lstm_cell_bwd(const float* dhd, const float* dh_part, int S, long long slab,
                        const float* dc_in, const float* act, const float* c_prev,
                        const float* c_cur, int B, int D, int bt, float* dgates, float* dc_out,
                        void* stream);
/* Pixel-duplicated features (models/encoder.py:92,108, AdaptiveAvgPool2d of an F x F map to
 * (F d) x (F d) with integer d: every pooled pixel is one input pixel repeated d x d times). The
 * decoder runs on the F*F distinct rows; these map its results back to the reference's positions.
 * alpha expansion: ap[r][pi][pj] = aq[r][pi/d][pj/d] / d^2 for rows r (= b*T + t), aq (rows, F*F). */
int capmi_att_alpha_expand(const float* aq, long long rows, int F, int d, float* ap, void* stream);
/* representatives: out[b][qi][qj] = in[b][qi*d][qj*d], in (B, (F d)^2), out (B, F*F) -- the
 * regulariser's d(loss)/d(alpha), equal over a duplicated group, as seen by the distinct rows */
int capmi_att_dup_pick(const float* in, int B, int F, int d, float* out, void* stream);
/* d(awe_g) = sum_s part[s]; dawe = d*gate; dgp = d*awe*gate*(1-gate) (if gate != NULL)
 * dalpha[b][p] = dawe . enc[b][p][:]; dawe -> dawe_out[b][E] when non-NULL (encoder fine-tune) */
int capmi_att_ctx_bwd(const float* part, int S, long long slab, const float* gate,
                      const float* awe, const float* enc, int B, int P, int E, float* dgp,
                      float* dalpha, float* dawe_out, void* stream);
/* gradient w.r.t. encoder_out (B,P,E) when the encoder is fine-tuned (models/encoder.py:112-121):
 * the context sums (:59-60) and the init-state mean (:161) contribute
 *   denc[b][p][e] = sum_t alpha[b*alpha_ld_b + t*P + p] * dawe[t][b][e] + dmean[b][e] / P
 * (dmean may be NULL); the enc_att term (:54) is a GEMM added on top (beta = 1). */
int capmi_att_enc_dinput(const float* alpha, long long alpha_ld_b, const float* dawe, const float* dmean,
                         int B, int T, int P, int E, float* denc, void* stream);
/* softmax backward with an extra dalpha term (dreg[b*dreg_ld_b + p], may be NULL: the alphas
 * output's own gradient) and the ReLU score backward:
 *   da = dalpha + dreg; de = alpha*(da - sum_p alpha*da); dad[b][a] = wf[a] sum_p de[p] [att_enc+ad > 0]
 * alpha read at alpha[b*alpha_ld_b + p]. rows b >= bt produce zeros. */
int capmi_att_score_bwd(const float* dalpha, const float* dreg, long long dreg_ld_b,
                        const float* alpha, long long alpha_ld_b, const float* att_enc,
                        const float* att_dec, const float* wf, int B, int P, int A, int bt,
                        float* de, float* dad, void* stream);
/* hoisted: datt_enc[b][p][a] = wf[a] sum_t de[t][b][p] [att_enc+ad_t > 0];
 * wf_part[blk][a] += sum de*relu(.) ; bf_part[blk] = sum de  (blk = one per (b, p-chunk)) */
int capmi_att_enc_grad(const float* de, const float* att_enc, const float* att_dec,
                       const float* wf, int T, int B, int P, int A, float* datt_enc,
                       float* wf_part, float* bf_part, int* nblk_out, void* stream);

/* ------------------------------------------------------------------------
 * Fused recurrence kernels (decoder_step.hip): three launches per timestep forward and three
 * backward instead of five each. Replace, per step t of models/attention.py:260-281:
 *   capmi_dstep_gemm, STORE2   : att_dec = dec_att(h) (:55) and gate = sigmoid(f_beta(h)) (:270)
 *   capmi_att_fwd_fused        : SoftAttention score, softmax, context (:56-60), gate * awe (:271)
 *   capmi_dstep_gemm, LSTM_FWD : LSTMCell([emb, gate*awe], (h, c)) (:277-278), the embedding
 *                                half of W_ih precomputed for all t (xemb, incl. both biases)
 * and the autograd backward of the same ops (LSTM_BWD: dh GEMM of step t+1 + the cell backward of
 * step t; GATE_BWD: d(gate*awe) GEMM + the gate/context split; capmi_att_bwd_fused: context,
 * softmax and score backward).
 *
 * capmi_dstep_gemm: C[M, N] = sum over segments i of A_i[M, K_i] * W_i[N, K_i]^T (both row-major,
 * k contiguous; every K_i % 32 == 0), fp32 MFMA (v_mfma_f32_16x16x4_f32), 64-row x nt-column tiles
 * (nt in {16, 32, 64}, N % nt == 0), k split S ways over workgroups. The S partials of a tile are
 * parked (write-through) and the LAST workgroup to arrive (one agent-scope counter per tile, reset
 * by that workgroup) adds them in split order -- deterministic -- and runs the epilogue.
 * gate_D > 0 (LSTM_FWD, nt = 64): tile tn's column c is W row (c/16)*gate_D + 16 tn + c%16, so a
 * tile holds the four gates i, f, g, o of 16 hidden units.
 * part: >= tiles*S*64*nt floats; counters: >= tiles ints, zero between launches.
 * ---------------------------------------------------------------------- */
typedef struct {
  const float* A;
  long long lda;
  const float* W;
  long long ldw;
  int K;
} capmi_dstep_seg;

#define CAPMI_DSTEP_STORE2 0   /* col < nsplit: out0 = v + bias0; else out1 = act1(v + bias1), act1 1 = sigmoid */
#define CAPMI_DSTEP_LSTM_FWD 1 /* gates = v + xemb -> h_out, c_out, act_out (i, f, g, o) */
#define CAPMI_DSTEP_LSTM_BWD 2 /* dh = v + dhd -> dgates, dc_out (rows >= bt: zeros) */
#define CAPMI_DSTEP_GATE_BWD 3 /* d = v: dawe_out = d * gate, dgp = d * awe * gate * (1 - gate) */

typedef struct {
  int mode;
  float* out0;
  long long ld0;
  const float* bias0;
  int nsplit;
  float* out1;
  long long ld1;
  const float* bias1;
  int act1;
  int D;                /* LSTM hidden size */
  const float* xemb;    /* LSTM_FWD: [M][4D] */
  const float* c_prev;  /* LSTM_FWD / LSTM_BWD: c_{t} [M][D] */
  float* h_out;
  float* c_out;
  float* act_out;       /* LSTM_FWD: [M][4D]; LSTM_BWD reads it (act) */
  const float* dhd;     /* LSTM_BWD: [M][D] or NULL */
  const float* dc_in;   /* LSTM_BWD: [M][D] or NULL */
  const float* act;     /* LSTM_BWD: [M][4D] */
  const float* c_cur;   /* LSTM_BWD: c_{t+1} */
  float* dgates;        /* LSTM_BWD: [M][4D] */
  float* dc_out;        /* LSTM_BWD: [M][D] */
  int bt;               /* LSTM_BWD: active rows */
  const float* gate;    /* GATE_BWD: [M][N] */
  const float* awe;     /* GATE_BWD: [M][N] */
  float* dawe_out;      /* GATE_BWD: [M][N] */
  float* dgp;           /* GATE_BWD: [M][N] */
} capmi_dstep_epi;

int capmi_dstep_gemm(const capmi_dstep_seg* segs, int nseg, int M, int N, int nt, int S, int gate_D,
                     const capmi_dstep_epi* epi, float* part, long long part_floats, int* counters,
                     int ncounters, void* stream);
/* capmi_att_score_fwd + capmi_att_softmax_ctx_fwd in one launch, on the distinct rows (P <= 56):
 * grid (E/512, B), each workgroup recomputes the P scores of its row b and writes its 512 columns
 * of awe and x = gate*awe; alphas of rows b >= bt are written as 0. att_dec: ad final [B][A]
 * (S_a = 0) or bias_da + the S_a split-K partials ad[s*slab_a + b*A + a] (then also written to
 * ad_out); gate: final sigmoid (S_g = 0) or sigmoid(bias_fb + partials), then written to gate_out.
 * Same arithmetic and summation order as the two kernels it replaces. */
int capmi_att_fwd_fused(const float* att_enc, const float* ad, int S_a, long long slab_a, const float* bias_da,
                        float* ad_out, const float* wf, const float* bf, const float* enc, const float* gate,
                        int S_g, long long slab_g, const float* bias_fb, float* gate_out, int B, int P, int A,
                        int E, int bt, float* alpha_out, long long alpha_ld_b, float* awe_out, float* x_out,
                        long long ld_x, void* stream);
/* capmi_att_ctx_bwd + capmi_att_score_bwd in one launch, one workgroup per row b: d(gate*awe) final
 * (S = 0: dx is dawe) or the S split-K partials (then dawe = d*gate -> dawe_out, dgp as
 * capmi_att_ctx_bwd), dalpha, softmax and ReLU-score backward. Bit-identical to the two kernels. */
int capmi_att_bwd_fused(const float* dx, int S, long long slab, const float* gate, const float* awe, float* dgp,
                        float* dawe_out, const float* enc, const float* alpha, long long alpha_ld_b,
                        const float* dreg, long long dreg_ld_b, const float* att_enc, const float* att_dec,
                        const float* wf, int B, int P, int A, int E, int bt, float* de, float* dad, void* stream);

/* ------------------------------------------------------------------------
 * Optimiser (train_utils.py:2-12 clamp + torch.optim.Adam, models/attention.py:352-355,423-430)
 * p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps) with g clamped to +-clip first.
 * step_dev == NULL: bc1 = 1 - beta1^t and bc2_sqrt = sqrt(1 - beta2^t) as passed (host step t);
 * else t = *step_dev and both are computed on the device in fp64 (graph-replayable).
 * ---------------------------------------------------------------------- */
int capmi_adam_clamp(float* p, const float* g, float* m, float* v, long long n, double lr,
                     double beta1, double beta2, double eps, double bc1, double bc2_sqrt, double clip,
                     const long long* step_dev, void* stream);
int capmi_adam_clamp_f64(double* p, const double* g, double* m, double* v, long long n, double lr,
                         double beta1, double beta2, double eps, double bc1, double bc2_sqrt,
                         double clip, const long long* step_dev, void* stream);
/* embedding gradient: demb[caps[b*L+t]][:] += dx[t][b][0:M] (atomic; fp32 or fp64 table) */
int capmi_embed_scatter_add(const float* dx, long long ld_dx, const long long* caps, int B, int L,
                            int T, const int* bt, int M, void* demb, int demb_is_f64, void* stream);

/* in[n] fp32 -> out[3][n] bf16 (n % 4 == 0): the exact split in = out[0] + out[1] + out[2], each
 * term the RNE bf16 rounding of the remainder (B operand of CAPMI_GEMM_X3). */
int capmi_split3_bf16(const float* in, long long n, void* out, void* stream);

/* x = relu(y * scale[c] + shift[c]) of y [rows][C] fp32 (scale = shift = NULL: x = y), written as
 * the three bf16 split planes out[3][rows * C] (the CAPMI_GEMM_X3P A operand); C % 4 == 0. */
int capmi_bn_relu_split3(const float* y, const float* scale, const float* shift, long long rows, int C, void* out,
                         void* stream);

/* ---- kernel timing inside HIP graphs (bench.py's roofline) -------------------------------
 * Timing events whose record becomes a graph node when `stream` is being captured
 * (hipEventRecordExternal), a plain record otherwise; after a replay has completed,
 * capmi_timing_elapsed_ms gives the time between two records (milliseconds). */
int capmi_timing_event_create(void** event);
int capmi_timing_event_destroy(void* event);
int capmi_timing_event_record(void* event, void* stream);
int capmi_timing_elapsed_ms(void* start, void* end, float* ms);
/* ABI 16: the next GEMM launch of the calling host thread (any capmi_gemm* entry point, eager, not
 * under capture) records its dispatch's own start / end timestamps into the two timing events
 * (hipExtLaunchKernel: the kernel duration rocprofv3 reports); capmi_timing_disarm drops a pair no
 * launch consumed and returns 1 if there was one. */
int capmi_timing_arm(void* start, void* stop);
int capmi_timing_disarm(void);

const char* capmi_strerror(int code);
int capmi_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* CAPMI_H */
