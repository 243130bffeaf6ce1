/*
 * libvcg_hip — MI355X (gfx950) native kernels for the video-segment-point clip scorer of
 * SeoYeonnLee/Video-Chapter-Generation (TwoStream = TSM-ResNet-50 + BERT-base + ChapterHead).
 *
 * C ABI conventions
 *   - device pointers + explicit int sizes; no torch types; `dtype` is VCG_F32 (0) or VCG_BF16 (1)
 *     and selects the storage type of activation tensors (parameters/grads are always fp32);
 *   - activations are NHWC (vision) / row-major [tokens][hidden] (text);
 *   - every call is asynchronous on `stream` and returns 0 or a negative vcg_status; the
 *     message of the last failure on the calling thread is vcg_last_error();
 *   - workspaces are caller-allocated; size them with the matching *_ws_bytes query;
 *   - gradients are ACCUMULATED (+=) into fp32 buffers so micro-batch accumulation is free.
 *
 * Each entry point cites the reference code it replaces (paths relative to
 * video_chapter_generation/ in the reference repository).
 */
#ifndef VCG_HIP_H
#define VCG_HIP_H
#include <hip/hip_runtime.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define VCG_API
enum { VCG_F32 = 0, VCG_BF16 = 1 };
/* vcg_ln_bwd / vcg_embed_ln_bwd dtype flag (VCG_BF16 | VCG_GRAD_F32): the incoming gradient dout and the residual
   gradient dres are fp32 while x / res / dx stay bf16 -- BERT's residual-gradient stream kept in fp32 between its
   LayerNorm backwards, as torch autocast keeps it (the LayerNorm outputs it flows back into are fp32 there) */
enum { VCG_GRAD_F32 = 0x10 };
enum { VCG_OK = 0, VCG_ERR_INVALID = -1, VCG_ERR_UNSUPPORTED = -2, VCG_ERR_HIP = -3 };
enum { VCG_ACT_NONE = 0, VCG_ACT_RELU = 1, VCG_ACT_GELU = 2, VCG_ACT_TANH = 3, VCG_ACT_GELU_BWD = 4 };
/* vcg_gemm act flag: with a residual, round alpha * AB + bias to the storage dtype BEFORE adding the residual (the
   unfolded conv3 -> bn3 path stores y3 in bf16; the scoring forward's folded conv3 sets it to match). Without it the
   residual is added to the f32 accumulator value. */
enum { VCG_ACT_FLAG_ROUND_PRE = 0x100 };
/* vcg_gemm act flag: run this GEMM on the wide-tile engine (csrc/igemm_wide.hip: 128 x 128/192/256 tiles, one
   512-thread workgroup per CU, persistent) -- BERT's Linear layers (transformers BertModel, model/lang/bert_hugface.py:20)
   and the trunk's stride-2 downsample input gradient set it. Taken, whatever M, for bf16 GEMMs with K-contiguous
   operands (transA = transB = 0), alpha = 1 and 16-B aligned rows whose epilogue is a bias (act NONE), bias + GELU
   (aux: the bf16 pre-activation; the GELU of the unrounded value, as the 128 x 128 engine), GELU' of a residual, or a
   residual addend (residual != C); any other flagged GEMM runs on the 128 x 128 engine (vcg_gemm_census shows which
   ran). */
enum { VCG_ACT_FLAG_WIDE = 0x200 };
/* vcg_gemm act flag with VCG_ACT_FLAG_WIDE and a residual: the residual and the output C are fp32 (the operands bf16):
   BERT's input gradients added to its fp32 residual-gradient stream (C = A B^T + residual, one rounding to fp32) */
enum { VCG_ACT_FLAG_F32_OUT = 0x400 };
/* GEMM census (tests, bench.py): while enabled, every GEMM dispatch of vcg_gemm / vcg_gemm_splitk / the conv entry
   points adds one to the count of its key "<engine> M=.. N=.. K=.. <epilogue>"; enabling (or disabling) clears it.
   vcg_gemm_census_size returns the number of keys; vcg_gemm_census_get(i) writes key i (NUL-terminated, at most n
   bytes) and its count. */
VCG_API int vcg_gemm_census_enable(int on);
VCG_API int vcg_gemm_census_size(void);
VCG_API int vcg_gemm_census_get(int i, char* key, int n, long long* count);

/* ---- library ---------------------------------------------------------------------------- */
VCG_API const char* vcg_last_error(void);
VCG_API int vcg_version(void);
VCG_API int vcg_init(int device);      /* per-device handle; fails unless the device is gfx950 */
VCG_API int vcg_finalize(void);
VCG_API int vcg_sync(hipStream_t stream);
/* Live launch timing (bench.py's dominant-kernel roofline): while enabled, every fast-GEMM / wgrad launch is
   bracketed with HIP events on its stream; query sums durations (ms), launches and algorithmic FLOPs per kernel
   id (0 igemm_fast_kernel, 1 wgrad_fast_kernel, 2 igemm_kernel, 3 conv3x3_patch_kernel, 4 gemm_wide_kernel).
   Enabling (or disabling) clears the records. */
VCG_API int vcg_timing_enable(int on);
VCG_API int vcg_timing_query(int kernel_id, double* ms_total, long long* launches, double* flops);
/* per-launch roofline of the recorded launches: ideal_ms = sum over launches of max(flops / peak_tflops,
   algorithmic bytes / peak_gbs) (bytes: operands read once, outputs written once), with their total time */
VCG_API int vcg_timing_roofline(int kernel_id, double peak_tflops, double peak_gbs, double* ms_total, double* ideal_ms, double* bytes, double* flops);
/* Profiling aid (no reference counterpart): phase stamps (s_memtime) of workgroup 0 / wave 0 of the last
   conv3x3_patch_kernel launch made with VCG_PATCH_STAMPS=1 in the environment, 6 per tile for the first 64 tiles:
   tile top, after the DMA wait + barrier, after the next DMA issue, after the MFMAs, after the barrier, after the
   epilogue. Returns 1 when no stamped launch happened. */
VCG_API int vcg_patch_stamps(unsigned long long* out, int n);
/* Profiling aid: per-tile phase stamps of workgroup 0 / wave 0 of the last igemm_fast launch, 4 per tile (first
   k-step, after the last MFMAs, after the output staging, after the epilogue) -- only in a library built with
   -DVCG_FAST_STAMPS (make EXTRA=-DVCG_FAST_STAMPS); returns 1 otherwise. */
VCG_API int vcg_fast_stamps(unsigned long long* out, int n);
/* profiling aid: s_memtime phase stamps of the last 256-tile GEMM (a -DVCG_G256_STAMPS build; 1 otherwise) */
VCG_API int vcg_g256_stamps(unsigned long long* out, int n);
/* profiling aid: s_memtime phase stamps of the last wide-tile GEMM (a -DVCG_WIDE_STAMPS build; 1 otherwise): waves 0
   and 4 of workgroup 0, k-steps 8..23, both phases, 4 points each */
VCG_API int vcg_wide_stamps(unsigned long long* out, int n);

/* ---- MFMA implicit-GEMM engine (igemm.hip) ---------------------------------------------- */
/* torchvision conv2d inside Resnet50TSM.base_model (model/vision/resnet50_tsm.py:15,68-77), with
 * TemporalShift.shift (ops/temporal_shift.py:33-51, inserted by make_temporal_shift :133-144)
 * fused into the input gather; optional BatchNorm partial statistics from the epilogue.
 * stats (optional): float2 [Cout + 1][vcg_conv_stats_tiles(M)] — per column and slot (mean, M2) of
 * the slot's rows, then the count row (rows per slot, 0 = unused slot); merged by vcg_bn_finalize.
 * bf16 with C = 4 (RGB0, the stem): the pair-packed stem -- stride 2, even W; w in the layout of
 * vcg_weight_prep(transposed = 2 + pad); two stride-2 taps per 16-B chunk (GEMM K 224 instead of 392). */
VCG_API int vcg_conv_stats_tiles(int M);
VCG_API int vcg_conv_fwd(int dtype, const void* x, const void* w, void* y, float* stats, int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad, int tsm_T, int tsm_fold, hipStream_t stream);
/* y = act(conv(x, w) + bias[col]) (act 0 none / 1 ReLU), no statistics: a conv with its running-statistics BN folded
   into w (vcg_weight_fold) and the BN shift as bias -- the scoring (eval) forward, test_video_segment_point.py:116-122 */
VCG_API int vcg_conv_fwd_bias_act(int dtype, const void* x, const void* w, const float* bias, int act, void* y, int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad, int tsm_T, int tsm_fold, hipStream_t stream);
/* autograd of conv2d: input gradient (transposed-conv gather) */
VCG_API int vcg_conv_dgrad(int dtype, const void* dy, const void* wt, void* dx, int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad, hipStream_t stream);
/* vcg_conv_dgrad fused with the trunk backward's next steps (igemm.h BwdEpi): TSM adjoint (tsm_fold > 0:
   ops/temporal_shift.py:33-51 autograd), + res, ReLU mask (bits or fma(y, mscale, mshift) > 0), stored as g, and
   the BatchNorm backward reductions against y (and y2) -> sum_g / sum_gx (/ sum_gx2), dgamma / dbeta
   (/ dgamma2 / dbeta2) accumulated. res_stride 2: `res` is the compact [N][ceil(H/2)][ceil(W/2)][C] input
   gradient of a 1x1 stride-2 conv (the downsample branch), added at the even (h, w) rows only. A 3x3 / stride-2
   dgrad runs as four sub-pixel classes (dx pixels of one (h, w) parity) over only the taps reaching each.
   bf16 fast engine only; VCG_ERR_UNSUPPORTED elsewhere. */
VCG_API long long vcg_conv_dgrad_bwd_ws_bytes(int C, int Cout, int KH, int KW);
/* a2 (optional, with bits and no y): the previous block's conv3 input [N*H*W][a2_c] bf16 (a2_c 64; K <= 128); the kernel then
   also accumulates pg [C][a2_c] f32 = g^T a2 (the conv3 weight-gradient product that gives bn3's sum_gx) from the g
   tiles it stores, with the partial slabs in pws (vcg_conv_dgrad_bwd_p_ws_bytes). VCG_ERR_UNSUPPORTED when that
   product does not apply to the shape (the streaming 1x1 kernel only): the caller runs the plain call and the GEMM. */
VCG_API long long vcg_conv_dgrad_bwd_p_ws_bytes(int C, int a2_c);
VCG_API int vcg_conv_dgrad_bwd(int dtype, const void* dy, const void* wt, void* g, int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad, int tsm_T, int tsm_fold, const void* res, int res_stride, const unsigned char* bits, const void* y, const float* mean, const float* invstd, const float* mscale, const float* mshift, const void* y2, const float* mean2, const float* invstd2, float* ws, long long ws_bytes, float* sum_g, float* sum_gx, float* dgamma, float* dbeta, float* sum_gx2, float* dgamma2, float* dbeta2, const void* a2, int a2_c, float* pg, float* pws, long long pws_bytes, hipStream_t s);
/* autograd of conv2d: weight gradient, split-K over pixels, written in OIHW (state-dict layout); bf16 C = 4:
   the pair-packed stem gather (as vcg_conv_fwd) */
VCG_API long long vcg_conv_wgrad_ws_bytes(int dtype, int N, int H, int W, int C, int Cout, int KH, int KW, int stride, int pad);
VCG_API int vcg_conv_wgrad(int dtype, const void* x, const void* dy, float* dw, int accumulate, float* ws, long long ws_bytes, int N, int H, int W, int C, int Cin, int Cout, int KH, int KW, int stride, int pad, int tsm_T, int tsm_fold, hipStream_t stream);
/* A batch-statistics BatchNorm backward (torch BatchNorm2d autograd: dy = A g + B y + Cc per channel, as
   vcg_bn_bwd_apply) folded into the two gradients of the 1x1 conv that consumes dy (bottleneck conv3 after
   bn3, model/vision/resnet50_tsm.py:15 via torchvision Bottleneck), so dy is never stored (bf16 only):
   vcg_bn_bwd_fold_weights: wt [N][K] (the dgrad's B operand) -> wfold [N][2K] = [A_k wt | B_k wt] (bf16) and the
   per-column constant bias [N] (f32); vcg_conv_dgrad_bwd_bnfold: the input gradient of that conv as one GEMM over
   [g | yg] (K = Cout + Ky; yg = y, Ky = Cout) with vcg_conv_dgrad_bwd's light epilogue (ReLU mask fma(y, mscale, mshift) > 0, sums against
   y); vcg_conv_wgrad_bnfold: dw[Cout][C] (+)= its weight gradient, one GEMM with 2 Cout rows ([g | yg]^T x)
   combined per row with colsum_x = the column sums of x (f32 [C]). VCG_ERR_UNSUPPORTED where the engine does not
   apply. */
/* torchvision Bottleneck's bn3 + identity + ReLU (model/vision/resnet50_tsm.py:15) as a second pass of conv3's GEMM:
   out[M][N] = relu(bf16(x[M][K] wfold[N][K]^T + bias) + res') and the ReLU mask bits (vcg_bn_apply's layout),
   res' = res or fma(res, res_scale[n], res_shift[n]) (a layer's first block: the downsample BN's output), with
   wfold = the conv3 weight rows scaled by the batch-statistics BN scale (vcg_weight_fold), bias = its shift: the stored
   conv output is not read back (bf16 fast engine; VCG_ERR_UNSUPPORTED elsewhere) */
VCG_API int vcg_conv1x1_bn_res_relu(const void* x, const void* wfold, const float* bias, const void* res, const float* res_scale, const float* res_shift, void* out, unsigned char* bits, int M, int N, int K, hipStream_t stream);
VCG_API int vcg_bn_bwd_fold_weights(const void* wt, int N, int K, const float* mean, const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx, float inv_count, void* wfold, float* bias, hipStream_t stream);
/* the fold with the conv3 input a2 [M][C] as the second source instead of y3 = a2 w3^T (y3 never read):
   vcg_bn_bwd_fold_weights_a2: wfold [C][K + C] = [A_k wt | w3^T diag(B) w3] and the bias, colsum_a = column sums of
   a2 (f32 [C]); the dgrad then runs vcg_conv_dgrad_bwd_bnfold with yg = a2, Ky = C; vcg_bn_bwd_fold_wgrad_a2:
   dw[K][C] (+)= A P + B (w3 G) + Cc colsum_a from P = g^T a2 and G = a2^T a2 (f32, vcg_conv_wgrad products) and
   the f32 conv3 weight w3 [K][C]. Shapes: fold_weights_a2 needs K % 64 == 0 and a 16-B aligned wt, fold_wgrad_a2
   C % 16 == 0 (VCG_ERR_INVALID otherwise). */
/* bn3 with y3 never stored (the forward keeps only its statistics, vcg_conv1x1_stats, and applies it by
   vcg_conv1x1_bn_res_relu): sum_gx of its backward from P = g^T a2 (vcg_conv_wgrad) and the forward's bf16 conv weight
   w [K][C]: sum_gx[k] = invstd_k (sum_j w[k][j] P[k][j] - mean_k sum_g[k]), dgamma (optional) += sum_gx; sum_g
   comes from the producing dgrad's epilogue run with the mask bits and no y (vcg_conv_dgrad_bwd: y NULL, bits,
   sum_g / sum_gx given: sum_gx written as 0). */
/* vcg_bn_apply without a residual (bf16) that also writes the column sums of the stored output (f32 [C]): conv3's
   input a2 and its colsum for the bn3 fold's centring in one pass */
VCG_API long long vcg_bn_apply_colsum_ws_bytes(long long P, int C);
VCG_API int vcg_bn_apply_colsum(const void* y, const float* scale, const float* shift, int relu, void* out, float* colsum, float* ws, long long ws_bytes, long long P, int C, hipStream_t s);
/* vcg_bn_apply_colsum (ReLU, bf16, C = 64 / 128 / 256) that also returns gram = out^T out (f32 [C][C], summed in a
   fixed order: deterministic): the bottleneck's bn2 -> relu -> a2 with the a2 statistics that bn3's batch statistics
   (vcg_bn_stats_from_gram) and the a2 form of the bn3 backward fold need, so that neither reads a2 again.
   mean / invstd: the statistics that scale / shift fold. g64 (double [C * C + 2 C]): the same Gram matrix and column
   sums accumulated centred per channel, with the centres ([Gc | d | c]; c = bf16(beta) for channels whose BN shift
   beta exceeds 6 |gamma|, else 0): the input of vcg_bn_stats_from_gram, free of E[y^2] - E[y]^2 cancellation. */
VCG_API long long vcg_bn_apply_gram_ws_bytes(long long P, int C);
VCG_API int vcg_bn_apply_gram(const void* y, const float* scale, const float* shift, const float* mean, const float* invstd, void* out, float* colsum, float* gram, double* g64, float* ws, long long ws_bytes, long long P, int C, hipStream_t s);
/* Batch statistics of y = x w^T (w bf16 [N][C], the conv's forward GEMM weights; M rows) from x's g64 of
   vcg_bn_apply_gram: mean_n = w_n . mu, var_n = w_n^T Cov w_n with Cov = Gc / M - (d / M)(d / M)^T, mu = c + d / M, in
   double -- torchvision Bottleneck bn3 over conv3's output (model/vision/resnet50_tsm.py:15) without a statistics
   pass over a2. Writes the vcg_conv_fwd stats layout (one used slot) for vcg_bn_finalize. */
VCG_API int vcg_bn_stats_from_gram(const double* g64, const void* w, long long M, int N, int C, float* stats, int mtiles, hipStream_t s);
/* vcg_bn_stats_from_gram + vcg_bn_finalize for its one slot of M rows (running_mean / running_var updated with
   momentum when given, both or neither) + vcg_weight_fold of the f32 master weight w32 [N][C] by the new scale into
   wfold (bf16 [N][C]; both or neither) in one launch, with the same values as the three calls: bn3's state and the
   folded weight of the y3-drop block's GEMM pass (model/two_stream.py:VideoEncoder -> torchvision Bottleneck.bn3).
   C <= 256, C % 16 == 0 (VCG_ERR_INVALID otherwise). */
VCG_API int vcg_bn_finalize_from_gram(const double* g64, const void* w, long long M, int N, int C, const float* gamma,
                                      const float* beta, float* mean, float* invstd, float* scale, float* shift,
                                      float* running_mean, float* running_var, float momentum, float eps,
                                      const float* w32, void* wfold, hipStream_t s);
VCG_API int vcg_conv1x1_stats(const void* x, const void* w, float* stats, int M, int N, int K, hipStream_t stream);
VCG_API int vcg_bn_bwd_sumgx_from_wgrad(const float* P, const void* w, int K, int C, const float* mean, const float* invstd, const float* sum_g, float* sum_gx, float* dgamma, hipStream_t stream);
VCG_API int vcg_bn_bwd_fold_weights_a2(const void* wt, int C, int K, const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx, float inv_count, const float* colsum_a, void* wfold, float* bias, hipStream_t stream);
VCG_API int vcg_bn_bwd_fold_wgrad_a2(const float* P, const float* G, const float* w3, int K, int C, const float* mean, const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx, float inv_count, const float* colsum_a, float* dw, int accumulate, hipStream_t stream);
VCG_API int vcg_conv_dgrad_bwd_bnfold(const void* g, const void* yg, int Ky, const void* wfold, const float* bias, void* out, int N, int H, int W, int C, int Cout, const void* y, const float* mean, const float* invstd, const float* mscale, const float* mshift, float* ws, long long ws_bytes, float* sum_g, float* sum_gx, float* dgamma, float* dbeta, hipStream_t stream);
VCG_API long long vcg_conv_wgrad_bnfold_ws_bytes(int N, int H, int W, int C, int Cout);
VCG_API int vcg_conv_wgrad_bnfold(const void* x, const void* g, const void* yg, const float* mean, const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx, float inv_count, const float* colsum_x, float* dw, int accumulate, float* ws, long long ws_bytes, int N, int H, int W, int C, int Cout, hipStream_t stream);
/* nn.Linear / BertSelfAttention matmuls (HF BertModel via model/lang/bert_hugface.py:20; ChapterHead
 * projections model/fusion/two_stream.py:60-61,79-85) */
VCG_API int vcg_gemm(int dtype, int transA, int transB, int M, int N, int K, const void* A, long long lda, const void* B, long long ldb, void* C, long long ldc, const float* bias, int act, const void* residual, long long ldr, void* aux, float alpha, hipStream_t stream);
VCG_API int vcg_gemm_batched(int dtype, int transA, int transB, int M, int N, int K, const void* A, long long lda, long long a_so, long long a_si, const void* B, long long ldb, long long b_so, long long b_si, void* C, long long ldc, long long c_so, long long c_si, int batch_outer, int batch_inner, const float* bias, int act, float alpha, hipStream_t stream);
VCG_API long long vcg_gemm_splitk_ws_bytes(int dtype, int M, int N, int K);
VCG_API int vcg_gemm_splitk(int dtype, int transA, int transB, int M, int N, int K, const void* A, long long lda, const void* B, long long ldb, float* out, int accumulate, float* ws, long long ws_bytes, hipStream_t stream);

/* ---- vision support (vision.hip) --------------------------------------------------------- */
/* nn.BatchNorm2d (train: batch stats + running update; eval: running stats; the test driver's
 * batch-stat eval test_video_segment_point.py:116-122) */
VCG_API int vcg_bn_finalize(const float* stats, int mtiles, int M, int C, const float* gamma, const float* beta, float* mean_out, float* invstd_out, float* scale_out, float* shift_out, float* running_mean, float* running_var, float momentum, float eps, hipStream_t s);
VCG_API int vcg_bn_eval_params(const float* gamma, const float* beta, const float* rm, const float* rv, float eps, int C, float* mean_out, float* invstd_out, float* scale, float* shift, hipStream_t s);
/* bits (optional): ReLU mask of out, one byte per 16-byte vector (bit e = element e), for VCG_MASK_BITS. */
VCG_API int vcg_bn_apply(int dtype, const void* y, const float* scale, const float* shift, const void* res, const float* rscale, const float* rshift, int relu, void* out, unsigned char* bits, long long P, int C, hipStream_t s);
VCG_API long long vcg_bn_bwd_ws_bytes(long long P, int C);
/* ReLU mask of the upstream gradient (mask_mode): 0 none, 1 tensor (mask > 0), 2 bits from vcg_bn_apply,
   3 affine (fma(y, mscale[c], mshift[c]) > 0: the forward BN+ReLU decision recomputed from y). */
VCG_API int vcg_bn_bwd_reduce(int dtype, const void* dout, int mask_mode, const void* mask, const unsigned char* mbits, const float* mscale, const float* mshift, const void* y, const float* mean, const float* invstd, long long P, int C, float* ws, long long ws_bytes, float* sum_g, float* sum_gx, float* dgamma, float* dbeta, int accumulate, hipStream_t s);
VCG_API int vcg_bn_bwd_apply(int dtype, const void* dout, int mask_mode, const void* mask, const unsigned char* mbits, const float* mscale, const float* mshift, const void* y, const float* mean, const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx, long long count, int train_stats, void* dy, void* gout, long long P, int C, hipStream_t s);
/* two batch-stat BN backward applies sharing one masked gradient g (bn3 + the downsample BN of a layer's first
   bottleneck, resnet50_tsm.py:15 via torchvision Bottleneck): dy = bn3' (g, y), dyd = bn_d' (g, yd), g read once */
VCG_API int vcg_bn_bwd_apply_dual(int dtype, const void* g, const void* y, const float* mean, const float* invstd, const float* gamma, const float* sum_g, const float* sum_gx, const void* yd, const float* mean_d, const float* invstd_d, const float* gamma_d, const float* sum_g_d, const float* sum_gx_d, long long count, void* dy, void* dyd, long long P, int C, hipStream_t s);
/* torchvision stem maxpool 3x3/2 and avgpool + fc=Identity (resnet50_tsm.py:19) */
VCG_API int vcg_maxpool_fwd(int dtype, const void* x, void* y, unsigned char* idx, int N, int H, int W, int C, hipStream_t s);
VCG_API int vcg_maxpool_bwd(int dtype, const void* dy, const unsigned char* idx, void* dx, int N, int H, int W, int C, hipStream_t s);
/* maxpool backward fused with the stem BatchNorm backward reduction (BN + ReLU before the pool): g = mask(dx),
   mask = fma(y, mscale, mshift) > 0; sum_g / sum_gx finalized, dgamma / dbeta accumulated; g = NULL: the sums
   only (for vcg_maxpool_bwd_bn_apply) */
VCG_API long long vcg_maxpool_bwd_bn_ws_bytes(int C);
VCG_API int vcg_maxpool_bwd_bn(int dtype, const void* dy, const unsigned char* idx, void* g, int N, int H, int W, int C, const void* y, const float* mean, const float* invstd, const float* mscale, const float* mshift, float* ws, long long ws_bytes, float* sum_g, float* sum_gx, float* dgamma, float* dbeta, hipStream_t s);
/* the sums of vcg_maxpool_bwd_bn (g = NULL) from the pooled activation mp [N][OH][OW][C] (vcg_bn_relu_maxpool's
   output) instead of the pre-pool y: a window's gradient reaches its argmax pixel, whose ReLU output is mp, so the
   mask is mp > 0 and y - mean = (mp - mshift) / mscale - mean there (mscale != 0). The stem BN + ReLU + max-pool
   backward of Resnet50TSM.base_model (model/vision/resnet50_tsm.py:15, torchvision bn1 -> relu -> maxpool). */
VCG_API int vcg_maxpool_bwd_bn_sums_pooled(int dtype, const void* dy, const void* mp, const unsigned char* idx, const void* y, int N, int H, int W, int C, const float* mean, const float* invstd, const float* mscale, const float* mshift, float* ws, long long ws_bytes, float* sum_g, float* sum_gx, float* dgamma, float* dbeta, hipStream_t s);
/* the stem backward in two streaming passes (reference resnet50_tsm.py:19 torchvision stem: conv1 -> bn1 -> relu ->
   maxpool): dx = BN-backward-apply(g) with g = mask(maxpool_bwd(dy)) recomputed (rounded to dtype), sums from
   vcg_maxpool_bwd_bn(g = NULL) -- vcg_maxpool_bwd_bn + vcg_bn_bwd_apply without the g tensor */
VCG_API int vcg_maxpool_bwd_bn_apply(int dtype, const void* dy, const unsigned char* idx, void* dx, int N, int H, int W, int C, const void* y, const float* mean, const float* invstd, const float* mscale, const float* mshift, const float* gamma, const float* sum_g, const float* sum_gx, long long count, int train_stats, hipStream_t s);
/* the stem backward from the pooled-output gradient to the stem conv's weight gradient in ONE pass (bf16; reference
   resnet50_tsm.py:19 torchvision stem conv1 7x7/2 -> bn1 -> relu -> maxpool): vcg_maxpool_bwd_bn_apply's dy0 of each
   conv-output row pair computed into LDS and contracted at once with the pair-packed frames x [N][2H][2W][4] into
   dW [64][3][7][7] (fp32, added to when accumulate) -- dy0 never reaches HBM. y [N][H][W][64], dy / idx
   [N][H/2][W/2][64]; H even, W % 8 == 0, W <= 112. Equals vcg_maxpool_bwd_bn_apply + vcg_conv_wgrad up to the
   fp32 summation order (fixed: deterministic). Returns VCG_ERR_UNSUPPORTED unless vcg_stem_bwd_fused_fits(N, H, W)
   (every operand below 4 GB: 32-bit buffer offsets; the caller then runs the apply pass + weight gradient). */
VCG_API long long vcg_stem_bwd_fused_ws_bytes(void);
VCG_API int vcg_stem_bwd_fused_fits(int N, int H, int W);
VCG_API int vcg_stem_bwd_fused(const void* dy, const unsigned char* idx, const void* y, const void* x, int N, int H, int W, const float* mean, const float* invstd, const float* mscale, const float* mshift, const float* gamma, const float* sum_g, const float* sum_gx, long long count, int train_stats, float* ws, long long ws_bytes, float* dw, int accumulate, hipStream_t s);
/* the stem forward's BN + ReLU + maxpool 3x3/2 in one pass: out / idx = maxpool(relu(fma(y, scale, shift))) with the
   activation rounded to dtype (bit-identical to vcg_bn_apply then vcg_maxpool_fwd; no activation tensor) */
VCG_API int vcg_bn_relu_maxpool(int dtype, const void* y, const float* scale, const float* shift, void* out, unsigned char* idx, int N, int H, int W, int C, hipStream_t s);
VCG_API int vcg_avgpool_fwd(int dtype, const void* x, float* y, int N, int HW, int C, hipStream_t s);
VCG_API int vcg_avgpool_bwd(int dtype, const float* dy, void* dx, int N, int HW, int C, hipStream_t s);
/* rearrange 'b t c h w -> (b t) c h w' (two_stream.py:183) + NCHW->NHWC staging */
VCG_API int vcg_frames_to_nhwc(int dtype, const float* src, void* dst, int N, int C, int H, int W, int Cpad, hipStream_t s);
/* Frame ingest (§8f rank 2): u8 RGB frames [F][H][W][3] gathered by a window frame table idx[n_rows] (int64,
   0-based; youtube_dataset.py:180-190 offsets applied by the caller, see data/clip_windows.py:frame_index_table) and
   normalised like ToTensor+Normalize (train_video_segment_point.py:383-386) into NHWC [n_rows][H][W][8]. mean3/std3
   are HOST pointers to 3 floats. */
VCG_API int vcg_window_frames_u8(int dtype, const uint8_t* frames, const long long* idx, void* dst, long long n_rows, int F, int H, int W, const float* mean3, const float* std3, hipStream_t s);
/* the same into NHWC [n_rows][H][W][Cpad], Cpad 4 (the pair-packed bf16 stem / fp32) or 8 */
VCG_API int vcg_window_frames_u8_cpad(int dtype, const uint8_t* frames, const long long* idx, void* dst, long long n_rows, int F, int H, int W, int Cpad, const float* mean3, const float* std3, hipStream_t s);
/* OIHW f32 -> GEMM operand: transposed 0 [Cout][KH][KW][Cpad], 1 [Cin][KH][KW][Cout], 2 + pad the pair-packed
   stem [Cout][KH][KWp][8] (bf16, Cin <= 4; element 4j + c of super tap kwp = w[.][c][kh][2 (kwp - pwp) + j + pad],
   pwp = -floor(-pad / 2), KWp = floor((KW - 1 - pad) / 2) + pwp + 1) */
VCG_API int vcg_weight_prep(int dtype, const float* w, void* out, int Cout, int Cin, int KH, int KW, int Cpad, int transposed, hipStream_t s);
/* out[r][c] = w[r][c] * scale[r] (f32 master -> dtype): a running-statistics BN (scale = gamma * invstd) folded into the
   1x1 conv before it, for scoring (eval) forwards; the shift becomes the GEMM bias */
VCG_API int vcg_weight_fold(int dtype, const float* w, const float* scale, void* out, int rows, int cols, hipStream_t s);
/* every conv of the trunk in one launch: desc = DEVICE array of n x 8 int64 (src OIHW f32 ptr, dst bf16 ptr, Cout,
   Cin, KH, KW, Cpad, transposed), each as vcg_weight_prep; bf16 only, each tensor < 2^31 elements */
VCG_API int vcg_weight_prep_multi(int dtype, const long long* desc, int n, hipStream_t s);
/* out[c][r] = in[r][c] ([rows][cols], leading dims ld_in / ld_out): W^T for the BERT input-gradient GEMMs */
VCG_API int vcg_transpose(int dtype, const void* in, void* out, int rows, int cols, long long ld_in, long long ld_out, hipStream_t s);
/* Batched bf16 transpose: desc (DEVICE int64 [n][5]) = (src, dst, rows, cols, first tile), [rows][cols] -> [cols][rows],
   rows and cols multiples of 8, first tile = the running sum of ceil(rows/64) * ceil(cols/64); total_tiles = the sum.
   (BERT's Linear weights transposed once per weight generation for the input-gradient GEMMs.) */
VCG_API int vcg_transpose_multi(const long long* desc, int n, int total_tiles, hipStream_t s);
VCG_API int vcg_cast_from_f32(int dtype, const float* in, void* out, long long n, hipStream_t s);
VCG_API int vcg_cast_to_f32(int dtype, const void* in, float* out, long long n, hipStream_t s);
/* TemporalShift.shift (ops/temporal_shift.py:33-51) on NCHW; direction 1 = its adjoint */
VCG_API int vcg_tsm_shift(int dtype, const void* x, void* y, long long n_batch, int T, int C, long long HW, int fold_div, int direction, hipStream_t s);
VCG_API int vcg_tsm_unshift_add(int dtype, const void* dshift, const void* other, const unsigned char* other_bits, void* dx, long long NT, int T, long long HW, int C, int fold, hipStream_t s);

/* ---- BERT support (bert.hip) ------------------------------------------------------------- */
VCG_API int vcg_embed_ln_fwd(int dtype, const long long* ids, const float* word, const float* pos, const float* type, const float* gamma, const float* beta, void* out, float* mean, float* rstd, int B, int L, int H, float eps, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API long long vcg_ln_bwd_ws_bytes(int rows, int H);
VCG_API int vcg_embed_ln_bwd(int dtype, const void* dout, const long long* ids, const float* word, const float* pos, const float* type, const float* gamma, const float* mean, const float* rstd, float* word_grad, float* pos_grad, float* type_grad, float* gamma_grad, float* beta_grad, float* ws, long long ws_bytes, int B, int L, int H, float dropout_p, unsigned long long seed, long long pad_idx, hipStream_t s);
VCG_API int vcg_ln_fwd(int dtype, const void* x, const void* res, const float* gamma, const float* beta, void* out, float* mean, float* rstd, int rows, int H, float eps, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API int vcg_ln_bwd(int dtype, const void* dout, const void* x, const void* res, const float* gamma, const float* mean, const float* rstd, void* dx, void* dres, float* gamma_grad, float* beta_grad, float* bias_grad, float* ws, long long ws_bytes, int rows, int H, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API long long vcg_colsum_ws_bytes(int rows, int N);
VCG_API int vcg_colsum(int dtype, const void* x, long long ld, int rows, int N, float* out, int accumulate, float* ws, long long ws_bytes, hipStream_t s);
VCG_API int vcg_attn_softmax_fwd(int dtype, const void* S, const long long* mask, void* P, void* Pd, int B, int nh, int L, int Lp, float scale, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API int vcg_attn_softmax_bwd(int dtype, const void* dPd, const void* P, void* dS, int Z, int L, int Lp, float scale, float dropout_p, unsigned long long seed, hipStream_t s);
/* fused self-attention (bert_attn.hip), bf16, L <= 128, head dim 64: ctx = dropout(softmax(scale QK^T + mask)) V
   per (sequence, head) in one workgroup, nothing L x L in HBM; stats [B*nh][128] float2 (row max, 1 / row sum)
   for the backward, which recomputes P and writes dQ | dK | dV into dqkv [B*L][3*H] (its ctx argument may be
   NULL: the row term rowsum(dP o P) comes from the fp32 products, not from the forward's output). Same semantics and dropout
   mask as vcg_attn_softmax_fwd/bwd + the batched GEMMs (HF BertSelfAttention, bert_hugface.py:20). */
VCG_API int vcg_bert_attn_fwd(const void* qkv, const long long* mask, void* ctx, void* stats, int B, int nh, int L, int Lp, float scale, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API int vcg_bert_attn_bwd(const void* qkv, const void* dctx, const void* ctx, const long long* mask, const void* stats, void* dqkv, int B, int nh, int L, int Lp, float scale, float dropout_p, unsigned long long seed, hipStream_t s);
/* packed (unpadded) sequences -- BERT with the padded positions dropped (they feed neither the pooler's CLS row nor any
   kept row: masked keys), reference HF BertModel via bert_hugface.py:20 / two_stream.py:178-179: sequence b's rows are
   seq[b] .. seq[b+1]-1 (int32 [B+1] prefix offsets, each <= Lmax <= 128 rows) of qkv [rows][3H] / ctx / dqkv, mask the
   key flag of every packed row (NULL: all keys); stats and the dropout counters keep the padded [B*nh][Lmax] space */
VCG_API int vcg_bert_attn_fwd_varlen(const void* qkv, const long long* mask, const int* seq, void* ctx, void* stats, int B, int nh, int Lmax, int Lp, float scale, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API int vcg_bert_attn_bwd_varlen(const void* qkv, const void* dctx, const long long* mask, const int* seq, const void* stats, void* dqkv, int B, int nh, int Lmax, int Lp, float scale, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API int vcg_tanh_bwd(int dtype, const void* dy, const void* t, void* dx, long long n, hipStream_t s);

/* ---- fusion head + loss (head.hip): ChapterHead mlp (two_stream.py:51-95), softmax (:189),
 *      F.cross_entropy (train_video_segment_point.py:165) ----------------------------------- */
VCG_API int vcg_head_mlp_fwd(int dtype, const void* Vout, const void* Lout, const float* W, const float* bias, float* logits, float* prob, int B, int T, int hid, int O, hipStream_t s);
VCG_API int vcg_head_mlp_bwd(int dtype, const void* Vout, const void* Lout, const float* W, const float* dlogits, void* dV, void* dL, float* dW, float* dbias, int B, int T, int hid, int O, int relu_mask, hipStream_t s);
/* ChapterHead head_type "attn" (head_attn.hip; also the window ChapterHead "self_attn", O = hid <= 256): SelfAttention(hid, n_head, O) (two_stream.py:8-48) over the T+1
 * fused tokens cat([Vout [B*T][hid], Lout [B][hid]]) of each window, output proj of token 0, softmax. Weights are
 * the fp32 nn.Linear parameters ([out][in]). `saved` (f32, vcg_head_attn_saved_floats) keeps the state of the
 * backward; dropout_p = attn_drop.p in training (counter-hash mask, regenerated by the backward with `seed`). */
VCG_API long long vcg_head_attn_saved_floats(int B, int T, int hid, int nh);
VCG_API int vcg_head_attn_fwd(int dtype, const void* Vout, const void* Lout, const float* Wq, const float* bq, const float* Wk, const float* bk, const float* Wv, const float* bv, const float* Wp, const float* bp, float* saved, long long saved_floats, float* logits, float* prob, int B, int T, int hid, int nh, int O, float dropout_p, unsigned long long seed, hipStream_t s);
/* dVout / dLout = ReLU-masked input gradients (relu_mask: the projections' ReLU); parameter grads (nullable)
   are accumulated (+=). ws: f32 workspace of vcg_head_attn_bwd_ws_floats. */
VCG_API long long vcg_head_attn_bwd_ws_floats(int B, int T, int hid);
VCG_API int vcg_head_attn_bwd(int dtype, const float* saved, const float* Wq, const float* Wk, const float* Wv, const float* Wp, const float* dlogits, void* dVout, void* dLout, float* dWq, float* dbq, float* dWk, float* dbk, float* dWv, float* dbv, float* dWp, float* dbp, float* ws, long long ws_floats, int B, int T, int hid, int nh, int O, float dropout_p, unsigned long long seed, int relu_mask, hipStream_t s);
/* Window transformer StackedVideoChapterAttention, inference (window_attn.hip; replaces the module at
 * model/fusion/stacked_window_self_attention.py:150-223 as called by two_stream_window.py:444): emb [B][S][H] f32
 * per-clip fusion embeddings (S = 2w+1 <= 16, S*H <= 2048), 16 heads in the reference (nh), P = 2w+1 entries of
 * window_pos_bias. `weights` = the f32 parameters packed by vcg_hip/window.py pack_window_weights (Linear weights
 * transposed to [in][out]); logits / prob [B][2]. */
VCG_API long long vcg_window_attn_weight_floats(int H, int nh, int P);
VCG_API int vcg_window_attn_fwd(const float* emb, const float* weights, long long weight_floats, float* logits, float* prob, int B, int S, int H, int nh, int P, hipStream_t s);
/* CrossAttention of the window ChapterHead, head_type "cross_attn" (two_stream_window.py:11-91): lang [B][H] and vis
 * [B][T][H] (the ReLU'd projections) -> out [B][H]; 2 <= T <= 16, T*H <= 2048. `weights` packed by
 * vcg_hip/window.py pack_cross_attn_weights (LN / pos-encoding vectors, then q, k|v, out Linear weights as W^T). */
VCG_API long long vcg_cross_attn_weight_floats(int H);
VCG_API int vcg_cross_attn_fwd(const float* lang, const float* vis, const float* weights, long long weight_floats, float* out, int B, int T, int H, int nh, hipStream_t s);
/* Window ChapterHead "multiplication" / "bilinear" pieces (two_stream_window.py:269-281): out = a * b over n f32
 * (n % 4 == 0); out[b][r] = sum_i U[b][r][i] x[b][i] + bias[r] (nn.Bilinear's second contraction after U = x2 A^T). */
VCG_API int vcg_mul_fwd(const float* a, const float* b, float* out, long long n, hipStream_t s);
VCG_API int vcg_rowdot_fwd(const float* U, const float* x, const float* bias, float* out, int B, int R, int K, hipStream_t s);
/* its backward (the bilinear window head in training): dU[b][r][i] = dy[b][r] x[b][i], dx[b][i] = sum_r dy[b][r] U[b][r][i]
   (dx may be null) */
VCG_API int vcg_rowdot_bwd(const float* U, const float* x, const float* dy, float* dU, float* dx, int B, int R, int K, hipStream_t s);
/* out = act(LayerNorm(x) * gamma + beta) over `rows` rows of D f32 features (window ChapterHead's Linear -> LN -> ReLU
 * chains, two_stream_window.py:145-176); act 0 = none, 1 = ReLU, 2 = GELU (erf). */
VCG_API int vcg_ln_act_fwd(const float* x, const float* gamma, const float* beta, float* out, int rows, int D, float eps, int act, hipStream_t s);
VCG_API int vcg_cross_entropy_fwd(const float* logits, const long long* labels, float* loss, int B, int C, hipStream_t s);
VCG_API int vcg_cross_entropy_bwd(const float* logits, const long long* labels, const float* dloss, float* dlogits, int B, int C, hipStream_t s);

/* ---- optimiser (optim.hip): clip_grad_norm_ (train_video_segment_point.py:204) + AdamW with the
 *      two groups of TwoStream.configure_optimizers (two_stream.py:127-169) ------------------- */
VCG_API long long vcg_sumsq_ws_bytes(void);
VCG_API int vcg_sumsq(const float* x, long long n, float* ws, float* out, hipStream_t s);
VCG_API int vcg_adamw(float* p, const float* g, float* m, float* v, const unsigned char* wd_flags, int flag_shift, long long n, float lr, float beta1, float beta2, float eps, float wd, float step_size, float bc2_sqrt, const float* sumsq, float max_norm, float grad_scale, void* bf16_shadow, hipStream_t s);

/* ---- window-model training (wtrain.hip): model/fusion/two_stream_window.py ChapterHead chains / CrossAttention and
 *      stacked_window_self_attention.py (trained by train_video_segment_ddp.py:294-342). fp32 [rows][D]; dropout masks
 *      regenerated in the backward from (seed, element index); act 0 none / 1 ReLU / 2 erf-GELU ------------------- */
/* out = Dropout(act(LayerNorm(x))) (nn.LayerNorm, eps given); mean / rstd [rows] saved for the backward */
VCG_API int vcg_ln_act_drop_fwd(const float* x, const float* gamma, const float* beta, float* out, float* mean, float* rstd, int rows, int D, float eps, int act, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API long long vcg_ln_act_drop_bwd_ws_bytes(int rows, int D);
/* dx (written) and gamma_grad / beta_grad (accumulated, fixed-order reduction) */
VCG_API int vcg_ln_act_drop_bwd(const float* dout, const float* x, const float* gamma, const float* beta, const float* mean, const float* rstd, float* dx, float* gamma_grad, float* beta_grad, float* ws, long long ws_bytes, int rows, int D, int act, float dropout_p, unsigned long long seed, hipStream_t s);
/* out = Dropout(act(x)) (+ res) ; dx = d/dx of Dropout(act(x)) */
VCG_API int vcg_act_drop_fwd(const float* x, const float* res, float* out, long long n, int act, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API int vcg_act_drop_bwd(const float* dout, const float* x, float* dx, long long n, int act, float dropout_p, unsigned long long seed, hipStream_t s);
/* da = dout * b, db = dout * a (either may be NULL) */
VCG_API int vcg_mul_bwd(const float* dout, const float* a, const float* b, float* da, float* db, long long n, hipStream_t s);
/* multi-head attention of short windows (VideoChapterWindowAttention.forward stacked_window_self_attention.py:55-95,
   CrossAttention.forward two_stream_window.py:55-91): per window b, Sq queries over Sk keys (<= 32), nh heads of dh
   (<= 16) columns of row-major q / k / v (leading dims given), scores * scale + bias[h][j] (bias [nh][Pb] or NULL),
   softmax -> probs [B][nh][Sq][Sk] (saved), dropout, ctx = P V. Backward: dq / dk / dv written, dbias accumulated. */
VCG_API int vcg_mha_small_fwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv, const float* bias, int Pb, float* ctx, long long ldc, float* probs, int B, int Sq, int Sk, int nh, int dh, float scale, float dropout_p, unsigned long long seed, hipStream_t s);
VCG_API long long vcg_mha_small_bwd_ws_bytes(int B, int nh, int Pb);
VCG_API int vcg_mha_small_bwd(const float* q, long long ldq, const float* k, long long ldk, const float* v, long long ldv, const float* probs, const float* dctx, long long lddc, float* dq, long long lddq, float* dk, long long lddk, float* dv, long long lddv, float* dbias, int Pb, float* ws, long long ws_bytes, int B, int Sq, int Sk, int nh, int dh, float scale, float dropout_p, unsigned long long seed, hipStream_t s);

/* Linear(1, H) position encoding of token r % S added to row r: out = x + pos[r % S] * w + b; backward accumulates
   dw / db (fixed row order); the input gradient is dout itself */
VCG_API int vcg_posenc_fwd(const float* x, const float* pos, const float* w, const float* b, float* out, long long rows, int S, int H, hipStream_t s);
VCG_API int vcg_posenc_bwd(const float* d, const float* pos, float* dw, float* db, long long rows, int S, int H, hipStream_t s);
/* Linear layers narrower than the GEMM's 16-byte tiles (K or N % 4 != 0: the 2-way classifiers):
   y = act(x W^T + b + res); backward: dx written, dw / db accumulated (fixed order) */
VCG_API int vcg_linear_small_fwd(const float* x, const float* W, const float* b, const float* res, float* y, int M, int N, int K, int act, hipStream_t s);
VCG_API int vcg_linear_small_bwd(const float* g, const float* x, const float* W, float* dx, float* dw, float* db, int M, int N, int K, hipStream_t s);
/* softmax over the C entries of each row (the window model's prob output) */
VCG_API int vcg_softmax_rows(const float* x, float* out, int rows, int C, hipStream_t s);

/* ---- gradient exchange over RCCL / xGMI (comm.hip) --------------------------------------------
 * Replaces the NCCL communicator of DDP(model) in train_video_segment_ddp.py:64-86 (init_process_group) and :148
 * (bucketed gradient all-reduce on every backward) and the parameter broadcast of :261-263. One communicator per
 * process (one process per GPU); RCCL is the one already mapped into the process (PyTorch-ROCm's) or
 * /opt/rocm/lib/librccl.so.1. Calls are asynchronous on `s`: issue them on a side stream that waits for the
 * bucket's producer to overlap the exchange with the backward (vcg_hip/comm.py). */
VCG_API int vcg_comm_unique_id(void* uid_out, int uid_bytes);                 /* rank 0: 128-byte id */
VCG_API int vcg_comm_init(int rank, int world, const void* uid, int uid_bytes); /* collective */
VCG_API int vcg_comm_world(int* rank, int* world);
VCG_API int vcg_allreduce_bucket(void* ptr, long long count, int dtype, hipStream_t s);  /* in-place SUM */
VCG_API int vcg_broadcast_bucket(void* ptr, long long count, int dtype, int root, hipStream_t s);
VCG_API int vcg_comm_finalize(void);

/* ---- synthetic inputs (synth.hip): seeded clip windows / weights, bit-identical to numpy ---- */
VCG_API int vcg_synth(int kind, void* out, long long n, unsigned long long key, double a, double b, hipStream_t s);

#ifdef __cplusplus
}
#endif
#endif
