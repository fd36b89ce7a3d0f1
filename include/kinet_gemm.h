/* kinet_amd C-ABI: MFMA GEMM and implicit-GEMM NHWC convolution with fused epilogues.
 *
 * Replaces, on the detection hot path, the cuBLAS/cuDNN work the reference delegates
 * to PyTorch ("Dense ops on the hot path"):
 *   nn.Linear in MSDeformAttn          (ms_deform_attn.py:27-30)
 *   FFN linear1/linear2                (deformable_transformer.py:273-276, 350-353)
 *   nn.MultiheadAttention in/out proj  (deformable_transformer.py:345, :371)
 *   class / bbox MLP heads             (deformable_detr.py:98-108, detr.py:937-951)
 *   ResNet convs + FrozenBatchNorm2d   (backbone.py:22-58, :102)  -- BN folded into scale/bias
 *   input_proj 1x1 / 3x3-s2 convs      (deformable_detr.py:63-71)
 *
 *   C[m, n] = epi( sum_k A[m, k] * B[n, k] )
 *   epi(v)  = relu?( v * scale[n] + bias[n] + R[m, n] ),  rows with row_mask[m] != 0 -> 0
 *
 * A, B, C, R row-major with leading dims lda, ldb, ldc, ldr (elements).  B is the
 * PyTorch weight layout (out_features, in_features), i.e. K-contiguous.  scale/bias
 * are f32 (NULL = 1 / 0).  in_dtype in {F32, BF16, F16} for A and B; out_dtype for C
 * and R in {F32, BF16, F16}.  bf16/f16 run v_mfma_f32_16x16x32_{bf16,f16}; f32 runs the
 * exact-f32 v_mfma_f32_16x16x4_f32 (parity mode).  Requirements: K % 8 == 0, lda/ldb
 * multiples of 8, 16-byte aligned A/B.
 */
#ifndef KINET_GEMM_H_
#define KINET_GEMM_H_

#include "kinet_common.h"

#ifdef __cplusplus
extern "C" {
#endif

int kinet_gemm(const void* A, const void* B, void* C, int M, int N, int K,
               int lda, int ldb, int ldc, int in_dtype,
               const float* scale, const float* bias, const void* R, int ldr,
               int relu, int out_dtype, const uint8_t* row_mask, int reserved,
               kinet_stream_t stream);

/* Extended form: A2 (optional, same layout as A) is added to A at load time
 * (q = src + pos feeding a projection, deformable_transformer.py:292, :369, :377);
 * ln_gamma/ln_beta (optional, f32, N <= 320) apply LayerNorm(eps) over each output row
 * after the bias + residual add -- the post-norm of a transformer sub-layer
 * (deformable_transformer.py:287, :294, :364, :374, :380) fused into the GEMM epilogue. */
int kinet_gemm_ex(const void* A, const void* A2, const void* B, void* C, int M, int N, int K,
                  int lda, int ldb, int ldc, int in_dtype,
                  const float* scale, const float* bias, const void* R, int ldr, int relu,
                  const float* ln_gamma, const float* ln_beta, float ln_eps,
                  int out_dtype, const uint8_t* row_mask, kinet_stream_t stream);

/* Convolution, NHWC activations, weights (Cout, KH, KW, Cin) = PyTorch OIHW permuted.
 *   X (batch, Hin, Win, Cin) with Cin % 8 == 0 (pad channels with zeros otherwise)
 *   Y (batch, Hout, Wout, Cout) written with row stride ldy (>= Cout) so outputs can land
 *   directly inside a larger flattened buffer; R residual with the same layout (ldr).
 *   Hout = (Hin + 2*pad - KH) / stride + 1 (dilation 1). */
int kinet_conv2d(const void* X, const void* Wt, void* Y, int batch, int Hin, int Win, int Cin,
                 int Hout, int Wout, int Cout, int KH, int KW, int stride, int pad,
                 int in_dtype, const float* scale, const float* bias, const void* R, int ldr,
                 int relu, int ldy, kinet_stream_t stream);

/* kinet_conv2d with separate vertical / horizontal stride and padding
 * (Hout = (Hin + 2*pad_h - KH)/stride_h + 1, Wout = (Win + 2*pad_w - KW)/stride_w + 1);
 * used for the tap-folded ResNet stem (kinet_pack_image_kwfold). */
int kinet_conv2d_ex(const void* X, const void* Wt, void* Y, int batch, int Hin, int Win, int Cin,
                    int Hout, int Wout, int Cout, int KH, int KW, int stride_h, int stride_w, int pad_h,
                    int pad_w, int in_dtype, const float* scale, const float* bias, const void* R, int ldr,
                    int relu, int ldy, kinet_stream_t stream);

/* value_proj for MSDA: C = (A @ B^T + bias) with rows masked, stored HEAD-MAJOR:
 * row r = b*rows_per_batch + s, column n = g*head_dim + d  ->  C[((g*batch + b)*rows_per_batch + s)*head_dim + d]
 * i.e. (N/head_dim, batch, rows_per_batch, head_dim) -- the layout kinet_msda_fused_forward
 * gathers from best (ms_deform_attn.py:64-67 produce the same values in (N, S, M, D)).
 * out_dtype: in_dtype, or KINET_F16 from KINET_BF16 operands (f16 values feed the sampling
 * kernel's mixed-precision FMA; post-LayerNorm projections are far inside f16 range). */
int kinet_gemm_headmajor(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                         int in_dtype, int out_dtype, const float* bias, const uint8_t* row_mask,
                         int rows_per_batch, int head_dim, kinet_stream_t stream);

/* kinet_gemm_headmajor with A + A2 as the left operand (the position embedding added at load
 * time, `with_pos_embed` of deformable_transformer.py:278); the MSDA offsets / logits
 * projection of the encoder writes (M, N, Lq, L*P*3) head-major this way
 * (kinet_msda_encoder_forward).  a2_rows: 0 = A2 has M rows like A; else A2 has a2_rows rows
 * (>= 32, dividing M) and row m adds A2 row m % a2_rows -- one frame's position embedding
 * shared by every frame of an unpadded batch (the same values the reference adds per frame). */
int kinet_gemm_headmajor_ex(const void* A, const void* A2, const void* B, void* C, int M, int N, int K,
                            int lda, int ldb, int in_dtype, int out_dtype, const float* bias,
                            const uint8_t* row_mask, int rows_per_batch, int head_dim, int a2_rows,
                            kinet_stream_t stream);

/* Split head-major store (round 5, the head_dim-36 MSDA value of configs 3-5): the weight rows
 * are ordered [every head's first head_dim channels | every head's last tail_dim channels];
 * columns [0, split_cols) go head-major (split_cols/head_dim, B, S, head_dim) to C and columns
 * [split_cols, N) head-major (heads, B, S, tail_dim) right after that plane, at
 * C + split_cols*M elements.  kinet_msda_encoder_forward_split reads the two planes.  Replaces
 * the value_proj + view of ms_deform_attn.py:64-66 for that kernel. */
int kinet_gemm_headmajor_split(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb,
                               int in_dtype, int out_dtype, const float* bias, const uint8_t* row_mask,
                               int rows_per_batch, int head_dim, int split_cols, int tail_dim,
                               kinet_stream_t stream);

/* Split-K forms for small-M / long-K problems (few output tiles): K is cut into `ksplit`
 * slices (rounded to whole 64-element K-steps) whose f32 partial tiles go to `workspace`
 * (ksplit * M * N floats, caller-allocated), then one finalize pass sums the slices and
 * applies the same epilogue (scale/bias, residual, ReLU, LayerNorm for N <= 1024, row mask)
 * into C / Y.  Deterministic (no atomics). */
int kinet_gemm_splitk(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                      int in_dtype, const float* scale, const float* bias, const void* R, int ldr, int relu,
                      const float* ln_gamma, const float* ln_beta, float ln_eps, int out_dtype,
                      const uint8_t* row_mask, float* workspace, int ksplit, kinet_stream_t stream);
int kinet_conv2d_splitk(const void* X, const void* Wt, void* Y, int batch, int Hin, int Win, int Cin,
                        int Hout, int Wout, int Cout, int KH, int KW, int stride, int pad, int in_dtype,
                        const float* scale, const float* bias, const void* R, int ldr, int relu, int ldy,
                        float* workspace, int ksplit, kinet_stream_t stream);

/* ResNet stem from the image (torchvision conv1, 7x7 / stride 2 / pad 3, 3 -> 64, + folded
 * FrozenBN + ReLU; the reference's backbone.py:102 body, IntermediateLayerGetter input): img
 * f32 NCHW (N, 3, H, W) -> Y NHWC (N, (H-1)/2+1, (W-1)/2+1, 64) in dtype (KINET_BF16 /
 * KINET_F16).  Replaces kinet_pack_image_kwfold + kinet_conv2d_ex over the folded layout
 * (same values: the image is rounded to dtype once, the tap-folded rows are built in LDS);
 * w_packed = the folded stem weights (64, 7, 1, 24) of that path; scale / bias (64) f32. */
int kinet_stem_conv_image(const float* img, const void* w_packed, const float* scale, const float* bias,
                          void* Y, int N, int H, int W, int dtype, kinet_stream_t stream);

/* Diagnostic kernel-selection knob (no reference counterpart; used by the kernel
 * benchmarks to A/B GEMM kernels in one process).  bit 1: allow the 512-thread
 * 256x256-tile LDS-DMA kernel for large-M problems; bit 2: never use the
 * resident-weight streaming kernel; bit 8 (256): keep K = 512 problems off it (the
 * tiled kernel, as before round 3); bit 1024: never the direct 3x3 64 -> 64 channel
 * convolution (the implicit GEMM instead); bit 2048: strided 1x1 convolutions (the stage-2
 * downsample) on the implicit-GEMM kernel instead of the resident-weight conv-row kernel;
 * bit 268435456: the resident-weight kernel's 4-wave column groups everywhere (round 6 runs the
 * x + pos projections, K = 512 / N = 256, residual N > 256 and K = 288 N > 384 launches on
 * 8-wave groups); bit 1073741824: 32-column head-major stores without the LDS transpose.
 * All of these select among bit-identical kernels.  Returns the previous flags.  Per CALLING THREAD: torch
 * runs autograd backward for device tensors on its own engine thread, so flags set here do
 * NOT reach the backward kernels launched through autograd (only forward / direct calls). */
int kinet_gemm_set_flags(int flags);

/* Launch-fill policy (no reference counterpart), process-wide.  1 = "solo": the caller keeps one
 * batch in flight, so no other stream's work fills CUs a launch leaves idle -- shapes whose
 * default tiles cover under 60 % of one round of workgroups per CU (config 5's stage-3 3x3
 * convolutions and D = 256 bottleneck pairs, M = 32,640 rows) switch to tiles half as tall that
 * fill the chip: config 5 on one stream 239 -> 257 frames/s.  0 (default) = throughput mode:
 * with several batches in flight the other streams fill those CUs and the taller tiles' better
 * per-CU efficiency wins (config 5 on 3 streams 294 vs 290 frames/s).  Same outputs bit for bit
 * either way.  Returns the previous policy. */
int kinet_set_solo_launch(int on);

#ifdef __cplusplus
}
#endif

#endif /* KINET_GEMM_H_ */
