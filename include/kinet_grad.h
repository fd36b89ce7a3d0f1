/* kinet_amd C-ABI: backward-pass kernels of the training path.
 *
 * The reference trains with losses.backward() (src/trackformer/engine.py:145-149), i.e. the
 * autograd of torch's Conv2d / Linear / LayerNorm / GroupNorm / MultiheadAttention modules
 * (cuDNN / cuBLAS / ATen) around the MSDeformAttn CUDA backward (ms_deform_attn_cuda.cu:
 * 89-168, replaced by kinet_msda_backward, kinet_msda.h).  kinet_amd/autograd.py wires these
 * kernels into torch.autograd.Functions; the forward halves reuse kinet_gemm.h / kinet_ops.h.
 * Conventions as in kinet_common.h (device pointers, caller's stream, caller workspace, int
 * status).  Every reduction runs in a fixed order (no float atomics): gradients are
 * bit-identical across reruns.
 */
#ifndef KINET_GRAD_H_
#define KINET_GRAD_H_

#include "kinet_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* dst (cols x rows, row stride ld_dst) = src^T (src rows x cols, row stride ld_src); 2/4-byte
 * element types (F32, BF16, F16). */
int kinet_transpose(const void* src, void* dst, int rows, int cols, int64_t ld_src, int64_t ld_dst,
                    int dtype, kinet_stream_t stream);

/* Patch matrix of an NHWC convolution (torch Conv2d geometry, backbone.py / deformable_detr.py:63-71):
 *   cols[(n*Ho + ho)*Wo + wo][(kh*KW + kw)*C + c] = x[n][ho*sh - ph + kh][wo*sw - pw + kw][c]
 * (0 outside the image); C % 4 == 0. */
int kinet_im2col_nhwc(const void* x, void* cols, int B, int H, int W, int C, int Ho, int Wo, int KH, int KW,
                      int sh, int sw, int ph, int pw, int dtype, kinet_stream_t stream);

/* Adjoint of kinet_im2col_nhwc (the input gradient of the convolution given the gradient of
 * its patch matrix): dx[n][h][w][c] = sum of the cols entries that read x[n][h][w][c], summed
 * per pixel in (kh, kw) order; dx fully overwritten. */
int kinet_col2im_nhwc(const void* cols, void* dx, int B, int H, int W, int C, int Ho, int Wo, int KH, int KW,
                      int sh, int sw, int ph, int pw, int dtype, kinet_stream_t stream);

/* C (M x N, f32, row stride ldc) = A^T B (+ C if accumulate), A (K x M) and B (K x N) row-major
 * in dtype (F32: exact-f32 MFMA; BF16/F16 widened to f32).  The weight gradient of a Linear
 * (dW = dY^T X) and of a convolution (dW = dZ^T im2col(X)).  Split over K when the output has
 * few tiles: `workspace` must then hold kinet_gemm_tn_workspace(M, N, K) floats (0 = none
 * needed; accumulate always needs at least M*N). */
int64_t kinet_gemm_tn_workspace(int M, int N, int K);
int kinet_gemm_tn(const void* A, const void* B, float* C, int M, int N, int K, int64_t lda, int64_t ldb,
                  int64_t ldc, int dtype, int accumulate, float* workspace, kinet_stream_t stream);

/* out[c] (+)= sum_r A[r*lda + c] (f32): bias gradients.  workspace: kinet_colsum_workspace floats. */
int64_t kinet_colsum_workspace(int rows, int cols);
int kinet_colsum(const void* A, float* out, int rows, int cols, int64_t lda, int dtype, int accumulate,
                 float* workspace, kinet_stream_t stream);

/* nn.LayerNorm backward over the last dim d <= 1024 (statistics recomputed from x):
 * dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma; dgamma = sum dy*xhat,
 * dbeta = sum dy (either may be NULL).  workspace: kinet_layernorm_backward_workspace floats. */
int64_t kinet_layernorm_backward_workspace(int rows, int d);
int kinet_layernorm_backward(const void* dy, const void* x, const float* gamma, void* dx, float* dgamma,
                             float* dbeta, int rows, int d, float eps, int dtype, float* workspace,
                             kinet_stream_t stream);

/* nn.GroupNorm(groups, C) backward on NHWC (N, HW, C) input (the forward is kinet_groupnorm).
 * workspace: kinet_groupnorm_backward_workspace floats. */
int64_t kinet_groupnorm_backward_workspace(int N, int HW, int C, int groups);
int kinet_groupnorm_backward(const void* dy, const void* x, const float* gamma, void* dx, float* dgamma,
                             float* dbeta, int N, int HW, int C, int groups, float eps, int dtype,
                             float* workspace, kinet_stream_t stream);

/* Backward of kinet_mha_core / kinet_mha_core_dropout (f32): given Q, K, V (row strides ld*),
 * dO, writes dQ, dK, dV (same layouts and strides as Q, K, V).  head_dim <= 64.  workspace:
 * kinet_mha_backward_workspace floats (the dropped probabilities and the score gradient).
 * dropout_p / dropout_seed: those of the forward (0 / NULL: no dropout); the keep mask is
 * regenerated from the seed (include/kinet_ops.h kinet_dropout_mask). */
int64_t kinet_mha_backward_workspace(int batch, int Lq, int Lk, int heads);
int kinet_mha_backward(const float* Q, int ldq, const float* K, int ldk, const float* V, int ldv,
                       const float* dO, int ldo, float* dQ, float* dK, float* dV, int batch, int Lq, int Lk,
                       int heads, int head_dim, float scale, const uint8_t* key_mask, float* workspace,
                       float dropout_p, const int64_t* dropout_seed, kinet_stream_t stream);

/* ---- training-path glue (kinet_amd/csrc/train_ops.hip), f32, replacing torch elementwise ops.
 * Dropout keep masks: the counter hash of kinet_dropout_mask (include/kinet_ops.h) over the
 * element's flat index, keyed by the device int64 *dropout_seed; kept values scaled 1/(1-p). */

/* Post-norm residual sub-layer y = LayerNorm(x + dropout_p(r)) over rows of d <= 1024
 * (deformable_transformer.py:100,108,186,196,199: `norm(src + dropout(src2))`). */
int kinet_dropout_add_layernorm(const float* x, const float* r, const float* gamma, const float* beta, float* y,
                                int rows, int d, float eps, float dropout_p, const int64_t* dropout_seed,
                                kinet_stream_t stream);
/* Its backward (x + dropout(r) recomputed from x, r and the seed): dx = dL/d(x + Z r), dr = Z dx,
 * dgamma / dbeta (both or neither; fixed-order partial sums in `workspace`, sized by
 * kinet_dropout_add_layernorm_backward_workspace floats).  dx or dr may be NULL. */
int64_t kinet_dropout_add_layernorm_backward_workspace(int rows, int d);
int kinet_dropout_add_layernorm_backward(const float* dy, const float* x, const float* r, const float* gamma,
                                         float* dx, float* dr, float* dgamma, float* dbeta, int rows, int d,
                                         float eps, float dropout_p, const int64_t* dropout_seed, float* workspace,
                                         kinet_stream_t stream);

/* y = dropout_p(relu ? max(x, 0) : x), n elements (the FFN hidden, deformable_transformer.py:99,185);
 * backward dx = Z * dy * (relu ? [y > 0] : 1).  16-byte aligned buffers. */
int kinet_dropout_act(const float* x, float* y, int64_t n, int relu, float dropout_p, const int64_t* dropout_seed,
                      kinet_stream_t stream);
int kinet_dropout_act_backward(const float* dy, const float* y, float* dx, int64_t n, int relu, float dropout_p,
                               const int64_t* dropout_seed, kinet_stream_t stream);

/* MSDeformAttn sampling preparation (ms_deform_attn.py:64-82) from the packed projection output
 * offlog (nq = N*Lq rows of stride ld floats: heads*L*P*2 sampling offsets (m, l, p, xy), then
 * heads*L*P attention logits (m, l, p) -- one GEMM over the concatenated sampling_offsets |
 * attention_weights weights): per (row, head) attw = softmax over the L*P logits (0 where
 * query_mask), loc = ref + off / (H_l, W_l) for 2-d refs (the reference's divisor order) or
 * ref_xy + off / P * ref_wh * 0.5 for 4-d refs.  loc (nq, heads, L, P, 2), attw (nq, heads, L, P),
 * refs (nq, L, ref_dim), shapes (L, 2) int64 (H, W). */
int kinet_msda_prep(const float* offlog, int64_t ld, const float* refs, const int64_t* shapes,
                    const uint8_t* query_mask, float* loc, float* attw, int64_t nq, int heads, int levels, int points,
                    int ref_dim, kinet_stream_t stream);
/* Its backward: grad_offlog (same layout and stride as offlog: offset gradients, then the softmax
 * backward through attw), grad_refs (summed over heads and points); either may be NULL.  heads a
 * power of two <= 64. */
int kinet_msda_prep_backward(const float* grad_loc, const float* grad_attw, const float* attw, const float* offlog,
                             int64_t ld, const float* refs, const int64_t* shapes, float* grad_offlog,
                             float* grad_refs, int64_t nq, int heads, int levels, int points, int ref_dim,
                             kinet_stream_t stream);

/* inverse_sigmoid (util/misc.py:609-613): y = log(max(c, eps) / max(1 - c, eps)), c = clamp(x, 0, 1),
 * and its backward through the clamps' gradient masks. */
int kinet_inverse_sigmoid(const float* x, float* y, int64_t n, float eps, kinet_stream_t stream);
int kinet_inverse_sigmoid_backward(const float* dy, const float* x, float* dx, int64_t n, float eps,
                                   kinet_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* KINET_GRAD_H_ */
