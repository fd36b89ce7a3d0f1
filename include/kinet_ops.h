/* kinet_amd C-ABI: normalisation / pooling / attention kernels on the detection path.
 * dtype codes: include/kinet_common.h.  All tensors contiguous unless a stride is given.
 */
#ifndef KINET_OPS_H_
#define KINET_OPS_H_

#include "kinet_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* y = LayerNorm(x (+ r)) over the last dim d (nn.LayerNorm, eps) -- the post-norm of every
 * encoder/decoder sub-layer (deformable_transformer.py:287, :294, :374, :380, :364).
 * x, r, y: (rows, d) in `dtype`; gamma/beta f32; r may be NULL. */
int kinet_layernorm(const void* x, const void* r, const float* gamma, const float* beta, void* y,
                    int rows, int d, float eps, int dtype, int reserved, kinet_stream_t stream);

/* nn.GroupNorm(groups, C) on NHWC input (deformable_detr.py:64, :70):
 * x (N, HW, C) contiguous; y written at y + n*y_batch_stride + p*C + c (so a level can land
 * inside the flattened multi-level src buffer, deformable_transformer.py:145-153).
 * `stats`: caller-provided scratch of kinet_groupnorm_workspace(N, HW, C, groups, dtype) floats;
 * its first 2*N*groups floats hold (sum, sumsq) per image x group on return.  Every reduction
 * runs in a fixed order (no float atomics): reruns are bit-identical. */
long kinet_groupnorm_workspace(int N, int HW, int C, int groups, int dtype);
int kinet_groupnorm(const void* x, const float* gamma, const float* beta, void* y,
                    int N, int HW, int C, int groups, int y_batch_stride, float eps, int dtype,
                    float* stats, kinet_stream_t stream);

/* ResNet stem max-pool 3x3/2 pad 1 (torchvision), NHWC. */
int kinet_maxpool2d_3x3s2(const void* x, void* y, int N, int H, int W, int C, int dtype,
                          kinet_stream_t stream);

/* (N, 3, H, W) f32 NCHW image -> (N, H, W, Cpad) NHWC in dtype, channels >= 3 zero. */
int kinet_pack_image_nhwc(const float* x, void* y, int N, int H, int W, int Cpad, int dtype,
                          kinet_stream_t stream);

/* Stem input with the horizontal taps of a KW-wide, stride-s filter folded into channels:
 * (N, 3, H, W) f32 NCHW -> (N, H, Wo, Cg) in bf16/f16/f32 with y[n][h][ow][kw*3 + c] =
 * x[n][c][h][ow*stride - pad + kw] (0 outside the image and for channels >= 3*KW),
 * Wo = (W + 2*pad - KW)/stride + 1, Cg % 8 == 0.  The KHxKW stride-s convolution of the image
 * (ResNet conv1, backbone.py) is then the KHx1 convolution of y with strides (s, 1), pads
 * (pad, 0) and weights w'[o][kh][0][kw*3 + c] = w[o][c][kh][kw] (kinet_conv2d_ex). */
int kinet_pack_image_kwfold(const float* x, void* y, int N, int H, int W, int KW, int stride, int pad,
                            int Cg, int dtype, kinet_stream_t stream);

/* y = a + b, n elements. */
int kinet_add(const void* a, const void* b, void* y, int64_t n_lo, int dtype, kinet_stream_t stream);

/* Scaled-dot-product core of nn.MultiheadAttention (deformable_transformer.py:371):
 *   O[b, i, h*D:(h+1)*D] = softmax_j( Q_bh[i] . K_bh[j] * scale  (-inf where key_mask[b,j]) ) V_bh[j]
 * Q/K/V/O row-major with row strides ldq/ldk/ldv/ldo (elements), batch strides = rows*ld. */
int kinet_mha_core(const void* Q, int ldq, const void* Kt, int ldk, const void* V, int ldv,
                   void* O, int ldo, int batch, int Lq, int Lk, int heads, int head_dim,
                   float scale, int dtype, const uint8_t* key_mask, kinet_stream_t stream);

/* kinet_mha_core with attention-probability dropout, the training form of
 * nn.MultiheadAttention(d, heads, dropout=p) (deformable_transformer.py:345; torch applies
 * F.dropout to the softmax output):
 *   O[b, i, h] = sum_j softmax_j(...)[j] * Z[b, h, i, j] * V_bh[j],  Z in {0, 1/(1-p)}
 * Z from kinet_dropout_mask's counter-based hash of (*dropout_seed, ((b*heads + h)*Lq + i)*Lk + j)
 * (dropout_seed: a device int64, so drawing it needs no host sync).  Runs the FMA kernel. */
int kinet_mha_core_dropout(const void* Q, int ldq, const void* Kt, int ldk, const void* V, int ldv,
                           void* O, int ldo, int batch, int Lq, int Lk, int heads, int head_dim,
                           float scale, int dtype, const uint8_t* key_mask, float dropout_p,
                           const int64_t* dropout_seed, kinet_stream_t stream);

/* The keep mask those kernels use: keep[idx] = 1 if element idx (0 <= idx < n) is kept at
 * dropout probability p under *dropout_seed (tests, and callers that need the mask). */
int kinet_dropout_mask(const int64_t* dropout_seed, int64_t n, float dropout_p, uint8_t* keep,
                       kinet_stream_t stream);

/* Diagnostic knob (no reference counterpart): 1 (default) = kinet_mha_core runs head_dim 32,
 * bf16/f16, Lk <= 384 on the MFMA kernel (attn.hip), 0 = always the FMA kernel.  Returns the
 * previous setting. */
int kinet_mha_set_mfma(int enable);

/* Iterative box refinement (deformable_transformer.py:414-425) fused with the next
 * layer's reference input (:406-411):
 *   new_ref = sigmoid(tmp + inverse_sigmoid(ref))        (ref_dim 4)
 *   new_ref = sigmoid([tmp[:2] + inverse_sigmoid(ref), tmp[2:]])   (ref_dim 2)
 *   ref_input[b,q,l,:] = new_ref * [vr_l, vr_l]
 * tmp (N*Q, 4) f32, ref (N*Q, ref_dim) f32, valid_ratios (N, L, 2) f32;
 * new_ref (N*Q, 4) f32, ref_input (N*Q, L, 4) f32. */
int kinet_box_refine(const float* tmp, const float* ref, int ref_dim, const float* valid_ratios,
                     float* new_ref, float* ref_input, int N, int Q, int L, kinet_stream_t stream);

/* Sine position embedding of a padding mask (PositionEmbeddingSine, position_encoding.py:85-121;
 * PositionEmbeddingSine3D, :12-81, one frame `frame` of `frames` at a time), written as NHWC rows:
 *   out[b*out_batch_stride + (h*W + w)*C + c] = pe(b, h, w, c) (+ level_embed[c] if non-NULL)
 * C = 2*num_pos_feats ([y | x]) or 3*num_pos_feats ([z | y | x]); channel 2k = sin(e / dim_t[2k]),
 * 2k+1 = cos(e / dim_t[2k+1]) with e the (normalised) cumulative count of unmasked pixels.
 * dim_t (num_pos_feats f32, device): temperature ** (2 * (k // 2) / num_pos_feats) as the caller
 * computes it (kinet_amd evaluates it with torch on the host, as the reference does). */
int kinet_sine_position_embed(const uint8_t* mask, const float* dim_t, const float* level_embed, void* out,
                              int B, int H, int W, int num_pos_feats, int three_d, int frame, int frames,
                              int normalize, float scale, int64_t out_batch_stride, int out_dtype,
                              kinet_stream_t stream);

/* Greedy non-maximum suppression with torchvision.ops.nms semantics (the tracker's track /
 * detection NMS, tracker.py:437, :511): boxes (n, 4) xyxy f32, scores (n) f32 -> keep[i] = 1 for
 * the kept boxes (in order of descending score, ties by index; a box is dropped when its IoU
 * with a kept higher-ranked box exceeds iou_threshold).  n <= 4096, one workgroup. */
int kinet_nms(const float* boxes, const float* scores, uint8_t* keep, int n, float iou_threshold,
              kinet_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* KINET_OPS_H_ */
